"""Host-staged rank transport over torch.distributed (gloo).

The library's default multi-rank transport is RCCL on the context stream
(gh_ctx_create_dist).  This one moves the same two collectives — an
all-gather of a few words per rank and the pairwise exchange of state rows at
a resample — through host memory with a CPU process group.  It
lets several ranks share one GPU (the one-GPU test box) and runs the
multi-rank algorithm where RCCL peer access is unavailable.  It synchronises
the stream at every collective, so it is a correctness transport, not the
benchmark path.
"""
from __future__ import annotations

import ctypes
from ctypes import CFUNCTYPE, POINTER, c_int, c_uint64, c_void_p

import numpy as np

ALLGATHER_FN = CFUNCTYPE(c_int, c_void_p, c_void_p, c_void_p, c_uint64)
SENDRECV_FN = CFUNCTYPE(
    c_int, c_void_p,
    c_int, POINTER(c_int), POINTER(c_void_p), POINTER(c_uint64),
    c_int, POINTER(c_int), POINTER(c_void_p), POINTER(c_uint64),
)


class HostComm(ctypes.Structure):
    _fields_ = [("user", c_void_p), ("allgather", ALLGATHER_FN), ("sendrecv", SENDRECV_FN)]


def _host_bytes(ptr: int, n: int) -> np.ndarray:
    return np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(ptr))


class GlooTransport:
    """Callbacks for gh_ctx_create_hostcomm over a torch.distributed group."""

    def __init__(self, group=None):
        import torch.distributed as dist

        if not dist.is_initialized():
            raise RuntimeError("GlooTransport needs an initialised torch.distributed process group")
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self._ag = ALLGATHER_FN(self._allgather)
        self._sr = SENDRECV_FN(self._sendrecv)
        self.struct = HostComm(None, self._ag, self._sr)
        self.calls = {"allgather": 0, "sendrecv": 0}

    def _allgather(self, _user, send, recv, nbytes):
        try:
            import torch

            t = torch.from_numpy(_host_bytes(send, nbytes).copy())
            outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
            self.dist.all_gather(outs, t, group=self.group)
            dst = _host_bytes(recv, nbytes * self.world)
            for r, o in enumerate(outs):
                dst[r * nbytes : (r + 1) * nbytes] = o.numpy()
            self.calls["allgather"] += 1
            return 0
        except Exception as e:  # an exception must not cross the C boundary
            print(f"GlooTransport.allgather failed: {e!r}", flush=True)
            return 1

    def _sendrecv(self, _user, ns, speers, sbufs, sbytes, nr, rpeers, rbufs, rbytes):
        try:
            import torch

            reqs, recv_t = [], []
            for i in range(ns):
                t = torch.from_numpy(_host_bytes(sbufs[i], int(sbytes[i])).copy())
                reqs.append(self.dist.isend(t, int(speers[i]), group=self.group))
            for i in range(nr):
                t = torch.empty(int(rbytes[i]), dtype=torch.uint8)
                recv_t.append((t, rbufs[i], int(rbytes[i])))
                reqs.append(self.dist.irecv(t, int(rpeers[i]), group=self.group))
            for r in reqs:
                r.wait()
            for t, ptr, n in recv_t:
                _host_bytes(ptr, n)[:] = t.numpy()
            self.calls["sendrecv"] += 1
            return 0
        except Exception as e:
            print(f"GlooTransport.sendrecv failed: {e!r}", flush=True)
            return 1


class LocalTransport:
    """A one-rank transport (world 1): the all-gather is a copy.  With
    Context(peer=True) it runs the multi-rank code path of the peer transport
    on one process (the mailboxes are its own), e.g. to time that path."""

    def __init__(self):
        self.rank, self.world = 0, 1
        self._ag = ALLGATHER_FN(self._allgather)
        self._sr = SENDRECV_FN(lambda *a: 0)
        self.struct = HostComm(None, self._ag, self._sr)

    @staticmethod
    def _allgather(_user, send, recv, nbytes):
        ctypes.memmove(recv, send, nbytes)
        return 0
