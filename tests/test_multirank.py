"""Multi-rank particle filter.

CPU tests (gloo, world_size 2..4):
  * the product's exchange plan (gh_sys_plan, host code) against a brute-force
    systematic resampler over the global CDF;
  * the host transport callbacks (gen_amd.transport.GlooTransport) moving
    bytes between two processes;
  * the sharded oracle driven by the product's plan and real gloo messages
    reproduces the single-rank oracle bit for bit.
GPU test: 2 and 3 ranks sharing GPU 0 through the host transport reproduce
the single-rank oracle (states, weights, parents bit-exact; log-ML 1e-9).
"""
import ctypes
import os
import socket
import subprocess
import sys
from ctypes import POINTER, c_int64, c_uint64

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gen_amd import _lib  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def plan(n, R, q, totals, o):
    lib = _lib.load()
    tot = np.ascontiguousarray(totals, dtype=np.uint64)
    out = [np.zeros(R, dtype=np.int64) for _ in range(4)]
    _lib.check(lib.gh_sys_plan(n, R, q, tot.ctypes.data_as(POINTER(c_uint64)), int(o),
                               *[a.ctypes.data_as(POINTER(c_int64)) for a in out]))
    return out


def brute_source_rank(n, totals, o):
    """rank owning the ancestor of every global slot (systematic, global CDF)."""
    S = int(sum(int(t) for t in totals))
    bounds = np.cumsum([int(t) for t in totals])
    src = np.empty(n, dtype=np.int64)
    for j in range(n):
        T = (j * S + o) // n
        src[j] = int(np.searchsorted(bounds, T, side="right"))
    return src


@pytest.mark.parametrize("R", [2, 3, 5, 8])
def test_sys_plan_matches_bruteforce(R):
    rng = np.random.default_rng(R)
    for trial in range(30):
        n = int(rng.integers(R, 400))
        totals = rng.integers(0, 1 << 40, size=R).astype(np.uint64)
        if trial % 3 == 0:
            totals[rng.integers(0, R, size=R // 2 + 1)] = 0  # empty ranks
        if totals.sum() == 0:
            totals[0] = 7
        S = int(sum(int(t) for t in totals))
        o = int(rng.integers(0, S))
        src = brute_source_rank(n, totals, o)
        plans = [plan(n, R, q, totals, o) for q in range(R)]
        for q in range(R):
            slo, shi, rlo, rhi = plans[q]
            lo, hi = (n * q) // R, (n * (q + 1)) // R
            # every slot of q is received from exactly its source rank
            got = np.full(hi - lo, -1)
            for r in range(R):
                got[rlo[r] - lo : rhi[r] - lo] = r
            assert np.array_equal(got, src[lo:hi])
            for r in range(R):
                # what q sends to r is what r receives from q
                assert (slo[r], shi[r]) == (plans[r][2][q], plans[r][3][q])


def exchange_lists(n, R, q, totals, o, d):
    lib = _lib.load()
    tot = np.ascontiguousarray(totals, dtype=np.uint64)
    ns, nr = ctypes.c_int(), ctypes.c_int()
    sp, rp = np.zeros(R, dtype=np.int32), np.zeros(R, dtype=np.int32)
    sb, rb = np.zeros(R, dtype=np.uint64), np.zeros(R, dtype=np.uint64)
    i32 = POINTER(ctypes.c_int)
    _lib.check(lib.gh_debug_exchange_lists(
        n, R, q, tot.ctypes.data_as(POINTER(c_uint64)), int(o), d, ctypes.byref(ns),
        sp.ctypes.data_as(i32), sb.ctypes.data_as(POINTER(c_uint64)), ctypes.byref(nr), rp.ctypes.data_as(i32),
        rb.ctypes.data_as(POINTER(c_uint64))))
    return sp[: ns.value], sb[: ns.value], rp[: nr.value], rb[: nr.value]


@pytest.mark.parametrize("R", [2, 3, 5, 8])
def test_exchange_lists_pair_up(R):
    """The grouped messages both transports post (finish_plan's lists): every
    send of q to r is the receive of r from q with the same byte count, the
    rows are gh_sys_plan's slot ranges, no rank messages itself, and peers are
    in rank order on both sides (RCCL's grouped send/recv and the host
    transport's sendrecv take the lists as they are)."""
    rng = np.random.default_rng(100 + R)
    d = 4
    for trial in range(20):
        n = int(rng.integers(R, 5000))
        totals = rng.integers(0, 1 << 40, size=R).astype(np.uint64)
        if trial % 4 == 0:  # one rank holds (nearly) all the weight: it sends to everyone
            totals[:] = 0
            totals[rng.integers(0, R)] = 1 << 41
        if totals.sum() == 0:
            totals[0] = 7
        o = int(rng.integers(0, int(sum(int(t) for t in totals))))
        lists = [exchange_lists(n, R, q, totals, o, d) for q in range(R)]
        for q in range(R):
            sp, sb, rp, rb = lists[q]
            slo, shi, rlo, rhi = plan(n, R, q, totals, o)
            assert q not in sp and q not in rp
            assert list(sp) == sorted(sp) and list(rp) == sorted(rp)
            for peer, b in zip(sp, sb):
                assert b == (shi[peer] - slo[peer]) * (d + 1) * 8
                osp, osb, orp, orb = lists[peer]
                assert b == orb[list(orp).index(q)]
            for peer, b in zip(rp, rb):
                assert b == (rhi[peer] - rlo[peer]) * (d + 1) * 8
            assert len(rp) == sum(1 for r in range(R) if r != q and rhi[r] > rlo[r])


def test_sys_plan_rejects_bad_arguments():
    lib = _lib.load()
    tot = np.array([0, 0], dtype=np.uint64)
    z = np.zeros(2, dtype=np.int64)
    p = z.ctypes.data_as(POINTER(c_int64))
    rc = lib.gh_sys_plan(10, 2, 0, tot.ctypes.data_as(POINTER(c_uint64)), 0, p, p, p, p)
    assert rc == 1
    tot = np.array([5, 5], dtype=np.uint64)
    rc = lib.gh_sys_plan(10, 2, 2, tot.ctypes.data_as(POINTER(c_uint64)), 0, p, p, p, p)
    assert rc == 1


def _run_workers(script_args, world, timeout=300):
    env = dict(os.environ)
    env["MASTER_ADDR"] = "127.0.0.1"
    env["MASTER_PORT"] = str(_free_port())
    env["WORLD_SIZE"] = str(world)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable] + script_args, env=e, cwd=ROOT,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out.decode(errors="replace"))
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-4000:]
    return outs


_CPU_WORKER = r'''
import os, sys, ctypes
import numpy as np
import torch, torch.distributed as dist
sys.path.insert(0, os.environ["GH_ROOT"])
from gen_amd import _lib, LinearGaussianSSM
from gen_amd.transport import GlooTransport
from oracle import oracle as O
from tests.test_multirank import plan

dist.init_process_group("gloo")
rank, R = dist.get_rank(), dist.get_world_size()
out = os.environ["GH_OUT"]

# 1) transport callbacks through their C function pointers
tr = GlooTransport()
send = (ctypes.c_uint8 * 5)(*[rank * 10 + i for i in range(5)])
recv = (ctypes.c_uint8 * (5 * R))()
assert tr.struct.allgather(None, ctypes.addressof(send), ctypes.addressof(recv), 5) == 0
assert list(recv) == [r * 10 + i for r in range(R) for i in range(5)]
peers = [p for p in range(R) if p != rank]
sb = [(ctypes.c_uint8 * (3 + rank))(*([rank + 1] * (3 + rank))) for _ in peers]
rb = [(ctypes.c_uint8 * (3 + p))() for p in peers]
IA = ctypes.c_int * len(peers); VA = ctypes.c_void_p * len(peers); UA = ctypes.c_uint64 * len(peers)
rc = tr.struct.sendrecv(None, len(peers), IA(*peers), VA(*[ctypes.addressof(b) for b in sb]),
                        UA(*[3 + rank] * len(peers)), len(peers), IA(*peers),
                        VA(*[ctypes.addressof(b) for b in rb]), UA(*[3 + p for p in peers]))
assert rc == 0
for p, b in zip(peers, rb):
    assert list(b) == [p + 1] * (3 + p)

# 2) sharded oracle, routed by the product's plan over gloo
m = LinearGaussianSSM.benchmark(4)
_, ys = m.simulate(8, np.random.default_rng(5))
n, seed = 3001, 9
lo, hi = (n * rank) // R, (n * (rank + 1)) // R
pf = O.OraclePF(m, n, seed, lo=lo, n_local=hi - lo)
pf.init(ys[0])
for t, y in enumerate(ys[1:], start=1):
    st = torch.from_numpy(pf.local_stats())
    allst = [torch.empty(3, dtype=torch.float64) for _ in range(R)]
    dist.all_gather(allst, st)
    dec, L, ess, M = O.combine_stats(torch.cat(allst).numpy(), n, n)
    assert dec == 1
    tot = torch.tensor([pf.qtotal(M)], dtype=torch.int64)
    allt = [torch.empty(1, dtype=torch.int64) for _ in range(R)]
    dist.all_gather(allt, tot)
    totals = np.array([int(x.item()) for x in allt], dtype=np.uint64)
    S = int(sum(int(x) for x in totals))
    w = O.philox([0xFFFFFFFF, 0xFFFFFFFF, t, (3 << 16) | 0], [seed & 0xFFFFFFFF, seed >> 32])
    u = ((w[0] >> 5) << 26) | (w[1] >> 6)
    o = (u * S) >> 53
    slo, shi, rlo, rhi = plan(n, R, rank, totals, o)
    slots, ancs, sts = pf.emit(M, totals, rank)
    reqs, bufs = [], []
    for r in range(R):
        if r == rank:
            continue
        sel = (slots >= slo[r]) & (slots < shi[r])
        assert sel.sum() == shi[r] - slo[r]
        if sel.sum():
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(slots[sel])), r))
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(ancs[sel])), r))
            reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(sts[sel])), r))
        k = rhi[r] - rlo[r]
        if k:
            b = (torch.empty(k, dtype=torch.int64), torch.empty(k, dtype=torch.int64),
                 torch.empty((k, m.d), dtype=torch.float64))
            for x in b:
                reqs.append(dist.irecv(x, r))
            bufs.append(b)
    for q in reqs:
        q.wait()
    own = (slots >= lo) & (slots < hi)
    all_s = np.concatenate([slots[own]] + [b[0].numpy() for b in bufs])
    all_a = np.concatenate([ancs[own]] + [b[1].numpy() for b in bufs])
    all_x = np.concatenate([sts[own]] + [b[2].numpy() for b in bufs])
    assert np.array_equal(np.sort(all_s), np.arange(lo, hi))
    pf.apply(L, all_s, all_a, all_x)
    pf.step(y)
np.savez(f"{out}.rank{rank}.npz", states=pf.state(), parents=pf.parents())
dist.barrier()
dist.destroy_process_group()
'''


@pytest.mark.parametrize("R", [2, 3])
def test_gloo_sharded_oracle_with_product_plan(tmp_path, R):
    from gen_amd import LinearGaussianSSM
    from oracle import oracle as O

    script = tmp_path / "w.py"
    script.write_text(_CPU_WORKER)
    out = str(tmp_path / "o")
    os.environ["GH_ROOT"] = ROOT
    os.environ["GH_OUT"] = out
    try:
        _run_workers([str(script)], R, timeout=240)
    finally:
        os.environ.pop("GH_OUT", None)
    m = LinearGaussianSSM.benchmark(4)
    _, ys = m.simulate(8, np.random.default_rng(5))
    ref = O.run_pf(m, ys, 3001, 9, thr=3001)
    parts = [np.load(f"{out}.rank{r}.npz") for r in range(R)]
    assert np.array_equal(np.concatenate([p["states"] for p in parts], axis=1), ref.state())
    assert np.array_equal(np.concatenate([p["parents"] for p in parts]), ref.parents())


@pytest.mark.gpu
# thr: a number is passed through (0.0 never resamples: `ess < 0`); None is the
# reference's default N/2 (the worker passes no --thr)
@pytest.mark.parametrize("model,R,thr,n", [("lg4", 2, 3001.0, 3001), ("lg4", 3, None, 3001), ("kit", 2, None, 3001),
                                            ("kit", 2, 0.0, 3001), ("lg10", 2, 3001.0, 3001),
                                            ("lg4", 2, 1e9, 20011), ("kit", 4, 1e9, 4003),
                                            ("kit_sharp", 4, None, 4003), ("kit", 8, 1e9, 8003),
                                            ("lg4", 8, None, 8192)])
def test_gpu_multirank_host_transport_equals_single_rank(tmp_path, model, R, thr, n):
    """R ranks share GPU 0 through the gloo host transport; the gathered shards
    equal the single-rank oracle bit for bit (log-ML within 1e-9).  n = 20011
    spans several 4096-particle tiles per rank; R = 4 with the peaked
    Kitagawa weights moves rows across several ranks; kit_sharp (var_y = 0.01)
    puts nearly all the weight on one rank, whose rows overflow the bounded send
    buffer (2 n rows) and are written by the regrow path (k_rows_fill)."""
    from oracle import oracle as O
    from tests.mr_worker import build_model

    out = str(tmp_path / "g")
    T, seed = 8, 9
    _run_workers([os.path.join(ROOT, "tests", "mr_worker.py"), "--model", model, "--n", str(n), "--T", str(T),
                  *([] if thr is None else ["--thr", str(thr)]), "--seed", str(seed), "--out", out], R, timeout=400)
    m = build_model(model)
    _, ys = m.simulate(T, np.random.default_rng(5))
    ref = O.run_pf(m, ys, n, seed, thr=thr)
    parts = [np.load(f"{out}.rank{r}.npz") for r in range(R)]
    states = np.concatenate([p["states"] for p in parts], axis=0)  # [n, d]
    assert np.array_equal(states.T, ref.state())
    assert np.array_equal(np.concatenate([p["logw"] for p in parts]), ref.log_weights())
    assert np.array_equal(np.concatenate([p["parents"] for p in parts]), ref.parents())
    lml = float(parts[0]["lml"])
    assert all(float(p["lml"]) == lml for p in parts)
    assert abs(lml - ref.log_ml_estimate()) <= 1e-9 * abs(ref.log_ml_estimate())


def _check_against_oracle(out, model, R, n, T, seed, thr, resampler="systematic"):
    from oracle import oracle as O
    from tests.mr_worker import build_model

    m = build_model(model)
    _, ys = m.simulate(T, np.random.default_rng(5))
    ref = O.run_pf(m, ys, n, seed, thr=thr, resampler=O.MULTINOMIAL if resampler == "multinomial" else O.SYSTEMATIC)
    parts = [np.load(f"{out}.rank{r}.npz") for r in range(R)]
    states = np.concatenate([p["states"] for p in parts], axis=0)  # [n, d]
    assert np.array_equal(states.T, ref.state())
    assert np.array_equal(np.concatenate([p["logw"] for p in parts]), ref.log_weights())
    assert np.array_equal(np.concatenate([p["parents"] for p in parts]), ref.parents())
    lml = float(parts[0]["lml"])
    assert all(float(p["lml"]) == lml for p in parts)
    assert abs(lml - ref.log_ml_estimate()) <= 1e-9 * abs(ref.log_ml_estimate())


@pytest.mark.gpu
@pytest.mark.parametrize("model,R,thr,n", [("lg4", 2, None, 3001), ("lg4", 3, 1e9, 20011), ("kit", 2, None, 4096),
                                            ("kit", 4, 1e9, 8192), ("kit_sharp", 4, None, 4003),
                                            ("lg10", 2, 3001.0, 3001), ("kit", 8, 1e9, 16384),
                                            ("kit_sharp", 8, None, 8003)])
def test_gpu_multirank_batched_host_transport(tmp_path, model, R, thr, n):
    """The batched loop on R ranks (gh_pf_run: max-only steps whose maxima go to
    the atomic-max shards, the shards' all-gather, k_rank_a2's quantisation +
    sums, the records' all-gather, k_rank_b's decision; the Kitagawa ranks
    whose first particle is a multiple of 128 step with the pair kernel, split
    around the row exchange) equals the single-rank oracle bit for bit."""
    out = str(tmp_path / "b")
    T, seed = 8, 9
    _run_workers([os.path.join(ROOT, "tests", "mr_worker.py"), "--model", model, "--n", str(n), "--T", str(T),
                  *([] if thr is None else ["--thr", str(thr)]), "--seed", str(seed), "--batched", "--out", out], R,
                 timeout=400)
    _check_against_oracle(out, model, R, n, T, seed, thr)


@pytest.mark.gpu
@pytest.mark.parametrize("model,thr,n,batched", [("lg4", None, 20011, False), ("lg4", None, 20011, True),
                                                  ("lg10", 1e9, 9000, True), ("kit", None, 8192, True),
                                                  ("kit", 1e9, 8192, False), ("kit_sharp", None, 4003, True)])
def test_gpu_multirank_path_over_rccl_one_rank(tmp_path, model, thr, n, batched):
    """gh_ctx_force_multirank: one rank on the multi-rank code path over a
    one-rank RCCL communicator (ncclAllGather of the triples / shards / records,
    k_rank_a or k_rank_a2, k_rank_b, the split step) equals the single-rank
    oracle bit for bit.  (A one-rank exchange sends no rows: the grouped
    send/recv is exercised by the 2..4-rank host-transport tests.)"""
    out = str(tmp_path / "r")
    T, seed = 8, 9
    _run_workers([os.path.join(ROOT, "tests", "mr_worker.py"), "--model", model, "--n", str(n), "--T", str(T),
                  *([] if thr is None else ["--thr", str(thr)]), "--seed", str(seed), "--transport", "rccl1",
                  "--device", "0", *(["--batched"] if batched else []), "--out", out], 1, timeout=300)
    _check_against_oracle(out, model, 1, n, T, seed, thr)


@pytest.mark.gpu
@pytest.mark.parametrize("model,R,thr,n,batched", [("lg4", 2, None, 3001, True), ("lg4", 3, 1e9, 20011, True),
                                                    ("kit", 2, None, 4096, True), ("kit", 4, 1e9, 8192, True),
                                                    ("kit_sharp", 4, None, 4003, True), ("lg10", 2, 3001.0, 3001, True),
                                                    ("lg4", 2, None, 3001, False), ("kit", 3, 1e9, 4003, False),
                                                    ("kit", 8, 1e9, 8192, True), ("lg4", 8, None, 4096, False)])
def test_gpu_multirank_peer_transport(tmp_path, model, R, thr, n, batched):
    """The peer transport (gh_ctx_create_peer): R processes share GPU 0, map
    each other's mailboxes and row buffers by IPC handle (swapped once over
    gloo), and exchange the rank maxima, the records and the state rows with
    device stores and tagged words — k_rank_a2 / k_rank_b / k_peer_* inside
    the step loop, no host collective.  The gathered shards equal the
    single-rank oracle bit for bit (log-ML 1e-9), batched (gh_pf_run) and
    call by call (the small all-gathers through k_peer_allgather)."""
    out = str(tmp_path / "p")
    T, seed = 8, 9
    _run_workers([os.path.join(ROOT, "tests", "mr_worker.py"), "--model", model, "--n", str(n), "--T", str(T),
                  *([] if thr is None else ["--thr", str(thr)]), "--seed", str(seed), "--transport", "peer",
                  *(["--batched"] if batched else []), "--out", out], R, timeout=400)
    _check_against_oracle(out, model, R, n, T, seed, thr)


@pytest.mark.gpu
@pytest.mark.parametrize("transport,model,R,thr,n,batched", [
    ("gloo", "lg4", 2, None, 3001, False), ("gloo", "kit", 3, 1e9, 4003, False), ("gloo", "kit_sharp", 4, None, 4003, True),
    ("gloo", "lg10", 2, 3001.0, 3001, True), ("rccl1", "lg4", 1, 1e9, 3001, False),
    ("peer", "lg4", 2, None, 3001, False), ("peer", "kit", 3, 1e9, 4003, True), ("peer", "kit_sharp", 4, None, 4003, True),
    ("gloo", "kit", 8, 1e9, 8003, True), ("peer", "count", 3, 1e9, 4003, False)])
def test_gpu_multirank_multinomial(tmp_path, gh_ctx, transport, model, R, thr, n, batched):
    """Multinomial resampling (the reference's own resampler, Categorical draws
    per slot, particle_filter.jl:200) on R ranks: every rank evaluates the
    targets of all slots, the rank holding a slot's target sends that slot's
    ancestor row to its owner, both ordering by slot.  States, weights, parents
    and the genealogy queries equal the single-rank multinomial oracle bit for
    bit (log-ML 1e-9), call by call and batched."""
    out = str(tmp_path / "mn")
    T, seed = 8, 9
    _run_workers([os.path.join(ROOT, "tests", "mr_worker.py"), "--model", model, "--n", str(n), "--T", str(T),
                  *([] if thr is None else ["--thr", str(thr)]), "--seed", str(seed), "--transport", transport,
                  *(["--device", "0"] if transport == "rccl1" else []), *(["--batched"] if batched else []),
                  "--resampler", "multinomial", "--genealogy", "--out", out], R, timeout=400)
    _check_against_oracle(out, model, R, n, T, seed, thr, resampler="multinomial")
    _check_genealogy(out, model, R, n, T, seed, thr, batched, resampler="multinomial")


@pytest.mark.gpu
@pytest.mark.parametrize("transport,model,R,thr,n", [("gloo", "lg4", 2, None, 3001), ("gloo", "kit", 3, 1e9, 4003),
                                                      ("rccl1", "lg4", 1, 1e9, 3001), ("peer", "lg4", 2, None, 3001),
                                                      ("peer", "kit", 3, 1e9, 4003), ("peer", "count", 2, None, 3001)])
def test_gpu_multirank_conditional_smc(tmp_path, transport, model, R, thr, n):
    """Conditional SMC (examples/pmmh/smc.jl:100-151) on R ranks: particle 0
    (rank 0's first) is pinned to the reference and is its own parent, the
    others resample multinomially across ranks; states, weights, parents and
    the trajectories equal the single-rank oracle's conditional run bit for bit."""
    from oracle import oracle as O
    from tests.mr_worker import build_model

    out = str(tmp_path / "cs")
    T, seed = 8, 9
    _run_workers([os.path.join(ROOT, "tests", "mr_worker.py"), "--model", model, "--n", str(n), "--T", str(T),
                  *([] if thr is None else ["--thr", str(thr)]), "--seed", str(seed), "--transport", transport,
                  *(["--device", "0"] if transport == "rccl1" else []), "--csmc", "--genealogy", "--out", out], R,
                 timeout=400)
    m = build_model(model)
    xs, ys = m.simulate(T, np.random.default_rng(5))
    ref_traj = np.asarray(xs, dtype=np.float64).reshape(len(ys), -1) * 0.9
    orc = O.run_csmc(m, ys, n, seed, ref_traj, thr=thr)
    parts = [np.load(f"{out}.rank{r}.npz") for r in range(R)]
    states = np.concatenate([p["states"] for p in parts], axis=0)
    assert np.array_equal(states.T.view(np.uint64), orc.state().view(np.uint64))
    assert np.array_equal(np.concatenate([p["logw"] for p in parts]).view(np.uint64), orc.log_weights().view(np.uint64))
    assert np.array_equal(np.concatenate([p["parents"] for p in parts]), orc.parents())
    lml = float(parts[0]["lml"])
    assert abs(lml - orc.log_ml_estimate()) <= 1e-9 * abs(orc.log_ml_estimate())
    for t in sorted({1, min(5, T), T}):
        got = np.concatenate([p[f"traj{t}"] for p in parts], axis=0)
        assert np.array_equal(got.T.view(np.uint64), orc.trajectory(t).view(np.uint64)), t
        assert np.array_equal(got[0], ref_traj[t - 1]), t  # the distinguished particle's line is the reference


def _check_genealogy(out, model, R, n, T, seed, thr, batched, resampler="systematic"):
    """Trajectories at t = 1, 5, T and the score columns of the gathered shards
    equal the single-rank oracle bit for bit; the 500 sample_unweighted_traces
    indices equal a one-rank GPU filter's (the same global integer CDF)."""
    import gen_amd as gen
    from oracle import oracle as O
    from tests.mr_worker import build_model, obs_at

    m = build_model(model)
    _, ys = m.simulate(T, np.random.default_rng(5))
    ref = O.run_pf(m, ys, n, seed, thr=thr, resampler=O.MULTINOMIAL if resampler == "multinomial" else O.SYSTEMATIC)
    parts = [np.load(f"{out}.rank{r}.npz") for r in range(R)]
    for t in sorted({1, min(5, T), T}):
        got = np.concatenate([p[f"traj{t}"] for p in parts], axis=0)  # [n, d]
        assert np.array_equal(got.T.view(np.uint64), ref.trajectory(t).view(np.uint64)), t
    rtot, rps = ref.scores(per_step=True)
    assert np.array_equal(np.concatenate([p["score_tot"] for p in parts]).view(np.uint64), rtot.view(np.uint64))
    assert np.array_equal(np.concatenate([p["score_ps"] for p in parts], axis=2).view(np.uint64), rps.view(np.uint64))
    # the same filter on one rank of this process's GPU
    st = gen.initialize_particle_filter(m, (1,), obs_at(m, ys[0], 1), n, seed=seed, resampler=resampler)
    if batched:
        gen.run_particle_filter(st, list(ys[1:T]), thr)
    else:
        for t in range(2, T + 1):
            gen.maybe_resample(st, thr)
            gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), obs_at(m, ys[t - 1], t))
    _, idx = gen.sample_unweighted_traces(st, 500, seed=3)
    st.close()
    for p in parts:
        assert np.array_equal(p["samp"], idx)


@pytest.mark.gpu
@pytest.mark.parametrize("transport,model,R,thr,n,batched", [
    ("gloo", "lg4", 2, None, 3001, False), ("gloo", "kit", 3, 1e9, 4003, True), ("gloo", "kit_sharp", 3, None, 4003, True),
    ("peer", "lg4", 2, 1e9, 3001, True), ("peer", "kit", 3, None, 4096, True), ("peer", "lg10", 2, 3001.0, 3001, False),
    ("rccl1", "lg4", 1, None, 3001, True), ("gloo", "kit", 2, 1e9, 3001, "mid"), ("peer", "lg4", 3, 1e9, 3001, "mid"),
    ("peer", "count", 3, None, 4003, True), ("gloo", "count", 2, 1e9, 3001, False), ("rccl1", "count", 1, 1e9, 3001, True),
    ("peer", "switch", 3, 1e9, 4003, False), ("peer", "slds", 2, 1e9, 3001, True), ("gloo", "deps", 2, None, 3001, False)])
def test_gpu_multirank_genealogy(tmp_path, gh_ctx, transport, model, R, thr, n, batched):
    """The genealogy across ranks (get_traces at earlier steps, the trace score
    columns, sample_unweighted_traces; particle_filter.jl:31-34, 62-70): each
    rank keeps its slots' ancestors and the rows it received, and the queries
    walk them collectively — against the single-rank oracle bit for bit.
    "mid": queries between maybe_resample and the step at t = 4 too (that
    step then reads materialised ancestors that name received rows)."""
    out = str(tmp_path / "gen")
    T, seed = 8, 9
    mid = batched == "mid"
    batched = batched is True
    _run_workers([os.path.join(ROOT, "tests", "mr_worker.py"), "--model", model, "--n", str(n), "--T", str(T),
                  *([] if thr is None else ["--thr", str(thr)]), "--seed", str(seed), "--transport", transport,
                  *(["--device", "0"] if transport == "rccl1" else []), *(["--batched"] if batched else []),
                  *(["--mid-query"] if mid else []), "--genealogy", "--out", out], R, timeout=400)
    _check_against_oracle(out, model, R, n, T, seed, thr)
    _check_genealogy(out, model, R, n, T, seed, thr, batched)


@pytest.mark.gpu
@pytest.mark.parametrize("R,sleep,timeout", [(2, "1:4:4.0", None), (3, "0:3:3.5", 60.0)])
def test_gpu_multirank_peer_slow_rank(tmp_path, R, sleep, timeout):
    """Peer transport, a slow rank: one rank sleeps seconds (longer than the
    round-5 bound of ~2.5 s of polls) before a call-by-call step while the
    others' kernels wait on the device for its maxima and rows.  The device
    waits are bounded in time (30 s by default, gh_ctx_set_peer_timeout), so
    they wait for it and the filter finishes bit-exact against the oracle."""
    out = str(tmp_path / "slow")
    model, n, T, seed, thr = "kit", 4003, 6, 9, 1e9
    _run_workers([os.path.join(ROOT, "tests", "mr_worker.py"), "--model", model, "--n", str(n), "--T", str(T),
                  "--thr", str(thr), "--seed", str(seed), "--transport", "peer", "--sleep", sleep,
                  *([] if timeout is None else ["--peer-timeout", str(timeout)]), "--out", out], R, timeout=300)
    _check_against_oracle(out, model, R, n, T, seed, thr)


@pytest.mark.gpu
@pytest.mark.parametrize("transport,R,value", [("gloo", 2, 3001 // 2 + 7), ("gloo", 2, -1_000_000), ("rccl1", 1, 5000),
                                               ("peer", 2, -1_000_000)])
def test_gpu_multirank_broken_genealogy_raises(tmp_path, gh_ctx, transport, R, value):
    """A genealogy walk that meets a broken record (an ancestor index outside
    the rank's particles, or a received row that was never kept) raises
    GH_E_STATE through the filter's device error word — the collective
    trajectory and score queries fail on the rank whose walk broke instead of
    returning NaN or another particle's trajectory."""
    out = str(tmp_path / "bad")
    n, T = 3001, 6
    _run_workers([os.path.join(ROOT, "tests", "mr_worker.py"), "--model", "lg4", "--n", str(n), "--T", str(T),
                  "--thr", "1e9", "--seed", "9", "--transport", transport,
                  *(["--device", "0"] if transport == "rccl1" else []), "--corrupt", str(value), "--out", out], R,
                 timeout=300)
    r0 = np.load(f"{out}.rank0.npz")
    for q in ("traj", "scores"):
        msg = str(r0[f"err_{q}"])
        assert msg.startswith("GenHipError: GH_E_STATE") and "genealogy" in msg, (q, msg)


@pytest.mark.gpu
@pytest.mark.parametrize("transport,model,R", [("gloo", "lg4", 2), ("peer", "kit", 3), ("peer", "count", 2)])
def test_gpu_multirank_step_params(tmp_path, transport, model, R):
    """particle_filter_step with changed Unfold parameters on R ranks
    (gh_pf_step_params: every particle re-scored along its genealogy, which
    crosses ranks) equals the single-rank oracle's orc_pf_step_params run bit
    for bit, and later steps under the new parameters too."""
    from oracle import oracle as O
    from tests.mr_worker import build_model, changed_model

    out = str(tmp_path / "sp")
    T, seed, n, K = 8, 9, 3001, 5
    _run_workers([os.path.join(ROOT, "tests", "mr_worker.py"), "--model", model, "--n", str(n), "--T", str(T),
                  "--seed", str(seed), "--transport", transport, "--params-step", str(K), "--out", out], R,
                 timeout=400)
    m, m2 = build_model(model), changed_model(model)
    _, ys = m.simulate(T, np.random.default_rng(5))
    orc = O.OraclePF(m, n, seed, O.SYSTEMATIC)
    orc.init(ys[0])
    for t in range(2, T + 1):
        orc.maybe_resample(None)
        if t == K:
            orc.step_params(m2, ys[t - 1])
        else:
            orc.step(ys[t - 1])
    parts = [np.load(f"{out}.rank{r}.npz") for r in range(R)]
    assert np.array_equal(np.concatenate([p["states"] for p in parts], axis=0).T.view(np.uint64),
                          orc.state().view(np.uint64))
    assert np.array_equal(np.concatenate([p["logw"] for p in parts]).view(np.uint64), orc.log_weights().view(np.uint64))
    assert np.array_equal(np.concatenate([p["parents"] for p in parts]), orc.parents())
    lml = float(parts[0]["lml"])
    assert abs(lml - orc.log_ml_estimate()) <= 1e-9 * abs(orc.log_ml_estimate())
