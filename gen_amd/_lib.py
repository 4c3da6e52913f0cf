"""ctypes binding of libgen_hip.so (the C ABI in include/gen_hip.h).

The product path has no fallback: if the HIP library is missing, importing
the binding raises.  Nothing here imports or calls the CPU oracle.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_uint8, c_uint32, c_uint64, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GEN_HIP_LIB") or os.path.join(HERE, "libgen_hip.so")

GH_OK = 0
STATUS = {
    1: "GH_E_INVAL",
    2: "GH_E_DISCARD",
    3: "GH_E_NUMERIC",
    4: "GH_E_NOMEM",
    5: "GH_E_HIP",
    6: "GH_E_RCCL",
    7: "GH_E_STATE",
}

FAMILY_LGSSM, FAMILY_HMM, FAMILY_KITAGAWA, FAMILY_REGRESSION, FAMILY_SLOTS = 1, 2, 3, 4, 5
SLOT_INPUT = -1  # gh_obs.slot of a step's latent input (GH_SLOT_INPUT)
RESAMPLE_SYSTEMATIC, RESAMPLE_MULTINOMIAL = 0, 1
PROPOSAL_DEFAULT, PROPOSAL_OPTIMAL, PROPOSAL_GAUSSIAN, PROPOSAL_LINEAR = 0, 1, 2, 3


class GenHipError(RuntimeError):
    """Raised for a non-zero gh_status (the reference raises `error(...)`)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code


class ModelDesc(ctypes.Structure):
    _fields_ = [
        ("family", c_int32),
        ("d", c_int32),
        ("dy", c_int32),
        ("k", c_int32),
        ("v", c_int32),
        ("params", POINTER(c_double)),
        ("n_params", c_int64),
    ]


class Obs(ctypes.Structure):
    pass


Obs._fields_ = [("values", POINTER(c_double)), ("n_values", c_int32), ("present", c_int32), ("slot", c_int32),
                ("reserved", c_int32), ("next", POINTER(Obs))]


class PFOpts(ctypes.Structure):
    _fields_ = [
        ("resampler", c_int32),
        ("record_history", c_int32),
        ("history_capacity", c_int32),
        ("block_size", c_int32),
        ("time_kernels", c_int32),
        ("reserved", c_int32 * 3),
    ]


# name -> (restype, argtypes); restype int means a gh_status
SIGNATURES = {
    "gh_ctx_create": (c_int, [c_int, c_void_p, POINTER(c_void_p)]),
    "gh_comm_unique_id": (c_int, [POINTER(c_uint8)]),
    "gh_ctx_create_dist": (c_int, [c_int, c_int, c_int, POINTER(c_uint8), c_void_p, POINTER(c_void_p)]),
    "gh_ctx_create_hostcomm": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, POINTER(c_void_p)]),
    "gh_ctx_create_peer": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p, POINTER(c_void_p)]),
    "gh_ctx_destroy": (c_int, [c_void_p]),
    "gh_ctx_force_multirank": (c_int, [c_void_p]),
    "gh_pf_step_params": (c_int, [c_void_p, POINTER(Obs), c_int, c_void_p]),
    "gh_pf_step_params_conditional": (c_int, [c_void_p, POINTER(Obs), c_void_p, POINTER(c_double)]),
    "gh_ctx_rank": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int)]),
    "gh_ctx_stream": (c_int, [c_void_p, POINTER(c_void_p)]),
    "gh_ctx_synchronize": (c_int, [c_void_p]),
    "gh_model_create": (c_int, [c_void_p, POINTER(ModelDesc), POINTER(c_void_p)]),
    "gh_model_destroy": (c_int, [c_void_p]),
    "gh_model_state_dim": (c_int, [c_void_p, POINTER(c_int)]),
    "gh_pf_opts_default": (None, [POINTER(PFOpts)]),
    "gh_pf_init": (c_int, [c_void_p, POINTER(Obs), c_int, c_int64, c_uint64, POINTER(PFOpts), POINTER(c_void_p)]),
    "gh_pf_destroy": (c_int, [c_void_p]),
    "gh_pf_step": (c_int, [c_void_p, POINTER(Obs), c_int]),
    "gh_pf_init_q": (c_int, [c_void_p, POINTER(Obs), c_int, POINTER(c_double), c_int, c_int64, c_uint64,
                             POINTER(PFOpts), POINTER(c_void_p)]),
    "gh_pf_step_q": (c_int, [c_void_p, POINTER(Obs), c_int, POINTER(c_double), c_int]),
    "gh_pf_maybe_resample": (c_int, [c_void_p, c_double, POINTER(c_int), POINTER(c_double)]),
    "gh_pf_run": (c_int, [c_void_p, c_int, POINTER(Obs), c_int, c_double]),
    "gh_pf_log_ml_estimate": (c_int, [c_void_p, POINTER(c_double)]),
    "gh_pf_num_particles": (c_int, [c_void_p, POINTER(c_int64), POINTER(c_int64), POINTER(c_int64)]),
    "gh_pf_num_steps": (c_int, [c_void_p, POINTER(c_int)]),
    "gh_pf_get_log_weights": (c_int, [c_void_p, POINTER(c_double)]),
    "gh_pf_get_states": (c_int, [c_void_p, POINTER(c_double)]),
    "gh_pf_get_parents": (c_int, [c_void_p, POINTER(c_int64)]),
    "gh_pf_get_trajectory": (c_int, [c_void_p, c_int, POINTER(c_double)]),
    "gh_pf_sample_unweighted": (c_int, [c_void_p, c_int64, c_uint64, POINTER(c_int64)]),
    "gh_pf_rejuvenate": (c_int, [c_void_p, c_int, POINTER(c_int64)]),
    "gh_pf_mh_select": (c_int, [c_void_p, ctypes.c_uint32, c_int, POINTER(c_int64)]),
    "gh_pf_mh_drift": (c_int, [c_void_p, ctypes.c_uint32, POINTER(c_double), c_int, POINTER(c_int64)]),
    "gh_pf_get_scores": (c_int, [c_void_p, POINTER(c_double), POINTER(c_double)]),
    "gh_debug_mark_bits": (c_int, [c_void_p, c_int]),
    "gh_debug_count_window": (c_int, [c_void_p, c_int]),
    "gh_debug_set_ancestor": (c_int, [c_void_p, c_int, c_int64, c_int32]),
    "gh_ctx_set_peer_timeout": (c_int, [c_void_p, c_double]),
    "gh_debug_exchange_lists": (c_int, [c_int64, c_int, c_int, POINTER(c_uint64), c_uint64, c_int, POINTER(c_int),
                                        POINTER(c_int), POINTER(c_uint64), POINTER(c_int), POINTER(c_int),
                                        POINTER(c_uint64)]),
    "gh_dist_logpdf": (c_int, [c_void_p, c_void_p, c_int64, POINTER(c_double), POINTER(c_double)]),
    "gh_dist_random": (c_int, [c_void_p, c_void_p, c_int64, c_uint64, POINTER(c_double)]),
    "gh_dist_logpdf_dev": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "gh_dist_random_dev": (c_int, [c_void_p, c_void_p, c_int64, c_uint64, c_void_p]),
    "gh_simulate": (c_int, [c_void_p, c_int, c_int64, c_uint64, POINTER(c_double), POINTER(c_double),
                            POINTER(c_double), POINTER(c_double)]),
    "gh_simulate_inputs": (c_int, [c_void_p, c_int, c_int64, c_uint64, POINTER(c_double), POINTER(c_double),
                                   POINTER(c_double), POINTER(c_double), POINTER(c_double)]),
    "gh_pf_init_conditional": (c_int, [c_void_p, POINTER(Obs), c_int64, c_uint64, POINTER(PFOpts), POINTER(c_double),
                                       POINTER(c_void_p)]),
    "gh_pf_step_conditional": (c_int, [c_void_p, POINTER(Obs), POINTER(c_double)]),
    "gh_pf_get_ess_history": (c_int, [c_void_p, c_int, POINTER(c_double), POINTER(c_int32)]),
    "gh_pf_kernel_time": (c_int, [c_void_p, POINTER(c_double), POINTER(c_int64), c_int]),
    "gh_sys_plan": (c_int, [c_int64, c_int, c_int, POINTER(c_uint64), c_uint64, POINTER(c_int64), POINTER(c_int64), POINTER(c_int64), POINTER(c_int64)]),
    "gh_pmmh_run": (c_int, [c_void_p, c_int64, c_int64, c_int, POINTER(c_double), c_int, c_int, c_int, c_uint64, c_int,
                            POINTER(c_double), POINTER(c_double), POINTER(c_double), POINTER(c_int32),
                            POINTER(c_double), POINTER(c_double)]),
    "gh_coal_run": (c_int, [c_void_p, c_int64, c_int64, POINTER(c_double), c_int, c_int, c_int, c_uint64, c_int,
                            POINTER(c_double), POINTER(c_int32), POINTER(c_int32), POINTER(c_double)]),
    "gh_coal_create": (c_int, [c_void_p, c_int64, c_int64, POINTER(c_double), c_int, c_uint64, POINTER(c_void_p)]),
    "gh_coal_set_kernel": (c_int, [c_void_p, c_int]),
    "gh_coal_step": (c_int, [c_void_p, c_int, POINTER(c_int32), POINTER(c_int32), POINTER(c_double)]),
    "gh_coal_read_state": (c_int, [c_void_p, POINTER(c_double)]),
    "gh_coal_write_state": (c_int, [c_void_p, POINTER(c_double), c_int]),
    "gh_coal_destroy": (c_int, [c_void_p]),
    "gh_is_run": (c_int, [c_void_p, POINTER(Obs), c_int, c_int64, c_uint64, POINTER(c_double), POINTER(c_double), POINTER(c_double)]),
    "gh_last_error": (c_char_p, []),
    "gh_version": (c_char_p, []),
    "gh_selftest_math": (c_int, [c_void_p, c_int64, POINTER(c_double), POINTER(c_double), POINTER(c_double), POINTER(c_double), POINTER(c_double)]),
    "gh_selftest_boxmuller": (c_int, [c_void_p, c_int64, POINTER(ctypes.c_uint32), POINTER(c_double)]),
    "gh_selftest_normals": (c_int, [c_void_p, c_uint64, c_int64, c_uint32, c_uint32, c_int, POINTER(c_double)]),
}

_LIB = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libgen_hip.so and declare every C-ABI symbol; raises if absent."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise ImportError(
            f"libgen_hip.so not found at {path}: build it with `python -m gen_amd.build` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback."
        )
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        if name.startswith("gh_debug_") and not hasattr(lib, name):
            continue  # (test hooks: an older library built for an A/B run may lack one)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def check(rc: int) -> None:
    if rc != GH_OK:
        msg = load().gh_last_error()
        raise GenHipError(rc, msg.decode() if msg else "")


def dptr(a):
    """POINTER(c_double) to a C-contiguous float64 numpy array (or None)."""
    if a is None:
        return None
    return a.ctypes.data_as(POINTER(c_double))
