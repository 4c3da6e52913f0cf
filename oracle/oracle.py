"""ctypes wrapper of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker.  Never imported by gen_amd/.
See gh_oracle.h for what the oracle restates (reference file:line) and how
it is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_double, c_int, c_int32, c_int64, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
OMP_PATH = os.path.join(HERE, "liboracle_omp.so")  # the same oracle on every host core (CPU baseline only)

LGSSM, HMM, KITAGAWA, REGRESSION, SLOTS = 1, 2, 3, 4, 5
SYSTEMATIC, MULTINOMIAL = 0, 1
DEFAULT, OPTIMAL, GAUSSIAN, LINEAR = 0, 1, 2, 3

_lib = None
_libs = {}
_use_omp = False


def build(force: bool = False, target: str = "liboracle.so") -> str:
    src = os.path.join(HERE, "gh_oracle.c")
    path = os.path.join(HERE, target)
    if force or not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", HERE] + (["-B"] if force else []) + [target], check=True)
    return path


def set_openmp(on: bool) -> None:
    """Route the module's calls (and OraclePFs created afterwards) to the
    OpenMP build (all host cores) or back to the scalar build."""
    global _lib, _use_omp
    _use_omp = bool(on)
    _lib = None


def num_threads() -> int:
    return lib().orc_num_threads()


def lib():
    global _lib
    if _lib is None:
        target = "liboracle_omp.so" if _use_omp else "liboracle.so"
        if target not in _libs:
            _libs[target] = _load(build(target=target))
        _lib = _libs[target]
    return _lib


def _load(path):
    if True:
        L = ctypes.CDLL(path)
        D, I, I64, U64, U32, V = POINTER(c_double), c_int, c_int64, c_uint64, c_uint32, c_void_p
        sig = {
            "orc_philox4x32_10": (None, [POINTER(c_uint32), POINTER(c_uint32), POINTER(c_uint32)]),
            "orc_exp": (c_double, [c_double]),
            "orc_log": (c_double, [c_double]),
            "orc_log_unit": (c_double, [c_double]),
            "orc_cos": (c_double, [c_double]),
            "orc_sincos_2pi": (None, [c_double, D, D]),
            "orc_sincos_2pi_u32": (None, [U32, D, D]),
            "orc_box_muller": (None, [U32, U32, U32, D, D]),
            "orc_normals": (None, [U64, U64, U32, U32, I, D]),
            "orc_pf_create": (V, [I, I, I, I, I, D, I64, I64, I64, I64, U64, I, I]),
            "orc_pf_destroy": (None, [V]),
            "orc_pf_init": (I, [V, D, I, I]),
            "orc_pf_step": (I, [V, D, I, I]),
            "orc_pf_set_proposal_args": (I, [V, D, I]),
            "orc_pf_maybe_resample": (I, [V, c_double, D]),
            "orc_pf_rejuvenate": (I, [V, I, POINTER(c_int64)]),
            "orc_pf_mh_select": (I, [V, U32, I, POINTER(c_int64)]),
            "orc_pf_mh_drift": (I, [V, U32, D, I, POINTER(c_int64)]),
            "orc_pf_init_conditional": (I, [V, D, I, D]),
            "orc_pf_step_conditional": (I, [V, D, I, D]),
            "orc_pf_log_ml_estimate": (c_double, [V]),
            "orc_pf_get_log_weights": (None, [V, D]),
            "orc_pf_get_state": (None, [V, D]),
            "orc_pf_get_parents": (None, [V, POINTER(c_int64)]),
            "orc_pf_num_steps": (I, [V]),
            "orc_pf_get_history": (I, [V, I, D, POINTER(c_int32), POINTER(c_int)]),
            "orc_pf_get_scores": (I, [V, D, D]),
            "orc_pf_step_params": (I, [V, D, I64, D, I, I]),
            "orc_lgamma": (c_double, [c_double]),
            "orc_log1p": (c_double, [c_double]),
            "orc_dist_logpdf": (I, [I, I, I, I, D, I64, D, D]),
            "orc_dist_random": (I, [I, I, I, I, D, I64, U64, D]),
            "orc_simulate": (I, [I, I, I, I, I, D, I64, I, I64, U64, D, D, D, D]),
            "orc_simulate_inputs": (I, [I, I, I, I, I, D, I64, I, I64, U64, D, D, D, D, D]),
            "orc_pf_local_stats": (None, [V, D]),
            "orc_combine_stats": (I, [D, I, I64, c_double, D, D, D]),
            "orc_pf_local_qtotal": (U64, [V, c_double]),
            "orc_pf_resample_emit": (I64, [V, c_double, POINTER(c_uint64), I, I, POINTER(c_int64), POINTER(c_int64), D]),
            "orc_pf_resample_apply": (None, [V, c_double, I64, POINTER(c_int64), POINTER(c_int64), D]),
            "orc_importance_sampling": (I, [I, I, I, I, I, D, I64, D, I, I, I64, U64, D, D, D]),
            "orc_normal_logpdf": (c_double, [c_double, c_double, c_double]),
            "orc_pmmh_run": (I, [I64, I64, I, D, I, I, I, U64, I, D, D, D, POINTER(ctypes.c_int32), D]),
            "orc_coal_run": (I, [I64, I64, D, I, I, I, U64, I, D, POINTER(ctypes.c_int32), POINTER(ctypes.c_int32), I]),
            "orc_coal_regen_k": (c_double, [D, D, I, D, D]),
            "orc_coal_score": (c_double, [D, D, I]),
            "orc_coal_propose": (c_double, [D, D, I, I, D, D]),
            "orc_pmmh_loglik": (c_double, [U64, U64, U32, c_double, c_double, I, D, I]),
        }
        sig["orc_num_threads"] = (I, [])
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
    return L


def _d(a):
    return None if a is None else a.ctypes.data_as(POINTER(c_double))


def philox(ctr, key):
    c = (c_uint32 * 4)(*ctr)
    k = (c_uint32 * 2)(*key)
    o = (c_uint32 * 4)()
    lib().orc_philox4x32_10(c, k, o)
    return list(o)


def box_muller_words(words):
    """[n, 3] uint32 words -> [n, 2] normals (the oracle's Box–Muller)."""
    out = np.empty((len(words), 2))
    a, b = c_double(), c_double()
    f = lib().orc_box_muller
    for i, (x, y, z) in enumerate(np.asarray(words, dtype=np.uint64)):
        f(int(x), int(y), int(z), ctypes.byref(a), ctypes.byref(b))
        out[i] = a.value, b.value
    return out


def normals(seed, id_, step, stream, n):
    z = np.empty(n)
    lib().orc_normals(seed, id_, step, stream, n, _d(z))
    return z


def model_args(model):
    """(family, d, dy, k, v, params) from a gen_amd.models.Model (duck-typed)."""
    p = np.ascontiguousarray(model.params(), dtype=np.float64)
    return model.family, model.d, model.dy, model.k, model.v, p


def slot_obs(model, value):
    """A slot model's observation (a {slot name: value} dict) as the oracle
    takes it (gh_oracle.h ORC_SLOTS): the slots' values in slot order (m for
    an mvnormal slot, one otherwise) and the bitmask of the present slots; a
    "__input__" entry is the step's latent input (bit 4, d values after them)."""
    vals = value if isinstance(value, dict) else {model.names[0]: value}
    vec = np.zeros(max(1, model.dy) + model.d)
    mask, row = 0, 0
    for k, s in enumerate(model.slots):
        rows = s["m"] if s["dist"] == "mvnormal" else 1
        if vals.get(s["name"]) is not None:
            vec[row:row + rows] = np.atleast_1d(np.asarray(vals[s["name"]], dtype=np.float64)).ravel()
            mask |= 1 << k
        row += rows
    if vals.get("__input__") is not None:  # a model with per-step inputs: u_t after the dy values, bit 4
        vec[model.dy:model.dy + model.d] = np.asarray(vals["__input__"], dtype=np.float64).reshape(model.d)
        mask |= 1 << 4
    return vec, mask


class OraclePF:
    """CPU restatement of ParticleFilterState over particles [lo, lo+n_local)."""

    def __init__(self, model, n_global, seed, resampler=SYSTEMATIC, lo=0, n_local=None, record_history=True):
        fam, d, dy, k, v, p = model_args(model)
        self.L = lib()
        self._p = p
        self.d = d if fam in (LGSSM, REGRESSION, SLOTS) else 1
        self.n_global = n_global
        self.lo = lo
        self.n = n_global if n_local is None else n_local
        self.h = self.L.orc_pf_create(fam, d, dy, k, v, _d(p), p.size, n_global, lo, self.n, seed, resampler,
                                     int(record_history))
        if not self.h:
            raise ValueError("oracle: bad model parameters")
        self.model = model

    def __del__(self):
        if getattr(self, "h", None):
            self.L.orc_pf_destroy(self.h)
            self.h = None

    def _obs(self, y):
        if y is None:
            return None, 0
        if self.model.family == SLOTS:  # the slots' values in slot order, bitmask of the present ones
            a, mask = slot_obs(self.model, y)
            return np.ascontiguousarray(a), mask
        a = np.ascontiguousarray(np.atleast_1d(np.asarray(y, dtype=np.float64)))
        return a, 1

    def set_proposal_args(self, args):
        """(alpha, beta, gamma, sigma_q) of the GAUSSIAN proposal (nonlinear SSM)"""
        a = np.ascontiguousarray(args, dtype=np.float64)
        if self.L.orc_pf_set_proposal_args(self.h, _d(a), a.size):
            raise ValueError("oracle: proposal arguments (alpha, beta, gamma, sigma_q > 0)")

    def init(self, y, proposal=DEFAULT):
        a, has = self._obs(y)
        if self.L.orc_pf_init(self.h, _d(a), has, proposal):
            raise ValueError("oracle: proposal not available for this model")

    def step(self, y, proposal=DEFAULT):
        a, has = self._obs(y)
        if self.L.orc_pf_step(self.h, _d(a), has, proposal):
            raise ValueError("oracle: this filter does not take plain steps")

    def step_params(self, model, y, proposal=DEFAULT):
        """particle_filter_step! with the Unfold's parameters changed to `model`'s
        (same family and dimensions): every particle's weight gains its
        trajectory's score under the new parameters minus under the old ones."""
        fam, d, dy, k, v, p = model_args(model)
        a, has = self._obs(y)
        self._p = p
        if self.L.orc_pf_step_params(self.h, _d(p), p.size, _d(a), has, proposal):
            raise ValueError("oracle: parameter change needs one shard with its history, a matching model")
        self.model = model

    def init_conditional(self, y, ref):
        a, has = self._obs(y)
        r = np.ascontiguousarray(np.atleast_1d(np.asarray(ref, dtype=np.float64)))
        if self.L.orc_pf_init_conditional(self.h, _d(a), has, _d(r)):
            raise ValueError("oracle: conditional SMC needs the multinomial resampler on one shard")

    def step_conditional(self, y, ref):
        a, has = self._obs(y)
        r = np.ascontiguousarray(np.atleast_1d(np.asarray(ref, dtype=np.float64)))
        if self.L.orc_pf_step_conditional(self.h, _d(a), has, _d(r)):
            raise ValueError("oracle: not a conditional filter")

    def maybe_resample(self, thr=None):
        thr = self.n_global / 2 if thr is None else thr
        ess = c_double()
        r = self.L.orc_pf_maybe_resample(self.h, thr, ctypes.byref(ess))
        if r < 0:
            raise FloatingPointError("oracle: all log-weights are -Inf/NaN")
        return bool(r), ess.value

    def rejuvenate(self, n_moves):
        """n_moves mh(trace, select(x_t)) moves on every particle; returns accepted moves."""
        acc = c_int64()
        if self.L.orc_pf_rejuvenate(self.h, n_moves, ctypes.byref(acc)):
            raise RuntimeError("oracle: rejuvenate after a resample / too many moves")
        return acc.value

    def mh_select(self, mask, n_moves=1):
        """mh(trace, selection) on every particle (mask over the step's latent addresses)."""
        acc = c_int64()
        if self.L.orc_pf_mh_select(self.h, int(mask), n_moves, ctypes.byref(acc)):
            raise RuntimeError("oracle: bad selection / mh after a resample")
        return acc.value

    def mh_drift(self, mask, sd, n_moves=1):
        """mh(trace, drift, (sd,)) on every particle: Gaussian drift of the selected latent addresses."""
        acc = c_int64()
        sdv = np.ascontiguousarray(np.atleast_1d(sd), dtype=np.float64)
        if self.L.orc_pf_mh_drift(self.h, int(mask), _d(sdv), n_moves, ctypes.byref(acc)):
            raise RuntimeError("oracle: bad drift arguments / mh after a resample")
        return acc.value

    def log_ml_estimate(self):
        return self.L.orc_pf_log_ml_estimate(self.h)

    def log_weights(self):
        o = np.empty(self.n)
        self.L.orc_pf_get_log_weights(self.h, _d(o))
        return o

    def state(self):
        o = np.empty((self.d, self.n))
        self.L.orc_pf_get_state(self.h, _d(o))
        return o

    def parents(self):
        o = np.empty(self.n, dtype=np.int64)
        self.L.orc_pf_get_parents(self.h, o.ctypes.data_as(POINTER(c_int64)))
        return o

    def history(self, t):
        x = np.empty((self.d, self.n))
        anc = np.empty(self.n, dtype=np.int32)
        res = c_int()
        rc = self.L.orc_pf_get_history(self.h, t, _d(x), anc.ctypes.data_as(POINTER(c_int32)), ctypes.byref(res))
        if rc:
            raise ValueError("no history")
        return x, (anc if res.value else None)

    def scores(self, per_step=False):
        """get_score of every particle's trace (and the [t, 2, n] choice scores)."""
        tot = np.empty(self.n)
        ps = np.empty((self.L.orc_pf_num_steps(self.h), 2, self.n)) if per_step else None
        if self.L.orc_pf_get_scores(self.h, _d(tot), _d(ps)):
            raise ValueError("oracle: scores need the history on one shard")
        return (tot, ps) if per_step else tot

    def trajectory(self, t):
        """latent of step t along the genealogy of the current particles (single rank)."""
        T = self.L.orc_pf_num_steps(self.h)
        idx = np.arange(self.n)
        for s in range(T, t, -1):
            _, anc = self.history(s)
            if anc is not None:
                idx = anc[idx]
        x, _ = self.history(t)
        return x[:, idx]

    # distributed building blocks
    def local_stats(self):
        o = np.empty(3)
        self.L.orc_pf_local_stats(self.h, _d(o))
        return o

    def qtotal(self, M):
        return self.L.orc_pf_local_qtotal(self.h, M)

    def emit(self, M, totals, rank):
        tot = np.ascontiguousarray(totals, dtype=np.uint64)
        n = self.n_global
        slots = np.empty(n, dtype=np.int64)
        ancs = np.empty(n, dtype=np.int64)
        st = np.empty(n * self.d)
        c = self.L.orc_pf_resample_emit(self.h, M, tot.ctypes.data_as(POINTER(c_uint64)), tot.size, rank,
                                       slots.ctypes.data_as(POINTER(c_int64)), ancs.ctypes.data_as(POINTER(c_int64)),
                                       _d(st))
        return slots[:c].copy(), ancs[:c].copy(), st[: c * self.d].reshape(c, self.d).copy()

    def apply(self, L, slots, ancs, states):
        slots = np.ascontiguousarray(slots, dtype=np.int64)
        ancs = np.ascontiguousarray(ancs, dtype=np.int64)
        states = np.ascontiguousarray(states, dtype=np.float64)
        self.L.orc_pf_resample_apply(self.h, L, slots.size, slots.ctypes.data_as(POINTER(c_int64)),
                                    ancs.ctypes.data_as(POINTER(c_int64)), _d(states))


def combine_stats(stats, n_global, thr):
    st = np.ascontiguousarray(stats, dtype=np.float64).ravel()
    L, ess, M = c_double(), c_double(), c_double()
    r = lib().orc_combine_stats(_d(st), st.size // 3, n_global, thr, ctypes.byref(L), ctypes.byref(ess),
                                ctypes.byref(M))
    return r, L.value, ess.value, M.value


def importance_sampling(model, y, n, seed, proposal=DEFAULT):
    fam, d, dy, k, v, p = model_args(model)
    a = None if y is None else np.ascontiguousarray(np.atleast_1d(np.asarray(y, dtype=np.float64)))
    dd = d if fam in (LGSSM, REGRESSION) else 1
    lnw = np.empty(n)
    st = np.empty((dd, n))
    lml = c_double()
    rc = lib().orc_importance_sampling(fam, d, dy, k, v, _d(p), p.size, _d(a), int(a is not None), proposal, n, seed,
                                       _d(lnw), _d(st), ctypes.byref(lml))
    if rc:
        raise ValueError("oracle IS failed")
    return st, lnw, lml.value


def simulate(model, T, n, seed, inputs=None):
    """simulate(model, (T,)) n times — (T, U) with a slot model's per-step
    inputs U [T, d] — : (xs [T, d, n], ys [T, dy, n], per_step [T, 2, n], total [n])."""
    fam, d, dy, k, v, p = model_args(model)
    dd = d if fam in (LGSSM, REGRESSION, SLOTS) else 1
    ddy = dy if fam in (LGSSM, REGRESSION, SLOTS) else 1
    xs, ys = np.empty((T, dd, n)), np.empty((T, ddy, n))
    ps, tot = np.empty((T, 2, n)), np.empty(n)
    if inputs is not None:
        U = np.ascontiguousarray(np.asarray(inputs, dtype=np.float64).reshape(T, dd))
        rc = lib().orc_simulate_inputs(fam, d, dy, k, v, _d(p), p.size, T, n, seed, _d(U), _d(xs), _d(ys), _d(ps),
                                       _d(tot))
    else:
        rc = lib().orc_simulate(fam, d, dy, k, v, _d(p), p.size, T, n, seed, _d(xs), _d(ys), _d(ps), _d(tot))
    if rc:
        raise ValueError("oracle simulate failed")
    return xs, ys, ps, tot


DISTS = {"normal": 1, "broadcasted_normal": 2, "mvnormal": 3, "uniform_continuous": 4, "uniform_discrete": 5,
         "bernoulli": 6, "categorical": 7, "gamma": 8, "inv_gamma": 9, "beta": 10, "exponential": 11, "poisson": 12,
         "binomial": 13, "neg_binomial": 14, "geometric": 15, "laplace": 16, "cauchy": 17, "piecewise_uniform": 18,
         "beta_uniform": 19}


def dist_logpdf(name, params, x, dim=1, per_value=False):
    """logpdf of n values x ([dim, n] or [n]) under one shared parameter row
    (or, per_value, rows params[n, n_params])."""
    p = np.ascontiguousarray(params, dtype=np.float64)
    xv = np.ascontiguousarray(x, dtype=np.float64)
    n = xv.shape[-1]
    np_ = p.shape[-1] if per_value else p.size
    out = np.empty(n)
    if lib().orc_dist_logpdf(DISTS[name], dim, np_, np_ if per_value else 0, _d(p), n, _d(xv), _d(out)):
        raise ValueError("oracle dist_logpdf failed")
    return out


def dist_random(name, params, n, seed, dim=1, per_value=False):
    p = np.ascontiguousarray(params, dtype=np.float64)
    np_ = p.shape[-1] if per_value else p.size
    out = np.empty((dim, n)) if dim > 1 else np.empty(n)
    if lib().orc_dist_random(DISTS[name], dim, np_, np_ if per_value else 0, _d(p), n, seed, _d(out)):
        raise ValueError("oracle dist_random failed")
    return out


def run_pf(model, ys, n, seed, thr=None, resampler=SYSTEMATIC, proposal=DEFAULT, record_history=True):
    """The reference caller loop (test/inference/particle_filter.jl:152-162)."""
    pf = OraclePF(model, n, seed, resampler, record_history=record_history)
    pf.init(ys[0], proposal)
    for y in ys[1:]:
        pf.maybe_resample(thr)
        pf.step(y, proposal)
    return pf


def run_csmc(model, ys, n, seed, reference, thr=None):
    """conditional_smc (examples/pmmh/smc.jl:100-151) on the oracle; reference [T, d]."""
    ref = np.asarray(reference, dtype=np.float64).reshape(len(ys), -1)
    pf = OraclePF(model, n, seed, MULTINOMIAL)
    pf.init_conditional(ys[0], ref[0])
    for t in range(1, len(ys)):
        pf.maybe_resample(thr)
        pf.step_conditional(ys[t], ref[t])
    return pf


def pmmh_run(ys, n_chains, n_inner, n_iters, seed, chain0=0, iter0=0, state=None, history=False):
    """CPU PMMH (orc_pmmh_run): returns (lvx, lvy, lml, accepts[n,4], hist)."""
    ys = np.ascontiguousarray(np.asarray(ys, dtype=np.float64))
    if state is None:
        lvx, lvy, lml = np.zeros(n_chains), np.zeros(n_chains), np.zeros(n_chains)
        init = 1
    else:
        lvx, lvy, lml = (np.array(a, dtype=np.float64) for a in state)
        init = 0
    acc = np.zeros((n_chains, 4), dtype=np.int32)
    hist = np.zeros((n_chains, max(n_iters, 1), 2)) if history else None
    rc = lib().orc_pmmh_run(chain0, n_chains, n_inner, _d(ys), ys.size, n_iters, iter0, seed, init, _d(lvx),
                            _d(lvy), _d(lml), acc.ctypes.data_as(POINTER(ctypes.c_int32)), _d(hist))
    if rc:
        raise ValueError("oracle PMMH failed")
    return lvx, lvy, lml, acc, hist


COAL_W = 68


def coal_run(events, n_chains, n_iters, seed, chain0=0, iter0=0, state=None, khist=False, simple=False):
    """CPU RJMCMC on the coal model (orc_coal_run): (state[n,68], accepts[n,3], khist).
    simple: simple_mcmc_step (regenerate k as the third move)."""
    ev = np.ascontiguousarray(np.asarray(events, dtype=np.float64))
    st = np.zeros((n_chains, COAL_W)) if state is None else np.array(state, dtype=np.float64)
    acc = np.zeros((n_chains, 3), dtype=np.int32)
    kh = np.zeros((n_chains, max(n_iters, 1)), dtype=np.int32) if khist else None
    rc = lib().orc_coal_run(chain0, n_chains, _d(ev), ev.size, n_iters, iter0, seed, 1 if state is None else 0,
                            _d(st), acc.ctypes.data_as(POINTER(ctypes.c_int32)),
                            None if kh is None else kh.ctypes.data_as(POINTER(ctypes.c_int32)), int(simple))
    if rc:
        raise ValueError("oracle coal failed")
    return st, acc, kh


def coal_regen_k(row, events, u):
    """mh(trace, select(:k)) on one row with explicit uniforms u[66] (u[0]: k',
    u[i]: change point i, u[32 + i]: rate i): (weight, proposed row)."""
    ev = np.ascontiguousarray(np.asarray(events, dtype=np.float64))
    r = np.ascontiguousarray(row, dtype=np.float64)
    uu = np.ascontiguousarray(u, dtype=np.float64)
    out = np.zeros(COAL_W)
    a = lib().orc_coal_regen_k(_d(r), _d(ev), ev.size, _d(uu), _d(out))
    return a, out


def coal_score(row, events):
    """The oracle's score of one 68-double coal row (k, score, cp[32], h[33], pad)."""
    r = np.ascontiguousarray(row, dtype=np.float64)
    ev = np.ascontiguousarray(events, dtype=np.float64)
    return lib().orc_coal_score(_d(r), _d(ev), ev.size)


COAL_MOVES = {"rate": 0, "position": 1, "birth": 2, "death": 3}


def coal_propose(row, events, move, u):
    """One coal move from explicit uniforms u (3): (alpha, proposed row)."""
    r = np.ascontiguousarray(row, dtype=np.float64)
    ev = np.ascontiguousarray(events, dtype=np.float64)
    uu = np.ascontiguousarray(np.resize(np.asarray(u, dtype=np.float64), 3))
    out = np.zeros(COAL_W)
    a = lib().orc_coal_propose(_d(r), _d(ev), ev.size, COAL_MOVES[move], _d(uu), _d(out))
    return a, out


def pmmh_loglik(ys, lvx, lvy, n_inner, seed, chain, u=0):
    """The PMMH inner particle filter's log-ML estimate (orc_pmmh_loglik)."""
    y = np.ascontiguousarray(np.asarray(ys, dtype=np.float64))
    return lib().orc_pmmh_loglik(seed, chain, u, lvx, lvy, n_inner, _d(y), y.size)
