"""Gen's particle-filter API over libgen_hip.so.

Same names, argument meaning and error behaviour as
src/inference/particle_filter.jl (Julia `!` dropped from the names):

    initialize_particle_filter(model, model_args, observations, num_particles)     :99-108
    initialize_particle_filter(model, model_args, observations, proposal, (), N)   :79-91
    particle_filter_step(state, new_args, argdiffs, observations[, proposal, args]):139-180
    maybe_resample(state, ess_threshold=N/2, verbose=False) -> bool               :189-213
    log_ml_estimate(state)                                                          :52-55
    get_traces / get_log_weights / sample_unweighted_traces                         :31-70
    importance_sampling(model, model_args, observations, N)     src/inference/importance.jl:20-52
    importance_resampling(model, model_args, observations, N)   src/inference/importance.jl:70-85

Every per-particle loop runs on the GPU; this module only translates
Gen-style arguments (tuples, choice maps, argdiffs) into gh_* calls.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import byref, c_double, c_int, c_int64, c_void_p

import numpy as np

from . import _lib
from .choicemap import ChoiceMap
from .models import Model


# ------------------------------------------------------------------ argdiffs
class NoChange:  # src/diff.jl:39
    def __repr__(self):
        return "NoChange()"


class UnknownChange:  # src/diff.jl:46
    def __repr__(self):
        return "UnknownChange()"


class OptimalProposal:
    """The locally optimal proposal (categorical HMM): q(z_t) ∝ p(z_t|z_{t-1}) p(x_t|z_t).
    Stands for the reference test's `init_proposal` / `step_proposal`
    (test/inference/particle_filter.jl:104-127)."""


class GaussianProposal:
    """A user-parameterised custom proposal for the nonlinear SSM (a proposal
    generative function in Gen's sense, particle_filter.jl:79-91,139-154):
    x_t ~ normal(alpha * m + beta * y_t + gamma, sigma_q), m the model's prior
    mean of x_t; proposal_args = (alpha, beta, gamma, sigma_q).  The weight is
    log p(x_t | x_{t-1}) + log p(y_t | x_t) - log q(x_t)
    (trace_translators.jl:775-802)."""


class LinearGaussianProposal:
    """The LG-SSM's user-parameterised custom proposal (the same translator):

        @gen function linear_proposal(trace, P, Sigma_q, u)
            x_prev = trace[:chain => t - 1 => :x]          # absent at t = 1
            @trace(mvnormal(P * x_prev + u, Sigma_q), :chain => t => :x)

    proposal_args = (P, Sigma_q, u) — or (u,) alone to keep P and Sigma_q
    (e.g. a data-driven mean offset per step).  weight = model score of the
    new choices - proposal score."""


def _qargs(proposal, proposal_args):
    if proposal is LinearGaussianProposal or isinstance(proposal, LinearGaussianProposal):
        if not proposal_args:
            return None, 0
        parts = [np.asarray(a, dtype=np.float64).ravel() for a in proposal_args]
        a = np.ascontiguousarray(np.concatenate(parts))
        return a, a.size
    if not (proposal is GaussianProposal or isinstance(proposal, GaussianProposal)):
        return None, 0
    a = np.ascontiguousarray(proposal_args, dtype=np.float64)
    if a.size != 4:
        raise _lib.GenHipError(1, "GaussianProposal takes proposal_args = (alpha, beta, gamma, sigma_q)")
    return a, 4


# ------------------------------------------------------------------ context
class Context:
    """One GPU (and, for multi-GPU, one rank of an RCCL communicator)."""

    def __init__(self, device: int | None = None, rank: int = 0, world: int = 1, unique_id: bytes | None = None,
                 transport=None, force_multirank: bool = False, peer: bool = False):
        """`unique_id`: RCCL communicator id (Context.unique_id() on rank 0,
        broadcast to the others).  `transport`: a host-staged transport
        (gen_amd.transport.GlooTransport) used instead of RCCL.
        `force_multirank`: filters take the multi-rank path even at world 1
        (a one-rank RCCL communicator; gh_ctx_force_multirank, for tests and
        timing on one GPU).  `peer`: with a `transport`, the ranks exchange
        through each other's mapped device memory (gh_ctx_create_peer); the
        transport only swaps the IPC handles."""
        lib = _lib.load()
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        self.device = device
        self.transport = transport
        h = c_void_p()
        if transport is not None and peer:
            rank, world = transport.rank, transport.world
            _lib.check(lib.gh_ctx_create_peer(device, rank, world, byref(transport.struct), None, byref(h)))
        elif transport is not None:
            rank, world = transport.rank, transport.world
            _lib.check(lib.gh_ctx_create_hostcomm(device, rank, world, byref(transport.struct), None, byref(h)))
        elif world > 1:
            if unique_id is None or len(unique_id) != 128:
                raise ValueError("multi-rank context needs the 128-byte RCCL unique id")
            buf = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
            _lib.check(lib.gh_ctx_create_dist(device, rank, world, buf, None, byref(h)))
        else:
            _lib.check(lib.gh_ctx_create(device, None, byref(h)))
        self.h = h
        self.rank, self.world = rank, world
        self._models = {}
        if force_multirank:
            _lib.check(lib.gh_ctx_force_multirank(h))

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        _lib.check(_lib.load().gh_comm_unique_id(buf))
        return bytes(buf)

    def model_handle(self, model: Model):
        key = id(model)
        if key not in self._models:
            desc, keep = model.desc()
            h = c_void_p()
            _lib.check(_lib.load().gh_model_create(self.h, byref(desc), byref(h)))
            self._models[key] = (h, model, keep)
        return self._models[key][0]

    def stream(self) -> int:
        s = c_void_p()
        _lib.check(_lib.load().gh_ctx_stream(self.h, byref(s)))
        return s.value or 0

    def synchronize(self):
        _lib.check(_lib.load().gh_ctx_synchronize(self.h))

    def set_peer_timeout(self, seconds: float):
        """Bound of every device wait on another rank (peer transport; 30 s
        by default): a rank that has not posted by then is taken as gone and
        the waiting filter raises GH_E_STATE."""
        _lib.check(_lib.load().gh_ctx_set_peer_timeout(self.h, float(seconds)))

    def close(self):
        if self.h:
            lib = _lib.load()
            for h, _, _ in self._models.values():
                lib.gh_model_destroy(h)
            self._models.clear()
            lib.gh_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_DEFAULT_CTX: Context | None = None


def default_context() -> Context:
    global _DEFAULT_CTX
    if _DEFAULT_CTX is None:
        _DEFAULT_CTX = Context()
    return _DEFAULT_CTX


def set_default_context(ctx: Context) -> None:
    global _DEFAULT_CTX
    _DEFAULT_CTX = ctx


# ------------------------------------------------------------- observations
def _step_obs(model: Model, t: int, observations, u=None) -> tuple[_lib.Obs, np.ndarray | None]:
    """The gh_obs of step t from a ChoiceMap / dict / array / None (and a slot
    model's per-step input u_t)."""
    val = None
    if observations is None:
        val = None
    elif isinstance(observations, (ChoiceMap, dict)):
        cm = observations if isinstance(observations, ChoiceMap) else ChoiceMap(observations)
        val = model.obs_from_choicemap(cm, t)
    else:
        val = observations
    if u is not None:
        return model.gh_obs(val, u)  # (a slot model with inputs: the chain with an input entry)
    if val is None:
        return _lib.Obs(None, 0, 0, 0, 0, None), None
    return model.gh_obs(val)  # (a slot model: the chain of its constrained addresses)


def _proposal_code(proposal) -> int:
    if proposal is None:
        return _lib.PROPOSAL_DEFAULT
    if proposal is OptimalProposal or isinstance(proposal, OptimalProposal) or proposal == "optimal":
        return _lib.PROPOSAL_OPTIMAL
    if proposal is GaussianProposal or isinstance(proposal, GaussianProposal):
        return _lib.PROPOSAL_GAUSSIAN
    if proposal is LinearGaussianProposal or isinstance(proposal, LinearGaussianProposal):
        return _lib.PROPOSAL_LINEAR
    raise _lib.GenHipError(1, f"unsupported proposal {proposal!r}: the engine lowers the model's default "
                              "proposal and the locally optimal proposal")


# ------------------------------------------------------------------- state
class ParticleFilterState:
    """Mirror of `ParticleFilterState{U}` (particle_filter.jl:18-24) whose
    traces, weights and parents live in HBM as structure-of-arrays."""

    def __init__(self, ctx: Context, model: Model, handle, num_particles: int):
        self.ctx, self.model, self.h = ctx, model, handle
        self.num_particles = num_particles
        self.moves = 0  # MH moves applied (trace views drop their cached columns when it changes)
        ng, nl, lo = c_int64(), c_int64(), c_int64()
        _lib.check(_lib.load().gh_pf_num_particles(handle, byref(ng), byref(nl), byref(lo)))
        self.n_local, self.first = nl.value, lo.value
        # the observations of every step (host copies) for trace materialisation
        self.observations: dict[int, np.ndarray | None] = {}

    def _log_obs(self, t: int, arr) -> None:
        if isinstance(arr, tuple):  # a slot model's (chain, {name: values})
            self.observations[t] = {k: np.array(v, copy=True) for k, v in arr[1].items()}
        else:
            self.observations[t] = None if arr is None else np.array(arr, copy=True)

    @property
    def t(self) -> int:
        t = c_int()
        _lib.check(_lib.load().gh_pf_num_steps(self.h, byref(t)))
        return t.value

    def close(self):
        if self.h:
            _lib.load().gh_pf_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # accessors ---------------------------------------------------------
    @property
    def log_weights(self) -> np.ndarray:
        return get_log_weights(self)

    @property
    def parents(self) -> np.ndarray:
        out = np.empty(self.n_local, dtype=np.int64)
        _lib.check(_lib.load().gh_pf_get_parents(self.h, out.ctypes.data_as(ctypes.POINTER(c_int64))))
        return out

    def states(self, t: int | None = None) -> np.ndarray:
        """[n_local, d] latent of step t (default: current) along each particle's genealogy."""
        d = self.model.d
        out = np.empty((d, self.n_local), dtype=np.float64)
        lib = _lib.load()
        if t is None:
            _lib.check(lib.gh_pf_get_states(self.h, _lib.dptr(out)))
        else:
            _lib.check(lib.gh_pf_get_trajectory(self.h, int(t), _lib.dptr(out)))
        return out.T.copy()

    def ess_history(self):
        T = self.t
        ess = np.empty(T)
        did = np.empty(T, dtype=np.int32)
        _lib.check(_lib.load().gh_pf_get_ess_history(self.h, T, _lib.dptr(ess),
                                                     did.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return ess, did.astype(bool)

    def kernel_time_ms(self, reset: bool = False) -> tuple[float, int]:
        ms, n = c_double(), c_int64()
        _lib.check(_lib.load().gh_pf_kernel_time(self.h, byref(ms), byref(n), int(reset)))
        return ms.value, n.value


class ParticleTraces:
    """`get_traces(state)`: the particles' traces, materialised lazily from the
    SoA history.  `traces[i][addr]` reads one choice; `traces.column(addr)`
    reads an address across all particles."""

    def __init__(self, state: ParticleFilterState):
        self.state = state
        self._cache = {}
        self._moves = state.moves

    def _fresh(self):
        # an MH move rewrote the current step's latents in place: cached columns are stale
        if self._moves != self.state.moves:
            self._cache.clear()
            self._moves = self.state.moves

    def __len__(self):
        return self.state.n_local

    def _step_of(self, addr):
        m = self.state.model
        for t in range(1, self.state.t + 1):
            for k, la in enumerate(m.latent_addresses(t)):
                if tuple(la) == addr:
                    return t, ("latent", k)
            if m.obs_address(t) == addr or (hasattr(m, "names") and len(addr) == 3 and addr[:2] == ("chain", t)
                                            and addr[2] in m.names):
                return t, "obs"
        raise KeyError(addr)

    def column(self, addr) -> np.ndarray:
        if self.state.model.static:  # the regression: :slope, :intercept are the two latent components
            comp = {("slope",): 0, ("intercept",): 1}.get(tuple(addr))
            if comp is None:
                raise KeyError(addr)
            return self.step_states(1)[:, comp]
        t, kind = self._step_of(tuple(addr))
        if kind == "obs":
            raise KeyError(f"{addr} is an observation; it is constrained to the same value in every trace")
        self._fresh()
        if t not in self._cache:
            self._cache[t] = self.state.states(t)
        return self.state.model.latent_part_column(kind[1], self._cache[t])

    def __getitem__(self, i):
        return _TraceView(self, int(i))

    def step_states(self, t: int) -> np.ndarray:
        """[n_local, d] latents of step t along every particle's genealogy (cached)."""
        self._fresh()
        if t not in self._cache:
            self._cache[t] = self.state.states(t)
        return self._cache[t]

    def scores(self, per_step: bool = False):
        """The traces' score columns, computed on the device from the history
        (gh_pf_get_scores): get_score of every trace [n_local], and with
        per_step the [t, 2, n_local] scores of each step's latent and
        observation choices."""
        key = "_scores_ps" if per_step else "_scores"
        self._fresh()
        if key not in self._cache:
            st = self.state
            tot = np.empty(st.n_local)
            ps = np.empty((st.t, 2, st.n_local)) if per_step else None
            _lib.check(_lib.load().gh_pf_get_scores(st.h, _lib.dptr(tot), _lib.dptr(ps) if ps is not None else None))
            self._cache[key] = (tot, ps) if per_step else tot
        return self._cache[key]


class _TraceView:
    """One particle's trace (`get_traces(state)[i]`): the Unfold's latent
    trajectory along the particle's genealogy plus the observations, with the
    trace accessors of src/gen_fn_interface.jl (`get_args`, `get_choices`,
    `get_score`; `trace[addr]` as `getindex`)."""

    def __init__(self, traces: ParticleTraces, i: int):
        self.traces, self.i = traces, i

    def __getitem__(self, addr):
        return self.traces.column(addr)[self.i]

    def get_args(self) -> tuple:
        """The model arguments: (T,) for the Unfold models, () for a static model."""
        st = self.traces.state
        return () if st.model.static else (st.t,)

    def trajectory(self) -> np.ndarray:
        """[T, d] latent of every step of this particle's ancestral line."""
        st = self.traces.state
        return np.stack([self.traces.step_states(t)[self.i] for t in range(1, st.t + 1)])

    def _obs(self):
        st = self.traces.state
        return [st.observations.get(t) for t in range(1, st.t + 1)]

    def get_choices(self) -> ChoiceMap:
        """get_choices(trace): every latent choice and observation by address."""
        st = self.traces.state
        m = st.model
        cm = ChoiceMap()
        xs = self.trajectory()
        if m.static:  # BayesianLinearRegression: :slope, :intercept, "y-i"
            cm[("slope",)] = float(xs[0, 0])
            cm[("intercept",)] = float(xs[0, 1])
            ys = st.observations.get(1)
            if ys is not None:
                for i, y in enumerate(np.asarray(ys).ravel()):
                    cm[m.y_address(i + 1)] = float(y)
            return cm
        for t in range(1, st.t + 1):
            x = xs[t - 1]
            for k, la in enumerate(m.latent_addresses(t)):
                cm[la] = m.latent_part(k, x)
            y = st.observations.get(t)
            if isinstance(y, dict):  # a slot model: every constrained slot
                for name, v in y.items():
                    v = np.asarray(v).ravel()
                    cm[("chain", t, name)] = float(v[0]) if v.size == 1 else v.copy()
            elif y is not None:
                y = np.asarray(y).ravel()
                cm[m.obs_address(t)] = float(y[0]) if y.size == 1 else y.copy()
        return cm

    def get_score(self) -> float:
        """get_score(trace) = log p(every choice): the device score column
        (gh_pf_get_scores) of this particle."""
        return float(self.traces.scores()[self.i])

    def project(self, selection) -> float:
        """project(trace, selection) (src/static_ir/project.jl:8-28): the sum
        of the selected choices' scores, from the device score columns (the
        regression's :slope / :intercept scores separately on the host)."""
        from .choicemap import Selection, select as _select

        sel = selection if isinstance(selection, Selection) else _select(*selection)
        st = self.traces.state
        m = st.model
        _, ps = self.traces.scores(per_step=True)
        total = 0.0
        for a in sel:
            a = tuple(a)
            if m.static:
                x = self.trajectory()[0]
                if a == ("slope",):
                    total += _normal_lp(x[0], m.mu_s, m.sd_s)
                elif a == ("intercept",):
                    total += _normal_lp(x[1], m.mu_i, m.sd_i)
                elif len(a) == 1 and isinstance(a[0], str) and a[0].startswith("y-"):
                    i = int(a[0][2:]) - 1
                    ys = st.observations.get(1)
                    if ys is not None:
                        total += _normal_lp(float(ys[i]), x[0] * m.xs[i] + x[1], m.sigma)
                continue
            for t in range(1, st.t + 1):
                las = [tuple(la) for la in m.latent_addresses(t)]
                if a in las and len(las) > 1:  # one of several latent addresses: its own score on the host
                    tr = self.trajectory()
                    total += m.latent_part_logpdf(las.index(a), t, tr[t - 2] if t > 1 else None, tr[t - 1])
                elif a == tuple(m.latent_address(t)):
                    total += ps[t - 1, 0, self.i]
                elif hasattr(m, "names") and len(a) == 3 and a[:2] == ("chain", t) and a[2] in m.names:
                    # one slot of a slot model (the device column sums the step's slots): its logpdf on the host
                    y = (st.observations.get(t) or {}).get(a[2])
                    if y is not None:
                        total += m.slot_logpdf(m.names.index(a[2]), np.asarray(y).ravel() if
                                               m.slots[m.names.index(a[2])]["dist"] == "mvnormal" else
                                               float(np.asarray(y).ravel()[0]), self.trajectory()[t - 1],
                                               st.observations.get(t))
                elif a == tuple(m.obs_address(t)):
                    total += ps[t - 1, 1, self.i]
        return float(total)


def _normal_lp(x, mu, sd) -> float:
    """normal.jl:56-60"""
    v = sd * sd
    return float(-((x - mu) ** 2) / (2.0 * v) - 0.5 * np.log(2.0 * np.pi * v))


# --------------------------------------------------------------- the API
def _opts(resampler: str, record_history: bool, history_capacity: int, time_kernels: int) -> _lib.PFOpts:
    o = _lib.PFOpts()
    _lib.load().gh_pf_opts_default(byref(o))
    o.resampler = {"systematic": _lib.RESAMPLE_SYSTEMATIC, "multinomial": _lib.RESAMPLE_MULTINOMIAL}[resampler]
    o.record_history = int(record_history)
    o.history_capacity = int(history_capacity)
    o.time_kernels = int(time_kernels)
    return o


def initialize_particle_filter(model: Model, model_args: tuple, observations, *args, seed: int = 0,
                               resampler: str = "systematic", record_history: bool = True,
                               history_capacity: int = 0, time_kernels: int = 0,
                               ctx: Context | None = None) -> ParticleFilterState:
    """initialize_particle_filter(model, model_args, observations, num_particles)
    initialize_particle_filter(model, model_args, observations, proposal, proposal_args, num_particles)

    Resampling scheme: Gen's maybe_resample! draws parents multinomially
    (`Distributions.rand!(Categorical(..))`, particle_filter.jl:200); this
    engine defaults to SYSTEMATIC resampling (the north-star setting, the
    lower-variance scheme, and the only one the multi-rank path exchanges).
    Pass resampler="multinomial" for Gen's distribution of parents; both are
    unbiased, so log-ML estimates agree in expectation, not draw for draw."""
    proposal_args = ()
    if len(args) == 1:
        proposal, num_particles = None, args[0]
    elif len(args) == 3:
        proposal, proposal_args, num_particles = args
    else:
        raise TypeError("expected (num_particles) or (proposal, proposal_args, num_particles)")
    if not model.static and tuple(model_args)[:1] not in ((1,), ()):
        raise _lib.GenHipError(1, "the particle filter starts at model_args = (1,)")
    ctx = ctx or default_context()
    mh = ctx.model_handle(model)
    obs, keep = _step_obs(model, 1, observations)
    h = c_void_p()
    opts = _opts(resampler, record_history, history_capacity, time_kernels)
    qa, nq = _qargs(proposal, proposal_args)
    _lib.check(_lib.load().gh_pf_init_q(mh, byref(obs), _proposal_code(proposal),
                                        _lib.dptr(qa) if qa is not None else None, nq, int(num_particles),
                                        int(seed) & 0xFFFFFFFFFFFFFFFF, byref(opts), byref(h)))
    st = ParticleFilterState(ctx, model, h, int(num_particles))
    st._log_obs(1, keep)
    return st


def particle_filter_step(state: ParticleFilterState, new_args: tuple, argdiffs: tuple, observations,
                         proposal=None, proposal_args: tuple = ()) -> None:
    """particle_filter_step!(state, new_args, argdiffs, observations[, proposal,
    proposal_args]) (particle_filter.jl:139-180).  new_args = (t,) extends the
    Unfold by one step; new_args = (t, model') also changes the Unfold's
    parameters to those of model' (the same family and dimensions) with an
    UnknownChange() argdiff for them: every retained kernel application is
    re-scored (gh_pf_step_params), as the Unfold's update does.  A slot model
    with per-step inputs takes new_args = (t, u_t) or (t, model', u_t): the
    Unfold's argument vector extended by one value (earlier steps keep theirs,
    so nothing is re-scored for it)."""
    t = state.t + 1
    new_args = tuple(new_args)
    argdiffs = tuple(argdiffs)
    if new_args[:1] != (t,):
        raise _lib.GenHipError(1, f"new_args must extend the Unfold by one step: expected ({t}, ...), got {new_args}")
    if argdiffs and not isinstance(argdiffs[0], UnknownChange):
        raise _lib.GenHipError(1, "the length argument changes: its argdiff must be UnknownChange()")
    u = None
    if getattr(state.model, "inputs", False) and len(new_args) >= 2 and not isinstance(new_args[-1], Model):
        u = new_args[-1]  # (t, u_t) / (t, model', u_t)
        new_args = new_args[:-1]
        argdiffs = argdiffs[:len(new_args)]
    if len(new_args) > 2:
        raise _lib.GenHipError(1, "new_args = (t,) or (t, model with the new parameters)")
    new_model = new_args[1] if len(new_args) == 2 else None
    if new_model is not None and new_model is not state.model:
        diff = argdiffs[1] if len(argdiffs) > 1 else UnknownChange()
        if isinstance(diff, NoChange):
            raise _lib.GenHipError(1, "the parameters differ from the filter's but their argdiff is NoChange()")
        if type(new_model) is not type(state.model):
            raise _lib.GenHipError(1, "new parameters of another model family")
        obs, keep = _step_obs(new_model, t, observations, u)
        if proposal_args:
            raise _lib.GenHipError(1, "a parameter change takes the proposal's stored arguments")
        mh = state.ctx.model_handle(new_model)
        _lib.check(_lib.load().gh_pf_step_params(state.h, byref(obs), _proposal_code(proposal), mh))
        state.model = new_model
        state._log_obs(t, keep)
        return
    obs, keep = _step_obs(state.model, t, observations, u)
    qa, nq = _qargs(proposal, proposal_args)
    _lib.check(_lib.load().gh_pf_step_q(state.h, byref(obs), _proposal_code(proposal),
                                        _lib.dptr(qa) if qa is not None else None, nq))
    state._log_obs(t, keep)


def maybe_resample(state: ParticleFilterState, ess_threshold: float | None = None, verbose: bool = False) -> bool:
    thr = state.num_particles / 2 if ess_threshold is None else float(ess_threshold)
    did, ess = c_int(), c_double()
    _lib.check(_lib.load().gh_pf_maybe_resample(state.h, thr, byref(did), byref(ess)))
    if verbose:
        print(f"effective sample size: {ess.value}, doing resample: {bool(did.value)}")
    return bool(did.value)


def maybe_resample_async(state: ParticleFilterState, ess_threshold: float | None = None) -> None:
    """maybe_resample! whose decision stays on the device (no host round trip)."""
    thr = state.num_particles / 2 if ess_threshold is None else float(ess_threshold)
    _lib.check(_lib.load().gh_pf_maybe_resample(state.h, thr, None, None))


class ObservationBatch:
    """The gh_obs array of several consecutive steps, built once (the host-side
    marshalling of run_particle_filter, done ahead of a timed loop)."""

    def __init__(self, model: Model, observations_per_step, inputs_per_step=None):
        ins = [None] * len(observations_per_step) if inputs_per_step is None else list(inputs_per_step)
        if len(ins) != len(observations_per_step):
            raise ValueError("one input per step")
        built = [(_lib.Obs(None, 0, 0, 0, 0, None), None) if v is None and u is None
                 else (model.gh_obs(v, u) if u is not None else model.gh_obs(v))
                 for v, u in zip(observations_per_step, ins)]
        self.values = [keep for _, keep in built]  # (kept alive with the array: the gh_obs point into them)
        self.arr = (_lib.Obs * max(1, len(self.values)))()
        for i, (o, _) in enumerate(built):
            self.arr[i] = o

    def __len__(self):
        return len(self.values)


def prepare_observations(model: Model, observations_per_step, inputs_per_step=None) -> ObservationBatch:
    return ObservationBatch(model, observations_per_step, inputs_per_step)


def run_particle_filter(state: ParticleFilterState, observations_per_step, ess_threshold: float | None = None,
                        proposal=None, proposal_args: tuple | None = None, inputs_per_step=None) -> None:
    """The reference caller loop {maybe_resample!; particle_filter_step!} over
    the given per-step observations (arrays or None, or an ObservationBatch of
    them), enqueued without host sync.  A proposal with arguments uses
    proposal_args, or the last ones given.  inputs_per_step: a slot model's
    per-step inputs u_t (None entries: no input)."""
    model = state.model
    if isinstance(observations_per_step, ObservationBatch):
        if inputs_per_step is not None:
            raise ValueError("run_particle_filter: inputs with a prepared ObservationBatch (prepare them with it)")
        if proposal_args is not None:
            raise ValueError("run_particle_filter: proposal_args with a prepared ObservationBatch; pass the "
                             "observations as a list (its first step takes the arguments) or set them with a "
                             "particle_filter_step first")
        batch = observations_per_step
    else:
        if proposal_args is not None and len(observations_per_step) > 0:
            qa, nq = _qargs(proposal, proposal_args)
            if qa is not None:  # store them (the library keeps the last arguments)
                maybe_resample_async(state, ess_threshold)
                u0 = None if inputs_per_step is None else inputs_per_step[0]
                particle_filter_step(state, (state.t + 1,) + (() if u0 is None else (u0,)),
                                     (UnknownChange(),) * (1 if u0 is None else 2), observations_per_step[0],
                                     proposal, proposal_args)
                observations_per_step = list(observations_per_step)[1:]
                if inputs_per_step is not None:
                    inputs_per_step = list(inputs_per_step)[1:]
        batch = ObservationBatch(model, observations_per_step, inputs_per_step)
    t0 = state.t
    thr = state.num_particles / 2 if ess_threshold is None else float(ess_threshold)
    _lib.check(_lib.load().gh_pf_run(state.h, len(batch), batch.arr, _proposal_code(proposal), thr))
    for i, a in enumerate(batch.values):
        state._log_obs(t0 + 1 + i, a)


def log_ml_estimate(state: ParticleFilterState) -> float:
    out = c_double()
    _lib.check(_lib.load().gh_pf_log_ml_estimate(state.h, byref(out)))
    return out.value


def get_log_weights(state: ParticleFilterState) -> np.ndarray:
    out = np.empty(state.n_local, dtype=np.float64)
    _lib.check(_lib.load().gh_pf_get_log_weights(state.h, _lib.dptr(out)))
    return out


def get_traces(state: ParticleFilterState) -> ParticleTraces:
    return ParticleTraces(state)


def sample_unweighted_traces(state: ParticleFilterState, num_samples: int, seed: int = 0):
    """Indices (and views) of num_samples traces drawn ∝ normalised weights."""
    idx = np.empty(int(num_samples), dtype=np.int64)
    _lib.check(_lib.load().gh_pf_sample_unweighted(state.h, int(num_samples), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                                   idx.ctypes.data_as(ctypes.POINTER(c_int64))))
    tr = get_traces(state)
    # (on R ranks the indices are global: this rank's views of its own ones)
    lo, nl = state.first, state.n_local
    return [tr[i - lo] if lo <= i < lo + nl else None for i in idx], idx


def rejuvenate(state: ParticleFilterState, n_moves: int = 1) -> int:
    """Rejuvenation between steps: for every particle i, n_moves times
    ``state.traces[i], _ = mh(state.traces[i], select(:chain => t => :x))``
    (src/inference/mh.jl:14-26) on the current step t.  Weights are unchanged.
    Call after a step and before maybe_resample.  Returns the accepted moves
    summed over this rank's particles."""
    acc = c_int64()
    _lib.check(_lib.load().gh_pf_rejuvenate(state.h, int(n_moves), byref(acc)))
    state.moves += 1
    return int(acc.value)


class GaussianDriftProposal:
    """The Gaussian drift proposal generative function, the proposal form of
    ``metropolis_hastings(trace, proposal, proposal_args)`` (src/inference/mh.jl:41-62):

        @gen function gaussian_drift(trace, selection, sd)
            for a in selection: @trace(normal(trace[a], sd), a)   # mvnormal(x, diag(sd^2)) for a vector latent

    ``proposal_args = (selection, sd)``, sd a scalar or one value per state
    component."""

    def __repr__(self):
        return "gaussian_drift"


gaussian_drift = GaussianDriftProposal()


def _latent_mask(state: ParticleFilterState, selection) -> int:
    from .choicemap import Selection, select as _select

    sel = selection if isinstance(selection, Selection) else _select(*selection)
    m = state.model
    if m.static:
        names = {("slope",): 1, ("intercept",): 2}
    else:
        names = {tuple(a): 1 for a in m.latent_addresses(state.t)}
        if len(names) > 1 and not all(a in set(map(tuple, sel)) for a in names):  # (a switching slot model)
            raise _lib.GenHipError(1, f"selection must name every latent address of the step together: {sorted(names)}")
    mask = 0
    for a in sel:
        if a not in names:
            raise _lib.GenHipError(1, f"selection names {a}: only {sorted(names)} (the current step's latent "
                                      "addresses) are lowered")
        mask |= names[a]
    return mask


def metropolis_hastings(state: ParticleFilterState, selection, *args, n_moves: int | None = None) -> int:
    """``metropolis_hastings`` (alias ``mh``) applied to every particle's trace;
    the particles' log weights are unchanged.  Returns the accepted moves over
    this rank's particles.

    * ``mh(state, selection[, n_moves])`` — the selection form (mh.jl:14-28):
      regenerate the selected choices from their prior, accept with
      log(rand()) < the regenerate weight.  The selection names latent
      addresses of the current step: the regression's "slope" / "intercept"
      (examples/regression/quickstart.jl:17-22), or the Unfold models' latent
      of the last step.
    * ``mh(state, gaussian_drift, (selection, sd)[, n_moves])`` — the proposal
      form (mh.jl:41-62) with the Gaussian drift proposal: accept with
      log(rand()) < update weight - forward score + backward score."""
    if selection is gaussian_drift or isinstance(selection, GaussianDriftProposal):
        pargs = tuple(args[0]) if args else ()
        n = n_moves if n_moves is not None else (int(args[1]) if len(args) > 1 else 1)
        if len(pargs) != 2:
            raise _lib.GenHipError(1, "gaussian_drift takes proposal_args = (selection, sd)")
        mask = _latent_mask(state, pargs[0])
        d = state.model.d
        sd = np.ascontiguousarray(np.broadcast_to(np.asarray(pargs[1], dtype=np.float64), (d,)))
        acc = c_int64()
        _lib.check(_lib.load().gh_pf_mh_drift(state.h, mask, _lib.dptr(sd), int(n), byref(acc)))
        state.moves += 1
        return int(acc.value)
    n = n_moves if n_moves is not None else (int(args[0]) if args else 1)
    mask = _latent_mask(state, selection)
    acc = c_int64()
    _lib.check(_lib.load().gh_pf_mh_select(state.h, mask, int(n), byref(acc)))
    state.moves += 1
    return int(acc.value)


mh = metropolis_hastings


# ------------------------------------------------------ conditional SMC
def _ref_state(model: Model, x) -> np.ndarray:
    a = np.ascontiguousarray(np.atleast_1d(np.asarray(x, dtype=np.float64)).ravel())
    if a.size != model.d:
        raise _lib.GenHipError(1, f"a reference state has {model.d} values, got {a.size}")
    return a


def initialize_conditional_particle_filter(model: Model, model_args: tuple, observations, num_particles: int,
                                           reference_x1, seed: int = 0, record_history: bool = True,
                                           history_capacity: int = 0, ctx: Context | None = None
                                           ) -> ParticleFilterState:
    """conditional_smc's initialisation (examples/pmmh/smc.jl:110-119):
    particle 0 is the distinguished particle, pinned to reference_x1 with
    weight init_score = log p(y_1 | x_1); multinomial resampling."""
    if tuple(model_args)[:1] not in ((1,), ()):
        raise _lib.GenHipError(1, "the particle filter starts at model_args = (1,)")
    ctx = ctx or default_context()
    mh = ctx.model_handle(model)
    obs, keep = _step_obs(model, 1, observations)
    ref = _ref_state(model, reference_x1)
    h = c_void_p()
    opts = _opts("multinomial", record_history, history_capacity, 0)
    _lib.check(_lib.load().gh_pf_init_conditional(mh, byref(obs), int(num_particles), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                                  byref(opts), _lib.dptr(ref), byref(h)))
    st = ParticleFilterState(ctx, model, h, int(num_particles))
    st._log_obs(1, keep)
    return st


def conditional_particle_filter_step(state: ParticleFilterState, new_args: tuple, argdiffs: tuple, observations,
                                     reference_xt) -> None:
    """One step of conditional_smc (smc.jl:138-147): the distinguished particle
    takes reference_xt, its own parent, weight += log p(y_t | x_t).  new_args =
    (t, model') also changes the Unfold's parameters (every retained kernel
    application re-scored, as particle_filter_step does)."""
    t = state.t + 1
    new_args = tuple(new_args)
    if new_args[:1] != (t,) or len(new_args) > 2:
        raise _lib.GenHipError(1, f"new_args must extend the Unfold by one step: expected ({t},) or ({t}, model'), "
                                  f"got {new_args}")
    new_model = new_args[1] if len(new_args) == 2 else None
    if new_model is not None and new_model is not state.model:
        if type(new_model) is not type(state.model):
            raise _lib.GenHipError(1, "new parameters of another model family")
        obs, keep = _step_obs(new_model, t, observations)
        ref = _ref_state(new_model, reference_xt)
        mh = state.ctx.model_handle(new_model)
        _lib.check(_lib.load().gh_pf_step_params_conditional(state.h, byref(obs), mh, _lib.dptr(ref)))
        state.model = new_model
        state._log_obs(t, keep)
        return
    obs, keep = _step_obs(state.model, t, observations)
    ref = _ref_state(state.model, reference_xt)
    _lib.check(_lib.load().gh_pf_step_conditional(state.h, byref(obs), _lib.dptr(ref)))
    state._log_obs(t, keep)


def conditional_smc(model: Model, observations_per_step, num_particles: int, reference, seed: int = 0,
                    ess_threshold: float | None = None, ctx: Context | None = None) -> ParticleFilterState:
    """conditional_smc(scheme, distinguished_particle) (smc.jl:100-151) with the
    model's own proposal: the whole sweep, reference = [T, d] trajectory."""
    T = len(observations_per_step)
    ref = np.asarray(reference, dtype=np.float64).reshape(T, -1)
    addr = model.obs_address
    st = initialize_conditional_particle_filter(model, (1,), {addr(1): observations_per_step[0]}, num_particles,
                                                ref[0], seed=seed, history_capacity=T, ctx=ctx)
    for t in range(2, T + 1):
        maybe_resample_async(st, ess_threshold)
        conditional_particle_filter_step(st, (t,), (UnknownChange(),), {addr(t): observations_per_step[t - 1]},
                                         ref[t - 1])
    return st


def get_particle(state: ParticleFilterState, index: int) -> np.ndarray:
    """get_particle(result, final_index) (smc.jl:153-163): the [T, d] trajectory
    of one final particle, following its ancestors back."""
    T = state.t
    return np.stack([state.states(t)[index] for t in range(1, T + 1)])


def particle_gibbs(model: Model, observations_per_step, num_particles: int, reference, num_sweeps: int,
                   seed: int = 0, ess_threshold: float | None = None, ctx: Context | None = None):
    """Particle Gibbs: repeat {conditional_smc; draw a final particle with
    probability proportional to its weight; take its trajectory as the next
    reference}.  Returns the list of references after each sweep and the
    log-ML estimates of the sweeps."""
    refs, lmls = [], []
    ref = np.asarray(reference, dtype=np.float64)
    for k in range(num_sweeps):
        st = conditional_smc(model, observations_per_step, num_particles, ref, seed=seed + 1000003 * k,
                             ess_threshold=ess_threshold, ctx=ctx)
        _, idx = sample_unweighted_traces(st, 1, seed=seed + 1000003 * k + 1)
        ref = get_particle(st, int(idx[0]))
        refs.append(ref)
        lmls.append(log_ml_estimate(st))
        st.close()
    return refs, lmls


def importance_sampling(model: Model, model_args: tuple, observations, *args, seed: int = 0,
                        ctx: Context | None = None):
    """(traces, log_normalized_weights, lml_est) (importance.jl:20-52)."""
    if len(args) == 1:
        proposal, n = None, args[0]
    elif len(args) == 3:
        proposal, _, n = args
    else:
        raise TypeError("expected (num_samples) or (proposal, proposal_args, num_samples)")
    ctx = ctx or default_context()
    mh = ctx.model_handle(model)
    obs, keep = _step_obs(model, 1, observations)
    lnw = np.empty(int(n))
    states = np.empty((model.d, int(n)))
    lml = c_double()
    _lib.check(_lib.load().gh_is_run(mh, byref(obs), _proposal_code(proposal), int(n), int(seed),
                                     _lib.dptr(lnw), _lib.dptr(states), byref(lml)))
    del keep
    return states.T.copy(), lnw, lml.value


def importance_resampling(model: Model, model_args: tuple, observations, *args, seed: int = 0,
                          ctx: Context | None = None):
    """(trace, lml_est) (importance.jl:70-108).  The reference's streaming SIR
    keeps one candidate with probability w_i / sum_{j<=i} w_j; the draw here
    is the distribution-equivalent single categorical draw over all N weights
    (SURVEY.md Appendix A.8)."""
    states, lnw, lml = importance_sampling(model, model_args, observations, *args, seed=seed, ctx=ctx)
    w = np.exp(lnw - lnw.max())
    rng = np.random.default_rng(seed)
    i = int(rng.choice(w.size, p=w / w.sum()))
    return states[i], lml
