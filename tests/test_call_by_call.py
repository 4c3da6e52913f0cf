"""The reference caller loop through the C ABI, one call per operation
(test/inference/particle_filter.jl:130-137, examples/pmmh/pf.jl:48-54):
maybe_resample! then particle_filter_step!, with the weight sums and the
decision read in every way a caller can ask for them.

On one rank every step writes block maxima only; the next maybe_resample!
sums the weights in its own pass and any other reader (log_ml_estimate, the
ESS readers, a second maybe_resample! without a step) has them recomputed
(k_block_sums: the same block geometry and order as a full-partials step).
maybe_resample!'s Bool comes back through a host-mapped mailbox that
k_resample1 posts as soon as it has decided.  All of it must be the same
filter as the oracle's, bit for bit (log-ML 1e-9)."""
import numpy as np
import pytest

import gen_amd as gen
from gen_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _model(name):
    return gen.LinearGaussianSSM.benchmark(10) if name == "lg10" else gen.KitagawaSSM(10.0, 1.0)


@pytest.mark.parametrize("name", ["lg10", "kit"])
@pytest.mark.parametrize("decision", ["mailbox", "none", "mixed"])
def test_call_by_call_matches_oracle(gh_ctx, name, decision):
    """Every step compared with the oracle; log_ml_estimate asked for in the
    middle of the run (after a max-only step: the recomputed sums) and the
    returned decisions equal to the oracle's."""
    m = _model(name)
    _, ys = m.simulate(14, np.random.default_rng(31))
    n = 70001
    st = gen.initialize_particle_filter(m, (1,), {m.obs_address(1): ys[0]}, n, seed=17)
    orc = O.OraclePF(m, n, 17, O.SYSTEMATIC)
    orc.init(ys[0])
    for t in range(2, len(ys) + 1):
        thr = None if t % 4 else n / 20  # some steps that do not resample
        odid, oess = orc.maybe_resample(thr)
        ask = decision == "mailbox" or (decision == "mixed" and t % 2 == 0)
        if ask:
            assert gen.maybe_resample(st, thr) == odid, t
        else:
            gen.maybe_resample_async(st, thr)
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), {m.obs_address(t): ys[t - 1]})
        orc.step(ys[t - 1])
        if t % 3 == 0:  # a reader of the sums between steps
            a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
            assert abs(a - b) <= 1e-9 * max(1.0, abs(b)), (t, a, b)
        assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64)), t
        assert np.array_equal(st.parents, orc.parents()), t
    ess, did = st.ess_history()
    a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
    assert abs(a - b) <= 1e-9 * max(1.0, abs(b)), (a, b)


def test_mailbox_decision_and_ess_equal_device_history(gh_ctx):
    """The (did, ess) a caller gets from the mailbox are the values the device
    committed (ess_history), step by step, and the oracle's decision."""
    m = _model("lg10")
    _, ys = m.simulate(10, np.random.default_rng(4))
    n = 30011
    st = gen.initialize_particle_filter(m, (1,), {m.obs_address(1): ys[0]}, n, seed=3)
    orc = O.OraclePF(m, n, 3, O.SYSTEMATIC)
    orc.init(ys[0])
    lib = _lib.load()
    import ctypes

    got = []
    for t in range(2, len(ys) + 1):
        did, ess = ctypes.c_int(), ctypes.c_double()
        _lib.check(lib.gh_pf_maybe_resample(st.h, float(n / 2), ctypes.byref(did), ctypes.byref(ess)))
        odid, oess = orc.maybe_resample(None)
        assert bool(did.value) == odid
        assert abs(ess.value - oess) <= 1e-9 * oess
        got.append((bool(did.value), ess.value))
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), {m.obs_address(t): ys[t - 1]})
        orc.step(ys[t - 1])
    hess, hdid = st.ess_history()
    for s, (d, e) in enumerate(got, start=1):
        assert bool(hdid[s - 1]) == d and hess[s - 1] == e, s


def test_second_maybe_resample_after_max_only_step(gh_ctx):
    """Two maybe_resample! without a step in between after a max-only step:
    the second decides on recomputed sums (k_decide after k_block_sums)."""
    m = _model("kit")
    _, ys = m.simulate(8, np.random.default_rng(12))
    n = 20001
    st = gen.initialize_particle_filter(m, (1,), {m.obs_address(1): ys[0]}, n, seed=8)
    orc = O.OraclePF(m, n, 8, O.SYSTEMATIC)
    orc.init(ys[0])
    for t in range(2, len(ys) + 1):
        for _ in range(2 if t in (3, 6) else 1):
            assert gen.maybe_resample(st, n) == orc.maybe_resample(n)[0]
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), {m.obs_address(t): ys[t - 1]})
        orc.step(ys[t - 1])
    assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64))
    assert np.array_equal(st.parents, orc.parents())
    a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
    assert abs(a - b) <= 1e-9 * max(1.0, abs(b)), (a, b)


def test_force_multirank_refused_with_live_filter():
    """A filter keeps the path it was created on: switching its context to the
    multi-rank path while it exists is GH_E_STATE (its multi-rank buffers were
    never allocated)."""
    ctx = gen.Context(device=0)
    try:
        m = _model("lg10")
        _, ys = m.simulate(2, np.random.default_rng(0))
        st = gen.initialize_particle_filter(m, (1,), {m.obs_address(1): ys[0]}, 1000, seed=1, ctx=ctx)
        with pytest.raises(_lib.GenHipError, match="GH_E_STATE"):
            _lib.check(_lib.load().gh_ctx_force_multirank(ctx.h))
        st.close()
        _lib.check(_lib.load().gh_ctx_force_multirank(ctx.h))  # no filter left: allowed
    finally:
        ctx.close()


class _NoTransport:
    """A two-rank host transport whose collectives must never run (the
    refusal comes before any)."""

    def __init__(self):
        from gen_amd.transport import ALLGATHER_FN, SENDRECV_FN, HostComm

        self.rank, self.world = 0, 2
        self._ag = ALLGATHER_FN(lambda *a: 1)
        self._sr = SENDRECV_FN(lambda *a: 1)
        self.struct = HostComm(None, self._ag, self._sr)


def test_multirank_needs_a_particle_per_rank():
    """Fewer particles than ranks is refused on the multi-rank path (every
    rank must post the same collectives)."""
    ctx = gen.Context(device=0, transport=_NoTransport())
    try:
        m = _model("kit")
        _, ys = m.simulate(2, np.random.default_rng(0))
        with pytest.raises(_lib.GenHipError, match="GH_E_INVAL"):
            gen.initialize_particle_filter(m, (1,), {m.obs_address(1): ys[0]}, 1, seed=1, ctx=ctx)
    finally:
        ctx.close()
