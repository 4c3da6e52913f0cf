"""The one-shard bound path of the resample.

A one-rank filter quantises the weights against the a-priori bound
U = (the last decision's maximum, or 0 after a resample) + the step's weight
bound (the observation density's maximum) instead of their maximum M, when
every weight is <= U and M - U >= -20 ln 2: then k_step's per-block integer
totals are the resample's, and k_resample1 runs without its grid barrier.
Otherwise (an outlier observation, a proposal without a bound, a second
decision on the same weights, N > 2^22) it quantises against M as before.

The bound path changes which uniform falls in which particle only at the
quantisation's rounding (relative 2^-32 at worst), so its parents equal the
exact path's except at such ties; the fall-back cases are bit-identical to the
exact path.  CPU: the oracle's two rules.  GPU: the engine bit-exact against
the oracle under both rules (gh_pf_opts.exact_quantisation).
"""
import numpy as np
import pytest

import gen_amd as gen
from gen_amd.models import KitagawaSSM, LinearGaussianSSM
from oracle import oracle as O


def _run(m, ys, n, seed, resampler, exact, thr):
    pf = O.OraclePF(m, n, seed, resampler, exact_quantisation=exact)
    pf.init(ys[0])
    fired = []
    for y in ys[1:]:
        fired.append(pf.maybe_resample(thr)[0])
        pf.step(y)
    return pf, fired


def _cases():
    k = KitagawaSSM(10.0, 1.0)
    _, ys = k.simulate(12, np.random.default_rng(4))
    ys = [float(y) for y in ys]
    lg = LinearGaussianSSM.benchmark(4)
    _, yl = lg.simulate(12, np.random.default_rng(5))
    return [("kitagawa", k, ys), ("lg4", lg, list(yl))]


CASES = _cases()


@pytest.mark.parametrize("case", range(len(CASES)), ids=[c[0] for c in CASES])
@pytest.mark.parametrize("resampler", [O.SYSTEMATIC, O.MULTINOMIAL])
def test_oracle_bound_path_parents_are_the_exact_paths(case, resampler):
    """Same seed, both rules, resampling every step: every resample takes the
    bound path, and its parents equal the exact path's but for rounding ties."""
    _, m, ys = CASES[case]
    n = 20000
    a, fa = _run(m, ys, n, 3, resampler, False, n + 1)
    b, fb = _run(m, ys, n, 3, resampler, True, n + 1)
    assert all(fa) and all(fb)
    assert a.bound_uses() == len(ys) - 1 and b.bound_uses() == 0
    # trajectories part at the first tie, so compare one resample at a time
    for k in range(2, 6):
        a1, _ = _run(m, ys[:k], n, 3, resampler, False, n + 1)
        b1, _ = _run(m, ys[:k], n, 3, resampler, True, n + 1)
        if not np.array_equal(a1.state(), b1.state()):
            break
        assert np.mean(a1.parents() == b1.parents()) >= 0.999, k
    # the same law: the log-ML estimates agree to Monte Carlo error
    assert abs(a.log_ml_estimate() - b.log_ml_estimate()) <= 0.05 * max(1.0, abs(b.log_ml_estimate()))


def test_oracle_no_bound_without_an_earlier_decision_or_after_a_second():
    """U needs the last decision's maximum: a step after no decision, and a
    second decision on the same weights, quantise against M."""
    m, ys = CASES[0][1], CASES[0][2]
    n = 4000
    pf = O.OraclePF(m, n, 1)
    pf.init(ys[0])
    pf.step(ys[1])  # no decision before this step: U = +inf
    assert pf.maybe_resample(n + 1)[0] and pf.bound_uses() == 0
    pf.step(ys[2])  # after a resample: U = the step's bound
    assert pf.maybe_resample(0.0)[0] is False
    assert pf.maybe_resample(n + 1)[0] and pf.bound_uses() == 0  # the second decision
    pf.step(ys[3])
    assert pf.maybe_resample(n + 1)[0] and pf.bound_uses() == 1


def test_oracle_outlier_observation_falls_back_to_the_maximum():
    """An observation far from every particle puts M far below U: the bound
    path is refused and that resample is the exact one, bit for bit."""
    m = KitagawaSSM(10.0, 1.0)
    ys = [0.5, 1.0, 400.0]
    n = 5000
    a, fa = _run(m, ys + [2.0], n, 8, O.SYSTEMATIC, False, n + 1)
    b, _ = _run(m, ys + [2.0], n, 8, O.SYSTEMATIC, True, n + 1)
    assert a.bound_uses() == 2  # the two ordinary steps' resamples
    a0, _ = _run(m, ys, n, 8, O.SYSTEMATIC, False, n + 1)
    b0, _ = _run(m, ys, n, 8, O.SYSTEMATIC, True, n + 1)
    if np.array_equal(a0.state(), b0.state()):  # same particles before the outlier's resample
        assert np.array_equal(a.parents(), b.parents())


# ------------------------------------------------------------------ GPU
def _gpu_vs_oracle(m, ys, n, seed, resampler, exact, thr, every=None):
    rs = {O.SYSTEMATIC: "systematic", O.MULTINOMIAL: "multinomial"}[resampler]
    addr = m.obs_address
    st = gen.initialize_particle_filter(m, (1,), {addr(1): ys[0]}, n, seed=seed, resampler=rs,
                                        exact_quantisation=exact)
    orc = O.OraclePF(m, n, seed, resampler, exact_quantisation=exact)
    orc.init(ys[0])
    for t in range(2, len(ys) + 1):
        th = thr(t) if callable(thr) else thr
        assert gen.maybe_resample(st, th) == orc.maybe_resample(th)[0], t
        if every and t % every == 0:  # a second decision on the same weights
            assert gen.maybe_resample(st, n + 1) == orc.maybe_resample(n + 1)[0], t
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), {addr(t): ys[t - 1]})
        orc.step(ys[t - 1])
        assert np.array_equal(st.parents, orc.parents()), t
    assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64))
    assert np.array_equal(gen.get_log_weights(st).view(np.uint64), orc.log_weights().view(np.uint64))
    a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
    assert abs(a - b) <= 1e-9 * max(1.0, abs(b))
    st.close()
    return orc.bound_uses()


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(CASES)), ids=[c[0] for c in CASES])
@pytest.mark.parametrize("resampler", [O.SYSTEMATIC, O.MULTINOMIAL])
@pytest.mark.parametrize("exact", [False, True], ids=["bound", "exact"])
def test_gpu_bound_and_exact_paths_bitexact(gh_ctx, case, resampler, exact):
    _, m, ys = CASES[case]
    n = 300007  # ragged: not a multiple of any block
    uses = _gpu_vs_oracle(m, ys, n, 21, resampler, exact, lambda t: n + 1 if t % 4 else n * 0.5, every=5)
    assert (uses == 0) if exact else (uses >= 6)


@pytest.mark.gpu
def test_gpu_outlier_observations_fall_back(gh_ctx):
    m = KitagawaSSM(10.0, 1.0)
    ys = [0.5, 1.0, 400.0, 2.0, -300.0, 1.5, 0.2, 1e4]
    assert _gpu_vs_oracle(m, ys, 100003, 5, O.SYSTEMATIC, False, 100004) >= 2


@pytest.mark.gpu
def test_gpu_bound_path_across_block_sizes(gh_ctx):
    """Particle counts at and around the pairs kernel's and k_step's block
    boundaries, and the first-step bound (no earlier weights).  One particle
    never takes the bound path (its total reaches 2^shift only if its weight
    equals U), so there the test is the exact path's parity alone."""
    m = KitagawaSSM(10.0, 1.0)
    _, ys = m.simulate(5, np.random.default_rng(9))
    ys = [float(y) for y in ys]
    for n in (1, 63, 512, 513, 4096, 65537):
        assert _gpu_vs_oracle(m, ys, n, 2, O.SYSTEMATIC, False, n + 1) >= (0 if n == 1 else 3)
