"""Config C1: Bayesian linear regression (examples/regression/quickstart.jl:3-9,
data :26-27) through importance sampling / resampling (importance.jl:20-108)
and rejuvenation moves.

The oracle is pinned by the conjugate answer: y ~ N(X m0, X S0 X' + I) gives
the exact log p(y), and the exact posterior of (slope, intercept).
CPU: oracle log-ML against the exact value; constraint handling of the host
mirror.  GPU: bit-exact against the oracle at the C1 size (N = 1000, seed 42);
log-ML at N = 2^22 within Monte-Carlo error of the exact value; MH
rejuvenation at t = 1 moves the particles to the exact posterior.
"""
import numpy as np
import pytest

import gen_amd as gen
from oracle import oracle as O


def _c1():
    return gen.BayesianLinearRegression.quickstart()


def test_oracle_is_log_ml_matches_conjugate():
    m, ys = _c1()
    exact = m.log_marginal(ys)
    ls = [O.importance_sampling(m, ys, 1 << 18, s)[2] for s in range(4)]
    assert abs(np.mean(ls) - exact) < 0.15
    # the weights are the data log-likelihood of the prior draws
    st, lnw, lml = O.importance_sampling(m, ys, 64, 3)
    X = np.stack([m.xs, np.ones_like(m.xs)], axis=1)
    mu = X @ st  # [n_data, 64]
    ll = (-0.5 * (np.asarray(ys)[:, None] - mu) ** 2 - 0.5 * np.log(2 * np.pi)).sum(0)
    w = ll - np.logaddexp.reduce(ll)
    assert np.allclose(lnw, w, atol=1e-9)


def test_regression_constraints_are_checked():
    m, ys = _c1()
    cm = gen.choicemap(*m.constraints(ys).items())
    assert np.array_equal(m.obs_from_choicemap(cm, 1), ys)
    with pytest.raises(gen.GenHipError):
        m.obs_from_choicemap(gen.choicemap(*m.constraints(ys[:3]).items()), 1)  # partial
    with pytest.raises(gen.GenHipError):
        m.obs_from_choicemap(gen.choicemap((("slope",), 1.0)), 1)
    with pytest.raises(gen.GenHipError):
        m.obs_from_choicemap(gen.choicemap((("y-11",), 1.0)), 1)
    with pytest.raises(ValueError):
        gen.BayesianLinearRegression(np.arange(33.0))


@pytest.mark.gpu
def test_gpu_c1_importance_sampling_bitexact(gh_ctx):
    m, ys = _c1()
    cm = m.constraints(ys)
    traces, lnw, lml = gen.importance_sampling(m, (m.xs,), cm, 1000, seed=42)
    ost, olnw, olml = O.importance_sampling(m, ys, 1000, 42)
    assert np.array_equal(traces.T.view(np.uint64), ost.view(np.uint64))
    assert np.allclose(lnw, olnw, rtol=0, atol=1e-12)
    assert abs(lml - olml) <= 1e-9 * abs(olml)
    tr, lml2 = gen.importance_resampling(m, (m.xs,), cm, 1000, seed=42)
    assert lml2 == lml and tr.shape == (2,)


@pytest.mark.gpu
def test_gpu_c1_large_n_log_ml_and_rejuvenation(gh_ctx):
    m, ys = _c1()
    exact = m.log_marginal(ys)
    _, _, lml = gen.importance_sampling(m, (m.xs,), m.constraints(ys), 1 << 22, seed=7)
    assert abs(lml - exact) < 0.1
    # rejuvenation at t = 1: independence MH from the prior targets the posterior
    n = 1 << 16
    st = gen.initialize_particle_filter(m, (m.xs,), m.constraints(ys), n, seed=5)
    acc = gen.rejuvenate(st, 30000)
    assert acc > 0
    x = st.states()  # [n, 2]
    mean, cov = m.posterior(ys)
    sd = np.sqrt(np.diag(cov))
    assert np.all(np.abs(x.mean(0) - mean) < 0.03 * sd)  # MC error ~ sd / 256
    assert np.allclose(np.cov(x.T), cov, rtol=0.05, atol=0)
    with pytest.raises(gen.GenHipError):
        gen.particle_filter_step(st, (2,), (gen.UnknownChange(),), None)


@pytest.mark.gpu
def test_gpu_regression_rejuvenation_bitexact(gh_ctx):
    m, ys = _c1()
    n = 3001
    st = gen.initialize_particle_filter(m, (m.xs,), m.constraints(ys), n, seed=13)
    orc = O.OraclePF(m, n, 13)
    orc.init(ys)
    # 4100 moves cross into the second block of MH streams (move 4096 onwards)
    assert gen.rejuvenate(st, 4090) + gen.rejuvenate(st, 10) == orc.rejuvenate(4090) + orc.rejuvenate(10)
    assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64))
    assert np.array_equal(gen.get_log_weights(st).view(np.uint64), orc.log_weights().view(np.uint64))


# ------------------------------------------------ mh(trace, select(...))
def test_oracle_single_address_mh_reaches_posterior():
    """The quickstart's inference loop (examples/regression/quickstart.jl:17-22):
    each iteration mh(trace, select(:slope)) then mh(trace, select(:intercept)),
    one independent chain per particle.  The chains' states reproduce the
    conjugate posterior; a move leaves the unselected address untouched."""
    m, ys = _c1()
    n = 1024
    orc = O.OraclePF(m, n, 21)
    orc.init(ys)
    x0 = orc.state().copy()
    orc.mh_select(1, 1)
    x1 = orc.state()
    assert np.array_equal(x1[1], x0[1]) and not np.array_equal(x1[0], x0[0])
    orc.mh_select(2, 1)
    assert np.array_equal(orc.state()[0], x1[0])
    for _ in range(2000):  # prior proposals on a correlated posterior: ~1000 sweeps to mix
        orc.mh_select(1, 1)
        orc.mh_select(2, 1)
    x = orc.state().T
    mean, cov = m.posterior(ys)
    sd = np.sqrt(np.diag(cov))
    assert np.all(np.abs(x.mean(0) - mean) < 0.15 * sd), (x.mean(0), mean)  # MC error ~ sd / 32
    assert np.allclose(np.sqrt(np.diag(np.cov(x.T))), sd, rtol=0.1)
    with pytest.raises(RuntimeError):
        orc.mh_select(4, 1)


@pytest.mark.gpu
def test_gpu_single_address_mh_bitexact(gh_ctx):
    m, ys = _c1()
    n = 3001
    st = gen.initialize_particle_filter(m, (m.xs,), m.constraints(ys), n, seed=17)
    orc = O.OraclePF(m, n, 17)
    orc.init(ys)
    for sel, mask in [(("slope",), 1), (("intercept",), 2), (("slope", "intercept"), 3), (("slope",), 1)]:
        assert gen.mh(st, gen.select(*sel), 3) == orc.mh_select(mask, 3)
        assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64))
    with pytest.raises(gen.GenHipError):
        gen.mh(st, gen.select("noise"))
    # the quickstart loop: slope, intercept alternately, 2000 iterations
    for _ in range(2000):
        gen.mh(st, gen.select("slope"))
        gen.mh(st, gen.select("intercept"))
    x = st.states()
    mean, cov = m.posterior(ys)
    assert np.all(np.abs(x.mean(0) - mean) < 0.12 * np.sqrt(np.diag(cov)))
