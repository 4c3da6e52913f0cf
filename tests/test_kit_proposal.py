"""Custom proposal of the nonlinear SSM: the user-parameterised Gaussian
proposal q(x_t | x_{t-1}, y_t) = normal(alpha m + beta y_t + gamma, sigma_q)
(m the prior mean), with Gen's custom-proposal weight
log p(x_t | x_{t-1}) + log p(y_t | x_t) - log q(x_t)
(particle_filter.jl:79-91,139-154 via trace_translators.jl:775-802).

CPU: the oracle's weights against scipy's densities, the bootstrap special
case, log-ML agreement with the bootstrap filter.  GPU: bit-exact against the
oracle, arguments changing between steps, argument errors."""
import math

import numpy as np
import pytest
from scipy import stats

import gen_amd as gen
from oracle import oracle as O

Q = (0.8, 0.5, 0.1, 4.0)  # (alpha, beta, gamma, sigma_q)


def prior_mean(m, v, t):
    return v / 2 + 25 * v / (1 + v * v) + 8 * math.cos(1.2 * t)


def test_weights_are_the_custom_proposal_weights():
    m = gen.KitagawaSSM(10.0, 1.0)
    _, ys = m.simulate(3, np.random.default_rng(11))
    n = 257
    pf = O.OraclePF(m, n, 3)
    pf.set_proposal_args(Q)
    pf.init(ys[0], O.GAUSSIAN)
    x1 = pf.state()[0].copy()
    a, b, g, sq = Q
    mq = a * m.mu1 + b * ys[0] + g
    w1 = (stats.norm.logpdf(x1, m.mu1, m.s1) + stats.norm.logpdf(ys[0], x1 * x1 / 20, math.sqrt(m.var_y))
          - stats.norm.logpdf(x1, mq, sq))
    assert np.allclose(pf.log_weights(), w1, rtol=1e-12, atol=1e-11)
    # x1 ~ q: standardised draws are standard normal
    z = (x1 - mq) / sq
    assert abs(z.mean()) < 0.3 and abs(z.std() - 1) < 0.2
    pf.maybe_resample(0.0)  # ESS < 0 never holds: parents stay the identity
    pf.step(ys[1], O.GAUSSIAN)
    x2 = pf.state()[0]
    mean = prior_mean(m, x1, 2)
    mq2 = a * mean + b * ys[1] + g
    w2 = w1 + (stats.norm.logpdf(x2, mean, math.sqrt(m.var_x))
               + stats.norm.logpdf(ys[1], x2 * x2 / 20, math.sqrt(m.var_y)) - stats.norm.logpdf(x2, mq2, sq))
    assert np.allclose(pf.log_weights(), w2, rtol=1e-12, atol=1e-10)


def test_missing_observation_drops_the_data_term():
    m = gen.KitagawaSSM(10.0, 1.0)
    n = 64
    pf = O.OraclePF(m, n, 5)
    pf.set_proposal_args(Q)
    pf.init(None, O.GAUSSIAN)
    x1 = pf.state()[0]
    a, _, g, sq = Q
    mq = a * m.mu1 + g
    w = stats.norm.logpdf(x1, m.mu1, m.s1) - stats.norm.logpdf(x1, mq, sq)
    assert np.allclose(pf.log_weights(), w, rtol=1e-12, atol=1e-11)


def test_bootstrap_special_case():
    """alpha = 1, beta = gamma = 0, sigma_q = sqrt(var_x) draws exactly the
    prior's values; the weights equal the bootstrap weights up to rounding."""
    m = gen.KitagawaSSM(10.0, 1.0)
    _, ys = m.simulate(6, np.random.default_rng(12))
    n = 1000
    a = O.OraclePF(m, n, 8)
    b = O.OraclePF(m, n, 8)
    b.set_proposal_args((1.0, 0.0, 0.0, math.sqrt(m.var_x)))
    a.init(ys[0])
    # at t = 1 the prior is normal(mu1, s1): use sigma_q = s1 there
    b.set_proposal_args((1.0, 0.0, 0.0, m.s1))
    b.init(ys[0], O.GAUSSIAN)
    assert np.array_equal(a.state(), b.state())
    assert np.allclose(a.log_weights(), b.log_weights(), rtol=0, atol=1e-12)
    b.set_proposal_args((1.0, 0.0, 0.0, math.sqrt(m.var_x)))
    for y in ys[1:]:
        a.maybe_resample()
        b.maybe_resample()
        a.step(y)
        b.step(y, O.GAUSSIAN)
    assert np.array_equal(a.state(), b.state())
    assert np.allclose(a.log_weights(), b.log_weights(), rtol=0, atol=1e-10)


def test_log_ml_agrees_with_bootstrap():
    """Both filters estimate the same log p(y_1..T): their estimates at
    N = 2^14 agree within their Monte-Carlo spread."""
    m = gen.KitagawaSSM(10.0, 1.0)
    _, ys = m.simulate(15, np.random.default_rng(13))
    n = 1 << 14
    boot, cust = [], []
    for seed in range(3):
        boot.append(O.run_pf(m, ys, n, seed).log_ml_estimate())
        pf = O.OraclePF(m, n, seed)
        pf.set_proposal_args(Q)
        pf.init(ys[0], O.GAUSSIAN)
        for y in ys[1:]:
            pf.maybe_resample()
            pf.step(y, O.GAUSSIAN)
        cust.append(pf.log_ml_estimate())
    assert abs(np.mean(boot) - np.mean(cust)) < 1.0, (boot, cust)


def test_oracle_rejects_bad_arguments():
    m = gen.KitagawaSSM()
    pf = O.OraclePF(m, 10, 1)
    with pytest.raises(ValueError):
        pf.set_proposal_args((1.0, 0.0, 0.0, 0.0))
    with pytest.raises(ValueError):
        pf.init(np.array([0.3]), O.GAUSSIAN)  # no arguments set
    with pytest.raises(ValueError):
        O.OraclePF(gen.LinearGaussianSSM.benchmark(2), 10, 1).init(np.zeros(2), O.GAUSSIAN)


# ------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("n", [1000, 70001])
def test_gpu_gaussian_proposal_bitexact(gh_ctx, n):
    m = gen.KitagawaSSM(10.0, 1.0)
    _, ys = m.simulate(10, np.random.default_rng(14))
    ys = [y if t != 5 else None for t, y in enumerate(ys)]  # one step without an observation
    args = [Q if t % 4 else (1.0, 0.2, -0.3, 3.0) for t in range(len(ys))]  # arguments change between steps
    st = gen.initialize_particle_filter(m, (1,), {m.obs_address(1): ys[0]}, gen.GaussianProposal, args[0], n,
                                        seed=17)
    orc = O.OraclePF(m, n, 17)
    orc.set_proposal_args(args[0])
    orc.init(ys[0], O.GAUSSIAN)
    for t in range(2, len(ys) + 1):
        thr = n if t % 3 else None
        assert gen.maybe_resample(st, thr) == orc.maybe_resample(thr)[0]
        obs = {m.obs_address(t): ys[t - 1]} if ys[t - 1] is not None else {}
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), obs, gen.GaussianProposal, args[t - 1])
        orc.set_proposal_args(args[t - 1])
        orc.step(ys[t - 1], O.GAUSSIAN)
        assert np.array_equal(gen.get_log_weights(st).view(np.uint64), orc.log_weights().view(np.uint64)), t
        assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64)), t
        assert np.array_equal(st.parents, orc.parents()), t
    a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
    assert abs(a - b) <= 1e-9 * abs(b)


@pytest.mark.gpu
def test_gpu_gaussian_proposal_batched_run(gh_ctx):
    """run_particle_filter with a proposal: the library keeps the last arguments."""
    m = gen.KitagawaSSM(10.0, 1.0)
    _, ys = m.simulate(8, np.random.default_rng(15))
    n = 5000
    st = gen.initialize_particle_filter(m, (1,), {m.obs_address(1): ys[0]}, gen.GaussianProposal, Q, n, seed=4)
    gen.run_particle_filter(st, list(ys[1:]), proposal=gen.GaussianProposal, proposal_args=Q)
    orc = O.OraclePF(m, n, 4)
    orc.set_proposal_args(Q)
    orc.init(ys[0], O.GAUSSIAN)
    for y in ys[1:]:
        orc.maybe_resample()
        orc.step(y, O.GAUSSIAN)
    assert np.array_equal(st.states().T, orc.state())
    assert np.array_equal(st.parents, orc.parents())


@pytest.mark.gpu
def test_gpu_gaussian_proposal_argument_errors(gh_ctx):
    m = gen.KitagawaSSM(10.0, 1.0)
    with pytest.raises(gen.GenHipError):
        gen.initialize_particle_filter(m, (1,), {m.obs_address(1): 1.0}, gen.GaussianProposal, (1.0, 0.0, 0.0), 10)
    with pytest.raises(gen.GenHipError):
        gen.initialize_particle_filter(m, (1,), {m.obs_address(1): 1.0}, gen.GaussianProposal, (1.0, 0.0, 0.0, -1.0),
                                       10)
    lg = gen.LinearGaussianSSM.benchmark(2)
    with pytest.raises(gen.GenHipError):
        gen.initialize_particle_filter(lg, (1,), {lg.obs_address(1): np.zeros(2)}, gen.GaussianProposal, Q, 10)
