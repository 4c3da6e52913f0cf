"""metropolis_hastings(trace, proposal, proposal_args) with the Gaussian drift
proposal on every particle (src/inference/mh.jl:41-62; row a20).

CPU: the oracle's move (orc_pf_mh_drift) takes the proposal from its draws and
accepts exactly when log u < (scipy log-joint at the proposal) - (at the
current state), the drift's forward and backward scores cancelling; long
chains on every particle reproduce the conjugate posteriors of the regression
(quickstart.jl) and of a 1-D linear-Gaussian step.
GPU: gh_pf_mh_drift reproduces the oracle bit for bit (states, acceptance
counts) for the regression's selections, the LG-SSM and the nonlinear SSM
after several steps; invalid calls are refused.
"""
import numpy as np
import pytest
from scipy import stats

import gen_amd as gen
from gen_amd.models import BayesianLinearRegression, KitagawaSSM, LinearGaussianSSM
from oracle import oracle as O

S_MH = 6


def _lg1():
    return LinearGaussianSSM([[0.9]], [[0.5]], [[1.0]], [[0.8]], [0.0], [[1.0]])


def reg_joint(m, x, ys):
    return (stats.norm.logpdf(x[0], m.mu_s, m.sd_s) + stats.norm.logpdf(x[1], m.mu_i, m.sd_i)
            + stats.norm.logpdf(ys, x[0] * m.xs + x[1], m.sigma).sum())


def test_oracle_drift_acceptance_is_the_update_weight():
    m, ys = BayesianLinearRegression.quickstart()
    n, seed, sd = 64, 5, np.array([0.2, 1.5])
    pf = O.OraclePF(m, n, seed)
    pf.init(ys)
    x0 = pf.state().copy()
    acc = pf.mh_drift(3, sd, 1)
    x1 = pf.state()
    n_acc = 0
    for i in range(n):
        z = O.normals(seed, i, 1, S_MH, 2)  # move 0: stream MH, draws 0..
        y = x0[:, i] + sd * z
        w = O.philox([i & 0xFFFFFFFF, i >> 32, 1, (S_MH << 16) | 15], [seed & 0xFFFFFFFF, seed >> 32])
        u = (((w[0] >> 5) << 26) | (w[1] >> 6)) * 2.0**-53
        alpha = reg_joint(m, y, ys) - reg_joint(m, x0[:, i], ys)
        if abs(np.log(u) - alpha) < 1e-9:
            continue  # too close to call at double precision
        want = y if np.log(u) < alpha else x0[:, i]
        np.testing.assert_allclose(x1[:, i], want, rtol=0, atol=0)
        n_acc += np.log(u) < alpha
    assert acc == n_acc
    # a selection of one address drifts that component only
    pf2 = O.OraclePF(m, n, seed)
    pf2.init(ys)
    pf2.mh_drift(2, sd, 3)
    assert np.array_equal(pf2.state()[0], x0[0]) and not np.array_equal(pf2.state()[1], x0[1])


def test_oracle_drift_chains_reach_the_regression_posterior():
    m, ys = BayesianLinearRegression.quickstart()
    n = 512
    pf = O.OraclePF(m, n, 11)
    pf.init(ys)
    acc = pf.mh_drift(3, [0.15, 0.8], 1500)
    assert 0.15 * n * 1500 < acc < 0.9 * n * 1500
    mean, cov = m.posterior(ys)
    x = pf.state()
    assert np.all(np.abs(x.mean(axis=1) - mean) < 5 * np.sqrt(np.diag(cov) / n) + 0.02), (x.mean(axis=1), mean)
    np.testing.assert_allclose(np.cov(x), cov, rtol=0.25, atol=0.01)


def test_oracle_drift_chains_reach_the_filtering_posterior_lg1():
    """x_1 | y_1 of a 1-D LG model: N(P0 H (H P0 H + R)^-1 y, ...) (Kalman)."""
    m = _lg1()
    y1 = np.array([1.3])
    n = 1024
    pf = O.OraclePF(m, n, 3)
    pf.init(y1)
    pf.mh_drift(1, [0.8], 400)
    P0, H, R = m.P0[0, 0], m.H[0, 0], m.R[0, 0]
    k = P0 * H / (H * P0 * H + R)
    mean, var = m.mu0[0] + k * (y1[0] - H * m.mu0[0]), (1 - k * H) * P0
    x = pf.state()[0]
    assert abs(x.mean() - mean) < 5 * np.sqrt(var / n) + 0.01
    assert abs(x.var() - var) < 0.15 * var


def test_oracle_drift_refusals():
    from tests.test_scores import hmm

    h = hmm()
    pf = O.OraclePF(h, 16, 1)
    pf.init([0])
    with pytest.raises(RuntimeError):
        pf.mh_drift(1, [1.0], 1)  # a discrete latent
    m = _lg1()
    pf = O.OraclePF(m, 16, 1)
    pf.init([0.1])
    with pytest.raises(RuntimeError):
        pf.mh_drift(1, [0.0], 1)  # sd must be > 0


# ------------------------------------------------------------------ GPU
def _filters(m, ys, n, seed, steps):
    st = gen.initialize_particle_filter(m, (1,), ys[0], n, seed=seed)
    pf = O.OraclePF(m, n, seed)
    pf.init(ys[0])
    for t in range(2, steps + 1):
        gen.maybe_resample(st)
        pf.maybe_resample()
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), ys[t - 1])
        pf.step(ys[t - 1])
    return st, pf


@pytest.mark.gpu
@pytest.mark.parametrize("mask", [1, 2, 3])
def test_gpu_drift_regression_bitexact(gh_ctx, mask):
    m, ys = BayesianLinearRegression.quickstart()
    n, seed = 3001, 9
    st = gen.initialize_particle_filter(m, (m.xs,), m.constraints(ys), n, seed=seed)
    sel = {1: ("slope",), 2: ("intercept",), 3: ("slope", "intercept")}[mask]
    acc = gen.mh(st, gen.gaussian_drift, (gen.select(*sel), [0.2, 1.5]), 7)
    pf = O.OraclePF(m, n, seed)
    pf.init(ys)
    oacc = pf.mh_drift(mask, [0.2, 1.5], 7)
    assert acc == oacc
    assert np.array_equal(st.states().T.view(np.uint64), pf.state().view(np.uint64))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["lg4", "kit"])
def test_gpu_drift_ssm_bitexact(gh_ctx, name):
    m = LinearGaussianSSM.benchmark(4) if name == "lg4" else KitagawaSSM(10.0, 1.0)
    _, ys = m.simulate(5, np.random.default_rng(4))
    ys = list(ys)
    n, seed = 4099, 13
    st, pf = _filters(m, ys, n, seed, 4)
    sd = 0.3 if name == "lg4" else 1.0
    tr = gen.get_traces(st)
    before = tr.step_states(4).copy()
    score_before = tr.scores().copy()
    acc = gen.mh(st, gen.gaussian_drift, (gen.select(m.latent_address(4)), sd), n_moves=5)
    acc2 = gen.mh(st, gen.select(m.latent_address(4)), 2)  # then selection moves: fresh draw windows
    oacc = pf.mh_drift(1, np.full(m.d if name == "lg4" else 1, sd), 5)
    oacc2 = pf.mh_select(1, 2)
    assert (acc, acc2) == (oacc, oacc2)
    assert np.array_equal(st.states().T.view(np.uint64), pf.state().view(np.uint64))
    # the moved particles keep their weights
    assert np.array_equal(gen.get_log_weights(st).view(np.uint64), pf.log_weights().view(np.uint64))
    # a traces view taken before the moves reads the moved latents and scores
    assert np.array_equal(tr.step_states(4).T.view(np.uint64), pf.state().view(np.uint64))
    assert not np.array_equal(tr.step_states(4), before)
    assert not np.array_equal(tr.scores(), score_before)


@pytest.mark.gpu
def test_gpu_drift_refusals(gh_ctx):
    from tests.test_scores import hmm

    h = hmm()
    st = gen.initialize_particle_filter(h, (1,), [0], 64, seed=1)
    with pytest.raises(gen.GenHipError):
        gen.mh(st, gen.gaussian_drift, (gen.select(h.latent_address(1)), 1.0))
    m = _lg1()
    st = gen.initialize_particle_filter(m, (1,), [0.1], 64, seed=1)
    with pytest.raises(gen.GenHipError):
        gen.mh(st, gen.gaussian_drift, (gen.select(m.latent_address(1)), -1.0))
    gen.maybe_resample(st, 1e9)
    with pytest.raises(gen.GenHipError):  # after maybe_resample and before the next step
        gen.mh(st, gen.gaussian_drift, (gen.select(m.latent_address(1)), 0.5))
