"""User-parameterised custom proposal of the linear-Gaussian SSM:
q(x_t | x_{t-1}) = mvnormal(P x_{t-1} + u_t, Sigma_q) (t = 1: mvnormal(u_1, Sigma_q)),
proposal_args (P, Sigma_q, u) or (u,) per step, with Gen's custom-proposal
weight log p(x_t | x_{t-1}) + log p(y_t | x_t) - log q(x_t)
(particle_filter.jl:79-91,139-154 via trace_translators.jl:775-802).

CPU: the oracle's weights against scipy's multivariate-normal densities, its
draws are q's (whitened residuals standard normal), the proposal equal to the
prior reproduces the bootstrap filter's states and weights.
GPU: bit-exact against the oracle with arguments changing between steps (full and u-only forms), a step without observation, a
parameter change on top, argument errors."""
import numpy as np
import pytest
from scipy import stats

import gen_amd as gen
from oracle import oracle as O
from tests.test_oracle_lg_pins import dense_model


def _args(m, rng, scale=1.0):
    d = m.d
    P = 0.7 * m.A + 0.05 * rng.standard_normal((d, d))
    G = rng.standard_normal((d, d))
    S = scale * (0.3 * m.Q + 0.05 * G @ G.T)
    u = 0.2 * rng.standard_normal(d)
    return P, S, u


def _flat(*a):
    return np.concatenate([np.asarray(x, dtype=np.float64).ravel() for x in a])


def test_oracle_weights_are_the_custom_proposal_weights():
    m = dense_model()
    _, ys = m.simulate(3, np.random.default_rng(11))
    n = 300
    rng = np.random.default_rng(1)
    P, S, u1 = _args(m, rng)
    pf = O.OraclePF(m, n, 3)
    pf.set_proposal_args(_flat(P, S, u1))
    pf.init(ys[0], O.LINEAR)
    x1 = pf.state().copy()  # [d, n]
    w1 = np.array([stats.multivariate_normal.logpdf(x1[:, i], m.mu0, m.P0)
                   + stats.multivariate_normal.logpdf(ys[0], m.H @ x1[:, i] + m.c, m.R)
                   - stats.multivariate_normal.logpdf(x1[:, i], u1, S) for i in range(n)])
    np.testing.assert_allclose(pf.log_weights(), w1, rtol=1e-11, atol=1e-10)
    r = np.linalg.solve(np.linalg.cholesky(S), x1 - u1[:, None])
    for c in range(m.d):
        assert stats.kstest(r[c], "norm").pvalue > 1e-4
    u2 = np.array([0.3, -0.1, 0.2][: m.d] + [0.0] * max(0, m.d - 3))
    pf.set_proposal_args(u2)  # u alone: P and Sigma_q kept
    pf.maybe_resample(0.0)  # no resample: particle i's parent is i
    pf.step(ys[1], O.LINEAR)
    x2 = pf.state()
    w2 = w1 + np.array([stats.multivariate_normal.logpdf(x2[:, i], m.A @ x1[:, i] + m.b, m.Q)
                        + stats.multivariate_normal.logpdf(ys[1], m.H @ x2[:, i] + m.c, m.R)
                        - stats.multivariate_normal.logpdf(x2[:, i], P @ x1[:, i] + u2, S) for i in range(n)])
    np.testing.assert_allclose(pf.log_weights(), w2, rtol=1e-11, atol=1e-9)


def test_oracle_prior_as_proposal_is_the_bootstrap_filter():
    """q = the prior (P = A, u_t = b, Sigma_q = Q; t = 1: u = mu0, Sigma_q = P0
    needs its own arguments) draws the same latents as the bootstrap filter
    (same normals, x = mean + L z) and the weights agree to rounding."""
    m = gen.LinearGaussianSSM.benchmark(4)
    _, ys = m.simulate(5, np.random.default_rng(2))
    n = 500
    boot = O.run_pf(m, ys, n, 9, thr=0.0)
    pf = O.OraclePF(m, n, 9)
    pf.set_proposal_args(_flat(m.A, m.P0, m.mu0))
    pf.init(ys[0], O.LINEAR)
    pf.set_proposal_args(_flat(m.A, m.Q, m.b))
    for y in ys[1:]:
        pf.maybe_resample(0.0)
        pf.step(y, O.LINEAR)
    np.testing.assert_allclose(pf.state(), boot.state(), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(pf.log_weights(), boot.log_weights(), rtol=1e-10, atol=1e-9)


def test_oracle_refuses_bad_arguments():
    m = gen.LinearGaussianSSM.benchmark(2)
    pf = O.OraclePF(m, 10, 1)
    with pytest.raises(ValueError):
        pf.set_proposal_args(np.zeros(2))  # u alone before P, Sigma_q
    with pytest.raises(ValueError):
        pf.set_proposal_args(_flat(np.eye(2), -np.eye(2), np.zeros(2)))  # Sigma_q not PD
    with pytest.raises(ValueError):
        pf.init(np.zeros(2), O.LINEAR)  # no arguments yet


# ------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["dense", "lg10"])
def test_gpu_linear_proposal_bitexact(gh_ctx, name):
    m = dense_model() if name == "dense" else gen.LinearGaussianSSM.benchmark(10)
    _, ys = m.simulate(9, np.random.default_rng(14))
    ys = [y if t != 4 else None for t, y in enumerate(ys)]  # one step without an observation
    rng = np.random.default_rng(5)
    full = [_flat(*_args(m, rng, 1.0 + 0.5 * (t % 3))) for t in range(len(ys))]
    n, seed = 20011, 17
    st = gen.initialize_particle_filter(m, (1,), {m.obs_address(1): ys[0]}, gen.LinearGaussianProposal,
                                        (full[0],), n, seed=seed)
    orc = O.OraclePF(m, n, seed)
    orc.set_proposal_args(full[0])
    orc.init(ys[0], O.LINEAR)
    for t in range(2, len(ys) + 1):
        thr = n if t % 3 else None
        assert gen.maybe_resample(st, thr) == orc.maybe_resample(thr)[0]
        # full arguments on even steps, u alone on odd ones
        args = (full[t - 1],) if t % 2 == 0 else (full[t - 1][-m.d:],)
        obs = {m.obs_address(t): ys[t - 1]} if ys[t - 1] is not None else {}
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), obs, gen.LinearGaussianProposal, args)
        orc.set_proposal_args(args[0])
        orc.step(ys[t - 1], O.LINEAR)
        assert np.array_equal(gen.get_log_weights(st).view(np.uint64), orc.log_weights().view(np.uint64)), t
        assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64)), t
        assert np.array_equal(st.parents, orc.parents()), t
    a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
    assert abs(a - b) <= 1e-9 * abs(b)
    # the trace scores are the model's, whatever proposal made the particles
    assert np.array_equal(gen.get_traces(st).scores().view(np.uint64), orc.scores().view(np.uint64))
    # a parameter change on top: the filter keeps its proposal arguments
    m2 = gen.LinearGaussianSSM(0.8 * m.A, 1.5 * m.Q, m.H, 0.7 * m.R, m.mu0, m.P0, b=m.b, c=m.c)
    t = len(ys) + 1
    gen.particle_filter_step(st, (t, m2), (gen.UnknownChange(), gen.UnknownChange()), {m.obs_address(t): ys[1]},
                             gen.LinearGaussianProposal)
    orc.step_params(m2, ys[1], O.LINEAR)
    assert np.array_equal(gen.get_log_weights(st).view(np.uint64), orc.log_weights().view(np.uint64))
    assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64))
    st.close()


@pytest.mark.gpu
def test_gpu_linear_proposal_argument_errors(gh_ctx):
    m = gen.LinearGaussianSSM.benchmark(2)
    y = {m.obs_address(1): np.zeros(2)}
    with pytest.raises(gen.GenHipError):  # u alone at init
        gen.initialize_particle_filter(m, (1,), y, gen.LinearGaussianProposal, (np.zeros(2),), 10)
    with pytest.raises(gen.GenHipError):  # Sigma_q not positive definite
        gen.initialize_particle_filter(m, (1,), y, gen.LinearGaussianProposal,
                                       (np.eye(2), -np.eye(2), np.zeros(2)), 10)
    k = gen.KitagawaSSM(10.0, 1.0)
    with pytest.raises(gen.GenHipError):  # an LG-SSM proposal
        gen.initialize_particle_filter(k, (1,), {k.obs_address(1): 1.0}, gen.LinearGaussianProposal,
                                       (np.eye(1), np.eye(1), np.zeros(1)), 10)
