"""simulate(model, (T,)) (src/static_ir/simulate.jl:23-34, 50-83; unfold/simulate.jl).

CPU: the oracle's simulate (orc_simulate) records, per choice, the logpdf of
the value it sampled: every per-step score equals the scipy density of that
choice given its parents (mvnormal.jl:12-16, normal.jl:56-60, categorical.jl),
and get_score equals the host log-joint; the sampled values follow the
model's distributions (moment / KS / chi-square checks); trace i does not
depend on the number of traces.
GPU: gh_simulate reproduces the oracle bit for bit, and the trace accessors
read the same values.
"""
import numpy as np
import pytest
from scipy import stats

import gen_amd as gen
from gen_amd.models import BayesianLinearRegression, DiscreteHMM, KitagawaSSM, LinearGaussianSSM
from oracle import oracle as O
from tests.test_oracle_lg_pins import dense_model


def hmm():
    prior = np.array([0.2, 0.3, 0.5])
    T = np.array([[0.1, 0.2, 0.7], [0.2, 0.7, 0.1], [0.7, 0.2, 0.1]]).T
    E = np.array([[0.9, 0.05, 0.05], [0.05, 0.9, 0.05], [0.05, 0.05, 0.9]]).T
    return DiscreteHMM(prior, T, E)


def regression():
    m, _ = BayesianLinearRegression.quickstart()
    return m


MODELS = {
    "lg4": (lambda: LinearGaussianSSM.benchmark(4), 6),
    "lg10": (lambda: LinearGaussianSSM.benchmark(10), 4),
    "lg_dense": (dense_model, 5),
    "kitagawa": (lambda: KitagawaSSM(10.0, 1.0), 7),
    "hmm": (hmm, 6),
    "regression": (regression, 1),
}


def step_scores(m, x, y, xp, t):
    """scipy densities of one step's latent and observation choices."""
    if isinstance(m, LinearGaussianSSM):
        mean, cov = (m.mu0, m.P0) if t == 1 else (m.A @ xp + m.b, m.Q)
        return (stats.multivariate_normal.logpdf(x, mean, cov),
                stats.multivariate_normal.logpdf(y, m.H @ x + m.c, m.R))
    if isinstance(m, KitagawaSSM):
        if t == 1:
            lat = stats.norm.logpdf(x[0], m.mu1, m.s1)
        else:
            v = xp[0]
            lat = stats.norm.logpdf(x[0], v / 2 + 25 * v / (1 + v * v) + 8 * np.cos(1.2 * t), np.sqrt(m.var_x))
        return lat, stats.norm.logpdf(y[0], x[0] ** 2 / 20.0, np.sqrt(m.var_y))
    if isinstance(m, DiscreteHMM):
        z = int(x[0])
        lat = np.log(m.prior[z] if t == 1 else m.T[z, int(xp[0])])
        return lat, np.log(m.E[int(y[0]), z])
    lat = stats.norm.logpdf(x[0], m.mu_s, m.sd_s) + stats.norm.logpdf(x[1], m.mu_i, m.sd_i)
    return lat, stats.norm.logpdf(y, x[0] * m.xs + x[1], m.sigma).sum()


@pytest.mark.parametrize("name", list(MODELS))
def test_oracle_simulate_scores_are_scipy_logpdfs(name):
    make, T = MODELS[name]
    m = make()
    n = 40
    xs, ys, ps, tot = O.simulate(m, T, n, seed=3)
    for i in range(n):
        for t in range(1, T + 1):
            lat, ob = step_scores(m, xs[t - 1, :, i], ys[t - 1, :, i], xs[t - 2, :, i] if t > 1 else None, t)
            assert ps[t - 1, 0, i] == pytest.approx(lat, rel=1e-11, abs=1e-10), (t, i)
            assert ps[t - 1, 1, i] == pytest.approx(ob, rel=1e-11, abs=1e-10), (t, i)
        # get_score = the host log-joint of the trace's choices
        if isinstance(m, LinearGaussianSSM):
            want = m.log_joint(xs[:, :, i], list(ys[:, :, i]))
        elif isinstance(m, KitagawaSSM):
            want = m.log_joint(xs[:, 0, i], list(ys[:, 0, i]))
        elif isinstance(m, DiscreteHMM):
            want = m.log_joint(xs[:, 0, i], list(ys[:, :, i]))
        else:
            want = m.log_joint(xs[0, :, i], ys[0, :, i])
        assert tot[i] == pytest.approx(want, rel=1e-11, abs=1e-9)
    np.testing.assert_allclose(ps.sum(axis=(0, 1)), tot, rtol=1e-12, atol=1e-10)


@pytest.mark.parametrize("name", ["lg_dense", "hmm"])
def test_oracle_simulate_is_independent_of_n(name):
    make, T = MODELS[name]
    m = make()
    a = O.simulate(m, T, 7, seed=11)
    b = O.simulate(m, T, 30, seed=11)
    for u, v in zip(a, b):
        assert np.array_equal(u, v[..., :7])


def test_oracle_simulate_distributions():
    n = 20000
    # LG-SSM: x_1 ~ N(mu0, P0); y_t - H x_t - c ~ N(0, R)  (whitened: chi-square with dy dof)
    m = dense_model()
    xs, ys, _, _ = O.simulate(m, 2, n, seed=5)
    x1 = xs[0].T
    np.testing.assert_allclose(x1.mean(0), m.mu0, atol=5 * np.sqrt(np.diag(m.P0).max() / n))
    np.testing.assert_allclose(np.cov(x1.T), m.P0, atol=0.06 * np.abs(m.P0).max())
    LR = np.linalg.cholesky(m.R)
    r = np.linalg.solve(LR, ys[1] - (m.H @ xs[1]) - m.c[:, None])
    assert stats.kstest((r**2).sum(0), stats.chi2(m.dy).cdf).pvalue > 1e-3
    # x_2 | x_1 ~ N(A x_1 + b, Q)
    LQ = np.linalg.cholesky(m.Q)
    e = np.linalg.solve(LQ, xs[1] - (m.A @ xs[0]) - m.b[:, None])
    assert stats.kstest((e**2).sum(0), stats.chi2(m.d).cdf).pvalue > 1e-3
    # Kitagawa: y - x^2/20 ~ N(0, sqrt(var_y)); x_1 ~ N(mu1, s1)
    k = KitagawaSSM(10.0, 2.0)
    xs, ys, _, _ = O.simulate(k, 3, n, seed=6)
    assert stats.kstest(ys[2, 0] - xs[2, 0] ** 2 / 20.0, stats.norm(0, np.sqrt(2.0)).cdf).pvalue > 1e-3
    assert stats.kstest(xs[0, 0], stats.norm(k.mu1, k.s1).cdf).pvalue > 1e-3
    # HMM: z_1 ~ prior, x_t | z_t ~ E[:, z_t]
    h = hmm()
    xs, ys, _, _ = O.simulate(h, 2, n, seed=7)
    z1 = xs[0, 0].astype(int)
    assert stats.chisquare(np.bincount(z1, minlength=3), h.prior * n).pvalue > 1e-3
    for z in range(3):
        sel = xs[1, 0].astype(int) == z
        assert stats.chisquare(np.bincount(ys[1, 0, sel].astype(int), minlength=3),
                               h.E[:, z] * sel.sum()).pvalue > 1e-3
    # regression: y_i - (slope x_i + intercept) ~ N(0, sigma)
    r = regression()
    xs, ys, _, _ = O.simulate(r, 1, n, seed=8)
    res = ys[0] - (xs[0, 0][None, :] * r.xs[:, None] + xs[0, 1][None, :])
    assert stats.kstest(res.ravel(), stats.norm(0, r.sigma).cdf).pvalue > 1e-3
    assert stats.kstest(xs[0, 0], stats.norm(r.mu_s, r.sd_s).cdf).pvalue > 1e-3


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", list(MODELS))
def test_gpu_simulate_bitexact(gh_ctx, name):
    make, T = MODELS[name]
    m = make()
    n = 3001
    tr = gen.simulate(m, () if m.static else (T,), num_traces=n, seed=13)
    xs, ys, ps, tot = O.simulate(m, T, n, seed=13)
    for got, want in ((tr.xs, xs), (tr.ys, ys), (tr.per_step, ps), (tr.total, tot)):
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
    one = tr[17]
    assert one.get_score() == tot[17]
    cm = one.get_choices()
    if m.static:
        assert cm[("slope",)] == xs[0, 0, 17] and cm[m.y_address(2)] == ys[0, 1, 17]
        assert one.project(gen.select("slope", "intercept")) == pytest.approx(ps[0, 0, 17], rel=1e-12)
    else:
        assert np.all(np.atleast_1d(cm[m.latent_address(T)]) == xs[T - 1, :, 17])
        assert np.all(np.atleast_1d(cm[m.obs_address(1)]) == ys[0, :, 17])
        sel = gen.select(m.latent_address(1), m.obs_address(T))
        assert one.project(sel) == pytest.approx(ps[0, 0, 17] + ps[T - 1, 1, 17], rel=1e-15)


@pytest.mark.gpu
def test_gpu_simulate_single_trace_and_errors(gh_ctx):
    m = KitagawaSSM(10.0, 1.0)
    one = gen.simulate(m, (4,), seed=2)
    xs, ys, ps, tot = O.simulate(m, 4, 1, seed=2)
    assert one.get_score() == tot[0] and one.get_args() == (4,)
    assert one[m.obs_address(3)] == ys[2, 0, 0]
    with pytest.raises(gen.GenHipError):
        gen.simulate(m, (0,), num_traces=4)
    # the simulated observations drive a filter whose log-ML matches the oracle's
    obs = [float(y) for y in ys[:, 0, 0]]
    st = gen.initialize_particle_filter(m, (1,), obs[0], 4096, seed=1)
    for t, y in enumerate(obs[1:], start=2):
        gen.maybe_resample(st)
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), y)
    ref = O.run_pf(m, obs, 4096, 1)
    assert gen.log_ml_estimate(st) == pytest.approx(ref.log_ml_estimate(), abs=1e-9)
