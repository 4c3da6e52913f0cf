"""Pin the oracle's linear-Gaussian weight and transition path (CPU only).

The C2 headline filter's arithmetic in oracle/gh_oracle.c is checked against
densities and samplers written independently of it:
  * the per-particle weight increments (Gen's generate/update weight of the
    constrained :y, src/static_ir/generate.jl:31-34 with the mvnormal logpdf of
    src/modeling_library/distributions/mvnormal.jl:12-16) equal
    scipy.stats.multivariate_normal.logpdf(y; H x + c, R) to 1e-12;
  * the latent draws are mvnormal(A x_prev + b, Q) (mvnormal.jl:30-33) built
    from the oracle's own standard normals with numpy's Cholesky of Q;
  * the log-ML estimate of the seeded d = 10 fixture (tests/golden/kalman.json
    "lg10", exact Kalman value) at N = 2^17 is within Monte-Carlo error over
    several seeds.
Both the structured C2 model (LGModel<10,3>: diagonal chol(Q), H = I) and a
dense random model (no exact zeros; b, c non-zero) are covered.
"""
import json
import os

import numpy as np
import pytest
from scipy import stats

from gen_amd.models import LinearGaussianSSM
from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")
STREAM_INIT, STREAM_STEP = 1, 2


def dense_model(d=5, dy=3, seed=11):
    rng = np.random.default_rng(seed)
    A = 0.3 * rng.standard_normal((d, d))
    G = rng.standard_normal((d, d))
    Q = G @ G.T / d + 0.2 * np.eye(d)
    H = rng.standard_normal((dy, d))
    F = rng.standard_normal((dy, dy))
    R = F @ F.T / dy + 0.3 * np.eye(dy)
    P = rng.standard_normal((d, d))
    P0 = P @ P.T / d + 0.5 * np.eye(d)
    return LinearGaussianSSM(A, Q, H, R, rng.standard_normal(d), P0, b=rng.standard_normal(d),
                             c=rng.standard_normal(dy))


MODELS = {"c2_d10": lambda: LinearGaussianSSM.benchmark(10), "dense_d5_dy3": dense_model}


@pytest.mark.parametrize("name", sorted(MODELS))
def test_weights_equal_scipy_mvnormal(name):
    m = MODELS[name]()
    _, ys = m.simulate(3, np.random.default_rng(7))
    n, seed = 64, 1234
    pf = O.OraclePF(m, n, seed)
    pf.init(ys[0])
    x1 = pf.state()                      # [d][n]
    w1 = pf.log_weights()
    want1 = np.array([stats.multivariate_normal.logpdf(ys[0], m.H @ x1[:, i] + m.c, m.R) for i in range(n)])
    np.testing.assert_allclose(w1, want1, rtol=1e-12, atol=1e-12)
    # x_1 = mu0 + chol(P0) z, z the oracle's INIT-stream normals of particle i
    L0 = np.linalg.cholesky(m.P0)
    for i in range(n):
        z = O.normals(seed, i, 1, STREAM_INIT, m.d)
        np.testing.assert_allclose(x1[:, i], m.mu0 + L0 @ z, rtol=0, atol=1e-12)
    # a step without resampling (threshold 0 never fires): the increment is the
    # new observation's logpdf, the latent mvnormal(A x_prev + b, Q)
    did, _ = pf.maybe_resample(0.0)
    assert not did
    pf.step(ys[1])
    x2 = pf.state()
    inc = pf.log_weights() - w1
    want2 = np.array([stats.multivariate_normal.logpdf(ys[1], m.H @ x2[:, i] + m.c, m.R) for i in range(n)])
    np.testing.assert_allclose(inc, want2, rtol=1e-12, atol=1e-11)
    LQ = np.linalg.cholesky(m.Q)
    for i in range(n):
        z = O.normals(seed, i, 2, STREAM_STEP, m.d)
        np.testing.assert_allclose(x2[:, i], m.A @ x1[:, i] + m.b + LQ @ z, rtol=0, atol=1e-12)
    # a step with no observation adds nothing (the :y choice is unconstrained)
    pf.maybe_resample(0.0)
    pf.step(None)
    np.testing.assert_array_equal(pf.log_weights(), w1 + inc)


def test_resampled_weights_restart_from_scipy_increment():
    """After a resample the weights are 0 (particle_filter.jl:204) and the next
    step's weight is exactly the new increment; log_ml_est absorbs L - log N."""
    m = LinearGaussianSSM.benchmark(10)
    _, ys = m.simulate(2, np.random.default_rng(8))
    n = 256
    pf = O.OraclePF(m, n, 5)
    pf.init(ys[0])
    w1 = pf.log_weights()
    mx = w1.max()
    L = mx + np.log(np.exp(w1 - mx).sum())
    did, ess = pf.maybe_resample(n + 1.0)
    assert did
    assert ess == pytest.approx(np.exp(2 * L - (mx * 2 + np.log(np.exp(2 * (w1 - mx)).sum()))), rel=1e-12)
    pf.step(ys[1])
    x2 = pf.state()
    want = np.array([stats.multivariate_normal.logpdf(ys[1], m.H @ x2[:, i] + m.c, m.R) for i in range(n)])
    np.testing.assert_allclose(pf.log_weights(), want, rtol=1e-12, atol=1e-11)
    lw = pf.log_weights()
    mx2 = lw.max()
    expect = (L - np.log(n)) + (mx2 + np.log(np.exp(lw - mx2).sum()) - np.log(n))
    assert pf.log_ml_estimate() == pytest.approx(expect, rel=1e-12)


def test_lg10_fixture_log_ml_within_monte_carlo_error():
    """The seeded C2-shape fixture (d = 10, T = 100): 8 oracle runs at
    N = 2^17.  The particle filter's Z estimate is unbiased, so log Z-hat is
    biased low; at this N the bias is about -1.05 with a spread of ~0.5
    (measured over 16 runs) and
    log Z-hat is skewed to the left, so the mean + var/2 correction of a
    normal log Z-hat does not hold here.  The mean sits in [-2.5, 0.5] of the
    exact Kalman log-ML and no run above it by more than 4 spreads."""
    k = json.load(open(os.path.join(GOLD, "kalman.json")))["lg10"]
    d = k["d"]
    m = LinearGaussianSSM(np.array(k["A"]), 0.1 * np.eye(d), np.eye(d), 0.5 * np.eye(d), np.zeros(d), np.eye(d))
    ys = np.array(k["ys"])
    assert m.kalman_log_marginal(ys) == pytest.approx(k["log_ml"], rel=1e-12)
    from concurrent.futures import ThreadPoolExecutor  # ctypes calls release the GIL

    with ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        ests = np.array(list(ex.map(
            lambda s: O.run_pf(m, ys, 1 << 17, s, record_history=False).log_ml_estimate(), range(8))))
    var = ests.var(ddof=1)
    assert np.sqrt(var) < 2.0, ests
    assert -2.5 < ests.mean() - k["log_ml"] < 0.5, (ests, k["log_ml"])
    assert ests.max() < k["log_ml"] + 4 * np.sqrt(var), ests
