"""Trace score columns: get_score / per-choice scores (src/static_ir/trace.jl:91-129).

CPU: the oracle's score columns (orc_pf_get_scores: the model's densities
along each particle's genealogy) equal the host log-joint of the materialised
trajectories (models.py log_joint: numpy Cholesky mvnormal, normal.jl,
categorical.jl), per step and in total, for every family, across resamples,
a pending resample and a missing observation.
GPU: gh_pf_get_scores reproduces the oracle bit for bit, and the Python trace
views read it (get_score, project).
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


def family_cases():
    out = []
    m = LinearGaussianSSM.benchmark(4)
    _, ys = m.simulate(6, np.random.default_rng(1))
    out.append(("lg4", m, list(ys)))
    m = dense_model()
    _, ys = m.simulate(6, np.random.default_rng(2))
    ys = list(ys)
    ys[3] = None  # a step without observation: its :y is not a choice of the trace
    out.append(("lg_dense", m, ys))
    m = KitagawaSSM(10.0, 1.0)
    _, ys = m.simulate(7, np.random.default_rng(3))
    out.append(("kitagawa", m, [float(y) for y in ys]))
    h = hmm()
    out.append(("hmm", h, [[0], [1], [2], [2], [1], [0]]))
    return out


CASES = family_cases()


def run_oracle(m, ys, n, seed, pending=False):
    pf = O.OraclePF(m, n, seed)
    pf.init(ys[0])
    for y in ys[1:]:
        pf.maybe_resample(n * 0.9)  # resample often: the genealogy matters
        pf.step(y)
    if pending:
        pf.maybe_resample(n + 1)
    return pf


def host_scores(m, pf, ys, pending=False):
    """log_joint of every particle's trajectory (the host restatement); after
    a resample the particles' traces are their parents' (particle_filter.jl:202-206)."""
    T = len(ys)
    traj = np.stack([pf.trajectory(t) for t in range(1, T + 1)])  # [T, d, n]
    if pending:
        traj = traj[:, :, pf.parents()]
    out = []
    for i in range(traj.shape[2]):
        xs = traj[:, :, i]
        if isinstance(m, LinearGaussianSSM):
            out.append(m.log_joint(xs, ys))
        elif isinstance(m, KitagawaSSM):
            out.append(m.log_joint(xs[:, 0], ys))
        else:
            out.append(m.log_joint(xs[:, 0], [y[0] if y is not None else None for y in ys]))
    return np.array(out)


@pytest.mark.parametrize("case", range(len(CASES)), ids=[c[0] for c in CASES])
@pytest.mark.parametrize("pending", [False, True])
def test_oracle_scores_equal_host_log_joint(case, pending):
    name, m, ys = CASES[case]
    pf = run_oracle(m, ys, 200, 7, pending)
    tot, ps = pf.scores(per_step=True)
    want = host_scores(m, pf, ys, pending)
    np.testing.assert_allclose(tot, want, rtol=1e-11, atol=1e-9)
    np.testing.assert_allclose(ps.sum(axis=(0, 1)), tot, rtol=1e-12, atol=1e-10)
    # an unobserved step contributes no observation score
    for t, y in enumerate(ys):
        if y is None:
            assert not ps[t, 1].any()


def test_oracle_lg_step_scores_are_mvnormal_logpdfs():
    m = dense_model()
    _, ys = m.simulate(3, np.random.default_rng(5))
    pf = run_oracle(m, list(ys), 50, 3)
    _, ps = pf.scores(per_step=True)
    x1, x2, x3 = (pf.trajectory(t) for t in (1, 2, 3))
    for i in range(50):
        assert ps[0, 0, i] == pytest.approx(stats.multivariate_normal.logpdf(x1[:, i], m.mu0, m.P0), rel=1e-12)
        assert ps[2, 0, i] == pytest.approx(
            stats.multivariate_normal.logpdf(x3[:, i], m.A @ x2[:, i] + m.b, m.Q), rel=1e-12)
        assert ps[2, 1, i] == pytest.approx(
            stats.multivariate_normal.logpdf(ys[2], m.H @ x3[:, i] + m.c, m.R), rel=1e-12)


def test_oracle_regression_scores():
    m, ys = BayesianLinearRegression.quickstart()
    pf = O.OraclePF(m, 64, 9)
    pf.init(ys)
    pf.mh_select(1, 5)
    tot = pf.scores()
    x = pf.state()
    want = [m.log_joint(x[:, i], ys) for i in range(64)]
    np.testing.assert_allclose(tot, want, rtol=1e-12)


# ------------------------------------------------------------------ GPU
def gpu_filter(m, ys, n, seed, pending=False):
    st = gen.initialize_particle_filter(m, (1,), ys[0], n, seed=seed)
    for t, y in enumerate(ys[1:], start=2):
        gen.maybe_resample(st, n * 0.9)
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), y)
    if pending:
        gen.maybe_resample(st, n + 1)
    return st


@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(CASES)), ids=[c[0] for c in CASES])
@pytest.mark.parametrize("pending", [False, True])
def test_gpu_scores_bitexact(gh_ctx, case, pending):
    name, m, ys = CASES[case]
    n = 3001
    st = gpu_filter(m, ys, n, 11, pending)
    pf = run_oracle(m, ys, n, 11, pending)
    tr = gen.get_traces(st)
    tot, ps = tr.scores(per_step=True)
    otot, ops = pf.scores(per_step=True)
    assert np.array_equal(tot.view(np.uint64), otot.view(np.uint64))
    assert np.array_equal(ps.view(np.uint64), ops.view(np.uint64))
    assert tr[17].get_score() == otot[17]
    T = len(ys)
    sel = gen.select(m.latent_address(T), m.latent_address(1))
    assert tr[5].project(sel) == pytest.approx(ops[T - 1, 0, 5] + ops[0, 0, 5], rel=1e-15)


@pytest.mark.gpu
def test_gpu_regression_scores_bitexact(gh_ctx):
    m, ys = BayesianLinearRegression.quickstart()
    n = 1000
    st = gen.initialize_particle_filter(m, (m.xs,), m.constraints(ys), n, seed=9)
    gen.mh(st, gen.select("slope"), 5)
    pf = O.OraclePF(m, n, 9)
    pf.init(ys)
    pf.mh_select(1, 5)
    tot = gen.get_traces(st).scores()
    assert np.array_equal(tot.view(np.uint64), pf.scores().view(np.uint64))
    tr = gen.get_traces(st)[3]
    want = stats.norm.logpdf(tr[("slope",)], m.mu_s, m.sd_s)
    assert tr.project(gen.select("slope")) == pytest.approx(want, rel=1e-12)
