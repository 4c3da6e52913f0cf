"""particle_filter_step! with changed model parameters (new_args with an
UnknownChange() argdiff on them; src/inference/particle_filter.jl:162-180).

Gen's Unfold update re-visits every retained kernel application when its
parameters change (src/modeling_library/unfold/generic_update.jl:9-16); with no
new constraints on them each contributes new score - old score, and the new
application is generated under the new parameters.  So a particle's weight
after the step is (its weight, or 0 after a resample) + log p'(y_t | x_t) +
log p'(x_1..t-1, y_1..t-1) - log p(x_1..t-1, y_1..t-1) along its trajectory.

CPU: the oracle (orc_pf_step_params) against that formula evaluated by the
host log-joint restatements (models.py, scipy-pinned in tests/test_scores.py),
with and without a pending resample, for the three Unfold families; the new
step's transition is the new one (whitened residuals standard normal).
GPU: gh_pf_step_params bit-exact against the oracle (states, weights,
parents, later steps and resamples under the new parameters).
"""
import numpy as np
import pytest
from scipy import stats

import gen_amd as gen
from gen_amd.models import DiscreteHMM, KitagawaSSM, LinearGaussianSSM
from oracle import oracle as O
from tests.test_oracle_lg_pins import dense_model


def _hmm(p):
    prior = np.array([0.2, 0.3, 0.5])
    T = np.array([[0.1, 0.2, 0.7], [0.2, 0.7, 0.1], [0.7, 0.2, 0.1]]).T
    E = np.array([[0.9, 0.05, 0.05], [0.05, 0.9, 0.05], [0.05, 0.05, 0.9]]).T
    if p:
        T = np.array([[0.3, 0.3, 0.4], [0.5, 0.4, 0.1], [0.2, 0.2, 0.6]]).T
        E = np.array([[0.8, 0.1, 0.1], [0.1, 0.8, 0.1], [0.2, 0.2, 0.6]]).T
    return DiscreteHMM(prior, T, E)


def cases():
    m = dense_model()
    m2 = LinearGaussianSSM(0.8 * m.A, 1.5 * m.Q, m.H, 0.7 * m.R, m.mu0 + 0.1, m.P0, b=m.b + 0.05, c=m.c - 0.1)
    _, ys = m.simulate(7, np.random.default_rng(2))
    ys = list(ys)
    ys[2] = None  # an unobserved step
    out = [("lg_dense", m, m2, ys)]
    k, k2 = KitagawaSSM(10.0, 1.0), KitagawaSSM(6.0, 2.0)
    _, ys = k.simulate(7, np.random.default_rng(3))
    out.append(("kitagawa", k, k2, [float(y) for y in ys]))
    out.append(("hmm", _hmm(0), _hmm(1), [[0], [1], [2], [2], [1], [0], [1]]))
    return out


CASES = cases()


def _joint(m, traj_j, ys):
    if isinstance(m, LinearGaussianSSM):
        return m.log_joint(traj_j, ys)
    if isinstance(m, KitagawaSSM):
        return m.log_joint(traj_j[:, 0], ys)
    return m.log_joint(traj_j[:, 0], [y[0] if y is not None else None for y in ys])


def run_oracle(m, m2, ys, n, seed, pending, k):
    """steps 1..k under m, then the step k+1 with m2's parameters"""
    pf = O.OraclePF(m, n, seed)
    pf.init(ys[0])
    for y in ys[1:k]:
        pf.maybe_resample(n * 0.9)
        pf.step(y)
    if pending:
        assert pf.maybe_resample(n + 1)[0]
    return pf


@pytest.mark.parametrize("case", range(len(CASES)), ids=[c[0] for c in CASES])
@pytest.mark.parametrize("pending", [False, True])
def test_oracle_step_params_weight_is_the_rescoring(case, pending):
    name, m, m2, ys = CASES[case]
    n, k = 300, 5
    pf = run_oracle(m, m2, ys, n, 7, pending, k)
    lw0 = pf.log_weights()
    pf.step_params(m2, ys[k])
    lw = pf.log_weights()
    traj = np.stack([pf.trajectory(t) for t in range(1, k + 2)])  # [k+1, d, n]
    past, now = ys[:k], ys[: k + 1]
    unobs = list(now[:k]) + [None]
    for j in range(n):
        tj = traj[:, :, j]
        inc = _joint(m2, tj, now) - _joint(m2, tj, unobs)  # log p'(y_t | x_t): the bootstrap step's weight
        delta = _joint(m2, tj[:k], past) - _joint(m, tj[:k], past)
        want = (0.0 if pending else lw0[j]) + inc + delta
        assert lw[j] == pytest.approx(want, rel=1e-10, abs=1e-9), (name, j)
    # the trace scores now follow the new parameters
    tot = pf.scores()
    want = [_joint(m2, traj[:, :, j], now) for j in range(n)]
    np.testing.assert_allclose(tot, want, rtol=1e-11, atol=1e-9)


def test_oracle_step_params_draws_from_the_new_transition():
    m = LinearGaussianSSM.benchmark(3)
    m2 = LinearGaussianSSM(0.5 * m.A, 2.0 * m.Q, m.H, m.R, m.mu0, m.P0, b=np.array([1.0, -2.0, 0.5]))
    _, ys = m.simulate(4, np.random.default_rng(5))
    n = 4000
    pf = O.OraclePF(m, n, 3)
    pf.init(ys[0])
    pf.step(ys[1])
    x_prev = pf.state().copy()  # no resample in between: particle j's parent is j
    pf.step_params(m2, ys[2])
    x = pf.state()
    L = np.linalg.cholesky(m2.Q)
    r = np.linalg.solve(L, x - (m2.A @ x_prev + m2.b[:, None]))
    for c in range(3):
        assert stats.kstest(r[c], "norm").pvalue > 1e-4


def test_oracle_step_params_refusals():
    m = LinearGaussianSSM.benchmark(3)
    _, ys = m.simulate(3, np.random.default_rng(5))
    pf = O.OraclePF(m, 10, 3, record_history=False)
    pf.init(ys[0])
    pf.step(ys[1])
    with pytest.raises(ValueError):
        pf.step_params(m, ys[2])  # the re-scoring needs the history
    pf = O.OraclePF(m, 10, 3)
    pf.init(ys[0])
    with pytest.raises(ValueError):
        pf.step_params(LinearGaussianSSM.benchmark(4), ys[1])  # other dimensions


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("case", range(len(CASES)), ids=[c[0] for c in CASES])
@pytest.mark.parametrize("pending", [False, True])
def test_gpu_step_params_bitexact(gh_ctx, case, pending):
    name, m, m2, ys = CASES[case]
    n, k, seed = 3001, 4, 11
    addr = m.obs_address
    st = gen.initialize_particle_filter(m, (1,), {addr(1): ys[0]}, n, seed=seed)
    orc = O.OraclePF(m, n, seed)
    orc.init(ys[0])
    for t in range(2, k + 1):
        assert gen.maybe_resample(st, n * 0.9) == orc.maybe_resample(n * 0.9)[0]
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), {addr(t): ys[t - 1]})
        orc.step(ys[t - 1])
    if pending:
        assert gen.maybe_resample(st, n + 1) and orc.maybe_resample(n + 1)[0]
    gen.particle_filter_step(st, (k + 1, m2), (gen.UnknownChange(), gen.UnknownChange()), {addr(k + 1): ys[k]})
    orc.step_params(m2, ys[k])
    assert st.model is m2
    # later steps and resamples under the new parameters
    for t in range(k + 2, len(ys) + 1):
        assert gen.maybe_resample(st, n * 0.9) == orc.maybe_resample(n * 0.9)[0]
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), {addr(t): ys[t - 1]})
        orc.step(ys[t - 1])
    assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64))
    assert np.array_equal(gen.get_log_weights(st).view(np.uint64), orc.log_weights().view(np.uint64))
    assert np.array_equal(st.parents, orc.parents())
    a, b = gen.log_ml_estimate(st), orc.log_ml_estimate()
    assert abs(a - b) <= 1e-9 * max(1.0, abs(b))
    tot = gen.get_traces(st).scores()
    assert np.array_equal(tot.view(np.uint64), orc.scores().view(np.uint64))
    st.close()


@pytest.mark.gpu
def test_gpu_step_params_refusals(gh_ctx):
    m = LinearGaussianSSM.benchmark(3)
    _, ys = m.simulate(3, np.random.default_rng(5))
    st = gen.initialize_particle_filter(m, (1,), {("chain", 1, "y"): ys[0]}, 64, seed=1)
    with pytest.raises(gen.GenHipError):
        gen.particle_filter_step(st, (2, LinearGaussianSSM.benchmark(4)), (gen.UnknownChange(), gen.UnknownChange()),
                                 {("chain", 2, "y"): ys[1]})
    with pytest.raises(gen.GenHipError):
        gen.particle_filter_step(st, (2, LinearGaussianSSM.benchmark(3, seed=5)), (gen.UnknownChange(), gen.NoChange()),
                                 {("chain", 2, "y"): ys[1]})
    st.close()


@pytest.mark.gpu
def test_gpu_step_params_matches_reference_update_params_kat(gh_ctx):
    """The reference's own update_params KAT (test/modeling_library/unfold.jl
    :303-326; numbers in tests/golden/unfold_kats.json) through
    gh_pf_step_params itself: the Unfold x ~ normal(alpha x_prev + beta, 1)
    (unfold.jl:5-8) is the LG-SSM at d = 1, its literal trajectory (x1 1.1,
    x2 1.2 from x_init 0.1) the distinguished particle of a conditional
    filter, no observations (weights 0).  Changing alpha 0.2 -> 0.5 re-scores
    both retained applications: particle 0's weight gains exactly the KAT's
    weight (0.1929) and its score columns of steps 1, 2 sum to the KAT's new
    score; the new step 3 (pinned to 1.4) is scored under alpha 0.5."""
    import json
    import os

    from gen_amd import dists as D

    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "unfold_kats.json")))
    a, want = g["args"], g["cases"]["update_params"]
    xi, al, be, x1, x2 = a["x_init"], a["alpha"], a["beta"], a["x1"], a["x2"]
    an, x3 = 0.5, 1.4

    def unfold(alpha):
        return gen.LinearGaussianSSM([[alpha]], [[1.0]], [[1.0]], [[1.0]], [alpha * xi + be], [[1.0]], b=[be])

    m_old, m_new = unfold(al), unfold(an)
    st = gen.initialize_conditional_particle_filter(m_old, (1,), None, 64, [x1], seed=5)
    gen.conditional_particle_filter_step(st, (2,), (gen.UnknownChange(),), None, [x2])
    w_before = gen.get_log_weights(st)[0]
    assert w_before == 0.0
    gen.conditional_particle_filter_step(st, (3, m_new), (gen.UnknownChange(), gen.UnknownChange()), None, [x3])
    w = gen.get_log_weights(st)[0]
    assert abs(w - want["weight"]) <= 1e-12 * max(1.0, abs(want["weight"])), (w, want)
    tr = gen.get_traces(st)
    assert [tr.step_states(t)[0, 0] for t in (1, 2, 3)] == [x1, x2, x3]
    _, ps = tr.scores(per_step=True)
    lat = ps[:, 0, 0]
    assert abs(lat[0] + lat[1] - want["score"]) <= 1e-13 * max(1.0, abs(want["score"])), (lat, want)
    assert abs(lat[2] - D.normal.logpdf(x3, an * x2 + be, 1.0)) <= 1e-13
    st.close()
