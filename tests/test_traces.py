"""Trace materialisation: `get_traces(state)[i]`
exposes one particle's Gen trace — `get_args`, `get_choices`, `get_score`,
`trace[addr]` (src/gen_fn_interface.jl) — from the SoA history and the
genealogy, and choice maps flatten with `to_array` / `from_array`
(src/choice_map.jl:163-225).

CPU: to_array/from_array round trips and errors; the models' trace scores
against scipy densities.  GPU: a trace's choices are the oracle's trajectory
along the particle's genealogy (bit-exact) and its score is the model density
of that trajectory.
"""
import numpy as np
import pytest
from scipy.stats import multivariate_normal, norm

import gen_amd as gen
from gen_amd.choicemap import ChoiceMap, choicemap
from oracle import oracle as O


def test_to_array_from_array_round_trip():
    cm = choicemap((("chain", 1, "x"), np.array([1.0, 2.0])), (("chain", 1, "y"), 3.5),
                   (("chain", 2, "x"), np.array([[4.0, 5.0], [6.0, 7.0]])))
    arr = cm.to_array()
    assert np.array_equal(arr, [1.0, 2.0, 3.5, 4.0, 5.0, 6.0, 7.0])
    back = cm.from_array(arr * 2)
    assert back[("chain", 1, "y")] == 7.0
    assert np.array_equal(back[("chain", 2, "x")], [[8.0, 10.0], [12.0, 14.0]])
    assert np.array_equal(back.to_array(), arr * 2)
    with pytest.raises(ValueError):
        cm.from_array(arr[:-1])
    with pytest.raises(ValueError):
        cm.from_array(np.concatenate([arr, [0.0]]))
    assert ChoiceMap().to_array().size == 0


def test_lgssm_trace_score_is_the_joint_density():
    m = gen.LinearGaussianSSM.benchmark(3)
    xs, ys = m.simulate(4, np.random.default_rng(0))
    ref = multivariate_normal(m.mu0, m.P0).logpdf(xs[0])
    for t in range(1, 4):
        ref += multivariate_normal(m.A @ xs[t - 1] + m.b, m.Q).logpdf(xs[t])
    for t in range(4):
        ref += multivariate_normal(m.H @ xs[t] + m.c, m.R).logpdf(ys[t])
    assert abs(m.log_joint(xs, list(ys)) - ref) < 1e-10 * abs(ref)
    # an absent observation contributes nothing
    ys2 = list(ys)
    ys2[2] = None
    assert abs(m.log_joint(xs, ys2) - (ref - multivariate_normal(m.H @ xs[2] + m.c, m.R).logpdf(ys[2]))) < 1e-9


def test_kitagawa_and_hmm_trace_scores():
    k = gen.KitagawaSSM(10.0, 1.0)
    xs, ys = k.simulate(3, np.random.default_rng(1))
    ref = norm(0.0, 5.0).logpdf(xs[0])
    for t in (2, 3):
        v = xs[t - 2]
        ref += norm(v / 2 + 25 * v / (1 + v * v) + 8 * np.cos(1.2 * t), np.sqrt(10.0)).logpdf(xs[t - 1])
    ref += sum(norm(x * x / 20.0, 1.0).logpdf(y) for x, y in zip(xs, ys))
    assert abs(k.log_joint(xs, list(ys)) - ref) < 1e-10 * abs(ref)
    h = gen.DiscreteHMM([0.2, 0.8], [[0.9, 0.3], [0.1, 0.7]], [[0.6, 0.1], [0.4, 0.9]])
    zs, xo = [1, 1, 0], [1, 0, 0]
    ref = np.log(0.8 * 0.7 * 0.3) + np.log(0.9 * 0.1 * 0.6)
    assert abs(h.log_joint(zs, xo) - ref) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["lg4", "kit"])
def test_gpu_traces_follow_the_genealogy(gh_ctx, name):
    m = gen.LinearGaussianSSM.benchmark(4) if name == "lg4" else gen.KitagawaSSM(10.0, 1.0)
    _, ys = m.simulate(6, np.random.default_rng(3))
    n = 5003
    st = gen.initialize_particle_filter(m, (1,), {m.obs_address(1): ys[0]}, n, seed=13)
    orc = O.OraclePF(m, n, 13)
    orc.init(ys[0])
    for t in range(2, 7):
        gen.maybe_resample(st, n)
        orc.maybe_resample(n)
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), {m.obs_address(t): ys[t - 1]})
        orc.step(ys[t - 1])
    traces = gen.get_traces(st)
    for i in (0, 17, n - 1):
        tr = traces[i]
        assert tr.get_args() == (6,)
        cm = tr.get_choices()
        traj = np.stack([orc.trajectory(t)[:, i] for t in range(1, 7)])
        for t in range(1, 7):
            assert np.array_equal(np.atleast_1d(cm[m.latent_address(t)]), traj[t - 1])
            assert np.array_equal(np.atleast_1d(cm[m.obs_address(t)]), np.atleast_1d(ys[t - 1]))
            assert np.array_equal(np.atleast_1d(tr[m.latent_address(t)]), traj[t - 1])
        ref = m.log_joint(traj if m.d > 1 else traj[:, 0], list(ys))
        assert abs(tr.get_score() - ref) <= 1e-12 * abs(ref)
        assert np.array_equal(cm.from_array(cm.to_array()).to_array(), cm.to_array())


@pytest.mark.gpu
def test_gpu_regression_trace(gh_ctx):
    m, ys = gen.BayesianLinearRegression.quickstart()
    st = gen.initialize_particle_filter(m, (), m.constraints(ys), 1000, seed=4)
    tr = gen.get_traces(st)[7]
    cm = tr.get_choices()
    x = st.states()[7]
    assert cm[("slope",)] == x[0] and cm[("intercept",)] == x[1]
    assert cm[m.y_address(3)] == ys[2]
    assert tr.get_args() == ()
    assert abs(tr.get_score() - m.log_joint(x, ys)) < 1e-12 * abs(m.log_joint(x, ys))
