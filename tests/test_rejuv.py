"""Rejuvenation moves (gh_pf_rejuvenate, gen_amd.rejuvenate).

The reference applies ``mh(trace, select(:chain => t => :x))`` to every
particle between steps (src/inference/mh.jl:14-26): regenerate the current
latent from its prior given the parent, accept iff log(u) < log p(y|x') -
log p(y|x); log weights unchanged.

CPU (oracle): weights untouched; the moves sample the one-step posterior (a
conjugate 1-D Gaussian at t = 1, checked by moments); refused after a resample.
GPU: states, weights, parents and accept counts bit-exact against the oracle
on every family, with and without resampling before the step, history on and
off, and on 2 ranks sharing the GPU through the host transport.
"""
import os

import numpy as np
import pytest

import gen_amd as gen
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lg1():
    # x_1 ~ N(0, 4); y ~ N(x, 1)  =>  x | y ~ N(4y/5, 4/5)
    return gen.LinearGaussianSSM([[0.8]], [[0.5]], [[1.0]], [[1.0]], [0.0], [[4.0]])


def test_oracle_rejuvenation_targets_the_posterior():
    m = _lg1()
    n, y = 40000, 2.5
    orc = O.OraclePF(m, n, 7)
    orc.init([y])
    w0 = orc.log_weights().copy()
    acc = orc.rejuvenate(30)
    assert 0 < acc < 30 * n
    x = orc.state()[0]
    # log weights are not touched by MH
    assert np.array_equal(orc.log_weights(), w0)
    mu, var = 4 * y / 5, 4 / 5
    assert abs(x.mean() - mu) < 4 * np.sqrt(var / n) * 3  # MH chains are correlated: loose
    assert abs(x.var() - var) < 0.05


def test_oracle_rejuvenation_step_keeps_parent_and_weights():
    m = gen.KitagawaSSM(10.0, 1.0)
    _, ys = m.simulate(4, np.random.default_rng(2))
    n = 2000
    orc = O.OraclePF(m, n, 3)
    orc.init(ys[0])
    for t in range(2, 5):
        orc.maybe_resample(None)
        orc.step(ys[t - 1])
        w = orc.log_weights().copy()
        orc.rejuvenate(2)
        assert np.array_equal(orc.log_weights(), w)
    # the rejuvenated states are what the history records
    x, _ = orc.history(4)
    assert np.array_equal(x, orc.state())


def test_oracle_rejuvenation_refused_after_resample():
    m = gen.LinearGaussianSSM.benchmark(4)
    _, ys = m.simulate(3, np.random.default_rng(1))
    orc = O.OraclePF(m, 500, 1)
    orc.init(ys[0])
    did, _ = orc.maybe_resample(1e9)
    assert did
    with pytest.raises(RuntimeError):
        orc.rejuvenate(1)


# ------------------------------------------------------------------ GPU
def _run_pair(model, ys, n, seed, thr, moves, record_history=True):
    st = gen.initialize_particle_filter(model, (1,), {model.obs_address(1): ys[0]}, n, seed=seed,
                                        record_history=record_history)
    orc = O.OraclePF(model, n, seed, record_history=record_history)
    orc.init(ys[0])
    a, b = gen.rejuvenate(st, moves), orc.rejuvenate(moves)
    assert a == b
    for t in range(2, len(ys) + 1):
        assert gen.maybe_resample(st, thr) == orc.maybe_resample(thr)[0]
        gen.particle_filter_step(st, (t,), (gen.UnknownChange(),), {model.obs_address(t): ys[t - 1]})
        orc.step(ys[t - 1])
        # two calls at one step continue the move counter
        a = gen.rejuvenate(st, moves) + gen.rejuvenate(st, 1)
        b = orc.rejuvenate(moves) + orc.rejuvenate(1)
        assert a == b, t
        assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64)), t
        assert np.array_equal(gen.get_log_weights(st).view(np.uint64), orc.log_weights().view(np.uint64)), t
    assert np.array_equal(st.parents, orc.parents())
    lml, olml = gen.log_ml_estimate(st), orc.log_ml_estimate()
    assert abs(lml - olml) <= 1e-9 * abs(olml)
    return st, orc


@pytest.mark.gpu
@pytest.mark.parametrize("name,thr", [("lg4", 1e9), ("lg4", None), ("lg10", 1e9), ("lg16", 1e9), ("kit", None),
                                      ("kit", 1e9)])
def test_gpu_rejuvenation_bitexact(gh_ctx, name, thr):
    m = {"lg4": lambda: gen.LinearGaussianSSM.benchmark(4), "lg10": lambda: gen.LinearGaussianSSM.benchmark(10),
         "lg16": lambda: gen.LinearGaussianSSM.benchmark(16), "kit": lambda: gen.KitagawaSSM(10.0, 1.0)}[name]()
    _, ys = m.simulate(6, np.random.default_rng(4))
    _run_pair(m, ys, 5003, 11, thr, 3)


@pytest.mark.gpu
def test_gpu_rejuvenation_hmm_and_no_history(gh_ctx):
    import json

    with open(os.path.join(ROOT, "tests", "golden", "hmm.json")) as f:
        g = json.load(f)["pf_test"]
    m = gen.DiscreteHMM(g["prior"], np.array(g["transition"]), np.array(g["emission"]))
    _run_pair(m, g["obs"], 4099, 5, 4099.0, 2)
    lg = gen.LinearGaussianSSM.benchmark(4)
    _, ys = lg.simulate(5, np.random.default_rng(8))
    _run_pair(lg, ys, 70001, 2, 1e9, 2, record_history=False)


@pytest.mark.gpu
def test_gpu_rejuvenation_state_errors(gh_ctx):
    m = gen.LinearGaussianSSM.benchmark(4)
    _, ys = m.simulate(3, np.random.default_rng(1))
    st = gen.initialize_particle_filter(m, (1,), {m.obs_address(1): ys[0]}, 1000, seed=1)
    gen.maybe_resample(st, 1e9)
    with pytest.raises(gen.GenHipError):
        gen.rejuvenate(st, 1)
    gen.particle_filter_step(st, (2,), (gen.UnknownChange(),), {m.obs_address(2): ys[1]})
    gen.rejuvenate(st, 4000)
    with pytest.raises(gen.GenHipError):
        gen.rejuvenate(st, (1 << 24) - 3999)  # 2^24 moves per step at most
    assert gen.rejuvenate(st, 0) == 0


@pytest.mark.gpu
def test_gpu_rejuvenation_multirank_host_transport(tmp_path):
    from tests.mr_worker import build_model
    from tests.test_multirank import _run_workers

    out = str(tmp_path / "r")
    n, T, seed, R = 3001, 6, 9, 2
    _run_workers([os.path.join(ROOT, "tests", "mr_worker.py"), "--model", "lg4", "--n", str(n), "--T", str(T),
                  "--thr", "1e9", "--seed", str(seed), "--rejuv", "2", "--out", out], R, timeout=400)
    m = build_model("lg4")
    _, ys = m.simulate(T, np.random.default_rng(5))
    orc = O.OraclePF(m, n, seed)
    orc.init(ys[0])
    orc.rejuvenate(2)
    for t in range(2, T + 1):
        orc.maybe_resample(1e9)
        orc.step(ys[t - 1])
        orc.rejuvenate(2)
    parts = [np.load(f"{out}.rank{r}.npz") for r in range(R)]
    states = np.concatenate([p["states"] for p in parts], axis=0)
    assert np.array_equal(states.T, orc.state())
    assert np.array_equal(np.concatenate([p["logw"] for p in parts]), orc.log_weights())
    assert np.array_equal(np.concatenate([p["parents"] for p in parts]), orc.parents())
