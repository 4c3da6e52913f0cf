"""Conditional SMC / particle Gibbs (examples/pmmh/smc.jl:100-163).

CPU (oracle): the distinguished particle keeps the given trajectory, its own
parent and the init_score / forward_score weights; a particle-Gibbs chain on
a 1-D linear-Gaussian model reproduces the exact (Kalman/RTS) smoothing means.
GPU: the C-ABI conditional filter equals the oracle bit for bit (states,
weights, parents, genealogy; log-ML 1e-9) on LG and Kitagawa models, and the
GPU particle-Gibbs chain reproduces the smoothing means.
"""
import numpy as np
import pytest

import gen_amd as gen
from oracle import oracle as O


def _lg1():
    return gen.LinearGaussianSSM([[0.9]], [[0.5]], [[1.0]], [[0.8]], [0.0], [[1.0]])


def _rts_means(m, ys):
    """Exact smoothing means of a 1-D LG model (Kalman filter + RTS)."""
    a, q, h, r = m.A[0, 0], m.Q[0, 0], m.H[0, 0], m.R[0, 0]
    mf, pf, mp, pp = [], [], [], []
    mu, P = m.mu0[0], m.P0[0, 0]
    for t, y in enumerate(np.asarray(ys).ravel()):
        if t > 0:
            mu, P = a * mu, a * a * P + q
        mp.append(mu)
        pp.append(P)
        k = P * h / (h * h * P + r)
        mu, P = mu + k * (y - h * mu), (1 - k * h) * P
        mf.append(mu)
        pf.append(P)
    ms = list(mf)
    for t in range(len(ms) - 2, -1, -1):
        g = pf[t] * a / pp[t + 1]
        ms[t] = mf[t] + g * (ms[t + 1] - mp[t + 1])
    return np.array(ms)


def _kit_loglik(m, y, x):
    return -((y - x * x / 20.0) ** 2) / (2 * m.var_y) - 0.5 * np.log(2 * np.pi * m.var_y)


def test_oracle_distinguished_particle_follows_reference():
    m = gen.KitagawaSSM(10.0, 1.0)
    xs, ys = m.simulate(8, np.random.default_rng(3))
    ref = xs + 0.25
    n = 500
    pf = O.OraclePF(m, n, 5, O.MULTINOMIAL)
    pf.init_conditional(ys[0], ref[0])
    w = _kit_loglik(m, ys[0], ref[0])
    for t in range(1, len(ys)):
        did, _ = pf.maybe_resample(n)  # resample every step
        assert did
        pf.step_conditional(ys[t], ref[t])
        assert pf.state()[0, 0] == ref[t]
        assert pf.parents()[0] == 0
        w = _kit_loglik(m, ys[t], ref[t])
        assert abs(pf.log_weights()[0] - w) < 1e-9
    # the lineage of particle 0 is the reference trajectory
    assert np.array_equal(np.array([pf.trajectory(t + 1)[0, 0] for t in range(len(ys))]), ref)
    with pytest.raises(ValueError):
        pf.step(ys[0])  # plain steps are refused on a conditional filter
    with pytest.raises(RuntimeError):
        pf.rejuvenate(1)


def test_oracle_csmc_needs_multinomial():
    m = _lg1()
    pf = O.OraclePF(m, 100, 1, O.SYSTEMATIC)
    with pytest.raises(ValueError):
        pf.init_conditional([0.3], [0.0])


def test_oracle_particle_gibbs_matches_smoother():
    m = _lg1()
    _, ys = m.simulate(5, np.random.default_rng(11))
    exact = _rts_means(m, ys)
    rng = np.random.default_rng(0)
    n, sweeps, burn = 32, 3000, 200
    ref = np.zeros((len(ys), 1))
    acc = np.zeros(len(ys))
    for k in range(sweeps):
        pf = O.run_csmc(m, ys, n, 100 + k, ref)
        w = pf.log_weights()
        p = np.exp(w - w.max())
        i = rng.choice(n, p=p / p.sum())
        ref = np.array([pf.trajectory(t + 1)[:, i] for t in range(len(ys))])
        if k >= burn:
            acc += ref[:, 0]
    est = acc / (sweeps - burn)
    assert np.max(np.abs(est - exact)) < 0.08, (est, exact)


# ------------------------------------------------------------------ GPU
def _pair(model, ys, ref, n, seed, thr):
    st = gen.initialize_conditional_particle_filter(model, (1,), {model.obs_address(1): ys[0]}, n, ref[0], seed=seed)
    orc = O.OraclePF(model, n, seed, O.MULTINOMIAL)
    orc.init_conditional(ys[0], ref[0])
    for t in range(2, len(ys) + 1):
        assert gen.maybe_resample(st, thr) == orc.maybe_resample(thr)[0]
        gen.conditional_particle_filter_step(st, (t,), (gen.UnknownChange(),), {model.obs_address(t): ys[t - 1]},
                                             ref[t - 1])
        orc.step_conditional(ys[t - 1], ref[t - 1])
        assert np.array_equal(st.states().T.view(np.uint64), orc.state().view(np.uint64)), t
        assert np.array_equal(gen.get_log_weights(st).view(np.uint64), orc.log_weights().view(np.uint64)), t
        assert np.array_equal(st.parents, orc.parents()), t
    lml, olml = gen.log_ml_estimate(st), orc.log_ml_estimate()
    assert abs(lml - olml) <= 1e-9 * abs(olml)
    T = len(ys)
    for t in (1, T // 2, T):
        assert np.array_equal(st.states(t).T, orc.trajectory(t)), t
    return st


@pytest.mark.gpu
@pytest.mark.parametrize("name,thr", [("lg4", None), ("lg4", 1e9), ("kit", None), ("kit", 1e9)])
def test_gpu_csmc_bitexact(gh_ctx, name, thr):
    m = gen.LinearGaussianSSM.benchmark(4) if name == "lg4" else gen.KitagawaSSM(10.0, 1.0)
    xs, ys = m.simulate(7, np.random.default_rng(6))
    ref = np.asarray(xs, dtype=np.float64).reshape(len(ys), -1) * 0.9
    st = _pair(m, ys, ref, 3001, 17, thr)
    # the distinguished particle's genealogy is the reference
    assert np.array_equal(np.stack([st.states(t)[0] for t in range(1, len(ys) + 1)]), ref)
    assert np.array_equal(gen.get_particle(st, 0), ref)
    with pytest.raises(gen.GenHipError):
        gen.particle_filter_step(st, (8,), (gen.UnknownChange(),), {m.obs_address(8): ys[0]})
    with pytest.raises(gen.GenHipError):
        gen.rejuvenate(st, 1)


@pytest.mark.gpu
def test_gpu_particle_gibbs_matches_smoother(gh_ctx):
    m = _lg1()
    _, ys = m.simulate(10, np.random.default_rng(12))
    exact = _rts_means(m, ys)
    refs, lmls = gen.particle_gibbs(m, [y for y in ys], 256, np.zeros((10, 1)), 600, seed=3)
    est = np.mean(np.stack(refs[100:])[:, :, 0], axis=0)
    assert np.max(np.abs(est - exact)) < 0.06, (est, exact)
    assert np.all(np.isfinite(lmls))
