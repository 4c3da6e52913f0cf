"""Particle-marginal MH (config C5, examples/pmmh/example.jl:20-79).

CPU: the oracle's PMMH is deterministic, continues across calls exactly, and
moves.  GPU: one workgroup per chain reproduces the oracle bit for bit
(parameters, acceptance counts) with log-ML estimates within 1e-9.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gen_amd import KitagawaSSM  # noqa: E402
from oracle import oracle as O  # noqa: E402


def data(T=25, seed=3):
    # example.jl:45-57: var_x = 4, var_y = 1 (the reference's synthetic set)
    _, ys = KitagawaSSM(4.0, 1.0, 0.0, 5.0).simulate(T, np.random.default_rng(seed))
    return ys


@pytest.mark.parametrize("lvx,lvy", [(np.log(4.0), 0.0), (1.0, 0.3), (1.6, -0.3)])
def test_oracle_pmmh_inner_filter_is_the_particle_filter(lvx, lvy):
    """The likelihood term of the PMMH (the ParticleFilterCombinator's
    log_ml_estimate, examples/pmmh/pf.jl:40-56) is the particle filter of
    src/inference/particle_filter.jl on the model of example.jl:5-22: its
    estimates over 300 chains (independent random streams) have the mean and
    spread of the PF oracle's (O.run_pf, KitagawaSSM(exp(lvx), exp(lvy), 0, 5),
    N = 256, 300 seeds), and the average of the Z estimates (Z-hat is
    unbiased) agrees with a 2^16-particle estimate."""
    ys = data(T=25)
    m = KitagawaSSM(float(np.exp(lvx)), float(np.exp(lvy)), 0.0, 5.0)
    n = 300
    a = np.array([O.pmmh_loglik(ys, lvx, lvy, 256, seed=3, chain=c) for c in range(n)])
    b = np.array([O.run_pf(m, ys, 256, s, record_history=False).log_ml_estimate() for s in range(n)])
    se = np.sqrt(a.var(ddof=1) / n + b.var(ddof=1) / n)
    assert abs(a.mean() - b.mean()) < 4 * se, (a.mean(), b.mean(), se)
    assert 0.7 < a.var(ddof=1) / b.var(ddof=1) < 1.4
    big = np.mean([O.run_pf(m, ys, 1 << 16, s, record_history=False).log_ml_estimate() for s in range(2)])
    for x in (a, b):
        log_mean_z = x.max() + np.log(np.mean(np.exp(x - x.max())))
        assert abs(log_mean_z - big) < 0.5, (log_mean_z, big)
        assert x.mean() < big  # log Z-hat is biased low


def test_oracle_pmmh_deterministic_and_continues():
    ys = data()
    a = O.pmmh_run(ys, 3, 64, 4, seed=11, chain0=2)
    b = O.pmmh_run(ys, 3, 64, 4, seed=11, chain0=2)
    for x, y in zip(a[:4], b[:4]):
        assert np.array_equal(x, y)
    # 2 + 2 iterations == 4 iterations
    c1 = O.pmmh_run(ys, 3, 64, 2, seed=11, chain0=2)
    c2 = O.pmmh_run(ys, 3, 64, 2, seed=11, chain0=2, iter0=2, state=c1[:3])
    assert np.array_equal(c2[0], a[0]) and np.array_equal(c2[1], a[1]) and np.array_equal(c2[2], a[2])
    assert np.array_equal(c1[3] + c2[3], a[3])
    assert a[3].sum() > 0  # the chains move
    assert np.all(np.isfinite(a[2]))


@pytest.mark.gpu
@pytest.mark.parametrize("n_inner", [64, 256])
def test_gpu_pmmh_matches_oracle(gh_ctx, n_inner):
    from gen_amd.pmmh import PMMHChains

    ys = data()
    ref = O.pmmh_run(ys, 3, n_inner, 3, seed=11, chain0=5, history=True)
    ch = PMMHChains(ys, 3, n_inner, seed=11, chain0=5, ctx=gh_ctx)
    hist = ch.run(3, history=True)
    assert np.array_equal(ch.lvx, ref[0]) and np.array_equal(ch.lvy, ref[1])
    assert np.array_equal(ch.accepts, ref[3])
    assert np.array_equal(hist, ref[4])
    assert np.allclose(ch.lml, ref[2], rtol=1e-9, atol=0)
    # continuing on the device equals one longer run on the oracle
    ch.run(2)
    ref5 = O.pmmh_run(ys, 3, n_inner, 5, seed=11, chain0=5)
    assert np.array_equal(ch.lvx, ref5[0]) and np.array_equal(ch.lvy, ref5[1])
    assert np.array_equal(ch.accepts, ref5[3])


@pytest.mark.gpu
def test_gpu_pmmh_concentrates_near_truth(gh_ctx):
    """256 chains x 40 iterations on 60 observations of the var_x = 4,
    var_y = 1 model: the pooled late-iteration posterior of var_y sits near 1
    and of var_x in a broad band around 4 (PMMH is noisy at 128 particles)."""
    from gen_amd.pmmh import PMMHChains

    ys = data(T=60, seed=5)
    ch = PMMHChains(ys, 256, 128, seed=7, ctx=gh_ctx)
    hist = ch.run(40, history=True)
    late = np.exp(hist[:, 20:, :]).reshape(-1, 2)
    vx, vy = np.median(late[:, 0]), np.median(late[:, 1])
    assert 1.0 < vx < 16.0, vx
    assert 0.2 < vy < 5.0, vy
    assert (ch.accepts.sum(axis=0) > 0).all()
