"""Reversible-jump MH on the coal change-point model (config C3).

CPU: the oracle (orc_coal_run) is deterministic, continues across calls
exactly, keeps every state inside the model's support with a consistent
cached score, and its posterior over k matches the reference analysis (Green
1995, the source of examples/coal: mass on 1..7 change points, mode 2-3).
GPU: one thread per chain reproduces the oracle bit for bit (states, scores,
acceptance counts, k histories).
"""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

EV = json.load(open(os.path.join(ROOT, "tests", "golden", "coal_events.json")))
EVENTS = np.array(EV["events"])


def _valid(st):
    T = EVENTS[-1]
    for row in st:
        k = int(row[0])
        cp = row[2 : 2 + k]
        h = row[34 : 34 + k + 1]
        assert 0 <= k <= 32
        assert np.all(np.diff(np.concatenate([[0.0], cp, [T]])) > 0)
        assert np.all(h > 0)


def test_fixture():
    assert EV["n"] == 190 and EVENTS[0] == 0.0 and np.all(np.diff(EVENTS) >= 0)


def test_oracle_coal_deterministic_continues_and_valid():
    a = O.coal_run(EVENTS, 8, 60, seed=3, chain0=4, khist=True)
    b = O.coal_run(EVENTS, 8, 60, seed=3, chain0=4, khist=True)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
    c1 = O.coal_run(EVENTS, 8, 25, seed=3, chain0=4)
    c2 = O.coal_run(EVENTS, 8, 35, seed=3, chain0=4, iter0=25, state=c1[0])
    assert np.array_equal(c2[0], a[0]) and np.array_equal(c1[1] + c2[1], a[1])
    _valid(a[0])


def test_oracle_coal_posterior_over_k():
    st, acc, kh = O.coal_run(EVENTS, 32, 3000, seed=1, khist=True)
    post = np.bincount(kh[:, 1000:].ravel(), minlength=33) / kh[:, 1000:].size
    assert post[0] < 0.01  # a single rate is ruled out by the data
    assert post[1:8].sum() > 0.97
    assert 2 <= int(np.argmax(post)) <= 3
    rates = acc.sum(axis=0) / (32 * 3000)
    assert np.all((rates > 0.05) & (rates < 0.8)), rates


def test_oracle_simple_mcmc_posterior_over_k():
    """simple_mcmc_step (rate, position, mh(trace, select(:k))) targets the same
    posterior as mcmc_step: the regenerate of k leaves it invariant."""
    st, acc, kh = O.coal_run(EVENTS, 32, 4000, seed=2, khist=True, simple=True)
    _valid(st)
    post = np.bincount(kh[:, 1500:].ravel(), minlength=33) / kh[:, 1500:].size
    assert post[0] < 0.01
    assert post[1:8].sum() > 0.97
    assert 2 <= int(np.argmax(post)) <= 3
    st2, _, kh2 = O.coal_run(EVENTS, 32, 4000, seed=2, khist=True)
    post2 = np.bincount(kh2[:, 1500:].ravel(), minlength=33) / kh2[:, 1500:].size
    assert np.abs(post[:8] - post2[:8]).max() < 0.08, (post[:8], post2[:8])
    assert 0.001 < acc[:, 2].sum() / (32 * 4000) < 0.5
    for row in st:  # the cached scores are the scores of the states
        assert row[1] == pytest.approx(O.coal_score(row, EVENTS), rel=1e-11, abs=1e-8)


@pytest.mark.gpu
def test_gpu_coal_simple_matches_oracle(gh_ctx):
    from gen_amd.coal import CoalChains

    ref = O.coal_run(EVENTS, 300, 40, seed=5, chain0=3, khist=True, simple=True)
    ch = CoalChains(EVENTS, 300, seed=5, chain0=3, ctx=gh_ctx, kernel="simple_mcmc_step")
    kh = ch.run(40, k_history=True)
    assert np.array_equal(ch.state, ref[0])
    assert np.array_equal(ch.accepts, ref[1])
    assert np.array_equal(kh, ref[2])


@pytest.mark.gpu
def test_gpu_coal_matches_oracle(gh_ctx):
    from gen_amd.coal import CoalChains

    ref = O.coal_run(EVENTS, 300, 30, seed=11, chain0=7, khist=True)
    ch = CoalChains(EVENTS, 300, seed=11, chain0=7, ctx=gh_ctx)
    kh = ch.run(30, k_history=True)
    assert np.array_equal(ch.state, ref[0])
    assert np.array_equal(ch.accepts, ref[1])
    assert np.array_equal(kh, ref[2])
    ch.run(20)
    ref2 = O.coal_run(EVENTS, 300, 20, seed=11, chain0=7, iter0=30, state=ref[0])
    assert np.array_equal(ch.state, ref2[0])


@pytest.mark.gpu
def test_gpu_coal_run_stateless_matches_oracle(gh_ctx):
    """gh_coal_run (host rows in and out, transposed to the device's SoA layout
    at the boundary): generate + 25 iterations, then a continuation from the
    returned rows, against the oracle."""
    from ctypes import POINTER, byref, c_double, c_int32

    from gen_amd import _lib

    lib = _lib.load()
    ev = np.ascontiguousarray(np.sort(EVENTS))
    n = 257
    st = np.zeros((n, 68))
    acc = np.zeros((n, 3), dtype=np.int32)
    ms = c_double()
    _lib.check(lib.gh_coal_run(gh_ctx.h, 3, n, _lib.dptr(ev), ev.size, 25, 0, 5, 1, _lib.dptr(st),
                               acc.ctypes.data_as(POINTER(c_int32)), None, byref(ms)))
    ref = O.coal_run(EVENTS, n, 25, seed=5, chain0=3)
    assert np.array_equal(st, ref[0]) and np.array_equal(acc, ref[1])
    _lib.check(lib.gh_coal_run(gh_ctx.h, 3, n, _lib.dptr(ev), ev.size, 10, 25, 5, 0, _lib.dptr(st),
                               acc.ctypes.data_as(POINTER(c_int32)), None, byref(ms)))
    ref2 = O.coal_run(EVENTS, n, 10, seed=5, chain0=3, iter0=25, state=ref[0])
    assert np.array_equal(st, ref2[0]) and np.array_equal(acc, ref2[1])


@pytest.mark.gpu
@pytest.mark.parametrize("simple", [False, True])
def test_gpu_coal_many_change_points_bitexact(gh_ctx, simple):
    """Chains resumed from states with more change points than the kernel's LDS
    window (k_coal keeps cp 1..8, h 1..9 in LDS; the rest of a row is read and
    written in place in HBM): synthetic rows with k = 7..32 (the window's edge,
    the k = 31 kind of test_coal_pins.py, the capacity) run 30 iterations of
    either MCMC kernel bit-exact against the oracle — births past the window,
    deaths back into it, regenerated k' across it."""
    from gen_amd.coal import CoalChains

    ev = np.sort(np.asarray(EVENTS, dtype=np.float64))
    T = float(ev[-1])
    rng = np.random.default_rng(21)
    rows = []
    for i in range(320):
        k = int([7, 8, 9, 10, 16, 24, 31, 32][i % 8])
        r = np.zeros(68)
        r[0] = k
        r[2 : 2 + k] = np.sort(rng.uniform(0, T, k))
        r[34 : 34 + k + 1] = rng.gamma(1.0, 1.0 / 200.0, k + 1) + 1e-4
        r[1] = O.coal_score(r, ev)
        rows.append(r)
    st = np.array(rows)
    ref = O.coal_run(ev, len(rows), 30, seed=8, chain0=11, iter0=4, state=st, simple=simple)
    ch = CoalChains(ev, len(rows), seed=8, chain0=11, ctx=gh_ctx,
                    kernel="simple_mcmc_step" if simple else "mcmc_step")
    ch.load_state(st, 4)
    ch.run(30)
    assert np.array_equal(ch.state, ref[0]) and np.array_equal(ch.accepts, ref[1])
    # chains past the window at the end too (the simple kernel regenerates k
    # from its prior, so most of its chains are back inside it by then)
    assert (ref[0][:, 0] > 8).sum() > (3 if simple else 20)
    ch.close()
