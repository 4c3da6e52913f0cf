"""Pin the coal oracle to the reference model and moves (CPU only).

The oracle (oracle/gh_oracle.c, orc_coal_*) scores a state by its segment
decomposition and each move by its score difference.  Here both are checked
against an independent restatement written from the reference files:
  * the score against the reference's own terms — scipy poisson(3).logpmf(k),
    the min_uniform_continuous logpdf of examples/coal/coal.jl:21-27 for every
    change point, scipy gamma(1, scale=1/200).logpdf for every rate, and the
    piecewise Poisson process logpdf of examples/coal/poisson_process.jl:32-51
    (sorted events walked through the segments, minus the integrated rate);
  * every move's acceptance ratio against the involutive MH weight of
    src/inference/mh.jl:85-98 / trace_translators.jl:848-876 — new score - old
    score + bwd proposal score - fwd proposal score + log|J| — with the
    proposal distributions of coal.jl:103-318 and the birth / death Jacobian
    of new_rates / new_rates_inverse (coal.jl:211-238) by central finite
    differences (the reference uses ForwardDiff);
  * the proposed states against the reference's birth / death transforms
    (coal.jl:260-305).
"""
import json
import math
import os

import numpy as np
import pytest
from scipy import stats

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EV = np.array(json.load(open(os.path.join(ROOT, "tests", "golden", "coal_events.json")))["events"])
T = EV[-1]
KMAX = 32


# ------------------------------------------------ the reference, restated
def min_uniform_logpdf(x, lower, upper, k):  # coal.jl:21-27
    if lower < x < upper:
        return (k - 1) * math.log(upper - x) + math.log(k) - k * math.log(upper - lower)
    return -math.inf


def piecewise_poisson_logpdf(x, bounds, rates):  # poisson_process.jl:9-51
    cur = 0
    upper = bounds[cur + 1]
    lpdf = 0.0
    for xi in sorted(x):
        assert bounds[0] <= xi <= bounds[-1]
        while xi > upper:
            cur += 1
            upper = bounds[cur + 1]
        lpdf += math.log(rates[cur])
    total, ascending = 0.0, True
    for i in range(len(rates)):
        ln = bounds[i + 1] - bounds[i]
        ascending = ascending and ln > 0
        total += ln * rates[i]
    return lpdf - total if ascending else -math.inf


def ref_score(k, cp, h):  # coal.jl:47-62
    lp = stats.poisson.logpmf(k, 3.0)
    lower = 0.0
    for i in range(1, k + 1):
        lp += min_uniform_logpdf(cp[i - 1], lower, T, k - i + 1)
        lower = cp[i - 1]
    lp += stats.gamma.logpdf(np.asarray(h), a=1.0, scale=1.0 / 200.0).sum()
    return lp + piecewise_poisson_logpdf(EV, [0.0] + list(cp) + [T], list(h))


def new_rates(cur_rate, u, cur_cp, prev_cp, next_cp):  # coal.jl:211-223
    d_prev, d_next = cur_cp - prev_cp, next_cp - cur_cp
    d_total = d_prev + d_next
    log_ratio = math.log(1 - u) - math.log(u)
    return (math.exp(math.log(cur_rate) - (d_next / d_total) * log_ratio),
            math.exp(math.log(cur_rate) + (d_prev / d_total) * log_ratio))


def new_rates_inverse(prev_rate, next_rate, cur_cp, prev_cp, next_cp):  # coal.jl:225-238
    d_prev, d_next = cur_cp - prev_cp, next_cp - cur_cp
    d_total = d_prev + d_next
    cur = math.exp((d_prev / d_total) * math.log(prev_rate) + (d_next / d_total) * math.log(next_rate))
    return cur, prev_rate / (prev_rate + next_rate)


def log_abs_jac(f, a, b):
    """log |det d f(a, b) / d(a, b)| by central differences."""
    ha, hb = 1e-6 * abs(a), 1e-6 * abs(b)
    fa = (np.array(f(a + ha, b)) - np.array(f(a - ha, b))) / (2 * ha)
    fb = (np.array(f(a, b + hb)) - np.array(f(a, b - hb))) / (2 * hb)
    return math.log(abs(fa[0] * fb[1] - fa[1] * fb[0]))


def unif_logpdf(lo, hi):
    return -math.log(hi - lo)


def ref_move(k, cp, h, move, u):
    """(alpha, k', cp', h') of one move with explicit uniforms (coal.jl:103-318)."""
    cp, h = list(cp), list(h)
    old = ref_score(k, cp, h)
    if move == "rate":  # rate_proposal / rate_involution
        i = int(u[0] * (k + 1)) + 1
        cur = h[i - 1]
        nh = cur / 2 + (cur * 2 - cur / 2) * u[1]
        h2 = h.copy()
        h2[i - 1] = nh
        fwd = -math.log(k + 1) + unif_logpdf(cur / 2, cur * 2)
        bwd = -math.log(k + 1) + unif_logpdf(nh / 2, nh * 2)
        return ref_score(k, cp, h2) - old + bwd - fwd, k, cp, h2
    if move == "position":  # position_proposal / position_involution
        i = int(u[0] * k) + 1
        lower = 0.0 if i == 1 else cp[i - 2]
        upper = T if i == k else cp[i]
        cp2 = cp.copy()
        cp2[i - 1] = lower + (upper - lower) * u[1]
        fwd = -math.log(k) + unif_logpdf(lower, upper)
        return ref_score(k, cp2, h) - old + fwd - fwd, k, cp2, h
    if move == "birth":  # birth_death_proposal (is_birth) / birth(k, i)
        i = int(u[0] * (k + 1)) + 1
        lower = 0.0 if i == 1 else cp[i - 2]
        upper = T if i == k + 1 else cp[i - 1]
        x = lower + (upper - lower) * u[1]
        hp, hn = new_rates(h[i - 1], u[2], x, lower, upper)
        cp2 = cp[: i - 1] + [x] + cp[i - 1:]
        h2 = h[: i - 1] + [hp, hn] + h[i:]
        fwd = (math.log(0.5) if k > 0 else 0.0) - math.log(k + 1) + unif_logpdf(lower, upper) + 0.0
        bwd = math.log(0.5) - math.log(k + 1)
        lj = log_abs_jac(lambda a, b: new_rates(a, b, x, lower, upper), h[i - 1], u[2])
        return ref_score(k + 1, cp2, h2) - old + bwd - fwd + lj, k + 1, cp2, h2
    # death: birth_death_proposal (not is_birth) / death(k, i)
    i = int(u[0] * k) + 1
    x = cp[i - 1]
    lower = 0.0 if i == 1 else cp[i - 2]
    upper = T if i == k else cp[i]
    cur, _ = new_rates_inverse(h[i - 1], h[i], x, lower, upper)
    cp2 = cp[: i - 1] + cp[i:]
    h2 = h[: i - 1] + [cur] + h[i + 1:]
    fwd = math.log(0.5) - math.log(k)
    bwd = (math.log(0.5) if k - 1 > 0 else 0.0) - math.log(k) + unif_logpdf(lower, upper) + 0.0
    lj = log_abs_jac(lambda a, b: new_rates_inverse(a, b, x, lower, upper), h[i - 1], h[i])
    return ref_score(k - 1, cp2, h2) - old + bwd - fwd + lj, k - 1, cp2, h2


def row(k, cp, h):
    r = np.zeros(68)
    r[0] = k
    r[2 : 2 + k] = cp
    r[34 : 34 + k + 1] = h
    r[1] = O.coal_score(r, EV)
    return r


def states():
    """Chain states of every size the posterior visits, the prior's k = 0, and
    synthetic states with many change points."""
    out = [O.coal_run(EV, 24, n, seed=9)[0] for n in (0, 3, 40)]
    rows = [r for st in out for r in st]
    rng = np.random.default_rng(4)
    for k in (0, 1, 5, 12, 31):
        cp = np.sort(rng.uniform(0, T, k))
        h = rng.gamma(1.0, 1.0 / 200.0, k + 1) + 1e-4
        rows.append(row(k, cp, h))
    return rows


STATES = states()


def test_states_cover_sizes():
    ks = {int(r[0]) for r in STATES}
    assert {0, 1, 5, 12, 31} <= ks and len(STATES) >= 70


def test_score_equals_reference_terms():
    """orc_coal_score (segment decomposition) = the reference's sum of
    logpdfs; the chains' cached scores are the scores of their states."""
    for r in STATES:
        k = int(r[0])
        cp, h = list(r[2 : 2 + k]), list(r[34 : 34 + k + 1])
        want = ref_score(k, cp, h)
        assert O.coal_score(r, EV) == pytest.approx(want, rel=1e-12, abs=1e-9), k
        assert r[1] == pytest.approx(want, rel=1e-11, abs=1e-8), k
    # outside the support: change points out of order / outside [0, T], a zero rate
    r = STATES[-2].copy()
    r[2], r[3] = r[3], r[2]
    assert O.coal_score(r, EV) == -math.inf
    r = STATES[-2].copy()
    r[34] = 0.0
    assert O.coal_score(r, EV) == -math.inf


@pytest.mark.parametrize("move", ["rate", "position", "birth", "death"])
def test_move_alpha_equals_involutive_mh_weight(move):
    rng = np.random.default_rng({"rate": 1, "position": 2, "birth": 3, "death": 4}[move])
    n = 0
    for r in STATES:
        k = int(r[0])
        if move in ("position", "death") and k == 0:
            continue
        if move == "birth" and k >= KMAX:
            continue
        for _ in range(3):
            u = rng.uniform(0.001, 0.999, 3)
            a, out = O.coal_propose(r, EV, move, u)
            want, k2, cp2, h2 = ref_move(k, list(r[2 : 2 + k]), list(r[34 : 34 + k + 1]), move, u)
            tol = 1e-6 if move in ("birth", "death") else 1e-8  # finite-difference Jacobian
            assert a == pytest.approx(want, abs=tol, rel=1e-10), (move, k, u)
            assert int(out[0]) == k2
            np.testing.assert_allclose(out[2 : 2 + k2], cp2, rtol=1e-13)
            np.testing.assert_allclose(out[34 : 34 + k2 + 1], h2, rtol=1e-13)
            assert not out[2 + k2 : 34].any() and not out[34 + k2 + 1 :].any()  # canonical zero padding
            # the proposed row's score (old score + the move's difference) is its score
            assert out[1] == pytest.approx(ref_score(k2, cp2, h2), rel=1e-11, abs=1e-8)
            n += 1
    assert n >= 60


def ref_regen_k(k, cp, h, u):
    """regenerate(trace, select(:k)) of the Dynamic DSL (src/dynamic/regenerate.jl:
    kept unselected choices add new score - old score; new choices are drawn
    from their distributions; discarded choices drop out) on the coal model,
    with k' from poisson(3)'s inverse CDF."""
    kk, cum = 0, stats.poisson.pmf(0, 3.0)
    while u[0] >= cum:
        kk += 1
        cum += stats.poisson.pmf(kk, 3.0)
    w, lower = 0.0, 0.0
    for i in range(1, min(k, kk) + 1):  # kept change points: min_uniform(lower, T, k - i + 1) -> (.., kk - i + 1)
        w += min_uniform_logpdf(cp[i - 1], lower, T, kk - i + 1) - min_uniform_logpdf(cp[i - 1], lower, T, k - i + 1)
        lower = cp[i - 1]
    cp2, h2 = list(cp[: min(k, kk)]), list(h[: min(k, kk) + 1])
    for i in range(k + 1, kk + 1):  # new change points by min_uniform's inverse CDF (coal.jl:28-32)
        x = T - (T - lower) * (1.0 - u[i]) ** (1.0 / (kk - i + 1))
        cp2.append(x)
        lower = x
    for i in range(k + 2, kk + 2):  # new rates: gamma(1, 1/200) by inversion
        h2.append(-math.log(1.0 - u[32 + i]) / 200.0)
    w += piecewise_poisson_logpdf(EV, [0.0] + cp2 + [T], h2) - piecewise_poisson_logpdf(EV, [0.0] + list(cp[:k]) + [T],
                                                                                        list(h[: k + 1]))
    return w, kk, cp2, h2


def test_regen_k_weight_equals_dynamic_regenerate():
    rng = np.random.default_rng(7)
    n = 0
    for r in STATES:
        k = int(r[0])
        for _ in range(3):
            u = rng.uniform(0.001, 0.999, 66)
            u[0] = rng.uniform(0.0, 0.97)  # k' <= 7 mostly, all sizes over the loop
            a, out = O.coal_regen_k(r, EV, u)
            want, kk, cp2, h2 = ref_regen_k(k, list(r[2 : 2 + k]), list(r[34 : 34 + k + 1]), u)
            assert int(out[0]) == kk
            np.testing.assert_allclose(out[2 : 2 + kk], cp2, rtol=1e-13)
            np.testing.assert_allclose(out[34 : 34 + kk + 1], h2, rtol=1e-13)
            assert not out[2 + kk : 34].any() and not out[34 + kk + 1 : 67].any()
            assert a == pytest.approx(want, rel=1e-10, abs=1e-8), (k, kk)
            assert out[1] == pytest.approx(ref_score(kk, cp2, h2), rel=1e-11, abs=1e-8)
            n += 1
    assert n >= 200


def test_birth_is_refused_at_capacity_and_outside_support():
    full = row(KMAX, np.sort(np.random.default_rng(5).uniform(0, T, KMAX)), np.full(KMAX + 1, 0.002))
    a, _ = O.coal_propose(full, EV, "birth", [0.5, 0.5, 0.5])
    assert a == -math.inf  # k_max = 32: the engine's fixed capacity
    a, _ = O.coal_propose(STATES[0], EV, "birth", [0.5, 0.5, 0.0])
    assert a == -math.inf  # u = 0: log(u) = -inf in new_rates
