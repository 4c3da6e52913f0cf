"""Pin the CPU oracle before trusting it (CPU only).

The oracle (oracle/gh_oracle.c) is checked against the reference's own
known-answer tests, re-expressed as the golden vectors in tests/golden/, and
against analytic oracles.  Gen.jl cannot run in this container (no Julia).
"""
import json
import math
import os

import numpy as np
import pytest

from oracle import oracle as O
from gen_amd.models import DiscreteHMM, KitagawaSSM, LinearGaussianSSM

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def gold(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def test_philox_known_answers():
    for v in gold("philox_kat.json")["vectors"]:
        assert O.philox(v["ctr"], v["key"]) == v["out"]


def test_exp_log_within_one_ulp_of_libm():
    L = O.lib()
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.uniform(-745, 709, 20000), rng.uniform(-1, 1, 20000), [0.0, -0.0, 1e-300, -1e-300]])
    e = np.array([L.orc_exp(x) for x in xs])
    ref = np.exp(xs)
    assert np.all(np.abs(e - ref) <= np.spacing(ref))
    ys = np.concatenate([np.exp(rng.uniform(-700, 700, 20000)), rng.uniform(0.5, 2, 20000), [5e-324, 1e-310, 1.0]])
    lg = np.array([L.orc_log(y) for y in ys])
    ref = np.log(ys)
    assert np.all(np.abs(lg - ref) <= np.spacing(np.abs(ref)) + 0.0)
    assert L.orc_log(0.0) == -math.inf and math.isnan(L.orc_log(-1.0))
    assert L.orc_exp(-1000.0) == 0.0 and L.orc_exp(800.0) == math.inf


def test_unit_log_within_one_ulp_of_libm():
    """The table-driven Box-Muller log over [2^-53, 1]: every bin, both bins
    touching 1 (no cancellation near 1), the ends of the interval."""
    L = O.lib()
    rng = np.random.default_rng(5)
    k = rng.integers(1, 1 << 53, 40000, dtype=np.uint64)
    u = np.concatenate([1.0 - k.astype(np.float64) * 2.0**-53, rng.uniform(0, 1, 20000) + 2.0**-53,
                        2.0 ** -rng.uniform(0, 53, 20000), 1.0 - 2.0 ** -np.arange(1, 54),
                        [1.0, 2.0**-53, 0.5, 0.70703125, 0.7071067811865476, np.nextafter(1.0, 0)]])
    lg = np.array([L.orc_log_unit(x) for x in u])
    ref = np.log(u)
    assert np.all(np.abs(lg - ref) <= np.spacing(np.abs(ref)))
    assert L.orc_log_unit(1.0) == 0.0
    # any positive normal argument (the coal score's log j, log(T - x), log h)
    x = np.concatenate([np.exp(rng.uniform(-700, 700, 20000)), np.arange(1.0, 200.0), [2.0**-1022, 1.7e308]])
    lg = np.array([L.orc_log_unit(v) for v in x])
    assert np.all(np.abs(lg - np.log(x)) <= np.spacing(np.abs(np.log(x))))


def test_trig():
    L = O.lib()
    rng = np.random.default_rng(1)
    xs = rng.uniform(0, 2000, 5000)
    assert np.max(np.abs(np.array([L.orc_cos(x) for x in xs]) - np.cos(xs))) < 5e-16
    import ctypes

    s, c = ctypes.c_double(), ctypes.c_double()
    for u in rng.uniform(0, 1, 5000):
        L.orc_sincos_2pi(u, ctypes.byref(s), ctypes.byref(c))
        assert abs(s.value - math.sin(2 * math.pi * u)) < 2e-15
        assert abs(c.value - math.cos(2 * math.pi * u)) < 2e-15


def test_trig_u32_angle_words():
    """sincos of a 32-bit angle word (the Box–Muller angle): every octant
    boundary and random words against libm at 2 pi c 2^-32."""
    import ctypes

    L = O.lib()
    rng = np.random.default_rng(2)
    words = list(rng.integers(0, 1 << 32, 20000, dtype=np.uint64))
    words += [k << 29 for k in range(8)] + [(k << 29) - 1 for k in range(1, 8)] + [0xFFFFFFFF, 1]
    s, c = ctypes.c_double(), ctypes.c_double()
    for w in words:
        L.orc_sincos_2pi_u32(int(w), ctypes.byref(s), ctypes.byref(c))
        ang = 2 * math.pi * (int(w) / 2.0**32)
        assert abs(s.value - math.sin(ang)) < 2e-15 and abs(c.value - math.cos(ang)) < 2e-15, w
    L.orc_sincos_2pi_u32(0, ctypes.byref(s), ctypes.byref(c))
    assert (s.value, c.value) == (0.0, 1.0)


def test_normals_are_standard():
    from scipy import stats

    z = np.concatenate([O.normals(7, i, 3, 2, 10) for i in range(20000)])
    assert abs(z.mean()) < 0.01 and abs(z.var() - 1) < 0.01
    assert stats.kstest(z, "norm").pvalue > 1e-3
    # each coordinate of the d = 10 layout (pairs straddle Philox blocks) is standard
    zz = z.reshape(-1, 10)
    for k in range(10):
        assert stats.kstest(zz[:, k], "norm").pvalue > 1e-4, k
    assert np.max(np.abs(np.corrcoef(zz.T) - np.eye(10))) < 0.04
    # the same counter gives the same draws, a different one different draws
    assert np.array_equal(O.normals(7, 5, 3, 2, 10), O.normals(7, 5, 3, 2, 10))
    assert not np.array_equal(O.normals(7, 5, 3, 2, 10), O.normals(7, 5, 4, 2, 10))


def test_normal_logpdf_golden():
    L = O.lib()
    for row in gold("unfold_kats.json")["normal_logpdf"]:
        got = L.orc_normal_logpdf(row["x"], row["mu"], row["std"])
        assert got == pytest.approx(row["logpdf"], rel=1e-15, abs=1e-15)


def test_unfold_update_regenerate_kats():
    """The Unfold update / regenerate weights and scores of the reference's
    known-answer tests (test/modeling_library/unfold.jl:116-481, kernel
    x ~ normal(alpha x_prev + beta, 1), unfold.jl:5-8), recomposed from the
    oracle's normal logpdf exactly as the reference states them.  The PF step's
    weight (update extending the chain, constrained new choices) is the
    `update_extend_change` shape: new-step logpdf plus the re-scored changes."""
    g = gold("unfold_kats.json")
    a = g["args"]
    lp = O.lib().orc_normal_logpdf
    xi, al, be, x1, x2 = a["x_init"], a["alpha"], a["beta"], a["x1"], a["x2"]
    an, s = 0.5, 1.0
    want = g["cases"]
    got = {
        "update_extend_change": (
            lp(x1, xi * an + be, s) + lp(1.3, x1 * an + be, s) + lp(1.4, 1.3 * an + be, s),
            lp(1.4, 1.3 * an + be, s) + lp(1.3, x1 * an + be, s) - lp(x2, x1 * al + be, s)
            + lp(x1, xi * an + be, s) - lp(x1, xi * al + be, s)),
        "update_shrink_change": (
            lp(1.3, xi * an + be, s),
            lp(1.3, xi * an + be, s) - lp(x1, xi * al + be, s) - lp(x2, x1 * al + be, s)),
        "update_nochange": (lp(x1, xi * al + be, s) + lp(x2, x1 * al + be, s), 0.0),
        "update_change_x2": (
            lp(x1, xi * al + be, s) + lp(3.3, x1 * al + be, s),
            lp(3.3, x1 * al + be, s) - lp(x2, x1 * al + be, s)),
        "update_params": (
            lp(x1, xi * an + be, s) + lp(x2, x1 * an + be, s),
            lp(x1, xi * an + be, s) - lp(x1, xi * al + be, s) + lp(x2, x1 * an + be, s) - lp(x2, x1 * al + be, s)),
        "regenerate_init": (
            lp(x1, -0.1 * al + be, s) + lp(x2, x1 * al + be, s),
            lp(x1, -0.1 * al + be, s) - lp(x1, xi * al + be, s)),
    }
    assert set(got) == set(want)
    for k, (score, weight) in got.items():
        assert score == pytest.approx(want[k]["score"], rel=1e-13, abs=1e-13), k
        assert weight == pytest.approx(want[k]["weight"], rel=1e-12, abs=1e-12), k


def hmm_forward(prior, E, T, obs):
    ml = 1.0
    alpha = np.asarray(prior)
    for i in range(1, len(obs)):
        pp = alpha * E[obs[i - 1], :]
        den = pp.sum()
        alpha = T @ (pp / den)
        ml *= den
    return ml * (alpha * E[obs[-1], :]).sum()


def test_hmm_forward_kat():
    # test/inference/particle_filter.jl:29-48
    k = gold("hmm.json")["forward_kat"]
    got = hmm_forward(k["prior"], np.array(k["emission"]), np.array(k["transition"]), k["obs"])
    assert got == pytest.approx(k["marg_lik"])


@pytest.mark.parametrize("proposal", [O.DEFAULT, O.OPTIMAL])
def test_oracle_pf_matches_hmm_forward(proposal):
    # test/inference/particle_filter.jl:96-168: N=10000, resample every step,
    # atol 0.01 against the exact forward-algorithm log-ML.
    g = gold("hmm.json")["pf_test"]
    m = DiscreteHMM(g["prior"], np.array(g["transition"]), np.array(g["emission"]))
    pf = O.run_pf(m, [[o] for o in g["obs"]], g["num_particles"], 0, thr=g["ess_threshold"], proposal=proposal)
    assert abs(pf.log_ml_estimate() - g["log_ml"]) < g["atol"]
    # the assertion is statistical: over 8 seeds the mean error is well inside it
    errs = [
        O.run_pf(m, [[o] for o in g["obs"]], g["num_particles"], s, thr=g["ess_threshold"], proposal=proposal)
        .log_ml_estimate() - g["log_ml"]
        for s in range(1, 9)
    ]
    assert abs(np.mean(errs)) < g["atol"]


def test_oracle_pf_matches_kalman():
    k = gold("kalman.json")["lg2"]
    d = k["d"]
    m = LinearGaussianSSM(np.array(k["A"]), 0.1 * np.eye(d), np.eye(d), 0.5 * np.eye(d), np.zeros(d), np.eye(d))
    ests = [O.run_pf(m, np.array(k["ys"]), 20000, s).log_ml_estimate() for s in range(4)]
    assert abs(np.mean(ests) - k["log_ml"]) < 0.05


def test_resampling_invariants():
    m = KitagawaSSM(10.0, 1.0)
    _, ys = m.simulate(12, np.random.default_rng(3))
    for resampler in (O.SYSTEMATIC, O.MULTINOMIAL):
        pf = O.OraclePF(m, 5000, 11, resampler)
        pf.init(ys[0])
        for y in ys[1:]:
            did, ess = pf.maybe_resample(5000 + 1)  # always resample
            assert did
            par = pf.parents()
            assert par.min() >= 0 and par.max() < 5000
            if resampler == O.SYSTEMATIC:
                assert np.all(np.diff(par) >= 0)  # systematic ancestors are sorted
            assert np.all(pf.log_weights() == 0.0)
            pf.step(y)


def test_systematic_offspring_counts_are_floor_or_ceil():
    """Systematic resampling gives particle i either floor(N w_i) or ceil(N w_i)
    children (w_i from the integer-quantised weights)."""
    m = KitagawaSSM(10.0, 1.0)
    _, ys = m.simulate(3, np.random.default_rng(4))
    n = 4096
    pf = O.OraclePF(m, n, 5)
    pf.init(ys[0])
    lw = pf.log_weights()
    pf.maybe_resample(n + 1)
    counts = np.bincount(pf.parents(), minlength=n)
    w = np.exp(lw - lw.max())
    w /= w.sum()
    assert np.all(counts >= np.floor(n * w) - 1) and np.all(counts <= np.ceil(n * w) + 1)
    assert counts.sum() == n


def test_importance_sampling_normalised():
    # test/inference/importance_sampling.jl:19-30: logsumexp(lnw) == 0 within 1e-14
    m = KitagawaSSM(10.0, 1.0)
    _, lnw, lml = O.importance_sampling(m, [2.0], 4, 0)
    mx = lnw.max()
    assert abs(mx + math.log(np.exp(lnw - mx).sum())) < 1e-14
    assert not math.isnan(lml)


def test_sharded_oracle_equals_single_rank():
    """Two ranks run the distributed algorithm (stats all-gather, integer totals
    all-gather, emit/apply exchange) and reproduce the single-rank run bit for bit."""
    m = LinearGaussianSSM.benchmark(4)
    _, ys = m.simulate(8, np.random.default_rng(5))
    n = 3001
    ref = O.run_pf(m, ys, n, 9, thr=n)  # resample every step
    for R in (2, 3):
        los = [(n * r) // R for r in range(R + 1)]
        pfs = [O.OraclePF(m, n, 9, lo=los[r], n_local=los[r + 1] - los[r]) for r in range(R)]
        for p in pfs:
            p.init(ys[0])
        for y in ys[1:]:
            stats = np.concatenate([p.local_stats() for p in pfs])
            dec, L, ess, M = O.combine_stats(stats, n, n)
            assert dec == 1
            totals = [p.qtotal(M) for p in pfs]
            emitted = [p.emit(M, totals, r) for r, p in enumerate(pfs)]
            slots = np.concatenate([e[0] for e in emitted])
            ancs = np.concatenate([e[1] for e in emitted])
            sts = np.concatenate([e[2] for e in emitted])
            assert np.array_equal(np.sort(slots), np.arange(n))
            for p in pfs:
                p.apply(L, slots, ancs, sts)
            for p in pfs:
                p.step(y)
        got = np.concatenate([p.state() for p in pfs], axis=1)
        assert np.array_equal(got, ref.state())
        assert np.array_equal(np.concatenate([p.parents() for p in pfs]), ref.parents())
