"""The distribution library (src/modeling_library/distributions/, rows a14-a17).

CPU: the oracle's restatement (orc_dist_logpdf) equals scipy's closed-form
densities for every distribution, including the support edges; its samplers
(orc_dist_random) follow the distributions (KS / chi-square / moment checks,
large-parameter regimes included); values do not depend on the batch size;
per-value parameter rows equal the shared row.
GPU: gh_dist_logpdf / gh_dist_random reproduce the oracle bit for bit, with
shared and per-value parameters, through the gen_amd.dists objects.
"""
import math

import numpy as np
import pytest
from scipy import special, stats

import gen_amd as gen
from gen_amd import dists as D
from oracle import oracle as O

COV3 = np.array([[2.0, 0.3, -0.4], [0.3, 1.0, 0.2], [-0.4, 0.2, 1.5]])
PW_B, PW_P = np.array([0.0, 1.0, 3.0, 4.0]), np.array([0.2, 0.5, 0.3])


def pw_logpdf(x):
    out = np.full(np.shape(x), -np.inf)
    for i in range(3):
        m = (x > PW_B[i]) & (x <= PW_B[i + 1]) & (x > PW_B[0]) & (x < PW_B[-1])
        out[m] = np.log(PW_P[i]) - np.log(PW_B[i + 1] - PW_B[i])
    return out


def bu_logpdf(x):
    with np.errstate(divide="ignore"):
        v = np.log(0.7 * stats.beta(2.0, 3.0).pdf(x) + 0.3)
    return np.where((x >= 0) & (x <= 1), v, -np.inf)


# name, args, dim, logpdf test points, scipy logpdf, discrete
CASES = {
    "normal": ((0.3, 1.7), 1, np.linspace(-6, 6, 41), stats.norm(0.3, 1.7).logpdf, False),
    "broadcasted_normal": ((np.array([0.0, 1.0, 2.0]), np.array([1.0, 0.5, 2.0])), 3,
                           np.random.default_rng(0).normal(size=(3, 25)),
                           lambda x: stats.norm(np.array([[0.0], [1.0], [2.0]]), np.array([[1.0], [0.5], [2.0]])).logpdf(x).sum(0),
                           False),
    "mvnormal": ((np.array([1.0, -1.0, 0.5]), COV3), 3, np.random.default_rng(1).normal(size=(3, 25)),
                 lambda x: stats.multivariate_normal(np.array([1.0, -1.0, 0.5]), COV3).logpdf(x.T), False),
    "uniform_continuous": ((-1.0, 2.5), 1, np.array([-1.5, -1.0, 0.0, 2.5, 2.6]),
                           stats.uniform(-1.0, 3.5).logpdf, False),
    "uniform_discrete": ((2.0, 7.0), 1, np.arange(0.0, 10.0), stats.randint(2, 8).logpmf, True),
    "bernoulli": ((0.3,), 1, np.array([0.0, 1.0]), stats.bernoulli(0.3).logpmf, True),
    "categorical": ((np.array([0.1, 0.2, 0.3, 0.4]),), 1, np.arange(0.0, 6.0),
                    lambda x: np.where((x >= 1) & (x <= 4), np.log(np.array([1, .1, .2, .3, .4, 1])[np.clip(x, 0, 5).astype(int)]), -np.inf),
                    True),
    "gamma": ((2.5, 0.7), 1, np.array([-1.0, 0.0, 1e-3, 0.5, 1.7, 4.0, 20.0]), stats.gamma(2.5, scale=0.7).logpdf, False),
    "inv_gamma": ((3.0, 2.0), 1, np.array([-1.0, 0.05, 0.5, 1.0, 3.0, 40.0]), stats.invgamma(3.0, scale=2.0).logpdf, False),
    "beta": ((2.0, 5.0), 1, np.array([-0.1, 0.01, 0.3, 0.5, 0.99, 1.2]), stats.beta(2.0, 5.0).logpdf, False),
    "exponential": ((1.5,), 1, np.array([-1.0, 0.0, 0.2, 3.0, 10.0]), stats.expon(scale=1 / 1.5).logpdf, False),
    "poisson": ((3.5,), 1, np.arange(0.0, 25.0), stats.poisson(3.5).logpmf, True),
    "binomial": ((20.0, 0.3), 1, np.arange(0.0, 21.0), stats.binom(20, 0.3).logpmf, True),
    "neg_binomial": ((3.5, 0.4), 1, np.arange(0.0, 40.0), stats.nbinom(3.5, 0.4).logpmf, True),
    "geometric": ((0.3,), 1, np.arange(0.0, 30.0), lambda x: stats.geom(0.3).logpmf(x + 1), True),
    "laplace": ((1.0, 2.0), 1, np.linspace(-10, 10, 21), stats.laplace(1.0, 2.0).logpdf, False),
    "cauchy": ((0.5, 1.5), 1, np.linspace(-30, 30, 31), stats.cauchy(0.5, 1.5).logpdf, False),
    "piecewise_uniform": ((PW_B, PW_P), 1, np.array([-1.0, 0.0, 0.5, 1.0, 2.0, 3.5, 4.0]), pw_logpdf, False),
    "beta_uniform": ((0.7, 2.0, 3.0), 1, np.array([-0.1, 0.0, 0.2, 0.5, 0.9, 1.0, 1.1]), bu_logpdf, False),
}
# the scipy distribution each sampler is checked against (continuous: KS; discrete: chi-square)
SAMPLING = {
    "normal": stats.norm(0.3, 1.7), "uniform_continuous": stats.uniform(-1.0, 3.5),
    "uniform_discrete": stats.randint(2, 8), "bernoulli": stats.bernoulli(0.3),
    "gamma": stats.gamma(2.5, scale=0.7), "inv_gamma": stats.invgamma(3.0, scale=2.0), "beta": stats.beta(2.0, 5.0),
    "exponential": stats.expon(scale=1 / 1.5), "poisson": stats.poisson(3.5), "binomial": stats.binom(20, 0.3),
    "neg_binomial": stats.nbinom(3.5, 0.4), "laplace": stats.laplace(1.0, 2.0), "cauchy": stats.cauchy(0.5, 1.5),
}


def flat(args):
    if len(args) == 2 and np.ndim(args[1]) == 2:  # mvnormal
        return np.concatenate([args[0], np.ravel(args[1])])
    return np.concatenate([np.atleast_1d(np.asarray(a, dtype=np.float64)) for a in args])


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_logpdf_equals_scipy(name):
    args, dim, x, ref, _ = CASES[name]
    got = O.dist_logpdf(name, flat(args), x, dim=dim)
    want = ref(x)
    assert np.array_equal(np.isneginf(got), np.isneginf(want)), (got, want)
    fin = np.isfinite(want)
    np.testing.assert_allclose(got[fin], want[fin], rtol=1e-12, atol=1e-12)


def test_oracle_special_functions():
    xs = np.array([1e-300, 1e-8, 0.1, 0.5, 1.0, 1.5, 2.0, 3.7, 7.99, 8.0, 12.5, 171.3, 1e4, 1e9, 1e100])
    for x in xs:
        assert O.lib().orc_lgamma(x) == pytest.approx(special.gammaln(x), rel=1e-14, abs=1e-13)
    for y in [-0.999, -0.5, -1e-10, 1e-300, 1e-12, 0.3, 2.0, 1e10]:
        assert O.lib().orc_log1p(y) == pytest.approx(math.log1p(y), rel=4e-16, abs=0)
    assert O.lib().orc_log1p(-1.0) == -math.inf


@pytest.mark.parametrize("name", list(SAMPLING))
def test_oracle_samplers_follow_the_distribution(name):
    args, dim, _, _, discrete = CASES[name]
    n = 20000
    s = O.dist_random(name, flat(args), n, seed=17)
    dist = SAMPLING[name]
    if discrete:
        ks = np.arange(s.min(), s.max() + 1)
        assert np.all(s == np.floor(s))
        obs = np.array([(s == k).sum() for k in ks])
        exp = dist.pmf(ks) * n
        # merge sparse tails so every expected count is >= 5
        keep = exp >= 5
        o2, e2 = list(obs[keep]), list(exp[keep])
        o2.append(n - sum(o2))
        e2.append(n - sum(e2))
        if e2[-1] < 5:
            ro, re = o2.pop(), e2.pop()
            o2[-1] += ro
            e2[-1] += re
        assert stats.chisquare(o2, e2).pvalue > 1e-4, name
    else:
        assert stats.kstest(s, dist.cdf).pvalue > 1e-4, name


def test_oracle_samplers_vector_and_mixture_distributions():
    n = 20000
    mu, std = np.array([0.0, 1.0, 2.0]), np.array([1.0, 0.5, 2.0])
    s = O.dist_random("broadcasted_normal", flat((mu, std)), n, 3, dim=3)
    for k in range(3):
        assert stats.kstest(s[k], stats.norm(mu[k], std[k]).cdf).pvalue > 1e-4
    m = np.array([1.0, -1.0, 0.5])
    s = O.dist_random("mvnormal", flat((m, COV3)), n, 4, dim=3)
    np.testing.assert_allclose(s.mean(1), m, atol=0.05)
    np.testing.assert_allclose(np.cov(s), COV3, atol=0.08)
    L = np.linalg.cholesky(COV3)
    assert stats.kstest((np.linalg.solve(L, s - m[:, None]) ** 2).sum(0), stats.chi2(3).cdf).pvalue > 1e-4
    s = O.dist_random("categorical", [0.1, 0.2, 0.3, 0.4], n, 5)
    assert stats.chisquare(np.bincount(s.astype(int), minlength=5)[1:], np.array([0.1, 0.2, 0.3, 0.4]) * n).pvalue > 1e-4
    s = O.dist_random("piecewise_uniform", flat((PW_B, PW_P)), n, 6)
    cdf = lambda x: np.interp(x, PW_B, np.concatenate([[0], np.cumsum(PW_P)]))
    assert stats.kstest(s, cdf).pvalue > 1e-4
    s = O.dist_random("beta_uniform", [0.7, 2.0, 3.0], n, 7)
    assert stats.kstest(s, lambda x: 0.7 * stats.beta(2.0, 3.0).cdf(x) + 0.3 * np.clip(x, 0, 1)).pvalue > 1e-4
    s = O.dist_random("geometric", [0.3], n, 8)
    assert s.mean() == pytest.approx(0.7 / 0.3, rel=0.03)


@pytest.mark.parametrize("name,args,mean,var", [
    ("poisson", (0.05,), 0.05, 0.05), ("poisson", (40.0,), 40.0, 40.0), ("poisson", (1e5,), 1e5, 1e5),
    ("binomial", (1e6, 0.4), 4e5, 2.4e5), ("binomial", (50.0, 0.97), 48.5, 1.455),
    ("gamma", (0.05, 3.0), 0.15, 0.45), ("gamma", (400.0, 0.01), 4.0, 0.04),
    ("neg_binomial", (0.5, 0.1), 4.5, 45.0), ("beta", (0.3, 0.4), 0.3 / 0.7, 0.3 * 0.4 / (0.49 * 1.7)),
])
def test_oracle_samplers_extreme_parameters(name, args, mean, var):
    n = 20000
    s = O.dist_random(name, list(args), n, seed=23)
    assert np.all(np.isfinite(s))
    assert s.mean() == pytest.approx(mean, abs=5 * math.sqrt(var / n))
    assert s.var() == pytest.approx(var, rel=0.12)


def test_oracle_per_value_rows_and_batch_independence():
    a = O.dist_random("gamma", [2.5, 0.7], 50, seed=2)
    b = O.dist_random("gamma", [2.5, 0.7], 7, seed=2)
    assert np.array_equal(a[:7], b)
    rows = np.tile([2.5, 0.7], (50, 1))
    c = O.dist_random("gamma", rows, 50, seed=2, per_value=True)
    assert np.array_equal(a, c)
    x = np.linspace(0.1, 3, 50)
    assert np.array_equal(O.dist_logpdf("gamma", rows, x, per_value=True), O.dist_logpdf("gamma", [2.5, 0.7], x))


# ------------------------------------------------------------------ GPU
def dist_obj(name):
    return {"binomial": D.binom, "neg_binomial": D.neg_binom}.get(name) or getattr(D, name)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_gpu_dists_bitexact(gh_ctx, name):
    args, dim, x, _, _ = CASES[name]
    d = dist_obj(name)
    got = d.logpdf(x, *args)
    want = O.dist_logpdf(name, flat(args), x, dim=dim)
    assert np.array_equal(np.asarray(got).view(np.uint64), want.view(np.uint64))
    n = 5003
    s = d.random(*args, n=n, seed=31)
    w = O.dist_random(name, flat(args), n, seed=31, dim=dim)
    assert np.array_equal(s.view(np.uint64), w.view(np.uint64))
    assert np.array_equal(d.random(*args, n=100, seed=31), s[..., :100])


@pytest.mark.gpu
def test_gpu_dists_per_value_parameters(gh_ctx):
    n = 4001
    rng = np.random.default_rng(3)
    shape, scale = rng.uniform(0.2, 5.0, n), rng.uniform(0.1, 3.0, n)
    s = D.gamma.random(shape, scale, n=n, seed=5)
    w = O.dist_random("gamma", np.stack([shape, scale], 1), n, seed=5, per_value=True)
    assert np.array_equal(s.view(np.uint64), w.view(np.uint64))
    lp = D.gamma.logpdf(s, shape, scale)
    np.testing.assert_allclose(lp, stats.gamma(shape, scale=scale).logpdf(s), rtol=1e-11, atol=1e-11)
    lam = rng.uniform(0.0, 300.0, n)
    k = D.poisson.random(lam, n=n, seed=6)
    assert np.array_equal(k, O.dist_random("poisson", lam[:, None], n, seed=6, per_value=True))
    probs = rng.dirichlet(np.ones(5), n)
    c = D.categorical.random(probs, n=n, seed=7)
    assert np.array_equal(c, O.dist_random("categorical", probs, n, seed=7, per_value=True))
    assert c.min() >= 1 and c.max() <= 5
    # Gen's call forms
    assert isinstance(D.normal(0.0, 1.0), float)
    assert D.logpdf(D.normal, 0.5, 0.0, 1.0) == O.dist_logpdf("normal", [0.0, 1.0], [0.5])[0]
    with pytest.raises(gen.GenHipError):
        D.gamma.random(1.0, n=3)


@pytest.mark.gpu
def test_gpu_unseeded_draws_are_fresh(gh_ctx):
    """Gen's random(dist, args...) draws fresh randomness on every call: two
    unseeded calls differ; reseeding the host generator reproduces a sequence."""
    a = [D.normal(0.0, 1.0) for _ in range(4)]
    assert len(set(a)) == 4
    assert not np.array_equal(D.gamma.random(2.0, 1.0, n=64), D.gamma.random(2.0, 1.0, n=64))
    D.seed(123)
    s1 = [D.normal(0.0, 1.0), D.poisson.random(3.0)]
    D.seed(123)
    s2 = [D.normal(0.0, 1.0), D.poisson.random(3.0)]
    D.seed(None)
    assert s1 == s2
