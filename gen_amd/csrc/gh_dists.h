// gh_dists.h — Gen's distribution library on the device.
//
// Every distribution of src/modeling_library/distributions/ as a pair of
// device functions, `logpdf(x, args...)` and `random(args...)`
// (modeling_library.jl:15-41), evaluated by one thread per value in the batch
// kernels k_dist_logpdf / k_dist_random (gh_dist_logpdf / gh_dist_random).
// The logpdfs follow the reference files' formulas in their operation order
// (file:line at each); the samplers are exact algorithms on the Philox
// stream STREAM_DIST keyed (seed, value index, 0, STREAM_DIST | draw), so a
// value does not depend on the batch size or the launch shape:
//   normal, broadcasted_normal, mvnormal   Box–Muller (gh_math.h)
//   uniform_continuous / _discrete, bernoulli, categorical, piecewise_uniform
//                                          one 53-bit uniform (inversion)
//   gamma, inv_gamma, beta, beta_uniform   Marsaglia–Tsang squeeze/rejection,
//                                          boosted by U^(1/a) for shape < 1
//   exponential, geometric, laplace, cauchy inversion
//   poisson, binomial                      inversion by chop-down search from
//                                          the mode (expected O(sd) steps)
//   neg_binomial                           poisson(gamma(r, (1-p)/p)), as
//                                          Distributions.jl samples it
// Special functions are the engine's own (gh_log, gh_exp, gh_lgamma below),
// bit-identical between device and the oracle's C restatement.
// Values are doubles; discrete values are integers stored exactly, bernoulli
// is 0/1, categorical (and piecewise_uniform's bin) are 1-based as in Gen.
#pragma once
#include "gh_math.h"

namespace gh {

enum : uint32_t { STREAM_DIST = 8 };

enum DistId : int {
  DIST_NORMAL = 1,
  DIST_BROADCASTED_NORMAL = 2,
  DIST_MVNORMAL = 3,
  DIST_UNIFORM_CONTINUOUS = 4,
  DIST_UNIFORM_DISCRETE = 5,
  DIST_BERNOULLI = 6,
  DIST_CATEGORICAL = 7,
  DIST_GAMMA = 8,
  DIST_INV_GAMMA = 9,
  DIST_BETA = 10,
  DIST_EXPONENTIAL = 11,
  DIST_POISSON = 12,
  DIST_BINOMIAL = 13,
  DIST_NEG_BINOMIAL = 14,
  DIST_GEOMETRIC = 15,
  DIST_LAPLACE = 16,
  DIST_CAUCHY = 17,
  DIST_PIECEWISE_UNIFORM = 18,
  DIST_BETA_UNIFORM = 19,
  DIST_LAST = 19
};

constexpr double kPi = 0x1.921fb54442d18p+1;
constexpr int kGammaIters = 60;       // Marsaglia–Tsang rounds (acceptance >= 0.95 each)
constexpr uint32_t kGammaBoost = 120;  // draw of the U^(1/a) boost
constexpr uint32_t kSecond = 128;      // second variate's draws (beta's G2, neg_binomial's poisson)
constexpr int kChopMax = 1 << 24;

// ------------------------------------------------------------ special functions
// log1p(y) = log(u) - ((u - 1) - y) / u with u = 1 + y (a few ulp)
GH_HD double gh_log1p(double y) {
  const double u = 1.0 + y;
  if (u == 1.0) return y;
  if (u == 0.0) return -INFINITY;
  return gh_log(u) - ((u - 1.0) - y) / u;
}

// log Gamma(x), x > 0: shift to x >= 8 by the recurrence, then Stirling's
// series through x^-13 (absolute error < 1e-14 on (0, 1e305)).
GH_HD double gh_lgamma(double x) {
  if (x != x) return x;
  if (x <= 0.0) return x == 0.0 ? INFINITY : NAN;
  if (x == INFINITY) return x;
  double prod = 1.0;
  while (x < 8.0) {
    prod *= x;
    x += 1.0;
  }
  const double r = 1.0 / x, r2 = r * r;
  double s = 1.0 / 156.0;
  s = fma(s, r2, -691.0 / 360360.0);
  s = fma(s, r2, 1.0 / 1188.0);
  s = fma(s, r2, -1.0 / 1680.0);
  s = fma(s, r2, 1.0 / 1260.0);
  s = fma(s, r2, -1.0 / 360.0);
  s = fma(s, r2, 1.0 / 12.0);
  const double st = ((x - 0.5) * gh_log(x) - x) + (0x1.d67f1c864beb5p-1 + s * r);  // 0.5 log(2 pi)
  return prod == 1.0 ? st : st - gh_log(prod);
}

// x log(y) with 0 log(y) = 0, x log1p(y) likewise (StatsFuns xlogy / xlog1py)
GH_HD double xlogy(double x, double y) { return x == 0.0 ? 0.0 : x * gh_log(y); }
GH_HD double xlog1py(double x, double y) { return x == 0.0 ? 0.0 : x * gh_log1p(y); }

GH_HD double normal_logpdf(double x, double mu, double std) {  // normal.jl:56-60
  const double var = std * std;
  const double diff = x - mu;
  return -(diff * diff) / (2.0 * var) - 0.5 * gh_log(2.0 * kPi * var);
}

// ----------------------------------------------------------------- draws
// (the distribution kernels draw from (seed, id, 0, STREAM_DIST, draw); a slot
// model's simulate from (seed, particle, t, STREAM_SIM, base + draw))
struct DistRng {
  uint64_t seed, id;
  uint32_t t = 0, stream = STREAM_DIST, base = 0;
};
GH_HD u32x4 dist_block(const DistRng& r, uint32_t draw) {
  return rng_block(r.seed, r.id, r.t, r.stream, r.base + draw);
}
GH_HD double dist_u(const DistRng& r, uint32_t draw) {  // [0, 1)
  const u32x4 w = dist_block(r, draw);
  return u53(w.x, w.y);
}
GH_HD double dist_upos(const DistRng& r, uint32_t draw) {  // (0, 1]
  const u32x4 w = dist_block(r, draw);
  return one_minus_u53(w.x, w.y);
}
GH_HD double dist_normal(const DistRng& r, uint32_t draw, const double* tab) {
  double z0, z1;
  normal_pair(dist_block(r, draw), &z0, &z1, tab);
  return z0;
}

// inverse-CDF categorical over p[0..K) (sequential sums; 0-based result)
GH_HD int dist_cat(const double* p, int K, double u) {
  double total = 0.0;
  for (int k = 0; k < K; ++k) total += p[k];
  const double target = u * total;
  double cum = 0.0;
  int last = -1;
  for (int k = 0; k < K; ++k) {
    cum += p[k];
    if (p[k] > 0.0) last = k;
    if (cum > target && p[k] > 0.0) return k;
  }
  return last;
}

// Gamma(a, 1), Marsaglia & Tsang (2000): round i draws a normal from block
// d0 + 2i and the acceptance uniform from d0 + 2i + 1
GH_HD double gamma_std(const DistRng& r, double a, uint32_t d0, const double* tab) {
  if (!(a > 0.0)) return NAN;
  double boost = 1.0;
  if (a < 1.0) {
    boost = gh_exp(gh_log(dist_upos(r, d0 + kGammaBoost)) / a);
    a = a + 1.0;
  }
  const double d = a - 1.0 / 3.0;
  const double c = 1.0 / sqrt(9.0 * d);
  for (int i = 0; i < kGammaIters; ++i) {
    const double x = dist_normal(r, d0 + 2u * (uint32_t)i, tab);
    double v = 1.0 + c * x;
    if (v <= 0.0) continue;
    v = v * v * v;
    const double u = dist_upos(r, d0 + 2u * (uint32_t)i + 1u);
    const double x2 = x * x;
    if (u < 1.0 - 0.0331 * (x2 * x2)) return (d * v) * boost;
    if (gh_log(u) < 0.5 * x2 + d * ((1.0 - v) + gh_log(v))) return (d * v) * boost;
  }
  return NAN;
}

// Poisson(lam) by chop-down inversion from the mode m = floor(lam): subtract
// pmf(m), then alternately pmf(m+1), pmf(m-1), pmf(m+2), ... from one uniform
// u in [0, 1) (poisson_chop; poisson_draw takes u from the DIST stream)
GH_HD double poisson_chop(double lam, double u) {
  if (lam == 0.0) return 0.0;
  if (!(lam > 0.0) || lam == INFINITY) return NAN;
  const double m = floor(lam);
  const double pm = gh_exp(xlogy(m, lam) - lam - gh_lgamma(m + 1.0));
  u -= pm;
  if (u <= 0.0) return m;
  double lo = m, hi = m, pl = pm, ph = pm;
  for (int it = 0; it < kChopMax; ++it) {
    hi += 1.0;
    ph = ph * lam / hi;
    u -= ph;
    if (u <= 0.0) return hi;
    if (lo > 0.0) {
      pl = pl * lo / lam;
      lo -= 1.0;
      u -= pl;
      if (u <= 0.0) return lo;
    }
    if (ph == 0.0 && (lo <= 0.0 || pl == 0.0)) break;  // rounding residue: all mass visited
  }
  return m;
}
GH_HD double poisson_draw(const DistRng& r, double lam, uint32_t draw) {
  if (lam == 0.0) return 0.0;
  if (!(lam > 0.0) || lam == INFINITY) return NAN;
  return poisson_chop(lam, dist_u(r, draw));
}

// Binomial(n, p), the same chop-down from the mode floor((n + 1) p)
GH_HD double binomial_draw(const DistRng& r, double n, double p, uint32_t draw) {
  if (!(p >= 0.0 && p <= 1.0) || !(n >= 0.0)) return NAN;
  if (p == 0.0 || n == 0.0) return 0.0;
  if (p == 1.0) return n;
  const double q = 1.0 - p;
  double m = floor((n + 1.0) * p);
  if (m > n) m = n;
  double u = dist_u(r, draw);
  const double pm =
      gh_exp(((gh_lgamma(n + 1.0) - gh_lgamma(m + 1.0)) - gh_lgamma(n - m + 1.0)) + xlogy(m, p) + xlog1py(n - m, -p));
  u -= pm;
  if (u <= 0.0) return m;
  const double pq = p / q, qp = q / p;
  double lo = m, hi = m, pl = pm, ph = pm;
  for (int it = 0; it < kChopMax; ++it) {
    if (hi < n) {
      ph = ph * ((n - hi) / (hi + 1.0)) * pq;
      hi += 1.0;
      u -= ph;
      if (u <= 0.0) return hi;
    }
    if (lo > 0.0) {
      pl = pl * (lo / (n - lo + 1.0)) * qp;
      lo -= 1.0;
      u -= pl;
      if (u <= 0.0) return lo;
    }
    if ((hi >= n || ph == 0.0) && (lo <= 0.0 || pl == 0.0)) break;
  }
  return m;
}

// ------------------------------------------------------------------ one value
// P: the value's parameter row; D: value components (vector distributions);
// K: categorical / piecewise_uniform bins.  mvnormal's row is host-derived:
// mu[D] | L[D*D] (lower Cholesky factor of the covariance) | cst =
// -0.5 (D log 2pi + log det).
template <int DIST>
GH_HD double dist_logpdf(const double* x, int64_t xs, const double* P, int D, int K) {
  const double v = x[0];
  if constexpr (DIST == DIST_NORMAL) {
    return normal_logpdf(v, P[0], P[1]);
  } else if constexpr (DIST == DIST_BROADCASTED_NORMAL) {  // normal.jl:62-71
    double s = 0.0;
    for (int k = 0; k < D; ++k) {
      const double std = P[D + k];
      const double var = std * std;
      const double diff = x[k * xs] - P[k];
      s += -(diff * diff) / (2.0 * var) - 0.5 * gh_log(2.0 * kPi * var);
    }
    return s;
  } else if constexpr (DIST == DIST_MVNORMAL) {  // mvnormal.jl:12-16, forward substitution
    const double* L = P + D;
    double u[32];
    double quad = 0.0;
    for (int i = 0; i < D; ++i) {
      double rr = x[i * xs] - P[i];
      for (int k = 0; k < i; ++k) rr = fma(-L[i * D + k], u[k], rr);
      u[i] = rr / L[i * D + i];
      quad = fma(u[i], u[i], quad);
    }
    return P[D + D * D] - 0.5 * quad;
  } else if constexpr (DIST == DIST_UNIFORM_CONTINUOUS) {  // uniform_continuous.jl:12-14
    return (v >= P[0] && v <= P[1]) ? -gh_log(P[1] - P[0]) : -INFINITY;
  } else if constexpr (DIST == DIST_UNIFORM_DISCRETE) {  // uniform_discrete.jl:10-13 (DiscreteUniform)
    return (v >= P[0] && v <= P[1] && v == floor(v)) ? -gh_log((P[1] - P[0]) + 1.0) : -INFINITY;
  } else if constexpr (DIST == DIST_BERNOULLI) {  // bernoulli.jl:10-12
    return v != 0.0 ? gh_log(P[0]) : gh_log(1.0 - P[0]);
  } else if constexpr (DIST == DIST_CATEGORICAL) {  // categorical.jl:10-12, 1-based
    return (v > 0.0 && v <= (double)K && v == floor(v)) ? gh_log(P[(int)v - 1]) : -INFINITY;
  } else if constexpr (DIST == DIST_GAMMA) {  // gamma.jl:10-16
    const double shape = P[0], scale = P[1];
    return v > 0.0 ? (((shape - 1.0) * gh_log(v) - (v / scale)) - shape * gh_log(scale)) - gh_lgamma(shape)
                   : -INFINITY;
  } else if constexpr (DIST == DIST_INV_GAMMA) {  // inv_gamma.jl:12-18
    const double shape = P[0], scale = P[1];
    return v > 0.0 ? ((shape * gh_log(scale) - (shape + 1.0) * gh_log(v)) - gh_lgamma(shape)) - (scale / v)
                   : -INFINITY;
  } else if constexpr (DIST == DIST_BETA) {  // beta.jl:13-16, logbeta = lgamma a + lgamma b - lgamma(a + b)
    const double a = P[0], b = P[1];
    if (v < 0.0 || v > 1.0) return -INFINITY;
    const double lb = (gh_lgamma(a) + gh_lgamma(b)) - gh_lgamma(a + b);
    return ((a - 1.0) * gh_log(v) + (b - 1.0) * gh_log1p(-v)) - lb;
  } else if constexpr (DIST == DIST_EXPONENTIAL) {  // exponential.jl:10-13: Exponential(scale = 1/rate)
    const double scale = 1.0 / P[0];
    return v < 0.0 ? -INFINITY : -gh_log(scale) - v / scale;
  } else if constexpr (DIST == DIST_POISSON) {  // poisson.jl:10-12
    return v < 0.0 ? -INFINITY : (v * gh_log(P[0]) - P[0]) - gh_lgamma(v + 1.0);
  } else if constexpr (DIST == DIST_BINOMIAL) {  // binom.jl:10-12 (Distributions.Binomial)
    const double n = P[0], p = P[1];
    if (v < 0.0 || v > n || v != floor(v)) return -INFINITY;
    return (((gh_lgamma(n + 1.0) - gh_lgamma(v + 1.0)) - gh_lgamma(n - v + 1.0)) + xlogy(v, p)) + xlog1py(n - v, -p);
  } else if constexpr (DIST == DIST_NEG_BINOMIAL) {  // neg_binom.jl:12-14 (failures before the r-th success)
    const double rr = P[0], p = P[1];
    if (v < 0.0 || v != floor(v)) return -INFINITY;
    return (((gh_lgamma(v + rr) - gh_lgamma(rr)) - gh_lgamma(v + 1.0)) + xlogy(rr, p)) + xlog1py(v, -p);
  } else if constexpr (DIST == DIST_GEOMETRIC) {  // geometric.jl:10-12 (failures before the first success)
    if (v < 0.0 || v != floor(v)) return -INFINITY;
    return gh_log(P[0]) + xlog1py(v, -P[0]);
  } else if constexpr (DIST == DIST_LAPLACE) {  // laplace.jl:10-13
    const double diff = fabs(v - P[0]);
    return -diff / P[1] - gh_log(2.0 * P[1]);
  } else if constexpr (DIST == DIST_CAUCHY) {  // cauchy.jl:10-12 (Distributions.Cauchy)
    const double z = (v - P[0]) / P[1];
    return -(gh_log(kPi * P[1]) + gh_log1p(z * z));
  } else if constexpr (DIST == DIST_PIECEWISE_UNIFORM) {  // piecewise_uniform.jl:30-43: bounds[K+1] | probs[K]
    const double* b = P;
    if (v <= b[0] || v >= b[K]) return -INFINITY;
    int bin = 0;
    while (v > b[bin + 1]) ++bin;
    return gh_log(P[K + 1 + bin]) - gh_log(b[bin + 1] - b[bin]);
  } else {  // DIST_BETA_UNIFORM, beta_uniform.jl:12-20: logsumexp(log theta + beta, log(1 - theta))
    if (v < 0.0 || v > 1.0) return -INFINITY;
    const double th = P[0];
    const double lbeta = gh_log(th) + dist_logpdf<DIST_BETA>(x, xs, P + 1, 1, 0);
    const double lunif = gh_log(1.0 - th);
    const double m = lbeta > lunif ? lbeta : lunif;
    if (m == -INFINITY) return m;
    return m + gh_log(gh_exp(lbeta - m) + gh_exp(lunif - m));
  }
}

template <int DIST>
GH_HD void dist_random(const DistRng& r, double* x, int64_t xs, const double* P, int D, int K, const double* tab) {
  if constexpr (DIST == DIST_NORMAL) {  // normal.jl:96: mu + std * randn()
    x[0] = P[0] + P[1] * dist_normal(r, 0, tab);
  } else if constexpr (DIST == DIST_BROADCASTED_NORMAL || DIST == DIST_MVNORMAL) {
    double z[32];
    for (int p = 0; 2 * p < D; ++p) {  // normals_rt's word layout, draws from 0
      double a, c;
      const int k0 = 3 * p;
      uint32_t wd[3];
      for (int q = 0; q < 3; ++q) {
        const int k = k0 + q;
        const u32x4 w = dist_block(r, (uint32_t)(k >> 2));
        const int e = k & 3;
        wd[q] = e == 0 ? w.x : (e == 1 ? w.y : (e == 2 ? w.z : w.w));
      }
      box_muller(wd[0], wd[1], wd[2], &a, &c, tab);
      z[2 * p] = a;
      if (2 * p + 1 < D) z[2 * p + 1] = c;
    }
    if constexpr (DIST == DIST_BROADCASTED_NORMAL) {  // normal.jl:99-104: mu .+ std .* randn(shape)
      for (int k = 0; k < D; ++k) x[k * xs] = P[k] + P[D + k] * z[k];
    } else {  // mvnormal.jl:30-33: mu + L z
      const double* L = P + D;
      for (int i = 0; i < D; ++i) {
        double acc = P[i];
        for (int k = 0; k <= i; ++k) acc = fma(L[i * D + k], z[k], acc);
        x[i * xs] = acc;
      }
    }
  } else if constexpr (DIST == DIST_UNIFORM_CONTINUOUS) {  // uniform_continuous.jl:21-23
    x[0] = dist_u(r, 0) * (P[1] - P[0]) + P[0];
  } else if constexpr (DIST == DIST_UNIFORM_DISCRETE) {
    x[0] = P[0] + floor(dist_u(r, 0) * ((P[1] - P[0]) + 1.0));
  } else if constexpr (DIST == DIST_BERNOULLI) {  // bernoulli.jl:19: rand() < prob
    x[0] = dist_u(r, 0) < P[0] ? 1.0 : 0.0;
  } else if constexpr (DIST == DIST_CATEGORICAL) {
    x[0] = (double)(dist_cat(P, K, dist_u(r, 0)) + 1);
  } else if constexpr (DIST == DIST_GAMMA) {
    x[0] = P[1] * gamma_std(r, P[0], 0, tab);
  } else if constexpr (DIST == DIST_INV_GAMMA) {  // InverseGamma(a, s) = s / Gamma(a, 1)
    x[0] = P[1] / gamma_std(r, P[0], 0, tab);
  } else if constexpr (DIST == DIST_BETA) {  // G1 / (G1 + G2)
    const double g1 = gamma_std(r, P[0], 0, tab), g2 = gamma_std(r, P[1], kSecond, tab);
    x[0] = g1 / (g1 + g2);
  } else if constexpr (DIST == DIST_EXPONENTIAL) {  // scale * randexp()
    x[0] = (1.0 / P[0]) * -gh_log(dist_upos(r, 0));
  } else if constexpr (DIST == DIST_POISSON) {
    x[0] = poisson_draw(r, P[0], 0);
  } else if constexpr (DIST == DIST_BINOMIAL) {
    x[0] = binomial_draw(r, P[0], P[1], 0);
  } else if constexpr (DIST == DIST_NEG_BINOMIAL) {  // poisson(gamma(r, (1 - p) / p))
    const double lam = ((1.0 - P[1]) / P[1]) * gamma_std(r, P[0], 0, tab);
    x[0] = poisson_draw(r, lam, kSecond);
  } else if constexpr (DIST == DIST_GEOMETRIC) {  // floor(log(U) / log1p(-p))
    x[0] = floor(gh_log(dist_upos(r, 0)) / gh_log1p(-P[0])) + 0.0;
  } else if constexpr (DIST == DIST_LAPLACE) {  // loc +- scale * randexp(), the sign from a third word
    const u32x4 w = dist_block(r, 0);
    const double e = -gh_log(one_minus_u53(w.x, w.y));
    x[0] = P[0] + P[1] * ((w.z & 1u) ? -e : e);
  } else if constexpr (DIST == DIST_CAUCHY) {  // x0 + gamma tan(pi (u - 1/2)) = x0 - gamma cot(pi u)
    const u32x4 w = dist_block(r, 0);
    const double u = ((double)u53_bits(w.x, w.y) + 0.5) * 0x1p-53;  // (0, 1)
    double s, c;
    sincos_2pi(u * 0.5, &s, &c);
    x[0] = P[0] - P[1] * (c / s);
  } else if constexpr (DIST == DIST_PIECEWISE_UNIFORM) {  // piecewise_uniform.jl:46-50
    const int bin = dist_cat(P + K + 1, K, dist_u(r, 0));
    x[0] = dist_u(r, 1) * (P[bin + 1] - P[bin]) + P[bin];
  } else {  // DIST_BETA_UNIFORM, beta_uniform.jl:36-42
    if (dist_u(r, 255) < P[0]) {
      const double g1 = gamma_std(r, P[1], 0, tab), g2 = gamma_std(r, P[2], kSecond, tab);
      x[0] = g1 / (g1 + g2);
    } else {
      x[0] = dist_u(r, 254);
    }
  }
}

// ------------------------------------------------------------------ kernels
struct DistArgs {
  int64_t n;
  int dim;           // value components (vector distributions), else 1
  int K;             // bins (categorical, piecewise_uniform)
  int prow;          // doubles per parameter row
  int pstride;       // 0: one row for every value; prow: row i for value i
  const double* params;
  const double* x;   // [dim][n] (logpdf)
  double* out;       // logpdf: [n]; random: [dim][n]
  uint64_t seed;
};

template <int DIST>
__global__ __launch_bounds__(256) void k_dist_logpdf(DistArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  a.out[i] = dist_logpdf<DIST>(a.x + i, a.n, a.params + i * a.pstride, a.dim, a.K);
}

template <int DIST>
__global__ __launch_bounds__(256) void k_dist_random(DistArgs a) {
  __shared__ double tab[kMathTabDoubles];
  load_math_tab(tab);
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  dist_random<DIST>(DistRng{a.seed, (uint64_t)i}, a.out + i, a.n, a.params + i * a.pstride, a.dim, a.K, tab);
}

}  // namespace gh
