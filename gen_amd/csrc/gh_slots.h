// gh_slots.h — the slot-described state-space family (GH_FAMILY_SLOTS).
//
// A Static-DSL Unfold kernel whose choices are given as address slots rather
// than as a hand-lowered family: one latent address and up to kMaxSlots
// observed addresses per step, each {distribution, dimension, mean form}
// (include/gen_hip.h documents the parameter layout).  The device functor
// below evaluates what Gen's generated code computes for one particle of
// such a kernel (static_ir/generate.jl:24-43, 68-109: every constrained
// choice adds its logpdf to the weight, every unconstrained one is drawn):
//
//   latent   x_t ~ mvnormal(A x_{t-1} + b, Q)      (x_1 ~ mvnormal(mu0, P0); with per-step
//            inputs b + u_t, u_t the step's kernel argument)
//         or z_t ~ categorical(T[:, z_{t-1}])       (z_1 ~ categorical(prior); stored one-hot, d = K)
//         or x_t ~ normal(x/2 + 25x/(1+x^2) + 8cos(1.2t), sd_x)   (d = 1;
//            x_1 ~ normal(mu1, s1)) — examples/pmmh/model.jl:9-13
//         or two latent addresses, a switching linear-Gaussian state:
//            z_t ~ categorical(T[:, z_{t-1}]), x_t ~ mvnormal(A_z x_{t-1} + b_z, Q_z)
//            (z_1 ~ categorical(prior), x_1 ~ mvnormal(mu0, P0)); stored as
//            x (dx values) then z one-hot (nz values), d = dx + nz
//   slots    mvnormal(H x + c, R)                         mvnormal.jl:12-16
//            normal(h.x + c, sd) or normal(x^2/20, sd)    normal.jl:56-60
//            normal(h.x + c, exp(g.x + s))                normal.jl:56-60 (stochastic volatility)
//            poisson(exp(h.x + c))                        poisson.jl:10-12
//            bernoulli(1 / (1 + exp(-(h.x + c))))         bernoulli.jl:10-12
//            categorical(softmax(W x + c))                categorical.jl:10-12 (0-based values)
//            any scalar distribution of Gen's library (gh_dists.h: normal, uniform,
//            uniform_discrete, bernoulli, gamma, inv_gamma, beta, exponential, poisson,
//            binom, neg_binom, geometric, laplace, cauchy, beta_uniform) whose
//            arguments are each link_j(h_j.x + c_j), link identity / exp / logistic
//
// Each step constrains any subset of the observed slots (a gh_obs chain with
// slot ids, choice_map.jl:163-225); the weight is the sum of the present
// slots' logpdfs in slot order.  The arithmetic follows the hand-tuned
// families where they coincide, so an LGSSM written as slots (affine latent,
// one mvnormal slot) and the nonlinear SSM written as slots (Kitagawa latent,
// one normal slot with the x^2/20 mean) give the LGSSM / Kitagawa families'
// states, weights and ancestors bit for bit; those families stay the fast
// specialisations.  oracle/gh_oracle.c restates every line (slot_* there).
#pragma once
#include "gh_dists.h"
#include "gh_models.h"

namespace gh {

constexpr int kMaxSlots = 4;        // observed addresses per step
constexpr int kMaxSlotD = 16;       // latent dimension (SlotModel<1..16> instantiated)
constexpr int kMaxSlotClasses = 16;  // categorical slot classes
constexpr uint32_t kSlotSimDraws = 32;  // simulate(): slot k draws from kSimObsDraw + 32 k

enum SlotDist : int {
  SLOT_MVNORMAL = 1, SLOT_NORMAL = 2, SLOT_POISSON = 3, SLOT_BERNOULLI = 4, SLOT_CATEGORICAL = 5,
  SLOT_LIBRARY = 6  // m = the gh_dists.h distribution id
};
constexpr uint32_t kSlotLibDraw = 1024;  // simulate(): library slot k draws from kSlotLibDraw + 256 k

// A library slot's distribution: its argument count (0: not a scalar
// distribution a slot may name)
GH_HD int lib_nargs(int dist) {
  switch (dist) {
    case DIST_BERNOULLI: case DIST_EXPONENTIAL: case DIST_POISSON: case DIST_GEOMETRIC:
      return 1;
    case DIST_NORMAL: case DIST_UNIFORM_CONTINUOUS: case DIST_UNIFORM_DISCRETE: case DIST_GAMMA:
    case DIST_INV_GAMMA: case DIST_BETA: case DIST_BINOMIAL: case DIST_NEG_BINOMIAL: case DIST_LAPLACE:
    case DIST_CAUCHY:
      return 2;
    case DIST_BETA_UNIFORM:
      return 3;
    default:
      return 0;
  }
}
// argument j of a library slot: link (0 identity, 2 exp, 3 logistic) applied to c + h.x
// (the block holds link h[d] c per argument)
enum : int { LIB_IDENTITY = 0, LIB_EXP = 2, LIB_LOGISTIC = 3 };
GH_HD double lib_link(int link, double eta) {
  return link == LIB_EXP ? gh_exp(eta) : (link == LIB_LOGISTIC ? 1.0 / (1.0 + gh_exp(-eta)) : eta);
}
// the library's logpdf and sampler by run-time id (out of line, in the
// extended instantiations only; the sampler reads the Box–Muller tables from
// the constant copy: an LDS table pointer handed to the call came back unusable
// to the caller's later normal draws — see DESIGN.md §5)
static __device__ __noinline__ double lib_logpdf(int dist, double v, double a0, double a1, double a2) {
  const double P[3] = {a0, a1, a2};
  switch (dist) {
    case DIST_NORMAL: return dist_logpdf<DIST_NORMAL>(&v, 1, P, 1, 0);
    case DIST_UNIFORM_CONTINUOUS: return dist_logpdf<DIST_UNIFORM_CONTINUOUS>(&v, 1, P, 1, 0);
    case DIST_UNIFORM_DISCRETE: return dist_logpdf<DIST_UNIFORM_DISCRETE>(&v, 1, P, 1, 0);
    case DIST_BERNOULLI: return dist_logpdf<DIST_BERNOULLI>(&v, 1, P, 1, 0);
    case DIST_GAMMA: return dist_logpdf<DIST_GAMMA>(&v, 1, P, 1, 0);
    case DIST_INV_GAMMA: return dist_logpdf<DIST_INV_GAMMA>(&v, 1, P, 1, 0);
    case DIST_BETA: return dist_logpdf<DIST_BETA>(&v, 1, P, 1, 0);
    case DIST_EXPONENTIAL: return dist_logpdf<DIST_EXPONENTIAL>(&v, 1, P, 1, 0);
    case DIST_POISSON: return dist_logpdf<DIST_POISSON>(&v, 1, P, 1, 0);
    case DIST_BINOMIAL: return dist_logpdf<DIST_BINOMIAL>(&v, 1, P, 1, 0);
    case DIST_NEG_BINOMIAL: return dist_logpdf<DIST_NEG_BINOMIAL>(&v, 1, P, 1, 0);
    case DIST_GEOMETRIC: return dist_logpdf<DIST_GEOMETRIC>(&v, 1, P, 1, 0);
    case DIST_LAPLACE: return dist_logpdf<DIST_LAPLACE>(&v, 1, P, 1, 0);
    case DIST_CAUCHY: return dist_logpdf<DIST_CAUCHY>(&v, 1, P, 1, 0);
    default: return dist_logpdf<DIST_BETA_UNIFORM>(&v, 1, P, 1, 0);
  }
}
static __device__ __noinline__ double lib_random(int dist, uint64_t seed, uint64_t pid, uint32_t t, uint32_t base, double a0,
                                          double a1, double a2) {
  const double* tab = gh_math_tab_dev;
  const double P[3] = {a0, a1, a2};
  const DistRng r{seed, pid, t, STREAM_SIM, base};
  double x = 0.0;
  switch (dist) {
    case DIST_NORMAL: dist_random<DIST_NORMAL>(r, &x, 1, P, 1, 0, tab); break;
    case DIST_UNIFORM_CONTINUOUS: dist_random<DIST_UNIFORM_CONTINUOUS>(r, &x, 1, P, 1, 0, tab); break;
    case DIST_UNIFORM_DISCRETE: dist_random<DIST_UNIFORM_DISCRETE>(r, &x, 1, P, 1, 0, tab); break;
    case DIST_BERNOULLI: dist_random<DIST_BERNOULLI>(r, &x, 1, P, 1, 0, tab); break;
    case DIST_GAMMA: dist_random<DIST_GAMMA>(r, &x, 1, P, 1, 0, tab); break;
    case DIST_INV_GAMMA: dist_random<DIST_INV_GAMMA>(r, &x, 1, P, 1, 0, tab); break;
    case DIST_BETA: dist_random<DIST_BETA>(r, &x, 1, P, 1, 0, tab); break;
    case DIST_EXPONENTIAL: dist_random<DIST_EXPONENTIAL>(r, &x, 1, P, 1, 0, tab); break;
    case DIST_POISSON: dist_random<DIST_POISSON>(r, &x, 1, P, 1, 0, tab); break;
    case DIST_BINOMIAL: dist_random<DIST_BINOMIAL>(r, &x, 1, P, 1, 0, tab); break;
    case DIST_NEG_BINOMIAL: dist_random<DIST_NEG_BINOMIAL>(r, &x, 1, P, 1, 0, tab); break;
    case DIST_GEOMETRIC: dist_random<DIST_GEOMETRIC>(r, &x, 1, P, 1, 0, tab); break;
    case DIST_LAPLACE: dist_random<DIST_LAPLACE>(r, &x, 1, P, 1, 0, tab); break;
    case DIST_CAUCHY: dist_random<DIST_CAUCHY>(r, &x, 1, P, 1, 0, tab); break;
    default: dist_random<DIST_BETA_UNIFORM>(r, &x, 1, P, 1, 0, tab); break;
  }
  return x;
}
enum SlotLink : int {
  LINK_AFFINE = 0, LINK_KITAGAWA = 1, LINK_EXP = 2, LINK_LOGISTIC = 3, LINK_SOFTMAX = 4,
  LINK_LOGSCALE = 5  // normal slot with a log-linear standard deviation
};
// (latent form 2 — affine with per-step inputs — is SLOT_LAT_AFFINE with uoff >= 0)
enum SlotLatent : int { SLOT_LAT_AFFINE = 0, SLOT_LAT_KITAGAWA = 1, SLOT_LAT_CATEGORICAL = 3, SLOT_LAT_SWITCHING = 4 };
constexpr int kMaxRegimes = 8;  // switching latent: regimes

struct SlotParams {
  const double* base;
  // affine latent: A | b | chol(Q) | mu0 | chol(P0) in the device buffer
  const double *A, *b, *LQ, *mu0, *L0;
  // categorical latent (K = d classes, one-hot state): prior[K] | T[K*K], T[new*K + prev]
  const double *cprior, *cT;
  double cstQ, cst0;  // their log-normalisers (score columns)
  // switching latent (nz regimes, state x[dx] | one-hot z[nz]): prior | T as above,
  // then per regime A_z [dx*dx] | b_z [dx] | chol(Q_z) [dx*dx] (SW), mu0 [dx] | chol(P0) [dx*dx]
  const double* SW;
  int nz;
  double cstQz[kMaxRegimes];
  KitParams kit;      // Kitagawa latent (mu1, s1, sx, inv2vx, cstx, inv2v1, cst1)
  int lat, K;
  int dist[kMaxSlots], m[kMaxSlots], link[kMaxSlots];
  int voff[kMaxSlots];  // the slot's values in StepObs::v
  int yoff[kMaxSlots];  // the slot's rows in simulate()'s output
  // per slot: mvnormal M = L_R^-1 H [m*d] | H [m*d] | c [m] | L_R [m*m];
  // normal / poisson / bernoulli h [d] | c (log-linear normal: h [d] | c | g [d] | s);
  // categorical W [m*d] | c [m]; library (link | h [d] | c) per argument
  const double* P[kMaxSlots];
  double cst[kMaxSlots];    // mvnormal -0.5 (m log 2pi + log det R); normal -0.5 log(2 pi sd^2)
  double inv2v[kMaxSlots];  // normal 1 / (2 sd^2)
  double sd[kMaxSlots];     // normal sd (simulate)
  // (the observed values fill StepObs::v[0..voff of the last slot + its count); a poisson slot takes 2)
  // dependencies between the observed addresses of one step: slot k's linear
  // predictor adds delta_k = sum_{j<k} dg[k][j] y_j over its scalar parent slots
  // (dep: the slots with parents; filtering reads delta_k from v[doff + k], the
  // host's fma chain over the constrained parents; simulate forms it from the draws)
  int dep, doff;
  double dg[kMaxSlots][kMaxSlots];
  int uoff;                 // the step's latent input u_t (affine latent with inputs) in v[uoff..], or -1
  int qoff;                 // the linear proposal's mean offset in v[qoff..] (after the input, if any)
  // the linear custom proposal (SlotLinModel): the filter's own buffer,
  // absolute pointers (not rebased): P d*d | chol(Sigma_q) d*d
  const double* QP;
  const double* QL;
  double cstq;              // -0.5 (d log 2pi + log det Sigma_q)
  __device__ SlotParams rebase(const double* __restrict__ prm) const {
    SlotParams q = *this;
    q.A = rebased(*this, prm, A);
    q.b = rebased(*this, prm, b);
    q.LQ = rebased(*this, prm, LQ);
    q.mu0 = rebased(*this, prm, mu0);
    q.L0 = rebased(*this, prm, L0);
    q.cprior = rebased(*this, prm, cprior);
    q.cT = rebased(*this, prm, cT);
    q.SW = rebased(*this, prm, SW);
#pragma unroll
    for (int k = 0; k < kMaxSlots; ++k) q.P[k] = rebased(*this, prm, P[k]);
    return q;
  }
};

// EXT: the extended instantiations, for a model with a library slot (its
// logpdf and sampler are out-of-line calls) or the switching latent; the
// others keep the leaner call-free kernels
template <int D, bool EXT = false>
struct SlotModel {
  static constexpr int kD = D;
  static constexpr int kMinWaves = D <= 3 ? 8 : (D <= 6 ? 6 : (D <= 10 ? 4 : 3));
  using Params = SlotParams;

  // c + h.x (fma over the components ascending)
  __device__ static double affine(const double* h, double c, const double* x) {
    double acc = c;
#pragma unroll
    for (int j = 0; j < D; ++j) acc = fma(h[j], x[j], acc);
    return acc;
  }

  // normal.jl:56-60 literally, with std = exp(eta): var = std * std,
  // -(diff * diff) / (2 var) - 0.5 log(2 pi var)
  __device__ static double normal_logscale_lpdf(double diff, double eta) {
    const double sd = gh_exp(eta);
    const double var = sd * sd;
    return -(diff * diff) / (2.0 * var) - 0.5 * gh_log(0x1.921fb54442d18p+2 * var);
  }

  // a library slot's arguments at latent x (the parent term joins the first one)
  __device__ static void lib_args(const Params& p, const double* P, int na, const double* x, int k, double dk,
                                  double a[3]) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const double* B = P + j * (D + 2);
      a[j] = j < na ? lib_link((int)B[0], j == 0 ? eta(p, B + 1, B[D + 1], x, k, dk) : affine(B + 1, B[D + 1], x))
                    : 0.0;
    }
  }

  // the regime of a switching state (its one-hot tail x[dx..D))
  __device__ static int regime(const Params& p, const double* x) {
    const int dx = D - p.nz;
    int z = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) z = (j >= dx && x[j] != 0.0) ? j - dx : z;
    return z;
  }

  // the class of a one-hot categorical latent
  __device__ static int onehot(const double* x) {
    int z = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) z = x[j] != 0.0 ? j : z;
    return z;
  }

  // c + h.x, plus slot k's parent term when it has parents
  __device__ static double eta(const Params& p, const double* h, double c, const double* x, int k, double dk) {
    const double e = affine(h, c, x);
    return ((p.dep >> k) & 1) ? e + dk : e;
  }

  // the logpdf of slot k's value (o.v + voff) at latent x; dk: its parent term
  __device__ static double slot_lpdf(const Params& p, const StepObs& o, int k, const double* x) {
    return slot_lpdf_d(p, o.v + p.voff[k], k, x, ((p.dep >> k) & 1) ? o.v[p.doff + k] : 0.0);
  }
  __device__ static double slot_lpdf_d(const Params& p, const double* v, int k, const double* x, double dk) {
    const double* P = p.P[k];
    const int m = p.m[k];
    switch (p.dist[k]) {
      case SLOT_LIBRARY: {  // the library's logpdf (gh_dists.h, the reference's formulas)
        if constexpr (EXT) {
          double a[3];
          lib_args(p, P, lib_nargs(m), x, k, dk, a);
          return lib_logpdf(m, v[0], a[0], a[1], a[2]);
        } else {
          return NAN;  // (never: the host picks the EXT instantiation for such a model)
        }
      }
      case SLOT_MVNORMAL: {  // LGModel::obs (dense): v = L_R^-1 (y - c)
        double quad = 0.0;
        for (int r = 0; r < m; ++r) {
          double acc = v[r];
#pragma unroll
          for (int j = 0; j < D; ++j) acc = fma(-P[r * D + j], x[j], acc);
          quad = fma(acc, acc, quad);
        }
        return p.cst[k] - 0.5 * quad;
      }
      case SLOT_NORMAL: {
        const double mean = p.link[k] == LINK_KITAGAWA ? div20(x[0] * x[0]) : eta(p, P, P[D], x, k, dk);
        const double diff = v[0] - mean;
        if (p.link[k] == LINK_LOGSCALE) return normal_logscale_lpdf(diff, affine(P + D + 1, P[2 * D + 1], x));
        return -(diff * diff) * p.inv2v[k] + p.cst[k];
      }
      case SLOT_POISSON: {  // poisson.jl:10-12 with lambda = exp(h.x + c); v[1] = log Gamma(y + 1)
        const double lam = gh_exp(eta(p, P, P[D], x, k, dk));
        return v[0] < 0.0 ? -INFINITY : (v[0] * gh_log(lam) - lam) - v[1];
      }
      case SLOT_BERNOULLI: {  // bernoulli.jl:10-12 with prob = 1 / (1 + exp(-(h.x + c)))
        const double prob = 1.0 / (1.0 + gh_exp(-eta(p, P, P[D], x, k, dk)));
        return v[0] != 0.0 ? gh_log(prob) : gh_log(1.0 - prob);
      }
      default: {  // categorical.jl:10-12 with probs = softmax(W x + c): exp(eta - max) / sum
        // (eta_j recomputed per pass: no per-lane array indexed at run time)
        double mx = -INFINITY;
        for (int j = 0; j < m; ++j) mx = fmax(mx, affine(P + j * D, P[m * D + j], x));
        double s = 0.0, ey = 0.0;
        const int y = (int)v[0];
        for (int j = 0; j < m; ++j) {
          const double e = gh_exp(affine(P + j * D, P[m * D + j], x) - mx);
          s += e;
          if (j == y) ey = e;
        }
        return gh_log(ey / s);
      }
    }
  }

  // the weight: the present slots' logpdfs (o.present bit k) in slot order
  __device__ static double loglik(const Params& p, const StepObs& o, const double* x) {
    double w = 0.0;
#pragma unroll
    for (int k = 0; k < kMaxSlots; ++k)
      if (k < p.K && ((o.present >> k) & 1)) w = w + slot_lpdf(p, o, k, x);
    return w;
  }

  // the latent's logpdf (LGModel<D, 0>::score / KitModel::score forms)
  __device__ static double latent_lpdf(const Params& p, const StepObs& o, uint32_t t, const double* xp,
                                       const double* x) {
    if (p.lat == SLOT_LAT_CATEGORICAL)  // categorical.jl:10-12: log prior[z] or log T[z | z_prev]
      return gh_log(t == 1 ? p.cprior[onehot(x)] : p.cT[onehot(x) * D + onehot(xp)]);
    if (EXT && p.lat == SLOT_LAT_SWITCHING) {  // log p(z | z_prev) + mvnormal.jl:12-16 under regime z, in that order
      const int dx = D - p.nz, z = regime(p, x);
      const double* blk = p.SW + z * (2 * dx * dx + dx);
      const double lz = gh_log(t == 1 ? p.cprior[z] : p.cT[z * p.nz + regime(p, xp)]);
      const double* L = t == 1 ? p.L0 : blk + dx * dx + dx;
      double u[D];
      double quad = 0.0;
#pragma unroll
      for (int i = 0; i < D; ++i) {
        if (i >= dx) break;
        double mean;
        if (t == 1) {
          mean = p.mu0[i];
        } else {
          mean = blk[dx * dx + i];
#pragma unroll
          for (int k = 0; k < D; ++k)
            if (k < dx) mean = fma(blk[i * dx + k], xp[k], mean);
        }
        double r = x[i] - mean;
#pragma unroll
        for (int k = 0; k < i; ++k) r = fma(-L[i * dx + k], u[k], r);
        u[i] = r / L[i * dx + i];
        quad = fma(u[i], u[i], quad);
      }
      return lz + ((t == 1 ? p.cst0 : p.cstQz[z]) - 0.5 * quad);
    }
    if (p.lat == SLOT_LAT_KITAGAWA) {
      double mean = p.kit.mu1, inv2 = p.kit.inv2v1, cst = p.kit.cst1;
      if (t > 1) {
        mean = KitModel::mean(o, xp[0]);
        inv2 = p.kit.inv2vx;
        cst = p.kit.cstx;
      }
      const double d = x[0] - mean;
      return -(d * d) * inv2 + cst;
    }
    const double* L = t == 1 ? p.L0 : p.LQ;
    double u[D];
    double quad = 0.0;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double mean;
      if (t == 1) {
        mean = p.mu0[i];
      } else {
        mean = p.uoff >= 0 ? p.b[i] + o.v[p.uoff + i] : p.b[i];  // (the step's input u_t: an Unfold argument)
#pragma unroll
        for (int k = 0; k < D; ++k) mean = fma(p.A[i * D + k], xp[k], mean);
      }
      double r = x[i] - mean;
#pragma unroll
      for (int k = 0; k < i; ++k) r = fma(-L[i * D + k], u[k], r);
      u[i] = r / L[i * D + i];
      quad = fma(u[i], u[i], quad);
    }
    return (t == 1 ? p.cst0 : p.cstQ) - 0.5 * quad;
  }

  __device__ static void score(const Params& p, const StepObs& o, uint32_t t, const double* xp, const double* x,
                               double* lat, double* ob) {
    *lat = latent_lpdf(p, o, t, xp, x);
    *ob = loglik(p, o, x);
  }

  // the latent draw of step t (t = 1: from the initial distribution)
  __device__ static void draw_latent(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid, uint32_t t,
                                     const double* xp, double* x, const Draw& dr) {
    if (p.lat == SLOT_LAT_CATEGORICAL) {  // inverse-CDF draw (categorical.jl:20-22), as HMMModel's
      const u32x4 w = rng_block(seed, pid, t, dr.stream, dr.base);
      const double u = u53(w.x, w.y);
      const int z = t == 1 ? cat_sample(p.cprior, D, 1, u) : cat_sample(p.cT + onehot(xp), D, D, u);
#pragma unroll
      for (int j = 0; j < D; ++j) x[j] = j == z ? 1.0 : 0.0;
      return;
    }
    if (EXT && p.lat == SLOT_LAT_SWITCHING) {  // the regime (inverse CDF, draw base), then x given it (normals from base + 1)
      const int dx = D - p.nz;
      const u32x4 w = rng_block(seed, pid, t, dr.stream, dr.base);
      const double u = u53(w.x, w.y);
      const int z = t == 1 ? cat_sample(p.cprior, p.nz, 1, u) : cat_sample(p.cT + regime(p, xp), p.nz, p.nz, u);
      const double* blk = p.SW + z * (2 * dx * dx + dx);
      const double* L = t == 1 ? p.L0 : blk + dx * dx + dx;
      double zn[D + 1];
      normals_n<D>(seed, pid, t, dr.stream, dr.base + 1, zn, dr.tab);
#pragma unroll
      for (int i = 0; i < D; ++i) {
        if (i < dx) {
          double acc;
          if (t == 1) {
            acc = p.mu0[i];
          } else {
            acc = blk[dx * dx + i];
#pragma unroll
            for (int k = 0; k < D; ++k)
              if (k < dx) acc = fma(blk[i * dx + k], xp[k], acc);
          }
#pragma unroll
          for (int k = 0; k <= i; ++k) acc = fma(L[i * dx + k], zn[k], acc);
          x[i] = acc;
        } else {
          x[i] = i - dx == z ? 1.0 : 0.0;
        }
      }
      return;
    }
    if (p.lat == SLOT_LAT_KITAGAWA) {  // the nonlinear SSM's paired normals (KitModel::znorm)
      const double z = KitModel::znorm(seed, pid, t, dr);
      x[0] = t == 1 ? p.kit.mu1 + p.kit.s1 * z : KitModel::mean(o, xp[0]) + p.kit.sx * z;
      return;
    }
    double z[D + 1];
    normals_n<D>(seed, pid, t, dr.stream, dr.base, z, dr.tab);
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double acc;
      if (t == 1) {
        acc = p.mu0[i];
#pragma unroll
        for (int k = 0; k <= i; ++k) acc = fma(p.L0[i * D + k], z[k], acc);
      } else {
        acc = p.uoff >= 0 ? p.b[i] + o.v[p.uoff + i] : p.b[i];
#pragma unroll
        for (int k = 0; k < D; ++k) acc = fma(p.A[i * D + k], xp[k], acc);
#pragma unroll
        for (int k = 0; k <= i; ++k) acc = fma(p.LQ[i * D + k], z[k], acc);
      }
      x[i] = acc;
    }
  }

  __device__ static double init(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid, int /*proposal*/,
                                double* x, Draw dr = {STREAM_INIT, 0}) {
    draw_latent(p, o, seed, pid, 1, nullptr, x, dr);
    return loglik(p, o, x);
  }

  __device__ static double step(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid, uint32_t t,
                                int /*proposal*/, const double* xp, double* x, Draw dr = {STREAM_STEP, 0}) {
    draw_latent(p, o, seed, pid, t, xp, x, dr);
    return loglik(p, o, x);
  }

  // simulate(): every slot's value drawn from the model (slot k from its own
  // draws kSimObsDraw + 32 k of the SIM stream), written to rows yoff[k].. with
  // stride ys, and the sum of their logpdfs
  __device__ static double sim_obs(const Params& p, uint64_t seed, uint64_t pid, uint32_t t, const double* x,
                                   double* y, int64_t ys, const double* tab) {
    double total = 0.0;
    double ysc[kMaxSlots];  // the scalar slots' draws (the parents of later slots)
    // (a rolled loop: the unrolled form of the extended instantiation, four
    // copies of every slot kind around the library calls, came out with wrong
    // draws after the first call — DESIGN.md §5)
#pragma unroll 1
    for (int k = 0; k < kMaxSlots; ++k) {
      if (k >= p.K) break;
      const double* P = p.P[k];
      const int m = p.m[k];
      const uint32_t draw = kSimObsDraw + kSlotSimDraws * (uint32_t)k;
      double* yk = y + (int64_t)p.yoff[k] * ys;
      double dk = 0.0;  // the parent term, as the host forms it for a step (fma over the parents in slot order)
      if ((p.dep >> k) & 1) {
#pragma unroll
        for (int j = 0; j < kMaxSlots; ++j)
          if (j < k && p.dg[k][j] != 0.0) dk = fma(p.dg[k][j], ysc[j], dk);
      }
      double lp;
      switch (p.dist[k]) {
        case SLOT_LIBRARY: {  // the library's sampler (gh_dists.h) on draws kSlotLibDraw + 256 k
          if constexpr (EXT) {
            double a[3];
            lib_args(p, P, lib_nargs(m), x, k, dk, a);
            yk[0] = lib_random(m, seed, pid, t, kSlotLibDraw + 256u * (uint32_t)k, a[0], a[1], a[2]);
            lp = lib_logpdf(m, yk[0], a[0], a[1], a[2]);
          } else {
            yk[0] = NAN;
            lp = NAN;
          }
          break;
        }
        case SLOT_MVNORMAL: {  // y = H x + c + L_R z, scored through L_R^-1 (y - c) (LGModel::sim_obs)
          const double *H = P + m * D, *c = H + m * D, *LR = c + m;
          double z[kMaxObs], v[kMaxObs];
          normals_rt(seed, pid, t, STREAM_SIM, draw, m, z, tab);
          for (int r = 0; r < m; ++r) {
            double acc = c[r];
#pragma unroll
            for (int j = 0; j < D; ++j) acc = fma(H[r * D + j], x[j], acc);
            for (int q = 0; q <= r; ++q) acc = fma(LR[r * m + q], z[q], acc);
            yk[r * ys] = acc;
            double s = acc - c[r];
            for (int q = 0; q < r; ++q) s = fma(-LR[r * m + q], v[q], s);
            v[r] = s / LR[r * m + r];
          }
          double quad = 0.0;
          for (int r = 0; r < m; ++r) {
            double acc = v[r];
#pragma unroll
            for (int j = 0; j < D; ++j) acc = fma(-P[r * D + j], x[j], acc);
            quad = fma(acc, acc, quad);
          }
          lp = p.cst[k] - 0.5 * quad;
          break;
        }
        case SLOT_NORMAL: {
          double z0, z1;
          normal_pair(rng_block(seed, pid, t, STREAM_SIM, draw), &z0, &z1, tab);
          const double mean = p.link[k] == LINK_KITAGAWA ? div20(x[0] * x[0]) : eta(p, P, P[D], x, k, dk);
          if (p.link[k] == LINK_LOGSCALE) {
            const double eta = affine(P + D + 1, P[2 * D + 1], x);
            yk[0] = mean + gh_exp(eta) * z0;
            lp = normal_logscale_lpdf(yk[0] - mean, eta);
            break;
          }
          yk[0] = mean + p.sd[k] * z0;
          const double diff = yk[0] - mean;
          lp = -(diff * diff) * p.inv2v[k] + p.cst[k];
          break;
        }
        case SLOT_POISSON: {
          const u32x4 w = rng_block(seed, pid, t, STREAM_SIM, draw);
          const double lam = gh_exp(eta(p, P, P[D], x, k, dk));
          const double v = poisson_chop(lam, u53(w.x, w.y));
          yk[0] = v;
          lp = (v * gh_log(lam) - lam) - gh_lgamma(v + 1.0);
          break;
        }
        case SLOT_BERNOULLI: {  // bernoulli.jl:19: rand() < prob
          const u32x4 w = rng_block(seed, pid, t, STREAM_SIM, draw);
          const double prob = 1.0 / (1.0 + gh_exp(-eta(p, P, P[D], x, k, dk)));
          const bool b = u53(w.x, w.y) < prob;
          yk[0] = b ? 1.0 : 0.0;
          lp = b ? gh_log(prob) : gh_log(1.0 - prob);
          break;
        }
        default: {  // categorical: inverse CDF over the softmax weights e_j (dist_cat's sums)
          const u32x4 w = rng_block(seed, pid, t, STREAM_SIM, draw);
          double mx = -INFINITY;
          for (int j = 0; j < m; ++j) mx = fmax(mx, affine(P + j * D, P[m * D + j], x));
          double s = 0.0;
          for (int j = 0; j < m; ++j) s += gh_exp(affine(P + j * D, P[m * D + j], x) - mx);
          const double target = u53(w.x, w.y) * s;
          double cum = 0.0, ey = 0.0, elast = 0.0;
          int yv = -1, last = -1;
          for (int j = 0; j < m && yv < 0; ++j) {
            const double e = gh_exp(affine(P + j * D, P[m * D + j], x) - mx);
            cum += e;
            if (e > 0.0) {
              last = j;
              elast = e;
            }
            if (cum > target && e > 0.0) {
              yv = j;
              ey = e;
            }
          }
          if (yv < 0) {
            yv = last;
            ey = elast;
          }
          yk[0] = (double)yv;
          lp = gh_log(ey / s);
          break;
        }
      }
      total = total + lp;
      ysc[k] = yk[0];
    }
    return total;
  }
};

// A user-parameterised linear-Gaussian custom proposal for the slot family
// (GH_PROPOSAL_LINEAR; the LG-SSM's LGLinModel over any slot model):
// q(x_t | x_{t-1}) = mvnormal(P x_{t-1} + u_t, Sigma_q) (t = 1: mvnormal(u_1,
// Sigma_q)), u_t per step after the slot values (and the latent input).  The weight is Gen's
// custom-proposal weight (particle_filter.jl:79-91,139-154 via
// trace_translators.jl:775-802): the model's score of the new choices — the
// latent's logpdf (affine or Kitagawa) and the present slots' — minus q's
// logpdf of the drawn value.
template <int D, bool EXT = false>
struct SlotLinModel {
  static constexpr int kD = D;
  static constexpr int kMinWaves = SlotModel<D, EXT>::kMinWaves;
  using Params = SlotParams;
  using Prior = SlotModel<D, EXT>;

  __device__ static double loglik(const Params& p, const StepObs& o, const double* x) { return Prior::loglik(p, o, x); }

  // x = mean + L_q z with mean = u (+ P xp); returns log q(x), the mean
  // recomputed in the same order (LGLinModel::draw)
  __device__ static double draw(const Params& p, const StepObs& o, const double* xp, const double* z, double* x) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double acc = o.v[p.qoff + i];
      if (xp) {
#pragma unroll
        for (int k = 0; k < D; ++k) acc = fma(p.QP[i * D + k], xp[k], acc);
      }
#pragma unroll
      for (int k = 0; k <= i; ++k) acc = fma(p.QL[i * D + k], z[k], acc);
      x[i] = acc;
    }
    double w[D];
    double quad = 0.0;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double mean = o.v[p.qoff + i];
      if (xp) {
#pragma unroll
        for (int k = 0; k < D; ++k) mean = fma(p.QP[i * D + k], xp[k], mean);
      }
      double r = x[i] - mean;
#pragma unroll
      for (int k = 0; k < i; ++k) r = fma(-p.QL[i * D + k], w[k], r);
      w[i] = r / p.QL[i * D + i];
      quad = fma(w[i], w[i], quad);
    }
    return p.cstq - 0.5 * quad;
  }

  __device__ static double init(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid, int /*proposal*/,
                                double* x, Draw dr = {STREAM_INIT, 0}) {
    double z[D + 1];
    normals_n<D>(seed, pid, 1, dr.stream, dr.base, z, dr.tab);
    const double lq = draw(p, o, nullptr, z, x);
    double lat, ob;
    Prior::score(p, o, 1, x, x, &lat, &ob);
    return (lat + ob) - lq;
  }

  __device__ static double step(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid, uint32_t t,
                                int /*proposal*/, const double* xp, double* x, Draw dr = {STREAM_STEP, 0}) {
    double z[D + 1];
    normals_n<D>(seed, pid, t, dr.stream, dr.base, z, dr.tab);
    const double lq = draw(p, o, xp, z, x);
    double lat, ob;
    Prior::score(p, o, t, xp, x, &lat, &ob);
    return (lat + ob) - lq;
  }
};

}  // namespace gh
