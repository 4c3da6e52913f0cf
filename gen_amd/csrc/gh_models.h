// gh_models.h — the model families the engine lowers to device code.
//
// Each family is the hand-lowered form of one Static-DSL model wrapped in an
// Unfold combinator.  The per-particle functions are exactly what Gen's
// generated code computes for one particle:
//
//   init(..)  = generate(model, (1, ...), obs_1)       static_ir/generate.jl:24-43
//               constrained choice  -> weight += logpdf (generate.jl:31-34)
//               unconstrained choice-> value = random   (generate.jl:35-37)
//   step(..)  = update(trace, (t, ...), (UnknownChange(),), obs_t) restricted to
//               the newly appended Unfold application (unfold/update.jl:54-78):
//               sample the new latent from the prior, weight = logpdf(obs | latent)
//
// With the "optimal" proposal the weight is model_weight - proposal_score
// (particle_filter.jl:79-91,139-154 via trace_translators.jl:775-802), which
// for a categorical latent collapses to log sum_z p(z|z_prev) p(x|z).
//
// The arithmetic (operation order, explicit fma) is the specification in
// DESIGN.md §5 and is mirrored by oracle/gh_oracle.c.
#pragma once
#include "gh_math.h"

namespace gh {

constexpr int kMaxObs = 32;

// Where a particle's draws come from: the step / init streams for the filter,
// the MH stream (with a per-move draw offset) for rejuvenation proposals.
struct Draw {
  uint32_t stream;
  uint32_t base;               // first draw index
  const double* tab = nullptr;  // log table for Box–Muller (LDS copy; nullptr: constant memory)
};

// per-step observation, passed by value in the kernel arguments
struct StepObs {
  double v[kMaxObs];  // LGSSM: L_R^{-1}(y - c); Kitagawa: y; HMM: symbol
  double ct;          // Kitagawa: 8 cos(1.2 t); LGSSM optimal proposal at t = 1: the (constant) weight
  int present;
  int sym;            // HMM symbol (integer copy of v[0])
};

// ------------------------------------------------------------------ LGSSM
// Parameter blocks hold pointers into one device buffer.  rebase() re-derives
// them from the kernel's `const double* __restrict__` argument so the
// compiler can prove no store of the kernel clobbers them and reads them
// through the scalar cache (s_load) instead of per-lane vector loads.
template <class P>
__device__ __forceinline__ const double* rebased(const P& p, const double* __restrict__ prm, const double* ptr) {
  return prm + (ptr - p.base);
}

struct LGParams {
  const double* base; // start of the device parameter buffer
  const double* A;    // d*d
  const double* b;    // d
  const double* LQ;   // d*d lower Cholesky factor of Q
  const double* M;    // dy*d  L_R^{-1} H
  const double* mu0;  // d
  const double* L0;   // d*d lower Cholesky factor of P0
  // locally optimal proposal (LGOptModel): N(F A x + g_t, Sigma), weight
  // log N(y; H (A x + b) + c, S) with S = H Q H^T + R, F = I - K H
  const double* FA;   // d*d F A
  const double* LSig; // d*d chol(Sigma), Sigma = F Q
  const double* WA;   // dy*d L_S^{-1} H A
  const double* LSig1;// d*d chol((I - K_1 H) P0), the t = 1 proposal
  const double* H;    // dy*d  observation matrix  (simulate: y = H x + c + L_R z)
  const double* cv;   // dy    observation offset c
  const double* LR;   // dy*dy lower Cholesky factor of R
  // user-parameterised linear-Gaussian proposal (LGLinModel): the filter's own
  // buffer, absolute pointers (not rebased): QP d*d, QL d*d chol(Sigma_q)
  const double* QP = nullptr;
  const double* QL = nullptr;
  double cstq = 0.0;  // -0.5 (d log 2pi + log det Sigma_q)
  int dy;
  double cstR;        // -0.5 (dy log 2pi + log det R)
  double cstS;        // -0.5 (dy log 2pi + log det S)
  double cstQ, cst0;  // the same for Q and P0 (trace scores, gh_pf_get_scores)
  __device__ LGParams rebase(const double* __restrict__ prm) const {
    LGParams q = *this;
    q.A = rebased(*this, prm, A);
    q.b = rebased(*this, prm, b);
    q.LQ = rebased(*this, prm, LQ);
    q.M = rebased(*this, prm, M);
    q.mu0 = rebased(*this, prm, mu0);
    q.L0 = rebased(*this, prm, L0);
    q.FA = rebased(*this, prm, FA);
    q.LSig = rebased(*this, prm, LSig);
    q.WA = rebased(*this, prm, WA);
    q.LSig1 = rebased(*this, prm, LSig1);
    q.H = rebased(*this, prm, H);
    q.cv = rebased(*this, prm, cv);
    q.LR = rebased(*this, prm, LR);
    return q;
  }
};

// S: structure known at model-compile time (host detects exact zeros):
//   bit 0 — chol(Q) is diagonal:   L z needs only the diagonal terms
//   bit 1 — L_R^{-1} H is diagonal (dy == d): the residual needs only x_r
// The skipped terms are exactly-zero matrix entries; the oracle applies the
// same rule, so both paths stay bit-identical.
template <int D, int S = 0>
struct LGModel {
  static constexpr int kD = D;
  // spill-free register budgets measured with tools/regs.py
  #if defined(GH_LG10_WAVES)  // timing-only variants: occupancy target of the d<=10 diagonal case
  static constexpr int kMinWaves = (D <= 4) ? 8 : (D <= 10 ? (S == 3 ? GH_LG10_WAVES : 5) : 4);
#else
  static constexpr int kMinWaves =
      (D <= 3) ? 8 : (D <= 5 ? 7 : (D < 10 ? (S == 3 && D != 7 && D != 9 ? 6 : 5) : (D == 10 ? (S == 3 ? 7 : 5) : 4)));
#endif
  using Params = LGParams;

  // mvnormal(H x + c, R) logpdf with the Cholesky factor applied on the host
  __device__ static double obs(const Params& p, const StepObs& o, const double* x) {
    if (!o.present) return 0.0;
    double quad = 0.0;
    if (S & 2) {
#pragma unroll
      for (int r = 0; r < D; ++r) {
        const double acc = fma(-p.M[r * D + r], x[r], o.v[r]);
        quad = fma(acc, acc, quad);
      }
    } else {
      for (int r = 0; r < p.dy; ++r) {
        double acc = o.v[r];
#pragma unroll
        for (int j = 0; j < D; ++j) acc = fma(-p.M[r * D + j], x[j], acc);
        quad = fma(acc, acc, quad);
      }
    }
    return p.cstR - 0.5 * quad;
  }

  __device__ static double loglik(const Params& p, const StepObs& o, const double* x) { return obs(p, o, x); }

  // the trace's choice scores of step t (Gen's per-choice score fields,
  // static_ir/trace.jl:91-129): *lat = logpdf(mvnormal(A x_prev + b, Q), x)
  // (t = 1: mvnormal(mu0, P0)) by forward substitution with the Cholesky factor
  // (mvnormal.jl:12-16), *ob = logpdf(mvnormal(H x + c, R), y) (0 if unobserved)
  __device__ static void score(const Params& p, const StepObs& o, uint32_t t, const double* xp, const double* x,
                               double* lat, double* ob) {
    const double* L = t == 1 ? p.L0 : p.LQ;
    double u[D];
    double quad = 0.0;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double mean;
      if (t == 1) {
        mean = p.mu0[i];
      } else {
        mean = p.b[i];
#pragma unroll
        for (int k = 0; k < D; ++k) mean = fma(p.A[i * D + k], xp[k], mean);
      }
      double r = x[i] - mean;
      if (t == 1 || !(S & 1)) {
#pragma unroll
        for (int k = 0; k < i; ++k) r = fma(-L[i * D + k], u[k], r);
      }
      u[i] = r / L[i * D + i];
      quad = fma(u[i], u[i], quad);
    }
    *lat = (t == 1 ? p.cst0 : p.cstQ) - 0.5 * quad;
    *ob = obs(p, o, x);
  }

  // simulate()'s observation (static_ir/simulate.jl:23-34: value = random,
  // score = logpdf of that value): y = H x + c + L_R z written with stride ys,
  // scored as the filter scores a given y (make_obs: v = L_R^{-1}(y - c); obs())
  __device__ static double sim_obs(const Params& p, uint64_t seed, uint64_t pid, uint32_t t, const double* x,
                                   double* y, int64_t ys, const double* tab) {
    double z[kMaxObs], v[kMaxObs];
    normals_rt(seed, pid, t, STREAM_SIM, kSimObsDraw, p.dy, z, tab);
    for (int r = 0; r < p.dy; ++r) {
      double acc = p.cv[r];
#pragma unroll
      for (int j = 0; j < D; ++j) acc = fma(p.H[r * D + j], x[j], acc);
      for (int k = 0; k <= r; ++k) acc = fma(p.LR[r * p.dy + k], z[k], acc);
      y[r * ys] = acc;
      double s = acc - p.cv[r];
      for (int k = 0; k < r; ++k) s = fma(-p.LR[r * p.dy + k], v[k], s);
      v[r] = s / p.LR[r * p.dy + r];
    }
    double quad = 0.0;
    if (S & 2) {
#pragma unroll
      for (int r = 0; r < D; ++r) {
        const double acc = fma(-p.M[r * D + r], x[r], v[r]);
        quad = fma(acc, acc, quad);
      }
    } else {
      for (int r = 0; r < p.dy; ++r) {
        double acc = v[r];
#pragma unroll
        for (int j = 0; j < D; ++j) acc = fma(-p.M[r * D + j], x[j], acc);
        quad = fma(acc, acc, quad);
      }
    }
    return p.cstR - 0.5 * quad;
  }

  __device__ static double init(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid,
                                int /*proposal*/, double* x, Draw dr = {STREAM_INIT, 0}) {
    double z[D + 1];
    normals_n<D>(seed, pid, 1, dr.stream, dr.base, z, dr.tab);
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double acc = p.mu0[i];
#pragma unroll
      for (int k = 0; k <= i; ++k) acc = fma(p.L0[i * D + k], z[k], acc);
      x[i] = acc;
    }
    return obs(p, o, x);
  }

  __device__ static double step(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid,
                                uint32_t t, int /*proposal*/, const double* xp, double* x,
                                Draw dr = {STREAM_STEP, 0}) {
    double z[D + 1];
    normals_n<D>(seed, pid, t, dr.stream, dr.base, z, dr.tab);
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double acc = p.b[i];
#pragma unroll
      for (int k = 0; k < D; ++k) acc = fma(p.A[i * D + k], xp[k], acc);
      if (S & 1) {
        acc = fma(p.LQ[i * D + i], z[i], acc);
      } else {
#pragma unroll
        for (int k = 0; k <= i; ++k) acc = fma(p.LQ[i * D + k], z[k], acc);
      }
      x[i] = acc;
    }
    return obs(p, o, x);
  }
};

// ------------------------------------------------ LGSSM, optimal proposal
// The locally optimal proposal of the linear-Gaussian SSM, a custom proposal
// in Gen's sense (particle_filter.jl:79-91,139-154 via the
// SimpleExtendingTraceTranslator, trace_translators.jl:775-802): x_t is drawn
// from p(x_t | x_{t-1}, y_t) = N(mu, Sigma) and the weight
//   model weight - proposal score = log p(x_t|x_{t-1}) + log p(y_t|x_t) - log q(x_t)
// collapses to log p(y_t | x_{t-1}) = log N(y_t; H (A x_{t-1} + b) + c, S),
// evaluated in that closed form (as the HMM's optimal proposal is).  Host
// precomputes: S = H Q H^T + R, K = Q H^T S^-1, F = I - K H,
// Sigma = F Q; per step the vectors g_t = F b + K (y_t - c) (o.v[i], i < d) and
// v_t = L_S^-1 (y_t - c) - L_S^-1 H b (o.v[d + r]); at t = 1 the proposal mean
// mu_1 (o.v[i]) and the constant weight log N(y_1; H mu0 + c, H P0 H^T + R)
// (o.ct).  Without an observation the proposal is the prior (LGModel).
template <int D>
struct LGOptModel {
  static constexpr int kD = D;
  static constexpr int kMinWaves = (D <= 4) ? 8 : (D <= 8 ? 5 : (D <= 14 ? 4 : 3));
  using Params = LGParams;
  using Prior = LGModel<D, 0>;

  __device__ static double loglik(const Params& p, const StepObs& o, const double* x) { return Prior::loglik(p, o, x); }

  __device__ static double init(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid, int proposal,
                                double* x, Draw dr = {STREAM_INIT, 0}) {
    if (!o.present) return Prior::init(p, o, seed, pid, proposal, x, dr);
    double z[D + 1];
    normals_n<D>(seed, pid, 1, dr.stream, dr.base, z, dr.tab);
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double acc = o.v[i];
#pragma unroll
      for (int k = 0; k <= i; ++k) acc = fma(p.LSig1[i * D + k], z[k], acc);
      x[i] = acc;
    }
    return o.ct;
  }

  __device__ static double step(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid, uint32_t t,
                                int proposal, const double* xp, double* x, Draw dr = {STREAM_STEP, 0}) {
    if (!o.present) return Prior::step(p, o, seed, pid, t, proposal, xp, x, dr);
    double z[D + 1];
    normals_n<D>(seed, pid, t, dr.stream, dr.base, z, dr.tab);
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double acc = o.v[i];
#pragma unroll
      for (int k = 0; k < D; ++k) acc = fma(p.FA[i * D + k], xp[k], acc);
#pragma unroll
      for (int k = 0; k <= i; ++k) acc = fma(p.LSig[i * D + k], z[k], acc);
      x[i] = acc;
    }
    double quad = 0.0;
    for (int r = 0; r < p.dy; ++r) {
      double u = o.v[D + r];
#pragma unroll
      for (int k = 0; k < D; ++k) u = fma(-p.WA[r * D + k], xp[k], u);
      quad = fma(u, u, quad);
    }
    return p.cstS - 0.5 * quad;
  }
};

// --------------------------------- LGSSM, user-parameterised linear proposal
// A custom proposal in Gen's sense (particle_filter.jl:79-91,139-154 via the
// SimpleExtendingTraceTranslator, trace_translators.jl:775-802) whose
// arguments the caller supplies: q(x_t | x_{t-1}) = N(P x_{t-1} + u_t, Sigma_q)
// (t = 1: N(u_1, Sigma_q)), P and chol(Sigma_q) in the filter's buffer, u_t
// per step in o.v[dy + i] (after the observation's L_R^{-1}(y - c)).  The
// weight is the translator's model weight - proposal score:
//   log p(x_t | x_{t-1}) + log p(y_t | x_t) - log q(x_t)
// with the model's densities as the trace's score columns compute them
// (LGModel<D, 0>::score) and q's logpdf of the drawn value by forward
// substitution.
template <int D>
struct LGLinModel {
  static constexpr int kD = D;
  static constexpr int kMinWaves = (D <= 4) ? 8 : (D <= 8 ? 5 : (D <= 14 ? 4 : 3));
  using Params = LGParams;
  using Prior = LGModel<D, 0>;

  __device__ static double loglik(const Params& p, const StepObs& o, const double* x) { return Prior::loglik(p, o, x); }

  // x = mean + L_q z with mean = u (+ P xp); returns log q(x) recomputing the
  // mean in the same order (the logpdf of the value, as mvnormal.jl:14 scores it)
  __device__ static double draw(const Params& p, const StepObs& o, const double* xp, const double* z, double* x) {
#pragma unroll
    for (int i = 0; i < D; ++i) {
      double acc = o.v[p.dy + i];
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
      double mean = o.v[p.dy + i];
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

// -------------------------------------------------------------------- HMM
struct HMMParams {
  const double* base;
  const double* prior;  // k
  const double* T;      // k*k, T[new*k + prev]
  const double* E;      // v*k, E[x*k + z]
  const double* logE;   // v*k
  int k;
  int v;
  __device__ HMMParams rebase(const double* __restrict__ prm) const {
    HMMParams q = *this;
    q.prior = rebased(*this, prm, prior);
    q.T = rebased(*this, prm, T);
    q.E = rebased(*this, prm, E);
    q.logE = rebased(*this, prm, logE);
    return q;
  }
};

// inverse-CDF categorical draw over p[0], p[stride], ... (sequential sums)
__device__ __forceinline__ int cat_sample(const double* p, int K, int stride, double u) {
  double total = 0.0;
  for (int k = 0; k < K; ++k) total += p[k * stride];
  const double target = u * total;
  double cum = 0.0;
  int last = -1;
  for (int k = 0; k < K; ++k) {
    const double pk = p[k * stride];
    cum += pk;
    if (pk > 0.0) last = k;
    if (cum > target && pk > 0.0) return k;
  }
  return last;
}

// draw from p_k = a[k*sa] * e[k] without storing p (locally optimal proposal)
__device__ __forceinline__ int cat_sample_prod(const double* a, int sa, const double* e, int K,
                                               double u, double* total_out) {
  double total = 0.0;
  for (int k = 0; k < K; ++k) total += a[k * sa] * e[k];
  *total_out = total;
  const double target = u * total;
  double cum = 0.0;
  int last = -1;
  for (int k = 0; k < K; ++k) {
    const double pk = a[k * sa] * e[k];
    cum += pk;
    if (pk > 0.0) last = k;
    if (cum > target && pk > 0.0) return k;
  }
  return last;
}

struct HMMModel {
  static constexpr int kD = 1;
  static constexpr int kMinWaves = 8;
  using Params = HMMParams;

  __device__ static double loglik(const Params& p, const StepObs& o, const double* x) {
    return o.present ? p.logE[o.sym * p.k + (int)x[0]] : 0.0;
  }
  // categorical.jl:10-12: log prior[z] (t = 1) or log T[z | z_prev]; the emission
  __device__ static void score(const Params& p, const StepObs& o, uint32_t t, const double* xp, const double* x,
                               double* lat, double* ob) {
    const int z = (int)x[0];
    *lat = gh_log(t == 1 ? p.prior[z] : p.T[z * p.k + (int)xp[0]]);
    *ob = loglik(p, o, x);
  }
  // simulate(): the symbol ~ categorical(E[:, z]) and its log emission
  __device__ static double sim_obs(const Params& p, uint64_t seed, uint64_t pid, uint32_t t, const double* x,
                                   double* y, int64_t, const double*) {
    const int z = (int)x[0];
    const u32x4 w = rng_block(seed, pid, t, STREAM_SIM, kSimObsDraw);
    const int sym = cat_sample(p.E + z, p.v, p.k, u53(w.x, w.y));
    y[0] = (double)sym;
    return p.logE[sym * p.k + z];
  }
  __device__ static double init(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid,
                                int proposal, double* x, Draw dr = {STREAM_INIT, 0}) {
    const u32x4 w = rng_block(seed, pid, 1, dr.stream, dr.base);
    const double u = u53(w.x, w.y);
    if (proposal == 1 && o.present) {
      double total;
      const int z = cat_sample_prod(p.prior, 1, p.E + o.sym * p.k, p.k, u, &total);
      x[0] = (double)z;
      return gh_log(total);
    }
    const int z = cat_sample(p.prior, p.k, 1, u);
    x[0] = (double)z;
    return o.present ? p.logE[o.sym * p.k + z] : 0.0;
  }

  __device__ static double step(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid,
                                uint32_t t, int proposal, const double* xp, double* x,
                                Draw dr = {STREAM_STEP, 0}) {
    const u32x4 w = rng_block(seed, pid, t, dr.stream, dr.base);
    const double u = u53(w.x, w.y);
    const int zp = (int)xp[0];
    if (proposal == 1 && o.present) {
      double total;
      const int z = cat_sample_prod(p.T + zp, p.k, p.E + o.sym * p.k, p.k, u, &total);
      x[0] = (double)z;
      return gh_log(total);
    }
    const int z = cat_sample(p.T + zp, p.k, p.k, u);
    x[0] = (double)z;
    return o.present ? p.logE[o.sym * p.k + z] : 0.0;
  }
};

// --------------------------------------------------------------- Kitagawa
struct KitParams {
  double mu1, s1;   // x_1 ~ normal(mu1, s1)
  double sx;        // sqrt(var_x)
  double inv2vy;    // 1 / (2 var_y)
  double csty;      // -0.5 log(2 pi var_y)
  double inv2vx, cstx;  // the prior densities (Gaussian custom proposal's weight): 1/(2 var_x), -0.5 log(2 pi var_x)
  double inv2v1, cst1;  //   and at t = 1: 1/(2 s1^2), -0.5 log(2 pi s1^2)
  double sy;            // sqrt(var_y) (simulate)
  __device__ KitParams rebase(const double* __restrict__) const { return *this; }
};

// The Kitagawa latent draws come in pairs: particles p and p + 64 of every
// 128-particle group (the two 64-particle tiles a pair-stepping lane owns)
// share one Philox block and its Box–Muller pair — z0 for p, z1 for p + 64 —
// so k_step_pairs spends one counter block and one log / sqrt / sincos per two
// particles.  The draw of a particle is a function of its global id alone.
__device__ __forceinline__ uint64_t kit_pair_id(uint64_t pid) { return ((pid >> 7) << 6) | (pid & 63); }

struct KitModel {
  static constexpr int kD = 1;
  static constexpr int kMinWaves = 8;
  static constexpr bool kPairs = true;  // k_step_pairs: two particles per lane
  using Params = KitParams;

  __device__ static double obs(const Params& p, const StepObs& o, double x) {
    if (!o.present) return 0.0;
    const double diff = o.v[0] - div20(x * x);
    return -(diff * diff) * p.inv2vy + p.csty;
  }
  __device__ static double loglik(const Params& p, const StepObs& o, const double* x) { return obs(p, o, x[0]); }
  // normal.jl:56-60 for x_t | x_{t-1} (t = 1: normal(mu1, s1)) and y_t | x_t
  __device__ static void score(const Params& p, const StepObs& o, uint32_t t, const double* xp, const double* x,
                               double* lat, double* ob) {
    double mean = p.mu1, inv2 = p.inv2v1, cst = p.cst1;
    if (t > 1) {
      const double v = xp[0];
      mean = ((v / 2.0) + 25.0 * (v / (1.0 + v * v))) + o.ct;
      inv2 = p.inv2vx;
      cst = p.cstx;
    }
    const double d = x[0] - mean;
    *lat = -(d * d) * inv2 + cst;
    *ob = obs(p, o, x[0]);
  }
  // simulate(): y ~ normal(x^2 / 20, sqrt(var_y)) (examples/pmmh/model.jl) and its logpdf
  __device__ static double sim_obs(const Params& p, uint64_t seed, uint64_t pid, uint32_t t, const double* x,
                                   double* y, int64_t, const double* tab) {
    double z0, z1;
    normal_pair(rng_block(seed, pid, t, STREAM_SIM, kSimObsDraw), &z0, &z1, tab);
    const double m = div20(x[0] * x[0]);
    y[0] = m + p.sy * z0;
    const double diff = y[0] - m;
    return -(diff * diff) * p.inv2vy + p.csty;
  }
  __device__ static double mean(const StepObs& o, double v) { return ((v / 2.0) + 25.0 * (v / (1.0 + v * v))) + o.ct; }
  // the particle's standard normal of step t (its half of the shared pair)
  __device__ static double znorm(uint64_t seed, uint64_t pid, uint32_t t, const Draw& dr) {
    double z0, z1;
    normal_pair(rng_block(seed, kit_pair_id(pid), t, dr.stream, dr.base), &z0, &z1, dr.tab);
    return ((pid >> 6) & 1) ? z1 : z0;
  }
  __device__ static double init(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid,
                                int /*proposal*/, double* x, Draw dr = {STREAM_INIT, 0}) {
    x[0] = p.mu1 + p.s1 * znorm(seed, pid, 1, dr);
    return obs(p, o, x[0]);
  }
  __device__ static double step(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid,
                                uint32_t t, int /*proposal*/, const double* xp, double* x,
                                Draw dr = {STREAM_STEP, 0}) {
    x[0] = mean(o, xp[0]) + p.sx * znorm(seed, pid, t, dr);
    return obs(p, o, x[0]);
  }
  // both particles of a pair (pid0 with bit 6 clear, pid0 + 64) from one block:
  // the same values as init / step of each
  __device__ static void init2(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid0, double* x0,
                               double* x1, double* w0, double* w1, const Draw& dr) {
    double z0, z1;
    normal_pair(rng_block(seed, kit_pair_id(pid0), 1, dr.stream, dr.base), &z0, &z1, dr.tab);
    *x0 = p.mu1 + p.s1 * z0;
    *x1 = p.mu1 + p.s1 * z1;
    *w0 = obs(p, o, *x0);
    *w1 = obs(p, o, *x1);
  }
  __device__ static void step2(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid0, uint32_t t,
                               double xp0, double xp1, double* x0, double* x1, double* w0, double* w1,
                               const Draw& dr) {
    double z0, z1;
    normal_pair(rng_block(seed, kit_pair_id(pid0), t, dr.stream, dr.base), &z0, &z1, dr.tab);
    *x0 = mean(o, xp0) + p.sx * z0;
    *x1 = mean(o, xp1) + p.sx * z1;
    *w0 = obs(p, o, *x0);
    *w1 = obs(p, o, *x1);
  }
};

// ------------------------------------- nonlinear SSM, Gaussian custom proposal
// (draws: the nonlinear SSM's paired normals, KitModel::znorm)
// A user-parameterised custom proposal in Gen's sense (particle_filter.jl:
// 79-91,139-154 via the SimpleExtendingTraceTranslator, trace_translators.jl:
// 775-802): x_t ~ q = normal(mu_q, sigma_q), mu_q = alpha m + beta y_t + gamma
// with m the prior mean (m = mu1 at t = 1; beta y_t only when y_t is
// observed); the weight is model weight - proposal score =
// log p(x_t | x_{t-1}) + log p(y_t | x_t) - log q(x_t).  (alpha, beta, gamma,
// sigma_q) are the step's proposal arguments, passed with 1/(2 sigma_q^2) and
// -0.5 log(2 pi sigma_q^2) in o.v[1..6] (gh_pf_step_q).  alpha = 1, beta =
// gamma = 0, sigma_q = sqrt(var_x) is the bootstrap proposal.
struct KitGaussModel {
  static constexpr int kD = 1;
  static constexpr int kMinWaves = 8;
  using Params = KitParams;
  __device__ static double lpn(double x, double mu, double inv2, double cst) {
    const double d = x - mu;
    return -(d * d) * inv2 + cst;
  }
  __device__ static double propose(const Params& p, const StepObs& o, double mean, double inv2p, double cstp,
                                   double z, double* x) {
    double mq = o.v[1] * mean;
    if (o.present) mq = mq + o.v[2] * o.v[0];
    mq = mq + o.v[3];
    x[0] = mq + o.v[4] * z;
    double w = lpn(x[0], mean, inv2p, cstp);
    if (o.present) w = w + KitModel::obs(p, o, x[0]);
    return w - lpn(x[0], mq, o.v[5], o.v[6]);
  }
  __device__ static double loglik(const Params& p, const StepObs& o, const double* x) { return KitModel::obs(p, o, x[0]); }
  __device__ static double init(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid,
                                int /*proposal*/, double* x, Draw dr = {STREAM_INIT, 0}) {
    return propose(p, o, p.mu1, p.inv2v1, p.cst1, KitModel::znorm(seed, pid, 1, dr), x);
  }
  __device__ static double step(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid,
                                uint32_t t, int /*proposal*/, const double* xp, double* x,
                                Draw dr = {STREAM_STEP, 0}) {
    return propose(p, o, KitModel::mean(o, xp[0]), p.inv2vx, p.cstx, KitModel::znorm(seed, pid, t, dr), x);
  }
};

// ------------------------------------------------- Bayesian linear regression
// examples/regression/quickstart.jl:3-9 (config C1):
//   slope ~ normal(mu_s, sd_s); intercept ~ normal(mu_i, sd_i);
//   y_i ~ normal(slope * x_i + intercept, sigma), i = 1..n (n <= kMaxObs)
// A static model (no Unfold): generate only (importance sampling), plus
// rejuvenation moves at t = 1.  State = (slope, intercept).
struct RegParams {
  double mu_s, sd_s, mu_i, sd_i;
  double inv2v;  // 1 / (2 sigma^2)
  double cst;    // -0.5 log(2 pi sigma^2)
  double inv2s, csts, inv2i, csti;  // the same for the slope and intercept priors
  double sigma;
  int n;
  double xs[kMaxObs];
  __device__ RegParams rebase(const double* __restrict__) const { return *this; }
};

struct RegModel {
  static constexpr int kD = 2;
  static constexpr int kMinWaves = 8;
  using Params = RegParams;

  __device__ static double loglik(const Params& p, const StepObs& o, const double* x) {
    if (!o.present) return 0.0;
    double s = 0.0;
    for (int i = 0; i < p.n; ++i) {
      const double diff = o.v[i] - (x[0] * p.xs[i] + x[1]);
      s += -(diff * diff) * p.inv2v + p.cst;
    }
    return s;
  }
  __device__ static double init(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid,
                                int /*proposal*/, double* x, Draw dr = {STREAM_INIT, 0}) {
    double z0, z1;
    normal_pair(rng_block(seed, pid, 1, dr.stream, dr.base), &z0, &z1, dr.tab);
    x[0] = p.mu_s + p.sd_s * z0;
    x[1] = p.mu_i + p.sd_i * z1;
    return loglik(p, o, x);
  }
  // :slope and :intercept scores (normal.jl:56-60) and the y's
  __device__ static void score(const Params& p, const StepObs& o, uint32_t, const double*, const double* x,
                               double* lat, double* ob) {
    const double ds = x[0] - p.mu_s, di = x[1] - p.mu_i;
    *lat = (-(ds * ds) * p.inv2s + p.csts) + (-(di * di) * p.inv2i + p.csti);
    *ob = loglik(p, o, x);
  }
  // simulate(): y_i ~ normal(slope x_i + intercept, sigma) and their logpdfs in data order
  __device__ static double sim_obs(const Params& p, uint64_t seed, uint64_t pid, uint32_t t, const double* x,
                                   double* y, int64_t ys, const double* tab) {
    double z[kMaxObs];
    normals_rt(seed, pid, t, STREAM_SIM, kSimObsDraw, p.n, z, tab);
    double s = 0.0;
    for (int i = 0; i < p.n; ++i) {
      const double m = x[0] * p.xs[i] + x[1];
      const double yi = m + p.sigma * z[i];
      y[i * ys] = yi;
      const double diff = yi - m;
      s += -(diff * diff) * p.inv2v + p.cst;
    }
    return s;
  }
  // regenerate the selected addresses from their prior (bit 0 :slope, bit 1
  // :intercept; the same draws as init), keep the others: the proposal of
  // mh(trace, select(...)) (src/inference/mh.jl:14-28).  The returned value is
  // the new log-likelihood: the selected choices' prior scores cancel in the
  // regenerate weight, the unselected roots' do not change.
  __device__ static double init_select(const Params& p, const StepObs& o, uint64_t seed, uint64_t pid, uint32_t sel,
                                       const double* xc, double* x, Draw dr = {STREAM_INIT, 0}) {
    double z0, z1;
    normal_pair(rng_block(seed, pid, 1, dr.stream, dr.base), &z0, &z1, dr.tab);
    x[0] = (sel & 1u) ? p.mu_s + p.sd_s * z0 : xc[0];
    x[1] = (sel & 2u) ? p.mu_i + p.sd_i * z1 : xc[1];
    return loglik(p, o, x);
  }
  // no time structure: the host refuses particle_filter_step for this family
  __device__ static double step(const Params&, const StepObs&, uint64_t, uint64_t, uint32_t, int,
                                const double* xp, double* x, Draw = {STREAM_STEP, 0}) {
    x[0] = xp[0];
    x[1] = xp[1];
    return 0.0;
  }
};

}  // namespace gh
