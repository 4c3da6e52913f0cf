// gh_pmmh.h — particle-marginal Metropolis–Hastings (config C5).
//
// Reference: examples/pmmh/example.jl:26-79 (model, proposals, do_inference)
// over examples/pmmh/pf.jl:14-73 (ParticleFilterCombinator: a generative
// function whose generate/update/regenerate weight is a particle filter's
// log-ML estimate) and src/inference/mh.jl:14-62 (both MH forms).
//
// One workgroup runs one outer chain; its threads are the inner particles
// (states, weights and the integer CDF live in registers and LDS).  Each
// iteration applies the four moves of do_inference (example.jl:67-70):
//   0  mh(tr, select(:var_x))       regenerate log var_x from its prior
//   1  mh(tr, select(:var_y))       regenerate log var_y from its prior
//   2  mh(tr, var_x_proposal, ())   random walk on log var_x, sd sqrt(0.5)
//   3  mh(tr, var_y_proposal, ())   random walk on log var_y, sd sqrt(0.5)
// and every move re-runs the inner filter (pseudo-marginal).  The inner
// filter is the reference's PF loop (pf.jl:40-56) on the Kitagawa model with
// the engine's systematic integer resampling.
//
// Randomness: move counter u = 0 for the initial generate,
// u = 1 + 4k + m for move m of (global) iteration k; particle p of chain c uses id
// (u << 32) | (c << 10) | p; the chain's own draws (prior / proposal,
// acceptance, resampling offsets) use id (u << 32) | (c << 10).  The state
// noise of steps t and t + 1 (t even) is the pair (z0, z1) of ONE Box–Muller
// evaluation of the block at step t: half the Philox and Box–Muller work of a
// filter (the kernel is VALU-bound), still a function of (seed, id, t) alone.
#pragma once
#include "gh_kernels.h"

namespace gh {

constexpr int kPmmhMaxInner = 1024;
constexpr int kPmmhMaxT = 1024;

struct PmmhArgs {
  const double* ys;     // [T] observations
  const double* ct;     // [T] 8 cos(1.2 t), t = 1..T (host gh_cos)
  int T;
  int n_iters;
  int iter0;            // iterations already run (continues the move counters)
  uint64_t seed;
  int64_t chain0;       // global index of this launch's first chain
  int64_t n_chains;
  double* lvx;          // [n_chains] log var_x (in: start values if init == 0; out: last state)
  double* lvy;          // [n_chains] log var_y
  double* lml;          // [n_chains] log-ML estimate of the current state
  int32_t* accepts;     // [n_chains][4]
  double* hist;         // optional [n_chains][n_iters][2] (log var_x, log var_y) after each iteration
  int init;             // 1: draw the start from the prior and run the first filter (generate)
};

// The kernel is compiled in its own unit (gh_inst_pmmh.hip, GH_PMMH_KERNEL)
// with fma_c as a plain fma (GH_FMA_C_PLAIN): the SGPR-operand form that
// helps the particle-filter kernels cost this VALU-bound persistent kernel
// 192.1 -> 177.6 ms per C5 launch pair (three interleaved runs each on one
// box, round 6).  The values are the same: one correctly rounded fma.
#if !defined(GH_PMMH_KERNEL)
__global__ __launch_bounds__(kPmmhMaxInner) void k_pmmh(PmmhArgs a);
#else

// normal(mu, sd) logpdf in the reference's form (normal.jl:56-60)
__device__ __forceinline__ double normal_lpdf(double x, double mu, double sd) {
  const double var = sd * sd;
  const double diff = x - mu;
  return -(diff * diff) / (2.0 * var) - 0.5 * gh_log(2.0 * 0x1.921fb54442d18p+1 * var);
}

// 256..1024-thread block reductions (nw waves), result broadcast
__device__ __forceinline__ double blkn_max(double v, double* sm, int nw) {
  v = wave_max(v);
  lds_barrier();
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  lds_barrier();
  double r = sm[0];
  for (int k = 1; k < nw; ++k) r = fmax(r, sm[k]);
  return r;
}
__device__ __forceinline__ double blkn_sum(double v, double* sm, int nw) {
  v = wave_sum(v);
  lds_barrier();
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  lds_barrier();
  double r = sm[0];
  for (int k = 1; k < nw; ++k) r += sm[k];
  return r;
}
// two sums in one LDS round (the same per-value order as blkn_sum; sm holds 32)
__device__ __forceinline__ void blkn_sum2(double* a, double* b, double* sm, int nw) {
  const double wa = wave_sum(*a), wb = wave_sum(*b);
  lds_barrier();
  if ((threadIdx.x & 63) == 0) {
    sm[threadIdx.x >> 6] = wa;
    sm[16 + (threadIdx.x >> 6)] = wb;
  }
  lds_barrier();
  double ra = sm[0], rb = sm[16];
  for (int k = 1; k < nw; ++k) {
    ra += sm[k];
    rb += sm[16 + k];
  }
  *a = ra;
  *b = rb;
}
__device__ __forceinline__ uint64_t blkn_incl_u64(uint64_t v, uint64_t* sm, int nw) {
  const int w = threadIdx.x >> 6;
  v = wave_incl_sum_u64(v);
  lds_barrier();
  if ((threadIdx.x & 63) == 63) sm[w] = v;
  lds_barrier();
  for (int k = 0; k < w; ++k) v += sm[k];
  return v;
}

struct PmmhShared {
  double x[kPmmhMaxInner];
  uint64_t C[kPmmhMaxInner];
  double tab[kMathTabDoubles];  // Box–Muller log / angle tables
  double smd[32];
  uint64_t smu[16];
};

// One run of the inner particle filter (pf.jl:35-57) for chain c, move u;
// returns log_ml_estimate (block-uniform).
__device__ double pmmh_filter(const PmmhArgs& a, PmmhShared& sh, uint64_t c, uint32_t u, double log_vx,
                              double log_vy) {
  const int N = blockDim.x, nw = N >> 6, j = threadIdx.x;
  const double var_x = gh_exp(log_vx), var_y = gh_exp(log_vy);
  const double sx = sqrt(var_x);
  const double inv2vy = 1.0 / (2.0 * var_y);
  const double csty = -0.5 * gh_log(2.0 * 0x1.921fb54442d18p+1 * var_y);
  const uint64_t cid = ((uint64_t)u << 32) | (c << 10);
  const uint64_t pid = cid | (uint64_t)j;
  const double logN = gh_log((double)N);
  const double invN = 1.0 / (double)N;
  const int shift = quant_shift((uint64_t)N);
  auto obs = [&](double y, double x) {
    const double diff = y - div20(x * x);
    return -(diff * diff) * inv2vy + csty;
  };
  // generate: x_1 ~ normal(0, 5), weight = emission logpdf (pf.jl:23-27)
  double z0, z1;
  normal_pair(rng_block(a.seed, pid, 1, STREAM_INIT, 0), &z0, &z1, sh.tab);
  double x = 0.0 + 5.0 * z0;
  double lw = obs(a.ys[0], x);
  double log_ml = 0.0;
  double zk = 0.0;  // the second normal of the last even step's pair
  for (int t = 2; t <= a.T; ++t) {
    // maybe_resample! (particle_filter.jl:189-213), threshold N/2
    const double M = blkn_max(lw, sh.smd, nw);
    // lw - M <= 0: the branch-free exp (gh_exp's values); the same e gives
    // the quantised weight (= quantize_weight(lw, M, shift))
    const double e = lw > -INFINITY ? gh_exp_nonpos(lw - M) : 0.0;
    double S = e, S2 = e * e;
    blkn_sum2(&S, &S2, sh.smd, nw);
    double xp = x, base = lw;
    if ((S * S) / S2 < (double)N / 2.0) {
      log_ml += (M + gh_log(S)) - logN;
      const uint64_t qv = (uint64_t)(e * as_f64((uint64_t)(shift + 1023) << 52));
      const uint64_t incl = blkn_incl_u64(qv, sh.smu, nw);
      sh.C[j] = incl;
      sh.x[j] = x;
      lds_barrier();
      // the block constants on the scalar unit; per lane, floor((j Rs + o) / N)
      // = o / N + floor((j Rs + o % N) / N) with j Rs + o % N < 2^21: a
      // double estimate and one correction (the same integers as the
      // reference division)
      const uint64_t Stot = readfirstlane_u64(sh.C[N - 1]);
      const u32x4 w = rng_block(a.seed, cid, (uint32_t)(t - 1), STREAM_RESAMPLE, 0);
      const uint64_t o = readfirstlane_u64(scale_u53(u53_bits(w.x, w.y), Stot));
      const uint64_t Qs = Stot / (uint64_t)N, Rs = Stot - Qs * (uint64_t)N;
      const uint64_t oq = o / (uint64_t)N, orr = o - oq * (uint64_t)N;
      const uint32_t num = (uint32_t)((uint64_t)j * Rs + orr);
      uint32_t qq = (uint32_t)((double)num * invN);
      qq += (qq + 1u) * (uint32_t)N <= num ? 1u : 0u;
      qq -= qq * (uint32_t)N > num ? 1u : 0u;
      const uint64_t target = (uint64_t)j * Qs + oq + qq;
      int lo = 0, hi = N - 1;  // first i with C[i] > target
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sh.C[mid] > target) hi = mid;
        else lo = mid + 1;
      }
      xp = sh.x[lo];
      base = 0.0;
      lds_barrier();
    }
    // particle_filter_step!: x_t ~ normal(x_mean(x_{t-1}, t), sqrt(var_x))
    double z = zk;
    if ((t & 1) == 0) {  // uniform: a new pair every second step
      normal_pair(rng_block(a.seed, pid, (uint32_t)t, STREAM_STEP, 0), &z0, &z1, sh.tab);
      z = z0;
      zk = z1;
    }
    const double mean = ((xp / 2.0) + 25.0 * (xp / (1.0 + xp * xp))) + a.ct[t - 1];
    x = mean + sx * z;
    lw = base + obs(a.ys[t - 1], x);
  }
  // log_ml_estimate (particle_filter.jl:52-55)
  const double M = blkn_max(lw, sh.smd, nw);
  const double e = lw > -INFINITY ? gh_exp_nonpos(lw - M) : 0.0;
  const double S = blkn_sum(e, sh.smd, nw);
  return log_ml + (M + gh_log(S)) - logN;
}

__global__ __launch_bounds__(kPmmhMaxInner) void k_pmmh(PmmhArgs a) {
  __shared__ PmmhShared sh;
  const int64_t cl = blockIdx.x;
  if (cl >= a.n_chains) return;
  load_math_tab(sh.tab);
  lds_barrier();
  const uint64_t c = (uint64_t)(a.chain0 + cl);
  const double sd_rw = 0x1.6a09e667f3bcdp-1;  // sqrt(0.5)
  double lvx, lvy, lml;
  if (a.init) {
    // generate(model, (), observations): priors normal(0, 2) (example.jl:24-25)
    double z0, z1;
    normal_pair(rng_block(a.seed, c << 10, 0, STREAM_MH, 0), &z0, &z1, sh.tab);
    lvx = 0.0 + 2.0 * z0;
    lvy = 0.0 + 2.0 * z1;
    lml = pmmh_filter(a, sh, c, 0, lvx, lvy);
  } else {
    lvx = a.lvx[cl];
    lvy = a.lvy[cl];
    lml = a.lml[cl];
  }
  int acc[4] = {0, 0, 0, 0};
  for (int k = 0; k < a.n_iters; ++k) {
    for (int m = 0; m < 4; ++m) {
      const uint32_t u = 1u + 4u * (uint32_t)(a.iter0 + k) + (uint32_t)m;
      const uint64_t cid = ((uint64_t)u << 32) | (c << 10);
      double z0, z1;
      normal_pair(rng_block(a.seed, cid, 0, STREAM_MH, 0), &z0, &z1, sh.tab);
      const u32x4 wa = rng_block(a.seed, cid, 0, STREAM_MH, 1);
      const double logu = gh_log(u53(wa.x, wa.y));
      const bool on_x = (m & 1) == 0;
      const double cur = on_x ? lvx : lvy;
      double prop, alpha, lml_new;
      if (m < 2) {
        // regenerate from the prior: weight = new log-ML - old log-ML
        prop = 0.0 + 2.0 * z0;
        lml_new = on_x ? pmmh_filter(a, sh, c, u, prop, lvy) : pmmh_filter(a, sh, c, u, lvx, prop);
        alpha = lml_new - lml;
      } else {
        // random walk: alpha = weight - fwd + bwd (mh.jl:48-55)
        prop = cur + sd_rw * z0;
        lml_new = on_x ? pmmh_filter(a, sh, c, u, prop, lvy) : pmmh_filter(a, sh, c, u, lvx, prop);
        const double weight = (normal_lpdf(prop, 0.0, 2.0) - normal_lpdf(cur, 0.0, 2.0)) + (lml_new - lml);
        const double fwd = normal_lpdf(prop, cur, sd_rw);
        const double bwd = normal_lpdf(cur, prop, sd_rw);
        alpha = (weight - fwd) + bwd;
      }
      if (logu < alpha) {
        if (on_x) lvx = prop;
        else lvy = prop;
        lml = lml_new;
        acc[m] += 1;
      }
    }
    if (a.hist && threadIdx.x == 0) {
      a.hist[(cl * a.n_iters + k) * 2] = lvx;
      a.hist[(cl * a.n_iters + k) * 2 + 1] = lvy;
    }
  }
  if (threadIdx.x == 0) {
    a.lvx[cl] = lvx;
    a.lvy[cl] = lvy;
    a.lml[cl] = lml;
    for (int m = 0; m < 4; ++m) a.accepts[cl * 4 + m] = acc[m];
  }
}

#endif  // GH_PMMH_KERNEL

}  // namespace gh
