// gh_kernels.h — HIP kernels of the particle-filter hot path (gfx950, wave64).
//
// Kernel map (DESIGN.md §6 has the roofline of each):
//   k_step<Model,INIT>  generate (INIT) / update of every particle, fused with
//                       the ancestor gather of the previous resample, the
//                       log-weight update and the block partials of
//                       (max, sum e, sum e^2); the last block to arrive folds
//                       the partials into this rank's (M, S, S2).
//                       particle_filter.jl:99-108 / 162-180 + inference.jl:3-6
//   k_decide            ESS test + log-ML update (particle_filter.jl:189-201)
//   k_qsum / k_qscan /
//   k_cdf               integer-quantised weight CDF
//   k_search            systematic / multinomial ancestor search, composes
//                       ancestors on a second resample without a step
//   k_traj              genealogy walk (get_traces along the Unfold history)
#pragma once
#include "gh_models.h"

namespace gh {

constexpr int kBlock = 256;
constexpr int kScanItems = 8;                    // items per thread in the CDF kernels
constexpr int kScanTile = kBlock * kScanItems;   // particles per CDF block

// Device-resident state of one particle filter (one rank).
struct DevScalars {
  double stats[3];     // this rank's (max, sum exp(w-max), sum exp(w-max)^2)
  double log_ml_est;   // ParticleFilterState.log_ml_est
  double M, L, ess;    // last decision: global max, logsumexp, ESS
  double sM;           // max used by sample_unweighted
  uint64_t S;          // global integer total of the quantised weights
  uint64_t base;       // this rank's offset in the global integer CDF
  uint64_t local;      // this rank's integer total
  uint64_t o, Qs, Rs;  // systematic offset, S / N, S % N
  int pending;         // a resample happened since the last step
  int fire;            // the current maybe_resample decided to resample
  int spend;           // sample_unweighted: weights are all equal
  int one;             // constant 1 (gate for unconditional launches)
  int error;           // gh_status raised on the device
  unsigned ticket;     // last-block-done counter of k_step
  int pad[2];
};

struct StepArgs {
  const double* xprev;   // [D][ld_prev] states of the previous step
  int64_t ld_prev;
  const int32_t* anc;    // ancestors for this step (used when a resample is pending)
  const double* remote;  // multi-rank: states received from other ranks [D][ld_remote]
  int64_t ld_remote;
  double* xout;          // [D][ld_out]
  int64_t ld_out;
  double* logw;
  int64_t n;             // particles on this rank
  int64_t lo;            // global id of the first one
  uint64_t seed;
  uint32_t t;            // 1-based step index
  int proposal;
  DevScalars* dev;
  double* pm;            // block partials: max
  double* ps;            //                 sum e
  double* ps2;           //                 sum e^2
  double* stats_out;     // where the rank's (M, S, S2) goes
};

// ------------------------------------------------------------ reductions
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block (256 threads) max / sum, result broadcast to every thread
__device__ __forceinline__ double block_max(double v, double* sm) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sm[w] = v;
  __syncthreads();
  return fmax(fmax(sm[0], sm[1]), fmax(sm[2], sm[3]));
}
__device__ __forceinline__ double block_sum(double v, double* sm) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sm[w] = v;
  __syncthreads();
  return (sm[0] + sm[1]) + (sm[2] + sm[3]);
}

// Combine per-block (m, s, s2) partials into the rank's triple.  Called by
// the last block of k_step after the agent-scope acquire.
__device__ void fold_partials(const double* pm, const double* ps, const double* ps2, int nb,
                              double* sm, double* out) {
  double m = -INFINITY;
  for (int b = threadIdx.x; b < nb; b += kBlock) m = fmax(m, pm[b]);
  const double M = block_max(m, sm);
  double s = 0.0, s2 = 0.0;
  if (M > -INFINITY) {
    for (int b = threadIdx.x; b < nb; b += kBlock) {
      const double mb = pm[b];
      if (mb > -INFINITY) {
        const double e = gh_exp(mb - M);
        s += ps[b] * e;
        s2 += ps2[b] * (e * e);
      }
    }
  }
  s = block_sum(s, sm);
  s2 = block_sum(s2, sm);
  if (threadIdx.x == 0) {
    out[0] = M;
    out[1] = s;
    out[2] = s2;
  }
}

// ---------------------------------------------------------------- k_step
template <class Model, bool INIT>
__global__ __launch_bounds__(kBlock) void k_step(typename Model::Params p, StepObs o, StepArgs a) {
  constexpr int D = Model::kD;
  __shared__ double sm[8];
  __shared__ int am_last;
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  int pend = 0;
  if (!INIT) pend = a.dev->pending | a.dev->fire;
  double lw = -INFINITY;
  if (j < a.n) {
    double x[D];
    double inc;
    if (INIT) {
      inc = Model::init(p, o, a.seed, (uint64_t)(a.lo + j), a.proposal, x);
      lw = inc;
    } else {
      double xp[D];
      if (pend) {
        const int32_t s = a.anc[j];
        if (s >= 0) {
#pragma unroll
          for (int k = 0; k < D; ++k) xp[k] = a.xprev[k * a.ld_prev + s];
        } else {
#pragma unroll
          for (int k = 0; k < D; ++k) xp[k] = a.remote[k * a.ld_remote + (-1 - s)];
        }
      } else {
#pragma unroll
        for (int k = 0; k < D; ++k) xp[k] = a.xprev[k * a.ld_prev + j];
      }
      inc = Model::step(p, o, a.seed, (uint64_t)(a.lo + j), a.t, a.proposal, xp, x);
      lw = (pend ? 0.0 : a.logw[j]) + inc;
    }
#pragma unroll
    for (int k = 0; k < D; ++k) a.xout[k * a.ld_out + j] = x[k];
    a.logw[j] = lw;
  }
  // block partials of (max, sum e, sum e^2)
  const double mb = block_max(lw, sm);
  double e = 0.0;
  if (mb > -INFINITY && lw > -INFINITY) e = gh_exp(lw - mb);
  const double sb = block_sum(e, sm);
  const double s2b = block_sum(e * e, sm);
  if (threadIdx.x == 0) {
    a.pm[blockIdx.x] = mb;
    a.ps[blockIdx.x] = sb;
    a.ps2[blockIdx.x] = s2b;
    // publish: stores drained, agent release, then the ticket (Guideline 16)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev =
        __hip_atomic_fetch_add(&a.dev->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    am_last = (prev == gridDim.x - 1);
  }
  __syncthreads();
  if (!am_last) return;
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  fold_partials(a.pm, a.ps, a.ps2, (int)gridDim.x, sm, a.stats_out);
  if (threadIdx.x == 0) {
    __hip_atomic_store(&a.dev->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!INIT) {
      a.dev->pending = 0;
      a.dev->fire = 0;
    }
  }
}

// --------------------------------------------------------------- k_decide
// maybe_resample! (particle_filter.jl:189-201): combine the ranks' triples in
// rank order, ESS = S^2 / S2 (= exp(-logsumexp(2 lnw))), resample iff ESS < thr.
__global__ void k_decide(DevScalars* dev, double* stats_all, int R, int64_t n_global, double thr,
                         double* ess_hist, int32_t* res_hist, int t) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (dev->fire) {  // second maybe_resample without a step: commit the first
    dev->pending = 1;
    dev->fire = 0;
  }
  double M = -INFINITY;
  for (int r = 0; r < R; ++r) M = fmax(M, stats_all[3 * r]);
  if (!(M > -INFINITY) || M == INFINITY || M != M) {
    dev->error = 3;  // GH_E_NUMERIC
    dev->ess = NAN;
    if (ess_hist) ess_hist[t] = NAN;
    return;
  }
  double S = 0.0, S2 = 0.0;
  for (int r = 0; r < R; ++r) {
    if (!(stats_all[3 * r] > -INFINITY)) continue;
    const double e = gh_exp(stats_all[3 * r] - M);
    S += stats_all[3 * r + 1] * e;
    S2 += stats_all[3 * r + 2] * (e * e);
  }
  const double L = M + gh_log(S);
  const double ess = (S * S) / S2;
  const int fire = ess < thr;
  dev->M = M;
  dev->L = L;
  dev->ess = ess;
  dev->fire = fire;
  if (fire) {
    dev->log_ml_est += L - gh_log((double)n_global);
    // after the resample every weight is 0
    for (int r = 0; r < R; ++r) {
      const int64_t nr = (n_global * (r + 1)) / R - (n_global * r) / R;
      stats_all[3 * r] = 0.0;
      stats_all[3 * r + 1] = (double)nr;
      stats_all[3 * r + 2] = (double)nr;
    }
  }
  if (ess_hist) ess_hist[t] = ess;
  if (res_hist) res_hist[t + 1] = dev->pending | fire;
}

// ------------------------------------------------------ integer CDF kernels
struct GateArgs {
  const int* gate;     // launch does nothing unless *gate
  const double* M;     // max log-weight used for quantisation
  const int* zero_w;   // weights are all 0 (resampled since last step)
  int shift;           // quantisation shift
};

__device__ __forceinline__ uint64_t qweight(const double* logw, int64_t i, double M, int zero,
                                            int shift) {
  return quantize_weight(zero ? 0.0 : logw[i], M, shift);
}

__global__ __launch_bounds__(kBlock) void k_qsum(const double* logw, int64_t n, GateArgs g,
                                                 uint64_t* bsum) {
  if (!*g.gate) return;
  __shared__ uint64_t sm[4];
  const double M = *g.M;
  const int zero = *g.zero_w;
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int64_t i = base + threadIdx.x + (int64_t)k * kBlock;
    if (i < n) s += qweight(logw, i, M, zero, g.shift);
  }
  s = wave_sum_u64(s);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = (sm[0] + sm[1]) + (sm[2] + sm[3]);
}

// exclusive scan of the block sums in place (one 1024-thread block); writes
// the rank total into dev->local.
__global__ __launch_bounds__(1024) void k_qscan(uint64_t* bsum, int64_t nb, GateArgs g,
                                                DevScalars* dev) {
  if (!*g.gate) return;
  __shared__ uint64_t sm[1024];
  const int64_t per = (nb + 1023) / 1024;
  const int64_t b0 = (int64_t)threadIdx.x * per;
  uint64_t s = 0;
  for (int64_t b = b0; b < b0 + per && b < nb; ++b) s += bsum[b];
  sm[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    uint64_t v = threadIdx.x >= (unsigned)off ? sm[threadIdx.x - off] : 0;
    __syncthreads();
    sm[threadIdx.x] += v;
    __syncthreads();
  }
  uint64_t run = sm[threadIdx.x] - s;  // exclusive
  for (int64_t b = b0; b < b0 + per && b < nb; ++b) {
    const uint64_t v = bsum[b];
    bsum[b] = run;
    run += v;
  }
  if (threadIdx.x == 1023) dev->local = sm[1023];
}

// global integer constants of the resample: S, base, systematic offset
__global__ void k_rs_const(GateArgs g, DevScalars* dev, const uint64_t* totals, int R, int rank,
                           int64_t n_global, uint64_t seed, uint32_t t, uint32_t stream) {
  if (!*g.gate || threadIdx.x != 0) return;
  uint64_t S = 0, base = 0;
  if (totals) {
    for (int r = 0; r < R; ++r) {
      if (r < rank) base += totals[r];
      S += totals[r];
    }
  } else {
    S = dev->local;
  }
  dev->S = S;
  dev->base = base;
  const u32x4 w = rng_block(seed, ~0ull, t, stream, 0);
  dev->o = scale_u53(u53_bits(w.x, w.y), S);
  dev->Qs = S / (uint64_t)n_global;
  dev->Rs = S % (uint64_t)n_global;
}

// inclusive global CDF C[i]
__global__ __launch_bounds__(kBlock) void k_cdf(const double* logw, int64_t n, GateArgs g,
                                                const uint64_t* boff, const DevScalars* dev,
                                                uint64_t* C) {
  if (!*g.gate) return;
  __shared__ uint64_t sm[kBlock];
  const double M = *g.M;
  const int zero = *g.zero_w;
  const int64_t i0 = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  uint64_t q[kScanItems];
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    q[k] = (i0 + k < n) ? qweight(logw, i0 + k, M, zero, g.shift) : 0;
    s += q[k];
  }
  sm[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < kBlock; off <<= 1) {
    uint64_t v = threadIdx.x >= (unsigned)off ? sm[threadIdx.x - off] : 0;
    __syncthreads();
    sm[threadIdx.x] += v;
    __syncthreads();
  }
  uint64_t run = dev->base + boff[blockIdx.x] + sm[threadIdx.x] - s;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    run += q[k];
    if (i0 + k < n) C[i0 + k] = run;
  }
}

enum SearchMode { SEARCH_SYSTEMATIC = 0, SEARCH_MULTINOMIAL = 1, SEARCH_SAMPLE = 2 };

struct SearchArgs {
  const uint64_t* C;     // inclusive CDF of this rank's particles, offset by dev->base
  int64_t n_cdf;
  int64_t n_slots;       // slots handled by this launch
  int64_t slot_lo;       // global index of slot 0
  int64_t n_global;
  uint64_t seed;
  uint32_t t;
  int mode;
  const int32_t* anc_old;  // compose when a resample is already pending
  int32_t* anc_out;
};

__device__ __forceinline__ uint64_t slot_target(const SearchArgs& s, const DevScalars* dev,
                                                int64_t g) {
  if (s.mode == SEARCH_SYSTEMATIC) {
    const uint64_t gg = (uint64_t)g;
    return gg * dev->Qs + (gg * dev->Rs + dev->o) / (uint64_t)s.n_global;
  }
  const uint32_t stream = s.mode == SEARCH_SAMPLE ? STREAM_SAMPLE : STREAM_RESAMPLE;
  const u32x4 w = rng_block(s.seed, (uint64_t)g, s.t, stream, 0);
  return scale_u53(u53_bits(w.x, w.y), dev->S);
}

__global__ __launch_bounds__(kBlock) void k_search(SearchArgs s, GateArgs g, const DevScalars* dev) {
  if (!*g.gate) return;
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= s.n_slots) return;
  const uint64_t target = slot_target(s, dev, s.slot_lo + j) - dev->base;
  int64_t lo = 0, hi = s.n_cdf - 1;
  while (lo < hi) {  // first i with C[i] - base > target
    const int64_t mid = lo + ((hi - lo) >> 1);
    if (s.C[mid] - dev->base > target) hi = mid;
    else lo = mid + 1;
  }
  const int zero = *g.zero_w;
  s.anc_out[j] = (zero && s.anc_old) ? s.anc_old[lo] : (int32_t)lo;
}

__global__ void k_copy_anc(const int* gate, const int32_t* src, int32_t* dst, int64_t n) {
  if (!*gate) return;
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j < n) dst[j] = src[j];
}

// ------------------------------------------------------------- genealogy
struct TrajArgs {
  const double* const* xs;    // device array of per-step state slots (index t-1)
  const int32_t* const* ancs; // device array of per-step ancestor arrays (index t-1)
  const int32_t* res_before;  // res_before[t]: a resample preceded step t
  const int32_t* anc_pending; // ancestors of a resample pending after the last step
  int64_t n, ld;
  int t_target, t_cur, D;
  double* out;                // [D][n]
};

__global__ __launch_bounds__(kBlock) void k_traj(TrajArgs a, const DevScalars* dev) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= a.n) return;
  int64_t idx = j;
  if ((dev->pending | dev->fire) && a.anc_pending) idx = a.anc_pending[idx];
  for (int s = a.t_cur; s > a.t_target; --s)
    if (a.res_before[s]) idx = a.ancs[s - 1][idx];
  const double* x = a.xs[a.t_target - 1];
  for (int k = 0; k < a.D; ++k) a.out[k * a.n + j] = x[k * a.ld + idx];
}

// sample_unweighted: prepare max / equal-weight flag from the current stats
__global__ void k_prep_sample(DevScalars* dev, const double* stats_all, int R) {
  if (threadIdx.x != 0) return;
  double M = -INFINITY;
  for (int r = 0; r < R; ++r) M = fmax(M, stats_all[3 * r]);
  dev->spend = dev->pending | dev->fire;
  dev->sM = dev->spend ? 0.0 : M;
  dev->one = 1;
}

// ------------------------------------------------------------ self tests
__global__ void k_selftest_math(int64_t n, const double* in, double* oe, double* ol, double* os,
                                double* od) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const double x = in[i];
  oe[i] = gh_exp(x);
  ol[i] = gh_log(fabs(x));
  os[i] = sqrt(fabs(x));
  od[i] = x / in[(i + 1) % n];
}

__global__ void k_selftest_normals(uint64_t seed, int64_t n, uint32_t step, uint32_t stream,
                                   int dim, double* out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  for (int j = 0; 2 * j < dim; ++j) {
    double a, b;
    normal_pair(rng_block(seed, (uint64_t)i, step, stream, (uint32_t)j), &a, &b);
    out[i * dim + 2 * j] = a;
    if (2 * j + 1 < dim) out[i * dim + 2 * j + 1] = b;
  }
}

}  // namespace gh
