// gh_coal.h — reversible-jump MH chains on the coal-mining change-point model
// (config C3).
//
// Reference: examples/coal/coal.jl:47-62 (model), :18-33 (min_uniform_continuous),
// examples/coal/poisson_process.jl:9-67 (piecewise Poisson process), and the
// three moves of mcmc_step (coal.jl:329-336): rate_move (:103-134),
// position_move (:140-167), birth_death_move (:173-318), each an involutive
// MH step (src/inference/mh.jl:85-98 over trace_translators.jl:848-876:
// log_weight = new score - old score + bwd score - fwd score + log|J|).
// The Jacobian of the birth map (h, u) -> (h_prev, h_next) is taken in closed
// form, |J| = (h_prev + h_next)^2 / h (Green 1995), where the reference
// differentiates the transform with ForwardDiff (trace_translators.jl:534-589).
//
// The score, written for the state (k, cp[1..k], h[1..k+1]) with b_0 = 0,
// b_{k+1} = T, c_i = #events in segment i and len_i = b_i - b_{i-1}:
//   poisson(3) + the k sequential min_uniform_continuous terms + gamma priors
//   + piecewise Poisson process
//   = k (log 3 - log T) - 3 + sum_i [-log(theta) - h_i / theta]
//     + sum_i [c_i log h_i - len_i h_i]
// (the order-statistic densities telescope to log k! - k log T, and log k!
// cancels against the Poisson prior's; tests/test_coal_pins.py checks this
// against the reference's formulas term by term).  Each move changes one or
// two segments, so it is scored by its difference alone: a rate move touches
// segment i, a position move segments i and i+1, a birth / death the segment
// split or merged — no copy of the state, no full re-score.
//
// One thread per chain; a window of a chain's change points and rates (cp
// 1..kCoalWin, h 1..kCoalWin+1) lives in LDS for the whole launch
// ([field][lane] per wave: conflict-free for any per-lane index), k and the
// score in registers; the fields past the window (a chain with more than
// kCoalWin change points: the posterior puts ~0.4 % of its mass above k = 8) are
// read and written in place in the chain's HBM row.  The window keeps a
// chain's LDS at 17 fields instead of 65, so four waves per SIMD fit instead
// of one (the kernel waits on dependent LDS reads; more resident waves hide
// them; measured: window 15 / 10 / 8 / 7 / 6 with 128- or 256-thread blocks,
// DESIGN.md §7c).  HBM:
// the window read once and written once per launch.  Event counts come from the sorted event times in LDS through a
// bucket table (start index) and a short scan.  The oracle
// (oracle/gh_oracle.c, orc_coal_run) restates the same arithmetic.
#pragma once
#include "gh_kernels.h"

namespace gh {

constexpr int kCoalKMax = 32;
constexpr int kCoalW = 2 + kCoalKMax + (kCoalKMax + 1) + 1;  // 68: k, score, cp[32], h[33], pad
constexpr int kCoalF = kCoalKMax + (kCoalKMax + 1);          // 65 LDS fields per chain: cp[32], h[33]
constexpr int kCoalMaxEvents = 4096;
#ifndef GH_COAL_WIN
#define GH_COAL_WIN 8
#endif
constexpr int kCoalWin = GH_COAL_WIN;                        // change points in LDS (rates: kCoalWin + 1)
constexpr int kCoalLF = 2 * kCoalWin + 1;                    // LDS fields per chain
#ifndef GH_COAL_BLOCK
#define GH_COAL_BLOCK 256
#endif
constexpr int kCoalBlock = GH_COAL_BLOCK;                    // four waves: 4 blocks (34.8 KB window each + tables) per CU
constexpr int kCoalBuckets = 256;                            // event-count start table
constexpr double kCoalRate = 200.0;                          // gamma(1, 1/200) rate prior: 1 / theta (coal.jl:56-58)

struct CoalArgs {
  const double* events;  // sorted event times
  const int32_t* bucket; // [kCoalBuckets] start index of the event scan per bucket of [0, T]
  int E;
  double T;              // observation window [0, T]
  double bscale;         // kCoalBuckets / T
  double kb;             // log 3 - log T: the score per change point
  double ktheta;         // -log(theta): the gamma prior's constant per rate
  double lhalf;          // log 0.5 (the is_birth bernoulli)
  int64_t chain0, n_chains;
  uint64_t seed;
  int n_iters, iter0;
  int init;              // 1: draw the start from the prior (generate)
  double* state;         // SoA [kCoalW][ld] rows (k, score, cp[32], h[33], pad); unused fields 0
  int64_t ld;            // chains per field column (>= n_chains)
  int32_t* accepts;      // [n_chains][3] rate, position, birth/death (simple: regenerate k)
  int32_t* khist;        // optional [n_chains][n_iters] k after each iteration
  int simple;            // 1: simple_mcmc_step (coal.jl:338-345), mh(trace, select(K)) as the third move
};

// the two uniforms of Philox block b of an iteration: u53(x, y), u53(z, w);
// 1 - u as the exact one_minus_u53 of the same words
struct CoalU {
  uint32_t x, y, z, w;
};
__device__ __forceinline__ CoalU coal_block(uint64_t seed, uint64_t c, uint32_t step, uint32_t b) {
  const u32x4 r = rng_block(seed, c, step, STREAM_MH, b);
  return CoalU{r.x, r.y, r.z, r.w};
}

// #events <= y: start from the bucket before y's (a lower bound of the
// count whatever the rounding of y * bscale), scan forward, and step back if
// the start overshot — exact for any table.
__device__ __forceinline__ int coal_count(const double* ev, const int32_t* bk, int E, double bscale, double y) {
  int bi = (int)(y * bscale);
  bi = bi < 1 ? 0 : (bi > kCoalBuckets ? kCoalBuckets - 1 : bi - 1);
  int j = bk[bi];
  while (j < E && ev[j] <= y) ++j;
  while (j > 0 && ev[j - 1] > y) --j;
  return j;
}

// one chain's fields: cp[i] (i = 1..k) and h[i] (i = 1..k+1) in the LDS window
// (cp at f = i - 1, h at f = kCoalWin + i - 1), past it in the chain's HBM row
// (field 2 + i - 1, resp. 2 + kCoalKMax + i - 1, of the SoA rows)
struct CoalLds {
  double* p;  // wave base + lane
  double* g;  // the chain's HBM row: field f at g[f * ld]
  int64_t ld;
  __device__ __forceinline__ double cp(int i) const {
    return i <= kCoalWin ? p[(i - 1) * 64] : g[(2 + i - 1) * ld];
  }
  __device__ __forceinline__ double h(int i) const {
    return i <= kCoalWin + 1 ? p[(kCoalWin + i - 1) * 64] : g[(2 + kCoalKMax + i - 1) * ld];
  }
  __device__ __forceinline__ void set_cp(int i, double v) const {
    if (i <= kCoalWin) p[(i - 1) * 64] = v;
    else g[(2 + i - 1) * ld] = v;
  }
  __device__ __forceinline__ void set_h(int i, double v) const {
    if (i <= kCoalWin + 1) p[(kCoalWin + i - 1) * 64] = v;
    else g[(2 + kCoalKMax + i - 1) * ld] = v;
  }
  // zero cp(i), h(i + 1) for i = k + 1 .. kCoalKMax: the whole window, past it
  // only up to khi (the largest k this row held: beyond that the row is 0)
  __device__ __forceinline__ void clear_above(int k, int khi) const {
    for (int i = k + 1; i <= kCoalKMax; ++i) {
      if (i > kCoalWin && i > khi) break;
      set_cp(i, 0.0);
    }
    for (int i = k + 2; i <= kCoalKMax + 1; ++i) {
      if (i > kCoalWin + 1 && i > khi + 1) break;
      set_h(i, 0.0);
    }
  }
};

__device__ __forceinline__ double coal_u(uint64_t seed, uint64_t c, uint32_t step, uint32_t d) {
  const u32x4 w = rng_block(seed, c, step, STREAM_MH, d);
  return u53(w.x, w.y);
}

// the piecewise Poisson process's logpdf (poisson_process.jl:32-51) in the
// segment form sum_i [c_i log h_i - len_i h_i], segments in order
__device__ __forceinline__ double coal_events_lp(const CoalArgs& a, int k, const CoalLds& s, const double* ev,
                                                 const int32_t* bk, const double* tab) {
  double lp = 0.0, b_lo = 0.0;
  int n_lo = 0;
  for (int i = 1; i <= k + 1; ++i) {
    const double b_hi = i <= k ? s.cp(i) : a.T;
    const int n_hi = i <= k ? coal_count(ev, bk, a.E, a.bscale, b_hi) : a.E;
    const double h = s.h(i);
    lp += (double)(n_hi - n_lo) * gh_log_unit(h, tab) - (b_hi - b_lo) * h;
    n_lo = n_hi;
    b_lo = b_hi;
  }
  return lp;
}

// the score from scratch (the decomposition of the header), segment by segment
__device__ __forceinline__ double coal_full_score(const CoalArgs& a, int k, const CoalLds& s, const double* ev,
                                                  const int32_t* bk, const double* tab) {
  double sc = (double)k * a.kb - 3.0;
  int n_lo = 0;
  double b_lo = 0.0;
  for (int i = 1; i <= k + 1; ++i) {
    const double b_hi = i <= k ? s.cp(i) : a.T;
    const int n_hi = i <= k ? coal_count(ev, bk, a.E, a.bscale, b_hi) : a.E;
    const double h = s.h(i);
    sc += a.ktheta - h * kCoalRate;
    sc += (double)(n_hi - n_lo) * gh_log_unit(h, tab) - (b_hi - b_lo) * h;
    n_lo = n_hi;
    b_lo = b_hi;
  }
  return sc;
}

// generate(model, (T,), observations): k, change points and rates from the
// prior (attempt a uses draws 100 a + ...; a degenerate draw retries), then
// the score from scratch.  Returns k.
__device__ int coal_init(const CoalArgs& a, uint64_t c, const CoalLds& s, const double* ev, const int32_t* bk,
                         const double* tab, double* score, int* khi) {
  int k = 0;
  bool done = false;
  for (int att = 0; att < 64 && !done; ++att) {
    const uint32_t d0 = 100u * (uint32_t)att;
    // k ~ poisson(3) by inverse CDF
    const double u = coal_u(a.seed, c, 0, d0);
    double p = gh_exp(-3.0), cum = p;
    k = 0;
    while (u >= cum && k < 200) {
      ++k;
      p = p * (3.0 / (double)k);
      cum += p;
    }
    if (k > kCoalKMax) continue;
    *khi = k > *khi ? k : *khi;  // (a retried attempt may leave fields up to here)
    bool ok = true;
    double lower = 0.0;
    for (int i = 1; i <= k; ++i) {
      // min_uniform_continuous(lower, T, m): upper - (upper - lower) (1 - p)^(1/m)  (coal.jl:28-32)
      const double q = coal_u(a.seed, c, 0, d0 + 1u + (uint32_t)i);
      const double m = (double)(k - i + 1);
      const double x = a.T - (a.T - lower) * gh_exp(gh_log(1.0 - q) / m);
      if (!(x > lower && x < a.T)) ok = false;
      s.set_cp(i, x);
      lower = x;
    }
    for (int i = 1; i <= k + 1; ++i) {
      // gamma(1, theta) = exponential: -theta log(1 - q)
      const double q = coal_u(a.seed, c, 0, d0 + 40u + (uint32_t)i);
      const double x = -gh_log(1.0 - q) / kCoalRate;
      if (!(x > 0.0)) ok = false;
      s.set_h(i, x);
    }
    done = ok;
  }
  if (!done) {  // unreachable in practice: k = 0 with the mean rate
    k = 0;
    s.set_h(1, (double)a.E / a.T);
  }
  s.clear_above(k, *khi);
  *score = coal_full_score(a, k, s, ev, bk, tab);
  return k;
}

// mh(trace, select(K)) (coal.jl:338-345 simple_mcmc_step; the Dynamic DSL's
// regenerate, src/dynamic/regenerate.jl): k' ~ poisson(3); change points
// 1..min(k, k') and rates 1..min(k, k')+1 keep their values, the others are
// drawn from their distributions under the new k' (min_uniform_continuous,
// gamma) or discarded; the weight is, over the kept unselected choices, new
// score - old score (change point i: its min_uniform_continuous(cp_{i-1}, T,
// k - i + 1) density under k' and under k; the rates' gamma arguments do not
// change) plus the events' new logpdf - old.  Draws of iteration `step`:
// block 6 (k', acceptance), 8 + i (new change point i), 48 + i (new rate i).
// Returns whether the move was accepted (the LDS row and k, score updated).
__device__ bool coal_regen_k(const CoalArgs& a, uint64_t c, uint32_t step, const CoalLds& s, const double* ev,
                             const int32_t* bk, const double* tab, int* k_io, double* score_io, int* khi) {
  const int k = *k_io;
  const CoalU B6 = coal_block(a.seed, c, step, 6);
  const double u = u53(B6.x, B6.y);
  double p = gh_exp(-3.0), cum = p;
  int kk = 0;
  while (u >= cum && kk < 200) {
    ++kk;
    p = p * (3.0 / (double)kk);
    cum += p;
  }
  if (kk > kCoalKMax) return false;  // beyond the engine's capacity: refused (P < 1e-21)
  *khi = kk > *khi ? kk : *khi;
  const double T = a.T;
  const int m = k < kk ? k : kk;
  const double dk = (double)(kk - k);
  double w = 0.0, lower = 0.0;
  for (int i = 1; i <= m; ++i) {  // kept change points, re-scored under k'
    const double x = s.cp(i);
    w += dk * (gh_log_unit(T - x, tab) - gh_log_unit(T - lower, tab)) +
         (gh_log_unit((double)(kk - i + 1), tab) - gh_log_unit((double)(k - i + 1), tab));
    lower = x;
  }
  const double old_ev = coal_events_lp(a, k, s, ev, bk, tab);
  // the new choices, written into the free LDS fields (zeroed again on rejection)
  bool ok = true;
  for (int i = k + 1; i <= kk; ++i) {
    const double q = coal_u(a.seed, c, step, 8u + (uint32_t)i);
    const double mm = (double)(kk - i + 1);
    const double x = T - (T - lower) * gh_exp(gh_log(1.0 - q) / mm);
    if (!(x > lower && x < T)) ok = false;
    s.set_cp(i, x);
    lower = x;
  }
  for (int i = k + 2; i <= kk + 1; ++i) {
    const double q = coal_u(a.seed, c, step, 48u + (uint32_t)i);
    const double x = -gh_log(1.0 - q) / kCoalRate;
    if (!(x > 0.0)) ok = false;
    s.set_h(i, x);
  }
  double alpha = -INFINITY;
  if (ok) alpha = w + (coal_events_lp(a, kk, s, ev, bk, tab) - old_ev);
  const bool acc = gh_log_unit(one_minus_u53(B6.z, B6.w), tab) < alpha;
  const int keep = acc ? kk : k;
  s.clear_above(keep, *khi);
  if (acc) {
    *k_io = kk;
    *score_io = coal_full_score(a, kk, s, ev, bk, tab);
  }
  return acc;
}

__global__ __launch_bounds__(kCoalBlock) void k_coal(CoalArgs a) {
  __shared__ double st[kCoalBlock / 64][kCoalLF * 64];  // per wave: [field][lane]
  __shared__ double tab[kMathTabDoubles / 3];          // the log bins (gh_log_unit)
  extern __shared__ double dyn[];                      // E event times, then the bucket table
  double* ev = dyn;
  int32_t* bk = reinterpret_cast<int32_t*>(dyn + a.E);
  for (int i = threadIdx.x; i < kMathTabDoubles / 3; i += kCoalBlock) tab[i] = gh_math_tab_dev[i];
  for (int i = threadIdx.x; i < a.E; i += kCoalBlock) ev[i] = a.events[i];
  for (int i = threadIdx.x; i < kCoalBuckets; i += kCoalBlock) bk[i] = a.bucket[i];
  __syncthreads();
  const int64_t cl = (int64_t)blockIdx.x * kCoalBlock + threadIdx.x;
  if (cl >= a.n_chains) return;  // no block barrier below
  const int lane = threadIdx.x & 63;
  double* g = a.state + cl;  // field f at g[f * ld]
  const CoalLds s{&st[threadIdx.x >> 6][lane], g, a.ld};
  const uint64_t c = (uint64_t)(a.chain0 + cl);
  const double T = a.T;
  int k, khi = 0;  // khi: the largest k the row has held (its fields past khi are 0)
  double score;
  if (a.init) {
    k = coal_init(a, c, s, ev, bk, tab, &score, &khi);
  } else {
    k = (int)g[0];
    khi = k;
    score = g[a.ld];
    // the window: cp 1..kCoalWin (row fields 0..), h 1..kCoalWin+1 (row fields kCoalKMax..)
#pragma unroll
    for (int f = 0; f < kCoalWin; ++f) s.p[f * 64] = g[(2 + f) * a.ld];
#pragma unroll
    for (int f = 0; f <= kCoalWin; ++f) s.p[(kCoalWin + f) * 64] = g[(2 + kCoalKMax + f) * a.ld];
  }
  int acc[3] = {0, 0, 0};
  for (int it = 0; it < a.n_iters; ++it) {
    const uint32_t step = (uint32_t)(a.iter0 + it + 1);
    const CoalU B0 = coal_block(a.seed, c, step, 0);
    const CoalU B1 = coal_block(a.seed, c, step, 1);
    // ---- rate move (coal.jl:103-134): segment i's rate h -> nh ~ U(h/2, 2h)
    {
      const int i = (int)(u53(B0.x, B0.y) * (double)(k + 1)) + 1;  // uniform_discrete(1, k+1)
      const double h = s.h(i);  // (a read past the window goes to HBM)
      const double lo = h * 0.5, hi = h * 2.0;
      const double nh = lo + (hi - lo) * u53(B0.z, B0.w);
      const double b_lo = i == 1 ? 0.0 : s.cp(i - 1);
      const double b_hi = i == k + 1 ? T : s.cp(i);
      const int n_lo = i == 1 ? 0 : coal_count(ev, bk, a.E, a.bscale, b_lo);
      const int n_hi = i == k + 1 ? a.E : coal_count(ev, bk, a.E, a.bscale, b_hi);
      const double dh = nh - h;
      const double delta =
          ((double)(n_hi - n_lo) * (gh_log_unit(nh, tab) - gh_log_unit(h, tab)) - (b_hi - b_lo) * dh) - dh * kCoalRate;
      // fwd - bwd: the uniform_discrete terms cancel; the new_rate densities
      const double alpha = delta + (gh_log_unit(hi - lo, tab) - gh_log_unit(nh * 2.0 - nh * 0.5, tab));
      if (gh_log_unit(one_minus_u53(B1.x, B1.y), tab) < alpha) {
        s.set_h(i, nh);
        score += delta;
        acc[0] += 1;
      }
    }
    // ---- position move (coal.jl:140-167), if k > 0: cp_i -> U(cp_{i-1}, cp_{i+1})
    if (k > 0) {
      const CoalU B2 = coal_block(a.seed, c, step, 2);
      const int i = (int)(u53(B1.z, B1.w) * (double)k) + 1;  // uniform_discrete(1, k)
      const double lower = i == 1 ? 0.0 : s.cp(i - 1);
      const double upper = i == k ? T : s.cp(i + 1);
      const double x = s.cp(i);
      const double nx = lower + (upper - lower) * u53(B2.x, B2.y);
      double alpha = -INFINITY, delta = 0.0;
      if (nx > lower && nx < upper) {
        const double hi_ = s.h(i), hn = s.h(i + 1);
        const int dc = coal_count(ev, bk, a.E, a.bscale, nx) - coal_count(ev, bk, a.E, a.bscale, x);
        delta = (double)dc * (gh_log_unit(hi_, tab) - gh_log_unit(hn, tab)) - (nx - x) * (hi_ - hn);
        alpha = delta;  // the neighbours bound both proposals: fwd == bwd
      }
      if (gh_log_unit(one_minus_u53(B2.z, B2.w), tab) < alpha) {
        s.set_cp(i, nx);
        score += delta;
        acc[1] += 1;
      }
    }
    // ---- simple_mcmc_step: regenerate k (coal.jl:338-345)
    if (a.simple) {
      if (coal_regen_k(a, c, step, s, ev, bk, tab, &k, &score, &khi)) acc[2] += 1;
    } else {  // ---- birth / death move (coal.jl:173-318)
      const CoalU B3 = coal_block(a.seed, c, step, 3);
      const CoalU B4 = coal_block(a.seed, c, step, 4);
      const bool birth = k == 0 || u53(B3.x, B3.y) < 0.5;
      double alpha = -INFINITY, delta = 0.0;
      int i = 0;
      double x = 0.0, hp = 0.0, hn = 0.0, h = 0.0;
      if (birth) {
        i = (int)(u53(B3.z, B3.w) * (double)(k + 1)) + 1;  // CHOSEN: segment to split
        const double lower = i == 1 ? 0.0 : s.cp(i - 1);
        const double upper = i == k + 1 ? T : s.cp(i);
        x = lower + (upper - lower) * u53(B4.x, B4.y);
        const double uu = u53(B4.z, B4.w);
        const double d_prev = x - lower, d_next = upper - x;
        if (k < kCoalKMax && d_prev > 0.0 && d_next > 0.0 && uu > 0.0) {
          // new_rates (coal.jl:211-223)
          h = s.h(i);
          const double d_total = d_prev + d_next;
          const double lh = gh_log_unit(h, tab);
          const double lr = gh_log_unit(one_minus_u53(B4.z, B4.w), tab) - gh_log_unit(uu, tab);
          hp = gh_exp(lh - (d_next / d_total) * lr);
          hn = gh_exp(lh + (d_prev / d_total) * lr);
          const int n_lo = i == 1 ? 0 : coal_count(ev, bk, a.E, a.bscale, lower);
          const int n_hi = i == k + 1 ? a.E : coal_count(ev, bk, a.E, a.bscale, upper);
          const int n_x = coal_count(ev, bk, a.E, a.bscale, x);
          const double lhp = gh_log_unit(hp, tab), lhn = gh_log_unit(hn, tab);
          delta = ((a.kb + a.ktheta) - ((hp + hn) - h) * kCoalRate) +
                  (((double)(n_x - n_lo) * lhp + (double)(n_hi - n_x) * lhn) - (double)(n_hi - n_lo) * lh) -
                  ((d_prev * hp + d_next * hn) - (upper - lower) * h);
          const double fwd = ((k > 0 ? a.lhalf : 0.0) - gh_log_unit((double)(k + 1), tab)) -
                             gh_log_unit(upper - lower, tab);
          const double bwd = a.lhalf - gh_log_unit((double)(k + 1), tab);
          const double logj = 2.0 * gh_log_unit(hp + hn, tab) - lh;
          alpha = ((delta + bwd) - fwd) + logj;
        }
      } else {
        i = (int)(u53(B3.z, B3.w) * (double)k) + 1;  // CHOSEN: change point to delete
        x = s.cp(i);
        const double lower = i == 1 ? 0.0 : s.cp(i - 1);
        const double upper = i == k ? T : s.cp(i + 1);
        const double d_prev = x - lower, d_next = upper - x;
        if (d_prev > 0.0 && d_next > 0.0) {
          // new_rates_inverse (coal.jl:225-238)
          hp = s.h(i);
          hn = s.h(i + 1);
          const double d_total = d_prev + d_next;
          const double lhp = gh_log_unit(hp, tab), lhn = gh_log_unit(hn, tab);
          h = gh_exp((d_prev / d_total) * lhp + (d_next / d_total) * lhn);
          const double lh = gh_log_unit(h, tab);
          const int n_lo = i == 1 ? 0 : coal_count(ev, bk, a.E, a.bscale, lower);
          const int n_hi = i == k ? a.E : coal_count(ev, bk, a.E, a.bscale, upper);
          const int n_x = coal_count(ev, bk, a.E, a.bscale, x);
          delta = (-(a.kb + a.ktheta) - (h - (hp + hn)) * kCoalRate) +
                  ((double)(n_hi - n_lo) * lh - ((double)(n_x - n_lo) * lhp + (double)(n_hi - n_x) * lhn)) -
                  ((upper - lower) * h - (d_prev * hp + d_next * hn));
          const double fwd = a.lhalf - gh_log_unit((double)k, tab);
          const double bwd = ((k - 1 > 0 ? a.lhalf : 0.0) - gh_log_unit((double)k, tab)) -
                             gh_log_unit(upper - lower, tab);
          const double logj = lh - 2.0 * gh_log_unit(hp + hn, tab);
          alpha = ((delta + bwd) - fwd) + logj;
        }
      }
      const CoalU B5 = coal_block(a.seed, c, step, 5);
      if (gh_log_unit(one_minus_u53(B5.x, B5.y), tab) < alpha) {
        if (birth) {  // birth(k, i) (coal.jl:260-283): insert cp at i, rates (hp, hn) at (i, i+1)
          for (int j = k; j >= i; --j) s.set_cp(j + 1, s.cp(j));
          s.set_cp(i, x);
          for (int j = k + 1; j >= i + 1; --j) s.set_h(j + 1, s.h(j));
          s.set_h(i, hp);
          s.set_h(i + 1, hn);
          k += 1;
          khi = k > khi ? k : khi;
        } else {  // death(k, i) (coal.jl:285-305): remove cp i, rate h at i
          for (int j = i; j <= k - 1; ++j) s.set_cp(j, s.cp(j + 1));
          s.set_cp(k, 0.0);
          s.set_h(i, h);
          for (int j = i + 1; j <= k; ++j) s.set_h(j, s.h(j + 1));
          s.set_h(k + 1, 0.0);
          k -= 1;
        }
        score += delta;
        acc[2] += 1;
      }
    }
    if (a.khist) a.khist[cl * a.n_iters + it] = (int32_t)k;
  }
  g[0] = (double)k;
  g[a.ld] = score;
#pragma unroll
  for (int f = 0; f < kCoalWin; ++f) g[(2 + f) * a.ld] = s.p[f * 64];
#pragma unroll
  for (int f = 0; f <= kCoalWin; ++f) g[(2 + kCoalKMax + f) * a.ld] = s.p[(kCoalWin + f) * 64];
  g[(kCoalW - 1) * a.ld] = 0.0;
  for (int m = 0; m < 3; ++m) a.accepts[cl * 3 + m] = acc[m];
}

// AoS rows [n][kCoalW] (the host layout) <-> SoA fields [kCoalW][ld]
__global__ void k_coal_rows(double* soa, int64_t ld, double* aos, int64_t n, int to_soa) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * kCoalW) return;
  const int64_t c = i / kCoalW, f = i - c * kCoalW;  // aos index: coalesced on the AoS side
  if (to_soa) soa[f * ld + c] = aos[i];
  else aos[i] = soa[f * ld + c];
}

}  // namespace gh
