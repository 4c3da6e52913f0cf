// gh_coal.h — reversible-jump MH chains on the coal-mining change-point model
// (config C3).
//
// Reference: examples/coal/coal.jl:47-62 (model), :18-33 (min_uniform_continuous),
// examples/coal/poisson_process.jl:9-67 (piecewise Poisson process), and the
// three moves of mcmc_step (coal.jl:329-336): rate_move (:126-150),
// position_move (:156-184), birth_death_move (:190-318), each an involutive
// MH step (src/inference/mh.jl:85-98 over trace_translators.jl:848-876:
// log_weight = new score - old score + bwd score - fwd score + log|J|).
// The Jacobian of the birth map (h, u) -> (h_prev, h_next) is taken in closed
// form, |J| = (h_prev + h_next)^2 / h (Green 1995), where the reference
// differentiates the transform with ForwardDiff (trace_translators.jl:534-589).
//
// One thread per chain.  A chain's state lives in HBM as one row of
// kCoalW doubles (k, score, change points, rates); the 190 event times live
// in LDS.  The full specification (score order, draw indices) is DESIGN.md
// §7c and is restated by oracle/gh_oracle.c (orc_coal_run).
#pragma once
#include "gh_kernels.h"

namespace gh {

constexpr int kCoalKMax = 32;
constexpr int kCoalW = 2 + kCoalKMax + (kCoalKMax + 1) + 1;  // 68: k, score, cp[32], h[33], pad
constexpr int kCoalMaxEvents = 4096;
constexpr double kCoalTheta = 1.0 / 200.0;  // gamma(1, 1/200) rate prior (coal.jl:56-58)

struct CoalArgs {
  const double* events;  // sorted event times
  int E;
  double T;              // observation window [0, T]
  int64_t chain0, n_chains;
  uint64_t seed;
  int n_iters, iter0;
  int init;              // 1: draw the start from the prior (generate)
  double* state;         // SoA [2][kCoalW][ld]: current row fields, then proposal row fields
  int64_t ld;            // chains per field column (>= n_chains)
  int32_t* accepts;      // [n_chains][3] rate, position, birth/death
  int32_t* khist;        // optional [n_chains][n_iters] k after each iteration
};

// one chain's row (k, score, cp[32], h[33], pad) in the SoA state: field i
// of chain c at p[i * ld] — a wave's 64 chains read one field coalesced
struct CoalRow {
  double* p;
  int64_t ld;
  __device__ __forceinline__ double& operator[](int i) const { return p[(int64_t)i * ld]; }
};

__device__ __forceinline__ double coal_u(uint64_t seed, uint64_t c, uint32_t step, uint32_t d) {
  const u32x4 w = rng_block(seed, c, step, STREAM_MH, d);
  return u53(w.x, w.y);
}

// number of events <= x (events sorted, in LDS)
__device__ __forceinline__ int coal_upper(const double* ev, int E, double x) {
  int lo = 0, hi = E;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (ev[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// score of the state row s (coal.jl:47-62 with poisson_process.jl:34-51)
__device__ double coal_score(const CoalRow& s, const double* ev, int E, double T, const double* tab) {
  const int k = (int)s[0];
  const CoalRow cp{s.p + 2 * s.ld, s.ld};
  const CoalRow h{s.p + (2 + kCoalKMax) * s.ld, s.ld};
  // k ~ poisson(3): k log 3 - 3 - log k!
  double lf = 0.0;
  for (int j = 2; j <= k; ++j) lf += gh_log_unit((double)j, tab);
  double lp = ((double)k * gh_log(3.0) - 3.0) - lf;
  // cp_i ~ min_uniform_continuous(cp_{i-1}, T, k - i + 1)
  double lower = 0.0, l_lower = gh_log(T);
  for (int i = 1; i <= k; ++i) {
    const double x = cp[i - 1];
    if (!(x > lower && x < T)) return -INFINITY;
    const double m = (double)(k - i + 1);
    const double l_x = gh_log_unit(T - x, tab);
    lp += ((m - 1.0) * l_x + gh_log_unit(m, tab)) - m * l_lower;
    lower = x;
    l_lower = l_x;
  }
  // h_i ~ gamma(1, theta): -log theta - x / theta
  const double l_theta = gh_log(kCoalTheta);
  for (int i = 1; i <= k + 1; ++i) {
    const double x = h[i - 1];
    if (!(x > 0.0)) return -INFINITY;
    lp += -l_theta - x / kCoalTheta;
  }
  // events ~ piecewise_poisson_process([0, cp..., T], h)
  double A = 0.0, B = 0.0, b_lo = 0.0;
  int c_lo = 0;
  for (int i = 1; i <= k + 1; ++i) {
    const double b_hi = i <= k ? cp[i - 1] : T;
    const int c_hi = coal_upper(ev, E, b_hi);
    A += (double)(c_hi - c_lo) * gh_log_unit(h[i - 1], tab);
    B += (b_hi - b_lo) * h[i - 1];
    b_lo = b_hi;
    c_lo = c_hi;
  }
  return lp + (A - B);
}

__device__ __forceinline__ void coal_copy(const CoalRow& src, const CoalRow& dst) {
  const int k = (int)src[0];
  dst[0] = src[0];
  for (int i = 0; i < k; ++i) dst[2 + i] = src[2 + i];
  for (int i = 0; i <= k; ++i) dst[2 + kCoalKMax + i] = src[2 + kCoalKMax + i];
}

// generate(model, (T,), observations): k, change points and rates from the
// prior (attempt a uses draws 100 a + ...; a degenerate draw retries)
__device__ void coal_init(const CoalArgs& a, uint64_t c, const CoalRow& s) {
  for (int att = 0; att < 64; ++att) {
    const uint32_t d0 = 100u * (uint32_t)att;
    // k ~ poisson(3) by inverse CDF
    const double u = coal_u(a.seed, c, 0, d0);
    double p = gh_exp(-3.0), cum = p;
    int k = 0;
    while (u >= cum && k < 200) {
      ++k;
      p = p * (3.0 / (double)k);
      cum += p;
    }
    if (k > kCoalKMax) continue;
    bool ok = true;
    double lower = 0.0;
    for (int i = 1; i <= k; ++i) {
      // min_uniform_continuous(lower, T, m): upper - (upper - lower) (1 - p)^(1/m)  (coal.jl:28-32)
      const double q = coal_u(a.seed, c, 0, d0 + 1u + (uint32_t)i);
      const double m = (double)(k - i + 1);
      const double x = a.T - (a.T - lower) * gh_exp(gh_log(1.0 - q) / m);
      if (!(x > lower && x < a.T)) ok = false;
      s[2 + i - 1] = x;
      lower = x;
    }
    for (int i = 1; i <= k + 1; ++i) {
      // gamma(1, theta) = exponential: -theta log(1 - q)
      const double q = coal_u(a.seed, c, 0, d0 + 40u + (uint32_t)i);
      const double x = -kCoalTheta * gh_log(1.0 - q);
      if (!(x > 0.0)) ok = false;
      s[2 + kCoalKMax + i - 1] = x;
    }
    if (!ok) continue;
    s[0] = (double)k;
    return;
  }
  s[0] = 0.0;  // unreachable in practice: k = 0 with a mean rate
  s[2 + kCoalKMax] = (double)a.E / a.T;
}

__global__ __launch_bounds__(256) void k_coal(CoalArgs a) {
  extern __shared__ double ev[];  // the E event times (dynamic LDS: E doubles)
  __shared__ double tab[kMathTabDoubles];  // the log table, per-lane reads from LDS
  load_math_tab(tab);
  for (int i = threadIdx.x; i < a.E; i += blockDim.x) ev[i] = a.events[i];
  __syncthreads();
  const int64_t cl = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (cl >= a.n_chains) return;
  const uint64_t c = (uint64_t)(a.chain0 + cl);
  const CoalRow cur{a.state + cl, a.ld};
  const CoalRow prop{a.state + kCoalW * a.ld + cl, a.ld};
  const double T = a.T;
  if (a.init) {
    coal_init(a, c, cur);
    cur[1] = coal_score(cur, ev, a.E, T, tab);
  }
  int acc[3] = {0, 0, 0};
  for (int it = 0; it < a.n_iters; ++it) {
    const uint32_t step = (uint32_t)(a.iter0 + it + 1);
    // ---- rate move (coal.jl:126-150)
    {
      const int k = (int)cur[0];
      const double ui = coal_u(a.seed, c, step, 0);
      const int i = (int)(ui * (double)(k + 1)) + 1;  // uniform_discrete(1, k+1)
      const double h = cur[2 + kCoalKMax + i - 1];
      const double lo = h / 2.0, hi = h * 2.0;
      const double nh = lo + (hi - lo) * coal_u(a.seed, c, step, 1);
      coal_copy(cur, prop);
      prop[2 + kCoalKMax + i - 1] = nh;
      const double sn = coal_score(prop, ev, a.E, T, tab);
      const double fwd = -gh_log((double)(k + 1)) - gh_log(hi - lo);
      const double bwd = -gh_log((double)(k + 1)) - gh_log(nh * 2.0 - nh / 2.0);
      const double alpha = ((sn - cur[1]) + bwd) - fwd;
      if (gh_log(coal_u(a.seed, c, step, 2)) < alpha) {
        cur[2 + kCoalKMax + i - 1] = nh;
        cur[1] = sn;
        acc[0] += 1;
      }
    }
    // ---- position move (coal.jl:156-184), if k > 0
    if ((int)cur[0] > 0) {
      const int k = (int)cur[0];
      const int i = (int)(coal_u(a.seed, c, step, 3) * (double)k) + 1;  // uniform_discrete(1, k)
      const double lower = i == 1 ? 0.0 : cur[2 + i - 2];
      const double upper = i == k ? T : cur[2 + i];
      const double ncp = lower + (upper - lower) * coal_u(a.seed, c, step, 4);
      coal_copy(cur, prop);
      prop[2 + i - 1] = ncp;
      const double sn = coal_score(prop, ev, a.E, T, tab);
      const double fwd = -gh_log((double)k) - gh_log(upper - lower);
      const double bwd = fwd;  // the neighbours bound both proposals
      const double alpha = ((sn - cur[1]) + bwd) - fwd;
      if (gh_log(coal_u(a.seed, c, step, 5)) < alpha) {
        cur[2 + i - 1] = ncp;
        cur[1] = sn;
        acc[1] += 1;
      }
    }
    // ---- birth / death move (coal.jl:190-318)
    {
      const int k = (int)cur[0];
      const bool birth = k == 0 || coal_u(a.seed, c, step, 6) < 0.5;
      double alpha = -INFINITY, sn = -INFINITY;
      if (birth) {
        const int i = (int)(coal_u(a.seed, c, step, 7) * (double)(k + 1)) + 1;  // CHOSEN
        const double lower = i == 1 ? 0.0 : cur[2 + i - 2];
        const double upper = i == k + 1 ? T : cur[2 + i - 1];
        const double ncp = lower + (upper - lower) * coal_u(a.seed, c, step, 8);
        const double uu = coal_u(a.seed, c, step, 9);
        const double d_prev = ncp - lower, d_next = upper - ncp;
        if (k < kCoalKMax && d_prev > 0.0 && d_next > 0.0 && uu > 0.0) {
          // new_rates (coal.jl:222-235)
          const double h = cur[2 + kCoalKMax + i - 1];
          const double d_total = d_prev + d_next;
          const double lr = gh_log(1.0 - uu) - gh_log(uu);
          const double hp = gh_exp(gh_log(h) - (d_next / d_total) * lr);
          const double hn = gh_exp(gh_log(h) + (d_prev / d_total) * lr);
          // birth(k, i) (coal.jl:273-297): insert cp at i, rates (hp, hn) at (i, i+1)
          prop[0] = (double)(k + 1);
          for (int j = 1; j < i; ++j) prop[2 + j - 1] = cur[2 + j - 1];
          prop[2 + i - 1] = ncp;
          for (int j = i + 1; j <= k + 1; ++j) prop[2 + j - 1] = cur[2 + j - 2];
          for (int j = 1; j < i; ++j) prop[2 + kCoalKMax + j - 1] = cur[2 + kCoalKMax + j - 1];
          prop[2 + kCoalKMax + i - 1] = hp;
          prop[2 + kCoalKMax + i] = hn;
          for (int j = i + 2; j <= k + 2; ++j) prop[2 + kCoalKMax + j - 1] = cur[2 + kCoalKMax + j - 2];
          sn = coal_score(prop, ev, a.E, T, tab);
          const double fwd = ((k > 0 ? gh_log(0.5) : 0.0) - gh_log((double)(k + 1))) - gh_log(upper - lower);
          const double bwd = gh_log(0.5) - gh_log((double)(k + 1));
          const double logj = 2.0 * gh_log(hp + hn) - gh_log(h);
          alpha = (((sn - cur[1]) + bwd) - fwd) + logj;
        }
      } else {
        const int i = (int)(coal_u(a.seed, c, step, 7) * (double)k) + 1;  // CHOSEN
        const double cpd = cur[2 + i - 1];
        const double lower = i == 1 ? 0.0 : cur[2 + i - 2];
        const double upper = i == k ? T : cur[2 + i];
        const double d_prev = cpd - lower, d_next = upper - cpd;
        if (d_prev > 0.0 && d_next > 0.0) {
          // new_rates_inverse (coal.jl:237-250)
          const double hp = cur[2 + kCoalKMax + i - 1], hn = cur[2 + kCoalKMax + i];
          const double d_total = d_prev + d_next;
          const double h = gh_exp((d_prev / d_total) * gh_log(hp) + (d_next / d_total) * gh_log(hn));
          // death(k, i) (coal.jl:299-318): remove cp i, rate h at i
          prop[0] = (double)(k - 1);
          for (int j = 1; j < i; ++j) prop[2 + j - 1] = cur[2 + j - 1];
          for (int j = i; j <= k - 1; ++j) prop[2 + j - 1] = cur[2 + j];
          for (int j = 1; j < i; ++j) prop[2 + kCoalKMax + j - 1] = cur[2 + kCoalKMax + j - 1];
          prop[2 + kCoalKMax + i - 1] = h;
          for (int j = i + 1; j <= k; ++j) prop[2 + kCoalKMax + j - 1] = cur[2 + kCoalKMax + j];
          sn = coal_score(prop, ev, a.E, T, tab);
          const double fwd = gh_log(0.5) - gh_log((double)k);
          const double bwd = ((k - 1 > 0 ? gh_log(0.5) : 0.0) - gh_log((double)k)) - gh_log(upper - lower);
          const double logj = gh_log(h) - 2.0 * gh_log(hp + hn);
          alpha = (((sn - cur[1]) + bwd) - fwd) + logj;
        }
      }
      if (gh_log(coal_u(a.seed, c, step, 10)) < alpha) {
        coal_copy(prop, cur);
        cur[1] = sn;
        acc[2] += 1;
      }
    }
    if (a.khist) a.khist[cl * a.n_iters + it] = (int32_t)cur[0];
  }
  for (int m = 0; m < 3; ++m) a.accepts[cl * 3 + m] = acc[m];
}

// AoS rows [n][kCoalW] (the host layout) <-> SoA current fields [kCoalW][ld]
__global__ void k_coal_rows(double* soa, int64_t ld, double* aos, int64_t n, int to_soa) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * kCoalW) return;
  const int64_t c = i / kCoalW, f = i - c * kCoalW;  // aos index: coalesced on the AoS side
  if (to_soa) soa[f * ld + c] = aos[i];
  else aos[i] = soa[f * ld + c];
}

}  // namespace gh
