// gh_rejuv.h — rejuvenation moves on the particles of a filter.
//
// The reference leaves rejuvenation to the caller: after a step it applies
// an MH kernel to every trace, typically
//     state.traces[i], _ = mh(state.traces[i], select(:x => t))
// (src/inference/mh.jl:14-26, selection form: regenerate the selected choices
// from their prior; accept iff log(rand()) < weight), and the particle's log
// weight is left as it is (mh keeps the target of the trace).  Regenerating the
// current latent x_t from its prior given x_{t-1} gives
//     weight = log p(y_t | x'_t) - log p(y_t | x_t)
// because the transition density cancels between the new score and the
// proposal.  At t = 1 the prior is the initial-state distribution.  A static
// model with several latent addresses (the regression's :slope, :intercept)
// regenerates the selected ones only (mh(trace, select(:slope)),
// examples/regression/quickstart.jl:17-22): weight = the log-likelihood
// difference again (the selected choices' prior scores cancel, the
// unselected roots' are unchanged).
//
// One particle per lane; the current state and its parent's state live in
// registers for all moves.  Move w (counted from the step) draws its proposal
// from draw window (w mod 4096) * kRejuvDraws of stream STREAM_MH + 16 (w / 4096)
// and its acceptance uniform from the last draw of that window;
// the first 4096 moves use the MH stream itself.
#pragma once
#include <type_traits>

#include "gh_kernels.h"

namespace gh {

constexpr uint32_t kRejuvDraws = 16;           // draw window per move (LG d <= 16 uses 8)
constexpr uint32_t kRejuvMaxMoves = 1u << 24;  // 4096 windows x 4096 stream blocks

__device__ __host__ __forceinline__ Draw rejuv_draw(uint32_t w) {
  return Draw{(uint32_t)STREAM_MH + ((w >> 12) << 4), (w & 4095u) * kRejuvDraws};
}

struct RejuvArgs {
  const double* xprev;    // wave-tiled states of step t-1 (t >= 2)
  const int32_t* anc;     // ancestors consumed by step t (valid when *res)
  const int32_t* res;     // res_hist + t: a resample preceded step t
  const double* remote;   // multi-rank rows received by the last exchange
  int64_t ld_remote;
  double* x;              // wave-tiled states of step t, rewritten in place
  int64_t n, lo;
  uint64_t seed;
  uint32_t t;
  uint32_t move0;         // moves already applied at this step
  uint32_t select;        // selected latent addresses of the step (the regression: bit 0 :slope, bit 1 :intercept)
  int n_moves;
  unsigned long long* accepted;  // accepted moves (summed over particles)
};

// the drift's standard deviation per state component (0: not selected)
struct DriftSd {
  double v[16];
};

template <class Model, bool INIT>
__global__ __launch_bounds__(kBlock) void k_rejuv(const double* __restrict__ prm, typename Model::Params p0,
                                                  StepObs o, RejuvArgs a) {
  constexpr int D = Model::kD;
  const typename Model::Params p = p0.rebase(prm);
  __shared__ double tab[kMathTabDoubles];  // Box–Muller tables (LDS reads)
  load_math_tab(tab);
  lds_barrier();
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  unsigned acc = 0;
  if (j < a.n) {
    const uint64_t pid = (uint64_t)(a.lo + j);
    double x[D], xp[D], y[D];
#pragma unroll
    for (int k = 0; k < D; ++k) x[k] = a.x[xidx(j, k, D)];
    if (!INIT) {
      const int64_t src = *a.res ? (int64_t)a.anc[j] : j;
      if (src >= 0) {
#pragma unroll
        for (int k = 0; k < D; ++k) xp[k] = a.xprev[xidx(src, k, D)];
      } else {
#pragma unroll
        for (int k = 0; k < D; ++k) xp[k] = ld_sys(&a.remote[(-1 - src) * a.ld_remote + k]);
      }
    }
    double ll = Model::loglik(p, o, x);
    for (int m = 0; m < a.n_moves; ++m) {
      Draw dr = rejuv_draw(a.move0 + (uint32_t)m);
      dr.tab = tab;
      // the prior proposal's weight increment is the observation log-density
      double ll2;
      if constexpr (INIT && std::is_same<Model, RegModel>::value)
        ll2 = Model::init_select(p, o, a.seed, pid, a.select, x, y, dr);
      else
        ll2 = INIT ? Model::init(p, o, a.seed, pid, 0, y, dr) : Model::step(p, o, a.seed, pid, a.t, 0, xp, y, dr);
      const u32x4 w = rng_block(a.seed, pid, a.t, dr.stream, dr.base + kRejuvDraws - 1);
      const double logu = gh_log(u53(w.x, w.y));
      if (logu < ll2 - ll) {
#pragma unroll
        for (int k = 0; k < D; ++k) x[k] = y[k];
        ll = ll2;
        ++acc;
      }
    }
#pragma unroll
    for (int k = 0; k < D; ++k) a.x[xidx(j, k, D)] = x[k];
  }
  const uint64_t tot = wave_sum_u64((uint64_t)acc);
  if ((threadIdx.x & 63) == 0 && tot) atomicAdd(a.accepted, (unsigned long long)tot);
}

}  // namespace gh

namespace gh {

// mh(trace, drift, (sd,)) on every particle (src/inference/mh.jl:41-62, the
// proposal form): a Gaussian drift proposal — `@trace(normal(trace[a], sd), a)`
// for each selected latent address a of the current step (the LG-SSM's :x
// drifts componentwise by the sd vector, a diagonal mvnormal) — then
// update and accept iff log(rand()) < weight - fwd score + bwd score.  The
// drift is symmetric, its forward and backward scores are the same number
// ((x' - x)^2 = (x - x')^2 in floating point), so the acceptance ratio is the
// update weight: the step's latent and observation scores (Model::score, the
// trace's score columns) at x' minus those at x — the current step's latent
// has no children yet.  Draws: move w's window as k_rejuv (normals from its
// first blocks, the uniform from its last).
template <class Model, bool INIT>
__global__ __launch_bounds__(kBlock) void k_mh_drift(const double* __restrict__ prm, typename Model::Params p0,
                                                     StepObs o, RejuvArgs a, DriftSd sd) {
  constexpr int D = Model::kD;
  const typename Model::Params p = p0.rebase(prm);
  __shared__ double tab[kMathTabDoubles];
  load_math_tab(tab);
  lds_barrier();
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  unsigned acc = 0;
  if (j < a.n) {
    const uint64_t pid = (uint64_t)(a.lo + j);
    double x[D], xp[D], y[D], z[D + 1];
#pragma unroll
    for (int k = 0; k < D; ++k) x[k] = a.x[xidx(j, k, D)];
#pragma unroll
    for (int k = 0; k < D; ++k) xp[k] = 0.0;
    if (!INIT) {
      const int64_t src = *a.res ? (int64_t)a.anc[j] : j;
      if (src >= 0) {
#pragma unroll
        for (int k = 0; k < D; ++k) xp[k] = a.xprev[xidx(src, k, D)];
      } else {
#pragma unroll
        for (int k = 0; k < D; ++k) xp[k] = ld_sys(&a.remote[(-1 - src) * a.ld_remote + k]);
      }
    }
    double lat, ob;
    Model::score(p, o, a.t, xp, x, &lat, &ob);
    double s = lat + ob;
    for (int m = 0; m < a.n_moves; ++m) {
      const Draw dr = rejuv_draw(a.move0 + (uint32_t)m);
      normals_n<D>(a.seed, pid, a.t, dr.stream, dr.base, z, tab);
#pragma unroll
      for (int k = 0; k < D; ++k) y[k] = sd.v[k] > 0.0 ? x[k] + sd.v[k] * z[k] : x[k];
      Model::score(p, o, a.t, xp, y, &lat, &ob);
      const double s2 = lat + ob;
      const u32x4 w = rng_block(a.seed, pid, a.t, dr.stream, dr.base + kRejuvDraws - 1);
      const double logu = gh_log(u53(w.x, w.y));
      if (logu < s2 - s) {
#pragma unroll
        for (int k = 0; k < D; ++k) x[k] = y[k];
        s = s2;
        ++acc;
      }
    }
#pragma unroll
    for (int k = 0; k < D; ++k) a.x[xidx(j, k, D)] = x[k];
  }
  const uint64_t tot = wave_sum_u64((uint64_t)acc);
  if ((threadIdx.x & 63) == 0 && tot) atomicAdd(a.accepted, (unsigned long long)tot);
}

}  // namespace gh
