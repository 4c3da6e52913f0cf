// gh_scores.h — the trace score columns of a filter's particles.
//
// A Static-IR trace keeps a value AND a score per random choice
// (src/static_ir/trace.jl:91-129), and get_score(trace) is their total.  The
// engine's traces are the SoA history (one state slot per step + the
// genealogy); their score columns are materialised on the device from it on
// demand: for every current particle k_scores walks the genealogy from the
// last step back to t = 1 (as get_traces does, k_traj) and writes, per step,
// the latent choice's score logpdf(x_t | x_{t-1}) and the observation's
// score logpdf(y_t | x_t) — the model's own densities (Model::score), whatever
// proposal generated the particle — then the trace's total, summed in time
// order (step score = latent + observation, the Unfold's order).  Nothing is
// added to the filter's hot step: the columns cost one pass over the history
// when asked for (gh_pf_get_scores).
#pragma once
#include "gh_kernels.h"

namespace gh {

struct ScoreArgs {
  const double* const* xs;     // device array of per-step state slots (index t-1)
  const int32_t* const* ancs;  // device array of per-step ancestor arrays (index t-1)
  const int32_t* res_before;   // res_before[t]: a resample preceded step t
  const int32_t* anc_pending;  // ancestors of a resample pending after the last step
  int live;                    // the device resample flags are current
  const StepObs* obs;          // [T] each step's observation (prior form)
  int64_t n;
  int T;
  double* per_step;            // [T][2][n]: latent score, observation score
  double* total;               // [n]
};

template <class Model>
__global__ __launch_bounds__(kBlock) void k_scores(const double* __restrict__ prm, typename Model::Params p0, ScoreArgs a,
                                                   const DevScalars* dev) {
  constexpr int D = Model::kD;
  const typename Model::Params p = p0.rebase(prm);
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= a.n) return;
  int64_t idx = j;
  if (a.live && (dev->pending | dev->fire) && a.anc_pending) idx = a.anc_pending[idx];
  double x[D], xp[D];
#pragma unroll
  for (int k = 0; k < D; ++k) x[k] = a.xs[a.T - 1][xidx(idx, k, D)];
  for (int s = a.T; s >= 1; --s) {
    int64_t parent = idx;
    if (s > 1) {
      if (a.res_before[s]) parent = a.ancs[s - 1][idx];
#pragma unroll
      for (int k = 0; k < D; ++k) xp[k] = a.xs[s - 2][xidx(parent, k, D)];
    }
    double lat, ob;
    Model::score(p, a.obs[s - 1], (uint32_t)s, xp, x, &lat, &ob);
    a.per_step[((int64_t)(s - 1) * 2) * a.n + j] = lat;
    a.per_step[((int64_t)(s - 1) * 2 + 1) * a.n + j] = ob;
#pragma unroll
    for (int k = 0; k < D; ++k) x[k] = xp[k];
    idx = parent;
  }
  double tot = 0.0;
  for (int s = 1; s <= a.T; ++s)
    tot += a.per_step[((int64_t)(s - 1) * 2) * a.n + j] + a.per_step[((int64_t)(s - 1) * 2 + 1) * a.n + j];
  a.total[j] = tot;
}

// gh_pf_step_params: after the step under the new parameters, every particle's
// weight gains its trajectory's re-scoring, logw += new - old, and the step
// kernel's block partials are taken again from the new weights (256-particle
// blocks, block_partial's arithmetic) for the next fold / resample.
static __global__ __launch_bounds__(kBlock) void k_add_delta(double* logw, const double* snew, const double* sold,
                                                             int64_t n, double* pm, double* ps, double* ps2) {
  __shared__ double sm[3][4];
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double lw = -INFINITY;
  if (j < n) {
    lw = logw[j] + (snew[j] - sold[j]);
    logw[j] = lw;
  }
  block_partial(lw, sm, pm + blockIdx.x, ps + blockIdx.x, ps2 + blockIdx.x);
}

}  // namespace gh
