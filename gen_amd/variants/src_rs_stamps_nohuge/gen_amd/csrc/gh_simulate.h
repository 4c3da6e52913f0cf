// gh_simulate.h — simulate(model, (T,)) for N independent traces.
//
// Static-IR simulate (src/static_ir/simulate.jl:23-34, :50-83) visits the
// model's nodes in order: each random choice takes value = random(dist, args)
// and adds logpdf(dist, value, args) to the trace's score; the Unfold
// (src/modeling_library/unfold/simulate.jl) runs the kernel once per step on
// the previous state.  For the lowered families one thread is one trace: per
// step it draws the latent exactly as the filter's generate/update would
// (Model::init / Model::step on the SIM stream, no observation), then the
// observation (Model::sim_obs, draws from kSimObsDraw on), and writes both
// with their scores (Model::score for the latent — the same densities as the
// trace score columns, gh_scores.h).  Outputs are time-major SoA, so every
// store of a step is coalesced across the wave:
//   xs[t][k][n]  latent component k of step t+1
//   ys[t][r][n]  observation component r (HMM: the symbol; regression: y_r)
//   per_step[t][2][n]  latent score, observation score; total[n] = get_score
// Draws are keyed (seed, trace id, t, STREAM_SIM | draw): a trace's choices do
// not depend on N or on the launch shape.
#pragma once
#include "gh_kernels.h"

namespace gh {

struct SimArgs {
  uint64_t seed;
  int64_t n;
  int T;
  int dy;                 // observation components per step
  const StepObs* obs;     // [T] per-step constants (Kitagawa ct), present = 0
  double* xs;             // [T][d][n]
  double* ys;             // [T][dy][n]
  double* per_step;       // [T][2][n]
  double* total;          // [n]
};

template <class Model>
__global__ __launch_bounds__(kBlock) void k_simulate(const double* __restrict__ prm, typename Model::Params p0,
                                                     SimArgs a) {
  constexpr int D = Model::kD;
  const typename Model::Params p = p0.rebase(prm);
  __shared__ double tab[kMathTabDoubles];  // Box–Muller tables (device callers pass one, gh_math.h)
  load_math_tab(tab);
  __syncthreads();
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= a.n) return;
  const Draw dr{STREAM_SIM, 0, tab};
  double x[D], xp[D];
#pragma unroll
  for (int k = 0; k < D; ++k) xp[k] = 0.0;
  double tot = 0.0;
  for (int t = 1; t <= a.T; ++t) {
    const StepObs& o = a.obs[t - 1];
    if (t == 1)
      Model::init(p, o, a.seed, (uint64_t)j, 0, x, dr);
    else
      Model::step(p, o, a.seed, (uint64_t)j, (uint32_t)t, 0, xp, x, dr);
    double* y = a.ys + ((int64_t)(t - 1) * a.dy) * a.n + j;
    const double ob = Model::sim_obs(p, a.seed, (uint64_t)j, (uint32_t)t, x, y, a.n, tab);
    double lat, ob0;
    Model::score(p, o, (uint32_t)t, xp, x, &lat, &ob0);
#pragma unroll
    for (int k = 0; k < D; ++k) a.xs[((int64_t)(t - 1) * D + k) * a.n + j] = x[k];
    a.per_step[((int64_t)(t - 1) * 2) * a.n + j] = lat;
    a.per_step[((int64_t)(t - 1) * 2 + 1) * a.n + j] = ob;
    tot += lat + ob;
#pragma unroll
    for (int k = 0; k < D; ++k) xp[k] = x[k];
  }
  a.total[j] = tot;
}

}  // namespace gh
