// gh_csmc.h — conditional SMC (the particle-Gibbs sweep).
//
// Reference: examples/pmmh/smc.jl:100-151 (conditional_smc).  Particle 0 (the
// reference's ONE) is the distinguished particle: its state at every step is
// given, its parent is itself, and its weight accumulates the score the
// proposal would have given that state:
//     init_score(x_1)          = log p(y_1 | x_1)            (smc.jl:115)
//     forward_score(x', x, t)  = log p(y_t | x_t)            (smc.jl:141)
// for the model's own (prior) proposal, whose weight increment is the
// observation log-density.  The other particles are the ordinary filter
// (smc.jl:143-147); their multinomial ancestors may pick particle 0.
//
// The step kernel is left untouched: k_pin_pre saves the distinguished
// particle's new weight before the step overwrites its old one, k_pin_post
// writes its state and weight after the step and recomputes block 0's
// partial (max, sum e, sum e^2) with the step kernel's own reduction, so the
// statistics are those a step with particle 0 pinned would have produced.
#pragma once
#include "gh_kernels.h"

namespace gh {

struct PinArgs {
  const double* ref;      // [D] the distinguished state of this step
  double* w0;             // scratch: its new log weight
  const DevScalars* dev;  // resample flags (read when `resampled`)
  int resampled;          // a maybe_resample! was enqueued since the last step
  double* x;              // wave-tiled states of this step (xidx)
  double* logw;
  int64_t n;
  double* pm;             // block-0 partial of the step kernel
  double* ps;
  double* ps2;
};

template <class Model, bool INIT>
__global__ void k_pin_pre(const double* __restrict__ prm, typename Model::Params p0, StepObs o, PinArgs a) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const typename Model::Params p = p0.rebase(prm);
  constexpr int D = Model::kD;
  double x[D];
#pragma unroll
  for (int k = 0; k < D; ++k) x[k] = a.ref[k];
  double base = 0.0;
  if (!INIT) {
    const int pend = a.resampled ? (a.dev->pending | a.dev->fire) : 0;
    base = pend ? 0.0 : a.logw[0];
  }
  *a.w0 = base + Model::loglik(p, o, x);
}

static __global__ __launch_bounds__(kBlock) void k_pin_post(PinArgs a, int D) {
  __shared__ double sm[3][4];
  const int64_t j = threadIdx.x;
  double lw = j < a.n ? a.logw[j] : -INFINITY;
  if (j == 0) {
    for (int k = 0; k < D; ++k) a.x[xidx(0, k, D)] = a.ref[k];  // particle 0
    lw = *a.w0;
    a.logw[0] = lw;
  }
  block_partial(lw, sm, a.pm, a.ps, a.ps2);
}

}  // namespace gh
