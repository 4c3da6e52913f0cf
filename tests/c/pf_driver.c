/* pf_driver.c — the particle filter driven from C through the C ABI alone
 * (include/gen_hip.h), the way a Julia `ccall` shim would drive it
 * (INTEGRATION.md): no Python, no torch.  Test infrastructure, run by
 * tests/test_c_abi.py on the GPU.
 *
 * It runs the reference's HMM particle-filter test
 * (test/inference/particle_filter.jl:145-168: default proposal, resample when
 * ESS < threshold, log_ml_estimate) twice over the same observations:
 *   1. call by call: gh_pf_maybe_resample + gh_pf_step per step (the caller
 *      loop of particle_filter.jl:157-162), decisions read back every step;
 *   2. batched: gh_pf_run over the same steps (no host round trip per step);
 * and prints both log-ML estimates, the resample count and the final parents'
 * checksum; then checks the error path (a NULL filter -> GH_E_INVAL with a
 * message from gh_last_error, as the reference raises `error(...)`).
 *
 * usage: pf_driver k v n seed thr T  prior[k] trans[k*k] emis[v*k] obs[T]
 *   trans[new*k + prev], emis[x*k + z] (gen_hip.h GH_FAMILY_HMM), obs 0-based
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gen_hip.h"

#define TRY(call)                                                                      \
  do {                                                                                 \
    int rc_ = (call);                                                                  \
    if (rc_ != GH_OK) {                                                                \
      fprintf(stderr, "%s failed: status %d: %s\n", #call, rc_, gh_last_error());     \
      return 2;                                                                        \
    }                                                                                  \
  } while (0)

static gh_obs obs_at(const double* xs, int t) {
  gh_obs o = {0};  /* slot 0, no chained observations */
  o.values = &xs[t];
  o.n_values = 1;
  o.present = 1;
  return o;
}

int main(int argc, char** argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: %s k v n seed thr T prior trans emis obs\n", argv[0]);
    return 1;
  }
  const int k = atoi(argv[1]), v = atoi(argv[2]);
  const long long n = atoll(argv[3]);
  const unsigned long long seed = strtoull(argv[4], NULL, 10);
  const double thr = atof(argv[5]);
  const int T = atoi(argv[6]);
  const int np = k + k * k + v * k;
  if (k < 1 || v < 1 || T < 1 || argc != 7 + np + T) {
    fprintf(stderr, "expected %d numbers after the header, got %d\n", np + T, argc - 7);
    return 1;
  }
  double* params = (double*)malloc(sizeof(double) * (size_t)np);
  double* xs = (double*)malloc(sizeof(double) * (size_t)T);
  for (int i = 0; i < np; ++i) params[i] = atof(argv[7 + i]);
  for (int t = 0; t < T; ++t) xs[t] = atof(argv[7 + np + t]);

  gh_ctx* ctx = NULL;
  TRY(gh_ctx_create(0, NULL, &ctx));
  gh_model_desc desc;
  memset(&desc, 0, sizeof(desc));
  desc.family = GH_FAMILY_HMM;
  desc.k = k;
  desc.v = v;
  desc.params = params;
  desc.n_params = np;
  gh_model* m = NULL;
  TRY(gh_model_create(ctx, &desc, &m));
  gh_pf_opts opts;
  gh_pf_opts_default(&opts);

  /* 1. call by call */
  gh_pf* pf = NULL;
  gh_obs o0 = obs_at(xs, 0);
  TRY(gh_pf_init(m, &o0, GH_PROPOSAL_DEFAULT, n, seed, &opts, &pf));
  int resamples = 0;
  for (int t = 1; t < T; ++t) {
    int did = 0;
    double ess = 0.0;
    TRY(gh_pf_maybe_resample(pf, thr, &did, &ess));
    resamples += did;
    gh_obs o = obs_at(xs, t);
    TRY(gh_pf_step(pf, &o, GH_PROPOSAL_DEFAULT));
  }
  double lml1 = 0.0;
  TRY(gh_pf_log_ml_estimate(pf, &lml1));
  int64_t n_global = 0, n_local = 0, first = 0;
  TRY(gh_pf_num_particles(pf, &n_global, &n_local, &first));
  int64_t* parents = (int64_t*)malloc(sizeof(int64_t) * (size_t)n_local);
  TRY(gh_pf_get_parents(pf, parents));
  unsigned long long psum = 0;
  for (int64_t i = 0; i < n_local; ++i) psum = psum * 1000003ull + (unsigned long long)parents[i];

  /* 2. batched: the same filter through gh_pf_run */
  gh_pf* pf2 = NULL;
  TRY(gh_pf_init(m, &o0, GH_PROPOSAL_DEFAULT, n, seed, &opts, &pf2));
  gh_obs* os = (gh_obs*)malloc(sizeof(gh_obs) * (size_t)(T > 1 ? T - 1 : 1));
  for (int t = 1; t < T; ++t) os[t - 1] = obs_at(xs, t);
  TRY(gh_pf_run(pf2, T - 1, os, GH_PROPOSAL_DEFAULT, thr));
  double lml2 = 0.0;
  TRY(gh_pf_log_ml_estimate(pf2, &lml2));
  TRY(gh_pf_get_parents(pf2, parents));
  unsigned long long psum2 = 0;
  for (int64_t i = 0; i < n_local; ++i) psum2 = psum2 * 1000003ull + (unsigned long long)parents[i];

  /* the error path: a NULL filter is an argument error with a message */
  const int bad = gh_pf_step(NULL, &o0, GH_PROPOSAL_DEFAULT);
  const char* msg = gh_last_error();
  const int err_ok = bad == GH_E_INVAL && msg != NULL && msg[0] != '\0';

  printf("log_ml_calls %.17g\nlog_ml_run %.17g\nresamples %d\nparents_equal %d\nn %lld\nerror_path_ok %d\n",
         lml1, lml2, resamples, psum == psum2, (long long)n_global, err_ok);
  TRY(gh_pf_destroy(pf2));
  TRY(gh_pf_destroy(pf));
  TRY(gh_model_destroy(m));
  TRY(gh_ctx_destroy(ctx));
  free(os);
  free(parents);
  free(params);
  free(xs);
  return err_ok ? 0 : 3;
}
