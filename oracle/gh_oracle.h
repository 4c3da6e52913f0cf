/* gh_oracle.h — CPU restatement of Gen's particle-filter hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is linked into, loaded by
 * or called from the product (gen_amd/, libgen_hip.so).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the
 * checker / the CPU baseline.
 *
 * Parity status: pinned.  The restatement is checked (tests/test_oracle.py)
 * against (a) the reference's own known-answer tests re-expressed as golden
 * vectors in tests/golden/ (HMM forward algorithm hand enumeration,
 * test/inference/particle_filter.jl:29-48; PF log-ML within atol 0.01 of the
 * exact HMM forward log-ML at N=10000 with resampling every step,
 * test/inference/particle_filter.jl:96-168; Unfold update/regenerate weight
 * closed forms, test/modeling_library/unfold.jl:116-481), and (b) analytic
 * oracles (Kalman-filter log-ML).  Gen.jl itself cannot run here (no Julia).
 *
 * Algorithm sources (reference file:line):
 *   ParticleFilterState            src/inference/particle_filter.jl:18-24
 *   initialize_particle_filter     src/inference/particle_filter.jl:79-108
 *   particle_filter_step!          src/inference/particle_filter.jl:139-180
 *   maybe_resample!                src/inference/particle_filter.jl:189-213
 *   effective_sample_size          src/inference/particle_filter.jl:3-6
 *   log_ml_estimate                src/inference/particle_filter.jl:52-55
 *   logsumexp                      src/inference/inference.jl:3-6
 *   normal logpdf / random         src/modeling_library/distributions/normal.jl:56-60,96
 *   mvnormal logpdf / random       src/modeling_library/distributions/mvnormal.jl:12-16,30-33
 *   categorical logpdf / random    src/modeling_library/distributions/categorical.jl:10-12,20-22
 *   Unfold step semantics          src/modeling_library/unfold/update.jl:54-78
 * RNG, transcendental and resampling arithmetic follow DESIGN.md §4 so that
 * the GPU path can be compared bit-for-bit.
 */
#ifndef GH_ORACLE_H
#define GH_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_LGSSM = 1, ORC_HMM = 2, ORC_KITAGAWA = 3, ORC_REGRESSION = 4,
       /* slot-described Unfold kernel (gen_amd/csrc/gh_slots.h, include/gen_hip.h
          GH_FAMILY_SLOTS): an observation is the slots' values concatenated in
          slot order (m values for an mvnormal slot, one for the others) and
          has_obs the bitmask of the slots present; with per-step inputs
          (latent form 2) bit 4 marks the step's input u_t, d values after
          the dy slot values */
       ORC_SLOTS = 5 };
enum { ORC_SYSTEMATIC = 0, ORC_MULTINOMIAL = 1 };
enum { ORC_PROPOSAL_DEFAULT = 0, ORC_PROPOSAL_OPTIMAL = 1, ORC_PROPOSAL_GAUSSIAN = 2, ORC_PROPOSAL_LINEAR = 3 };

typedef struct orc_pf orc_pf;

/* math primitives (exported so tests can check them against libm / KATs) */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double orc_exp(double x);
double orc_log(double x);
double orc_log_unit(double x); /* x in [2^-53, 1]: the Box–Muller radius log (table-driven) */
double orc_cos(double x);
void orc_sincos_2pi(double u, double* s, double* c);
void orc_sincos_2pi_u32(uint32_t c, double* s, double* co);
void orc_box_muller(uint32_t a, uint32_t b, uint32_t c, double* z0, double* z1);
void orc_normals(uint64_t seed, uint64_t id, uint32_t step, uint32_t stream, int n, double* z);

/* particle filter over particles [lo, lo+n_local) of a global set of n_global */
orc_pf* orc_pf_create(int family, int d, int dy, int k, int v, const double* params, int64_t n_params,
                      int64_t n_global, int64_t lo, int64_t n_local, uint64_t seed, int resampler,
                      int record_history);
void orc_pf_destroy(orc_pf* pf);
int orc_pf_init(orc_pf* pf, const double* obs, int has_obs, int proposal);
int orc_pf_step(orc_pf* pf, const double* obs, int has_obs, int proposal);
/* arguments of the Gaussian custom proposal (alpha, beta, gamma, sigma_q), used
   by init / step with ORC_PROPOSAL_GAUSSIAN (nonlinear SSM) until changed */
int orc_pf_set_proposal_args(orc_pf* pf, const double* args, int n);
/* single-rank maybe_resample!: returns 1/0, or -1 on numeric error */
int orc_pf_maybe_resample(orc_pf* pf, double ess_threshold, double* ess_out);
/* rejuvenation: n_moves mh(trace, select(x_t)) moves per particle (src/inference/mh.jl:14-26);
   -1 if a resample is pending */
int orc_pf_rejuvenate(orc_pf* pf, int n_moves, int64_t* accepted);
/* mh(trace, selection) on every particle: mask over the step's latent addresses
   (the regression: bit 0 :slope, bit 1 :intercept; the Unfold families: bit 0) */
int orc_pf_mh_select(orc_pf* pf, uint32_t mask, int n_moves, int64_t* accepted);
/* conditional SMC (examples/pmmh/smc.jl:100-151): particle 0 pinned to ref
   (multinomial resampler, one shard); a conditional filter steps only with
   orc_pf_step_conditional.  -1 on misuse */
int orc_pf_init_conditional(orc_pf* pf, const double* obs, int has_obs, const double* ref);
int orc_pf_step_conditional(orc_pf* pf, const double* obs, int has_obs, const double* ref);
double orc_pf_log_ml_estimate(orc_pf* pf);
void orc_pf_get_log_weights(orc_pf* pf, double* out);     /* n_local */
void orc_pf_get_state(orc_pf* pf, double* out);           /* [d][n_local] */
void orc_pf_get_parents(orc_pf* pf, int64_t* out);        /* n_local, global ids */
int orc_pf_num_steps(orc_pf* pf);
int orc_pf_get_history(orc_pf* pf, int t, double* x_out, int32_t* anc_out, int* resampled);
/* get_score of every current particle's trace (total [n]) and the per-step
   latent / observation choice scores (per_step [t][2][n], nullable); one shard */
int orc_pf_mh_drift(orc_pf* pf, uint32_t mask, const double* sd, int n_moves, int64_t* accepted);
int orc_pf_get_scores(orc_pf* pf, double* total, double* per_step);
/* a step whose Unfold parameters change (new_args with UnknownChange on them):
   every retained application re-scored, weight += new - old score (see .c) */
int orc_pf_step_params(orc_pf* pf, const double* params, int64_t np, const double* obs, int has_obs, int proposal);
double orc_log1p(double y);
double orc_lgamma(double x);
int orc_dist_logpdf(int dist, int dim, int np, int stride, const double* params, int64_t n, const double* x,
                    double* out);
int orc_dist_random(int dist, int dim, int np, int stride, const double* params, int64_t n, uint64_t seed,
                    double* out);
int orc_simulate(int family, int d, int dy, int k, int v, const double* params, int64_t np, int T, int64_t n,
                 uint64_t seed, double* xs, double* ys, double* per_step, double* total);
int orc_simulate_inputs(int family, int d, int dy, int k, int v, const double* params, int64_t np, int T, int64_t n,
                        uint64_t seed, const double* inputs, double* xs, double* ys, double* per_step,
                        double* total);

/* distributed building blocks (sharded oracle, exercised with gloo) */
void orc_pf_local_stats(orc_pf* pf, double out[3]);      /* (max, sum e, sum e^2) local */
int orc_combine_stats(const double* stats, int R, int64_t n_global, double thr, double* L,
                      double* ess, double* M);
uint64_t orc_pf_local_qtotal(orc_pf* pf, double M);
/* after the collectives: for every global slot j whose target falls in this
   rank's CDF range, emit (j, ancestor global id, state[d]).  Returns count. */
int64_t orc_pf_resample_emit(orc_pf* pf, double M, const uint64_t* totals, int R, int rank,
                             int64_t* slot_out, int64_t* anc_out, double* state_out);
/* install incoming (slot, anc, state) for this rank's own slots and mark the
   resample as done; log_ml update is applied from (L) */
void orc_pf_resample_apply(orc_pf* pf, double L, int64_t count, const int64_t* slots,
                           const int64_t* ancs, const double* states);

/* importance sampling (importance.jl:20-52) on the first step of a model */
int orc_importance_sampling(int family, int d, int dy, int k, int v, const double* params,
                            int64_t n_params, const double* obs, int has_obs, int proposal,
                            int64_t n, uint64_t seed, double* log_norm_weights, double* states,
                            double* lml);

/* particle-marginal MH (config C5): chains [chain0, chain0 + n_chains) of the
   Kitagawa PMMH of examples/pmmh/example.jl:20-79 over pf.jl:14-73 */
int orc_pmmh_run(int64_t chain0, int64_t n_chains, int n_inner, const double* ys, int T, int n_iters,
                 int iter0, uint64_t seed, int init, double* lvx, double* lvy, double* lml, int32_t* accepts,
                 double* hist);

/* reversible-jump MH on the coal change-point model (config C3,
   examples/coal/coal.jl:47-62, :103-336): chains [chain0, chain0 + n_chains);
   state rows of 68 doubles (k, score, cp[32], h[33], pad; unused fields 0) */
int orc_coal_run(int64_t chain0, int64_t n_chains, const double* events, int E, int n_iters, int iter0,
                 uint64_t seed, int init, double* state, int32_t* accepts, int32_t* khist, int simple);
double orc_coal_regen_k(const double* row, const double* ev, int E, const double* u, double* out);
/* the score of a row from scratch, and one move's proposal (move 0 rate, 1
   position, 2 birth, 3 death) from explicit uniforms u[3]: returns the MH
   log acceptance ratio, writes the proposed row (tests/test_coal_pins.py) */
double orc_coal_score(const double* row, const double* events, int E);
double orc_coal_propose(const double* row, const double* events, int E, int move, const double* u, double* out);
/* the inner particle filter of the PMMH (its log-ML estimate) for chain c and
   move counter u at parameters (log var_x, log var_y) */
double orc_pmmh_loglik(uint64_t seed, uint64_t chain, uint32_t u, double lvx, double lvy, int n_inner,
                       const double* ys, int T);

/* host threads the loops use: 1, or the OpenMP team size of liboracle_omp.so
   (the all-cores CPU baseline) */
int orc_num_threads(void);

/* static weight helpers used by the golden-vector tests */
double orc_normal_logpdf(double x, double mu, double std);

#ifdef __cplusplus
}
#endif
#endif
