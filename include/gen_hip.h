/* gen_hip.h — C ABI of libgen_hip.so, the MI355X particle-inference engine.
 *
 * This is the drop-in boundary for Gen's sequential-Monte-Carlo hot path.
 * The reference has no FFI: its interface is Julia multiple dispatch on
 * `ParticleFilterState{U}` and the generative-function interface (GFI).  Each
 * entry point below replaces one reference function; the Julia `ccall`
 * binding a maintainer adds is spelled out in INTEGRATION.md.
 *
 *   gh_pf_init              initialize_particle_filter   src/inference/particle_filter.jl:79-108
 *   gh_pf_step              particle_filter_step!        src/inference/particle_filter.jl:139-180
 *   gh_pf_maybe_resample    maybe_resample!              src/inference/particle_filter.jl:189-213
 *   gh_pf_log_ml_estimate   log_ml_estimate              src/inference/particle_filter.jl:52-55
 *   gh_pf_get_log_weights   get_log_weights              src/inference/particle_filter.jl:43-45
 *   gh_pf_get_states /
 *   gh_pf_get_trajectory    get_traces (SoA columns)     src/inference/particle_filter.jl:31-34
 *   gh_pf_get_parents       ParticleFilterState.parents  src/inference/particle_filter.jl:23
 *   gh_pf_get_scores        get_score / per-choice scores src/static_ir/trace.jl:91-129
 *   gh_pf_sample_unweighted sample_unweighted_traces     src/inference/particle_filter.jl:62-70
 *   gh_pf_rejuvenate        mh(trace, select(x_t)) on    src/inference/mh.jl:14-26 (applied per
 *                           every particle               particle, as callers of the PF do)
 *   gh_pf_mh_select         mh(trace, selection) on      src/inference/mh.jl:14-28,
 *                           every particle               examples/regression/quickstart.jl:17-22
 *   gh_pf_mh_drift          mh(trace, drift, (sd,)) on   src/inference/mh.jl:41-62 (proposal form)
 *                           every particle
 *   gh_pf_init_conditional /
 *   gh_pf_step_conditional  conditional_smc              examples/pmmh/smc.jl:100-151
 *   gh_is_run               importance_sampling          src/inference/importance.jl:20-52
 *   gh_pmmh_run             PMMH (mh over a PF-estimated  examples/pmmh/example.jl:20-79,
 *                           likelihood)                   examples/pmmh/pf.jl:14-73
 *   gh_coal_run             involutive (RJ) MH chains     examples/coal/coal.jl:126-336,
 *                                                         src/inference/mh.jl:85-98
 *   gh_simulate             simulate(model, (T,)) for N  src/static_ir/simulate.jl:23-34,50-83,
 *                           traces                       src/modeling_library/unfold/simulate.jl
 *   gh_dist_logpdf /        logpdf / random of the       src/modeling_library/modeling_library.jl:15-41,
 *   gh_dist_random          distribution library         src/modeling_library/distributions/ (all files)
 *   gh_model_create         a Static-DSL model + Unfold  src/static_ir/, src/modeling_library/unfold/
 *
 * Conventions
 *  - Every function returns an int status (GH_OK = 0); the message of the
 *    last failure on this thread is gh_last_error().  Julia's `error(...)`
 *    sites map to status codes (see gh_status).
 *  - Handles are opaque; the library owns all device memory.  Host inputs are
 *    copied at call time, outputs are written into caller-allocated buffers.
 *  - Particle indices are 0-based (Julia's are 1-based).
 *  - A gh_pf is driven by one host thread (as the reference's mutable state is);
 *    distinct handles may run concurrently on distinct streams.  The resample
 *    kernels synchronise their whole grid (sized to the co-resident capacity of
 *    an idle device, no cooperative launch: it costs ~16 us per step), so they
 *    assume no other kernel occupies the GPU while they run.  If blocks are
 *    not co-resident the bounded barrier wait expires, the kernel writes
 *    nothing and the next synchronising call returns GH_E_STATE.
 *  - Multi-GPU: one process per GPU.  Create the context with
 *    gh_ctx_create_dist(); particles [rank*n/world, (rank+1)*n/world) live on
 *    each rank and every gh_pf_* call is collective over the ranks.
 */
#ifndef GEN_HIP_H
#define GEN_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  GH_OK = 0,
  GH_E_INVAL = 1,    /* bad argument (cf. unfold.jl:57-61 negative length, vector.jl:110) */
  GH_E_DISCARD = 2,  /* a constraint hit an existing choice inside a PF step (particle_filter.jl:168-170) */
  GH_E_NUMERIC = 3,  /* all log-weights -Inf / NaN (Categorical with NaN probabilities) */
  GH_E_NOMEM = 4,
  GH_E_HIP = 5,
  GH_E_RCCL = 6,
  GH_E_STATE = 7     /* call out of order (e.g. step before init); resample grid barrier timed out */
} gh_status;

typedef enum {
  /* x_1 ~ mvnormal(mu0, P0); x_t ~ mvnormal(A x_{t-1} + b, Q); y_t ~ mvnormal(H x_t + c, R)
     params (row-major doubles): A[d*d] b[d] Q[d*d] H[dy*d] c[dy] R[dy*dy] mu0[d] P0[d*d]
     supported d: 1..16; dy <= 32.  Multi-rank filters use systematic resampling. */
  GH_FAMILY_LGSSM = 1,
  /* categorical HMM (test/inference/particle_filter.jl:50-78):
     z_1 ~ categorical(prior); z_t ~ categorical(T[:, z_{t-1}]); x_t ~ categorical(E[:, z_t])
     params: prior[k] T[k*k] (T[new*k + prev]) E[v*k] (E[x*k + z]); k <= 64 */
  GH_FAMILY_HMM = 2,
  /* nonlinear "Kitagawa" SSM (examples/pmmh/model.jl:9-13,40-46):
     x_1 ~ normal(mu1, s1); x_t ~ normal(x/2 + 25x/(1+x^2) + 8cos(1.2t), sqrt(var_x));
     y_t ~ normal(x_t^2/20, sqrt(var_y));  params: mu1 s1 var_x var_y */
  GH_FAMILY_KITAGAWA = 3,
  /* Bayesian linear regression (examples/regression/quickstart.jl:3-9), a static
     model (generate / importance sampling / rejuvenation; no steps):
     slope ~ normal(mu_s, sd_s); intercept ~ normal(mu_i, sd_i);
     y_i ~ normal(slope x_i + intercept, sigma), i = 1..dy (dy <= 32 data points)
     params: mu_s sd_s mu_i sd_i sigma x[dy]; the observation is y[dy];
     state (d = 2) = (slope, intercept) */
  GH_FAMILY_REGRESSION = 4,
  /* slot-described Unfold kernel (Static-DSL models other than the four
     above, static_ir/generate.jl:24-43): one latent address and K = 1..4
     observed addresses ("slots") per step, any subset of which a step
     constrains (gh_obs.slot / .next).  d (latent dimension) 1..16.
       params = [lat, K, (dist_k, m_k, link_k) for k < K, latent block, slot blocks]
     latent block, lat = GH_SLOT_LAT_AFFINE (0):   A[d*d] b[d] Q[d*d] mu0[d] P0[d*d]
         x_1 ~ mvnormal(mu0, P0); x_t ~ mvnormal(A x_{t-1} + b, Q)
                   lat = GH_SLOT_LAT_AFFINE_INPUT (2): the same block, and
         x_t ~ mvnormal(A x_{t-1} + (b + u_t), Q) with u_t the step's input (a
         gh_obs entry with slot GH_SLOT_INPUT and d values; zero when a step
         gives none): the Unfold's kernel arguments extended by one value per
         step, new_args = (t, u_t) (no re-scoring: earlier steps keep theirs);
         simulate(model, (T, U)) is gh_simulate_inputs (gh_simulate refuses)
                   lat = GH_SLOT_LAT_KITAGAWA (1), d = 1: mu1 s1 sd_x
         x_1 ~ normal(mu1, s1); x_t ~ normal(x/2 + 25x/(1+x^2) + 8cos(1.2t), sd_x)
                   lat = GH_SLOT_LAT_CATEGORICAL (3), d = K classes (2..16): prior[K] T[K*K]
         z_1 ~ categorical(prior); z_t ~ categorical(T[:, z_{t-1}]) (T[new*K + prev]);
         the state is stored one-hot (K values), so a slot's affine mean h.x + c
         is h[z] + c (per-class parameters); no drift MH, no linear proposal
                   lat = GH_SLOT_LAT_SWITCHING (4), two latent addresses, d = dx + nz:
         nz (2..8) prior[nz] T[nz*nz], per regime A_z[dx*dx] b_z[dx] Q_z[dx*dx], mu0[dx] P0[dx*dx]
         z_1 ~ categorical(prior), x_1 ~ mvnormal(mu0, P0); z_t ~ categorical(T[:, z_{t-1}]),
         x_t ~ mvnormal(A_z x_{t-1} + b_z, Q_z) with z = z_t; the state is x (dx values) then
         z one-hot (nz values), so a slot's h.x + c loads x and adds h[dx + z];
         no drift MH, no linear proposal, MH selections name both addresses
     slot blocks (m_k values of the slot; its value rows in simulate's output
     follow slot order, one row for a scalar slot):
       GH_SLOT_MVNORMAL, link GH_LINK_AFFINE, m <= 32: H[m*d] c[m] R[m*m]   y ~ mvnormal(H x + c, R)
       GH_SLOT_NORMAL, m = 1, GH_LINK_AFFINE: h[d] c sd                     y ~ normal(h.x + c, sd)
                              GH_LINK_KITAGAWA (d = 1): sd                  y ~ normal(x^2/20, sd)
                              GH_LINK_LOGSCALE: h[d] c g[d] s   y ~ normal(h.x + c, exp(g.x + s))
         (a log-linear standard deviation: the stochastic-volatility emission
         y_t ~ normal(0, exp(x_t / 2)) is h = 0, c = 0, g = 1/2, s = 0)
       GH_SLOT_POISSON, m = 1, GH_LINK_EXP: h[d] c                         y ~ poisson(exp(h.x + c))
       GH_SLOT_BERNOULLI, m = 1, GH_LINK_LOGISTIC: h[d] c   y ~ bernoulli(1 / (1 + exp(-(h.x + c)))) (0 / 1)
       GH_SLOT_CATEGORICAL, m = classes 2..16, GH_LINK_SOFTMAX: W[m*d] c[m]
                                     y ~ categorical(softmax(W x + c)), 0-based class
       GH_SLOT_LIBRARY, m = a scalar distribution of Gen's library by its
         gh_dist_desc id (GH_DIST_NORMAL, _UNIFORM_CONTINUOUS, _UNIFORM_DISCRETE,
         _BERNOULLI, _GAMMA, _INV_GAMMA, _BETA, _EXPONENTIAL, _POISSON, _BINOMIAL,
         _NEG_BINOMIAL, _GEOMETRIC, _LAPLACE, _CAUCHY, _BETA_UNIFORM), link 0:
         per argument (Gen's order) link_j h_j[d] c_j, the argument being
         link_j(h_j.x + c_j) with link_j GH_ARG_IDENTITY, GH_ARG_EXP or
         GH_ARG_LOGISTIC; y ~ dist(args...) scored by the library's logpdf
         (gh_dist_logpdf's formulas) and drawn by its sampler in simulate
     Optional trailing block, dependencies between a step's observed addresses:
       nd, then nd triples (child k, parent j < k, g): the child's linear
       predictor (a normal slot's affine mean, a poisson / bernoulli slot's
       h.x + c, a library slot's first argument) adds the fma chain of g * y_j
       over its parents in slot order; parents are scalar slots; a step that
       constrains a child constrains its parents (else GH_E_INVAL); simulate
       draws the parents first.
     At most 32 observed values per step (a poisson slot counts 2).  An LGSSM
     or Kitagawa model written as slots filters bit for bit as its family does
     (those stay the fast paths); the default proposal or GH_PROPOSAL_LINEAR
     (d + observed values <= 32); gh_pf_step_params takes a new slot model
     with the same latent form and slot layout (only the numbers change). */
  GH_FAMILY_SLOTS = 5
} gh_family;

enum { GH_SLOT_LAT_AFFINE = 0, GH_SLOT_LAT_KITAGAWA = 1, GH_SLOT_LAT_AFFINE_INPUT = 2, GH_SLOT_LAT_CATEGORICAL = 3,
       GH_SLOT_LAT_SWITCHING = 4 };
/* gh_obs.slot of a step's latent input u_t (latent form 2): d values, an
   argument of the step's kernel application, not a choice */
enum { GH_SLOT_INPUT = -1 };
enum { GH_SLOT_MVNORMAL = 1, GH_SLOT_NORMAL = 2, GH_SLOT_POISSON = 3, GH_SLOT_BERNOULLI = 4, GH_SLOT_CATEGORICAL = 5,
       GH_SLOT_LIBRARY = 6 };
enum { GH_ARG_IDENTITY = 0, GH_ARG_EXP = 2, GH_ARG_LOGISTIC = 3 };  /* a library slot's argument links */
enum { GH_LINK_AFFINE = 0, GH_LINK_KITAGAWA = 1, GH_LINK_EXP = 2, GH_LINK_LOGISTIC = 3, GH_LINK_SOFTMAX = 4,
       GH_LINK_LOGSCALE = 5 };

typedef enum { GH_RESAMPLE_SYSTEMATIC = 0, GH_RESAMPLE_MULTINOMIAL = 1 } gh_resampler;

typedef enum {
  GH_PROPOSAL_DEFAULT = 0, /* the model's internal proposal (prior) */
  GH_PROPOSAL_OPTIMAL = 1, /* locally optimal proposal p(x_t | x_{t-1}, y_t) as a custom
                              proposal (particle_filter.jl:79-91,139-154): HMM (the proposal
                              of test/inference/particle_filter.jl:104-127) and LGSSM
                              (Gaussian, d + dy <= 32); weight log p(y_t | x_{t-1}) */
  GH_PROPOSAL_GAUSSIAN = 2 /* user-parameterised custom proposal of the nonlinear SSM
                              (particle_filter.jl:79-91,139-154 via trace_translators.jl:
                              775-802): x_t ~ normal(alpha m + beta y_t + gamma, sigma_q),
                              m the prior mean; proposal_args = (alpha, beta, gamma, sigma_q)
                              through gh_pf_init_q / gh_pf_step_q; weight log p(x_t|x_{t-1})
                              + log p(y_t|x_t) - log q(x_t) */,
  GH_PROPOSAL_LINEAR = 3  /* user-parameterised custom proposal of the LGSSM and of slot models (the same
                              translator): x_t ~ mvnormal(P x_{t-1} + u_t, Sigma_q) (t = 1:
                              mvnormal(u_1, Sigma_q)); proposal_args = P[d*d] Sigma_q[d*d] u[d]
                              (required at gh_pf_init_q), or u[d] alone to keep P and Sigma_q
                              (none: keep u too); d + dy <= 32; weight log p(x_t|x_{t-1})
                              + log p(y_t|x_t) - log q(x_t) */
} gh_proposal;

typedef struct gh_ctx gh_ctx;
typedef struct gh_model gh_model;
typedef struct gh_pf gh_pf;

typedef struct {
  int32_t family; /* gh_family */
  int32_t d;      /* latent dimension (LGSSM) */
  int32_t dy;     /* observation dimension (LGSSM) */
  int32_t k;      /* number of hidden states (HMM) */
  int32_t v;      /* number of observation symbols (HMM) */
  const double* params;
  int64_t n_params;
} gh_model_desc;

/* The observations of one step: the value(s) at address :chain => t => :y.
   values == NULL or present == 0 means "no observation at this step".
   GH_FAMILY_SLOTS: `slot` names the observed address (0..K-1) and `next`
   chains the step's other constrained addresses (NULL ends the chain; a
   slot constrained twice is GH_E_DISCARD); an entry with slot
   GH_SLOT_INPUT (-1) carries the step's latent input u_t (latent form 2, d
   values, at most one per step); the other families take slot 0 and no
   chain. */
typedef struct gh_obs {
  const double* values;
  int32_t n_values;
  int32_t present;
  int32_t slot;
  int32_t reserved;
  const struct gh_obs* next;
} gh_obs;

typedef struct {
  int32_t resampler;      /* gh_resampler */
  int32_t record_history; /* 1: keep every step's states + genealogy (Gen trace semantics) */
  int32_t history_capacity; /* steps to preallocate when record_history (0 = grow) */
  int32_t block_size;     /* 0 = default (256) */
  int32_t time_kernels;   /* k > 0: time every k-th step kernel with hipEvents (gh_pf_kernel_time) */
  int32_t reserved[3];
} gh_pf_opts;

/* ---- context ------------------------------------------------------------ */
int gh_ctx_create(int device, void* hip_stream /* NULL = own stream */, gh_ctx** out);
int gh_comm_unique_id(uint8_t id[128]);
int gh_ctx_create_dist(int device, int rank, int world, const uint8_t id[128], void* hip_stream,
                       gh_ctx** out);
/* Host-staged transport (e.g. several ranks sharing one GPU, or a cluster
   without RCCL peer access): the library stages device buffers through host
   memory and calls these functions, which move host buffers between ranks.
   Return 0 on success. */
typedef struct {
  void* user;
  /* every rank contributes `bytes`; recv receives world*bytes in rank order */
  int (*allgather)(void* user, const void* send, void* recv, uint64_t bytes);
  /* point-to-point exchange: the calls of all ranks match pairwise */
  int (*sendrecv)(void* user, int n_send, const int* send_peers, const void* const* send_bufs,
                  const uint64_t* send_bytes, int n_recv, const int* recv_peers, void* const* recv_bufs,
                  const uint64_t* recv_bytes);
} gh_host_comm;
int gh_ctx_create_hostcomm(int device, int rank, int world, const gh_host_comm* comm, void* hip_stream,
                           gh_ctx** out);
/* Peer transport: the ranks' kernels exchange through device memory they map
   from each other (a fine-grained mailbox per rank, and every filter's
   received-row buffer), with tagged words and bounded polls — no collective
   call and no host round trip on the step path.  The bootstrap's allgather
   (host buffers) swaps the IPC handles once, at context and filter creation
   (both collective over the ranks, and fail-together: a rank that fails its
   part makes every rank's call return an error, none is left waiting), and
   fences the ranks at gh_ctx_destroy and at gh_pf_destroy of a multi-rank
   filter — on this transport both destroys are COLLECTIVE: every rank calls
   them, in the same order.  Ranks on one GPU (processes sharing a device) or
   on GPUs that map each other's memory (xGMI peers of one node).
   world <= 64.  Systematic resampling moves its rows inside the fused
   kernels; the other forms (multinomial, conditional SMC, the generic
   exchange) move theirs through the bootstrap's sendrecv when it is given
   (GH_E_STATE without it).  Every device wait on another rank is bounded
   in time (gh_ctx_set_peer_timeout, 30 s by default): a rank that stops
   posting makes the others' waits end in GH_E_STATE ("peer transport: ...");
   a slow one is waited for. */
int gh_ctx_create_peer(int device, int rank, int world, const gh_host_comm* bootstrap, void* hip_stream,
                       gh_ctx** out);
/* the bound of every device wait on another rank (peer transport; later
   launches), seconds in (0, 86400]; no effect on the other transports */
int gh_ctx_set_peer_timeout(gh_ctx* ctx, double seconds);
int gh_ctx_destroy(gh_ctx* ctx);
/* Debug / timing: filters created on this context afterwards take the
   multi-rank code path (collectives, split step after a resample, k_rank_a/b)
   even at world 1 — over a one-rank RCCL communicator for a gh_ctx_create /
   gh_ctx_create_dist context, over the user's functions for a host-comm one.
   Results are the same filter's (bit-exact against the one-rank path).
   GH_E_STATE while a filter exists on the context (its buffers were
   allocated for the path chosen when it was created). */
int gh_ctx_force_multirank(gh_ctx* ctx);
int gh_ctx_rank(const gh_ctx* ctx, int* rank, int* world);
int gh_ctx_stream(const gh_ctx* ctx, void** hip_stream);
int gh_ctx_synchronize(gh_ctx* ctx);

/* ---- models --------------------------------------------------------------- */
int gh_model_create(gh_ctx* ctx, const gh_model_desc* desc, gh_model** out);
int gh_model_destroy(gh_model* m);
int gh_model_state_dim(const gh_model* m, int* d);
/* simulate(model, (T,)) n times (static_ir/simulate.jl:23-34: every choice
   sampled from its distribution, score += logpdf of the sampled value; the
   Unfold runs its kernel T times).  Trace i draws from (seed, i, t, simulate
   stream), independent of n.  Outputs (host, each nullable, time-major):
     xs[t-1][k][i]        latent component k of :chain => t => :x (regression: slope, intercept)
     ys[t-1][r][i]        observation component r of :chain => t => :y (HMM: the symbol;
                          regression: y-(r+1)); r < dy (1 for HMM and Kitagawa)
     per_step[t-1][0|1][i] the latent's / the observation's score
     total[i]             get_score(trace i), the scores summed in time order
   The regression model takes T = 1. */
int gh_simulate(gh_model* m, int T, int64_t n, uint64_t seed, double* xs, double* ys, double* per_step,
                double* total);
/* simulate(model, (T, U)) for a slot model with per-step inputs (latent form
   2; gh_simulate refuses one): inputs[T*d], row t-1 the input u_t of step t
   (row 0 unused); outputs as gh_simulate. */
int gh_simulate_inputs(gh_model* m, int T, int64_t n, uint64_t seed, const double* inputs, double* xs, double* ys,
                       double* per_step, double* total);

/* ---- distributions ----------------------------------------------------------- */
/* Gen's distribution library (src/modeling_library/distributions/), batched:
   n values, one parameter row shared by all (param_stride 0) or one row per
   value (param_stride = n_params).  Parameter rows, in Gen's argument order:
     NORMAL mu std | BROADCASTED_NORMAL mu[dim] std[dim] | MVNORMAL mu[dim] cov[dim*dim]
     UNIFORM_CONTINUOUS low high | UNIFORM_DISCRETE low high | BERNOULLI prob
     CATEGORICAL probs[K] (K = n_params) | GAMMA shape scale | INV_GAMMA shape scale
     BETA alpha beta | EXPONENTIAL rate | POISSON lambda | BINOMIAL n p
     NEG_BINOMIAL r p | GEOMETRIC p | LAPLACE loc scale | CAUCHY x0 gamma
     PIECEWISE_UNIFORM bounds[K+1] probs[K] | BETA_UNIFORM theta alpha beta
   Values are doubles, component-major [dim][n] for the vector distributions;
   integer values are stored exactly, bernoulli is 0/1, categorical is 1-based
   (as Gen's).  random(): value i draws from the Philox stream keyed
   (seed, i), independent of n.  The *_dev forms take device x / out and
   enqueue on the context's stream (params_on_device: params is a device
   pointer; not for MVNORMAL, whose Cholesky factor is taken on the host). */
typedef enum {
  GH_DIST_NORMAL = 1, GH_DIST_BROADCASTED_NORMAL = 2, GH_DIST_MVNORMAL = 3, GH_DIST_UNIFORM_CONTINUOUS = 4,
  GH_DIST_UNIFORM_DISCRETE = 5, GH_DIST_BERNOULLI = 6, GH_DIST_CATEGORICAL = 7, GH_DIST_GAMMA = 8,
  GH_DIST_INV_GAMMA = 9, GH_DIST_BETA = 10, GH_DIST_EXPONENTIAL = 11, GH_DIST_POISSON = 12, GH_DIST_BINOMIAL = 13,
  GH_DIST_NEG_BINOMIAL = 14, GH_DIST_GEOMETRIC = 15, GH_DIST_LAPLACE = 16, GH_DIST_CAUCHY = 17,
  GH_DIST_PIECEWISE_UNIFORM = 18, GH_DIST_BETA_UNIFORM = 19
} gh_dist;

typedef struct {
  int32_t dist;             /* gh_dist */
  int32_t dim;              /* value components (BROADCASTED_NORMAL, MVNORMAL); else 1 */
  int32_t n_params;         /* doubles per parameter row */
  int32_t param_stride;     /* 0: one shared row; n_params: row i for value i */
  int32_t params_on_device; /* *_dev forms: params is a device pointer */
  int32_t reserved;
  const double* params;
} gh_dist_desc;

int gh_dist_logpdf(gh_ctx* ctx, const gh_dist_desc* d, int64_t n, const double* x /* [dim][n] */,
                   double* out /* [n] */);
int gh_dist_random(gh_ctx* ctx, const gh_dist_desc* d, int64_t n, uint64_t seed, double* out /* [dim][n] */);
int gh_dist_logpdf_dev(gh_ctx* ctx, const gh_dist_desc* d, int64_t n, const double* x, double* out);
int gh_dist_random_dev(gh_ctx* ctx, const gh_dist_desc* d, int64_t n, uint64_t seed, double* out);

/* ---- particle filter -------------------------------------------------------- */
void gh_pf_opts_default(gh_pf_opts* o);
int gh_pf_init(gh_model* m, const gh_obs* obs, int proposal, int64_t n_particles, uint64_t seed,
               const gh_pf_opts* opts, gh_pf** out);
int gh_pf_destroy(gh_pf* pf);  /* collective for a multi-rank filter on the peer transport */
int gh_pf_step(gh_pf* pf, const gh_obs* obs, int proposal);
/* initialize_particle_filter(model, args, obs, proposal, proposal_args, N) and
   particle_filter_step!(state, args, argdiffs, obs, proposal, proposal_args)
   (particle_filter.jl:79-91, 139-154) for proposals with arguments
   (GH_PROPOSAL_GAUSSIAN: 4 doubles).  The arguments are kept: gh_pf_step and
   gh_pf_run reuse the last ones given. */
int gh_pf_init_q(gh_model* m, const gh_obs* obs, int proposal, const double* proposal_args, int n_proposal_args,
                 int64_t n_particles, uint64_t seed, const gh_pf_opts* opts, gh_pf** out);
int gh_pf_step_q(gh_pf* pf, const gh_obs* obs, int proposal, const double* proposal_args, int n_proposal_args);
/* particle_filter_step!(state, (t, params'...), (UnknownChange(), UnknownChange()...),
   observations) (particle_filter.jl:162-180) with the Unfold's parameters
   changed to those of new_model (same family and dimensions, same context):
   the Unfold's update re-visits every retained kernel application
   (unfold/generic_update.jl:9-16), so every particle's weight gains its
   trajectory's score under the new parameters minus under the old ones, and
   the new step is generated under the new parameters, which the filter keeps
   from then on (new_model must outlive it).  record_history; on R ranks
   every rank calls it (the re-scoring walks the genealogy across ranks). */
int gh_pf_step_params(gh_pf* pf, const gh_obs* obs, int proposal, gh_model* new_model);
/* The same for a conditional filter (gh_pf_init_conditional): the re-scoring,
   then the conditional step of gh_pf_step_conditional with the distinguished
   particle pinned to ref_xt[d] (particle Gibbs with a parameter move between
   sweeps, examples/pmmh/smc.jl:138-147).  The reference's Unfold update KAT
   with changed parameters (test/modeling_library/unfold.jl:303-326) is driven
   through this entry: tests/test_step_params.py. */
int gh_pf_step_params_conditional(gh_pf* pf, const gh_obs* obs, gh_model* new_model, const double* ref_xt);
/* ess_threshold NaN means the reference's default N/2; any other value >= 0 is
   the threshold as given (resample iff ESS < ess_threshold, so 0 never
   resamples, as in Gen); a negative threshold is GH_E_INVAL (before round 3,
   values <= 0 selected N/2).  If did_resample/ess are non-NULL the
   call synchronises and reports them; otherwise the decision stays on the
   device and the call is asynchronous. */
int gh_pf_maybe_resample(gh_pf* pf, double ess_threshold, int* did_resample, double* ess);
/* run {maybe_resample!; particle_filter_step!} for n_steps consecutive steps
   (the reference caller loop, test/inference/particle_filter.jl:157-162),
   observations obs[0..n_steps-1]; no host synchronisation inside. */
int gh_pf_run(gh_pf* pf, int n_steps, const gh_obs* obs, int proposal, double ess_threshold);
int gh_pf_log_ml_estimate(gh_pf* pf, double* out);
int gh_pf_num_particles(const gh_pf* pf, int64_t* n_global, int64_t* n_local, int64_t* first);
int gh_pf_num_steps(const gh_pf* pf, int* t);
int gh_pf_get_log_weights(gh_pf* pf, double* host_out /* n_local */);
int gh_pf_get_states(gh_pf* pf, double* host_out /* [d][n_local] current latent */);
int gh_pf_get_parents(gh_pf* pf, int64_t* host_out /* n_local, global ids */);
/* latent of step t (1-based) of the current particles' traces: follows the
   genealogy back from the current step (record_history required) */
int gh_pf_get_trajectory(gh_pf* pf, int t, double* host_out /* [d][n_local] */);
/* The score columns of the current particles' traces (the per-choice score
   fields of static_ir/trace.jl:91-129): total[i] = get_score(trace i), and
   (nullable) per_step[t-1][0][i] / per_step[t-1][1][i] = the scores of the
   latent :chain => t => :x and the observation :chain => t => :y (0 when not
   observed) — the model's densities, whatever proposal made the particles.
   Computed on the device from the history (record_history, one rank). */
int gh_pf_get_scores(gh_pf* pf, double* total /* [n_local] */, double* per_step /* [t][2][n_local] */);
int gh_pf_sample_unweighted(gh_pf* pf, int64_t n_samples, uint64_t seed, int64_t* host_idx);
/* Rejuvenation: n_moves MH moves on every particle, each regenerating the
   current latent x_t from its prior given x_{t-1} (x_1 from the initial
   distribution) and accepting with log(rand()) < log p(y_t|x'_t) - log p(y_t|x_t).
   Log weights are unchanged.  Call after gh_pf_init / gh_pf_step and before
   gh_pf_maybe_resample (GH_E_STATE otherwise); at most 2^24 moves per step.
   *accepted (optional, synchronises) = accepted moves summed over the local
   particles. */
int gh_pf_rejuvenate(gh_pf* pf, int n_moves, int64_t* accepted);
/* metropolis_hastings(trace, selection) on every particle (src/inference/mh.jl:14-28,
   the selection form): regenerate the selected latent addresses of the current
   step from their prior, accept with log(rand()) < the regenerate weight.
   selection is a bit mask over the step's latent addresses: the Unfold families
   have one (bit 0: :chain => t => :x, the same move as gh_pf_rejuvenate); the
   regression has two (bit 0 :slope, bit 1 :intercept; quickstart.jl:17-22's
   mh(trace, select(:slope)) / mh(trace, select(:intercept))).  The moves share
   gh_pf_rejuvenate's draw windows and per-step move counter. */
int gh_pf_mh_select(gh_pf* pf, uint32_t selection, int n_moves, int64_t* accepted);
/* mh(trace, drift, (sd,)) on every particle (src/inference/mh.jl:41-62, a
   proposal generative function): the Gaussian drift proposal
   `@trace(normal(trace[a], sd), a)` on the selected latent addresses of the
   current step (bit layout as gh_pf_mh_select; the LG-SSM's vector :x drifts
   componentwise with sd[0..d), a diagonal mvnormal), accept iff log(rand()) <
   update weight - fwd score + bwd score (the symmetric drift's two scores
   cancel exactly).  sd[d]: > 0 for the selected components.  Not for the
   HMM (a discrete latent).  Same calling rules and draws as gh_pf_rejuvenate. */
int gh_pf_mh_drift(gh_pf* pf, uint32_t selection, const double* sd /* [d] */, int n_moves, int64_t* accepted);
/* Conditional SMC (examples/pmmh/smc.jl:100-151, the particle-Gibbs sweep):
   particle 0 is the distinguished particle, pinned to ref_x1 at init and to
   ref_xt at each step, its parent always itself, its weight the observation
   log-density of the given state (init_score / forward_score of the model's
   own proposal).  Requires opts->resampler == GH_RESAMPLE_MULTINOMIAL and one
   rank.  Such a filter steps only with gh_pf_step_conditional. */
int gh_pf_init_conditional(gh_model* m, const gh_obs* obs, int64_t n_particles, uint64_t seed,
                           const gh_pf_opts* opts, const double* ref_x1 /* [d] */, gh_pf** out);
int gh_pf_step_conditional(gh_pf* pf, const gh_obs* obs, const double* ref_xt /* [d] */);
/* per-step resampling record: ess and did_resample for steps 1..t */
int gh_pf_get_ess_history(gh_pf* pf, int max_steps, double* ess, int32_t* did);
/* average duration (ms) of the step kernel over the timed launches (opts.time_kernels) */
int gh_pf_kernel_time(gh_pf* pf, double* avg_ms, int64_t* n_launches, int reset);

/* multi-rank systematic resampling plan (host only, no GPU): given every
   rank's integer weight total and the shared offset o < sum(totals), the global
   slot ranges rank `rank` sends to ([send_lo[r], send_hi[r])) and receives from
   ([recv_lo[r], recv_hi[r])) each rank r; empty ranges have lo == hi.  This is
   the plan gh_pf_maybe_resample follows; exposed for tests and integrators. */
int gh_sys_plan(int64_t n_global, int world, int rank, const uint64_t* totals, uint64_t offset,
                int64_t* send_lo, int64_t* send_hi, int64_t* recv_lo, int64_t* recv_hi);
/* the grouped messages that plan becomes (host only): peers and byte counts of
   the sends and receives, rows of d + 1 doubles, in the order both transports
   post them (RCCL ncclSend/ncclRecv in one group, or gh_host_comm.sendrecv).
   Arrays hold up to world - 1 entries. */
int gh_debug_exchange_lists(int64_t n_global, int world, int rank, const uint64_t* totals, uint64_t offset, int d,
                            int* n_send, int* send_peer, uint64_t* send_bytes, int* n_recv, int* recv_peer,
                            uint64_t* recv_bytes);

/* test hook: widen the ancestor field of the filter's 32-bit range marks to
   `bits` (at least what the particle count needs, at most 31), which shortens
   the epoch field, so that a short run crosses several epoch wraps (the marks
   are cleared at each).  Only before the first resample is pending. */
int gh_debug_mark_bits(gh_pf* pf, int bits);

/* test hook: overwrite the genealogy record of step t (2 <= t <= current):
   particle j's ancestor index becomes `value` (a corrupted record, so that a
   test can check that a genealogy query reports GH_E_STATE instead of
   returning a wrong trajectory).  The filter is unusable afterwards. */
int gh_debug_set_ancestor(gh_pf* pf, int t, int64_t j, int32_t value);

/* test hook: the systematic slot counts are taken in floating point and
   recounted exactly when within a window of an integer (2^(ceil(log2 N) + 7 - 53)
   by default, so rarely); log2_inv > 0 sets the window to 2^-log2_inv for every
   later resample on the context's device, so that the exact recount runs often
   (0 restores the default).  Results do not change. */
int gh_debug_count_window(gh_ctx* ctx, int log2_inv);

/* ---- importance sampling ---------------------------------------------------- */
int gh_is_run(gh_model* m, const gh_obs* obs, int proposal, int64_t n, uint64_t seed,
              double* host_log_norm_weights /* may be NULL */, double* host_states /* may be NULL */,
              double* lml);

/* ---- particle-marginal MH (config C5) ------------------------------------------
   examples/pmmh/example.jl:20-79: log var_x, log var_y ~ normal(0, 2); the
   likelihood is the log-ML estimate of an inner particle filter with n_inner
   particles on the Kitagawa model (examples/pmmh/pf.jl:14-73); each
   iteration applies mh(select(:var_x)), mh(select(:var_y)) and the two
   random-walk moves (sd sqrt(0.5)) (src/inference/mh.jl:14-62).  One
   workgroup per chain, chains [chain0, chain0 + n_chains) (a rank's share).
   init = 1 draws the start from the prior (generate); otherwise lvx / lvy /
   lml hold the state to continue from, after iter0 iterations.  Host buffers; hist (nullable) gets
   [n_chains][n_iters][2]; accepts [n_chains][4] counts per move. */
int gh_pmmh_run(gh_ctx* ctx, int64_t chain0, int64_t n_chains, int n_inner, const double* ys, int T,
                int n_iters, int iter0, uint64_t seed, int init, double* lvx, double* lvy, double* lml, int32_t* accepts,
                double* hist, double* kernel_ms);

/* ---- reversible-jump MH on the coal change-point model (config C3) ---------------
   examples/coal/coal.jl:47-62 model, mcmc_step (:329-336) = rate_move,
   position_move (k > 0), birth_death_move, each an involutive MH step
   (src/inference/mh.jl:85-98, trace_translators.jl:848-876).  One thread per
   chain; events sorted, T = events[E-1].  state: host [n_chains][68] rows
   (k, score, cp[32], h[33], pad), written on return and read when init == 0
   (continuing after iter0 iterations).  accepts [n_chains][3]; khist
   (nullable) [n_chains][n_iters] = k after each iteration. */
int gh_coal_run(gh_ctx* ctx, int64_t chain0, int64_t n_chains, const double* events, int E, int n_iters,
                int iter0, uint64_t seed, int init, double* state, int32_t* accepts, int32_t* khist,
                double* kernel_ms);

/* Device-resident chains (the same kernel, state kept in HBM between calls:
   no per-call state upload/download).  gh_coal_step's first call draws the
   start from the prior (generate) and then runs n_iters iterations; later
   calls continue.  accepts (nullable) [n_chains][3]: this call's counts;
   khist as gh_coal_run.  gh_coal_read_state: the [n_chains][68] rows. */
typedef struct gh_coal gh_coal;
int gh_coal_create(gh_ctx* ctx, int64_t chain0, int64_t n_chains, const double* events, int E, uint64_t seed,
                   gh_coal** out);
int gh_coal_step(gh_coal* h, int n_iters, int32_t* accepts, int32_t* khist, double* kernel_ms);
/* the MCMC kernel of the following gh_coal_step calls: 0 = mcmc_step (rate,
   position, birth/death; coal.jl:329-336, the default), 1 = simple_mcmc_step
   (rate, position, then mh(trace, select(:k)) — the Dynamic DSL regenerate of
   k with the change points and rates it adds or drops; coal.jl:338-345);
   accepts[2] counts the third move's acceptances either way */
int gh_coal_set_kernel(gh_coal* h, int kernel);
int gh_coal_read_state(gh_coal* h, double* state);
/* Resume the chains from given rows ([n_chains][68], the layout of
   gh_coal_read_state: fields past k / k+1 zero); the next gh_coal_step
   continues at iteration iter0 + 1 (its draws are those of that iteration). */
int gh_coal_write_state(gh_coal* h, const double* state, int iter0);
int gh_coal_destroy(gh_coal* h);

/* ---- diagnostics ------------------------------------------------------------ */
const char* gh_last_error(void);
const char* gh_version(void);
/* device self-test: evaluates gh_exp/gh_log/sqrt/div/normals on n inputs on the
   GPU so tests can compare them bit-for-bit with the CPU oracle (out_div: the
   even entries in[i] / in[i+1], the odd ones the models' in[i] / 20) */
int gh_selftest_math(gh_ctx* ctx, int64_t n, const double* in, double* out_exp, double* out_log,
                     double* out_sqrt, double* out_div);
/* Box–Muller stages for n word triples (a, b, c): out[4i..4i+3] =
   (1 - u53(a, b), sqrt(-2 log(.)), z0, z1) as the kernels compute them */
int gh_selftest_boxmuller(gh_ctx* ctx, int64_t n, const uint32_t* words, double* out);
int gh_selftest_normals(gh_ctx* ctx, uint64_t seed, int64_t n, uint32_t step, uint32_t stream,
                        int dim, double* out /* [n][dim] */);

#ifdef __cplusplus
}
#endif
#endif
