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
constexpr int kScanItems = 4;                    // items per thread in the CDF kernels
constexpr int kScanTile = kBlock * kScanItems;   // particles per CDF block

// Wave-tiled state slots: the states of one step are stored in
// 64-particle tiles, a tile's D components one contiguous run of 64·D
// doubles: component pairs (2c, 2c+1) interleaved per particle, [D/2][64][2],
// then for odd D the last component as a plain [64] column — component k of
// particle i at xidx(i, k, D).  A lane reads or writes a component pair as one
// 16-byte word (a wave: 1 KiB contiguous).  (The column-major [D][n] layout
// put a particle's D components n·8 bytes apart — 8 MiB at 2^20 — and its
// gather+store skeleton ran 14 % slower through HBM; 8-byte words per
// component 3 % slower: tools/ubench_layout.hip.)
constexpr int kTileP = 64;
__host__ __device__ __forceinline__ int64_t tbase(int64_t i, int D) { return (i >> 6) * (int64_t)(kTileP * D); }
__host__ __device__ __forceinline__ int64_t xidx(int64_t i, int k, int D) {
  const int l = (int)(i & 63);
  return tbase(i, D) + (k < (D & ~1) ? (k >> 1) * (2 * kTileP) + 2 * l + (k & 1) : (D - 1) * kTileP + l);
}
__host__ __device__ __forceinline__ int64_t slot_doubles(int64_t n, int D) {
  return ((n + kTileP - 1) / kTileP) * (int64_t)(kTileP * D);
}

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
  double invN;         // 1 / N (division estimate, corrected exactly)
  double invS;         // 1 / S (slot-count estimate, exact unless near an integer)
  int pending;         // a resample happened since the last step
  int fire;            // the current maybe_resample decided to resample
  int spend;           // sample_unweighted: weights are all equal
  int one;             // constant 1 (gate for unconditional launches)
  int error;           // gh_status raised on the device
  unsigned ticket;     // (unused; kept for layout)
  unsigned ticket_q;
  unsigned ticket_c;
  // decision pre-evaluated by k_fold for the threshold the host expects the
  // next maybe_resample! to use (single rank); committed by k_qsum
  double cM, cL, cess;
  int cfire, cerr;
  unsigned bar_gen;    // k_resample1 / k_rank_a grid barriers completed
  int64_t ra, rb;      // multi-rank: local slots [0, ra) and [rb, n) take received rows
  unsigned fire_streak;  // k_resample1: consecutive resamples that fired (its speculation policy)
};

// DevScalars::error: a gh_status in the low byte, the cause above it (the
// host reports both: dev_error_msg in gh_api.hip)
constexpr int kErrBarrier = 7;             // GH_E_STATE: a grid barrier timed out (blocks not co-resident)
constexpr int kErrGenealogy = 7 | 1 << 8;  // GH_E_STATE: a genealogy walk met a broken record
constexpr int kErrPeer = 7 | 2 << 8;       // GH_E_STATE: another rank never published (bounded wait)

struct StepArgs {
  const double* xprev;   // wave-tiled states of the previous step (xidx)
  int32_t* anc;          // ancestors for this step (read when a resample is pending;
                         // written here when they come from the systematic marks)
  const uint32_t* mark;  // systematic range marks + per-64-slot-group carries (mark_mode):
  const uint32_t* carry; //   (epoch tag | ancestor), the ancestor in the low bits of mark_idx
  uint32_t mark_idx;
  int mark_mode;          // 1: systematic marks (one rank); 2: marks + received rows (multi-rank)
  int resampled;         // a maybe_resample! was enqueued since the last step
                         // (otherwise the device flags are stale and ignored)
  int buf;               // state slots < 4 GiB: address them by buffer descriptors
  const double* remote;  // multi-rank: rows received from other ranks, row r at
  int64_t ld_remote;     // remote[r * ld_remote] = (x_0 .. x_{D-1}, global id)
  double* xout;          // wave-tiled states of this step (xidx)
  double* logw;
  int64_t n;             // particles on this rank
  int64_t nvb;           // virtual blocks of kBlock particles (= partial count)
  int max_only;          // write block maxima only (the fused resample sums the weights)
  int64_t lo;            // global id of the first one
  uint64_t seed;
  uint32_t t;            // 1-based step index
  int proposal;
  DevScalars* dev;
  double* pm;            // block partials: max
  double* ps;            //                 sum e
  double* ps2;           //                 sum e^2
  double* stats_out;     // where the rank's (M, S, S2) goes
  uint64_t* amax;        // max_only steps of gh_pf_run: the block maximum also goes into
                         // kAmaxShards order-keyed atomic-max words (k_resample1 folds
                         // those instead of every block maximum); nullptr: not written
  // multi-rank split of a step after a resample: part 1 runs
  // every tile before the received rows exist (its results for slots [0, ra)
  // and [rb, n) are discarded), part 2 runs again the tiles holding such
  // slots, once the rows are in, and overwrites them (the draws are
  // counter-based and a resample resets the weights, so the tiles' other
  // slots get the same values again).  A part-2 launch over a later tile range
  // gets every per-slot pointer advanced by j0 slots (j0 = 0 otherwise).
  int part;              // host only: 0 one launch; 1, 2 the halves of a split step
  int64_t j0;            // slot offset of this launch (the received-row index only)
  // part 2 as ONE launch over the block ranges [0, vb_split) and
  // [vb_split + vb_skip, ...): block b >= vb_split steps block b + vb_skip
  // (vb_skip = 0: every block its own)
  int64_t vb_split, vb_skip;
  int64_t grid_blocks;   // host only: the launch's blocks when nonzero
  // part 2 (record_history): every received row used here is also kept,
  // row-indexed (D components + global id), as this step's genealogy record of
  // the parents that lived on other ranks (rows_recv is overwritten by the
  // next resample); nullptr: not kept
  double* rhist;
};

// ------------------------------------------------------------ reductions
// Wave-level reductions and scans on DPP lane moves (quad_perm, row_shr,
// row_bcast:15/31) instead of LDS-routed shuffles: each step is two
// v_mov_dpp (64-bit payload) + the operation, a few cycles instead of an LDS
// round trip.  Reductions leave the total in lane 63, read back with
// readlane.  Integer sums, maxima and scans are exact in any order; the
// floating sums only feed the statistics (log-ML / ESS), not the ancestors.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v, uint64_t old) {
  const int lo = __builtin_amdgcn_update_dpp((int)(uint32_t)old, (int)(uint32_t)v, CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(uint32_t)(old >> 32), (int)(uint32_t)(v >> 32), CTRL, ROW_MASK,
                                             0xf, false);
  return ((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo;
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_f64(double v, double old) {
  return as_f64(dpp_u64<CTRL, ROW_MASK>(as_u64(v), as_u64(old)));
}
__device__ __forceinline__ uint64_t readfirstlane_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t readlane63_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
  return ((uint64_t)hi << 32) | lo;
}

// Lane moves for reductions read at lane 63 only: lane 63's operands are
// always valid sources, so the other lanes may take garbage — a plain
// v_mov_dpp (bound_ctrl, no "old" operand) needs no register copy per step.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint64_t dpp_red_u64(uint64_t v) {
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, ROW_MASK, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, ROW_MASK, 0xf, true);
  return ((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo;
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_red_f64(double v) {
  return as_f64(dpp_red_u64<CTRL, ROW_MASK>(as_u64(v)));
}

template <class Op>
__device__ __forceinline__ double wave_reduce_f64(double v, Op op) {
  v = op(v, dpp_red_f64<0xb1>(v));         // quad_perm [1,0,3,2]
  v = op(v, dpp_red_f64<0x4e>(v));         // quad_perm [2,3,0,1]
  v = op(v, dpp_red_f64<0x114>(v));        // row_shr:4
  v = op(v, dpp_red_f64<0x118>(v));        // row_shr:8
  v = op(v, dpp_red_f64<0x142, 0xa>(v));   // row_bcast:15
  v = op(v, dpp_red_f64<0x143, 0xc>(v));   // row_bcast:31
  return as_f64(readlane63_u64(as_u64(v)));
}
__device__ __forceinline__ double wave_max(double v) {
  return wave_reduce_f64(v, [](double a, double b) { return fmax(a, b); });
}
__device__ __forceinline__ double wave_sum(double v) {
  return wave_reduce_f64(v, [](double a, double b) { return a + b; });
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  v += dpp_red_u64<0xb1>(v);
  v += dpp_red_u64<0x4e>(v);
  v += dpp_red_u64<0x114>(v);
  v += dpp_red_u64<0x118>(v);
  v += dpp_red_u64<0x142, 0xa>(v);
  v += dpp_red_u64<0x143, 0xc>(v);
  return readlane63_u64(v);
}
// inclusive scans over the 64 lanes (lane order)
// (lanes without a DPP source — shifted out of their row, or in a row outside
// ROW_MASK — keep the "old" operand 0, which adds nothing: no lane conditions)
__device__ __forceinline__ uint64_t wave_incl_sum_u64(uint64_t v) {
  v += dpp_u64<0x111>(v, 0);        // row_shr:1
  v += dpp_u64<0x112>(v, 0);        // row_shr:2
  v += dpp_u64<0x114>(v, 0);        // row_shr:4
  v += dpp_u64<0x118>(v, 0);        // row_shr:8
  v += dpp_u64<0x142, 0xa>(v, 0);   // row_bcast:15 into rows 1, 3
  v += dpp_u64<0x143, 0xc>(v, 0);   // row_bcast:31 into rows 2, 3
  return v;
}
// lanes without a DPP source (row_shr shifted out, rows outside ROW_MASK) read 0
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp0_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, false);
}
// inclusive max over the lanes (0 is the identity: no lane conditions)
__device__ __forceinline__ uint32_t wave_incl_max_u32(uint32_t v) {
  v = max(v, dpp0_u32<0x111>(v));       // row_shr:1
  v = max(v, dpp0_u32<0x112>(v));       // row_shr:2
  v = max(v, dpp0_u32<0x114>(v));       // row_shr:4
  v = max(v, dpp0_u32<0x118>(v));       // row_shr:8
  v = max(v, dpp0_u32<0x142, 0xa>(v));  // row_bcast:15 into rows 1, 3
  v = max(v, dpp0_u32<0x143, 0xc>(v));  // row_bcast:31 into rows 2, 3
  return v;
}
__device__ __forceinline__ uint64_t wave_incl_max_u64(uint64_t v) {
  const int lane = threadIdx.x & 63, rl = lane & 15;
  uint64_t t;
  t = dpp_u64<0x111>(v, 0); if (rl >= 1 && t > v) v = t;
  t = dpp_u64<0x112>(v, 0); if (rl >= 2 && t > v) v = t;
  t = dpp_u64<0x114>(v, 0); if (rl >= 4 && t > v) v = t;
  t = dpp_u64<0x118>(v, 0); if (rl >= 8 && t > v) v = t;
  t = dpp_u64<0x142>(v, 0); if ((lane & 31) >= 16 && t > v) v = t;
  t = dpp_u64<0x143>(v, 0); if (lane >= 32 && t > v) v = t;
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

// agent-scope relaxed accesses: global_load/store ... sc1 (L1 bypassed; the
// store writes through and drops the line from the XCD's L2)
template <class T>
__device__ __forceinline__ T ld_sc1(T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// system-scope accesses: the stores write through to memory, the loads
// bypass the caches (the words may be written by other processes' kernels: the peer
// transport's mailboxes and received rows)
template <class T>
__device__ __forceinline__ T ld_sys(const T* p) {
  return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <class T>
__device__ __forceinline__ void st_sys(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------- buffer accesses
// A buffer descriptor (wave-uniform, from kernel arguments) + a 32-bit
// per-lane byte offset + a uniform SGPR offset per state component: one
// offset VGPR serves all d component loads/stores of a particle instead of d
// 64-bit addresses.
typedef unsigned int gh_v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gh_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)0xffffffff, 0x00020000);
}
__device__ __forceinline__ double buf_ld_f64(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, (int)soff, 0));
}
__device__ __forceinline__ void buf_st_f64(double v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(gh_v2u, v), r, (int)voff, (int)soff, 0);
}
typedef unsigned int gh_v4u __attribute__((ext_vector_type(4)));
// a component pair (16 bytes) of the wave-tiled slots
__device__ __forceinline__ void buf_ld_f64x2(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, double* out) {
  const gh_v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0);
  out[0] = __builtin_bit_cast(double, ((uint64_t)v.y << 32) | v.x);
  out[1] = __builtin_bit_cast(double, ((uint64_t)v.w << 32) | v.z);
}
__device__ __forceinline__ void buf_st_f64x2(const double* in, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  const uint64_t a = __builtin_bit_cast(uint64_t, in[0]), b = __builtin_bit_cast(uint64_t, in[1]);
  const gh_v4u v = {(unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)voff, (int)soff, 0);
}

// ---------------------------------------------------------------- k_step
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// accesses (lgkmcnt) but not for its global stores, so the states a wave has
// just written drain while it computes the next tile.  (__syncthreads()'s
// release fence would emit vmcnt(0) and expose every store's latency.)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Block partial of the step kernel: the block max first (wave DPP max, then
// the 4 waves through LDS), then every lane's e = exp(lw - max) and the wave
// sums of e and e^2 — partial sums on one reference, so the 4 waves add
// without rescaling; thread 0 stores the block's triple.  Safe to call in a
// loop on the same `sm`: sm[0] is read before the second barrier, sm[1..2]
// (thread 0) before thread 0 reaches the next call's first barrier.
__device__ __forceinline__ void block_partial(double lw, double (*sm)[4], double* pm, double* ps, double* ps2) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double mw = wave_max(lw);
  if (lane == 0) sm[0][w] = mw;
  lds_barrier();
  const double mb = fmax(fmax(sm[0][0], sm[0][1]), fmax(sm[0][2], sm[0][3]));
  double e = 0.0;
  if (lw > -INFINITY) e = gh_exp_nonpos(lw - mb);
  if (lw != lw) e = lw;  // NaN poisons the statistics
  const double sw = wave_sum(e), s2w = wave_sum(e * e);
  if (lane == 0) {
    sm[1][w] = sw;
    sm[2][w] = s2w;
  }
  lds_barrier();
  if (threadIdx.x == 0) {
    *pm = mb;
    *ps = (sm[1][0] + sm[1][1]) + (sm[1][2] + sm[1][3]);
    *ps2 = (sm[2][0] + sm[2][1]) + (sm[2][2] + sm[2][3]);
  }
}

// The rank maximum of a max_only step, folded by the step kernel itself:
// every block adds its maximum to one of kAmaxShards words (128 B apart) by an
// agent-scope atomic max on an order-preserving key, so the resample reads 32
// words instead of every block's maximum (MI355X_MICROARCH.md: one address
// takes ~11-13 ns per atomic; 4096 blocks over 32 shards and a ~36 us launch
// is far below that).  NaN maxima are keyed as -inf, as fmax ignores them.
constexpr int kAmaxShards = 32;
constexpr int kAmaxStride = 16;  // u64 words between shards
constexpr uint64_t kAmaxEmpty = 0x000fffffffffffffull;  // the key of -inf
__host__ __device__ __forceinline__ uint64_t amax_key(double x) {
  const uint64_t b = x == x ? as_u64(x) : as_u64(-INFINITY);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__host__ __device__ __forceinline__ double amax_value(uint64_t k) {
  return as_f64((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k);
}

// Block maximum only (the fused resample computes the weight sums in its own
// pass over the log-weights, where it evaluates exp(w - M) anyway).
__device__ __forceinline__ void block_max_partial(double lw, double (*sm)[4], double* pm, uint64_t* amax,
                                                  int64_t vb) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double mw = wave_max(lw);
  if (lane == 0) sm[0][w] = mw;
  lds_barrier();
  if (threadIdx.x == 0) {
    const double mb = fmax(fmax(sm[0][0], sm[0][1]), fmax(sm[0][2], sm[0][3]));
    *pm = mb;
    if (amax)
      __hip_atomic_fetch_max(&amax[(vb & (kAmaxShards - 1)) * kAmaxStride], amax_key(mb), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
}

// One particle per lane, 64-particle tiles per wave, 4 waves per block, one
// 256-particle block per workgroup (straight-line code: a persistent
// grid-stride loop was measured slower — the loop-invariant parameters,
// observations and descriptors hoisted out of it spill).  Systematic ancestors
// come from the range marks by a wave-level prefix max seeded with the carry
// of the tile's 64-slot group (no block barrier).  The Box–Muller log and angle
// tables are copied into LDS once per block.  Each block writes one (max, sum e, sum e^2)
// partial with plain stores; k_resample1 / k_fold combine them in the next
// launch (a per-block ticket would serialise ~4k atomics per 1M particles at
// the memory side), and the block barrier waits for LDS only, so a block's
// state stores are not waited for before it retires.
template <class Model, bool INIT, bool SPLIT = false>
__global__ __launch_bounds__(kBlock, Model::kMinWaves) void k_step(const double* __restrict__ prm,
                                                                    typename Model::Params p0, StepObs o,
                                                                    StepArgs a) {
  constexpr int D = Model::kD;
  const typename Model::Params p = p0.rebase(prm);
  __shared__ double sm[3][4];
  __shared__ double logtab[kMathTabDoubles];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // (the remap lives in its own instantiation: the compare on two kernel
  // arguments made every other launch's waves wait for them before their
  // first loads — k_step 35.6 -> 37.5 us, A/B on one box)
  const int64_t vb = SPLIT ? (int64_t)blockIdx.x + (blockIdx.x >= a.vb_split ? a.vb_skip : 0) : (int64_t)blockIdx.x;
  const int64_t tile = vb * (kBlock / 64) + w;
  const int64_t j = tile * 64 + lane;
  // The device flags and this slot's range mark + carry are loaded before the
  // table copy, so one memory round trip covers all three (the marks are
  // read whenever a resample was enqueued; they are used only if it fired).
  // (clamped indices, no per-lane branch: a value merged at a divergent join
  // would be waited for right here)
  uint32_t mv = 0, cv = 0;
  int pending = 0, fire = 0;
  if (!INIT && a.resampled) {
    pending = a.dev->pending;
    fire = a.dev->fire;
    if (a.mark_mode) {
      const int64_t last = a.n > 0 ? a.n - 1 : 0;
      mv = a.mark[j < last ? j : last];
      cv = a.carry[tile < (last >> 6) ? tile : (last >> 6)];
    }
  }
  load_math_tab256(logtab);
  lds_barrier();
  // the marks are used from here on (the compiler would otherwise compute
  // their max where they are loaded, and wait for them there)
  asm volatile("" : "+v"(mv), "+v"(cv));
  const int pend = pending | fire;
  const int use_marks = a.mark_mode && fire && !pending;
  const Draw dr_init{STREAM_INIT, 0, logtab}, dr_step{STREAM_STEP, 0, logtab};
  double lw = -INFINITY;
  if (tile * 64 < a.n) {  // wave-uniform
    int64_t src = j;
    if (use_marks) {
      const uint32_t v = wave_incl_max_u32(max(j < a.n ? mv : 0u, cv));
      src = (int64_t)(v & a.mark_idx);
      if (a.mark_mode == 2) {  // slots outside [ra, rb) take the received rows in slot order
        const int64_t ra = a.dev->ra, rb = a.dev->rb, js = a.j0 + j;
        if (js < ra) src = -1 - js;
        else if (js >= rb) src = -1 - (ra + (js - rb));
      }
      if (j < a.n) a.anc[j] = (int32_t)src;  // genealogy record
    }
    // part 1 of a split multi-rank step: slots that take a received row are
    // stepped by part 2 once the rows have landed (no read of rows_recv here)
    if (j < a.n && !(a.part == 1 && src < 0)) {
      double x[D];
      if (INIT) {
        lw = Model::init(p, o, a.seed, (uint64_t)(a.lo + j), a.proposal, x, dr_init);
      } else {
        double xp[D];
        if (pend && !use_marks) src = a.anc[j];
        // one load sequence per uniform case (no per-lane branch: values
        // defined on divergent paths make the register allocator spill).  The
        // buffer path whenever no lane of the wave takes a received row (a
        // negative ancestor: multi-rank only, and only in the waves at the
        // rank's [0, ra) / [rb, n) edges) — the general path's system-scope
        // loads cannot be if-converted, and taking it for every wave of a
        // multi-rank step cost k_step 37 -> 44 us at world 1 (round 5)
        if (a.buf && __builtin_amdgcn_ballot_w64(src < 0) == 0) {  // local rows, slots < 4 GiB: 16-byte buffer loads of component pairs
          const __amdgpu_buffer_rsrc_t rp = gh_rsrc(a.xprev);
          const uint32_t tb = ((uint32_t)src >> 6) * (uint32_t)(kTileP * D * 8), l = (uint32_t)src & 63u;
#pragma unroll
          for (int c = 0; c < D / 2; ++c) buf_ld_f64x2(rp, tb + l * 16u, (uint32_t)(c * kTileP * 16), &xp[2 * c]);
          if (D & 1) xp[D - 1] = buf_ld_f64(rp, tb + l * 8u, (uint32_t)((D - 1) * kTileP * 8));
        } else {  // general: a local tile (xidx) or a received row (stride 1)
          const bool loc = src >= 0;
#pragma unroll
          for (int k = 0; k < D; ++k)
            xp[k] = loc ? a.xprev[xidx(src, k, D)] : ld_sys(&a.remote[(-1 - src) * a.ld_remote + k]);
          if (SPLIT && !loc && a.rhist) {  // the parent's row, kept for the genealogy
            double* h = a.rhist + (-1 - src) * (int64_t)(D + 1);
#pragma unroll
            for (int k = 0; k < D; ++k) h[k] = xp[k];
            h[D] = ld_sys(&a.remote[(-1 - src) * a.ld_remote + D]);
          }
        }
        const double inc = Model::step(p, o, a.seed, (uint64_t)(a.lo + j), a.t, a.proposal, xp, x, dr_step);
        lw = (pend ? 0.0 : a.logw[j]) + inc;
      }

      if (a.buf) {
        const __amdgpu_buffer_rsrc_t ro = gh_rsrc(a.xout);
        const uint32_t tb = (uint32_t)tile * (uint32_t)(kTileP * D * 8);
#pragma unroll
        for (int c = 0; c < D / 2; ++c) buf_st_f64x2(&x[2 * c], ro, tb + (uint32_t)lane * 16u, (uint32_t)(c * kTileP * 16));
        if (D & 1) buf_st_f64(x[D - 1], ro, tb + (uint32_t)lane * 8u, (uint32_t)((D - 1) * kTileP * 8));
      } else {
#pragma unroll
        for (int k = 0; k < D; ++k) a.xout[xidx(j, k, D)] = x[k];
      }
      a.logw[j] = lw;
    }
  }
  if (a.max_only) block_max_partial(lw, sm, a.pm + vb, a.amax, vb);
  else block_partial(lw, sm, a.pm + vb, a.ps + vb, a.ps2 + vb);
}

// k_step for one-dimensional models whose particles p, p + 64 share their
// draws (Model::kPairs, KitModel): each lane steps the particle of its lane in
// two consecutive 64-particle tiles, so one counter block and one Box–Muller
// evaluation serve both; a 256-thread block covers 512 particles and writes
// one partial.  Particle offset lo a multiple of 128 (the pair mates are then
// in the same lane); values identical to k_step's.  Multi-rank (mark_mode 2,
// received rows, split steps) as k_step; a part-2 launch starts at a multiple
// of 512 slots.
__device__ __forceinline__ void block_partial2(double lw0, double lw1, double (*sm)[4], double* pm, double* ps,
                                               double* ps2) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double mw = wave_max(fmax(lw0, lw1));
  if (lane == 0) sm[0][w] = mw;
  lds_barrier();
  const double mb = fmax(fmax(sm[0][0], sm[0][1]), fmax(sm[0][2], sm[0][3]));
  double e0 = 0.0, e1 = 0.0;
  if (lw0 > -INFINITY) e0 = gh_exp_nonpos(lw0 - mb);
  if (lw1 > -INFINITY) e1 = gh_exp_nonpos(lw1 - mb);
  if (lw0 != lw0) e0 = lw0;  // NaN poisons the statistics
  if (lw1 != lw1) e1 = lw1;
  const double sw = wave_sum(e0 + e1), s2w = wave_sum(e0 * e0 + e1 * e1);
  if (lane == 0) {
    sm[1][w] = sw;
    sm[2][w] = s2w;
  }
  lds_barrier();
  if (threadIdx.x == 0) {
    *pm = mb;
    *ps = (sm[1][0] + sm[1][1]) + (sm[1][2] + sm[1][3]);
    *ps2 = (sm[2][0] + sm[2][1]) + (sm[2][2] + sm[2][3]);
  }
}

template <class Model, bool INIT, bool SPLIT = false>
__global__ __launch_bounds__(kBlock, Model::kMinWaves) void k_step_pairs(const double* __restrict__ prm,
                                                                          typename Model::Params p0, StepObs o,
                                                                          StepArgs a) {
  static_assert(Model::kD == 1 && Model::kPairs, "pair stepping: one-dimensional paired models");
  const typename Model::Params p = p0.rebase(prm);
  __shared__ double sm[3][4];
  __shared__ double logtab[kMathTabDoubles];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // (the remap lives in its own instantiation: the compare on two kernel
  // arguments made every other launch's waves wait for them before their
  // first loads — k_step 35.6 -> 37.5 us, A/B on one box)
  const int64_t vb = SPLIT ? (int64_t)blockIdx.x + (blockIdx.x >= a.vb_split ? a.vb_skip : 0) : (int64_t)blockIdx.x;
  const int64_t tile0 = (vb * (kBlock / 64) + w) * 2;
  const int64_t j0 = tile0 * 64 + lane, j1 = j0 + 64;
  uint32_t mv0 = 0, mv1 = 0, cv0 = 0, cv1 = 0;
  int pending = 0, fire = 0;
  if (!INIT && a.resampled) {
    pending = a.dev->pending;
    fire = a.dev->fire;
    if (a.mark_mode) {
      const int64_t last = a.n > 0 ? a.n - 1 : 0, lt = last >> 6;
      mv0 = a.mark[j0 < last ? j0 : last];
      mv1 = a.mark[j1 < last ? j1 : last];
      cv0 = a.carry[tile0 < lt ? tile0 : lt];
      cv1 = a.carry[tile0 + 1 < lt ? tile0 + 1 : lt];
    }
  }
  load_math_tab256(logtab);
  lds_barrier();
  asm volatile("" : "+v"(mv0), "+v"(cv0), "+v"(mv1), "+v"(cv1));
  const int pend = pending | fire;
  const int use_marks = a.mark_mode && fire && !pending;
  const Draw dr_init{STREAM_INIT, 0, logtab}, dr_step{STREAM_STEP, 0, logtab};
  double lw0 = -INFINITY, lw1 = -INFINITY;
  if (tile0 * 64 < a.n) {  // wave-uniform
    const bool has1 = j1 < a.n;
    int64_t s0 = j0, s1 = j1;
    if (use_marks) {  // both tiles: prefix max seeded with the tile's carry
      const uint32_t v0 = wave_incl_max_u32(max(j0 < a.n ? mv0 : 0u, cv0));
      const uint32_t v1 = wave_incl_max_u32(max(has1 ? mv1 : 0u, cv1));
      s0 = (int64_t)(v0 & a.mark_idx);
      s1 = (int64_t)(v1 & a.mark_idx);
      if (a.mark_mode == 2) {  // multi-rank: slots outside [ra, rb) take the received rows in slot order
        const int64_t ra = a.dev->ra, rb = a.dev->rb, js0 = a.j0 + j0, js1 = a.j0 + j1;
        if (js0 < ra) s0 = -1 - js0;
        else if (js0 >= rb) s0 = -1 - (ra + (js0 - rb));
        if (js1 < ra) s1 = -1 - js1;
        else if (js1 >= rb) s1 = -1 - (ra + (js1 - rb));
      }
      if (j0 < a.n) a.anc[j0] = (int32_t)s0;
      if (has1) a.anc[j1] = (int32_t)s1;
    }
    if (j0 < a.n) {
      const uint64_t g0 = (uint64_t)(a.lo + j0);
      double x0, x1, w0, w1;
      // part 1 of a split multi-rank step: a slot that takes a received row is
      // computed from a stand-in and not stored (part 2 steps it once the rows
      // have landed; the pair's draws do not depend on the parent)
      bool skip0 = false, skip1 = false;
      if (INIT) {
        Model::init2(p, o, a.seed, g0, &x0, &x1, &w0, &w1, dr_init);
      } else {
        if (pend && !use_marks) {
          s0 = a.anc[j0];
          s1 = has1 ? a.anc[j1] : s0;
        }
        if (!has1) s1 = s0;
        double xp0, xp1;
        // (wave-uniform: the general path only for a wave with a received row)
        if (a.remote && __builtin_amdgcn_ballot_w64(s0 < 0 || s1 < 0) != 0) {  // a negative ancestor is row -1 - s of the receive buffer
          skip0 = a.part == 1 && s0 < 0;
          skip1 = a.part == 1 && s1 < 0;
          xp0 = s0 >= 0 ? a.xprev[s0] : (skip0 ? 0.0 : ld_sys(&a.remote[(-1 - s0) * a.ld_remote]));
          xp1 = s1 >= 0 ? a.xprev[s1] : (skip1 ? 0.0 : ld_sys(&a.remote[(-1 - s1) * a.ld_remote]));
          if (SPLIT && a.rhist) {  // received parents' rows, kept for the genealogy
            if (s0 < 0) {
              a.rhist[(-1 - s0) * 2] = xp0;
              a.rhist[(-1 - s0) * 2 + 1] = ld_sys(&a.remote[(-1 - s0) * a.ld_remote + 1]);
            }
            if (has1 && s1 < 0) {
              a.rhist[(-1 - s1) * 2] = xp1;
              a.rhist[(-1 - s1) * 2 + 1] = ld_sys(&a.remote[(-1 - s1) * a.ld_remote + 1]);
            }
          }
        } else {
          xp0 = a.xprev[s0];
          xp1 = a.xprev[s1];
        }
        Model::step2(p, o, a.seed, g0, a.t, xp0, xp1, &x0, &x1, &w0, &w1, dr_step);
        w0 = (pend ? 0.0 : a.logw[j0]) + w0;
        if (has1) w1 = (pend ? 0.0 : a.logw[j1]) + w1;
      }
      if (!skip0) {
        a.xout[j0] = x0;
        a.logw[j0] = w0;
        lw0 = w0;
      }
      if (has1 && !skip1) {
        a.xout[j1] = x1;
        a.logw[j1] = w1;
        lw1 = w1;
      }
    }
  }
  if (a.max_only) block_max_partial(fmax(lw0, lw1), sm, a.pm + vb, a.amax, vb);
  else block_partial2(lw0, lw1, sm, a.pm + vb, a.ps + vb, a.ps2 + vb);
}

// The weight sums of a max-only step, recomputed when something other than
// the next maybe_resample! asks for them (log_ml_estimate, the ESS readers, a
// second maybe_resample! without a step).  Same block geometry, block maxima
// (the step kernel's pm) and reduction order as block_partial (PAIRS:
// block_partial2), so ps / ps2 are exactly what a full-partials step would
// have written.  One rank: every step writes maxima only, so a caller loop of
// maybe_resample! + particle_filter_step! runs the batched loop's kernels.
template <bool PAIRS>
__global__ __launch_bounds__(kBlock) void k_block_sums(const double* __restrict__ logw, int64_t n,
                                                        const double* __restrict__ pm, double* ps, double* ps2) {
  __shared__ double sm[2][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t vb = blockIdx.x;
  const double mb = pm[vb];
  double sw, s2w;
  if (!PAIRS) {
    const int64_t j = (vb * (kBlock / 64) + w) * 64 + lane;
    const double lw = j < n ? logw[j] : -INFINITY;
    double e = 0.0;
    if (lw > -INFINITY) e = gh_exp_nonpos(lw - mb);
    if (lw != lw) e = lw;
    sw = wave_sum(e);
    s2w = wave_sum(e * e);
  } else {
    const int64_t j0 = (vb * (kBlock / 64) + w) * 2 * 64 + lane, j1 = j0 + 64;
    const double lw0 = j0 < n ? logw[j0] : -INFINITY, lw1 = j1 < n ? logw[j1] : -INFINITY;
    double e0 = 0.0, e1 = 0.0;
    if (lw0 > -INFINITY) e0 = gh_exp_nonpos(lw0 - mb);
    if (lw1 > -INFINITY) e1 = gh_exp_nonpos(lw1 - mb);
    if (lw0 != lw0) e0 = lw0;
    if (lw1 != lw1) e1 = lw1;
    sw = wave_sum(e0 + e1);
    s2w = wave_sum(e0 * e0 + e1 * e1);
  }
  if (lane == 0) {
    sm[0][w] = sw;
    sm[1][w] = s2w;
  }
  lds_barrier();
  if (threadIdx.x == 0) {
    ps[vb] = (sm[0][0] + sm[0][1]) + (sm[0][2] + sm[0][3]);
    ps2[vb] = (sm[1][0] + sm[1][1]) + (sm[1][2] + sm[1][3]);
  }
}

// --------------------------------------------------------------- decision
// maybe_resample! (particle_filter.jl:189-201): combine the ranks' triples in
// rank order, ESS = S^2 / S2 (= exp(-logsumexp(2 lnw))), resample iff
// ESS < thr (strict).  `uniform` = every weight is 0 (a resample is pending).
struct DecideArgs {
  const double* stats_all;  // [3*R]
  int R;
  int64_t n_global;
  double log_n;      // gh_log(n_global), evaluated on the host (same function, same bits)
  double inv_n;      // 1 / n_global (division estimate, corrected exactly)
  double thr;
  double* ess_hist;  // indexed by step
  int32_t* res_hist; // res_hist[t+1]: a resample precedes step t+1
  int t;
};

struct Decision {
  double M, L, ess;
  int fire, err;
};

__device__ __forceinline__ Decision decide(const DecideArgs& d, bool uniform) {
  Decision r{};
  double M = -INFINITY;
  if (uniform) M = 0.0;
  else
    for (int q = 0; q < d.R; ++q) M = fmax(M, d.stats_all[3 * q]);
  if (!(M > -INFINITY) || M == INFINITY || M != M) {
    r.err = 3;  // GH_E_NUMERIC: the reference's Categorical would get NaN probabilities
    r.ess = NAN;
    r.M = M;
    return r;
  }
  double S = 0.0, S2 = 0.0;
  for (int q = 0; q < d.R; ++q) {
    if (uniform) {
      const double nq = (double)((d.n_global * (q + 1)) / d.R - (d.n_global * q) / d.R);
      S += nq * 1.0;
      S2 += nq * 1.0;
      continue;
    }
    if (!(d.stats_all[3 * q] > -INFINITY)) continue;
    const double e = gh_exp(d.stats_all[3 * q] - M);
    S += d.stats_all[3 * q + 1] * e;
    S2 += d.stats_all[3 * q + 2] * (e * e);
  }
  r.M = M;
  r.L = M + gh_log(S);
  r.ess = (S * S) / S2;
  r.fire = r.ess < d.thr;
  return r;
}

__device__ __forceinline__ void commit_decision(const DecideArgs& d, const Decision& r, DevScalars* dev,
                                                int pending) {
  dev->M = r.M;
  dev->L = r.L;
  dev->ess = r.ess;
  dev->fire = r.fire;
  if (r.err) dev->error = r.err;
  if (r.fire) dev->log_ml_est += r.L - d.log_n;
  if (d.ess_hist) d.ess_hist[d.t] = r.ess;
  if (d.res_hist) d.res_hist[d.t + 1] = pending | r.fire;
}

// Stand-alone decision: used for a second maybe_resample without a step in
// between (commits the first one; weights are then all 0).
static __global__ void k_decide(DecideArgs d, DevScalars* dev) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (dev->fire) {
    dev->pending = 1;
    dev->fire = 0;
  }
  const Decision r = decide(d, dev->pending != 0);
  commit_decision(d, r, dev, dev->pending);
}

// Fold the step kernel's block partials into the rank's (M, S, S2) and clear
// the resample flags the step consumed (one 1024-thread block, partial loads
// issued eight at a time).  On a single rank it also pre-evaluates the next
// maybe_resample! decision for `thr_hint` (> 0), so k_qsum's blocks need not.
static __global__ __launch_bounds__(1024) void k_fold(const double* pm, const double* ps, const double* ps2, int nb,
                                               double* stats_out, DevScalars* dev, int clear_flags,
                                               double thr_hint, int64_t n_global) {
  __shared__ double sm[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double m = -INFINITY;
  for (int b0 = threadIdx.x; b0 < nb; b0 += 1024 * 8) {
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = (b0 + 1024 * k < nb) ? pm[b0 + 1024 * k] : -INFINITY;
#pragma unroll
    for (int k = 0; k < 8; ++k) m = fmax(m, v[k]);
  }
  m = wave_max(m);
  if (lane == 0) sm[w] = m;
  __syncthreads();
  double M = -INFINITY;
  for (int k = 0; k < 16; ++k) M = fmax(M, sm[k]);
  double s = 0.0, s2 = 0.0;
  if (M > -INFINITY) {
    for (int b0 = threadIdx.x; b0 < nb; b0 += 1024 * 8) {
      double mv[8], sv[8], s2v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int b = b0 + 1024 * k;
        mv[k] = b < nb ? pm[b] : -INFINITY;
        sv[k] = b < nb ? ps[b] : 0.0;
        s2v[k] = b < nb ? ps2[b] : 0.0;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (mv[k] > -INFINITY) {
          const double f = gh_exp(mv[k] - M);
          s += sv[k] * f;
          s2 += s2v[k] * (f * f);
        }
    }
  }
  s = wave_sum(s);
  s2 = wave_sum(s2);
  __syncthreads();
  if (lane == 0) sm[w] = s;
  __syncthreads();
  double S = 0.0;
  for (int k = 0; k < 16; ++k) S += sm[k];
  __syncthreads();
  if (lane == 0) sm[w] = s2;
  __syncthreads();
  if (threadIdx.x == 0) {
    double S2 = 0.0;
    for (int k = 0; k < 16; ++k) S2 += sm[k];
    stats_out[0] = M;
    stats_out[1] = S;
    stats_out[2] = S2;
    if (clear_flags) {
      dev->pending = 0;
      dev->fire = 0;
    }
    if (thr_hint > 0.0) {
      DecideArgs d{};
      d.stats_all = stats_out;
      d.R = 1;
      d.n_global = n_global;
      d.thr = thr_hint;
      const Decision r = decide(d, false);
      dev->cM = r.M;
      dev->cL = r.L;
      dev->cess = r.ess;
      dev->cfire = r.fire;
      dev->cerr = r.err;
    }
  }
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

__device__ __forceinline__ uint64_t block_sum_u64(uint64_t s, uint64_t* sm) {
  s = wave_sum_u64(s);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = s;
  __syncthreads();
  return (sm[0] + sm[1]) + (sm[2] + sm[3]);
}


// Block-wide (256 threads) inclusive scans of one value per thread.
__device__ __forceinline__ uint64_t block_incl_sum_u64(uint64_t v, uint64_t* sm4) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_incl_sum_u64(v);
  __syncthreads();
  if (lane == 63) sm4[w] = v;
  __syncthreads();
  for (int k = 0; k < w; ++k) v += sm4[k];
  return v;
}
__device__ __forceinline__ uint64_t block_incl_max_u64(uint64_t v, uint64_t* sm4) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_incl_max_u64(v);
  __syncthreads();
  if (lane == 63) sm4[w] = v;
  __syncthreads();
  for (int k = 0; k < w; ++k) v = sm4[k] > v ? sm4[k] : v;
  return v;
}

// Last-block-done ticket (Guideline 16): the block's sc1 stores are drained
// by every storing wave, then one lane takes a ticket; returns true in the
// block that arrived last (which then reads the published values with sc1
// loads).  The last block re-arms the counter.
__device__ __forceinline__ bool last_block(unsigned* ticket, int* sm_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *sm_flag = prev == gridDim.x - 1;
  }
  __syncthreads();
  const bool last = *sm_flag != 0;
  if (last && threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return last;
}


// Integer block sums of the quantised weights.  With `fused` the launch also
// takes the maybe_resample! decision: every block evaluates it from the same
// inputs (identical result), block 0 commits it, blocks exit unless it fires.
static __global__ __launch_bounds__(kBlock) void k_qsum(const double* logw, int64_t n, GateArgs g,
                                                 uint64_t* bsum, int fused, DecideArgs d,
                                                 DevScalars* dev) {
  __shared__ uint64_t sm[4];
  __shared__ double sM;
  __shared__ int sfire;
  if (fused) {
    if (threadIdx.x == 0) {
      Decision r;
      if (fused == 2) {  // pre-evaluated by k_fold for this threshold
        r.M = dev->cM;
        r.L = dev->cL;
        r.ess = dev->cess;
        r.fire = dev->cfire;
        r.err = dev->cerr;
      } else {
        r = decide(d, false);
      }
      if (blockIdx.x == 0) commit_decision(d, r, dev, 0);
      sM = r.M;
      sfire = r.fire;
    }
    __syncthreads();
    if (!sfire) return;
  } else {
    if (!*g.gate) return;
    if (threadIdx.x == 0) sM = *g.M;
    __syncthreads();
  }
  const double M = sM;
  const int zero = fused ? 0 : *g.zero_w;
  const int64_t base = (int64_t)blockIdx.x * kScanTile;
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int64_t i = base + threadIdx.x + (int64_t)k * kBlock;
    if (i < n) s += qweight(logw, i, M, zero, g.shift);
  }
  s = block_sum_u64(s, sm);
  if (threadIdx.x == 0) bsum[blockIdx.x] = s;
}

// multi-rank: this rank's integer total (input of the all-gather)
static __global__ __launch_bounds__(kBlock) void k_rank_total(const int* gate, const uint64_t* bsum, int64_t nb,
                                                       DevScalars* dev) {
  if (!*gate) return;
  __shared__ uint64_t sm[4];
  uint64_t s = 0;
  for (int64_t b = threadIdx.x; b < nb; b += kBlock) s += bsum[b];
  s = block_sum_u64(s, sm);
  if (threadIdx.x == 0) dev->local = s;
}

// ------------------------------------------------ systematic slot ranges
// floor(num / N) for num < 2^63: double estimate, then exact correction.
__device__ __forceinline__ uint64_t udiv_n(uint64_t num, uint64_t N, double invN) {
  uint64_t q = (uint64_t)((double)num * invN);
  if (q > (1ull << 50)) return num / N;  // estimate too coarse: exact division
  int64_t r = (int64_t)(num - q * N);
  while (r < 0) { --q; r += (int64_t)N; }
  while (r >= (int64_t)N) { ++q; r -= (int64_t)N; }
  return q;
}

// 1 / x for the slot-count estimates (x >= 1): the hardware reciprocal and two
// Newton steps (within 2 ulp; sys_count's exactness argument allows far more)
// instead of the ~30-instruction IEEE division on the resample's serial path.
__device__ __forceinline__ double recip_est(double x) {
  double y = __builtin_amdgcn_rcp(x);
  double e = fma(-x, y, 1.0);
  y = fma(y, e, y);
  e = fma(-x, y, 1.0);
  return fma(y, e, y);
}

// systematic target of global slot j: floor((j S + o) / N)
__device__ __forceinline__ uint64_t sys_target(const DevScalars* dev, uint64_t N, uint64_t j) {
  return j * dev->Qs + udiv_n(j * dev->Rs + dev->o, N, dev->invN);
}

// #{ j in [0, N) : T_j < X }: the first slot whose target reaches X.
// Particle i owns the slots [count(C_{i-1}), count(C_i)).
__device__ __forceinline__ int64_t sys_count_exact(const DevScalars* dev, uint64_t N, uint64_t X) {
  if (X == 0) return 0;
  if (X >= dev->S) return (int64_t)N;
  const double est = ((double)X * (double)N - (double)dev->o) * dev->invS;  // (a start only: corrected below)
  int64_t j = est <= 0.0 ? 0 : (est >= (double)N ? (int64_t)N : (int64_t)est);
  while (j > 0 && sys_target(dev, N, (uint64_t)(j - 1)) >= X) --j;
  while (j < (int64_t)N && sys_target(dev, N, (uint64_t)j) < X) ++j;
  return j;
}

// sys_count_exact out of line, for loops that call it rarely (one copy, and
// the caller's registers are not shaped by its search loops)
__device__ __noinline__ int32_t sys_count_exact_call(const DevScalars* dev, uint32_t N, uint64_t X) {
  return (int32_t)sys_count_exact(dev, N, X);
}

// The float slot counts below are taken exactly when v lies within this
// window of an integer: 2^(ceil(log2 N) + 7 - 53) >= 128 N 2^-53, at least
// four times the worst-case error of v (8 N 2^-53 + 2^-53 for one
// evaluation, 31 N 2^-53 + 2^-53 for k_resample1's incremental counts).  So
// the exact count runs with probability ~2^-24 per count at N = 2^21 (a
// fixed 2^-16 window made it ~2^-15: a hundred exact counts per C4 resample,
// each holding its wave ~1.7 us past the others, the launch ending with them).
// (tests, gh_debug_count_window: k > 0 makes the window 2^-k, so that the
// exact counts run often)
static __device__ int g_count_window_log2 = 0;
__device__ __forceinline__ double count_window(uint64_t N) {
  const int lg = N <= 1 ? 0 : 64 - __builtin_clzll(N - 1);  // ceil(log2 N)
  const int k = g_count_window_log2;
  return as_f64((uint64_t)(k > 0 ? 1023 - k : 1023 + lg + 7 - 53) << 52);
}

// The same count from v = (X N - o) / S in floating point: count = ceil(v)
// clamped to [0, N].  With 1/S within 2 ulp (recip_est) the computed v is
// within 8 N 2^-53 + 2^-53 of the exact quotient (the error of X's and o's
// conversions, of the FMA, of 1/S and of the product), so ceil is exact
// whenever v is more than count_window(N) away from an integer; otherwise
// count exactly.
__device__ __forceinline__ int64_t sys_count(const DevScalars* dev, uint64_t N, uint64_t X) {
  if (X == 0) return 0;
  if (X >= dev->S) return (int64_t)N;
  const double v = fma((double)X, (double)N, -(double)dev->o) * dev->invS;
  const double fl = floor(v);
  const double fr = v - fl;
  const double w = count_window(N);
  if (fr > w && fr < 1.0 - w) {
    const double j = fl + 1.0;
    if (j <= 0.0) return 0;
    if (j >= (double)N) return (int64_t)N;
    return N < (1ull << 31) ? (int64_t)(int32_t)j : (int64_t)j;  // v_cvt_i32_f64 when it fits
  }
  return sys_count_exact(dev, N, X);
}

// sys_count for whole waves: the estimate and its clamps as selects, and the
// exact count (rare: count_window) behind a wave-uniform branch, so
// the marks loops run straight-line code instead of nested divergent branches
// (k_resample1's marks phase: 2.7 us of the C2 resample).  Same results.
__device__ __forceinline__ int64_t sys_count_w(const DevScalars* dev, uint64_t N, uint64_t X) {
  const double v = fma((double)X, (double)N, -(double)dev->o) * dev->invS;
  const double fl = floor(v);
  const double fr = v - fl;
  const double jd = fmin(fmax(fl + 1.0, 0.0), (double)N);
  int64_t j = N < (1ull << 31) ? (int64_t)(int32_t)jd : (int64_t)jd;
  const bool edge = X == 0 || X >= dev->S;
  j = X == 0 ? 0 : (X >= dev->S ? (int64_t)N : j);
  const double w = count_window(N);
  const bool near = !edge && !(fr > w && fr < 1.0 - w);
  if (__builtin_amdgcn_ballot_w64(near) != 0) {
    if (near) j = sys_count_exact(dev, N, X);
  }
  return j;
}

// Range marks are 32-bit words: the resample's epoch tag in the high bits and
// the ancestor (a local particle index) in the low ceil(log2 n) bits, so the
// newest epoch's words are the largest; the host clears both arrays when the
// epoch field wraps.  k_resample1's marks loop takes its slot
// counts incrementally, as 32-bit slot indices (N < 2^31, as gh_pf_init
// enforces), so its slot and group arithmetic runs on 32-bit integers.

struct MarkArgs {
  uint32_t* mark;     // [n slots] tagged ancestor at each range start
  uint32_t* cmark;    // [64-slot groups] tagged ancestor of the group's first slot
  uint32_t tag;       // this resample's epoch tag (epoch << index bits)
  int64_t n_global;
  int64_t n_groups;   // 64-slot groups (entries of cmark)
  int enabled;        // systematic single-rank path
};

struct CdfArgs {
  const uint64_t* bsum;    // integer block sums of k_qsum
  int64_t nb;              // number of them
  const uint64_t* totals;  // multi-rank: all-gathered rank totals (nullptr: one rank)
  int R, rank;
  int64_t n_global;
  uint64_t seed;
  uint32_t t;
  uint32_t stream;
};

// Every block derives what it needs from the block sums itself (no separate
// scan launch): its exclusive offset, the rank total, the global total S,
// this rank's base and the systematic constants (block 0 also stores them).
// Then it writes either the inclusive CDF C (multinomial / sampling) or, for
// systematic resampling on one rank, the range marks: particle i owns slots
// [count(C_{i-1}), count(C_i)); its range start gets a tagged mark, and every
// step-block start slot the block's particles cover gets its ancestor in cmark.
static __global__ __launch_bounds__(kBlock) void k_cdf(const double* logw, int64_t n, GateArgs g, CdfArgs ca,
                                                DevScalars* dev, uint64_t* C, MarkArgs mk) {
  if (!*g.gate) return;
  __shared__ uint64_t sm4[4];
  __shared__ DevScalars sd;       // block copy of the resample constants
  __shared__ uint64_t sboff;
  __shared__ int32_t se[kScanTile];  // slot end of each particle of the block
  __shared__ int64_t sfirst;
  // ---- prologue: offsets and constants from the block sums
  uint64_t before = 0, all = 0;
  for (int64_t b = threadIdx.x; b < ca.nb; b += kBlock) {
    const uint64_t v = ca.bsum[b];
    all += v;
    if (b < (int64_t)blockIdx.x) before += v;
  }
  before = block_sum_u64(before, sm4);
  all = block_sum_u64(all, sm4);
  if (threadIdx.x == 0) {
    uint64_t S = all, base = 0;
    if (ca.totals) {
      S = 0;
      for (int r = 0; r < ca.R; ++r) {
        if (r < ca.rank) base += ca.totals[r];
        S += ca.totals[r];
      }
    }
    sd.S = S;
    sd.base = base;
    sd.local = all;
    const u32x4 w = rng_block(ca.seed, ~0ull, ca.t, ca.stream, 0);
    sd.o = scale_u53(u53_bits(w.x, w.y), S);
    sd.Qs = S / (uint64_t)ca.n_global;
    sd.Rs = S % (uint64_t)ca.n_global;
    sd.invN = 1.0 / (double)ca.n_global;
    sd.invS = 1.0 / (double)S;
    sboff = base + before;
    if (blockIdx.x == 0) {
      dev->S = sd.S;
      dev->base = sd.base;
      dev->local = sd.local;
      dev->o = sd.o;
      dev->Qs = sd.Qs;
      dev->Rs = sd.Rs;
      dev->invN = sd.invN;
    }
  }
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
  const uint64_t incl = block_incl_sum_u64(s, sm4);  // (its barriers also publish sd)
  uint64_t run = sboff + incl - s;
  if (!mk.enabled) {
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
      run += q[k];
      if (i0 + k < n) C[i0 + k] = run;
    }
    return;
  }
  const uint64_t N = (uint64_t)mk.n_global;
  int64_t s_i = sys_count(&sd, N, run);
  if (threadIdx.x == 0) sfirst = s_i;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    run += q[k];
    const int64_t e_i = (i0 + k < n && q[k]) ? sys_count(&sd, N, run) : s_i;
    se[threadIdx.x * kScanItems + k] = (int32_t)e_i;
    if (e_i > s_i) mk.mark[s_i] = mk.tag | (uint32_t)(i0 + k);
    s_i = e_i;
  }
  __syncthreads();
  // 64-slot group starts inside [first slot, last slot end) of this particle block
  const int64_t s_lo = sfirst, s_hi = se[kScanTile - 1];
  const int64_t pbase = (int64_t)blockIdx.x * kScanTile;
  for (int64_t b = (s_lo + 63) / 64 + threadIdx.x; b * 64 < s_hi; b += kBlock) {
    const int32_t slot = (int32_t)(b * 64);
    int lo = 0, hi = kScanTile - 1;  // first particle p with se[p] > slot
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (se[mid] > slot) hi = mid;
      else lo = mid + 1;
    }
    mk.cmark[b] = mk.tag | (uint32_t)(pbase + lo);
  }
}

// systematic ancestors (materialised outside a step): wave-level prefix max
// of the slot marks seeded with the carry of the 64-slot group
static __global__ __launch_bounds__(kBlock) void k_sys_ancestors(const int* gate, const int* zero_w,
                                                          const uint32_t* mark, const uint32_t* carry,
                                                          uint32_t idx, int64_t n, const int32_t* anc_old,
                                                          int32_t* anc_out, const DevScalars* dev, int mode) {
  if (!*gate) return;
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int lane = threadIdx.x & 63;
  if ((j & ~63LL) >= n) return;  // whole wave past the end
  const uint32_t v = wave_incl_max_u32(max(j < n ? mark[j] : 0u, carry[j >> 6]));
  (void)lane;
  if (j >= n) return;
  int32_t a = (int32_t)(v & idx);
  if (mode == 2) {  // multi-rank: slots outside [ra, rb) take received rows
    if (j < dev->ra) a = (int32_t)(-1 - j);
    else if (j >= dev->rb) a = (int32_t)(-1 - (dev->ra + (j - dev->rb)));
  }
  anc_out[j] = (*zero_w && anc_old) ? anc_old[a] : a;
}

// ----------------------------------------------- fused single-rank resample
// maybe_resample! on one rank in ONE launch: every block folds
// the step kernel's partials itself and takes the (identical) decision, so no
// block waits for another to decide; if it fires, each block quantises its
// 4096-particle tile, publishes the tile's integer total and crosses one grid
// barrier; then it derives its CDF offset and the systematic constants from
// the published totals and writes the range marks (or the CDF).  The grid is
// co-resident (cooperative launch, grid <= resident capacity).
constexpr int kRsBlock = 1024;
constexpr int kRsItems = 4;
constexpr int kRsTile = kRsBlock * kRsItems;  // particles per block
constexpr int kRsPart = 4;                    // step partials per thread (nb_part <= 4096)
constexpr int kRsPoll = 8;                    // polling waves x 64 tiles: grid <= 512
#if defined(GH_SPEC_STREAK)  // A/B only
constexpr unsigned kSpecStreak = GH_SPEC_STREAK;
#else
constexpr unsigned kSpecStreak = 8;           // resamples in a row that fired: speculative marks
#endif

struct Resample1Args {
  const double* pm;        // step-kernel block partials
  const double* ps;
  const double* ps2;
  int nb_part;
  const double* logw;
  int64_t n;
  int shift;
  double* stats_out;       // (M, S, S2) of this rank
  DevScalars* dev;
  DecideArgs d;
  uint64_t* tsum;          // [grid] published tile totals (bit 63: generation parity)
  uint64_t* ts1;           // sums_in_pass: [grid] tile sums of e = exp(w - M), e^2 (tagged bits)
  uint64_t* ts2;
  int sums_in_pass;        // the step wrote block maxima only: S, S2 from this pass
  MarkArgs mk;             // enabled: systematic marks; else write C
  uint64_t* C;
  const uint64_t* amax_in; // the step's atomic-max shards (sums-in-pass only; nullptr: fold pm)
  uint64_t* amax_reset;    // the other parity's shards, emptied for the next step
  uint64_t seed;
  uint32_t t;
  uint64_t* hdec;          // host-mapped decision mailbox [tag, fire | err << 32, ess] (nullptr: none);
  uint64_t htag;           //   block 0 posts the decision as soon as it is known, then this tag
};

// maybe_resample!'s return value for the host (block 0, thread 0): the
// decision words, a system-scope release, then the tag the host polls
// (gh_pf_maybe_resample with did / ess: no stream synchronisation).  An
// error an earlier kernel raised (the filter's error word: a grid-barrier or
// peer-wait timeout) is posted in place of the decision's own, so the call
// reports it; a barrier timeout later in this same launch surfaces at the
// filter's next synchronising call.
__device__ __forceinline__ void post_decision(uint64_t* hdec, uint64_t htag, const Decision& dec, const int* derr) {
  if (!hdec) return;
  const int prior = __hip_atomic_load(const_cast<int*>(derr), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int err = prior ? prior : dec.err;
  hdec[1] = (uint64_t)(uint32_t)dec.fire | ((uint64_t)(uint32_t)err << 32);
  hdec[2] = as_u64(dec.ess);
  __threadfence_system();
  __hip_atomic_store(&hdec[0], htag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// 1024-thread block reductions (16 waves), result broadcast; LDS-only
// barriers (outstanding global loads/stores are not waited for)
__device__ __forceinline__ double blk16_max(double v, double* sm) {
  v = wave_max(v);
  lds_barrier();
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  lds_barrier();
  double r = sm[0];
#pragma unroll
  for (int k = 1; k < 16; ++k) r = fmax(r, sm[k]);
  return r;
}
__device__ __forceinline__ double blk16_sum(double v, double* sm) {
  v = wave_sum(v);
  lds_barrier();
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  lds_barrier();
  double r = sm[0];
#pragma unroll
  for (int k = 1; k < 16; ++k) r += sm[k];
  return r;
}
// two sums in one pass (same per-value order as blk16_sum; sm holds 32)
__device__ __forceinline__ void blk16_sum2(double* a, double* b, double* sm) {
  const double wa = wave_sum(*a), wb = wave_sum(*b);
  lds_barrier();
  if ((threadIdx.x & 63) == 0) {
    sm[threadIdx.x >> 6] = wa;
    sm[16 + (threadIdx.x >> 6)] = wb;
  }
  lds_barrier();
  double ra = sm[0], rb = sm[16];
#pragma unroll
  for (int k = 1; k < 16; ++k) {
    ra += sm[k];
    rb += sm[16 + k];
  }
  *a = ra;
  *b = rb;
}
__device__ __forceinline__ uint64_t blk16_sum_u64(uint64_t v, uint64_t* sm) {
  v = wave_sum_u64(v);
  lds_barrier();
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = v;
  lds_barrier();
  uint64_t r = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) r += sm[k];
  return r;
}
// sum of the first w of the 16 wave totals: all 16 read at once (no serial
// LDS round trips), the rest masked
__device__ __forceinline__ uint64_t blk16_excl(const uint64_t* sm, int w) {
  uint64_t r = 0;
#pragma unroll
  for (int k = 0; k < 15; ++k) r += k < w ? sm[k] : 0ull;
  return r;
}
// inclusive scan of v and the sums of a, b in one LDS round (same per-value
// orders as blk16_incl_u64 and blk16_sum2)
__device__ __forceinline__ uint64_t blk16_incl_sum2(uint64_t v, double* a, double* b, uint64_t* smu, double* smd) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_incl_sum_u64(v);
  const double wa = wave_sum(*a), wb = wave_sum(*b);
  lds_barrier();
  if (lane == 63) smu[w] = v;
  if (lane == 0) {
    smd[w] = wa;
    smd[16 + w] = wb;
  }
  lds_barrier();
  v += blk16_excl(smu, w);
  double ra = smd[0], rb = smd[16];
#pragma unroll
  for (int k = 1; k < 16; ++k) {
    ra += smd[k];
    rb += smd[16 + k];
  }
  *a = ra;
  *b = rb;
  return v;
}
// inclusive scan over the block's threads
__device__ __forceinline__ uint64_t blk16_incl_u64(uint64_t v, uint64_t* sm) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_incl_sum_u64(v);
  lds_barrier();
  if (lane == 63) sm[w] = v;
  lds_barrier();
  return v + blk16_excl(sm, w);
}

// The resample kernel's block scan, with the cross-wave work done once: the
// 16 wave totals are scanned by wave 0 (one DPP scan over lanes 0..15) and
// each wave reads its one exclusive offset, instead of every wave summing 16
// LDS values under a mask; with `sums`, thread 0 alone adds the 16 wave sums
// of a and b (the block totals it publishes; same order as blk16_sum2).
// smu: 32 u64 (totals, offsets), smd: 32 doubles.  Inclusive scan returned;
// *a, *b hold the block sums in thread 0 only.
template <bool SUMS>
__device__ __forceinline__ uint64_t blk16_scan(uint64_t v, double* a, double* b, uint64_t* smu, double* smd) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_incl_sum_u64(v);
  double wa = 0.0, wb = 0.0;
  if (SUMS) {
    wa = wave_sum(*a);
    wb = wave_sum(*b);
  }
  lds_barrier();
  if (lane == 63) smu[w] = v;
  if (SUMS && lane == 0) {
    smd[w] = wa;
    smd[16 + w] = wb;
  }
  lds_barrier();
  if (w == 0) {
    const uint64_t t = lane < 16 ? smu[lane] : 0ull;
    const uint64_t inc = wave_incl_sum_u64(t);
    if (lane < 16) smu[16 + lane] = inc - t;
    if (SUMS && lane == 0) {
      double ra = smd[0], rb = smd[16];
#pragma unroll
      for (int k = 1; k < 16; ++k) {
        ra += smd[k];
        rb += smd[16 + k];
      }
      *a = ra;
      *b = rb;
    }
  }
  lds_barrier();
  return v + smu[16 + w];
}

// block max (16 waves): wave 0 folds the 16 wave maxima, every thread reads one
// LDS value (fmax is exact in any order)
__device__ __forceinline__ double blk16_max1(double v, double* sm) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_max(v);
  lds_barrier();
  if (lane == 0) sm[w] = v;
  lds_barrier();
  if (w == 0) {
    double r = lane < 16 ? sm[lane] : -INFINITY;
    r = wave_max(r);
    if (lane == 0) sm[16] = r;
  }
  lds_barrier();
  return sm[16];
}

// (uint64)x for 0 <= x <= 2^52 in three instructions: floor, then the integer
// read off the mantissa of floor(x) + 2^52 (exact below 2^53); the generic
// f64 -> u64 conversion is a dozen
__device__ __forceinline__ uint64_t f64_to_u52(double x) {
  return as_u64(floor(x) + 0x1p52) - 0x4330000000000000ull;
}
// and back, (double)q for q <= 2^52: the bits of 2^52 plus q (2^52 + q, exact
// below 2^53; q = 2^52 carries into the exponent: 2^53), minus 2^52 (two
// instructions; the generic u64 -> f64 conversion is four)
__device__ __forceinline__ double u52_to_f64(uint64_t q) {
  return as_f64(q + 0x4330000000000000ull) - 0x1p52;
}

template <bool MARKS, int IT, bool SUMS>
__global__ __launch_bounds__(kRsBlock, IT <= 4 ? 8 : 1) void k_resample1(Resample1Args r) {
  __shared__ double smd[32];
  __shared__ uint64_t smu[32];
  __shared__ DevScalars sd;
  __shared__ uint64_t sbase;
  __shared__ unsigned sgen;
  __shared__ int sfail;  // the barrier wait timed out: write nothing
  __shared__ int sspec;  // speculative marks (see below)
  // barrier generation of this launch and the fire streak: read before this
  // block publishes (so before block 0 can commit this launch's decision)
  if (threadIdx.x == 0) {
    sgen = r.dev->bar_gen + 1;
    sspec = r.dev->fire_streak >= kSpecStreak;
    sfail = 0;
  }
  // ---- fold the step partials (same order in every block: same result)
  // this tile's log-weights are loaded up front, beside the partials
  const int64_t i0 = (int64_t)blockIdx.x * (kRsBlock * IT) + (int64_t)threadIdx.x * IT;
  double lw[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) lw[k] = (i0 + k < r.n) ? r.logw[i0 + k] : -INFINITY;
  double M, s1 = 0.0, s2 = 0.0;
  constexpr bool sums = SUMS;  // the step wrote block maxima only: the sums come from this pass
  // KP partials per thread stay in registers (one round trip for the maxima;
  // the sums of small tiles ride along, larger tiles load them once M is known)
  constexpr int KP = IT > kRsPart ? IT : kRsPart;
  constexpr bool kSumsEarly = IT <= kRsPart;
  if (threadIdx.x < kAmaxShards && blockIdx.x == 0 && r.amax_reset)
    r.amax_reset[threadIdx.x * kAmaxStride] = kAmaxEmpty;  // the next step's shards (read by nobody here)
  if (sums && r.amax_in) {  // uniform: the step folded its maxima itself; every wave reads the shards
    const int lane = threadIdx.x & 63;
    uint64_t key = lane < kAmaxShards ? r.amax_in[lane * kAmaxStride] : 0ull;
    key = wave_incl_max_u64(key);
    M = amax_value(readlane63_u64(key));
  } else if (IT <= 8 && r.nb_part <= KP * kRsBlock) {  // uniform; always true at IT <= kRsPart (host-checked)
    double pmv[KP], psv[kSumsEarly ? KP : 1], ps2v[kSumsEarly ? KP : 1];
#pragma unroll
    for (int k = 0; k < KP; ++k) {
      const int b = threadIdx.x + k * kRsBlock;
      const bool ok = b < r.nb_part;
      pmv[k] = ok ? r.pm[b] : -INFINITY;
      if constexpr (kSumsEarly) {
        psv[k] = ok && !sums ? r.ps[b] : 0.0;
        ps2v[k] = ok && !sums ? r.ps2[b] : 0.0;
      }
    }
    double m = pmv[0];
#pragma unroll
    for (int k = 1; k < KP; ++k) m = fmax(m, pmv[k]);
    M = blk16_max1(m, smd);
    if (!sums && M > -INFINITY) {
      double a1[KP], a2[KP];
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        const int b = threadIdx.x + k * kRsBlock;
        const bool ok = b < r.nb_part;
        if constexpr (kSumsEarly) {
          a1[k] = psv[k];
          a2[k] = ps2v[k];
        } else {
          a1[k] = ok ? r.ps[b] : 0.0;
          a2[k] = ok ? r.ps2[b] : 0.0;
        }
      }
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        // pm - M <= 0: the branch-free exp (same values as gh_exp there)
        const double f = gh_exp_nonpos(pmv[k] - M);
        if (pmv[k] > -INFINITY) {
          s1 += a1[k] * f;
          s2 += a2[k] * (f * f);
        }
      }
    }
  } else {  // larger sets: max pass, then a sum pass over the (cache-hot) partials
    double m = -INFINITY;
    for (int b = threadIdx.x; b < r.nb_part; b += kRsBlock) m = fmax(m, r.pm[b]);
    M = blk16_max(m, smd);
    if (!sums && M > -INFINITY)
      for (int b = threadIdx.x; b < r.nb_part; b += kRsBlock) {
        const double mb = r.pm[b];
        if (mb > -INFINITY) {
          const double f = gh_exp(mb - M);
          s1 += r.ps[b] * f;
          s2 += r.ps2[b] * (f * f);
        }
      }
  }
  const bool m_ok = M > -INFINITY && M != INFINITY && M == M;
  double S1 = 0.0, S2 = 0.0;
  // the resample test alone (ESS = S^2 / S2 < thr, exactly as decide()):
  // block 0 commits the full decision (logsumexp, log-ML) at its end.  With
  // sums_in_pass the sums come from this pass's own exp(w - M) and the test
  // follows the grid barrier.
  __shared__ int sfire;
  __shared__ double sS[2];
  // block 0 posts the decision to the host as soon as it is taken (before the
  // marks), and commits it to the device scalars at its end
  bool posted = false;
  auto decision = [&]() {
    double st[3] = {M, S1, S2};
    DecideArgs d = r.d;
    d.stats_all = st;
    d.R = 1;
    return decide(d, false);
  };
  if (!sums) {
    blk16_sum2(&s1, &s2, smd);
    S1 = s1;
    S2 = s2;
    if (threadIdx.x == 0) {
      sfire = m_ok && ((S1 * S1) / S2 < r.d.thr);
      if (blockIdx.x == 0) {
        post_decision(r.hdec, r.htag, decision(), &r.dev->error);
        posted = true;
      }
    }
    lds_barrier();
  }
  // (thread 0 keeps M in LDS for the commit: no registers held through the marks)
  __shared__ double sMv;
  if (threadIdx.x == 0) sMv = M;
  auto commit = [&]() {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      M = sMv;
      const Decision dec = decision();
      r.stats_out[0] = M;
      r.stats_out[1] = S1;
      r.stats_out[2] = S2;
      r.dev->pending = 0;
      commit_decision(r.d, dec, r.dev, 0);
      r.dev->fire_streak = dec.fire ? r.dev->fire_streak + 1u : 0u;
      if (!posted) post_decision(r.hdec, r.htag, dec, &r.dev->error);
    }
  };
  if (sums ? !m_ok : !sfire) {  // uniform over the grid: nobody publishes
    commit();
    return;
  }
  const double Mq = M;
  // ---- quantise this block's tile (IT consecutive particles per thread);
  // sums_in_pass: the same e = exp(w - M) also feed this tile's sums
  const double qscale = as_f64((uint64_t)(r.shift + 1023) << 52);
  uint64_t q[IT];
  uint64_t tsum = 0;
  s1 = 0.0;
  s2 = 0.0;
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const bool in = i0 + k < r.n;
    const double e = in ? gh_exp_nonpos(lw[k] - Mq) : 0.0;
    q[k] = e == e ? f64_to_u52(e * qscale) : 0;  // = quantize_weight_nonpos (e * 2^shift <= 2^52)
    tsum += q[k];
    if (sums) {
      const double ee = lw[k] != lw[k] ? lw[k] : e;  // NaN poisons the statistics
      s1 += ee;
      s2 += ee * ee;
    }
  }
  const uint64_t incl = sums ? blk16_scan<true>(tsum, &s1, &s2, smu, smd) : blk16_scan<false>(tsum, &s1, &s2, smu, smd);
  // ---- grid barrier: each tile total (< 2^62) is published as ONE 8-byte
  // agent-scope store tagged in bit 63 with the generation's parity, and read
  // back with agent-scope loads until every tag matches (the payload is its
  // own flag: no counter, no fence).  sums_in_pass: the tile sums (>= 0, so
  // their sign bit is free) are published and polled the same way.
  const uint64_t kTag = 1ull << 63;
  const uint64_t par = (sgen & 1u) ? kTag : 0ull;
  // ts1/ts2 are published on EVERY generation (0 when the sums are not in
  // this pass), so each of the three words alternates its tag strictly and a
  // matching tag always means this generation's value: a poller can never
  // pair a fresh tile total with sums left over from two generations back.
  if (threadIdx.x == kRsBlock - 1) st_sc1(&r.tsum[blockIdx.x], incl | par);
  if (threadIdx.x == 0) {
    st_sc1(&r.ts1[blockIdx.x], (as_u64(s1) & ~kTag) | par);
    st_sc1(&r.ts2[blockIdx.x], (as_u64(s2) & ~kTag) | par);
  }
  // waves 0..7 read the tile words, 64 tiles each (grid <= 512, host-checked):
  // one poll in flight per lane, so the kernel's register budget stays at two
  // resident 1024-thread blocks per CU; the wave sums (integer totals in any
  // order, the weight sums by the DPP tree) are combined by thread 0 in wave
  // order — the same arithmetic in every block
  __shared__ uint64_t spa[8], spb[8];
  __shared__ double spg[2][8];
  __shared__ uint64_t su53;
  // sums_in_pass after a run of resamples that all fired (kSpecStreak): the
  // blocks write the marks without waiting for the weight sums, and block 0
  // reads them and takes the decision after its marks; a resample that then
  // does not fire leaves marks no step reads
  // (not when the host waits for the decision: the call-by-call loop with
  // maybe_resample!'s Bool asked for gets it before the marks, as without)
  const bool spec = sums && sspec && !r.hdec;  // (grid-uniform)
  {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 8 * 64) {  // a non-polling wave draws the systematic offset's uniform meanwhile
      const u32x4 wr = rng_block(r.seed, ~0ull, r.t, STREAM_RESAMPLE, 0);  // independent of the totals
      su53 = u53_bits(wr.x, wr.y);
    }
    if (w < 8) {
      const unsigned b = (unsigned)(w * 64 + lane);
      const bool mine = b < gridDim.x;
      // the totals alone while the grid publishes, then the tile sums
      // (published with them) until their tags match too: a third of the
      // polling traffic while lagging blocks still load their tiles (C4, 512
      // tiles: barrier 2.2 us sooner, 39.7 -> 37.8 us per step; C2 -0.9 us)
      uint64_t v = par, v1 = par, v2 = par;
      bool ok = !mine, timed_out = false;  // (wave-uniform)
      for (unsigned spins = 0;; ++spins) {  // bounded (~0.5 s): a grid that is not co-resident errors out
        if (!ok) v = ld_sc1(&r.tsum[b]);
        ok = ok || (v & kTag) == par;
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        if (spins == (1u << 22)) {
          r.dev->error = 7;  // GH_E_STATE
          sfail = 1;
          timed_out = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      ok = !mine || !sums || spec || timed_out;  // (a timed-out wave does not wait a second time)
      for (unsigned spins = 0;; ++spins) {
        if (!ok) {
          v1 = ld_sc1(&r.ts1[b]);
          v2 = ld_sc1(&r.ts2[b]);
        }
        ok = ok || ((v1 & kTag) == par && (v2 & kTag) == par);
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        if (spins == (1u << 22)) {
          r.dev->error = 7;
          sfail = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      const uint64_t x = mine ? (v & ~kTag) : 0ull;
      const uint64_t all = wave_sum_u64(x);
      const uint64_t before = wave_sum_u64(b < blockIdx.x ? x : 0ull);
      double g1 = 0.0, g2 = 0.0;
      if (sums) {
        g1 = wave_sum(mine ? as_f64(v1 & ~kTag) : 0.0);
        g2 = wave_sum(mine ? as_f64(v2 & ~kTag) : 0.0);
      }
      if (lane == 0) {
        spa[w] = all;
        spb[w] = before;
        spg[0][w] = g1;
        spg[1][w] = g2;
      }
    }
  }
  lds_barrier();
  if (threadIdx.x == 0) {
    uint64_t all = 0, before = 0;
    double g1 = 0.0, g2 = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      all += spa[k];
      before += spb[k];
      g1 += spg[0][k];
      g2 += spg[1][k];
    }
    if (sums) {
      sS[0] = g1;
      sS[1] = g2;
      sfire = (g1 * g1) / g2 < r.d.thr;
      if (blockIdx.x == 0 && !sfail && !spec) {
        S1 = g1;
        S2 = g2;
        post_decision(r.hdec, r.htag, decision(), &r.dev->error);
        posted = true;
      }
    }
    const uint64_t N = (uint64_t)r.d.n_global;
    sd.S = all;
    sd.base = 0;
    sd.local = all;
    sd.o = scale_u53(su53, all);
    sd.invN = r.d.inv_n;
    sd.Qs = udiv_n(all, N, sd.invN);
    sd.Rs = all - sd.Qs * N;
    sd.invS = recip_est((double)all);
    sbase = before;
    if (blockIdx.x == 0) {
      r.dev->bar_gen = sgen;  // every block has published, so has read the old value
      r.dev->S = sd.S;
      r.dev->base = 0;
      r.dev->local = sd.local;
      r.dev->o = sd.o;
      r.dev->Qs = sd.Qs;
      r.dev->Rs = sd.Rs;
      r.dev->invN = sd.invN;
      r.dev->invS = sd.invS;
    }
  }
  lds_barrier();
  // Not co-resident (the device runs other kernels, so some blocks of this
  // grid never started): the totals are partial.  The block leaves without
  // marks or decision; the error surfaces as GH_E_STATE at the next sync.
  if (sfail) return;
  // (sums_in_pass, not speculative: thread 0 reads the sums from LDS at the
  // commit, so no registers hold them through the marks)
  auto sums_from_lds = [&]() {
    if (sums && !spec) {
      S1 = sS[0];
      S2 = sS[1];
    }
  };
  if (sums && !spec && !sfire) {
    sums_from_lds();
    commit();
    return;
  }
  // speculative: block 0 reads the tile sums and takes the decision after
  // its marks or CDF
  auto decide_late = [&]() {
    if (!spec || blockIdx.x != 0) return;  // (block-uniform)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (w < 8) {
      const unsigned b = (unsigned)(w * 64 + lane);
      const bool mine = b < gridDim.x;
      uint64_t v1 = ld_sc1(&r.ts1[mine ? b : 0u]);  // (every lane: no merged values)
      uint64_t v2 = ld_sc1(&r.ts2[mine ? b : 0u]);
      bool ok = !mine || ((v1 & kTag) == par && (v2 & kTag) == par);
      for (unsigned spins = 0; __builtin_amdgcn_ballot_w64(!ok) != 0; ++spins) {  // (rarely taken)
        if (spins == (1u << 22)) {
          r.dev->error = 7;  // GH_E_STATE
          sfail = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        if (!ok) {
          v1 = ld_sc1(&r.ts1[b]);
          v2 = ld_sc1(&r.ts2[b]);
        }
        ok = ok || ((v1 & kTag) == par && (v2 & kTag) == par);
      }
      const double g1 = wave_sum(mine ? as_f64(v1 & ~kTag) : 0.0);
      const double g2 = wave_sum(mine ? as_f64(v2 & ~kTag) : 0.0);
      if (lane == 0) {
        spg[0][w] = g1;
        spg[1][w] = g2;
      }
    }
    lds_barrier();
    if (threadIdx.x == 0) {
      double g1 = 0.0, g2 = 0.0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        g1 += spg[0][k];
        g2 += spg[1][k];
      }
      S1 = g1;
      S2 = g2;
    }
  };
  uint64_t run = sbase + incl - tsum;
  if (!MARKS) {
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      run += q[k];
      if (i0 + k < r.n) r.C[i0 + k] = run;
    }
    decide_late();
    sums_from_lds();
    if (!sfail) commit();
    return;
  }
  const uint32_t N = (uint32_t)r.mk.n_global;  // < 2^31: 32-bit slots and groups
  // The slot counts count(X) = ceil(v), v = (X N - o) / S, as sys_count, but
  // v advances by q N / S per particle (one FMA on the quantised weight, exact
  // as a double) instead of being re-derived from the 64-bit X.  Error: v_0 is
  // within 8 N 2^-53 + 2^-53 of the exact quotient (sys_count); ns = N / S to
  // within 6 units of 2^-53 (1/S within 2 ulp, one product), so the tile's
  // increments q ns add at most 6 N 2^-53 (their exact sum is <= N); each FMA
  // rounds by at most N 2^-53: |v - v*| <= (14 + IT) N 2^-53 + 2^-53 <=
  // 31 N 2^-53 + 2^-53 for IT <= 16, a quarter of count_window(N), so ceil(v)
  // is exact outside the window and the count is taken exactly inside it.  No
  // clamps or edge tests: for 0 < X < S, v* lies in (-1, N); X = 0 and X = S
  // give v* = -o/S and N - o/S, whose ceilings are 0 and N (o small: inside
  // the window, so the exact count).
  static_assert(IT <= 16, "the error bound of the incremental slot counts");
  const double ns = as_f64(readfirstlane_u64(as_u64((double)N * sd.invS)));  // (uniform: SGPRs)
  // near the integers: |fr - 1/2| >= 1/2 - w (1/2 - w is a double, so the
  // rounding of fr - 1/2 never takes a near value out; it may take a value
  // just outside the window in, which only costs an exact count)
  const double hw = as_f64(readfirstlane_u64(as_u64(0.5 - count_window(N))));
  double v = fma((double)run, (double)N, -(double)sd.o) * sd.invS;
  auto count = [&](uint64_t X) {
    const double fl = floor(v);
    const double fr = v - fl;
    int32_t j = (int32_t)fl + 1;
    const bool near = fabs(fr - 0.5) >= hw;
    if (near) j = sys_count_exact_call(&sd, N, X);  // (exec-masked call, skipped when no lane is near)
    return j;
  };
  int32_t s_i = count(run);
  // particle i owns the slots [s_i, e_i): a tagged mark at s_i, and the carry
  // of every 64-slot group that starts inside the range; a lane writes up to
  // two carries itself, a longer range (a particle with > 128 offspring) gets
  // its carries from the whole wave (one wave-wide store loop per such
  // particle, no block barrier)
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    run += q[k];
    v = fma(u52_to_f64(q[k]), ns, v);
    // (a particle past n or of zero weight leaves run, v, hence the count, unchanged)
    const int32_t e_i = count(run);
    const uint32_t tagged = r.mk.tag | (uint32_t)(i0 + k);
    if (e_i > s_i) r.mk.mark[(uint32_t)s_i] = tagged;
    const uint32_t g0 = ((uint32_t)s_i + 63u) >> 6, g1 = ((uint32_t)e_i + 63u) >> 6;  // groups g with 64 g in [s_i, e_i)
    const bool many = g1 - g0 > 2u;
    if (!many) {
      if (g1 > g0) r.mk.cmark[g0] = tagged;
      if (g1 > g0 + 1u) r.mk.cmark[g0 + 1u] = tagged;
    }
    uint64_t bm = __builtin_amdgcn_ballot_w64(many);
    while (bm) {
      const int L = __builtin_ctzll(bm);
      bm &= bm - 1;
      const int32_t a0 = __builtin_amdgcn_readlane((int32_t)g0, L), a1 = __builtin_amdgcn_readlane((int32_t)g1, L);
      const uint32_t tg = r.mk.tag | (uint32_t)__builtin_amdgcn_readlane((int32_t)(i0 + k), L);
      for (int32_t g = a0 + (threadIdx.x & 63); g < a1; g += 64) r.mk.cmark[g] = tg;
    }
    s_i = e_i;
  }
  decide_late();
  sums_from_lds();
  if (!sfail) commit();
}

// ------------------------------------------------ multi-rank resample (R > 1)
// DESIGN.md §7.  Phase A (before the all-gather of the rank totals): every
// block takes the decision from the all-gathered (M, S, S2) triples, then
// quantises its tile, publishes the tile total and crosses one grid barrier
// (as k_resample1); block 0 leaves the rank total in dev->local.
struct RankAArgs {
  const double* logw;
  int64_t n;
  int shift;
  DevScalars* dev;
  DecideArgs d;      // stats_all = the R all-gathered triples
  uint64_t* tsum;    // [grid] tile totals (bit 63: generation parity)
  uint64_t* ts1;     // [grid] the tile-sum words k_rank_a2 and k_resample1 poll: published here
  uint64_t* ts2;     //   too (0, tagged), so each word's tag alternates with every generation
};

template <int IT>
__global__ __launch_bounds__(kRsBlock) void k_rank_a(RankAArgs r) {
  __shared__ uint64_t smu[16];
  __shared__ int sfire;
  __shared__ double sM;
  __shared__ unsigned sgen;
  if (threadIdx.x == 0) {
    sgen = r.dev->bar_gen + 1;
    const Decision dec = decide(r.d, false);
    sfire = dec.fire;
    sM = dec.M;
    if (blockIdx.x == 0) {
      r.dev->pending = 0;
      commit_decision(r.d, dec, r.dev, 0);
    }
  }
  __syncthreads();
  if (!sfire) return;
  const double M = sM;
  const int64_t i0 = (int64_t)blockIdx.x * (kRsBlock * IT) + (int64_t)threadIdx.x * IT;
  uint64_t tsum = 0;
  const double qscale = as_f64((uint64_t)(r.shift + 1023) << 52);
#pragma unroll
  for (int k = 0; k < IT; ++k) {  // (= quantize_weight: the branch-free exp, 3-instruction conversion)
    const double e = (i0 + k < r.n) ? gh_exp_nonpos(r.logw[i0 + k] - M) : 0.0;
    tsum += e == e ? f64_to_u52(e * qscale) : 0;
  }
  const uint64_t tot = blk16_sum_u64(tsum, smu);
  const uint64_t kTag = 1ull << 63;
  const uint64_t par = (sgen & 1u) ? kTag : 0ull;
  if (threadIdx.x == 0) {
    st_sc1(&r.tsum[blockIdx.x], tot | par);
    // (a generation that skipped these would leave them one parity behind:
    // the next k_rank_a2 would take a tile's sums from two generations back)
    st_sc1(&r.ts1[blockIdx.x], par);
    st_sc1(&r.ts2[blockIdx.x], par);
  }
  uint64_t all = 0;
  unsigned failed = 0;
  for (int b = threadIdx.x; b < (int)gridDim.x; b += kRsBlock) {
    uint64_t v = ld_sc1(&r.tsum[b]);
    unsigned spins = 0;
    while ((v & kTag) != par) {
      __builtin_amdgcn_s_sleep(1);
      v = ld_sc1(&r.tsum[b]);
      if (++spins == (1u << 22)) {
        r.dev->error = 7;  // GH_E_STATE: not co-resident (see k_resample1)
        failed = 1;
        break;
      }
    }
    all += v & ~kTag;
  }
  all = blk16_sum_u64(all, smu);
  if (__syncthreads_or(failed)) return;  // partial totals: publish nothing
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    r.dev->local = all;
    r.dev->bar_gen = sgen;
  }
}

// Multi-rank resample of the batched loop (gh_pf_run), phase A
// with the weight sums in the quantisation pass: the step kernels wrote their
// block maxima into kAmaxShards order-keyed atomic-max words per rank (no fold
// launch), all-gathered.  Every block folds the R x kAmaxShards keys into the
// global max M, quantises its tile against M, sums e = exp(w - M) and e^2 from
// the same exps and publishes the tile total and sums (tagged, as
// k_resample1).  Only block 0 needs the rank's totals: it alone polls the tile
// words and writes the rank record (integer total, S_r, S2_r, M) that the
// second all-gather carries; the other blocks leave after publishing.  The
// decision is taken from the R records by k_rank_b (and by the host, the same
// arithmetic, for the split of the next step).
constexpr int kRecWords = 4;  // rank record: integer total, S_r, S2_r (f64 bits), M (f64 bits)
// ---------------------------------------------- peer transport primitives
// (gh_peer.h: the transport's design; gh_ctx_create_peer)
constexpr int kAgWords = 8;  // largest small all-gather payload (u64 words)
constexpr int kPeerMaxRanks = 64;
constexpr double kPeerWaitDefaultS = 30.0;  // default bound of a device wait on a peer (gh_ctx_set_peer_timeout)

// mailbox layout (u64 words), for R ranks
__host__ __device__ __forceinline__ int64_t mb_sh(int R, int par, int r) { return (int64_t)par * R + r; }
__host__ __device__ __forceinline__ int64_t mb_sh_tag(int R, int par, int r) { return 2LL * R + (int64_t)par * R + r; }
__host__ __device__ __forceinline__ int64_t mb_rec(int R, int par, int r) {
  return 4LL * R + ((int64_t)par * R + r) * kRecWords;
}
__host__ __device__ __forceinline__ int64_t mb_rec_tag(int R, int par, int r) {
  return 4LL * R + 2LL * R * kRecWords + (int64_t)par * R + r;
}
__host__ __device__ __forceinline__ int64_t mb_ag(int R, int par, int r) {
  return 6LL * R + 2LL * R * kRecWords + ((int64_t)par * R + r) * kAgWords;
}
__host__ __device__ __forceinline__ int64_t mb_ag_tag(int R, int par, int r) {
  return 6LL * R + 2LL * R * kRecWords + 2LL * R * kAgWords + (int64_t)par * R + r;
}
__host__ __device__ __forceinline__ int64_t mb_words(int R) { return 8LL * R + 2LL * R * kRecWords + 2LL * R * kAgWords; }

// every rank's mailbox, as this process maps it (peer[rank] is its own)
struct PeerBox {
  uint64_t* peer[kPeerMaxRanks];
  int R, rank;
  uint64_t wait_ticks;  // the wait bound in wall-clock ticks (gh_ctx_set_peer_timeout)
};

// Wave-level poll: lanes r < R wait until word (base + stride * r) of the own
// mailbox reaches `want` (monotonic tags).  Returns false once `ticks` of the
// constant-rate wall clock (s_memrealtime, 100 MHz) have passed: a backstop
// against a rank that never comes, measured in time rather than polls (a
// slow peer — host I/O, a first launch, descheduling — is waited for up to the
// context's bound, 30 s by default; round 5's bound was ~2.5 s of polls).
__device__ __forceinline__ bool peer_poll(const uint64_t* own, int64_t base, int R, uint64_t want, uint64_t ticks,
                                          int skip = -1) {
  const int lane = threadIdx.x & 63;
  bool ok = lane >= R || lane == skip;
  const uint64_t t0 = wall_clock64();
  for (unsigned spins = 0;; ++spins) {
    if (!ok) ok = ld_sys(own + base + lane) >= want;
    if (__builtin_amdgcn_ballot_w64(!ok) == 0) return true;
    if ((spins & 63) == 63 && wall_clock64() - t0 > ticks) return false;
    __builtin_amdgcn_s_sleep(2);
  }
}

// Publish `words` u64 values (lane l holds value l; lanes < words) to slot
// `slot` of every rank's mailbox, then the tag at `tag` behind a system-scope
// release.  One whole wave calls it.
__device__ __forceinline__ void peer_publish(const PeerBox& pb, int64_t slot, int64_t tag, uint64_t lane_val,
                                             int words, uint64_t use) {
  const int lane = threadIdx.x & 63;
  for (int q = 0; q < pb.R; ++q)
    if (lane < words) st_sys(pb.peer[q] + slot + lane, lane_val);
  __threadfence_system();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane < pb.R) st_sys(pb.peer[lane] + tag, use);
}

struct RankA2Args {
  const double* logw;
  int64_t n;
  int shift;
  DevScalars* dev;
  const uint64_t* amax_all;  // [R][kAmaxShards * kAmaxStride] all-gathered shard words
  int R;
  uint64_t* amax_reset;      // this rank's shards just consumed (read from the gathered copy): emptied
  uint64_t* tsum;            // [grid] tile totals (bit 63: generation parity)
  uint64_t* ts1;             // [grid] tile sums of e, e^2 (tagged bits)
  uint64_t* ts2;
  uint64_t* rec;             // [kRecWords] this rank's record (input of the second all-gather)
  // peer transport (pb.R > 0): no all-gathers — every block folds this rank's
  // own shards (amax_own), block 0 publishes the rank maximum to every
  // mailbox (SH, use_sh), every block polls its own for all R; at the end
  // block 0 publishes the record (REC, use_rec) for k_rank_b.  The shards are
  // then emptied by k_rank_b (every block of this launch reads them).
  PeerBox pb;
  const uint64_t* amax_own;
  uint64_t use_sh, use_rec;
};

template <int IT>
__global__ __launch_bounds__(kRsBlock, IT <= 4 ? 8 : 1) void k_rank_a2(RankA2Args r) {
  __shared__ double smd[32];
  __shared__ uint64_t smu[32];
  __shared__ unsigned sgen;
  __shared__ int sfail;
  __shared__ uint64_t spa[8];
  __shared__ double spg[2][8];
  if (threadIdx.x == 0) {
    sgen = r.dev->bar_gen + 1;
    sfail = 0;
  }
  const int64_t i0 = (int64_t)blockIdx.x * (kRsBlock * IT) + (int64_t)threadIdx.x * IT;
  double lw[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) lw[k] = (i0 + k < r.n) ? r.logw[i0 + k] : -INFINITY;
  const bool peer = r.pb.R > 0;  // (uniform)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ uint64_t srec[kRecWords];
  double M;
  if (!peer) {
    // the global max from every rank's shards (the same keys, the same M in every block)
    uint64_t key = kAmaxEmpty;
    for (int idx = threadIdx.x; idx < r.R * kAmaxShards; idx += kRsBlock) {
      const uint64_t v = r.amax_all[(idx / kAmaxShards) * (kAmaxShards * kAmaxStride) + (idx % kAmaxShards) * kAmaxStride];
      key = v > key ? v : key;
    }
    M = blk16_max1(amax_value(key), smd);
    if (blockIdx.x == 0 && threadIdx.x < kAmaxShards) r.amax_reset[threadIdx.x * kAmaxStride] = kAmaxEmpty;
  } else {
    // this rank's maximum (every block the same), then the R ranks' through the mailboxes
    const uint64_t k0 = threadIdx.x < kAmaxShards ? r.amax_own[threadIdx.x * kAmaxStride] : kAmaxEmpty;
    const double Ml = blk16_max1(amax_value(k0), smd);
    __shared__ double sM;
    if (w == 0) {
      const int par = (int)(r.use_sh & 1);
      const uint64_t* own = r.pb.peer[r.pb.rank];
      if (blockIdx.x == 0)
        peer_publish(r.pb, mb_sh(r.pb.R, par, r.pb.rank), mb_sh_tag(r.pb.R, par, r.pb.rank), amax_key(Ml), 1, r.use_sh);
      const bool ok = peer_poll(own, mb_sh_tag(r.pb.R, par, 0), r.pb.R, r.use_sh, r.pb.wait_ticks);
      uint64_t kk = ok && lane < r.pb.R ? ld_sys(own + mb_sh(r.pb.R, par, lane)) : kAmaxEmpty;
      kk = readlane63_u64(wave_incl_max_u64(kk));
      if (lane == 0) {
        sM = ok ? amax_value(kk) : NAN;
        if (!ok) {
          sfail = 1;
          r.dev->error = kErrPeer;  // a rank never published
        }
      }
    }
    lds_barrier();
    M = sM;
  }
  const bool m_ok = M > -INFINITY && M != INFINITY && M == M;
  if (!m_ok) {  // uniform over every rank's grid: no tile publishes; the decision raises GH_E_NUMERIC
    if (blockIdx.x == 0) {
      if (threadIdx.x == 0) {
        r.rec[0] = 0;
        r.rec[1] = 0;
        r.rec[2] = 0;
        r.rec[3] = as_u64(M);
        r.dev->local = 0;
      }
      if (peer && w == 0) {
        const int par = (int)(r.use_rec & 1);
        const uint64_t v = lane == 3 ? as_u64(M) : 0ull;
        peer_publish(r.pb, mb_rec(r.pb.R, par, r.pb.rank), mb_rec_tag(r.pb.R, par, r.pb.rank), v, kRecWords, r.use_rec);
      }
    }
    return;
  }
  const double qscale = as_f64((uint64_t)(r.shift + 1023) << 52);
  uint64_t tsum = 0;
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const bool in = i0 + k < r.n;
    const double e = in ? gh_exp_nonpos(lw[k] - M) : 0.0;
    tsum += e == e ? f64_to_u52(e * qscale) : 0;  // = quantize_weight (k_rank_b re-quantises the same)
    const double ee = lw[k] != lw[k] ? lw[k] : e;  // NaN poisons the statistics
    s1 += ee;
    s2 += ee * ee;
  }
  const uint64_t incl = blk16_scan<true>(tsum, &s1, &s2, smu, smd);
  const uint64_t kTag = 1ull << 63;
  const uint64_t par = (sgen & 1u) ? kTag : 0ull;
  if (threadIdx.x == kRsBlock - 1) st_sc1(&r.tsum[blockIdx.x], incl | par);
  if (threadIdx.x == 0) {
    st_sc1(&r.ts1[blockIdx.x], (as_u64(s1) & ~kTag) | par);
    st_sc1(&r.ts2[blockIdx.x], (as_u64(s2) & ~kTag) | par);
  }
  if (blockIdx.x != 0) return;
  // block 0: the rank totals (waves 0..7 poll 64 tiles each, as k_resample1)
  if (w < 8) {
    const unsigned b = (unsigned)(w * 64 + lane);
    const bool mine = b < gridDim.x;
    uint64_t v = par, v1 = par, v2 = par;
    bool ok = !mine, fail = false;
    for (unsigned spins = 0;; ++spins) {  // bounded (~0.5 s): a grid that is not co-resident errors out
      if (!ok) {
        v = ld_sc1(&r.tsum[b]);
        v1 = ld_sc1(&r.ts1[b]);
        v2 = ld_sc1(&r.ts2[b]);
      }
      ok = ok || ((v & kTag) == par && (v1 & kTag) == par && (v2 & kTag) == par);
      if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
      if (spins == (1u << 22)) {
        fail = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const uint64_t all = wave_sum_u64(mine ? (v & ~kTag) : 0ull);
    const double g1 = wave_sum(mine ? as_f64(v1 & ~kTag) : 0.0);
    const double g2 = wave_sum(mine ? as_f64(v2 & ~kTag) : 0.0);
    if (lane == 0) {
      spa[w] = all;
      spg[0][w] = g1;
      spg[1][w] = g2;
      if (fail) sfail = 1;
    }
  }
  lds_barrier();
  if (threadIdx.x == 0) {
    uint64_t all = 0;
    double g1 = 0.0, g2 = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      all += spa[k];
      g1 += spg[0][k];
      g2 += spg[1][k];
    }
    if (sfail) {
      r.dev->error = 7;  // GH_E_STATE: partial totals
      g1 = NAN;
    }
    r.rec[0] = all;
    r.rec[1] = as_u64(g1);
    r.rec[2] = as_u64(g2);
    r.rec[3] = as_u64(M);
    srec[0] = all;
    srec[1] = as_u64(g1);
    srec[2] = as_u64(g2);
    srec[3] = as_u64(M);
    r.dev->local = all;
    r.dev->bar_gen = sgen;  // every block has published, so has read the old value
  }
  if (peer) {  // the record to every rank's mailbox (k_rank_b polls for all R)
    lds_barrier();
    if (w == 0) {
      const int par = (int)(r.use_rec & 1);
      peer_publish(r.pb, mb_rec(r.pb.R, par, r.pb.rank), mb_rec_tag(r.pb.R, par, r.pb.rank),
                   lane < kRecWords ? srec[lane] : 0ull, kRecWords, r.use_rec);
    }
  }
}

// The decision of a multi-rank resample from the R rank records (rank order):
// the sums share the global max, so S = sum S_r, S2 = sum S2_r; host and
// device evaluate the same arithmetic (finish_plan needs the fire flag before
// the device has taken it).
GH_HD Decision decide_records(const uint64_t* recs, int R, double thr) {
  Decision d{};
  const double M = as_f64(recs[3]);
  double S = 0.0, S2 = 0.0;
  for (int q = 0; q < R; ++q) {
    S += as_f64(recs[kRecWords * q + 1]);
    S2 += as_f64(recs[kRecWords * q + 2]);
  }
  d.M = M;
  if (!(M > -INFINITY) || M == INFINITY || M != M) {
    d.err = 3;  // GH_E_NUMERIC
    d.ess = NAN;
    return d;
  }
  d.L = M + gh_log(S);
  d.ess = (S * S) / S2;
  d.fire = d.ess < thr;
  return d;
}

// Phase B (after the all-gather): every block derives the global systematic
// constants and the slot coverage of every rank from the totals (the same
// integers on every rank), re-quantises its tile, and for each particle's
// slot range writes a range mark where the slots are this rank's own and a
// state row (x, global id) where they belong to another rank, packed by
// destination rank and slot.  Slots of this rank covered by other ranks are
// [0, ra) and [rb, n): the step kernel reads them from the received rows.
constexpr int kMaxRanks = 64;
struct RankBArgs {
  const double* logw;
  int64_t n;
  int shift;
  DevScalars* dev;
  const uint64_t* tsum;   // tile totals of phase A (tagged)
  const uint64_t* totals; // all-gathered rank totals, rank k's at totals[k * tot_stride]
  int tot_stride;         // 1: k_rank_a's totals; kRecWords: k_rank_a2's records
  const uint64_t* recs;   // k_rank_a2's records: this launch takes (and block 0 commits) the decision
  const int64_t* dlo;     // [R + 1] floor(N k / R): rank k's first global slot (host table)
  uint64_t* hplan;        // (with recs) host-mapped plan mailbox: block 0 copies the R records to
  uint64_t htag;          //   hplan[1..] and then writes htag to hplan[0] (the host polls it)
  DecideArgs d;           //   (with recs) the decision's threshold and histories
  int R, rank;
  int64_t lo;             // global id of this rank's first particle
  uint64_t seed;
  uint32_t t;
  MarkArgs mk;            // marks / carries in this rank's local slot space
  const double* xprev;    // wave-tiled states of the current step (xidx)
  int D;
  double* rows;           // send rows [(D+1)] per slot
  int64_t rows_cap;
  uint64_t* C;            // more rows than rows_cap: the inclusive CDF, for k_rows_fill
  // peer transport (pb.R > 0): the records come from the own mailbox (REC,
  // use_rec; every block polls), the rows go straight into every receiving
  // rank's row buffer prow[k] at the row its slot takes there, and block 0
  // empties the shards k_rank_a2 read (amax_reset)
  PeerBox pb;
  uint64_t use_rec;
  int peer_rows;          // the rows go to prow (peer transport, either resample form)
  double* prow[kPeerMaxRanks];
  uint64_t* amax_reset;
};

// The send layout of one rank's resample (as gh_sys_plan): destination rank k
// owns global slots [dlo_k, dhi_k); this rank's particles cover [cov_lo,
// cov_hi); the rows for rank k != rank start at soff_k, in slot order.
__device__ __forceinline__ int64_t send_tables(const DevScalars* sd, uint64_t N, int R, int q, uint64_t local,
                                               const int64_t* dlo_tab, int64_t* dst_lo, int64_t* seg_lo,
                                               int64_t* soffs, int64_t* cov_lo_out, int64_t* cov_hi_out) {
  const int64_t cov_lo = sys_count_exact(sd, N, sd->base);
  const int64_t cov_hi = sys_count_exact(sd, N, sd->base + local);
  int64_t soff = 0;
  for (int k = 0; k < R; ++k) {
    const int64_t dlo = dlo_tab[k], dhi = dlo_tab[k + 1];  // floor(N k / R), from the host
    const int64_t a = cov_lo > dlo ? cov_lo : dlo, b = cov_hi < dhi ? cov_hi : dhi;
    dst_lo[k] = dlo;
    seg_lo[k] = a;
    soffs[k] = soff;
    if (k != q && b > a) soff += b - a;
  }
  *cov_lo_out = cov_lo;
  *cov_hi_out = cov_hi;
  return soff;
}

// the state rows of particle i's slots [s0, s1) that other ranks own
__device__ __forceinline__ void send_rows(int64_t s0, int64_t s1, int64_t i, int64_t own_lo, int64_t own_hi, int R,
                                          uint64_t N, const int64_t* dst_lo, const int64_t* seg_lo,
                                          const int64_t* soffs, int64_t rows_cap, double* rows, const double* xprev,
                                          int D, int64_t lo) {
  for (int64_t sl = s0; sl < s1; ++sl) {
    if (sl >= own_lo && sl < own_hi) {
      sl = own_hi - 1;  // skip the own block
      continue;
    }
    int dst = (int)(((__int128)sl * R) / (int64_t)N);  // owner of global slot sl
    while (dst + 1 < R && dst_lo[dst + 1] <= sl) ++dst;
    while (dst > 0 && dst_lo[dst] > sl) --dst;
    const int64_t row = soffs[dst] + (sl - seg_lo[dst]);
    if (row < rows_cap) {
      double* rw = rows + row * (D + 1);
      for (int c = 0; c < D; ++c) rw[c] = xprev[xidx(i, c, D)];
      rw[D] = __longlong_as_double(lo + i);
    }
  }
}

// the same rows written into the receivers' own buffers (peer transport):
// rank k's slot j (local) takes row j below ra_k and ra_k + j - rb_k from rb_k
__device__ __forceinline__ void send_rows_peer(int64_t s0, int64_t s1, int64_t i, int64_t own_lo, int64_t own_hi,
                                               int R, uint64_t N, const int64_t* dst_lo, const int64_t* ra,
                                               const int64_t* rb, double* const* prow, const double* xprev, int D,
                                               int64_t lo) {
  for (int64_t sl = s0; sl < s1; ++sl) {
    if (sl >= own_lo && sl < own_hi) {
      sl = own_hi - 1;  // skip the own block
      continue;
    }
    int dst = (int)(((__int128)sl * R) / (int64_t)N);  // owner of global slot sl
    while (dst + 1 < R && dst_lo[dst + 1] <= sl) ++dst;
    while (dst > 0 && dst_lo[dst] > sl) --dst;
    const int64_t j = sl - dst_lo[dst];
    const int64_t row = j < ra[dst] ? j : ra[dst] + (j - rb[dst]);
    double* rw = prow[dst] + row * (D + 1);
    for (int c = 0; c < D; ++c) st_sys(rw + c, xprev[xidx(i, c, D)]);
    st_sys(rw + D, __longlong_as_double(lo + i));
  }
}

template <int IT>
__global__ __launch_bounds__(kRsBlock) void k_rank_b(RankBArgs r) {
  __shared__ int sfire;
  __shared__ double sMq;
  // this tile's log-weights and the tile totals before it are loaded first,
  // so their round trip overlaps the decision's and thread 0's plan
  const int64_t i0 = (int64_t)blockIdx.x * (kRsBlock * IT) + (int64_t)threadIdx.x * IT;
  double lw[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) lw[k] = (i0 + k < r.n) ? r.logw[i0 + k] : 0.0;
  uint64_t before = 0;  // tile offset within the rank
  for (int b = threadIdx.x; b < (int)blockIdx.x; b += kRsBlock) before += r.tsum[b] & ~(1ull << 63);
  __shared__ uint64_t su53;
  if (threadIdx.x == 64) {  // another wave draws the systematic offset's uniform meanwhile (independent of the totals)
    const u32x4 w = rng_block(r.seed, ~0ull, r.t, STREAM_RESAMPLE, 0);
    su53 = u53_bits(w.x, w.y);
  }
  // peer transport: the R records from the own mailbox (wave 0 polls, LDS copy)
  const bool peer = r.pb.R > 0;  // (uniform)
  __shared__ uint64_t srecs[kPeerMaxRanks * kRecWords];
  const uint64_t* recs = r.recs;
  const uint64_t* totals = r.totals;
  if (peer) {
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x & 63, par = (int)(r.use_rec & 1);
      const uint64_t* own = r.pb.peer[r.pb.rank];
      const bool ok = peer_poll(own, mb_rec_tag(r.pb.R, par, 0), r.pb.R, r.use_rec, r.pb.wait_ticks);
      if (lane < r.pb.R)
        for (int k = 0; k < kRecWords; ++k)
          srecs[lane * kRecWords + k] = ok ? ld_sys(own + mb_rec(r.pb.R, par, lane) + k) : (k == 3 ? as_u64(NAN) : 0ull);
      if (!ok && lane == 0) r.dev->error = kErrPeer;  // a rank never published its record
      if (blockIdx.x == 0 && lane < kAmaxShards) r.amax_reset[lane * kAmaxStride] = kAmaxEmpty;
    }
    lds_barrier();
    recs = srecs;
    totals = srecs;
  }
  if (threadIdx.x == 0) {
    if (recs) {  // the decision from the R rank records (every block the same)
      const Decision dec = decide_records(recs, r.R, r.d.thr);
      sfire = dec.fire;
      sMq = dec.M;
      if (blockIdx.x == 0) {
        r.dev->pending = 0;
        commit_decision(r.d, dec, r.dev, 0);
        if (r.hplan) {  // the host's copy of the records, then the tag behind a system-scope release
          for (int w = 0; w < r.R * kRecWords; ++w) r.hplan[1 + w] = recs[w];
          __threadfence_system();
          __hip_atomic_store(&r.hplan[0], r.htag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    } else {  // k_rank_a decided
      sfire = r.dev->fire;
      sMq = r.dev->M;
    }
  }
  __shared__ uint64_t smu[16];
  __shared__ DevScalars sd;
  __shared__ int64_t sdst_lo[kMaxRanks], sseg_lo[kMaxRanks], ssoff[kMaxRanks];
  __shared__ int64_t sra_all[kMaxRanks], srb_all[kMaxRanks];
  __shared__ int64_t sown_lo, sown_hi, sra, srb, ssend;
  __shared__ uint64_t sbase;
  const int R = r.R, q = r.rank;
  const uint64_t N = (uint64_t)r.mk.n_global;
  // (the block sum's LDS barriers also publish the decision)
  before = blk16_sum_u64(before, smu);
  if (!sfire) return;
  if (threadIdx.x == 0) {
    uint64_t S = 0, base = 0;
    for (int k = 0; k < R; ++k) {
      if (k < q) base += totals[k * r.tot_stride];
      S += totals[k * r.tot_stride];
    }
    sd.S = S;
    sd.base = base;
    sd.local = totals[q * r.tot_stride];
    sd.o = scale_u53(su53, S);
    sd.invN = r.d.inv_n;
    sd.Qs = udiv_n(S, N, sd.invN);
    sd.Rs = S - sd.Qs * N;
    sd.invS = recip_est((double)S);
    const int64_t own_lo = r.lo, own_hi = r.lo + r.n;
    // rows this rank sends: destination blocks in rank order (lower ranks,
    // then higher ranks), each the part of [cov_lo, cov_hi) it owns
    int64_t cov_lo, cov_hi;
    ssend = send_tables(&sd, N, R, q, sd.local, r.dlo, sdst_lo, sseg_lo, ssoff, &cov_lo, &cov_hi);
    sown_lo = own_lo;
    sown_hi = own_hi;
    const int64_t ca = cov_lo < own_lo ? own_lo : (cov_lo > own_hi ? own_hi : cov_lo);
    const int64_t cb = cov_hi < own_lo ? own_lo : (cov_hi > own_hi ? own_hi : cov_hi);
    sra = ca - own_lo;
    srb = cb - own_lo;
    sbase = base + before;
    if (r.peer_rows) {  // every receiving rank's [0, ra) / [rb, n) split (its rows' layout)
      uint64_t bk = 0;
      for (int k = 0; k < R; ++k) {
        const uint64_t tk = totals[k * r.tot_stride];
        const int64_t dl = r.dlo[k], dh = r.dlo[k + 1];
        const int64_t lo_k = sys_count_exact(&sd, N, bk), hi_k = sys_count_exact(&sd, N, bk + tk);
        sra_all[k] = (lo_k < dl ? dl : (lo_k > dh ? dh : lo_k)) - dl;
        srb_all[k] = (hi_k < dl ? dl : (hi_k > dh ? dh : hi_k)) - dl;
        bk += tk;
      }
    }
    if (blockIdx.x == 0) {
      r.dev->S = S;
      r.dev->base = base;
      r.dev->o = sd.o;
      r.dev->Qs = sd.Qs;
      r.dev->Rs = sd.Rs;
      r.dev->invN = sd.invN;
      r.dev->invS = sd.invS;
      r.dev->ra = sra;
      r.dev->rb = srb;
    }
  }
  __syncthreads();
  const double M = sMq;
  uint64_t qv[IT];
  uint64_t tsum = 0;
  const double qscale = as_f64((uint64_t)(r.shift + 1023) << 52);
#pragma unroll
  for (int k = 0; k < IT; ++k) {  // (k_rank_a2's form: the branch-free exp, 3-instruction conversion)
    const double e = (i0 + k < r.n) ? gh_exp_nonpos(lw[k] - M) : 0.0;
    qv[k] = e == e ? f64_to_u52(e * qscale) : 0;
    tsum += qv[k];
  }
  const uint64_t incl = blk16_incl_u64(tsum, smu);
  uint64_t run = sbase + incl - tsum;
  // (32-bit slots: N < 2^31, gh_pf_init; the clamp is one v_med3_i32)
  const int32_t own_lo = (int32_t)sown_lo, own_hi = (int32_t)sown_hi;
  const uint32_t N32 = (uint32_t)N;
  // more rows than the bounded send buffer holds (this rank carries most of
  // the weight): keep the CDF, the host regrows the buffer and k_rows_fill
  // writes every row from it (rare; the hot path only tests the flag)
  const bool spill = ssend > r.rows_cap;
  // particle i's slots [s_i, e_i) (global) by k_resample1's incremental
  // counts (its error bound: exact outside count_window, the exact count
  // inside); the part this rank owns, [l0, l1) in local slots, gets a tagged
  // mark at l0 and the carry of every 64-slot group starting inside it — a
  // lane writes up to two carries, a longer range gets them from its whole
  // wave (no LDS copy of the range ends, no block barrier)
  static_assert(IT <= 16, "the error bound of the incremental slot counts");
  const double ns = as_f64(readfirstlane_u64(as_u64((double)N32 * sd.invS)));
  const double hw = as_f64(readfirstlane_u64(as_u64(0.5 - count_window(N32))));
  double v = fma((double)run, (double)N32, -(double)sd.o) * sd.invS;
  auto count = [&](uint64_t X) {
    const double fl = floor(v);
    const double fr = v - fl;
    int32_t j = (int32_t)fl + 1;
    const bool near = fabs(fr - 0.5) >= hw;
    if (near) j = sys_count_exact_call(&sd, N32, X);  // (exec-masked call, skipped when no lane is near)
    return j;
  };
  auto local = [&](int32_t sl) { return (uint32_t)(min(max(sl, own_lo), own_hi) - own_lo); };
  int32_t s_i = count(run);
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    run += qv[k];
    v = fma(u52_to_f64(qv[k]), ns, v);
    const int64_t i = i0 + k;
    // (a particle past n or of zero weight leaves run, v, hence the count, unchanged)
    const int32_t e_i = count(run);
    const uint32_t l0 = local(s_i), l1 = local(e_i);
    const uint32_t tagged = r.mk.tag | (uint32_t)i;
    if (l1 > l0) r.mk.mark[l0] = tagged;
    const uint32_t g0 = (l0 + 63u) >> 6, g1 = (l1 + 63u) >> 6;  // local groups g with 64 g in [l0, l1)
    const bool many = g1 - g0 > 2u;
    if (!many) {
      if (g1 > g0) r.mk.cmark[g0] = tagged;
      if (g1 > g0 + 1u) r.mk.cmark[g0 + 1u] = tagged;
    }
    uint64_t bm = __builtin_amdgcn_ballot_w64(many);
    while (bm) {
      const int L = __builtin_ctzll(bm);
      bm &= bm - 1;
      const int32_t a0 = __builtin_amdgcn_readlane((int32_t)g0, L), a1 = __builtin_amdgcn_readlane((int32_t)g1, L);
      const uint32_t tg = r.mk.tag | (uint32_t)__builtin_amdgcn_readlane((int32_t)i, L);
      for (int32_t g = a0 + (threadIdx.x & 63); g < a1; g += 64) r.mk.cmark[g] = tg;
    }
    if (spill && i < r.n) r.C[i] = run;
    // slots of other ranks (only a range that crosses this rank's block edge):
    // state rows, by destination then slot
    if (e_i > s_i && (s_i < own_lo || e_i > own_hi)) {
      if (r.peer_rows)
        send_rows_peer(s_i, e_i, i, own_lo, own_hi, R, N, sdst_lo, sra_all, srb_all, r.prow, r.xprev, r.D, r.lo);
      else if (!spill)
        send_rows(s_i, e_i, i, own_lo, own_hi, R, N, sdst_lo, sseg_lo, ssoff, r.rows_cap, r.rows, r.xprev, r.D,
                  r.lo);
    }
    s_i = e_i;
  }
}

// The send rows of a resample whose rows overflowed the bounded buffer, from
// the CDF k_rank_b kept (one thread per particle; the plan's scalars from dev)
struct RowsFillArgs {
  const uint64_t* C;
  int64_t n;
  int R, rank;
  int64_t lo;
  const DevScalars* dev;
  const uint64_t* totals;  // rank k's total at totals[k * tot_stride] (as RankBArgs)
  int tot_stride;
  int64_t n_global;
  const double* xprev;
  int D;
  double* rows;
  int64_t rows_cap;
  const int64_t* dlo;      // [R + 1] floor(N k / R), from the host
};

static __global__ __launch_bounds__(256) void k_rows_fill(RowsFillArgs r) {
  __shared__ DevScalars sd;
  __shared__ int64_t sdst_lo[kMaxRanks], sseg_lo[kMaxRanks], ssoff[kMaxRanks];
  const uint64_t N = (uint64_t)r.n_global;
  if (threadIdx.x == 0) {
    sd = *r.dev;
    int64_t a, b;
    send_tables(&sd, N, r.R, r.rank, r.totals[r.rank * r.tot_stride], r.dlo, sdst_lo, sseg_lo, ssoff, &a, &b);
  }
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= r.n) return;
  const uint64_t prev = i == 0 ? sd.base : r.C[i - 1], cur = r.C[i];
  const int64_t s0 = sys_count(&sd, N, prev);
  const int64_t s1 = cur > prev ? sys_count(&sd, N, cur) : s0;
  send_rows(s0, s1, i, r.lo, r.lo + r.n, r.R, N, sdst_lo, sseg_lo, ssoff, r.rows_cap, r.rows, r.xprev, r.D, r.lo);
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
  int own_only;            // multi-rank sampling: only the targets in this rank's CDF range (others: -1)
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

// first i in [lo, hi] with C[i] - base > target (C[hi] - base > target holds)
__device__ __forceinline__ int64_t cdf_search(const uint64_t* C, uint64_t base, uint64_t target,
                                              int64_t lo, int64_t hi) {
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    if (C[mid] - base > target) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

constexpr int kSearchWin = 256;  // CDF entries a wave stages in LDS

// Ancestor search.  Systematic targets are monotone in the slot, so a wave's
// 64 slots need a contiguous CDF window: the wave finds the window's ends
// with two (wave-uniform) binary searches, stages up to 256 entries in LDS
// and each lane finishes with an 8-step LDS search.  Wider windows (many
// zero-offspring particles between the wave's ancestors) and random targets
// (multinomial, sampling) use a per-lane binary search over the global CDF.
static __global__ __launch_bounds__(kBlock) void k_search(SearchArgs s, GateArgs g, const DevScalars* dev) {
  if (!*g.gate) return;
  __shared__ uint64_t win[kBlock / 64][kSearchWin];
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t jc = j < s.n_slots ? j : s.n_slots - 1;  // clamp: padding lanes mirror the last slot
  const uint64_t base = dev->base;
  const uint64_t tg = slot_target(s, dev, s.slot_lo + jc);
  const uint64_t target = tg - base;
  const bool mine = !s.own_only || (tg >= base && target < dev->local);
  const int64_t hi_all = s.n_cdf - 1;
  int64_t a;
  if (s.mode == SEARCH_SYSTEMATIC) {
    const uint64_t t_lo = __shfl(target, 0, 64);
    const uint64_t t_hi = __shfl(target, 63, 64);
    const int64_t a_lo = cdf_search(s.C, base, t_lo, 0, hi_all);
    const int64_t a_hi = cdf_search(s.C, base, t_hi, a_lo, hi_all);
    if (a_hi - a_lo < kSearchWin) {
#pragma unroll
      for (int k = 0; k < kSearchWin / 64; ++k) {
        const int64_t i = a_lo + lane + 64 * k;
        win[w][lane + 64 * k] = i <= a_hi ? s.C[i] - base : ~0ull;
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      int lo = 0, hi = (int)(a_hi - a_lo);
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (win[w][mid] > target) hi = mid;
        else lo = mid + 1;
      }
      a = a_lo + lo;
    } else {
      a = cdf_search(s.C, base, target, a_lo, a_hi);
    }
  } else {
    a = mine ? cdf_search(s.C, base, target, 0, hi_all) : -1;
  }
  if (j >= s.n_slots) return;
  const int zero = *g.zero_w;
  s.anc_out[j] = (zero && s.anc_old) ? s.anc_old[a] : (int32_t)a;
}

// ------------------------------------------------- multinomial on R ranks
// DESIGN.md §7.  Slot j's multinomial target T_j (its own RESAMPLE draw scaled
// by the global total: k_search's target on one rank) lies in the CDF range of
// one rank, the slot's key.  k_mn_keys writes the keys of a slot range and, per
// 256-slot block, how many of the block's slots carry each key; k_mn_pos ranks
// every slot among the earlier slots of the range with its key (stable, from
// the per-block offsets the host scans).  The rank that holds a slot's target
// sends that slot's ancestor row to the rank that owns the slot, in slot order.
struct MnArgs {
  int64_t slot_lo;          // global index of the range's first slot
  int64_t n_slots;
  uint64_t seed;
  uint32_t t;
  const uint64_t* totals;   // the R all-gathered rank totals
  int R;
  int32_t* key;             // [n_slots] the rank holding the slot's target
  int32_t* bcnt;            // [blocks][R] slots per key in each block
};
static __global__ __launch_bounds__(kBlock) void k_mn_keys(MnArgs m, const int* gate, const DevScalars* dev) {
  if (!*gate) return;
  __shared__ int hist[kMaxRanks];
  for (int k = threadIdx.x; k < m.R; k += kBlock) hist[k] = 0;
  __syncthreads();
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j < m.n_slots) {
    const u32x4 w = rng_block(m.seed, (uint64_t)(m.slot_lo + j), m.t, STREAM_RESAMPLE, 0);
    const uint64_t T = scale_u53(u53_bits(w.x, w.y), dev->S);  // < S
    uint64_t base = 0;
    int k = 0;
    for (; k < m.R - 1; ++k) {  // (an empty rank's range holds no target)
      const uint64_t nb = base + m.totals[k];
      if (T < nb) break;
      base = nb;
    }
    m.key[j] = k;
    atomicAdd(&hist[k], 1);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < m.R; k += kBlock) m.bcnt[(int64_t)blockIdx.x * m.R + k] = hist[k];
}
// pos[j] = the block's offset for key[j] + the slots of the block before j
// with that key (per wave: one ballot per distinct key of the wave)
static __global__ __launch_bounds__(kBlock) void k_mn_pos(const int32_t* key, int64_t n, const int32_t* boff, int R,
                                                         int32_t* pos, const int* gate) {
  if (!*gate) return;
  __shared__ int wcnt[kBlock / 64][kMaxRanks];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < (kBlock / 64) * kMaxRanks; i += kBlock) wcnt[i / kMaxRanks][i % kMaxRanks] = 0;
  __syncthreads();
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int k = j < n ? key[j] : -1;
  int rl = 0;
  uint64_t todo = __builtin_amdgcn_ballot_w64(k >= 0);
  while (todo) {
    const int L = __builtin_ctzll(todo);
    const int kk = __builtin_amdgcn_readlane(k, L);
    const uint64_t mk = __builtin_amdgcn_ballot_w64(k == kk);
    if (k == kk) rl = __builtin_popcountll(mk & ((1ull << lane) - 1ull));
    if (lane == 0) wcnt[w][kk] = __builtin_popcountll(mk);
    todo &= ~mk;
  }
  __syncthreads();
  if (k >= 0) {
    int before = 0;
    for (int v = 0; v < w; ++v) before += wcnt[v][k];
    pos[j] = boff[(int64_t)blockIdx.x * R + k] + before + rl;
  }
}
// sender: the slots of a range that take one of this rank's particles, in slot
// order (pos among them), with their local ancestors (k_search, own_only)
static __global__ __launch_bounds__(kBlock) void k_mn_send(const int32_t* anc, const int32_t* pos, int64_t n,
                                                          int32_t* xanc, const int* gate) {
  if (!*gate) return;
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j < n && anc[j] >= 0) xanc[pos[j]] = anc[j];
}
struct MnRecvOff {
  int32_t off[kMaxRanks];  // first received row from each rank (rows_recv in rank order)
};
// receiver: this rank's slots take a local ancestor or received row
// off[key] + pos (the slot's rank among this rank's slots with that key)
static __global__ __launch_bounds__(kBlock) void k_mn_recv(const int32_t* anc_loc, const int32_t* key,
                                                          const int32_t* pos, int64_t n, MnRecvOff ro,
                                                          int32_t* anc_out, const int* gate) {
  if (!*gate) return;
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j < n) anc_out[j] = anc_loc[j] >= 0 ? anc_loc[j] : -1 - (ro.off[key[j]] + pos[j]);
}

// ------------------------------------------------- multi-rank exchange
// Rows sent to other ranks: row j = (x[:, anc[j]], global id of anc[j]).
static __global__ __launch_bounds__(kBlock) void k_pack_rows(const int32_t* anc, int64_t rows, const double* x,
                                                      int D, int64_t lo, double* out) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= rows) return;
  const int32_t a = anc[j];
  double* r = out + j * (D + 1);
  for (int k = 0; k < D; ++k) r[k] = x[xidx(a, k, D)];
  r[D] = __longlong_as_double(lo + a);
}

// slots fed by received rows: ancestor = -1 - (row index in the receive buffer)
static __global__ void k_assign_remote(int32_t* anc, int64_t len, int64_t row0) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j < len) anc[j] = (int32_t)(-1 - (row0 + j));
}

// global parent ids of this rank's slots after an exchange
static __global__ void k_global_parents(const int32_t* anc, int64_t n, int64_t lo, const double* rows, int D,
                                 int64_t* gparent) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  const int32_t a = anc[j];
  gparent[j] = a >= 0 ? lo + a : __double_as_longlong(rows[(int64_t)(-1 - a) * (D + 1) + D]);
}

static __global__ void k_copy_anc(const int* gate, const int32_t* src, int32_t* dst, int64_t n) {
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
  int64_t n;
  int t_target, t_cur, D;
  int live;                   // the device resample flags are current
  double* out;                // [D][n]
};

static __global__ __launch_bounds__(kBlock) void k_traj(TrajArgs a, const DevScalars* dev) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= a.n) return;
  int64_t idx = j;
  if (a.live && (dev->pending | dev->fire) && a.anc_pending) idx = a.anc_pending[idx];
  for (int s = a.t_cur; s > a.t_target; --s)
    if (a.res_before[s]) idx = a.ancs[s - 1][idx];
  const double* x = a.xs[a.t_target - 1];
  for (int k = 0; k < a.D; ++k) a.out[k * a.n + j] = x[xidx(idx, k, a.D)];
}

// ------------------------------------- multi-rank genealogy (queries only)
// get_traces / the score columns / sample_unweighted_traces on R ranks
// (particle_filter.jl:31-34, 62-70): the genealogy is kept where it was made —
// each rank's per-step ancestors of its own slots (local index, or -1 - row of
// the rows it received, whose global ids and states the step's part-2 launch
// kept) — and a query walks it collectively: every step back, each rank turns
// its slots' ancestors into global parent ids, the ranks all-gather them
// (padded to `pad` per rank), and every cursor moves to its parent.  The
// position of global particle c in such an all-gather is its owner's block
// plus its local index.
__device__ __forceinline__ int64_t mr_pos(int64_t c, const int64_t* dlo, int R, int64_t N, int64_t pad, int64_t* local) {
  int r = (int)(((__int128)c * R) / N);
  while (r + 1 < R && dlo[r + 1] <= c) ++r;
  while (r > 0 && dlo[r] > c) --r;
  *local = c - dlo[r];
  return (int64_t)r * pad;
}

static __global__ void k_iota64(int64_t* out, int64_t n, int64_t lo) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j < n) out[j] = lo + j;
}

// global parent ids of this rank's slots at one step (rows: the received rows
// the slots' negative ancestors index; read at system scope: the peer
// transport's row buffer is written by other processes)
// A record that names no particle (a local index outside [0, n), a received
// row outside the nrows kept, or any received row when none were kept; nrows
// < 0: the count is not known here) raises kErrGenealogy through the filter's
// error word and the query returns GH_E_STATE — a wrong trajectory is never
// returned.  The cursor becomes -1, which every later walk kernel also reports.
static __global__ void k_mr_gparents(const int32_t* anc, int64_t n, int64_t lo, const double* rows, int64_t nrows,
                                     int D, int64_t* gp, int* err) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  const int32_t a = anc[j];
  const int64_t row = -1 - (int64_t)a;
  int64_t g = -1;
  if (a >= 0 && a < n) g = lo + a;
  else if (a < 0 && rows && (nrows < 0 || row < nrows)) g = __double_as_longlong(ld_sys(&rows[row * (D + 1) + D]));
  else *err = kErrGenealogy;
  gp[j] = g;
}

// every cursor one step back: cur = parent of the slot it names
static __global__ void k_mr_back(int64_t* cur, int64_t n, const int64_t* gp_all, const int64_t* dlo, int R, int64_t N,
                                 int64_t pad, int* err) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  if (cur[j] < 0 || cur[j] >= N) {  // (a broken walk: reported, not followed)
    *err = kErrGenealogy;
    return;
  }
  int64_t i;
  const int64_t b = mr_pos(cur[j], dlo, R, N, pad, &i);
  cur[j] = gp_all[b + i];
}

// the cursors' states from an all-gather of every rank's (wave-tiled) slot,
// rank r's at r * stride doubles: out[k * n + j]
static __global__ void k_mr_states(const int64_t* cur, int64_t n, const double* slab, int64_t stride,
                                   const int64_t* dlo, int R, int64_t N, int D, double* out, int* err) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  if (cur[j] < 0 || cur[j] >= N) {  // (the query returns GH_E_STATE, these values are not handed out)
    for (int k = 0; k < D; ++k) out[k * n + j] = NAN;
    *err = kErrGenealogy;
    return;
  }
  int64_t i;
  const int64_t r = mr_pos(cur[j], dlo, R, N, 1, &i);
  for (int k = 0; k < D; ++k) out[k * n + j] = slab[r * stride + xidx(i, k, D)];
}

// The score columns of this rank's slots at step s, as k_scores evaluates them
// along a walk through the slot: Model::score of the slot's state given its
// parent's (a local slot of step s - 1, a received row kept for step s, or the
// slot itself when no resample preceded s; unused at s = 1).  Into the
// all-gather's send block: lat at [0, pad), ob at [pad, 2 pad).
template <class Model>
__global__ __launch_bounds__(kBlock) void k_mr_slot_scores(const double* __restrict__ prm, typename Model::Params p0,
                                                           StepObs o, int s, const double* xs, const double* xprev,
                                                           const int32_t* anc, const double* rows, int64_t nrows,
                                                           int64_t n, int64_t pad, double* out, int* err) {
  constexpr int D = Model::kD;
  const typename Model::Params p = p0.rebase(prm);
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  double x[D], xp[D];
#pragma unroll
  for (int k = 0; k < D; ++k) x[k] = xs[xidx(j, k, D)];
  if (s > 1) {
    const int64_t a = anc ? anc[j] : j;
    if (a >= 0 && a < n) {
#pragma unroll
      for (int k = 0; k < D; ++k) xp[k] = xprev[xidx(a, k, D)];
    } else if (a < 0 && rows && (nrows < 0 || -1 - a < nrows)) {
#pragma unroll
      for (int k = 0; k < D; ++k) xp[k] = rows[(-1 - a) * (D + 1) + k];
    } else {  // a broken record: reported (the query returns GH_E_STATE)
#pragma unroll
      for (int k = 0; k < D; ++k) xp[k] = NAN;
      *err = kErrGenealogy;
    }
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) xp[k] = 0.0;
  }
  double lat, ob;
  Model::score(p, o, (uint32_t)s, xp, x, &lat, &ob);
  out[j] = lat;
  out[pad + j] = ob;
}

// the cursors' step-s columns from the all-gathered slot scores
static __global__ void k_mr_take_scores(const int64_t* cur, int64_t n, const double* all, const int64_t* dlo, int R,
                                        int64_t N, int64_t pad, double* lat, double* ob, int* err) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  if (cur[j] < 0 || cur[j] >= N) {  // (reported: the query returns GH_E_STATE)
    lat[j] = NAN;
    ob[j] = NAN;
    *err = kErrGenealogy;
    return;
  }
  int64_t i;
  const int64_t b = mr_pos(cur[j], dlo, R, N, 2 * pad, &i);
  lat[j] = all[b + i];
  ob[j] = all[b + pad + i];
}

// get_score: the columns summed in time order (k_scores' order)
static __global__ void k_score_total(const double* per_step, int T, int64_t n, double* total) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= n) return;
  double tot = 0.0;
  for (int s = 1; s <= T; ++s)
    tot += per_step[((int64_t)(s - 1) * 2) * n + j] + per_step[((int64_t)(s - 1) * 2 + 1) * n + j];
  total[j] = tot;
}

// sample_unweighted: prepare max / equal-weight flag from the current stats
static __global__ void k_prep_sample(DevScalars* dev, const double* stats_all, int R, int live) {
  if (threadIdx.x != 0) return;
  double M = -INFINITY;
  for (int r = 0; r < R; ++r) M = fmax(M, stats_all[3 * r]);
  dev->spend = live ? (dev->pending | dev->fire) : 0;
  dev->sM = dev->spend ? 0.0 : M;
  dev->one = 1;
}

// ------------------------------------------------------------ self tests
static __global__ void k_selftest_math(int64_t n, const double* in, double* oe, double* ol, double* os,
                                double* od) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const double x = in[i];
  oe[i] = gh_exp(x);
  ol[i] = gh_log(fabs(x));
  os[i] = sqrt(fabs(x));
  od[i] = (i & 1) ? div20(x) : x / in[(i + 1) % n];  // (odd entries: the models' a / 20)
}

// Box–Muller stages for given words: u1, r, z0, z1 per triple
static __global__ void k_selftest_boxmuller(int64_t n, const uint32_t* w, double* out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const uint32_t a = w[3 * i], b = w[3 * i + 1], c = w[3 * i + 2];
  const double u1 = one_minus_u53(a, b);
  out[4 * i] = u1;
  out[4 * i + 1] = sqrt_radius(-2.0 * gh_log_unit(u1, gh_math_tab_dev));
  double z0, z1;
  box_muller(a, b, c, &z0, &z1, gh_math_tab_dev);
  out[4 * i + 2] = z0;
  out[4 * i + 3] = z1;
}

static __global__ void k_selftest_normals(uint64_t seed, int64_t n, uint32_t step, uint32_t stream,
                                   int dim, double* out) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  // the multi-block layout of normals_n (pair p = words 3p..3p+2)
  for (int p = 0; 2 * p < dim; ++p) {
    uint32_t wd[3];
    for (int q = 0; q < 3; ++q) {
      const int k = 3 * p + q;
      const u32x4 w = rng_block(seed, (uint64_t)i, step, stream, (uint32_t)(k >> 2));
      const int r = k & 3;
      wd[q] = r == 0 ? w.x : r == 1 ? w.y : r == 2 ? w.z : w.w;
    }
    double a, b;
    box_muller(wd[0], wd[1], wd[2], &a, &b, gh_math_tab_dev);
    out[i * dim + 2 * p] = a;
    if (2 * p + 1 < dim) out[i * dim + 2 * p + 1] = b;
  }
}

}  // namespace gh
