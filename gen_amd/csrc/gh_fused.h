// gh_fused.h — maybe_resample! and particle_filter_step! in ONE launch (one
// rank, systematic resampling: the gh_pf_run loop; DESIGN.md §3 "fused step").
//
// The two-kernel step (k_resample1, then k_step) pays the resample's launch
// ramp, one dependent kernel boundary and the step kernel's own prologue on
// top of the resample's latency-bound phases.  Here one grid of 256-thread
// blocks carries both roles:
//   blocks [0, G)       the resample (G = tiles of 4096 particles, 16 per
//                       thread): fold of the previous step's block maxima,
//                       quantisation, ONE grid barrier among these G blocks,
//                       systematic range marks (sc1 stores), decision commit;
//                       then every block signals "done" on a per-XCD-sharded
//                       counter (agent-scope atomic add after its stores
//                       drained: MI355X_MICROARCH.md hand-off row "one lane of
//                       each storing workgroup ... agent-scope atomic add");
//   blocks [G, G + nb)  the step of particle_filter_step!: each copies the
//                       Box–Muller tables into LDS, waits for the counter to
//                       reach gen * G (sc1 polls of every shard), reads the
//                       fire word and its marks with sc1 loads, then runs
//                       exactly k_step's body.
// Blocks are dispatched in index order, so the G resample blocks are resident
// before any step block can hold a slot (the same co-residency k_resample1's
// barrier needs); every wait is bounded and raises GH_E_STATE instead of
// hanging.  The step blocks' table copies and launch ramp overlap the
// resample; the arithmetic is k_resample1's and k_step's, so the results are
// the same bits (the floating weight sums only change their tree).
#pragma once
#include "gh_kernels.h"

namespace gh {

constexpr int kFzIT = 16;                 // resample role: particles per thread
constexpr int kFzTile = kBlock * kFzIT;   // 4096 particles per tile
static_assert(kFzTile == kRsTile, "the fused resample shares k_resample1's tiles and tile words");
constexpr int kFzMaxTiles = 2 * kBlock;   // tile words polled two per lane by the four waves
constexpr int kFzShards = 8;              // done-counter replicas, 1 KiB apart
constexpr int kFzShardStride = 256;       // unsigned words between replicas
#ifndef GH_FZ_SLEEP
#define GH_FZ_SLEEP 16
#endif

struct FusedArgs {
  Resample1Args r;  // the resample role (tiles of kFzTile particles: G of them)
  unsigned* cnt;    // [kFzShards * kFzShardStride] cumulative done counters
  unsigned* fire;   // block 0 publishes (gen << 1) | fire
  unsigned gen;     // 1, 2, ... per fused launch of this filter
  int G;            // resample-role blocks
};

// 4-wave block helpers (results in every thread)
__device__ __forceinline__ double fz_blk_max(double v, double* sm) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_max(v);
  lds_barrier();
  if (lane == 0) sm[w] = v;
  lds_barrier();
  return fmax(fmax(sm[0], sm[1]), fmax(sm[2], sm[3]));
}

// every storing wave drains its stores, then wave 0 signals for the block:
// one atomic-add instruction whose lanes 0..7 add 1 to the eight counter
// replicas (each consumer polls one replica; MI355X_MICROARCH.md hand-off row
// "a counter kept in R replicas"); block 0 first publishes the decision word
__device__ __forceinline__ void fz_signal(const FusedArgs& f, int fire) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  lds_barrier();
  if (threadIdx.x < 64) {
    if (blockIdx.x == 0) {
      if (threadIdx.x == 0) st_sc1(f.fire, (f.gen << 1) | (unsigned)(fire ? 1 : 0));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (threadIdx.x < kFzShards)
      __hip_atomic_fetch_add(&f.cnt[threadIdx.x * kFzShardStride], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// sys_count (gh_kernels.h) without branches: the same exact count
// #{j : T_j < X} = clamp(ceil(v), 0, N), v = (X N - o) / S.  Away from an
// integer (|v - rint v| > 2^-16) ceil(v) of the estimate is exact (sys_count's
// error bound); near one the count is m or m + 1 for m = rint(v), and one
// target T_m = m Qs + floor((m Rs + o) / N) decides which (count <= m iff
// T_m >= X).  The quotient's double estimate is within one of the truth
// (m Rs + o < 2^63, quotient < 2^44 for N <= 2^21), so one correction is exact.
__device__ __forceinline__ int32_t fz_count(const DevScalars* d, uint64_t N, uint64_t X) {
  const double v = fma((double)X, (double)N, -(double)d->o) * d->invS;
  const double m = rint(v);
  const bool near = fabs(v - m) <= 0x1p-16;
  const int64_t mc = (int64_t)fmin(fmax(m, 0.0), (double)(N - 1));
  const uint64_t num = (uint64_t)mc * d->Rs + d->o;
  uint64_t qd = (uint64_t)((double)num * d->invN);
  const int64_t rr = (int64_t)(num - qd * N);
  qd = rr < 0 ? qd - 1 : (rr >= (int64_t)N ? qd + 1 : qd);
  const uint64_t T = (uint64_t)mc * d->Qs + qd;
  const int64_t ex = T >= X ? mc : mc + 1;
  const int64_t fast = (int64_t)fmin(fmax(ceil(v), 0.0), (double)N);
  const int64_t c = near ? ex : fast;
  return (int32_t)(X == 0 ? 0 : (X >= d->S ? (int64_t)N : c));
}

// The resample role: k_resample1<true, ., SUMS> for 256-thread blocks with 16
// particles per thread (same tiles, same tile words and barrier generation).
__device__ __forceinline__ void fz_resample(const FusedArgs& f) {
  const Resample1Args& r = f.r;
  __shared__ double fsm[8];
  __shared__ uint64_t fsu[4];
  __shared__ DevScalars fsd;
  __shared__ uint64_t fbase;
  __shared__ unsigned fgen;
  __shared__ int ffire, ffail;
  __shared__ double fS[2];
  __shared__ uint64_t fpa[4], fpb[4];
  __shared__ double fpg[2][4];
  // the resample is the critical path: its waves issue ahead of the step
  // blocks sharing the CU
  __builtin_amdgcn_s_setprio(3);
  GH_RS_STAMP(0);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    fgen = r.dev->bar_gen + 1;
    ffail = 0;
  }
  const bool sums = r.sums_in_pass != 0;
  // this thread's 16 log-weights (the array is padded to whole tiles), loaded
  // beside the step partials
  const int64_t i0 = (int64_t)blockIdx.x * kFzTile + (int64_t)threadIdx.x * kFzIT;
  double lw[kFzIT];
  {
    const double2* p2 = reinterpret_cast<const double2*>(r.logw + i0);
#pragma unroll
    for (int k = 0; k < kFzIT / 2; ++k) {
      const double2 v = p2[k];
      lw[2 * k] = v.x;
      lw[2 * k + 1] = v.y;
    }
  }
  double m = -INFINITY;
  if (r.nb_part <= 16 * kBlock) {
    double pmv[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int b = threadIdx.x + k * kBlock;
      pmv[k] = b < r.nb_part ? r.pm[b] : -INFINITY;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) m = fmax(m, pmv[k]);
  } else {
    for (int b = threadIdx.x; b < r.nb_part; b += kBlock) m = fmax(m, r.pm[b]);
  }
#pragma unroll
  for (int k = 0; k < kFzIT; ++k)
    if (i0 + k >= r.n) lw[k] = -INFINITY;
  const double M = fz_blk_max(m, fsm);
  GH_RS_STAMP(7);
  const bool m_ok = M > -INFINITY && M != INFINITY && M == M;
  double S1 = 0.0, S2 = 0.0;
  if (!sums) {  // the step wrote full partials: the sums come from them (second, cache-hot pass)
    double s1 = 0.0, s2 = 0.0;
    if (m_ok)
      for (int b = threadIdx.x; b < r.nb_part; b += kBlock) {
        const double mb = r.pm[b];
        if (mb > -INFINITY) {
          const double e = gh_exp(mb - M);
          s1 += r.ps[b] * e;
          s2 += r.ps2[b] * (e * e);
        }
      }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    lds_barrier();
    if (lane == 0) {
      fsm[w] = s1;
      fsm[4 + w] = s2;
    }
    lds_barrier();
    S1 = (fsm[0] + fsm[1]) + (fsm[2] + fsm[3]);
    S2 = (fsm[4] + fsm[5]) + (fsm[6] + fsm[7]);
    if (threadIdx.x == 0) ffire = m_ok && ((S1 * S1) / S2 < r.d.thr);
    lds_barrier();
  }
  auto commit = [&]() {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      double st[3] = {M, S1, S2};
      DecideArgs d = r.d;
      d.stats_all = st;
      d.R = 1;
      const Decision dec = decide(d, false);
      r.stats_out[0] = M;
      r.stats_out[1] = S1;
      r.stats_out[2] = S2;
      r.dev->pending = 0;
      commit_decision(r.d, dec, r.dev, 0);
    }
  };
  if (sums ? !m_ok : !ffire) {  // uniform over the role: nobody publishes
    commit();
    fz_signal(f, 0);
    return;
  }
  GH_RS_STAMP(1);
  // ---- quantise this tile (e = exp(w - M) also feeds the tile sums)
  const double qscale = as_f64((uint64_t)(r.shift + 1023) << 52);
  // the quantised weights are parked in r.C (this thread's own 128 bytes,
  // L2-resident) across the barrier instead of 32 registers, and read back
  // while the block's systematic constants are computed
  uint64_t tsum = 0;
  double s1 = 0.0, s2 = 0.0;
  ulonglong2* qp = reinterpret_cast<ulonglong2*>(r.C + i0);
#pragma unroll
  for (int k = 0; k < kFzIT; k += 2) {
    uint64_t qq[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const double e = gh_exp_nonpos(lw[k + h] - M);  // slots past n hold -inf: e = 0
      qq[h] = e == e ? f64_to_u52(e * qscale) : 0;
      tsum += qq[h];
      if (sums) {
        const double ee = lw[k + h] != lw[k + h] ? lw[k + h] : e;  // NaN poisons the statistics
        s1 += ee;
        s2 += ee * ee;
      }
    }
    qp[k / 2] = make_ulonglong2(qq[0], qq[1]);
  }
  // block scan of the thread totals over the four waves
  uint64_t v = wave_incl_sum_u64(tsum);
  const double ws1 = sums ? wave_sum(s1) : 0.0, ws2 = sums ? wave_sum(s2) : 0.0;
  lds_barrier();
  if (lane == 63) fsu[w] = v;
  if (lane == 0) {
    fsm[w] = ws1;
    fsm[4 + w] = ws2;
  }
  lds_barrier();
  const uint64_t t0 = fsu[0], t1 = fsu[1], t2 = fsu[2], t3 = fsu[3];
  v += (w > 0 ? t0 : 0ull) + (w > 1 ? t1 : 0ull) + (w > 2 ? t2 : 0ull);
  const uint64_t incl = v;
  GH_RS_STAMP(2);
  // ---- grid barrier among the G resample blocks (k_resample1's protocol:
  // tagged tile words, parity of the barrier generation in bit 63)
  const uint64_t kTag = 1ull << 63;
  const uint64_t par = (fgen & 1u) ? kTag : 0ull;
  if (threadIdx.x == 0) {
    const uint64_t total = ((t0 + t1) + t2) + t3;
    const double b1 = (fsm[0] + fsm[1]) + (fsm[2] + fsm[3]);
    const double b2 = (fsm[4] + fsm[5]) + (fsm[6] + fsm[7]);
    st_sc1(&r.tsum[blockIdx.x], total | par);
    st_sc1(&r.ts1[blockIdx.x], (as_u64(b1) & ~kTag) | par);
    st_sc1(&r.ts2[blockIdx.x], (as_u64(b2) & ~kTag) | par);
  }
  {
    const unsigned ba = (unsigned)(w * 64 + lane), bb = ba + 4u * 64u;
    const bool ma = ba < (unsigned)f.G, mb = bb < (unsigned)f.G;
    uint64_t va = par, va1 = par, va2 = par, vb = par, vb1 = par, vb2 = par;
    bool oka = !ma, okb = !mb;
    for (unsigned spins = 0;; ++spins) {  // bounded (~0.5 s)
      if (!oka) {
        va = ld_sc1(&r.tsum[ba]);
        if (sums) {
          va1 = ld_sc1(&r.ts1[ba]);
          va2 = ld_sc1(&r.ts2[ba]);
        }
      }
      if (!okb) {
        vb = ld_sc1(&r.tsum[bb]);
        if (sums) {
          vb1 = ld_sc1(&r.ts1[bb]);
          vb2 = ld_sc1(&r.ts2[bb]);
        }
      }
      oka = oka || ((va & kTag) == par && (va1 & kTag) == par && (va2 & kTag) == par);
      okb = okb || ((vb & kTag) == par && (vb1 & kTag) == par && (vb2 & kTag) == par);
      if (__builtin_amdgcn_ballot_w64(!(oka && okb)) == 0) break;
      if (spins == (1u << 22)) {
        r.dev->error = 7;  // GH_E_STATE: the role's blocks were not co-resident
        ffail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const uint64_t xa = ma ? (va & ~kTag) : 0ull, xb = mb ? (vb & ~kTag) : 0ull;
    const uint64_t all = wave_sum_u64(xa + xb);
    const uint64_t before = wave_sum_u64((ba < blockIdx.x ? xa : 0ull) + (bb < blockIdx.x ? xb : 0ull));
    double g1 = 0.0, g2 = 0.0;
    if (sums) {
      g1 = wave_sum((ma ? as_f64(va1 & ~kTag) : 0.0) + (mb ? as_f64(vb1 & ~kTag) : 0.0));
      g2 = wave_sum((ma ? as_f64(va2 & ~kTag) : 0.0) + (mb ? as_f64(vb2 & ~kTag) : 0.0));
    }
    if (lane == 0) {
      fpa[w] = all;
      fpb[w] = before;
      fpg[0][w] = g1;
      fpg[1][w] = g2;
    }
  }
  GH_RS_STAMP(3);
  // the quantised weights back from their parking (they land while thread 0
  // derives the systematic constants)
  uint64_t q[kFzIT];
#pragma unroll
  for (int k = 0; k < kFzIT; k += 2) {
    const ulonglong2 v2 = qp[k / 2];
    q[k] = v2.x;
    q[k + 1] = v2.y;
  }
  lds_barrier();
  if (threadIdx.x == 0) {
    const u32x4 wr = rng_block(r.seed, ~0ull, r.t, STREAM_RESAMPLE, 0);
    const uint64_t all = ((fpa[0] + fpa[1]) + fpa[2]) + fpa[3];
    const uint64_t before = ((fpb[0] + fpb[1]) + fpb[2]) + fpb[3];
    if (sums) {
      const double g1 = (fpg[0][0] + fpg[0][1]) + (fpg[0][2] + fpg[0][3]);
      const double g2 = (fpg[1][0] + fpg[1][1]) + (fpg[1][2] + fpg[1][3]);
      fS[0] = g1;
      fS[1] = g2;
      ffire = (g1 * g1) / g2 < r.d.thr;
    }
    const uint64_t N = (uint64_t)r.d.n_global;
    fsd.S = all;
    fsd.base = 0;
    fsd.local = all;
    fsd.o = scale_u53(u53_bits(wr.x, wr.y), all);
    fsd.invN = r.d.inv_n;
    fsd.Qs = udiv_n(all, N, fsd.invN);
    fsd.Rs = all - fsd.Qs * N;
    fsd.invS = recip_est((double)all);
    fbase = before;
    if (blockIdx.x == 0) {
      r.dev->bar_gen = fgen;  // every role block has published, so has read the old value
      r.dev->S = fsd.S;
      r.dev->base = 0;
      r.dev->local = fsd.local;
      r.dev->o = fsd.o;
      r.dev->Qs = fsd.Qs;
      r.dev->Rs = fsd.Rs;
      r.dev->invN = fsd.invN;
      r.dev->invS = fsd.invS;
    }
  }
  lds_barrier();
  if (ffail) {  // partial totals: no marks; the error surfaces at the next sync
    fz_signal(f, 0);
    return;
  }
  if (sums) {
    S1 = fS[0];
    S2 = fS[1];
    if (!ffire) {
      commit();
      fz_signal(f, 0);
      return;
    }
  }
  // ---- systematic range marks (k_resample1's), stored sc1 for the step
  // blocks of this launch; a particle with more than two 64-slot group starts
  // in its range gets its carries from the whole wave
  GH_RS_STAMP(4);
  uint64_t run = fbase + incl - tsum;
  const uint64_t N = (uint64_t)r.mk.n_global;
  // slot-range ends of the 16 particles first (registers: the q die as the
  // ends are born), then every mark and carry store — no load waits behind
  // the write-through stores
  const int32_t s0 = fz_count(&fsd, N, run);
  int32_t e[kFzIT];
#pragma unroll
  for (int k = 0; k < kFzIT; ++k) {
    run += q[k];
    const int32_t prev = k ? e[k - 1] : s0;
    e[k] = (i0 + k < r.n && q[k]) ? fz_count(&fsd, N, run) : prev;
    __builtin_amdgcn_sched_barrier(0);  // one count at a time (registers)
  }
  int32_t s_i = s0;
#pragma unroll
  for (int k = 0; k < kFzIT; ++k) {
    const int32_t e_i = e[k];
    const uint64_t tagged = (r.mk.epoch << 32) | (uint64_t)(i0 + k);
    if (e_i > s_i) st_sc1(&r.mk.mark[s_i], tagged);
    const int32_t g0 = (s_i + 63) >> 6, g1 = (e_i + 63) >> 6;  // groups g with 64 g in [s_i, e_i)
    const bool many = g1 - g0 > 2;
    if (!many) {
      if (g1 > g0) st_sc1(&r.mk.cmark[g0], tagged);
      if (g1 > g0 + 1) st_sc1(&r.mk.cmark[g0 + 1], tagged);
    }
    uint64_t bm = __builtin_amdgcn_ballot_w64(many);
    while (bm) {  // rare: one wave-wide loop per such particle
      const int L = __builtin_ctzll(bm);
      bm &= bm - 1;
      const int32_t a0 = __builtin_amdgcn_readlane(g0, L), a1 = __builtin_amdgcn_readlane(g1, L);
      const uint64_t tg = (r.mk.epoch << 32) | (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(i0 + k), L);
      for (int32_t g = a0 + lane; g < a1; g += 64) st_sc1(&r.mk.cmark[g], tg);
    }
    s_i = e_i;
  }
  GH_RS_STAMP(5);
  commit();
  fz_signal(f, 1);
  GH_RS_STAMP(6);
}

// The step blocks' wait: lane 0 polls one counter replica (sc1) until the
// resample role's G blocks have all signalled in this launch's generation,
// then reads the decision word; the other waves wait at the block barrier.
// Returns the decision (0 after a timeout, with GH_E_STATE raised).
__device__ __forceinline__ int fz_wait(const FusedArgs& f, DevScalars* dev, int vb, int* sflag) {
  if (threadIdx.x == 0) {
    const unsigned target = f.gen * (unsigned)f.G;  // cumulative over launches (mod 2^32)
    const unsigned* c = &f.cnt[(vb & (kFzShards - 1)) * kFzShardStride];
    bool ok = false;
    for (unsigned spins = 0;; ++spins) {
      if (ld_sc1(c) == target) {
        ok = true;
        break;
      }
      if (spins == (1u << 20)) {
        dev->error = 7;  // GH_E_STATE
        break;
      }
      __builtin_amdgcn_s_sleep(GH_FZ_SLEEP);
    }
    const unsigned fw = ok ? ld_sc1(f.fire) : 0u;
    *sflag = (ok && (fw >> 1) == f.gen) ? (int)(fw & 1u) : 0;
  }
  lds_barrier();
  return *sflag;
}

// The step role: k_step<Model, false>'s body after the wait (one rank,
// systematic marks, weights reset iff the resample fired).
template <class Model>
__device__ __forceinline__ void fz_step(const double* __restrict__ prm, const typename Model::Params& p0,
                                        const StepObs& o, const StepArgs& a, const FusedArgs& f) {
  constexpr int D = Model::kD;
  const typename Model::Params p = p0.rebase(prm);
  __shared__ double sm[3][4];
  __shared__ double logtab[kMathTabDoubles];
  __shared__ int sflag;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t vb = (int64_t)blockIdx.x - f.G;
  const int64_t tile = vb * (kBlock / 64) + w;
  const int64_t j = tile * 64 + lane;
  GH_RS_STAMP(0);
  load_math_tab256(logtab);
  const int fire = fz_wait(f, a.dev, (int)vb, &sflag);
  GH_RS_STAMP(2);
#if defined(GH_FZ_STEPSKIP)  // timing-only variant: the resample role and the wait alone
  return;
#endif
  uint64_t mv = 0, cv = 0;
  if (fire) {
    const int64_t last = a.n > 0 ? a.n - 1 : 0;
    mv = ld_sc1(&a.mark[j < last ? j : last]);
    cv = ld_sc1(&a.carry[tile < (last >> 6) ? tile : (last >> 6)]);
  }
  asm volatile("" : "+v"(mv), "+v"(cv));
  const Draw dr_step{STREAM_STEP, 0, logtab};
  double lw = -INFINITY;
  if (tile * 64 < a.n) {  // wave-uniform
    int64_t src = j;
    if (fire) {
      uint64_t v = j < a.n ? mv : 0;
      v = wave_incl_max_u64(v > cv ? v : cv);
      src = (int64_t)(uint32_t)v;
      if (j < a.n) a.anc[j] = (int32_t)src;  // genealogy record
    }
    if (j < a.n) {
      double x[D], xp[D];
      const __amdgpu_buffer_rsrc_t rp = gh_rsrc(a.xprev);
      const uint32_t tb = ((uint32_t)src >> 6) * (uint32_t)(kTileP * D * 8), l = (uint32_t)src & 63u;
#pragma unroll
      for (int c = 0; c < D / 2; ++c) buf_ld_f64x2(rp, tb + l * 16u, (uint32_t)(c * kTileP * 16), &xp[2 * c]);
      if (D & 1) xp[D - 1] = buf_ld_f64(rp, tb + l * 8u, (uint32_t)((D - 1) * kTileP * 8));
      const double inc = Model::step(p, o, a.seed, (uint64_t)(a.lo + j), a.t, a.proposal, xp, x, dr_step);
      lw = (fire ? 0.0 : a.logw[j]) + inc;
      const __amdgpu_buffer_rsrc_t ro = gh_rsrc(a.xout);
      const uint32_t tbo = (uint32_t)tile * (uint32_t)(kTileP * D * 8);
#pragma unroll
      for (int c = 0; c < D / 2; ++c) buf_st_f64x2(&x[2 * c], ro, tbo + (uint32_t)lane * 16u, (uint32_t)(c * kTileP * 16));
      if (D & 1) buf_st_f64(x[D - 1], ro, tbo + (uint32_t)lane * 8u, (uint32_t)((D - 1) * kTileP * 8));
      a.logw[j] = lw;
    }
  }
  if (a.max_only) block_max_partial(lw, sm, a.pm + vb);
  else block_partial(lw, sm, a.pm + vb, a.ps + vb, a.ps2 + vb);
  GH_RS_STAMP(6);
}

// The step role for pair-stepped one-dimensional models (k_step_pairs' body).
template <class Model>
__device__ __forceinline__ void fz_step_pairs(const double* __restrict__ prm, const typename Model::Params& p0,
                                              const StepObs& o, const StepArgs& a, const FusedArgs& f) {
  const typename Model::Params p = p0.rebase(prm);
  __shared__ double sm[3][4];
  __shared__ double logtab[kMathTabDoubles];
  __shared__ int sflag;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t vb = (int64_t)blockIdx.x - f.G;
  const int64_t tile0 = (vb * (kBlock / 64) + w) * 2;
  const int64_t j0 = tile0 * 64 + lane, j1 = j0 + 64;
  GH_RS_STAMP(0);
  load_math_tab256(logtab);
  const int fire = fz_wait(f, a.dev, (int)vb, &sflag);
  GH_RS_STAMP(2);
  uint64_t mv0 = 0, mv1 = 0, cv0 = 0, cv1 = 0;
  if (fire) {
    const int64_t last = a.n > 0 ? a.n - 1 : 0, lt = last >> 6;
    mv0 = ld_sc1(&a.mark[j0 < last ? j0 : last]);
    mv1 = ld_sc1(&a.mark[j1 < last ? j1 : last]);
    cv0 = ld_sc1(&a.carry[tile0 < lt ? tile0 : lt]);
    cv1 = ld_sc1(&a.carry[tile0 + 1 < lt ? tile0 + 1 : lt]);
  }
  asm volatile("" : "+v"(mv0), "+v"(cv0), "+v"(mv1), "+v"(cv1));
  const Draw dr_step{STREAM_STEP, 0, logtab};
  double lw0 = -INFINITY, lw1 = -INFINITY;
  if (tile0 * 64 < a.n) {  // wave-uniform
    const bool has1 = j1 < a.n;
    int64_t s0 = j0, s1 = j1;
    if (fire) {
      uint64_t v0 = j0 < a.n ? mv0 : 0, v1 = has1 ? mv1 : 0;
      v0 = wave_incl_max_u64(v0 > cv0 ? v0 : cv0);
      v1 = wave_incl_max_u64(v1 > cv1 ? v1 : cv1);
      s0 = (int64_t)(uint32_t)v0;
      s1 = (int64_t)(uint32_t)v1;
      if (j0 < a.n) a.anc[j0] = (int32_t)s0;
      if (has1) a.anc[j1] = (int32_t)s1;
    }
    if (j0 < a.n) {
      const uint64_t g0 = (uint64_t)(a.lo + j0);
      double x0, x1, w0, w1;
      if (!has1) s1 = s0;
      Model::step2(p, o, a.seed, g0, a.t, a.xprev[s0], a.xprev[s1], &x0, &x1, &w0, &w1, dr_step);
      w0 = (fire ? 0.0 : a.logw[j0]) + w0;
      if (has1) w1 = (fire ? 0.0 : a.logw[j1]) + w1;
      a.xout[j0] = x0;
      a.logw[j0] = w0;
      lw0 = w0;
      if (has1) {
        a.xout[j1] = x1;
        a.logw[j1] = w1;
        lw1 = w1;
      }
    }
  }
  if (a.max_only) block_max_partial(fmax(lw0, lw1), sm, a.pm + vb);
  else block_partial2(lw0, lw1, sm, a.pm + vb, a.ps + vb, a.ps2 + vb);
}

// occupancy: the step family's target, at most 7 waves per SIMD (72 VGPRs:
// what the resample role needs without spilling)
template <class Model, bool PAIRS>
__global__ __launch_bounds__(kBlock, Model::kMinWaves < 7 ? Model::kMinWaves : 7) void k_fused(const double* __restrict__ prm,
                                                                     typename Model::Params p0, StepObs o,
                                                                     StepArgs a, FusedArgs f) {
  if ((int)blockIdx.x < f.G) {
    fz_resample(f);
    return;
  }
  if constexpr (PAIRS) fz_step_pairs<Model>(prm, p0, o, a, f);
  else fz_step<Model>(prm, p0, o, a, f);
}

}  // namespace gh
