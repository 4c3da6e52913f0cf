// gh_rank_ab.h — the batched loop's multi-rank resample on the peer transport
// in ONE launch.
//
// maybe_resample! (particle_filter.jl:189-213) on R ranks after a max-only
// step was two launches: k_rank_a2 (the global maximum through the mailboxes,
// quantisation and the weight sums, tile totals behind one grid barrier that
// only block 0 waited on, the rank record published to every rank) and
// k_rank_b (every block polls the R records, takes the decision, re-reads its
// log-weights, quantises them AGAIN, re-sums the tile totals before it, and
// writes the range marks and the rows other ranks take).  On the peer
// transport every exchange is a device-side poll, so nothing forces the
// launch boundary: k_rank_ab keeps each thread's quantised weights in
// registers from the quantisation to the marks, every block reads the tile
// totals it needs in the barrier it crosses anyway (as k_resample1 does), and
// the marks loop is k_resample1's (32-bit slots, incremental slot counts,
// exact recount near integers) on the global CDF.  The values — tile
// totals, records, decision, marks, rows — are the two-kernel path's bit for
// bit (tests/test_multirank.py peer cases against the single-rank oracle).
#pragma once
#include "gh_kernels.h"

namespace gh {

struct RankABArgs {
  RankA2Args a;  // the fold, quantisation, tile words and record (pb, amax_own, use_sh, use_rec)
  RankBArgs b;   // the decision, marks and rows (pb, use_rec, prow, amax_reset, hplan / htag, d)
};

template <int IT>
__global__ __launch_bounds__(kRsBlock, IT <= 4 ? 8 : 1) void k_rank_ab(RankABArgs args) {
  const RankA2Args& ra = args.a;
  const RankBArgs& rb = args.b;
  __shared__ double smd[32];
  __shared__ uint64_t smu[32];
  __shared__ unsigned sgen;
  __shared__ int sfail, sfire;
  __shared__ uint64_t spa[8], spb[8];
  __shared__ double spg[2][8];
  __shared__ double sM;
  __shared__ uint64_t su53, sbefore;
  __shared__ uint64_t srec[kRecWords];
  __shared__ uint64_t srecs[kPeerMaxRanks * kRecWords];
  __shared__ DevScalars sd;
  __shared__ int64_t sdst_lo[kPeerMaxRanks], sra_all[kPeerMaxRanks], srb_all[kPeerMaxRanks];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int R = ra.pb.R;
  if (threadIdx.x == 0) {
    sgen = ra.dev->bar_gen + 1;  // (read before this block publishes)
    sfail = 0;
  }
  const int64_t i0 = (int64_t)blockIdx.x * (kRsBlock * IT) + (int64_t)threadIdx.x * IT;
  double lw[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) lw[k] = (i0 + k < ra.n) ? ra.logw[i0 + k] : -INFINITY;
  // ---- the global maximum: this rank's shards (every block), published to
  // every rank by block 0, the R ranks' polled from the own mailbox
  {
    const uint64_t k0 = threadIdx.x < kAmaxShards ? ra.amax_own[threadIdx.x * kAmaxStride] : kAmaxEmpty;
    const double Ml = blk16_max1(amax_value(k0), smd);
    if (w == 0) {
      const int par = (int)(ra.use_sh & 1);
      const uint64_t* own = ra.pb.peer[ra.pb.rank];
      if (blockIdx.x == 0)
        peer_publish(ra.pb, mb_sh(R, par, ra.pb.rank), mb_sh_tag(R, par, ra.pb.rank), amax_key(Ml), 1, ra.use_sh);
      const bool ok = peer_poll(own, mb_sh_tag(R, par, 0), R, ra.use_sh, ra.pb.wait_ticks);
      uint64_t kk = ok && lane < R ? ld_sys(own + mb_sh(R, par, lane)) : kAmaxEmpty;
      kk = readlane63_u64(wave_incl_max_u64(kk));
      if (lane == 0) {
        sM = ok ? amax_value(kk) : NAN;
        if (!ok) {
          sfail = 1;
          ra.dev->error = kErrPeer;  // a rank never published
        }
      }
    }
    if (threadIdx.x == 8 * 64) {  // a non-polling wave draws the systematic offset's uniform meanwhile
      const u32x4 wr = rng_block(rb.seed, ~0ull, rb.t, STREAM_RESAMPLE, 0);
      su53 = u53_bits(wr.x, wr.y);
    }
    lds_barrier();
  }
  const double M = sM;
  const bool m_ok = M > -INFINITY && M != INFINITY && M == M;  // (uniform over every rank's grid)
  // ---- quantise the tile (the weights stay in registers for the marks), the
  // tile's sums, one tagged word each, and the grid barrier every block
  // crosses: its tile offset (the totals before it), the rank total and sums
  const double qscale = as_f64((uint64_t)(ra.shift + 1023) << 52);
  uint64_t q[IT];
  uint64_t tsum = 0, incl = 0;
  if (m_ok) {
    double s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const bool in = i0 + k < ra.n;
      const double e = in ? gh_exp_nonpos(lw[k] - M) : 0.0;
      q[k] = e == e ? f64_to_u52(e * qscale) : 0;  // = quantize_weight (k_rank_b's re-quantisation)
      tsum += q[k];
      const double ee = lw[k] != lw[k] ? lw[k] : e;  // NaN poisons the statistics
      s1 += ee;
      s2 += ee * ee;
    }
    incl = blk16_scan<true>(tsum, &s1, &s2, smu, smd);
    const uint64_t kTag = 1ull << 63;
    const uint64_t par = (sgen & 1u) ? kTag : 0ull;
    if (threadIdx.x == kRsBlock - 1) st_sc1(&ra.tsum[blockIdx.x], incl | par);
    if (threadIdx.x == 0) {
      st_sc1(&ra.ts1[blockIdx.x], (as_u64(s1) & ~kTag) | par);
      st_sc1(&ra.ts2[blockIdx.x], (as_u64(s2) & ~kTag) | par);
    }
    if (w < 8) {  // waves 0..7 poll 64 tiles each (k_resample1's barrier)
      const unsigned b = (unsigned)(w * 64 + lane);
      const bool mine = b < gridDim.x;
      uint64_t v = par, v1 = par, v2 = par;
      bool ok = !mine, timed_out = false;
      for (unsigned spins = 0;; ++spins) {  // bounded: a grid that is not co-resident errors out
        if (!ok) v = ld_sc1(&ra.tsum[b]);
        ok = ok || (v & kTag) == par;
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        if (spins == (1u << 22)) {
          timed_out = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      ok = !mine || timed_out;
      for (unsigned spins = 0;; ++spins) {
        if (!ok) {
          v1 = ld_sc1(&ra.ts1[b]);
          v2 = ld_sc1(&ra.ts2[b]);
        }
        ok = ok || ((v1 & kTag) == par && (v2 & kTag) == par);
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        if (spins == (1u << 22)) {
          timed_out = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      const uint64_t x = mine ? (v & ~kTag) : 0ull;
      const uint64_t all = wave_sum_u64(x);
      const uint64_t before = wave_sum_u64(b < blockIdx.x ? x : 0ull);
      const double g1 = wave_sum(mine ? as_f64(v1 & ~kTag) : 0.0);
      const double g2 = wave_sum(mine ? as_f64(v2 & ~kTag) : 0.0);
      if (lane == 0) {
        spa[w] = all;
        spb[w] = before;
        spg[0][w] = g1;
        spg[1][w] = g2;
        if (timed_out) sfail = 1;
      }
    }
    lds_barrier();
    if (threadIdx.x == 0) {  // (k_rank_a2's record: the same sums in the same order)
      uint64_t all = 0, before = 0;
      double g1 = 0.0, g2 = 0.0;
#pragma unroll 1
      for (int k = 0; k < 8; ++k) {  // (not unrolled: 32 LDS values at once would spill the kept weights)
        all += spa[k];
        before += spb[k];
        g1 += spg[0][k];
        g2 += spg[1][k];
      }
      if (sfail) {
        ra.dev->error = kErrBarrier;  // partial totals
        g1 = NAN;
      }
      sbefore = before;
      srec[0] = all;
      srec[1] = as_u64(g1);
      srec[2] = as_u64(g2);
      srec[3] = as_u64(M);
      if (blockIdx.x == 0) {
        ra.dev->local = all;
        ra.dev->bar_gen = sgen;  // every block has published, so has read the old value
      }
    }
  } else if (threadIdx.x == 0) {  // no tile publishes: the record carries M, the decision raises GH_E_NUMERIC
    sbefore = 0;
    srec[0] = 0;
    srec[1] = 0;
    srec[2] = 0;
    srec[3] = as_u64(M);
    if (blockIdx.x == 0) ra.dev->local = 0;
  }
  lds_barrier();
  // ---- the rank records: block 0 publishes this rank's to every mailbox,
  // every block polls the R records from its own
  if (w == 0) {
    const int par = (int)(ra.use_rec & 1);
    if (blockIdx.x == 0) {
      if (lane < kRecWords) ra.rec[lane] = srec[lane];  // (the host's copy: the plan mailbox below)
      peer_publish(ra.pb, mb_rec(R, par, ra.pb.rank), mb_rec_tag(R, par, ra.pb.rank),
                   lane < kRecWords ? srec[lane] : 0ull, kRecWords, ra.use_rec);
    }
    const uint64_t* own = ra.pb.peer[ra.pb.rank];
    const bool ok = peer_poll(own, mb_rec_tag(R, par, 0), R, ra.use_rec, ra.pb.wait_ticks);
    if (lane < R)
      for (int k = 0; k < kRecWords; ++k)
        srecs[lane * kRecWords + k] = ok ? ld_sys(own + mb_rec(R, par, lane) + k) : (k == 3 ? as_u64(NAN) : 0ull);
    if (!ok && lane == 0) {
      ra.dev->error = kErrPeer;  // a rank never published its record
      sfail = 1;
    }
    if (blockIdx.x == 0 && lane < kAmaxShards) rb.amax_reset[lane * kAmaxStride] = kAmaxEmpty;  // (read above)
  }
  lds_barrier();
  // ---- the decision from the R records (every block the same), committed by block 0
  if (threadIdx.x == 0) {
    const Decision dec = decide_records(srecs, R, rb.d.thr);
    sfire = dec.fire && !sfail;
    if (blockIdx.x == 0) {
      rb.dev->pending = 0;
      commit_decision(rb.d, dec, rb.dev, 0);
      if (rb.hplan) {  // the host's copy of the records, then the tag behind a system-scope release
        for (int k = 0; k < R * kRecWords; ++k) rb.hplan[1 + k] = srecs[k];
        __threadfence_system();
        __hip_atomic_store(&rb.hplan[0], rb.htag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  lds_barrier();
  if (!sfire) return;
  // ---- the plan (thread 0): the global systematic constants, every rank's
  // slot block and the part of it other ranks cover (the rows' layout there)
  const uint32_t N = (uint32_t)rb.mk.n_global;  // < 2^31 (host-checked): 32-bit slots
  if (threadIdx.x == 0) {
    uint64_t S = 0, base = 0;
    for (int k = 0; k < R; ++k) {
      if (k < rb.rank) base += srecs[k * kRecWords];
      S += srecs[k * kRecWords];
    }
    sd.S = S;
    sd.base = base;
    sd.local = srecs[rb.rank * kRecWords];
    sd.o = scale_u53(su53, S);
    sd.invN = rb.d.inv_n;
    sd.Qs = udiv_n(S, N, sd.invN);
    sd.Rs = S - sd.Qs * N;
    sd.invS = recip_est((double)S);
    uint64_t bk = 0;
    for (int k = 0; k < R; ++k) {
      const uint64_t tk = srecs[k * kRecWords];
      const int64_t dl = rb.dlo[k], dh = rb.dlo[k + 1];
      const int64_t lo_k = sys_count_exact(&sd, N, bk), hi_k = sys_count_exact(&sd, N, bk + tk);
      sdst_lo[k] = dl;
      sra_all[k] = (lo_k < dl ? dl : (lo_k > dh ? dh : lo_k)) - dl;
      srb_all[k] = (hi_k < dl ? dl : (hi_k > dh ? dh : hi_k)) - dl;
      bk += tk;
    }
    if (blockIdx.x == 0) {
      rb.dev->S = S;
      rb.dev->base = base;
      rb.dev->o = sd.o;
      rb.dev->Qs = sd.Qs;
      rb.dev->Rs = sd.Rs;
      rb.dev->invN = sd.invN;
      rb.dev->invS = sd.invS;
      rb.dev->ra = sra_all[rb.rank];
      rb.dev->rb = srb_all[rb.rank];
    }
  }
  lds_barrier();
  // ---- the marks (k_resample1's loop on the global CDF: incremental slot
  // counts, the exact recount near integers) clamped to this rank's slots,
  // and the rows of slots other ranks own, stored into their buffers
  // (32-bit: N < 2^31, so the clamp below is one v_med3_i32, not 64-bit compares and selects)
  const int32_t own_lo = (int32_t)rb.lo, own_hi = (int32_t)(rb.lo + rb.n);
  uint64_t run = sd.base + sbefore + incl - tsum;
  const double ns = as_f64(readfirstlane_u64(as_u64((double)N * sd.invS)));
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
  auto local = [&](int32_t s) {  // clamp to [own_lo, own_hi), local index
    return (uint32_t)(min(max(s, own_lo), own_hi) - own_lo);
  };
  int32_t s_i = count(run);
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    run += q[k];
    v = fma(u52_to_f64(q[k]), ns, v);
    const int32_t e_i = count(run);
    const uint32_t l0 = local(s_i), l1 = local(e_i);
    const uint32_t tagged = rb.mk.tag | (uint32_t)(i0 + k);
    if (l1 > l0) rb.mk.mark[l0] = tagged;
    const uint32_t g0 = (l0 + 63u) >> 6, g1 = (l1 + 63u) >> 6;  // local groups g with 64 g in [l0, l1)
    const bool many = g1 - g0 > 2u;
    if (!many) {
      if (g1 > g0) rb.mk.cmark[g0] = tagged;
      if (g1 > g0 + 1u) rb.mk.cmark[g0 + 1u] = tagged;
    }
    uint64_t bm = __builtin_amdgcn_ballot_w64(many);
    while (bm) {
      const int L = __builtin_ctzll(bm);
      bm &= bm - 1;
      const int32_t a0 = __builtin_amdgcn_readlane((int32_t)g0, L), a1 = __builtin_amdgcn_readlane((int32_t)g1, L);
      const uint32_t tg = rb.mk.tag | (uint32_t)__builtin_amdgcn_readlane((int32_t)(i0 + k), L);
      for (int32_t g = a0 + lane; g < a1; g += 64) rb.mk.cmark[g] = tg;
    }
    // slots other ranks own (only a range that crosses this rank's block edge)
    if (e_i > s_i && (s_i < own_lo || e_i > own_hi))
      send_rows_peer(s_i, e_i, i0 + k, own_lo, own_hi, R, N, sdst_lo, sra_all, srb_all, rb.prow, rb.xprev, rb.D,
                     rb.lo);
    s_i = e_i;
  }
}

}  // namespace gh
