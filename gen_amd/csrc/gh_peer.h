// gh_peer.h — the peer transport of the multi-rank filter (DESIGN.md §7,
// gh_ctx_create_peer): ranks exchange through device memory they map from
// each other (IPC handles swapped once over the user's host transport), with
// tagged words and bounded polls instead of collective calls.
//
// Every rank owns a mailbox of fine-grained device memory; the others write
// into it with system-scope stores and then a tag, the owner polls its own
// mailbox.  The regions below are used in the same order on every rank
// (every rank posts the same sequence of operations, as with RCCL), each
// with its own use counter: a use writes slot [use & 1][sender] and tags it
// with the use count, so two uses in flight never share a slot — a rank can
// be at most one use ahead of another (it cannot finish use k + 1 before
// every rank has published use k + 1, i.e. consumed use k).
//
//   SH   k_rank_a2's rank maxima (one order key per rank) — its global max
//   REC  k_rank_a2's rank records (kRecWords per rank) — read by k_rank_b
//   AG   small all-gathers (the (M, S, S2) triples, the rank totals)
//
// The resample's state rows go straight into the receiving filter's row
// buffer (fine-grained, mapped by every rank), behind one tag per sender
// at its end (k_peer_signal / k_peer_wait).  Every wait is bounded and
// raises GH_E_STATE through the filter's device error word.
#pragma once
#include "gh_kernels.h"

namespace gh {

// (the mailbox layout, PeerBox and the poll / publish primitives are in
// gh_kernels.h, beside k_rank_a2 and k_rank_b, which use them too)

// Small all-gather (payload <= kAgWords words per rank): one wave publishes
// this rank's words to every mailbox, polls its own for every rank's tag and
// copies the R slots to recv (rank-major, as ncclAllGather).
static __global__ __launch_bounds__(64) void k_peer_allgather(const uint64_t* send, uint64_t* recv, int words,
                                                              PeerBox pb, uint64_t use, int* err) {
  const int lane = threadIdx.x & 63;
  const int par = (int)(use & 1);
  peer_publish(pb, mb_ag(pb.R, par, pb.rank), mb_ag_tag(pb.R, par, pb.rank), lane < words ? send[lane] : 0ull, words,
               use);
  const uint64_t* own = pb.peer[pb.rank];
  if (!peer_poll(own, mb_ag_tag(pb.R, par, 0), pb.R, use, pb.wait_ticks)) {
    if (lane == 0) *err = kErrPeer;  // GH_E_STATE
    return;
  }
  for (int r = 0; r < pb.R; ++r)
    if (lane < words) recv[r * words + lane] = ld_sys(own + mb_ag(pb.R, par, r) + lane);
}

// The state rows of one resample are in the receivers' buffers (the previous
// kernel on this stream, k_rank_b, stored them): tag every other rank's row
// buffer with this exchange's count.
struct PeerRowTags {
  uint64_t* tag[kPeerMaxRanks];  // rank q's row-tag words (R of them, indexed by sender), as mapped here
  int R, rank;
};
static __global__ __launch_bounds__(64) void k_peer_signal(PeerRowTags pt, uint64_t use) {
  const int lane = threadIdx.x & 63;
  __threadfence_system();
  if (lane < pt.R && lane != pt.rank) st_sys(pt.tag[lane] + pt.rank, use);
}
// ... and wait for every other rank's tag in the own row buffer
static __global__ __launch_bounds__(64) void k_peer_wait(const uint64_t* own_tags, int R, int rank, uint64_t use,
                                                         uint64_t ticks, int* err) {
  if (!peer_poll(own_tags, 0, R, use, ticks, rank) && (threadIdx.x & 63) == 0) *err = kErrPeer;
}

}  // namespace gh
