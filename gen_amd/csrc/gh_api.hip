// gh_api.hip — host side of libgen_hip.so: the C ABI declared in
// include/gen_hip.h, implemented over the kernels in gh_kernels.h.
//
// Mirrors the reference's ParticleFilterState machine
// (src/inference/particle_filter.jl:18-216): init -> {maybe_resample!, step!}*
// -> log_ml_estimate, with every per-particle loop moved to the device and
// every decision (ESS test, resample) kept device-resident so that a whole
// filter can be enqueued without a host round trip.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/gen_hip.h"
#include "gh_kernels.h"
#include "gh_pmmh.h"
#include "gh_coal.h"
#include "gh_scores.h"
#include "gh_simulate.h"
#include "gh_dists.h"
#include "gh_rejuv.h"
#include "gh_csmc.h"
#include "gh_inst.h"
#include "gh_peer.h"
#include "gh_rank_ab.h"

using namespace gh;

// LG-SSM kernels come from gh_inst_lg*.hip (parallel build units)
GH_LG_UNIT0(GH_EXTERN_TEMPLATE)
GH_LG_UNIT1(GH_EXTERN_TEMPLATE)
GH_LG_UNIT2(GH_EXTERN_TEMPLATE)
GH_LG_UNIT3(GH_EXTERN_TEMPLATE)
GH_LG_UNIT4(GH_EXTERN_TEMPLATE)
GH_LG_UNIT5(GH_EXTERN_TEMPLATE)
GH_LG_UNIT6(GH_EXTERN_TEMPLATE)
GH_SL_UNIT0(GH_EXTERN_TEMPLATE)
GH_SL_UNIT1(GH_EXTERN_TEMPLATE)
GH_SL_UNIT2(GH_EXTERN_TEMPLATE)
GH_SL_UNIT3(GH_EXTERN_TEMPLATE)
GH_SL_UNIT4(GH_EXTERN_TEMPLATE)
GH_SL_UNIT5(GH_EXTERN_TEMPLATE)
GH_SL_UNIT6(GH_EXTERN_TEMPLATE)
GH_SL_UNIT7(GH_EXTERN_TEMPLATE)

// ------------------------------------------------------------------ errors
static thread_local std::string g_err;

static int set_err(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

// message for a status the device raised (DevScalars::error)
// (the low byte is the gh_status, the byte above it the cause: kErr* in gh_kernels.h)
static const char* dev_error_msg(int code) {
  switch (code) {
    case GH_E_NUMERIC: return "maybe_resample: all log-weights are -Inf or NaN";
    case kErrBarrier:
      return "resample grid barrier timed out: its blocks were not co-resident (the device is running other "
             "kernels); this filter's state is no longer valid";
    case kErrGenealogy:
      return "genealogy walk met a broken record (an ancestor that names no particle or no kept row); this "
             "filter's state is no longer valid";
    case kErrPeer:
      return "peer transport: another rank did not publish within the wait bound (gh_ctx_set_peer_timeout); "
             "this filter's state is no longer valid";
    default: return "error raised on the device";
  }
}
// a device-raised error as the call's status
static int dev_fail(int code) { return set_err(code & 0xff, "%s", dev_error_msg(code)); }

#define HIP_TRY(x)                                                                       \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) return set_err(GH_E_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

#define NCCL_TRY(x)                                                                           \
  do {                                                                                        \
    ncclResult_t r_ = (x);                                                                    \
    if (r_ != ncclSuccess) return set_err(GH_E_RCCL, "%s: %s", #x, ncclGetErrorString(r_));   \
  } while (0)

#define CHECK(x)            \
  do {                      \
    int rc_ = (x);          \
    if (rc_ != GH_OK) return rc_; \
  } while (0)

extern "C" const char* gh_last_error(void) { return g_err.c_str(); }
extern "C" const char* gh_version(void) { return "gen_hip 0.1.0 (gfx950)"; }

// --------------------------------------------------------------- context
struct gh_ctx {
  int device = 0;
  int cus = 256;  // compute units
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int rank = 0, world = 1;
  ncclComm_t comm = nullptr;
  // host-staged transport (gh_ctx_create_hostcomm)
  bool host_comm = false;
  gh_host_comm hc{};
  char* stage = nullptr;  // pinned staging buffer
  size_t stage_bytes = 0;
  // gh_ctx_force_multirank: filters take the multi-rank path even at world 1
  // (a one-rank RCCL communicator; tests and timing on a one-GPU box)
  bool force_multi = false;
  int n_filters = 0;  // live filters (their buffers follow the path chosen at their creation)
  // peer transport (gh_ctx_create_peer, gh_peer.h): every rank's mailbox as
  // mapped here (mpeer[rank] = mbox, the own one, fine-grained), the
  // bootstrap callbacks (hc; setup only) and each region's use counter
  bool peer = false;
  uint64_t* mbox = nullptr;
  uint64_t* mpeer[kPeerMaxRanks] = {};
  uint64_t use_sh = 0, use_rec = 0, use_ag = 0;
  uint64_t peer_wait_ticks = 0;  // bound of every device wait on a peer (wall-clock ticks)
  int wall_khz = 100000;         // the device wall clock's rate (hipDeviceAttributeWallClockRate)
};

static PeerBox peer_box(const gh_ctx* c) {
  PeerBox pb{};
  for (int r = 0; r < c->world; ++r) pb.peer[r] = c->mpeer[r];
  pb.R = c->world;
  pb.rank = c->rank;
  pb.wait_ticks = c->peer_wait_ticks;
  return pb;
}

// The peer transport's bootstrap rounds (the user's host all-gather) are
// fail-together: every rank takes part in every round of a collective set-up
// whatever happened locally, each round carries the sender's ok flag, and a
// round in which any rank failed ends the set-up on every rank at that round
// (no rank is left waiting in a later collective).  PeerRounds counts the
// rounds a set-up has completed; peer_abort runs the next one with a failed
// flag.
struct PeerRounds {
  int next = 0;      // rounds completed
  bool over = false;  // a round reported a failure (or the set-up finished)
};
static int peer_round(gh_ctx* c, PeerRounds& pr, bool ok, const void* payload, size_t plen, std::vector<uint8_t>* all) {
  const size_t rec = plen + 8;
  std::vector<uint8_t> send(rec, 0), recv(rec * (size_t)c->world, 0);
  if (payload && plen) memcpy(send.data(), payload, plen);
  send[plen] = ok ? 1 : 0;
  const int rc = c->hc.allgather(c->hc.user, send.data(), recv.data(), rec);
  pr.next++;
  if (rc) {
    pr.over = true;
    return set_err(GH_E_RCCL, "peer transport: bootstrap allgather failed");
  }
  int bad = -1;
  for (int r = 0; r < c->world; ++r)
    if (!recv[rec * (size_t)r + plen]) bad = r;
  if (bad >= 0) {
    pr.over = true;
    return ok ? set_err(GH_E_STATE, "peer transport: rank %d failed its part of a collective set-up", bad) : GH_E_STATE;
  }
  if (all) {
    all->resize(plen * (size_t)c->world);
    for (int r = 0; r < c->world; ++r) memcpy(all->data() + plen * (size_t)r, recv.data() + rec * (size_t)r, plen);
  }
  return GH_OK;
}
static void peer_abort(gh_ctx* c, PeerRounds& pr) {
  if (pr.over) return;
  peer_round(c, pr, false, nullptr, 0, nullptr);
  pr.over = true;
}

static void ipc_close(const gh_ctx* c, void* const* mapped) {
  for (int r = 0; r < c->world; ++r)
    if (r != c->rank && mapped[r]) {
      hipIpcCloseMemHandle(mapped[r]);
    }
}

// Bootstrap exchange of IPC handles (two rounds: the handles, then whether
// every rank mapped every other's): map every other rank's buffer (out[rank]
// = own).  Fails on every rank or on none; on failure nothing stays mapped.
static int ipc_exchange(gh_ctx* c, PeerRounds& pr, void* own, void** out) {
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle size");
  for (int r = 0; r < c->world; ++r) out[r] = nullptr;
  uint8_t hbuf[64] = {};
  hipIpcMemHandle_t h;
  const bool got = hipIpcGetMemHandle(&h, own) == hipSuccess;
  if (got) memcpy(hbuf, &h, sizeof h);
  std::vector<uint8_t> all;
  int rc = peer_round(c, pr, got, hbuf, 64, &all);
  if (rc) return got ? rc : set_err(GH_E_HIP, "peer transport: hipIpcGetMemHandle failed");
  bool opened = true;
  for (int r = 0; r < c->world && opened; ++r) {
    if (r == c->rank) continue;
    hipIpcMemHandle_t hr;
    memcpy(&hr, all.data() + 64 * (size_t)r, sizeof hr);
    void* p = nullptr;
    opened = hipIpcOpenMemHandle(&p, hr, hipIpcMemLazyEnablePeerAccess) == hipSuccess;
    out[r] = opened ? p : nullptr;
  }
  rc = peer_round(c, pr, opened, nullptr, 0, nullptr);
  if (rc) {
    ipc_close(c, out);
    for (int r = 0; r < c->world; ++r) out[r] = nullptr;
    return opened ? rc : set_err(GH_E_HIP, "peer transport: hipIpcOpenMemHandle failed");
  }
  out[c->rank] = own;
  return GH_OK;
}

// the filter's multi-rank path (collectives, split steps) is in use
static bool mr(const gh_ctx* c) { return c->world > 1 || c->force_multi; }

static int ctx_setup(int device, void* stream, gh_ctx* c) {
  c->device = device;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device));
  if (stream) {
    c->stream = (hipStream_t)stream;
  } else {
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->own_stream = true;
  }
  return GH_OK;
}

extern "C" int gh_ctx_create(int device, void* hip_stream, gh_ctx** out) {
  if (!out) return set_err(GH_E_INVAL, "gh_ctx_create: out is NULL");
  gh_ctx* c = new gh_ctx();
  int rc = ctx_setup(device, hip_stream, c);
  if (rc) { delete c; return rc; }
  *out = c;
  return GH_OK;
}

extern "C" int gh_comm_unique_id(uint8_t id[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u));
  memcpy(id, &u, 128);
  return GH_OK;
}

extern "C" int gh_ctx_create_dist(int device, int rank, int world, const uint8_t id[128],
                                  void* hip_stream, gh_ctx** out) {
  if (!out || world < 1 || rank < 0 || rank >= world)
    return set_err(GH_E_INVAL, "gh_ctx_create_dist: bad rank/world %d/%d", rank, world);
  gh_ctx* c = new gh_ctx();
  int rc = ctx_setup(device, hip_stream, c);
  if (rc) { delete c; return rc; }
  c->rank = rank;
  c->world = world;
  if (world > 1) {
    ncclUniqueId u;
    memcpy(&u, id, 128);
    ncclResult_t r = ncclCommInitRank(&c->comm, world, u, rank);
    if (r != ncclSuccess) {
      delete c;
      return set_err(GH_E_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
  }
  *out = c;
  return GH_OK;
}

extern "C" int gh_ctx_create_hostcomm(int device, int rank, int world, const gh_host_comm* comm,
                                      void* hip_stream, gh_ctx** out) {
  if (!out || !comm || !comm->allgather || !comm->sendrecv || world < 1 || rank < 0 || rank >= world)
    return set_err(GH_E_INVAL, "gh_ctx_create_hostcomm: bad argument (rank/world %d/%d)", rank, world);
  gh_ctx* c = new gh_ctx();
  int rc = ctx_setup(device, hip_stream, c);
  if (rc) { delete c; return rc; }
  c->rank = rank;
  c->world = world;
  c->host_comm = true;
  c->hc = *comm;
  *out = c;
  return GH_OK;
}

extern "C" int gh_ctx_create_peer(int device, int rank, int world, const gh_host_comm* bootstrap, void* hip_stream,
                                  gh_ctx** out) {
  if (!out || !bootstrap || !bootstrap->allgather || world < 1 || world > kPeerMaxRanks || rank < 0 || rank >= world)
    return set_err(GH_E_INVAL, "gh_ctx_create_peer: bad argument (rank/world %d/%d, at most %d ranks)", rank, world,
                   kPeerMaxRanks);
  gh_ctx* c = new gh_ctx();
  c->rank = rank;
  c->world = world;
  c->peer = true;
  c->hc = *bootstrap;
  PeerRounds pr;
  // (a local failure still runs the exchange's first round, flagged, so the
  // other ranks fail with it instead of waiting)
  auto fail = [&](int rc) {
    peer_abort(c, pr);
    if (c->mbox) hipFree(c->mbox);
    if (c->own_stream) hipStreamDestroy(c->stream);
    delete c;
    return rc;
  };
  int rc = ctx_setup(device, hip_stream, c);
  if (rc) return fail(rc);
  if (hipDeviceGetAttribute(&c->wall_khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || c->wall_khz <= 0)
    c->wall_khz = 100000;
  c->peer_wait_ticks = (uint64_t)(kPeerWaitDefaultS * 1e3 * c->wall_khz);
  const size_t bytes = sizeof(uint64_t) * (size_t)mb_words(world);
  if (hipExtMallocWithFlags((void**)&c->mbox, bytes, hipDeviceMallocFinegrained) != hipSuccess) {
    c->mbox = nullptr;
    return fail(set_err(GH_E_NOMEM, "peer transport: mailbox"));
  }
  if (hipMemset(c->mbox, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return fail(set_err(GH_E_HIP, "peer transport: mailbox init"));
  rc = ipc_exchange(c, pr, c->mbox, (void**)c->mpeer);
  if (rc) return fail(rc);
  *out = c;
  return GH_OK;
}

extern "C" int gh_ctx_set_peer_timeout(gh_ctx* c, double seconds) {
  if (!c || !(seconds > 0.0) || seconds > 86400.0) return set_err(GH_E_INVAL, "gh_ctx_set_peer_timeout: bad argument");
  if (!c->peer) return GH_OK;  // (no device waits on peers on the other transports)
  c->peer_wait_ticks = (uint64_t)(seconds * 1e3 * c->wall_khz);
  return GH_OK;
}

extern "C" int gh_ctx_force_multirank(gh_ctx* c) {
  if (!c) return set_err(GH_E_INVAL, "null ctx");
  if (c->force_multi) return GH_OK;
  // a live filter allocated the one-rank path's buffers only; switching it
  // would run the multi-rank kernels and collectives on missing buffers
  if (c->n_filters > 0)
    return set_err(GH_E_STATE, "gh_ctx_force_multirank: %d filter(s) exist on this context", c->n_filters);
  if (c->world == 1 && !c->host_comm && !c->peer && !c->comm) {  // a one-rank RCCL communicator
    ncclUniqueId u;
    NCCL_TRY(ncclGetUniqueId(&u));
    HIP_TRY(hipSetDevice(c->device));
    NCCL_TRY(ncclCommInitRank(&c->comm, 1, u, 0));
  }
  c->force_multi = true;
  return GH_OK;
}

extern "C" int gh_ctx_destroy(gh_ctx* c) {
  if (!c) return GH_OK;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->stage) hipHostFree(c->stage);
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->peer) {
    // every rank is done writing into the others' mailboxes before any frees its own
    uint8_t one = 1;
    std::vector<uint8_t> all((size_t)c->world);
    c->hc.allgather(c->hc.user, &one, all.data(), 1);
    ipc_close(c, (void**)c->mpeer);
    hipFree(c->mbox);
  }
  if (c->own_stream) hipStreamDestroy(c->stream);
  delete c;
  return GH_OK;
}

extern "C" int gh_ctx_rank(const gh_ctx* c, int* rank, int* world) {
  if (!c) return set_err(GH_E_INVAL, "null ctx");
  if (rank) *rank = c->rank;
  if (world) *world = c->world;
  return GH_OK;
}

extern "C" int gh_ctx_stream(const gh_ctx* c, void** s) {
  if (!c || !s) return set_err(GH_E_INVAL, "null ctx");
  *s = (void*)c->stream;
  return GH_OK;
}

// ---------------------------------------------------------- transport
// Two collectives cover the path: an all-gather of a few words per rank and a
// grouped point-to-point exchange of state rows.  RCCL runs them on the
// context stream with no host synchronisation; the host-staged transport
// copies through pinned memory and calls the user's functions.
struct CommMsg {
  int peer;
  void* dptr;
  size_t bytes;
};

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

static int stage_reserve(gh_ctx* c, size_t bytes) {
  if (bytes <= c->stage_bytes) return GH_OK;
  size_t nb = c->stage_bytes ? c->stage_bytes : (1 << 16);
  while (nb < bytes) nb *= 2;
  if (c->stage) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    hipHostFree(c->stage);
    c->stage = nullptr;
    c->stage_bytes = 0;
  }
  HIP_TRY(hipHostMalloc((void**)&c->stage, nb, hipHostMallocDefault));
  c->stage_bytes = nb;
  return GH_OK;
}

static int comm_allgather(gh_ctx* c, const void* dsend, void* drecv, size_t bytes, hipStream_t s, int* derr) {
  if (c->peer) {  // one wave through the mailboxes (gh_peer.h)
    if (bytes % 8 || bytes > sizeof(uint64_t) * kAgWords)
      return set_err(GH_E_INVAL, "peer transport: all-gather of %zu bytes", bytes);
    hipLaunchKernelGGL(k_peer_allgather, dim3(1), dim3(64), 0, s, (const uint64_t*)dsend, (uint64_t*)drecv,
                       (int)(bytes / 8), peer_box(c), ++c->use_ag, derr);
    HIP_TRY(hipGetLastError());
    return GH_OK;
  }
  if (!c->host_comm) {
    NCCL_TRY(ncclAllGather(dsend, drecv, bytes, ncclUint8, c->comm, s));
    return GH_OK;
  }
  const size_t off = align_up(bytes);
  CHECK(stage_reserve(c, off + bytes * (size_t)c->world));
  HIP_TRY(hipMemcpyAsync(c->stage, dsend, bytes, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (c->hc.allgather(c->hc.user, c->stage, c->stage + off, bytes))
    return set_err(GH_E_RCCL, "host transport: allgather failed");
  HIP_TRY(hipMemcpyAsync(drecv, c->stage + off, bytes * (size_t)c->world, hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  return GH_OK;
}

static int comm_exchange(gh_ctx* c, const std::vector<CommMsg>& sends, const std::vector<CommMsg>& recvs,
                         hipStream_t s) {
  if (sends.empty() && recvs.empty()) return GH_OK;
  // peer transport: the systematic rows move inside the resample kernels; the
  // other resamplers' rows (multinomial, conditional SMC, the generic exchange)
  // go through the bootstrap's host send/recv when it has one
  if (c->peer && !c->hc.sendrecv)
    return set_err(GH_E_STATE, "peer transport without a bootstrap sendrecv: rows move inside the systematic "
                               "resample kernels only");
  if (!c->host_comm && !c->peer) {
    // an error inside the group still closes it (an open group leaves the
    // communicator unusable); the first error is reported
    NCCL_TRY(ncclGroupStart());
    ncclResult_t r = ncclSuccess;
    const char* what = "";
    for (const auto& m : sends)
      if (r == ncclSuccess && (r = ncclSend(m.dptr, m.bytes, ncclUint8, m.peer, c->comm, s)) != ncclSuccess) what = "ncclSend";
    for (const auto& m : recvs)
      if (r == ncclSuccess && (r = ncclRecv(m.dptr, m.bytes, ncclUint8, m.peer, c->comm, s)) != ncclSuccess) what = "ncclRecv";
    const ncclResult_t re = ncclGroupEnd();
    if (r != ncclSuccess) return set_err(GH_E_RCCL, "%s: %s", what, ncclGetErrorString(r));
    if (re != ncclSuccess) return set_err(GH_E_RCCL, "ncclGroupEnd: %s", ncclGetErrorString(re));
    return GH_OK;
  }
  size_t total = 0;
  for (const auto& m : sends) total += align_up(m.bytes);
  for (const auto& m : recvs) total += align_up(m.bytes);
  CHECK(stage_reserve(c, total));
  std::vector<int> sp, rp;
  std::vector<const void*> sb;
  std::vector<void*> rb;
  std::vector<uint64_t> sn, rn;
  size_t off = 0;
  for (const auto& m : sends) {
    HIP_TRY(hipMemcpyAsync(c->stage + off, m.dptr, m.bytes, hipMemcpyDeviceToHost, s));
    sp.push_back(m.peer);
    sb.push_back(c->stage + off);
    sn.push_back(m.bytes);
    off += align_up(m.bytes);
  }
  for (const auto& m : recvs) {
    rp.push_back(m.peer);
    rb.push_back(c->stage + off);
    rn.push_back(m.bytes);
    off += align_up(m.bytes);
  }
  HIP_TRY(hipStreamSynchronize(s));
  if (c->hc.sendrecv(c->hc.user, (int)sp.size(), sp.data(), sb.data(), sn.data(), (int)rp.size(), rp.data(),
                     rb.data(), rn.data()))
    return set_err(GH_E_RCCL, "host transport: sendrecv failed");
  for (size_t i = 0; i < recvs.size(); ++i)
    HIP_TRY(hipMemcpyAsync(recvs[i].dptr, rb[i], recvs[i].bytes, hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  return GH_OK;
}

// All-gather of a large buffer for the genealogy queries (off the step
// path): RCCL, or staged through host memory and the user's all-gather (the
// host and peer transports).  Synchronous.
static int bulk_allgather(gh_ctx* c, const void* dsend, void* drecv, size_t bytes, hipStream_t s) {
  if (c->comm) {
    NCCL_TRY(ncclAllGather(dsend, drecv, bytes, ncclUint8, c->comm, s));
    HIP_TRY(hipStreamSynchronize(s));
    return GH_OK;
  }
  if (!c->hc.allgather) return set_err(GH_E_STATE, "no transport for the genealogy all-gather");
  std::vector<uint8_t> hs(bytes), hr(bytes * (size_t)c->world);
  HIP_TRY(hipMemcpyAsync(hs.data(), dsend, bytes, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (c->hc.allgather(c->hc.user, hs.data(), hr.data(), bytes))
    return set_err(GH_E_RCCL, "genealogy all-gather failed");
  HIP_TRY(hipMemcpyAsync(drecv, hr.data(), hr.size(), hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  return GH_OK;
}

extern "C" int gh_ctx_synchronize(gh_ctx* c) {
  if (!c) return set_err(GH_E_INVAL, "null ctx");
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GH_OK;
}

// ------------------------------------------------ host linear algebra (§5.1)
// Same operation order as oracle/gh_oracle.c so derived parameters agree bit
// for bit (Cholesky–Banachiewicz, forward substitution, log-det).
static int chol(int d, const double* S, double* L) {
  for (int i = 0; i < d * d; ++i) L[i] = 0.0;
  for (int i = 0; i < d; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = S[i * d + j];
      for (int k = 0; k < j; ++k) s = fma(-L[i * d + k], L[j * d + k], s);
      if (i == j) {
        if (!(s > 0.0)) return -1;
        L[i * d + i] = sqrt(s);
      } else {
        L[i * d + j] = s / L[j * d + j];
      }
    }
  return 0;
}
static void fwdsub(int d, int m, const double* L, const double* B, double* Y) {
  for (int c = 0; c < m; ++c)
    for (int i = 0; i < d; ++i) {
      double s = B[i * m + c];
      for (int k = 0; k < i; ++k) s = fma(-L[i * d + k], Y[k * m + c], s);
      Y[i * m + c] = s / L[i * d + i];
    }
}
// X = L^{-T} B for B (d x m) row-major (backward substitution on L^T)
static void bwdsub(int d, int m, const double* L, const double* B, double* X) {
  for (int c = 0; c < m; ++c)
    for (int i = d - 1; i >= 0; --i) {
      double s = B[i * m + c];
      for (int k = i + 1; k < d; ++k) s = fma(-L[k * d + i], X[k * m + c], s);
      X[i * m + c] = s / L[i * d + i];
    }
}
// C = A B (A: n x k, B: k x m), fma over the inner index ascending
static void matmul(int n, int k, int m, const double* A, const double* B, double* C) {
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < m; ++j) {
      double acc = 0.0;
      for (int l = 0; l < k; ++l) acc = fma(A[i * k + l], B[l * m + j], acc);
      C[i * m + j] = acc;
    }
}
static double gauss_cst(int d, const double* L) {
  double acc = 0.0;
  for (int i = 0; i < d; ++i) acc += gh_log(L[i * d + i]);
  const double logdet = 2.0 * acc;
  return -0.5 * ((double)d * LOG_2PI + logdet);
}

// ------------------------------------------------------------------ models
struct gh_model {
  gh_ctx* ctx = nullptr;
  int family = 0, d = 0, dy = 0, k = 0, v = 0;
  double* dparams = nullptr;  // device copy of the derived parameters
  // host copies needed per step
  std::vector<double> LR, c;  // LGSSM: chol(R), offset c
  // LGSSM locally optimal proposal (LGOptModel): host halves
  bool lg_opt = false;        // derivable (S, Sigma positive definite, d + dy <= kMaxObs)
  std::vector<double> LS, Kt, Fb, Wb;       // chol(S), K^T (dy x d), F b, L_S^-1 H b
  std::vector<double> H, mu0, LS1, Kt1;     // t = 1: H, mu0, chol(S_1), K_1^T
  double cstS1 = 0.0;
  LGParams lg{};
  int lg_struct = 0;  // LGModel<D, S> structure bits (gh_models.h)
  HMMParams hmm{};
  KitParams kit{};
  RegParams reg{};
  // slot family (gh_slots.h): the device description and, per mvnormal slot,
  // the host halves of its observation whitening L_R^-1 (y - c)
  SlotParams slots{};
  bool slot_ext = false;  // a library slot or the switching latent: the SlotModel<D, true> instantiations
  std::vector<double> slot_c[kMaxSlots], slot_LR[kMaxSlots];
};

static bool lg_supported(int d) { return d >= 1 && d <= 16; }
static bool slots_supported(int d) { return d >= 1 && d <= kMaxSlotD; }

// GH_FAMILY_SLOTS: parse the slot description (include/gen_hip.h), derive the
// device parameters into h (offsets into it in *off) and the model's host
// halves.  Returns an error message or nullptr.
static const char* slots_build(gh_model* m, const double* p, int64_t np, std::vector<double>& h,
                               int64_t off[5 + kMaxSlots]) {
  const int d = m->d;
  if (!slots_supported(d)) return "slots: latent dimension d must be in 1..16";
  if (np < 2) return "slots: need the latent form and the slot count";
  SlotParams& sp = m->slots;
  const int form = (int)p[0];
  sp.lat = form == GH_SLOT_LAT_AFFINE_INPUT ? SLOT_LAT_AFFINE : form;
  const bool inputs = form == GH_SLOT_LAT_AFFINE_INPUT;
  sp.K = (int)p[1];
  if (p[0] != form || (form != SLOT_LAT_AFFINE && form != SLOT_LAT_KITAGAWA && !inputs &&
                       form != SLOT_LAT_CATEGORICAL && form != SLOT_LAT_SWITCHING))
    return "slots: latent form must be 0 (affine mvnormal), 1 (Kitagawa), 2 (affine with per-step inputs), 3 "
           "(categorical) or 4 (switching linear-Gaussian)";
  if (form == SLOT_LAT_CATEGORICAL && d < 2) return "slots: a categorical latent has d = K >= 2 classes";
  if (sp.lat == SLOT_LAT_KITAGAWA && d != 1) return "slots: the Kitagawa latent has d = 1";
  if (p[1] != sp.K || sp.K < 1 || sp.K > kMaxSlots) return "slots: 1..4 observed slots";
  int64_t i = 2 + 3 * (int64_t)sp.K;
  if (np < i) return "slots: too few parameters (slot headers)";
  int voff = 0, yoff = 0;
  for (int k = 0; k < sp.K; ++k) {
    const double* hd = p + 2 + 3 * k;
    sp.dist[k] = (int)hd[0];
    sp.m[k] = (int)hd[1];
    sp.link[k] = (int)hd[2];
    if (hd[0] != sp.dist[k] || hd[1] != sp.m[k] || hd[2] != sp.link[k]) return "slots: slot header not integral";
    const int dist = sp.dist[k], mm = sp.m[k], link = sp.link[k];
    int nv = 1;
    if (dist == SLOT_MVNORMAL) {
      if (link != LINK_AFFINE || mm < 1 || mm > kMaxObs) return "slots: mvnormal slot needs the affine mean, 1..32 values";
      nv = mm;
    } else if (dist == SLOT_NORMAL) {
      if (mm != 1 || !(link == LINK_AFFINE || link == LINK_LOGSCALE || (link == LINK_KITAGAWA && d == 1)))
        return "slots: normal slot: one value, affine mean (or x^2/20 with d = 1), fixed or log-linear sd";
    } else if (dist == SLOT_POISSON) {
      if (mm != 1 || link != LINK_EXP) return "slots: poisson slot: one count, rate exp(h.x + c)";
      nv = 2;  // (y, log Gamma(y + 1))
    } else if (dist == SLOT_BERNOULLI) {
      if (mm != 1 || link != LINK_LOGISTIC) return "slots: bernoulli slot: one value, prob 1/(1 + exp(-(h.x + c)))";
    } else if (dist == SLOT_CATEGORICAL) {
      if (mm < 2 || mm > kMaxSlotClasses || link != LINK_SOFTMAX)
        return "slots: categorical slot: 2..16 classes, probs softmax(W x + c)";
    } else if (dist == SLOT_LIBRARY) {
      if (lib_nargs(mm) == 0 || link != 0) return "slots: library slot: m names a scalar distribution (gen_hip.h)";
      m->slot_ext = true;
    } else {
      return "slots: unknown slot distribution";
    }
    sp.voff[k] = voff;
    sp.yoff[k] = yoff;
    voff += nv;
    yoff += dist == SLOT_MVNORMAL ? mm : 1;
  }
  if (voff + (inputs ? d : 0) > kMaxObs || yoff > kMaxObs)
    return "slots: more than 32 observed values (and inputs) per step";
  m->dy = yoff;
  sp.uoff = inputs ? voff : -1;
  sp.qoff = voff + (inputs ? d : 0);
  // latent block
  off[0] = (int64_t)h.size();
  if (sp.lat == SLOT_LAT_AFFINE) {
    const int64_t need = 3LL * d * d + 2LL * d;
    if (np < i + need) return "slots: too few parameters (affine latent: A b Q mu0 P0)";
    const double *A = p + i, *b = A + d * d, *Q = b + d, *mu0 = Q + d * d, *P0 = mu0 + d;
    std::vector<double> LQ(d * d), L0(d * d);
    if (chol(d, Q, LQ.data())) return "slots: Q not positive definite";
    if (chol(d, P0, L0.data())) return "slots: P0 not positive definite";
    h.insert(h.end(), A, A + d * d);
    h.insert(h.end(), b, b + d);
    h.insert(h.end(), LQ.begin(), LQ.end());
    h.insert(h.end(), mu0, mu0 + d);
    h.insert(h.end(), L0.begin(), L0.end());
    sp.cstQ = gauss_cst(d, LQ.data());
    sp.cst0 = gauss_cst(d, L0.data());
    i += need;
  } else if (sp.lat == SLOT_LAT_SWITCHING) {  // nz prior[nz] T[nz*nz] (A_z b_z Q_z per regime) mu0 P0
    if (np < i + 1) return "slots: too few parameters (switching latent)";
    const int nz = (int)p[i];
    const int dx = d - nz;
    if (p[i] != nz || nz < 2 || nz > kMaxRegimes || dx < 1)
      return "slots: a switching latent has 2..8 regimes and d = dx + regimes with dx >= 1";
    sp.nz = nz;
    m->slot_ext = true;
    const int64_t per = 2LL * dx * dx + dx;
    const int64_t need = 1 + nz + (int64_t)nz * nz + nz * per + dx + (int64_t)dx * dx;
    if (np < i + need) return "slots: too few parameters (switching latent: nz prior T (A b Q per regime) mu0 P0)";
    const double* pr = p + i + 1;
    for (int64_t j = 0; j < nz + (int64_t)nz * nz; ++j)
      if (!(pr[j] >= 0.0) || !std::isfinite(pr[j])) return "slots: regime probabilities must be >= 0";
    h.insert(h.end(), pr, pr + nz + nz * nz);
    const double* rb = pr + nz + nz * nz;
    std::vector<double> L(dx * dx);
    for (int z = 0; z < nz; ++z, rb += per) {
      const double *A = rb, *b = rb + dx * dx, *Q = b + dx;
      if (chol(dx, Q, L.data())) return "slots: a regime's Q is not positive definite";
      h.insert(h.end(), A, A + dx * dx);
      h.insert(h.end(), b, b + dx);
      h.insert(h.end(), L.begin(), L.end());
      sp.cstQz[z] = gauss_cst(dx, L.data());
    }
    const double *mu0 = rb, *P0 = rb + dx;
    if (chol(dx, P0, L.data())) return "slots: P0 not positive definite";
    h.insert(h.end(), mu0, mu0 + dx);
    h.insert(h.end(), L.begin(), L.end());
    sp.cst0 = gauss_cst(dx, L.data());
    i += need;
  } else if (sp.lat == SLOT_LAT_CATEGORICAL) {
    const int64_t need = (int64_t)d + (int64_t)d * d;
    if (np < i + need) return "slots: too few parameters (categorical latent: prior[K] T[K*K])";
    for (int64_t j = 0; j < need; ++j)
      if (!(p[i + j] >= 0.0) || !std::isfinite(p[i + j])) return "slots: categorical latent probabilities must be >= 0";
    h.insert(h.end(), p + i, p + i + need);  // prior | T (T[new*K + prev], as the HMM family)
    i += need;
  } else {
    if (np < i + 3) return "slots: too few parameters (Kitagawa latent: mu1 s1 sd_x)";
    const double mu1 = p[i], s1 = p[i + 1], sdx = p[i + 2];
    if (!(s1 > 0.0) || !(sdx > 0.0)) return "slots: Kitagawa latent standard deviations must be > 0";
    // normal.jl:56-60 with the standard deviations given (var = sd * sd)
    sp.kit.mu1 = mu1;
    sp.kit.s1 = s1;
    sp.kit.sx = sdx;
    sp.kit.inv2vx = 1.0 / (2.0 * (sdx * sdx));
    sp.kit.cstx = -0.5 * gh_log(2.0 * 0x1.921fb54442d18p+1 * (sdx * sdx));
    sp.kit.inv2v1 = 1.0 / (2.0 * (s1 * s1));
    sp.kit.cst1 = -0.5 * gh_log(2.0 * 0x1.921fb54442d18p+1 * (s1 * s1));
    h.push_back(0.0);
    i += 3;
  }
  // slot blocks
  for (int k = 0; k < sp.K; ++k) {
    const int dist = sp.dist[k], mm = sp.m[k];
    off[5 + k] = (int64_t)h.size();
    if (dist == SLOT_MVNORMAL) {
      const int64_t need = (int64_t)mm * d + mm + (int64_t)mm * mm;
      if (np < i + need) return "slots: too few parameters (mvnormal slot: H c R)";
      const double *H = p + i, *c = H + mm * d, *R = c + mm;
      m->slot_LR[k].assign(mm * mm, 0.0);
      if (chol(mm, R, m->slot_LR[k].data())) return "slots: an mvnormal slot's R is not positive definite";
      std::vector<double> M(mm * d);
      fwdsub(mm, d, m->slot_LR[k].data(), H, M.data());
      m->slot_c[k].assign(c, c + mm);
      h.insert(h.end(), M.begin(), M.end());
      h.insert(h.end(), H, H + mm * d);
      h.insert(h.end(), c, c + mm);
      h.insert(h.end(), m->slot_LR[k].begin(), m->slot_LR[k].end());
      sp.cst[k] = gauss_cst(mm, m->slot_LR[k].data());
      i += need;
    } else if (dist == SLOT_NORMAL && sp.link[k] == LINK_LOGSCALE) {  // h c g s: sd = exp(g.x + s)
      const int64_t need = 2LL * d + 2;
      if (np < i + need) return "slots: too few parameters (log-linear normal slot: h c g s)";
      h.insert(h.end(), p + i, p + i + need);
      i += need;
    } else if (dist == SLOT_NORMAL) {
      const int64_t need = sp.link[k] == LINK_AFFINE ? d + 2 : 1;
      if (np < i + need) return "slots: too few parameters (normal slot: h c sd, or sd)";
      if (sp.link[k] == LINK_AFFINE) h.insert(h.end(), p + i, p + i + d + 1);
      else h.push_back(0.0);
      const double sd = p[i + need - 1];
      if (!(sd > 0.0)) return "slots: a normal slot's sd must be > 0";
      sp.sd[k] = sd;
      sp.inv2v[k] = 1.0 / (2.0 * (sd * sd));
      sp.cst[k] = -0.5 * gh_log(2.0 * 0x1.921fb54442d18p+1 * (sd * sd));
      i += need;
    } else if (dist == SLOT_LIBRARY) {  // (link h[d] c) per argument
      const int na = lib_nargs(mm);
      const int64_t need = (int64_t)na * (d + 2);
      if (np < i + need) return "slots: too few parameters (library slot: link h c per argument)";
      for (int j = 0; j < na; ++j) {
        const double l = p[i + j * (d + 2)];
        if (!(l == LIB_IDENTITY || l == LIB_EXP || l == LIB_LOGISTIC))
          return "slots: a library slot's argument link is 0 (identity), 2 (exp) or 3 (logistic)";
      }
      h.insert(h.end(), p + i, p + i + need);
      i += need;
    } else if (dist == SLOT_CATEGORICAL) {
      const int64_t need = (int64_t)mm * d + mm;
      if (np < i + need) return "slots: too few parameters (categorical slot: W c)";
      h.insert(h.end(), p + i, p + i + need);
      i += need;
    } else {  // poisson, bernoulli: h c
      if (np < i + d + 1) return "slots: too few parameters (h c)";
      h.insert(h.end(), p + i, p + i + d + 1);
      i += d + 1;
    }
  }
  // optional: dependencies between the step's observed addresses, nd then
  // (child k, parent j < k, coefficient g) per dependency
  sp.dep = 0;
  sp.doff = sp.qoff + d;
  for (int k = 0; k < kMaxSlots; ++k)
    for (int j = 0; j < kMaxSlots; ++j) sp.dg[k][j] = 0.0;
  if (np > i) {
    const int nd = (int)p[i];
    if (p[i] != nd || nd < 0 || np < i + 1 + 3LL * nd) return "slots: dependency block: nd then (child, parent, g) per dependency";
    auto scalar = [&](int k) { return sp.dist[k] != SLOT_MVNORMAL; };
    auto child_ok = [&](int k) {
      return sp.dist[k] == SLOT_POISSON || sp.dist[k] == SLOT_BERNOULLI || sp.dist[k] == SLOT_LIBRARY ||
             (sp.dist[k] == SLOT_NORMAL && sp.link[k] != LINK_KITAGAWA);
    };
    for (int q = 0; q < nd; ++q) {
      const double* e = p + i + 1 + 3 * q;
      const int k = (int)e[0], j = (int)e[1];
      if (e[0] != k || e[1] != j || k < 0 || k >= sp.K || j < 0 || j >= k || !std::isfinite(e[2]))
        return "slots: a dependency names a child slot and an earlier parent slot";
      if (!child_ok(k) || !scalar(j))
        return "slots: dependencies: a normal (affine mean), poisson, bernoulli or library child; a scalar parent";
      sp.dg[k][j] = e[2];
      sp.dep |= 1 << k;
    }
    if (sp.dep && sp.doff + sp.K > kMaxObs) return "slots: too many observed values for the dependency terms";
  }
  return nullptr;
}

extern "C" int gh_model_create(gh_ctx* ctx, const gh_model_desc* desc, gh_model** out) {
  if (!ctx || !desc || !out) return set_err(GH_E_INVAL, "gh_model_create: null argument");
  HIP_TRY(hipSetDevice(ctx->device));
  gh_model* m = new gh_model();
  m->ctx = ctx;
  m->family = desc->family;
  m->d = desc->d;
  m->dy = desc->dy;
  m->k = desc->k;
  m->v = desc->v;
  std::vector<double> h;  // packed derived parameters
  int64_t slot_off[5 + kMaxSlots] = {};  // GH_FAMILY_SLOTS: the latent's and each slot's offset in h
  const double* p = desc->params;
  auto fail = [&](int code, const char* msg) {
    delete m;
    return set_err(code, "gh_model_create: %s", msg);
  };
  if (!p) return fail(GH_E_INVAL, "params is NULL");
  if (desc->family == GH_FAMILY_LGSSM) {
    const int d = desc->d, dy = desc->dy;
    if (!lg_supported(d)) return fail(GH_E_INVAL, "LGSSM: unsupported d (1..16)");
    if (dy < 1 || dy > kMaxObs) return fail(GH_E_INVAL, "LGSSM: dy must be in 1..32");
    const int64_t need = (int64_t)d * d + d + (int64_t)d * d + (int64_t)dy * d + dy +
                         (int64_t)dy * dy + d + (int64_t)d * d;
    if (desc->n_params < need) return fail(GH_E_INVAL, "LGSSM: too few parameters");
    const double *A = p, *b = A + d * d, *Q = b + d, *H = Q + d * d, *c = H + dy * d, *R = c + dy,
                 *mu0 = R + dy * dy, *P0 = mu0 + d;
    std::vector<double> LQ(d * d), L0(d * d), M(dy * d);
    m->LR.assign(dy * dy, 0.0);
    if (chol(d, Q, LQ.data())) return fail(GH_E_INVAL, "LGSSM: Q not positive definite");
    if (chol(dy, R, m->LR.data())) return fail(GH_E_INVAL, "LGSSM: R not positive definite");
    if (chol(d, P0, L0.data())) return fail(GH_E_INVAL, "LGSSM: P0 not positive definite");
    fwdsub(dy, d, m->LR.data(), H, M.data());
    m->c.assign(c, c + dy);
    // layout: A | b | LQ | M | mu0 | L0 | FA | LSig | WA | LSig1 (below)
    h.insert(h.end(), A, A + d * d);
    h.insert(h.end(), b, b + d);
    h.insert(h.end(), LQ.begin(), LQ.end());
    h.insert(h.end(), M.begin(), M.end());
    h.insert(h.end(), mu0, mu0 + d);
    h.insert(h.end(), L0.begin(), L0.end());
    m->lg.dy = dy;
    m->lg.cstR = gauss_cst(dy, m->LR.data());
    m->lg.cstQ = gauss_cst(d, LQ.data());
    m->lg.cst0 = gauss_cst(d, L0.data());
    bool lq_diag = true, m_diag = dy == d;
    for (int i = 0; i < d; ++i)
      for (int j = 0; j < i; ++j) lq_diag = lq_diag && LQ[i * d + j] == 0.0;
    for (int r = 0; m_diag && r < dy; ++r)
      for (int j = 0; j < d; ++j) m_diag = m_diag && (j == r || M[r * d + j] == 0.0);
    m->lg_struct = (lq_diag ? 1 : 0) | (m_diag ? 2 : 0);
    // locally optimal proposal: S = H Q H^T + R, K^T = S^-1 H Q, F = I - K H,
    // Sigma = F Q (the same operations as oracle/gh_oracle.c lg_opt_build)
    std::vector<double> FA(d * d, 0.0), LSig(d * d, 0.0), WA(dy * d, 0.0), LSig1(d * d, 0.0);
    auto derive = [&](const double* P, std::vector<double>& LSo, std::vector<double>& Kto,
                      std::vector<double>& Lsigo, std::vector<double>* F_out) -> bool {
      std::vector<double> HP(dy * d), Sm(dy * dy), Y(dy * d), F(d * d), Sig(d * d);
      matmul(dy, d, d, H, P, HP.data());
      for (int r = 0; r < dy; ++r)
        for (int q = 0; q < dy; ++q) {
          double acc = R[r * dy + q];
          for (int j = 0; j < d; ++j) acc = fma(HP[r * d + j], H[q * d + j], acc);
          Sm[r * dy + q] = acc;
        }
      LSo.assign(dy * dy, 0.0);
      if (chol(dy, Sm.data(), LSo.data())) return false;
      fwdsub(dy, d, LSo.data(), HP.data(), Y.data());
      Kto.assign(dy * d, 0.0);
      bwdsub(dy, d, LSo.data(), Y.data(), Kto.data());
      for (int i = 0; i < d; ++i)
        for (int j = 0; j < d; ++j) {
          double acc = i == j ? 1.0 : 0.0;
          for (int r = 0; r < dy; ++r) acc = fma(-Kto[r * d + i], H[r * d + j], acc);
          F[i * d + j] = acc;
        }
      matmul(d, d, d, F.data(), P, Sig.data());
      Lsigo.assign(d * d, 0.0);
      if (chol(d, Sig.data(), Lsigo.data())) return false;
      if (F_out) *F_out = F;
      return true;
    };
    std::vector<double> F, LSigv, LSig1v;
    m->lg_opt = d + dy <= kMaxObs && derive(Q, m->LS, m->Kt, LSigv, &F) && derive(P0, m->LS1, m->Kt1, LSig1v, nullptr);
    if (m->lg_opt) {
      matmul(d, d, d, F.data(), A, FA.data());
      m->Fb.assign(d, 0.0);
      matmul(d, d, 1, F.data(), b, m->Fb.data());
      std::vector<double> W(dy * d);
      fwdsub(dy, d, m->LS.data(), H, W.data());
      matmul(dy, d, d, W.data(), A, WA.data());
      m->Wb.assign(dy, 0.0);
      matmul(dy, d, 1, W.data(), b, m->Wb.data());
      LSig = LSigv;
      LSig1 = LSig1v;
      m->lg.cstS = gauss_cst(dy, m->LS.data());
      m->cstS1 = gauss_cst(dy, m->LS1.data());
      m->H.assign(H, H + dy * d);
      m->mu0.assign(mu0, mu0 + d);
    }
    // proposal blocks after the prior's (zeros when not derivable)
    h.insert(h.end(), FA.begin(), FA.end());
    h.insert(h.end(), LSig.begin(), LSig.end());
    h.insert(h.end(), WA.begin(), WA.end());
    h.insert(h.end(), LSig1.begin(), LSig1.end());
    // simulate(): H | c | L_R
    h.insert(h.end(), H, H + dy * d);
    h.insert(h.end(), c, c + dy);
    h.insert(h.end(), m->LR.begin(), m->LR.end());
  } else if (desc->family == GH_FAMILY_HMM) {
    const int K = desc->k, V = desc->v;
    if (K < 1 || K > 64 || V < 1) return fail(GH_E_INVAL, "HMM: need 1 <= k <= 64, v >= 1");
    if (desc->n_params < (int64_t)K + K * K + (int64_t)V * K) return fail(GH_E_INVAL, "HMM: too few parameters");
    m->d = 1;
    h.insert(h.end(), p, p + K + K * K + V * K);  // prior | T | E
    for (int i = 0; i < V * K; ++i) h.push_back(gh_log(p[K + K * K + i]));  // logE
    m->hmm.k = K;
    m->hmm.v = V;
  } else if (desc->family == GH_FAMILY_KITAGAWA) {
    if (desc->n_params < 4) return fail(GH_E_INVAL, "Kitagawa: need mu1 s1 var_x var_y");
    if (!(p[2] > 0.0) || !(p[3] > 0.0)) return fail(GH_E_INVAL, "Kitagawa: variances must be > 0");
    m->d = 1;
    m->kit.mu1 = p[0];
    m->kit.s1 = p[1];
    m->kit.sx = sqrt(p[2]);
    m->kit.inv2vy = 1.0 / (2.0 * p[3]);
    m->kit.csty = -0.5 * gh_log(2.0 * 0x1.921fb54442d18p+1 * p[3]);
    m->kit.inv2vx = 1.0 / (2.0 * p[2]);
    m->kit.cstx = -0.5 * gh_log(2.0 * 0x1.921fb54442d18p+1 * p[2]);
    m->kit.inv2v1 = 1.0 / (2.0 * (p[1] * p[1]));
    m->kit.cst1 = -0.5 * gh_log(2.0 * 0x1.921fb54442d18p+1 * (p[1] * p[1]));
    m->kit.sy = sqrt(p[3]);
    h.push_back(0.0);
  } else if (desc->family == GH_FAMILY_REGRESSION) {
    const int n = desc->dy;
    if (n < 1 || n > kMaxObs) return fail(GH_E_INVAL, "regression: dy (data points) must be in 1..32");
    if (desc->n_params < 5 + (int64_t)n) return fail(GH_E_INVAL, "regression: need mu_s sd_s mu_i sd_i sigma x[dy]");
    if (!(p[1] > 0.0) || !(p[3] > 0.0) || !(p[4] > 0.0))
      return fail(GH_E_INVAL, "regression: standard deviations must be > 0");
    m->d = 2;
    m->reg.mu_s = p[0];
    m->reg.sd_s = p[1];
    m->reg.mu_i = p[2];
    m->reg.sd_i = p[3];
    const double var = p[4] * p[4];
    m->reg.inv2v = 1.0 / (2.0 * var);
    m->reg.cst = -0.5 * gh_log(2.0 * 0x1.921fb54442d18p+1 * var);
    m->reg.inv2s = 1.0 / (2.0 * (p[1] * p[1]));
    m->reg.csts = -0.5 * gh_log(2.0 * 0x1.921fb54442d18p+1 * (p[1] * p[1]));
    m->reg.inv2i = 1.0 / (2.0 * (p[3] * p[3]));
    m->reg.csti = -0.5 * gh_log(2.0 * 0x1.921fb54442d18p+1 * (p[3] * p[3]));
    m->reg.sigma = p[4];
    m->reg.n = n;
    for (int i = 0; i < n; ++i) m->reg.xs[i] = p[5 + i];
    h.push_back(0.0);
  } else if (desc->family == GH_FAMILY_SLOTS) {
    if (const char* e = slots_build(m, p, desc->n_params, h, slot_off)) return fail(GH_E_INVAL, e);
  } else {
    return fail(GH_E_INVAL, "unknown family");
  }
  if (hipMalloc(&m->dparams, h.size() * sizeof(double)) != hipSuccess) return fail(GH_E_NOMEM, "hipMalloc params");
  if (hipMemcpy(m->dparams, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
    return fail(GH_E_HIP, "hipMemcpy params");
  if (m->family == GH_FAMILY_LGSSM) {
    const int d = m->d, dy = m->dy;
    double* q = m->dparams;
    m->lg.base = m->dparams;
    m->lg.A = q; q += d * d;
    m->lg.b = q; q += d;
    m->lg.LQ = q; q += d * d;
    m->lg.M = q; q += dy * d;
    m->lg.mu0 = q; q += d;
    m->lg.L0 = q; q += d * d;
    m->lg.FA = q; q += d * d;
    m->lg.LSig = q; q += d * d;
    m->lg.WA = q; q += dy * d;
    m->lg.LSig1 = q; q += d * d;
    m->lg.H = q; q += dy * d;
    m->lg.cv = q; q += dy;
    m->lg.LR = q;
  } else if (m->family == GH_FAMILY_HMM) {
    const int K = m->k, V = m->v;
    m->hmm.base = m->dparams;
    m->hmm.prior = m->dparams;
    m->hmm.T = m->dparams + K;
    m->hmm.E = m->dparams + K + K * K;
    m->hmm.logE = m->dparams + K + K * K + V * K;
  } else if (m->family == GH_FAMILY_SLOTS) {
    const int d = m->d;
    SlotParams& sp = m->slots;
    double* q = m->dparams + slot_off[0];
    sp.base = m->dparams;
    sp.A = q;
    sp.b = sp.lat == SLOT_LAT_AFFINE ? q + d * d : q;
    sp.LQ = sp.lat == SLOT_LAT_AFFINE ? q + d * d + d : q;
    sp.mu0 = sp.lat == SLOT_LAT_AFFINE ? q + 2 * d * d + d : q;
    sp.L0 = sp.lat == SLOT_LAT_AFFINE ? q + 2 * d * d + 2 * d : q;
    sp.cprior = q;
    sp.cT = sp.lat == SLOT_LAT_CATEGORICAL ? q + d : q;
    sp.SW = q;
    if (sp.lat == SLOT_LAT_SWITCHING) {
      const int nz = sp.nz, dx = d - nz;
      sp.cT = q + nz;
      sp.SW = q + nz + nz * nz;
      sp.mu0 = sp.SW + nz * (2 * dx * dx + dx);
      sp.L0 = sp.mu0 + dx;
    }
    for (int k = 0; k < kMaxSlots; ++k) sp.P[k] = m->dparams + (k < sp.K ? slot_off[5 + k] : 0);
  }
  *out = m;
  return GH_OK;
}

extern "C" int gh_model_destroy(gh_model* m) {
  if (!m) return GH_OK;
  hipSetDevice(m->ctx->device);
  if (m->dparams) hipFree(m->dparams);
  delete m;
  return GH_OK;
}

extern "C" int gh_model_state_dim(const gh_model* m, int* d) {
  if (!m || !d) return set_err(GH_E_INVAL, "null model");
  *d = m->d;
  return GH_OK;
}

// host preprocessing of one step's observation
// the slot family's observations: a chain of gh_obs, one per constrained slot
// (any subset, each at most once), into StepObs::v at the slots' offsets and
// the present bits
static int make_obs_slots(const gh_model* m, const gh_obs* in, StepObs* o) {
  const SlotParams& sp = m->slots;
  int n = 0;
  bool has_input = false;
  for (const gh_obs* e = in; e; e = e->next) {
    if (++n > kMaxSlots + 1)
      return set_err(GH_E_INVAL, "slots: more than %d observations (and an input) in one step", kMaxSlots);
    if (!e->present || !e->values) continue;
    const int k = e->slot;
    if (k == GH_SLOT_INPUT) {  // the step's latent input u_t (an Unfold argument, not a choice)
      if (sp.uoff < 0) return set_err(GH_E_INVAL, "slots: a step input for a model without inputs (latent form 2)");
      if (has_input) return set_err(GH_E_INVAL, "slots: two inputs in one step");
      if (e->n_values != m->d) return set_err(GH_E_INVAL, "slots: the input has d = %d values, got %d", m->d, e->n_values);
      for (int j = 0; j < m->d; ++j) {
        if (!std::isfinite(e->values[j])) return set_err(GH_E_INVAL, "slots: non-finite input");
        o->v[sp.uoff + j] = e->values[j];
      }
      has_input = true;
      continue;
    }
    if (k < 0 || k >= sp.K) return set_err(GH_E_INVAL, "slots: observation for slot %d (the model has %d)", k, sp.K);
    if ((o->present >> k) & 1)
      return set_err(GH_E_DISCARD, "slots: slot %d constrained twice in one step", k);  // (particle_filter.jl:168-170)
    const int mm = sp.m[k], dist = sp.dist[k];
    const int nv = dist == SLOT_MVNORMAL ? mm : 1;
    if (e->n_values != nv) return set_err(GH_E_INVAL, "slots: slot %d takes %d values, got %d", k, nv, e->n_values);
    double* v = o->v + sp.voff[k];
    const double y = e->values[0];
    if (dist == SLOT_MVNORMAL) {
      double r[kMaxObs];
      for (int j = 0; j < mm; ++j) r[j] = e->values[j] - m->slot_c[k][j];
      fwdsub(mm, 1, m->slot_LR[k].data(), r, v);
    } else if (dist == SLOT_POISSON) {
      if (!(y >= 0.0) || y != floor(y) || y > 0x1p52)
        return set_err(GH_E_INVAL, "slots: poisson value %g is not a count (poisson.jl: x::Int)", y);
      v[0] = y;
      v[1] = gh_lgamma(y + 1.0);
    } else if (dist == SLOT_BERNOULLI) {
      if (!(y == 0.0 || y == 1.0)) return set_err(GH_E_INVAL, "slots: bernoulli value %g is not 0 or 1", y);
      v[0] = y;
    } else if (dist == SLOT_CATEGORICAL) {
      if (!(y >= 0.0) || y >= (double)mm || y != floor(y))
        return set_err(GH_E_INVAL, "slots: categorical value %g is not a class in 0..%d", y, mm - 1);
      v[0] = y;
    } else {
      v[0] = y;
    }
    o->present |= 1 << k;
  }
  // the dependent slots' parent terms: fma over the (constrained) parents in slot order
  for (int k = 0; k < sp.K; ++k) {
    if (!((sp.dep >> k) & 1) || !((o->present >> k) & 1)) continue;
    double dk = 0.0;
    for (int j = 0; j < k; ++j) {
      if (sp.dg[k][j] == 0.0) continue;
      if (!((o->present >> j) & 1))
        return set_err(GH_E_INVAL, "slots: slot %d is constrained but slot %d, which it depends on, is not", k, j);
      dk = std::fma(sp.dg[k][j], o->v[sp.voff[j]], dk);
    }
    o->v[sp.doff + k] = dk;
  }
  return GH_OK;
}

static int make_obs(const gh_model* m, int t, const gh_obs* in, StepObs* o) {
  memset(o, 0, sizeof(*o));
  if (m->family == GH_FAMILY_SLOTS) {
    if (m->slots.lat == SLOT_LAT_KITAGAWA) o->ct = 8.0 * gh_cos(1.2 * (double)t);
    return make_obs_slots(m, in, o);
  }
  if (in && (in->next || in->slot != 0))
    return set_err(GH_E_INVAL, "this family has one observed address (slot 0, no chained observations)");
  o->present = (in && in->present && in->values) ? 1 : 0;
  if (m->family == GH_FAMILY_KITAGAWA) o->ct = 8.0 * gh_cos(1.2 * (double)t);
  if (!o->present) return GH_OK;
  if (m->family == GH_FAMILY_LGSSM) {
    if (in->n_values != m->dy) return set_err(GH_E_INVAL, "observation has %d values, dy = %d", in->n_values, m->dy);
    double r[kMaxObs];
    for (int i = 0; i < m->dy; ++i) r[i] = in->values[i] - m->c[i];
    fwdsub(m->dy, 1, m->LR.data(), r, o->v);
  } else if (m->family == GH_FAMILY_REGRESSION) {
    if (in->n_values != m->dy) return set_err(GH_E_INVAL, "observation has %d values, expected %d", in->n_values, m->dy);
    for (int i = 0; i < m->dy; ++i) o->v[i] = in->values[i];
  } else if (m->family == GH_FAMILY_HMM) {
    const double s = in->values[0];
    if (!(s >= 0.0) || s >= (double)m->v || s != floor(s))
      return set_err(GH_E_INVAL, "HMM observation %g is not a symbol in 0..%d", s, m->v - 1);
    o->v[0] = s;
    o->sym = (int)s;
  } else {
    o->v[0] = in->values[0];
  }
  return GH_OK;
}

// The Gaussian custom proposal's arguments (KitGaussModel): o.v[1..4] =
// (alpha, beta, gamma, sigma_q), o.v[5] = 1/(2 sigma_q^2), o.v[6] =
// -0.5 log(2 pi sigma_q^2).
static int make_obs_gauss(const gh_model* m, int t, const gh_obs* in, const double* q, StepObs* o) {
  CHECK(make_obs(m, t, in, o));
  if (!(q[3] > 0.0)) return set_err(GH_E_INVAL, "Gaussian proposal: sigma_q must be > 0");
  const double v = q[3] * q[3];
  for (int i = 0; i < 4; ++i) o->v[1 + i] = q[i];
  o->v[5] = 1.0 / (2.0 * v);
  o->v[6] = -0.5 * gh_log(2.0 * 0x1.921fb54442d18p+1 * v);
  return GH_OK;
}

// The optimal proposal's per-step vectors (LGOptModel): t = 1: o.v[0, d) =
// mu_1 = mu0 + K_1 (y - c - H mu0), o.ct = log N(y; H mu0 + c, S_1); t >= 2:
// o.v[0, d) = g_t = F b + K (y - c), o.v[d, d + dy) = L_S^-1 (y - c) - L_S^-1 H b.
// the observation with u_t of the linear proposal behind it (o.v[dy + i])
static int make_obs_lin(const gh_model* m, int t, const gh_obs* in, const double* u, StepObs* o) {
  CHECK(make_obs(m, t, in, o));
  const int at = m->family == GH_FAMILY_SLOTS ? m->slots.qoff : m->dy;
  for (int i = 0; i < m->d; ++i) o->v[at + i] = u[i];
  return GH_OK;
}

static int make_obs_opt(const gh_model* m, int t, const gh_obs* in, StepObs* o) {
  CHECK(make_obs(m, t, in, o));
  if (!o->present) return GH_OK;
  const int d = m->d, dy = m->dy;
  double r[kMaxObs];
  for (int i = 0; i < dy; ++i) r[i] = in->values[i] - m->c[i];
  if (t == 1) {
    double e[kMaxObs], u[kMaxObs];
    for (int q = 0; q < dy; ++q) {
      double acc = r[q];
      for (int j = 0; j < d; ++j) acc = fma(-m->H[q * d + j], m->mu0[j], acc);
      e[q] = acc;
    }
    fwdsub(dy, 1, m->LS1.data(), e, u);
    double quad = 0.0;
    for (int q = 0; q < dy; ++q) quad = fma(u[q], u[q], quad);
    o->ct = m->cstS1 - 0.5 * quad;
    for (int i = 0; i < d; ++i) {
      double acc = m->mu0[i];
      for (int q = 0; q < dy; ++q) acc = fma(m->Kt1[q * d + i], e[q], acc);
      o->v[i] = acc;
    }
    return GH_OK;
  }
  double ls[kMaxObs];
  fwdsub(dy, 1, m->LS.data(), r, ls);
  for (int i = 0; i < d; ++i) {
    double acc = 0.0;
    for (int q = 0; q < dy; ++q) acc = fma(m->Kt[q * d + i], r[q], acc);
    o->v[i] = m->Fb[i] + acc;
  }
  for (int q = 0; q < dy; ++q) o->v[d + q] = ls[q] - m->Wb[q];
  return GH_OK;
}

static bool proposal_ok(const gh_model* m, int proposal) {
  if (proposal == GH_PROPOSAL_DEFAULT) return true;
  if (proposal == GH_PROPOSAL_GAUSSIAN) return m->family == GH_FAMILY_KITAGAWA;
  if (proposal == GH_PROPOSAL_LINEAR)  // (u_t follows the step's observed values)
    return (m->family == GH_FAMILY_LGSSM && m->d + m->dy <= kMaxObs) ||
           (m->family == GH_FAMILY_SLOTS && m->slots.lat != SLOT_LAT_CATEGORICAL && m->slots.lat != SLOT_LAT_SWITCHING &&
            m->d + m->slots.qoff <= kMaxObs);
  if (proposal != GH_PROPOSAL_OPTIMAL) return false;
  return m->family == GH_FAMILY_HMM || (m->family == GH_FAMILY_LGSSM && m->lg_opt);
}

// ------------------------------------------------------------ the PF state
struct gh_pf {
  gh_model* m = nullptr;
  gh_ctx* ctx = nullptr;
  hipStream_t s = nullptr;
  int D = 0;
  int64_t n_global = 0, n = 0, lo = 0;
  uint64_t seed = 0;
  gh_pf_opts opts{};
  int t = 0;                      // completed steps
  int resample_calls = 0;         // maybe_resample calls since the last step
  // states: history slots (record_history) or 2 ping-pong slots
  std::vector<double*> xs;        // index t-1 (history) or t&1
  std::vector<int32_t*> ancs;     // index t-1: ancestors used by step t
  int32_t* anc_scratch = nullptr;
  double* logw = nullptr;
  uint64_t* C = nullptr;
  uint32_t* mark = nullptr;       // systematic: tagged range starts per slot
  uint32_t* cmark = nullptr;      // systematic: tagged carry per 64-slot group
  uint64_t epoch = 0;             // resample counter for the tags (since the last clear)
  int mark_bits = 1;              // low bits of a mark word holding the ancestor
  bool marks_pending = false;     // last resample's ancestors only exist as marks
  bool stats_valid = false;       // stats_all holds the last step's (M, S, S2) (one rank)
  uint64_t* tsum = nullptr;       // k_resample1: published tile totals (+ tile sums, 3 x n_tiles)
  int64_t n_tiles = 0;
  bool max_only = false;          // the last step wrote block maxima only (sums left to k_resample1)
  bool step_max_only = false;     // gh_pf_run: the next step may write block maxima only
  int rs_grid = 0;                // k_resample1 / k_rank_* tiles (blocks); 0: not usable
  int rs_it = 0;                  // particles per thread of those kernels (4, 8 or 16)
  uint64_t* amax = nullptr;       // [2][kAmaxShards * kAmaxStride] a max_only step's atomic-max shards (by t & 1)
  bool amax_armed = false;        // k_resample1 emptied the shards of the next step
  bool amax_valid = false;        // the last step wrote its shards
  uint64_t* bsum = nullptr;
  int64_t nb_scan = 0;
  int64_t nb_step = 0;
  int64_t nb_part = 0;             // block partials the last step kernel wrote (pair kernels: n / 512)
  bool pairs = false;             // the default step runs the pair kernel (512 particles per block)
  bool last_pairs = false;        // the last step kernel was the pair kernel
  double *pm = nullptr, *ps = nullptr, *ps2 = nullptr;
  DevScalars* dev = nullptr;
  double* stats_all = nullptr;    // [3*world]
  uint64_t* totals_all = nullptr; // [world]
  int cap = 0;                    // history/ess capacity (steps)
  double* ess_hist = nullptr;     // [cap+2]
  int32_t* res_hist = nullptr;    // [cap+2]
  // multi-rank resample exchange
  double* rows_recv = nullptr;    // [n][D+1] rows received for this rank's slots
  double* rows_send = nullptr;    // [send_cap][D+1] rows this rank sends
  int32_t* xanc = nullptr;        // [send_cap] local ancestors of the sent rows
  int64_t send_cap = 0;
  // multinomial on R ranks (exchange_states_mn): per global slot its key (the
  // rank holding its target), its rank among the range's slots with that key
  // and its local ancestor when the key is this rank; per-block key counts
  int32_t* mn_key = nullptr;
  int32_t* mn_pos = nullptr;
  int32_t* mn_anc = nullptr;
  int32_t* mn_bcnt = nullptr;
  int32_t* mn_boff = nullptr;
  int send_grows = 0;              // resamples whose rows overflowed the bounded send buffer
  int64_t* gparent = nullptr;     // [n] global parent ids of the last exchange
  hipStream_t aux = nullptr;      // multi-rank: side stream (the plan's D2H read, the row exchange)
  hipEvent_t ev_tot = nullptr;    // multi-rank: totals all-gathered
  hipEvent_t ev_plan = nullptr;   //   fire flag + totals landed in h_plan
  hipEvent_t ev_rb = nullptr;     //   k_rank_b packed the rows
  hipEvent_t ev_x = nullptr;      //   rows exchanged
  uint64_t* h_plan = nullptr;     // pinned: [fire, totals[R]] (k_rank_a) or the R rank records (k_rank_a2)
  uint64_t* h_mail = nullptr;     // pinned, coherent: [tag, R rank records] written by k_rank_b (batched loop)
  uint64_t* d_mail = nullptr;     //   its device alias (the kernels' pointer)
  // maybe_resample!'s decision for the host (one rank): pinned, coherent [tag,
  // fire | err << 32, ess] posted by k_resample1's block 0 (no stream sync)
  uint64_t* h_dec = nullptr;
  uint64_t* d_dec = nullptr;
  uint64_t dec_seq = 0;           // the tag of the last decision posted there
  bool dec_posted = false;        // the last maybe_resample! posts its decision to h_dec
  bool no_max_only = false;       // gh_pf_step_params: the step writes full partials
  bool mr_stale = false;          // multi-rank: the last step left its weight sums to the next resample
  // peer transport: every rank's row buffer as mapped here (prow[rank] =
  // rows_recv, fine-grained, followed by R tag words indexed by sender) and
  // the row exchanges posted so far
  double* prow[kPeerMaxRanks] = {};
  PeerRounds pr;                  // the set-up's bootstrap rounds (fail-together)
  bool peer_ready = false;        // set up on every rank: destruction fences the ranks
  bool ab_fits = false;           // the grid is co-resident for k_rank_ab (it polls every tile)
  bool no_fused_rank = false;     // (GH_NO_FUSED_RANK in the environment: the two-kernel peer resample, for A/B)
  uint64_t* ptag[kPeerMaxRanks] = {};
  uint64_t row_use = 0;
  // multi-rank genealogy (record_history): per step, the rows received for
  // it (the parents on other ranks; D + 1 doubles each, row-indexed), kept by
  // the step's part-2 launch; chunked device storage
  std::vector<double*> rh_step;   // index t-1 (nullptr: none received)
  std::vector<int64_t> rh_cnt;    // index t-1: rows kept for step t
  std::vector<char*> rh_chunks;
  size_t rh_used = 0, rh_cap = 0;
  int64_t* dlo = nullptr;         // [R + 1] floor(N k / R): the ranks' first global slots
  uint64_t mail_seq = 0;          //   the tag of the last plan posted there
  bool plan_recs = false;         // the pending plan is k_rank_a2's records (the host takes the decision)
  double plan_thr = 0.0;          //   at this threshold
  uint64_t* amax_all = nullptr;   // multi-rank: [R][kAmaxShards * kAmaxStride] all-gathered shard words
  uint64_t* rec = nullptr;        // multi-rank: [kRecWords] this rank's record (k_rank_a2)
  uint64_t* recs_all = nullptr;   //   [R][kRecWords] all-gathered
  bool plan_pending = false;      // k_rank_b enqueued; the host has not read the totals yet
  bool rem_fire = false;          // the resample fired (read by finish_plan)
  int64_t rem_ra = 0, rem_rb = 0; // local slots [0, ra) and [rb, n) take received rows
  int mark_mode = 1;              // 1: one-rank marks; 2: marks + received rows
  // rejuvenation (gh_pf_rejuvenate): the current step's observation and the
  // MH moves already applied at this step (their draw windows)
  StepObs last_obs{};
  std::vector<StepObs> obs_hist;  // every step's observation (prior form), index t-1: trace scores
  std::vector<std::vector<double>> raw_obs;  // every step's observation as given (index t-1; empty: none)
  uint32_t rejuv_moves = 0;
  unsigned long long* acc_count = nullptr;
  // the Gaussian custom proposal's last arguments (alpha, beta, gamma, sigma_q)
  double qargs[4] = {0, 0, 0, 0};
  bool has_q = false;
  // the LGSSM's linear-Gaussian custom proposal (GH_PROPOSAL_LINEAR): device P | chol(Sigma_q)
  double* qlin = nullptr;
  double cstq = 0.0;
  bool has_qlin = false;
  std::vector<double> qlin_u;     // u_t of the next steps
  // conditional SMC (gh_csmc.h): particle 0 is pinned to a given trajectory
  bool cond = false;
  double* pin = nullptr;          // [D] this step's distinguished state, [D] its new log weight
  std::vector<void*> chunks;      // history allocations (record_history)
  // kernel timing
  std::vector<hipEvent_t> ev;
  size_t ev_used = 0;
  double ev_ms = 0.0;
  int64_t ev_count = 0;
};

static int64_t split_lo(int64_t n, int r, int R) { return (n * r) / R; }

static void log_raw_obs(gh_pf* pf, int t, const gh_obs* obs);

// Tile size of the one-launch resample kernels: the smallest 1024 x IT tile
// whose grid fits the co-resident capacity (their grid barrier needs every
// block resident), IT = 4 only while the step partials fit its registers.
template <class K>
static int occ_blocks(K kernel) {
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, kRsBlock, 0) != hipSuccess) occ = 0;
  return occ;
}
template <int IT>
static int resample_cap(int cus) {  // one rank: k_resample1's co-resident blocks
  int o = std::min(occ_blocks(k_resample1<true, IT, true>), occ_blocks(k_resample1<true, IT, false>));
  o = std::min(o, std::min(occ_blocks(k_resample1<false, IT, true>), occ_blocks(k_resample1<false, IT, false>)));
  return o * cus;
}
template <int IT>
static int rank_cap(int cus) {  // multi-rank: k_rank_a's (k_rank_b has no grid barrier)
  return occ_blocks(k_rank_a<IT>) * cus;
}
template <int IT>
static int rank_ab_cap(int cus) {  // the fused peer resample's co-resident blocks
  return occ_blocks(k_rank_ab<IT>) * cus;
}
static void pick_ab(gh_pf* pf) {  // the fused kernel only where its grid fits
  const int cus = pf->ctx->cus;
  const int cap = pf->rs_it == 4 ? rank_ab_cap<4>(cus) : pf->rs_it == 8 ? rank_ab_cap<8>(cus)
                : pf->rs_it == 16 ? rank_ab_cap<16>(cus) : 0;
  // judged on the largest shard's grid, as the tiles are, so that every rank
  // takes the same path
  const int64_t n = (pf->n_global + pf->ctx->world - 1) / pf->ctx->world;
  const int64_t g = pf->rs_it ? (n + (int64_t)pf->rs_it * kRsBlock - 1) / ((int64_t)pf->rs_it * kRsBlock) : 0;
  pf->ab_fits = pf->rs_grid > 0 && g <= cap;
}
static void pick_resample_tiles_(gh_pf* pf, int64_t n);
static void pick_resample_tiles(gh_pf* pf, int64_t n) {
  pick_resample_tiles_(pf, n);
  if (mr(pf->ctx) && pf->ctx->peer) pick_ab(pf);
}
static void pick_resample_tiles_(gh_pf* pf, int64_t n) {
  const int cus = pf->ctx->cus;
  pf->rs_grid = 0;
  pf->rs_it = 0;
  // multi-rank: the choice (tile size, usable or not) is made for the largest
  // shard, ceil(N / R), so that every rank takes the same resample path and
  // posts the same collectives; each rank's grid covers its own particles
  const int64_t n_own = n;
  if (mr(pf->ctx)) n = (pf->n_global + pf->ctx->world - 1) / pf->ctx->world;
  // the polling waves read at most 64 * kRsPoll tile words
  const int64_t gmax = 64 * kRsPoll;
  auto grid_of = [&](int it) { return (n + (int64_t)it * kRsBlock - 1) / ((int64_t)it * kRsBlock); };
  // the smallest tile whose grid is co-resident: more waves per CU, fewer
  // particles per thread in every phase; IT <= kRsPart keeps the partials in
  // registers only while they fit
  struct Cand {
    int it;
    int cap;
  };
  std::vector<Cand> cands;
  if (!mr(pf->ctx)) {
    // (IT = 2, two 1024-thread blocks per CU, measured slower: 59.4 vs 54.7 us per C2 step)
    cands = {{4, resample_cap<4>(cus)}, {8, resample_cap<8>(cus)}, {16, resample_cap<16>(cus)}};
  } else {
    cands = {{4, rank_cap<4>(cus)}, {8, rank_cap<8>(cus)}, {16, rank_cap<16>(cus)}};
  }
  for (const Cand& c : cands) {
    const int64_t nb_part = (n + (pf->pairs ? 2 : 1) * kBlock - 1) / ((pf->pairs ? 2 : 1) * kBlock);
    if (c.it <= kRsPart && nb_part > (int64_t)kRsPart * kRsBlock) continue;
    const int64_t g = grid_of(c.it);
    if (g <= std::min<int64_t>(gmax, c.cap)) {
      pf->rs_it = c.it;
      pf->rs_grid = (int)std::max<int64_t>(1, (n_own + (int64_t)c.it * kRsBlock - 1) / ((int64_t)c.it * kRsBlock));
      return;
    }
  }
}

// device -> host copy ordered after everything enqueued on the filter's stream
// (the stream is non-blocking, so a plain hipMemcpy could overtake it)
static int d2h(gh_pf* pf, void* dst, const void* src, size_t bytes) {
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, pf->s));
  HIP_TRY(hipStreamSynchronize(pf->s));
  return GH_OK;
}

static double* slot_x(gh_pf* pf, int t) {  // states of step t (1-based)
  return pf->opts.record_history ? pf->xs[t - 1] : pf->xs[t & 1];
}

static int ensure_capacity(gh_pf* pf, int steps) {
  // history slots, ancestor slots and per-step records for steps 1..steps
  if (steps <= pf->cap) return GH_OK;
  int nc = pf->cap ? pf->cap : 16;
  while (nc < steps) nc *= 2;
  const size_t xbytes = sizeof(double) * (size_t)slot_doubles(pf->n, pf->D);
  const size_t abytes = sizeof(int32_t) * (size_t)(pf->n ? pf->n : 1);
  if (pf->opts.record_history) {
    // allocate the new slots as one chunk (no hipMalloc per step)
    const int add = nc - pf->cap;
    char* chunk = nullptr;
    if (hipMalloc(&chunk, (xbytes + abytes) * (size_t)add) != hipSuccess)
      return set_err(GH_E_NOMEM, "history: cannot allocate %d more steps", add);
    pf->chunks.push_back(chunk);
    for (int i = 0; i < add; ++i) {
      pf->xs.push_back((double*)(chunk + (xbytes + abytes) * i));
      pf->ancs.push_back((int32_t*)(chunk + (xbytes + abytes) * i + xbytes));
    }
  }
  double* ne = nullptr;
  int32_t* nr = nullptr;
  HIP_TRY(hipMalloc(&ne, sizeof(double) * (nc + 2)));
  HIP_TRY(hipMalloc(&nr, sizeof(int32_t) * (nc + 2)));
  HIP_TRY(hipMemsetAsync(nr, 0, sizeof(int32_t) * (nc + 2), pf->s));
  HIP_TRY(hipMemsetAsync(ne, 0, sizeof(double) * (nc + 2), pf->s));
  if (pf->ess_hist) {
    HIP_TRY(hipMemcpyAsync(ne, pf->ess_hist, sizeof(double) * (pf->cap + 2), hipMemcpyDeviceToDevice, pf->s));
    HIP_TRY(hipMemcpyAsync(nr, pf->res_hist, sizeof(int32_t) * (pf->cap + 2), hipMemcpyDeviceToDevice, pf->s));
    HIP_TRY(hipStreamSynchronize(pf->s));
    hipFree(pf->ess_hist);
    hipFree(pf->res_hist);
  }
  pf->ess_hist = ne;
  pf->res_hist = nr;
  pf->cap = nc;
  return GH_OK;
}

static int32_t* anc_for_step(gh_pf* pf, int t) {  // ancestors consumed by step t
  return pf->opts.record_history ? pf->ancs[t - 1] : pf->ancs[0];
}

extern "C" void gh_pf_opts_default(gh_pf_opts* o) {
  memset(o, 0, sizeof(*o));
  o->resampler = GH_RESAMPLE_SYSTEMATIC;
  o->record_history = 1;
}

static void pf_free(gh_pf* pf) {
  if (!pf) return;
  hipSetDevice(pf->ctx->device);
  hipStreamSynchronize(pf->s);
  if (pf->aux) hipStreamSynchronize(pf->aux);
  if (pf->peer_ready) {
    // peer transport: other ranks' kernels store rows and tags into this
    // rank's row buffer; every rank has drained its stream before this fence,
    // so none is still writing when the buffer is freed (gh_pf_destroy is
    // collective on this transport)
    uint8_t one = 1;
    std::vector<uint8_t> all((size_t)pf->ctx->world);
    pf->ctx->hc.allgather(pf->ctx->hc.user, &one, all.data(), 1);
  }
  for (auto c : pf->chunks) hipFree(c);
  for (auto e : pf->ev) hipEventDestroy(e);
  hipFree(pf->logw); hipFree(pf->C); hipFree(pf->mark); hipFree(pf->cmark); hipFree(pf->bsum); hipFree(pf->pm); hipFree(pf->ps);
  hipFree(pf->ps2); hipFree(pf->dev); hipFree(pf->tsum); hipFree(pf->stats_all); hipFree(pf->totals_all);
  hipFree(pf->ess_hist); hipFree(pf->res_hist); hipFree(pf->anc_scratch);
  hipFree(pf->rows_recv); hipFree(pf->rows_send); hipFree(pf->xanc); hipFree(pf->gparent);
  hipFree(pf->mn_key); hipFree(pf->mn_pos); hipFree(pf->mn_anc); hipFree(pf->mn_bcnt); hipFree(pf->mn_boff);
  hipFree(pf->acc_count); hipFree(pf->pin); hipFree(pf->amax);
  hipFree(pf->amax_all); hipFree(pf->rec); hipFree(pf->recs_all); hipFree(pf->qlin);
  if (pf->aux) hipStreamDestroy(pf->aux);
  if (pf->ev_tot) hipEventDestroy(pf->ev_tot);
  if (pf->ev_plan) hipEventDestroy(pf->ev_plan);
  if (pf->ev_rb) hipEventDestroy(pf->ev_rb);
  if (pf->ev_x) hipEventDestroy(pf->ev_x);
  if (pf->h_plan) hipHostFree(pf->h_plan);
  if (pf->h_mail) hipHostFree(pf->h_mail);
  if (pf->h_dec) hipHostFree(pf->h_dec);
  for (auto c : pf->rh_chunks) hipFree(c);
  if (pf->ctx->peer) ipc_close(pf->ctx, (void**)pf->prow);
  hipFree(pf->dlo);
  if (!pf->opts.record_history) {
    for (auto p : pf->xs) hipFree(p);
    for (auto p : pf->ancs) hipFree(p);
  }
  pf->ctx->n_filters--;
  delete pf;
}

extern "C" int gh_pf_destroy(gh_pf* pf) {
  pf_free(pf);
  return GH_OK;
}

// ----------------------------------------------------------- kernel launch
// Kernel-timing events: no system-scope fence when an event is recorded.  The
// default event writes back and invalidates the caches at the kernel's end,
// so a timed step kernel pushed the ~80 MB of states it had just written out
// of L2 / Infinity Cache synchronously and the run lost 25-60 us per timed
// launch (C2, measured); the timestamps are read after a stream
// synchronisation, which acquires anyway.
constexpr unsigned kTimingEventFlags = hipEventDisableSystemFence;

template <class M, class = void>
struct has_pairs : std::false_type {};
template <class M>
struct has_pairs<M, std::void_t<decltype(M::kPairs)>> : std::bool_constant<M::kPairs> {};

// the pair kernel steps the filters of paired models (pair mates in one lane
// needs a particle offset that is a multiple of 128; every rank decides for
// itself — the values are the same either way)
template <class Model>
static bool use_pairs(const gh_pf* pf) {
  // (conditional filters re-fold block 0 as 256 particles: k_pin_post)
  if constexpr (has_pairs<Model>::value) return (pf->lo & 127) == 0 && !pf->cond;
  return false;
}

template <class Model>
static void launch_step_t(gh_pf* pf, const typename Model::Params& p, const StepObs& o,
                          const StepArgs& a0, bool init, hipEvent_t e0, hipEvent_t e1) {
  StepArgs a = a0;
  a.nvb = (a.n + kBlock - 1) / kBlock;
  if constexpr (has_pairs<Model>::value) {
    if (use_pairs<Model>(pf)) {
      const dim3 grid((unsigned)(a.grid_blocks > 0 ? a.grid_blocks : (a.n + 2 * kBlock - 1) / (2 * kBlock))),
          block(kBlock);
      if (a.part != 2) {
        pf->nb_part = grid.x;
        pf->last_pairs = true;
      }
      if (init)
        hipExtLaunchKernelGGL((k_step_pairs<Model, true>), grid, block, 0, pf->s, e0, e1, 0,
                              (const double*)pf->m->dparams, p, o, a);
      else if (a.part == 2)
        hipExtLaunchKernelGGL((k_step_pairs<Model, false, true>), grid, block, 0, pf->s, e0, e1, 0,
                              (const double*)pf->m->dparams, p, o, a);
      else
        hipExtLaunchKernelGGL((k_step_pairs<Model, false>), grid, block, 0, pf->s, e0, e1, 0,
                              (const double*)pf->m->dparams, p, o, a);
      return;
    }
  }
  if (a.part != 2) {
    pf->nb_part = pf->nb_step;
    pf->last_pairs = false;
  }
  const dim3 grid((unsigned)(a.grid_blocks > 0 ? a.grid_blocks : (a.part == 2 ? a.nvb : pf->nb_step))), block(kBlock);
  // the timed launch records its events at the kernel's own start and end
  if (init)
    hipExtLaunchKernelGGL((k_step<Model, true>), grid, block, 0, pf->s, e0, e1, 0, (const double*)pf->m->dparams,
                          p, o, a);
  else if (a.part == 2)  // one launch over two block ranges (the block remap's own instantiation)
    hipExtLaunchKernelGGL((k_step<Model, false, true>), grid, block, 0, pf->s, e0, e1, 0,
                          (const double*)pf->m->dparams, p, o, a);
  else
    hipExtLaunchKernelGGL((k_step<Model, false>), grid, block, 0, pf->s, e0, e1, 0, (const double*)pf->m->dparams,
                          p, o, a);
}

// fold the step kernel's block partials (nb of them) into the rank's (M, S, S2)
static void launch_fold(gh_pf* pf, const StepArgs& a, bool init, int64_t nb) {
  hipLaunchKernelGGL(k_fold, dim3(1), dim3(1024), 0, pf->s, pf->pm, pf->ps, pf->ps2, (int)nb, a.stats_out, pf->dev,
                     init ? 0 : 1, 0.0, pf->n_global);
}

// one rank: make stats_all current (the fold is otherwise done by k_resample1).
// After a max-only step the block sums are recomputed first (k_block_sums:
// the values a full-partials step would have written).
static int ensure_stats(gh_pf* pf) {
  if (mr(pf->ctx)) {
    // (recomputing them here would be a collective only this caller enters)
    if (pf->mr_stale)
      return set_err(GH_E_STATE, "multi-rank: the last step left its weight sums to the next maybe_resample "
                                 "(a gh_pf_run that stopped early); step again first");
    return GH_OK;
  }
  if (pf->stats_valid) return GH_OK;
  if (pf->max_only && pf->n > 0) {
    if (pf->last_pairs)
      hipLaunchKernelGGL(k_block_sums<true>, dim3((unsigned)pf->nb_part), dim3(kBlock), 0, pf->s,
                         (const double*)pf->logw, pf->n, (const double*)pf->pm, pf->ps, pf->ps2);
    else
      hipLaunchKernelGGL(k_block_sums<false>, dim3((unsigned)pf->nb_part), dim3(kBlock), 0, pf->s,
                         (const double*)pf->logw, pf->n, (const double*)pf->pm, pf->ps, pf->ps2);
  }
  hipLaunchKernelGGL(k_fold, dim3(1), dim3(1024), 0, pf->s, pf->pm, pf->ps, pf->ps2, (int)pf->nb_part,
                     pf->stats_all, pf->dev, 0, 0.0, pf->n_global);
  HIP_TRY(hipGetLastError());
  pf->stats_valid = true;
  return GH_OK;
}

// the device resample flags describe the current particles only if a
// maybe_resample! was enqueued since the last step
static int flags_live(const gh_pf* pf) { return pf->resample_calls > 0 ? 1 : 0; }

// Call f(Model{}, params) with the device model type of m (the one switch
// over families and instantiated LGSSM shapes).
template <class F>
static int with_model(const gh_model* m, F&& f) {
  switch (m->family) {
    case GH_FAMILY_LGSSM:
      switch (m->d) {
#define GH_LG_CASE(DD)                                   \
  case DD:                                               \
    switch (m->lg_struct) {                              \
      case 1: f(LGModel<DD, 1>{}, m->lg); break;         \
      case 2: f(LGModel<DD, 2>{}, m->lg); break;         \
      case 3: f(LGModel<DD, 3>{}, m->lg); break;         \
      default: f(LGModel<DD, 0>{}, m->lg); break;        \
    }                                                    \
    break;
        GH_LG_CASE(1) GH_LG_CASE(2) GH_LG_CASE(3) GH_LG_CASE(4) GH_LG_CASE(5) GH_LG_CASE(6)
        GH_LG_CASE(7) GH_LG_CASE(8) GH_LG_CASE(9) GH_LG_CASE(10) GH_LG_CASE(11) GH_LG_CASE(12)
        GH_LG_CASE(13) GH_LG_CASE(14) GH_LG_CASE(15) GH_LG_CASE(16)
#undef GH_LG_CASE
        default: return set_err(GH_E_INVAL, "LGSSM d=%d not instantiated", m->d);
      }
      break;
    case GH_FAMILY_HMM: f(HMMModel{}, m->hmm); break;
    case GH_FAMILY_KITAGAWA: f(KitModel{}, m->kit); break;
    case GH_FAMILY_REGRESSION: f(RegModel{}, m->reg); break;
    case GH_FAMILY_SLOTS:
      switch (m->d) {
#define GH_SL_CASE(DD) \
  case DD:                                                    \
    if (m->slot_ext) f(SlotModel<DD, true>{}, m->slots);      \
    else f(SlotModel<DD>{}, m->slots);                        \
    break;
        GH_SL_CASE(1) GH_SL_CASE(2) GH_SL_CASE(3) GH_SL_CASE(4) GH_SL_CASE(5) GH_SL_CASE(6) GH_SL_CASE(7)
        GH_SL_CASE(8) GH_SL_CASE(9) GH_SL_CASE(10) GH_SL_CASE(11) GH_SL_CASE(12) GH_SL_CASE(13) GH_SL_CASE(14)
        GH_SL_CASE(15) GH_SL_CASE(16)
#undef GH_SL_CASE
        default: return set_err(GH_E_INVAL, "slots d=%d not instantiated", m->d);
      }
      break;
    default: return set_err(GH_E_INVAL, "unknown family");
  }
  return GH_OK;
}

static int launch_step(gh_pf* pf, const StepObs& o, const StepArgs& a, bool init, hipEvent_t e0 = nullptr,
                       hipEvent_t e1 = nullptr) {
  if (!init && pf->m->family == GH_FAMILY_REGRESSION)
    return set_err(GH_E_INVAL, "the regression model has no time steps");
  if (a.proposal == GH_PROPOSAL_GAUSSIAN) {  // Kitagawa only (proposal_ok); its own functor
    launch_step_t<KitGaussModel>(pf, pf->m->kit, o, a, init, e0, e1);
    HIP_TRY(hipGetLastError());
    return GH_OK;
  }
  if (a.proposal == GH_PROPOSAL_LINEAR && pf->m->family == GH_FAMILY_SLOTS) {  // (proposal_ok)
    SlotParams p = pf->m->slots;
    p.QP = pf->qlin;
    p.QL = pf->qlin + pf->D * pf->D;
    p.cstq = pf->cstq;
    switch (pf->m->d) {
#define GH_SLL_CASE(DD) \
  case DD:                                                                     \
    if (pf->m->slot_ext) launch_step_t<SlotLinModel<DD, true>>(pf, p, o, a, init, e0, e1); \
    else launch_step_t<SlotLinModel<DD>>(pf, p, o, a, init, e0, e1);                     \
    break;
      GH_SLL_CASE(1) GH_SLL_CASE(2) GH_SLL_CASE(3) GH_SLL_CASE(4) GH_SLL_CASE(5) GH_SLL_CASE(6)
      GH_SLL_CASE(7) GH_SLL_CASE(8) GH_SLL_CASE(9) GH_SLL_CASE(10) GH_SLL_CASE(11) GH_SLL_CASE(12)
      GH_SLL_CASE(13) GH_SLL_CASE(14) GH_SLL_CASE(15) GH_SLL_CASE(16)
#undef GH_SLL_CASE
      default: return set_err(GH_E_INVAL, "slot model d=%d not instantiated", pf->m->d);
    }
    HIP_TRY(hipGetLastError());
    return GH_OK;
  }
  if (a.proposal == GH_PROPOSAL_LINEAR) {  // LGSSM (proposal_ok); P and chol(Sigma_q) in the filter's buffer
    LGParams p = pf->m->lg;
    p.QP = pf->qlin;
    p.QL = pf->qlin + pf->D * pf->D;
    p.cstq = pf->cstq;
    switch (pf->m->d) {
#define GH_LGL_CASE(DD) \
  case DD: launch_step_t<LGLinModel<DD>>(pf, p, o, a, init, e0, e1); break;
      GH_LGL_CASE(1) GH_LGL_CASE(2) GH_LGL_CASE(3) GH_LGL_CASE(4) GH_LGL_CASE(5) GH_LGL_CASE(6)
      GH_LGL_CASE(7) GH_LGL_CASE(8) GH_LGL_CASE(9) GH_LGL_CASE(10) GH_LGL_CASE(11) GH_LGL_CASE(12)
      GH_LGL_CASE(13) GH_LGL_CASE(14) GH_LGL_CASE(15) GH_LGL_CASE(16)
#undef GH_LGL_CASE
      default: return set_err(GH_E_INVAL, "LGSSM d=%d not instantiated", pf->m->d);
    }
    HIP_TRY(hipGetLastError());
    return GH_OK;
  }
  if (a.proposal == GH_PROPOSAL_OPTIMAL && pf->m->family == GH_FAMILY_LGSSM) {
    // the LGSSM's locally optimal proposal is its own functor (the default
    // step kernel stays free of the proposal's code and registers)
    switch (pf->m->d) {
#define GH_LGO_CASE(DD) \
  case DD: launch_step_t<LGOptModel<DD>>(pf, pf->m->lg, o, a, init, e0, e1); break;
      GH_LGO_CASE(1) GH_LGO_CASE(2) GH_LGO_CASE(3) GH_LGO_CASE(4) GH_LGO_CASE(5) GH_LGO_CASE(6)
      GH_LGO_CASE(7) GH_LGO_CASE(8) GH_LGO_CASE(9) GH_LGO_CASE(10) GH_LGO_CASE(11) GH_LGO_CASE(12)
      GH_LGO_CASE(13) GH_LGO_CASE(14) GH_LGO_CASE(15) GH_LGO_CASE(16)
#undef GH_LGO_CASE
      default: return set_err(GH_E_INVAL, "LGSSM d=%d not instantiated", pf->m->d);
    }
    HIP_TRY(hipGetLastError());
    return GH_OK;
  }
  CHECK(with_model(pf->m, [&](auto model, const auto& p) {
    launch_step_t<decltype(model)>(pf, p, o, a, init, e0, e1);
  }));
  HIP_TRY(hipGetLastError());
  return GH_OK;
}

static int finish_plan(gh_pf* pf);

// The genealogy record of step t's received rows (count of them): chunked
// device storage, released with the filter.
static int rhist_reserve(gh_pf* pf, int t, int64_t count, double** out) {
  *out = nullptr;
  if ((int)pf->rh_step.size() < t) pf->rh_step.resize(t, nullptr);
  if ((int)pf->rh_cnt.size() < t) pf->rh_cnt.resize(t, 0);
  pf->rh_step[t - 1] = nullptr;
  pf->rh_cnt[t - 1] = 0;
  if (count <= 0) return GH_OK;
  const size_t bytes = (sizeof(double) * (size_t)(pf->D + 1) * (size_t)count + 255) & ~(size_t)255;
  if (pf->rh_used + bytes > pf->rh_cap) {
    const size_t cap = std::max(bytes, (size_t)64 << 20);
    char* c = nullptr;
    if (hipMalloc(&c, cap) != hipSuccess) return set_err(GH_E_NOMEM, "genealogy rows (%zu bytes)", cap);
    pf->rh_chunks.push_back(c);
    pf->rh_used = 0;
    pf->rh_cap = cap;
  }
  *out = (double*)(pf->rh_chunks.back() + pf->rh_used);
  pf->rh_used += bytes;
  pf->rh_step[t - 1] = *out;
  pf->rh_cnt[t - 1] = count;
  return GH_OK;
}

// Multi-rank, after the step kernel: when the step followed a resample it was
// enqueued before the host read the plan (part 1); now the plan is read, the
// rows exchanged and the tiles holding slots that take received rows run
// again (part 2).  Then the fold of the block partials.
static int finish_split(gh_pf* pf, const StepObs& o, const StepArgs& a, bool init) {
  if (a.part == 1) {
    CHECK(finish_plan(pf));
    if (pf->rem_fire) {
      // tiles [0, tA) and [tB, nb) hold the slots [0, ra) and [rb, n) (tiles
      // of the step kernel's blocks: 512 slots for the pair kernel)
      const int64_t kb = pf->last_pairs ? 2 * kBlock : kBlock;
      const int64_t n = pf->n, nb = (n + kb - 1) / kb, ra = pf->rem_ra, rb = pf->rem_rb;
      int64_t tA = (ra + kb - 1) / kb;
      int64_t tB = rb < n ? rb / kb : nb;
      if (tB <= tA) {  // the ranges meet: one launch over every tile
        tA = nb;
        tB = nb;
      }
      if (tA > 0 || tB < nb) {  // one launch: blocks [0, tA) and, remapped, [tB, nb)
        StepArgs b = a;
        b.part = 2;
        b.vb_split = tA;
        b.vb_skip = tB - tA;
        b.grid_blocks = tA + (nb - tB);
        if (pf->opts.record_history) CHECK(rhist_reserve(pf, (int)a.t, ra + (n - rb), &b.rhist));
        CHECK(launch_step(pf, o, b, init));
      }
    }
  }
  if (!a.max_only) launch_fold(pf, a, init, pf->nb_part);
  return GH_OK;
}

// the step kernel (timed alone when opts.time_kernels).  Multi-rank: the
// fold follows at once (its triple is all-gathered every step); one rank: the
// next maybe_resample! folds inside k_resample1, other readers fold on demand.
static int timed_step(gh_pf* pf, const StepObs& o, const StepArgs& a, bool init) {
  pf->stats_valid = false;
  // time_kernels = k > 0: time every k-th step kernel (events add queue packets)
  const int every = pf->opts.time_kernels;
  if (every <= 0 || (a.t - 1) % (uint32_t)every != 0) {
    CHECK(launch_step(pf, o, a, init));
    if (mr(pf->ctx)) CHECK(finish_split(pf, o, a, init));
    HIP_TRY(hipGetLastError());
    return GH_OK;
  }
  if (pf->ev_used + 2 > pf->ev.size()) {
    for (int i = 0; i < 64; ++i) {
      hipEvent_t e;
      HIP_TRY(hipEventCreateWithFlags(&e, kTimingEventFlags));
      pf->ev.push_back(e);
    }
  }
  hipEvent_t e0 = pf->ev[pf->ev_used], e1 = pf->ev[pf->ev_used + 1];
  pf->ev_used += 2;
  CHECK(launch_step(pf, o, a, init, e0, e1));
  if (mr(pf->ctx)) CHECK(finish_split(pf, o, a, init));
  HIP_TRY(hipGetLastError());
  return GH_OK;
}

// after the step kernel: share the rank's (M, S, S2) with every rank
static int share_stats(gh_pf* pf) {
  if (!mr(pf->ctx)) return GH_OK;
  return comm_allgather(pf->ctx, pf->dev->stats, pf->stats_all, 3 * sizeof(double), pf->s, &pf->dev->error);
}

// Conditional SMC: pin particle 0 around the step kernel (gh_csmc.h).  pre =
// before the step (saves the new weight), post = after it.
static int pin_launch(gh_pf* pf, const StepObs& o, bool init, bool pre) {
  if (pf->lo != 0) return GH_OK;  // (R ranks: the distinguished particle 0 lives on rank 0)
  PinArgs a{};
  a.ref = pf->pin;
  a.w0 = pf->pin + pf->D;
  a.dev = pf->dev;
  a.resampled = flags_live(pf);
  a.x = slot_x(pf, init ? 1 : pf->t + 1);
  a.logw = pf->logw;
  a.n = pf->n;
  a.pm = pf->pm;
  a.ps = pf->ps;
  a.ps2 = pf->ps2;
  if (pre) {
    CHECK(with_model(pf->m, [&](auto model, const auto& p) {
      using M = decltype(model);
      if (init)
        hipLaunchKernelGGL((k_pin_pre<M, true>), dim3(1), dim3(64), 0, pf->s, (const double*)pf->m->dparams, p, o, a);
      else
        hipLaunchKernelGGL((k_pin_pre<M, false>), dim3(1), dim3(64), 0, pf->s, (const double*)pf->m->dparams, p, o,
                           a);
    }));
  } else {
    hipLaunchKernelGGL(k_pin_post, dim3(1), dim3(kBlock), 0, pf->s, a, pf->D);
  }
  HIP_TRY(hipGetLastError());
  return GH_OK;
}

static int pin_upload(gh_pf* pf, const double* ref) {
  if (!pf->pin) HIP_TRY(hipMalloc(&pf->pin, sizeof(double) * (pf->D + 1)));
  HIP_TRY(hipMemcpyAsync(pf->pin, ref, sizeof(double) * pf->D, hipMemcpyHostToDevice, pf->s));
  return GH_OK;
}

static int pf_init_impl(gh_model* m, const gh_obs* obs, int proposal, int64_t n_particles, uint64_t seed,
                        const gh_pf_opts* opts, const double* pin_ref, gh_pf** out,
                        const double* qargs = nullptr, int nq = 0);

extern "C" int gh_pf_init(gh_model* m, const gh_obs* obs, int proposal, int64_t n_particles,
                          uint64_t seed, const gh_pf_opts* opts, gh_pf** out) {
  return pf_init_impl(m, obs, proposal, n_particles, seed, opts, nullptr, out);
}

extern "C" int gh_pf_init_q(gh_model* m, const gh_obs* obs, int proposal, const double* proposal_args,
                            int n_proposal_args, int64_t n_particles, uint64_t seed, const gh_pf_opts* opts,
                            gh_pf** out) {
  return pf_init_impl(m, obs, proposal, n_particles, seed, opts, nullptr, out, proposal_args, n_proposal_args);
}

// the stored arguments of the Gaussian custom proposal (4: alpha, beta, gamma, sigma_q)
static int set_qargs(double* dst, bool* has, int proposal, const double* q, int nq) {
  if (!q || nq == 0) return proposal == GH_PROPOSAL_GAUSSIAN && !*has
                              ? set_err(GH_E_INVAL, "the Gaussian proposal needs (alpha, beta, gamma, sigma_q)")
                              : GH_OK;
  if (nq != 4 || !(q[3] > 0.0))
    return set_err(GH_E_INVAL, "Gaussian proposal arguments: (alpha, beta, gamma, sigma_q > 0)");
  for (int i = 0; i < 4; ++i) dst[i] = q[i];
  *has = true;
  return GH_OK;
}

// GH_PROPOSAL_LINEAR's arguments: P[d*d] Sigma_q[d*d] u[d] (P and chol(Sigma_q)
// to the filter's device buffer), or u[d] alone, or none (keep everything)
static int set_qlin(gh_pf* pf, const double* q, int nq) {
  const int d = pf->D;
  if (!q || nq == 0) {
    if (!pf->has_qlin)
      return set_err(GH_E_INVAL, "the linear proposal needs (P[d*d], Sigma_q[d*d], u[d]) first");
    return GH_OK;
  }
  if (nq == d) {
    if (!pf->has_qlin) return set_err(GH_E_INVAL, "the linear proposal needs (P[d*d], Sigma_q[d*d], u[d]) first");
    pf->qlin_u.assign(q, q + d);
    return GH_OK;
  }
  if (nq != 2 * d * d + d)
    return set_err(GH_E_INVAL, "linear proposal arguments: P[d*d] Sigma_q[d*d] u[d] (%d values) or u[d] (%d), got %d",
                   2 * d * d + d, d, nq);
  std::vector<double> buf(2 * d * d);
  for (int i = 0; i < d * d; ++i) buf[i] = q[i];
  if (chol(d, q + d * d, buf.data() + d * d))
    return set_err(GH_E_INVAL, "linear proposal: Sigma_q is not positive definite");
  for (int i = 0; i < 2 * d * d; ++i)
    if (!std::isfinite(buf[i])) return set_err(GH_E_INVAL, "linear proposal: non-finite P or Sigma_q");
  if (!pf->qlin && hipMalloc(&pf->qlin, sizeof(double) * 2 * d * d) != hipSuccess)
    return set_err(GH_E_NOMEM, "linear proposal buffer");
  // ordered on the filter's stream; synchronous so that buf may go (off the hot path)
  HIP_TRY(hipMemcpyAsync(pf->qlin, buf.data(), sizeof(double) * 2 * d * d, hipMemcpyHostToDevice, pf->s));
  HIP_TRY(hipStreamSynchronize(pf->s));
  pf->cstq = gauss_cst(d, buf.data() + d * d);
  pf->qlin_u.assign(q + 2 * d * d, q + 2 * d * d + d);
  pf->has_qlin = true;
  return GH_OK;
}

extern "C" int gh_pf_init_conditional(gh_model* m, const gh_obs* obs, int64_t n_particles, uint64_t seed,
                                      const gh_pf_opts* opts, const double* ref_x1, gh_pf** out) {
  if (!m || !ref_x1 || !out) return set_err(GH_E_INVAL, "gh_pf_init_conditional: null argument");
  if (!opts || opts->resampler != GH_RESAMPLE_MULTINOMIAL)
    return set_err(GH_E_INVAL, "conditional SMC uses multinomial resampling (examples/pmmh/smc.jl:132)");
  if (mr(m->ctx) && m->ctx->peer && !m->ctx->hc.sendrecv)
    return set_err(GH_E_INVAL, "conditional SMC on R ranks over the peer transport needs a bootstrap with sendrecv "
                               "(the multinomial rows go through the host)");
  if (m->family == GH_FAMILY_REGRESSION) return set_err(GH_E_INVAL, "conditional SMC needs a state-space model");
  return pf_init_impl(m, obs, GH_PROPOSAL_DEFAULT, n_particles, seed, opts, ref_x1, out);
}

static int pf_init_impl(gh_model* m, const gh_obs* obs, int proposal, int64_t n_particles, uint64_t seed,
                        const gh_pf_opts* opts, const double* pin_ref, gh_pf** out, const double* qargs, int nq) {
  if (!m || !out) return set_err(GH_E_INVAL, "gh_pf_init: null argument");
  double q0[4] = {0, 0, 0, 0};
  bool has_q = false;
  if (proposal != GH_PROPOSAL_LINEAR) CHECK(set_qargs(q0, &has_q, proposal, qargs, nq));
  if (n_particles < 1 || n_particles > 0x7fffffffLL)
    return set_err(GH_E_INVAL, "gh_pf_init: num_particles must be in 1..2^31-1");
  if (!proposal_ok(m, proposal))
    return set_err(GH_E_INVAL, "gh_pf_init: proposal %d is not available for this model (the optimal proposal: "
                               "HMM, and LGSSM with d + dy <= %d; the Gaussian proposal: the nonlinear SSM)",
                   proposal, kMaxObs);
  gh_ctx* ctx = m->ctx;
  // every rank holds at least one particle, so each rank takes the same path
  // through every collective (a rank with none would skip kernels whose
  // all-gathers the others post)
  if (mr(ctx) && n_particles < ctx->world)
    return set_err(GH_E_INVAL, "gh_pf_init: %lld particles for %d ranks (at least one per rank)",
                   (long long)n_particles, ctx->world);
  HIP_TRY(hipSetDevice(ctx->device));
  gh_pf* pf = new gh_pf();
  pf->m = m;
  pf->ctx = ctx;
  ctx->n_filters++;  // (pf_free undoes it on every failure below)
  pf->s = ctx->stream;
  pf->D = m->d;
  pf->cond = pin_ref != nullptr;  // before the first step kernel (use_pairs)
  pf->no_fused_rank = getenv("GH_NO_FUSED_RANK") != nullptr;
  for (int i = 0; i < 4; ++i) pf->qargs[i] = q0[i];
  pf->has_q = has_q;
  if (opts) pf->opts = *opts;
  else gh_pf_opts_default(&pf->opts);
  if (pf->opts.resampler != GH_RESAMPLE_SYSTEMATIC && pf->opts.resampler != GH_RESAMPLE_MULTINOMIAL) {
    const int r = pf->opts.resampler;
    pf->ctx->n_filters--;
    delete pf;
    return set_err(GH_E_INVAL, "unknown resampler %d", r);
  }
  pf->n_global = n_particles;
  pf->lo = split_lo(n_particles, ctx->rank, ctx->world);
  pf->n = split_lo(n_particles, ctx->rank + 1, ctx->world) - pf->lo;
  pf->seed = seed;
  const int64_t n = pf->n > 0 ? pf->n : 1;
  pf->nb_step = (n + kBlock - 1) / kBlock;
  pf->nb_part = pf->nb_step;
  {  // the partial count of the family's step kernel (resample tile choice)
    bool pairs = false;
    with_model(m, [&](auto model, const auto&) { pairs = use_pairs<decltype(model)>(pf); });
    pf->pairs = pairs;
    if (pairs) pf->nb_part = (n + 2 * kBlock - 1) / (2 * kBlock);
  }
  pf->nb_scan = (n + kScanTile - 1) / kScanTile;
  // peer transport: the set-up's bootstrap rounds are fail-together (a rank
  // that fails runs the next round flagged, so every rank fails with it)
  const bool peer_setup = mr(ctx) && ctx->peer;
  auto fail = [&](int rc) {
    if (peer_setup) peer_abort(ctx, pf->pr);
    pf_free(pf);
    return rc;
  };
#define ALLOC(ptr, bytes) \
  if (hipMalloc(&(ptr), (bytes)) != hipSuccess) return fail(set_err(GH_E_NOMEM, "hipMalloc %s", #ptr));
  ALLOC(pf->logw, sizeof(double) * n);
  ALLOC(pf->C, sizeof(uint64_t) * n);
  ALLOC(pf->mark, sizeof(uint32_t) * n);
  ALLOC(pf->cmark, sizeof(uint32_t) * ((n + 63) / 64));
  while (pf->mark_bits < 31 && (1ll << pf->mark_bits) < n) ++pf->mark_bits;
  ALLOC(pf->bsum, sizeof(uint64_t) * pf->nb_scan);
  ALLOC(pf->pm, sizeof(double) * pf->nb_step);
  ALLOC(pf->ps, sizeof(double) * pf->nb_step);
  ALLOC(pf->ps2, sizeof(double) * pf->nb_step);
  ALLOC(pf->dev, sizeof(DevScalars));
  ALLOC(pf->stats_all, sizeof(double) * 3 * ctx->world);
  ALLOC(pf->totals_all, sizeof(uint64_t) * ctx->world);
  ALLOC(pf->anc_scratch, sizeof(int32_t) * n);
  // tile totals, then the tile sums of e and e^2 (k_resample1 sums-in-pass)
  pf->n_tiles = (n + kRsTile - 1) / kRsTile;
  ALLOC(pf->tsum, sizeof(uint64_t) * 3 * std::max<int64_t>(1, pf->n_tiles));
  pick_resample_tiles(pf, n);
  ALLOC(pf->amax, sizeof(uint64_t) * 2 * kAmaxShards * kAmaxStride);
  if (mr(ctx)) {
    if (pf->opts.resampler != GH_RESAMPLE_SYSTEMATIC && ((ctx->peer && !ctx->hc.sendrecv) || ctx->world > kMaxRanks))
      return fail(set_err(GH_E_INVAL, "multinomial resampling on R ranks needs at most %d ranks and, on the peer "
                                      "transport, a bootstrap with sendrecv (its rows go through the host)",
                          kMaxRanks));
    if (!ctx->peer) {
      ALLOC(pf->rows_recv, sizeof(double) * (pf->D + 1) * n);
    } else {
      // the received rows (written by the senders' k_rank_b), then R tag
      // words; fine-grained, mapped by every rank (bootstrap exchange)
      const size_t rb = sizeof(double) * (pf->D + 1) * n + sizeof(uint64_t) * ctx->world;
      if (hipExtMallocWithFlags((void**)&pf->rows_recv, rb, hipDeviceMallocFinegrained) != hipSuccess)
        return fail(set_err(GH_E_NOMEM, "peer transport: row buffer"));
      if (hipMemset(pf->rows_recv, 0, rb) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
        return fail(set_err(GH_E_HIP, "peer transport: row buffer init"));
      const int rc = ipc_exchange(ctx, pf->pr, pf->rows_recv, (void**)pf->prow);
      if (rc) return fail(rc);
      for (int r = 0; r < ctx->world; ++r) {
        const int64_t nr = std::max<int64_t>(1, split_lo(pf->n_global, r + 1, ctx->world) - split_lo(pf->n_global, r, ctx->world));
        pf->ptag[r] = (uint64_t*)(pf->prow[r] + (pf->D + 1) * nr);
      }
    }
    ALLOC(pf->gparent, sizeof(int64_t) * n);
    ALLOC(pf->amax_all, sizeof(uint64_t) * kAmaxShards * kAmaxStride * ctx->world);
    ALLOC(pf->rec, sizeof(uint64_t) * kRecWords);
    ALLOC(pf->recs_all, sizeof(uint64_t) * kRecWords * ctx->world);
    ALLOC(pf->dlo, sizeof(int64_t) * (ctx->world + 1));
    {
      std::vector<int64_t> t(ctx->world + 1);
      for (int k = 0; k <= ctx->world; ++k) t[k] = (int64_t)(((__int128)pf->n_global * k) / ctx->world);
      if (hipMemcpy(pf->dlo, t.data(), sizeof(int64_t) * t.size(), hipMemcpyHostToDevice) != hipSuccess)
        return fail(set_err(GH_E_HIP, "rank slot table"));
    }
    // the shards are empty between uses: k_rank_a2 empties what it consumed
    pf->amax_armed = true;
    if (hipStreamCreateWithFlags(&pf->aux, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&pf->ev_tot, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&pf->ev_plan, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&pf->ev_rb, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&pf->ev_x, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc((void**)&pf->h_mail, sizeof(uint64_t) * (1 + kRecWords * ctx->world),
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostMalloc((void**)&pf->h_plan, sizeof(uint64_t) * std::max(ctx->world + 1, kRecWords * ctx->world),
                      hipHostMallocDefault) != hipSuccess)
      return fail(set_err(GH_E_NOMEM, "multi-rank plan buffers"));
    // tags count from 1: a reused pinned page must not hold one already
    memset(pf->h_mail, 0, sizeof(uint64_t) * (1 + kRecWords * ctx->world));
    if (hipHostGetDevicePointer((void**)&pf->d_mail, pf->h_mail, 0) != hipSuccess)
      return fail(set_err(GH_E_HIP, "plan mailbox: device alias"));
  }
  if (hipHostMalloc((void**)&pf->h_dec, sizeof(uint64_t) * 4, hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer((void**)&pf->d_dec, pf->h_dec, 0) != hipSuccess)
    return fail(set_err(GH_E_NOMEM, "decision mailbox"));
  memset(pf->h_dec, 0, sizeof(uint64_t) * 4);
  if (!pf->opts.record_history) {
    for (int i = 0; i < 2; ++i) {
      double* x = nullptr;
      ALLOC(x, sizeof(double) * slot_doubles(n, pf->D));
      pf->xs.push_back(x);
    }
    int32_t* a = nullptr;
    ALLOC(a, sizeof(int32_t) * n);
    pf->ancs.push_back(a);
  }
#undef ALLOC
  {
    DevScalars z;
    memset(&z, 0, sizeof z);
    z.one = 1;
    if (hipMemcpyAsync(pf->dev, &z, sizeof z, hipMemcpyHostToDevice, pf->s) != hipSuccess)
      return fail(set_err(GH_E_HIP, "init scalars"));
    if (hipMemsetAsync(pf->mark, 0, sizeof(uint32_t) * n, pf->s) != hipSuccess ||
        hipMemsetAsync(pf->tsum, 0, sizeof(uint64_t) * 3 * std::max<int64_t>(1, pf->n_tiles), pf->s) != hipSuccess ||
        hipMemsetAsync(pf->cmark, 0, sizeof(uint32_t) * ((n + 63) / 64), pf->s) != hipSuccess)
      return fail(set_err(GH_E_HIP, "init marks"));
    if (pf->amax) {
      std::vector<uint64_t> e(2 * kAmaxShards * kAmaxStride, kAmaxEmpty);
      if (hipMemcpyAsync(pf->amax, e.data(), sizeof(uint64_t) * e.size(), hipMemcpyHostToDevice, pf->s) != hipSuccess)
        return fail(set_err(GH_E_HIP, "init shards"));
    }
    if (hipStreamSynchronize(pf->s) != hipSuccess) return fail(set_err(GH_E_HIP, "sync"));
  }
  const int cap0 = pf->opts.history_capacity > 0 ? pf->opts.history_capacity : 16;
  {
    int rc = ensure_capacity(pf, cap0);
    if (rc) return fail(rc);
  }
  StepObs o, o_prior;
  int rc = make_obs(m, 1, obs, &o_prior);
  if (!rc && proposal == GH_PROPOSAL_LINEAR) rc = set_qlin(pf, qargs, nq);
  if (!rc) {
    o = o_prior;
    if (proposal == GH_PROPOSAL_OPTIMAL && m->family == GH_FAMILY_LGSSM) rc = make_obs_opt(m, 1, obs, &o);
    if (proposal == GH_PROPOSAL_GAUSSIAN) rc = make_obs_gauss(m, 1, obs, pf->qargs, &o);
    if (proposal == GH_PROPOSAL_LINEAR) rc = make_obs_lin(m, 1, obs, pf->qlin_u.data(), &o);
  }
  if (rc) return fail(rc);
  StepArgs a{};
  a.xout = slot_x(pf, 1);
  a.logw = pf->logw;
  a.n = pf->n;
  a.lo = pf->lo;
  a.seed = seed;
  a.t = 1;
  a.proposal = proposal;
  a.dev = pf->dev;
  a.pm = pf->pm;
  a.ps = pf->ps;
  a.ps2 = pf->ps2;
  a.stats_out = !mr(ctx) ? pf->stats_all : pf->dev->stats;
  a.buf = slot_doubles(pf->n, pf->D) * 8 < (1LL << 32) ? 1 : 0;
  rc = timed_step(pf, o, a, true);
  if (rc) return fail(rc);
  if (pin_ref) {
    pf->cond = true;
    rc = pin_upload(pf, pin_ref);
    if (!rc) rc = pin_launch(pf, o, true, true);
    if (!rc) rc = pin_launch(pf, o, true, false);
    if (rc) return fail(rc);
    if (mr(ctx) && pf->lo == 0) launch_fold(pf, a, true, pf->nb_part);  // (the fold, again with particle 0 pinned)
  }
  rc = share_stats(pf);
  if (rc) return fail(rc);
  if (peer_setup) {  // every rank created its shard (the last round), or every rank fails here
    rc = peer_round(ctx, pf->pr, true, nullptr, 0, nullptr);
    if (rc) return fail(rc);
    pf->pr.over = true;
    pf->peer_ready = true;
  }
  pf->t = 1;
  pf->last_obs = o_prior;  // rejuvenation scores under the model (prior form)
  pf->obs_hist.assign(1, o_prior);
  log_raw_obs(pf, 1, obs);
  *out = pf;
  return GH_OK;
}

static int grow_for_step(gh_pf* pf, int t) { return ensure_capacity(pf, t + 1); }

// the observation of step t as given (rebuilt under other parameters: gh_pf_step_params)
static void log_raw_obs(gh_pf* pf, int t, const gh_obs* obs) {
  if ((int)pf->raw_obs.size() < t) pf->raw_obs.resize(t);
  auto& r = pf->raw_obs[t - 1];
  r.clear();
  if (pf->m->family == GH_FAMILY_SLOTS) {  // the chain as (slot, count, values...) records (make_obs validated it)
    for (const gh_obs* e = obs; e; e = e->next) {
      if (!e->present || !e->values) continue;
      r.push_back((double)e->slot);
      r.push_back((double)e->n_values);
      r.insert(r.end(), e->values, e->values + e->n_values);
    }
    return;
  }
  if (obs && obs->present && obs->values && obs->n_values > 0) r.assign(obs->values, obs->values + obs->n_values);
}

// a slot model's logged step (log_raw_obs) as a gh_obs chain again, in
// chain[0..kMaxSlots) (nullptr: nothing observed)
static const gh_obs* slot_chain(const std::vector<double>& r, gh_obs* chain) {
  int k = 0;
  for (size_t i = 0; i + 1 < r.size() && k < kMaxSlots; ++k) {
    const int nv = (int)r[i + 1];
    chain[k] = gh_obs{};
    chain[k].values = r.data() + i + 2;
    chain[k].n_values = nv;
    chain[k].present = 1;
    chain[k].slot = (int32_t)r[i];
    if (k > 0) chain[k - 1].next = &chain[k];
    i += 2 + (size_t)nv;
  }
  return k ? chain : nullptr;
}

// the same slot layout (a parameter change keeps every address and its form)
static bool same_slots(const gh_model* a, const gh_model* b) {
  const SlotParams &p = a->slots, &q = b->slots;
  if (p.lat != q.lat || p.K != q.K || (p.uoff >= 0) != (q.uoff >= 0) || p.nz != q.nz) return false;
  if (p.dep != q.dep) return false;
  for (int k = 0; k < p.K; ++k) {
    if (p.dist[k] != q.dist[k] || p.m[k] != q.m[k] || p.link[k] != q.link[k]) return false;
    for (int j = 0; j < k; ++j)
      if ((p.dg[k][j] != 0.0) != (q.dg[k][j] != 0.0)) return false;
  }
  return true;
}

static int pf_step_impl(gh_pf* pf, const gh_obs* obs, int proposal, const double* pin_ref);

// a step's proposal arguments: the Gaussian (nonlinear SSM) or linear (LGSSM) custom proposal's
static int step_qargs(gh_pf* pf, int proposal, const double* q, int nq) {
  if (proposal == GH_PROPOSAL_LINEAR) return proposal_ok(pf->m, proposal) ? set_qlin(pf, q, nq) : GH_OK;
  return set_qargs(pf->qargs, &pf->has_q, proposal, q, nq);
}

extern "C" int gh_pf_step(gh_pf* pf, const gh_obs* obs, int proposal) {
  if (pf && pf->cond) return set_err(GH_E_STATE, "a conditional filter steps with gh_pf_step_conditional");
  if (pf) CHECK(step_qargs(pf, proposal, nullptr, 0));
  return pf_step_impl(pf, obs, proposal, nullptr);
}

extern "C" int gh_pf_step_q(gh_pf* pf, const gh_obs* obs, int proposal, const double* proposal_args,
                            int n_proposal_args) {
  if (!pf) return set_err(GH_E_INVAL, "null pf");
  if (pf->cond) return set_err(GH_E_STATE, "a conditional filter steps with gh_pf_step_conditional");
  CHECK(step_qargs(pf, proposal, proposal_args, n_proposal_args));
  return pf_step_impl(pf, obs, proposal, nullptr);
}

extern "C" int gh_pf_step_conditional(gh_pf* pf, const gh_obs* obs, const double* ref_xt) {
  if (!pf || !ref_xt) return set_err(GH_E_INVAL, "gh_pf_step_conditional: null argument");
  if (!pf->cond) return set_err(GH_E_STATE, "gh_pf_step_conditional on a filter not made by gh_pf_init_conditional");
  return pf_step_impl(pf, obs, GH_PROPOSAL_DEFAULT, ref_xt);
}

static int pf_step_impl(gh_pf* pf, const gh_obs* obs, int proposal, const double* pin_ref) {
  if (!pf) return set_err(GH_E_INVAL, "null pf");
  if (!proposal_ok(pf->m, proposal))
    return set_err(GH_E_INVAL, "proposal %d is not available for this model (the optimal proposal: HMM, and "
                               "LGSSM with d + dy <= %d)", proposal, kMaxObs);
  if (pf->m->family == GH_FAMILY_REGRESSION)
    return set_err(GH_E_INVAL, "the regression model has no time steps (particle_filter_step needs an Unfold)");
  const int t = pf->t + 1;
  CHECK(grow_for_step(pf, t));
  StepObs o, o_prior;
  CHECK(make_obs(pf->m, t, obs, &o_prior));
  o = o_prior;
  if (proposal == GH_PROPOSAL_OPTIMAL && pf->m->family == GH_FAMILY_LGSSM) CHECK(make_obs_opt(pf->m, t, obs, &o));
  if (proposal == GH_PROPOSAL_GAUSSIAN) CHECK(make_obs_gauss(pf->m, t, obs, pf->qargs, &o));
  if (proposal == GH_PROPOSAL_LINEAR) CHECK(make_obs_lin(pf->m, t, obs, pf->qlin_u.data(), &o));
  StepArgs a{};
  a.xprev = slot_x(pf, t - 1);
  a.anc = anc_for_step(pf, t);
  a.mark = pf->mark;
  a.carry = pf->cmark;
  a.mark_idx = (uint32_t)((1ull << pf->mark_bits) - 1);
  a.mark_mode = pf->marks_pending ? pf->mark_mode : 0;
  a.resampled = flags_live(pf);
  a.remote = pf->rows_recv;
  a.ld_remote = pf->D + 1;
  a.xout = slot_x(pf, t);
  a.logw = pf->logw;
  a.n = pf->n;
  a.lo = pf->lo;
  a.seed = pf->seed;
  a.t = (uint32_t)t;
  a.proposal = proposal;
  a.dev = pf->dev;
  a.pm = pf->pm;
  a.ps = pf->ps;
  a.ps2 = pf->ps2;
  a.stats_out = !mr(pf->ctx) ? pf->stats_all : pf->dev->stats;
  a.buf = slot_doubles(pf->n, pf->D) * 8 < (1LL << 32) ? 1 : 0;
  const bool multi = mr(pf->ctx);
  // (multi-rank, a resample whose ancestors were materialised by a genealogy
  // query between maybe_resample! and this step: they may name received rows
  // (negative); the kernels test each wave's ancestors for that themselves)
  // One rank: every step writes block maxima only — the next maybe_resample!
  // sums the weights in its own pass, any other reader recomputes the sums
  // (ensure_stats) — so a caller's maybe_resample! + particle_filter_step!
  // loop runs what gh_pf_run runs.  Multi-rank: gh_pf_run's steps, which
  // need the shards (the rank maximum has no other fold).
  const bool lazy = !multi && pf->rs_grid > 0 && !pf->cond && pf->n > 0 && !pf->no_max_only;
  a.max_only = (pf->step_max_only || lazy) && !pin_ref && (!multi || pf->amax_armed) ? 1 : 0;
  // The block maxima also go into the atomic-max shards, so the resample
  // reads 32 words instead of every block's maximum (the pair kernel too:
  // C4 39.45 -> 39.06 us per step, four runs each on one box, round 5).
  a.amax = a.max_only && pf->amax_armed ? pf->amax + (t & 1) * kAmaxShards * kAmaxStride : nullptr;
  // multi-rank after a resample: the local half now, the rest once the rows arrive
  a.part = pf->plan_pending && a.mark_mode == 2 ? 1 : 0;
  if (pin_ref) {
    CHECK(pin_upload(pf, pin_ref));
    CHECK(pin_launch(pf, o, false, true));
  }
  CHECK(timed_step(pf, o, a, false));
  if (pin_ref) {
    CHECK(pin_launch(pf, o, false, false));
    // R ranks: the step folded its partials already; again with particle 0 pinned
    if (multi && pf->lo == 0) launch_fold(pf, a, false, pf->nb_part);
  }
  if (!a.max_only) CHECK(share_stats(pf));  // (max-only: the resample's own all-gathers)
  pf->t = t;
  pf->max_only = a.max_only != 0;
  pf->mr_stale = multi && a.max_only;
  pf->amax_valid = a.amax != nullptr;
  if (!multi) pf->amax_armed = false;
  pf->resample_calls = 0;
  pf->marks_pending = false;
  pf->last_obs = o_prior;  // rejuvenation scores under the model (prior form)
  if ((int)pf->obs_hist.size() < t) pf->obs_hist.resize(t);
  pf->obs_hist[t - 1] = o_prior;
  log_raw_obs(pf, t, obs);
  pf->rejuv_moves = 0;
  return GH_OK;
}

// Expand pending systematic marks into the ancestor array of step t+1 (for
// genealogy reads before the next step, or a second resample).
static int finish_plan(gh_pf* pf);

// The next resample's epoch tag for the range marks (MarkArgs::tag: the epoch
// above the mark_bits index bits).  When the epoch field is used up, both mark
// arrays are cleared on the filter's stream first (every consumer of the old
// marks is enqueued before), so all older words stay below the new tags.
static int next_mark_tag(gh_pf* pf, uint32_t* tag) {
  if (pf->epoch + 1 >= (1ull << (32 - pf->mark_bits))) {
    HIP_TRY(hipMemsetAsync(pf->mark, 0, sizeof(uint32_t) * pf->n, pf->s));
    HIP_TRY(hipMemsetAsync(pf->cmark, 0, sizeof(uint32_t) * ((pf->n + 63) / 64), pf->s));
    pf->epoch = 0;
  }
  *tag = (uint32_t)(++pf->epoch << pf->mark_bits);
  return GH_OK;
}

static int materialize_marks(gh_pf* pf) {
  CHECK(finish_plan(pf));
  if (!pf->marks_pending) return GH_OK;
  int32_t* anc_target = anc_for_step(pf, pf->t + 1);
  hipLaunchKernelGGL(k_sys_ancestors, dim3((unsigned)pf->nb_step), dim3(kBlock), 0, pf->s, &pf->dev->fire,
                     &pf->dev->pending, pf->mark, pf->cmark, (uint32_t)((1ull << pf->mark_bits) - 1), pf->n,
                     (const int32_t*)nullptr, anc_target,
                     (const DevScalars*)pf->dev, pf->mark_mode);
  HIP_TRY(hipGetLastError());
  pf->marks_pending = false;
  // multi-rank: the next step reads these ancestors in one launch (no part 2,
  // which would keep the received rows), so the rows received for it are
  // kept here as that step's genealogy record
  if (pf->mark_mode == 2 && pf->rem_fire && pf->opts.record_history) {
    const int64_t cnt = pf->rem_ra + (pf->n - pf->rem_rb);
    double* dst = nullptr;
    CHECK(rhist_reserve(pf, pf->t + 1, cnt, &dst));
    if (dst)
      HIP_TRY(hipMemcpyAsync(dst, pf->rows_recv, sizeof(double) * (pf->D + 1) * (size_t)cnt, hipMemcpyDeviceToDevice,
                             pf->s));
  }
  return GH_OK;
}

// multi-rank exchange of ancestor states; defined below
static int exchange_states(gh_pf* pf, int32_t* anc_out);
static int exchange_states_mn(gh_pf* pf, int32_t* anc_out);

static void sys_plan(int64_t N, int R, int q, const uint64_t* totals, uint64_t o, int64_t* send_lo,
                     int64_t* send_hi, int64_t* recv_lo, int64_t* recv_hi);
static int64_t sys_count_host(uint64_t X, uint64_t N, uint64_t S, uint64_t o);

static void launch_rank_b(gh_pf* pf, const RankBArgs& rb) {
  switch (pf->rs_it) {
    case 4: hipLaunchKernelGGL(k_rank_b<4>, dim3((unsigned)pf->rs_grid), dim3(kRsBlock), 0, pf->s, rb); break;
    case 8: hipLaunchKernelGGL(k_rank_b<8>, dim3((unsigned)pf->rs_grid), dim3(kRsBlock), 0, pf->s, rb); break;
    default: hipLaunchKernelGGL(k_rank_b<16>, dim3((unsigned)pf->rs_grid), dim3(kRsBlock), 0, pf->s, rb); break;
  }
}

// The grouped exchange of one multi-rank resample: to / from each other rank r
// the rows of its slot block, packed by rank (sends at their k_rank_b offsets)
static void exchange_lists(int R, int q, int D, const int64_t* slo, const int64_t* shi, const int64_t* rlo,
                           const int64_t* rhi, double* rows_send, double* rows_recv, std::vector<CommMsg>* sends,
                           std::vector<CommMsg>* recvs) {
  const size_t row_bytes = sizeof(double) * (D + 1);
  int64_t soff = 0, roff = 0;
  for (int r = 0; r < R; ++r) {
    if (r == q) continue;
    const int64_t ls = shi[r] - slo[r], lr = rhi[r] - rlo[r];
    if (ls > 0) sends->push_back({r, rows_send + soff * (D + 1), (size_t)ls * row_bytes});
    if (lr > 0) recvs->push_back({r, rows_recv + roff * (D + 1), (size_t)lr * row_bytes});
    soff += ls > 0 ? ls : 0;
    roff += lr > 0 ? lr : 0;
  }
}

// Multi-rank systematic resample: decision + quantise + rank
// total (k_rank_a), all-gather of the totals, marks + outgoing rows
// (k_rank_b).  Nothing here waits for the device: the fire flag and the
// totals are copied to pinned memory on the side stream, and finish_plan
// (called by the next step after it has enqueued the local half of its work)
// reads them, derives the row counts (gh_sys_plan's arithmetic) and posts
// the grouped send/recv on the side stream.
static int rank_resample(gh_pf* pf, const DecideArgs& d, int shift, int t) {
  gh_ctx* c = pf->ctx;
  const int R = c->world, q = c->rank;
  const int D = pf->D;
  if (pf->send_cap < 1) {
    // bounded: up to twice this rank's own particles (the worst case, every
    // other rank's slots, grows with the world size); a resample that needs
    // more keeps its CDF and finish_plan regrows the buffer (k_rows_fill)
    const int64_t cap = std::max<int64_t>(std::min<int64_t>(pf->n_global - pf->n, 2 * pf->n), 1);
    if (hipMalloc(&pf->rows_send, sizeof(double) * (D + 1) * cap) != hipSuccess)
      return set_err(GH_E_NOMEM, "send rows (%lld)", (long long)cap);
    pf->send_cap = cap;
  }
  // after a max-only step (gh_pf_run): the shards' all-gather, k_rank_a2
  // (global max, quantisation + sums, rank record), the records' all-gather;
  // otherwise k_rank_a on the all-gathered triples and the totals' all-gather
  const bool sums = pf->max_only && pf->amax_valid;
  uint64_t* shards = pf->amax + (t & 1) * kAmaxShards * kAmaxStride;
  // peer transport, batched loop: ONE launch (k_rank_ab, gh_rank_ab.h) for
  // k_rank_a2 + k_rank_b — nothing between them needs the host
  const bool fused = sums && c->peer && pf->ab_fits && pf->n_global < (1LL << 31) && !pf->no_fused_rank;
  RankA2Args a2{};
  if (sums) {
    // peer transport: the shards' and the records' all-gathers happen inside
    // k_rank_a2 / k_rank_b through the mailboxes
    if (!c->peer)
      CHECK(comm_allgather(c, shards, pf->amax_all, sizeof(uint64_t) * kAmaxShards * kAmaxStride, pf->s,
                           &pf->dev->error));
    a2.logw = pf->logw;
    a2.n = pf->n;
    a2.shift = shift;
    a2.dev = pf->dev;
    a2.amax_all = pf->amax_all;
    a2.R = R;
    a2.amax_reset = shards;
    a2.tsum = pf->tsum;
    a2.ts1 = pf->tsum + pf->n_tiles;
    a2.ts2 = pf->tsum + 2 * pf->n_tiles;
    a2.rec = pf->rec;
    if (c->peer) {
      a2.pb = peer_box(c);
      a2.amax_own = shards;
      a2.amax_reset = nullptr;  // (k_rank_b empties them: every block here reads them)
      a2.use_sh = ++c->use_sh;
      a2.use_rec = ++c->use_rec;
    }
    if (!fused) {
      switch (pf->rs_it) {
        case 4: hipLaunchKernelGGL(k_rank_a2<4>, dim3((unsigned)pf->rs_grid), dim3(kRsBlock), 0, pf->s, a2); break;
        case 8: hipLaunchKernelGGL(k_rank_a2<8>, dim3((unsigned)pf->rs_grid), dim3(kRsBlock), 0, pf->s, a2); break;
        default: hipLaunchKernelGGL(k_rank_a2<16>, dim3((unsigned)pf->rs_grid), dim3(kRsBlock), 0, pf->s, a2); break;
      }
      HIP_TRY(hipGetLastError());
    }
    if (!c->peer) CHECK(comm_allgather(c, pf->rec, pf->recs_all, sizeof(uint64_t) * kRecWords, pf->s, &pf->dev->error));
  } else {
    RankAArgs ra{};
    ra.logw = pf->logw;
    ra.n = pf->n;
    ra.shift = shift;
    ra.dev = pf->dev;
    ra.d = d;
    ra.tsum = pf->tsum;
    ra.ts1 = pf->tsum + pf->n_tiles;
    ra.ts2 = pf->tsum + 2 * pf->n_tiles;
    switch (pf->rs_it) {
      case 4: hipLaunchKernelGGL(k_rank_a<4>, dim3((unsigned)pf->rs_grid), dim3(kRsBlock), 0, pf->s, ra); break;
      case 8: hipLaunchKernelGGL(k_rank_a<8>, dim3((unsigned)pf->rs_grid), dim3(kRsBlock), 0, pf->s, ra); break;
      default: hipLaunchKernelGGL(k_rank_a<16>, dim3((unsigned)pf->rs_grid), dim3(kRsBlock), 0, pf->s, ra); break;
    }
    HIP_TRY(hipGetLastError());
    CHECK(comm_allgather(c, &pf->dev->local, pf->totals_all, sizeof(uint64_t), pf->s, &pf->dev->error));
    HIP_TRY(hipEventRecord(pf->ev_tot, pf->s));
  }
  RankBArgs rb{};
  rb.logw = pf->logw;
  rb.n = pf->n;
  rb.shift = shift;
  rb.dev = pf->dev;
  rb.tsum = pf->tsum;
  rb.totals = sums ? pf->recs_all : pf->totals_all;
  rb.tot_stride = sums ? kRecWords : 1;
  rb.recs = sums ? pf->recs_all : nullptr;
  if (sums) {  // the plan comes back through the host-mapped mailbox (no event, no copy, no stream wait)
    rb.hplan = pf->d_mail;
    rb.htag = ++pf->mail_seq;
  }
  rb.d = d;
  rb.R = R;
  rb.rank = q;
  rb.lo = pf->lo;
  rb.seed = pf->seed;
  rb.t = (uint32_t)t;
  rb.mk.mark = pf->mark;
  rb.mk.cmark = pf->cmark;
  CHECK(next_mark_tag(pf, &rb.mk.tag));
  rb.mk.n_global = pf->n_global;
  rb.mk.n_groups = (pf->n + 63) / 64;
  rb.mk.enabled = 1;
  rb.xprev = slot_x(pf, t);
  rb.D = D;
  rb.rows = pf->rows_send;
  rb.rows_cap = pf->send_cap;
  rb.C = pf->C;
  rb.dlo = pf->dlo;
  if (c->peer) {  // records from the mailboxes (sums), rows straight into the receivers' buffers
    if (sums) {
      rb.pb = peer_box(c);
      rb.use_rec = c->use_rec;
      rb.amax_reset = shards;
    }
    rb.peer_rows = 1;
    for (int r = 0; r < R; ++r) rb.prow[r] = pf->prow[r];
    rb.rows_cap = INT64_MAX;
  }
  if (fused) {
    const RankABArgs ab{a2, rb};
    switch (pf->rs_it) {
      case 4: hipLaunchKernelGGL(k_rank_ab<4>, dim3((unsigned)pf->rs_grid), dim3(kRsBlock), 0, pf->s, ab); break;
      case 8: hipLaunchKernelGGL(k_rank_ab<8>, dim3((unsigned)pf->rs_grid), dim3(kRsBlock), 0, pf->s, ab); break;
      default: hipLaunchKernelGGL(k_rank_ab<16>, dim3((unsigned)pf->rs_grid), dim3(kRsBlock), 0, pf->s, ab); break;
    }
  } else {
    launch_rank_b(pf, rb);
  }
  HIP_TRY(hipGetLastError());
  if (c->peer) {
    // every rank tags every other rank's row buffer once its rows are in
    // (fired or not: the tags count the exchanges); finish_plan waits
    if (R > 1) {
      PeerRowTags pt{};
      for (int r = 0; r < R; ++r) pt.tag[r] = pf->ptag[r];
      pt.R = R;
      pt.rank = q;
      hipLaunchKernelGGL(k_peer_signal, dim3(1), dim3(64), 0, pf->s, pt, ++pf->row_use);
      HIP_TRY(hipGetLastError());
    }
  } else if (R > 1) {
    // the row exchange starts on the side stream once k_rank_b packed the rows
    HIP_TRY(hipEventRecord(pf->ev_rb, pf->s));
  }
  if (!sums) {  // the decision and the totals, read on the side stream while k_rank_b runs
    HIP_TRY(hipStreamWaitEvent(pf->aux, pf->ev_tot, 0));
    HIP_TRY(hipMemcpyAsync(pf->h_plan, &pf->dev->fire, sizeof(int), hipMemcpyDeviceToHost, pf->aux));
    HIP_TRY(hipMemcpyAsync(pf->h_plan + 1, pf->totals_all, sizeof(uint64_t) * R, hipMemcpyDeviceToHost, pf->aux));
    HIP_TRY(hipEventRecord(pf->ev_plan, pf->aux));
  }
  pf->plan_recs = sums;
  pf->plan_thr = d.thr;
  pf->mark_mode = 2;
  pf->marks_pending = true;  // harmless when it did not fire: k_step gates on the device flag
  pf->plan_pending = true;
  pf->rem_fire = false;
  return GH_OK;
}

// The host half of rank_resample: wait for the fire flag and the totals, post
// the row exchange on the side stream and make the filter's stream wait for
// it (work already enqueued on the filter's stream — the local half of the
// next step — runs meanwhile).  Sets the received-row slot ranges.
// The batched loop's plan: k_rank_b's block 0 writes the R records and then
// the launch's tag into pinned, coherent host memory.  The host spins on the
// tag (the records were copied before it, behind a system-scope release).  A
// kernel that never writes it (a fault) ends the wait through the stream's
// error after a bounded spin.
static int wait_tag(gh_pf* pf, volatile uint64_t* tag, uint64_t want, const char* what) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t spins = 0; __atomic_load_n(tag, __ATOMIC_ACQUIRE) != want; ++spins) {
    __builtin_ia32_pause();
    if ((spins & 0xfffff) == 0xfffff) {  // every ~1M polls: is the stream still alive?
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
        return set_err(GH_E_STATE, "%s wait: nothing posted after 60 s", what);
      const hipError_t e = hipStreamQuery(pf->s);
      if (e != hipSuccess && e != hipErrorNotReady) return set_err(GH_E_HIP, "%s wait: %s", what, hipGetErrorString(e));
      if (e == hipSuccess && __atomic_load_n(tag, __ATOMIC_ACQUIRE) != want)
        return set_err(GH_E_STATE, "%s wait: the stream drained without it (tag %llu, want %llu)", what,
                       (unsigned long long)*tag, (unsigned long long)want);
    }
  }
  return GH_OK;
}
static int wait_mailbox(gh_pf* pf) { return wait_tag(pf, pf->h_mail, pf->mail_seq, "plan"); }
static int wait_decision(gh_pf* pf) { return wait_tag(pf, pf->h_dec, pf->dec_seq, "decision"); }

static int finish_plan(gh_pf* pf) {
  if (!pf->plan_pending) return GH_OK;
  pf->plan_pending = false;
  gh_ctx* c = pf->ctx;
  const int R = c->world, q = c->rank;
  const int D = pf->D;
  const int t = pf->t;
  int fire = 0;
  std::vector<uint64_t> totv(R);
  if (pf->plan_recs) {  // k_rank_b takes the same decision from the same records
    CHECK(wait_mailbox(pf));
    const uint64_t* recs = pf->h_mail + 1;
    fire = decide_records(recs, R, pf->plan_thr).fire;
    for (int r = 0; r < R; ++r) totv[r] = recs[kRecWords * r];
  } else {
    HIP_TRY(hipEventSynchronize(pf->ev_plan));
    memcpy(&fire, pf->h_plan, sizeof(int));
    for (int r = 0; r < R; ++r) totv[r] = pf->h_plan[1 + r];
  }
  if (!fire) return GH_OK;
  const uint64_t* tot = totv.data();
  uint64_t S = 0, base = 0;
  for (int r = 0; r < R; ++r) {
    if (r < q) base += tot[r];
    S += tot[r];
  }
  if (S == 0) return GH_OK;  // the device raised GH_E_NUMERIC
  pf->rem_fire = true;
  const u32x4 w = rng_block(pf->seed, ~0ull, (uint32_t)t, STREAM_RESAMPLE, 0);
  const uint64_t o = scale_u53(u53_bits(w.x, w.y), S);
  // this rank's own slots covered by other ranks: [0, ra) and [rb, n) (as k_rank_b)
  const uint64_t N = (uint64_t)pf->n_global;
  const int64_t own_lo = pf->lo, own_hi = pf->lo + pf->n;
  auto clamp_own = [&](int64_t v) { return v < own_lo ? own_lo : (v > own_hi ? own_hi : v); };
  pf->rem_ra = clamp_own(sys_count_host(base, N, S, o)) - own_lo;
  pf->rem_rb = clamp_own(sys_count_host(base + tot[q], N, S, o)) - own_lo;
  if (c->peer) {
    // the senders' k_rank_b stored the rows here; part 2 of the step reads
    // them behind this wait (on the filter's stream, after part 1)
    if (R > 1) {
      hipLaunchKernelGGL(k_peer_wait, dim3(1), dim3(64), 0, pf->s, (const uint64_t*)pf->ptag[q], R, q, pf->row_use,
                         c->peer_wait_ticks, &pf->dev->error);
      HIP_TRY(hipGetLastError());
    }
    return GH_OK;
  }
  std::vector<int64_t> slo(R), shi(R), rlo(R), rhi(R);
  sys_plan(pf->n_global, R, q, tot, o, slo.data(), shi.data(), rlo.data(), rhi.data());
  int64_t n_send = 0;
  for (int r = 0; r < R; ++r)
    if (r != q && shi[r] > slo[r]) n_send += shi[r] - slo[r];
  if (n_send > pf->send_cap) {
    // k_rank_b kept the CDF instead of the rows: regrow (synchronously: this
    // rank holds most of the weight, a rare step) and write every row from it
    HIP_TRY(hipStreamSynchronize(pf->s));
    hipFree(pf->rows_send);
    pf->rows_send = nullptr;
    pf->send_cap = 0;
    const int64_t cap = n_send + n_send / 4 + 64;
    if (hipMalloc(&pf->rows_send, sizeof(double) * (D + 1) * cap) != hipSuccess)
      return set_err(GH_E_NOMEM, "send rows (%lld)", (long long)cap);
    pf->send_cap = cap;
    RowsFillArgs fa{};
    fa.C = pf->C;
    fa.n = pf->n;
    fa.R = R;
    fa.rank = q;
    fa.lo = pf->lo;
    fa.dev = pf->dev;
    fa.totals = pf->plan_recs ? pf->recs_all : pf->totals_all;
    fa.tot_stride = pf->plan_recs ? kRecWords : 1;
    fa.n_global = pf->n_global;
    fa.xprev = slot_x(pf, t);
    fa.D = D;
    fa.rows = pf->rows_send;
    fa.rows_cap = pf->send_cap;
    fa.dlo = pf->dlo;
    hipLaunchKernelGGL(k_rows_fill, dim3((unsigned)((pf->n + 255) / 256)), dim3(256), 0, pf->s, fa);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(pf->ev_rb, pf->s));
    pf->send_grows++;
  }
  // the same message lists serve both transports (RCCL grouped send/recv,
  // or the host-staged sendrecv): exchange_lists, also exported for tests
  std::vector<CommMsg> sends, recvs;
  exchange_lists(R, q, D, slo.data(), shi.data(), rlo.data(), rhi.data(), pf->rows_send, pf->rows_recv, &sends,
                 &recvs);
  if (sends.empty() && recvs.empty()) return GH_OK;
  HIP_TRY(hipStreamWaitEvent(pf->aux, pf->ev_rb, 0));
  CHECK(comm_exchange(c, sends, recvs, pf->aux));
  HIP_TRY(hipEventRecord(pf->ev_x, pf->aux));
  HIP_TRY(hipStreamWaitEvent(pf->s, pf->ev_x, 0));
  return GH_OK;
}

// want_decision: the caller reads maybe_resample!'s Bool (or the ESS) now, so
// the fused kernel posts it to the host mailbox; the batched loop does not
// (block 0 then skips the post and its system-scope fence)
static int resample_enqueue(gh_pf* pf, double thr, bool want_decision) {
  const int t = pf->t;
  CHECK(grow_for_step(pf, t + 1));
  pf->dec_posted = false;
  const int R = pf->ctx->world;
  const bool multi = mr(pf->ctx);
  const int64_t n = pf->n;
  const bool second = pf->resample_calls > 0;
  DecideArgs d{};
  d.stats_all = pf->stats_all;
  d.R = R;
  d.n_global = pf->n_global;
  d.log_n = gh_log((double)pf->n_global);
  d.inv_n = 1.0 / (double)pf->n_global;
  d.thr = thr;
  d.ess_hist = pf->ess_hist;
  d.res_hist = pf->res_hist;
  d.t = t;
  GateArgs g;
  g.gate = &pf->dev->fire;
  g.M = &pf->dev->M;
  g.zero_w = &pf->dev->pending;
  g.shift = quant_shift((uint64_t)pf->n_global);
  // The common case fuses the decision into the first resample kernel; a
  // second call without a step (or an empty shard) decides in its own launch.
  const bool sys = pf->opts.resampler == GH_RESAMPLE_SYSTEMATIC;
  if (!multi && !second && n > 0 && pf->rs_grid > 0) {
    // one launch: fold + decision + quantise + one grid barrier + marks / CDF
    Resample1Args ra{};
    ra.pm = pf->pm;
    ra.ps = pf->ps;
    ra.ps2 = pf->ps2;
    ra.nb_part = (int)pf->nb_part;
    ra.logw = pf->logw;
    ra.n = n;
    ra.shift = g.shift;
    ra.stats_out = pf->stats_all;
    ra.dev = pf->dev;
    ra.d = d;
    ra.tsum = pf->tsum;
    ra.ts1 = pf->tsum + pf->n_tiles;
    ra.ts2 = pf->tsum + 2 * pf->n_tiles;
    ra.sums_in_pass = pf->max_only ? 1 : 0;
    ra.mk.mark = pf->mark;
    ra.mk.cmark = pf->cmark;
    CHECK(next_mark_tag(pf, &ra.mk.tag));
    ra.mk.n_global = pf->n_global;
    ra.mk.n_groups = (n + 63) / 64;
    ra.mk.enabled = sys ? 1 : 0;
    ra.C = pf->C;
    ra.seed = pf->seed;
    ra.t = (uint32_t)t;
    ra.hdec = want_decision ? pf->d_dec : nullptr;
    ra.htag = want_decision ? ++pf->dec_seq : 0;
    if (pf->amax) {  // the step's own max fold (when it wrote one); the next step's shards emptied
      ra.amax_in = pf->max_only && pf->amax_valid ? pf->amax + (t & 1) * kAmaxShards * kAmaxStride : nullptr;
      ra.amax_reset = pf->amax + ((t + 1) & 1) * kAmaxShards * kAmaxStride;
      pf->amax_armed = true;
    }
    // grid <= co-resident capacity of an idle device (rs_cap), so every block
    // is eventually resident; the barrier wait is bounded as a backstop
    const dim3 grid((unsigned)pf->rs_grid), blk(kRsBlock);
#define GH_RS1(SYS, IT)                                                                 \
  do {                                                                                  \
    if (ra.sums_in_pass) hipLaunchKernelGGL((k_resample1<SYS, IT, true>), grid, blk, 0, pf->s, ra); \
    else hipLaunchKernelGGL((k_resample1<SYS, IT, false>), grid, blk, 0, pf->s, ra);                \
  } while (0)
    switch (pf->rs_it * 2 + (sys ? 1 : 0)) {
      case 9: GH_RS1(true, 4); break;
      case 8: GH_RS1(false, 4); break;
      case 17: GH_RS1(true, 8); break;
      case 16: GH_RS1(false, 8); break;
      case 33: GH_RS1(true, 16); break;
      default: GH_RS1(false, 16); break;
    }
#undef GH_RS1
    pf->stats_valid = true;
    pf->dec_posted = want_decision;
    if (sys) {
      pf->marks_pending = true;
    } else {
      SearchArgs sa{};
      sa.C = pf->C;
      sa.n_cdf = n;
      sa.n_slots = n;
      sa.slot_lo = 0;
      sa.n_global = pf->n_global;
      sa.seed = pf->seed;
      sa.t = (uint32_t)t;
      sa.mode = SEARCH_MULTINOMIAL;
      sa.anc_old = nullptr;
      sa.anc_out = anc_for_step(pf, t + 1);
      hipLaunchKernelGGL(k_search, dim3((unsigned)pf->nb_step), dim3(kBlock), 0, pf->s, sa, g, pf->dev);
    }
    HIP_TRY(hipGetLastError());
    pf->resample_calls++;
    return GH_OK;
  }
  if (multi && R <= kMaxRanks && !second && n > 0 && sys && pf->rs_grid > 0) {
    CHECK(rank_resample(pf, d, g.shift, t));
    pf->resample_calls++;
    return GH_OK;
  }
  CHECK(ensure_stats(pf));
  const bool fused = !second && n > 0;
  if (second && pf->marks_pending) CHECK(materialize_marks(pf));
  if (!fused) hipLaunchKernelGGL(k_decide, dim3(1), dim3(64), 0, pf->s, d, pf->dev);
  const int fmode = fused ? 1 : 0;
  if (n > 0)
    hipLaunchKernelGGL(k_qsum, dim3((unsigned)pf->nb_scan), dim3(kBlock), 0, pf->s, pf->logw, n, g, pf->bsum,
                       fmode, d, pf->dev);
  if (multi) {
    hipLaunchKernelGGL(k_rank_total, dim3(1), dim3(kBlock), 0, pf->s, g.gate, pf->bsum, n > 0 ? pf->nb_scan : 0,
                       pf->dev);
    CHECK(comm_allgather(pf->ctx, &pf->dev->local, pf->totals_all, sizeof(uint64_t), pf->s, &pf->dev->error));
  }
  int32_t* anc_target = anc_for_step(pf, t + 1);
  const bool sys1 = !multi && pf->opts.resampler == GH_RESAMPLE_SYSTEMATIC;
  MarkArgs mk{};
  mk.mark = pf->mark;
  mk.cmark = pf->cmark;
  CHECK(next_mark_tag(pf, &mk.tag));
  mk.n_global = pf->n_global;
  mk.n_groups = (pf->n + 63) / 64;
  mk.enabled = sys1 ? 1 : 0;
  CdfArgs ca{};
  ca.bsum = pf->bsum;
  ca.nb = pf->nb_scan;
  ca.totals = multi ? pf->totals_all : nullptr;
  ca.R = R;
  ca.rank = pf->ctx->rank;
  ca.n_global = pf->n_global;
  ca.seed = pf->seed;
  ca.t = (uint32_t)t;
  ca.stream = STREAM_RESAMPLE;
  if (n > 0)
    hipLaunchKernelGGL(k_cdf, dim3((unsigned)pf->nb_scan), dim3(kBlock), 0, pf->s, pf->logw, n, g, ca, pf->dev,
                       pf->C, mk);
  if (sys1) {
    // systematic, one rank: the ancestors are the range marks; the next step
    // kernel expands them (no search, no ancestor array round trip)
    if (second) {
      hipLaunchKernelGGL(k_sys_ancestors, dim3((unsigned)pf->nb_step), dim3(kBlock), 0, pf->s, g.gate, g.zero_w,
                         pf->mark, pf->cmark, (uint32_t)((1ull << pf->mark_bits) - 1), n,
                         (const int32_t*)anc_target, pf->anc_scratch,
                         (const DevScalars*)pf->dev, 1);
      hipLaunchKernelGGL(k_copy_anc, dim3((unsigned)pf->nb_step), dim3(kBlock), 0, pf->s, &pf->dev->fire,
                         pf->anc_scratch, anc_target, n);
    } else {
      pf->marks_pending = true;
    }
  } else if (!multi) {
    SearchArgs sa{};
    sa.C = pf->C;
    sa.n_cdf = n;
    sa.n_slots = n;
    sa.slot_lo = 0;
    sa.n_global = pf->n_global;
    sa.seed = pf->seed;
    sa.t = (uint32_t)t;
    sa.mode = pf->opts.resampler == GH_RESAMPLE_SYSTEMATIC ? SEARCH_SYSTEMATIC : SEARCH_MULTINOMIAL;
    sa.anc_old = second ? anc_target : nullptr;
    sa.anc_out = second ? pf->anc_scratch : anc_target;
    hipLaunchKernelGGL(k_search, dim3((unsigned)pf->nb_step), dim3(kBlock), 0, pf->s, sa, g, pf->dev);
    if (second)
      hipLaunchKernelGGL(k_copy_anc, dim3((unsigned)pf->nb_step), dim3(kBlock), 0, pf->s, &pf->dev->fire,
                         pf->anc_scratch, anc_target, n);
  } else {
    if (second) return set_err(GH_E_STATE, "multi-rank: maybe_resample twice without a step is not supported");
    if (pf->opts.resampler == GH_RESAMPLE_MULTINOMIAL) CHECK(exchange_states_mn(pf, anc_target));
    else CHECK(exchange_states(pf, anc_target));
  }
  HIP_TRY(hipGetLastError());
  pf->resample_calls++;
  return GH_OK;
}

extern "C" int gh_pf_maybe_resample(gh_pf* pf, double thr, int* did, double* ess) {
  if (!pf) return set_err(GH_E_INVAL, "null pf");
  if (pf->t < 1) return set_err(GH_E_STATE, "maybe_resample before init");
  // NaN selects the reference's default N/2 (particle_filter.jl:190); any
  // other value is the threshold itself: ess < 0 never holds, so a threshold
  // <= 0 turns resampling off exactly as in maybe_resample! (:194)
  if (thr != thr) thr = (double)pf->n_global / 2.0;
  if (thr < 0.0)
    return set_err(GH_E_INVAL, "ess_threshold %g < 0: pass NaN for the default N/2, 0 to never resample", thr);
  CHECK(resample_enqueue(pf, thr, did || ess));
  // conditional SMC: the distinguished particle's parent is itself (smc.jl:139);
  // the ancestor array is only read if the resample fired
  if (pf->cond && !mr(pf->ctx)) HIP_TRY(hipMemsetAsync(anc_for_step(pf, pf->t + 1), 0, sizeof(int32_t), pf->s));
  if (did || ess) {
    // the fused one-rank resample posts its decision to the host mailbox as
    // soon as it is taken: wait for that, not for the stream (the caller's
    // next particle_filter_step! is enqueued while the marks are written)
    if (pf->dec_posted) {
      const int rc = wait_decision(pf);
      if (rc == GH_OK) {
        const uint64_t w = __atomic_load_n(&pf->h_dec[1], __ATOMIC_ACQUIRE);
        const int err = (int)(uint32_t)(w >> 32);
        if (err) return dev_fail(err);
        if (did) *did = (int)(uint32_t)w;
        if (ess) *ess = as_f64(__atomic_load_n(&pf->h_dec[2], __ATOMIC_ACQUIRE));
        return GH_OK;
      }
      if (rc != GH_E_STATE) return rc;  // (drained without a post: the device error below)
    }
    DevScalars h;
    HIP_TRY(hipMemcpyAsync(&h, pf->dev, sizeof h, hipMemcpyDeviceToHost, pf->s));
    HIP_TRY(hipStreamSynchronize(pf->s));
    if (h.error) return dev_fail(h.error);
    if (did) *did = h.fire;
    if (ess) *ess = h.ess;
  }
  return GH_OK;
}

extern "C" int gh_pf_run(gh_pf* pf, int n_steps, const gh_obs* obs, int proposal, double thr) {
  if (!pf || n_steps < 0) return set_err(GH_E_INVAL, "gh_pf_run: bad argument");
  // A step followed by this loop's own maybe_resample! leaves the weight sums
  // to the fused resample kernel (k_step writes block maxima only; one rank,
  // fused path only); the last step writes full partials for other readers.
  // Multi-rank (systematic): the maxima go to the step's atomic-max shards and
  // the sums into k_rank_a2's pass (no fold launch, no all-gather of triples).
  const bool multi = mr(pf->ctx);
  const bool fused = pf->rs_grid > 0 && !pf->cond && pf->n > 0 &&
                     (!multi || (pf->opts.resampler == GH_RESAMPLE_SYSTEMATIC && pf->ctx->world <= kMaxRanks));
  for (int i = 0; i < n_steps; ++i) {
    CHECK(gh_pf_maybe_resample(pf, thr, nullptr, nullptr));
    pf->step_max_only = fused && i + 1 < n_steps;
    const int rc = gh_pf_step(pf, obs ? &obs[i] : nullptr, proposal);
    pf->step_max_only = false;
    CHECK(rc);
  }
  return GH_OK;
}

static int read_scalars(gh_pf* pf, DevScalars* h, std::vector<double>* stats) {
  HIP_TRY(hipMemcpyAsync(h, pf->dev, sizeof *h, hipMemcpyDeviceToHost, pf->s));
  if (stats) {
    stats->resize(3 * pf->ctx->world);
    HIP_TRY(hipMemcpyAsync(stats->data(), pf->stats_all, sizeof(double) * stats->size(), hipMemcpyDeviceToHost, pf->s));
  }
  HIP_TRY(hipStreamSynchronize(pf->s));
  return GH_OK;
}

extern "C" int gh_pf_log_ml_estimate(gh_pf* pf, double* out) {
  if (!pf || !out) return set_err(GH_E_INVAL, "null argument");
  DevScalars h;
  std::vector<double> st;
  CHECK(ensure_stats(pf));
  CHECK(read_scalars(pf, &h, &st));
  if (h.error) return dev_fail(h.error);
  if (flags_live(pf) && (h.pending | h.fire)) {  // all weights are 0: logsumexp(w) - log N = 0
    *out = h.log_ml_est;
    return GH_OK;
  }
  // log_ml_est + logsumexp(log_weights) - log(N)   (particle_filter.jl:52-55)
  const int R = pf->ctx->world;
  double M = -INFINITY;
  for (int r = 0; r < R; ++r) M = fmax(M, st[3 * r]);
  if (!(M > -INFINITY)) {
    *out = -INFINITY;
    return GH_OK;
  }
  double S = 0.0;
  for (int r = 0; r < R; ++r)
    if (st[3 * r] > -INFINITY) S += st[3 * r + 1] * gh_exp(st[3 * r] - M);
  *out = h.log_ml_est + (M + gh_log(S)) - gh_log((double)pf->n_global);
  return GH_OK;
}

extern "C" int gh_pf_num_particles(const gh_pf* pf, int64_t* ng, int64_t* nl, int64_t* first) {
  if (!pf) return set_err(GH_E_INVAL, "null pf");
  if (ng) *ng = pf->n_global;
  if (nl) *nl = pf->n;
  if (first) *first = pf->lo;
  return GH_OK;
}

extern "C" int gh_pf_num_steps(const gh_pf* pf, int* t) {
  if (!pf || !t) return set_err(GH_E_INVAL, "null argument");
  *t = pf->t;
  return GH_OK;
}

extern "C" int gh_pf_get_log_weights(gh_pf* pf, double* out) {
  if (!pf || !out) return set_err(GH_E_INVAL, "null argument");
  DevScalars h;
  CHECK(read_scalars(pf, &h, nullptr));
  if (flags_live(pf) && (h.pending | h.fire)) {
    for (int64_t i = 0; i < pf->n; ++i) out[i] = 0.0;
    return GH_OK;
  }
  CHECK(d2h(pf, out, pf->logw, sizeof(double) * pf->n));
  return GH_OK;
}

// ------------------------------------------- multi-rank genealogy queries
// (kernels in gh_kernels.h "multi-rank genealogy").  Collective:
// every rank calls the same query.  Cursors = the global ids of this rank's
// particles' ancestors at the step the walk has reached.
struct DBuf {
  void* p = nullptr;
  ~DBuf() {
    if (p) hipFree(p);
  }
  template <class T>
  T* as() const {
    return (T*)p;
  }
};
static int dalloc(DBuf& b, size_t bytes) {
  if (hipMalloc(&b.p, bytes ? bytes : 8) != hipSuccess) return set_err(GH_E_NOMEM, "genealogy query: %zu bytes", bytes);
  return GH_OK;
}

struct MrWalk {
  gh_pf* pf = nullptr;
  int64_t n = 0, N = 0, pad = 0;
  int R = 1;
  std::vector<int32_t> res;  // res[s]: a resample preceded step s
  DBuf cur, gp, gp_all;
};

static const double* rh_of(const gh_pf* pf, int s) {
  return s >= 1 && s - 1 < (int)pf->rh_step.size() ? pf->rh_step[s - 1] : nullptr;
}
static int64_t rh_count(const gh_pf* pf, int s) {
  return s >= 1 && s - 1 < (int)pf->rh_cnt.size() ? pf->rh_cnt[s - 1] : 0;
}
// after a genealogy query's kernels: a broken record they met (kErrGenealogy)
static int walk_status(gh_pf* pf) {
  int e = 0;
  HIP_TRY(hipMemcpyAsync(&e, &pf->dev->error, sizeof(int), hipMemcpyDeviceToHost, pf->s));
  HIP_TRY(hipStreamSynchronize(pf->s));
  return e ? dev_fail(e) : GH_OK;
}

static int mr_walk_begin(gh_pf* pf, MrWalk& w) {
  CHECK(materialize_marks(pf));
  w.pf = pf;
  w.n = pf->n;
  w.N = pf->n_global;
  w.R = pf->ctx->world;
  w.pad = (w.N + w.R - 1) / w.R;
  w.res.assign(pf->cap + 2, 0);
  CHECK(d2h(pf, w.res.data(), pf->res_hist, sizeof(int32_t) * (pf->cap + 2)));
  DevScalars h;
  CHECK(d2h(pf, &h, pf->dev, sizeof h));
  // (a device error raised earlier does not end the walk here: the query is
  // collective, so every rank runs all of its all-gathers and the error is
  // reported at the end, walk_status — a rank that returned early would
  // leave the others waiting in the next all-gather)
  CHECK(dalloc(w.cur, sizeof(int64_t) * (size_t)w.n));
  CHECK(dalloc(w.gp, sizeof(int64_t) * (size_t)w.pad));
  CHECK(dalloc(w.gp_all, sizeof(int64_t) * (size_t)w.pad * w.R));
  const dim3 grid((unsigned)((w.n + kBlock - 1) / kBlock));
  if (flags_live(pf) && (h.pending | h.fire) && pf->cap >= pf->t + 1) {
    // a resample pending after the last step: the particles are its copies,
    // slot j's parent (local, or a row received for the next step)
    hipLaunchKernelGGL(k_mr_gparents, grid, dim3(kBlock), 0, pf->s, (const int32_t*)anc_for_step(pf, pf->t + 1), w.n,
                       pf->lo, (const double*)pf->rows_recv, w.n, pf->D, w.cur.as<int64_t>(),
                       &pf->dev->error);
  } else {
    hipLaunchKernelGGL(k_iota64, grid, dim3(kBlock), 0, pf->s, w.cur.as<int64_t>(), w.n, pf->lo);
  }
  HIP_TRY(hipGetLastError());
  return GH_OK;
}

// every cursor from step s back to step s - 1
static int mr_walk_back(MrWalk& w, int s) {
  gh_pf* pf = w.pf;
  if (!w.res[s]) return GH_OK;
  const dim3 grid((unsigned)((w.n + kBlock - 1) / kBlock));
  hipLaunchKernelGGL(k_mr_gparents, grid, dim3(kBlock), 0, pf->s, (const int32_t*)anc_for_step(pf, s), w.n, pf->lo,
                     rh_of(pf, s), rh_count(pf, s), pf->D, w.gp.as<int64_t>(), &pf->dev->error);
  HIP_TRY(hipGetLastError());
  CHECK(bulk_allgather(pf->ctx, w.gp.p, w.gp_all.p, sizeof(int64_t) * (size_t)w.pad, pf->s));
  hipLaunchKernelGGL(k_mr_back, grid, dim3(kBlock), 0, pf->s, w.cur.as<int64_t>(), w.n,
                     (const int64_t*)w.gp_all.as<int64_t>(), (const int64_t*)pf->dlo, w.R, w.N, w.pad,
                     &pf->dev->error);
  HIP_TRY(hipGetLastError());
  return GH_OK;
}

// get_traces at step t on R ranks: the states of this rank's particles' ancestors, [D][n] on the device
static int mr_trajectory(gh_pf* pf, int t, double* dout) {
  MrWalk w;
  CHECK(mr_walk_begin(pf, w));
  for (int s = pf->t; s > t; --s) CHECK(mr_walk_back(w, s));
  const int64_t pad_d = slot_doubles(w.pad, pf->D);
  DBuf send, slab;
  CHECK(dalloc(send, sizeof(double) * (size_t)pad_d));
  CHECK(dalloc(slab, sizeof(double) * (size_t)pad_d * w.R));
  HIP_TRY(hipMemsetAsync(send.p, 0, sizeof(double) * (size_t)pad_d, pf->s));
  HIP_TRY(hipMemcpyAsync(send.p, slot_x(pf, t), sizeof(double) * (size_t)slot_doubles(w.n, pf->D),
                         hipMemcpyDeviceToDevice, pf->s));
  CHECK(bulk_allgather(pf->ctx, send.p, slab.p, sizeof(double) * (size_t)pad_d, pf->s));
  hipLaunchKernelGGL(k_mr_states, dim3((unsigned)((w.n + kBlock - 1) / kBlock)), dim3(kBlock), 0, pf->s,
                     (const int64_t*)w.cur.as<int64_t>(), w.n, (const double*)slab.as<double>(), pad_d,
                     (const int64_t*)pf->dlo, w.R, w.N, pf->D, dout, &pf->dev->error);
  HIP_TRY(hipGetLastError());
  return walk_status(pf);
}

// the score columns on R ranks (k_scores' values): per step, every rank
// scores its own slots, the ranks all-gather them, each cursor takes its
// slot's pair, then the cursors step back
static int mr_scores(gh_pf* pf, const gh_model* m, const std::vector<StepObs>& obs, double* dtot, double* dper) {
  MrWalk w;
  CHECK(mr_walk_begin(pf, w));
  const int T = pf->t;
  const int64_t n = w.n;
  DBuf sc, sc_all;
  CHECK(dalloc(sc, sizeof(double) * 2 * (size_t)w.pad));
  CHECK(dalloc(sc_all, sizeof(double) * 2 * (size_t)w.pad * w.R));
  HIP_TRY(hipMemsetAsync(sc.p, 0, sizeof(double) * 2 * (size_t)w.pad, pf->s));
  const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
  for (int s = T; s >= 1; --s) {
    const int32_t* anc = s > 1 && w.res[s] ? anc_for_step(pf, s) : nullptr;
    CHECK(with_model(m, [&](auto model, const auto& p) {
      hipLaunchKernelGGL(k_mr_slot_scores<decltype(model)>, grid, dim3(kBlock), 0, pf->s, (const double*)m->dparams,
                         p, obs[s - 1], s, (const double*)slot_x(pf, s),
                         (const double*)(s > 1 ? slot_x(pf, s - 1) : nullptr), anc, rh_of(pf, s), rh_count(pf, s),
                         n, w.pad, sc.as<double>(), &pf->dev->error);
    }));
    HIP_TRY(hipGetLastError());
    CHECK(bulk_allgather(pf->ctx, sc.p, sc_all.p, sizeof(double) * 2 * (size_t)w.pad, pf->s));
    hipLaunchKernelGGL(k_mr_take_scores, grid, dim3(kBlock), 0, pf->s, (const int64_t*)w.cur.as<int64_t>(), n,
                       (const double*)sc_all.as<double>(), (const int64_t*)pf->dlo, w.R, w.N, w.pad,
                       dper + (int64_t)(s - 1) * 2 * n, dper + ((int64_t)(s - 1) * 2 + 1) * n, &pf->dev->error);
    HIP_TRY(hipGetLastError());
    if (s > 1) CHECK(mr_walk_back(w, s));
  }
  hipLaunchKernelGGL(k_score_total, grid, dim3(kBlock), 0, pf->s, (const double*)dper, T, n, dtot);
  HIP_TRY(hipGetLastError());
  return walk_status(pf);
}

extern "C" int gh_pf_get_trajectory(gh_pf* pf, int t, double* out) {
  if (!pf || !out) return set_err(GH_E_INVAL, "null argument");
  CHECK(materialize_marks(pf));
  if (t < 1 || t > pf->t) return set_err(GH_E_INVAL, "step %d outside 1..%d", t, pf->t);
  if (!pf->opts.record_history && t != pf->t)
    return set_err(GH_E_STATE, "record_history is off: only the current step is kept");
  const int64_t n = pf->n;
  if (n == 0) return GH_OK;
  if (mr(pf->ctx)) {  // collective: the walk crosses ranks
    DBuf d;
    CHECK(dalloc(d, sizeof(double) * pf->D * (size_t)n));
    CHECK(mr_trajectory(pf, t, d.as<double>()));
    HIP_TRY(hipMemcpy(out, d.p, sizeof(double) * pf->D * (size_t)n, hipMemcpyDeviceToHost));
    return GH_OK;
  }
  double* dout = nullptr;
  const double** dxs = nullptr;
  const int32_t** dancs = nullptr;
  HIP_TRY(hipMalloc(&dout, sizeof(double) * pf->D * n));
  const int T = pf->t;
  std::vector<const double*> hx(T);
  std::vector<const int32_t*> ha(T);
  for (int s = 1; s <= T; ++s) {
    hx[s - 1] = slot_x(pf, s);
    ha[s - 1] = anc_for_step(pf, s);
  }
  HIP_TRY(hipMalloc(&dxs, sizeof(double*) * T));
  HIP_TRY(hipMalloc(&dancs, sizeof(int32_t*) * T));
  HIP_TRY(hipMemcpyAsync(dxs, hx.data(), sizeof(double*) * T, hipMemcpyHostToDevice, pf->s));
  HIP_TRY(hipMemcpyAsync(dancs, ha.data(), sizeof(int32_t*) * T, hipMemcpyHostToDevice, pf->s));
  TrajArgs ta{};
  ta.xs = dxs;
  ta.ancs = dancs;
  ta.res_before = pf->res_hist;
  ta.anc_pending = (!mr(pf->ctx) && pf->cap >= T + 1) ? anc_for_step(pf, T + 1) : nullptr;
  ta.live = flags_live(pf);
  ta.n = n;
  ta.t_target = t;
  ta.t_cur = T;
  ta.D = pf->D;
  ta.out = dout;
  hipLaunchKernelGGL(k_traj, dim3((unsigned)pf->nb_step), dim3(kBlock), 0, pf->s, ta, pf->dev);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, dout, sizeof(double) * pf->D * n, hipMemcpyDeviceToHost, pf->s));
  HIP_TRY(hipStreamSynchronize(pf->s));
  hipFree(dout);
  hipFree(dxs);
  hipFree(dancs);
  return GH_OK;
}

// Trace score columns (gh_scores.h): per particle and step the latent's and
// the observation's score, and the trace's total (get_score).
// The trace score columns of every current particle (k_scores: the genealogy
// walk) under model m and the steps' observations obs[0..T): dtot[n] and the
// per-step scratch/output dper[T][2][n], device buffers, on the filter's stream.
static int mr_scores(gh_pf* pf, const gh_model* m, const std::vector<StepObs>& obs, double* dtot, double* dper);

static int scores_dev(gh_pf* pf, const gh_model* m, const std::vector<StepObs>& obs, double* dtot, double* dper) {
  if (mr(pf->ctx)) return mr_scores(pf, m, obs, dtot, dper);
  const int T = pf->t;
  const int64_t n = pf->n;
  const double** dxs = nullptr;
  const int32_t** dancs = nullptr;
  StepObs* dobs = nullptr;
  auto cleanup = [&]() { hipFree(dxs); hipFree(dancs); hipFree(dobs); };
  std::vector<const double*> hx(T);
  std::vector<const int32_t*> ha(T);
  for (int s = 1; s <= T; ++s) {
    hx[s - 1] = slot_x(pf, s);
    ha[s - 1] = anc_for_step(pf, s);
  }
  if (hipMalloc(&dxs, sizeof(double*) * T) != hipSuccess || hipMalloc(&dancs, sizeof(int32_t*) * T) != hipSuccess ||
      hipMalloc(&dobs, sizeof(StepObs) * T) != hipSuccess) {
    cleanup();
    return set_err(GH_E_NOMEM, "scores: %d steps", T);
  }
  int rc = GH_OK;
  do {
    if (hipMemcpyAsync(dxs, hx.data(), sizeof(double*) * T, hipMemcpyHostToDevice, pf->s) != hipSuccess ||
        hipMemcpyAsync(dancs, ha.data(), sizeof(int32_t*) * T, hipMemcpyHostToDevice, pf->s) != hipSuccess ||
        hipMemcpyAsync(dobs, obs.data(), sizeof(StepObs) * T, hipMemcpyHostToDevice, pf->s) != hipSuccess) {
      rc = set_err(GH_E_HIP, "scores: upload");
      break;
    }
    ScoreArgs sa{};
    sa.xs = dxs;
    sa.ancs = dancs;
    sa.res_before = pf->res_hist;
    sa.anc_pending = (!mr(pf->ctx) && pf->cap >= T + 1) ? anc_for_step(pf, T + 1) : nullptr;
    sa.live = flags_live(pf);
    sa.obs = dobs;
    sa.n = n;
    sa.T = T;
    sa.per_step = dper;
    sa.total = dtot;
    const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
    // the model's own densities, whatever proposal made the particles
    rc = with_model(m, [&](auto model, const auto& p) {
      hipLaunchKernelGGL(k_scores<decltype(model)>, grid, dim3(kBlock), 0, pf->s, (const double*)m->dparams, p, sa,
                         (const DevScalars*)pf->dev);
    });
    if (rc) break;
    if (hipGetLastError() != hipSuccess) rc = set_err(GH_E_HIP, "scores: launch");
    // the argument arrays are freed below: wait for the kernel
    if (!rc && hipStreamSynchronize(pf->s) != hipSuccess) rc = set_err(GH_E_HIP, "scores: sync");
  } while (0);
  cleanup();
  return rc;
}

static int scores_ready(gh_pf* pf, const char* who) {
  CHECK(materialize_marks(pf));
  const int T = pf->t;
  if (T < 1) return set_err(GH_E_STATE, "%s before init", who);
  if (!pf->opts.record_history && T > 1) return set_err(GH_E_STATE, "%s needs record_history", who);
  if ((int)pf->obs_hist.size() < T) return set_err(GH_E_STATE, "internal: observation history");
  return GH_OK;
}

extern "C" int gh_pf_get_scores(gh_pf* pf, double* total, double* per_step) {
  if (!pf || !total) return set_err(GH_E_INVAL, "null argument");
  CHECK(scores_ready(pf, "gh_pf_get_scores"));
  const int T = pf->t;
  const int64_t n = pf->n;
  if (n == 0) return GH_OK;
  double *dtot = nullptr, *dper = nullptr;
  if (hipMalloc(&dtot, sizeof(double) * n) != hipSuccess ||
      hipMalloc(&dper, sizeof(double) * 2 * (size_t)T * n) != hipSuccess) {
    hipFree(dtot);
    hipFree(dper);
    return set_err(GH_E_NOMEM, "gh_pf_get_scores: %d steps x %lld particles", T, (long long)n);
  }
  int rc = scores_dev(pf, pf->m, pf->obs_hist, dtot, dper);
  if (!rc && (hipMemcpyAsync(total, dtot, sizeof(double) * n, hipMemcpyDeviceToHost, pf->s) != hipSuccess ||
              (per_step && hipMemcpyAsync(per_step, dper, sizeof(double) * 2 * (size_t)T * n, hipMemcpyDeviceToHost,
                                          pf->s) != hipSuccess) ||
              hipStreamSynchronize(pf->s) != hipSuccess))
    rc = set_err(GH_E_HIP, "gh_pf_get_scores: download");
  hipFree(dtot);
  hipFree(dper);
  return rc;
}

// particle_filter_step!(state, (t, params'...), (UnknownChange(), UnknownChange()...), obs)
// (particle_filter.jl:162-180) with the Unfold's parameters changed to those of
// nm: the Unfold's update re-visits every retained kernel application
// (unfold/generic_update.jl:9-16), each contributing new score - old score
// (no new constraints on them), then generates the new application under the
// new parameters.  Delta_j = get_score under nm - under the old model along
// particle j's trajectory (k_scores twice; the past observations rebuilt under
// nm), the step under nm, then logw_j += Delta_j and the block partials again
// (k_add_delta).  One rank, history kept, same family and dimensions.
static int step_params_impl(gh_pf* pf, const gh_obs* obs, int proposal, gh_model* nm, const double* pin_ref);

extern "C" int gh_pf_step_params(gh_pf* pf, const gh_obs* obs, int proposal, gh_model* nm) {
  if (!pf || !nm) return set_err(GH_E_INVAL, "gh_pf_step_params: null argument");
  if (pf->cond)
    return set_err(GH_E_STATE, "gh_pf_step_params: a conditional filter steps with gh_pf_step_params_conditional");
  return step_params_impl(pf, obs, proposal, nm, nullptr);
}

// conditional SMC with changed parameters (particle Gibbs with parameter
// moves): the re-scoring of gh_pf_step_params, then the conditional step
// pinning the distinguished particle to ref_xt
extern "C" int gh_pf_step_params_conditional(gh_pf* pf, const gh_obs* obs, gh_model* nm, const double* ref_xt) {
  if (!pf || !nm || !ref_xt) return set_err(GH_E_INVAL, "gh_pf_step_params_conditional: null argument");
  if (!pf->cond)
    return set_err(GH_E_STATE, "gh_pf_step_params_conditional on a filter not made by gh_pf_init_conditional");
  return step_params_impl(pf, obs, GH_PROPOSAL_DEFAULT, nm, ref_xt);
}

static int step_params_impl(gh_pf* pf, const gh_obs* obs, int proposal, gh_model* nm, const double* pin_ref) {
  if (!pf->opts.record_history) return set_err(GH_E_STATE, "gh_pf_step_params needs record_history");
  const gh_model* m = pf->m;
  if (m->family == GH_FAMILY_SLOTS && (nm->family != m->family || !same_slots(m, nm)))
    return set_err(GH_E_INVAL, "gh_pf_step_params: the new slot model must keep the latent form and every slot's "
                               "distribution, size and mean form");
  if (nm->ctx != m->ctx || nm->family != m->family || nm->d != m->d || nm->dy != m->dy || nm->k != m->k ||
      nm->v != m->v)
    return set_err(GH_E_INVAL, "gh_pf_step_params: the new parameters must be of the same family and dimensions");
  if (!proposal_ok(nm, proposal)) return set_err(GH_E_INVAL, "gh_pf_step_params: proposal %d not available", proposal);
  CHECK(step_qargs(pf, proposal, nullptr, 0));
  CHECK(scores_ready(pf, "gh_pf_step_params"));
  const int T = pf->t;
  const int64_t n = pf->n;
  std::vector<StepObs> rebuilt(T);
  for (int s = 1; s <= T; ++s) {
    const auto& r = pf->raw_obs[s - 1];
    if (m->family == GH_FAMILY_SLOTS) {
      gh_obs chain[kMaxSlots];
      CHECK(make_obs(nm, s, slot_chain(r, chain), &rebuilt[s - 1]));
      continue;
    }
    const gh_obs in{r.empty() ? nullptr : r.data(), (int32_t)r.size(), r.empty() ? 0 : 1};
    CHECK(make_obs(nm, s, &in, &rebuilt[s - 1]));
  }
  double *dold = nullptr, *dnew = nullptr, *dper = nullptr;
  auto cleanup = [&]() { hipFree(dold); hipFree(dnew); hipFree(dper); };
  const size_t nn = (size_t)(n > 0 ? n : 1);
  if (hipMalloc(&dold, sizeof(double) * nn) != hipSuccess || hipMalloc(&dnew, sizeof(double) * nn) != hipSuccess ||
      hipMalloc(&dper, sizeof(double) * 2 * (size_t)T * nn) != hipSuccess) {
    cleanup();
    return set_err(GH_E_NOMEM, "gh_pf_step_params: re-scoring buffers (%d steps)", T);
  }
  int rc = GH_OK;
  if (n > 0) {
    rc = scores_dev(pf, m, pf->obs_hist, dold, dper);
    if (!rc) rc = scores_dev(pf, nm, rebuilt, dnew, dper);
  }
  if (rc) {
    cleanup();
    return rc;
  }
  {  // the new step's observation under the new parameters, checked before anything changes
    StepObs probe;
    rc = make_obs(nm, T + 1, obs, &probe);
    if (rc) {
      cleanup();
      return rc;
    }
  }
  const gh_model* m_old = pf->m;
  std::vector<StepObs> hist_old = pf->obs_hist;
  pf->m = nm;
  pf->obs_hist = rebuilt;
  pf->no_max_only = true;  // k_add_delta rewrites full partials of the changed weights
  rc = pf_step_impl(pf, obs, proposal, pin_ref);
  pf->no_max_only = false;
  if (rc && pf->t == T) {  // no step was taken: the filter keeps its model and history
    pf->m = const_cast<gh_model*>(m_old);
    pf->obs_hist = hist_old;
  }
  if (!rc && n > 0) {
    hipLaunchKernelGGL(k_add_delta, dim3((unsigned)pf->nb_step), dim3(kBlock), 0, pf->s, pf->logw,
                       (const double*)dnew, (const double*)dold, n, pf->pm, pf->ps, pf->ps2);
    if (hipGetLastError() != hipSuccess) rc = set_err(GH_E_HIP, "gh_pf_step_params: launch");
    pf->nb_part = pf->nb_step;
    pf->last_pairs = false;
    pf->stats_valid = false;
    pf->max_only = false;
    pf->amax_valid = false;
    if (mr(pf->ctx) && !rc) {  // the rank's (M, S, S2) of the changed weights, shared again
      hipLaunchKernelGGL(k_fold, dim3(1), dim3(1024), 0, pf->s, pf->pm, pf->ps, pf->ps2, (int)pf->nb_part,
                         pf->dev->stats, pf->dev, 1, 0.0, pf->n_global);
      rc = share_stats(pf);
    }
  }
  if (hipStreamSynchronize(pf->s) != hipSuccess && !rc) rc = set_err(GH_E_HIP, "gh_pf_step_params: sync");
  cleanup();
  return rc;
}

// simulate(model, (T,)) for n independent traces (gh_simulate.h).
static int simulate_impl(gh_model* m, int T, int64_t n, uint64_t seed, const double* inputs, double* xs, double* ys,
                         double* per_step, double* total);

extern "C" int gh_simulate(gh_model* m, int T, int64_t n, uint64_t seed, double* xs, double* ys, double* per_step,
                           double* total) {
  return simulate_impl(m, T, n, seed, nullptr, xs, ys, per_step, total);
}

// simulate(model, (T, U)) for a slot model with per-step inputs: U[T*d], row t-1
// the input of step t (row 0 unused: the transition starts at t = 2)
extern "C" int gh_simulate_inputs(gh_model* m, int T, int64_t n, uint64_t seed, const double* inputs, double* xs,
                                  double* ys, double* per_step, double* total) {
  if (!m || !inputs) return set_err(GH_E_INVAL, "gh_simulate_inputs: null argument");
  if (m->family != GH_FAMILY_SLOTS || m->slots.uoff < 0)
    return set_err(GH_E_INVAL, "gh_simulate_inputs: the model takes no per-step inputs (slot latent form 2)");
  return simulate_impl(m, T, n, seed, inputs, xs, ys, per_step, total);
}

static int simulate_impl(gh_model* m, int T, int64_t n, uint64_t seed, const double* inputs, double* xs, double* ys,
                         double* per_step, double* total) {
  if (!m) return set_err(GH_E_INVAL, "gh_simulate: null model");
  if (T < 1) return set_err(GH_E_INVAL, "gh_simulate: T = %d (need >= 1)", T);
  if (m->family == GH_FAMILY_REGRESSION && T != 1)
    return set_err(GH_E_INVAL, "gh_simulate: the regression model has no time steps (T = 1)");
  if (n < 0 || n > INT32_MAX) return set_err(GH_E_INVAL, "gh_simulate: n = %lld", (long long)n);
  if (m->family == GH_FAMILY_SLOTS && m->slots.uoff >= 0 && !inputs)
    return set_err(GH_E_INVAL, "gh_simulate: a slot model with per-step inputs takes them (gh_simulate_inputs)");
  if (n == 0) return GH_OK;
  HIP_TRY(hipSetDevice(m->ctx->device));
  const int d = m->d;
  const int dy = (m->family == GH_FAMILY_LGSSM || m->family == GH_FAMILY_REGRESSION || m->family == GH_FAMILY_SLOTS)
                     ? m->dy
                     : 1;
  std::vector<StepObs> hobs(T);
  for (int t = 1; t <= T; ++t) {
    CHECK(make_obs(m, t, nullptr, &hobs[t - 1]));
    if (inputs && t > 1)
      for (int j = 0; j < d; ++j) {
        const double u = inputs[(size_t)(t - 1) * d + j];
        if (!std::isfinite(u)) return set_err(GH_E_INVAL, "gh_simulate_inputs: non-finite input");
        hobs[t - 1].v[m->slots.uoff + j] = u;
      }
  }
  const size_t nx = (size_t)T * d * n, ny = (size_t)T * dy * n, ns = (size_t)T * 2 * n;
  double* buf = nullptr;
  StepObs* dobs = nullptr;
  if (hipMalloc(&buf, sizeof(double) * (nx + ny + ns + n)) != hipSuccess ||
      hipMalloc(&dobs, sizeof(StepObs) * T) != hipSuccess) {
    hipFree(buf);
    return set_err(GH_E_NOMEM, "gh_simulate: %d steps x %lld traces", T, (long long)n);
  }
  hipStream_t s = m->ctx->stream;
  int rc = GH_OK;
  do {
    if (hipMemcpyAsync(dobs, hobs.data(), sizeof(StepObs) * T, hipMemcpyHostToDevice, s) != hipSuccess) {
      rc = set_err(GH_E_HIP, "gh_simulate: upload");
      break;
    }
    SimArgs a{};
    a.seed = seed;
    a.n = n;
    a.T = T;
    a.dy = dy;
    a.obs = dobs;
    a.xs = buf;
    a.ys = buf + nx;
    a.per_step = buf + nx + ny;
    a.total = buf + nx + ny + ns;
    const dim3 grid((unsigned)((n + kBlock - 1) / kBlock));
    rc = with_model(m, [&](auto model, const auto& p) {
      hipLaunchKernelGGL(k_simulate<decltype(model)>, grid, dim3(kBlock), 0, s, (const double*)m->dparams, p, a);
    });
    if (rc) break;
    if (hipGetLastError() != hipSuccess) {
      rc = set_err(GH_E_HIP, "gh_simulate: launch");
      break;
    }
    if ((xs && hipMemcpyAsync(xs, a.xs, sizeof(double) * nx, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        (ys && hipMemcpyAsync(ys, a.ys, sizeof(double) * ny, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        (per_step && hipMemcpyAsync(per_step, a.per_step, sizeof(double) * ns, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        (total && hipMemcpyAsync(total, a.total, sizeof(double) * n, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        hipStreamSynchronize(s) != hipSuccess)
      rc = set_err(GH_E_HIP, "gh_simulate: download");
  } while (0);
  hipFree(buf);
  hipFree(dobs);
  return rc;
}

// ------------------------------------------------------------ distributions
// Batched logpdf / random of Gen's distribution library (gh_dists.h).
struct DistShape {
  int dim = 1, K = 0, prow = 0;  // value components, bins, doubles per device parameter row
};

static int dist_shape(const gh_dist_desc* d, DistShape* s) {
  const int np = d->n_params, dim = d->dim < 1 ? 1 : d->dim;
  auto need = [&](int k) { return np == k ? GH_OK : set_err(GH_E_INVAL, "distribution %d takes %d parameters, got %d", d->dist, k, np); };
  s->dim = 1;
  s->K = 0;
  s->prow = np;
  switch (d->dist) {
    case DIST_NORMAL: case DIST_UNIFORM_CONTINUOUS: case DIST_UNIFORM_DISCRETE: case DIST_GAMMA: case DIST_INV_GAMMA:
    case DIST_BETA: case DIST_BINOMIAL: case DIST_NEG_BINOMIAL: case DIST_LAPLACE: case DIST_CAUCHY:
      return need(2);
    case DIST_BERNOULLI: case DIST_EXPONENTIAL: case DIST_POISSON: case DIST_GEOMETRIC:
      return need(1);
    case DIST_BETA_UNIFORM:
      return need(3);
    case DIST_BROADCASTED_NORMAL:
      if (dim > 32) return set_err(GH_E_INVAL, "broadcasted_normal: dim <= 32");
      s->dim = dim;
      return need(2 * dim);
    case DIST_MVNORMAL:
      if (dim > 32) return set_err(GH_E_INVAL, "mvnormal: dim <= 32");
      if (d->param_stride != 0) return set_err(GH_E_INVAL, "mvnormal: one shared (mu, cov) row");
      s->dim = dim;
      s->prow = dim + dim * dim + 1;
      return need(dim + dim * dim);
    case DIST_CATEGORICAL:
      if (np < 1) return set_err(GH_E_INVAL, "categorical: at least one probability");
      s->K = np;
      return GH_OK;
    case DIST_PIECEWISE_UNIFORM:
      if (np < 3 || np % 2 == 0) return set_err(GH_E_INVAL, "piecewise_uniform: bounds[K+1] then probs[K]");
      s->K = (np - 1) / 2;
      return GH_OK;
    default:
      return set_err(GH_E_INVAL, "unknown distribution %d", d->dist);
  }
}

template <class F>
static void with_dist(int dist, F&& f) {
  switch (dist) {
#define GH_DIST_CASE(D) case D: f(std::integral_constant<int, D>{}); break;
    GH_DIST_CASE(DIST_NORMAL) GH_DIST_CASE(DIST_BROADCASTED_NORMAL) GH_DIST_CASE(DIST_MVNORMAL)
    GH_DIST_CASE(DIST_UNIFORM_CONTINUOUS) GH_DIST_CASE(DIST_UNIFORM_DISCRETE) GH_DIST_CASE(DIST_BERNOULLI)
    GH_DIST_CASE(DIST_CATEGORICAL) GH_DIST_CASE(DIST_GAMMA) GH_DIST_CASE(DIST_INV_GAMMA) GH_DIST_CASE(DIST_BETA)
    GH_DIST_CASE(DIST_EXPONENTIAL) GH_DIST_CASE(DIST_POISSON) GH_DIST_CASE(DIST_BINOMIAL)
    GH_DIST_CASE(DIST_NEG_BINOMIAL) GH_DIST_CASE(DIST_GEOMETRIC) GH_DIST_CASE(DIST_LAPLACE) GH_DIST_CASE(DIST_CAUCHY)
    GH_DIST_CASE(DIST_PIECEWISE_UNIFORM) GH_DIST_CASE(DIST_BETA_UNIFORM)
#undef GH_DIST_CASE
    default: break;
  }
}

// the device parameter rows: mvnormal's derived row, else the caller's rows
static int dist_params(gh_ctx* ctx, const gh_dist_desc* d, const DistShape& sh, int64_t n, double** dparams,
                       bool* owned) {
  *owned = false;
  if (!d->params) return set_err(GH_E_INVAL, "distribution parameters are NULL");
  if (d->param_stride != 0 && d->param_stride != d->n_params)
    return set_err(GH_E_INVAL, "param_stride must be 0 (shared row) or n_params (a row per value)");
  if (d->params_on_device) {
    if (d->dist == DIST_MVNORMAL) return set_err(GH_E_INVAL, "mvnormal parameters are host memory (Cholesky on the host)");
    *dparams = const_cast<double*>(d->params);
    return GH_OK;
  }
  std::vector<double> row;
  const double* src = d->params;
  size_t count = d->param_stride ? (size_t)n * d->n_params : (size_t)d->n_params;
  if (d->dist == DIST_MVNORMAL) {
    const int D = sh.dim;
    row.assign(sh.prow, 0.0);
    std::copy(src, src + D, row.begin());
    if (chol(D, src + D, row.data() + D)) return set_err(GH_E_INVAL, "mvnormal: covariance not positive definite");
    row[D + D * D] = gauss_cst(D, row.data() + D);
    src = row.data();
    count = row.size();
  }
  if (hipMalloc(dparams, sizeof(double) * (count ? count : 1)) != hipSuccess) return set_err(GH_E_NOMEM, "distribution parameters");
  *owned = true;
  if (hipMemcpyAsync(*dparams, src, sizeof(double) * count, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess)
    return set_err(GH_E_HIP, "distribution parameters: upload");
  return GH_OK;
}

static int dist_launch(gh_ctx* ctx, const gh_dist_desc* d, int64_t n, uint64_t seed, const double* x, double* out,
                       bool random) {
  if (!ctx || !d) return set_err(GH_E_INVAL, "null argument");
  if (n < 0 || n > ((int64_t)1 << 40)) return set_err(GH_E_INVAL, "batch size %lld", (long long)n);
  DistShape sh;
  CHECK(dist_shape(d, &sh));
  if (n == 0) return GH_OK;
  if (!out || (!random && !x)) return set_err(GH_E_INVAL, "null %s buffer", out ? "x" : "out");
  HIP_TRY(hipSetDevice(ctx->device));
  double* dp = nullptr;
  bool owned = false;
  int rc = dist_params(ctx, d, sh, n, &dp, &owned);
  if (rc == GH_OK) {
    DistArgs a{};
    a.n = n;
    a.dim = sh.dim;
    a.K = sh.K;
    a.prow = sh.prow;
    a.pstride = d->param_stride ? sh.prow : 0;
    a.params = dp;
    a.x = x;
    a.out = out;
    a.seed = seed;
    const dim3 grid((unsigned)((n + 255) / 256));
    with_dist(d->dist, [&](auto id) {
      constexpr int D = decltype(id)::value;
      if (random)
        hipLaunchKernelGGL(k_dist_random<D>, grid, dim3(256), 0, ctx->stream, a);
      else
        hipLaunchKernelGGL(k_dist_logpdf<D>, grid, dim3(256), 0, ctx->stream, a);
    });
    if (hipGetLastError() != hipSuccess) rc = set_err(GH_E_HIP, "distribution kernel launch");
  }
  if (owned) {
    if (hipStreamSynchronize(ctx->stream) != hipSuccess && rc == GH_OK) rc = set_err(GH_E_HIP, "distribution kernel");
    hipFree(dp);
  }
  return rc;
}

extern "C" int gh_dist_logpdf_dev(gh_ctx* ctx, const gh_dist_desc* d, int64_t n, const double* x, double* out) {
  return dist_launch(ctx, d, n, 0, x, out, false);
}
extern "C" int gh_dist_random_dev(gh_ctx* ctx, const gh_dist_desc* d, int64_t n, uint64_t seed, double* out) {
  return dist_launch(ctx, d, n, seed, nullptr, out, true);
}

// host-buffer forms: stage through device memory and synchronise
static int dist_host(gh_ctx* ctx, const gh_dist_desc* d, int64_t n, uint64_t seed, const double* x, double* out,
                     bool random) {
  if (!ctx || !d || !out || (!random && !x)) return set_err(GH_E_INVAL, "null argument");
  DistShape sh;
  CHECK(dist_shape(d, &sh));
  if (n <= 0) return n == 0 ? GH_OK : set_err(GH_E_INVAL, "batch size %lld", (long long)n);
  HIP_TRY(hipSetDevice(ctx->device));
  const size_t nx = (size_t)sh.dim * n, nout = random ? nx : (size_t)n;
  double *dx = nullptr, *dout = nullptr;
  if ((!random && hipMalloc(&dx, sizeof(double) * nx) != hipSuccess) || hipMalloc(&dout, sizeof(double) * nout) != hipSuccess) {
    hipFree(dx);
    return set_err(GH_E_NOMEM, "distribution batch of %lld", (long long)n);
  }
  int rc = GH_OK;
  if (!random && hipMemcpyAsync(dx, x, sizeof(double) * nx, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
    rc = set_err(GH_E_HIP, "distribution values: upload");
  if (rc == GH_OK) rc = dist_launch(ctx, d, n, seed, dx, dout, random);
  if (rc == GH_OK && (hipMemcpyAsync(out, dout, sizeof(double) * nout, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
                      hipStreamSynchronize(ctx->stream) != hipSuccess))
    rc = set_err(GH_E_HIP, "distribution results: download");
  hipFree(dx);
  hipFree(dout);
  return rc;
}

extern "C" int gh_dist_logpdf(gh_ctx* ctx, const gh_dist_desc* d, int64_t n, const double* x, double* out) {
  return dist_host(ctx, d, n, 0, x, out, false);
}
extern "C" int gh_dist_random(gh_ctx* ctx, const gh_dist_desc* d, int64_t n, uint64_t seed, double* out) {
  return dist_host(ctx, d, n, seed, nullptr, out, true);
}

extern "C" int gh_pf_get_states(gh_pf* pf, double* out) {
  if (!pf) return set_err(GH_E_INVAL, "null pf");
  if (mr(pf->ctx)) {
    DevScalars h;
    CHECK(read_scalars(pf, &h, nullptr));
    if (flags_live(pf) && (h.pending | h.fire))
      return set_err(GH_E_STATE, "multi-rank: states of a pending resample are materialised by the next step");
  }
  return gh_pf_get_trajectory(pf, pf->t, out);  // untiles the slot into [D][n]
}

extern "C" int gh_pf_get_parents(gh_pf* pf, int64_t* out) {
  if (!pf || !out) return set_err(GH_E_INVAL, "null argument");
  CHECK(materialize_marks(pf));
  // ParticleFilterState.parents: ancestors chosen by the most recent resample
  // (identity before the first one), as global 0-based ids.
  std::vector<int32_t> res(pf->cap + 2);
  CHECK(d2h(pf, res.data(), pf->res_hist, sizeof(int32_t) * (pf->cap + 2)));
  int s_last = -1;
  for (int s = pf->t + 1; s >= 2 && s < pf->cap + 2; --s)
    if (res[s]) { s_last = s; break; }
  if (s_last < 0) {
    for (int64_t i = 0; i < pf->n; ++i) out[i] = pf->lo + i;
    return GH_OK;
  }
  if (mr(pf->ctx)) {
    // the most recent resample (before step s_last): local ancestors plus the
    // global ids carried by the received rows
    hipLaunchKernelGGL(k_global_parents, dim3((unsigned)pf->nb_step), dim3(kBlock), 0, pf->s,
                       (const int32_t*)anc_for_step(pf, s_last), pf->n, pf->lo, (const double*)pf->rows_recv,
                       pf->D, pf->gparent);
    HIP_TRY(hipGetLastError());
    CHECK(d2h(pf, out, pf->gparent, sizeof(int64_t) * pf->n));
    return GH_OK;
  }
  std::vector<int32_t> a(pf->n);
  CHECK(d2h(pf, a.data(), anc_for_step(pf, s_last), sizeof(int32_t) * pf->n));
  for (int64_t i = 0; i < pf->n; ++i) out[i] = pf->lo + a[i];
  return GH_OK;
}

// ------------------------------------------------------------ rejuvenation
template <class Model>
static void launch_rejuv_t(gh_pf* pf, const typename Model::Params& p, const RejuvArgs& a, bool init) {
  const dim3 grid((unsigned)pf->nb_step), block(kBlock);
  if (init)
    hipLaunchKernelGGL((k_rejuv<Model, true>), grid, block, 0, pf->s, (const double*)pf->m->dparams, p,
                       pf->last_obs, a);
  else
    hipLaunchKernelGGL((k_rejuv<Model, false>), grid, block, 0, pf->s, (const double*)pf->m->dparams, p,
                       pf->last_obs, a);
}

static int launch_rejuv(gh_pf* pf, const RejuvArgs& a, bool init) {
  CHECK(with_model(pf->m, [&](auto model, const auto& p) { launch_rejuv_t<decltype(model)>(pf, p, a, init); }));
  HIP_TRY(hipGetLastError());
  return GH_OK;
}

// mh(trace, select(x_t)) on every particle (gh_rejuv.h).  The states of step t
// are rewritten in place; the parent states are those step t consumed: the
// previous slot through the step's ancestors, or rows received from other
// ranks (still resident until the next exchange).
// latent addresses of the current step a selection may name (bit i = address i)
static uint32_t latent_addresses(const gh_model* m) { return m->family == GH_FAMILY_REGRESSION ? 3u : 1u; }

extern "C" int gh_pf_rejuvenate(gh_pf* pf, int n_moves, int64_t* accepted) {
  if (!pf) return set_err(GH_E_INVAL, "null pf");
  return gh_pf_mh_select(pf, latent_addresses(pf->m), n_moves, accepted);
}

extern "C" int gh_pf_mh_select(gh_pf* pf, uint32_t selection, int n_moves, int64_t* accepted) {
  if (!pf) return set_err(GH_E_INVAL, "null pf");
  if (n_moves < 0) return set_err(GH_E_INVAL, "gh_pf_rejuvenate: n_moves < 0");
  if (selection == 0 || (selection & ~latent_addresses(pf->m)) != 0)
    return set_err(GH_E_INVAL, "gh_pf_mh_select: selection 0x%x names no latent address of this step (valid: 0x%x)",
                   selection, latent_addresses(pf->m));
  if (pf->m->family == GH_FAMILY_REGRESSION && pf->t != 1)
    return set_err(GH_E_STATE, "gh_pf_mh_select: the regression is a static model (t = 1)");
  if (pf->resample_calls > 0)
    return set_err(GH_E_STATE, "gh_pf_rejuvenate: call after a step and before maybe_resample");
  if (pf->cond) return set_err(GH_E_STATE, "gh_pf_rejuvenate: the distinguished particle of a conditional filter is fixed");
  if ((uint64_t)pf->rejuv_moves + (uint64_t)n_moves > kRejuvMaxMoves)
    return set_err(GH_E_INVAL, "gh_pf_rejuvenate: more than %u moves at one step", kRejuvMaxMoves);
  HIP_TRY(hipSetDevice(pf->ctx->device));
  if (!pf->acc_count) HIP_TRY(hipMalloc(&pf->acc_count, sizeof(unsigned long long)));
  HIP_TRY(hipMemsetAsync(pf->acc_count, 0, sizeof(unsigned long long), pf->s));
  const int t = pf->t;
  if (n_moves > 0 && pf->n > 0) {
    RejuvArgs a{};
    if (t >= 2) {
      a.xprev = slot_x(pf, t - 1);
      a.anc = anc_for_step(pf, t);
      a.res = pf->res_hist + t;
      a.remote = pf->rows_recv;
      a.ld_remote = pf->D + 1;
    }
    a.x = slot_x(pf, t);
    a.n = pf->n;
    a.lo = pf->lo;
    a.seed = pf->seed;
    a.t = (uint32_t)t;
    a.move0 = pf->rejuv_moves;
    a.select = selection;
    a.n_moves = n_moves;
    a.accepted = pf->acc_count;
    CHECK(launch_rejuv(pf, a, t == 1));
  }
  pf->rejuv_moves += (uint32_t)n_moves;
  if (accepted) {
    unsigned long long h = 0;
    CHECK(d2h(pf, &h, pf->acc_count, sizeof h));
    *accepted = (int64_t)h;
  }
  return GH_OK;
}

// mh(trace, drift, (sd,)) on every particle (gh_rejuv.h k_mh_drift)
extern "C" int gh_pf_mh_drift(gh_pf* pf, uint32_t selection, const double* sd, int n_moves, int64_t* accepted) {
  if (!pf || !sd) return set_err(GH_E_INVAL, "gh_pf_mh_drift: null argument");
  if (n_moves < 0) return set_err(GH_E_INVAL, "gh_pf_mh_drift: n_moves < 0");
  if (pf->m->family == GH_FAMILY_HMM ||
      (pf->m->family == GH_FAMILY_SLOTS &&
       (pf->m->slots.lat == SLOT_LAT_CATEGORICAL || pf->m->slots.lat == SLOT_LAT_SWITCHING)))
    return set_err(GH_E_INVAL, "gh_pf_mh_drift: a Gaussian drift needs a continuous latent (not a categorical one)");
  if (selection == 0 || (selection & ~latent_addresses(pf->m)) != 0)
    return set_err(GH_E_INVAL, "gh_pf_mh_drift: selection 0x%x names no latent address of this step (valid: 0x%x)",
                   selection, latent_addresses(pf->m));
  if (pf->m->family == GH_FAMILY_REGRESSION && pf->t != 1)
    return set_err(GH_E_STATE, "gh_pf_mh_drift: the regression is a static model (t = 1)");
  if (pf->resample_calls > 0) return set_err(GH_E_STATE, "gh_pf_mh_drift: call after a step and before maybe_resample");
  if (pf->cond) return set_err(GH_E_STATE, "gh_pf_mh_drift: the distinguished particle of a conditional filter is fixed");
  if ((uint64_t)pf->rejuv_moves + (uint64_t)n_moves > kRejuvMaxMoves)
    return set_err(GH_E_INVAL, "gh_pf_mh_drift: more than %u moves at one step", kRejuvMaxMoves);
  const int D = pf->D;
  DriftSd dsd{};
  for (int k = 0; k < D; ++k) {
    // the regression's components are its addresses; an Unfold latent drifts as a whole
    const bool sel = pf->m->family == GH_FAMILY_REGRESSION ? ((selection >> k) & 1u) != 0 : true;
    if (sel && !(sd[k] > 0.0 && sd[k] < INFINITY))
      return set_err(GH_E_INVAL, "gh_pf_mh_drift: sd[%d] = %g must be finite and > 0", k, sd[k]);
    dsd.v[k] = sel ? sd[k] : 0.0;
  }
  HIP_TRY(hipSetDevice(pf->ctx->device));
  if (!pf->acc_count) HIP_TRY(hipMalloc(&pf->acc_count, sizeof(unsigned long long)));
  HIP_TRY(hipMemsetAsync(pf->acc_count, 0, sizeof(unsigned long long), pf->s));
  const int t = pf->t;
  if (n_moves > 0 && pf->n > 0) {
    RejuvArgs a{};
    if (t >= 2) {
      a.xprev = slot_x(pf, t - 1);
      a.anc = anc_for_step(pf, t);
      a.res = pf->res_hist + t;
      a.remote = pf->rows_recv;
      a.ld_remote = pf->D + 1;
    }
    a.x = slot_x(pf, t);
    a.n = pf->n;
    a.lo = pf->lo;
    a.seed = pf->seed;
    a.t = (uint32_t)t;
    a.move0 = pf->rejuv_moves;
    a.select = selection;
    a.n_moves = n_moves;
    a.accepted = pf->acc_count;
    const dim3 grid((unsigned)pf->nb_step), block(kBlock);
    CHECK(with_model(pf->m, [&](auto model, const auto& p) {
      using M = decltype(model);
      if constexpr (!std::is_same<M, HMMModel>::value) {
        if (t == 1)
          hipLaunchKernelGGL((k_mh_drift<M, true>), grid, block, 0, pf->s, (const double*)pf->m->dparams, p,
                             pf->last_obs, a, dsd);
        else
          hipLaunchKernelGGL((k_mh_drift<M, false>), grid, block, 0, pf->s, (const double*)pf->m->dparams, p,
                             pf->last_obs, a, dsd);
      }
    }));
    HIP_TRY(hipGetLastError());
  }
  pf->rejuv_moves += (uint32_t)n_moves;
  if (accepted) {
    unsigned long long h = 0;
    CHECK(d2h(pf, &h, pf->acc_count, sizeof h));
    *accepted = (int64_t)h;
  }
  return GH_OK;
}

extern "C" int gh_pf_get_ess_history(gh_pf* pf, int max_steps, double* ess, int32_t* did) {
  if (!pf) return set_err(GH_E_INVAL, "null pf");
  const int T = pf->t < max_steps ? pf->t : max_steps;
  std::vector<double> e(pf->cap + 2);
  std::vector<int32_t> r(pf->cap + 2);
  CHECK(d2h(pf, e.data(), pf->ess_hist, sizeof(double) * (pf->cap + 2)));
  CHECK(d2h(pf, r.data(), pf->res_hist, sizeof(int32_t) * (pf->cap + 2)));
  // ess[s-1]: ESS measured by maybe_resample after step s; did[s-1]: resampled then
  for (int s = 1; s <= T; ++s) {
    if (ess) ess[s - 1] = e[s];
    if (did) did[s - 1] = r[s + 1];
  }
  return GH_OK;
}

extern "C" int gh_pf_sample_unweighted(gh_pf* pf, int64_t ns, uint64_t seed, int64_t* idx) {
  if (!pf || !idx || ns < 0) return set_err(GH_E_INVAL, "bad argument");
  if (ns == 0) return GH_OK;
  const int64_t n = pf->n;
  const bool multi = mr(pf->ctx);
  const int R = pf->ctx->world;
  CHECK(ensure_stats(pf));
  hipLaunchKernelGGL(k_prep_sample, dim3(1), dim3(64), 0, pf->s, pf->dev, pf->stats_all, R, flags_live(pf));
  GateArgs g;
  g.gate = &pf->dev->one;
  g.M = &pf->dev->sM;
  g.zero_w = &pf->dev->spend;
  g.shift = quant_shift((uint64_t)pf->n_global);
  CHECK(materialize_marks(pf));
  DecideArgs d{};
  hipLaunchKernelGGL(k_qsum, dim3((unsigned)pf->nb_scan), dim3(kBlock), 0, pf->s, pf->logw, n, g, pf->bsum, 0, d,
                     pf->dev);
  if (multi) {  // the global integer CDF: every rank's total (one word each)
    hipLaunchKernelGGL(k_rank_total, dim3(1), dim3(kBlock), 0, pf->s, g.gate, pf->bsum, pf->nb_scan, pf->dev);
    CHECK(comm_allgather(pf->ctx, &pf->dev->local, pf->totals_all, sizeof(uint64_t), pf->s, &pf->dev->error));
  }
  MarkArgs mk{};
  CdfArgs ca{};
  ca.bsum = pf->bsum;
  ca.nb = pf->nb_scan;
  ca.totals = multi ? pf->totals_all : nullptr;
  ca.R = R;
  ca.rank = pf->ctx->rank;
  ca.n_global = pf->n_global;
  ca.seed = seed;
  ca.t = (uint32_t)pf->t;
  ca.stream = STREAM_SAMPLE;
  hipLaunchKernelGGL(k_cdf, dim3((unsigned)pf->nb_scan), dim3(kBlock), 0, pf->s, pf->logw, n, g, ca, pf->dev, pf->C,
                     mk);
  int32_t* dout = nullptr;
  HIP_TRY(hipMalloc(&dout, sizeof(int32_t) * (ns + 1)));
  SearchArgs sa{};
  sa.C = pf->C;
  sa.n_cdf = n;
  sa.n_slots = ns;
  sa.slot_lo = 0;
  sa.n_global = pf->n_global;
  sa.seed = seed;
  sa.t = (uint32_t)pf->t;
  sa.mode = SEARCH_SAMPLE;
  sa.anc_old = nullptr;
  sa.anc_out = dout;
  sa.own_only = multi ? 1 : 0;  // each target is searched by the rank whose CDF range holds it
  hipLaunchKernelGGL(k_search, dim3((unsigned)((ns + kBlock - 1) / kBlock)), dim3(kBlock), 0, pf->s, sa, g,
                     pf->dev);
  HIP_TRY(hipGetLastError());
  if (!multi) {
    std::vector<int32_t> h(ns);
    HIP_TRY(hipMemcpyAsync(h.data(), dout, sizeof(int32_t) * ns, hipMemcpyDeviceToHost, pf->s));
    HIP_TRY(hipStreamSynchronize(pf->s));
    hipFree(dout);
    for (int64_t i = 0; i < ns; ++i) idx[i] = h[i];
    return GH_OK;
  }
  // every rank's answers (local index, -1 where another rank's range held the
  // target), all-gathered: each sample is the global id one rank found
  const size_t bytes = (sizeof(int32_t) * (size_t)ns + 7) & ~(size_t)7;
  DBuf all;
  int rc = dalloc(all, bytes * (size_t)R);
  if (!rc) rc = bulk_allgather(pf->ctx, dout, all.p, bytes, pf->s);
  hipFree(dout);
  CHECK(rc);
  std::vector<int32_t> h(bytes / sizeof(int32_t) * (size_t)R);
  HIP_TRY(hipMemcpy(h.data(), all.p, bytes * (size_t)R, hipMemcpyDeviceToHost));
  DevScalars hs;
  CHECK(d2h(pf, &hs, pf->dev, sizeof hs));
  if (hs.error) return dev_fail(hs.error);
  const size_t stride = bytes / sizeof(int32_t);
  for (int64_t i = 0; i < ns; ++i) {
    idx[i] = -1;
    for (int r = 0; r < R; ++r)
      if (h[(size_t)r * stride + i] >= 0) {
        idx[i] = split_lo(pf->n_global, r, R) + h[(size_t)r * stride + i];
        break;
      }
    if (idx[i] < 0) return set_err(GH_E_STATE, "sample_unweighted: sample %lld found by no rank", (long long)i);
  }
  return GH_OK;
}

extern "C" int gh_pf_kernel_time(gh_pf* pf, double* avg_ms, int64_t* nl, int reset) {
  if (!pf) return set_err(GH_E_INVAL, "null pf");
  HIP_TRY(hipStreamSynchronize(pf->s));
  for (size_t i = 0; i + 1 < pf->ev_used; i += 2) {
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, pf->ev[i], pf->ev[i + 1]));
    pf->ev_ms += ms;
    pf->ev_count += 1;
  }
  pf->ev_used = 0;
  if (avg_ms) *avg_ms = pf->ev_count ? pf->ev_ms / (double)pf->ev_count : 0.0;
  if (nl) *nl = pf->ev_count;
  if (reset) {
    pf->ev_ms = 0.0;
    pf->ev_count = 0;
  }
  return GH_OK;
}

// -------------------------------------------------- multi-rank exchange
// Systematic resampling over R ranks.  Global slot j takes the
// first particle whose global inclusive CDF exceeds T_j = floor((j S + o)/N);
// T is monotone, so the slots rank r's particles cover form one contiguous
// range [count(base_r), count(base_r + total_r)) with
//   count(X) = #{j : T_j < X} = clamp(ceil((X N - o) / S), 0, N).
// Intersecting those ranges with the slot blocks each rank owns gives every
// rank the same plan: which slot range it sends to / receives from each peer.
static int64_t sys_count_host(uint64_t X, uint64_t N, uint64_t S, uint64_t o) {
  if (X == 0) return 0;
  if (X >= S) return (int64_t)N;
  const __int128 num = (__int128)X * N - (__int128)o;
  if (num <= 0) return 0;
  const __int128 j = (num + S - 1) / S;
  return j > (__int128)N ? (int64_t)N : (int64_t)j;
}

static void sys_plan(int64_t N, int R, int q, const uint64_t* totals, uint64_t o, int64_t* send_lo,
                     int64_t* send_hi, int64_t* recv_lo, int64_t* recv_hi) {
  uint64_t S = 0;
  for (int r = 0; r < R; ++r) S += totals[r];
  std::vector<int64_t> cov_lo(R), cov_hi(R);
  uint64_t base = 0;
  for (int r = 0; r < R; ++r) {
    cov_lo[r] = sys_count_host(base, (uint64_t)N, S, o);
    base += totals[r];
    cov_hi[r] = sys_count_host(base, (uint64_t)N, S, o);
  }
  const int64_t my_lo = split_lo(N, q, R), my_hi = split_lo(N, q + 1, R);
  for (int r = 0; r < R; ++r) {
    const int64_t dlo = split_lo(N, r, R), dhi = split_lo(N, r + 1, R);
    int64_t a = cov_lo[q] > dlo ? cov_lo[q] : dlo, b = cov_hi[q] < dhi ? cov_hi[q] : dhi;
    send_lo[r] = a;
    send_hi[r] = b > a ? b : a;
    a = cov_lo[r] > my_lo ? cov_lo[r] : my_lo;
    b = cov_hi[r] < my_hi ? cov_hi[r] : my_hi;
    recv_lo[r] = a;
    recv_hi[r] = b > a ? b : a;
  }
}

extern "C" int gh_sys_plan(int64_t n_global, int world, int rank, const uint64_t* totals, uint64_t offset,
                           int64_t* send_lo, int64_t* send_hi, int64_t* recv_lo, int64_t* recv_hi) {
  if (n_global < 1 || world < 1 || rank < 0 || rank >= world || !totals || !send_lo || !send_hi || !recv_lo ||
      !recv_hi)
    return set_err(GH_E_INVAL, "gh_sys_plan: bad argument");
  uint64_t S = 0;
  for (int r = 0; r < world; ++r) S += totals[r];
  if (S == 0 || offset >= S) return set_err(GH_E_INVAL, "gh_sys_plan: offset must be < sum(totals) > 0");
  sys_plan(n_global, world, rank, totals, offset, send_lo, send_hi, recv_lo, recv_hi);
  return GH_OK;
}

// The message lists one rank posts for a resample with these totals (host
// arithmetic only; tests): peers and byte counts, sends then receives.
extern "C" int gh_debug_mark_bits(gh_pf* pf, int bits) {
  if (!pf) return set_err(GH_E_INVAL, "gh_debug_mark_bits: null filter");
  if (pf->marks_pending) return set_err(GH_E_STATE, "gh_debug_mark_bits: a resample's marks are pending");
  int need = 1;
  while (need < 31 && (1ll << need) < pf->n) ++need;
  pf->mark_bits = std::min(31, std::max(need, bits));
  HIP_TRY(hipMemsetAsync(pf->mark, 0, sizeof(uint32_t) * pf->n, pf->s));
  HIP_TRY(hipMemsetAsync(pf->cmark, 0, sizeof(uint32_t) * ((pf->n + 63) / 64), pf->s));
  pf->epoch = 0;
  return GH_OK;
}

extern "C" int gh_debug_set_ancestor(gh_pf* pf, int t, int64_t j, int32_t value) {
  if (!pf || t < 2 || t > pf->t || j < 0 || j >= pf->n) return set_err(GH_E_INVAL, "gh_debug_set_ancestor: bad argument");
  CHECK(materialize_marks(pf));
  HIP_TRY(hipMemcpyAsync(anc_for_step(pf, t) + j, &value, sizeof(int32_t), hipMemcpyHostToDevice, pf->s));
  HIP_TRY(hipStreamSynchronize(pf->s));
  return GH_OK;
}

extern "C" int gh_debug_count_window(gh_ctx* ctx, int log2_inv) {
  if (!ctx || log2_inv < 0 || log2_inv > 40) return set_err(GH_E_INVAL, "gh_debug_count_window: bad argument");
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_count_window_log2), &log2_inv, sizeof(int)));
  return GH_OK;
}

extern "C" int gh_debug_exchange_lists(int64_t n_global, int world, int rank, const uint64_t* totals, uint64_t offset,
                                       int D, int* n_send, int* send_peer, uint64_t* send_bytes, int* n_recv,
                                       int* recv_peer, uint64_t* recv_bytes) {
  if (world < 1 || world > kMaxRanks || D < 1 || !n_send || !n_recv) return set_err(GH_E_INVAL, "bad argument");
  std::vector<int64_t> slo(world), shi(world), rlo(world), rhi(world);
  CHECK(gh_sys_plan(n_global, world, rank, totals, offset, slo.data(), shi.data(), rlo.data(), rhi.data()));
  std::vector<CommMsg> sends, recvs;
  exchange_lists(world, rank, D, slo.data(), shi.data(), rlo.data(), rhi.data(), nullptr, nullptr, &sends, &recvs);
  *n_send = (int)sends.size();
  *n_recv = (int)recvs.size();
  for (size_t k = 0; k < sends.size(); ++k) {
    send_peer[k] = sends[k].peer;
    send_bytes[k] = sends[k].bytes;
  }
  for (size_t k = 0; k < recvs.size(); ++k) {
    recv_peer[k] = recvs[k].peer;
    recv_bytes[k] = recvs[k].bytes;
  }
  return GH_OK;
}

static int exchange_states(gh_pf* pf, int32_t* anc_out) {
  if (pf->ctx->peer && !pf->ctx->hc.sendrecv)
    return set_err(GH_E_STATE, "peer transport: this resample needs the fused multi-rank kernels (systematic, "
                               "at most %d ranks, co-resident tiles) or a bootstrap with sendrecv", kMaxRanks);
  gh_ctx* c = pf->ctx;
  const int R = c->world, q = c->rank;
  const int D = pf->D;
  const int t = pf->t;
  // the plan needs the decision and the totals on the host: one round trip
  DevScalars h;
  std::vector<uint64_t> tot(R);
  HIP_TRY(hipMemcpyAsync(&h, pf->dev, sizeof h, hipMemcpyDeviceToHost, pf->s));
  HIP_TRY(hipMemcpyAsync(tot.data(), pf->totals_all, sizeof(uint64_t) * R, hipMemcpyDeviceToHost, pf->s));
  HIP_TRY(hipStreamSynchronize(pf->s));
  if (h.error) return dev_fail(h.error);
  if (!h.fire) return GH_OK;
  uint64_t S = 0;
  for (int r = 0; r < R; ++r) S += tot[r];
  const u32x4 w = rng_block(pf->seed, ~0ull, (uint32_t)t, STREAM_RESAMPLE, 0);
  const uint64_t o = scale_u53(u53_bits(w.x, w.y), S);
  std::vector<int64_t> slo(R), shi(R), rlo(R), rhi(R);
  sys_plan(pf->n_global, R, q, tot.data(), o, slo.data(), shi.data(), rlo.data(), rhi.data());
  // rows to send, packed by destination rank
  int64_t n_send = 0;
  for (int r = 0; r < R; ++r)
    if (r != q) n_send += shi[r] - slo[r];
  if (n_send > pf->send_cap) {
    HIP_TRY(hipStreamSynchronize(pf->s));
    hipFree(pf->rows_send);
    hipFree(pf->xanc);
    pf->rows_send = nullptr;
    pf->xanc = nullptr;
    pf->send_cap = 0;
    int64_t cap = n_send + n_send / 4 + 64;
    if (hipMalloc(&pf->rows_send, sizeof(double) * (D + 1) * cap) != hipSuccess ||
        hipMalloc(&pf->xanc, sizeof(int32_t) * cap) != hipSuccess)
      return set_err(GH_E_NOMEM, "exchange: cannot allocate %lld send rows", (long long)cap);
    pf->send_cap = cap;
  }
  GateArgs g;
  g.gate = &pf->dev->fire;
  g.M = &pf->dev->M;
  g.zero_w = &pf->dev->pending;
  g.shift = quant_shift((uint64_t)pf->n_global);
  SearchArgs sa{};
  sa.C = pf->C;
  sa.n_cdf = pf->n;
  sa.n_global = pf->n_global;
  sa.seed = pf->seed;
  sa.t = (uint32_t)t;
  sa.mode = SEARCH_SYSTEMATIC;
  sa.anc_old = nullptr;
  std::vector<CommMsg> sends, recvs;
  const size_t row_bytes = sizeof(double) * (D + 1);
  int64_t soff = 0;
  for (int r = 0; r < R; ++r) {
    const int64_t len = shi[r] - slo[r];
    if (len <= 0) continue;
    sa.slot_lo = slo[r];
    sa.n_slots = len;
    sa.anc_out = r == q ? anc_out + (slo[r] - pf->lo) : pf->xanc + soff;
    hipLaunchKernelGGL(k_search, dim3((unsigned)((len + kBlock - 1) / kBlock)), dim3(kBlock), 0, pf->s, sa, g,
                       pf->dev);
    if (r != q) {
      sends.push_back({r, pf->rows_send + soff * (D + 1), (size_t)len * row_bytes});
      soff += len;
    }
  }
  if (n_send > 0)
    hipLaunchKernelGGL(k_pack_rows, dim3((unsigned)((n_send + kBlock - 1) / kBlock)), dim3(kBlock), 0, pf->s,
                       pf->xanc, n_send, slot_x(pf, t), D, pf->lo, pf->rows_send);
  int64_t roff = 0;
  for (int r = 0; r < R; ++r) {
    const int64_t len = rhi[r] - rlo[r];
    if (r == q || len <= 0) continue;
    recvs.push_back({r, pf->rows_recv + roff * (D + 1), (size_t)len * row_bytes});
    hipLaunchKernelGGL(k_assign_remote, dim3((unsigned)((len + kBlock - 1) / kBlock)), dim3(kBlock), 0, pf->s,
                       anc_out + (rlo[r] - pf->lo), len, roff);
    roff += len;
  }
  HIP_TRY(hipGetLastError());
  CHECK(comm_exchange(c, sends, recvs, pf->s));
  if (pf->n > 0)
    hipLaunchKernelGGL(k_global_parents, dim3((unsigned)pf->nb_step), dim3(kBlock), 0, pf->s, anc_out, pf->n,
                       pf->lo, pf->rows_recv, D, pf->gparent);
  HIP_TRY(hipGetLastError());
  // the received rows, kept as the next step's genealogy record (as the split
  // step's part 2 keeps them on the fused path)
  if (pf->opts.record_history && roff > 0) {
    double* dst = nullptr;
    CHECK(rhist_reserve(pf, t + 1, roff, &dst));
    if (dst) HIP_TRY(hipMemcpyAsync(dst, pf->rows_recv, row_bytes * (size_t)roff, hipMemcpyDeviceToDevice, pf->s));
  }
  return GH_OK;
}

// Multinomial resampling on R ranks.  Every rank evaluates the
// targets of all N slots (one Philox block each) and their keys; the rank
// holding a slot's target sends that slot's ancestor row to the slot's owner,
// both ranks ordering those rows by slot, so no index travels.  One host round
// trip (the decision, the totals and the per-block key counts), one grouped
// send/recv of rows.  The same ancestors as k_search on one rank.
static int exchange_states_mn(gh_pf* pf, int32_t* anc_out) {
  gh_ctx* c = pf->ctx;
  const int R = c->world, q = c->rank;
  const int D = pf->D;
  const int t = pf->t;
  const int64_t N = pf->n_global;
  DevScalars h;
  std::vector<uint64_t> tot(R);
  HIP_TRY(hipMemcpyAsync(&h, pf->dev, sizeof h, hipMemcpyDeviceToHost, pf->s));
  HIP_TRY(hipMemcpyAsync(tot.data(), pf->totals_all, sizeof(uint64_t) * R, hipMemcpyDeviceToHost, pf->s));
  HIP_TRY(hipStreamSynchronize(pf->s));
  if (h.error) return dev_fail(h.error);
  if (!h.fire) return GH_OK;
  // the slot ranges (= the particle ranges) and their blocks
  std::vector<int64_t> lo(R + 1), boff0(R + 1);
  for (int r = 0; r <= R; ++r) lo[r] = split_lo(N, r, R);
  boff0[0] = 0;
  for (int r = 0; r < R; ++r) boff0[r + 1] = boff0[r] + (lo[r + 1] - lo[r] + kBlock - 1) / kBlock;
  const int64_t nb = boff0[R];
  if (!pf->mn_key) {
    if (hipMalloc(&pf->mn_key, sizeof(int32_t) * N) != hipSuccess || hipMalloc(&pf->mn_pos, sizeof(int32_t) * N) != hipSuccess ||
        hipMalloc(&pf->mn_anc, sizeof(int32_t) * N) != hipSuccess ||
        hipMalloc(&pf->mn_bcnt, sizeof(int32_t) * nb * R) != hipSuccess ||
        hipMalloc(&pf->mn_boff, sizeof(int32_t) * nb * R) != hipSuccess)
      return set_err(GH_E_NOMEM, "multinomial exchange: %lld slots", (long long)N);
  }
  const int* gate = &pf->dev->fire;
  for (int r = 0; r < R; ++r) {
    const int64_t n_r = lo[r + 1] - lo[r];
    if (n_r <= 0) continue;
    MnArgs m{};
    m.slot_lo = lo[r];
    m.n_slots = n_r;
    m.seed = pf->seed;
    m.t = (uint32_t)t;
    m.totals = pf->totals_all;
    m.R = R;
    m.key = pf->mn_key + lo[r];
    m.bcnt = pf->mn_bcnt + boff0[r] * R;
    hipLaunchKernelGGL(k_mn_keys, dim3((unsigned)((n_r + kBlock - 1) / kBlock)), dim3(kBlock), 0, pf->s, m, gate,
                       (const DevScalars*)pf->dev);
  }
  HIP_TRY(hipGetLastError());
  std::vector<int32_t> cnt((size_t)(nb * R)), off((size_t)(nb * R));
  HIP_TRY(hipMemcpyAsync(cnt.data(), pf->mn_bcnt, sizeof(int32_t) * nb * R, hipMemcpyDeviceToHost, pf->s));
  HIP_TRY(hipStreamSynchronize(pf->s));
  // per range and key: exclusive scan over the range's blocks; the totals are
  // the rows rank q sends to range r's owner (key q) and receives (range q)
  std::vector<int64_t> kcount((size_t)R * R, 0);  // [range][key]
  for (int r = 0; r < R; ++r)
    for (int k = 0; k < R; ++k) {
      int64_t run = 0;
      for (int64_t b = boff0[r]; b < boff0[r + 1]; ++b) {
        off[(size_t)(b * R + k)] = (int32_t)run;
        run += cnt[(size_t)(b * R + k)];
      }
      kcount[(size_t)r * R + k] = run;
    }
  HIP_TRY(hipMemcpyAsync(pf->mn_boff, off.data(), sizeof(int32_t) * nb * R, hipMemcpyHostToDevice, pf->s));
  GateArgs g;
  g.gate = &pf->dev->fire;
  g.M = &pf->dev->M;
  g.zero_w = &pf->dev->pending;
  g.shift = quant_shift((uint64_t)N);
  SearchArgs sa{};
  sa.C = pf->C;
  sa.n_cdf = pf->n;
  sa.n_global = N;
  sa.seed = pf->seed;
  sa.t = (uint32_t)t;
  sa.mode = SEARCH_MULTINOMIAL;
  sa.anc_old = nullptr;
  sa.own_only = 1;
  int64_t n_send = 0;
  for (int r = 0; r < R; ++r)
    if (r != q) n_send += kcount[(size_t)r * R + q];
  if (n_send > pf->send_cap) {
    HIP_TRY(hipStreamSynchronize(pf->s));
    hipFree(pf->rows_send);
    hipFree(pf->xanc);
    pf->rows_send = nullptr;
    pf->xanc = nullptr;
    pf->send_cap = 0;
    const int64_t cap = n_send + n_send / 4 + 64;
    if (hipMalloc(&pf->rows_send, sizeof(double) * (D + 1) * cap) != hipSuccess ||
        hipMalloc(&pf->xanc, sizeof(int32_t) * cap) != hipSuccess)
      return set_err(GH_E_NOMEM, "exchange: cannot allocate %lld send rows", (long long)cap);
    pf->send_cap = cap;
  }
  std::vector<CommMsg> sends, recvs;
  const size_t row_bytes = sizeof(double) * (D + 1);
  int64_t soff = 0;
  for (int r = 0; r < R; ++r) {
    const int64_t n_r = lo[r + 1] - lo[r];
    if (n_r <= 0) continue;
    const unsigned grid = (unsigned)((n_r + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_mn_pos, dim3(grid), dim3(kBlock), 0, pf->s, (const int32_t*)pf->mn_key + lo[r], n_r,
                       (const int32_t*)pf->mn_boff + boff0[r] * R, R, pf->mn_pos + lo[r], gate);
    sa.slot_lo = lo[r];
    sa.n_slots = n_r;
    sa.anc_out = pf->mn_anc + lo[r];
    hipLaunchKernelGGL(k_search, dim3(grid), dim3(kBlock), 0, pf->s, sa, g, pf->dev);
    if (r == q) continue;
    const int64_t s_r = kcount[(size_t)r * R + q];
    if (s_r > 0) {
      hipLaunchKernelGGL(k_mn_send, dim3(grid), dim3(kBlock), 0, pf->s, (const int32_t*)pf->mn_anc + lo[r],
                         (const int32_t*)pf->mn_pos + lo[r], n_r, pf->xanc + soff, gate);
      sends.push_back({r, pf->rows_send + soff * (D + 1), (size_t)s_r * row_bytes});
      soff += s_r;
    }
  }
  if (n_send > 0)
    hipLaunchKernelGGL(k_pack_rows, dim3((unsigned)((n_send + kBlock - 1) / kBlock)), dim3(kBlock), 0, pf->s,
                       pf->xanc, n_send, slot_x(pf, t), D, pf->lo, pf->rows_send);
  MnRecvOff ro{};
  int64_t n_recv = 0;
  for (int k = 0; k < R; ++k) {
    ro.off[k] = (int32_t)n_recv;
    const int64_t c_k = kcount[(size_t)q * R + k];
    if (k == q || c_k <= 0) continue;
    recvs.push_back({k, pf->rows_recv + n_recv * (D + 1), (size_t)c_k * row_bytes});
    n_recv += c_k;
  }
  if (pf->n > 0)
    hipLaunchKernelGGL(k_mn_recv, dim3((unsigned)pf->nb_step), dim3(kBlock), 0, pf->s,
                       (const int32_t*)pf->mn_anc + pf->lo, (const int32_t*)pf->mn_key + pf->lo,
                       (const int32_t*)pf->mn_pos + pf->lo, pf->n, ro, anc_out, gate);
  // conditional SMC: the distinguished particle's parent is itself (smc.jl:139;
  // the row sent for slot 0, if any, goes unused)
  if (pf->cond && pf->lo == 0) HIP_TRY(hipMemsetAsync(anc_out, 0, sizeof(int32_t), pf->s));
  HIP_TRY(hipGetLastError());
  CHECK(comm_exchange(c, sends, recvs, pf->s));
  if (pf->n > 0)
    hipLaunchKernelGGL(k_global_parents, dim3((unsigned)pf->nb_step), dim3(kBlock), 0, pf->s, anc_out, pf->n,
                       pf->lo, pf->rows_recv, D, pf->gparent);
  HIP_TRY(hipGetLastError());
  // the received rows are the next step's parents on other ranks: kept as
  // that step's genealogy record (rows_recv is overwritten by the next resample)
  if (pf->opts.record_history && n_recv > 0) {
    double* dst = nullptr;
    CHECK(rhist_reserve(pf, t + 1, n_recv, &dst));
    if (dst)
      HIP_TRY(hipMemcpyAsync(dst, pf->rows_recv, row_bytes * (size_t)n_recv, hipMemcpyDeviceToDevice, pf->s));
  }
  return GH_OK;
}

// ------------------------------------------------------ importance sampling
extern "C" int gh_is_run(gh_model* m, const gh_obs* obs, int proposal, int64_t n, uint64_t seed,
                         double* lnw, double* states, double* lml) {
  if (!m || !lml) return set_err(GH_E_INVAL, "gh_is_run: null argument");
  gh_pf_opts o;
  gh_pf_opts_default(&o);
  o.record_history = 0;
  gh_pf* pf = nullptr;
  // importance_sampling = N independent generate() calls (importance.jl:20-33),
  // i.e. the PF's first step; the lml is logsumexp(w) - log N.
  CHECK(gh_pf_init(m, obs, proposal, n, seed, &o, &pf));
  int rc = gh_pf_log_ml_estimate(pf, lml);
  if (!rc && lnw) {
    rc = gh_pf_get_log_weights(pf, lnw);
    if (!rc) {
      // normalise: lnw - logsumexp(lnw) (importance.jl:29-31)
      const double L = *lml + gh_log((double)pf->n_global);
      for (int64_t i = 0; i < pf->n; ++i) lnw[i] -= L;
    }
  }
  if (!rc && states) rc = gh_pf_get_states(pf, states);
  gh_pf_destroy(pf);
  return rc;
}

// ------------------------------------------------------------------ PMMH
extern "C" int gh_pmmh_run(gh_ctx* ctx, int64_t chain0, int64_t n_chains, int n_inner, const double* ys, int T,
                           int n_iters, int iter0, uint64_t seed, int init, double* lvx, double* lvy, double* lml,
                           int32_t* accepts, double* hist, double* kernel_ms) {
  if (!ctx || !ys || !lvx || !lvy || !lml || !accepts || T < 1 || n_iters < 0 || n_chains < 0 || chain0 < 0)
    return set_err(GH_E_INVAL, "gh_pmmh_run: bad argument");
  if (n_inner < 64 || n_inner > kPmmhMaxInner || n_inner % 64)
    return set_err(GH_E_INVAL, "gh_pmmh_run: n_inner must be a multiple of 64 in 64..%d", kPmmhMaxInner);
  if (chain0 + n_chains > (1LL << 22))
    return set_err(GH_E_INVAL, "gh_pmmh_run: chain ids must stay below 2^22");
  if (iter0 < 0 || ((int64_t)iter0 + n_iters) * 4 + 1 >= (1LL << 32))
    return set_err(GH_E_INVAL, "gh_pmmh_run: too many iterations");
  if (n_chains == 0) return GH_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  std::vector<double> ct(T);
  for (int t = 1; t <= T; ++t) ct[t - 1] = 8.0 * gh_cos(1.2 * (double)t);
  const size_t nc = (size_t)n_chains;
  double *d_ys = nullptr, *d_ct = nullptr, *d_vx = nullptr, *d_vy = nullptr, *d_ml = nullptr, *d_hist = nullptr;
  int32_t* d_acc = nullptr;
  auto cleanup = [&]() {
    hipFree(d_ys); hipFree(d_ct); hipFree(d_vx); hipFree(d_vy); hipFree(d_ml); hipFree(d_acc); hipFree(d_hist);
  };
#define PM_ALLOC(p, bytes) \
  if (hipMalloc(&(p), (bytes)) != hipSuccess) { cleanup(); return set_err(GH_E_NOMEM, "gh_pmmh_run: %s", #p); }
  PM_ALLOC(d_ys, sizeof(double) * T);
  PM_ALLOC(d_ct, sizeof(double) * T);
  PM_ALLOC(d_vx, sizeof(double) * nc);
  PM_ALLOC(d_vy, sizeof(double) * nc);
  PM_ALLOC(d_ml, sizeof(double) * nc);
  PM_ALLOC(d_acc, sizeof(int32_t) * 4 * nc);
  if (hist) PM_ALLOC(d_hist, sizeof(double) * 2 * nc * (size_t)(n_iters > 0 ? n_iters : 1));
#undef PM_ALLOC
  int rc = GH_OK;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  do {
    if (hipMemcpyAsync(d_ys, ys, sizeof(double) * T, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_ct, ct.data(), sizeof(double) * T, hipMemcpyHostToDevice, s) != hipSuccess) {
      rc = set_err(GH_E_HIP, "gh_pmmh_run: upload");
      break;
    }
    if (!init &&
        (hipMemcpyAsync(d_vx, lvx, sizeof(double) * nc, hipMemcpyHostToDevice, s) != hipSuccess ||
         hipMemcpyAsync(d_vy, lvy, sizeof(double) * nc, hipMemcpyHostToDevice, s) != hipSuccess ||
         hipMemcpyAsync(d_ml, lml, sizeof(double) * nc, hipMemcpyHostToDevice, s) != hipSuccess)) {
      rc = set_err(GH_E_HIP, "gh_pmmh_run: upload state");
      break;
    }
    PmmhArgs a{};
    a.ys = d_ys;
    a.ct = d_ct;
    a.T = T;
    a.n_iters = n_iters;
    a.iter0 = iter0;
    a.seed = seed;
    a.chain0 = chain0;
    a.n_chains = n_chains;
    a.lvx = d_vx;
    a.lvy = d_vy;
    a.lml = d_ml;
    a.accepts = d_acc;
    a.hist = d_hist;
    a.init = init ? 1 : 0;
    if (kernel_ms) {
      hipEventCreateWithFlags(&e0, kTimingEventFlags);
      hipEventCreateWithFlags(&e1, kTimingEventFlags);
    }
    hipExtLaunchKernelGGL(k_pmmh, dim3((unsigned)n_chains), dim3((unsigned)n_inner), 0, s, e0, e1, 0, a);
    if (hipGetLastError() != hipSuccess) {
      rc = set_err(GH_E_HIP, "gh_pmmh_run: launch");
      break;
    }
    if (hipMemcpyAsync(lvx, d_vx, sizeof(double) * nc, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(lvy, d_vy, sizeof(double) * nc, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(lml, d_ml, sizeof(double) * nc, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(accepts, d_acc, sizeof(int32_t) * 4 * nc, hipMemcpyDeviceToHost, s) != hipSuccess ||
        (hist && hipMemcpyAsync(hist, d_hist, sizeof(double) * 2 * nc * n_iters, hipMemcpyDeviceToHost, s) !=
                     hipSuccess) ||
        hipStreamSynchronize(s) != hipSuccess) {
      rc = set_err(GH_E_HIP, "gh_pmmh_run: download");
      break;
    }
    if (kernel_ms) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      *kernel_ms = ms;
    }
  } while (0);
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  cleanup();
  return rc;
}

// ------------------------------------------------------------------ coal
// The model constants of k_coal (gh_coal.h) and the bucket table of event-scan
// start indices (any table is exact: coal_count corrects its start).
static void coal_consts(const double* events, int E, CoalArgs* a, std::vector<int32_t>* bucket) {
  a->E = E;
  a->T = events[E - 1];
  a->bscale = (double)kCoalBuckets / a->T;
  a->kb = gh_log(3.0) - gh_log(a->T);
  a->ktheta = gh_log(kCoalRate);
  a->lhalf = gh_log(0.5);
  bucket->assign(kCoalBuckets, 0);
  int j = 0;
  for (int b = 0; b < kCoalBuckets; ++b) {
    const double lo = (double)b / a->bscale;
    while (j < E && events[j] < lo) ++j;
    (*bucket)[b] = j;
  }
}

static size_t coal_lds_bytes(int E) { return sizeof(double) * (size_t)E + sizeof(int32_t) * kCoalBuckets; }

extern "C" int gh_coal_run(gh_ctx* ctx, int64_t chain0, int64_t n_chains, const double* events, int E, int n_iters,
                           int iter0, uint64_t seed, int init, double* state, int32_t* accepts, int32_t* khist,
                           double* kernel_ms) {
  if (!ctx || !events || !state || !accepts || E < 1 || E > kCoalMaxEvents || n_iters < 0 || iter0 < 0 ||
      n_chains < 0 || chain0 < 0)
    return set_err(GH_E_INVAL, "gh_coal_run: bad argument (events 1..%d)", kCoalMaxEvents);
  for (int i = 1; i < E; ++i)
    if (!(events[i] >= events[i - 1])) return set_err(GH_E_INVAL, "gh_coal_run: events must be sorted");
  if (!(events[E - 1] > 0.0)) return set_err(GH_E_INVAL, "gh_coal_run: the window [0, T] is empty");
  if (n_chains == 0) return GH_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  const size_t nc = (size_t)n_chains;
  double *d_ev = nullptr, *d_st = nullptr, *d_rows = nullptr;
  int32_t *d_acc = nullptr, *d_kh = nullptr, *d_bk = nullptr;
  auto cleanup = [&]() { hipFree(d_ev); hipFree(d_st); hipFree(d_rows); hipFree(d_acc); hipFree(d_kh); hipFree(d_bk); };
  const unsigned tgrid = (unsigned)((nc * kCoalW + 255) / 256);
  CoalArgs a{};
  std::vector<int32_t> bucket;
  coal_consts(events, E, &a, &bucket);
  if (hipMalloc(&d_ev, sizeof(double) * E) != hipSuccess || hipMalloc(&d_st, sizeof(double) * kCoalW * nc) != hipSuccess ||
      hipMalloc(&d_bk, sizeof(int32_t) * kCoalBuckets) != hipSuccess ||
      hipMalloc(&d_rows, sizeof(double) * kCoalW * nc) != hipSuccess ||
      hipMalloc(&d_acc, sizeof(int32_t) * 3 * nc) != hipSuccess ||
      (khist && n_iters > 0 && hipMalloc(&d_kh, sizeof(int32_t) * nc * n_iters) != hipSuccess)) {
    cleanup();
    return set_err(GH_E_NOMEM, "gh_coal_run: device buffers");
  }
  int rc = GH_OK;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  do {
    if (hipMemcpyAsync(d_ev, events, sizeof(double) * E, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_bk, bucket.data(), sizeof(int32_t) * kCoalBuckets, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemsetAsync(d_st, 0, sizeof(double) * kCoalW * nc, s) != hipSuccess ||
        (!init && hipMemcpyAsync(d_rows, state, sizeof(double) * kCoalW * nc, hipMemcpyHostToDevice, s) != hipSuccess)) {
      rc = set_err(GH_E_HIP, "gh_coal_run: upload");
      break;
    }
    if (!init) hipLaunchKernelGGL(k_coal_rows, dim3(tgrid), dim3(256), 0, s, d_st, (int64_t)nc, d_rows, (int64_t)nc, 1);
    a.events = d_ev;
    a.bucket = d_bk;
    a.chain0 = chain0;
    a.n_chains = n_chains;
    a.seed = seed;
    a.n_iters = n_iters;
    a.iter0 = iter0;
    a.init = init ? 1 : 0;
    a.state = d_st;
    a.ld = (int64_t)nc;
    a.accepts = d_acc;
    a.khist = d_kh;
    if (kernel_ms) {
      hipEventCreateWithFlags(&e0, kTimingEventFlags);
      hipEventCreateWithFlags(&e1, kTimingEventFlags);
    }
    hipExtLaunchKernelGGL(k_coal, dim3((unsigned)((nc + kCoalBlock - 1) / kCoalBlock)), dim3(kCoalBlock),
                          coal_lds_bytes(E), s, e0, e1, 0, a);
    if (hipGetLastError() != hipSuccess) {
      rc = set_err(GH_E_HIP, "gh_coal_run: launch");
      break;
    }
    hipLaunchKernelGGL(k_coal_rows, dim3(tgrid), dim3(256), 0, s, d_st, (int64_t)nc, d_rows, (int64_t)nc, 0);
    if (hipMemcpyAsync(state, d_rows, sizeof(double) * kCoalW * nc, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(accepts, d_acc, sizeof(int32_t) * 3 * nc, hipMemcpyDeviceToHost, s) != hipSuccess ||
        (d_kh && hipMemcpyAsync(khist, d_kh, sizeof(int32_t) * nc * n_iters, hipMemcpyDeviceToHost, s) != hipSuccess) ||
        hipStreamSynchronize(s) != hipSuccess) {
      rc = set_err(GH_E_HIP, "gh_coal_run: download");
      break;
    }
    if (kernel_ms) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      *kernel_ms = ms;
    }
  } while (0);
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  cleanup();
  return rc;
}

struct gh_coal {
  gh_ctx* ctx = nullptr;
  double* ev = nullptr;
  double* st = nullptr;     // SoA [kCoalW][n] rows
  int32_t* acc = nullptr;   // [n][3]
  int32_t* bk = nullptr;    // bucket table of the event scan
  CoalArgs consts{};        // model constants (coal_consts)
  int E = 0;
  double T = 0.0;
  int64_t chain0 = 0, n = 0;
  uint64_t seed = 0;
  int iters = 0;
  int simple = 0;           // 1: simple_mcmc_step (regenerate k as the third move)
  bool started = false;
  hipEvent_t e0 = nullptr, e1 = nullptr;
};

extern "C" int gh_coal_destroy(gh_coal* h) {
  if (!h) return GH_OK;
  hipSetDevice(h->ctx->device);
  hipStreamSynchronize(h->ctx->stream);
  hipFree(h->ev);
  hipFree(h->st);
  hipFree(h->acc);
  hipFree(h->bk);
  if (h->e0) hipEventDestroy(h->e0);
  if (h->e1) hipEventDestroy(h->e1);
  delete h;
  return GH_OK;
}

extern "C" int gh_coal_create(gh_ctx* ctx, int64_t chain0, int64_t n_chains, const double* events, int E,
                              uint64_t seed, gh_coal** out) {
  if (!ctx || !events || !out || E < 1 || E > kCoalMaxEvents || n_chains < 1 || chain0 < 0)
    return set_err(GH_E_INVAL, "gh_coal_create: bad argument (events 1..%d, n_chains >= 1)", kCoalMaxEvents);
  for (int i = 1; i < E; ++i)
    if (!(events[i] >= events[i - 1])) return set_err(GH_E_INVAL, "gh_coal_create: events must be sorted");
  if (!(events[E - 1] > 0.0)) return set_err(GH_E_INVAL, "gh_coal_create: the window [0, T] is empty");
  HIP_TRY(hipSetDevice(ctx->device));
  gh_coal* h = new gh_coal();
  h->ctx = ctx;
  h->E = E;
  h->T = events[E - 1];
  h->chain0 = chain0;
  h->n = n_chains;
  h->seed = seed;
  const size_t nc = (size_t)n_chains;
  std::vector<int32_t> bucket;
  coal_consts(events, E, &h->consts, &bucket);
  if (hipMalloc(&h->ev, sizeof(double) * E) != hipSuccess ||
      hipMalloc(&h->st, sizeof(double) * kCoalW * nc) != hipSuccess ||
      hipMalloc(&h->bk, sizeof(int32_t) * kCoalBuckets) != hipSuccess ||
      hipMalloc(&h->acc, sizeof(int32_t) * 3 * nc) != hipSuccess || hipEventCreateWithFlags(&h->e0, kTimingEventFlags) != hipSuccess ||
      hipEventCreateWithFlags(&h->e1, kTimingEventFlags) != hipSuccess) {
    gh_coal_destroy(h);
    return set_err(GH_E_NOMEM, "gh_coal_create: device buffers");
  }
  if (hipMemcpyAsync(h->ev, events, sizeof(double) * E, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
      hipMemcpyAsync(h->bk, bucket.data(), sizeof(int32_t) * kCoalBuckets, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
      hipMemsetAsync(h->st, 0, sizeof(double) * kCoalW * nc, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess) {
    gh_coal_destroy(h);
    return set_err(GH_E_HIP, "gh_coal_create: upload");
  }
  *out = h;
  return GH_OK;
}

// which MCMC kernel gh_coal_step applies: 0 = mcmc_step (rate, position,
// birth/death; coal.jl:329-336), 1 = simple_mcmc_step (rate, position,
// mh(trace, select(K)); coal.jl:338-345)
extern "C" int gh_coal_set_kernel(gh_coal* h, int kernel) {
  if (!h || kernel < 0 || kernel > 1) return set_err(GH_E_INVAL, "gh_coal_set_kernel: kernel 0 (mcmc_step) or 1 (simple_mcmc_step)");
  h->simple = kernel;
  return GH_OK;
}

extern "C" int gh_coal_step(gh_coal* h, int n_iters, int32_t* accepts, int32_t* khist, double* kernel_ms) {
  if (!h || n_iters < 0) return set_err(GH_E_INVAL, "gh_coal_step: bad argument");
  HIP_TRY(hipSetDevice(h->ctx->device));
  hipStream_t s = h->ctx->stream;
  const size_t nc = (size_t)h->n;
  int32_t* d_kh = nullptr;
  if (khist && n_iters > 0 && hipMalloc(&d_kh, sizeof(int32_t) * nc * n_iters) != hipSuccess)
    return set_err(GH_E_NOMEM, "gh_coal_step: k history");
  CoalArgs a = h->consts;
  a.events = h->ev;
  a.bucket = h->bk;
  a.chain0 = h->chain0;
  a.n_chains = h->n;
  a.seed = h->seed;
  a.n_iters = n_iters;
  a.iter0 = h->iters;
  a.init = h->started ? 0 : 1;
  a.state = h->st;
  a.ld = h->n;
  a.accepts = h->acc;
  a.khist = d_kh;
  a.simple = h->simple;
  hipExtLaunchKernelGGL(k_coal, dim3((unsigned)((nc + kCoalBlock - 1) / kCoalBlock)), dim3(kCoalBlock),
                        coal_lds_bytes(h->E), s, h->e0, h->e1, 0, a);
  int rc = GH_OK;
  if (hipGetLastError() != hipSuccess) rc = set_err(GH_E_HIP, "gh_coal_step: launch");
  if (!rc && accepts && hipMemcpyAsync(accepts, h->acc, sizeof(int32_t) * 3 * nc, hipMemcpyDeviceToHost, s) != hipSuccess)
    rc = set_err(GH_E_HIP, "gh_coal_step: accepts");
  if (!rc && d_kh && hipMemcpyAsync(khist, d_kh, sizeof(int32_t) * nc * n_iters, hipMemcpyDeviceToHost, s) != hipSuccess)
    rc = set_err(GH_E_HIP, "gh_coal_step: k history");
  if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = set_err(GH_E_HIP, "gh_coal_step: sync");
  if (!rc && kernel_ms) {
    float ms = 0.f;
    hipEventElapsedTime(&ms, h->e0, h->e1);
    *kernel_ms = ms;
  }
  hipFree(d_kh);
  if (!rc) {
    h->iters += n_iters;
    h->started = true;
  }
  return rc;
}

// resume the chains from given rows (a checkpoint, or states the prior rarely
// visits): the next gh_coal_step continues at iteration iter0 + 1
extern "C" int gh_coal_write_state(gh_coal* h, const double* state, int iter0) {
  if (!h || !state || iter0 < 0) return set_err(GH_E_INVAL, "gh_coal_write_state: bad argument");
  const size_t nc = (size_t)h->n;
  for (size_t c = 0; c < nc; ++c) {  // rows must keep the layout k_coal relies on
    const double* r = state + c * kCoalW;
    const double kd = r[0];
    if (!(kd >= 0.0 && kd <= (double)kCoalKMax) || kd != (double)(int)kd)
      return set_err(GH_E_INVAL, "gh_coal_write_state: chain %zu has k = %g (0..%d)", c, kd, kCoalKMax);
    const int k = (int)kd;
    for (int i = k; i < kCoalKMax; ++i)
      if (r[2 + i] != 0.0) return set_err(GH_E_INVAL, "gh_coal_write_state: chain %zu: change point %d past k is not 0", c, i + 1);
    for (int i = k + 1; i <= kCoalKMax; ++i)
      if (r[2 + kCoalKMax + i] != 0.0) return set_err(GH_E_INVAL, "gh_coal_write_state: chain %zu: rate %d past k+1 is not 0", c, i + 1);
  }
  HIP_TRY(hipSetDevice(h->ctx->device));
  double* rows = nullptr;
  if (hipMalloc(&rows, sizeof(double) * kCoalW * nc) != hipSuccess)
    return set_err(GH_E_NOMEM, "gh_coal_write_state: row buffer");
  int rc = GH_OK;
  if (hipMemcpyAsync(rows, state, sizeof(double) * kCoalW * nc, hipMemcpyHostToDevice, h->ctx->stream) != hipSuccess)
    rc = set_err(GH_E_HIP, "gh_coal_write_state: upload");
  if (!rc)
    hipLaunchKernelGGL(k_coal_rows, dim3((unsigned)((nc * kCoalW + 255) / 256)), dim3(256), 0, h->ctx->stream, h->st,
                       h->n, rows, h->n, 1);
  if (!rc && hipStreamSynchronize(h->ctx->stream) != hipSuccess) rc = set_err(GH_E_HIP, "gh_coal_write_state: sync");
  hipFree(rows);
  if (!rc) {
    h->iters = iter0;
    h->started = true;
  }
  return rc;
}

extern "C" int gh_coal_read_state(gh_coal* h, double* state) {
  if (!h || !state) return set_err(GH_E_INVAL, "gh_coal_read_state: null argument");
  HIP_TRY(hipSetDevice(h->ctx->device));
  const size_t nc = (size_t)h->n;
  double* rows = nullptr;
  if (hipMalloc(&rows, sizeof(double) * kCoalW * nc) != hipSuccess)
    return set_err(GH_E_NOMEM, "gh_coal_read_state: row buffer");
  hipLaunchKernelGGL(k_coal_rows, dim3((unsigned)((nc * kCoalW + 255) / 256)), dim3(256), 0, h->ctx->stream, h->st,
                     h->n, rows, h->n, 0);
  int rc = GH_OK;
  if (hipMemcpyAsync(state, rows, sizeof(double) * kCoalW * nc, hipMemcpyDeviceToHost, h->ctx->stream) != hipSuccess ||
      hipStreamSynchronize(h->ctx->stream) != hipSuccess)
    rc = set_err(GH_E_HIP, "gh_coal_read_state: download");
  hipFree(rows);
  return rc;
}

// ------------------------------------------------------------ self tests
extern "C" int gh_selftest_math(gh_ctx* ctx, int64_t n, const double* in, double* oe, double* ol,
                                double* os, double* od) {
  if (!ctx || n <= 0) return set_err(GH_E_INVAL, "bad argument");
  HIP_TRY(hipSetDevice(ctx->device));
  double* d = nullptr;
  HIP_TRY(hipMalloc(&d, sizeof(double) * n * 5));
  HIP_TRY(hipMemcpyAsync(d, in, sizeof(double) * n, hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(k_selftest_math, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     ctx->stream, n, d, d + n, d + 2 * n, d + 3 * n, d + 4 * n);
  HIP_TRY(hipGetLastError());
  double* outs[4] = {oe, ol, os, od};
  for (int i = 0; i < 4; ++i)
    if (outs[i])
      HIP_TRY(hipMemcpyAsync(outs[i], d + (i + 1) * n, sizeof(double) * n, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  hipFree(d);
  return GH_OK;
}

extern "C" int gh_selftest_boxmuller(gh_ctx* ctx, int64_t n, const uint32_t* words, double* out) {
  if (!ctx || n < 0 || (n && (!words || !out))) return set_err(GH_E_INVAL, "gh_selftest_boxmuller: bad argument");
  if (n == 0) return GH_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  uint32_t* dw = nullptr;
  double* dout = nullptr;
  if (hipMalloc(&dw, sizeof(uint32_t) * 3 * n) != hipSuccess || hipMalloc(&dout, sizeof(double) * 4 * n) != hipSuccess) {
    hipFree(dw);
    return set_err(GH_E_NOMEM, "gh_selftest_boxmuller");
  }
  int rc = GH_OK;
  if (hipMemcpyAsync(dw, words, sizeof(uint32_t) * 3 * n, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
    rc = set_err(GH_E_HIP, "copy");
  if (!rc) {
    hipLaunchKernelGGL(k_selftest_boxmuller, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       ctx->stream, n, (const uint32_t*)dw, dout);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(out, dout, sizeof(double) * 4 * n, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess)
      rc = set_err(GH_E_HIP, "gh_selftest_boxmuller");
  }
  hipFree(dw);
  hipFree(dout);
  return rc;
}

extern "C" int gh_selftest_normals(gh_ctx* ctx, uint64_t seed, int64_t n, uint32_t step, uint32_t stream,
                                   int dim, double* out) {
  if (!ctx || n <= 0 || dim <= 0) return set_err(GH_E_INVAL, "bad argument");
  HIP_TRY(hipSetDevice(ctx->device));
  double* d = nullptr;
  HIP_TRY(hipMalloc(&d, sizeof(double) * n * dim));
  hipLaunchKernelGGL(k_selftest_normals, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                     ctx->stream, seed, n, step, stream, dim, d);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, d, sizeof(double) * n * dim, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  hipFree(d);
  return GH_OK;
}
