// p2p_probe.hip — groundwork for the peer-mailbox multi-rank design:
// can two processes exchange tagged words through IPC-mapped device memory,
// and what does one hand-off cost?  Two processes on the one GPU of a box
// (the pool gives no second device), so this measures the mechanism and its
// same-device latency, not xGMI.
//
//   p2p_probe RANK DIR ITERS     (run RANK 0 and 1 concurrently; DIR shared)
//
// Each rank allocates a 4 KiB mailbox, exports its IPC handle to DIR/h<rank>,
// opens the peer's, then ping-pongs ITERS times in two ways:
//   kernel: a one-wave kernel stores the tag into the peer's mailbox (system
//           scope) and polls its own until the peer's tag arrives (bounded);
//   stream: hipStreamWriteValue64 into the peer's mailbox, then
//           hipStreamWaitValue64 on its own (stream memory operations; the
//           host only enqueues).
// Prints one JSON line per rank: round-trip microseconds for each way.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "rank %d: %s failed: %s\n", rank, #x, hipGetErrorString(e_));   \
      return 2;                                                                        \
    }                                                                                  \
  } while (0)

// one lane: send tag t to the peer (slot 0 of its mailbox), wait for tag t in
// our own slot 0 (rank 1 answers); bounded spin, error flag on timeout
__global__ void k_pingpong(uint64_t* mine, uint64_t* peer, int rank, int iters, int* fail) {
  if (threadIdx.x != 0) return;
  for (int i = 1; i <= iters; ++i) {
    const uint64_t want = (uint64_t)i;
    if (rank == 0) __hip_atomic_store(peer, want, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned spins = 0;
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins == (1u << 26)) {
        *fail = i;
        return;
      }
    }
    if (rank == 1) __hip_atomic_store(peer, want, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static bool read_file(const std::string& path, void* buf, size_t n) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  const size_t got = fread(buf, 1, n, f);
  fclose(f);
  return got == n;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: p2p_probe RANK DIR ITERS\n");
    return 1;
  }
  const int rank = atoi(argv[1]);
  const std::string dir = argv[2];
  const int iters = atoi(argv[3]);
  CK(hipSetDevice(0));
  uint64_t* box = nullptr;
  CK(hipExtMallocWithFlags((void**)&box, 4096, hipDeviceMallocFinegrained));
  CK(hipMemset(box, 0, 4096));
  hipIpcMemHandle_t h;
  CK(hipIpcGetMemHandle(&h, box));
  {
    const std::string tmp = dir + "/h" + std::to_string(rank) + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    fwrite(&h, 1, sizeof h, f);
    fclose(f);
    rename(tmp.c_str(), (dir + "/h" + std::to_string(rank)).c_str());
  }
  hipIpcMemHandle_t hp;
  const std::string peer_path = dir + "/h" + std::to_string(1 - rank);
  const auto t0 = std::chrono::steady_clock::now();
  while (!read_file(peer_path, &hp, sizeof hp)) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
      fprintf(stderr, "rank %d: no peer handle\n", rank);
      return 3;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  uint64_t* peer = nullptr;
  CK(hipIpcOpenMemHandle((void**)&peer, hp, hipIpcMemLazyEnablePeerAccess));
  int* dfail = nullptr;
  CK(hipMalloc(&dfail, sizeof(int)));
  CK(hipMemset(dfail, 0, sizeof(int)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));

  // kernel ping-pong (slot 0)
  auto k0 = std::chrono::steady_clock::now();
  hipLaunchKernelGGL(k_pingpong, dim3(1), dim3(64), 0, s, box, peer, rank, iters, dfail);
  CK(hipStreamSynchronize(s));
  const double kus = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - k0).count();
  int fail = 0;
  CK(hipMemcpy(&fail, dfail, sizeof(int), hipMemcpyDeviceToHost));

  // stream write/wait-value ping-pong (slot 64)
  int can_wait = 0;
  CK(hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, 0));
  double sus = -1.0;
  if (can_wait && !fail) {  // (only once the kernel hand-off worked both ways)
    auto s0 = std::chrono::steady_clock::now();
    for (int i = 1; i <= iters; ++i) {
      if (rank == 0) CK(hipStreamWriteValue64(s, peer + 64, (uint64_t)i, 0));
      CK(hipStreamWaitValue64(s, box + 64, (uint64_t)i, hipStreamWaitValueGte, ~0ull));
      if (rank == 1) CK(hipStreamWriteValue64(s, peer + 64, (uint64_t)i, 0));
    }
    CK(hipStreamSynchronize(s));
    sus = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - s0).count();
  }
  printf("{\"rank\": %d, \"iters\": %d, \"kernel_roundtrip_us\": %.3f, \"kernel_fail_at\": %d, "
         "\"stream_wait_value\": %d, \"stream_roundtrip_us\": %.3f}\n",
         rank, iters, kus / iters, fail, can_wait, sus >= 0 ? sus / iters : -1.0);
  CK(hipIpcCloseMemHandle(peer));
  return fail ? 4 : 0;
}
