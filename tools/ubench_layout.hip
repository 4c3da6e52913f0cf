// State-layout microbenchmark (timing-only tool, not part of the product):
// the C2 step's HBM skeleton (range marks -> DPP prefix max -> gather of the
// ancestor's D=10 fp64 components -> store of the new state, logw, ancestor)
// in record_history mode (16 rotating slots: every launch writes fresh lines)
// under different placements of the D components of one particle.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_layout.hip -o tools/ubench_layout && tools/ubench_layout
//
//   soa_pP    column k of slot s at s*SP + k*(N+P) doubles (P = pad)
//   tile_B    [N/B][D][B] per slot: a B-particle tile's components contiguous
//   copy_*    the same without marks/gather (anc = j)
//   rd / wr   read-only / write-only halves of soa_p0
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

constexpr int D = 10;
constexpr int64_t N = 1 << 20;
constexpr int kBlock = 256;
constexpr int kSlots = 16;

template <int CTRL>
__device__ __forceinline__ uint64_t dppmv(uint64_t v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, 0xf, 0xf, false);
  return ((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo;
}
__device__ __forceinline__ uint64_t wave_incl_max_u64(uint64_t v) {
  const int lane = threadIdx.x & 63, rl = lane & 15;
  uint64_t t;
  t = dppmv<0x111>(v); if (rl >= 1 && t > v) v = t;
  t = dppmv<0x112>(v); if (rl >= 2 && t > v) v = t;
  t = dppmv<0x114>(v); if (rl >= 4 && t > v) v = t;
  t = dppmv<0x118>(v); if (rl >= 8 && t > v) v = t;
  t = dppmv<0x142>(v); if ((lane & 31) >= 16 && t > v) v = t;
  t = dppmv<0x143>(v); if (lane >= 32 && t > v) v = t;
  return v;
}

struct Args {
  const double* x;
  double* y;
  const uint64_t* mark;
  const uint64_t* carry;
  int32_t* anc;
  double* logw;
};

// index of component k of particle i
// pair-interleaved 64-particle tiles: components (2c, 2c+1) of a particle are
// one 16-byte word, [N/64][D/2][64][2]
__device__ __forceinline__ int64_t at_pair(int64_t i, int c) { return (i >> 6) * (64 * D) + c * 128 + (i & 63) * 2; }

template <bool GATHER>
__global__ __launch_bounds__(kBlock) void k_pair(Args a) {
  const int lane = threadIdx.x & 63;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t j = tile * 64 + lane;
  int64_t src = j;
  if (GATHER) {
    uint64_t v = a.mark[j];
    const uint64_t c = a.carry[tile];
    v = wave_incl_max_u64(v > c ? v : c);
    src = (int64_t)(uint32_t)v;
    a.anc[j] = (int32_t)src;
  }
  double2 x[D / 2];
#pragma unroll
  for (int c = 0; c < D / 2; ++c) x[c] = *reinterpret_cast<const double2*>(&a.x[at_pair(src, c)]);
#pragma unroll
  for (int c = 0; c < D / 2; ++c) {
    double2 y = x[c];
    y.x += 1.0;
    y.y += 1.0;
    *reinterpret_cast<double2*>(&a.y[at_pair(j, c)]) = y;
  }
  a.logw[j] = 1.0;
}
template <bool GATHER>
static void launch_pair(Args a);

template <int L, int P>
__device__ __forceinline__ int64_t at(int64_t i, int k) {
  if (L == 0) return (int64_t)k * (N + P) + i;                       // SoA, padded pitch
  return (i / L) * (D * L + P) + (int64_t)k * L + (i % L);           // tiles of L particles, P doubles of tile padding
}

template <int L, int P, bool GATHER, int MODE>  // MODE 0 rw, 1 read-only, 2 write-only
__global__ __launch_bounds__(kBlock) void k_skel(Args a) {
  const int lane = threadIdx.x & 63;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t j = tile * 64 + lane;
  int64_t src = j;
  if (GATHER) {
    uint64_t v = a.mark[j];
    const uint64_t c = a.carry[tile];
    v = wave_incl_max_u64(v > c ? v : c);
    src = (int64_t)(uint32_t)v;
    a.anc[j] = (int32_t)src;
  }
  double x[D];
  double s = 0.0;
  if (MODE != 2) {
#pragma unroll
    for (int k = 0; k < D; ++k) x[k] = a.x[at<L, P>(src, k)];
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) x[k] = (double)(k + j);
  }
  if (MODE != 1) {
#pragma unroll
    for (int k = 0; k < D; ++k) a.y[at<L, P>(j, k)] = x[k] + 1.0;
  } else {
#pragma unroll
    for (int k = 0; k < D; ++k) s += x[k];
  }
  a.logw[j] = s;
}

static double* g_hist = nullptr;
static int64_t g_slot_pitch = 0;
static int g_slot = 0;

template <int L, int P, bool GATHER, int MODE>
static void launch(Args a) {
  a.x = g_hist + (size_t)(g_slot % kSlots) * g_slot_pitch;
  a.y = g_hist + (size_t)((g_slot + 1) % kSlots) * g_slot_pitch;
  ++g_slot;
  hipLaunchKernelGGL((k_skel<L, P, GATHER, MODE>), dim3(N / kBlock), dim3(kBlock), 0, 0, a);
}

template <bool GATHER>
static void launch_pair(Args a) {
  a.x = g_hist + (size_t)(g_slot % kSlots) * g_slot_pitch;
  a.y = g_hist + (size_t)((g_slot + 1) % kSlots) * g_slot_pitch;
  ++g_slot;
  hipLaunchKernelGGL((k_pair<GATHER>), dim3(N / kBlock), dim3(kBlock), 0, 0, a);
}

int main() {
  std::vector<uint64_t> mark(N, 0), carry(N / 64, 0);
  {  // a systematic-resampling pattern: ancestors drawn from skewed weights
    srand(1);
    std::vector<double> w(N);
    for (auto& v : w) { const double u = (rand() + 0.5) / (RAND_MAX + 1.0); v = u * u * u * u; }
    double S = 0;
    for (double v : w) S += v;
    double cum = 0;
    int64_t i = 0;
    std::vector<int64_t> anc(N);
    for (int64_t j = 0; j < N; ++j) {
      const double tgt = (j + 0.37) * S / N;
      while (i < N - 1 && cum + w[i] <= tgt) cum += w[i++];
      anc[j] = i;
    }
    const uint64_t ep = 5ull << 32;
    for (int64_t j = 0; j < N; ++j)
      if (j == 0 || anc[j] != anc[j - 1]) mark[j] = ep | (uint64_t)anc[j];
    for (int64_t g = 0; g < N / 64; ++g) carry[g] = ep | (uint64_t)anc[g * 64];
  }
  Args a{};
  uint64_t *dm, *dc;
  hipMalloc(&dm, sizeof(uint64_t) * N);
  hipMalloc(&dc, sizeof(uint64_t) * N / 64);
  hipMalloc(&a.anc, sizeof(int32_t) * N);
  hipMalloc(&a.logw, sizeof(double) * N);
  hipMemcpy(dm, mark.data(), sizeof(uint64_t) * N, hipMemcpyHostToDevice);
  hipMemcpy(dc, carry.data(), sizeof(uint64_t) * N / 64, hipMemcpyHostToDevice);
  a.mark = dm;
  a.carry = dc;
  constexpr int64_t kMaxPad = 8192;
  g_slot_pitch = (int64_t)D * (N + kMaxPad) + (N / 32) * 256 + 4096;  // slots never alias, fixed pitch for every variant
  hipMalloc(&g_hist, sizeof(double) * g_slot_pitch * kSlots);
  hipMemset(g_hist, 0, sizeof(double) * g_slot_pitch * kSlots);
  const double bytes = (double)N * (16.0 * D + 8.0 + 8.0 + 4.0);
  struct V {
    const char* name;
    double bytes;
    void (*f)(Args);
  } vs[] = {
      {"soa_p0", bytes, launch<0, 0, true, 0>},
      {"soa_p512", bytes, launch<0, 512, true, 0>},
      {"tile_64", bytes, launch<64, 0, true, 0>},
      {"pair_64", bytes, launch_pair<true>},
      {"pair_copy", (double)N * (16.0 * D + 8.0), launch_pair<false>},
      {"tile_256", bytes, launch<256, 0, true, 0>},
      {"tile_32", bytes, launch<32, 0, true, 0>},
      {"tile_128", bytes, launch<128, 0, true, 0>},
      {"copy_p0", (double)N * (16.0 * D + 8.0), launch<0, 0, false, 0>},
      {"copy_t256", (double)N * (16.0 * D + 8.0), launch<256, 0, false, 0>},
      {"copy_t64", (double)N * (16.0 * D + 8.0), launch<64, 0, false, 0>},
      {"rd_t64", (double)N * (8.0 * D + 8.0), launch<64, 0, false, 1>},
      {"wr_t64", (double)N * (8.0 * D + 8.0), launch<64, 0, false, 2>},
  };
  printf("N=%lld D=%d slots=%d\n", (long long)N, D, kSlots);
  for (int rep = 0; rep < 2; ++rep)
    for (auto& v : vs) {
      for (int i = 0; i < 4; ++i) v.f(a);
      hipDeviceSynchronize();
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      const int it = 32;
      hipEventRecord(e0);
      for (int i = 0; i < it; ++i) v.f(a);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / it;
      printf("%-12s %7.2f us  %6.0f GB/s (algorithmic)\n", v.name, us, v.bytes / (us * 1e-6) / 1e9);
    }
  return 0;
}
