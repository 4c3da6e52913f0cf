// Memory-skeleton microbenchmark of the step kernel (timing-only tool, not
// part of the product): what the C2 step's HBM pattern costs without its
// arithmetic.  N = 2^20 particles, D = 10 fp64 SoA columns.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_mem.hip -o tools/ubench_mem && tools/ubench_mem
//
// Variants (each one launch shape of 256-thread blocks, 1 particle per lane):
//   copy        y[k][j] = x[k][j] + 1, logw[j] = 0           (the floor)
//   copy_nt     same with nontemporal stores
//   gather      ancestors from systematic range marks (DPP prefix max), then
//               y[k][j] = x[k][anc] + 1, anc[j] and logw[j] written (the C2 skeleton)
//   gather_tab  gather + the 6 KB LDS table copy and block barrier per block
//   gather_2t   gather with two 64-particle tiles per wave (half the waves)
//   gather_pers gather as a grid-stride loop over co-resident blocks
//   gather_hist gather whose input/output slots advance through a 16-step
//               history (fresh pages every launch, as record_history)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

constexpr int D = 10;
constexpr int64_t N = 1 << 20;
constexpr int kBlock = 256;

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
  int64_t ld;
  const uint64_t* mark;
  const uint64_t* carry;
  int32_t* anc;
  double* logw;
  const double* tab;
};

__global__ __launch_bounds__(kBlock) void k_copy(Args a) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double v[D];
#pragma unroll
  for (int k = 0; k < D; ++k) v[k] = a.x[k * a.ld + j];
#pragma unroll
  for (int k = 0; k < D; ++k) a.y[k * a.ld + j] = v[k] + 1.0;
  a.logw[j] = 0.0;
}

__global__ __launch_bounds__(kBlock) void k_copy_nt(Args a) {
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  double v[D];
#pragma unroll
  for (int k = 0; k < D; ++k) v[k] = a.x[k * a.ld + j];
#pragma unroll
  for (int k = 0; k < D; ++k) __builtin_nontemporal_store(v[k] + 1.0, &a.y[k * a.ld + j]);
  __builtin_nontemporal_store(0.0, &a.logw[j]);
}

template <bool TAB>
__device__ __forceinline__ void gather_tile(const Args& a, int64_t tile, const double* lt) {
  const int lane = threadIdx.x & 63;
  const int64_t j = tile * 64 + lane;
  uint64_t v = a.mark[j];
  const uint64_t c = a.carry[tile];
  v = wave_incl_max_u64(v > c ? v : c);
  const int64_t src = (int64_t)(uint32_t)v;
  a.anc[j] = (int32_t)src;
  double x[D];
#pragma unroll
  for (int k = 0; k < D; ++k) x[k] = a.x[k * a.ld + src];
  double s = TAB ? lt[lane & 511] : 1.0;
#pragma unroll
  for (int k = 0; k < D; ++k) a.y[k * a.ld + j] = x[k] + s;
  a.logw[j] = s;
}

// gather writing y (plain or nontemporal) and optionally a second copy h
template <bool NT, bool DUAL, bool NT_H>
__global__ __launch_bounds__(kBlock) void k_gather_h(Args a, double* h) {
  const int lane = threadIdx.x & 63;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t j = tile * 64 + lane;
  uint64_t v = a.mark[j];
  const uint64_t c = a.carry[tile];
  v = wave_incl_max_u64(v > c ? v : c);
  const int64_t src = (int64_t)(uint32_t)v;
  a.anc[j] = (int32_t)src;
  double x[D];
#pragma unroll
  for (int k = 0; k < D; ++k) x[k] = a.x[k * a.ld + src];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    if (NT) __builtin_nontemporal_store(x[k] + 1.0, &a.y[k * a.ld + j]);
    else a.y[k * a.ld + j] = x[k] + 1.0;
    if (DUAL) {
      if (NT_H) __builtin_nontemporal_store(x[k] + 1.0, &h[k * a.ld + j]);
      else h[k * a.ld + j] = x[k] + 1.0;
    }
  }
  a.logw[j] = 1.0;
}

// gather with write-through (sc1) stores: no dirty L2 lines at the boundary
__global__ __launch_bounds__(kBlock) void k_gather_wt(Args a) {
  const int lane = threadIdx.x & 63;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t j = tile * 64 + lane;
  uint64_t v = a.mark[j];
  const uint64_t c = a.carry[tile];
  v = wave_incl_max_u64(v > c ? v : c);
  const int64_t src = (int64_t)(uint32_t)v;
  __hip_atomic_store(&a.anc[j], (int32_t)src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  double x[D];
#pragma unroll
  for (int k = 0; k < D; ++k) x[k] = a.x[k * a.ld + src];
#pragma unroll
  for (int k = 0; k < D; ++k) __hip_atomic_store(&a.y[k * a.ld + j], x[k] + 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&a.logw[j], 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// gather with 16-byte stores: lane pairs swap halves so that each lane holds
// two consecutive particles of D/2 columns (row_xmask DPP), then dwordx4 stores
__global__ __launch_bounds__(kBlock) void k_gather_st16(Args a) {
  const int lane = threadIdx.x & 63;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t j = tile * 64 + lane;
  uint64_t v = a.mark[j];
  const uint64_t c = a.carry[tile];
  v = wave_incl_max_u64(v > c ? v : c);
  const int64_t src = (int64_t)(uint32_t)v;
  a.anc[j] = (int32_t)src;
  double x[D];
#pragma unroll
  for (int k = 0; k < D; ++k) x[k] = a.x[k * a.ld + src] + 1.0;
  const bool odd = lane & 1;
  const int64_t j0 = j & ~1ll;
#pragma unroll
  for (int h = 0; h < D / 2; ++h) {
    // even lane keeps column h and sends column h + D/2; odd lane the reverse
    const double mine = odd ? x[h] : x[h + D / 2];
    const uint64_t u = __builtin_bit_cast(uint64_t, mine);
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, 0xb1, 0xf, 0xf, true);  // quad_perm [1,0,3,2]
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), 0xb1, 0xf, 0xf, true);
    const double other = __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
    const int col = odd ? h + D / 2 : h;
    double2 pr;
    pr.x = odd ? other : x[h];     // particle j0
    pr.y = odd ? x[h + D / 2] : other;  // particle j0 + 1
    *reinterpret_cast<double2*>(&a.y[col * a.ld + j0]) = pr;
  }
  a.logw[j] = 1.0;
}

// a dependent small kernel (the resample's fold: every block reads 4096 doubles)
__global__ __launch_bounds__(1024) void k_small(const double* p, double* out) {
  double m = -1e300;
  for (int i = threadIdx.x; i < 4096; i += 1024) m = fmax(m, p[i]);
  if (m == 12345.0) out[blockIdx.x] = m;
}

template <bool TAB>
__global__ __launch_bounds__(kBlock) void k_gather(Args a) {
  __shared__ double lt[768];
  if (TAB) {
    for (int i = threadIdx.x; i < 384; i += kBlock) reinterpret_cast<double2*>(lt)[i] = reinterpret_cast<const double2*>(a.tab)[i];
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  gather_tile<TAB>(a, (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), lt);
}

__global__ __launch_bounds__(kBlock) void k_gather_2t(Args a) {
  const int64_t t0 = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 6);
  gather_tile<false>(a, t0, nullptr);
  gather_tile<false>(a, t0 + 4, nullptr);
}

__global__ __launch_bounds__(kBlock) void k_gather_pers(Args a, int64_t nvb) {
  for (int64_t vb = blockIdx.x; vb < nvb; vb += gridDim.x) gather_tile<false>(a, vb * 4 + (threadIdx.x >> 6), nullptr);
}

static double* g_hist = nullptr;
static int g_slot = 0;
static int g_nslots = 16;

// touch one double per 64 KiB of a slot (translation warm-up only)
__global__ void k_touch(double* p, int64_t n, int64_t stride) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * stride;
  if (i < n) __builtin_nontemporal_store(0.0, p + i);
}
static double* g_pp = nullptr;
template <bool NT, bool DUAL, bool NT_H>
static void hist_launch2(const Args& a0, int64_t nvb) {
  Args a = a0;
  double* h = g_hist + (size_t)((g_slot + 1) % 16) * D * N;
  if (DUAL) {
    a.x = g_pp + (size_t)(g_slot % 2) * D * N;
    a.y = g_pp + (size_t)((g_slot + 1) % 2) * D * N;
  } else {
    a.x = g_hist + (size_t)(g_slot % 16) * D * N;
    a.y = h;
  }
  ++g_slot;
  hipLaunchKernelGGL((k_gather_h<NT, DUAL, NT_H>), dim3(nvb), dim3(kBlock), 0, 0, a, h);
}
static void hist_launch(const Args& a0, int64_t nvb, int touch) {
  Args a = a0;
  a.x = g_hist + (size_t)(g_slot % g_nslots) * D * N;
  a.y = g_hist + (size_t)((g_slot + 1) % g_nslots) * D * N;
  ++g_slot;
  if (touch) {
    const int64_t n = (int64_t)D * N, stride = 8192;
    hipLaunchKernelGGL(k_touch, dim3((unsigned)((n / stride + 255) / 256)), dim3(256), 0, 0, a.y, n, stride);
  }
  hipLaunchKernelGGL(k_gather<false>, dim3(nvb), dim3(kBlock), 0, 0, a);
}

int main() {
  const int64_t ld = N;
  std::vector<uint64_t> mark(N, 0), carry(N / 64, 0);
  // a systematic-resampling pattern: ancestors drawn from skewed weights
  std::vector<int64_t> anc(N);
  {
    srand(1);
    std::vector<double> w(N);
    for (auto& v : w) { const double u = (rand() + 0.5) / (RAND_MAX + 1.0); v = u * u * u * u; }
    double S = 0;
    for (double v : w) S += v;
    double cum = 0;
    int64_t i = 0;
    const double off = 0.37;
    for (int64_t j = 0; j < N; ++j) {
      const double tgt = (j + off) * S / N;
      while (i < N - 1 && cum + w[i] <= tgt) cum += w[i++];
      anc[j] = i;
    }
    const uint64_t ep = 5ull << 32;
    for (int64_t j = 0; j < N; ++j)
      if (j == 0 || anc[j] != anc[j - 1]) mark[j] = ep | (uint64_t)anc[j];
    for (int64_t g = 0; g < N / 64; ++g) carry[g] = ep | (uint64_t)anc[g * 64];
  }
  Args a{};
  double *x, *y, *logw, *tab;
  uint64_t *dm, *dc;
  int32_t* danc;
  hipMalloc(&x, sizeof(double) * D * N);
  hipMalloc(&y, sizeof(double) * D * N);
  hipMalloc(&logw, sizeof(double) * N);
  hipMalloc(&tab, sizeof(double) * 768);
  hipMalloc(&dm, sizeof(uint64_t) * N);
  hipMalloc(&dc, sizeof(uint64_t) * N / 64);
  hipMalloc(&danc, sizeof(int32_t) * N);
  hipMemset(x, 0, sizeof(double) * D * N);
  hipMalloc(&g_hist, sizeof(double) * D * N * 16);
  hipMalloc(&g_pp, sizeof(double) * D * N * 2);
  hipMemset(g_pp, 0, sizeof(double) * D * N * 2);
  hipMemset(g_hist, 0, sizeof(double) * D * N * 16);
  hipMemset(tab, 0, sizeof(double) * 768);
  hipMemcpy(dm, mark.data(), sizeof(uint64_t) * N, hipMemcpyHostToDevice);
  hipMemcpy(dc, carry.data(), sizeof(uint64_t) * N / 64, hipMemcpyHostToDevice);
  a = Args{x, y, ld, dm, dc, danc, logw, tab};
  int occ = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_gather_pers, kBlock, 0);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int64_t nvb = N / kBlock;
  const double bytes_copy = (double)N * (16.0 * D + 8.0);
  const double bytes_gather = (double)N * (16.0 * D + 8.0 + 8.0 + 4.0);
  struct V {
    const char* name;
    double bytes;
    void (*f)(const Args&, int64_t, int);
  } vs[] = {
      {"copy", bytes_copy, [](const Args& a, int64_t nvb, int) { hipLaunchKernelGGL(k_copy, dim3(nvb), dim3(kBlock), 0, 0, a); }},
      {"copy_nt", bytes_copy, [](const Args& a, int64_t nvb, int) { hipLaunchKernelGGL(k_copy_nt, dim3(nvb), dim3(kBlock), 0, 0, a); }},
      {"gather", bytes_gather, [](const Args& a, int64_t nvb, int) { hipLaunchKernelGGL(k_gather<false>, dim3(nvb), dim3(kBlock), 0, 0, a); }},
      {"gather_tab", bytes_gather, [](const Args& a, int64_t nvb, int) { hipLaunchKernelGGL(k_gather<true>, dim3(nvb), dim3(kBlock), 0, 0, a); }},
      {"gather_2t", bytes_gather, [](const Args& a, int64_t nvb, int) { hipLaunchKernelGGL(k_gather_2t, dim3(nvb / 2), dim3(kBlock), 0, 0, a); }},
      {"gather_hist", bytes_gather, [](const Args& a, int64_t nvb, int) { g_nslots = 16; hist_launch(a, nvb, 0); }},
      {"hist_touch", bytes_gather, [](const Args& a, int64_t nvb, int) { g_nslots = 16; hist_launch(a, nvb, 1); }},
      {"hist_nt", bytes_gather, [](const Args& a, int64_t nvb, int) { hist_launch2<true, false, false>(a, nvb); }},
      {"dual", bytes_gather, [](const Args& a, int64_t nvb, int) { hist_launch2<false, true, false>(a, nvb); }},
      {"dual_nt", bytes_gather, [](const Args& a, int64_t nvb, int) { hist_launch2<false, true, true>(a, nvb); }},
      {"pair_plain", bytes_gather, [](const Args& a, int64_t nvb, int) {
         g_nslots = 16; hist_launch(a, nvb, 0);
         hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, 0, a.logw, (double*)a.tab); }},
      {"pair_wt", bytes_gather, [](const Args& a0, int64_t nvb, int) {
         Args a = a0;
         a.x = g_hist + (size_t)(g_slot % 16) * D * N;
         a.y = g_hist + (size_t)((g_slot + 1) % 16) * D * N;
         ++g_slot;
         hipLaunchKernelGGL(k_gather_wt, dim3(nvb), dim3(kBlock), 0, 0, a);
         hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, 0, a.logw, (double*)a.tab); }},
      {"small_only", bytes_gather, [](const Args& a, int64_t nvb, int) {
         hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, 0, a.logw, (double*)a.tab); }},
      {"hist_st16", bytes_gather, [](const Args& a0, int64_t nvb, int) {
         Args a = a0;
         a.x = g_hist + (size_t)(g_slot % 16) * D * N;
         a.y = g_hist + (size_t)((g_slot + 1) % 16) * D * N;
         ++g_slot;
         hipLaunchKernelGGL(k_gather_st16, dim3(nvb), dim3(kBlock), 0, 0, a); }},
      {"st16_same", bytes_gather, [](const Args& a, int64_t nvb, int) {
         hipLaunchKernelGGL(k_gather_st16, dim3(nvb), dim3(kBlock), 0, 0, a); }},
      {"hist2", bytes_gather, [](const Args& a, int64_t nvb, int) { g_nslots = 2; hist_launch(a, nvb, 0); }},
      {"hist3", bytes_gather, [](const Args& a, int64_t nvb, int) { g_nslots = 3; hist_launch(a, nvb, 0); }},
      {"hist4", bytes_gather, [](const Args& a, int64_t nvb, int) { g_nslots = 4; hist_launch(a, nvb, 0); }},
      {"gather_pers", bytes_gather, [](const Args& a, int64_t nvb, int g) { hipLaunchKernelGGL(k_gather_pers, dim3(g), dim3(kBlock), 0, 0, a, nvb); }},
  };
  const int g = occ * cus;
  printf("CUs %d, persistent occupancy %d blocks/CU\n", cus, occ);
  for (int rep = 0; rep < 2; ++rep)
    for (auto& v : vs) {
      for (int i = 0; i < 3; ++i) v.f(a, nvb, g);
      hipDeviceSynchronize();
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      const int it = 20;
      hipEventRecord(e0);
      for (int i = 0; i < it; ++i) v.f(a, nvb, g);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 1e3 / it;
      printf("%-12s %7.2f us  %6.0f GB/s (algorithmic)\n", v.name, us, v.bytes / (us * 1e-6) / 1e9);
    }
  return 0;
}
