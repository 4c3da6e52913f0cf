// Timing-only tool: cost of the step kernel's random-number pieces in
// isolation, launched like k_step (2^20 threads, 256-thread blocks), each
// thread writing one double so nothing is dead code.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -mllvm -disable-machine-licm \
//         -Iinclude tools/ubench_rng.hip -o tools/ubench_rng && tools/ubench_rng
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../gen_amd/csrc/gh_math.h"

using namespace gh;

__global__ __launch_bounds__(256, 7) void k_philox4(double* out, uint64_t seed, uint32_t t) {
  const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const u32x4 w = rng_block(seed, id, t, STREAM_STEP, (uint32_t)b);
    acc ^= w.x ^ w.y ^ w.z ^ w.w;
  }
  out[id] = (double)acc;
}

__global__ __launch_bounds__(256, 7) void k_normals10(double* out, uint64_t seed, uint32_t t) {
  const uint64_t id = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  double z[11];
  normals_n<10>(seed, id, t, STREAM_STEP, 0, z);
  double s = 0;
#pragma unroll
  for (int k = 0; k < 10; ++k) s += z[k];
  out[id] = s;
}

__global__ __launch_bounds__(256, 7) void k_bm5(double* out, uint64_t seed, uint32_t t) {
  const uint32_t id = blockIdx.x * 256 + threadIdx.x;
  double s = 0;
#pragma unroll
  for (int p = 0; p < 5; ++p) {
    double a, c;
    box_muller(id * 0x9E3779B9u + p, id ^ (uint32_t)seed ^ (p << 20), id * 0x85EBCA6Bu + t + p, &a, &c);
    s += a + c;
  }
  out[id] = s;
}

__global__ __launch_bounds__(256, 7) void k_copy10(double* out, const double* in, uint32_t n) {
  const uint32_t id = blockIdx.x * 256 + threadIdx.x;
  double x[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) x[k] = in[(size_t)k * n + id];
#pragma unroll
  for (int k = 0; k < 10; ++k) out[(size_t)k * n + id] = x[k] * 1.5;
}

int main() {
  const uint32_t n = 1u << 20;
  double *out, *in;
  hipMalloc(&out, (size_t)n * 8 * 10);
  hipMalloc(&in, (size_t)n * 8 * 10);
  hipMemset(in, 0, (size_t)n * 80);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto time = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < 20; ++i) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-14s %8.2f us per launch (2^20 threads)\n", name, ms * 1000 / 20);
  };
  const dim3 g(n / 256), blk(256);
  time("philox x4", [&] { hipLaunchKernelGGL(k_philox4, g, blk, 0, 0, out, 42ull, 7u); });
  time("normals x10", [&] { hipLaunchKernelGGL(k_normals10, g, blk, 0, 0, out, 42ull, 7u); });
  time("box-muller x5", [&] { hipLaunchKernelGGL(k_bm5, g, blk, 0, 0, out, 42ull, 7u); });
  time("copy 10 cols", [&] { hipLaunchKernelGGL(k_copy10, g, blk, 0, 0, out, (const double*)in, n); });
  return 0;
}
