// Issue-cost microbenchmark for the instruction classes of the step kernel
// (timing-only tool, not part of the product).  One kernel per instruction:
// 8 independent chains per lane so latency is hidden, 7 waves per SIMD
// (the step kernel's occupancy), cycles per wave-instruction printed.
//
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_isa.hip -o tools/ubench_isa && tools/ubench_isa
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kIters = 4096;
constexpr int kChains = 8;

#define BODY_KERNEL(NAME, T, INIT, OP)                                               \
  __global__ __launch_bounds__(256) void NAME(T* out, T seed, long long* clk) {     \
    T v[kChains];                                                                    \
    _Pragma("unroll") for (int c = 0; c < kChains; ++c) v[c] = INIT;                 \
    const long long t0 = wall_clock64();                                             \
    for (int i = 0; i < kIters; ++i) {                                               \
      _Pragma("unroll") for (int c = 0; c < kChains; ++c) { OP; }                    \
    }                                                                                \
    const long long t1 = wall_clock64();                                             \
    T acc = v[0];                                                                    \
    _Pragma("unroll") for (int c = 1; c < kChains; ++c) acc += v[c];                 \
    out[blockIdx.x * 256 + threadIdx.x] = acc;                                       \
    if (threadIdx.x == 0 && blockIdx.x == 0) *clk = t1 - t0;                         \
  }

// every op is an asm statement so the compiler can neither fold nor hoist it
BODY_KERNEL(k_fma_f64, double, seed + c, asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(v[c])))
BODY_KERNEL(k_mul_f64, double, seed + c, asm volatile("v_mul_f64 %0, %0, %0" : "+v"(v[c])))
BODY_KERNEL(k_rcp_f64, double, seed + c, asm volatile("v_rcp_f64 %0, %0" : "+v"(v[c])))
BODY_KERNEL(k_rsq_f64, double, seed + c, asm volatile("v_rsq_f64 %0, %0" : "+v"(v[c])))
BODY_KERNEL(k_add_u32, uint32_t, (uint32_t)seed + c, asm volatile("v_add_u32 %0, %0, %0" : "+v"(v[c])))
BODY_KERNEL(k_xor3_u32, uint32_t, (uint32_t)seed + c, asm volatile("v_bitop3_b32 %0, %0, %0, %0 bitop3:0x96" : "+v"(v[c])))
BODY_KERNEL(k_mad_u64, uint64_t, (uint64_t)seed + c,
            { const uint32_t lo = (uint32_t)v[c]; asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, %0" : "+v"(v[c]) : "v"(lo) : "vcc"); })
BODY_KERNEL(k_mullo_u32, uint32_t, (uint32_t)seed + c, asm volatile("v_mul_lo_u32 %0, %0, %0" : "+v"(v[c])))
BODY_KERNEL(k_mulhi_u32, uint32_t, (uint32_t)seed + c, asm volatile("v_mul_hi_u32 %0, %0, %0" : "+v"(v[c])))
BODY_KERNEL(k_mulu24, uint32_t, (uint32_t)seed + c, asm volatile("v_mul_u32_u24 %0, %0, %0" : "+v"(v[c])))
BODY_KERNEL(k_cvt_f64_u32, double, seed + c, { const uint32_t lo = (uint32_t)__builtin_bit_cast(uint64_t, v[c]); asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(v[c]) : "v"(lo)); })
BODY_KERNEL(k_alignbit, uint32_t, (uint32_t)seed + c, asm volatile("v_alignbit_b32 %0, %0, %0, 13" : "+v"(v[c])))
BODY_KERNEL(k_fma_f32, float, (float)seed + c, asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(v[c])))
BODY_KERNEL(k_cndmask, uint32_t, (uint32_t)seed + c, asm volatile("v_cndmask_b32 %0, %0, %0, vcc" : "+v"(v[c])))
BODY_KERNEL(k_ldexp_f64, double, seed + c, asm volatile("v_ldexp_f64 %0, %0, 1" : "+v"(v[c])))
BODY_KERNEL(k_frexp_mant_f64, double, seed + c, asm volatile("v_frexp_mant_f64 %0, %0" : "+v"(v[c])))
BODY_KERNEL(k_div_fixup_f64, double, seed + c, asm volatile("v_div_fixup_f64 %0, %0, %0, %0" : "+v"(v[c])))
BODY_KERNEL(k_log_f32, float, (float)seed + c, asm volatile("v_log_f32 %0, %0" : "+v"(v[c])))

int main() {
  const int grid = 256 * 7;  // 7 blocks of 4 waves per CU = 7 waves per SIMD (256 CUs)
  void* out;
  long long* clk;
  hipMalloc(&out, (size_t)grid * 256 * 8);
  hipMalloc(&clk, 8);
  struct K {
    const char* name;
    void (*launch)(void*, long long*, int);
    int ops_per_iter;
  };
#define L(NAME, T) [](void* o, long long* c, int g) { hipLaunchKernelGGL(NAME, dim3(g), dim3(256), 0, 0, (T*)o, (T)1, c); }
  K ks[] = {
      {"v_fma_f64", L(k_fma_f64, double), 1},   {"v_mul_f64", L(k_mul_f64, double), 1},
      {"v_rcp_f64", L(k_rcp_f64, double), 1},   {"v_rsq_f64", L(k_rsq_f64, double), 1},
      {"v_add_u32", L(k_add_u32, uint32_t), 1}, {"v_bitop3_b32", L(k_xor3_u32, uint32_t), 1},
      {"v_mad_u64_u32", L(k_mad_u64, uint64_t), 1}, {"v_mul_lo_u32", L(k_mullo_u32, uint32_t), 1},
      {"v_mul_u32_u24", L(k_mulu24, uint32_t), 1}, {"v_cvt_f64_u32", L(k_cvt_f64_u32, double), 1},
      {"v_alignbit_b32", L(k_alignbit, uint32_t), 1}, {"v_fma_f32", L(k_fma_f32, float), 1},
      {"v_mul_hi_u32", L(k_mulhi_u32, uint32_t), 1}, {"v_cndmask_b32", L(k_cndmask, uint32_t), 1},
      {"v_ldexp_f64", L(k_ldexp_f64, double), 1}, {"v_frexp_mant_f64", L(k_frexp_mant_f64, double), 1},
      {"v_div_fixup_f64", L(k_div_fixup_f64, double), 1}, {"v_log_f32", L(k_log_f32, float), 1},
  };
  for (auto& k : ks) {
    k.launch(out, clk, grid);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    k.launch(out, clk, grid);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    // wave-instructions per SIMD = waves per SIMD (7) * iters * chains
    const double winst = 7.0 * kIters * kChains * k.ops_per_iter;
    const double cyc = ms * 1e-3 * 2.4e9 / winst;
    printf("%-24s %8.3f ms  %6.2f cycles per wave-instruction per SIMD (2.4 GHz)\n", k.name, ms, cyc);
  }
  return 0;
}
