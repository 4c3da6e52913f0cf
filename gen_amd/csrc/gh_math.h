// gh_math.h — deterministic fp64 math + counter-based RNG shared by the HIP
// kernels and the host-side preprocessing of libgen_hip.so.
//
// Why this exists: the reference draws randomness from Julia's task-global RNG
// (src/modeling_library/distributions/normal.jl:96 `mu + std * randn()`,
// src/inference/particle_filter.jl:200 `Distributions.rand!(Categorical(..))`),
// which is neither reproducible across processes nor partitionable across
// GPUs.  The engine replaces it with Philox4x32-10 keyed by (seed) and
// countered by (global particle id, step, stream, draw), so a particle's
// randomness does not depend on launch geometry or on how many GPUs share the
// particle set.  Every transcendental on the sampling path (exp/log/sin/cos)
// is evaluated with the explicit, IEEE-basic-op-only algorithms below so that
// the GPU path and the CPU oracle produce bit-identical particle states, and
// therefore bit-identical resampling ancestors.  Only +,-,*,/,sqrt,fma and
// rint are used (all correctly rounded on gfx950 and x86-64); the build uses
// -ffp-contract=off so the compiler cannot fuse a*b+c behind our back.
//
// The written specification of every function here is DESIGN.md §4.
#pragma once
#include <stdint.h>
#include <math.h>

#include "gh_tables.h"

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GH_HD __host__ __device__ __forceinline__
#else
#define GH_HD static inline
#endif

namespace gh {

// ---------------------------------------------------------------- bit casts
GH_HD double as_f64(uint64_t u) { return __builtin_bit_cast(double, u); }
GH_HD uint64_t as_u64(double d) { return __builtin_bit_cast(uint64_t, d); }

// ------------------------------------------------------------ Philox4x32-10
// Salmon et al., "Parallel random numbers: as easy as 1, 2, 3" (SC'11).
struct u32x4 {
  uint32_t x, y, z, w;
};

GH_HD uint32_t mulhi32(uint32_t a, uint32_t b) {
  return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

#ifndef GH_PHILOX_ROUNDS
#define GH_PHILOX_ROUNDS 10  // timing-only variants may lower it; the product uses 10
#endif
GH_HD u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < GH_PHILOX_ROUNDS; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    // one 32x32->64 multiply per word pair (v_mad_u64_u32) gives hi and lo
    const uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c.z;
#if defined(__HIP_DEVICE_COMPILE__)
    // three-input xor in one v_bitop3_b32 (truth table 0x96)
    c = u32x4{(uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96), (uint32_t)p1,
              (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96), (uint32_t)p0};
#else
    c = u32x4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1,
              (uint32_t)p0};
#endif
  }
  return c;
}

// Stream identifiers (counter word w, high 16 bits).  DESIGN.md §4.2.
enum : uint32_t {
  STREAM_INIT = 1,       // latent draws of generate() at the first step
  STREAM_STEP = 2,       // latent draws of update() at steps t >= 2
  STREAM_RESAMPLE = 3,   // systematic offset / multinomial positions
  STREAM_SAMPLE = 4,     // sample_unweighted_traces
  STREAM_IS = 5,         // importance sampling
  STREAM_MH = 6,         // MH proposals / accept tests
  STREAM_SIM = 7,        // simulate(): latents from draw 0, observations from draw kSimObsDraw
};
constexpr uint32_t kSimObsDraw = 32;

GH_HD u32x4 rng_block(uint64_t seed, uint64_t id, uint32_t step, uint32_t stream,
                      uint32_t draw) {
  return philox4x32_10(u32x4{(uint32_t)id, (uint32_t)(id >> 32), step, (stream << 16) | draw},
                       (uint32_t)seed, (uint32_t)(seed >> 32));
}

// 53-bit integer from two words, and the uniform in [0,1) it encodes.
GH_HD uint64_t u53_bits(uint32_t a, uint32_t b) {
  return ((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6);
}
GH_HD double u53(uint32_t a, uint32_t b) { return (double)u53_bits(a, b) * 0x1p-53; }

// ------------------------------------------------------------ a / 20
// a / 20.0 exactly as IEEE division rounds it: the product with y = RN(1/20)
// and two FMA corrections — the first leaves the quotient within an ulp, the
// second (Markstein's theorem: y correctly rounded, q faithful, the residual
// a - 20 q exact) rounds it correctly — five operations instead of the
// division's scale / reciprocal / fix-up sequence (the nonlinear SSM's
// observation mean x^2 / 20).  Outside [2^-1000, 2^1000] in magnitude (where
// the theorem's range conditions could fail: never for the model's states)
// and for 0, inf and NaN the division itself.
GH_HD double div20(double a) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(GH_DIV20_PLAIN)
  const double m = fabs(a);
  if (!(m >= 0x1p-1000 && m <= 0x1p1000)) return a / 20.0;
  const double y = 0.05;  // RN(1/20)
  double q = a * y;
  double r = fma(-20.0, q, a);
  q = fma(r, y, q);
  r = fma(-20.0, q, a);
  return fma(r, y, q);
#else
  return a / 20.0;
#endif
}

// ------------------------------------------------------------------- exp
// fma(a, b, c) for a constant c: on the device the constant goes to an SGPR
// pair operand of one v_fma_f64 (the compiler otherwise writes it into the
// destination VGPRs with two v_mov_b32 per Horner step and uses v_fmac);
// the same correctly rounded fused operation either way.
GH_HD double fma_c(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(GH_FMA_C_PLAIN)
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "s"(c));
  return d;
#else
  return fma(a, b, c);
#endif
}

// Cody–Waite reduction x = k ln2 + r, |r| <= ln2/2, degree-13 Taylor in r.
GH_HD double ldexp_exact(double p, int k) {
  // p in [0.5, 2); multiply by 2^k without relying on libm ldexp.
  if (k > -1022 && k < 1024) return p * as_f64((uint64_t)(k + 1023) << 52);
  if (k >= 1024) return (p * 0x1p1023) * 2.0;  // k == 1024 only
  // k <= -1022: two exact-then-rounding multiplies (deterministic IEEE).
  return (p * as_f64((uint64_t)(k + 600 + 1023) << 52)) * 0x1p-600;
}

GH_HD double gh_exp(double x) {
  if (x != x) return x;
  if (x < -745.5) return 0.0;
  if (x > 709.78) return INFINITY;
  const double k = rint(x * 0x1.71547652b82fep+0);
  double r = fma(-k, 0x1.62e42fee00000p-1, x);
  r = fma(-k, 0x1.a39ef35793c76p-33, r);
  double p = 0x1.6124613a86d09p-33;  // 1/13!
  p = fma(p, r, 0x1.1eed8eff8d898p-29);
  p = fma(p, r, 0x1.ae64567f544e4p-26);
  p = fma(p, r, 0x1.27e4fb7789f5cp-22);
  p = fma(p, r, 0x1.71de3a556c734p-19);
  p = fma(p, r, 0x1.a01a01a01a01ap-16);
  p = fma(p, r, 0x1.a01a01a01a01ap-13);
  p = fma(p, r, 0x1.6c16c16c16c17p-10);
  p = fma(p, r, 0x1.1111111111111p-7);
  p = fma(p, r, 0x1.5555555555555p-5);
  p = fma(p, r, 0x1.5555555555555p-3);
  p = fma(p, r, 0x1.0000000000000p-1);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp_exact(p, (int)k);
}

// gh_exp for x <= 0 (or NaN), branch-free: the same reduction, polynomial
// and 2^k scaling as gh_exp (so the same results), with the underflow cut and
// the subnormal scaling done by selects.  Used where whole waves evaluate it.
GH_HD double gh_exp_nonpos(double x) {
  const bool tiny = x < -745.5;
  const double xc = tiny ? 0.0 : x;
  const double k = rint(xc * 0x1.71547652b82fep+0);
  double r = fma(-k, 0x1.62e42fee00000p-1, xc);
  r = fma(-k, 0x1.a39ef35793c76p-33, r);
  double p = fma_c(0x1.6124613a86d09p-33, r, 0x1.1eed8eff8d898p-29);
  p = fma_c(p, r, 0x1.ae64567f544e4p-26);
  p = fma_c(p, r, 0x1.27e4fb7789f5cp-22);
  p = fma_c(p, r, 0x1.71de3a556c734p-19);
  p = fma_c(p, r, 0x1.a01a01a01a01ap-16);
  p = fma_c(p, r, 0x1.a01a01a01a01ap-13);
  p = fma_c(p, r, 0x1.6c16c16c16c17p-10);
  p = fma_c(p, r, 0x1.1111111111111p-7);
  p = fma_c(p, r, 0x1.5555555555555p-5);
  p = fma_c(p, r, 0x1.5555555555555p-3);
  p = fma(p, r, 0x1.0000000000000p-1);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  const int ki = (int)k;
  const bool sub = ki <= -1022;
  const double sc = as_f64((uint64_t)((sub ? ki + 600 : ki) + 1023) << 52);
  const double res = (p * sc) * (sub ? 0x1p-600 : 1.0);
  return tiny ? 0.0 : res;
}

// ------------------------------------------------------------------- log
// fdlibm e_log.c structure: x = 2^k m, m in [sqrt2/2, sqrt2), f = m-1,
// s = f/(2+f), log(1+f) = f - hfsq + s (hfsq + R(s^2)).
GH_HD double gh_log(double x) {
  if (x != x || x < 0.0) return NAN;
  if (x == 0.0) return -INFINITY;
  if (x == INFINITY) return x;
  int k = 0;
  uint64_t bits = as_u64(x);
  if (bits < 0x0010000000000000ull) {  // subnormal
    x *= 0x1p54;
    k = -54;
    bits = as_u64(x);
  }
  k += (int)(bits >> 52) - 1023;
  double m = as_f64((bits & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);
  if (m > 0x1.6a09e667f3bcdp+0) {
    m *= 0.5;
    k += 1;
  }
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s;
  const double w = z * z;
  const double t1 = w * (3.999999999940941908e-01 + w * (2.222219843214978396e-01 + w * 1.531383769920937332e-01));
  const double t2 = z * (6.666666666666735130e-01 +
                         w * (2.857142874366239149e-01 + w * (1.818357216161805012e-01 + w * 1.479819860511658591e-01)));
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double dk = (double)k;
  return dk * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + dk * 1.90821492927058770002e-10)) - f);
}

// --------------------------------------------------------- sin/cos kernels
// Taylor polynomials on |x| <= pi/4.
GH_HD double sin_kernel(double x) {
  const double x2 = x * x;
  double p = -0x1.ae7f3e733b81fp-41;  // -1/15!
  p = fma(p, x2, 0x1.6124613a86d09p-33);  //  1/13!
  p = fma(p, x2, -0x1.ae64567f544e4p-26);  // -1/11!
  p = fma(p, x2, 0x1.71de3a556c734p-19);   //  1/9!
  p = fma(p, x2, -0x1.a01a01a01a01ap-13);  // -1/7!
  p = fma(p, x2, 0x1.1111111111111p-7);    //  1/5!
  p = fma(p, x2, -0x1.5555555555555p-3);   // -1/3!
  return fma(x * x2, p, x);
}
GH_HD double cos_kernel(double x) {
  const double x2 = x * x;
  double p = 0x1.ae7f3e733b81fp-45;        //  1/16!
  p = fma(p, x2, -0x1.93974a8c07c9dp-37);  // -1/14!
  p = fma(p, x2, 0x1.1eed8eff8d898p-29);   //  1/12!
  p = fma(p, x2, -0x1.27e4fb7789f5cp-22);  // -1/10!
  p = fma(p, x2, 0x1.a01a01a01a01ap-16);   //  1/8!
  p = fma(p, x2, -0x1.6c16c16c16c17p-10);  // -1/6!
  p = fma(p, x2, 0x1.5555555555555p-5);    //  1/4!
  p = fma(p, x2, -0x1.0000000000000p-1);   // -1/2!
  return fma(x2, p, 1.0);
}

// sin(2*pi*u), cos(2*pi*u) for u in [0,1) (u a multiple of 2^-53).
// Octant o = floor(8u), f = 8u - o (both exact).  Even octants evaluate the
// kernels at f*pi/4, odd ones at (1-f)*pi/4 (1-f exact) with sin/cos swapped;
// the quadrant then permutes and negates.  Written with selects so a wave
// evaluates the two polynomials once, whatever its lanes' octants.
GH_HD void sincos_2pi(double u, double* s, double* c) {
  const double v = u * 8.0;               // exact
  const double o = floor(v);              // octant 0..7
  const double f = v - o;                 // exact, in [0,1)
  const int oi = (int)o;
  const bool odd = (oi & 1) != 0;
  const double a = (odd ? (1.0 - f) : f) * 0x1.921fb54442d18p-1;
  const double sk = sin_kernel(a), ck = cos_kernel(a);
  const double ss = odd ? ck : sk, cc = odd ? sk : ck;
  const int q = oi >> 1;
  // q=0: (ss, cc)  q=1: (cc, -ss)  q=2: (-ss, -cc)  q=3: (-cc, ss)
  const double s0 = (q & 1) ? cc : ss;
  const double c0 = (q & 1) ? ss : cc;
  *s = (q >= 2) ? -s0 : s0;
  *c = (q == 1 || q == 2) ? -c0 : c0;
}

// cos(x) for moderate |x| (< 2^19 * pi/2): fdlibm three-part pi/2 reduction.
GH_HD double gh_cos(double x) {
  const double k = rint(x * 0x1.45f306dc9c883p-1);  // 2/pi
  double r = fma(-k, 1.57079632673412561417e+00, x);
  r = fma(-k, 6.07710050630396597660e-11, r);
  r = fma(-k, 2.02226624871116645580e-21, r);
  const int q = ((int)k) & 3;
  switch (q) {
    case 0: return cos_kernel(r);
    case 1: return -sin_kernel(r);
    case 2: return -cos_kernel(r);
    default: return sin_kernel(r);
  }
}

// Constant tables of the Box–Muller (tools/gen_tables.py, shared with the
// oracle): [0, 256) the log bins {invc, logc}, [256, 768) {sin, cos}(2 pi j/256).
constexpr int kMathTabDoubles = 768;
constexpr int kTrigOff = 256;
static const double gh_math_tab_host[kMathTabDoubles] = {GH_LOG_TABLE_DATA, GH_TRIG_TABLE_DATA};
#if defined(__HIPCC__)
static __constant__ double gh_math_tab_dev[kMathTabDoubles] = {GH_LOG_TABLE_DATA, GH_TRIG_TABLE_DATA};
// Copy the tables into a block's LDS (kMathTabDoubles doubles); callers
// barrier before the first read.  Per-lane table reads then are ds_read_b128
// instead of vector-memory loads.
__device__ __forceinline__ void load_math_tab(double* lds) {
  for (int i = threadIdx.x; i < kMathTabDoubles / 2; i += blockDim.x)
    reinterpret_cast<double2*>(lds)[i] = reinterpret_cast<const double2*>(gh_math_tab_dev)[i];
}
// The same for a block of exactly 256 threads: both loads of a thread are
// issued before its first LDS write (one memory round trip, no loop).
__device__ __forceinline__ void load_math_tab256(double* lds) {
  static_assert(kMathTabDoubles / 2 > 256 && kMathTabDoubles / 2 <= 512, "two double2 per thread");
  const double2* src = reinterpret_cast<const double2*>(gh_math_tab_dev);
  double2* dst = reinterpret_cast<double2*>(lds);
  constexpr int n = kMathTabDoubles / 2;
  // entries [256, n) are written twice with the same value (unconditional
  // stores: a guarded one would let the compiler sink its load behind the
  // first wait)
  const int t = threadIdx.x, t1 = 256 + t % (n - 256);
  const double2 a = src[t];
  const double2 b = src[t1];
  dst[t] = a;
  dst[t1] = b;
}
#endif
// Device callers always pass a table (a block's LDS copy, or gh_math_tab_dev):
// a select between an LDS and a constant pointer would be a generic pointer,
// and its flat loads wait on vmcnt as well (every outstanding global load and
// store of the wave) instead of lgkmcnt alone.
GH_HD const double* math_tab(const double* tab) {
#if defined(__HIP_DEVICE_COMPILE__)
  return tab;
#else
  return tab ? tab : gh_math_tab_host;
#endif
}
// both doubles of table entry i (16 bytes) in one load
GH_HD void tab_pair(const double* t, uint32_t i, double* a, double* b) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double2 e = reinterpret_cast<const double2*>(t)[i];
  *a = e.x;
  *b = e.y;
#else
  *a = t[2 * i];
  *b = t[2 * i + 1];
#endif
}

// sin(2 pi c / 2^32), cos(2 pi c / 2^32) for a 32-bit angle word c, table
// driven: j = the nearest of 256 table angles (c + 2^23) >> 24 (mod 256),
// residual d = (int32)(c - j 2^24) (2 pi 2^-32), |d| <= pi/256, one rounding;
// sin d = d + d^3 (-1/6 + d^2 (1/120 - d^2/5040)), cos d - 1 =
// d^2 (-1/2 + d^2 (1/24 - d^2/720)) (truncation < 1e-20), then the rotation
// s = s_j + (s_j (cos d - 1) + c_j sin d), c = c_j + (c_j (cos d - 1) - s_j sin d).
// No branches, no selects; |error| < 4e-16.
GH_HD void sincos_2pi_u32(uint32_t c, double* s, double* co, const double* tab = nullptr) {
  const double* t = math_tab(tab) + kTrigOff;
  const uint32_t j = ((c + 0x800000u) >> 24) & 255u;
  const int32_t di = (int32_t)(c - (j << 24));
  const double d = (double)di * 0x1.921fb54442d18p-30;
  const double d2 = d * d;
  double ps = fma(d2, -0x1.a01a01a01a01ap-13, 0x1.1111111111111p-7);
  ps = fma_c(d2, ps, -0x1.5555555555555p-3);
  const double sd = fma(d * d2, ps, d);
  double pc = fma(d2, -0x1.6c16c16c16c17p-10, 0x1.5555555555555p-5);
  pc = fma(d2, pc, -0.5);
  const double cm1 = d2 * pc;
  double sj, cj;
  tab_pair(t, j, &sj, &cj);
  *s = sj + fma(sj, cm1, cj * sd);
  *co = cj + fma(cj, cm1, -(sj * sd));
}

// 1 - u53(a, b) in (0, 1], exactly: the 53-bit integer K = hi 2^32 + lo is
// never formed; 1 - hi 2^-21 and then - lo 2^-53 are both exact.
GH_HD double one_minus_u53(uint32_t a, uint32_t b) {
  const uint32_t hi = a >> 11;
  const uint32_t lo = ((a << 21) & 0xFC000000u) | (b >> 6);
  return fma(-(double)lo, 0x1p-53, fma(-(double)hi, 0x1p-21, 1.0));
}

// Table-driven log for positive normal finite x (the Box–Muller radius,
// x in [2^-53, 1], and the coal score terms): x = 2^e m, bin i = top 7 mantissa bits,
// bins i >= 53 take m/2 and k = e + 1, so the reduced m lies in
// [0.70703125, 1.4140625); r = fma(m, invc_i, -1) (|r| <= 2^-8, one rounding),
// log x = k ln2 + logc_i + log1p(r), log1p(r) = r + r^2 Q(r) with the Taylor
// terms through r^7 (truncation < 0.2 ulp).  No division and no branches;
// the table (tools/gen_tables.py) is shared with the oracle.
GH_HD double gh_log_unit(double x, const double* tab = nullptr) {
  const double* t = math_tab(tab);
  const uint64_t bits = as_u64(x);
  const uint32_t hi = (uint32_t)(bits >> 32);
  const uint32_t i = (hi >> 13) & 127u;
  const uint32_t up = i >= 53u ? 1u : 0u;
  const int k = (int)(hi >> 20) - 1023 + (int)up;
  // m: x's mantissa under exponent 0 (bins < 53) or -1 (bins >= 53)
  const double m = as_f64((bits & 0x000FFFFFFFFFFFFFull) | ((uint64_t)(1023u - up) << 52));
  double invc, logc;
  tab_pair(t, i, &invc, &logc);
  const double r = fma(m, invc, -1.0);
  const double r2 = r * r;
  double q = fma(0x1.2492492492492p-3, r, -0x1.5555555555555p-3);  // 1/7, -1/6
  q = fma_c(q, r, 0x1.999999999999ap-3);                          // 1/5
  q = fma_c(q, r, -0x1.0p-2);                                     // -1/4
  q = fma_c(q, r, 0x1.5555555555555p-2);                          // 1/3
  q = fma(q, r, -0x1.0p-1);                                       // -1/2
  const double kd = (double)k;
  const double h = fma(kd, 0x1.62e42fefa3800p-1, logc);           // ln2 high part: k ln2hi exact
  const double l = fma(kd, 0x1.ef35793c76730p-45, r);             // ln2 low part
  return h + fma(r2, q, l);
}

// IEEE sqrt for x = 0 or x in [2^-767, inf): on the device the correctly
// rounded rsq + Newton sequence the compiler emits for sqrt, minus its
// small-input scaling and class fix-up (x here is -2 log(u1) in [0, 75]);
// tests/test_gpu_parity.py checks it against the host's sqrt.
GH_HD double sqrt_radius(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y;
  double h = y * 0.5;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  double d = fma(-g, g, x);
  h = fma(h, r, h);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  g = fma(d, h, g);
  return x == 0.0 ? x : g;
#else
  return sqrt(x);
#endif
}

// ------------------------------------------------------------ normals
// Box–Muller on three 32-bit words: radius from the 53-bit uniform of (a, b),
// angle from the 32-bit word c.  Four Philox words per block
// serve 4/3 pairs, so d normals take ceil(3 ceil(d/2) / 4) blocks.
GH_HD void box_muller(uint32_t a, uint32_t b, uint32_t c, double* z0, double* z1, const double* tab = nullptr) {
  const double u1 = one_minus_u53(a, b);  // (0, 1]
  const double r = sqrt_radius(-2.0 * gh_log_unit(u1, tab));
  double s, co;
  sincos_2pi_u32(c, &s, &co, tab);
  *z0 = r * co;
  *z1 = r * s;
}

// two standard normals from one Philox block (words x, y, z)
GH_HD void normal_pair(u32x4 w, double* z0, double* z1, const double* tab = nullptr) {
  box_muller(w.x, w.y, w.z, z0, z1, tab);
}

// n standard normals from consecutive blocks draw0, draw0+1, ...: pair p takes
// words 3p, 3p+1, 3p+2 of the concatenated blocks.
#if defined(__HIPCC__)
template <int N>
__device__ __forceinline__ void normals_n(uint64_t seed, uint64_t id, uint32_t step, uint32_t stream,
                                          uint32_t draw0, double* z, const double* tab = nullptr) {
  constexpr int kPairs = (N + 1) / 2, kBlocks = (3 * kPairs + 3) / 4;
  uint32_t wd[4 * kBlocks];
#pragma unroll
  for (int b = 0; b < kBlocks; ++b) {
    const u32x4 w = rng_block(seed, id, step, stream, draw0 + (uint32_t)b);
    wd[4 * b] = w.x;
    wd[4 * b + 1] = w.y;
    wd[4 * b + 2] = w.z;
    wd[4 * b + 3] = w.w;
  }
#pragma unroll
  for (int p = 0; p < kPairs; ++p) {
    double a, c;
    box_muller(wd[3 * p], wd[3 * p + 1], wd[3 * p + 2], &a, &c, tab);
    z[2 * p] = a;
    if (2 * p + 1 < N) z[2 * p + 1] = c;
  }
}

// normals_n with a run-time count (n <= 64): the same word layout, each block
// generated when its first word is needed
__device__ __forceinline__ void normals_rt(uint64_t seed, uint64_t id, uint32_t step, uint32_t stream,
                                           uint32_t draw0, int n, double* z, const double* tab = nullptr) {
  u32x4 w{0, 0, 0, 0};
  int cur = -1;
  for (int p = 0; 2 * p < n; ++p) {
    uint32_t wd[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int k = 3 * p + q;
      if ((k >> 2) != cur) {
        cur = k >> 2;
        w = rng_block(seed, id, step, stream, draw0 + (uint32_t)cur);
      }
      const int e = k & 3;
      wd[q] = e == 0 ? w.x : (e == 1 ? w.y : (e == 2 ? w.z : w.w));
    }
    double a, c;
    box_muller(wd[0], wd[1], wd[2], &a, &c, tab);
    z[2 * p] = a;
    if (2 * p + 1 < n) z[2 * p + 1] = c;
  }
}
#endif

// (u53 * S) >> 53 without overflow: floor(u * S) for the integer CDF.
GH_HD uint64_t scale_u53(uint64_t u, uint64_t S) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t lo = u * S;
  const uint64_t hi = __umul64hi(u, S);
#else
  const unsigned __int128 p = (unsigned __int128)u * S;
  const uint64_t lo = (uint64_t)p, hi = (uint64_t)(p >> 64);
#endif
  return (hi << 11) | (lo >> 53);
}

// Integer weight quantisation shift for N particles: q = floor(e * 2^shift).
GH_HD int quant_shift(uint64_t n_global) {
  int lg = 0;
  while ((1ull << lg) < n_global) ++lg;
  int s = 62 - lg;
  return s > 52 ? 52 : s;
}

GH_HD uint64_t quantize_weight(double lw, double M, int shift) {
  const double e = gh_exp(lw - M);  // in [0, 1]
  return (uint64_t)(e * as_f64((uint64_t)(shift + 1023) << 52));
}

// quantize_weight for lw - M <= 0 (always the case: M is the maximum), with
// the branch-free exp (identical values)
GH_HD uint64_t quantize_weight_nonpos(double lw, double M, int shift) {
  const double e = gh_exp_nonpos(lw - M);
  return (uint64_t)(e * as_f64((uint64_t)(shift + 1023) << 52));
}

constexpr double LOG_2PI = 0x1.d67f1c864beb4p+0;

}  // namespace gh
