// What kernel-timing events cost a stream of dependent launches (timing-only
// tool, not part of the product).  20 launches of a 160 MB streaming kernel
// (the C2 step's size) alternating with a small kernel, as bench.py's timed
// region does; two of the streaming launches are timed in each mode:
//   0  no events
//   1  hipExtLaunchKernelGGL with start/stop events (hipEventDisableSystemFence)
//   2  the same, default events
//   3  hipEventRecord before/after the launch (hipEventDisableSystemFence)
//   4  hipEventRecord before/after the launch, default events
// Prints the median wall time of the 20-launch region per mode (10 repeats).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_events.hip -o tools/ubench_events && tools/ubench_events
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr int64_t N = (1 << 20) * 10;  // doubles per slot (80 MB)

__global__ __launch_bounds__(256) void k_stream(const double* __restrict__ x, double* __restrict__ y, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 2;
  if (i + 1 < n) {
    const double2 v = *reinterpret_cast<const double2*>(x + i);
    *reinterpret_cast<double2*>(y + i) = double2{v.x + 1.0, v.y + 1.0};
  }
}
__global__ __launch_bounds__(1024) void k_small(double* p) {
  if (threadIdx.x == 0) p[blockIdx.x] += 1.0;
}

int main() {
  double *x, *y, *s;
  CK(hipMalloc(&x, N * 8));
  CK(hipMalloc(&y, N * 8));
  CK(hipMalloc(&s, 4096 * 8));
  CK(hipMemset(x, 0, N * 8));
  CK(hipMemset(y, 0, N * 8));
  CK(hipMemset(s, 0, 4096 * 8));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ef[4], ed[4];
  for (int i = 0; i < 4; ++i) {
    CK(hipEventCreateWithFlags(&ef[i], hipEventDisableSystemFence));
    CK(hipEventCreate(&ed[i]));
  }
  const dim3 grid((unsigned)(N / 2 / 256)), blk(256);
  const char* names[] = {"none", "ext-launch nofence", "ext-launch default", "record nofence", "record default"};
  for (int mode = 0; mode < 5; ++mode) {
    std::vector<double> ts;
    float kms = 0.f;
    for (int rep = 0; rep < 11; ++rep) {
      CK(hipStreamSynchronize(st));
      const auto t0 = std::chrono::steady_clock::now();
      int ne = 0;
      for (int i = 0; i < 20; ++i) {
        hipLaunchKernelGGL(k_small, dim3(256), dim3(1024), 0, st, s);
        const bool timed = mode > 0 && (i == 0 || i == 10);
        hipEvent_t* e = (mode == 1 || mode == 3) ? ef : ed;
        double* a = (i & 1) ? y : x;
        double* b = (i & 1) ? x : y;
        if (!timed) {
          hipLaunchKernelGGL(k_stream, grid, blk, 0, st, a, b, N);
        } else if (mode <= 2) {
          hipExtLaunchKernelGGL(k_stream, grid, blk, 0, st, e[ne], e[ne + 1], 0, a, b, N);
          ne += 2;
        } else {
          CK(hipEventRecord(e[ne], st));
          hipLaunchKernelGGL(k_stream, grid, blk, 0, st, a, b, N);
          CK(hipEventRecord(e[ne + 1], st));
          ne += 2;
        }
      }
      CK(hipStreamSynchronize(st));
      const auto t1 = std::chrono::steady_clock::now();
      if (rep > 0) ts.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      if (mode > 0) {
        hipEvent_t* e = (mode == 1 || mode == 3) ? ef : ed;
        float a = 0.f, b = 0.f;
        CK(hipEventElapsedTime(&a, e[0], e[1]));
        CK(hipEventElapsedTime(&b, e[2], e[3]));
        kms = 0.5f * (a + b);
      }
    }
    std::sort(ts.begin(), ts.end());
    printf("%-20s region %.1f us (min %.1f)  timed kernel %.2f us\n", names[mode], ts[ts.size() / 2], ts[0],
           kms * 1e3f);
  }
  return 0;
}
