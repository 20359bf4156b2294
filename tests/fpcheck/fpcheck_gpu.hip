// tests/fpcheck/fpcheck_gpu.hip — TEST-ONLY exhaustive GPU check of the
// traversal's short correctly-rounded sequences (rtg_trace.h sqrt_rn /
// rcp_rn).  For EVERY binary32 bit pattern x:
//   * in the fast range: the short sequence's result equals the compiler's
//     correctly rounded sqrtf(x) / 1.f / x bit for bit, AND satisfies the
//     exact rounding criterion evaluated in f64 (the midpoints between the
//     result and its float neighbours bracket the true value; the squares and
//     products involved are exact in f64);
//   * everywhere: sqrt_rn / rcp_rn (fast path plus fallback) equal sqrtf /
//     1.f / x bit for bit (NaN included).
// Loaded by tests/test_gpu_parity.py through ctypes; not part of librtg.so.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "rtg_trace.h"

using namespace rtg;

enum { kSqrtIn, kSqrtLib, kSqrtExact, kSqrtAll, kRcpIn, kRcpLib, kRcpExact, kRcpAll, kSlots };

__device__ __forceinline__ float prevf(float v) { return __uint_as_float(__float_as_uint(v) - 1u); }
__device__ __forceinline__ float nextf(float v) { return __uint_as_float(__float_as_uint(v) + 1u); }

__global__ __launch_bounds__(256) void fpcheck_kernel(unsigned long long* out, uint64_t n) {
  unsigned long long c[kSlots] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float x = __uint_as_float((uint32_t)i);
    // ---- sqrt
    const float libS = sqrtf(x);
    if (sqrt_fast_range(x)) {
      ++c[kSqrtIn];
      const float s = sqrt_fast(x);
      if (__float_as_uint(s) != __float_as_uint(libS)) ++c[kSqrtLib];
      const double lo = 0.5 * ((double)s + (double)prevf(s));
      const double hi = 0.5 * ((double)s + (double)nextf(s));
      if (!(lo * lo < (double)x && (double)x < hi * hi)) ++c[kSqrtExact];
    }
    if (__float_as_uint(sqrt_rn(x)) != __float_as_uint(libS)) ++c[kSqrtAll];
    // ---- reciprocal
    const float libR = 1.f / x;
    if (rcp_fast_range(x)) {
      ++c[kRcpIn];
      const float y = rcp_fast(x);
      if (__float_as_uint(y) != __float_as_uint(libR)) ++c[kRcpLib];
      const double lo = 0.5 * ((double)y + (double)prevf(y));
      const double hi = 0.5 * ((double)y + (double)nextf(y));
      if (!((double)x * lo < 1.0 && 1.0 < (double)x * hi)) ++c[kRcpExact];
    }
    if (__float_as_uint(rcp_rn(x)) != __float_as_uint(libR)) ++c[kRcpAll];
  }
  __shared__ unsigned long long part[kSlots][256];
  for (int k = 0; k < kSlots; ++k) part[k][threadIdx.x] = c[k];
  __syncthreads();
  if (threadIdx.x < kSlots) {
    unsigned long long sum = 0;
    for (int t = 0; t < 256; ++t) sum += part[threadIdx.x][t];
    atomicAdd(&out[threadIdx.x], sum);
  }
}

// Runs the check over all 2^32 patterns (count = 0) or the first `count`;
// writes the kSlots counters to out8.  Returns 0 or a hipError_t.
extern "C" int fpcheck_run(unsigned long long count, unsigned long long* out8) {
  unsigned long long* d = nullptr;
  hipError_t e = hipMalloc(&d, kSlots * sizeof(unsigned long long));
  if (e != hipSuccess) return (int)e;
  e = hipMemset(d, 0, kSlots * sizeof(unsigned long long));
  const uint64_t n = count ? count : (1ull << 32);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(fpcheck_kernel, dim3(16384), dim3(256), 0, nullptr, d, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess)
    e = hipMemcpy(out8, d, kSlots * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  return (int)e;
}
