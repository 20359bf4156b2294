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
// And the f64 islands' short sequences (sqrt_d_unit, div_d_fresnel):
//   * sqrt_d_unit(1 - (double)(c * c)) == sqrt(...) bit for bit for EVERY
//     float c in [0, 1) (the operands of raytracer.h:683; -c gives the same);
//   * div_d_fresnel(num^2, den^2) == num^2 / den^2 bit for bit for 2^32
//     pseudo-random float pairs (l, r) of raytracer.h:380-393 (num = l - r,
//     den = l + r, den^2 >= 1e-6f) over wide exponent ranges.
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

enum { kF64SqrtIn, kF64SqrtBad, kF64DivIn, kF64DivBad, kF64Slots };

__device__ __forceinline__ uint32_t mix32(uint64_t v) {
  v ^= v >> 33;
  v *= 0xff51afd7ed558ccdull;
  v ^= v >> 33;
  v *= 0xc4ceb9fe1a85ec53ull;
  v ^= v >> 33;
  return (uint32_t)v;
}
// a float with a random sign, a mantissa and an exponent in [2^-30, 2^30]
// (mostly near 1, where refractive indices and cosines live); every 64th
// draw anywhere in the float range (the slow path's operands too)
__device__ __forceinline__ float rand_float(uint64_t key) {
  const uint32_t h = mix32(key);
  const uint32_t h2 = mix32(key ^ 0x9E3779B97F4A7C15ull);
  if ((h2 & 63u) == 0u) return __uint_as_float(h);
  const int e = (h2 & 3u) ? (int)(h2 >> 28) - 8 : (int)((h2 >> 8) % 61u) - 30;
  return __uint_as_float((h & 0x807FFFFFu) | ((uint32_t)(127 + e) << 23));
}

__global__ __launch_bounds__(256) void fpcheck_f64_kernel(unsigned long long* out, uint64_t n) {
  unsigned long long c[kF64Slots] = {0, 0, 0, 0};
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (i < 0x3F800000ull) {  // every float c in [0, 1)
      const float cf = __uint_as_float((uint32_t)i);
      const double y = 1.0 - (double)(cf * cf);
      ++c[kF64SqrtIn];
      if (__double_as_longlong(sqrt_d_unit(y)) != __double_as_longlong(sqrt(y))) ++c[kF64SqrtBad];
    }
    const float l = rand_float(2 * i), r = rand_float(2 * i + 1);
    const double num = (double)(l - r);
    double den = (double)(l + r);
    den *= den;
    if (den >= (double)1.0e-6f) {
      ++c[kF64DivIn];
      const double a = num * num;
      const bool fast = fabsf(l) <= 0x1p100f && fabsf(r) <= 0x1p100f;
      if (__double_as_longlong(div_d_fresnel(a, den, fast)) != __double_as_longlong(a / den))
        ++c[kF64DivBad];
    }
  }
  __shared__ unsigned long long part[kF64Slots][256];
  for (int k = 0; k < kF64Slots; ++k) part[k][threadIdx.x] = c[k];
  __syncthreads();
  if (threadIdx.x < kF64Slots) {
    unsigned long long sum = 0;
    for (int t = 0; t < 256; ++t) sum += part[threadIdx.x][t];
    atomicAdd(&out[threadIdx.x], sum);
  }
}

// The f64 checks over n = count (0: 2^32) indices; writes kF64Slots counters.
extern "C" int fpcheck_f64_run(unsigned long long count, unsigned long long* out4) {
  unsigned long long* d = nullptr;
  hipError_t e = hipMalloc(&d, kF64Slots * sizeof(unsigned long long));
  if (e != hipSuccess) return (int)e;
  e = hipMemset(d, 0, kF64Slots * sizeof(unsigned long long));
  const uint64_t n = count ? count : (1ull << 32);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(fpcheck_f64_kernel, dim3(16384), dim3(256), 0, nullptr, d, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess)
    e = hipMemcpy(out4, d, kF64Slots * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  return (int)e;
}
