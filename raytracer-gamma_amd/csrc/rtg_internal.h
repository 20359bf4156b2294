// rtg_internal.h — helpers shared by the host code and the kernels of librtg.so.
#pragma once

#include <stdarg.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RTG_HDI __host__ __device__ __forceinline__
#else
#define RTG_HDI inline
#endif

void rtg_set_error(const char* fmt, ...);
void rtg_clear_error();

namespace rtg {

// Row-cyclic sharding: block b = rows [b*B, (b+1)*B) -> shard b % G.
RTG_HDI unsigned shard_global_row(unsigned localRow, unsigned B, unsigned g, unsigned G) {
  const unsigned lb = localRow / B;
  return (lb * G + g) * B + (localRow % B);
}

RTG_HDI unsigned shard_row_count(unsigned H, unsigned B, unsigned g, unsigned G) {
  const unsigned nblk = (H + B - 1) / B;
  if (g >= nblk) return 0;
  const unsigned myBlocks = (nblk - g + G - 1) / G;  // blocks g, g+G, ...
  unsigned rows = myBlocks * B;
  const unsigned lastBlock = g + (myBlocks - 1) * G;
  if (lastBlock == nblk - 1) rows -= nblk * B - H;  // ragged final block
  return rows;
}

// main.cpp:71-76: (unsigned char)(std::min(1.f, c) * 255 / maxColourVal), with
// the reference x86 build's conversion: 32-bit truncation (cvttss2si, INT_MIN
// for NaN or out of range), low byte kept.
RTG_HDI unsigned char ppm_byte(float c, float mx) {
  const float m = (c < 1.f) ? c : 1.f;
  const float v = m * 255 / mx;
  int32_t i;
  if (v > -2147483649.0f && v < 2147483648.0f) i = (int32_t)v;
  else i = INT32_MIN;
  return (unsigned char)(i & 0xFF);
}

#if defined(__HIPCC__)
// Restores the caller's current HIP device when an ABI entry point returns:
// the entry points call hipSetDevice for their context's device, and a torch
// (or any HIP) caller must not find its later allocations and launches moved
// to another GPU.
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};
#endif

}  // namespace rtg
