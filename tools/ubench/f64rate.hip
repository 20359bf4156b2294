// tools/ubench/f64rate.hip — microbenchmark: issue rates of the f64 and
// conversion instructions of refraction's f64 islands (rtg_trace.h
// sqrt_d_unit, div_d_fresnel) against v_fma_f32 on gfx950: 8 independent
// chains per lane, full occupancy.  Prints instruction-lanes per second and
// each op's cost in v_fma_f32 issue slots.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define KERNEL_F32(name, ins)                                                           \
  __global__ __launch_bounds__(256) void name(float* out, int iters, float a) {         \
    float x[8];                                                                         \
    for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 0.001f + k + 1.0f;                 \
    for (int i = 0; i < iters; ++i) {                                                   \
      _Pragma("unroll") for (int k = 0; k < 8; ++k) asm volatile(ins : "+v"(x[k]) : "v"(a)); \
    }                                                                                   \
    float s = 0;                                                                        \
    for (int k = 0; k < 8; ++k) s += x[k];                                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                     \
  }
#define KERNEL_F64(name, ins)                                                           \
  __global__ __launch_bounds__(256) void name(float* out, int iters, float a) {         \
    double x[8];                                                                        \
    const double ad = a;                                                                \
    for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 0.001 + k + 1.0;                   \
    for (int i = 0; i < iters; ++i) {                                                   \
      _Pragma("unroll") for (int k = 0; k < 8; ++k) asm volatile(ins : "+v"(x[k]) : "v"(ad)); \
    }                                                                                   \
    double s = 0;                                                                       \
    for (int k = 0; k < 8; ++k) s += x[k];                                              \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s;                              \
  }

KERNEL_F32(k_fma32, "v_fma_f32 %0, %0, %1, %1")
KERNEL_F32(k_rcp32, "v_rcp_f32 %0, %0")
KERNEL_F32(k_rsq32, "v_rsq_f32 %0, %0")
KERNEL_F64(k_fma64, "v_fma_f64 %0, %0, %1, %1")
KERNEL_F64(k_mul64, "v_mul_f64 %0, %0, %1")
KERNEL_F64(k_rcp64, "v_rcp_f64 %0, %0")
KERNEL_F64(k_rsq64, "v_rsq_f64 %0, %0")

// conversions f32 <-> f64 in place: x (f64 pair) -> f32 in the low half -> back
__global__ __launch_bounds__(256) void k_cvt(float* out, int iters, float a) {
  double x[8];
  for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 0.001 + k + 1.0 + a;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      asm volatile("v_cvt_f32_f64 %0, %1\n\tv_cvt_f64_f32 %1, %0"
                   : "=&v"(a), "+v"(x[k]));
  }
  double s = 0;
  for (int k = 0; k < 8; ++k) s += x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (float)s;
}

typedef void (*Fn)(float*, int, float);

int main() {
  const int blocks = 256 * 8 * 4, threads = 256, iters = 2048;
  float* d;
  hipMalloc(&d, (size_t)blocks * threads * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct { const char* name; Fn fn; int per; } ks[] = {
      {"v_fma_f32", k_fma32, 1}, {"v_rcp_f32", k_rcp32, 1}, {"v_rsq_f32", k_rsq32, 1},
      {"v_fma_f64", k_fma64, 1}, {"v_mul_f64", k_mul64, 1}, {"v_rcp_f64", k_rcp64, 1},
      {"v_rsq_f64", k_rsq64, 1}, {"cvt f64->f32->f64 (2 instr)", k_cvt, 2}};
  double base = 0;
  for (int rep = 0; rep < 2; ++rep) {
    for (auto& k : ks) {
      float ms;
      hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0001f);
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0001f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
      const double lanes = (double)blocks * threads * iters * 8 * k.per;
      const double rate = lanes / ms / 1e9;  // T instr-lanes/s
      if (k.fn == k_fma32) base = rate;
      if (rep == 1)
        printf("%-28s %.3f ms  %6.1f T instr-lanes/s  %.2f v_fma_f32 slots each\n", k.name, ms,
               rate, base / rate);
    }
  }
  hipFree(d);
  return 0;
}
