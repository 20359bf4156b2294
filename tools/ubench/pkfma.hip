// tools/ubench/pkfma.hip — microbenchmark: issue rate of v_pk_fma_f32 (two
// f32 FMAs per lane) against v_fma_f32 on gfx950, 8 independent chains per
// lane, full occupancy.  Prints FMA lane-ops per second for both.
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float float2v __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_fma(float* out, int iters, float a, float b) {
  float x[8];
  for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 0.001f + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x[k]) : "v"(a), "v"(b));
  }
  float s = 0;
  for (int k = 0; k < 8; ++k) s += x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_pkfma(float* out, int iters, float a, float b) {
  float2v x[8];
  float2v av = {a, a}, bv = {b, b};
  for (int k = 0; k < 8; ++k) x[k] = float2v{threadIdx.x * 0.001f + k, (float)k};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x[k]) : "v"(av), "v"(bv));
  }
  float s = 0;
  for (int k = 0; k < 8; ++k) s += x[k].x + x[k].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_add(float* out, int iters, float a, float b) {
  float x[8];
  for (int k = 0; k < 8; ++k) x[k] = threadIdx.x * 0.001f + k;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x[k]) : "v"(a));
  }
  float s = 0;
  for (int k = 0; k < 8; ++k) s += x[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  const int blocks = 256 * 8 * 4, threads = 256, iters = 4096;
  float* d;
  hipMalloc(&d, (size_t)blocks * threads * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep) {
    float ms;
    hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0001f, 0.5f);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0001f, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    const double lanes = (double)blocks * threads * iters * 8;
    printf("v_fma_f32     : %.3f ms, %.1f T instr-lanes/s\n", ms, lanes / ms / 1e9);
    hipLaunchKernelGGL(k_pkfma, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0001f, 0.5f);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_pkfma, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0001f, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("v_pk_fma_f32  : %.3f ms, %.1f T instr-lanes/s (x2 FMAs each)\n", ms, lanes / ms / 1e9);
    hipLaunchKernelGGL(k_add, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0001f, 0.5f);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_add, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0001f, 0.5f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("v_add_f32     : %.3f ms, %.1f T instr-lanes/s\n", ms, lanes / ms / 1e9);
  }
  hipFree(d);
  return 0;
}
