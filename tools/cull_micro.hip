// tools/cull_micro.hip — what a C2-sized cull pass costs before it does any
// work: kernels of the cull pass's shape (1158 workgroups x 256 threads, or
// the same groups in 1024-thread workgroups), stripped down step by step, each
// timed over 200 back-to-back launches with HIP events (the kernel-to-kernel
// gaps are part of what a frame pays).
//   hipcc -O3 --offload-arch=gfx950 tools/cull_micro.hip -o /tmp/cull_micro && /tmp/cull_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

struct Big {  // a kernel-argument block the size of KernelArgs (304 bytes)
  float* dst;
  unsigned* cnt;
  unsigned* list;
  unsigned* cost;
  unsigned long long n;
  unsigned pad[66];
};

__global__ __launch_bounds__(256) void k_empty(Big a) {
  if (threadIdx.x == 999) a.dst[0] = 1.f;
}

// one 4-byte load per lane (a cost table), one LDS barrier
__global__ __launch_bounds__(256) void k_load(Big a) {
  const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
  __shared__ unsigned s[256];
  s[threadIdx.x] = g < a.n ? a.cost[g] : 0u;
  __syncthreads();
  if (s[255 - threadIdx.x] == 0xFFFFFFFFu) a.dst[0] = 1.f;
}

// + one atomic per workgroup on a shared counter, a second barrier, a store
__global__ __launch_bounds__(256) void k_atomic(Big a) {
  const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
  __shared__ unsigned s[256];
  __shared__ unsigned base;
  const unsigned v = g < a.n ? a.cost[g] : 0u;
  s[threadIdx.x] = v;
  __syncthreads();
  if (threadIdx.x == 0) base = atomicAdd(a.cnt, 37u);
  __syncthreads();
  if ((v & 7u) == 0u && g < a.n) a.list[(base + threadIdx.x) % a.n] = (unsigned)g;
}

// the same with the counter spread over S cache lines (block b on line b % S)
template <unsigned S>
__global__ __launch_bounds__(256) void k_atomicS(Big a) {
  const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
  __shared__ unsigned s[256];
  __shared__ unsigned base;
  const unsigned v = g < a.n ? a.cost[g] : 0u;
  s[threadIdx.x] = v;
  __syncthreads();
  if (threadIdx.x == 0) base = atomicAdd(a.cnt + 32 * (blockIdx.x % S), 37u);
  __syncthreads();
  if ((v & 7u) == 0u && g < a.n) a.list[(base + threadIdx.x) % a.n] = (unsigned)g;
}

// one-address atomic, 1024-thread workgroups (a quarter of the atomics)
__global__ __launch_bounds__(1024) void k_atomic1k(Big a) {
  const size_t g = (size_t)blockIdx.x * 1024 + threadIdx.x;
  __shared__ unsigned base;
  const unsigned v = g < a.n ? a.cost[g] : 0u;
  __syncthreads();
  if (threadIdx.x == 0) base = atomicAdd(a.cnt, 37u);
  __syncthreads();
  if ((v & 7u) == 0u && g < a.n) a.list[(base + threadIdx.x) % a.n] = (unsigned)g;
}

// one-address atomic without a returned value, no list store
__global__ __launch_bounds__(256) void k_atomic_noret(Big a) {
  const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
  const unsigned v = g < a.n ? a.cost[g] : 0u;
  __syncthreads();
  if (threadIdx.x == 0) (void)atomicAdd(a.cnt, 37u + v);
}

// + zero-fill of 21 floats per group, coalesced per wave (the cull's fill)
__global__ __launch_bounds__(256) void k_fill(Big a) {
  const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
  const unsigned lane = threadIdx.x & 63u;
  const size_t wg0 = g - lane;
  if (wg0 < a.n) {
    const size_t q0 = wg0 * 21, q1e = (wg0 + 64) * 21, lim = a.n * 21;
    const size_t q1 = q1e < lim ? q1e : lim;
    for (size_t q = q0 + lane; q < q1; q += 64) a.dst[q] = 0.f;
  }
}

// the fill as wide stores: 4 floats per lane per step
__global__ __launch_bounds__(256) void k_fill4(Big a) {
  const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
  const unsigned lane = threadIdx.x & 63u;
  const size_t wg0 = g - lane;
  if (wg0 < a.n) {
    // the wave's span [wg0 * 21, (wg0 + 64) * 21) floats: 1344 floats = 336 float4
    // when 16-byte aligned (wg0 multiple of 64: 64 * 21 * 4 bytes = 5376, a multiple of 16)
    const size_t q0 = wg0 * 21, q1e = (wg0 + 64) * 21, lim = a.n * 21;
    const size_t q1 = q1e < lim ? q1e : lim;
    float4* d4 = (float4*)(a.dst + q0);
    const size_t n4 = (q1 - q0) / 4;
    for (size_t q = lane; q < n4; q += 64) d4[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (size_t q = q0 + n4 * 4 + lane; q < q1; q += 64) a.dst[q] = 0.f;
  }
}

template <class F>
static float time_it(F launch, hipStream_t st, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) launch();
  CK(hipStreamSynchronize(st));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1, st));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ms * 1000.f / reps;
}

int main() {
  const unsigned long long n = 296229;  // C2's pixel groups
  Big a{};
  a.n = n;
  CK(hipMalloc(&a.dst, n * 21 * sizeof(float)));
  CK(hipMalloc(&a.cnt, 32 * 32 * 4));
  CK(hipMalloc(&a.list, n * sizeof(unsigned)));
  CK(hipMalloc(&a.cost, n * sizeof(unsigned)));
  CK(hipMemset(a.cost, 0, n * sizeof(unsigned)));
  CK(hipMemset(a.cnt, 0, 32 * 32 * 4));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const unsigned blocks = (unsigned)((n + 255) / 256);
  const int reps = 200;
  printf("blocks %u x 256 threads, n %llu, %d launches each\n", blocks, n, reps);
  printf("empty            %7.2f us\n", time_it([&] { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, st, a); }, st, reps));
  printf("load+barrier     %7.2f us\n", time_it([&] { hipLaunchKernelGGL(k_load, dim3(blocks), dim3(256), 0, st, a); }, st, reps));
  printf("+atomic+store    %7.2f us\n", time_it([&] { hipLaunchKernelGGL(k_atomic, dim3(blocks), dim3(256), 0, st, a); }, st, reps));
  printf("atomic 8 lines   %7.2f us\n", time_it([&] { hipLaunchKernelGGL(k_atomicS<8>, dim3(blocks), dim3(256), 0, st, a); }, st, reps));
  printf("atomic 32 lines  %7.2f us\n", time_it([&] { hipLaunchKernelGGL(k_atomicS<32>, dim3(blocks), dim3(256), 0, st, a); }, st, reps));
  printf("atomic 1k blocks %7.2f us\n", time_it([&] { hipLaunchKernelGGL(k_atomic1k, dim3((blocks + 3) / 4), dim3(1024), 0, st, a); }, st, reps));
  printf("atomic no-return %7.2f us\n", time_it([&] { hipLaunchKernelGGL(k_atomic_noret, dim3(blocks), dim3(256), 0, st, a); }, st, reps));
  printf("fill (dword)     %7.2f us\n", time_it([&] { hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(256), 0, st, a); }, st, reps));
  printf("fill (dwordx4)   %7.2f us\n", time_it([&] { hipLaunchKernelGGL(k_fill4, dim3(blocks), dim3(256), 0, st, a); }, st, reps));
  printf("memsetAsync 25MB %7.2f us\n", time_it([&] { (void)hipMemsetAsync(a.dst, 0, n * 21 * sizeof(float), st); }, st, reps));
  printf("empty x2 (pair)  %7.2f us\n", time_it([&] {
    hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, st, a); }, st, reps));
  printf("empty 1 block    %7.2f us\n", time_it([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, a); }, st, reps));
  CK(hipStreamSynchronize(st));
  return 0;
}
