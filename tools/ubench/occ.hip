// tools/ubench/occ.hip — resident-wave ceiling of one-wave workgroups on one
// SIMD: each wave records {start, end (s_memrealtime), HW_ID}; the host takes
// the peak number of waves whose [start, end) overlap on any SIMD.  Cases:
// plain, with 192 B/lane of dynamically indexed private memory (scratch), and
// with 5 KB of dynamic LDS, at <= 64 VGPRs.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <map>
#include <vector>

template <bool kScratch, int kSgpr = 0>
__global__ __launch_bounds__(64) void occ(uint4* rec, int spin, int idx) {
  extern __shared__ float lds[];
  // kSgpr: raise the kernel's SGPR count (clobbers) to test an SGPR ceiling
  if constexpr (kSgpr == 80) asm volatile("" ::: "s70", "s71", "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79");
  if constexpr (kSgpr == 88) asm volatile("" ::: "s80", "s81", "s82", "s83", "s84", "s85", "s86", "s87");
  if constexpr (kSgpr == 94) asm volatile("" ::: "s88", "s89", "s90", "s91", "s92", "s93");
  if constexpr (kSgpr == 100) asm volatile("" ::: "s94", "s95", "s96", "s97", "s98", "s99");
  const unsigned t0 = (unsigned)__builtin_amdgcn_s_memrealtime();
  float acc = (float)threadIdx.x;
  float priv[48];
  if (kScratch) {
#pragma unroll
    for (int k = 0; k < 48; ++k) priv[k] = acc + k;
  }
  for (int i = 0; i < spin; ++i) {
    acc = acc * 1.0000001f + 0.5f;
    if (kScratch) priv[(i + idx) % 48] += acc;
  }
  if (kScratch) acc += priv[idx % 48];
  lds[threadIdx.x] = acc;
  const unsigned t1 = (unsigned)__builtin_amdgcn_s_memrealtime();
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);
  if (threadIdx.x == 0) rec[blockIdx.x] = make_uint4(t0, t1, hw, xcc + (acc == 12345.f));
}

static void run(const char* name, void (*k)(uint4*, int, int), size_t lds, int spin) {
  const int n = 256 * 4 * 8 * 6;
  uint4* d;
  if (hipMalloc(&d, n * sizeof(uint4)) != hipSuccess) exit(1);
  hipLaunchKernelGGL(k, dim3(n), dim3(64), lds, 0, d, spin, 7);
  hipLaunchKernelGGL(k, dim3(n), dim3(64), lds, 0, d, spin, 7);
  if (hipDeviceSynchronize() != hipSuccess) exit(2);
  std::vector<uint4> h(n);
  hipMemcpy(h.data(), d, n * sizeof(uint4), hipMemcpyDeviceToHost);
  hipFree(d);
  std::map<unsigned, std::vector<std::pair<long, int>>> ev;
  for (auto& r : h) {
    const unsigned hw = r.z, x = r.w;
    const unsigned key = ((((x & 15) * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 16 +
                          ((hw >> 8) & 15)) * 4 + ((hw >> 4) & 3);
    long a = r.x, b = r.y;
    if (b < a) b += (1L << 32);
    ev[key].push_back({a, 1});
    ev[key].push_back({b, -1});
  }
  int peakMax = 0;
  double peakMean = 0;
  for (auto& kv : ev) {
    auto& e = kv.second;
    std::sort(e.begin(), e.end(), [](auto& p, auto& q) {
      return p.first < q.first || (p.first == q.first && p.second < q.second);
    });
    int cur = 0, pk = 0;
    for (auto& p : e) { cur += p.second; pk = std::max(pk, cur); }
    peakMax = std::max(peakMax, pk);
    peakMean += pk;
  }
  printf("%-10s simds %zu  peak resident waves per SIMD: max %d mean %.2f\n", name, ev.size(),
         peakMax, peakMean / ev.size());
}

int main() {
  const int spin = 20000;
  run("plain", occ<false>, 256, spin);
  run("scratch", occ<true>, 256, spin);
  run("lds5k", occ<false>, 5120, spin);
  run("scr+lds5k", occ<true>, 5120, spin);
  run("sgpr80", occ<false, 80>, 256, spin);
  run("sgpr88", occ<false, 88>, 256, spin);
  run("sgpr94", occ<false, 94>, 256, spin);
  run("sgpr100", occ<false, 100>, 256, spin);
  return 0;
}
