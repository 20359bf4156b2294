// rtg_kernel.hip — CDNA4 (gfx950) kernels and the device half of the C ABI.
//
// Replaces the OpenCL kernel `raytrace` (raytrace_kernel.cl:870-973) and its
// host orchestration (main.cpp:277-363, 456-468), computing the reference CPU
// path's framebuffer (raytracer.h) bit for bit; see rtg_trace.h for the
// traversal and DESIGN.md for the layout and roofline.
//
// Launch geometry: one work-item per pixel; a 256-thread workgroup covers a
// 16x16 pixel tile and each 64-lane wave an 8x8 sub-tile, so the rays of a
// wave are spatially coherent and take similar paths through the Whitted tree.
// The sphere loop index is wave-uniform, so sphere records are read with
// scalar loads into SGPRs (no VGPRs, no LDS traffic); per-lane material
// lookups (the hit sphere / refractive medium) come from an LDS copy of the
// material table staged once per workgroup.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>
#include <vector>

#include "rtg.h"
#include "rtg_internal.h"
#include "rtg_trace.h"
#include "rtg_scene_pack.h"

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) {                                                        \
      rtg_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                    __LINE__);                                                     \
      return RTG_ERR_HIP;                                                          \
    }                                                                              \
  } while (0)

namespace rtg {

constexpr int kBlock = 256;
// Materials staged in LDS when the table fits (n+1 records of 32 B).
constexpr unsigned kLdsMatMax = 1024 + 1;  // => <= 48 KiB of LDS per workgroup

// Device scene: geometry SoA-ish float4 {x, y, z, r*r}, (r + 1e-6f)^2, the
// material table (n+1 x 8 floats; [n] = background), lights (m x 6 floats).
// Read-only scene arrays are accessed through the constant address space
// (addrspace 4): with a wave-uniform index the loads become s_load into SGPRs.
#if defined(__HIP_DEVICE_COMPILE__)
#define RTG_CONST __attribute__((address_space(4)))
#else
#define RTG_CONST
#endif
typedef const RTG_CONST float* cfloat_p;

// Per-lane frame colours in LDS: level lv of thread t at lfr[lv * kBlock + t]
// (16-byte records, so a wave's ds_read_b128 covers 1 KiB contiguously and is
// bank-conflict free).
template <int kThreads>
struct LdsFrames {
  FrameC* base;  // already offset by threadIdx.x
  __device__ __forceinline__ FrameC& operator()(int lv) const { return base[lv * kThreads]; }
};

template <class MatPtr, bool kDiag = false, int kThreads = kBlock>
struct DevScene {
  FrameC* lfr;
  __device__ __forceinline__ bool all(bool b) const { return __ballot(!b) == 0ull; }
  __device__ __forceinline__ LdsFrames<kThreads> frames() const {
    return LdsFrames<kThreads>{lfr};
  }
  // Diagnostic cycle accounting (kDiag builds only): s_memtime deltas per
  // probe slot, summed per wave and added to KernelArgs::diag at exit.
  mutable unsigned long long acc[kProbeSlots];
  mutable unsigned long long t0[kProbeSlots];
  __device__ __forceinline__ void probe_begin(int slot) const {
    if constexpr (kDiag) {
      __builtin_amdgcn_sched_barrier(0);
      t0[slot] = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __device__ __forceinline__ void probe_end(int slot) const {
    if constexpr (kDiag) {
      __builtin_amdgcn_sched_barrier(0);
      acc[slot] += __builtin_amdgcn_s_memtime() - t0[slot];
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  cfloat_p geom;      // n x {x, y, z, r*r}
  cfloat_p crad2;
  MatPtr mats;        // LDS copy (float*) or the global table (cfloat_p)
  const float4* lgeom;  // LDS copy of geom (or the global array when it does not fit)
  cfloat_p lights;
  unsigned n, m;
  unsigned n4;  // geometry records incl. NaN padding to a multiple of 4

  __device__ __forceinline__ V3 sphere(unsigned i, float& r2) const {
    cfloat_p g = geom + 4 * i;
    r2 = g[3];
    return v3(g[0], g[1], g[2]);
  }
  // Four consecutive sphere records: one 64-byte scalar load.
  __device__ __forceinline__ void sphere4(unsigned i, V3* c, float* r2) const {
    cfloat_p g = geom + 4 * i;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c[k] = v3(g[4 * k + 0], g[4 * k + 1], g[4 * k + 2]);
      r2[k] = g[4 * k + 3];
    }
  }
  // Per-lane sphere record (divergent index): from the LDS copy.
  __device__ __forceinline__ V3 sphere_lane(unsigned i, float& r2) const {
    const float4 g = lgeom[i];
    r2 = g.w;
    return v3(g.x, g.y, g.z);
  }
  __device__ __forceinline__ float contain_r2(unsigned i) const { return crad2[i]; }
  // |0 - c_i|^2 - r_i^2: the c term of a ray from the origin (primary rays)
  __device__ __forceinline__ float origin_c(unsigned i) const { return crad2[n + i]; }
  __device__ __forceinline__ Mat mat(int i) const {
    const auto p = mats + 8 * i;
    Mat r;
    r.matte = v3(p[0], p[1], p[2]);
    r.gloss = v3(p[3], p[4], p[5]);
    r.opacity = p[6];
    r.refr = p[7];
    return r;
  }
  __device__ __forceinline__ float refr(int i) const { return mats[8 * i + 7]; }
  __device__ __forceinline__ void light(unsigned l, V3& pos, V3& col) const {
    cfloat_p p = lights + 6 * l;
    pos = v3(p[0], p[1], p[2]);
    col = v3(p[3], p[4], p[5]);
  }
};

struct KernelArgs;
typedef void (*TraceFn)(const KernelArgs);

struct KernelArgs {
  const float4* geom;
  const float* crad2;
  const float* mats;
  const float* lights;
  unsigned n, m, n4;
  Camera cam;
  unsigned W, rowsLocal, rowBlock, shard, nShards;
  const unsigned* rowList;  // explicit global rows (rtg_render_rows_device) or null
  float* dst;
  unsigned long long* diag;  // kProbeSlots counters (diagnostic variants only)
  uint4* timeline;           // per-wave records (RTG_LAUNCH_TIMELINE) or null
};

__device__ __forceinline__ float canon_nan(float v) {
  // x86 default NaN, what the reference CPU path writes (see rtg.h).
  return (v != v) ? __uint_as_float(0xFFC00000u) : v;
}

// Minimum waves per SIMD requested from the register allocator: 7 (<= 72
// VGPRs) where the LDS image of S-1 frame levels still admits 7 waves per
// SIMD (S <= 6 with a small scene); measured +1-2 % over the unconstrained
// 78-VGPR build at 6 waves/SIMD (C3, tile kernel).
template <int S, int kVariant>
struct MinWaves {
  static constexpr int value =
      ((kVariant % 100 == 0 || kVariant % 100 == 9 || kVariant >= 14) && S <= 6) ? 7 : 1;
};

// Workgroup prologue: the frame area and (kLds) the scene tables staged in LDS.
template <int S, bool kLds, int kThreads, class Sc>
__device__ __forceinline__ void stage_scene(const KernelArgs& a, Sc& sc) {
  extern __shared__ float4 lds4[];
  constexpr int NF = (S > 1) ? (S - 1) : 1;
  sc.lfr = reinterpret_cast<FrameC*>(lds4) + threadIdx.x;
  float4* sceneLds = lds4 + NF * kThreads;
  if constexpr (kLds) {
    float* lmats = reinterpret_cast<float*>(sceneLds);
    const unsigned nm = (a.n + 1) * 8;
    for (unsigned i = threadIdx.x; i < nm; i += kThreads) lmats[i] = a.mats[i];
    float4* lg = sceneLds + (a.n + 1) * 2;
    for (unsigned i = threadIdx.x; i < a.n4; i += kThreads)
      lg[i] = reinterpret_cast<const float4*>(a.geom)[i];
    __syncthreads();
    sc.mats = lmats;
    sc.lgeom = lg;
  } else {
    sc.mats = (cfloat_p)a.mats;
    sc.lgeom = reinterpret_cast<const float4*>(a.geom);
  }
  sc.geom = (cfloat_p)a.geom;
  sc.crad2 = (cfloat_p)a.crad2;
  sc.lights = (cfloat_p)a.lights;
  sc.n = a.n;
  sc.m = a.m;
  sc.n4 = a.n4;
}

// One 8 x 8 pixel tile per wave: tile (tx, ty) of the shard's local rows.
// Entered with the whole wave converged.
template <int S, int kVariant, class Sc>
__device__ __forceinline__ void trace_tile(const KernelArgs& a, Sc& sc, unsigned tx,
                                           unsigned ty) {
  constexpr bool kDiag = kVariant >= 100;
  constexpr int kBase = kDiag ? kVariant - 100 : kVariant;
  const unsigned lane = threadIdx.x & 63u;
  const unsigned x = tx * 8u + (lane & 7u);
  const unsigned lr = ty * 8u + (lane >> 3);
  const bool valid = x < a.W && lr < a.rowsLocal;
  const unsigned gy = !valid ? 0u
                     : a.rowList ? a.rowList[lr]
                                 : shard_global_row(lr, a.rowBlock, a.shard, a.nShards);

  // Primary-ray sphere cull for this wave (whole wave converged here): the
  // bounds of every sample direction of the wave's pixels, then one sphere
  // per lane against that bundle, then a ballot (see primary_sphere_possible).
  uint64_t primSel = ~0ull;
  bool usePrim = false;
  if constexpr (kBase == 0 || kBase == 8 || kBase == 9) {
    if (a.n <= 64) {
      float x0 = 3.0e38f, x1 = -3.0e38f, y0 = 3.0e38f, y1 = -3.0e38f;
      if (valid) primary_bounds(a.cam, x, gy, x0, x1, y0, y1);
      for (int off = 32; off > 0; off >>= 1) {
        x0 = fminf(x0, __shfl_xor(x0, off));
        x1 = fmaxf(x1, __shfl_xor(x1, off));
        y0 = fminf(y0, __shfl_xor(y0, off));
        y1 = fmaxf(y1, __shfl_xor(y1, off));
      }
      bool possible = false;
      if (lane < a.n) {
        const float4 g = sc.lgeom[lane];
        possible = primary_sphere_possible(v3(g.x, g.y, g.z), sqrtf(g.w), x0, x1, y0, y1,
                                           a.cam.zoom);
      }
      primSel = __ballot(possible);
      usePrim = true;
    }
  }
  if (!valid) return;
  V3 pix;
  unsigned long long tk0 = 0;
  if constexpr (kDiag) {
    for (int k = 0; k < kProbeSlots; ++k) sc.acc[k] = 0;
    tk0 = __builtin_amdgcn_s_memtime();
  }
  if constexpr (kBase == 0 || kBase == 9)
    pix = shade_pixel<S, 2, true>(sc, a.cam, x, gy, usePrim, primSel);
  else if constexpr (kBase == 6) pix = shade_pixel<S, 2, true>(sc, a.cam, x, gy);
  else if constexpr (kBase == 8) pix = shade_pixel<S, 3, true>(sc, a.cam, x, gy, usePrim, primSel);
  else if constexpr (kBase == 5) pix = shade_pixel<S, 2, false>(sc, a.cam, x, gy);
  else if constexpr (kBase == 1) pix = shade_pixel<S, 0>(sc, a.cam, x, gy);
  else if constexpr (kBase == 2) pix = shade_pixel_persistent<S, 2>(sc, a.cam, x, gy);
  else if constexpr (kBase == 3) pix = shade_pixel_persistent<S, 1>(sc, a.cam, x, gy);
  else pix = shade_pixel_nodes<S, 2>(sc, a.cam, x, gy);
  if constexpr (kDiag) {
    sc.acc[kProbeTotal] = __builtin_amdgcn_s_memtime() - tk0;
    // one wave-level add per slot (values are wave-uniform: s_memtime is scalar)
    if ((threadIdx.x & 63u) == (unsigned)__builtin_ctzll(__ballot(1)))
      for (int k = 0; k < kProbeSlots; ++k) atomicAdd(&a.diag[k], sc.acc[k]);
  }
  float* o = a.dst + ((size_t)lr * a.W + x) * 3;
  o[0] = canon_nan(pix.x);
  o[1] = canon_nan(pix.y);
  o[2] = canon_nan(pix.z);
}

// Timeline record of one wave (launch flag RTG_LAUNCH_TIMELINE): start/end
// s_memrealtime (100 MHz), HW_ID (hwreg 4) and XCC_ID (hwreg 20).  Called
// with the wave converged.
__device__ __forceinline__ void record_wave(const KernelArgs& a, unsigned t0, size_t w) {
  if (a.timeline == nullptr) return;
  const unsigned t1 = (unsigned)__builtin_amdgcn_s_memrealtime();
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);
  if ((threadIdx.x & 63u) == 0) a.timeline[w] = make_uint4(t0, t1, hw, xcc);
}

// Tile kernels: one 8 x 8 pixel tile per wave, all samples of a pixel in its
// lane; a workgroup is 2 x 2 tiles.
template <int S, bool kLds, int kVariant>
__global__ __launch_bounds__(kBlock, (MinWaves<S, kVariant>::value))
void trace_kernel(const KernelArgs a) {
  // LDS image: per-lane frame colours ((S-1) x threads x 16 B), then, when
  // kLds, the material table (n+1) x 8 floats and the geometry n x float4.
  constexpr int kThreads = kBlock;
  constexpr unsigned TW = 2u, TH = 2u;
  typedef typename std::conditional<kLds, const float*, cfloat_p>::type MatPtr;
  DevScene<MatPtr, (kVariant >= 100), kThreads> sc;
  stage_scene<S, kLds, kThreads>(a, sc);
  const unsigned wave = threadIdx.x >> 6;
  const unsigned t0 = (unsigned)__builtin_amdgcn_s_memrealtime();
  trace_tile<S, kVariant>(a, sc, blockIdx.x * TW + (wave % TW), blockIdx.y * TH + (wave / TW));
  record_wave(a, t0, ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * (kThreads / 64) + wave);
}

// Sample-parallel form (variant 14): each lane traces ONE primary sample, so
// a wave takes floor(64 / nAA^2) consecutive pixels (7 at 3 x 3) with their
// samples in lane order, instead of 64 pixels x all their samples.  A heavy
// region (deep refraction trees) is then spread over nAA^2 times as many
// waves, which keeps the frame's last waves short (the default kernel's
// 8 x 8 tiles of 9 samples ran up to 3 ms each on C3), and a
// wave's primary-ray bundle is a few pixels wide, so the cull is tighter.
// Each pixel's sum is formed in the reference's sample order
// (main.cpp:411-452: pix += c_s * inv for s = 0 .. nAA^2-1) by its first lane
// from the other lanes' values (ds_bpermute moves the bits unchanged).
// Requires nAA^2 <= 64; the host launches the default kernel otherwise.
// Pixel group gw (floor(64 / nAA^2) consecutive pixels of the shard's local
// rows, all their samples) traced by one wave, entered converged.
template <int S, class Sc>
__device__ __forceinline__ void trace_group(const KernelArgs& a, Sc& sc, size_t gw) {
  const unsigned lane = threadIdx.x & 63u;
  const unsigned nAA = (unsigned)a.cam.nAA;
  const unsigned SP = nAA * nAA;
  const unsigned PPW = 64u / SP;
  const unsigned pl = lane / SP, s = lane - pl * SP;
  const size_t p = gw * PPW + pl;
  const size_t total = (size_t)a.W * a.rowsLocal;
  const bool valid = pl < PPW && p < total;
  unsigned x = 0, lr = 0, gy = 0;
  if (valid) {
    if (total <= 0xFFFFFFFFull) {  // wave-uniform: 32-bit division
      lr = (unsigned)p / a.W;
      x = (unsigned)p - lr * a.W;
    } else {
      lr = (unsigned)(p / a.W);
      x = (unsigned)(p - (size_t)lr * a.W);
    }
    gy = a.rowList ? a.rowList[lr] : shard_global_row(lr, a.rowBlock, a.shard, a.nShards);
  }
  const int si = (int)(s / nAA), sj = (int)(s - (unsigned)si * nAA);
  float rx, ry;
  const V3 dir = sample_dir(a.cam, x, gy, si, sj, rx, ry);

  // Primary-ray cull over the wave's sample directions (wave converged).
  uint64_t primSel = ~0ull;
  bool usePrim = false;
  if (a.n <= 64) {
    float x0 = valid ? rx : 3.0e38f, x1 = valid ? rx : -3.0e38f;
    float y0 = valid ? ry : 3.0e38f, y1 = valid ? ry : -3.0e38f;
    for (int off = 32; off > 0; off >>= 1) {
      x0 = fminf(x0, __shfl_xor(x0, off));
      x1 = fmaxf(x1, __shfl_xor(x1, off));
      y0 = fminf(y0, __shfl_xor(y0, off));
      y1 = fmaxf(y1, __shfl_xor(y1, off));
    }
    bool possible = false;
    if (lane < a.n) {
      const float4 g = sc.lgeom[lane];
      possible = primary_sphere_possible(v3(g.x, g.y, g.z), sqrtf(g.w), x0, x1, y0, y1,
                                         a.cam.zoom);
    }
    primSel = __ballot(possible);
    usePrim = true;
  }
  V3 c = v3(0.f, 0.f, 0.f);
  if (valid) {
    c = trace_sample<S, 2>(sc, dir, sc.frames(), usePrim, primSel);
    c = vsmul(a.cam.inv, c);
  }
  // Ordered per-pixel sum (whole wave converged again).
  const unsigned base = pl * SP;
  V3 pix = v3(0.f, 0.f, 0.f);
  for (unsigned k = 0; k < SP; ++k) {
    const int src = (int)((base + k) & 63u);
    pix.x = pix.x + __shfl(c.x, src);
    pix.y = pix.y + __shfl(c.y, src);
    pix.z = pix.z + __shfl(c.z, src);
  }
  if (valid && s == 0) {
    float* o = a.dst + ((size_t)lr * a.W + x) * 3;
    o[0] = canon_nan(pix.x);
    o[1] = canon_nan(pix.y);
    o[2] = canon_nan(pix.z);
  }
}

template <int kVariant>
struct SampleThreads {
  static constexpr int value = (kVariant == 14) ? kBlock : (kVariant == 16) ? 128 : 64;
};

// One launch, one pixel group per wave: one-wave workgroups (default), or
// four-wave ones (variant 14).
template <int S, bool kLds, int kVariant>
__global__ __launch_bounds__(SampleThreads<kVariant>::value, (MinWaves<S, kVariant>::value))
void trace_samples_kernel(const KernelArgs a) {
  constexpr int kThreads = SampleThreads<kVariant>::value;
  typedef typename std::conditional<kLds, const float*, cfloat_p>::type MatPtr;
  DevScene<MatPtr, false, kThreads> sc;
  const unsigned t0 = (unsigned)__builtin_amdgcn_s_memrealtime();
  stage_scene<S, kLds, kThreads>(a, sc);
  const size_t gw = (size_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  trace_group<S>(a, sc, gw);
  record_wave(a, t0, gw);
}

// algebra.h:68-91 on the device: values are compared as floats (NaN never
// wins), the running max starts at +0 so only positive values can win, and a
// non-negative float orders like its bit pattern, so an integer atomicMax on
// the bits reduces across workgroups.
__global__ __launch_bounds__(256) void max_kernel(const float* __restrict__ c, size_t nval,
                                                  unsigned* __restrict__ out) {
  float mx = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nval;
       i += (size_t)gridDim.x * blockDim.x) {
    const float v = c[i];
    if (v > mx) mx = v;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const float o = __shfl_xor(mx, off);
    if (o > mx) mx = o;
  }
  __shared__ float part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w)
      if (part[w] > mx) mx = part[w];
    atomicMax(out, __float_as_uint(mx));
  }
}

__global__ void max_finish_kernel(unsigned* m) {
  if (__uint_as_float(*m) == 0.f) *m = __float_as_uint(1.f);
}

__global__ __launch_bounds__(256) void ppm_kernel(const float* __restrict__ c, size_t nval,
                                                  const float* __restrict__ mx,
                                                  unsigned char* __restrict__ out) {
  const float m = *mx;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nval;
       i += (size_t)gridDim.x * blockDim.x)
    out[i] = ppm_byte(c[i], m);
}

// Kernel variants (rtg_launch_opts.variant; results identical, speed differs):
//   0 (default) sample-parallel: one primary sample per lane, one-wave
//     workgroups, scene tables read from global memory (trace_samples_kernel);
//     falls back to 9 when nAA > 8
//   1 per-sample recursion, one sphere per step (first kernel)
//   2 one-query-per-iteration state machine + candidate masks
//   3 one-query-per-iteration state machine, four spheres per step
//   4 node-persistent: samples chained in one node loop + candidate masks
//   5 as 9 but frame colours in private memory instead of LDS
//   6 as 9 without the per-wave primary-ray sphere cull
//   (7, a converged loop with per-query bundle culls, was removed: DESIGN.md)
//   8 as 9 with the tuned two-pass query (prefetched groups, uniform quotient path)
//   9 tile kernel: an 8 x 8 pixel tile per wave, each lane all samples of its
//     pixel (per-sample recursion + two-pass candidate-mask queries + per-wave
//     primary cull), 7 waves/SIMD; the default until the sample-parallel kernel
//   14 as 0 with four-wave workgroups
//   15 same kernel as 0 (kept as an alias for A/B scripts)
//   16 as 17 with two-wave workgroups
//   17 as 0 with the materials/geometry staged in LDS per workgroup
//   (10-12: work-queue and workgroup-size trials of the tile kernel, removed: DESIGN.md)
//   100 + v: diagnostic build of v (s_memtime probes, rtg_diag_read); 100 = 9
template <int S, int V>
static TraceFn trace_fn_v(bool lds) {
  if constexpr (V == 14 || V == 16 || V == 17)
    return lds ? trace_samples_kernel<S, true, V> : trace_samples_kernel<S, false, V>;
  else if constexpr (V == 0 || V == 15)
    return trace_samples_kernel<S, false, V>;
  else
    return lds ? trace_kernel<S, true, V> : trace_kernel<S, false, V>;
}
template <int S>
static TraceFn trace_fn(bool lds, int variant) {
  switch (variant) {
    case 100: return trace_fn_v<S, 100>(lds);
    case 104: return trace_fn_v<S, 104>(lds);
    case 1: return trace_fn_v<S, 1>(lds);
    case 4: return trace_fn_v<S, 4>(lds);
    case 5: return trace_fn_v<S, 5>(lds);
    case 6: return trace_fn_v<S, 6>(lds);
    case 8: return trace_fn_v<S, 8>(lds);
    case 9: return trace_fn_v<S, 9>(lds);
    case 14: return trace_fn_v<S, 14>(lds);
    case 15: return trace_fn_v<S, 15>(lds);
    case 16: return trace_fn_v<S, 16>(lds);
    case 17: return trace_fn_v<S, 17>(lds);
    case 108: return trace_fn_v<S, 108>(lds);
    case 2: return trace_fn_v<S, 2>(lds);
    case 3: return trace_fn_v<S, 3>(lds);
    default: return trace_fn_v<S, 0>(lds);
  }
}

static TraceFn pick_trace(int S, bool lds, int variant) {
  switch (S) {
#define RTG_CASE(k) case k: return trace_fn<k>(lds, variant);
    RTG_CASE(1) RTG_CASE(2) RTG_CASE(3) RTG_CASE(4) RTG_CASE(5) RTG_CASE(6) RTG_CASE(7)
    RTG_CASE(8) RTG_CASE(9) RTG_CASE(10) RTG_CASE(11) RTG_CASE(12) RTG_CASE(13)
    RTG_CASE(14) RTG_CASE(15) RTG_CASE(16)
#undef RTG_CASE
    default: return nullptr;
  }
}

}  // namespace rtg

struct rtg_context {
  int device = 0;
  unsigned n = 0, m = 0, n4 = 0;
  float4* geom = nullptr;
  float* crad2 = nullptr;
  float* mats = nullptr;
  float* lights = nullptr;
  unsigned* maxScratch = nullptr;
  unsigned long long* diag = nullptr;  // probe counters of diagnostic variants
  uint4* timeline = nullptr;  // RTG_LAUNCH_TIMELINE records
  size_t timelineCap = 0, timelineCount = 0;
  rtg_launch_opts opts{};
  bool hasScene = false;
};

using namespace rtg;

static void free_scene(rtg_context* c) {
  (void)hipFree(c->geom);
  (void)hipFree(c->crad2);
  (void)hipFree(c->mats);
  (void)hipFree(c->lights);
  c->geom = nullptr;
  c->crad2 = nullptr;
  c->mats = nullptr;
  c->lights = nullptr;
  c->hasScene = false;
}

// Argument checks shared by the one-shot entry points (no HIP call made).
static int check_render_args(const rtg_sphere* spheres, unsigned sphNum, const rtg_light* lights,
                             unsigned lgtNum, unsigned width, unsigned height, float zoom,
                             float aliasFactor, int stackSize, const void* dst) {
  if (!dst) {
    rtg_set_error("render: null destination");
    return RTG_ERR_INVALID;
  }
  if ((sphNum && !spheres) || (lgtNum && !lights)) {
    rtg_set_error("render: null scene array");
    return RTG_ERR_INVALID;
  }
  if (stackSize < 1 || stackSize > RTG_MAX_STACK) {
    rtg_set_error("stackSize %d outside [1, %d]", stackSize, RTG_MAX_STACK);
    return RTG_ERR_INVALID;
  }
  Camera cam;
  return make_camera(width, height, zoom, aliasFactor, &cam);
}

extern "C" {

int rtg_device_count(int* count) {
  rtg_clear_error();
  if (!count) return RTG_ERR_INVALID;
  HIP_TRY(hipGetDeviceCount(count));
  return RTG_OK;
}

int rtg_device_info(int device, char* buf, size_t buflen) {
  rtg_clear_error();
  if (!buf || buflen == 0) return RTG_ERR_INVALID;
  hipDeviceProp_t p;
  HIP_TRY(hipGetDeviceProperties(&p, device));
  snprintf(buf, buflen, "%s (%s), %d CUs, %d MHz, %.1f GiB, LDS/block %zu KiB", p.name,
           p.gcnArchName, p.multiProcessorCount, p.clockRate / 1000,
           (double)p.totalGlobalMem / (1024.0 * 1024.0 * 1024.0),
           (size_t)p.sharedMemPerBlock / 1024);
  return RTG_OK;
}

int rtg_context_create(int device, rtg_context** out) {
  rtg_clear_error();
  if (!out) return RTG_ERR_INVALID;
  *out = nullptr;
  int cnt = 0;
  HIP_TRY(hipGetDeviceCount(&cnt));
  if (device < 0 || device >= cnt) {
    rtg_set_error("device %d not present (%d devices)", device, cnt);
    return RTG_ERR_NODEVICE;
  }
  HIP_TRY(hipSetDevice(device));
  rtg_context* c = new rtg_context();
  c->device = device;
  if (const char* v = getenv("RTG_VARIANT")) c->opts.variant = atoi(v);  // A/B knob
  if (hipMalloc(&c->maxScratch, 4) != hipSuccess) {
    delete c;
    rtg_set_error("hipMalloc failed");
    return RTG_ERR_NOMEM;
  }
  *out = c;
  return RTG_OK;
}

int rtg_context_destroy(rtg_context* ctx) {
  rtg_clear_error();
  if (!ctx) return RTG_OK;
  (void)hipSetDevice(ctx->device);
  free_scene(ctx);
  (void)hipFree(ctx->maxScratch);
  (void)hipFree(ctx->diag);
  (void)hipFree(ctx->timeline);
  delete ctx;
  return RTG_OK;
}

int rtg_diag_read(rtg_context* ctx, unsigned long long* out, int reset) {
  rtg_clear_error();
  if (!ctx || !out) return RTG_ERR_INVALID;
  if (!ctx->diag) {
    for (int k = 0; k < 8; ++k) out[k] = 0;
    return RTG_OK;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, ctx->diag, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  if (reset) HIP_TRY(hipMemset(ctx->diag, 0, 8 * sizeof(unsigned long long)));
  return RTG_OK;
}

int rtg_diag_timeline(rtg_context* ctx, unsigned* out4, size_t cap, size_t* count) {
  rtg_clear_error();
  if (!ctx || (cap && !out4) || !count) return RTG_ERR_INVALID;
  *count = ctx->timelineCount;
  const size_t k = cap < ctx->timelineCount ? cap : ctx->timelineCount;
  if (k == 0) return RTG_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out4, ctx->timeline, k * sizeof(uint4), hipMemcpyDeviceToHost));
  return RTG_OK;
}

int rtg_set_launch_opts(rtg_context* ctx, const rtg_launch_opts* opts) {
  rtg_clear_error();
  if (!ctx || !opts) return RTG_ERR_INVALID;
  ctx->opts = *opts;
  return RTG_OK;
}

int rtg_context_set_scene(rtg_context* ctx, const rtg_sphere* spheres, unsigned sphNum,
                          const rtg_light* lights, unsigned lgtNum) {
  rtg_clear_error();
  if (!ctx || (sphNum && !spheres) || (lgtNum && !lights)) {
    rtg_set_error("rtg_context_set_scene: invalid arguments");
    return RTG_ERR_INVALID;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  free_scene(ctx);
  PackedScene ps;
  pack_scene(spheres, sphNum, lights, lgtNum, &ps);
  std::vector<float4> geom(ps.geom.size() / 4);
  memcpy(geom.data(), ps.geom.data(), ps.geom.size() * sizeof(float));
  const std::vector<float>& crad2 = ps.crad2;
  const std::vector<float>& mats = ps.mats;
  const std::vector<float>& lg = ps.lights;
  if (hipMalloc(&ctx->geom, geom.size() * sizeof(float4)) != hipSuccess ||
      hipMalloc(&ctx->crad2, crad2.size() * sizeof(float)) != hipSuccess ||
      hipMalloc(&ctx->mats, mats.size() * sizeof(float)) != hipSuccess ||
      hipMalloc(&ctx->lights, lg.size() * sizeof(float)) != hipSuccess) {
    free_scene(ctx);
    rtg_set_error("hipMalloc failed for scene");
    return RTG_ERR_NOMEM;
  }
  HIP_TRY(hipMemcpy(ctx->geom, geom.data(), geom.size() * sizeof(float4),
                    hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(ctx->crad2, crad2.data(), crad2.size() * sizeof(float),
                    hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(ctx->mats, mats.data(), mats.size() * sizeof(float),
                    hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(ctx->lights, lg.data(), lg.size() * sizeof(float), hipMemcpyHostToDevice));
  ctx->n = sphNum;
  ctx->m = lgtNum;
  ctx->n4 = ps.n4;
  ctx->hasScene = true;
  return RTG_OK;
}

static int launch_trace(rtg_context* ctx, unsigned width, unsigned height, float zoom,
                        float aliasFactor, int stackSize, unsigned rowBlock, unsigned shard,
                        unsigned nShards, const unsigned* rowList, unsigned nRowList,
                        rtg_vec* dstDevice, void* stream) {
  if (!ctx || !ctx->hasScene) {
    rtg_set_error("render: no context/scene");
    return RTG_ERR_INVALID;
  }
  bool ldsMats = ctx->n + 1 <= kLdsMatMax;
  KernelArgs a;
  int rc = make_camera(width, height, zoom, aliasFactor, &a.cam);
  if (rc) return rc;
  int variant = ctx->opts.variant;
  // sample-parallel kernel: needs all of a pixel's samples in one wave
  // sample-parallel kernels need all of a pixel's samples in one wave
  const bool sampleKernel = variant == 0 || (variant >= 14 && variant <= 17);
  if (sampleKernel && (a.cam.nAA < 1 || a.cam.nAA > 8)) variant = 9;
  // the default sample kernel reads materials/geometry from global memory
  // (L1/L2-resident), not from a per-workgroup LDS copy (variant 17 keeps it)
  if (variant == 0 || variant == 15) ldsMats = false;
  TraceFn fn = pick_trace(stackSize, ldsMats, variant);
  if (!fn) {
    rtg_set_error("stackSize %d outside [1, %d]", stackSize, RTG_MAX_STACK);
    return RTG_ERR_INVALID;
  }
  unsigned rows;
  if (rowList) {
    rows = nRowList;
  } else {
    if (rowBlock == 0 || nShards == 0 || shard >= nShards) {
      rtg_set_error("render: bad sharding %u/%u block %u", shard, nShards, rowBlock);
      return RTG_ERR_INVALID;
    }
    rows = shard_row_count(height, rowBlock, shard, nShards);
  }
  if (rows == 0) return RTG_OK;
  if (!dstDevice) {
    rtg_set_error("render: null destination");
    return RTG_ERR_INVALID;
  }
  a.geom = ctx->geom;
  a.crad2 = ctx->crad2;
  a.mats = ctx->mats;
  a.lights = ctx->lights;
  a.n = ctx->n;
  a.m = ctx->m;
  a.n4 = ctx->n4;
  a.W = width;
  a.rowsLocal = rows;
  a.rowBlock = rowBlock ? rowBlock : 1;
  a.shard = shard;
  a.nShards = nShards ? nShards : 1;
  a.rowList = rowList;
  a.dst = reinterpret_cast<float*>(dstDevice);
  a.diag = nullptr;
  a.timeline = nullptr;
  if (variant >= 100) {
    if (!ctx->diag) {
      HIP_TRY(hipMalloc(&ctx->diag, 8 * sizeof(unsigned long long)));
      HIP_TRY(hipMemset(ctx->diag, 0, 8 * sizeof(unsigned long long)));
    }
    a.diag = ctx->diag;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  unsigned threads = (unsigned)kBlock;
  dim3 grid((width + 15u) / 16u, (rows + 15u) / 16u);
  if (variant == 0 || (variant >= 14 && variant <= 17)) {
    const unsigned ppw = 64u / (unsigned)(a.cam.nAA * a.cam.nAA);
    const size_t waves = ((size_t)width * rows + ppw - 1) / ppw;
    const unsigned tpb = variant == 14 ? 256u : variant == 16 ? 128u : 64u;
    const size_t blocks = (waves + tpb / 64 - 1) / (tpb / 64);
    threads = tpb;
    if (blocks > 0x7FFFFFFFu) {
      rtg_set_error("render: frame too large (%zu workgroups)", blocks);
      return RTG_ERR_INVALID;
    }
    grid = dim3((unsigned)blocks, 1);
  }
  const size_t frameLds = (size_t)(stackSize > 1 ? stackSize - 1 : 1) * threads * 16;
  const size_t lds = frameLds + (ldsMats ? ((size_t)(ctx->n + 1) * 8 * sizeof(float) +
                                            (size_t)ctx->n4 * 16)
                                         : 0);
  if (ctx->opts.flags & RTG_LAUNCH_TIMELINE) {
    const size_t waves = (size_t)grid.x * grid.y * (threads / 64);
    if (ctx->timelineCap < waves) {
      (void)hipFree(ctx->timeline);
      ctx->timeline = nullptr;
      ctx->timelineCap = 0;
      HIP_TRY(hipMalloc(&ctx->timeline, waves * sizeof(uint4)));
      ctx->timelineCap = waves;
    }
    ctx->timelineCount = waves;
    a.timeline = ctx->timeline;
  }
  hipLaunchKernelGGL(fn, grid, dim3(threads), lds, (hipStream_t)stream, a);
  HIP_TRY(hipGetLastError());
  return RTG_OK;
}

int rtg_render_device(rtg_context* ctx, unsigned width, unsigned height, float zoom,
                      float aliasFactor, int stackSize, unsigned rowBlock, unsigned shard,
                      unsigned nShards, rtg_vec* dstDevice, void* stream) {
  rtg_clear_error();
  return launch_trace(ctx, width, height, zoom, aliasFactor, stackSize, rowBlock, shard,
                      nShards, nullptr, 0, dstDevice, stream);
}

int rtg_render_rows_device(rtg_context* ctx, unsigned width, unsigned height, float zoom,
                           float aliasFactor, int stackSize, const unsigned* rowsDevice,
                           unsigned nRows, rtg_vec* dstDevice, void* stream) {
  rtg_clear_error();
  if (nRows && !rowsDevice) {
    rtg_set_error("rtg_render_rows_device: null row list");
    return RTG_ERR_INVALID;
  }
  if (nRows == 0) return RTG_OK;
  return launch_trace(ctx, width, height, zoom, aliasFactor, stackSize, 1, 0, 1, rowsDevice,
                      nRows, dstDevice, stream);
}

int rtg_render_rows(int device, const rtg_sphere* spheres, unsigned sphNum,
                    const rtg_light* lights, unsigned lgtNum, unsigned width, unsigned height,
                    float zoom, float aliasFactor, int stackSize, const unsigned* rows,
                    unsigned nRows, rtg_vec* dstHost) {
  rtg_clear_error();
  if (nRows && (!rows || !dstHost)) {
    rtg_set_error("rtg_render_rows: null argument");
    return RTG_ERR_INVALID;
  }
  if (nRows) {
    int rc0 = check_render_args(spheres, sphNum, lights, lgtNum, width, height, zoom,
                                aliasFactor, stackSize, dstHost);
    if (rc0) return rc0;
  }
  for (unsigned k = 0; k < nRows; ++k)
    if (rows[k] >= height) {
      rtg_set_error("rtg_render_rows: row %u >= height %u", rows[k], height);
      return RTG_ERR_INVALID;
    }
  if (nRows == 0) return RTG_OK;
  rtg_context* ctx = nullptr;
  int rc = rtg_context_create(device, &ctx);
  if (rc) return rc;
  rtg_vec* d = nullptr;
  unsigned* drows = nullptr;
  const size_t bytes = (size_t)width * nRows * sizeof(rtg_vec);
  rc = rtg_context_set_scene(ctx, spheres, sphNum, lights, lgtNum);
  if (!rc && (hipMalloc(&d, bytes) != hipSuccess ||
              hipMalloc(&drows, nRows * sizeof(unsigned)) != hipSuccess)) {
    rtg_set_error("hipMalloc failed");
    rc = RTG_ERR_NOMEM;
  }
  if (!rc && hipMemcpy(drows, rows, nRows * sizeof(unsigned), hipMemcpyHostToDevice) !=
                 hipSuccess) {
    rtg_set_error("row list upload failed");
    rc = RTG_ERR_HIP;
  }
  if (!rc)
    rc = rtg_render_rows_device(ctx, width, height, zoom, aliasFactor, stackSize, drows, nRows,
                                d, nullptr);
  if (!rc) {
    hipError_t e = hipMemcpy(dstHost, d, bytes, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      rtg_set_error("kernel/readback failed: %s", hipGetErrorString(e));
      rc = RTG_ERR_HIP;
    }
  }
  (void)hipFree(d);
  (void)hipFree(drows);
  rtg_context_destroy(ctx);
  return rc;
}

int rtg_max_colour_device(rtg_context* ctx, const rtg_vec* pixelsDevice, size_t n,
                          float* maxDevice, void* stream) {
  rtg_clear_error();
  if (!ctx || !maxDevice || (n && !pixelsDevice)) return RTG_ERR_INVALID;
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemsetAsync(maxDevice, 0, sizeof(float), s));
  if (n) {
    const size_t nval = n * 3;
    size_t blocks = (nval + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(max_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const float*)pixelsDevice, nval, (unsigned*)maxDevice);
    HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(max_finish_kernel, dim3(1), dim3(1), 0, s, (unsigned*)maxDevice);
  HIP_TRY(hipGetLastError());
  return RTG_OK;
}

int rtg_ppm_bytes_device(rtg_context* ctx, const rtg_vec* pixelsDevice, size_t n,
                         const float* maxDevice, unsigned char* outDevice, void* stream) {
  rtg_clear_error();
  if (!ctx || !maxDevice || (n && (!pixelsDevice || !outDevice))) return RTG_ERR_INVALID;
  if (n == 0) return RTG_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  const size_t nval = n * 3;
  size_t blocks = (nval + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(ppm_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (const float*)pixelsDevice, nval, maxDevice, outDevice);
  HIP_TRY(hipGetLastError());
  return RTG_OK;
}

int rtg_render(int device, const rtg_sphere* spheres, unsigned sphNum, const rtg_light* lights,
               unsigned lgtNum, unsigned width, unsigned height, float zoom, float aliasFactor,
               int stackSize, rtg_vec* dstHost) {
  rtg_clear_error();
  int rc0 = check_render_args(spheres, sphNum, lights, lgtNum, width, height, zoom, aliasFactor,
                              stackSize, dstHost);
  if (rc0) return rc0;
  rtg_context* ctx = nullptr;
  int rc = rtg_context_create(device, &ctx);
  if (rc) return rc;
  rtg_vec* d = nullptr;
  const size_t bytes = (size_t)width * height * sizeof(rtg_vec);
  rc = rtg_context_set_scene(ctx, spheres, sphNum, lights, lgtNum);
  if (!rc && hipMalloc(&d, bytes ? bytes : 4) != hipSuccess) {
    rtg_set_error("hipMalloc(%zu) failed", bytes);
    rc = RTG_ERR_NOMEM;
  }
  if (!rc)
    rc = rtg_render_device(ctx, width, height, zoom, aliasFactor, stackSize, 16, 0, 1, d,
                           nullptr);
  if (!rc) {
    hipError_t e = hipMemcpy(dstHost, d, bytes, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      rtg_set_error("kernel/readback failed: %s", hipGetErrorString(e));
      rc = RTG_ERR_HIP;
    }
  }
  (void)hipFree(d);
  rtg_context_destroy(ctx);
  return rc;
}

}  // extern "C"
