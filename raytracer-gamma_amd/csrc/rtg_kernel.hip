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

constexpr int kTileW = 16, kTileH = 16, kBlock = 256;
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
struct LdsFrames {
  FrameC* base;  // already offset by threadIdx.x
  __device__ __forceinline__ FrameC& operator()(int lv) const { return base[lv * kBlock]; }
};

// Wave-wide reductions with DPP (all 64 lanes must be active: the converged
// loop of trace_sample_cv guarantees it at every call site).
template <int kCtrl, int kRowMask>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), kCtrl, kRowMask, 0xF, false));
}
struct OpMax { __device__ float operator()(float a, float b) const { return fmaxf(a, b); } };
template <class Op>
__device__ __forceinline__ float wave_reduce(float v) {
  Op op;
  v = op(v, dpp_f<0xB1, 0xF>(v));   // quad_perm [1,0,3,2]
  v = op(v, dpp_f<0x4E, 0xF>(v));   // quad_perm [2,3,0,1]
  v = op(v, dpp_f<0x141, 0xF>(v));  // row_half_mirror
  v = op(v, dpp_f<0x140, 0xF>(v));  // row_mirror: every lane holds its row's result
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 15));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 31));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 47));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
  return op(op(r0, r1), op(r2, r3));
}

template <class MatPtr, bool kDiag = false>
struct DevScene {
  FrameC* lfr;
  __device__ __forceinline__ bool any(bool b) const { return __ballot(b) != 0ull; }
  __device__ __forceinline__ float wave_max(float v) const { return wave_reduce<OpMax>(v); }
  __device__ __forceinline__ int first_lane(bool b) const {
    const uint64_t m = __ballot(b);
    return m ? (int)__builtin_ctzll(m) : -1;
  }
  __device__ __forceinline__ float read_lane(float v, int l) const {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
  }
  // bit k (k < min(n, 64)) = pred(k), evaluated by lane k.
  __device__ __forceinline__ bool all(bool b) const { return __ballot(!b) == 0ull; }
  template <class F>
  __device__ __forceinline__ uint64_t sphere_mask(F pred) const {
    const unsigned lane = threadIdx.x & 63u;
    const bool p = (lane < n) ? pred(lane) : false;
    return __ballot(p);
  }
  __device__ __forceinline__ LdsFrames frames() const { return LdsFrames{lfr}; }
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
};

__device__ __forceinline__ float canon_nan(float v) {
  // x86 default NaN, what the reference CPU path writes (see rtg.h).
  return (v != v) ? __uint_as_float(0xFFC00000u) : v;
}

// Minimum waves per SIMD requested from the register allocator: 7 (<= 72
// VGPRs) where the LDS image of S-1 frame levels still admits 7 workgroups
// per CU (S <= 6 with a small scene); measured +1-2 % over the unconstrained
// 78-VGPR build at 6 waves/SIMD (C3).  Variant 9 forces it for any S.
template <int S, int kVariant>
struct MinWaves {
  static constexpr int value =
      ((kVariant % 100 == 0 && S <= 6) || kVariant % 100 == 9) ? 7 : 1;
};

template <int S, bool kLds, int kVariant>
__global__ __launch_bounds__(kBlock, (MinWaves<S, kVariant>::value)) void trace_kernel(
    const KernelArgs a) {
  // LDS image: per-lane frame colours ((S-1) x kBlock x 16 B), then, when
  // kLds, the material table (n+1) x 8 floats and the geometry n x float4.
  extern __shared__ float4 lds4[];
  typedef typename std::conditional<kLds, const float*, cfloat_p>::type MatPtr;
  constexpr bool kDiag = kVariant >= 100;
  constexpr int kBase = kDiag ? kVariant - 100 : kVariant;
  constexpr int NF = (S > 1) ? (S - 1) : 1;
  DevScene<MatPtr, kDiag> sc;
  if constexpr (kDiag)
    for (int k = 0; k < kProbeSlots; ++k) sc.acc[k] = 0;
  sc.lfr = reinterpret_cast<FrameC*>(lds4) + threadIdx.x;
  float4* sceneLds = lds4 + NF * kBlock;
  if constexpr (kLds) {
    float* lmats = reinterpret_cast<float*>(sceneLds);
    const unsigned nm = (a.n + 1) * 8;
    for (unsigned i = threadIdx.x; i < nm; i += kBlock) lmats[i] = a.mats[i];
    float4* lg = sceneLds + (a.n + 1) * 2;
    for (unsigned i = threadIdx.x; i < a.n4; i += kBlock)
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
  const unsigned lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const unsigned x = blockIdx.x * kTileW + (wave & 1u) * 8u + (lane & 7u);
  const unsigned lr = blockIdx.y * kTileH + (wave >> 1) * 8u + (lane >> 3);
  const bool valid = x < a.W && lr < a.rowsLocal;
  const unsigned gy = !valid ? 0u
                     : a.rowList ? a.rowList[lr]
                                 : shard_global_row(lr, a.rowBlock, a.shard, a.nShards);

  // Primary-ray sphere cull for this wave (whole wave converged here): the
  // bounds of every sample direction of the wave's pixels, then one sphere
  // per lane against that bundle, then a ballot (see primary_sphere_possible).
  uint64_t primSel = ~0ull;
  bool usePrim = false;
  if constexpr (kBase == 0 || kBase == 7 || kBase == 8 || kBase == 9) {
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
  if constexpr (kBase != 7) {
    if (!valid) return;
  }
  V3 pix;
  unsigned long long tk0 = 0;
  if constexpr (kDiag) tk0 = __builtin_amdgcn_s_memtime();
  if constexpr (kBase == 0) pix = shade_pixel<S, 2, true>(sc, a.cam, x, gy, usePrim, primSel);
  else if constexpr (kBase == 6) pix = shade_pixel<S, 2, true>(sc, a.cam, x, gy);
  else if constexpr (kBase == 8) pix = shade_pixel<S, 3, true>(sc, a.cam, x, gy, usePrim, primSel);
  else if constexpr (kBase == 9) pix = shade_pixel<S, 2, true>(sc, a.cam, x, gy, usePrim, primSel);
  else if constexpr (kBase == 7) pix = shade_pixel_cv<S>(sc, a.cam, x, gy, valid, usePrim, primSel);
  else if constexpr (kBase == 5) pix = shade_pixel<S, 2, false>(sc, a.cam, x, gy);
  else if constexpr (kBase == 1) pix = shade_pixel<S, 0>(sc, a.cam, x, gy);
  else if constexpr (kBase == 2) pix = shade_pixel_persistent<S, 2>(sc, a.cam, x, gy);
  else if constexpr (kBase == 3) pix = shade_pixel_persistent<S, 1>(sc, a.cam, x, gy);
  else pix = shade_pixel_nodes<S, 2>(sc, a.cam, x, gy);
  if (!valid) return;  // (variant 7 keeps every lane until here)
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

typedef void (*TraceFn)(const KernelArgs);
// Kernel variants (rtg_launch_opts.variant; results identical, speed differs):
//   0 (default) per-sample recursion + two-pass candidate-mask queries
//   1 per-sample recursion, one sphere per step (first kernel)
//   2 one-query-per-iteration state machine + candidate masks
//   3 one-query-per-iteration state machine, four spheres per step
//   4 node-persistent: samples chained in one node loop + candidate masks
//   5 as 0 but frame colours in private memory instead of LDS
//   6 as 0 without the per-wave primary-ray sphere cull
//   7 converged per-sample loop with per-query bundle culling (trace_sample_cv)
//   8 as 0 with the tuned two-pass query (prefetched groups, uniform quotient path)
//   9 as 0 compiled for 7 waves/SIMD (__launch_bounds__ min waves 7: <= 72 VGPRs)
//   100 + v: diagnostic build of v (s_memtime probes, rtg_diag_read)
template <int S, int V>
static TraceFn trace_fn_v(bool lds) {
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
    case 7: return trace_fn_v<S, 7>(lds);
    case 8: return trace_fn_v<S, 8>(lds);
    case 9: return trace_fn_v<S, 9>(lds);
    case 108: return trace_fn_v<S, 108>(lds);
    case 107: return trace_fn_v<S, 107>(lds);
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
  const bool ldsMats = ctx->n + 1 <= kLdsMatMax;
  TraceFn fn = pick_trace(stackSize, ldsMats, ctx->opts.variant);
  if (!fn) {
    rtg_set_error("stackSize %d outside [1, %d]", stackSize, RTG_MAX_STACK);
    return RTG_ERR_INVALID;
  }
  KernelArgs a;
  int rc = make_camera(width, height, zoom, aliasFactor, &a.cam);
  if (rc) return rc;
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
  if (ctx->opts.variant >= 100) {
    if (!ctx->diag) {
      HIP_TRY(hipMalloc(&ctx->diag, 8 * sizeof(unsigned long long)));
      HIP_TRY(hipMemset(ctx->diag, 0, 8 * sizeof(unsigned long long)));
    }
    a.diag = ctx->diag;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  dim3 grid((width + kTileW - 1) / kTileW, (rows + kTileH - 1) / kTileH);
  const size_t frameLds = (size_t)(stackSize > 1 ? stackSize - 1 : 1) * kBlock * 16;
  const size_t lds = frameLds + (ldsMats ? ((size_t)(ctx->n + 1) * 8 * sizeof(float) +
                                            (size_t)ctx->n4 * 16)
                                         : 0);
  hipLaunchKernelGGL(fn, grid, dim3(kBlock), lds, (hipStream_t)stream, a);
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
