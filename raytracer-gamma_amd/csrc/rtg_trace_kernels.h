// rtg_trace_kernels.h — the trace kernels of librtg.so (CDNA4 / gfx950) as
// templates over the stack capacity S (RTSTACK_MAXSIZE, raytraceStack.h:10)
// and the kernel variant.  Each rtg_trace_s<S>.hip translation unit
// instantiates one S (trace_fn<S>), so the 16 stack sizes compile in
// parallel; rtg_kernel.hip holds the launch code and the C ABI.
//
// Replaces the OpenCL kernel `raytrace` (raytrace_kernel.cl:870-973),
// computing the reference CPU path's framebuffer (raytracer.h) bit for bit;
// see rtg_trace.h for the traversal and DESIGN.md for the layout and roofline.
#pragma once

#include <hip/hip_runtime.h>

#include <stdint.h>

#include <type_traits>

#include "rtg.h"
#include "rtg_internal.h"
#include "rtg_trace.h"

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
typedef const RTG_CONST unsigned* cuint_p;

// Element i of a scene table with a 32-bit byte offset: base + zext(offset)
// is what the scalar (s_load sbase, soffset) and vector (global_load v, saddr)
// addressing modes take directly, so an index costs one 32-bit shift instead
// of 64-bit shift/add/add-with-carry pairs.  Tables are far below 4 GiB.
__device__ __forceinline__ cfloat_p fidx(cfloat_p p, unsigned i) {
  return (cfloat_p)((const RTG_CONST char*)p + i * 4u);
}
__device__ __forceinline__ cuint_p uidx(cuint_p p, unsigned i) {
  return (cuint_p)((const RTG_CONST char*)p + i * 4u);
}
#if defined(__HIP_DEVICE_COMPILE__)  // (one type on the host pass, where RTG_CONST is empty)
__device__ __forceinline__ const float* fidx(const float* p, unsigned i) { return p + i; }
#endif

// Per-lane frame colours in LDS: level lv of thread t at lfr[lv * kBlock + t]
// (16-byte records, so a wave's ds_read_b128 covers 1 KiB contiguously and is
// bank-conflict free).
template <int kThreads>
struct LdsFrames {
  FrameC* base;  // already offset by threadIdx.x
  __device__ __forceinline__ FrameC get(int lv) const { return base[lv * kThreads]; }
  __device__ __forceinline__ void set(int lv, const FrameC& v) const { base[lv * kThreads] = v; }
};
// The same with the deepest level `top` in four VGPRs instead of LDS (BVH
// kernels, stack capacity >= 3): one KiB less LDS per wave, which is what
// limits their occupancy (7 frame levels + the traversal stack at S = 8: 5
// waves per SIMD; 6 with this).  Level `top` holds a frame only while a node
// of depth S - 1 (a leaf) is being shaded below it.
// RTG_BVH_REG_LEVELS = 2 (A/B builds): the two deepest levels in VGPRs.
#ifndef RTG_BVH_REG_LEVELS
#define RTG_BVH_REG_LEVELS 1
#endif
template <int kThreads>
struct LdsFramesTop {
  FrameC* base;  // already offset by threadIdx.x; levels 0 .. top-1
  int top;
  mutable FrameC reg[RTG_BVH_REG_LEVELS];
  __device__ __forceinline__ FrameC get(int lv) const {
    const FrameC l = base[(lv < top ? lv : top - 1) * kThreads];
    if constexpr (RTG_BVH_REG_LEVELS == 1) return lv < top ? l : reg[0];
    else return lv < top ? l : lv == top ? reg[0] : reg[1];
  }
  __device__ __forceinline__ void set(int lv, const FrameC& v) const {
    if (lv < top) base[lv * kThreads] = v;
    else if (RTG_BVH_REG_LEVELS == 1 || lv == top) reg[0] = v;
    else reg[RTG_BVH_REG_LEVELS - 1] = v;
  }
};

// kBvh: the kernel instantiation for BVH scenes (n > 64); without it the BVH
// branches compile away, so small scenes keep the smaller, faster kernel.
// kFuse: Scene::fuse bits (kFusePrim / kFuseCone / kFuseShadow, rtg_trace.h).
// kMasks: the scene has shadow/overlap and cone masks (every finite scene of
// <= 64 spheres, rtg_scene_pack.h), so has_smask() / has_cone() are
// compile-time true and the kernel keeps no run-time flags for them.
// kCount: the executed-work counting build (kernel variant 120): count()
// accumulates every unit (rtg_trace.h kCnt* / kU*) per lane and, once per
// wave-level execution, on the wave's first active lane; flush_counts() adds
// the wave's sums to KernelArgs::counts.  Control flow is the default
// kernel's, so the counts are the default kernel's executed work.
template <class MatPtr, bool kDiag = false, int kThreads = kBlock, bool kBvh = false,
          int kFuse = 0, bool kMasks = false, bool kCount = false>
struct DevScene {
  static constexpr int fuse = kFuse;
  static constexpr bool kIsBvh = kBvh;
  FrameC* lfr;
  __device__ __forceinline__ bool all(bool b) const { return __ballot(!b) == 0ull; }
  __device__ __forceinline__ bool any(bool b) const { return __ballot(b) != 0ull; }
  // frame levels 0 .. nfl-1 in LDS (nfl = frame_lds_levels); BVH kernels keep
  // the deepest of NF levels in VGPRs (LdsFramesTop)
  int nfl;
  __device__ __forceinline__ auto frames() const {
    if constexpr (kBvh) return LdsFramesTop<kThreads>{lfr, nfl, {}};
    else return LdsFrames<kThreads>{lfr};
  }
  // Diagnostic cycle accounting (kDiag builds only): s_memtime deltas per
  // probe slot, summed per wave and added to KernelArgs::diag at exit.
  mutable unsigned long long acc[kProbeSlots];
  mutable unsigned long long t0[kProbeSlots];
  // RTG_DIAG_SPLIT builds (diagnostic A/B libraries only) re-assign slots 1
  // and 4-6 to the finer regions kProbeSplit* (rtg_trace.h).
  __device__ __forceinline__ static int probe_slot(int slot) {
    if (RTG_DIAG_SPLIT) {
      if (slot >= kProbeSplitBase) return slot - kProbeSplitBase;
      if (slot == kProbeShadow || (slot >= kProbeMatte && slot <= kProbeUnwind)) return -1;
      return slot;
    }
    return slot >= kProbeSplitBase ? -1 : slot;
  }
  __device__ __forceinline__ void probe_begin(int slot0) const {
    const int slot = probe_slot(slot0);
    if (slot < 0) return;
    if constexpr (kDiag) {
      __builtin_amdgcn_sched_barrier(0);
      t0[slot] = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __device__ __forceinline__ void probe_end(int slot0) const {
    const int slot = probe_slot(slot0);
    if (slot < 0) return;
    if constexpr (kDiag) {
      __builtin_amdgcn_sched_barrier(0);
      acc[slot] += __builtin_amdgcn_s_memtime() - t0[slot];
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  mutable unsigned cntW[kCount ? kCntSlots : 1];  // wave-level executions (first active lane)
  mutable unsigned cntL[kCount ? kCntSlots : 1];  // lane-level sum of the counted values
  __device__ __forceinline__ void count_reset() const {
    if constexpr (kCount)
      for (int k = 0; k < kCntSlots; ++k) cntW[k] = cntL[k] = 0u;
  }
  __device__ __forceinline__ void count(int slot, long v) const {
    if constexpr (kCount) {
      const uint64_t act = __ballot(1);
      const unsigned lane = threadIdx.x & 63u;
      cntW[slot] += (lane == (unsigned)__builtin_ctzll(act)) ? 1u : 0u;
      cntL[slot] += (unsigned)v;
    } else {
      (void)slot;
      (void)v;
    }
  }
  // Adds the wave's counters to out[0 .. kCntSlots) (wave-level) and
  // out[kCntSlots .. 2 kCntSlots) (lane-level); whole wave converged.
  __device__ __forceinline__ void flush_counts(unsigned long long* out) const {
    if constexpr (kCount) {
      for (int k = 0; k < kCntSlots; ++k) {
        unsigned w = cntW[k], l = cntL[k];
        for (int off = 32; off > 0; off >>= 1) {
          w += __shfl_xor(w, off);
          l += __shfl_xor(l, off);
        }
        if ((threadIdx.x & 63u) == 0) {
          if (w) atomicAdd(&out[k], (unsigned long long)w);
          if (l) atomicAdd(&out[kCntSlots + k], (unsigned long long)l);
        }
      }
    } else {
      (void)out;
    }
  }
  cfloat_p geom;      // n x {x, y, z, r*r}
  cfloat_p crad2;
  MatPtr mats;        // LDS copy (float*) or the global table (cfloat_p)
  const float4* lgeom;  // LDS copy of geom (or the global array when it does not fit)
  cfloat_p lights;
  cuint_p smask;  // m x n x {lo, hi} shadow masks, or null
  cuint_p cone;   // n x kConeCells x {lo, hi} secondary-ray cone masks, or null
  cfloat_p prim;  // n x {1/|c|, sin a, cos a, 0}: primary-cull sphere constants
  cfloat_p bvhNodes;  // BVH (build_bvh, rtg_scene_pack.h) or null
  int* bvhStk;        // this wave's 64-entry LDS traversal stack (BVH scenes)
  cfloat_p capRec, ovRec;  // sphere lists of BVH scenes (sphere_lists) or null
  cuint_p capOff, ovOff;
  unsigned n, m;
  unsigned n4;  // geometry records incl. NaN padding to a multiple of 4

  __device__ __forceinline__ V3 sphere(unsigned i, float& r2) const {
    cfloat_p g = fidx(geom, 4 * i);
    r2 = g[3];
    return v3(g[0], g[1], g[2]);
  }
  // r^2 of sphere i (wave-uniform i: one scalar load)
  __device__ __forceinline__ float sphere_r2(unsigned i) const { return fidx(geom, 4 * i)[3]; }
  // Four consecutive sphere records: one 64-byte scalar load.
  __device__ __forceinline__ void sphere4(unsigned i, V3* c, float* r2) const {
    cfloat_p g = fidx(geom, 4 * i);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c[k] = v3(g[4 * k + 0], g[4 * k + 1], g[4 * k + 2]);
      r2[k] = g[4 * k + 3];
    }
  }
  // The same with the pass-1 screen radius^2 (second half of geom).
  __device__ __forceinline__ void sphere4_screen(unsigned i, V3* c, float* rs) const {
    sphere4(n4 + 4 + i, c, rs);
  }
  // ... and with the containment radius^2 (third part of geom).
  __device__ __forceinline__ void sphere4_contain(unsigned i, V3* c, float* cr) const {
    sphere4(2 * (n4 + 4) + i, c, cr);
  }
  __device__ __forceinline__ V3 sphere_screen(unsigned i, float& rs) const {
    return sphere(n4 + 4 + i, rs);
  }
  // Fused record of sphere i (geom's fourth part, 32 bytes: one
  // s_load_dwordx8): centre, pass-1 screen radius^2, r^2 and the primary
  // rays' c term |0 - c|^2 - r^2, for the fused query loops.
  __device__ __forceinline__ V3 sphere_fused(unsigned i, float& rs, float& r2, float& oc) const {
    typedef float f8 __attribute__((ext_vector_type(8)));
    const f8 g = *(const RTG_CONST f8*)fidx(geom, 12 * (n4 + 4) + 8 * i);  // one load
    rs = g[3];
    r2 = g[4];
    oc = g[5];
    return v3(g[0], g[1], g[2]);
  }
  __device__ __forceinline__ V3 sphere_contain(unsigned i, float& cr) const {
    return sphere(2 * (n4 + 4) + i, cr);
  }
  // BVH node nd: four slots {centre, screen radius^2}, their children and
  // containment radii^2 (wave-uniform nd: scalar loads).
  // (the kBvh kernels run only for scenes with a BVH: pick_trace)
  __device__ __forceinline__ bool has_bvh() const { return kBvh; }
  __device__ __forceinline__ int* bvh_stack() const { return bvhStk; }
  // Sphere lists (BVH scenes): ranges and 32-byte records (one scalar load).
  __device__ __forceinline__ bool has_lists() const {
    if constexpr (kBvh) return capOff != nullptr;
    else return false;
  }
  // capsule list of (light l, sphere h, hit-point cell): one 8-byte scalar load
  __device__ __forceinline__ void cap_range(unsigned l, unsigned h, unsigned cell, unsigned& k0,
                                            unsigned& k1) const {
    const cuint_p o = uidx(capOff, 2u * ((l * n + h) * kCapCells + cell));
    k0 = o[0];
    k1 = o[1];
  }
  __device__ __forceinline__ void ov_range(unsigned h, unsigned& k0, unsigned& k1) const {
    const cuint_p o = uidx(ovOff, h);
    k0 = o[0];
    k1 = o[1];
  }
  __device__ __forceinline__ static V3 list_rec(cfloat_p base, unsigned k, float& rs, float& r2,
                                                float& cr, int& idx, float& rf) {
    typedef float f8 __attribute__((ext_vector_type(8)));
    const f8 g = *(const RTG_CONST f8*)fidx(base, 8u * k);
    rs = g[3];
    r2 = g[4];
    cr = g[5];
    idx = __float_as_int(g[6]);
    rf = g[7];
    return v3(g[0], g[1], g[2]);
  }
  // Records k and k + 1 of a list table with one 64-byte scalar load (the
  // tables end with a padding record, sphere_lists).
  __device__ __forceinline__ static void list_rec2(cfloat_p base, unsigned k, ListRec& r0,
                                                   ListRec& r1) {
    typedef float f16 __attribute__((ext_vector_type(16)));
    const f16 g = *(const RTG_CONST f16*)fidx(base, 8u * k);
    r0.c = v3(g[0], g[1], g[2]);
    r0.rs = g[3];
    r0.r2 = g[4];
    r0.cr = g[5];
    r0.idx = __float_as_int(g[6]);
    r0.rf = g[7];
    r1.c = v3(g[8], g[9], g[10]);
    r1.rs = g[11];
    r1.r2 = g[12];
    r1.cr = g[13];
    r1.idx = __float_as_int(g[14]);
    r1.rf = g[15];
  }
  // Capsule records k .. k + 3 (16-byte form) with one 64-byte scalar load.
  __device__ __forceinline__ void cap_rec4(unsigned k, CapRec* r) const {
    typedef float f16 __attribute__((ext_vector_type(16)));
    const f16 g = *(const RTG_CONST f16*)fidx(capRec, 4u * k);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r[j].c = v3(g[4 * j], g[4 * j + 1], g[4 * j + 2]);
      r[j].r2 = g[4 * j + 3];
    }
  }
  __device__ __forceinline__ void ov_rec2(unsigned k, ListRec& r0, ListRec& r1) const {
    list_rec2(ovRec, k, r0, r1);
  }
  __device__ __forceinline__ V3 ov_rec(unsigned k, float& rs, float& r2, float& cr, int& idx,
                                       float& rf) const {
    return list_rec(ovRec, k, rs, r2, cr, idx, rf);
  }
  // Node copy nd's record (BvhRec, rtg_trace.h): two 64-byte scalar loads
  // (issuing both from one asm block with one wait measured slower, DESIGN.md
  // §4 item 44).
  __device__ __forceinline__ void bvh_rec(unsigned nd, BvhRec& r) const {
    typedef float f16 __attribute__((ext_vector_type(16)));
    const RTG_CONST f16* p = (const RTG_CONST f16*)fidx(bvhNodes, kBvhWords * nd);
    const f16 a = p[0], b = p[1];
#pragma unroll
    for (int k = 0; k < 16; ++k) r.s[k] = a[k];
#pragma unroll
    for (int k = 0; k < 8; ++k) r.s[16 + k] = b[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      r.ch[k] = __float_as_int(b[8 + k]);
      r.cr[k] = b[12 + k];
    }
  }
  // One lane's value for wave-uniform decisions (traversal order, cone cull).
  __device__ __forceinline__ float first_lane(float v) const {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
  }
  // v of the first active lane with `pred` (some active lane has it).
  __device__ __forceinline__ int lane_with(int v, bool pred) const {
    return __builtin_amdgcn_readlane(v, (int)__builtin_ctzll(__ballot(pred)));
  }
  __device__ __forceinline__ int first_lane_i(int v) const {
    return __builtin_amdgcn_readfirstlane(v);
  }
  __device__ __forceinline__ V3 first_lane(V3 v) const {
    return v3(first_lane(v.x), first_lane(v.y), first_lane(v.z));
  }
  // Secondary-ray cone masks (cone_masks, rtg_scene_pack.h): n <= 64.
  // (BVH scenes have more than 64 spheres: never masks; their kernels drop
  // the masked paths at compile time)
  __device__ __forceinline__ bool has_cone() const {
    if constexpr (kMasks) return true;
    else if constexpr (kBvh) return false;
    else return cone != nullptr;
  }
  // Union over the active lanes' origin spheres h (all >= 0) of cone mask
  // (h, tier, cell): one scalar load per distinct h.
  __device__ __forceinline__ uint64_t cone_union(int h, unsigned tier, unsigned cell) const {
    const int hu = __builtin_amdgcn_readfirstlane(h);
    if (__ballot(h != hu) == 0ull) {  // coherent wave: one origin sphere, one load
      const cuint_p w = uidx(cone, 2u * (((unsigned)hu * kConeTiers + tier) * kConeCells + cell));
      return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    }
    uint64_t todo = __ballot(1);
    uint64_t u = 0;
    while (todo) {
      count(kUMaskIter, 1);
      const int src = __builtin_ctzll(todo);
      const int h0 = __builtin_amdgcn_readlane(h, src);
      const cuint_p w = uidx(cone, 2u * (((unsigned)h0 * kConeTiers + tier) * kConeCells + cell));
      u |= (uint64_t)w[0] | ((uint64_t)w[1] << 32);
      todo &= ~__ballot(h == h0);
    }
    return u;
  }
  // Shadow and overlap masks (rtg_scene_pack.h shadow_masks): n <= 64.
  __device__ __forceinline__ bool has_smask() const {
    if constexpr (kMasks) return true;
    else if constexpr (kBvh) return false;
    else return smask != nullptr;
  }
  __device__ __forceinline__ uint64_t overlap_mask(unsigned h) const {  // per lane
    const cuint_p w = uidx(smask, 2u * (m * n + h));
    return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  }
  __device__ __forceinline__ float guard_r2(unsigned i) const { return *fidx(crad2, 2 * n + i); }
  // Union of the active lanes' overlap masks (one scalar load per distinct
  // h) and, in `own`, each lane's own mask.
  __device__ __forceinline__ uint64_t overlap_union(int h, uint64_t& own) const {
    const int hu = __builtin_amdgcn_readfirstlane(h);
    if (__ballot(h != hu) == 0ull) {  // coherent wave: one sphere, one load
      const cuint_p w = uidx(smask, 2u * (m * n + (unsigned)hu));
      own = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
      return own;
    }
    uint64_t todo = __ballot(1);
    uint64_t u = 0;
    own = 0;
    while (todo) {
      count(kUMaskIter, 1);
      const int src = __builtin_ctzll(todo);
      const int h0 = __builtin_amdgcn_readlane(h, src);
      const cuint_p w = uidx(smask, 2u * (m * n + (unsigned)h0));
      const uint64_t mk = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
      u |= mk;
      if (h == h0) own = mk;
      todo &= ~__ballot(h == h0);
    }
    return u;
  }
  // Union of the active lanes' masks of table row `row` (wave-uniform): one
  // scalar mask load per distinct hit sphere among the lanes; every sphere if
  // a lane is not `ok` (its hit point failed the guard test).  Row l < m holds
  // light l's shadow masks, row m the overlap masks.
  __device__ __forceinline__ uint64_t mask_union(unsigned row, int hit, bool ok) const {
    if (__ballot(!ok)) return n >= 64 ? ~0ull : ((1ull << n) - 1ull);
    const int hu = __builtin_amdgcn_readfirstlane(hit);
    if (__ballot(hit != hu) == 0ull) {  // coherent wave: one hit sphere, one load
      const cuint_p w = uidx(smask, 2u * (row * n + (unsigned)hu));
      return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
    }
    uint64_t todo = __ballot(1);
    uint64_t u = 0;
    while (todo) {
      count(kUMaskIter, 1);
      const int src = __builtin_ctzll(todo);
      const int h0 = __builtin_amdgcn_readlane(hit, src);
      const cuint_p w = uidx(smask, 2u * (row * n + (unsigned)h0));
      u |= (uint64_t)w[0] | ((uint64_t)w[1] << 32);
      todo &= ~__ballot(hit == h0);
    }
    return u;
  }
  __device__ __forceinline__ uint64_t shadow_union(unsigned l, int hit, bool guardOK) const {
    return mask_union(l, hit, guardOK);
  }
  __device__ __forceinline__ uint64_t contain_union(int hit, bool ok) const {
    return mask_union(m, hit, ok);
  }
  // Per-lane sphere record (divergent index): from the LDS copy.
  __device__ __forceinline__ V3 sphere_lane(unsigned i, float& r2) const {
    const float4 g = lgeom[i];
    r2 = g.w;
    return v3(g.x, g.y, g.z);
  }
  __device__ __forceinline__ float contain_r2(unsigned i) const { return *fidx(crad2, i); }
  // primary_possible's per-sphere constants of sphere i
  __device__ __forceinline__ bool prim_possible(const PrimBundle& b, unsigned i, V3 c) const {
    const cfloat_p k = fidx(prim, 4 * i);
    return primary_possible(b, c, k[0], k[1], k[2]);
  }
  // |0 - c_i|^2 - r_i^2: the c term of a ray from the origin (primary rays)
  __device__ __forceinline__ float origin_c(unsigned i) const { return *fidx(crad2, n + i); }
  __device__ __forceinline__ Mat mat_at(decltype(mats) p) const {
    Mat r;
    r.matte = v3(p[0], p[1], p[2]);
    r.gloss = v3(p[3], p[4], p[5]);
    r.opacity = p[6];
    r.refr = p[7];
    return r;
  }
  // Material record i; when every active lane asks for the same record (the
  // background for primary misses, one sphere for a coherent wave) it comes
  // through scalar loads instead of a per-lane gather.
  __device__ __forceinline__ Mat mat(int i) const {
    if constexpr (std::is_same<MatPtr, cfloat_p>::value) {
      const int i0 = __builtin_amdgcn_readfirstlane(i);
      if (__ballot(i != i0) == 0ull) return mat_at(fidx(mats, 8u * (unsigned)i0));
    }
    return mat_at(fidx(mats, 8u * (unsigned)i));
  }
  __device__ __forceinline__ float refr(int i) const { return fidx(mats, 8u * (unsigned)i)[7]; }
  // The shading set-up's data of hit sphere i (>= 0): centre, guard radius^2
  // and material.  When every active lane hit the same sphere (a coherent
  // wave) they come through the scalar cache; otherwise per-lane gathers.
  __device__ __forceinline__ void hit_data(int i, V3& c, float& g2, float& r2, Mat& mt) const {
    const int i0 = __builtin_amdgcn_readfirstlane(i);
    if (__ballot(i != i0) == 0ull) {
      const cfloat_p g = fidx(geom, 4u * (unsigned)i0);
      c = v3(g[0], g[1], g[2]);
      r2 = g[3];
      g2 = *fidx(crad2, 2 * n + (unsigned)i0);
      mt = mat_at(fidx(mats, 8u * (unsigned)i0));
    } else {
      const cfloat_p g = fidx(geom, 4u * (unsigned)i);
      c = v3(g[0], g[1], g[2]);
      r2 = g[3];
      g2 = *fidx(crad2, 2 * n + (unsigned)i);
      mt = mat_at(fidx(mats, 8u * (unsigned)i));
    }
  }
  // Centre, r^2 and guard radius^2 of sphere h (>= 0), scalar when uniform.
  __device__ __forceinline__ V3 sphere_guard(int h, float& r2, float& g2) const {
    const int h0 = __builtin_amdgcn_readfirstlane(h);
    if (__ballot(h != h0) == 0ull) {
      const cfloat_p g = fidx(geom, 4u * (unsigned)h0);
      r2 = g[3];
      g2 = *fidx(crad2, 2 * n + (unsigned)h0);
      return v3(g[0], g[1], g[2]);
    }
    const cfloat_p g = fidx(geom, 4u * (unsigned)h);
    r2 = g[3];
    g2 = *fidx(crad2, 2 * n + (unsigned)h);
    return v3(g[0], g[1], g[2]);
  }
  __device__ __forceinline__ void light(unsigned l, V3& pos, V3& col) const {
    cfloat_p p = fidx(lights, 6 * l);
    pos = v3(p[0], p[1], p[2]);
    col = v3(p[3], p[4], p[5]);
  }
};

// Compacted launch: the group list's partitions, each with its run counters
// and cost sum on a 128-byte line of its own (cull_groups_kernel: device-scope
// atomics on one address serialise).  A multiple of kListParts persistent
// waves, so wave w always takes partition w % kListParts.
constexpr unsigned kListParts = 16;
constexpr unsigned kCountStride = 32;  // unsigned
constexpr unsigned kStatStride = 16;   // unsigned long long

struct KernelArgs;
typedef void (*TraceFn)(const KernelArgs);

struct KernelArgs {
  const float4* geom;
  const float* crad2;
  const float* mats;
  const float* lights;
  const unsigned* smask;  // shadow masks (PackedScene::smask) or null
  const unsigned* cone;   // cone masks (PackedScene::cone) or null
  const float* prim;      // primary-cull sphere constants (PackedScene::prim)
  const float* bvhNodes;  // BVH node records (PackedScene::bvhNodes) or null
  const float* capRec;    // sphere lists (PackedScene::cap*, ov*) or null
  const unsigned* capOff;
  const float* ovRec;
  const unsigned* ovOff;
  unsigned n, m, n4;
  Camera cam;
  unsigned W, rowsLocal, rowBlock, shard, nShards;
  double invW, invRowBlock;  // RN(1.0 / W), RN(1.0 / rowBlock) (divmod_u64)
  const unsigned* rowList;  // explicit global rows (rtg_render_rows_device) or null
  float* dst;
  // Compacted launch (cull_groups_kernel): the pixel groups some primary ray
  // may hit, their count, and the number of persistent waves; null otherwise.
  const unsigned* groupList;
  const unsigned long long* groupSel;  // the listed groups' primary-ray sphere masks
  // The list has kListParts partitions of 2 x groupCap entries; partition p
  // (at 2 p groupCap) holds four runs, read in this order: [0, count[0]) from
  // the front of its first half, count[1] entries from its back (groupCap - 1
  // down), count[2] from the front of the second half and count[3] from its
  // back (2 groupCap - 1 down); heaviest run first (cull_groups_kernel).
  // Partition p's run lengths are groupCount[p kCountStride + 0..3].
  const unsigned* groupCount;
  unsigned groupCap;
  unsigned nRuns;              // the list's longest-first runs: 4, or 8 for short launches
  unsigned lptMin;             // cull_groups_kernel's popcount threshold (no cost feedback)
  unsigned nPersist;
  // Launch-order feedback (compacted launches; null when off): each listed
  // group's trace time in 10 ns ticks (s_memrealtime), written by the trace
  // kernel and read by the next launch's cull pass of the same frame
  // geometry, which also sums what it reads (low 40 bits the ticks, high 24
  // the group count) for the launch after it.
  unsigned* groupCost;
  // per list partition, at p kStatStride:
  unsigned long long* costStat;        // this cull pass's sums (zeroed before it), or null
  const unsigned long long* costPrev;  // the previous cull pass's, or null
  // Counters of the NEXT launch that this launch's trace kernel zeroes (its
  // first wave, a lane per list partition), so that no memset precedes a cull
  // pass: the slot's other group-count set and the cost entry's next costStat
  // (or null).
  // Neither is in use while this launch's trace runs: the slot's previous
  // launch is complete (its event), and this launch's cull pass has read its
  // costPrev before the trace starts (one stream).
  unsigned* zeroCount;
  unsigned long long* zeroStat;
  unsigned long long* diag;  // kProbeSlots counters (diagnostic variants only)
  unsigned long long* counts;  // 2 x kCntSlots unit counters (counting build, variant 120)
  uint4* timeline;           // per-wave records (RTG_LAUNCH_TIMELINE) or null
};

// floor(a / d) for a <= 64, 1 <= d <= 64: (a + 0.5) / d is at least 1/128
// from an integer, far beyond the float product's error.
#ifndef RTG_PROBE_FLOOR
#define RTG_PROBE_FLOOR 0
#endif

__device__ __forceinline__ unsigned udiv_small(unsigned a, unsigned d) {
  return (unsigned)(((float)a + 0.5f) * (1.0f / (float)d));
}
// q = a / d, r = a % d for a < 2^53, d >= 1, invd = RN(1.0 / d) (host): the
// f64 quotient estimate is within one of the true quotient; one integer
// correction each way.
__device__ __forceinline__ void divmod_u64(uint64_t a, unsigned d, double invd, unsigned& q,
                                           unsigned& r) {
  uint64_t qq = (uint64_t)((double)a * invd);
  int64_t rr = (int64_t)(a - qq * d);
  if (rr < 0) { --qq; rr += d; }
  else if (rr >= (int64_t)d) { ++qq; rr -= d; }
  q = (unsigned)qq;
  r = (unsigned)rr;
}
// shard_global_row (rtg_internal.h) with the division by the block size done
// through divmod_u64.
__device__ __forceinline__ unsigned shard_global_row_fast(unsigned localRow, unsigned B,
                                                         double invB, unsigned g, unsigned G) {
  unsigned lb, rem;
  divmod_u64(localRow, B, invB, lb, rem);
  return (lb * G + g) * B + rem;
}

__device__ __forceinline__ float canon_nan(float v) {
  // x86 default NaN, what the reference CPU path writes (see rtg.h).
  return (v != v) ? __uint_as_float(0xFFC00000u) : v;
}

// Minimum waves per SIMD requested from the register allocator: 7 (<= 72
// VGPRs) where the LDS image of S-1 frame levels still admits 7 waves per
// SIMD (S <= 6 with a small scene); measured +1-2 % over the unconstrained
// 78-VGPR build at 6 waves/SIMD (C3, tile kernel).
// BVH kernels above S = 6 (C5: S = 8): 6 waves per SIMD, which their LDS
// image (S - 2 frame levels + the traversal stack, 6.25 KB at S = 8) admits
// (<= 80 VGPRs).
template <int S, int kVariant, bool kBvh = false>
#ifndef RTG_DEFAULT_MIN_WAVES  // compiler-setting A/B builds (tools/ab_build.sh) only
#define RTG_DEFAULT_MIN_WAVES 7
#endif
struct MinWaves {
  static constexpr int value =
      (kVariant == 120) ? 1  // counting build: its counters take registers
      : (kBvh && (kVariant == 0 || kVariant == 50) && S > 6) ? 5 + RTG_BVH_REG_LEVELS
      : (kVariant == 18 && S <= 6) ? 8
      : (kVariant == 0 && S <= 6) ? RTG_DEFAULT_MIN_WAVES
      : ((kVariant % 100 == 0 || kVariant % 100 == 9 || kVariant >= 14) && S <= 6) ? 7 : 1;
};

// Frame levels in LDS per lane: S - 1 ancestors (at least 1: the pixel sum
// parks samples in level 0), one fewer for BVH kernels from S = 3 on
// (LdsFramesTop keeps the deepest in VGPRs).  launch_trace sizes the LDS with
// the same rule.
constexpr int frame_lds_levels(int S, bool bvh) {
  return (S > 1 ? S - 1 : 1) -
         (!bvh || S < 3 ? 0 : S < 4 ? 1 : RTG_BVH_REG_LEVELS);
}

// Workgroup prologue: the frame area and (kLds) the scene tables staged in LDS.
template <int S, bool kLds, int kThreads, class Sc>
__device__ __forceinline__ void stage_scene(const KernelArgs& a, Sc& sc) {
  extern __shared__ float4 lds4[];
  constexpr int NFL = frame_lds_levels(S, Sc::kIsBvh);
  sc.lfr = reinterpret_cast<FrameC*>(lds4) + threadIdx.x;
  sc.nfl = NFL;
  float4* sceneLds = lds4 + NFL * kThreads;
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
  sc.smask = (cuint_p)a.smask;
  sc.cone = (cuint_p)a.cone;
  sc.prim = (cfloat_p)a.prim;
  sc.bvhNodes = (cfloat_p)a.bvhNodes;
  sc.capRec = (cfloat_p)a.capRec;
  sc.capOff = (cuint_p)a.capOff;
  sc.ovRec = (cfloat_p)a.ovRec;
  sc.ovOff = (cuint_p)a.ovOff;
  // BVH scenes: 64 stack entries per wave after the frames and scene tables
  // (the launcher adds them to the LDS size).
  sc.bvhStk = reinterpret_cast<int*>(sceneLds + (kLds ? (a.n + 1) * 2 + a.n4 : 0)) +
              (threadIdx.x >> 6) * 64;
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
  // per lane against that bundle, then a ballot (see primary_possible).
  uint64_t primSel = ~0ull;
  bool usePrim = false;
  if constexpr (kBase == 0 || kBase == 8 || kBase == 9 || kBase == 59) {
    if (a.n <= 64) {
      float x0 = 3.0e38f, x1 = -3.0e38f, y0 = 3.0e38f, y1 = -3.0e38f;
      if (valid) primary_bounds(a.cam, x, gy, x0, x1, y0, y1);
      for (int off = 32; off > 0; off >>= 1) {
        x0 = fminf(x0, __shfl_xor(x0, off));
        x1 = fmaxf(x1, __shfl_xor(x1, off));
        y0 = fminf(y0, __shfl_xor(y0, off));
        y1 = fmaxf(y1, __shfl_xor(y1, off));
      }
      const PrimBundle pb = primary_bundle(x0, x1, y0, y1, a.cam.zoom);
      bool possible = false;
      if (lane < a.n) {
        const float4 g = sc.lgeom[lane];
        possible = sc.prim_possible(pb, lane, v3(g.x, g.y, g.z));
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
  else if constexpr (kBase == 59)  // OpenCL semantics (rtg_context_set_semantics)
    pix = shade_pixel<S, 2, true, true>(sc, a.cam, x, gy, usePrim, primSel);
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
// with the wave converged.  `tag` (compacted launches) goes above XCC_ID's 4
// bits: the popcount of the wave's first group's sphere mask (7 bits) and that
// group's index (21 bits), for the launch-order analysis (tools/timeline.py).
__device__ __forceinline__ void record_wave(const KernelArgs& a, unsigned t0, size_t w,
                                            unsigned tag = 0) {
  if (a.timeline == nullptr) return;
  const unsigned t1 = (unsigned)__builtin_amdgcn_s_memrealtime();
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20) & 15u;
  if ((threadIdx.x & 63u) == 0) a.timeline[w] = make_uint4(t0, t1, hw, xcc | (tag << 4));
}
// The same record in two halves: the start at once (so the start time need
// not stay live through the wave), the rest at the end.
__device__ __forceinline__ void record_wave_start(const KernelArgs& a, unsigned t0, size_t w) {
  if (a.timeline != nullptr && (threadIdx.x & 63u) == 0) a.timeline[w].x = t0;
}
__device__ __forceinline__ void record_wave_end(const KernelArgs& a, size_t w, unsigned tag) {
  if (a.timeline == nullptr) return;
  const unsigned t1 = (unsigned)__builtin_amdgcn_s_memrealtime();
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20) & 15u;
  if ((threadIdx.x & 63u) == 0) {
    a.timeline[w].y = t1;
    a.timeline[w].z = hw;
    a.timeline[w].w = xcc | (tag << 4);
  }
}

// Tile kernels: one 8 x 8 pixel tile per wave, all samples of a pixel in its
// lane; a workgroup is 2 x 2 tiles.
template <int S, bool kLds, int kVariant, bool kBvh = false>
__global__ __launch_bounds__(kBlock, (MinWaves<S, kVariant>::value))
void trace_kernel(const KernelArgs a) {
  // LDS image: per-lane frame colours ((S-1) x threads x 16 B), then, when
  // kLds, the material table (n+1) x 8 floats and the geometry n x float4.
  constexpr int kThreads = kBlock;
  constexpr unsigned TW = 2u, TH = 2u;
  typedef typename std::conditional<kLds, const float*, cfloat_p>::type MatPtr;
  DevScene<MatPtr, (kVariant >= 100), kThreads, kBvh> sc;
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
// hasSel: the cull pass already gave the group's primary-ray sphere subset
// (gsel, compacted launch), so the wave skips its own cull.
// The kernel's argument block (the sample kernels' one by-value parameter, at
// offset 0 of the kernarg segment) through an opaque pointer: each call's
// field reads are fresh scalar loads where they are used, so the group set-up
// and epilogue values are not held in SGPRs (or spilled to VGPR lanes) across
// the whole trace.
__device__ __forceinline__ const RTG_CONST KernelArgs* kargs() {
  const RTG_CONST KernelArgs* p =
      (const RTG_CONST KernelArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}

template <int S, int Q, bool kDiag, class Sc, bool kShfl = false, bool kCL = false>
__device__ __forceinline__ void trace_group(const KernelArgs& a0, Sc& sc, size_t gw,
                                            bool hasSel = false, uint64_t gsel = 0) {
  (void)a0;
  const KernelArgs a = *kargs();  // == a0, read afresh for this group
  const unsigned lane = threadIdx.x & 63u;
  const unsigned nAA = (unsigned)a.cam.nAA;
  const unsigned SP = nAA * nAA;
  const unsigned PPW = 64u / SP;
  // No integer divisions by run-time values (each is a ~25-instruction
  // sequence on the GPU; a trivial wave's whole cost is this set-up): small
  // quotients through float reciprocals, the wave's first pixel through
  // divmod_u64, the lanes' rows by carrying from it.
  const unsigned pl = udiv_small(lane, SP), s = lane - pl * SP;
  const size_t p0 = gw * PPW;  // the wave's first pixel (wave-uniform)
  const size_t total = (size_t)a.W * a.rowsLocal;
  const size_t p = p0 + pl;
  const bool valid = pl < PPW && p < total;
  unsigned col0, r0;
  divmod_u64(p0, a.W, a.invW, r0, col0);
  unsigned x = col0 + pl, lr = r0, gy = 0;
  while (x >= a.W) {  // PPW <= 64 pixels past the first: rarely one row
    x -= a.W;
    ++lr;
  }
  if (valid)
    gy = a.rowList ? a.rowList[lr]
                   : shard_global_row_fast(lr, a.rowBlock, a.invRowBlock, a.shard, a.nShards);
  const int si = (int)udiv_small(s, nAA), sj = (int)(s - (unsigned)si * nAA);
  float rx, ry;
  const V3 dir = sample_dir(a.cam, x, gy, si, sj, rx, ry);

  // Primary-ray cull over the wave's sample directions (wave converged).
  uint64_t primSel = ~0ull;
  bool usePrim = false;
  if (hasSel) {
    primSel = gsel;
    usePrim = true;
  } else if (RTG_PROBE_FLOOR < 2 && !Sc::kIsBvh && a.n <= 64) {  // (BVH scenes: n > 64)
    float x0, x1, y0, y1;
    // Wave-uniform: do the wave's valid pixels lie in one row?  Then the
    // bounds are four lanes' values, since every float step of main.cpp:
    // 419-426 is monotone: rx grows with x and j (lane 0 has the smallest,
    // the last pixel's j = nAA-1 lane the largest) and ry with i (lane 0, and
    // lane nAA(nAA-1)).  Otherwise reduce across the wave.
    const unsigned nv = (unsigned)((total - p0 < PPW) ? (total - p0) : PPW);  // >= 1
    const bool oneRow = col0 + nv - 1 < a.W;
    if (oneRow && !kShfl) {
      x0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rx), 0));
      x1 = __int_as_float(
          __builtin_amdgcn_readlane(__float_as_int(rx), (int)((nv - 1) * SP + nAA - 1)));
      y0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry), 0));
      y1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ry), (int)((nAA - 1) * nAA)));
    } else {
      x0 = valid ? rx : 3.0e38f;
      x1 = valid ? rx : -3.0e38f;
      y0 = valid ? ry : 3.0e38f;
      y1 = valid ? ry : -3.0e38f;
      for (int off = 32; off > 0; off >>= 1) {
        x0 = fminf(x0, __shfl_xor(x0, off));
        x1 = fmaxf(x1, __shfl_xor(x1, off));
        y0 = fminf(y0, __shfl_xor(y0, off));
        y1 = fmaxf(y1, __shfl_xor(y1, off));
      }
    }
    const PrimBundle pb = primary_bundle(x0, x1, y0, y1, a.cam.zoom);
    bool possible = false;
    if (lane < a.n) {
      const float4 g = sc.lgeom[lane];
      possible = sc.prim_possible(pb, lane, v3(g.x, g.y, g.z));
    }
    primSel = __ballot(possible);
    usePrim = true;
  }
  V3 c = v3(0.f, 0.f, 0.f);
  unsigned long long tk0 = 0;
  if constexpr (kDiag) {
    for (int k = 0; k < kProbeSlots; ++k) sc.acc[k] = 0;
    tk0 = __builtin_amdgcn_s_memtime();
  }
#if RTG_PROBE_FLOOR >= 1  // diagnostic builds only (tools/probe_floor.py): no tracing
  (void)usePrim;
  c = vsmul(a.cam.inv, v3(dir.x, (float)__builtin_popcountll(primSel), 0.f));
#else
  if (valid) {
    sc.count(kUSample, 1);
    c = trace_sample<S, Q, kCL>(sc, dir, sc.frames(), usePrim, primSel);
    c = vsmul(kargs()->cam.inv, c);
  }
#endif
  if constexpr (kDiag) {  // wave converged again: one add per slot
    sc.acc[kProbeTotal] = __builtin_amdgcn_s_memtime() - tk0;
    if ((threadIdx.x & 63u) == 0)
      for (int k = 0; k < kProbeSlots; ++k) atomicAdd(&kargs()->diag[k], sc.acc[k]);
  }
  // Ordered per-pixel sum (whole wave converged again): every lane parks its
  // sample in its own level-0 frame slot (LDS, free again: the trace is done)
  // and each pixel's first lane reads its nAA^2 samples back in order.
  const unsigned base = pl * SP;
  V3 pix = v3(0.f, 0.f, 0.f);
  if constexpr (kShfl) {  // variant 19: cross-lane reads instead of LDS
    for (unsigned k = 0; k < SP; ++k) {
      const int src = (int)((base + k) & 63u);
      pix.x = pix.x + __shfl(c.x, src);
      pix.y = pix.y + __shfl(c.y, src);
      pix.z = pix.z + __shfl(c.z, src);
    }
  } else {
    FrameC* slot0 = sc.lfr - (threadIdx.x & 63u);  // this wave's level-0 slots
    sc.lfr->cx = c.x;
    sc.lfr->cy = c.y;
    sc.lfr->cz = c.z;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (s == 0) {
      for (unsigned k = 0; k < SP; ++k) {
        const FrameC& f = slot0[(base + k) & 63u];
        pix.x = pix.x + f.cx;
        pix.y = pix.y + f.cy;
        pix.z = pix.z + f.cz;
      }
    }
  }
  if (valid && s == 0) {
    const RTG_CONST KernelArgs* b = kargs();
    float* o = b->dst + ((size_t)lr * b->W + x) * 3;
    o[0] = canon_nan(pix.x);
    o[1] = canon_nan(pix.y);
    o[2] = canon_nan(pix.z);
  }
}

// Diagnostic builds: 100 + v are s_memtime probe builds of v (kDiag); 120 is
// the executed-work counting build of the default kernel (kCount).
template <int V>
struct IsCount {
  static constexpr bool value = V == 120;
};
template <int V>
struct IsDiag {
  static constexpr bool value = V >= 100 && V != 120;
};

// Fused query forms per variant (Scene::fuse bits, rtg_trace.h): every
// sample-kernel variant except 23 (the two-pass queries, for A/B).
template <int kVariant>
struct FuseOf {
  static constexpr int value =
      (kVariant == 23) ? 0 : (kFusePrim | kFuseCone | kFuseShadow | kFuseEnter);
};

template <int kVariant>
struct GroupsPerWave {
  static constexpr int value = (kVariant == 21) ? 4 : 1;
};

template <int kVariant>
struct SampleThreads {
  static constexpr int value = (kVariant == 14) ? kBlock : 64;
};

// One launch, one pixel group per wave: one-wave workgroups (default), or
// four-wave ones (variant 14).  kList: the compacted launch (the launcher
// guarantees a.groupList): the listed groups, dealt round-robin to the waves,
// with the cull pass's sphere masks; otherwise K consecutive groups per wave.
// Separate instantiations keep each loop's registers to itself.
// kMasks (compacted default kernel only): the launcher guarantees the
// scene's shadow/overlap and cone masks (DevScene).
// The body of the sample kernels (one per launch kind below).
template <int S, bool kLds, int kVariant, bool kBvh, bool kList, bool kMasks>
__device__ __forceinline__ void trace_samples_body(const KernelArgs& a) {
  constexpr int kThreads = SampleThreads<kVariant>::value;
  typedef typename std::conditional<kLds, const float*, cfloat_p>::type MatPtr;
  constexpr bool kCount = IsCount<kVariant>::value;
  DevScene<MatPtr, IsDiag<kVariant>::value, kThreads, kBvh, FuseOf<kVariant>::value, kMasks,
           kCount>
      sc;
  sc.count_reset();
  sc.count(kUWave, 1);  // every wave, those past the listed groups included
  const unsigned t0 = (unsigned)__builtin_amdgcn_s_memrealtime();
  stage_scene<S, kLds, kThreads>(a, sc);
  if constexpr (kVariant == 20) sc.cone = nullptr;  // A/B: no secondary-ray cone cull
  // the wave's index, wave-uniform (readfirstlane: an SGPR, so the list and
  // mask reads below are scalar loads and the group set-up is scalar work)
  const size_t gw = (size_t)blockIdx.x * (kThreads / 64) +
                    (unsigned)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // variant 15: the previous default (shadow rays screening every sphere)
  // variant 21: kGroupsPerWave consecutive pixel groups per wave, in turn
  constexpr int Q = (kVariant == 15) ? 2 : 4;
  constexpr bool kDiag = IsDiag<kVariant>::value;
  unsigned tag = 0;  // timeline tag (record_wave)
  if constexpr (kList) {
    const RTG_CONST unsigned* list = (const RTG_CONST unsigned*)a.groupList;
    // variant 24: the wave recomputes its primary cull (no cull-pass masks)
    const RTG_CONST unsigned long long* gsel = (const RTG_CONST unsigned long long*)a.groupSel;
    // List position of index idx: partition idx % kListParts (nPersist is a
    // multiple of kListParts, so a wave stays in one partition), its run-order
    // entry j = idx / kListParts (the four runs, heaviest first), or ~0u past
    // the partition's end; the run lengths are read afresh (scalar loads)
    // rather than held in SGPRs through the trace.
    auto pos = [](unsigned idx) {
      const unsigned part = idx % kListParts, j = idx / kListParts;
      const RTG_CONST KernelArgs* b = kargs();
      const RTG_CONST unsigned* gc =
          (const RTG_CONST unsigned*)b->groupCount + part * kCountStride;
      const unsigned cap = b->groupCap;
      if (b->nRuns == 8u) {  // short launches: runs 2k, 2k + 1 share [k cap, (k + 1) cap)
        unsigned jr = j;
#pragma unroll
        for (unsigned c = 0; c < 8u; ++c) {
          const unsigned n = gc[c];
          if (jr < n) return 4u * cap * part + (c >> 1) * cap + ((c & 1u) ? cap - 1u - jr : jr);
          jr -= n;
        }
        return ~0u;
      }
      const unsigned e0 = gc[0], e1 = e0 + gc[1], e2 = e1 + gc[2], e3 = e2 + gc[3];
      const unsigned r = j < e0 ? j
                       : j < e1 ? cap - 1u - (j - e0)
                       : j < e2 ? cap + (j - e1)
                       : j < e3 ? 2u * cap - 1u - (j - e2)
                                : ~0u;
      return r == ~0u ? r : 2u * cap * part + r;
    };
    record_wave_start(a, t0, gw);
    if (gw == 0) {  // the next launch's counters (KernelArgs), lane p: partition p's
      const RTG_CONST KernelArgs* b = kargs();
      const unsigned l = threadIdx.x & 63u;
      if (l < kListParts) {
        *(uint4*)(b->zeroCount + l * kCountStride) = make_uint4(0u, 0u, 0u, 0u);
        *(uint4*)(b->zeroCount + l * kCountStride + 4) = make_uint4(0u, 0u, 0u, 0u);
        if (unsigned long long* zs = b->zeroStat) zs[l * kStatStride] = 0ull;
      }
    }
    unsigned tg = t0;  // this group's start (the first one's includes the wave's set-up)
    for (unsigned idx = (unsigned)gw;; idx += kargs()->nPersist) {
      const unsigned at = pos(idx);
      if (at == ~0u) break;
      const unsigned g = __builtin_amdgcn_readfirstlane(list[at]);
      trace_group<S, Q, kDiag, decltype(sc), (kVariant == 19), (kVariant == 50)>(
          a, sc, g, kVariant != 24, kVariant != 24 ? (uint64_t)gsel[at] : 0ull);
      const unsigned now = (unsigned)__builtin_amdgcn_s_memrealtime();
      const RTG_CONST KernelArgs* b = kargs();
      if (b->groupCost != nullptr && (threadIdx.x & 63u) == 0)
        b->groupCost[g] = now - tg;  // launch-order feedback (a vector store)
      tg = now;
    }
    const unsigned at0 = a.timeline != nullptr ? pos((unsigned)gw) : ~0u;
    if (at0 != ~0u) {  // timeline tag: the wave's first group
      const unsigned at = at0;
      const unsigned g = list[at];
      tag = ((unsigned)__builtin_popcountll(gsel[at]) & 127u) | ((g < 0x1FFFFFu ? g : 0x1FFFFFu) << 7);
    }
  } else {
    constexpr int K = GroupsPerWave<kVariant>::value;
    for (int k = 0; k < K; ++k)
      trace_group<S, Q, kDiag, decltype(sc), (kVariant == 19), (kVariant == 50)>(a, sc,
                                                                                 gw * K + k);
  }
  if constexpr (kCount) sc.flush_counts(kargs()->counts);
  if constexpr (kList) record_wave_end(a, gw, tag);
  else record_wave(a, t0, gw);
}

template <int S, bool kLds, int kVariant, bool kBvh = false, bool kList = false,
          bool kMasks = false>
__global__ __launch_bounds__(SampleThreads<kVariant>::value, (MinWaves<S, kVariant, kBvh>::value))
void trace_samples_kernel(const KernelArgs a) {
  trace_samples_body<S, kLds, kVariant, kBvh, kList, kMasks>(a);
}

// The compacted default kernel of a masked scene with an SGPR budget
// (amdgpu_num_sgpr): on gfx950 a wave's SGPR allocation sets the resident-wave
// ceiling below the register allocator's model (tools/ubench/occ.hip: an SGPR
// count of 86-94 allows 7 waves per SIMD, 100+ only 6).  78 requested SGPRs
// (76 with VCC etc.) admit 8 waves, with 61 VGPRs and 5 KB of LDS per wave; the
// extra SGPR spills to VGPR lanes cost less than the eighth wave gains
// (A/B C3 1.755 vs 1.780 ms, C4 11.05 vs 11.35; resident waves per SIMD mean
// 7.1, peak 7.8, vs 6.4 / 6.8).  Instantiated for S <= 6 (trace_fn_v).
#ifndef RTG_NUM_SGPR
#define RTG_NUM_SGPR 78
#endif
template <int S>
__global__ __launch_bounds__(64, 8) __attribute__((amdgpu_num_sgpr(RTG_NUM_SGPR)))
void trace_samples_kernel_masked(const KernelArgs a) {
  trace_samples_body<S, false, 0, false, true, true>(a);
}

// Kernel variants (rtg_launch_opts.variant; results identical, speed differs):
//   0 (default) sample-parallel: one primary sample per lane, one-wave
//     workgroups, scene tables read from global memory (trace_samples_kernel),
//     fused sphere queries (FuseOf);
//     compacted launch for scenes of <= 64 spheres (cull_groups_kernel,
//     rtg_kernel.hip); falls back to 9 when nAA > 8
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
//   15 as 0 with shadow rays screening every sphere (no shadow masks)
//   18 as 0 built for 8 waves per SIMD (<= 64 VGPRs)
//   19 as 0 with shuffle reductions for the cull bounds and the pixel sum
//   20 as 0 without the secondary-ray cone cull (cone_masks)
//   21 as 0 with four consecutive pixel groups per wave
//   22 as 0 without the compacted launch (one wave per pixel group, every
//      group traced: the default before cull_groups_kernel)
//   23 as 0 with the two-pass queries (a screen loop, then a per-lane
//      candidate loop with per-lane record gathers) for primary, cone-culled,
//      shadow and entering rays: the default before the fused queries (FuseOf)
//   24 as 0 with each wave computing its primary-ray cull instead of taking
//      the cull pass's per-group sphere mask
//   50 / 59: 0 / 9 with the OpenCL kernel's semantics (RTG_SEMANTICS_OPENCL;
//     chosen by rtg_context_set_semantics, not by the variant knob)
//   (19-21, persistent sample kernels with static / atomic-queue dealing of
//    pixel groups, were removed: register spills made them slower)
//   (16, 17: as 0 with the materials/geometry staged in LDS per workgroup,
//    two- and one-wave workgroups; measured slower than the scalar-cache
//    reads in rounds 1-2 and removed in round 6: DESIGN.md §6)
//   (10-12: work-queue and workgroup-size trials of the tile kernel, removed: DESIGN.md)
//   100 + v: diagnostic build of v (s_memtime probes, rtg_diag_read); 100 = 9,
//     110 = the default sample kernel (0)
//   120 the default kernel's executed-work counting build (rtg_diag_counts):
//     same control flow, unit counters per wave (DevScene kCount)
// The one table of valid variants and their kernel kind; anything else is
// rejected (rtg_set_launch_opts, RTG_VARIANT) and trace_fn returns nullptr.
// kSemantic variants change results and are only chosen through
// rtg_context_set_semantics, never accepted as a launch option.
enum VariantKind : int { kVariantInvalid = 0, kVariantTile = 1, kVariantSample = 2 };
struct VariantInfo {
  int variant;
  int kind;
  bool semantic;
};
// The shipped library holds the default kernel (0), its tile fallback for
// nAA > 8 (9), the OpenCL-semantics forms (50, 59), the diagnostic builds of
// 9 and 0 (100, 110) and the counting build (120).  The A/B variants, each
// measured and not adopted, are compiled only into A/B
// libraries (`make AB=1`, -DRTG_AB_VARIANTS=1).
#ifndef RTG_AB_VARIANTS
#define RTG_AB_VARIANTS 0
#endif
constexpr VariantInfo kVariants[] = {
    {0, kVariantSample, false},  {9, kVariantTile, false},    {50, kVariantSample, true},
    {59, kVariantTile, true},    {100, kVariantTile, false},  {110, kVariantSample, false},
    {120, kVariantSample, false},
#if RTG_AB_VARIANTS
    {1, kVariantTile, false},    {2, kVariantTile, false},    {3, kVariantTile, false},
    {4, kVariantTile, false},    {5, kVariantTile, false},    {6, kVariantTile, false},
    {8, kVariantTile, false},    {14, kVariantSample, false}, {15, kVariantSample, false},
    {18, kVariantSample, false},
    {19, kVariantSample, false}, {20, kVariantSample, false}, {21, kVariantSample, false},
    {22, kVariantSample, false}, {23, kVariantSample, false}, {24, kVariantSample, false},
    {104, kVariantTile, false},  {108, kVariantTile, false},
#endif
};
inline const VariantInfo* variant_info(int v) {
  for (const VariantInfo& i : kVariants)
    if (i.variant == v) return &i;
  return nullptr;
}

// list: the compacted launch (kList instantiations exist for the one-wave
// sample kernels that the launcher compacts, CompactVariant).
// (launch_trace compacts every one-wave sample kernel but 21 and 22); a list
// request for any other variant gets nullptr, an error, never a wrong frame.
template <int V>
struct CompactVariant {
  static constexpr bool value = V == 0 || V == 15 || V == 18 || V == 19 || V == 20 ||
                                V == 23 || V == 24 || V == 50 || V == 110 || V == 120;
};
// list: 0 the direct launch, 1 the compacted launch, 2 the compacted launch
// of a scene with masks (kMasks instantiation of the default kernel).
template <int S, int V>
static TraceFn trace_fn_v(bool lds, int list) {
  if (list && !CompactVariant<V>::value) return nullptr;
  if constexpr (V == 0) {
    // S <= 6: the SGPR-budgeted 8-wave kernel; deeper stacks hold more LDS
    // per wave than 8 waves per SIMD admit anyway
    if (list == 2) {
      if constexpr (S <= 6) return trace_samples_kernel_masked<S>;
      else return trace_samples_kernel<S, false, 0, false, true, true>;
    }
    return list ? trace_samples_kernel<S, false, 0, false, true> : trace_samples_kernel<S, false, 0>;
  } else if constexpr (V == 120) {  // the counting build of exactly the masked kernel
    return list == 2 ? trace_samples_kernel<S, false, 120, false, true, true> : nullptr;
  } else if constexpr (V == 110) {  // the probe build of the compacted default kernel
    return list ? trace_samples_kernel<S, false, 110, false, true> : nullptr;
  } else if constexpr (V == 14) {
    return lds ? trace_samples_kernel<S, true, V> : trace_samples_kernel<S, false, V>;
  } else if constexpr (CompactVariant<V>::value) {
    return list ? trace_samples_kernel<S, false, V, false, true> : trace_samples_kernel<S, false, V>;
  } else if constexpr (V == 21 || V == 22) {
    return trace_samples_kernel<S, false, V>;
  } else if constexpr (V == 9 || V == 59 || V == 100) {
    (void)lds;  // the shipped tile kernels read the scene from global memory
    return trace_kernel<S, false, V>;
  } else {
    return lds ? trace_kernel<S, true, V> : trace_kernel<S, false, V>;
  }
}
// BVH scenes: the default kernels (and their diagnostic and OpenCL-semantics
// forms, the counting build) and the nAA > 8 tile fallback have kBvh
// instantiations; 59, 100 and the A/B variants run BVH scenes through their
// flat queries (same results, slower); the probe build 110 has none (an
// error on BVH scenes).  The launcher sizes a kBvh
// kernel's LDS by frame_lds_levels(S, true), so this list and
// has_bvh_kernel() must agree.
inline bool has_bvh_kernel(int variant) {
  return variant == 0 || variant == 50 || variant == 120 || variant == 9 ||
         (RTG_AB_VARIANTS && variant == 110);
}
template <int S>
static TraceFn trace_fn_bvh(bool lds, int variant) {
  switch (variant) {
    case 0: return trace_samples_kernel<S, false, 0, true>;
    case 50: return trace_samples_kernel<S, false, 50, true>;
    case 120: return trace_samples_kernel<S, false, 120, true>;
    case 9: (void)lds; return trace_kernel<S, false, 9, true>;
#if RTG_AB_VARIANTS
    case 110: return trace_samples_kernel<S, false, 110, true>;  // probe build, A/B libraries
#endif
    default: return nullptr;
  }
}
template <int S>
static TraceFn trace_fn(bool lds, int variant, bool bvh, int list) {
  if (bvh) {
    if (list) return nullptr;  // BVH scenes (n > 64) are never compacted
    if (TraceFn f = trace_fn_bvh<S>(lds, variant)) return f;
  }
  switch (variant) {
    case 0: return trace_fn_v<S, 0>(lds, list);
    case 9: return trace_fn_v<S, 9>(lds, list);
    case 50: return trace_fn_v<S, 50>(lds, list);
    case 59: return trace_fn_v<S, 59>(lds, list);
    case 100: return trace_fn_v<S, 100>(lds, list);
    case 110: return trace_fn_v<S, 110>(lds, list);
    case 120: return trace_fn_v<S, 120>(lds, list);
#if RTG_AB_VARIANTS
    case 1: return trace_fn_v<S, 1>(lds, list);
    case 2: return trace_fn_v<S, 2>(lds, list);
    case 3: return trace_fn_v<S, 3>(lds, list);
    case 4: return trace_fn_v<S, 4>(lds, list);
    case 5: return trace_fn_v<S, 5>(lds, list);
    case 6: return trace_fn_v<S, 6>(lds, list);
    case 8: return trace_fn_v<S, 8>(lds, list);
    case 14: return trace_fn_v<S, 14>(lds, list);
    case 15: return trace_fn_v<S, 15>(lds, list);
    case 16: return trace_fn_v<S, 16>(lds, list);
    case 17: return trace_fn_v<S, 17>(lds, list);
    case 18: return trace_fn_v<S, 18>(lds, list);
    case 19: return trace_fn_v<S, 19>(lds, list);
    case 20: return trace_fn_v<S, 20>(lds, list);
    case 21: return trace_fn_v<S, 21>(lds, list);
    case 22: return trace_fn_v<S, 22>(lds, list);
    case 23: return trace_fn_v<S, 23>(lds, list);
    case 24: return trace_fn_v<S, 24>(lds, list);
    case 104: return trace_fn_v<S, 104>(lds, list);
    case 108: return trace_fn_v<S, 108>(lds, list);
#endif
    default: return nullptr;  // not in kVariants
  }
}

// One per stack size, defined in rtg_trace_s<S>.hip.
#define RTG_DECL(k) TraceFn trace_fn_s##k(bool lds, int variant, bool bvh, int list);
RTG_DECL(1) RTG_DECL(2) RTG_DECL(3) RTG_DECL(4) RTG_DECL(5) RTG_DECL(6) RTG_DECL(7)
RTG_DECL(8) RTG_DECL(9) RTG_DECL(10) RTG_DECL(11) RTG_DECL(12) RTG_DECL(13)
RTG_DECL(14) RTG_DECL(15) RTG_DECL(16)
#undef RTG_DECL

}  // namespace rtg
