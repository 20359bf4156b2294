// rtg_trace.h — per-pixel Whitted traversal of raytracer-gamma, written for
// the CDNA4 kernels in rtg_trace_kernels.h.
//
// It computes exactly what the reference CPU path computes (raytracer.h +
// raytraceStack.h + main.cpp:411-452), bit for bit, but is restructured for a
// 64-lane wave:
//
//  * The reference's 168-byte snapshot stack (raytraceStack.h:13-35) becomes a
//    stack of 52-byte frames, one per ANCESTOR level 0..S-2.  A frame carries
//    the node colour, the pre-computed reflection child ray (the stage-1 work
//    of raytracer.h:552-618 depends only on stage-0 values, so it is done
//    before descending; same operations, same order) and the refractive
//    material index.
//  * The shared `colourSum` return register (raytracer.h:425) is kept as
//    `ret`.  Its "stale" value — read when a child hits with insignificant
//    intensity (raytracer.h:460 false branch) or when a child push was dropped
//    by a full stack (raytraceStack.h:52-58) — is always the parent's colour
//    at push time, which the code sets explicitly before every descent.
//  * Nodes at the last level (S-1) never get children: their refraction and
//    reflection children are dropped by the full stack, which the reference
//    turns into colour doubling (colour+colour, then again if the reflection
//    was significant).  The leaf path computes that directly, without a frame
//    and without the child rays.
//  * Shadow rays (raytracer.h:272-309) stop at the first blocker: blocked iff
//    some sphere has a valid root t < 1000 with |t*D|^2 < gap.  This is exact
//    because |fl(t*D)|^2 is monotone in t under round-to-nearest, so the
//    closest hit blocks whenever any hit does.  A light with incidence <= 0
//    (raytracer.h:349) contributes nothing, so its shadow ray is skipped.
//  * All per-sphere constants that the reference recomputes (r*r,
//    (r+1e-6f)^2) are precomputed on the host with the same float operation.
//
// Arithmetic follows the reference's operation order exactly; the file must
// be compiled with -ffp-contract=off and without fast-math (correctly rounded
// f32 division and sqrt are the HIP defaults and are checked by the GPU tests).
#pragma once

#include <string.h>

#include <stdint.h>
#include <math.h>

#include <type_traits>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RTG_HD __host__ __device__ __forceinline__
#else
#define RTG_HD inline
#endif

namespace rtg {

struct V3 { float x, y, z; };

RTG_HD V3 v3(float a, float b, float c) { V3 r; r.x = a; r.y = b; r.z = c; return r; }
// vec.h:34-41, operand order preserved.
RTG_HD V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
RTG_HD V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
RTG_HD V3 vmul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
RTG_HD V3 vsmul(float k, V3 b) { return v3(k * b.x, k * b.y, k * b.z); }
RTG_HD float vdot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// Correctly rounded square root and reciprocal, bit-identical to sqrtf(x)
// and 1.f / b (IEEE binary32, round to nearest), with a short sequence for
// the operand range the traversal meets and the compiler's full sequence for
// the rest (per lane; the wave skips it when no lane needs it).
//  * sqrt_rn, x in [2^-96, FLT_MAX]: s = v_sqrt_f32(x) (within 1 ulp), then
//    the neighbour s -+ 1 ulp whose residual fma(-s', s, x) shows that it is
//    the rounded root (the residuals are exact fused products; no scaling is
//    needed above 2^-96).  9 VALU instead of ~17 (the compiler's expansion
//    scales small operands and patches 0/inf with a class test).
//  * rcp_rn, b in [2^-125, 2^125]: y = v_rcp_f32(b), one Newton step
//    y + y (1 - b y) with fused operations (Markstein).  3 VALU instead of
//    the ~11 of a general division.
// tests/fpcheck/fpcheck_gpu.hip checks both against sqrtf / 1.f / b and
// against an exact (f64) rounding criterion for EVERY float in those ranges
// on the GPU (test_gpu_parity.py::test_fast_sqrt_rcp_exhaustive).
RTG_HD bool sqrt_fast_range(float x) {
  unsigned u;
  memcpy(&u, &x, 4);
  return u - 0x0F800000u <= 0x7F7FFFFFu - 0x0F800000u;  // 2^-96 <= x <= FLT_MAX
}
RTG_HD bool rcp_fast_range(float b) {
  unsigned u;
  memcpy(&u, &b, 4);
  return u - 0x01000000u <= 0x7E000000u - 0x01000000u;  // 2^-125 <= b <= 2^125
}
RTG_HD float sqrt_fast(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  float s = __builtin_amdgcn_sqrtf(x);
  const float sd = __uint_as_float(__float_as_uint(s) - 1u);
  const float su = __uint_as_float(__float_as_uint(s) + 1u);
  const float rd = fmaf(-sd, s, x);
  const float ru = fmaf(-su, s, x);
  s = (rd <= 0.f) ? sd : s;
  s = (ru > 0.f) ? su : s;
  return s;
#else
  return sqrtf(x);
#endif
}
RTG_HD float rcp_fast(float b) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float y = __builtin_amdgcn_rcpf(b);
  const float e = fmaf(-b, y, 1.0f);
  return fmaf(e, y, y);
#else
  return 1.f / b;
#endif
}
// The fallback stays a branch the wave skips when no lane needs it: the
// empty volatile asm keeps the compiler from speculating the (one-IR-op,
// long-expansion) sqrtf / fdiv into a select next to the short sequence.
RTG_HD void no_speculate() {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("");
#endif
}
// Whether any active lane needs the fallback: a wave-uniform test, so the
// common case costs one compare-to-mask and a scalar branch, with no exec-mask
// save/restore around the (skipped) fallback.
RTG_HD bool any_lane(bool b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_ballot_w64(b) != 0ull;
#else
  return b;
#endif
}
RTG_HD float sqrt_rn(float x) {
  float s = sqrt_fast(x);
  if (any_lane(!sqrt_fast_range(x))) {
    no_speculate();
    if (!sqrt_fast_range(x)) s = sqrtf(x);
  }
  return s;
}
RTG_HD float rcp_rn(float b) {
  float y = rcp_fast(b);
  if (any_lane(!rcp_fast_range(b))) {
    no_speculate();
    if (!rcp_fast_range(b)) y = 1.f / b;
  }
  return y;
}
// Approximate reciprocal square root (v_rsq_f32, ~1 ulp) for conservative
// culls only (primary_bundle, the cone cull); never for results.
RTG_HD float cull_rsq(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rsqf(x);
#else
  return 1.0f / sqrtf(x);
#endif
}
RTG_HD float rtg_sqrtf(float x) { return sqrt_rn(x); }
// rcp_rn(sqrt_rn(x)) with ONE range check: for x in sqrt_fast's range the
// rounded root lies in [2^-48, 2^64], inside rcp_fast's, so both short
// sequences hold; outside it, both compiler sequences (same results).
RTG_HD float rcp_sqrt_rn(float x) {
  float y = rcp_fast(sqrt_fast(x));
  if (any_lane(!sqrt_fast_range(x))) {
    no_speculate();
    if (!sqrt_fast_range(x)) y = 1.f / sqrtf(x);
  }
  return y;
}
// vec.h:41: l = 1.f / sqrt(dot); v *= l.
RTG_HD V3 vnorm(V3 v) { float l = rcp_sqrt_rn(vdot(v, v)); return vsmul(l, v); }
// raytracer.h:235-241
RTG_HD bool significant(V3 c) { return (c.x >= 0.001f) || (c.y >= 0.001f) || (c.z >= 0.001f); }

// Camera constants of main.cpp:384-402, computed once on the host.
struct Camera {
  float xs, ys, asp, st, inv, halfW, halfH, zoom;
  int nAA;  // iterations of `for (int i = 0; i < aliasFactor; ++i)`
};

// Material record (material.h:8-14) as 8 floats; index n is the background
// material {0,0,0, 0,0,0, opacity 0, n 1.0} (raytracer.h:694-697).
struct Mat { V3 matte, gloss; float opacity, refr; };

// Fused query forms (Scene::fuse bits; results identical, speed differs):
// screen and exact root test in ONE wave-uniform loop over a sphere subset,
// with scalar record loads, instead of a screen pass plus a per-lane
// candidate loop with per-lane record gathers.
enum : int { kFusePrim = 1, kFuseCone = 2, kFuseShadow = 4, kFuseEnter = 8 };

// Diagnostic probe slots (scenes without probes implement them as no-ops).
// Operation counters (host simulation only; sc.count is a no-op on the GPU).
// The kU* slots are the executed-work units of the roofline:
// one count per execution of a code unit; the device counting build (kernel
// variant 120, DevScene kCount) sums them per WAVE (a unit some lane of the
// wave executes costs the whole wave its instructions) and per lane.
enum : int { kCntSamples = 0, kCntPrimQ, kCntPrimSel, kCntPrimCand, kCntEnterQ, kCntEnterOK,
             kCntFullQ, kCntFullCand, kCntShadowQ, kCntShadowSel, kCntShadowCand,
             kCntContainMasked, kCntContainSel, kCntContainFull, kCntRefraction, kCntReflPush,
             kCntBvhNodeTests, kCntBvhSphereTests, kCntConeQ, kCntConeSel,
             kCntBvhShadowQ, kCntBvhShadowNodeTests, kCntBvhShadowSphereTests,
             kUQuery,       // make_query: a, 4a, 2a, screen factors, 1/2a
             kUPrimIter,    // closest_hit_sel_fused: one sphere's primary radicand
             kUPrimExact,   // ... its root test (sqrt, two quotients, accept, best)
             kUSelIter,     // closest_sel_fused: pass-1 screen of one sphere
             kUSelExact,    // ... exact root test + closest update
             kUShdIter,     // blocked_sel_fused: pass-1 screen of one sphere
             kUShdExact,    // ... exact root test + blocking test
             kUEnterHead,   // closest_enter_fused: sphere h's root test + guard tests
             kUEnterIter,   // ... one overlap sphere, loaded
             kUEnterExact,  // ... its root test + lexicographic update
             kUFullGroup,   // candidate_mask: pass-1 screens of 4 spheres
             kUFullExact,   // closest_hit_mask / blocked_mask: one candidate's root test
             kUBvhNode,     // BVH node visit: pop, records, front-to-back push
             kUBvhSlot,     // BVH slot: distance prune + bound / sphere screen
             kUBvhExact,    // BVH leaf sphere: root test + update (closest or shadow)
             kUContIter,    // primary_container_sel: one sphere's containment test
             kUCont4,       // primary_container: 4 spheres' containment tests
             kUContBvhNode, // container_bvh: one node (4 slots)
             kUCone,        // cone cull set-up (bundle axis, tier, cell)
             kUMaskIter,    // mask-union waterfall step (distinct sphere of the wave)
             kUNode,        // stage-0 node: query dispatch, miss / hit bookkeeping
             kUShade,       // significant hit: P, N, guard test, material, colour
             kULight,       // matte_light: one light (L - P, facing-away pre-test)
             kUShadow,      // a shadow ray's query set-up (incidence > 0)
             kULit,         // an unblocked light's intensity and sum
             kURefr,        // refraction with the refracted ray (interior node)
             kURefrLeaf,    // refraction without the ray (leaf: R and target only)
             kUPush,        // reflection child ray (calculateReflection) + frame write
             kUDescend,     // descent to the refraction child (frame, I, o, d)
             kUUnwind,      // one unwind step (stage 1/2 colour sums)
             kUSample,      // one primary sample: ray set-up, cull hand-over, pixel sum
             kUBvhPass,     // (diagnostic) a BVH child-node screen passes for the lane
             kUCapIter,     // blocked_cap: one capsule-list sphere (record, screen)
             kUOvIter,      // closest_enter_list / container_list: one overlap-list sphere
             kUDiagShdSame,   // (diagnostic) shadow query, every lane on one hit sphere
             kUDiagEnterAll,  // (diagnostic) closest query, every lane's ray entered a sphere
             kUDiagEnterSame, // (diagnostic) ... the same sphere
             kUDiagContSame,  // (diagnostic) refraction target query, one hit sphere
             kULightDir,    // matte_light: a light no facing-away test excluded (direction)
             kUDiagInsig,     // (diagnostic) stage-0 query; lane value: intensity insignificant
             kUDiagInsigAll,  // (diagnostic) stage-0 query whose every active lane is insignificant
             kUWave,        // one wave of the sample kernel: prologue, list walk, epilogue
             kCntSlots };
enum : int { kProbeClosest = 0, kProbeShadow = 1, kProbeRefraction = 2, kProbeTotal = 3,
             kProbeMatte = 4, kProbePush = 5, kProbeUnwind = 6, kProbeShade = 7,
             kProbeSlots = 8 };
// Finer regions, recorded only by RTG_DIAG_SPLIT builds (in slots 1, 4, 5, 6
// instead of shadow, matte, push, unwind): the shading set-up after the
// closest-hit query (hit record, P, N, material, guard test), the refraction
// target's containment search, the Fresnel factor, and sinA1.
#ifndef RTG_DIAG_SPLIT
#define RTG_DIAG_SPLIT 0
#endif
enum : int { kProbeSplitBase = 100, kProbeSplitSetup = 101, kProbeSplitContain = 104,
             kProbeSplitFresnel = 105, kProbeSplitSin = 106 };

// Split frame used by trace_sample: the part every unwind step touches
// (colour, stage flags, refractive material) is 16 bytes and can live in LDS;
// the pre-computed reflection ray is only read when that child is traced.
struct FrameC {
  float cx, cy, cz;
  unsigned meta;  // rm << 10 | inside << 9 | (1 + origin sphere) << 2 | flags
                  // (bit0: stage 2, bit1: reflection child significant;
                  // inside: the reflection child starts inside the origin sphere)
};
struct FrameR { V3 ro, rd, rI; };

// Local (private-memory) storage of the colour part, used when the scene does
// not provide per-lane LDS frames.
// Frame stores provide get(lv) / set(lv, frame) (trace_sample).
template <int NF>
struct LocalFrames {
  FrameC f[NF];
  RTG_HD FrameC get(int lv) const { return f[lv]; }
  RTG_HD void set(int lv, const FrameC& v) { f[lv] = v; }
};

// One ancestor frame.
struct Frame {
  V3 colour;
  V3 ro, rd, rI;   // pre-computed reflection child ray (valid if sig)
  int rm;          // refractive material index of this node (stage-1/2 use)
  int flags;       // bit0: stage==2, bit1: reflection child significant
};

// ---------------------------------------------------------------------------
// Quotient of the root test.  The reference divides twice per candidate
// sphere, (-b +- root) / (2a) (raytracer.h:112-116); both share the
// denominator, so the kernel takes y = 1/den once per ray (correctly rounded)
// and forms each quotient as q1 = fl(a*y) refined twice with FMA residuals
// (Markstein: q1 is faithful and y is within half an ulp of 1/den, so the
// second residual is exact and the result is the correctly rounded quotient).
// A quotient is only ever used through `u > 1e-5f && u < 10000.f` and its
// exact value when that holds; tests/fpcheck/markstein_check.c verifies that
// property over 1e9 operand pairs (incl. subnormal numerators and values at
// both thresholds) for den in [2^-60, 2^60].  Outside that range the correctly
// rounded division is used.
struct RayQ {
  V3 o, d;
  float a4, den, y;
  float ap;       // pass-1 screen: a (1 - K), K = 2^-16 (pass1_rad)
  bool fast;
  bool slow;      // some active lane of the wave is not `fast` (wave-uniform)
};

RTG_HD RayQ make_query(V3 o, V3 d) {
  RayQ q;
  q.o = o;
  q.d = d;
  const float a = vdot(d, d);
  q.a4 = 4.0f * a;
  q.den = 2.0f * a;
  q.ap = a * (1.0f - 0x1p-16f);
  q.fast = (q.den >= 0x1p-60f) && (q.den <= 0x1p60f);
  q.slow = any_lane(!q.fast);
  // y is used only when q.fast (quot, quot_k<true>); den is then in
  // [2^-60, 2^60], inside rcp_fast's range, so no range check is needed.
  q.y = rcp_fast(q.den);
  return q;
}

// The Markstein quotient for every lane; lanes outside its range take the
// division in a branch the wave skips unless one of its lanes needs it
// (q.slow, decided once per query).
RTG_HD float quot(float x, const RayQ& q) {
  const float q0 = x * q.y;
  const float r0 = fmaf(-q0, q.den, x);
  const float q1 = fmaf(r0, q.y, q0);
  const float r1 = fmaf(-q1, q.den, x);
  float r = fmaf(r1, q.y, q1);
  if (q.slow) {
    no_speculate();
    if (!q.fast) r = x / q.den;
  }
  return r;
}

// The same with the quotient path chosen for the whole wave (kFast: every
// lane's denominator is in the Markstein range, all(q.fast)).
template <bool kFast>
RTG_HD float quot_k(float x, const RayQ& q) {
  if constexpr (kFast) {
    const float q0 = x * q.y;
    const float r0 = fmaf(-q0, q.den, x);
    const float q1 = fmaf(r0, q.y, q0);
    const float r1 = fmaf(-q1, q.den, x);
    return fmaf(r1, q.y, q1);
  } else {
    return quot(x, q);
  }
}

// No root of the reference's test can be accepted (raytracer.h:105-138)
// when, in its own values b and cc, b > 0 and b < 16 a and either cc >= 0
// (the origin outside and the centre behind it: radicand <= fl(b b), so
// -b + root <= 2^-23 b (exact, Sterbenz) and u0 <= 2^-23 b / 2a < 1e-6), or
// cc < 0 with -cc < 8e-6 b (the origin inside by a rounding, typically the
// hit point on its own sphere: root <= (b + 2a |cc| / b)(1 + 2.0001 eps), so
// u0 <= |cc| / b (1 + 3 eps) + 2.0001 eps b / a (1 + eps) < 8.96e-6 < 1e-5);
// u1 < 0 in both cases.  Shadow rays test their own hit sphere (in their
// mask): its wave then skips the square root and the quotients unless a
// lane grazes it.  tests/test_oracle.py::
// test_no_root_is_exact checks it against the reference's test.
// Used by the masked scenes' shadow queries (C3 -0.9 %, C4 -1 %); in the
// BVH scenes' it cost the BVH kernel two VGPRs past 80, one wave per SIMD
// less: C5 145.5 vs 130.1 ms.
#ifndef RTG_NOROOT_K  // the inside bound (tests probe larger ones)
#define RTG_NOROOT_K 8e-6f
#endif
RTG_HD bool no_root(const RayQ& q, float b, float cc) {
  return b > 0.f && b < 4.f * q.a4 && (cc >= 0.f || -cc < RTG_NOROOT_K * b);
}

// Per-sphere ray test, raytracer.h:81-141.  Returns the smallest root in
// (1e-5, 10000) or 10000 when none (`res` tells).  kNone: lanes where
// no_root holds skip the roots (same answer).
// Both quotients' division fallback in one wave-uniform branch instead of
// one each (same values).
template <bool kNone = false>
RTG_HD float ray_sphere(const RayQ& q, V3 c, float r2, bool& res) {
  V3 disp = vsub(q.o, c);
  const float b = 2.0f * vdot(q.d, disp);
  const float cc = vdot(disp, disp) - r2;
  const float radicand = (b * b) - (q.a4 * cc);
  float sm = 10000.f;
  res = false;
  if (radicand >= 0.0f && !(kNone && no_root(q, b, cc))) {
    const float root = rtg_sqrtf(radicand);
    const float x0 = -b + root, x1 = -b - root;
    float u0 = quot_k<true>(x0, q);
    float u1 = quot_k<true>(x1, q);
    if (q.slow) {
      no_speculate();
      if (!q.fast) {
        u0 = x0 / q.den;
        u1 = x1 / q.den;
      }
    }
    if (u0 > 1.0e-5f) { if (u0 < sm) { sm = u0; res = true; } }
    if (u1 > 1.0e-5f) { if (u1 < sm) { sm = u1; res = true; } }
  }
  return sm;
}

// The BVH leaves' and sphere lists' root test (a select form of it, branch-
// free for lanes with a negative radicand, measured neutral on C5: DESIGN.md
// §4 item 45).
template <bool kNone = false>
RTG_HD float ray_sphere_leaf(const RayQ& q, V3 c, float r2, bool& res) {
  return ray_sphere<kNone>(q, c, r2, res);
}

template <bool kFast, bool kNone = false>
RTG_HD float ray_sphere_k(const RayQ& q, V3 c, float r2, bool& res) {
  V3 disp = vsub(q.o, c);
  const float b = 2.0f * vdot(q.d, disp);
  const float cc = vdot(disp, disp) - r2;
  const float radicand = (b * b) - (q.a4 * cc);
  float sm = 10000.f;
  res = false;
  if ((radicand >= 0.0f) & !(kNone && no_root(q, b, cc))) {  // one branch (blocked_sel_fused)
    const float root = rtg_sqrtf(radicand);
    const float u0 = quot_k<kFast>(-b + root, q);
    const float u1 = quot_k<kFast>(-b - root, q);
    if (u0 > 1.0e-5f) { if (u0 < sm) { sm = u0; res = true; } }
    if (u1 > 1.0e-5f) { if (u1 < sm) { sm = u1; res = true; } }
  }
  return sm;
}

// Closest hit, raytracer.h:145-194 (first index wins ties; minT starts 1000).
template <class Scene>
RTG_HD int closest_hit(const Scene& sc, V3 o, V3 d, float& tOut) {
  const RayQ q = make_query(o, d);
  float minT = 1000.f;
  int best = -1;
  const unsigned n = sc.n;
  for (unsigned i = 0; i < n; ++i) {
    float r2;
    V3 c = sc.sphere(i, r2);
    bool res;
    float t = ray_sphere(q, c, r2, res);
    if (res && t < minT) { minT = t; best = (int)i; }
  }
  tOut = minT;
  return best;
}

// Shadow query, raytracer.h:272-309 (see header note for the early exit).
template <class Scene>
RTG_HD bool blocked(const Scene& sc, V3 o, V3 d, float gap) {
  const RayQ q = make_query(o, d);
  const unsigned n = sc.n;
  for (unsigned i = 0; i < n; ++i) {
    float r2;
    V3 c = sc.sphere(i, r2);
    bool res;
    float t = ray_sphere(q, c, r2, res);
    if (res && t < 1000.f) {
      V3 dist = vsmul(t, d);
      if (vdot(dist, dist) < gap) return true;
    }
  }
  return false;
}

RTG_HD int lowest_bit(unsigned m) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_ctz(m);
#else
  return __builtin_ctz(m);
#endif
}

// raytracer.h:245-270: the first sphere i whose (r_i + 1e-6)^2 bounds
// |pt - c_i|^2 (same float operations), or -1.  Four spheres per step (one
// 64-byte scalar load of containment records {c, (r + 1e-6)^2}, NaN padding
// past n never matches); the first index is the lowest set bit, and the wave
// stops once every lane has its answer.
template <class Scene>
RTG_HD int container_bvh(const Scene& sc, V3 pt);

template <class Scene>
RTG_HD int primary_container(const Scene& sc, V3 pt) {
  if (sc.has_bvh()) return container_bvh(sc, pt);
  int found = -1;
  const unsigned n4 = sc.n4;
  for (unsigned k = 0; k < n4; k += 4) {  // wave-uniform
    sc.count(kUCont4, 1);
    V3 c[4];
    float cr[4];
    sc.sphere4_contain(k, c, cr);
    unsigned bits = 0;
#pragma unroll
    for (int j = 3; j >= 0; --j) {
      const V3 dist = vsub(pt, c[j]);
      bits = (bits << 1) | ((vdot(dist, dist) <= cr[j]) ? 1u : 0u);
    }
    if (found < 0 && bits) found = (int)(k + (unsigned)lowest_bit(bits));
    if (sc.all(found >= 0)) break;
  }
  return found;
}

// Direction length bound of the masked containment test: a lane uses its hit
// sphere's overlap mask for primary_container only when |D|^2 <= this^2
// (computed in float; primary, reflection and refraction directions are
// about unit length).  See contain_reach (rtg_scene_pack.h).
constexpr float kContainDirMax = 3.0f;

// primary_container over a wave-uniform subset `sel` of spheres 0..63 (the
// union of the active lanes' overlap masks, shadow_masks in rtg_scene_pack.h):
// every sphere outside `sel` provably fails the containment test for this
// point, so the first containing sphere of `sel` in index order is the
// reference's answer.  One scalar load of a containment record per sphere,
// and of the sphere's refractive index, returned in nT (the background's when
// no sphere contains pt), so the caller needs no per-lane material gather.
template <class Scene>
RTG_HD int primary_container_sel(const Scene& sc, V3 pt, uint64_t sel, float& nT) {
  int found = -1;
  nT = sc.refr((int)sc.n);  // background material (wave-uniform: scalar load)
  for (uint64_t m = sel; m;) {  // wave-uniform
    const unsigned i = (unsigned)__builtin_ctzll(m);
    m &= ~(1ull << i);  // (an asm s_bitset0_b64: neutral)
    sc.count(kUContIter, 1);
    float cr;
    const V3 c = sc.sphere_contain(i, cr);
    const float ni = sc.refr((int)i);  // scalar load, next to the record's
    const V3 dist = vsub(pt, c);
    if (found < 0 && vdot(dist, dist) <= cr) {
      found = (int)i;
      nT = ni;
    }
    if (sc.all(found >= 0)) break;
  }
  return found;
}

// Direction cells of the secondary-ray cull (cone_masks, rtg_scene_pack.h):
// a cube map of kConeGrid x kConeGrid cells per face.  A wave whose active
// lanes all trace rays from sphere origin balls (h_lane) and whose directions
// all lie within a bundle half-angle of the first lane's direction U tests
// only the union over its lanes' h of mask (h, tier, cell(U)); two tiers of
// bundle half-angle, the tighter one used when it holds.
constexpr int kConeGrid = 8;
constexpr int kConeCells = 6 * kConeGrid * kConeGrid;
constexpr int kConeTiers = 2;
constexpr double kConeHalf[kConeTiers] = {0.20943951023931953,   // 12 degrees
                                          0.61086523819801535};  // 35 degrees
constexpr float kConeCos[kConeTiers] = {0.97814760073380569f,   // cos, rounded up
                                        0.81915204428899179f};

// Hit-point cells of the capsule lists (BVH scenes; the geometry and why
// each cell's list holds every possible blocker: rtg_scene_pack.h, above
// cell_ball): 24 cells by e = P - c_h's largest axis and its components'
// signs, and kCapFull (the whole capsule list) for points the cells do not
// cover.
constexpr unsigned kCapCubeCells = 24;
constexpr unsigned kCapCells = kCapCubeCells + 1;
constexpr unsigned kCapFull = kCapCubeCells;
// The cell of hit point P = c_h + e on a sphere of r^2 = r2 (the float r * r
// of raytracer.h:100).  Needs |e| >= r_in = |r| (1 - 2^-8): |e|^2 computed
// (relative error < 5 2^-24) >= r2 (1 - 2^-9) computed implies it for
// r2 >= 2^-120 (cell_rin takes r_in = 0 below |r| = 2^-60), else kCapFull.
// The signs of the computed components are exact (one rounded subtraction
// each) and the largest computed component is within 2^-23 of the exact
// largest, which the cells' regions allow for.  NaN: kCapFull.
RTG_HD unsigned cap_cell(V3 e, float r2) {
  const float d2 = vdot(e, e);
  if (!(d2 >= r2 * 0x1.ffp-1f)) return kCapFull;
  const float ax = fabsf(e.x), ay = fabsf(e.y), az = fabsf(e.z);
  const bool xm = ax >= ay && ax >= az, ym = !xm && ay >= az;
  const float va = xm ? e.x : ym ? e.y : e.z;
  const float vp = xm ? e.y : e.x;
  const float vq = ym || xm ? e.z : e.y;
  return (xm ? 0u : ym ? 8u : 16u) + (va < 0.f ? 4u : 0u) + (vp < 0.f ? 2u : 0u) +
         (vq < 0.f ? 1u : 0u);
}

// Cube-map cell of direction U (any length): the face of the major axis and
// a kConeGrid x kConeGrid grid over the other two coordinates / |major|.  A
// direction near a cell border may land in either cell; the masks' 1e-3 rad
// margin covers that.
// Reciprocal of the major-axis magnitude (> 0): the hardware approximation
// (1 ulp) on the GPU; the cell only needs to be consistent with its border
// margin, which is 1e-3 rad (a 1-ulp quotient moves a border by ~1e-7).
RTG_HD float cone_rcp(float m) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcpf(m);
#else
  return 1.f / m;
#endif
}
RTG_HD int cone_cell(V3 U) {
  const float ax = fabsf(U.x), ay = fabsf(U.y), az = fabsf(U.z);
  int face;
  float m, a, b;
  if (ax >= ay && ax >= az) { face = U.x > 0.f ? 0 : 1; m = ax; a = U.y; b = U.z; }
  else if (ay >= az) { face = U.y > 0.f ? 2 : 3; m = ay; a = U.x; b = U.z; }
  else { face = U.z > 0.f ? 4 : 5; m = az; a = U.x; b = U.y; }
  const float im = cone_rcp(m);
  int ia = (int)((a * im + 1.f) * (0.5f * kConeGrid));
  int ib = (int)((b * im + 1.f) * (0.5f * kConeGrid));
  ia = ia < 0 ? 0 : (ia > kConeGrid - 1 ? kConeGrid - 1 : ia);
  ib = ib < 0 ? 0 : (ib > kConeGrid - 1 ? kConeGrid - 1 : ib);
  return (face * kConeGrid + ia) * kConeGrid + ib;
}

// Query strategies (defined below): see query_closest / query_blocked.
template <int Q, class Scene>
RTG_HD int query_closest(const Scene& sc, V3 o, V3 d, float& t);
template <int Q, class Scene>
RTG_HD bool query_blocked(const Scene& sc, V3 o, V3 d, float gap);
template <class Scene>
RTG_HD bool blocked_sel(const Scene& sc, V3 o, V3 d, float gap, uint64_t sel, int hit = -1,
                        V3 hc = V3{}, float hr2 = 0.f);
template <class Scene>
RTG_HD bool blocked_cap(const Scene& sc, const RayQ& q, float gap, unsigned l, int h,
                        unsigned cell);
template <class Scene>
RTG_HD int container_list(const Scene& sc, V3 pt, int h, float& nT);
template <class Scene>
RTG_HD bool blocked_cap_lanes(const Scene& sc, V3 o, V3 d, float gap, unsigned l, int h,
                              unsigned cell, V3 ch, float r2h, bool& full);
template <class Scene>
RTG_HD int closest_bvh(const Scene& sc, const RayQ& q, float& tOut);
// Most distinct spheres a wave walks the per-sphere lists of (blocked_cap_lanes
// and friends) before its remaining lanes take the BVH.
#ifndef RTG_LIST_WALKS  // A/B builds only (tools/ab_build.sh EXTRA=-DRTG_LIST_WALKS=N)
#define RTG_LIST_WALKS 5
#endif
constexpr int kListWalks = RTG_LIST_WALKS;
// ... and for shadow rays, whose walks are keyed by (sphere, hit-point cell)
#ifndef RTG_SHADOW_WALKS
#define RTG_SHADOW_WALKS 8
#endif
constexpr int kShadowWalks = RTG_SHADOW_WALKS;
template <class Scene>
RTG_HD int container_lanes(const Scene& sc, V3 pt, int h, float& nT, bool& full);
template <class Scene>
RTG_HD int closest_enter_list(const Scene& sc, const RayQ& q, int h, float& tOut, bool& ok);

// Does the scene type run the BVH kernels (DevScene::kIsBvh)?  Host scene
// types without the member count as not.
template <class S, class = void>
struct IsBvhScene : std::false_type {};
template <class S>
struct IsBvhScene<S, std::void_t<decltype(S::kIsBvh)>> : std::bool_constant<S::kIsBvh> {};

// raytracer.h:313-367, with the incidence test hoisted ahead of the shadow ray.
// Q == 4: shadow rays test only the union of the wave's shadow masks
// (shadow_masks, rtg_scene_pack.h) for the hit sphere `hit`; `guardOK` tells
// that P lies in that sphere's guard ball (else every sphere is tested).
template <int Q, class Scene>
RTG_HD V3 matte_light(const Scene& sc, V3 P, V3 N, int hit = -1, bool guardOK = false,
                      unsigned cell = kCapFull, V3 hc = V3{}, float hr2 = 0.f) {
  V3 sum = v3(0.f, 0.f, 0.f);
  const unsigned m = sc.m;
  for (unsigned l = 0; l < m; ++l) {
    sc.count(kULight, 1);
    V3 Lpos, Lcol;
    sc.light(l, Lpos, Lcol);
    V3 dist = vsub(Lpos, P);
#if !defined(RTG_NO_FACING_TEST)
    // (Not in the BVH kernels: measured slower there, C5 141.1 vs 139.4 ms.)
    // Facing-away test ahead of the light direction: the reference's
    // incidence (raytracer.h:337-349) is inv (N.dist) with relative
    // rounding below 2^-22 of m = sum |N_k dist_k| (dir = dist * inv, inv > 0,
    // its products and sums), so e = N.dist < -2^-20 m (computed here with
    // error below 3.1 2^-24 m) proves incidence < 0: the light adds nothing and
    // casts no shadow ray.  The wave skips the light when every lane proves it
    // (m >= 2^-100 keeps the bounds relative; NaN never skips).
    if constexpr (!IsBvhScene<Scene>::value) {
      const float fe = fmaf(N.x, dist.x, fmaf(N.y, dist.y, N.z * dist.z));
      const float fm = fmaf(fabsf(N.x), fabsf(dist.x),
                            fmaf(fabsf(N.y), fabsf(dist.y), fabsf(N.z * dist.z)));
      if (sc.all(fm >= 0x1p-100f && fmaf(fm, 0x1p-20f, fe) < 0.f)) continue;
    }
#endif
    sc.count(kULightDir, 1);
    const float gap = vdot(dist, dist);
    const V3 dir = vsmul(rcp_sqrt_rn(gap), dist);  // vnorm(dist)
    const float incidence = vdot(N, dir);
    if (incidence > 0.f) {
      sc.count(kUShadow, 1);
      sc.probe_begin(kProbeShadow);
      bool blk;
      if constexpr (Q == 4) {
        if (sc.has_smask()) {
          const uint64_t su = sc.shadow_union(l, hit, guardOK);
          sc.count(kCntShadowQ, 1);
          sc.count(kCntShadowSel, __builtin_popcountll(su));
          blk = blocked_sel(sc, P, dir, gap, su, hit, hc, hr2);
        } else {
          // BVH scene: each lane's hit sphere's capsule list for light l, the
          // wave's distinct hit spheres in turn (blocked_cap_lanes); the lanes
          // it leaves, or every lane, take the one full query below (one
          // inlined BVH traversal per kind keeps the kernel's code small:
          // DESIGN.md §4 item 66)
          bool full = true;
          blk = false;
          if (sc.has_lists() && sc.all(guardOK)) {
            if (sc.all(sc.first_lane_i(hit) == hit)) sc.count(kUDiagShdSame, 1);
            blk = blocked_cap_lanes(sc, P, dir, gap, l, hit, cell, hc, hr2, full);
          }
          if (sc.any(full))
            if (full) blk = query_blocked<2>(sc, P, dir, gap);
        }
      } else {
        blk = query_blocked<Q>(sc, P, dir, gap);
      }
      sc.probe_end(kProbeShadow);
      if (!blk) {
        sc.count(kULit, 1);
        const float intensity = incidence / gap;
        sum = vadd(sum, vsmul(intensity, Lcol));
      }
    }
  }
  return sum;
}

// The f64 islands' square root and quotient without the general
// sequences' scaling and special-case fix-ups, for the operands where those
// are the identity: the same operations as the compiler's IEEE expansions
// (v_rsq_f64 / v_rcp_f64 refined by fused Newton steps), so the same
// correctly rounded results.  tests/fpcheck/fpcheck_gpu.hip checks both
// against sqrt() and a / b bit for bit on the GPU (every sinA1 operand, and
// 2^32 random Fresnel operand pairs).
//  * sqrt_d_unit(y), y = 1 - (double)(c * c) for a float c in (-1, 1)
//    (calculateRefraction, raytracer.h:683): y is 0 or in [2^-24, 1] (or NaN,
//    which stays NaN); 0 is the one operand the refinement cannot take.
//  * div_d_fresnel(a, b, fast), a = num^2 and b = den^2 >= 1e-6 the exact
//    squares of polarisedReflection's float sums (raytracer.h:388-393):
//    `fast` (the caller's float check |l|, |r| <= 2^100) keeps both in
//    (2^-20, 2^202], where the general sequence scales nothing.
RTG_HD double sqrt_d_unit(double y) {
#if defined(__HIP_DEVICE_COMPILE__)
  const double g = __builtin_amdgcn_rsq(y);
  double s = y * g;
  double h = g * 0.5;
  const double r = fma(-h, s, 0.5);
  s = fma(s, r, s);
  h = fma(h, r, h);
  double d = fma(-s, s, y);
  s = fma(d, h, s);
  d = fma(-s, s, y);
  s = fma(d, h, s);
  return y == 0.0 ? 0.0 : s;
#else
  return sqrt(y);
#endif
}
RTG_HD double div_d_fresnel(double a, double b, bool fast) {
#if defined(__HIP_DEVICE_COMPILE__)
  double y = __builtin_amdgcn_rcp(b);
  double e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  e = fma(-b, y, 1.0);
  y = fma(y, e, y);
  const double q = a * y;
  const double r = fma(-b, q, a);
  double d = fma(r, y, q);
  if (any_lane(!fast)) {  // wave-uniform test: the rare fallback
    no_speculate();
    if (!fast) d = a / b;
  }
  return d;
#else
  (void)fast;
  return a / b;
#endif
}

// raytracer.h:370-403 (f64 island).  kCL: the OpenCL kernel's all-float
// version, raytrace_kernel.cl:399-432.
template <bool kCL = false>
RTG_HD float polarised_reflection(float n1, float n2, float cosA1, float cosA2) {
  const float left = n1 * cosA1;
  const float right = n2 * cosA2;
  if constexpr (kCL) {
    const float num = left - right;
    float den = left + right;
    den *= den;
    if (den < 1.0e-6f) return 1.f;
    float refl = (num * num) / den;
    if (refl > 1.f) refl = 1.f;
    return refl;
  }
  const double num = (double)(left - right);
  double den = (double)(left + right);
  den *= den;
  // den < 1e-6: the reference returns 1 without dividing (raytracer.h:387-391);
  // here the quotient of those lanes is computed and discarded (a select, not
  // a divergent early return)
  const bool tiny = den < (double)1.0e-6f;
  const bool fast = fabsf(left) <= 0x1p100f && fabsf(right) <= 0x1p100f;
  float refl = (float)div_d_fresnel(num * num, den, fast || tiny);
  if (refl > 1.f) refl = 1.f;
  return tiny ? 1.f : refl;
}

// raytracer.h:642-815.  Computes the reflection factor R and, when wantRay,
// the refracted direction.  Returns the target material index.
// hit >= 0: the sphere P lies on, and guardOK: P passed its guard-ball test;
// then (scenes with masks) the refraction target's containment test runs over
// the wave's union of overlap masks (primary_container_sel).
template <bool kCL = false, class Scene>
RTG_HD int refraction(const Scene& sc, V3 D, V3 P, V3 N, float nSrc, bool wantRay,
                      V3& dirOut, float& R, int hit = -1, bool guardOK = false) {
  float cosA1 = vdot(D, N);
  float sinA1 = 0.f;
  if (cosA1 <= -1.0f) { cosA1 = -1.f; sinA1 = 0.f; }
  else if (cosA1 >= 1.f) { cosA1 = 1.f; sinA1 = 0.f; }
  else {
    sc.probe_begin(kProbeSplitSin);
    sinA1 = (float)sqrt_d_unit(1.0 - (double)(cosA1 * cosA1));
    sc.probe_end(kProbeSplitSin);
  }

  sc.probe_begin(kProbeSplitContain);
  const V3 testPt = vadd(vsmul(0.01f, D), P);
  int tgt;
  float nTgt;
  if (hit >= 0 && sc.has_smask()) {
    const bool ok = guardOK && vdot(D, D) <= kContainDirMax * kContainDirMax;
    const uint64_t cu = sc.contain_union(hit, ok);
    sc.count(kCntContainMasked, 1);
    sc.count(kCntContainSel, __builtin_popcountll(cu));
    tgt = primary_container_sel(sc, testPt, cu, nTgt);
    if (tgt < 0) tgt = (int)sc.n;  // background material
  } else {
    // BVH scene: the first containing sphere of each lane's hit sphere's
    // overlap list, the wave's distinct hit spheres in turn (container_lanes);
    // the lanes it leaves, or every lane, take the one full query below
    bool full = true;
    tgt = -1;
    if (hit >= 0 && sc.has_lists() &&
        sc.all(guardOK && vdot(D, D) <= kContainDirMax * kContainDirMax)) {
      if (sc.all(sc.first_lane_i(hit) == hit)) sc.count(kUDiagContSame, 1);
      tgt = container_lanes(sc, testPt, hit, nTgt, full);
    }
    if (sc.any(full)) {
      if (full) {
        sc.count(kCntContainFull, 1);
        tgt = primary_container(sc, testPt);
        nTgt = sc.refr(tgt < 0 ? (int)sc.n : tgt);
      }
    }
    if (tgt < 0) tgt = (int)sc.n;  // background material
  }
  sc.probe_end(kProbeSplitContain);
  const float ratio = nSrc / nTgt;
  const float sinA2 = ratio * sinA1;

  if (wantRay) {
    // solveQuadratic(1, 2cosA1, 1 - 1/ratio^2), algebra.h:22-65 with a = 1.
    const float qb = 2.f * cosA1;
    const float qc = 1.f - rcp_rn(ratio * ratio);
    const float rad = (qb * qb) - ((4.f * 1.f) * qc);
    float r0, r1;
    int ns;
    if (fabsf(rad) < 0.001f) {
      r0 = -qb / (2.f * 1.f);
      r1 = 0.f;
      ns = 1;
    } else {
      const float root = rtg_sqrtf(rad);
      const float den = 2.0f * 1.f;
      r0 = (-qb + root) / den;
      r1 = (-qb - root) / den;
      ns = 2;
    }
    float maxAlign = (float)-0.1;
    V3 dir = v3(0.f, 0.f, 0.f);
    {
      V3 cur = vadd(D, vsmul(r0, N));
      float al = vdot(D, cur);
      if (al > maxAlign) { maxAlign = al; dir = cur; }
    }
    if (ns == 2) {
      V3 cur = vadd(D, vsmul(r1, N));
      float al = vdot(D, cur);
      if (al > maxAlign) { maxAlign = al; dir = cur; }
    }
    dirOut = dir;
  }
  sc.probe_begin(kProbeSplitFresnel);
  float cosA2 = rtg_sqrtf(1.f - (sinA2 * sinA2));
  if (cosA1 < 0.f) cosA2 = -cosA2;
  const float Rs = polarised_reflection<kCL>(nSrc, nTgt, cosA1, cosA2);
  const float Rp = polarised_reflection<kCL>(nSrc, nTgt, cosA2, cosA1);
  // (float)((double)(Rs + Rp) * 0.5) (raytracer.h:801): the f64 product is
  // exact, so its rounding to float is the float product's.
  R = (Rs + Rp) * 0.5f;
  sc.probe_end(kProbeSplitFresnel);
  return tgt;
}

// The reflection-child records in private memory (trace_sample's fr[]):
// BVH scenes (C5: S = 8, 54 GB of record traffic per frame) store and load
// them with the nontemporal (streaming) policy, so they do not push the scene's
// node and list lines out of the caches: C5 -1 to -1.2 %;
// the masked scenes keep the default policy (C3 +7.5 %, C4 +6.6 % with it:
// their records are re-read while still cached).
template <bool kNT>
RTG_HD void store_frame_r(FrameR& dst, const FrameR& r) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (kNT) {
    __builtin_nontemporal_store(r.ro.x, &dst.ro.x);
    __builtin_nontemporal_store(r.ro.y, &dst.ro.y);
    __builtin_nontemporal_store(r.ro.z, &dst.ro.z);
    __builtin_nontemporal_store(r.rd.x, &dst.rd.x);
    __builtin_nontemporal_store(r.rd.y, &dst.rd.y);
    __builtin_nontemporal_store(r.rd.z, &dst.rd.z);
    __builtin_nontemporal_store(r.rI.x, &dst.rI.x);
    __builtin_nontemporal_store(r.rI.y, &dst.rI.y);
    __builtin_nontemporal_store(r.rI.z, &dst.rI.z);
    return;
  }
#endif
  dst = r;
}
template <bool kNT>
RTG_HD FrameR load_frame_r(const FrameR& src) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (kNT) {
    FrameR r;
    r.ro = v3(__builtin_nontemporal_load(&src.ro.x), __builtin_nontemporal_load(&src.ro.y),
              __builtin_nontemporal_load(&src.ro.z));
    r.rd = v3(__builtin_nontemporal_load(&src.rd.x), __builtin_nontemporal_load(&src.rd.y),
              __builtin_nontemporal_load(&src.rd.z));
    r.rI = v3(__builtin_nontemporal_load(&src.rI.x), __builtin_nontemporal_load(&src.rI.y),
              __builtin_nontemporal_load(&src.rI.z));
    return r;
  }
#endif
  return src;
}

// Internal reflections of BVH scenes traced as entering rays (the sphere in
// the frame record, scenes below 2048 spheres): C5 -3.3 %, DESIGN.md §4
// item 63.  0 in A/B builds only.
#ifndef RTG_BVH_INSIDE
#define RTG_BVH_INSIDE 1
#endif
#ifndef RTG_SELF_SKIP  // the masked scenes' shadow self test (blocked_sel); 0: A/B builds
#define RTG_SELF_SKIP 1
#endif
// One primary sample: rayTrace(spheres, ..., ray, bgMaterial, 0),
// raytracer.h:410-636, for stack capacity S (RTSTACK_MAXSIZE).
// kCL: the reference OpenCL kernel's semantics (raytrace_kernel.cl:641-867):
// f32 Fresnel, and the return register zeroed by the reflection push
// (:835-845), so a reflection child that leaves it stale returns 0 and a
// leaf's colour is doubled once, not twice.  sinA1 stays f64: :507 is the CPU
// path's double expression, which the .cl compiled for gfx950 evaluates in
// double too (pinned against it, oracle/build_ref_cl.sh).
template <int S, int Q, bool kCL = false, class Scene, class FStore>
RTG_HD V3 trace_sample(const Scene& sc, V3 dir0, FStore&& fc, bool usePrim = false,
                       uint64_t primSel = ~0ull) {
  constexpr int NF = (S > 1) ? (S - 1) : 1;
  FrameR fr[NF];                        // reflection child rays (private memory)
  int sp = 0;                           // == level of the node being processed
  V3 ret = v3(0.f, 0.f, 0.f);           // colourSum register
  V3 o = v3(0.f, 0.f, 0.f), d = dir0, I = v3(1.f, 1.f, 1.f);
  int rm = (int)sc.n;                   // background material
  int enterH = -1;  // Q == 4: the sphere this ray entered (refraction child), or -1
  int originH = -1;  // Q == 4: the sphere whose origin ball holds this ray's origin, or -1
  for (;;) {
    // ---------------- stage 0 (raytracer.h:454-550) ----------------
    float t;
    sc.count(kUNode, 1);
    // insignificant intensity: hit or miss would do (:455-460, :542-546); a
    // hit-or-miss BVH query for waves of only such rays measured neutral on
    // C5 (13.6 % of its stage-0 waves)
    sc.count(kUDiagInsig, significant(I) ? 0 : 1);
    if (sc.all(!significant(I))) sc.count(kUDiagInsigAll, 1);
    sc.probe_begin(kProbeClosest);
    int hit = -1;
    // lanes left for the one full query after the chain below (one inlined
    // copy of each query kind keeps the kernel's code small: DESIGN.md §4
    // item 66)
    bool full = false;
    if (usePrim) {  // the primary ray: only spheres its wave's bundle can reach
      sc.count(kCntPrimQ, 1);
      sc.count(kCntPrimSel, __builtin_popcountll(primSel));
      hit = closest_hit_sel(sc, o, d, t, primSel);
      usePrim = false;
    } else if (Q == 4 && sc.has_smask() && sc.all(enterH >= 0)) {
      // every active lane traces a ray that entered a sphere: try h + overlaps
      bool ok;
      sc.count(kUQuery, 1);
      hit = closest_enter(sc, make_query(o, d), enterH, t, ok);
      sc.count(kCntEnterQ, 1);
      sc.count(kCntEnterOK, ok ? 1 : 0);
      if (!sc.all(ok)) {  // masked scenes only: a query site of its own
        sc.count(kCntFullQ, 1);
        hit = query_closest<2>(sc, o, d, t);
      }
    } else if (Q == 4 && sc.has_cone() && sc.all(originH >= 0)) {
      // secondary rays from sphere origin balls in a narrow bundle: only the
      // spheres of their cone masks for the bundle's cell
      sc.count(kUCone, 1);
      const V3 dh = vsmul(cull_rsq(vdot(d, d)), d);  // about unit length
      const V3 U = sc.first_lane(dh);
      const float cu = vdot(dh, U);
      const int tier = sc.all(cu >= kConeCos[0]) ? 0 : sc.all(cu >= kConeCos[1]) ? 1 : -1;
      if (tier >= 0) {
        uint64_t cm = sc.cone_union(originH, (unsigned)tier, (unsigned)cone_cell(U));
        const RayQ q = make_query(o, d);
        int skip = -1;
#if RTG_SELF_SKIP
        {
          // the origin sphere (in every cone mask of its own): a ray leaving
          // its surface (refraction out of it) or starting 0.01 off it
          // (reflection) accepts no root of it when no_root holds on the
          // reference's own b and cc (ray_sphere's operations), so those lanes
          // skip it; a wave whose lanes share it and all show it drops it
          float r2o, g2o;
          const V3 co = sc.sphere_guard(originH, r2o, g2o);
          const V3 e = vsub(q.o, co);
          if (no_root(q, 2.0f * vdot(q.d, e), vdot(e, e) - r2o)) skip = originH;
          const int h0 = sc.first_lane_i(originH);
          if (sc.all(skip == h0)) cm &= ~(1ull << h0);
        }
#endif
        sc.count(kCntConeQ, 1);
        sc.count(kCntConeSel, __builtin_popcountll(cm));
        sc.count(kUQuery, 1);
        hit = closest_sel(sc, q, cm, t, skip);
      } else {  // masked scenes only: a query site of its own
        sc.count(kCntFullQ, 1);
        hit = query_closest<2>(sc, o, d, t);
      }
    } else if (Q == 4 && sc.has_lists() && sc.any(enterH >= 0)) {
      // BVH scene, rays that entered a sphere: each lane's sphere and its
      // overlap list (closest_enter_list), the wave's distinct spheres in
      // turn; the other lanes, and the lanes a list does not settle, the BVH
      if (sc.all(enterH >= 0) && sc.all(sc.first_lane_i(enterH) == enterH))
        sc.count(kUDiagEnterSame, 1);
      const RayQ q = make_query(o, d);
      sc.count(kUQuery, 1);
      bool todo = enterH >= 0, done = false;
      hit = -1;
      t = 1000.f;
      for (int k = 0; k < kListWalks && sc.any(todo); ++k) {  // wave-uniform
        const int h0 = sc.lane_with(enterH, todo);
        if (todo && enterH == h0) {
          bool ok;
          // scalar h0 (blocked_cap_lanes)
          const int hh = closest_enter_list(sc, q, sc.first_lane_i(h0), t, ok);
          if (sc.all(ok)) {
            hit = hh;
            done = true;
          }
          todo = false;
        }
      }
      full = !done;
    } else if (!sc.has_bvh()) {  // masked and flat scenes: a query site of its own
      sc.count(kCntFullQ, 1);
      hit = query_closest<Q == 4 ? 2 : Q>(sc, o, d, t);
    } else {
      if (sc.all(enterH >= 0)) sc.count(kUDiagEnterAll, 1);
      full = true;
    }
    if (sc.any(full)) {
      if (full) {
        sc.count(kCntFullQ, 1);
        hit = query_closest<Q == 4 ? 2 : Q>(sc, o, d, t);
      }
    }
    enterH = -1;
    originH = -1;
    sc.probe_end(kProbeClosest);
    sc.probe_begin(kProbeShade);
    if (hit < 0) {
      ret = vmul(I, sc.mat(rm).matte);                       // :544
    } else if (significant(I)) {                             // :460
      sc.count(kUShade, 1);
      sc.probe_begin(kProbeSplitSetup);
      V3 c;
      float g2, r2h;
      Mat mh;
      sc.hit_data(hit, c, g2, r2h, mh);  // centre, guard radius^2, r^2, material of the hit sphere
      const V3 P = vadd(o, vsmul(t, d));
      const V3 N = vnorm(vsub(P, c));
      const float op = mh.opacity;
      const float tr = 1.f - op;
      V3 colour = v3(0.f, 0.f, 0.f);
      bool guardOK = false;
      unsigned cell = kCapFull;  // the hit point's capsule-list cell (BVH scenes)
      if constexpr (Q == 4) {  // P in the hit sphere's guard ball (shadow/overlap masks)
        const V3 e = vsub(P, c);
        guardOK = vdot(e, e) <= g2;
        if (sc.has_lists() && guardOK) cell = cap_cell(e, r2h);
      }
      sc.probe_end(kProbeSplitSetup);
      if (op > 0.f) {
        V3 tmp = vmul(I, mh.matte);
        tmp = vsmul(op, tmp);
        sc.probe_begin(kProbeMatte);
        const V3 mc = matte_light<Q>(sc, P, N, hit, guardOK, cell, c, r2h);
        sc.probe_end(kProbeMatte);
        tmp = vmul(mc, tmp);
        colour = vadd(tmp, colour);
      }
      if (tr > 0.f) {
        const bool leaf = (sp >= S - 1);
        const Mat mr = sc.mat(rm);
        V3 cdir;
        float R;
        sc.probe_begin(kProbeRefraction);
        sc.count(kCntRefraction, 1);
        sc.count(leaf ? kURefrLeaf : kURefr, 1);
        const int tgt = Q == 4 ? refraction<kCL>(sc, d, P, N, mr.refr, !leaf, cdir, R, hit, guardOK)
                               : refraction<kCL>(sc, d, P, N, mr.refr, !leaf, cdir, R);
        sc.probe_end(kProbeRefraction);
        // stage-1 reflection colour, raytracer.h:563-578
        const float prod = tr * R;
        V3 rc = vsmul(prod, v3(1.f, 1.f, 1.f));
        rc = vadd(rc, vsmul(mr.opacity, mh.gloss));
        rc = vmul(I, rc);
        const bool sigR = significant(rc);
        if (!leaf) {
          sc.probe_begin(kProbePush);
          const int lv = sp < NF ? sp : NF - 1;
          FrameC f;
          f.cx = colour.x; f.cy = colour.y; f.cz = colour.z;
          // bits 2..8: 1 + the sphere whose origin ball holds the
          // reflection ray's origin P + 0.01 rd (cone cull, n <= 64), or 0;
          // bit 9: the hit came from inside that sphere (d.N > 0), so its
          // reflection turns back into it: the child is traced like an
          // entering ray (closest_enter, which checks that it stays in the
          // sphere's guard ball and else takes the general query)
          const bool origin = sc.has_cone() && guardOK;
          const bool inside = Q == 4 && origin && vdot(d, N) > 0.f;
          f.meta = ((unsigned)rm << 10) | (inside ? 0x200u : 0u) |
                   ((unsigned)(origin ? hit + 1 : 0) << 2) | (sigR ? 2u : 0u);
#if RTG_BVH_INSIDE
          if constexpr (Q == 4 && IsBvhScene<Scene>::value) {
            // BVH scenes below 2048 spheres: the same for the sphere lists
            // (closest_enter_list), the sphere in bits 10..20 and rm in 21..31
            const bool in = sc.n < 2048u && guardOK && vdot(d, N) > 0.f;
            if (sc.n < 2048u)
              f.meta = ((unsigned)rm << 21) | ((unsigned)(in ? hit + 1 : 0) << 10) |
                       (in ? 0x200u : 0u) | (sigR ? 2u : 0u);
          }
#endif
          fc.set(lv, f);
          if (sigR) {
            sc.count(kCntReflPush, 1);
            sc.count(kUPush, 1);
            // calculateReflection, raytracer.h:817-842
            const float perp = 2.f * vdot(d, N);
            const V3 rd = vnorm(vsub(d, vsmul(perp, N)));
            FrameR r;
            r.rd = rd;
            r.ro = vadd(P, vsmul(0.01f, rd));
            r.rI = rc;
            store_frame_r<IsBvhScene<Scene>::value>(fr[lv], r);
          }
          sc.count(kUDescend, 1);
          ++sp;
          ret = colour;                                       // :538
          // refraction child: calculateRefraction's refracted ray (:805-809);
          // hit from outside (cosA1 < 0): the child starts in sphere `hit`
          if (Q == 4 && vdot(d, N) < 0.f) enterH = hit;
          if (Q == 4 && guardOK && sc.has_cone()) originH = hit;  // the child starts at P
          I = vsmul((1.f - R), vsmul(tr, I));
          o = P;
          d = cdir;
          rm = tgt;
          sc.probe_end(kProbePush);
          sc.probe_end(kProbeShade);
          continue;
        }
        // Leaf: both children dropped by the full stack.
        const V3 c1 = vadd(colour, colour);
        ret = (sigR && !kCL) ? vadd(c1, c1) : c1;
      } else {
        ret = colour;
      }
    }
    // else: hit but insignificant intensity -> ret unchanged (stale)
    sc.probe_end(kProbeShade);

    // ---------------- unwind (stages 1 and 2) ----------------
    sc.probe_begin(kProbeUnwind);
    bool descend = false;
    while (sp > 0) {
      sc.count(kUUnwind, 1);
      const int lv = sp - 1 < NF ? sp - 1 : NF - 1;
      FrameC f = fc.get(lv);
      const V3 fcol = vadd(ret, v3(f.cx, f.cy, f.cz));        // :553 / :622
      ret = fcol;                                             // :617 / :626
      if ((f.meta & 3u) == 2u) {                              // stage 1, reflection
        f.cx = fcol.x; f.cy = fcol.y; f.cz = fcol.z;
        f.meta = (f.meta & ~3u) | 1u;                         // -> stage 2
        fc.set(lv, f);
        const FrameR r = load_frame_r<IsBvhScene<Scene>::value>(fr[lv]);
        o = r.ro; d = r.rd; I = r.rI; rm = (int)(f.meta >> 10);
        originH = (int)((f.meta >> 2) & 0x7Fu) - 1;
        if (Q == 4 && (f.meta & 0x200u)) enterH = originH;  // reflection back into it
#if RTG_BVH_INSIDE
        if constexpr (Q == 4 && IsBvhScene<Scene>::value) {
          if (sc.n < 2048u) {
            rm = (int)(f.meta >> 21);
            originH = -1;
            enterH = (f.meta & 0x200u) ? (int)((f.meta >> 10) & 0x7FFu) - 1 : -1;
          }
        }
#endif
        if constexpr (kCL) ret = v3(0.f, 0.f, 0.f);           // raytrace_kernel.cl:845
        descend = true;
        break;
      }
      --sp;
    }
    sc.probe_end(kProbeUnwind);
    if (!descend) return ret;
  }
}

// ---------------------------------------------------------------------------
// v2: persistent per-lane state machine.
//
// Each iteration of the outer loop performs exactly ONE ray query for every
// lane that still has work: the closest hit of a tree node's ray, or the
// shadow ray of one light (raytracer.h:272-309, answered from the closest hit
// of that ray: blocked iff a hit exists and |t*D|^2 < gap — literally the
// reference's test).  The bookkeeping between queries (shading, refraction,
// frame push/pop, moving on to the next light / node / sample) runs after the
// query and leaves the lane with its next query.  So the sphere loop, where
// the time goes, runs with every unfinished lane of the wave active whatever
// stage of its Whitted tree or which of its 9 samples each lane is in, instead
// of idling lanes whose tree was shallower (v1 above).
//
// Closest-hit query over all spheres, 4 per step (one 64-byte scalar load
// when the scene supports it), first index wins ties: raytracer.h:145-194.
template <class Scene>
RTG_HD int closest_hit4(const Scene& sc, V3 o, V3 d, float& tOut) {
  const RayQ q = make_query(o, d);
  const float a4 = q.a4;
  float minT = 1000.f;
  int best = -1;
  const unsigned n = sc.n;
  unsigned i = 0;
  for (; i + 4 <= n; i += 4) {
    V3 c[4];
    float r2[4];
    sc.sphere4(i, c, r2);
    float b[4], rad[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const V3 disp = vsub(o, c[k]);
      b[k] = 2.0f * vdot(d, disp);
      const float cc = vdot(disp, disp) - r2[k];
      rad[k] = (b[k] * b[k]) - (a4 * cc);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (rad[k] >= 0.0f) {
        const float root = rtg_sqrtf(rad[k]);
        const float u0 = quot(-b[k] + root, q);
        const float u1 = quot(-b[k] - root, q);
        float sm = 10000.f;
        bool res = false;
        if (u0 > 1.0e-5f) { if (u0 < sm) { sm = u0; res = true; } }
        if (u1 > 1.0e-5f) { if (u1 < sm) { sm = u1; res = true; } }
        if (res && sm < minT) { minT = sm; best = (int)(i + k); }
      }
    }
  }
  for (; i < n; ++i) {
    float r2;
    V3 c = sc.sphere(i, r2);
    bool res;
    float t = ray_sphere(q, c, r2, res);
    if (res && t < minT) { minT = t; best = (int)i; }
  }
  tOut = minT;
  return best;
}

// Two-pass query (default).  Pass 1 runs over every sphere with a wave-
// uniform index and no branches: it only evaluates the radicand
// (raytracer.h:95-104) and sets bit k of a per-lane candidate mask when it is
// >= 0.  Pass 2 walks each lane's candidates in increasing index order (so the
// first index still wins ties) and does the expensive part — sqrt, the two
// divisions, the root selection (raytracer.h:105-138) — with the candidate's
// record fetched per lane (`sphere_lane`).  Lanes with candidates run pass 2
// together instead of every sphere's branch running for whichever lanes need
// it.  The radicand is recomputed with the same operations, so it is the same
// value.  Spheres are processed in chunks of 32 (one mask word).
// Shift the sign bit of v into acc from the right: acc = acc << 1 | sign(v)
// (one v_alignbit_b32).  rad >= 0 <=> sign clear for every radicand the query
// can produce except NaN (b*b is never -0, so rad is never -0); a NaN with
// the sign clear becomes a candidate, which pass 2 then rejects.
RTG_HD unsigned push_sign(unsigned acc, float v) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(acc, __float_as_uint(v), 31);
#else
  unsigned u;
  memcpy(&u, &v, 4);
  return (acc << 1) | (u >> 31);
#endif
}

// Pass-1 screen for one sphere: a value whose sign bit is clear whenever the
// reference's radicand test (raytracer.h:99-108, ray_sphere above) accepts.
// With p = o - c (the same float subtraction as the reference), x = d.p and
// cs = |p|^2 - rs evaluated with fused multiply-adds, where rs is the
// sphere's SCREEN radius^2 (screen_r2: r^2 (1 + K) / (1 - K) rounded up,
// precomputed on the host), it returns
//   x^2 - a (1 - K) cs + 2^-100  >=  x^2 - a cc + K a (|p|^2 + r^2) + tiny,
// i.e. the true radicand / 4 plus a slack of K = 2^-16 relative to its terms'
// magnitude a (|p|^2 + r^2).  Both this and the reference's own evaluation
// are within ~40 ulps of those magnitudes of the exact value, so the slack
// (2^8 ulps) covers both: a sphere the reference accepts always passes; the
// few near-tangent extras are rejected by pass 2's exact test.  The 2^-100
// floor keeps the screen open where the terms underflow.  12 VALU ops per
// sphere (3 sub, 3 for x, 3 for cs, 2 fma, 1 sign shift) instead of the
// reference's 19; tests/test_oracle.py checks the superset property on
// adversarial near-tangent cases.
RTG_HD float pass1_rad(const RayQ& q, V3 c, float rs) {
  const V3 p = vsub(q.o, c);
  const float x = fmaf(q.d.x, p.x, fmaf(q.d.y, p.y, q.d.z * p.z));
  const float cs = fmaf(p.x, p.x, fmaf(p.y, p.y, fmaf(p.z, p.z, -rs)));
  return fmaf(x, x, fmaf(-q.ap, cs, 0x1p-100f));
}

// Spheres wholly behind the ray's origin.  The reference accepts no root of
// sphere i (raytracer.h:105-138) when its b = 2 d.p > 0 and c = |p|^2 - r^2
// >= 0 (the origin outside, the centre ahead of it along -d) with b < 150 a:
// then radicand <= fl(b b) so root <= b (1 + 2^-23), -b + root <= 2^-23 b
// (exact, Sterbenz), u0 <= 2^-23 b / 2a (1 + 2^-24) < 9e-6 < 1e-5, and u1 < 0.
// `behind` proves those from the pass-1 screen's fused terms (p exactly the
// reference's, x = d.p and cs = |p|^2 - rs fused, rs >= r^2):
//  * x > 2^-20 (a + cs + rs): the reference's d.p and the fused one are both
//    within 3 2^-24 sum |d_k p_k| <= 1.5 2^-24 (a + |p|^2) of the exact dot;
//  * cs > 2^-18 rs: |p|^2 computed the reference's way exceeds r^2 (fused and
//    reference sums within 2^-22 relative of |p|^2);
//  * x < 75 a and cs + rs < 2^20 a (|p| < 1024 |d|): b < 150 a with the dot's
//    error below 2^-12 a.
// tests/test_oracle.py::test_behind_is_exact checks it against the reference's
// own float test on adversarial rays.  Used by the BVH scenes' queries (BVH
// leaves, sphere lists): C5 138.8-138.9 vs 139.3-139.4 ms without; the
// masked scenes' fused loops leave it out (C3 1.485-1.496 ms without it,
// 1.508-1.532 with).
RTG_HD bool behind(float a, float x, float cs, float rs) {
  const float pp = cs + rs;
  return x > 0x1p-20f * (a + pp) && cs > 0x1p-18f * rs && x < 75.f * a &&
         pp < 0x1p20f * a;
}
// pass1_rad's screen and `behind` in one: false when sphere (c, rs) can have
// no accepted root.
RTG_HD bool screen_ahead(const RayQ& q, V3 c, float rs) {
  const V3 p = vsub(q.o, c);
  const float x = fmaf(q.d.x, p.x, fmaf(q.d.y, p.y, q.d.z * p.z));
  const float cs = fmaf(p.x, p.x, fmaf(p.y, p.y, fmaf(p.z, p.z, -rs)));
  const float v = fmaf(x, x, fmaf(-q.ap, cs, 0x1p-100f));
  return !(v < 0.f) && !behind(0.5f * q.den, x, cs, rs);
}

// Screen radius^2 of pass1_rad, computed once per sphere on the host:
// r2 (1 + 2K + 4K^2) >= r2 (1 + K) / (1 - K) in double, rounded up to float
// (NaN stays NaN, overflow goes to +inf: both keep the screen open).
inline float screen_r2(float r2) {
  const double K = 1.0 / 65536.0;
  const double v = (double)r2 * (1.0 + 2.0 * K + 4.0 * K * K);
  float f = (float)v;
  if ((double)f < v) f = nextafterf(f, __builtin_inff());
  return f;
}

// ---------------------------------------------------------------------------
// BVH queries for scenes above 64 spheres (no shadow/overlap masks there).
// The host builds a 4-wide tree of axis-aligned boxes (build_bvh,
// rtg_scene_pack.h); the wave walks it together: a node's child is visited
// when the ray passes through the child's box for ANY active lane (ballot),
// so node indices, records and the stack stay wave-uniform (scalar loads, the
// stack in the wave's LDS).  Leaf spheres get the pass-1 screen and the
// reference's exact root test per lane.  The queries take the same answers as
// the flat ones whatever order the tree visits spheres in:
//  * closest hit (raytracer.h:145-194: index order, strict <, minT from
//    1000) = the lexicographic minimum of (t, i) over accepted roots t < 1000;
//  * shadow (raytracer.h:272-309) = does ANY accepted root block;
//  * container (raytracer.h:245-270) = the minimum index whose containment
//    test passes.
//
// Why a box keeps every sphere the reference accepts.  For an accepted root
// t* of sphere i (raytracer.h:105-138) the exact point X = o + t* d lies
// within r_i + mu_i of c_i, mu_i = 2^-8 (|p_i| + |r_i|), p_i = o - c_i: with
// f(t) = |p_i + t d|^2 - r_i^2 the quadratic, |X - c_i|^2 - r_i^2 = f(t*),
// and the radicand's rounding error E <= ~60 eps a (|p_i|^2 + r_i^2) bounds
// f(t*) by ~2E / (4a) whether the exact line hits (root error near tangency)
// or misses (a radicand >= 0 by rounding only), so |X - c_i| <= r_i +
// sqrt(30 eps) (|p_i| + |r_i|), and 2^-8 is twice sqrt(30 eps).  Every ray
// origin lies in the scene's origin box B* (the camera at 0 and hit points,
// each within mu of its sphere, plus the reference's 0.01 offsets), so |p_i|
// <= P_i, the distance from c_i to B*'s farthest corner; the builder grows
// sphere i's box by e_i = 2^-8 (P_i + |r_i|) plus 2^-18 (|c_i| + |r_i| + O)
// (O the largest coordinate of B*), the rounding of the slab test below
// (3 eps (|box coordinate| + |o|) along each axis), and rounds it outward.
// X is then inside every enclosing box with a margin that covers the slab
// arithmetic, so each axis' computed entry <= t* <= its exit, hence tn <= t*
// <= tf: the box passes when t* is within reach (t* <= minT for a closest
// query; t* < sqrt(gap / a) for a shadow ray, |t* D|^2 < gap).
// tests/test_oracle.py::test_bvh_bounds_are_conservative checks the box and
// the sphere slots' prune on adversarial near-tangent / far / on-surface
// rays, and that the check finds misses with a smaller margin.
RTG_HD float rcp_hw(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcpf(x);  // v_rcp_f32, within 1 ulp
#else
  return 1.0f / x;
#endif
}
RTG_HD float sqrt_hw(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_sqrtf(x);  // v_sqrt_f32, within 1 ulp
#else
  return sqrtf(x);
#endif
}

// Per-query slab constants: inv = 1/d per axis (a component below 2^-64 in
// magnitude taken as +2^-64: the line moves by < 2^-64 t, far inside the
// box margin) and on = o * inv, so an axis' plane parameter is one fused
// step, fma(plane, inv, -on).
struct BoxQ {
  V3 inv, on;
};
RTG_HD float slab_d(float v) { return fabsf(v) < 0x1p-64f ? 0x1p-64f : v; }  // NaN stays
RTG_HD BoxQ make_boxq(const RayQ& q) {
  BoxQ b;
  b.inv = v3(rcp_hw(slab_d(q.d.x)), rcp_hw(slab_d(q.d.y)), rcp_hw(slab_d(q.d.z)));
  b.on = v3(q.o.x * b.inv.x, q.o.y * b.inv.y, q.o.z * b.inv.z);
  return b;
}
// Does the ray pass through box [lo, hi] at a parameter in [0, reach]?
// (NaN rays pass: conservative.)
RTG_HD bool slab_pass(const BoxQ& b, V3 lo, V3 hi, float reach, float& tn) {
  const float x0 = fmaf(lo.x, b.inv.x, -b.on.x), x1 = fmaf(hi.x, b.inv.x, -b.on.x);
  const float y0 = fmaf(lo.y, b.inv.y, -b.on.y), y1 = fmaf(hi.y, b.inv.y, -b.on.y);
  const float z0 = fmaf(lo.z, b.inv.z, -b.on.z), z1 = fmaf(hi.z, b.inv.z, -b.on.z);
  tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), 0.0f));
  const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), reach));
  return tn <= tf;
}

// Wave-uniform traversal stack: 64 entries of the wave's LDS area
// (sc.bvh_stack()).  Every active lane writes the same entry and reads it
// back (LDS accesses of one wave complete in order); the popped index is made
// scalar with v_readfirstlane.  (A stack in the lanes of a VGPR does not
// survive the divergent callers: copies of a VGPR only move active lanes.)
struct BvhStack {
#if defined(__HIP_DEVICE_COMPILE__)
  int* v;
  unsigned sp = 0;
  __device__ __forceinline__ explicit BvhStack(int* lds) : v(lds) {}
  __device__ __forceinline__ void push(int x) {  // x, sp wave-uniform
    v[sp] = x;
    ++sp;
  }
  __device__ __forceinline__ int pop() {
    --sp;
    return __builtin_amdgcn_readfirstlane(v[sp]);
  }
#else
  int v[64];
  unsigned sp = 0;
  explicit BvhStack(int*) {}
  void push(int x) { v[sp++] = x; }
  int pop() { return v[--sp]; }
#endif
  RTG_HD bool empty() const { return sp == 0; }
};

// Distance pruning of sphere slots.  An accepted root t of sphere i lies on
// the ray no nearer than |p_i| - r_i - mu_i (mu_i above), i.e. t |d| >= |p_i|
// - r_i - mu_i.  So with rp >= r_i (1 + 2^-7) (the slot's prune radius) its
// accepted roots are beyond `reach` when
//   |p_i| (1 - 2^-8) > rp + reach,
// tested squared with p2 = |p_i|^2 (relative rounding below 2^-20 on both
// sides, covered by the two factors).  `reach` is minT |d|_up for a closest
// query (a root must be < minT, or == minT with a lower index, to win) and
// sqrt(gap)_up for a shadow ray (|t D|^2 < gap to block).
// tests/test_oracle.py::test_bvh_bounds_are_conservative checks the root
// bound on adversarial rays.
RTG_HD bool beyond(float p2, float rp, float reach) {
  const float s = rp + reach;
  return p2 * (0x1.fc02p-1f * (1.0f - 0x1p-18f)) > s * s * (1.0f + 0x1p-18f);
}
// |d| rounded up (v_sqrt_f32 is within 1 ulp).
RTG_HD float norm_up(float a) { return sqrt_hw(a) * (1.0f + 0x1p-20f); }

// BVH node record (build_bvh, rtg_scene_pack.h): kBvhWords words, read with
// two 64-byte scalar loads at the top of a node visit, so the four slots'
// tests run back to back on SGPR operands (no load latency per slot).
//   s[6k .. 6k+5]  slot k: a child node's box {lo.xyz, hi.xyz}, or a sphere's
//                  {c.xyz, screen r^2 (screen_r2), r*r (raytracer.h:100),
//                  prune radius rp}
//   ch[k]          > 0 child node, < 0 ~sphere index, 0 empty
//   cr[k]          a sphere slot's containment radius^2 (r + 1e-6f)^2
constexpr int kBvhWords = 32;
// Every node is stored 8 times, once per direction octant, with its child
// boxes in front-to-back order along that octant's diagonal by their near
// corners, then its sphere slots front to back by their near points
// (build_bvh); a query reads the copy of its wave's first lane's octant and
// pushes the passing children in that order instead of sorting them by entry
// parameter (no keys, no compare-exchanges): DESIGN.md §4 items 49, 51, 52.
constexpr unsigned kBvhCopies = 8u;
// One record of a sphere list (sphere_lists, rtg_scene_pack.h).
struct ListRec {
  V3 c;
  float rs, r2, cr, rf;
  int idx;
};
// Capsule-list records (sphere_lists, rtg_scene_pack.h): {x, y, z, r^2}, four
// to a 64-byte scalar load, the screen radius^2 derived on the device
// (cap_screen_r2).
constexpr int kCapWords = 4;
// One capsule-list record (16-byte form, kCapWords == 4): centre and r^2.
struct CapRec {
  V3 c;
  float r2;
};
// The pass-1 screen radius^2 of a 16-byte capsule record, on the device: any
// rs >= r^2 (1 + 2K + 4K^2) keeps pass1_rad's screen conservative (screen_r2
// rounds that up on the host); fma(r2, C, 2^-149) with C = (1 + 2K + 4K^2)
// (1 + 2^-22) rounded up is at least that for every r2 >= 0 (normal results
// lose under 2^-24 relative, subnormal ones under 2^-150, which the 2^-149
// covers), and NaN / inf stay NaN / inf.  A larger rs only lets more
// spheres through to the exact test, so the answer is the same.
RTG_HD float cap_screen_r2(float r2) { return fmaf(r2, 0x1.000206p+0f, 0x1p-149f); }
struct BvhRec {
  float s[24];
  int ch[4];
  float cr[4];
};

// One node of a ray query: distance pruning + pass-1 screens of its sphere
// slots (reach `reachD` in distance units), handed to `leaf(i, c, r2)` for
// the lanes that pass, then box tests of its child slots (reach `reachT` in
// ray parameter units); child nodes some active lane still needs come in the
// octant copy's front-to-back order (the nearest returned, the others pushed
// far first).  `active`: the lane still queries.  Returns the next node (> 0)
// or 0.
// The waves are scalar-issue bound (an extra scalar instruction per node
// costs 2.4 times an extra vector one), so:
//  * the sphere slots run in one unrolled pass and the box slots in a
//    second, each slot behind one wave-uniform test of its child word (an
//    empty / box / sphere if-else costs the structurizer's flow instructions
//    per slot: C5 -3.1 %, item 48);
//  * the sphere slots take the reach and activity the node's earlier sphere
//    slots left (`liveReach` = the closest query's minT, in ray units times
//    `liveDn`; `liveBlk` = the shadow query's blocked lanes), and the box
//    slots those the sphere slots left: still conservative (later visits use
//    them anyway), and a leaf hit in the node can cull its siblings (items
//    51-52).
template <class Scene, class Leaf>
RTG_HD int bvh_ray_node(const Scene& sc, const RayQ& q, const BoxQ& b, unsigned nd, bool active,
                        float reachT, float reachD, BvhStack& st, Leaf&& leaf,
                        bool shadowQ = false, unsigned oct = 0,
                        const float* liveReach = nullptr, const bool* liveBlk = nullptr,
                        float liveDn = 0.f) {
  BvhRec r;
  sc.bvh_rec(nd * kBvhCopies + oct, r);
  int pc[4];
  auto box_slot = [&](int k, int x) {
    const float* g = &r.s[6 * k];
    sc.count(kUBvhSlot, 1);
    sc.count(shadowQ ? kCntBvhShadowNodeTests : kCntBvhNodeTests, 1);
    float tn;
    const float rT = liveReach ? *liveReach : reachT;
    const bool act = liveBlk ? (active && !*liveBlk) : active;
    const bool pass = act && slab_pass(b, v3(g[0], g[1], g[2]), v3(g[3], g[4], g[5]), rT, tn);
    if (pass) sc.count(kUBvhPass, 1);
    if (sc.any(pass)) pc[k] = x;
  };
  auto sphere_slot = [&](int k, int x) {
    const float* g = &r.s[6 * k];
    sc.count(kUBvhSlot, 1);
    sc.count(shadowQ ? kCntBvhShadowSphereTests : kCntBvhSphereTests, 1);
    const V3 c = v3(g[0], g[1], g[2]);
    const V3 p = vsub(q.o, c);
    const float xd = fmaf(q.d.x, p.x, fmaf(q.d.y, p.y, q.d.z * p.z));
    const float p2 = fmaf(p.x, p.x, fmaf(p.y, p.y, p.z * p.z));
    const float cs = p2 - g[3];
    const float v = fmaf(xd, xd, fmaf(-q.ap, cs, 0x1p-100f));  // pass1_rad
    const float rD = liveReach ? *liveReach * liveDn : reachD;
    const bool act = liveBlk ? (active && !*liveBlk) : active;
    if (act && !beyond(p2, g[5], rD) && !(v < 0.f) && !behind(0.5f * q.den, xd, cs, g[3]))
      leaf((unsigned)~x, c, g[4]);
  };
#pragma unroll
  for (int k = 0; k < 4; ++k) pc[k] = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (r.ch[k] < 0) sphere_slot(k, r.ch[k]);  // wave-uniform
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (r.ch[k] > 0) box_slot(k, r.ch[k]);
  int nxt = 0;  // slots already front to back: the nearest next, the others pushed far first
#pragma unroll
  for (int k = 3; k >= 0; --k) {
    if (pc[k] > 0) {
      if (nxt > 0) st.push(nxt);
      nxt = pc[k];
    }
  }
  return nxt;
}

// The direction octant of the wave's first lane (the node copy it reads).
template <class Scene>
RTG_HD unsigned query_octant(const Scene& sc, const RayQ& q) {
  const V3 d = sc.first_lane(q.d);
  return (d.x < 0.f ? 1u : 0u) | (d.y < 0.f ? 2u : 0u) | (d.z < 0.f ? 4u : 0u);
}

// Closest-hit and shadow updates for an accepted root (BVH and list loops),
// as selects: the exact (t, index) order and the reference's |t D|^2 < gap
// test with no exec-mask branch, whose save/branch/restore costs scalar issue
// (C5 -3.2 %).  They need no root flag: ray_sphere
// returns exactly 10000 when it accepts no root, and minT <= 1000 and the
// shadow reach 1000 are below that, so t < minT, t == minT and t < 1000
// already imply an accepted root (C5 -0.5 %, item 50).
RTG_HD void take_closer(float t, int i, float& minT, int& best) {
  const bool b = (t < minT) | ((t == minT) & (i < best));
  minT = b ? t : minT;
  best = b ? i : best;
}
RTG_HD void take_blocker(float t, V3 d, float gap, bool& blk) {
  const V3 dist = vsmul(t, d);
  blk = blk | ((t < 1000.f) & (vdot(dist, dist) < gap));
}

// Closest hit: the lexicographic minimum of (t, i) over every accepted root
// below 1000 (minT from 1000, as calcIntersection).
template <class Scene>
RTG_HD int closest_bvh(const Scene& sc, const RayQ& q, float& tOut) {
  float minT = 1000.f;
  int best = -1;
  const float dn = norm_up(q.den * 0.5f);
  const BoxQ b = make_boxq(q);
  BvhStack st(sc.bvh_stack());
  const unsigned oct = query_octant(sc, q);
  unsigned nd = 0;  // the root
  for (;;) {        // wave-uniform
    sc.count(kUBvhNode, 1);
    const int nx = bvh_ray_node(sc, q, b, nd, true, minT, minT * dn, st,
                                [&](unsigned i, V3 ce, float r2) {
      sc.count(kCntFullCand, 1);
      sc.count(kUBvhExact, 1);
      bool res;
      const float t = ray_sphere_leaf(q, ce, r2, res);
      take_closer(t, (int)i, minT, best);
    }, false, oct, &minT, nullptr, dn);
    if (nx > 0) {
      nd = (unsigned)nx;
    } else {
      if (st.empty()) break;
      nd = (unsigned)st.pop();
    }
  }
  tOut = minT;
  return best;
}

// Shadow ray: blocked iff an accepted root t < 1000 has |t D|^2 < gap, so t
// < sqrt(gap / a) (1 + 2^-18) covers the float test's rounding; a lane
// outside the Markstein range (a tiny or huge) keeps the plain t < 1000.
template <class Scene>
RTG_HD bool blocked_bvh(const Scene& sc, const RayQ& q, float gap) {
  bool blk = false;
  const float reachD = norm_up(gap);
  float reachT = sqrt_hw(gap * rcp_hw(q.den * 0.5f)) * (1.0f + 0x1p-18f);
  reachT = q.fast ? fminf(reachT, 1000.f) : 1000.f;
  const BoxQ b = make_boxq(q);
  sc.count(kCntBvhShadowQ, 1);
  BvhStack st(sc.bvh_stack());
  const unsigned oct = query_octant(sc, q);
  unsigned nd = 0;  // the root
  for (;;) {        // wave-uniform
    sc.count(kUBvhNode, 1);
    const int nx = bvh_ray_node(sc, q, b, nd, !blk, reachT, reachD, st,
                                [&](unsigned, V3 ce, float r2) {
      sc.count(kCntShadowCand, 1);
      sc.count(kUBvhExact, 1);
      bool res;
      const float t = ray_sphere_leaf(q, ce, r2, res);
      take_blocker(t, q.d, gap, blk);
    }, true, oct, nullptr, &blk);
    if (sc.all(blk)) break;
    if (nx > 0) {
      nd = (unsigned)nx;
    } else {
      if (st.empty()) break;
      nd = (unsigned)st.pop();
    }
  }
  return blk;
}

// Containment: a sphere's containment ball (r + 1e-6, raytracer.h:259-264,
// which accepts at most a few ulps outside) lies inside its grown box, so a
// point outside a child's box is in none of its spheres; sphere slots take
// the reference's own test.
template <class Scene>
RTG_HD int container_bvh(const Scene& sc, V3 pt) {
  int found = 0x7FFFFFFF;
  BvhStack st(sc.bvh_stack());
  unsigned nd = 0;  // the root
  for (;;) {        // wave-uniform
    sc.count(kUContBvhNode, 1);
    BvhRec r;
    sc.bvh_rec(nd * kBvhCopies, r);
    int nxt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int x = r.ch[k];
      if (x == 0) continue;
      const float* g = &r.s[6 * k];
      if (x > 0) {
        const bool in = pt.x >= g[0] && pt.y >= g[1] && pt.z >= g[2] && pt.x <= g[3] &&
                        pt.y <= g[4] && pt.z <= g[5];
        if (sc.any(in)) {  // the last such child is the next node, no stack round trip
          if (nxt > 0) st.push(nxt);
          nxt = x;
        }
      } else {
        const V3 dist = vsub(pt, v3(g[0], g[1], g[2]));
        if (vdot(dist, dist) <= r.cr[k] && (int)~x < found) found = (int)~x;
      }
    }
    if (nxt > 0) {
      nd = (unsigned)nxt;
    } else {
      if (st.empty()) break;
      nd = (unsigned)st.pop();
    }
  }
  return found == 0x7FFFFFFF ? -1 : found;
}

// ---------------------------------------------------------------------------
// Queries of BVH scenes over the sphere lists (sphere_lists,
// rtg_scene_pack.h): the n <= 64 masks' sets as lists, walked with a
// wave-uniform index and scalar record loads, no stack.  The lanes of a wave
// on one list walk it together; a wave takes its distinct lists in turn (the
// *_lanes forms), and lanes left after a budget of walks take the BVH.

// Shadow ray from a hit point P of sphere h (guard test passed) to light l:
// only the spheres of the capsule list of (l, h, P's cell) can block it
// (shadow_masks' argument, with the cell's capsule: cell_ball), and the list
// holds the likeliest blockers first, so blocked lanes stop early; the walk
// ends once every lane on it is blocked.  Same answer as blocked_bvh: any
// blocker.
// The overlap-list loops below take records in pairs, k and k + 1, from one
// 64-byte scalar load (ov_rec2), so a wave waits on half as many loads; the
// second record of a pair past the list's end is handled as each says.
template <class Scene>
RTG_HD bool blocked_cap(const Scene& sc, const RayQ& q, float gap, unsigned l, int h,
                        unsigned cell) {
  sc.count(kUQuery, 1);
  unsigned k0, k1;
  sc.cap_range(l, (unsigned)h, cell, k0, k1);
  bool blk = false;
  // four 16-byte records per 64-byte scalar load, from the list's second
  // record (its first is h, which blocked_cap_lanes tests for every lane at
  // once); records past the list's end are the next list's (or the table's
  // padding): a real sphere can only block if it blocks, so testing it keeps
  // the answer; one exit test per load
  for (unsigned k = k0 + 1; k < k1; k += 4) {  // wave-uniform
    CapRec r[4];
    sc.cap_rec4(k, r);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sc.count(kUCapIter, 1);
      if (!blk && screen_ahead(q, r[j].c, cap_screen_r2(r[j].r2))) {
        sc.count(kUShdExact, 1);
        bool res;
        const float t = ray_sphere_leaf(q, r[j].c, r[j].r2, res);
        take_blocker(t, q.d, gap, blk);
      }
    }
    if (sc.all(blk)) break;
  }
  return blk;
}

// Closest hit of rays that entered sphere h (every active lane): as
// closest_enter_fused, with h's overlap list (index order) in place of the
// mask; `ok` false for a lane whose origin or exit point leaves B_h (the
// caller then runs the BVH query).  The winner is the lexicographic minimum of
// (t, index), which is what the reference's index-order scan keeps.
template <class Scene>
RTG_HD int closest_enter_list(const Scene& sc, const RayQ& q, int h, float& tOut, bool& ok) {
  sc.count(kUEnterHead, 1);
  float r2h, g2;
  const V3 ch = sc.sphere_guard(h, r2h, g2);
  bool res;
  const float th = ray_sphere(q, ch, r2h, res);
  const V3 e0 = vsub(q.o, ch);
  const V3 e1 = vsub(vadd(q.o, vsmul(th, q.d)), ch);
  ok = res && th < 1000.f && vdot(e0, e0) <= g2 && vdot(e1, e1) <= g2;
  tOut = 1000.f;
  if (!sc.all(ok)) return -1;
  float minT = th;
  int best = h;
  unsigned k0, k1;
  sc.ov_range((unsigned)h, k0, k1);
  auto step = [&](const ListRec& r) {
    const int j = r.idx;
    if (j == h) return;
    sc.count(kUOvIter, 1);
    if (screen_ahead(q, r.c, r.rs)) {
      sc.count(kUEnterExact, 1);
      bool rj;
      const float t = ray_sphere_leaf(q, r.c, r.r2, rj);
      take_closer(t, j, minT, best);
    }
  };
  for (unsigned k = k0; k < k1; k += 2) {  // wave-uniform
    ListRec r0, r1;
    sc.ov_rec2(k, r0, r1);
    step(r0);
    // past the list's end: the next list's sphere (or the padding record);
    // the answer is the lexicographic minimum over every sphere, so a real
    // extra sphere keeps it
    step(r1);
  }
  tOut = minT;
  return best;
}

// primary_container (raytracer.h:245-270) for refraction test points of hits
// on sphere h (every active lane; guard test passed, |D| <= kContainDirMax):
// the first containing sphere of h's overlap list in index order (the
// argument of primary_container_sel), and its refractive index in nT.
template <class Scene>
RTG_HD int container_list(const Scene& sc, V3 pt, int h, float& nT) {
  int found = -1;
  nT = sc.refr((int)sc.n);  // background material
  unsigned k0, k1;
  sc.ov_range((unsigned)h, k0, k1);
  auto step = [&](const ListRec& r) {
    sc.count(kUOvIter, 1);
    const V3 dist = vsub(pt, r.c);
    if (found < 0 && vdot(dist, dist) <= r.cr) {
      found = r.idx;
      nT = r.rf;
    }
  };
  for (unsigned k = k0; k < k1; k += 2) {  // wave-uniform
    ListRec r0, r1;
    sc.ov_rec2(k, r0, r1);
    step(r0);
    // a sphere past the list's end (the next list's) cannot contain the
    // point (primary_container_sel's argument: every container is listed)
    step(r1);
    if (sc.all(found >= 0)) break;
  }
  return found;
}

// The list queries above for waves whose lanes hit different spheres (every
// lane's point in its own sphere's guard ball): the wave takes its distinct
// spheres in turn, each walked by the lanes on it (the others inactive), up
// to kListWalks of them; lanes left after that take the BVH query.  The
// answer is each lane's own list answer, so the frame is the same as with
// the BVH (the lists' arguments hold per sphere).  A coherent wave is one
// walk.
template <class Scene>
RTG_HD bool blocked_cap_lanes(const Scene& sc, V3 o, V3 d, float gap, unsigned l, int h,
                              unsigned cell, V3 ch, float r2h, bool& full) {
  const RayQ q = make_query(o, d);
  full = false;
  // h itself (every list's first record: capsule_keep's order key) for every
  // lane at once, with the lane's own centre and r^2 (the records' values);
  // the walks then start at each list's second record
  sc.count(kUShdExact, 1);
  bool res;
  bool blk = false;
  take_blocker(ray_sphere_leaf(q, ch, r2h, res), q.d, gap, blk);
  // walks keyed by (hit sphere, hit-point cell): each key's capsule list
  // (cap_cell, sphere_lists)
  const int key = (h << 5) | (int)cell;
  bool todo = !blk;
  for (int k = 0; k < kShadowWalks; ++k) {  // wave-uniform
    if (!sc.any(todo)) return blk;
    const int k0 = sc.lane_with(key, todo);
    if (todo && key == k0) {
      // k0 made scalar again inside the branch: the compiler otherwise
      // substitutes the lane's own key (equal here, but a VGPR) and the walk's
      // range and record loads become per-lane vector loads
      const int ku = sc.first_lane_i(k0);
      blk = blocked_cap(sc, q, gap, l, ku >> 5, (unsigned)ku & 31u);
      todo = false;
    }
  }
  full = todo;  // the caller's one BVH query (matte_light)
  return blk;
}
template <class Scene>
RTG_HD int container_lanes(const Scene& sc, V3 pt, int h, float& nT, bool& full) {
  int found = -1;
  bool todo = true;
  full = false;
  for (int k = 0; k < kListWalks; ++k) {  // wave-uniform
    const int h0 = sc.lane_with(h, todo);
    if (todo && h == h0) {
      found = container_list(sc, pt, sc.first_lane_i(h0), nT);  // scalar h0 (above)
      todo = false;
    }
    if (!sc.any(todo)) return found;
  }
  full = todo;  // the caller's one full query (refraction)
  return found;
}

template <class Scene>
RTG_HD unsigned candidate_mask(const Scene& sc, unsigned base, unsigned cnt, const RayQ& q) {
  // Groups of 4 from the last to the first, so sphere base + k lands in bit k;
  // records past n are NaN padding (PackedScene), masked off below.
  unsigned neg = 0;
  for (int k = (int)((cnt + 3u) & ~3u) - 4; k >= 0; k -= 4) {
    sc.count(kUFullGroup, 1);
    V3 c[4];
    float r2[4];
    sc.sphere4_screen(base + (unsigned)k, c, r2);
#pragma unroll
    for (int j = 3; j >= 0; --j) neg = push_sign(neg, pass1_rad(q, c[j], r2[j]));
  }
  const unsigned all = cnt >= 32u ? ~0u : ((1u << cnt) - 1u);
  return ~neg & all;
}


template <class Scene>
RTG_HD int closest_hit_mask(const Scene& sc, V3 o, V3 d, float& tOut) {
  sc.count(kUQuery, 1);
  const RayQ q = make_query(o, d);
  if (sc.has_bvh()) return closest_bvh(sc, q, tOut);
  float minT = 1000.f;
  int best = -1;
  const unsigned n = sc.n;
  for (unsigned base = 0; base < n; base += 32) {
    const unsigned cnt = (n - base < 32u) ? (n - base) : 32u;
    unsigned mask = candidate_mask(sc, base, cnt, q);
    while (mask) {
      const unsigned i = base + (unsigned)lowest_bit(mask);
      mask &= mask - 1;
      sc.count(kCntFullCand, 1);
      sc.count(kUFullExact, 1);
      float r2;
      const V3 c = sc.sphere_lane(i, r2);
      bool res;
      const float t = ray_sphere(q, c, r2, res);
      if (res && t < minT) { minT = t; best = (int)i; }
    }
  }
  tOut = minT;
  return best;
}

// Shadow query with the two-pass scheme; stops at the first blocker.
template <class Scene>
RTG_HD bool blocked_mask(const Scene& sc, V3 o, V3 d, float gap) {
  sc.count(kUQuery, 1);
  const RayQ q = make_query(o, d);
  if (sc.has_bvh()) return blocked_bvh(sc, q, gap);
  const unsigned n = sc.n;
  for (unsigned base = 0; base < n; base += 32) {
    const unsigned cnt = (n - base < 32u) ? (n - base) : 32u;
    unsigned mask = candidate_mask(sc, base, cnt, q);
    while (mask) {
      const unsigned i = base + (unsigned)lowest_bit(mask);
      mask &= mask - 1;
      sc.count(kUFullExact, 1);
      float r2;
      const V3 c = sc.sphere_lane(i, r2);
      bool res;
      const float t = ray_sphere(q, c, r2, res);
      if (res && t < 1000.f) {
        const V3 dist = vsmul(t, d);
        if (vdot(dist, dist) < gap) return true;
      }
    }
  }
  return false;
}

// All-ones when the sign bit of v is set, else 0.
RTG_HD unsigned sign_mask(float v) {
  int32_t i;
  memcpy(&i, &v, 4);
  return (unsigned)(i >> 31);
}

// Shadow query over a wave-uniform subset `sel` of spheres 0..63 (the union
// of the wave's shadow masks): pass 1 screens only the spheres of `sel`, in
// increasing index order, one scalar load per sphere; pass 2 as blocked_mask.
// Spheres outside `sel` cannot block (shadow_masks), so the answer equals
// blocked_mask's, which equals the reference's hasClearLineOfSight.
// Fused form (sc.fuse & kFuseShadow): one wave-uniform loop over `sel` in
// index order; the lanes whose screen passes run the exact test right there
// with the sphere's r^2 from a scalar load (no per-lane record gather, no
// second loop), and the wave leaves once every lane is blocked.  Same answer:
// blocked iff any sphere of `sel` blocks.
template <bool kFast, class Scene>
RTG_HD bool blocked_sel_fused(const Scene& sc, const RayQ& q, float gap, uint64_t sel,
                              int skip = -1) {
  // One divergent branch per sphere: the lane's conditions combined without
  // short-circuit (no nested exec masks), and the blocked flag an integer in
  // a VGPR (a divergent bool lives as a lane mask in SGPRs, and every update
  // under a branch costs three scalar instructions to merge).  The masked
  // kernels are scalar-issue bound too: C3 -1.7 %, C2 -2.0 %, C4 -1.9 %
  // (DESIGN.md §4 item 69).
  unsigned blkv = 0u;
  for (uint64_t m = sel; m;) {  // wave-uniform
    const unsigned i = (unsigned)__builtin_ctzll(m);
    m &= ~(1ull << i);
    sc.count(kUShdIter, 1);
    float rs, r2, ocu;
    const V3 c = sc.sphere_fused(i, rs, r2, ocu);
    const bool cand = (blkv == 0u) & ((int)i != skip) & !(pass1_rad(q, c, rs) < 0.f);
    if (cand) {
      sc.count(kCntShadowCand, 1);
      sc.count(kUShdExact, 1);
      bool res;
      const float t = ray_sphere_k<kFast, true>(q, c, r2, res);
      const V3 dist = vsmul(t, q.d);
      blkv = (res & (t < 1000.f) & (vdot(dist, dist) < gap)) ? 1u : blkv;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    asm("" : "+v"(blkv));
#endif
    if (sc.all(blkv != 0u)) break;
  }
  return blkv != 0u;
}

template <class Scene>
RTG_HD bool blocked_sel(const Scene& sc, V3 o, V3 d, float gap, uint64_t sel, int hit,
                        V3 hc, float hr2) {
  sc.count(kUQuery, 1);
  const RayQ q = make_query(o, d);
  if (sc.fuse & kFuseShadow) {
    // The hit sphere itself (every shadow mask's own sphere): no_root on the
    // reference's own b and cc for it (ray_sphere's operations on the same
    // centre and r^2) shows for all but grazing rays that it accepts no root,
    // so it cannot block; those lanes skip it, and a wave whose lanes all hit
    // one sphere and all show it drops the sphere from the loop (DESIGN.md §4
    // item 64).
    int skip = -1;
#if RTG_SELF_SKIP
    if (hit >= 0) {
      const V3 e = vsub(q.o, hc);
      const float b = 2.0f * vdot(q.d, e);
      const float cc = vdot(e, e) - hr2;
      if (no_root(q, b, cc)) skip = hit;
      const int h0 = sc.first_lane_i(hit);
      if (sc.all(skip == h0)) sel &= ~(1ull << h0);
    }
#else
    (void)hit; (void)hc; (void)hr2;
#endif
    if (sc.all(q.fast)) return blocked_sel_fused<true>(sc, q, gap, sel, skip);
    return blocked_sel_fused<false>(sc, q, gap, sel, skip);
  }
  (void)hit; (void)hc; (void)hr2;
  for (unsigned base = 0; base < 64u; base += 32u) {
    const unsigned u = (unsigned)(sel >> base);
    unsigned cand = 0;
    for (unsigned mm = u; mm; mm &= mm - 1) {  // wave-uniform
      const unsigned k = (unsigned)__builtin_ctz(mm);
      float rs;
      const V3 c = sc.sphere_screen(base + k, rs);
      cand |= (1u << k) & ~sign_mask(pass1_rad(q, c, rs));
    }
    while (cand) {
      const unsigned i = base + (unsigned)lowest_bit(cand);
      cand &= cand - 1;
      sc.count(kCntShadowCand, 1);
      float r2;
      const V3 c = sc.sphere_lane(i, r2);
      bool res;
      const float t = ray_sphere(q, c, r2, res);
      if (res && t < 1000.f) {
        const V3 dist = vsmul(t, d);
        if (vdot(dist, dist) < gap) return true;
      }
    }
  }
  return false;
}

// Closest hit of a ray that starts inside sphere h's guard ball B_h (the
// refraction child of a hit on h from outside): sphere h's own root test
// (raytracer.h:81-141) gives t_h; when it is a hit and both the origin and the
// computed exit point o + t_h d lie in B_h (`ok`), no sphere outside h's
// overlap mask (shadow_masks, rtg_scene_pack.h) has an accepted root before
// t_h, so the reference's closest hit (raytracer.h:145-194: strict <, index
// order) is found among h and its overlap spheres, tested here in index order.
// When !ok the caller runs the full query.
// Fused form (sc.fuse & kFuseEnter), taken when every lane is `ok` (else it
// returns at once and the caller runs the full query): one wave-uniform loop
// over the union of the lanes' overlap masks, scalar record loads; a lane
// tests sphere j only when j is in its own mask (`own`).  The winner is the
// lexicographic minimum of (t, index) over h's root and the accepted roots
// of the lane's mask spheres, which is what the index-order scan with strict
// < keeps.
template <bool kFast, class Scene>
RTG_HD int closest_enter_fused(const Scene& sc, const RayQ& q, int h, float& tOut, bool& ok) {
  sc.count(kUEnterHead, 1);
  float r2, g2;
  const V3 c = sc.sphere_guard(h, r2, g2);
  bool res;
  const float th = ray_sphere_k<kFast>(q, c, r2, res);
  const V3 e0 = vsub(q.o, c);
  const V3 e1 = vsub(vadd(q.o, vsmul(th, q.d)), c);
  ok = res && th < 1000.f && vdot(e0, e0) <= g2 && vdot(e1, e1) <= g2;
  tOut = 1000.f;
  if (!sc.all(ok)) return -1;
  uint64_t own;
  const uint64_t u = sc.overlap_union(h, own);
  own &= ~(1ull << h);
  float minT = th;
  int best = h;
  for (uint64_t m = u; m;) {  // wave-uniform
    const unsigned j = (unsigned)__builtin_ctzll(m);
    m &= ~(1ull << j);
    sc.count(kUEnterIter, 1);
    float rj2;
    const V3 cj = sc.sphere(j, rj2);
    if ((own >> j) & 1ull) {
      sc.count(kUEnterExact, 1);
      bool rj;
      const float t = ray_sphere_k<kFast>(q, cj, rj2, rj);
      if (rj && (t < minT || (t == minT && (int)j < best))) { minT = t; best = (int)j; }
    }
  }
  tOut = minT;
  return best;
}

template <class Scene>
RTG_HD int closest_enter(const Scene& sc, const RayQ& q, int h, float& tOut, bool& ok) {
  if (sc.fuse & kFuseEnter) {
    if (sc.all(q.fast)) return closest_enter_fused<true>(sc, q, h, tOut, ok);
    return closest_enter_fused<false>(sc, q, h, tOut, ok);
  }
  float r2;
  const V3 c = sc.sphere_lane((unsigned)h, r2);
  bool res;
  const float th = ray_sphere(q, c, r2, res);
  const V3 e0 = vsub(q.o, c);
  const V3 e1 = vsub(vadd(q.o, vsmul(th, q.d)), c);
  const float g2 = sc.guard_r2((unsigned)h);
  ok = res && th < 1000.f && vdot(e0, e0) <= g2 && vdot(e1, e1) <= g2;
  float minT = 1000.f;
  int best = -1;
  uint64_t ov = ok ? (sc.overlap_mask((unsigned)h) & ~(1ull << h)) : 0ull;
  bool hDone = false;
  for (;;) {  // candidates in index order; h's result is already known
    const unsigned j = ov ? (unsigned)__builtin_ctzll(ov) : 64u;
    if (!hDone && (unsigned)h < j) {
      hDone = true;
      if (th < minT) { minT = th; best = h; }  // res holds when ok
      continue;
    }
    if (j == 64u) break;
    ov &= ov - 1;
    float rj2;
    const V3 cj = sc.sphere_lane(j, rj2);
    bool rj;
    const float t = ray_sphere(q, cj, rj2, rj);
    if (rj && t < minT) { minT = t; best = (int)j; }
  }
  tOut = minT;
  return best;
}

// Closest hit of any ray over a wave-uniform subset `sel` of spheres 0..63
// that holds every sphere the ray can hit (cone_masks): pass 1 screens the
// spheres of `sel` (one scalar load each), pass 2 tests the lane's candidates
// in index order, so the answer is closest_hit_mask's.
// Fused form (sc.fuse & kFuseCone): screen and exact test in one wave-uniform
// loop in index order (strict <, so the first index still wins ties).
template <bool kFast, class Scene>
RTG_HD int closest_sel_fused(const Scene& sc, const RayQ& q, uint64_t sel, float& tOut,
                             int skip = -1) {
  float minT = 1000.f;
  int best = -1;
  for (uint64_t m = sel; m;) {  // wave-uniform
    const unsigned i = (unsigned)__builtin_ctzll(m);
    m &= ~(1ull << i);
    sc.count(kUSelIter, 1);
    float rs, r2, ocu;
    const V3 c = sc.sphere_fused(i, rs, r2, ocu);
    if (((int)i != skip) & !(pass1_rad(q, c, rs) < 0.f)) {  // one branch (blocked_sel_fused)
      sc.count(kCntFullCand, 1);
      sc.count(kUSelExact, 1);
      bool res;
      const float t = ray_sphere_k<kFast>(q, c, r2, res);
      if (res && t < minT) { minT = t; best = (int)i; }
    }
  }
  tOut = minT;
  return best;
}

template <class Scene>
RTG_HD int closest_sel(const Scene& sc, const RayQ& q, uint64_t sel, float& tOut,
                       int skip) {
  if (sc.fuse & kFuseCone) {
    if (sc.all(q.fast)) return closest_sel_fused<true>(sc, q, sel, tOut, skip);
    return closest_sel_fused<false>(sc, q, sel, tOut, skip);
  }
  (void)skip;
  uint64_t cand = 0;
  for (uint64_t m = sel; m;) {  // wave-uniform
    const unsigned i = (unsigned)__builtin_ctzll(m);
    m &= ~(1ull << i);
    float rs;
    const V3 c = sc.sphere_screen(i, rs);
    cand |= (pass1_rad(q, c, rs) < 0.f) ? 0ull : (1ull << i);
  }
  float minT = 1000.f;
  int best = -1;
  while (cand) {
    const unsigned i = (unsigned)__builtin_ctzll(cand);
    cand &= cand - 1;
    sc.count(kCntFullCand, 1);
    float r2;
    const V3 c = sc.sphere_lane(i, r2);
    bool res;
    const float t = ray_sphere(q, c, r2, res);
    if (res && t < minT) { minT = t; best = (int)i; }
  }
  tOut = minT;
  return best;
}

// Closest hit restricted to a wave-uniform subset `sel` of spheres 0..63
// (bit i = sphere i may be hit; see primary_sphere_mask).  Spheres outside
// `sel` cannot produce a valid root, so the result equals closest_hit_mask's.
// Fused form (sc.fuse & kFusePrim): the roots straight from that radicand in
// the same wave-uniform loop.  bp = 2 d.c is -b (negation is exact), so
// -b + root = bp + root and -b - root = bp - root bit for bit (when b is a
// zero, its sign changes neither sum nor the accept decision).
template <bool kFast, class Scene>
RTG_HD int closest_hit_sel_fused(const Scene& sc, const RayQ& q, uint64_t sel, float& tOut) {
  float minT = 1000.f;
  int best = -1;
  const V3 d = q.d;
  for (uint64_t m = sel; m;) {  // wave-uniform
    const unsigned i = (unsigned)__builtin_ctzll(m);
    m &= ~(1ull << i);
    sc.count(kUPrimIter, 1);
    float rs, r2, oc;
    const V3 c = sc.sphere_fused(i, rs, r2, oc);
    const float bp = 2.0f * vdot(d, c);
    const float rad = (bp * bp) - (q.a4 * oc);
    if (rad >= 0.0f) {
      sc.count(kCntPrimCand, 1);
      sc.count(kUPrimExact, 1);
      const float root = rtg_sqrtf(rad);
      const float u0 = quot_k<kFast>(bp + root, q);
      const float u1 = quot_k<kFast>(bp - root, q);
      float sm = 10000.f;
      bool res = false;
      if (u0 > 1.0e-5f) { if (u0 < sm) { sm = u0; res = true; } }
      if (u1 > 1.0e-5f) { if (u1 < sm) { sm = u1; res = true; } }
      if (res && sm < minT) { minT = sm; best = (int)i; }
    }
  }
  tOut = minT;
  return best;
}

template <class Scene>
RTG_HD int closest_hit_sel(const Scene& sc, V3 o, V3 d, float& tOut, uint64_t sel) {
  sc.count(kUQuery, 1);
  const RayQ q = make_query(o, d);
  // The primary ray starts at the origin (main.cpp:417): disp = 0 - c = -c
  // exactly, so b = 2 d.disp = -(2 d.c) and b*b is (2 d.c)^2; the c term
  // |disp|^2 - r^2 is precomputed per sphere (origin_c).  Same radicand bits.
  (void)o;
  if (sc.fuse & kFusePrim) {
    if (sc.all(q.fast)) return closest_hit_sel_fused<true>(sc, q, sel, tOut);
    return closest_hit_sel_fused<false>(sc, q, sel, tOut);
  }
  float minT = 1000.f;
  int best = -1;
  uint64_t cand = 0;
  for (uint64_t m = sel; m;) {  // wave-uniform: scalar loop + scalar loads
    const unsigned i = (unsigned)__builtin_ctzll(m);
    m &= ~(1ull << i);
    float r2;
    const V3 c = sc.sphere(i, r2);
    const float b = 2.0f * vdot(d, c);
    const float rad = (b * b) - (q.a4 * sc.origin_c(i));
    cand |= (rad >= 0.0f) ? (1ull << i) : 0ull;
  }
  while (cand) {
    const unsigned i = (unsigned)__builtin_ctzll(cand);
    cand &= cand - 1;
    sc.count(kCntPrimCand, 1);
    float r2;
    const V3 c = sc.sphere_lane(i, r2);
    bool res;
    const float t = ray_sphere(q, c, r2, res);
    if (res && t < minT) { minT = t; best = (int)i; }
  }
  tOut = minT;
  return best;
}

// Conservative cull of spheres for a bundle of primary rays (origin 0,
// main.cpp:417): every ray direction is (X, Y, zoom) with X in [x0, x1],
// Y in [y0, y1] (main.cpp:432-436, before normalisation).  Returns false only
// if sphere c, r provably has no forward intersection with any such ray: the
// angle between the bundle's axis U and c exceeds the bundle's half-angle
// theta plus the sphere's angular radius alpha, compared through cosines,
// cos(angle) < cos(theta + alpha) - 2e-3 with
// cos(theta + alpha) = cos(theta) cos(alpha) - sin(theta) sin(alpha)
// (cos is 1-Lipschitz, so 2e-3 covers an angle margin of 2e-3 rad), and the
// radius inflated by 1e-3 relative + 1e-3 absolute.  Those margins are far
// above the float error of the bounds, of the hardware reciprocal square
// roots used here (about 1 ulp) and of the reference's own root test.
// Bundles wider than 60 degrees, and spheres at or around the origin, are
// never culled.

// The bundle half of the test: axis U, cos(theta) and sin(theta) of the
// bundle's half-angle, or `all` (no cull) for wide or degenerate bundles.
struct PrimBundle {
  V3 U;
  float cosT, st;
  bool all;
};
RTG_HD PrimBundle primary_bundle(float x0, float x1, float y0, float y1, float zoom) {
  PrimBundle b;
  b.all = true;
  b.U = v3(0.f, 0.f, 0.f);
  b.cosT = 1.f;
  b.st = 0.f;
  if (!(zoom != 0.f)) return b;
  const float xc = 0.5f * (x0 + x1), yc = 0.5f * (y0 + y1);
  const float ila = cull_rsq(xc * xc + yc * yc + zoom * zoom);
  b.U = v3(xc * ila, yc * ila, zoom * ila);
  float cosT = 1.f;
  const float xs[2] = {x0, x1}, ys[2] = {y0, y1};
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) {
      const float il = cull_rsq(xs[i] * xs[i] + ys[j] * ys[j] + zoom * zoom);
      cosT = fminf(cosT, (b.U.x * xs[i] + b.U.y * ys[j] + b.U.z * zoom) * il);
    }
  if (!(cosT >= 0.5f)) return b;  // wide (or NaN) bundle
  const float st2 = fmaxf(0.f, 1.f - cosT * cosT);
  b.cosT = cosT;
  b.st = st2 > 0.f ? st2 * cull_rsq(st2) : 0.f;
  b.all = false;
  return b;
}
// The sphere half: {1/|c|, sin(alpha), cos(alpha)} of sphere c, r, with the
// radius inflated to r * 1.001 + 1e-3, computed once per scene on the host
// (prim_consts, rtg_scene_pack.h; cos(alpha) = -3 for "always possible":
// the origin inside or near the sphere, or a non-finite sphere).
RTG_HD bool primary_possible(const PrimBundle& b, V3 c, float iL, float sa, float ca) {
  if (b.all) return true;
  const float cosLim = b.cosT * ca - b.st * sa;  // theta + alpha < 60 + 90 degrees
  const float cosPhi = vdot(b.U, c) * iL;
  return cosPhi >= cosLim - 2.0e-3f;
}

// Two-pass query for scenes of at most 64 spheres (the common case), tuned:
//  * the geometry array is padded with NaN spheres to a multiple of 4 plus one
//    extra group (PackedScene), so pass 1 has no remainder loop and can load
//    the next group of 4 records (one 64-byte scalar load) while testing the
//    current one; a NaN sphere's radicand is NaN, never a candidate;
//  * candidate bits of spheres 0..31 and 32..63 go to two 32-bit masks
//    (the half is wave-uniform);
//  * the Markstein quotient path is chosen once per query for the whole wave
//    when every lane's denominator is in range (all(q.fast)), so pass 2 has no
//    per-quotient branch.
template <class Scene>
RTG_HD void candidate_masks64(const Scene& sc, V3 o, V3 d, float a4, unsigned& lo,
                              unsigned& hi) {
  lo = 0;
  hi = 0;
  const unsigned n4 = sc.n4;
  V3 c[4];
  float r2[4];
  sc.sphere4(0, c, r2);
  for (unsigned k = 0; k < n4; k += 4) {
    V3 cn[4];
    float rn[4];
    sc.sphere4(k + 4, cn, rn);  // in bounds: one padding group past n4
    unsigned bits = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const V3 disp = vsub(o, c[q]);
      const float b = 2.0f * vdot(d, disp);
      const float cc = vdot(disp, disp) - r2[q];
      const float rad = (b * b) - (a4 * cc);
      bits |= (rad >= 0.0f) ? (1u << q) : 0u;
    }
    if (k < 32) lo |= bits << k;
    else hi |= bits << (k - 32);
#pragma unroll
    for (int q = 0; q < 4; ++q) { c[q] = cn[q]; r2[q] = rn[q]; }
  }
}

// Pass 2 over the candidates of one 32-sphere half; kShadow: stop at the first
// blocker (gap given), else closest hit (minT/best updated).
template <bool kFast, bool kShadow, class Scene>
RTG_HD bool pass2(const Scene& sc, const RayQ& q, unsigned mask, unsigned base, float gap,
                  float& minT, int& best) {
  while (mask) {
    const unsigned i = base + (unsigned)__builtin_ctz(mask);
    mask &= mask - 1;
    float r2;
    const V3 c = sc.sphere_lane(i, r2);
    bool res;
    const float t = ray_sphere_k<kFast>(q, c, r2, res);
    if constexpr (kShadow) {
      if (res && t < 1000.f) {
        const V3 dist = vsmul(t, q.d);
        if (vdot(dist, dist) < gap) return true;
      }
    } else {
      if (res && t < minT) { minT = t; best = (int)i; }
    }
  }
  return false;
}

template <class Scene>
RTG_HD int closest_hit64(const Scene& sc, V3 o, V3 d, float& tOut) {
  const RayQ q = make_query(o, d);
  unsigned lo, hi;
  candidate_masks64(sc, o, d, q.a4, lo, hi);
  float minT = 1000.f;
  int best = -1;
  if (sc.all(q.fast)) {
    pass2<true, false>(sc, q, lo, 0, 0.f, minT, best);
    pass2<true, false>(sc, q, hi, 32, 0.f, minT, best);
  } else {
    pass2<false, false>(sc, q, lo, 0, 0.f, minT, best);
    pass2<false, false>(sc, q, hi, 32, 0.f, minT, best);
  }
  tOut = minT;
  return best;
}

template <class Scene>
RTG_HD bool blocked64(const Scene& sc, V3 o, V3 d, float gap) {
  const RayQ q = make_query(o, d);
  unsigned lo, hi;
  candidate_masks64(sc, o, d, q.a4, lo, hi);
  float minT = 0.f;
  int best = 0;
  if (sc.all(q.fast))
    return pass2<true, true>(sc, q, lo, 0, gap, minT, best) ||
           pass2<true, true>(sc, q, hi, 32, gap, minT, best);
  return pass2<false, true>(sc, q, lo, 0, gap, minT, best) ||
         pass2<false, true>(sc, q, hi, 32, gap, minT, best);
}

// Query strategy selector: 0 = one sphere per step with a branch per sphere,
// 1 = four spheres per step, 2 = two-pass candidate masks, 3 = the tuned
// two-pass query (<= 64 spheres; larger scenes fall back to 2).
template <int Q, class Scene>
RTG_HD int query_closest(const Scene& sc, V3 o, V3 d, float& t) {
  if constexpr (Q == 0) return closest_hit(sc, o, d, t);
  else if constexpr (Q == 1) return closest_hit4(sc, o, d, t);
  else if constexpr (Q == 3) {
    if (sc.n4 <= 64) return closest_hit64(sc, o, d, t);
    return closest_hit_mask(sc, o, d, t);
  } else return closest_hit_mask(sc, o, d, t);
}
template <int Q, class Scene>
RTG_HD bool query_blocked(const Scene& sc, V3 o, V3 d, float gap) {
  if constexpr (Q == 3) {
    if (sc.n4 <= 64) return blocked64(sc, o, d, gap);
    return blocked_mask(sc, o, d, gap);
  } else if constexpr (Q == 2) return blocked_mask(sc, o, d, gap);
  else return blocked(sc, o, d, gap);
}

template <int S, int Q, class Scene>
RTG_HD V3 shade_pixel_persistent(const Scene& sc, const Camera& cam, unsigned x, unsigned y) {
  constexpr int NF = (S > 1) ? (S - 1) : 1;
  enum : int { kClosest = 0, kShadow = 1, kDone = 2 };
  const float pxX = (((float)x - cam.halfW)) * cam.xs;
  const float pxY = (cam.halfH - (float)y) * cam.ys;
  const int nSamples = cam.nAA * cam.nAA;
  V3 pix = v3(0.f, 0.f, 0.f);
  if (nSamples == 0) return pix;

  Frame st[NF];
  int sp = 0;                       // level of the current node
  int s = 0;                        // sample index, i = s / nAA, j = s % nAA
  V3 ret = v3(0.f, 0.f, 0.f);       // colourSum register
  V3 d, I;                          // current node ray (origin lives in qo)
  int rm = (int)sc.n;               // refractive material of the node
  V3 qo = v3(0.f, 0.f, 0.f), qd;    // the lane's pending query ray
  int phase = kClosest;
  // hit-node shading state (valid while phase == kShadow / within an iteration)
  V3 P = v3(0.f, 0.f, 0.f), N = v3(0.f, 0.f, 0.f), msum = v3(0.f, 0.f, 0.f);
  int hit = 0, li = 0;
  float lgap = 0.f, linc = 0.f;

  // primary ray of sample 0 (main.cpp:432-436)
  {
    const float rx = (pxX + (float)(((float)0) * cam.st)) * cam.asp;
    const float ry = (pxY + (float)(((float)0) * cam.st));
    d = vnorm(v3(rx, ry, cam.zoom));
    I = v3(1.f, 1.f, 1.f);
    qd = d;
  }

  while (phase != kDone) {
    float t;
    const int best = query_closest<Q>(sc, qo, qd, t);

    bool nextLight = false, afterMatte = false, unwind = false;
    if (phase == kClosest) {
      if (best < 0) {
        ret = vmul(I, sc.mat(rm).matte);                    // raytracer.h:544
        unwind = true;
      } else if (!significant(I)) {
        unwind = true;                                      // stale ret
      } else {
        float r2unused;
        const V3 c = sc.sphere((unsigned)best, r2unused);
        P = vadd(qo, vsmul(t, d));
        N = vnorm(vsub(P, c));
        hit = best;
        if (sc.mat(hit).opacity > 0.f) {
          msum = v3(0.f, 0.f, 0.f);
          li = -1;
          nextLight = true;
        } else {
          afterMatte = true;
        }
      }
    } else {  // kShadow: the query was light li's shadow ray
      bool blockedL = false;
      if (best >= 0) {
        const V3 dist = vsmul(t, qd);
        blockedL = vdot(dist, dist) < lgap;                 // raytracer.h:299
      }
      if (!blockedL) {
        V3 Lpos, Lcol;
        sc.light((unsigned)li, Lpos, Lcol);
        msum = vadd(msum, vsmul(linc / lgap, Lcol));        // raytracer.h:354-360
      }
      nextLight = true;
    }

    if (nextLight) {  // next light with positive incidence (raytracer.h:328-349)
      const int m = (int)sc.m;
      bool found = false;
      while (++li < m) {
        V3 Lpos, Lcol;
        sc.light((unsigned)li, Lpos, Lcol);
        const V3 dist = vsub(Lpos, P);
        const float gap = vdot(dist, dist);
        const V3 dir = vsmul(1.f / rtg_sqrtf(gap), dist);
        const float inc = vdot(N, dir);
        if (inc > 0.f) {
          lgap = gap;
          linc = inc;
          qo = P;
          qd = dir;
          found = true;
          break;
        }
      }
      if (found) {
        phase = kShadow;
      } else {
        afterMatte = true;
      }
    }

    if (afterMatte) {  // raytracer.h:463-539 after calculateMatte
      const Mat mh = sc.mat(hit);
      const float op = mh.opacity;
      const float tr = 1.f - op;
      V3 colour = v3(0.f, 0.f, 0.f);
      if (op > 0.f) {
        V3 tmp = vmul(I, mh.matte);
        tmp = vsmul(op, tmp);
        tmp = vmul(msum, tmp);
        colour = vadd(tmp, colour);
      }
      if (tr > 0.f) {
        const bool leaf = (sp >= S - 1);
        const Mat mr = sc.mat(rm);
        V3 cdir = v3(0.f, 0.f, 0.f);
        float R;
        const int tgt = refraction(sc, d, P, N, mr.refr, !leaf, cdir, R);
        const float prod = tr * R;
        V3 rc = vsmul(prod, v3(1.f, 1.f, 1.f));
        rc = vadd(rc, vsmul(mr.opacity, mh.gloss));
        rc = vmul(I, rc);
        const bool sigR = significant(rc);
        if (!leaf) {
          Frame& f = st[sp < NF ? sp : NF - 1];
          f.colour = colour;
          f.rm = rm;
          f.flags = sigR ? 2 : 0;
          if (sigR) {
            const float perp = 2.f * vdot(d, N);
            const V3 rd = vnorm(vsub(d, vsmul(perp, N)));
            f.rd = rd;
            f.ro = vadd(P, vsmul(0.01f, rd));
            f.rI = rc;
          }
          ++sp;
          ret = colour;
          I = vsmul((1.f - R), vsmul(tr, I));
          qo = P;
          d = cdir;
          qd = cdir;
          rm = tgt;
          phase = kClosest;
        } else {
          const V3 c1 = vadd(colour, colour);
          ret = sigR ? vadd(c1, c1) : c1;
          unwind = true;
        }
      } else {
        ret = colour;
        unwind = true;
      }
    }

    if (unwind) {
      bool descend = false;
      while (sp > 0) {
        Frame& f = st[sp - 1 < NF ? sp - 1 : NF - 1];
        f.colour = vadd(ret, f.colour);
        ret = f.colour;
        if ((f.flags & 3) == 2) {
          f.flags = 1;
          qo = f.ro; d = f.rd; qd = f.rd; I = f.rI; rm = f.rm;
          descend = true;
          break;
        }
        --sp;
      }
      if (descend) {
        phase = kClosest;
      } else {
        // sample finished: main.cpp:442-445
        pix = vadd(pix, vsmul(cam.inv, ret));
        ++s;
        if (s < nSamples) {
          const int si = s / cam.nAA, sj = s - si * cam.nAA;
          const float rx = (pxX + (float)(((float)sj) * cam.st)) * cam.asp;
          const float ry = (pxY + (float)(((float)si) * cam.st));
          d = vnorm(v3(rx, ry, cam.zoom));
          qo = v3(0.f, 0.f, 0.f);
          qd = d;
          I = v3(1.f, 1.f, 1.f);
          rm = (int)sc.n;
          ret = v3(0.f, 0.f, 0.f);
          phase = kClosest;
        } else {
          phase = kDone;
        }
      }
    }
  }
  return pix;
}

// v4: node-persistent.  Same node step as trace_sample (one whole node per
// iteration: closest hit, matte with its shadow rays, refraction, push), but
// the 9 samples of the pixel are chained inside ONE loop, so a lane whose
// sample tree is finished starts its next sample's primary ray at the next
// iteration instead of idling until the deepest tree of the wave is done.
template <int S, int Q, class Scene>
RTG_HD V3 shade_pixel_nodes(const Scene& sc, const Camera& cam, unsigned x, unsigned y) {
  constexpr int NF = (S > 1) ? (S - 1) : 1;
  const float pxX = (((float)x - cam.halfW)) * cam.xs;
  const float pxY = (cam.halfH - (float)y) * cam.ys;
  const int nSamples = cam.nAA * cam.nAA;
  V3 pix = v3(0.f, 0.f, 0.f);
  if (nSamples == 0) return pix;
  Frame st[NF];
  int sp = 0;
  int s = 0;
  V3 ret = v3(0.f, 0.f, 0.f);
  V3 o = v3(0.f, 0.f, 0.f), I = v3(1.f, 1.f, 1.f), d;
  int rm = (int)sc.n;
  {
    const float rx = (pxX + (float)(((float)0) * cam.st)) * cam.asp;
    const float ry = (pxY + (float)(((float)0) * cam.st));
    d = vnorm(v3(rx, ry, cam.zoom));
  }
  for (;;) {
    float t;
    sc.probe_begin(kProbeClosest);
    const int hit = query_closest<Q>(sc, o, d, t);
    sc.probe_end(kProbeClosest);
    bool descendNow = false;
    if (hit < 0) {
      ret = vmul(I, sc.mat(rm).matte);
    } else if (significant(I)) {
      float r2unused;
      const V3 c = sc.sphere((unsigned)hit, r2unused);
      const V3 P = vadd(o, vsmul(t, d));
      const V3 N = vnorm(vsub(P, c));
      const Mat mh = sc.mat(hit);
      const float op = mh.opacity;
      const float tr = 1.f - op;
      V3 colour = v3(0.f, 0.f, 0.f);
      if (op > 0.f) {
        V3 tmp = vmul(I, mh.matte);
        tmp = vsmul(op, tmp);
        const V3 mc = matte_light<Q>(sc, P, N);
        tmp = vmul(mc, tmp);
        colour = vadd(tmp, colour);
      }
      if (tr > 0.f) {
        const bool leaf = (sp >= S - 1);
        const Mat mr = sc.mat(rm);
        V3 cdir;
        float R;
        sc.probe_begin(kProbeRefraction);
        const int tgt = refraction(sc, d, P, N, mr.refr, !leaf, cdir, R);
        sc.probe_end(kProbeRefraction);
        const float prod = tr * R;
        V3 rc = vsmul(prod, v3(1.f, 1.f, 1.f));
        rc = vadd(rc, vsmul(mr.opacity, mh.gloss));
        rc = vmul(I, rc);
        const bool sigR = significant(rc);
        if (!leaf) {
          Frame& f = st[sp < NF ? sp : NF - 1];
          f.colour = colour;
          f.rm = rm;
          f.flags = sigR ? 2 : 0;
          if (sigR) {
            const float perp = 2.f * vdot(d, N);
            const V3 rd = vnorm(vsub(d, vsmul(perp, N)));
            f.rd = rd;
            f.ro = vadd(P, vsmul(0.01f, rd));
            f.rI = rc;
          }
          ++sp;
          ret = colour;
          I = vsmul((1.f - R), vsmul(tr, I));
          o = P;
          d = cdir;
          rm = tgt;
          descendNow = true;
        } else {
          const V3 c1 = vadd(colour, colour);
          ret = sigR ? vadd(c1, c1) : c1;
        }
      } else {
        ret = colour;
      }
    }
    if (descendNow) continue;
    bool descend = false;
    while (sp > 0) {
      Frame& f = st[sp - 1 < NF ? sp - 1 : NF - 1];
      f.colour = vadd(ret, f.colour);
      ret = f.colour;
      if ((f.flags & 3) == 2) {
        f.flags = 1;
        o = f.ro; d = f.rd; I = f.rI; rm = f.rm;
        descend = true;
        break;
      }
      --sp;
    }
    if (descend) continue;
    pix = vadd(pix, vsmul(cam.inv, ret));   // main.cpp:442-445
    if (++s >= nSamples) break;
    const int si = s / cam.nAA, sj = s - si * cam.nAA;
    const float rx = (pxX + (float)(((float)sj) * cam.st)) * cam.asp;
    const float ry = (pxY + (float)(((float)si) * cam.st));
    d = vnorm(v3(rx, ry, cam.zoom));
    o = v3(0.f, 0.f, 0.f);
    I = v3(1.f, 1.f, 1.f);
    rm = (int)sc.n;
    ret = v3(0.f, 0.f, 0.f);
  }
  return pix;
}

// Bounds of the primary-ray directions of pixel (x, y) (all its samples):
// X = (pxX + j*st)*asp, Y = pxY + i*st for i, j in [0, nAA).
RTG_HD void primary_bounds(const Camera& cam, unsigned x, unsigned y, float& x0, float& x1,
                           float& y0, float& y1) {
  const float pxX = (((float)x - cam.halfW)) * cam.xs;
  const float pxY = (cam.halfH - (float)y) * cam.ys;
  const float ext = (float)(cam.nAA > 0 ? cam.nAA - 1 : 0) * cam.st;
  const float a = pxX * cam.asp, b = (pxX + ext) * cam.asp;
  x0 = fminf(a, b);
  x1 = fmaxf(a, b);
  y0 = fminf(pxY, pxY + ext);
  y1 = fmaxf(pxY, pxY + ext);
}

// The primary ray of sample (i, j) of pixel (x, y): the screen-plane point
// (rx, ry) (main.cpp:419-426) and its normalised direction (main.cpp:428).
RTG_HD V3 sample_dir(const Camera& cam, unsigned x, unsigned y, int i, int j, float& rx,
                     float& ry) {
  const float pxX = (((float)x - cam.halfW)) * cam.xs;
  const float pxY = (cam.halfH - (float)y) * cam.ys;
  rx = (pxX + (float)(((float)j) * cam.st)) * cam.asp;
  ry = (pxY + (float)(((float)i) * cam.st));
  return vnorm(v3(rx, ry, cam.zoom));
}

// main.cpp:411-452 for pixel (x, y) of the frame.
template <int S, int Q, bool kSceneFrames = false, bool kCL = false, class Scene>
RTG_HD V3 shade_pixel(const Scene& sc, const Camera& cam, unsigned x, unsigned y,
                      bool usePrim = false, uint64_t primSel = ~0ull) {
  constexpr int NF = (S > 1) ? (S - 1) : 1;
  LocalFrames<NF> local;
  const float pxX = (((float)x - cam.halfW)) * cam.xs;
  const float pxY = (cam.halfH - (float)y) * cam.ys;
  V3 pix = v3(0.f, 0.f, 0.f);
  for (int i = 0; i < cam.nAA; ++i) {
    for (int j = 0; j < cam.nAA; ++j) {
      const float rx = (pxX + (float)(((float)j) * cam.st)) * cam.asp;
      const float ry = (pxY + (float)(((float)i) * cam.st));
      const V3 dir = vnorm(v3(rx, ry, cam.zoom));
      V3 c;
      if constexpr (kSceneFrames)
        c = trace_sample<S, Q, kCL>(sc, dir, sc.frames(), usePrim, primSel);
      else c = trace_sample<S, Q, kCL>(sc, dir, local, usePrim, primSel);
      c = vsmul(cam.inv, c);
      pix = vadd(pix, c);
    }
  }
  return pix;
}

}  // namespace rtg
