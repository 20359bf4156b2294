// rtg_scene_pack.h — host-side preparation of a scene and camera for the
// kernel (used by librtg.so; the test-only host simulation reuses it so that
// it exercises the same preparation).
//
// Everything here is arithmetic the reference does per use and that is
// hoisted to the host with the same float operation (-ffp-contract=off):
//   r*r                       raytracer.h:100
//   (radius + 1e-6f)^2        raytracer.h:259-264
//   |0 - c|^2 - r*r           raytracer.h:99-101 for a ray from the origin
//                              (every primary ray, main.cpp:417)
//   camera constants          main.cpp:384-402
#pragma once

#include <math.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <thread>
#include <utility>
#include <vector>

#include "rtg.h"
#include "rtg_internal.h"
#include "rtg_trace.h"

namespace rtg {

// Scenes above this many spheres have no masks; they get a BVH instead.
constexpr unsigned kMaskMaxSpheres = 64;

// Device image of a scene (crad2's third segment, guard_r2, and smask are
// the shadow-ray masks' data, see shadow_masks).  geom: n x {x, y, z, r*r} followed by NaN padding
// records up to n4 + 4 (n4 = n rounded up to 4), then the same n4 + 4 records
// with the pass-1 screen radius^2 (screen_r2) in place of r*r, then with the
// containment radius^2 (r + 1e-6f)^2 (primary_container), then n4 + 4 32-byte
// fused records {x, y, z, screen r^2, r^2, primary c term, 0, 0} (sphere_fused,
// the fused query loops: one scalar load per sphere); crad2: n x (r+1e-6)^2, then
// n x the primary-ray c term |0 - c|^2 - r^2 (same float operations and order
// as the query's vdot(disp, disp) - r2 with disp = 0 - c, exact negation);
// mats: (n+1) x {matte.xyz, gloss.xyz, opacity, n} with [n] = background
// {0,0,0, 0,0,0, 0, 1.0} (raytracer.h:694-697; opacity 0);
// lights: m x {pos.xyz, col.xyz}.  Arrays are never empty (padded to 1).
struct PackedScene {
  std::vector<float> geom, crad2, mats, lights;
  // Primary-cull sphere constants (prim_consts): n x {1/|c|, sin a, cos a, 0}.
  std::vector<float> prim;
  // Sphere masks (shadow_masks below): m x n shadow masks, then n overlap
  // masks, each {lo, hi} words, for 1 <= n <= 64 and a finite scene; empty
  // otherwise (every sphere is then tested).
  std::vector<unsigned> smask;
  // Secondary-ray cone masks (cone_masks): n x kConeTiers x kConeCells x {lo, hi}, with
  // the sphere masks; empty otherwise.
  std::vector<unsigned> cone;
  // BVH of scenes above kMaskMaxSpheres spheres (build_bvh): one 128-byte
  // record of kBvhWords words per node (rtg_trace.h BvhRec, loaded with two
  // 64-byte scalar loads); empty for small or non-finite scenes.
  std::vector<float> bvhNodes;
  // Sphere lists of BVH scenes (sphere_lists): capsule and overlap lists.
  std::vector<float> capRec, ovRec;
  std::vector<unsigned> capOff, ovOff;
  unsigned n = 0, m = 0;
  unsigned n4 = 0;  // n rounded up to a multiple of 4; geom holds 3 x (n4 + 4) records + the fused part
};

// Shadow-ray sphere masks.  A shadow ray of raytracer.h:272-309 starts at the
// hit point P of sphere h and ends at light l.  The kernel first checks that
// P lies in the guard ball B_h = ball(c_h, g_h) (guard_radius; the computed
// hit point is within a few ulps of the surface except after near-tangent
// hits), so the segment P -> L_l lies in the capsule of radius g_h around the
// segment c_h -> L_l (the capsule contains the convex hull of B_h and L_l).
// Sphere i can block only if the reference's root test accepts a root t in
// (1e-5, 1000) with |t D|^2 < |L - P|^2.  The reference's radicand carries a
// rounding error below ~14 eps a (|p|^2 + r_i^2) (p = P - c_i), so a line
// that misses ball i by mu can only look like a hit when mu^2 < 14 eps |p|^2,
// and computed roots move by less than sqrt(14 eps) (|p| + r_i) ~ 1e-3 (|p| +
// r_i); both are far below the margin
//   mu_i = 2^-8 (|c_i - c_h| + g_h + r_i) + 2^-16 (|L_l - c_h| + g_h)
// (the second term covers the ~eps direction error of vnorm(L - P) over the
// segment).  So if ball i grown by mu_i misses the capsule, every point of
// the segment is more than r_i + mu_i from c_i: the radicand near the segment
// stays negative and roots of the line outside the segment keep their side
// of 0 and of |L - P|, i.e. sphere i never blocks.  Bit i of mask (l, h) is
// set for i == h and for every sphere whose grown ball meets the capsule
// (double arithmetic with a further 1e-9 relative slack).  The kernel tests
// the union of its lanes' masks, and every sphere for a lane whose P fails
// the guard.  tests/test_oracle.py checks the superset property against the
// reference's own test on random segments and the kernel's frames bit for bit.
inline double guard_radius(const rtg_sphere& s) {
  const double r = fabs((double)s.radius);
  const double c = fabs((double)s.pos.x) + fabs((double)s.pos.y) + fabs((double)s.pos.z);
  return r * (1.0 + 0x1p-10) + 0x1p-20 * (c + r);
}

// g_h^2 (1 - 2^-20) rounded down: the float test |P - c_h|^2 <= guard_r2
// (relative error < 6 eps) then implies |P - c_h| <= g_h.  -1 (never passes)
// for non-finite or tiny spheres.
inline float guard_r2(const rtg_sphere& s) {
  const double g = guard_radius(s);
  if (!(g >= 0x1p-60 && g <= 0x1p60)) return -1.f;
  const double v = g * g * (1.0 - 0x1p-20);
  float f = (float)v;
  if ((double)f > v) f = nextafterf(f, 0.f);
  return f;
}

// Radius of the ball around c_h that holds every refraction test point
// P + 0.01f D (raytracer.h:690) with P in the guard ball B_h and
// |D| <= kContainDirMax (1 + 2^-20): 0.01 |D| with the float product's and
// the comparison's rounding, plus the rounding of the sum, below
// 2^-16 (|c_h| + g_h + 1).
inline double contain_reach(const rtg_sphere& s) {
  const double g = guard_radius(s);
  const double c = fabs((double)s.pos.x) + fabs((double)s.pos.y) + fabs((double)s.pos.z);
  return g + 0.01 * (double)kContainDirMax * (1.0 + 0x1p-16) + 0x1p-16 * (c + g + 1.0);
}

// The sphere half of the primary-ray cull (primary_possible, rtg_trace.h):
// seen from the camera origin, sphere c, r with the radius inflated to
// rr = |r| * 1.001 + 1e-3 has angular radius alpha, sin(alpha) = rr / |c|.
// Computed in double and rounded (the test's 2e-3 margin dwarfs that);
// cos(alpha) = -3, sin(alpha) = 0 mark "always possible" (sin(alpha) >= 0.999:
// the origin inside or near the sphere; or a non-finite or zero centre).
inline void prim_consts(const rtg_sphere& s, float* out) {
  const double cx = s.pos.x, cy = s.pos.y, cz = s.pos.z;
  const double L = sqrt(cx * cx + cy * cy + cz * cz);
  const double rr = fabs((double)s.radius) * 1.001 + 1e-3;
  const double sa = rr / L;
  out[3] = 0.f;
  if (!(sa < 0.999) || !(L > 0.0) || !(L < 1e30)) {
    out[0] = 0.f;
    out[1] = 0.f;
    out[2] = -3.f;
    return;
  }
  out[0] = (float)(1.0 / L);
  out[1] = (float)sa;
  out[2] = (float)sqrt(1.0 - sa * sa);
}

// The two mask predicates, shared by the masks (n <= 64) and the sphere lists
// of BVH scenes (sphere_lists): sphere i can block a shadow ray from B_h to
// light L (capsule_keep; *tOut = its centre's position along c_h -> L, 0..1),
// and sphere j can contain a refraction test point of h / be hit by a ray that
// entered h before it leaves B_h (overlap_keep).  See shadow_masks.
// Test hook (tests/hostsim only): a positive value moves capsule_keep's
// back plane forward by that fraction of g, so the check can show that the
// plane's position matters.
inline double g_capsuleBackSlack = 0.0;
inline bool capsule_keep(const rtg_sphere* spheres, unsigned h, unsigned i, const double L[3],
                         double* tOut = nullptr) {
  const rtg_sphere& sh = spheres[h];
  const double A[3] = {sh.pos.x, sh.pos.y, sh.pos.z};
  const double g = guard_radius(sh);
  double ab[3], ab2 = 0.0;
  for (int k = 0; k < 3; ++k) { ab[k] = L[k] - A[k]; ab2 += ab[k] * ab[k]; }
  const double lh = sqrt(ab2);
  const rtg_sphere& si = spheres[i];
  const double C[3] = {si.pos.x, si.pos.y, si.pos.z};
  const double ri = fabs((double)si.radius);
  double t = 0.0, dch = 0.0;
  for (int k = 0; k < 3; ++k) {
    const double ca = C[k] - A[k];
    t += ca * ab[k];
    dch += ca * ca;
  }
  dch = sqrt(dch);
  t = ab2 > 0.0 ? t / ab2 : 0.0;
  t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
  if (tOut) {
    // The capsule list's order key (sphere_lists): h itself first, then the
    // spheres whose extent along c_h -> L reaches back to the segment's start
    // (the likeliest blockers of a shadow ray from the hit point: P lies
    // inside or just behind them), largest first, then the others by where
    // their extent starts.  Only the order of the walk depends on it.
    double traw = 0.0;
    for (int k = 0; k < 3; ++k) traw += (C[k] - A[k]) * ab[k];
    traw = ab2 > 0.0 ? traw / ab2 : 0.0;
    const double start = traw - ri / (lh > 0.0 ? lh : 1.0);
    *tOut = (i == h) ? -1e300 : start < 0.0 ? -ri : start;
  }
  if (i == h) return true;
  double d2 = 0.0;
  for (int k = 0; k < 3; ++k) {
    const double e = C[k] - (A[k] + t * ab[k]);
    d2 += e * e;
  }
  const double mu = 0x1p-8 * (dch + g + ri) + 0x1p-16 * (lh + g);
  const double reach = (g + ri + mu) * (1.0 + 1e-9);
  if (sqrt(d2) > reach) return false;
  // The kernel casts a shadow ray only from a point P with incidence > 0
  // (matte_light): N.dir > 0 computed, so (P - c_h).(L - P) > -2^-20 |P -
  // c_h| |L - P| exactly, whence (P - c_h).u >= -2^-19 g with u the unit
  // vector c_h -> L (|L - P| <= 2 |L - c_h| for a light outside the guard
  // ball).  Every point of the segment P -> L then lies in that half-space,
  // and so does every blocking root's exact point, which is within r_i + mu
  // of c_i: a sphere whose grown ball lies wholly behind the plane
  // (c_i - c_h).u + r_i + mu < -(2^-16 g + 2^-20 |L - c_h|) blocks no
  // shadow ray of h.
  if (lh > 2.0 * g) {
    double proj = 0.0;
    for (int k = 0; k < 3; ++k) proj += (C[k] - A[k]) * ab[k];
    proj /= lh;
    if (proj + (ri + mu) * (1.0 + 1e-9) < -(0x1p-16 * g + 0x1p-20 * lh) + g_capsuleBackSlack * g)
      return false;
  }
  return true;
}
inline bool overlap_keep(const rtg_sphere* spheres, unsigned h, unsigned j) {
  if (j == h) return true;
  const rtg_sphere& sh = spheres[h];
  const double g = guard_radius(sh);
  const double reach = contain_reach(sh);
  const rtg_sphere& sj = spheres[j];
  const double dx = (double)sj.pos.x - sh.pos.x, dy = (double)sj.pos.y - sh.pos.y,
               dz = (double)sj.pos.z - sh.pos.z;
  const double d = sqrt(dx * dx + dy * dy + dz * dz);
  const double rj = fabs((double)sj.radius) + 1e-6;
  const double mu = 0x1p-8 * (d + g + rj);
  return !(d > (reach + rj + mu) * (1.0 + 1e-9));
}

inline void shadow_masks(const rtg_sphere* spheres, unsigned n, const rtg_light* lights,
                         unsigned m, std::vector<unsigned>* out) {
  out->clear();
  if (n == 0 || n > kMaskMaxSpheres) return;
  auto finite = [](double v) { return v == v && fabs(v) <= 1e30; };
  for (unsigned i = 0; i < n; ++i)
    if (!finite(spheres[i].pos.x) || !finite(spheres[i].pos.y) || !finite(spheres[i].pos.z) ||
        !finite(spheres[i].radius))
      return;
  for (unsigned l = 0; l < m; ++l)
    if (!finite(lights[l].pos.x) || !finite(lights[l].pos.y) || !finite(lights[l].pos.z))
      return;
  out->assign(((size_t)m * n + n) * 2, 0u);
  for (unsigned l = 0; l < m; ++l) {
    const double L[3] = {lights[l].pos.x, lights[l].pos.y, lights[l].pos.z};
    for (unsigned h = 0; h < n; ++h) {
      unsigned* w = &(*out)[((size_t)l * n + h) * 2];
      for (unsigned i = 0; i < n; ++i)
        if (capsule_keep(spheres, h, i, L)) w[i >> 5] |= 1u << (i & 31);
    }
  }
  // Overlap masks (closest_enter and primary_container_sel, rtg_trace.h): bit
  // j of mask h is set when ball(c_j, |r_j| + 1e-6) grown by
  // mu_j = 2^-8 (|c_j - c_h| + g_h + r_j) meets the ball B'_h = ball(c_h,
  // contain_reach(h)) around the guard ball B_h (and always for j == h).
  //  * closest_enter: a ray whose origin and computed exit point from sphere h
  //    both lie in B_h stays inside B_h up to that exit, so a sphere outside
  //    the mask has no accepted root before it (same error argument as
  //    above): the closest hit is h or a mask sphere.
  //  * primary_container_sel: the refraction test point P + 0.01f D
  //    (raytracer.h:690) of a hit point P in B_h with |D| <= kContainDirMax
  //    lies in B'_h (the reach covers 0.01 |D| and the rounding of the point),
  //    and the float containment test (raytracer.h:255-264) cannot accept a
  //    point more than mu_j outside ball(c_j, |r_j| + 1e-6); so the first
  //    containing sphere in index order is the first containing mask sphere.
  for (unsigned h = 0; h < n; ++h) {
    unsigned* w = &(*out)[((size_t)m * n + h) * 2];
    for (unsigned j = 0; j < n; ++j)
      if (overlap_keep(spheres, h, j)) w[j >> 5] |= 1u << (j & 31);
  }
}

// Hit-point cells of the capsule lists (BVH scenes).  A shadow ray starts at
// a hit point P of sphere h; the kernel classifies e = P - c_h (cap_cell,
// rtg_trace.h) into one of 24 cells: the axis a of e's largest component
// and the signs of e's three components, and only when |e| >= r_in =
// |r_h| (1 - 2^-8) (cells need the shell; else, or when the guard test
// fails, kCapFull).  Every classified P then lies in the cell's region
//   R = { c_h + e : r_in <= |e| <= g_h, e_a has the cell's sign, |e_a| >=
//         (1 - 2^-20) max(|e_p|, |e_q|), e_p, e_q have the cell's signs }
// (the computed e's signs are exact: one rounded subtraction each; its
// largest component can be 2^-23 below another's; its |e|^2 test is argued at
// cap_cell).  In gnomonic coordinates on face a the directions of R fill the
// rectangle [0, 1 + 2^-19]^2 (signed), so every direction of R is within the
// angle theta of the rectangle's centre direction v0 that its farthest corner
// has (the cap around v0 is convex in those coordinates), and R lies in the
// ball around c_h + beta v0 whose radius reaches the points at angle theta
// at |e| = r_in and |e| = g_h (cell_ball).  The segment P -> L lies within
// that radius of the segment b -> L, so the capsule argument of
// shadow_masks holds with (b, rho) in place of (c_h, g_h): a cell keeps the
// spheres of the full capsule list whose grown ball meets that capsule
// (cell_keep).  C5: 45 -> 25 capsule records per list on average.
inline double g_cellBallSlack = 0.0;  // test hook (tests/hostsim): shrinks the cell balls
inline double cell_rin(const rtg_sphere& s) {
  const double r = fabs((double)s.radius);
  return r < 0x1p-60 ? 0.0 : r * (1.0 - 0x1p-8);
}
// Centre b and radius rho of the ball holding cell `cell`'s region of sphere s.
inline void cell_ball(const rtg_sphere& s, unsigned cell, double b[3], double* rho) {
  const unsigned a = cell >> 3, p = a == 0 ? 1 : 0, q = a == 2 ? 1 : 2;
  const double sa = (cell & 4) ? -1.0 : 1.0, sp = (cell & 2) ? -1.0 : 1.0,
               sq = (cell & 1) ? -1.0 : 1.0;
  const double E = 1.0 + 0x1p-19;
  auto dir = [&](double pp, double qq, double v[3]) {
    v[a] = sa;
    v[p] = sp * pp;
    v[q] = sq * qq;
    const double l = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    for (int k = 0; k < 3; ++k) v[k] /= l;
  };
  double v0[3];
  dir(0.5 * E, 0.5 * E, v0);
  double cmin = 1.0;
  for (int k = 0; k < 4; ++k) {
    double v[3];
    dir((k & 1) ? E : 0.0, (k & 2) ? E : 0.0, v);
    const double c = v[0] * v0[0] + v[1] * v0[1] + v[2] * v0[2];
    cmin = c < cmin ? c : cmin;
  }
  cmin -= 1e-12;  // theta rounded up
  const double ri = cell_rin(s), g = guard_radius(s);
  auto f = [&](double beta) {  // squared distance to the farthest extreme point
    const double f1 = ri * ri + beta * beta - 2.0 * ri * beta * cmin;
    const double f2 = g * g + beta * beta - 2.0 * g * beta * cmin;
    return f1 > f2 ? f1 : f2;
  };
  // the minimum of the larger of two convex parabolas: at one's vertex or
  // where they cross
  double best = 1e300, bb = 0.0;
  const double cand[3] = {ri * cmin, g * cmin, cmin > 0.0 ? (g + ri) / (2.0 * cmin) : 0.0};
  for (double beta : cand) {
    beta = beta < 0.0 ? 0.0 : beta;
    if (f(beta) < best) { best = f(beta); bb = beta; }
  }
  b[0] = s.pos.x + bb * v0[0];
  b[1] = s.pos.y + bb * v0[1];
  b[2] = s.pos.z + bb * v0[2];
  const double cm = fabs((double)s.pos.x) + fabs((double)s.pos.y) + fabs((double)s.pos.z);
  *rho = sqrt(best) * (1.0 + 1e-9) * (1.0 - g_cellBallSlack) + 1e-12 * (g + cm);
}
// Is cell `cell` of sphere h wholly behind the plane through c_h facing
// light L (every direction e with e.u < 0)?  Such a cell holds no point a
// shadow ray is cast from (capsule_keep's back plane), so it shares the
// full list instead of a list of its own.
inline bool cell_behind(const rtg_sphere& s, unsigned cell, const double L[3]) {
  const unsigned a = cell >> 3, p = a == 0 ? 1 : 0, q = a == 2 ? 1 : 2;
  const double sa = (cell & 4) ? -1.0 : 1.0, sp = (cell & 2) ? -1.0 : 1.0,
               sq = (cell & 1) ? -1.0 : 1.0;
  const double u[3] = {L[0] - s.pos.x, L[1] - s.pos.y, L[2] - s.pos.z};
  const double ul = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
  if (!(ul > 2.0 * guard_radius(s))) return false;  // (the back plane's condition)
  const double E = 1.0 + 0x1p-19;
  for (int k = 0; k < 4; ++k) {  // e.u is linear in the gnomonic coordinates
    const double pp = (k & 1) ? E : 0.0, qq = (k & 2) ? E : 0.0;
    if (sa * u[a] + sp * pp * u[p] + sq * qq * u[q] > -1e-3 * ul) return false;
  }
  return true;
}
// Sphere i in cell `cell`'s capsule list for light L: its grown ball meets the
// capsule of radius rho around b -> L (cell_ball), with capsule_keep's margin.
inline bool cell_keep(const rtg_sphere* spheres, unsigned h, unsigned i, const double L[3],
                      const double b[3], double rho) {
  if (i == h) return true;
  const rtg_sphere& sh = spheres[h];
  const rtg_sphere& si = spheres[i];
  const double g = guard_radius(sh);
  const double C[3] = {si.pos.x, si.pos.y, si.pos.z};
  const double ri = fabs((double)si.radius);
  double ab[3], ab2 = 0.0, t = 0.0, dch = 0.0, lh = 0.0;
  for (int k = 0; k < 3; ++k) {
    ab[k] = L[k] - b[k];
    ab2 += ab[k] * ab[k];
    t += (C[k] - b[k]) * ab[k];
    const double ch = C[k] - (k == 0 ? sh.pos.x : k == 1 ? sh.pos.y : sh.pos.z);
    dch += ch * ch;
    const double lc = L[k] - (k == 0 ? sh.pos.x : k == 1 ? sh.pos.y : sh.pos.z);
    lh += lc * lc;
  }
  dch = sqrt(dch);
  lh = sqrt(lh);
  t = ab2 > 0.0 ? t / ab2 : 0.0;
  t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
  double d2 = 0.0;
  for (int k = 0; k < 3; ++k) {
    const double e = C[k] - (b[k] + t * ab[k]);
    d2 += e * e;
  }
  const double mu = 0x1p-8 * (dch + g + ri) + 0x1p-16 * (lh + g);
  return !(sqrt(d2) > (rho + ri + mu) * (1.0 + 1e-9));
}

// Sphere lists of BVH scenes (n > 64, where 64-bit masks do not reach): the
// masks' sets as lists of kListWords-word records, for the coherent-wave
// queries of rtg_trace.h (blocked_cap, closest_enter_list, container_list):
//  * capsule lists, one per (light l, sphere h): the spheres of shadow mask
//    (l, h) (capsule_keep) in the order of capsule_keep's key (h itself
//    first, then the spheres that reach back to the segment's start, largest
//    first: the likeliest blockers), records {x, y, z, screen r^2
//    (screen_r2), r^2, 0, 0, 0};
//  * overlap lists, one per sphere h: the spheres of overlap mask h
//    (overlap_keep) in index order, records {x, y, z, screen r^2, r^2,
//    (r + 1e-6f)^2, index, refractive index}.
// capOff[2 ((l n + h) kCapCells + c)] and [... + 1] delimit the capsule list of
// (light l, sphere h, hit-point cell c) (cells above; kCapFull the whole
// capsule list, which cells wholly behind the light's plane share), and
// ovOff[h] .. ovOff[h + 1] the overlap list.  Empty for non-finite scenes
// (the queries then use the BVH).
//
// Limits.  The kernel addresses the record tables with 32-bit byte offsets
// (fidx(capRec, 8k): 32 k bytes), and the lists grow as O(m n^2) records, so
// a table is capped at kListMaxRecords records (2^23: 256 MiB, far below the
// 2^27 records where the offsets would wrap); and building them costs
// m n^2 capsule tests plus n^2 overlap tests, so scenes where that exceeds
// kListMaxTests get no lists.  Either way the tables stay empty, has_lists()
// is false and every query takes the BVH (same answers, slower).
constexpr int kListWords = 8;
// records read past a list's end by one load: padding at each table's end
constexpr int kCapPad = 64 / (4 * kCapWords) - 1;
constexpr int kOvPad = 1;
constexpr size_t kListMaxRecords = size_t(1) << 23;
constexpr double kListMaxTests = 0x1p28;
inline void sphere_lists(const rtg_sphere* spheres, unsigned n, const rtg_light* lights,
                         unsigned m, PackedScene* ps, size_t maxRecords = kListMaxRecords) {
  ps->capRec.clear();
  ps->capOff.clear();
  ps->ovRec.clear();
  ps->ovOff.clear();
  if ((double)(m + 1) * n * n > kListMaxTests) return;  // (cells test only full-list members)
  auto finite = [](double v) { return v == v && fabs(v) <= 1e30; };
  for (unsigned i = 0; i < n; ++i)
    if (!finite(spheres[i].pos.x) || !finite(spheres[i].pos.y) || !finite(spheres[i].pos.z) ||
        !finite(spheres[i].radius))
      return;
  for (unsigned l = 0; l < m; ++l)
    if (!finite(lights[l].pos.x) || !finite(lights[l].pos.y) || !finite(lights[l].pos.z))
      return;
  auto rec = [&](std::vector<float>& v, unsigned i) {
    const rtg_sphere& s = spheres[i];
    const float r2 = s.radius * s.radius;  // raytracer.h:100
    const float rc = s.radius + 1.0e-6f;   // raytracer.h:259-264
    unsigned idx = i;
    float fi;
    memcpy(&fi, &idx, 4);
    const float w[kListWords] = {s.pos.x, s.pos.y, s.pos.z, screen_r2(r2), r2, rc * rc, fi,
                                 s.material.refractiveIndex};
    v.insert(v.end(), w, w + kListWords);
  };
  // capsule lists: per (l, h) the kept spheres sorted by capsule_keep's key,
  // then per cell the members its capsule keeps, in the same order (cells
  // wholly behind the light's plane: none, they share the full list); the
  // (l, h) pairs are independent, so they are built in parallel
  std::vector<std::vector<unsigned>> lists((size_t)m * n);
  std::vector<std::vector<unsigned>> cells((size_t)m * n * kCapCubeCells);
  std::vector<unsigned char> cellShared((size_t)m * n * kCapCubeCells, 0);
  auto work = [&](unsigned lo, unsigned hi) {
    std::vector<std::pair<double, unsigned>> tmp;
    for (unsigned q = lo; q < hi; ++q) {
      const unsigned l = q / n, h = q % n;
      const double L[3] = {lights[l].pos.x, lights[l].pos.y, lights[l].pos.z};
      tmp.clear();
      for (unsigned i = 0; i < n; ++i) {
        double t;
        if (capsule_keep(spheres, h, i, L, &t)) tmp.emplace_back(t, i);
      }
      std::sort(tmp.begin(), tmp.end());
      for (const auto& e : tmp) lists[q].push_back(e.second);
      for (unsigned c = 0; c < kCapCubeCells; ++c) {
        const size_t qc = (size_t)q * kCapCubeCells + c;
        if (cell_behind(spheres[h], c, L)) {
          cellShared[qc] = 1;
          continue;
        }
        double b[3], rho;
        cell_ball(spheres[h], c, b, &rho);
        for (unsigned i : lists[q])
          if (cell_keep(spheres, h, i, L, b, rho)) cells[qc].push_back(i);
      }
    }
  };
  const unsigned total = m * n;
  unsigned nt = std::thread::hardware_concurrency();
  nt = nt < 1 ? 1 : (nt > 16 ? 16 : nt);
  if (total < 256) nt = 1;
  std::vector<std::thread> pool;
  for (unsigned t = 0; t < nt; ++t)
    pool.emplace_back(work, (unsigned)((size_t)total * t / nt),
                      (unsigned)((size_t)total * (t + 1) / nt));
  for (auto& th : pool) th.join();
  size_t capTotal = 0;
  for (const auto& l : lists) capTotal += l.size();
  for (const auto& l : cells) capTotal += l.size();
  if (capTotal + kCapPad > maxRecords) return;  // (the padding records)
  std::vector<std::vector<unsigned>> ov(n);
  size_t ovTotal = 0;
  for (unsigned h = 0; h < n; ++h) {
    for (unsigned j = 0; j < n; ++j)
      if (overlap_keep(spheres, h, j)) ov[h].push_back(j);
    ovTotal += ov[h].size();
    if (ovTotal + 1 > maxRecords) return;
  }
  ps->capRec.reserve((capTotal + kCapPad) * kCapWords);
  ps->capOff.assign((size_t)total * kCapCells * 2, 0u);
  auto emit = [&](const std::vector<unsigned>& li, size_t slot) {
    ps->capOff[2 * slot] = (unsigned)(ps->capRec.size() / kCapWords);
    for (unsigned i : li) {
      const rtg_sphere& sp = spheres[i];
      const float w[kCapWords] = {sp.pos.x, sp.pos.y, sp.pos.z, sp.radius * sp.radius};  // raytracer.h:100
      ps->capRec.insert(ps->capRec.end(), w, w + kCapWords);
    }
    ps->capOff[2 * slot + 1] = (unsigned)(ps->capRec.size() / kCapWords);
  };
  for (unsigned q = 0; q < total; ++q) {
    const size_t full = (size_t)q * kCapCells + kCapFull;
    emit(lists[q], full);
    for (unsigned c = 0; c < kCapCubeCells; ++c) {
      const size_t qc = (size_t)q * kCapCubeCells + c, slot = (size_t)q * kCapCells + c;
      if (cellShared[qc]) {
        ps->capOff[2 * slot] = ps->capOff[2 * full];
        ps->capOff[2 * slot + 1] = ps->capOff[2 * full + 1];
      } else {
        emit(cells[qc], slot);
      }
    }
  }
  ps->ovRec.reserve((ovTotal + 1) * kListWords);
  ps->ovOff.push_back(0);
  for (unsigned h = 0; h < n; ++h) {
    for (unsigned j : ov[h]) rec(ps->ovRec, j);
    ps->ovOff.push_back((unsigned)(ps->ovRec.size() / kListWords));
  }
  // padding records past each table's end: the kernel reads a 64-byte
  // scalar load of records at a time (two overlap records, four capsule
  // records) and the ones past a list's end are the next list's or these,
  // whose NaN centres accept no root
  const float pad[kListWords] = {NAN, NAN, NAN, NAN, NAN, NAN, 0.f, 1.f};
  for (int k = 0; k < kCapPad; ++k) ps->capRec.insert(ps->capRec.end(), pad, pad + kCapWords);
  for (int k = 0; k < kOvPad; ++k) ps->ovRec.insert(ps->ovRec.end(), pad, pad + kListWords);
}

inline float round_up_f(double v) {
  float f = (float)v;
  if ((double)f < v) f = nextafterf(f, __builtin_inff());
  return f;
}
inline float round_down_f(double v) {
  float f = (float)v;
  if ((double)f > v) f = nextafterf(f, -__builtin_inff());
  return f;
}
// Secondary-ray cone masks.  A secondary ray of sphere h starts in the origin
// ball B''_h = ball(c_h, rho_h), rho_h = g_h + 0.0101 + 2^-20 (|c_h| + g_h):
// refraction children start at the hit point P (|P - c_h| <= g_h, the guard
// test) and reflection children at P + 0.01f rd with |rd| = 1 (vnorm)
// (raytracer.h:830-836).  Sphere i can take an accepted root (t > 1e-5) only
// if the ray points into the cone of directions from B''_h to ball(c_i, r'_i),
// r'_i = |r_i| + mu_i, mu_i = 2^-8 (D + rho_h + |r_i|) (D = |c_i - c_h|; the
// shadow masks' margin for the reference's rounding): its axis is
// u = (c_i - c_h) / D and its half-angle is at most
//   alpha = asin(r'_i / (D - rho_h)) + asin(rho_h / D)
// (every sphere when D <= rho_h + r'_i, and sphere h itself).  The kernel
// uses the masks of (h, tier, cell(U)) when every active lane's direction lies
// within the tier's half-angle kConeHalf[tier] of the first lane's U; U lies
// in its cube-map cell, whose directions are within beta (the largest angle
// from the cell's centre direction to a corner) of that centre.  So sphere i
// is in mask (h, tier, cell) when angle(centre, u) <= alpha + kConeHalf[tier]
// + beta + 1e-3 (the 1e-3 rad covers the float direction estimates and cell
// borders).  tests/test_oracle.py::test_cone_masks_are_conservative.
inline void cone_masks(const rtg_sphere* spheres, unsigned n, std::vector<unsigned>* out) {
  out->assign((size_t)n * kConeTiers * kConeCells * 2, 0u);
  const double kPi = 3.14159265358979323846;
  // cell centres and radii
  std::vector<double> cc((size_t)kConeCells * 3), cb(kConeCells);
  for (int face = 0; face < 6; ++face)
    for (int ia = 0; ia < kConeGrid; ++ia)
      for (int ib = 0; ib < kConeGrid; ++ib) {
        const int cell = (face * kConeGrid + ia) * kConeGrid + ib;
        const int major = face / 2;
        const double sg = (face % 2 == 0) ? 1.0 : -1.0;
        const int ax = major == 0 ? 1 : 0, bx = major == 2 ? 1 : 2;
        auto dirv = [&](double a, double b, double* v) {
          v[0] = v[1] = v[2] = 0.0;
          v[major] = sg;
          v[ax] = a;
          v[bx] = b;
          const double l = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
          for (int k = 0; k < 3; ++k) v[k] /= l;
        };
        const double a0 = -1.0 + 2.0 * ia / kConeGrid, a1 = a0 + 2.0 / kConeGrid;
        const double b0 = -1.0 + 2.0 * ib / kConeGrid, b1 = b0 + 2.0 / kConeGrid;
        double c[3];
        dirv(0.5 * (a0 + a1), 0.5 * (b0 + b1), c);
        double beta = 0.0;
        const double corners[4][2] = {{a0, b0}, {a0, b1}, {a1, b0}, {a1, b1}};
        for (const auto& co : corners) {
          double v[3];
          dirv(co[0], co[1], v);
          const double dt = c[0] * v[0] + c[1] * v[1] + c[2] * v[2];
          beta = fmax(beta, acos(fmin(1.0, fmax(-1.0, dt))));
        }
        for (int k = 0; k < 3; ++k) cc[(size_t)cell * 3 + k] = c[k];
        cb[cell] = beta;
      }
  // The angle test ang(cell centre, u) > X with X = A + beta_cell, A = alpha +
  // tier + 1e-3, is taken as cos: for X < pi, acos(dt) > X  <=>  dt < cos X,
  // and cos X = cos A cos beta - sin A sin beta from per-(h, i, tier) and
  // per-cell values; a sphere is kept when dt >= cos X - 1e-12 (the margin
  // covers the rounding of both sides, so the masks keep at least what the
  // acos form kept), and always when X >= pi.
  std::vector<double> cbc(kConeCells), cbs(kConeCells);
  for (int cell = 0; cell < kConeCells; ++cell) {
    cbc[cell] = cos(cb[cell]);
    cbs[cell] = sin(cb[cell]);
  }
  for (unsigned h = 0; h < n; ++h) {
    const rtg_sphere& sh = spheres[h];
    const double ch = fabs((double)sh.pos.x) + fabs((double)sh.pos.y) + fabs((double)sh.pos.z);
    const double g = guard_radius(sh);
    const double rho = g + 0.0101 + 0x1p-20 * (ch + g);
    for (unsigned i = 0; i < n; ++i) {
      const rtg_sphere& si = spheres[i];
      const double ux = (double)si.pos.x - sh.pos.x, uy = (double)si.pos.y - sh.pos.y,
                   uz = (double)si.pos.z - sh.pos.z;
      const double D = sqrt(ux * ux + uy * uy + uz * uz);
      const double ri = fabs((double)si.radius);
      const double rr = ri + 0x1p-8 * (D + rho + ri);
      const bool all = (i == h) || !(D > (rho + rr) * (1.0 + 1e-9));
      double alpha = 0.0;
      if (!all) alpha = asin(fmin(1.0, rr / (D - rho))) + asin(fmin(1.0, rho / D));
      for (int tier = 0; tier < kConeTiers; ++tier) {
        const double A = alpha + kConeHalf[tier] + 1e-3;
        const double cA = cos(A), sA = sin(A);
        for (int cell = 0; cell < kConeCells; ++cell) {
          bool keep = all || A + cb[cell] >= kPi;
          if (!keep) {
            const double* c = &cc[(size_t)cell * 3];
            const double dt = (c[0] * ux + c[1] * uy + c[2] * uz) / D;
            keep = dt >= cA * cbc[cell] - sA * cbs[cell] - 1e-12;
          }
          if (keep)
            (*out)[(((size_t)h * kConeTiers + tier) * kConeCells + cell) * 2 + (i >> 5)] |=
                1u << (i & 31);
        }
      }
    }
  }
}

// 4-wide BVH of axis-aligned boxes (the queries are closest_bvh, blocked_bvh
// and container_bvh in rtg_trace.h).  Each sphere gets a grown box (bvh_grow
// below: every point the reference's root test can accept, and its
// containment ball, lie inside with a margin for the kernel's slab
// arithmetic); a node's slot holds the union of its spheres' grown boxes.
// Top-down: a node's spheres are split in two by a surface-area sweep (split
// below), and each half again, into four groups; a group of one sphere
// becomes a sphere slot, a larger group a child node; nodes of <= 4 spheres
// hold sphere slots only.  Returns false (no BVH) for non-finite scenes,
// coordinates beyond 2^56 or an implausibly deep tree.

// The origin box B* of a scene: every ray origin the kernel queries — the
// camera at 0 (main.cpp:417), hit points (within r_h + mu_h of their sphere,
// mu_h = 2^-8 (|p| + |r_h|) <= 2^-8 (diam B* + r_max), rtg_trace.h) and the
// reference's offsets P + 0.01 rd (|rd| ~ 1) — lies inside it:
//   B* = box(0, c_i -+ |r_i|) grown by pad = 0.02 + 2^-6 (diagonal + r_max),
// which exceeds 2^-8 (diam B* + r_max) + 0.0101 (diam B* <= diagonal +
// 2 sqrt(3) pad).  `omax` is its largest coordinate magnitude.
struct OriginBox {
  double lo[3], hi[3], omax;
};
inline OriginBox origin_box(const rtg_sphere* spheres, unsigned n) {
  OriginBox b;
  double rmax = 0.0;
  for (int a = 0; a < 3; ++a) b.lo[a] = b.hi[a] = 0.0;
  for (unsigned i = 0; i < n; ++i) {
    const double c[3] = {spheres[i].pos.x, spheres[i].pos.y, spheres[i].pos.z};
    const double r = fabs((double)spheres[i].radius);
    rmax = fmax(rmax, r);
    for (int a = 0; a < 3; ++a) {
      b.lo[a] = fmin(b.lo[a], c[a] - r);
      b.hi[a] = fmax(b.hi[a], c[a] + r);
    }
  }
  double d2 = 0.0;
  for (int a = 0; a < 3; ++a) d2 += (b.hi[a] - b.lo[a]) * (b.hi[a] - b.lo[a]);
  const double pad = 0.02 + 0x1p-6 * (sqrt(d2) + rmax);
  b.omax = 0.0;
  for (int a = 0; a < 3; ++a) {
    b.lo[a] -= pad;
    b.hi[a] += pad;
    b.omax = fmax(b.omax, fmax(fabs(b.lo[a]), fabs(b.hi[a])));
  }
  return b;
}

// Sphere (c, r)'s grown box for rays whose origins lie within `pmax` of c
// and have coordinates of magnitude <= omax (rtg_trace.h, "Why a box keeps
// every sphere"): half-width |r| + 2^-8 (pmax + |r|) + 2^-18 (|c|_inf + |r| +
// omax) + 2^-20, in double, rounded outward to float.  `m` is the 2^-8
// margin (tests probe smaller ones).
inline void bvh_grow(const double c[3], double r, double pmax, double omax, float lo[3],
                     float hi[3], double m = 0x1p-8) {
  r = fabs(r);
  const double cm = fmax(fabs(c[0]), fmax(fabs(c[1]), fabs(c[2])));
  const double w = r + m * (pmax + r) + 0x1p-18 * (cm + r + omax) + 0x1p-20;
  for (int a = 0; a < 3; ++a) {
    lo[a] = round_down_f(c[a] - w);
    hi[a] = round_up_f(c[a] + w);
  }
}

inline bool build_bvh(const rtg_sphere* spheres, unsigned n, PackedScene* ps) {
  ps->bvhNodes.clear();
  if (n <= kMaskMaxSpheres) return false;
  auto finite = [](double v) { return v == v && fabs(v) <= 1e30; };
  for (unsigned i = 0; i < n; ++i)
    if (!finite(spheres[i].pos.x) || !finite(spheres[i].pos.y) || !finite(spheres[i].pos.z) ||
        !finite(spheres[i].radius))
      return false;
  const OriginBox ob = origin_box(spheres, n);
  // The slab test (rtg_trace.h make_boxq / slab_pass) multiplies origins and
  // box planes by 1/d, up to 2^64 for a near-axis direction: with every
  // coordinate below 2^57 (the origin box and the grown boxes within it) the
  // products stay below 2^121, finite.  Larger scenes take the flat queries.
  if (!(ob.omax <= 0x1p56)) return false;
  // grown boxes: 6 floats per sphere
  std::vector<float> gb((size_t)n * 6);
  for (unsigned i = 0; i < n; ++i) {
    const double c[3] = {spheres[i].pos.x, spheres[i].pos.y, spheres[i].pos.z};
    double p2 = 0.0;
    for (int a = 0; a < 3; ++a) {
      const double e = fmax(fabs(ob.lo[a] - c[a]), fabs(ob.hi[a] - c[a]));
      p2 += e * e;
    }
    bvh_grow(c, spheres[i].radius, sqrt(p2), ob.omax, &gb[6 * (size_t)i], &gb[6 * (size_t)i + 3]);
  }
  std::vector<unsigned> idx(n);
  for (unsigned i = 0; i < n; ++i) idx[i] = i;
  auto cen = [&](unsigned i, int ax) {
    return 0.5 * ((double)gb[6 * (size_t)i + ax] + (double)gb[6 * (size_t)i + 3 + ax]);
  };
  auto grow = [&](unsigned i, double* mn, double* mx) {
    for (int q = 0; q < 3; ++q) {
      mn[q] = fmin(mn[q], (double)gb[6 * (size_t)i + q]);
      mx[q] = fmax(mx[q], (double)gb[6 * (size_t)i + 3 + q]);
    }
  };
  auto area = [](const double* mn, const double* mx) {
    const double x = mx[0] - mn[0], y = mx[1] - mn[1], z = mx[2] - mn[2];
    return x * y + y * z + z * x;
  };
  // Split of idx[lo, hi) (>= 2 spheres) into two non-empty runs, returned as
  // the first index of the second run: the centroid order on each axis,
  // minimising n_left * area_left + n_right * area_right (the chance that a
  // line meets a box grows with its surface area).
  std::vector<double> suf;
  auto split = [&](unsigned lo, unsigned hi) {
    const unsigned cnt = hi - lo;
    double bestCost = 1e308;
    int bestAx = 0;
    unsigned bestK = cnt / 2;
    suf.assign(cnt + 1, 0.0);
    for (int ax = 0; ax < 3; ++ax) {
      std::sort(idx.begin() + lo, idx.begin() + hi, [&](unsigned a, unsigned b) {
        const double ca = cen(a, ax), cb = cen(b, ax);
        return ca < cb || (ca == cb && a < b);
      });
      double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
      for (unsigned k = cnt; k-- > 1;) {  // suffix boxes: runs [k, cnt)
        grow(idx[lo + k], mn, mx);
        suf[k] = area(mn, mx);
      }
      double pmn[3] = {1e300, 1e300, 1e300}, pmx[3] = {-1e300, -1e300, -1e300};
      for (unsigned k = 1; k < cnt; ++k) {  // prefix [0, k) | suffix [k, cnt)
        grow(idx[lo + k - 1], pmn, pmx);
        const double cost = k * area(pmn, pmx) + (cnt - k) * suf[k];
        if (cost < bestCost) {
          bestCost = cost;
          bestAx = ax;
          bestK = k;
        }
      }
    }
    std::sort(idx.begin() + lo, idx.begin() + hi, [&](unsigned a, unsigned b) {
      const double ca = cen(a, bestAx), cb = cen(b, bestAx);
      return ca < cb || (ca == cb && a < b);
    });
    return lo + bestK;
  };
  int maxDepth = 0;
  // node for idx[lo, hi), returns its index
  std::function<int(unsigned, unsigned, int)> build = [&](unsigned lo, unsigned hi,
                                                          int depth) -> int {
    maxDepth = depth > maxDepth ? depth : maxDepth;
    const int node = (int)(ps->bvhNodes.size() / kBvhWords);
    ps->bvhNodes.resize(ps->bvhNodes.size() + kBvhWords, 0.f);
    {  // empty slots: NaN geometry, child 0
      float* e = &ps->bvhNodes[(size_t)node * kBvhWords];
      for (int k = 0; k < 24; ++k) e[k] = __builtin_nanf("");
      for (int k = 28; k < 32; ++k) e[k] = -1.f;
    }
    unsigned g[5];
    const unsigned cnt = hi - lo;
    if (cnt <= 4) {
      for (unsigned k = 0; k <= cnt; ++k) g[k] = lo + k;
      for (unsigned k = cnt + 1; k <= 4; ++k) g[k] = hi;
    } else {
      g[0] = lo;
      g[4] = hi;
      g[2] = split(lo, hi);
      g[1] = split(lo, g[2]);
      g[3] = split(g[2], hi);
    }
    for (int k = 0; k < 4; ++k) {
      const unsigned a = g[k], b = g[k + 1];
      if (a >= b) continue;
      int child;
      float s[6], cr = -1.f;
      if (b - a == 1) {
        const unsigned i = idx[a];
        const rtg_sphere& sp = spheres[i];
        s[0] = sp.pos.x; s[1] = sp.pos.y; s[2] = sp.pos.z;
        const float r2 = sp.radius * sp.radius;  // raytracer.h:100, the exact root test
        s[3] = screen_r2(r2);
        s[4] = r2;
        s[5] = round_up_f(fabs((double)sp.radius) * (1.0 + 0x1p-7) * (1.0 + 0x1p-20));
        const float rc = sp.radius + 1.0e-6f;  // raytracer.h:259-264
        cr = rc * rc;
        child = ~(int)i;
      } else {
        float mn[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
        float mx[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
        for (unsigned t = a; t < b; ++t)
          for (int q = 0; q < 3; ++q) {
            mn[q] = fminf(mn[q], gb[6 * (size_t)idx[t] + q]);
            mx[q] = fmaxf(mx[q], gb[6 * (size_t)idx[t] + 3 + q]);
          }
        for (int q = 0; q < 3; ++q) {
          s[q] = mn[q];
          s[3 + q] = mx[q];
        }
        child = build(a, b, depth + 1);
      }
      float* rec = &ps->bvhNodes[(size_t)node * kBvhWords];
      for (int q = 0; q < 6; ++q) rec[6 * k + q] = s[q];
      memcpy(&rec[24 + k], &child, 4);
      rec[28 + k] = cr;
    }
    return node;
  };
  build(0, n, 0);
  if (maxDepth > 20) {  // the wave stack holds 3 * depth + 1 <= 64 entries
    ps->bvhNodes.clear();
    return false;
  }
  // DevScene::bvh_rec addresses a node copy by a 32-bit byte offset
  // (kBvhWords * 4 bytes per copy, kBvhCopies per node): a tree past 2^32
  // bytes takes the flat queries instead (about 4 M nodes, n ~ 5 M spheres).
  if ((double)(ps->bvhNodes.size() / kBvhWords) * kBvhCopies * kBvhWords * 4.0 >= 0x1p32) {
    ps->bvhNodes.clear();
    return false;
  }
  {  // a copy of every node per direction octant (rtg_trace.h kBvhCopies)
    const std::vector<float> src = ps->bvhNodes;
    const size_t nn = src.size() / kBvhWords;
    ps->bvhNodes.assign(nn * 8 * kBvhWords, 0.f);
    for (size_t nd = 0; nd < nn; ++nd) {
      const float* in = &src[nd * kBvhWords];
      for (unsigned oct = 0; oct < 8; ++oct) {
        const double sg[3] = {(oct & 1u) ? -1.0 : 1.0, (oct & 2u) ? -1.0 : 1.0,
                              (oct & 4u) ? -1.0 : 1.0};
        int ord[4] = {0, 1, 2, 3};
        double key[4];
        int cls[4];  // 0 child box, 1 sphere, 2 empty
        for (int k = 0; k < 4; ++k) {
          int ch;
          memcpy(&ch, &in[24 + k], 4);
          key[k] = 0.0;
          cls[k] = ch > 0 ? 0 : ch < 0 ? 1 : 2;
          if (ch > 0) {  // child box: its near corner along the octant's diagonal (item 51)
            for (int q = 0; q < 3; ++q) {
              const double lo = in[6 * k + q], hi = in[6 * k + 3 + q];
              key[k] += sg[q] * (sg[q] > 0 ? lo : hi);
            }
          } else if (ch < 0) {  // sphere: its near point along the diagonal (item 52)
            for (int q = 0; q < 3; ++q) key[k] += sg[q] * (double)in[6 * k + q];
            key[k] = key[k] * 0.5773502691896258 - (double)in[6 * k + 5];
          }
        }
        std::stable_sort(ord, ord + 4, [&](int a, int b) {
          return cls[a] != cls[b] ? cls[a] < cls[b] : key[a] < key[b];
        });
        float* out = &ps->bvhNodes[(nd * 8 + oct) * kBvhWords];
        for (int k = 0; k < 4; ++k) {
          const int j = ord[k];
          for (int q = 0; q < 6; ++q) out[6 * k + q] = in[6 * j + q];
          out[24 + k] = in[24 + j];
          out[28 + k] = in[28 + j];
        }
      }
    }
  }
  return true;
}

inline void pack_scene(const rtg_sphere* spheres, unsigned n, const rtg_light* lights,
                       unsigned m, PackedScene* ps) {
  ps->n = n;
  ps->m = m;
  ps->n4 = (n + 3u) & ~3u;
  // Padding records are NaN spheres: their radicand is NaN, never >= 0.
  // three parts of (n4 + 4) 16-byte records, then the fused part: (n4 + 4)
  // 32-byte records {x, y, z, screen r^2, r^2, primary c term, 0, 0}
  ps->geom.assign((size_t)(ps->n4 + 4) * 20, __builtin_nanf(""));
  ps->crad2.assign(n ? 3 * (size_t)n : 1, 0.f);
  ps->mats.assign((size_t)(n + 1) * 8, 0.f);
  ps->lights.assign((size_t)(m ? m : 1) * 6, 0.f);
  ps->prim.assign((size_t)(n ? n : 1) * 4, 0.f);
  for (unsigned i = 0; i < n; ++i) {
    const rtg_sphere& s = spheres[i];
    float* g = &ps->geom[(size_t)i * 4];
    g[0] = s.pos.x; g[1] = s.pos.y; g[2] = s.pos.z;
    g[3] = s.radius * s.radius;
    float* gs = &ps->geom[(size_t)(ps->n4 + 4 + i) * 4];
    gs[0] = g[0]; gs[1] = g[1]; gs[2] = g[2];
    gs[3] = screen_r2(g[3]);
    float* gc = &ps->geom[(size_t)(2 * (ps->n4 + 4) + i) * 4];
    gc[0] = g[0]; gc[1] = g[1]; gc[2] = g[2];
    const float rc = s.radius + 1.0e-6f;
    ps->crad2[i] = rc * rc;
    gc[3] = ps->crad2[i];
    const float dx = 0.f - s.pos.x, dy = 0.f - s.pos.y, dz = 0.f - s.pos.z;
    ps->crad2[n + i] = (((dx * dx) + (dy * dy)) + (dz * dz)) - g[3];
    ps->crad2[2 * (size_t)n + i] = guard_r2(s);
    float* gf = &ps->geom[(size_t)(ps->n4 + 4) * 12 + (size_t)i * 8];
    gf[0] = g[0]; gf[1] = g[1]; gf[2] = g[2];
    gf[3] = gs[3];
    gf[4] = g[3];
    gf[5] = ps->crad2[n + i];
    gf[6] = 0.f; gf[7] = 0.f;
    prim_consts(s, &ps->prim[(size_t)i * 4]);
    float* mt = &ps->mats[(size_t)i * 8];
    mt[0] = s.material.matteColour.x; mt[1] = s.material.matteColour.y;
    mt[2] = s.material.matteColour.z; mt[3] = s.material.glossColour.x;
    mt[4] = s.material.glossColour.y; mt[5] = s.material.glossColour.z;
    mt[6] = s.material.opacity; mt[7] = s.material.refractiveIndex;
  }
  ps->mats[(size_t)n * 8 + 7] = 1.00f;
  shadow_masks(spheres, n, lights, m, &ps->smask);
  if (!ps->smask.empty()) cone_masks(spheres, n, &ps->cone);
  else ps->cone.clear();
  if (build_bvh(spheres, n, ps)) {
    sphere_lists(spheres, n, lights, m, ps);
  }
  for (unsigned l = 0; l < m; ++l) {
    float* p = &ps->lights[(size_t)l * 6];
    p[0] = lights[l].pos.x; p[1] = lights[l].pos.y; p[2] = lights[l].pos.z;
    p[3] = lights[l].col.x; p[4] = lights[l].col.y; p[5] = lights[l].col.z;
  }
}

// main.cpp:384-402.
inline int make_camera(unsigned W, unsigned H, float zoom, float aa, Camera* cam) {
  if (W == 0 || H == 0) {
    rtg_set_error("empty frame %ux%u", W, H);
    return RTG_ERR_INVALID;
  }
  if (!(aa <= 256.f)) {  // also rejects NaN
    rtg_set_error("aliasFactor %g out of range", (double)aa);
    return RTG_ERR_INVALID;
  }
  cam->xs = 16.f / ((float)W);
  cam->ys = 12.f / ((float)H);
  cam->asp = 16.f / 12.f;
  cam->st = cam->xs / aa;
  const float tot = aa * aa;
  cam->inv = 1.f / tot;
  cam->halfW = W * 0.5f;
  cam->halfH = H * 0.5f;
  cam->zoom = zoom;
  int k = 0;
  while ((float)k < aa) ++k;  // `for (int i = 0; i < aliasFactor; ++i)`
  cam->nAA = k;
  return RTG_OK;
}

}  // namespace rtg
