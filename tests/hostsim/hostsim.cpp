// tests/hostsim/hostsim.cpp — TEST-ONLY host build of the GPU kernel's
// traversal (raytracer-gamma_amd/csrc/rtg_trace.h) over the same scene
// preparation (rtg_scene_pack.h).  It lets the CPU test suite check the
// kernel's restructured algorithm (frame stack, stale-register handling,
// leaf doubling, early-exit shadow rays) bit for bit against the oracle
// without a GPU.  It is not part of librtg.so and no product path calls it.
#include <math.h>
#include <string.h>

#include <vector>

#include "rtg.h"
#include "rtg_internal.h"
#include "rtg_scene_pack.h"
#include "rtg_trace.h"

void rtg_set_error(const char*, ...) {}
void rtg_clear_error() {}

long g_counts[rtg::kCntSlots];

namespace {
struct HostScene {
  void count(int slot, long v) const { g_counts[slot] += v; }
  const float* geom;
  const float* crad2;
  const float* mats;
  const float* lights;
  unsigned n, m, n4;
  bool all(bool b) const { return b; }
  bool any(bool b) const { return b; }
  int fuse = 0;  // fused query forms (rtg_trace.h kFuse*), set per variant
  const float* bvhNodes = nullptr;
  const float* capRec = nullptr;
  const unsigned* capOff = nullptr;
  const float* ovRec = nullptr;
  const unsigned* ovOff = nullptr;
  bool has_lists() const { return capOff != nullptr; }
  void cap_range(unsigned l, unsigned h, unsigned cell, unsigned& k0, unsigned& k1) const {
    const size_t slot = ((size_t)l * n + h) * rtg::kCapCells + cell;
    k0 = capOff[2 * slot];
    k1 = capOff[2 * slot + 1];
  }
  void ov_range(unsigned h, unsigned& k0, unsigned& k1) const {
    k0 = ovOff[h];
    k1 = ovOff[h + 1];
  }
  static rtg::V3 list_rec(const float* b, unsigned k, float& rs, float& r2, float& cr, int& idx,
                          float& rf) {
    const float* g = b + 8 * (size_t)k;
    rs = g[3];
    r2 = g[4];
    cr = g[5];
    memcpy(&idx, &g[6], 4);
    rf = g[7];
    return rtg::v3(g[0], g[1], g[2]);
  }
  static void list_rec2(const float* b, unsigned k, rtg::ListRec& r0, rtg::ListRec& r1) {
    r0.c = list_rec(b, k, r0.rs, r0.r2, r0.cr, r0.idx, r0.rf);
    r1.c = list_rec(b, k + 1, r1.rs, r1.r2, r1.cr, r1.idx, r1.rf);
  }
  void cap_rec4(unsigned k, rtg::CapRec* r) const {
    for (int j = 0; j < 4; ++j) {
      const float* g = capRec + 4 * ((size_t)k + j);
      r[j].c = rtg::v3(g[0], g[1], g[2]);
      r[j].r2 = g[3];
    }
  }
  void ov_rec2(unsigned k, rtg::ListRec& r0, rtg::ListRec& r1) const {
    list_rec2(ovRec, k, r0, r1);
  }
  rtg::V3 ov_rec(unsigned k, float& rs, float& r2, float& cr, int& idx, float& rf) const {
    return list_rec(ovRec, k, rs, r2, cr, idx, rf);
  }
  bool has_bvh() const { return bvhNodes != nullptr; }
  const float* prim = nullptr;
  const unsigned* cone = nullptr;
  bool has_cone() const { return cone != nullptr; }
  rtg::V3 first_lane(rtg::V3 v) const { return v; }
  uint64_t cone_union(int h, unsigned tier, unsigned cell) const {
    const unsigned* w =
        cone + 2u * (((unsigned)h * rtg::kConeTiers + tier) * rtg::kConeCells + cell);
    return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  }
  int* bvh_stack() const { return nullptr; }
  void bvh_rec(unsigned nd, rtg::BvhRec& r) const {
    const float* g = bvhNodes + (size_t)rtg::kBvhWords * nd;
    memcpy(r.s, g, 24 * 4);
    memcpy(r.ch, g + 24, 4 * 4);
    memcpy(r.cr, g + 28, 4 * 4);
  }
  float first_lane(float v) const { return v; }
  int first_lane_i(int v) const { return v; }
  int lane_with(int v, bool) const { return v; }
  rtg::V3 sphere(unsigned i, float& r2) const {
    const float* g = geom + 4 * i;
    r2 = g[3];
    return rtg::v3(g[0], g[1], g[2]);
  }
  rtg::V3 sphere_lane(unsigned i, float& r2) const { return sphere(i, r2); }
  float sphere_r2(unsigned i) const { return geom[4 * i + 3]; }
  rtg::V3 sphere_fused(unsigned i, float& rs, float& r2, float& oc) const {
    const float* g = geom + 12 * (n4 + 4) + 8 * i;
    rs = g[3];
    r2 = g[4];
    oc = g[5];
    return rtg::v3(g[0], g[1], g[2]);
  }
  void probe_begin(int) const {}
  struct Frames {
    rtg::FrameC* f;
    rtg::FrameC get(int lv) const { return f[lv]; }
    void set(int lv, const rtg::FrameC& v) const { f[lv] = v; }
  };
  mutable rtg::FrameC fr[16];
  Frames frames() const { return Frames{fr}; }
  void probe_end(int) const {}
  void sphere4(unsigned i, rtg::V3* c, float* r2) const {
    for (int k = 0; k < 4; ++k) c[k] = sphere(i + k, r2[k]);
  }
  void sphere4_screen(unsigned i, rtg::V3* c, float* rs) const { sphere4(n4 + 4 + i, c, rs); }
  rtg::V3 sphere_screen(unsigned i, float& rs) const { return sphere(n4 + 4 + i, rs); }
  void sphere4_contain(unsigned i, rtg::V3* c, float* cr) const { sphere4(2 * (n4 + 4) + i, c, cr); }
  rtg::V3 sphere_contain(unsigned i, float& cr) const { return sphere(2 * (n4 + 4) + i, cr); }
  uint64_t contain_union(int hit, bool ok) const {
    if (!ok) return n >= 64 ? ~0ull : ((1ull << n) - 1ull);
    return overlap_mask((unsigned)hit);
  }
  // shadow masks: a single lane, so the union is that lane's mask
  const unsigned* smask = nullptr;
  bool has_smask() const { return smask != nullptr; }
  uint64_t overlap_mask(unsigned h) const {
    const unsigned* w = smask + 2u * (m * n + h);
    return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  }
  float guard_r2(unsigned i) const { return crad2[2 * n + i]; }
  uint64_t overlap_union(int h, uint64_t& own) const {
    own = overlap_mask((unsigned)h);
    return own;
  }
  uint64_t shadow_union(unsigned l, int hit, bool guardOK) const {
    if (!guardOK) return n >= 64 ? ~0ull : ((1ull << n) - 1ull);
    const unsigned* w = smask + 2u * (l * n + (unsigned)hit);
    return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  }
  float contain_r2(unsigned i) const { return crad2[i]; }
  float origin_c(unsigned i) const { return crad2[n + i]; }
  rtg::Mat mat(int i) const {
    const float* p = mats + 8 * i;
    rtg::Mat r;
    r.matte = rtg::v3(p[0], p[1], p[2]);
    r.gloss = rtg::v3(p[3], p[4], p[5]);
    r.opacity = p[6];
    r.refr = p[7];
    return r;
  }
  float refr(int i) const { return mats[8 * i + 7]; }
  void hit_data(int i, rtg::V3& c, float& g2, float& r2, rtg::Mat& mt) const {
    c = sphere((unsigned)i, r2);
    g2 = guard_r2((unsigned)i);
    mt = mat(i);
  }
  rtg::V3 sphere_guard(int h, float& r2, float& g2) const {
    g2 = guard_r2((unsigned)h);
    return sphere((unsigned)h, r2);
  }
  void light(unsigned l, rtg::V3& pos, rtg::V3& col) const {
    const float* p = lights + 6 * l;
    pos = rtg::v3(p[0], p[1], p[2]);
    col = rtg::v3(p[3], p[4], p[5]);
  }
};

int g_variant = 0;
bool g_useBvh = true;
bool g_useLists = true;  // the sphere lists of BVH scenes (coherent-wave queries)
double g_boundM = 0.0;          // hostsim_bvh_bound_check: box margin probe (0: 2^-8)

template <int S>
void run(const HostScene& sc, const rtg::Camera& cam, unsigned W, unsigned y, float* out) {
  for (unsigned x = 0; x < W; ++x) {
    rtg::V3 p;
    switch (g_variant) {
      case 1: p = rtg::shade_pixel<S, 0>(sc, cam, x, y); break;
      case 2: p = rtg::shade_pixel_persistent<S, 2>(sc, cam, x, y); break;
      case 3: p = rtg::shade_pixel_persistent<S, 1>(sc, cam, x, y); break;
      case 4: p = rtg::shade_pixel_nodes<S, 2>(sc, cam, x, y); break;
      case 5: p = rtg::shade_pixel<S, 2, false>(sc, cam, x, y); break;
      case 8: p = rtg::shade_pixel<S, 3, true>(sc, cam, x, y); break;
      case 0:
      case 14:
      case 15:
      case 23:
      case 50: {  // sample-parallel kernel: samples traced one by one, summed in order
        // primary-ray cull over the pixel's samples (the kernel's is per wave)
        uint64_t sel = ~0ull;
        const bool use = sc.n <= 64;
        if (use) {
          float x0, x1, y0, y1;
          rtg::primary_bounds(cam, x, y, x0, x1, y0, y1);
          const rtg::PrimBundle pb = rtg::primary_bundle(x0, x1, y0, y1, cam.zoom);
          sel = 0;
          for (unsigned k = 0; k < sc.n; ++k) {
            float r2;
            const rtg::V3 c = sc.sphere(k, r2);
            const float* pk = sc.prim + 4 * k;
            if (rtg::primary_possible(pb, c, pk[0], pk[1], pk[2])) sel |= 1ull << k;
          }
        }
        p = rtg::v3(0.f, 0.f, 0.f);
        for (int s = 0; s < cam.nAA * cam.nAA; ++s) {
          float rx, ry;
          const rtg::V3 d = rtg::sample_dir(cam, x, y, s / cam.nAA, s % cam.nAA, rx, ry);
          rtg::V3 c = g_variant == 15   ? rtg::trace_sample<S, 2>(sc, d, sc.frames())
                      : g_variant == 50 ? rtg::trace_sample<S, 4, true>(sc, d, sc.frames(), use, sel)
                                        : rtg::trace_sample<S, 4>(sc, d, sc.frames(), use, sel);
          c = rtg::vsmul(cam.inv, c);
          p = rtg::vadd(p, c);
          g_counts[rtg::kCntSamples] += 1;
        }
        break;
      }
      default: {  // tile kernel (variant 9)
        // per-pixel primary cull: a stricter (smaller) bundle than the GPU's
        // per-wave one, so it exercises the cull's conservativeness harder
        uint64_t sel = ~0ull;
        bool use = sc.n <= 64;
        if (use) {
          float x0, x1, y0, y1;
          rtg::primary_bounds(cam, x, y, x0, x1, y0, y1);
          const rtg::PrimBundle pb = rtg::primary_bundle(x0, x1, y0, y1, cam.zoom);
          sel = 0;
          for (unsigned k = 0; k < sc.n; ++k) {
            float r2;
            const rtg::V3 c = sc.sphere(k, r2);
            const float* pk = sc.prim + 4 * k;
            if (rtg::primary_possible(pb, c, pk[0], pk[1], pk[2])) sel |= 1ull << k;
          }
        }
        p = rtg::shade_pixel<S, 2, true>(sc, cam, x, y, use, sel);
        break;
      }
    }
    out[3 * x + 0] = p.x;
    out[3 * x + 1] = p.y;
    out[3 * x + 2] = p.z;
  }
}
}  // namespace

extern "C" void hostsim_set_variant(int v) { g_variant = v; }
extern "C" void hostsim_use_bvh(int on) { g_useBvh = on != 0; }
extern "C" void hostsim_use_lists(int on) { g_useLists = on != 0; }
extern "C" void hostsim_capsule_back_slack(double s) { rtg::g_capsuleBackSlack = s; }
extern "C" void hostsim_bound_margin(double m) { g_boundM = m; }
// Operation counters of the kernel traversal (rtg_trace.h kCnt*), summed over
// the renders since the last reset (diagnostic; single-lane semantics, so the
// wave unions of the GPU are per-sample masks here).
extern "C" void hostsim_counts(long* out, int reset) {
  for (int k = 0; k < rtg::kCntSlots; ++k) {
    out[k] = g_counts[k];
    if (reset) g_counts[k] = 0;
  }
}

extern "C" int hostsim_render_rows(const rtg_sphere* spheres, unsigned n,
                                   const rtg_light* lights, unsigned m, unsigned W,
                                   unsigned H, float zoom, float aa, int S,
                                   const unsigned* rows, unsigned nrows, float* out) {
  rtg::PackedScene ps;
  rtg::pack_scene(spheres, n, lights, m, &ps);
  rtg::Camera cam;
  if (rtg::make_camera(W, H, zoom, aa, &cam)) return -1;
  HostScene sc{ps.geom.data(), ps.crad2.data(), ps.mats.data(), ps.lights.data(), n, m, ps.n4};
  sc.smask = ps.smask.empty() ? nullptr : ps.smask.data();
  sc.cone = ps.cone.empty() ? nullptr : ps.cone.data();
  sc.prim = ps.prim.data();
  // the kernel's FuseOf (rtg_trace_kernels.h): sample-kernel variants but 23
  sc.fuse = (g_variant == 0 || g_variant == 15 || g_variant == 50)
                ? (rtg::kFusePrim | rtg::kFuseCone | rtg::kFuseShadow | rtg::kFuseEnter)
                : 0;
  if (!ps.bvhNodes.empty() && g_useBvh) {
    sc.bvhNodes = ps.bvhNodes.data();
    if (!ps.capOff.empty() && g_useLists) {
      sc.capRec = ps.capRec.data();
      sc.capOff = ps.capOff.data();
      sc.ovRec = ps.ovRec.data();
      sc.ovOff = ps.ovOff.data();
    }
  }
  for (unsigned k = 0; k < nrows; ++k) {
    float* o = out + (size_t)k * W * 3;
    switch (S) {
#define C(s) case s: run<s>(sc, cam, W, rows[k], o); break;
      C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12)
#undef C
      default: return -1;
    }
  }
  return 0;
}

// Conservativeness of the primary-ray cull (primary_bundle + primary_possible
// with the host's prim_consts): over
// every group of `group` consecutive pixels of a W x H frame (the sample
// kernel's wave), bound the group's sample directions as the kernel does,
// then count spheres the cull drops although one of those samples hits them
// (exact ray_sphere from the origin).  *culled counts the drops in total.
extern "C" long hostsim_cull_violations(const rtg_sphere* spheres, unsigned n, unsigned W,
                                        unsigned H, float zoom, float aa, unsigned group,
                                        long* culled) {
  rtg::PackedScene ps;
  rtg::pack_scene(spheres, n, nullptr, 0, &ps);
  rtg::Camera cam;
  if (rtg::make_camera(W, H, zoom, aa, &cam)) return -1;
  HostScene sc{ps.geom.data(), ps.crad2.data(), ps.mats.data(), ps.lights.data(), n, 0, ps.n4};
  long bad = 0, drop = 0;
  const size_t total = (size_t)W * H;
  for (size_t p0 = 0; p0 < total; p0 += group) {
    float x0 = 3e38f, x1 = -3e38f, y0 = 3e38f, y1 = -3e38f;
    for (size_t p = p0; p < p0 + group && p < total; ++p)
      for (int i = 0; i < cam.nAA; ++i)
        for (int j = 0; j < cam.nAA; ++j) {
          float rx, ry;
          rtg::sample_dir(cam, (unsigned)(p % W), (unsigned)(p / W), i, j, rx, ry);
          x0 = fminf(x0, rx); x1 = fmaxf(x1, rx); y0 = fminf(y0, ry); y1 = fmaxf(y1, ry);
        }
    const rtg::PrimBundle pb = rtg::primary_bundle(x0, x1, y0, y1, cam.zoom);
    for (unsigned k = 0; k < n; ++k) {
      float r2;
      const rtg::V3 c = sc.sphere(k, r2);
      const float* pk = &ps.prim[(size_t)k * 4];
      if (rtg::primary_possible(pb, c, pk[0], pk[1], pk[2])) continue;
      ++drop;
      for (size_t p = p0; p < p0 + group && p < total; ++p)
        for (int i = 0; i < cam.nAA; ++i)
          for (int j = 0; j < cam.nAA; ++j) {
            float rx, ry;
            const rtg::V3 d = rtg::sample_dir(cam, (unsigned)(p % W), (unsigned)(p / W), i, j, rx, ry);
            const rtg::RayQ q = rtg::make_query(rtg::v3(0.f, 0.f, 0.f), d);
            bool res;
            rtg::ray_sphere(q, c, r2, res);
            if (res) ++bad;
          }
    }
  }
  if (culled) *culled = drop;
  return bad;
}

// Pass-1 screen (pass1_rad) vs the reference's radicand test on adversarial
// ray/sphere pairs: random origins, directions (unnormalised too) and scales,
// with the radius set so the ray passes within a relative 1e-7..1e-3 of
// tangency, and origins on the sphere surface (secondary rays).  Returns the
// number of pairs the reference accepts but the screen drops; *accepted and
// *extra count reference accepts and screen-only accepts.
extern "C" long hostsim_pass1_check(long trials, unsigned long long seed, long* accepted,
                                    long* extra) {
  unsigned long long st = seed * 0x9E3779B97F4A7C15ull + 1;
  auto u01 = [&]() {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    return (double)(st >> 11) * (1.0 / 9007199254740992.0);
  };
  long bad = 0, acc = 0, ext = 0;
  for (long t = 0; t < trials; ++t) {
    const double scale = pow(10.0, -3.0 + 6.0 * u01());
    rtg::V3 c = rtg::v3((float)((u01() - 0.5) * 20 * scale), (float)((u01() - 0.5) * 20 * scale),
                        (float)((u01() - 0.5) * 20 * scale));
    double dx = u01() - 0.5, dy = u01() - 0.5, dz = u01() - 0.5;
    const double dl = sqrt(dx * dx + dy * dy + dz * dz);
    const double dscale = (t % 3 == 0) ? 1.0 / dl : (0.1 + 3.0 * u01());
    rtg::V3 d = rtg::v3((float)(dx * dscale), (float)(dy * dscale), (float)(dz * dscale));
    rtg::V3 o;
    float r;
    const int mode = (int)(t % 4);
    if (mode == 3) {  // origin on the sphere surface, random direction
      r = (float)(scale * (0.1 + u01()));
      double ux = u01() - 0.5, uy = u01() - 0.5, uz = u01() - 0.5;
      const double ul = sqrt(ux * ux + uy * uy + uz * uz);
      o = rtg::v3((float)(c.x + r * ux / ul), (float)(c.y + r * uy / ul), (float)(c.z + r * uz / ul));
    } else {  // origin elsewhere, radius = distance(center, line) * (1 +- tiny)
      o = rtg::v3((float)((u01() - 0.5) * 20 * scale), (float)((u01() - 0.5) * 20 * scale),
                  (float)((u01() - 0.5) * 20 * scale));
      const double px = (double)o.x - c.x, py = (double)o.y - c.y, pz = (double)o.z - c.z;
      const double dd = (double)d.x * d.x + (double)d.y * d.y + (double)d.z * d.z;
      const double pd = px * d.x + py * d.y + pz * d.z;
      const double dist2 = px * px + py * py + pz * pz - pd * pd / dd;
      const double rel = pow(10.0, -7.0 + 4.0 * u01()) * (u01() < 0.5 ? -1.0 : 1.0);
      r = (float)(sqrt(fmax(dist2, 0.0)) * (1.0 + rel));
    }
    const float r2 = r * r;
    const rtg::RayQ q = rtg::make_query(o, d);
    // reference radicand (raytracer.h:99-108)
    const rtg::V3 disp = rtg::vsub(o, c);
    const float b = 2.0f * rtg::vdot(d, disp);
    const float cc = rtg::vdot(disp, disp) - r2;
    const float rad = (b * b) - (q.a4 * cc);
    const bool ref = rad >= 0.0f;
    const float s = rtg::pass1_rad(q, c, rtg::screen_r2(r2));
    unsigned u;
    memcpy(&u, &s, 4);
    const bool scr = (u >> 31) == 0;
    if (ref) ++acc;
    if (ref && !scr) ++bad;
    if (!ref && scr) ++ext;
  }
  if (accepted) *accepted = acc;
  if (extra) *extra = ext;
  return bad;
}

// Shadow masks (shadow_masks, rtg_scene_pack.h) against the reference's own
// blocking test (raytracer.h:272-309 with ray_sphere = raytracer.h:81-141):
// random scenes of `n` spheres, half of them placed just outside the reach of
// a random (light, sphere h) capsule; for every sphere i NOT in mask (l, h),
// `points` random hit points P inside h's guard ball (most within 1e-3 of the
// surface, half of them on the side facing sphere i) must not be blocked by
// sphere i.  Returns the violations;
// *tested counts the (P, i) pairs checked.
extern "C" long hostsim_shadow_mask_check(long scenes, unsigned n, long points,
                                          unsigned long long seed, long* tested) {
  unsigned long long st = seed * 0x9E3779B97F4A7C15ull + 7;
  auto u01 = [&]() {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    return (double)(st >> 11) * (1.0 / 9007199254740992.0);
  };
  long bad = 0, cnt = 0;
  std::vector<rtg_sphere> sph(n);
  rtg_light lg[2];
  for (long sc = 0; sc < scenes; ++sc) {
    const double scale = pow(10.0, -2.0 + 4.0 * u01());
    for (unsigned i = 0; i < n; ++i) {
      memset(&sph[i], 0, sizeof(rtg_sphere));
      sph[i].pos.x = (float)((u01() - 0.5) * 24 * scale);
      sph[i].pos.y = (float)((u01() - 0.5) * 16 * scale);
      sph[i].pos.z = (float)((-6 - 34 * u01()) * scale);
      sph[i].radius = (float)((0.3 + 3 * u01()) * scale);
    }
    for (int l = 0; l < 2; ++l) {
      lg[l].pos.x = (float)((u01() - 0.5) * 120 * scale);
      lg[l].pos.y = (float)((10 + 70 * u01()) * scale);
      lg[l].pos.z = (float)((u01() - 0.5) * 130 * scale);
    }
    // a quarter of the spheres: just behind sphere 0's plane facing light 0
    // (wholly on the far side of c_0, within the capsule's radius), which only
    // rays from points with incidence <= 0 could cross
    for (unsigned i = n / 4; i < n / 2; ++i) {
      const rtg_sphere& h = sph[0];
      const double A[3] = {h.pos.x, h.pos.y, h.pos.z};
      const double L[3] = {lg[0].pos.x, lg[0].pos.y, lg[0].pos.z};
      double ab[3], ab2 = 0.0;
      for (int k = 0; k < 3; ++k) { ab[k] = L[k] - A[k]; ab2 += ab[k] * ab[k]; }
      const double lh = sqrt(ab2);
      double v[3] = {u01() - 0.5, u01() - 0.5, u01() - 0.5};
      const double pr = (v[0] * ab[0] + v[1] * ab[1] + v[2] * ab[2]) / ab2;
      for (int k = 0; k < 3; ++k) v[k] -= pr * ab[k];
      const double vl = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
      const double ri = sph[i].radius;
      const double g = rtg::guard_radius(h);
      // centre this far behind: the sphere's front just behind or just ahead
      // of the plane
      const double back = ri * (1.0 + (u01() < 0.5 ? -1.0 : 1.0) * pow(10.0, -6.0 + 4.0 * u01()));
      const double lat = (g + ri) * u01();
      for (int k = 0; k < 3; ++k) {
        const double c = A[k] - back * ab[k] / lh + lat * v[k] / vl;
        (k == 0 ? sph[i].pos.x : k == 1 ? sph[i].pos.y : sph[i].pos.z) = (float)c;
      }
    }
    // half of the spheres: just outside (or on) the capsule of (light 0, sphere 0)
    for (unsigned i = n / 2; i < n; ++i) {
      const rtg_sphere& h = sph[0];
      const double t = (i & 1) ? u01() : 0.05 * u01() * u01();  // mostly near sphere 0
      const double A[3] = {h.pos.x, h.pos.y, h.pos.z};
      const double L[3] = {lg[0].pos.x, lg[0].pos.y, lg[0].pos.z};
      double p[3], ab[3];
      for (int k = 0; k < 3; ++k) { ab[k] = L[k] - A[k]; p[k] = A[k] + t * ab[k]; }
      // a unit vector orthogonal to ab
      double v[3] = {u01() - 0.5, u01() - 0.5, u01() - 0.5};
      const double ab2 = ab[0] * ab[0] + ab[1] * ab[1] + ab[2] * ab[2];
      const double pr = (v[0] * ab[0] + v[1] * ab[1] + v[2] * ab[2]) / ab2;
      for (int k = 0; k < 3; ++k) v[k] -= pr * ab[k];
      const double vl = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
      const double ri = sph[i].radius;
      const double g = rtg::guard_radius(h);
      const double dist = (g + ri) * (1.0 + pow(10.0, -4.0 + 2.5 * u01()));
      sph[i].pos.x = (float)(p[0] + dist * v[0] / vl);
      sph[i].pos.y = (float)(p[1] + dist * v[1] / vl);
      sph[i].pos.z = (float)(p[2] + dist * v[2] / vl);
    }
    std::vector<unsigned> masks;
    rtg::shadow_masks(sph.data(), n, lg, 2, &masks);
    if (masks.empty()) continue;  // (m * n shadow masks come first)
    for (int l = 0; l < 2; ++l)
      for (unsigned h = 0; h < n; ++h) {
        const unsigned* w = &masks[((size_t)l * n + h) * 2];
        const rtg_sphere& sh = sph[h];
        const double g = rtg::guard_radius(sh);
        const float G2 = rtg::guard_r2(sh);
        for (unsigned i = 0; i < n; ++i) {
          if (w[i >> 5] & (1u << (i & 31))) continue;
          for (long k = 0; k < points; ++k) {
            // P inside the guard ball, mostly near the sphere surface, half of
            // them on the side facing sphere i (grazing shadow rays)
            double ux = u01() - 0.5, uy = u01() - 0.5, uz = u01() - 0.5;
            if (k & 1) {
              const double cx = (double)sph[i].pos.x - sh.pos.x, cy = (double)sph[i].pos.y - sh.pos.y,
                           cz = (double)sph[i].pos.z - sh.pos.z;
              const double cl = sqrt(cx * cx + cy * cy + cz * cz) + 1e-300;
              const double spread = pow(10.0, -3.0 * u01());
              ux = cx / cl + spread * ux; uy = cy / cl + spread * uy; uz = cz / cl + spread * uz;
            }
            if (k % 4 == 3) {  // on h's rim facing light l, toward sphere i (grazing rays)
              const double lx = (double)lg[l].pos.x - sh.pos.x, ly = (double)lg[l].pos.y - sh.pos.y,
                           lz = (double)lg[l].pos.z - sh.pos.z;
              const double ll = sqrt(lx * lx + ly * ly + lz * lz) + 1e-300;
              double cx = (double)sph[i].pos.x - sh.pos.x, cy = (double)sph[i].pos.y - sh.pos.y,
                     cz = (double)sph[i].pos.z - sh.pos.z;
              const double pr = (cx * lx + cy * ly + cz * lz) / (ll * ll);
              cx -= pr * lx; cy -= pr * ly; cz -= pr * lz;
              const double cl = sqrt(cx * cx + cy * cy + cz * cz) + 1e-300;
              const double up = pow(10.0, -5.0 + 4.0 * u01());
              const double side = 1e-3 * (u01() - 0.5);
              ux = cx / cl + up * lx / ll + side * (u01() - 0.5);
              uy = cy / cl + up * ly / ll + side * (u01() - 0.5);
              uz = cz / cl + up * lz / ll + side * (u01() - 0.5);
            }
            const double ul = sqrt(ux * ux + uy * uy + uz * uz);
            const double rad = (k % 6 == 0) ? g * u01()
                                             : fabs((double)sh.radius) * (1.0 + (u01() - 0.7) * 2e-3);
            const rtg::V3 P = rtg::v3((float)(sh.pos.x + rad * ux / ul),
                                      (float)(sh.pos.y + rad * uy / ul),
                                      (float)(sh.pos.z + rad * uz / ul));
            const rtg::V3 e = rtg::vsub(P, rtg::v3(sh.pos.x, sh.pos.y, sh.pos.z));
            if (!(rtg::vdot(e, e) <= G2)) continue;  // the kernel tests every sphere then
            const rtg::V3 Lp = rtg::v3(lg[l].pos.x, lg[l].pos.y, lg[l].pos.z);
            const rtg::V3 dist = rtg::vsub(Lp, P);
            const float gap = rtg::vdot(dist, dist);
            const rtg::V3 D = rtg::vsmul(1.f / sqrtf(gap), dist);
            // the kernel casts a shadow ray only when the incidence is > 0
            // (matte_light, raytracer.h:337-349)
            const rtg::V3 N = rtg::vnorm(e);
            if (!(rtg::vdot(N, D) > 0.f)) continue;
            const rtg::RayQ q = rtg::make_query(P, D);
            ++cnt;
            bool res;
            const float t = rtg::ray_sphere(q, rtg::v3(sph[i].pos.x, sph[i].pos.y, sph[i].pos.z),
                                            sph[i].radius * sph[i].radius, res);
            if (res && t < 1000.f) {
              const rtg::V3 tv = rtg::vsmul(t, D);
              if (rtg::vdot(tv, tv) < gap) ++bad;
            }
          }
        }
      }
  }
  if (tested) *tested = cnt;
  return bad;
}

// Sizes of the shadow masks of a scene: *total = sum of popcounts over the
// m x n masks (-1 when the scene has none).
extern "C" long hostsim_shadow_mask_bits(const rtg_sphere* spheres, unsigned n,
                                         const rtg_light* lights, unsigned m) {
  std::vector<unsigned> masks;
  rtg::shadow_masks(spheres, n, lights, m, &masks);
  if (masks.empty()) return -1;
  long bits = 0;
  for (unsigned w : masks) bits += __builtin_popcount(w);
  return bits;
}

// Overlap masks as containment candidates (primary_container_sel): for a hit
// point P in sphere h's guard ball and a direction D with |D|^2 <= 9 (float),
// the refraction test point P + 0.01f D (raytracer.h:690) is never inside a
// sphere j outside mask h by the reference's own float test
// (raytracer.h:255-264).  Random scenes, half of the spheres placed just
// outside h's containment reach; returns the violations, *tested = points x
// spheres checked.
extern "C" long hostsim_contain_mask_check(long scenes, unsigned n, long points,
                                           unsigned long long seed, long* tested) {
  unsigned long long st = seed * 0x9E3779B97F4A7C15ull + 11;
  auto u01 = [&]() {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    return (double)(st >> 11) * (1.0 / 9007199254740992.0);
  };
  long bad = 0, cnt = 0;
  std::vector<rtg_sphere> sph(n);
  for (long sc = 0; sc < scenes; ++sc) {
    const double scale = pow(10.0, -1.5 + 3.0 * u01());
    for (unsigned i = 0; i < n; ++i) {
      memset(&sph[i], 0, sizeof(rtg_sphere));
      sph[i].pos.x = (float)((u01() - 0.5) * 24 * scale);
      sph[i].pos.y = (float)((u01() - 0.5) * 16 * scale);
      sph[i].pos.z = (float)((-6 - 34 * u01()) * scale);
      sph[i].radius = (float)((0.3 + 3 * u01()) * scale) * (u01() < 0.1 ? -1.f : 1.f);
    }
    // half of the spheres: just outside sphere 0's containment reach
    for (unsigned i = n / 2; i < n; ++i) {
      const rtg_sphere& h = sph[0];
      double v[3] = {u01() - 0.5, u01() - 0.5, u01() - 0.5};
      const double vl = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
      const double ri = fabs((double)sph[i].radius) + 1e-6;
      const double dist = (rtg::contain_reach(h) + ri) * (1.0 + pow(10.0, -5.0 + 3.0 * u01()));
      sph[i].pos.x = (float)(h.pos.x + dist * v[0] / vl);
      sph[i].pos.y = (float)(h.pos.y + dist * v[1] / vl);
      sph[i].pos.z = (float)(h.pos.z + dist * v[2] / vl);
    }
    std::vector<unsigned> masks;
    rtg::shadow_masks(sph.data(), n, nullptr, 0, &masks);
    if (masks.empty()) continue;  // m = 0: the n overlap masks only
    for (unsigned h = 0; h < n; ++h) {
      const unsigned* w = &masks[(size_t)h * 2];
      const rtg_sphere& sh = sph[h];
      const double g = rtg::guard_radius(sh);
      const float G2 = rtg::guard_r2(sh);
      for (unsigned j = 0; j < n; ++j) {
        if (w[j >> 5] & (1u << (j & 31))) continue;
        const float rc = sph[j].radius + 1.0e-6f;
        const float cr = rc * rc;
        const rtg::V3 cj = rtg::v3(sph[j].pos.x, sph[j].pos.y, sph[j].pos.z);
        for (long k = 0; k < points; ++k) {
          // P in the guard ball, mostly on h's surface facing sphere j; D
          // pointing at j, up to the length bound
          double ux = u01() - 0.5, uy = u01() - 0.5, uz = u01() - 0.5;
          const double cx = (double)cj.x - sh.pos.x, cy = (double)cj.y - sh.pos.y,
                       cz = (double)cj.z - sh.pos.z;
          const double cl = sqrt(cx * cx + cy * cy + cz * cz) + 1e-300;
          if (k & 1) {
            const double spread = pow(10.0, -3.0 * u01());
            ux = cx / cl + spread * ux; uy = cy / cl + spread * uy; uz = cz / cl + spread * uz;
          }
          const double ul = sqrt(ux * ux + uy * uy + uz * uz);
          const double rad = (k % 6 == 0) ? g * u01() : g * (1.0 - 1e-3 * u01());
          const rtg::V3 P = rtg::v3((float)(sh.pos.x + rad * ux / ul),
                                    (float)(sh.pos.y + rad * uy / ul),
                                    (float)(sh.pos.z + rad * uz / ul));
          const rtg::V3 e = rtg::vsub(P, rtg::v3(sh.pos.x, sh.pos.y, sh.pos.z));
          if (!(rtg::vdot(e, e) <= G2)) continue;  // the kernel scans every sphere then
          const double dl = rtg::kContainDirMax * (k % 3 == 0 ? u01() : 1.0 - 1e-6 * u01());
          const double sp = 0.05 * u01();
          double dx = cx / cl + sp * (u01() - 0.5), dy = cy / cl + sp * (u01() - 0.5),
                 dz = cz / cl + sp * (u01() - 0.5);
          const double dn = sqrt(dx * dx + dy * dy + dz * dz);
          const rtg::V3 D = rtg::v3((float)(dx / dn * dl), (float)(dy / dn * dl), (float)(dz / dn * dl));
          if (!(rtg::vdot(D, D) <= rtg::kContainDirMax * rtg::kContainDirMax)) continue;
          const rtg::V3 pt = rtg::vadd(rtg::vsmul(0.01f, D), P);
          ++cnt;
          const rtg::V3 dist = rtg::vsub(pt, cj);
          if (rtg::vdot(dist, dist) <= cr) ++bad;
        }
      }
    }
  }
  if (tested) *tested = cnt;
  return bad;
}

// BVH bounds against the reference's own root test (raytracer.h:81-141), on
// adversarial ray/sphere pairs (near-tangent lines, far spheres, origins on
// the surface, unnormalised directions, scales 1e-3..1e3):
//  * grown box (bvh_grow with the 2^-8 margin, origins within |o - c|):
//    the kernel's slab test passes every accepted sphere's box within the
//    closest query's reach t* and the shadow ray's reach;  -> *bad_screen
//  * root distance (beyond): an accepted root t never lies nearer than
//    |p| - r - 2^-8 (|p| + r) along the ray, so beyond() with reach just
//    below t |d| never prunes it.  -> return value
// *accepted counts accepted pairs.
extern "C" long hostsim_bvh_bound_check(long trials, unsigned long long seed, long* accepted,
                                        long* bad_screen) {
  unsigned long long st = seed * 0x9E3779B97F4A7C15ull + 5;
  auto u01 = [&]() {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    return (double)(st >> 11) * (1.0 / 9007199254740992.0);
  };
  long bad = 0, badS = 0, acc = 0;
  for (long t = 0; t < trials; ++t) {
    const double scale = pow(10.0, -3.0 + 6.0 * u01());
    rtg::V3 c = rtg::v3((float)((u01() - 0.5) * 20 * scale), (float)((u01() - 0.5) * 20 * scale),
                        (float)((u01() - 0.5) * 20 * scale));
    double dx = u01() - 0.5, dy = u01() - 0.5, dz = u01() - 0.5;
    const double dl = sqrt(dx * dx + dy * dy + dz * dz);
    const double dscale = (t % 3 == 0) ? 1.0 / dl : (0.1 + 3.0 * u01());
    rtg::V3 d = rtg::v3((float)(dx * dscale), (float)(dy * dscale), (float)(dz * dscale));
    rtg::V3 o;
    float r;
    const int mode = (int)(t % 4);
    const double far = (t % 5 == 0) ? pow(10.0, 1.0 + 2.0 * u01()) : 1.0;  // far, small spheres
    if (mode == 3) {  // origin on the sphere surface, random direction
      r = (float)(scale * (0.1 + u01()));
      double ux = u01() - 0.5, uy = u01() - 0.5, uz = u01() - 0.5;
      const double ul = sqrt(ux * ux + uy * uy + uz * uz);
      o = rtg::v3((float)(c.x + r * ux / ul), (float)(c.y + r * uy / ul), (float)(c.z + r * uz / ul));
    } else {  // radius = distance(centre, line) * (1 +- tiny), or a far sphere
              // the line misses by up to 3e-3 |p| (accepted only by rounding)
      o = rtg::v3((float)(c.x + (u01() - 0.5) * 20 * scale * far),
                  (float)(c.y + (u01() - 0.5) * 20 * scale * far),
                  (float)(c.z + (u01() - 0.5) * 20 * scale * far));
      const double px = (double)o.x - c.x, py = (double)o.y - c.y, pz = (double)o.z - c.z;
      const double dd = (double)d.x * d.x + (double)d.y * d.y + (double)d.z * d.z;
      const double pd = px * d.x + py * d.y + pz * d.z;
      const double dist2 = px * px + py * py + pz * pz - pd * pd / dd;
      const double dist = sqrt(fmax(dist2, 0.0));
      if (t % 2 == 0 && far > 1.0) {
        const double pl = sqrt(px * px + py * py + pz * pz);
        r = (float)(dist - 3e-3 * pl * u01() * u01());
        if (!(r > 0.f)) r = (float)(dist * 0.5);
      } else {
        const double rel = pow(10.0, -7.0 + 4.0 * u01()) * (u01() < 0.5 ? -1.0 : 1.0);
        r = (float)(dist * (1.0 + rel));
      }
    }
    if (t % 4 == 1) {  // tiny far sphere, line aimed just outside it: the
                       // reference accepts misses of up to ~7e-4 |p| here
      double ux = u01() - 0.5, uy = u01() - 0.5, uz = u01() - 0.5;
      const double ul = sqrt(ux * ux + uy * uy + uz * uz);
      ux /= ul; uy /= ul; uz /= ul;
      const double L = scale * pow(10.0, 1.0 + 2.0 * u01());
      o = rtg::v3((float)(c.x + L * ux), (float)(c.y + L * uy), (float)(c.z + L * uz));
      const double rr = L * pow(10.0, -7.0 + 4.0 * u01());
      const double miss = rr + L * 2e-3 * pow(u01(), 3);
      double vx = u01() - 0.5, vy = u01() - 0.5, vz = u01() - 0.5;
      const double vd = vx * ux + vy * uy + vz * uz;
      vx -= vd * ux; vy -= vd * uy; vz -= vd * uz;
      const double vl = sqrt(vx * vx + vy * vy + vz * vz) + 1e-300;
      const double ds = 0.1 + 3 * u01();
      d = rtg::v3((float)((c.x + miss * vx / vl - o.x) * ds / L),
                  (float)((c.y + miss * vy / vl - o.y) * ds / L),
                  (float)((c.z + miss * vz / vl - o.z) * ds / L));
      r = (float)rr;
    }
    const float r2 = r * r;
    const rtg::RayQ q = rtg::make_query(o, d);
    bool res;
    const float tr = rtg::ray_sphere(q, c, r2, res);
    if (!res) continue;
    ++acc;
    // grown box (bvh_grow) for origins within |o - c| of c: the ray passes
    // through it within reach t* (a closest query's minT) and within a
    // shadow ray's reach for the smallest gap that makes t* block
    {
      const double cd[3] = {c.x, c.y, c.z};
      const double px = (double)o.x - c.x, py = (double)o.y - c.y, pz = (double)o.z - c.z;
      const double pm = sqrt(px * px + py * py + pz * pz) * (1.0 + 1e-12);
      const double om = fmax(fabs((double)o.x), fmax(fabs((double)o.y), fabs((double)o.z)));
      float lo[3], hi[3];
      rtg::bvh_grow(cd, r, pm, om, lo, hi, g_boundM > 0.0 ? g_boundM : 0x1p-8);
      const rtg::BoxQ bq = rtg::make_boxq(q);
      float tn;
      bool ok = rtg::slab_pass(bq, rtg::v3(lo[0], lo[1], lo[2]), rtg::v3(hi[0], hi[1], hi[2]), tr, tn);
      const rtg::V3 dist = rtg::vsmul(tr, d);
      const float gap = nextafterf(rtg::vdot(dist, dist), __builtin_inff());
      if (ok && tr < 1000.f && q.fast) {
        const float rt = fminf(sqrtf(gap * (1.0f / (q.den * 0.5f))) * (1.0f + 0x1p-18f), 1000.f);
        ok = rtg::slab_pass(bq, rtg::v3(lo[0], lo[1], lo[2]), rtg::v3(hi[0], hi[1], hi[2]), rt, tn);
      }
      if (!ok) ++badS;
    }
    // root distance: reach = 0.999999 t |d| must not prune the sphere itself
    const float rp = rtg::round_up_f(fabs((double)r) * (1.0 + 0x1p-7) * (1.0 + 0x1p-20));
    const rtg::V3 p = rtg::vsub(o, c);
    const float p2 = fmaf(p.x, p.x, fmaf(p.y, p.y, p.z * p.z));
    const double tl = (double)tr * sqrt((double)q.den * 0.5) * (1.0 - 1e-6);
    if (rtg::beyond(p2, rp, (float)tl)) ++bad;
  }
  if (accepted) *accepted = acc;
  if (bad_screen) *bad_screen = badS;
  return bad;
}

// Cone masks (cone_masks, rtg_scene_pack.h) against the reference's own root
// test: random scenes; for random (h, i), an origin in h's origin ball
// (mostly on its boundary towards i), a direction d aimed at a point of
// sphere i's silhouette (grazing, in or slightly out), and a bundle direction
// U up to kConeHalf away from d; if i is not in mask (h, cone_cell(U)) the
// reference must not accept a root of sphere i.  Returns the violations;
// *tested counts the rays the reference accepts for sphere i.
extern "C" long hostsim_cone_mask_check(long scenes, unsigned n, long rays,
                                        unsigned long long seed, long* tested) {
  unsigned long long st = seed * 0x9E3779B97F4A7C15ull + 3;
  auto u01 = [&]() {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    return (double)(st >> 11) * (1.0 / 9007199254740992.0);
  };
  auto unit = [&](double* v) {
    double l;
    do {
      for (int k = 0; k < 3; ++k) v[k] = 2.0 * u01() - 1.0;
      l = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    } while (l < 1e-3 || l > 1.0);
    for (int k = 0; k < 3; ++k) v[k] /= l;
  };
  long bad = 0, cnt = 0;
  std::vector<rtg_sphere> sph(n);
  for (long sc = 0; sc < scenes; ++sc) {
    const double scale = pow(10.0, -1.5 + 3.0 * u01());
    for (unsigned i = 0; i < n; ++i) {
      memset(&sph[i], 0, sizeof(rtg_sphere));
      sph[i].pos.x = (float)((u01() - 0.5) * 24 * scale);
      sph[i].pos.y = (float)((u01() - 0.5) * 16 * scale);
      sph[i].pos.z = (float)((-6 - 34 * u01()) * scale);
      sph[i].radius = (float)((0.2 + 3 * u01()) * scale);
    }
    std::vector<unsigned> masks;
    rtg::cone_masks(sph.data(), n, &masks);
    for (long r = 0; r < rays; ++r) {
      const unsigned h = (unsigned)(u01() * n) % n, i = (unsigned)(u01() * n) % n;
      if (i == h) continue;
      const rtg_sphere& sh = sph[h];
      const rtg_sphere& si = sph[i];
      const double ch = fabs((double)sh.pos.x) + fabs((double)sh.pos.y) + fabs((double)sh.pos.z);
      const double g = rtg::guard_radius(sh);
      const double rho = g + 0.0101 + 0x1p-20 * (ch + g);
      // origin: on the origin ball's boundary, biased towards i
      double v[3];
      unit(v);
      const double ci[3] = {si.pos.x, si.pos.y, si.pos.z}, chv[3] = {sh.pos.x, sh.pos.y, sh.pos.z};
      double w[3] = {ci[0] - chv[0], ci[1] - chv[1], ci[2] - chv[2]};
      const double wl = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]) + 1e-300;
      const double bias = u01();
      for (int k = 0; k < 3; ++k) v[k] = bias * w[k] / wl + (1.0 - bias) * v[k];
      const double vl = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]) + 1e-300;
      const double orad = rho * (r % 4 == 0 ? u01() : 1.0 - 1e-9);
      double O[3];
      for (int k = 0; k < 3; ++k) O[k] = chv[k] + orad * v[k] / vl;
      // target on i's silhouette as seen from O, pushed out by up to 1e-3 r_i
      double a[3] = {ci[0] - O[0], ci[1] - O[1], ci[2] - O[2]};
      const double al = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]) + 1e-300;
      double p[3];
      unit(p);
      const double pd = (p[0] * a[0] + p[1] * a[1] + p[2] * a[2]) / al;
      for (int k = 0; k < 3; ++k) p[k] -= pd * a[k] / al;
      const double pl = sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]) + 1e-300;
      const double off = fabs((double)si.radius) * (1.0 + 1e-3 * (u01() - 0.3));
      double d[3];
      for (int k = 0; k < 3; ++k) d[k] = ci[k] + off * p[k] / pl - O[k];
      // bundle direction U: d rotated by up to kConeHalf
      const double dl = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]) + 1e-300;
      double q[3];
      unit(q);
      const double qd = (q[0] * d[0] + q[1] * d[1] + q[2] * d[2]) / dl;
      for (int k = 0; k < 3; ++k) q[k] -= qd * d[k] / dl;
      const double ql = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]) + 1e-300;
      const unsigned tier = (unsigned)(r & 1);
      const double ang = rtg::kConeHalf[tier] * (r % 3 == 0 ? u01() : 1.0 - 1e-6);
      double U[3];
      for (int k = 0; k < 3; ++k) U[k] = cos(ang) * d[k] / dl + sin(ang) * q[k] / ql;
      const int cell = rtg::cone_cell(rtg::v3((float)U[0], (float)U[1], (float)U[2]));
      const unsigned* mw = &masks[(((size_t)h * rtg::kConeTiers + tier) * rtg::kConeCells + cell) * 2];
      const double ds = 0.2 + 2.0 * u01();
      const rtg::RayQ qr = rtg::make_query(
          rtg::v3((float)O[0], (float)O[1], (float)O[2]),
          rtg::v3((float)(d[0] / dl * ds), (float)(d[1] / dl * ds), (float)(d[2] / dl * ds)));
      bool res;
      rtg::ray_sphere(qr, rtg::v3(si.pos.x, si.pos.y, si.pos.z), si.radius * si.radius, res);
      if (!res) continue;
      ++cnt;
      if (!(mw[i >> 5] & (1u << (i & 31)))) ++bad;
    }
  }
  if (tested) *tested = cnt;
  return bad;
}

// Sphere-list sizes of a scene (sphere_lists, rtg_scene_pack.h) under a
// record budget: out = {capsule records, overlap records, BVH nodes} (0, 0 when
// the scene gets no lists: over the budget or the build-cost threshold).
extern "C" void hostsim_list_records(const rtg_sphere* spheres, unsigned n,
                                     const rtg_light* lights, unsigned m,
                                     unsigned long long maxRecords, unsigned long long* out) {
  rtg::PackedScene ps;
  out[0] = out[1] = out[2] = 0;
  if (!rtg::build_bvh(spheres, n, &ps)) return;
  out[2] = ps.bvhNodes.size() / (rtg::kBvhWords * rtg::kBvhCopies);
  rtg::sphere_lists(spheres, n, lights, m, &ps, (size_t)maxRecords);
  if (ps.capOff.empty()) return;
  out[0] = ps.capRec.size() / rtg::kCapWords - rtg::kCapPad;  // without the padding records
  out[1] = ps.ovRec.size() / rtg::kListWords - rtg::kOvPad;
}

// `behind` (rtg_trace.h) never rejects a sphere the reference's root test
// accepts: adversarial rays from just outside a sphere, pointing away from
// it or grazing it, at scales 1e-3 .. 1e3, unit and unnormalised directions,
// against ray_sphere (raytracer.h:81-141's float operations).  Returns the
// violations; *rejected counts the spheres behind() rejected, *loose the
// accepted roots a margin-free version (x > 0, |p|^2 - r^2 > 0) would drop.
extern "C" long hostsim_behind_check(long trials, unsigned long long seed, long* rejected,
                                     long* loose) {
  unsigned long long st = seed;
  auto u01 = [&st]() {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    return (double)(st >> 11) * 0x1p-53;
  };
  long bad = 0;
  *rejected = 0;
  *loose = 0;
  for (long k = 0; k < trials; ++k) {
    const double scale = pow(10.0, -3.0 + 6.0 * u01());
    const double r = scale * (0.05 + u01());
    rtg::V3 c = rtg::v3((float)(scale * (u01() * 20 - 10)), (float)(scale * (u01() * 20 - 10)),
                        (float)(scale * (u01() * 20 - 10)));
    // a random unit normal n; the origin at distance r (1 + e) along n
    double nx = u01() * 2 - 1, ny = u01() * 2 - 1, nz = u01() * 2 - 1;
    const double nl = sqrt(nx * nx + ny * ny + nz * nz) + 1e-300;
    nx /= nl; ny /= nl; nz /= nl;
    const int kind = (int)(u01() * 4);
    const double e = kind == 0 ? pow(10.0, -9.0 + 8.0 * u01()) : kind == 1 ? u01() * 3.0
                   : pow(10.0, -7.0 + 7.0 * u01());
    const float rf = (float)r;
    rtg::V3 o = rtg::v3((float)(c.x + r * (1 + e) * nx), (float)(c.y + r * (1 + e) * ny),
                        (float)(c.z + r * (1 + e) * nz));
    // direction: away from the sphere with a tangential part (grazing when small)
    double tx = u01() * 2 - 1, ty = u01() * 2 - 1, tz = u01() * 2 - 1;
    const double tn = tx * nx + ty * ny + tz * nz;
    tx -= tn * nx; ty -= tn * ny; tz -= tn * nz;
    const double away = kind == 3 ? pow(10.0, -8.0 + 8.0 * u01()) : u01();
    double dx = nx * away + tx, dy = ny * away + ty, dz = nz * away + tz;
    const double dl = sqrt(dx * dx + dy * dy + dz * dz) + 1e-300;
    const double dscale = (u01() < 0.5) ? 1.0 : pow(10.0, -1.5 + 3.0 * u01());
    rtg::V3 d = rtg::v3((float)(dx / dl * dscale), (float)(dy / dl * dscale),
                        (float)(dz / dl * dscale));
    const rtg::RayQ q = rtg::make_query(o, d);
    const float r2 = rf * rf;
    const float rs = rtg::screen_r2(r2);
    const rtg::V3 p = rtg::vsub(q.o, c);
    const float x = fmaf(q.d.x, p.x, fmaf(q.d.y, p.y, q.d.z * p.z));
    const float cs = fmaf(p.x, p.x, fmaf(p.y, p.y, fmaf(p.z, p.z, -rs)));
    bool res;
    (void)rtg::ray_sphere(q, c, r2, res);
    if (rtg::behind(0.5f * q.den, x, cs, rs)) {
      ++*rejected;
      if (res) ++bad;
    } else if (res && x > 0.f && fmaf(p.x, p.x, fmaf(p.y, p.y, fmaf(p.z, p.z, -r2))) > 0.f) {
      ++*loose;  // outside and receding by the fused terms, yet a root is accepted
    }
  }
  return bad;
}

// no_root (rtg_trace.h) never skips a root the reference accepts: rays from
// on, just inside or just outside a sphere's surface (the shadow ray of a
// hit point on its own sphere), leaving it at any angle down to grazing, at
// scales 1e-3 .. 1e2 with unit and unnormalised directions.  Returns the
// violations; *skipped counts the tests no_root skipped, *accepted the roots
// the reference accepted (self-shadowing acne: the check has cases to miss).
extern "C" long hostsim_no_root_check(long trials, unsigned long long seed, long* skipped,
                                      long* accepted) {
  unsigned long long st = seed;
  auto u01 = [&st]() {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    return (double)(st >> 11) * 0x1p-53;
  };
  long bad = 0;
  *skipped = 0;
  *accepted = 0;
  for (long k = 0; k < trials; ++k) {
    const double scale = pow(10.0, -3.0 + 5.0 * u01());
    const double r = scale * (0.05 + u01());
    const rtg::V3 c = rtg::v3((float)(scale * (u01() * 20 - 10)), (float)(scale * (u01() * 20 - 10)),
                              (float)(scale * (u01() * 20 - 10)));
    double nx = u01() * 2 - 1, ny = u01() * 2 - 1, nz = u01() * 2 - 1;
    const double nl = sqrt(nx * nx + ny * ny + nz * nz) + 1e-300;
    nx /= nl; ny /= nl; nz /= nl;
    const double e = (u01() - 0.5) * pow(10.0, -8.0 + 5.0 * u01());  // on / inside / outside
    const rtg::V3 o = rtg::v3((float)(c.x + r * (1 + e) * nx), (float)(c.y + r * (1 + e) * ny),
                              (float)(c.z + r * (1 + e) * nz));
    double tx = u01() * 2 - 1, ty = u01() * 2 - 1, tz = u01() * 2 - 1;
    const double tn = tx * nx + ty * ny + tz * nz;
    tx -= tn * nx; ty -= tn * ny; tz -= tn * nz;
    const double tl = sqrt(tx * tx + ty * ty + tz * tz) + 1e-300;
    const double cosv = (u01() < 0.5) ? pow(10.0, -7.0 + 7.0 * u01()) : u01();  // to grazing
    const double sinv = sqrt(1 - cosv * cosv);
    const double dscale = (u01() < 0.5) ? 1.0 : pow(10.0, -1.0 + 2.0 * u01());
    const rtg::V3 d = rtg::v3((float)((nx * cosv + tx / tl * sinv) * dscale),
                              (float)((ny * cosv + ty / tl * sinv) * dscale),
                              (float)((nz * cosv + tz / tl * sinv) * dscale));
    const rtg::RayQ q = rtg::make_query(o, d);
    const float r2 = (float)r * (float)r;
    const rtg::V3 disp = rtg::vsub(q.o, c);
    const float b = 2.0f * rtg::vdot(q.d, disp);
    const float cc = rtg::vdot(disp, disp) - r2;
    bool res;
    (void)rtg::ray_sphere(q, c, r2, res);
    if (res) ++*accepted;
    if (rtg::no_root(q, b, cc)) {
      ++*skipped;
      if (res) ++bad;
    }
  }
  return bad;
}

// cap_screen_r2 (rtg_trace.h, the device's screen radius^2 of a 16-byte
// capsule record) never falls below the host's screen_r2, which pass1_rad's
// conservativeness argument assumes: every non-negative binary32 value r2 at
// a stride (all subnormals and the values around every power of two below
// it included), plus inf and NaN.  Returns the violations; *checked counts
// the values tested.
extern "C" long hostsim_cap_screen_check(unsigned stride, long* checked) {
  long bad = 0;
  *checked = 0;
  auto one = [&](uint32_t bits) {
    float r2;
    memcpy(&r2, &bits, 4);
    const float a = rtg::cap_screen_r2(r2), b = rtg::screen_r2(r2);
    ++*checked;
    if (r2 != r2) {
      if (a == a) ++bad;
    } else if (!(a >= b)) {
      ++bad;
    }
  };
  for (uint64_t u = 0; u <= 0x7FC00000u; u += stride) one((uint32_t)u);
  for (uint32_t e = 0; e < 256; ++e)  // both sides of every binade boundary
    for (uint32_t m = 0; m < 64; ++m) {
      one((e << 23) + m);
      if (e > 0) one((e << 23) - 1 - m);
    }
  for (uint32_t m = 0; m < 0x800000u; m += 7) one(m);  // subnormals
  return bad;
}

// The capsule lists' hit-point cells (cap_cell, cell_ball, cell_keep,
// cell_behind in rtg_scene_pack.h): a sphere left out of the list of cell c
// of (light l, sphere h) never blocks a shadow ray cast from a hit point P
// that the kernel classifies into cell c (guard and shell tests passed,
// incidence > 0), by the reference's own test.  Random scenes at scales
// 1e-2..1e2; half of the spheres are placed just outside (or on) a random
// cell capsule of sphere 0 and light 0, and the points P are drawn in that
// cell near the surface, at the shell's inner radius, near the cell's edges
// (components near 0, two components of near equal size) and toward the
// placed spheres.  Returns the violations; *tested counts the (P, sphere)
// pairs tested.
extern "C" long hostsim_cell_list_check(long scenes, unsigned n, long points,
                                        unsigned long long seed, long* tested) {
  unsigned long long st = seed * 0x9E3779B97F4A7C15ull + 11;
  auto u01 = [&]() {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    return (double)(st >> 11) * (1.0 / 9007199254740992.0);
  };
  long bad = 0, cnt = 0;
  std::vector<rtg_sphere> sph(n);
  rtg_light lg[2];
  for (long sc = 0; sc < scenes; ++sc) {
    const double scale = pow(10.0, -2.0 + 4.0 * u01());
    for (unsigned i = 0; i < n; ++i) {
      memset(&sph[i], 0, sizeof(rtg_sphere));
      sph[i].pos.x = (float)((u01() - 0.5) * 24 * scale);
      sph[i].pos.y = (float)((u01() - 0.5) * 16 * scale);
      sph[i].pos.z = (float)((-6 - 34 * u01()) * scale);
      sph[i].radius = (float)((0.3 + 3 * u01()) * scale);
    }
    for (int l = 0; l < 2; ++l) {
      lg[l].pos.x = (float)((u01() - 0.5) * 120 * scale);
      lg[l].pos.y = (float)((10 + 70 * u01()) * scale);
      lg[l].pos.z = (float)((u01() - 0.5) * 130 * scale);
    }
    const double L0[3] = {lg[0].pos.x, lg[0].pos.y, lg[0].pos.z};
    const unsigned c0 = (unsigned)(u01() * 24) % 24;
    double b0[3], rho0;
    rtg::cell_ball(sph[0], c0, b0, &rho0);
    for (unsigned i = n / 2; i < n; ++i) {  // just outside cell c0's capsule
      const double t = (i & 1) ? u01() : 0.05 * u01() * u01();
      double p[3], ab[3];
      for (int k = 0; k < 3; ++k) { ab[k] = L0[k] - b0[k]; p[k] = b0[k] + t * ab[k]; }
      double v[3] = {u01() - 0.5, u01() - 0.5, u01() - 0.5};
      const double ab2 = ab[0] * ab[0] + ab[1] * ab[1] + ab[2] * ab[2];
      const double pr = (v[0] * ab[0] + v[1] * ab[1] + v[2] * ab[2]) / ab2;
      for (int k = 0; k < 3; ++k) v[k] -= pr * ab[k];
      const double vl = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
      const double ri = sph[i].radius;
      const double dist = (rho0 + ri) * (1.0 + (u01() < 0.3 ? -0.1 : 1.0) * pow(10.0, -4.0 + 2.5 * u01()));
      sph[i].pos.x = (float)(p[0] + dist * v[0] / vl);
      sph[i].pos.y = (float)(p[1] + dist * v[1] / vl);
      sph[i].pos.z = (float)(p[2] + dist * v[2] / vl);
    }
    for (int l = 0; l < 2; ++l) {
      const double L[3] = {lg[l].pos.x, lg[l].pos.y, lg[l].pos.z};
      for (unsigned h = 0; h < (l == 0 ? 4u : 2u); ++h) {
        const rtg_sphere& sh = sph[h];
        const float G2 = rtg::guard_r2(sh);
        const float r2h = sh.radius * sh.radius;
        const double rh = fabs((double)sh.radius);
        for (unsigned cell = 0; cell < rtg::kCapCubeCells; ++cell) {
          if (h == 0 && l == 0 && cell != c0 && u01() < 0.7) continue;
          const bool shared = rtg::cell_behind(sh, cell, L);
          double b[3], rho;
          rtg::cell_ball(sh, cell, b, &rho);
          const unsigned a = cell >> 3, pa = a == 0 ? 1 : 0, qa = a == 2 ? 1 : 2;
          const double sa = (cell & 4) ? -1.0 : 1.0, sp = (cell & 2) ? -1.0 : 1.0,
                       sq = (cell & 1) ? -1.0 : 1.0;
          for (unsigned i = 0; i < n; ++i) {
            if (rtg::capsule_keep(sph.data(), h, i, L) &&
                (shared || rtg::cell_keep(sph.data(), h, i, L, b, rho)))
              continue;  // in the cell's list
            for (long k = 0; k < points; ++k) {
              // a direction in the cell: gnomonic coordinates in [0, 1]^2,
              // often at an edge (0 or 1), or toward sphere i
              double pp = u01(), qq = u01();
              const int edge = (int)(k % 5);
              if (edge == 1) pp = pow(10.0, -9.0 * u01());
              if (edge == 2) qq = 1.0 - pow(10.0, -9.0 * u01());
              if (edge == 3) { pp = 1.0 - pow(10.0, -8.0 * u01()); qq = pow(10.0, -8.0 * u01()); }
              double u[3];
              u[a] = sa; u[pa] = sp * pp; u[qa] = sq * qq;
              if (edge == 4) {  // toward sphere i (clamped into the cell)
                double cv[3] = {(double)sph[i].pos.x - sh.pos.x, (double)sph[i].pos.y - sh.pos.y,
                                (double)sph[i].pos.z - sh.pos.z};
                const double ca = fabs(cv[a]) + 1e-300;
                double p2 = sp * cv[pa] / ca, q2 = sq * cv[qa] / ca;
                p2 = p2 < 0 ? 0 : (p2 > 1 ? 1 : p2);
                q2 = q2 < 0 ? 0 : (q2 > 1 ? 1 : q2);
                u[pa] = sp * p2; u[qa] = sq * q2;
              }
              const double ul = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
              const double rad = (k % 7 == 0) ? rh * (1.0 - 0x1p-8) * (1.0 + (u01() - 0.5) * 1e-6)
                                               : rh * (1.0 + (u01() - 0.7) * 2e-3);
              const rtg::V3 P = rtg::v3((float)(sh.pos.x + rad * u[0] / ul),
                                        (float)(sh.pos.y + rad * u[1] / ul),
                                        (float)(sh.pos.z + rad * u[2] / ul));
              const rtg::V3 e = rtg::vsub(P, rtg::v3(sh.pos.x, sh.pos.y, sh.pos.z));
              if (!(rtg::vdot(e, e) <= G2)) continue;
              if (rtg::cap_cell(e, r2h) != cell) continue;  // another cell's list serves it
              const rtg::V3 Lp = rtg::v3(lg[l].pos.x, lg[l].pos.y, lg[l].pos.z);
              const rtg::V3 dist = rtg::vsub(Lp, P);
              const float gap = rtg::vdot(dist, dist);
              const rtg::V3 D = rtg::vsmul(1.f / sqrtf(gap), dist);
              const rtg::V3 N = rtg::vnorm(e);
              if (!(rtg::vdot(N, D) > 0.f)) continue;
              const rtg::RayQ q = rtg::make_query(P, D);
              ++cnt;
              bool res;
              const float t = rtg::ray_sphere(q, rtg::v3(sph[i].pos.x, sph[i].pos.y, sph[i].pos.z),
                                              sph[i].radius * sph[i].radius, res);
              if (res && t < 1000.f) {
                const rtg::V3 tv = rtg::vsmul(t, D);
                if (rtg::vdot(tv, tv) < gap) ++bad;
              }
            }
          }
        }
      }
    }
  }
  if (tested) *tested = cnt;
  return bad;
}
extern "C" void hostsim_cell_ball_slack(double s) { rtg::g_cellBallSlack = s; }
