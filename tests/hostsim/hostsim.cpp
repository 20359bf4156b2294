// tests/hostsim/hostsim.cpp — TEST-ONLY host build of the GPU kernel's
// traversal (raytracer-gamma_amd/csrc/rtg_trace.h) over the same scene
// preparation (rtg_scene_pack.h).  It lets the CPU test suite check the
// kernel's restructured algorithm (frame stack, stale-register handling,
// leaf doubling, early-exit shadow rays) bit for bit against the oracle
// without a GPU.  It is not part of librtg.so and no product path calls it.
#include <vector>

#include "rtg.h"
#include "rtg_internal.h"
#include "rtg_scene_pack.h"
#include "rtg_trace.h"

void rtg_set_error(const char*, ...) {}
void rtg_clear_error() {}

namespace {
struct HostScene {
  const float* geom;
  const float* crad2;
  const float* mats;
  const float* lights;
  unsigned n, m, n4;
  bool all(bool b) const { return b; }
  rtg::V3 sphere(unsigned i, float& r2) const {
    const float* g = geom + 4 * i;
    r2 = g[3];
    return rtg::v3(g[0], g[1], g[2]);
  }
  rtg::V3 sphere_lane(unsigned i, float& r2) const { return sphere(i, r2); }
  void probe_begin(int) const {}
  struct Frames {
    rtg::FrameC* f;
    rtg::FrameC& operator()(int lv) const { return f[lv]; }
  };
  mutable rtg::FrameC fr[16];
  Frames frames() const { return Frames{fr}; }
  void probe_end(int) const {}
  void sphere4(unsigned i, rtg::V3* c, float* r2) const {
    for (int k = 0; k < 4; ++k) c[k] = sphere(i + k, r2[k]);
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
  void light(unsigned l, rtg::V3& pos, rtg::V3& col) const {
    const float* p = lights + 6 * l;
    pos = rtg::v3(p[0], p[1], p[2]);
    col = rtg::v3(p[3], p[4], p[5]);
  }
};

int g_variant = 0;

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
      case 14: {  // sample-parallel kernel: samples traced one by one, summed in order
        p = rtg::v3(0.f, 0.f, 0.f);
        for (int s = 0; s < cam.nAA * cam.nAA; ++s) {
          float rx, ry;
          const rtg::V3 d = rtg::sample_dir(cam, x, y, s / cam.nAA, s % cam.nAA, rx, ry);
          rtg::V3 c = rtg::trace_sample<S, 2>(sc, d, sc.frames());
          c = rtg::vsmul(cam.inv, c);
          p = rtg::vadd(p, c);
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
          sel = 0;
          for (unsigned k = 0; k < sc.n; ++k) {
            float r2;
            const rtg::V3 c = sc.sphere(k, r2);
            if (rtg::primary_sphere_possible(c, sqrtf(r2), x0, x1, y0, y1, cam.zoom))
              sel |= 1ull << k;
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

extern "C" int hostsim_render_rows(const rtg_sphere* spheres, unsigned n,
                                   const rtg_light* lights, unsigned m, unsigned W,
                                   unsigned H, float zoom, float aa, int S,
                                   const unsigned* rows, unsigned nrows, float* out) {
  rtg::PackedScene ps;
  rtg::pack_scene(spheres, n, lights, m, &ps);
  rtg::Camera cam;
  if (rtg::make_camera(W, H, zoom, aa, &cam)) return -1;
  HostScene sc{ps.geom.data(), ps.crad2.data(), ps.mats.data(), ps.lights.data(), n, m, ps.n4};
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

// Conservativeness of the primary-ray cull (primary_sphere_possible): over
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
    for (unsigned k = 0; k < n; ++k) {
      float r2;
      const rtg::V3 c = sc.sphere(k, r2);
      if (rtg::primary_sphere_possible(c, sqrtf(r2), x0, x1, y0, y1, cam.zoom)) continue;
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
