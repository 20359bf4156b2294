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

#include <string.h>

#include <vector>

#include "rtg.h"
#include "rtg_internal.h"
#include "rtg_trace.h"

namespace rtg {

// Device image of a scene.  geom: n x {x, y, z, r*r} followed by NaN padding
// records up to n4 + 4 (n4 = n rounded up to 4); crad2: n x (r+1e-6)^2, then
// n x the primary-ray c term |0 - c|^2 - r^2 (same float operations and order
// as the query's vdot(disp, disp) - r2 with disp = 0 - c, exact negation);
// mats: (n+1) x {matte.xyz, gloss.xyz, opacity, n} with [n] = background
// {0,0,0, 0,0,0, 0, 1.0} (raytracer.h:694-697; opacity 0);
// lights: m x {pos.xyz, col.xyz}.  Arrays are never empty (padded to 1).
struct PackedScene {
  std::vector<float> geom, crad2, mats, lights;
  unsigned n = 0, m = 0;
  unsigned n4 = 0;  // n rounded up to a multiple of 4; geom holds n4 + 4 records
};

inline void pack_scene(const rtg_sphere* spheres, unsigned n, const rtg_light* lights,
                       unsigned m, PackedScene* ps) {
  ps->n = n;
  ps->m = m;
  ps->n4 = (n + 3u) & ~3u;
  // Padding records are NaN spheres: their radicand is NaN, never >= 0.
  ps->geom.assign((size_t)(ps->n4 + 4) * 4, __builtin_nanf(""));
  ps->crad2.assign(n ? 2 * (size_t)n : 1, 0.f);
  ps->mats.assign((size_t)(n + 1) * 8, 0.f);
  ps->lights.assign((size_t)(m ? m : 1) * 6, 0.f);
  for (unsigned i = 0; i < n; ++i) {
    const rtg_sphere& s = spheres[i];
    float* g = &ps->geom[(size_t)i * 4];
    g[0] = s.pos.x; g[1] = s.pos.y; g[2] = s.pos.z;
    g[3] = s.radius * s.radius;
    const float rc = s.radius + 1.0e-6f;
    ps->crad2[i] = rc * rc;
    const float dx = 0.f - s.pos.x, dy = 0.f - s.pos.y, dz = 0.f - s.pos.z;
    ps->crad2[n + i] = (((dx * dx) + (dy * dy)) + (dz * dz)) - g[3];
    float* mt = &ps->mats[(size_t)i * 8];
    mt[0] = s.material.matteColour.x; mt[1] = s.material.matteColour.y;
    mt[2] = s.material.matteColour.z; mt[3] = s.material.glossColour.x;
    mt[4] = s.material.glossColour.y; mt[5] = s.material.glossColour.z;
    mt[6] = s.material.opacity; mt[7] = s.material.refractiveIndex;
  }
  ps->mats[(size_t)n * 8 + 7] = 1.00f;
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
