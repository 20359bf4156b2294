// oracle/ref_harness.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// Drives the reference's own CPU raytracer (raytracer.h, compiled in place from
// /root/reference/raytracer_gamma via -I, never copied) so that the C
// restatement in oracle/rtg_oracle.c and the HIP kernel can be pinned against
// the real thing.  The reference ships its CPU per-pixel loop only as a
// commented-out block (main.cpp:383-453); this file restates that loop as a
// row-range driver and exposes it over a C ABI for ctypes.
//
// Built by oracle/build_ref.sh into oracle/_ref/librtgref_S<S>.so, one library
// per RTSTACK_MAXSIZE (S = depth + 1, raytraceStack.h:10).
//
// Deterministic recipe: clang++ -O2 -ffp-contract=off
// -ftrivial-auto-var-init=zero -DRSIZE_MAX=0x7FFFFFFF.  The zero auto-init
// makes the uninitialised bgMaterial.opacity read at raytracer.h:694-697
// deterministic (= 0), matching the explicit zero used by the harness below
// for the primary-ray background material (main.cpp:423-426).
// For S != 6 the build passes -DRTG_STACK_HEADER=<patched copy>; its include
// guard (_RAYTRACE_STACK_H) then makes raytracer.h's own include of
// raytraceStack.h a no-op.  For S == 6 nothing is substituted.
#ifdef RTG_STACK_HEADER
#include RTG_STACK_HEADER
#endif
#include <raytracer.h>

#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

namespace {

// One pixel of the CPU path, main.cpp:411-452 (commented-out block).
void shade_pixel(struct Sphere* spheres, unsigned sphNum, struct Light* lights,
                 unsigned lgtNum, unsigned kScreenWidth, unsigned kScreenHeight,
                 float zoomFactor, float aliasFactor, unsigned gid, float* dst) {
  const float kImageWorldWidth = 16.f;                       // main.cpp:384
  const float kImageWorldHeight = 12.f;                      // main.cpp:385
  const float kRayXStep = kImageWorldWidth / ((float)kScreenWidth);   // :388
  const float kRayYStep = kImageWorldHeight / ((float)kScreenHeight); // :389
  const float aspectRatio = kImageWorldWidth / kImageWorldHeight;     // :390
  const float kAliasFactorStepInv = kRayXStep / aliasFactor;          // :398
  const float kSamplesTot = aliasFactor * aliasFactor;                // :400
  const float kSamplesTotinv = 1.f / kSamplesTot;                     // :402

  const float kPxWorldX =
      ((((float)(gid % kScreenWidth) - (kScreenWidth * 0.5f))) * kRayXStep);  // :411
  const float kPxWorldY =
      ((kScreenHeight * 0.5f) - ((float)(gid / kScreenWidth))) * kRayYStep;  // :413

  struct Ray ray;
  vinit(ray.origin, 0.f, 0.f, 0.f);
  vinit(ray.intensity, 1.f, 1.f, 1.f);                       // :417
  Vec pixelCol = {0.f, 0.f, 0.f};                            // :420

  struct Material bgMaterial;                                // :423-426
  std::memset(&bgMaterial, 0, sizeof bgMaterial);            // opacity := 0 (UB in ref)
  Vec black;
  vinit(black, 0.f, 0.f, 0.f);
  setMatteGlossBalance(&bgMaterial, 0.f, &black, &black);
  setMatRefractivityIndex(&bgMaterial, 1.00f);

  for (int i = 0; i < aliasFactor; ++i) {                    // :429
    for (int j = 0; j < aliasFactor; ++j) {                  // :430
      float x = (kPxWorldX + (float)(((float)j) * kAliasFactorStepInv)) * aspectRatio;
      float y = (kPxWorldY + (float)(((float)i) * kAliasFactorStepInv));
      vinit(ray.dir, x, y, zoomFactor);
      vnorm(ray.dir);                                        // :436
      Vec currentSampleCol =
          rayTrace(spheres, sphNum, lights, lgtNum, ray, bgMaterial, 0);  // :439
      vsmul(currentSampleCol, kSamplesTotinv, currentSampleCol);        // :442
      vadd(pixelCol, pixelCol, currentSampleCol);                       // :445
    }
  }
  dst[0] = pixelCol.x;                                       // :450-452
  dst[1] = pixelCol.y;
  dst[2] = pixelCol.z;
}

}  // namespace

extern "C" {

int ref_stack_size(void) { return RTSTACK_MAXSIZE; }

int ref_sizeof(int which) {
  switch (which) {
    case 0: return (int)sizeof(Vec);
    case 1: return (int)sizeof(struct Ray);
    case 2: return (int)sizeof(struct Material);
    case 3: return (int)sizeof(struct Sphere);
    case 4: return (int)sizeof(struct Light);
    case 5: return (int)sizeof(struct Intersection);
    default: return -1;
  }
}

// Material built with the reference's own setters, in main.cpp:126-145 order.
void ref_make_material(float opacity, float glossFactor, const float* matte,
                       const float* gloss, float refIndex, void* out) {
  struct Material m;
  std::memset(&m, 0, sizeof m);
  Vec vm, vg;
  vinit(vm, matte[0], matte[1], matte[2]);
  vinit(vg, gloss[0], gloss[1], gloss[2]);
  setMatOpacity(&m, opacity);
  setMatteGlossBalance(&m, glossFactor, &vm, &vg);
  setMatRefractivityIndex(&m, refIndex);
  std::memcpy(out, &m, sizeof m);
}

// Render the listed rows (row-major, rows[k] in [0,H)) into out[k*W*3 ..].
void ref_render_rows(const void* spheres, unsigned sphNum, const void* lights,
                     unsigned lgtNum, unsigned W, unsigned H, float zoom,
                     float aliasFactor, const unsigned* rows, unsigned nrows,
                     float* out, int nthreads) {
  std::vector<struct Sphere> sph(sphNum);
  std::vector<struct Light> lgt(lgtNum);
  if (sphNum) std::memcpy(sph.data(), spheres, sphNum * sizeof(struct Sphere));
  if (lgtNum) std::memcpy(lgt.data(), lights, lgtNum * sizeof(struct Light));
  std::atomic<unsigned> next(0);
  auto worker = [&]() {
    for (;;) {
      unsigned k = next.fetch_add(1);
      if (k >= nrows) break;
      unsigned y = rows[k];
      for (unsigned x = 0; x < W; ++x)
        shade_pixel(sph.data(), sphNum, lgt.data(), lgtNum, W, H, zoom, aliasFactor,
                    y * W + x, out + ((size_t)k * W + x) * 3);
    }
  };
  if (nthreads <= 1) {
    worker();
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < nthreads; ++t) pool.emplace_back(worker);
    for (auto& t : pool) t.join();
  }
}

// Render the listed pixels (gid = y * W + x, each < W * H) into out[k*3 ..]:
// the sampled-pixel fixtures of configs too slow to render whole (C5).
void ref_render_pixels(const void* spheres, unsigned sphNum, const void* lights,
                       unsigned lgtNum, unsigned W, unsigned H, float zoom,
                       float aliasFactor, const unsigned* gids, unsigned npx,
                       float* out, int nthreads) {
  std::vector<struct Sphere> sph(sphNum);
  std::vector<struct Light> lgt(lgtNum);
  if (sphNum) std::memcpy(sph.data(), spheres, sphNum * sizeof(struct Sphere));
  if (lgtNum) std::memcpy(lgt.data(), lights, lgtNum * sizeof(struct Light));
  std::atomic<unsigned> next(0);
  auto worker = [&]() {
    for (;;) {
      const unsigned k0 = next.fetch_add(64);  // 64 pixels per grab
      if (k0 >= npx) break;
      const unsigned k1 = k0 + 64 < npx ? k0 + 64 : npx;
      for (unsigned k = k0; k < k1; ++k)
        shade_pixel(sph.data(), sphNum, lgt.data(), lgtNum, W, H, zoom, aliasFactor, gids[k],
                    out + (size_t)k * 3);
    }
  };
  if (nthreads <= 1) {
    worker();
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < nthreads; ++t) pool.emplace_back(worker);
    for (auto& t : pool) t.join();
  }
}

// algebra.h:68-91, called directly.
float ref_max_colour(const float* fb, unsigned long long npx) {
  return maxColourValuePixelBuffer((const Vec*)fb, (size_t)npx);
}

}  // extern "C"
