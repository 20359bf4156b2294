// rtg_host.cpp — host-side pieces of librtg.so that carry reference
// semantics outside the kernel: scene construction (main.cpp:104-168 +
// SURVEY.md §8d generator), the PPM writer (main.cpp:43-91), the colour max
// (algebra.h:68-91), row sharding and error reporting.
//
// Compiled with -ffp-contract=off like the kernel: material construction and
// generator arithmetic must round exactly as the reference's host does.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>

#include "rtg.h"
#include "rtg_internal.h"

static_assert(sizeof(rtg_vec) == 12, "Vec is 12 B (vec.h:27-29)");
static_assert(sizeof(rtg_material) == 32, "Material is 32 B (material.h:8-14)");
static_assert(sizeof(rtg_sphere) == 48, "Sphere is 48 B (sphere.h:9-14)");
static_assert(offsetof(rtg_sphere, radius) == 12, "Sphere.radius @12");
static_assert(offsetof(rtg_sphere, material) == 16, "Sphere.material @16");
static_assert(offsetof(rtg_material, opacity) == 24, "Material.opacity @24");
static_assert(offsetof(rtg_material, refractiveIndex) == 28, "Material.n @28");
static_assert(sizeof(rtg_light) == 24, "Light is 24 B (raytracer.h:20-25)");

namespace {
thread_local std::string g_last_error;
}

void rtg_set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
}
void rtg_clear_error() { g_last_error.clear(); }

extern "C" {

const char* rtg_last_error(void) { return g_last_error.c_str(); }
int rtg_abi_version(void) { return RTG_ABI_VERSION; }

// raytracer.h:53-74: setMatOpacity, setMatteGlossBalance, setMatRefractivityIndex.
void rtg_make_material(float opacity, float glossFactor, const rtg_vec* matte,
                       const rtg_vec* gloss, float refractiveIndex, rtg_material* out) {
  rtg_material m;
  memset(&m, 0, sizeof m);
  m.opacity = opacity;
  const float km = (float)(1.0 - glossFactor);  // vsmul(newMatte, (1.0 - glossFactor), *matte)
  m.matteColour.x = km * matte->x;
  m.matteColour.y = km * matte->y;
  m.matteColour.z = km * matte->z;
  const float kg = glossFactor;                  // vsmul(newGloss, glossFactor, *gloss)
  m.glossColour.x = kg * gloss->x;
  m.glossColour.y = kg * gloss->y;
  m.glossColour.z = kg * gloss->z;
  m.refractiveIndex = refractiveIndex;
  *out = m;
}

int rtg_scene_generate(unsigned long long seed, unsigned sphNum, unsigned lgtNum,
                       rtg_sphere* spheres, rtg_light* lights) {
  rtg_clear_error();
  if ((sphNum && !spheres) || (lgtNum && !lights)) {
    rtg_set_error("rtg_scene_generate: null output array");
    return RTG_ERR_INVALID;
  }
  // main.cpp:113-145
  const rtg_vec red = {0.8f, 1.f, 0.7f}, green = {0.4f, 0.5f, 0.7f};
  const rtg_vec col1 = {0.01f, 0.8f, 0.01f};
  rtg_material M[3];
  rtg_make_material(0.8f, 0.2f, &green, &red, 1.5500f, &M[0]);
  rtg_make_material(0.3f, 0.95f, &green, &red, 1.5500f, &M[1]);
  rtg_make_material(0.6f, 0.0f, &col1, &col1, 1.5500f, &M[2]);
  // splitmix64, u01 = (float)(next >> 40) * 2^-24, U(a,b) = a + (b-a)*u01.
  uint64_t state = seed;
  auto next = [&state]() {
    uint64_t z = (state += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
  };
  auto U = [&next](float a, float b) {
    const float u01 = (float)(next() >> 40) * 0x1p-24f;
    return a + (b - a) * u01;
  };
  static const float fixedSph[3][4] = {{-9.f, 0.f, -13.f, 5.f},   // main.cpp:151-153
                                       {-4.f, 1.5f, -5.f, 2.f},   // :154-156
                                       {1.f, -1.f, -7.f, 3.f}};   // :157-159
  for (unsigned i = 0; i < sphNum; ++i) {
    rtg_sphere s;
    memset(&s, 0, sizeof s);
    s.material = M[i % 3];
    if (i < 3) {
      s.pos.x = fixedSph[i][0]; s.pos.y = fixedSph[i][1]; s.pos.z = fixedSph[i][2];
      s.radius = fixedSph[i][3];
    } else {
      s.pos.x = U(-12.f, 12.f);
      s.pos.y = U(-8.f, 8.f);
      s.pos.z = U(-40.f, -6.f);
      s.radius = U(0.5f, 3.f);
    }
    spheres[i] = s;
  }
  static const float fixedLgt[2][3] = {{-45.f, 10.f, 85.f}, {20.f, 60.f, -5.f}};  // :165-168
  for (unsigned l = 0; l < lgtNum; ++l) {
    rtg_light L;
    if (l < 2) {
      L.pos.x = fixedLgt[l][0]; L.pos.y = fixedLgt[l][1]; L.pos.z = fixedLgt[l][2];
    } else {
      L.pos.x = U(-60.f, 60.f);
      L.pos.y = U(10.f, 80.f);
      L.pos.z = U(-40.f, 90.f);
    }
    L.col.x = 0.5f; L.col.y = 0.5f; L.col.z = 0.5f;  // lowerWhite, main.cpp:117
    lights[l] = L;
  }
  return RTG_OK;
}

// algebra.h:68-91 — NaN-skipping max over every channel; 0 -> 1.
float rtg_max_colour(const rtg_vec* pixels, size_t n) {
  float mx = 0.f;
  for (size_t i = 0; i < n; ++i) {
    if (pixels[i].x > mx) mx = pixels[i].x;
    if (pixels[i].y > mx) mx = pixels[i].y;
    if (pixels[i].z > mx) mx = pixels[i].z;
  }
  if (mx == 0.f) mx = 1.f;
  return mx;
}

void rtg_ppm_bytes(const rtg_vec* pixels, size_t n, float maxColourVal, unsigned char* out) {
  const float* c = (const float*)pixels;
  for (size_t i = 0; i < n * 3; ++i) out[i] = rtg::ppm_byte(c[i], maxColourVal);
}

// main.cpp:43-91.  The reference prints and returns on failure; here the
// failure is also returned.
int rtg_save_ppm(const rtg_vec* pixels, const char* filename, int width, int height,
                 float maxColourVal) {
  rtg_clear_error();
  if (width == 0 || height == 0) {
    fprintf(stderr, "Can't save an empty image\n");
    rtg_set_error("Can't save an empty image");
    return RTG_ERR_INVALID;
  }
  FILE* f = fopen(filename, "wb");
  if (!f) {
    fprintf(stderr, "Can't open output file\n");
    rtg_set_error("Can't open output file %s", filename);
    return RTG_ERR_IO;
  }
  fprintf(f, "P6\n%d %d\n255\n", width, height);
  const size_t npx = (size_t)width * (size_t)height;
  const size_t chunk = 1 << 16;
  unsigned char buf[3 * (1 << 16)];
  for (size_t i = 0; i < npx; i += chunk) {
    const size_t k = (npx - i < chunk) ? npx - i : chunk;
    rtg_ppm_bytes(pixels + i, k, maxColourVal, buf);
    if (fwrite(buf, 1, 3 * k, f) != 3 * k) {
      fclose(f);
      rtg_set_error("short write to %s", filename);
      return RTG_ERR_IO;
    }
  }
  if (fclose(f) != 0) {
    rtg_set_error("close failed for %s", filename);
    return RTG_ERR_IO;
  }
  return RTG_OK;
}

int rtg_shard_rows(unsigned height, unsigned rowBlock, unsigned shard, unsigned nShards,
                   unsigned* rows) {
  rtg_clear_error();
  if (!rows || rowBlock == 0 || nShards == 0 || shard >= nShards) {
    rtg_set_error("rtg_shard_rows: invalid arguments");
    return RTG_ERR_INVALID;
  }
  *rows = rtg::shard_row_count(height, rowBlock, shard, nShards);
  return RTG_OK;
}

unsigned rtg_shard_global_row(unsigned localRow, unsigned rowBlock, unsigned shard,
                              unsigned nShards) {
  return rtg::shard_global_row(localRow, rowBlock, shard, nShards);
}

}  // extern "C"
