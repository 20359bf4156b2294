// rtg_scene_file.cpp — scene files for the host: the
// reference hard-codes its scene in main.cpp:104-168; this text format lets a
// host load spheres, lights and materials instead.
//
//   # comment
//   material NAME opacity glossFactor mr mg mb gr gg gb refractiveIndex
//       -> setMatOpacity + setMatteGlossBalance + setMatRefractivityIndex
//          (raytracer.h:53-74, rtg_make_material), as main.cpp:126-145 does
//   sphere x y z radius NAME          sphere with a named material
//   sphere_raw x y z radius mr mg mb gr gg gb opacity n
//                                     material.h fields as stored (exact)
//   light x y z r g b                 raytracer.h:20-25
//
// Numbers are parsed with strtof (correctly rounded), and rtg_scene_save
// writes %.9g, so save -> load reproduces every float bit for bit.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <string>
#include <vector>

#include "rtg.h"
#include "rtg_internal.h"

namespace {

bool parse_floats(char** save, float* out, int n) {
  for (int k = 0; k < n; ++k) {
    const char* tok = strtok_r(nullptr, " \t\r\n", save);
    if (!tok) return false;
    char* end;
    out[k] = strtof(tok, &end);
    if (*end) return false;
  }
  return true;
}

}  // namespace

extern "C" {

int rtg_scene_load(const char* path, rtg_sphere* spheres, unsigned sphCap, unsigned* sphNum,
                   rtg_light* lights, unsigned lgtCap, unsigned* lgtNum) {
  rtg_clear_error();
  if (!path || !sphNum || !lgtNum || (sphCap && !spheres) || (lgtCap && !lights)) {
    rtg_set_error("rtg_scene_load: invalid arguments");
    return RTG_ERR_INVALID;
  }
  FILE* f = fopen(path, "r");
  if (!f) {
    rtg_set_error("rtg_scene_load: cannot open %s", path);
    return RTG_ERR_IO;
  }
  std::map<std::string, rtg_material> mats;
  unsigned ns = 0, nl = 0, line = 0;
  char buf[4096];
  int rc = RTG_OK;
  while (rc == RTG_OK && fgets(buf, sizeof buf, f)) {
    ++line;
    if (!strchr(buf, '\n') && !feof(f)) {
      rtg_set_error("%s:%u: line too long", path, line);
      rc = RTG_ERR_INVALID;
      break;
    }
    char* save = nullptr;
    const char* kw = strtok_r(buf, " \t\r\n", &save);
    if (!kw || kw[0] == '#') continue;
    if (!strcmp(kw, "material")) {
      const char* name = strtok_r(nullptr, " \t\r\n", &save);
      float v[9];
      if (!name || !parse_floats(&save, v, 9) || strtok_r(nullptr, " \t\r\n", &save)) {
        rtg_set_error("%s:%u: expected: material NAME opacity glossFactor mr mg mb gr gg gb n",
                      path, line);
        rc = RTG_ERR_INVALID;
        break;
      }
      const rtg_vec matte = {v[2], v[3], v[4]}, gloss = {v[5], v[6], v[7]};
      rtg_material m;
      rtg_make_material(v[0], v[1], &matte, &gloss, v[8], &m);
      mats[name] = m;
    } else if (!strcmp(kw, "sphere") || !strcmp(kw, "sphere_raw")) {
      const bool raw = kw[6] == '_';
      float v[12];
      rtg_sphere s;
      memset(&s, 0, sizeof s);
      bool ok = parse_floats(&save, v, 4);
      if (ok && raw) {
        ok = parse_floats(&save, v + 4, 8);
        if (ok) {
          s.material.matteColour = {v[4], v[5], v[6]};
          s.material.glossColour = {v[7], v[8], v[9]};
          s.material.opacity = v[10];
          s.material.refractiveIndex = v[11];
        }
      } else if (ok) {
        const char* name = strtok_r(nullptr, " \t\r\n", &save);
        auto it = name ? mats.find(name) : mats.end();
        if (it == mats.end()) {
          rtg_set_error("%s:%u: unknown material %s", path, line, name ? name : "(none)");
          rc = RTG_ERR_INVALID;
          break;
        }
        s.material = it->second;
      }
      if (!ok || strtok_r(nullptr, " \t\r\n", &save)) {
        rtg_set_error("%s:%u: expected: %s", path, line,
                      raw ? "sphere_raw x y z radius mr mg mb gr gg gb opacity n"
                          : "sphere x y z radius MATERIAL");
        rc = RTG_ERR_INVALID;
        break;
      }
      s.pos = {v[0], v[1], v[2]};
      s.radius = v[3];
      if (ns < sphCap) spheres[ns] = s;
      ++ns;
    } else if (!strcmp(kw, "light")) {
      float v[6];
      if (!parse_floats(&save, v, 6) || strtok_r(nullptr, " \t\r\n", &save)) {
        rtg_set_error("%s:%u: expected: light x y z r g b", path, line);
        rc = RTG_ERR_INVALID;
        break;
      }
      if (nl < lgtCap) lights[nl] = rtg_light{{v[0], v[1], v[2]}, {v[3], v[4], v[5]}};
      ++nl;
    } else {
      rtg_set_error("%s:%u: unknown keyword %s", path, line, kw);
      rc = RTG_ERR_INVALID;
    }
  }
  if (rc == RTG_OK && ferror(f)) {
    rtg_set_error("rtg_scene_load: read error on %s", path);
    rc = RTG_ERR_IO;
  }
  fclose(f);
  if (rc == RTG_OK) {
    *sphNum = ns;
    *lgtNum = nl;
  }
  return rc;
}

int rtg_scene_save(const char* path, const rtg_sphere* spheres, unsigned sphNum,
                   const rtg_light* lights, unsigned lgtNum) {
  rtg_clear_error();
  if (!path || (sphNum && !spheres) || (lgtNum && !lights)) {
    rtg_set_error("rtg_scene_save: invalid arguments");
    return RTG_ERR_INVALID;
  }
  FILE* f = fopen(path, "w");
  if (!f) {
    rtg_set_error("rtg_scene_save: cannot open %s", path);
    return RTG_ERR_IO;
  }
  fprintf(f, "# raytracer-gamma scene: %u spheres, %u lights (rtg_scene_save)\n", sphNum, lgtNum);
  for (unsigned i = 0; i < sphNum; ++i) {
    const rtg_sphere& s = spheres[i];
    const rtg_material& m = s.material;
    fprintf(f, "sphere_raw %.9g %.9g %.9g %.9g  %.9g %.9g %.9g  %.9g %.9g %.9g  %.9g %.9g\n",
            s.pos.x, s.pos.y, s.pos.z, s.radius, m.matteColour.x, m.matteColour.y,
            m.matteColour.z, m.glossColour.x, m.glossColour.y, m.glossColour.z, m.opacity,
            m.refractiveIndex);
  }
  for (unsigned l = 0; l < lgtNum; ++l)
    fprintf(f, "light %.9g %.9g %.9g  %.9g %.9g %.9g\n", lights[l].pos.x, lights[l].pos.y,
            lights[l].pos.z, lights[l].col.x, lights[l].col.y, lights[l].col.z);
  if (fclose(f) != 0) {
    rtg_set_error("rtg_scene_save: write error on %s", path);
    return RTG_ERR_IO;
  }
  return RTG_OK;
}

}  // extern "C"
