// rtg_main.cpp — the reference's host program (main.cpp) on librtg.so.
//
// Same flow as main.cpp:94-508: build the scene (main.cpp:104-168, or the
// seeded generator for larger scenes), render on the GPU through the C ABI
// (replacing the OpenCL setup/enqueue/readback of main.cpp:182-468), compute
// the colour max (algebra.h:68) and write the P6 PPM (main.cpp:43-91).  Errors
// print a message and exit(EXIT_FAILURE), like checkError (err_code.h:143-155).
// Device selection follows device_picker.h:70-119 (--list, --device N, -h).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "rtg.h"

static void check(int rc, const char* what) {
  if (rc != RTG_OK) {
    fprintf(stderr, "Error: %s failed (%d): %s\n", what, rc, rtg_last_error());
    exit(EXIT_FAILURE);
  }
}

static void usage() {
  printf("\nUsage: ./rtg_main [OPTIONS]\n\n");
  printf("Options:\n");
  printf("  -h  --help               Print the message\n");
  printf("      --list               List available devices\n");
  printf("      --device     INDEX   Select device at INDEX (default 0)\n");
  printf("      --width      W       Frame width  (default 800, main.cpp:105)\n");
  printf("      --height     H       Frame height (default 600, main.cpp:106)\n");
  printf("      --spheres    N       Spheres (default 3 = main.cpp scene)\n");
  printf("      --lights     M       Lights  (default 2 = main.cpp scene)\n");
  printf("      --depth      D       Recursion depth = RTSTACK_MAXSIZE - 1 (default 5)\n");
  printf("      --aa         F       Alias factor (default 3 -> 3x3 samples)\n");
  printf("      --zoom       Z       Zoom factor (default -4)\n");
  printf("      --seed       S       Scene generator seed (default 42)\n");
  printf("      --out        FILE    Output PPM (default testPPM.ppm)\n");
  printf("      --repeat     K       Render K times, report the best time\n");
  printf("      --scene      FILE    Load the scene from FILE (format: include/rtg.h)\n");
  printf("      --save-scene FILE    Write the scene used to FILE\n");
  printf("      --gpus       N       Render on devices 0..N-1 (row-cyclic shards, RCCL gather)\n");
  printf("      --semantics  MODE    cpu (default: raytracer.h, bit-exact) or opencl\n");
  printf("                           (raytrace_kernel.cl; use with --depth 4 = its stack of 5)\n");
  printf("\n");
}

static bool parse_uint(const char* s, unsigned* out) {
  char* end;
  unsigned long v = strtoul(s, &end, 10);
  if (*end) return false;
  *out = (unsigned)v;
  return true;
}

int main(int argc, char** argv) {
  unsigned device = 0, W = 800, H = 600, nSph = 3, nLgt = 2, depth = 5, repeat = 1;
  unsigned long long seed = 42;
  float aa = 3.f, zoom = -4.f;
  std::string out = "testPPM.ppm", sceneIn, sceneOut;
  unsigned gpus = 0;
  int semantics = RTG_SEMANTICS_CPU;
  for (int i = 1; i < argc; ++i) {
    auto need = [&](const char* opt) -> const char* {
      if (++i >= argc) {
        printf("Missing value for %s\n", opt);
        exit(1);
      }
      return argv[i];
    };
    const char* a = argv[i];
    if (!strcmp(a, "-h") || !strcmp(a, "--help")) {
      usage();
      return 0;
    } else if (!strcmp(a, "--list")) {
      int n = 0;
      check(rtg_device_count(&n), "rtg_device_count");
      if (n == 0) printf("No devices found.\n");
      printf("\nDevices:\n");
      for (int d = 0; d < n; ++d) {
        char buf[256];
        check(rtg_device_info(d, buf, sizeof buf), "rtg_device_info");
        printf("%2d: %s\n", d, buf);
      }
      printf("\n");
      return 0;
    } else if (!strcmp(a, "--device")) {
      if (!parse_uint(need(a), &device)) { printf("Invalid device index\n"); return 1; }
    } else if (!strcmp(a, "--width")) {
      if (!parse_uint(need(a), &W)) { printf("Invalid width\n"); return 1; }
    } else if (!strcmp(a, "--height")) {
      if (!parse_uint(need(a), &H)) { printf("Invalid height\n"); return 1; }
    } else if (!strcmp(a, "--spheres")) {
      if (!parse_uint(need(a), &nSph)) { printf("Invalid sphere count\n"); return 1; }
    } else if (!strcmp(a, "--lights")) {
      if (!parse_uint(need(a), &nLgt)) { printf("Invalid light count\n"); return 1; }
    } else if (!strcmp(a, "--depth")) {
      if (!parse_uint(need(a), &depth)) { printf("Invalid depth\n"); return 1; }
    } else if (!strcmp(a, "--repeat")) {
      if (!parse_uint(need(a), &repeat) || repeat == 0) { printf("Invalid repeat\n"); return 1; }
    } else if (!strcmp(a, "--aa")) {
      aa = strtof(need(a), nullptr);
    } else if (!strcmp(a, "--zoom")) {
      zoom = strtof(need(a), nullptr);
    } else if (!strcmp(a, "--seed")) {
      seed = strtoull(need(a), nullptr, 10);
    } else if (!strcmp(a, "--out")) {
      out = need(a);
    } else if (!strcmp(a, "--scene")) {
      sceneIn = need(a);
    } else if (!strcmp(a, "--save-scene")) {
      sceneOut = need(a);
    } else if (!strcmp(a, "--semantics")) {
      const char* v = need(a);
      if (!strcmp(v, "cpu")) semantics = RTG_SEMANTICS_CPU;
      else if (!strcmp(v, "opencl")) semantics = RTG_SEMANTICS_OPENCL;
      else { printf("Invalid semantics %s (cpu|opencl)\n", v); return 1; }
    } else if (!strcmp(a, "--gpus")) {
      if (!parse_uint(need(a), &gpus) || gpus == 0) { printf("Invalid GPU count\n"); return 1; }
    } else {
      printf("Unknown option %s\n", a);
      usage();
      return 1;
    }
  }

  std::vector<rtg_sphere> spheres;
  std::vector<rtg_light> lights;
  if (!sceneIn.empty()) {
    check(rtg_scene_load(sceneIn.c_str(), nullptr, 0, &nSph, nullptr, 0, &nLgt),
          "rtg_scene_load");
    spheres.resize(nSph);
    lights.resize(nLgt);
    check(rtg_scene_load(sceneIn.c_str(), spheres.data(), nSph, &nSph, lights.data(), nLgt,
                         &nLgt),
          "rtg_scene_load");
  } else {
    spheres.resize(nSph);
    lights.resize(nLgt);
    check(rtg_scene_generate(seed, nSph, nLgt, spheres.data(), lights.data()),
          "rtg_scene_generate");
  }
  if (!sceneOut.empty())
    check(rtg_scene_save(sceneOut.c_str(), spheres.data(), nSph, lights.data(), nLgt),
          "rtg_scene_save");

  char info[256];
  check(rtg_device_info((int)device, info, sizeof info), "rtg_device_info");
  printf("Device %u: %s\n", device, info);

  std::vector<rtg_vec> pixels((size_t)W * H);
  rtg_multi* mg = nullptr;  // --gpus: one communicator for every repeat
  if (gpus) {
    std::vector<int> devs(gpus);
    for (unsigned g = 0; g < gpus; ++g) devs[g] = (int)g;
    check(rtg_multi_create(devs.data(), (int)gpus, &mg), "rtg_multi_create");
    check(rtg_multi_set_scene(mg, spheres.data(), nSph, lights.data(), nLgt),
          "rtg_multi_set_scene");
  }
  double best = 1e30;
  for (unsigned r = 0; r < repeat; ++r) {
    auto t0 = std::chrono::steady_clock::now();
    if (semantics != RTG_SEMANTICS_CPU) {  // persistent context: semantics is per context
      if (gpus) { printf("--semantics opencl renders on one device\n"); return 1; }
      rtg_context* ctx = nullptr;
      check(rtg_context_create((int)device, &ctx), "rtg_context_create");
      check(rtg_context_set_semantics(ctx, semantics), "rtg_context_set_semantics");
      check(rtg_context_set_scene(ctx, spheres.data(), nSph, lights.data(), nLgt),
            "rtg_context_set_scene");
      rtg_vec* d = nullptr;
      if (hipMalloc(&d, pixels.size() * sizeof(rtg_vec)) != hipSuccess)
        check(RTG_ERR_NOMEM, "hipMalloc");
      check(rtg_render_device(ctx, W, H, zoom, aa, (int)depth + 1, 16, 0, 1, d, nullptr),
            "rtg_render_device");
      if (hipMemcpy(pixels.data(), d, pixels.size() * sizeof(rtg_vec),
                    hipMemcpyDeviceToHost) != hipSuccess)
        check(RTG_ERR_HIP, "readback");
      (void)hipFree(d);
      rtg_context_destroy(ctx);
    } else if (gpus) {
      float tm[3];
      check(rtg_multi_render(mg, W, H, zoom, aa, (int)depth + 1, 16, pixels.data(), tm),
            "rtg_multi_render");
      printf("  %u GPUs: render %.3f ms (slowest device), gather+assemble %.3f ms\n", gpus,
             (double)tm[0], (double)tm[1]);
    } else {
      check(rtg_render((int)device, spheres.data(), nSph, lights.data(), nLgt, W, H, zoom, aa,
                       (int)depth + 1, pixels.data()),
            "rtg_render");
    }
    auto t1 = std::chrono::steady_clock::now();
    double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    if (ms < best) best = ms;
  }
  if (mg) rtg_multi_destroy(mg);
  // main.cpp:374 prints integer milliseconds; report the measured value.
  printf("Exec time: %.5f ms (end to end: upload, render, readback)\n", best);

  const float mx = rtg_max_colour(pixels.data(), pixels.size());
  check(rtg_save_ppm(pixels.data(), out.c_str(), (int)W, (int)H, mx), "rtg_save_ppm");
  printf("Wrote %s (%ux%u, %u spheres, %u lights, depth %u, max colour %.8g)\n", out.c_str(), W,
         H, nSph, nLgt, depth, (double)mx);
  return 0;
}
