/*
 * rtg.h — C ABI of the MI355X-native raytracer-gamma hot path (librtg.so).
 *
 * This header is the drop-in boundary that replaces the reference's OpenCL
 * enqueue of the per-pixel kernel:
 *
 *   reference (snowzurfer/raytracer-gamma)            replaced by
 *   ------------------------------------------------  ------------------------------
 *   clCreateBuffer/clEnqueueWriteBuffer scene          rtg_render (one-shot) or
 *     main.cpp:277-294                                 rtg_context_set_scene
 *   clSetKernelArg x11, clEnqueueNDRangeKernel,        rtg_render / rtg_render_device /
 *     clFinish  main.cpp:339-363                       rtg_render_rows[_device]
 *     (kernel raytrace_kernel.cl:870-881)
 *   clEnqueueReadBuffer  main.cpp:460                  rtg_render (dstHost) or the
 *                                                      caller's copy of dstDevice
 *   maxColourValuePixelBuffer  algebra.h:68-91         rtg_max_colour (host) /
 *                                                      rtg_max_colour_device
 *   savePPM  main.cpp:43-91                            rtg_save_ppm / rtg_ppm_bytes
 *   rayTrace(...)  raytracer.h:410-636 (CPU entry)     (inside the HIP kernel)
 *   (8-GPU node, SURVEY.md §8e: none in the reference) rtg_render_multi (RCCL gather)
 *   checkError -> exit(EXIT_FAILURE)  err_code.h:143   negative return + rtg_last_error
 *   output_device_info  device_info.cpp:30             rtg_device_info
 *   parseArguments --list/--device  device_picker.h:70 rtg_device_count / device index args
 *
 * Scene records are byte-identical to the reference structs (static_asserts in
 * the implementation): a `struct Sphere*` / `struct Light*` / `Vec*` from the
 * reference host can be passed by a plain pointer cast.
 *
 * Semantics: the output is the framebuffer the reference CPU path
 * (raytracer.h, main.cpp:404-453) produces, bit for bit (NaNs are written as
 * the x86 default NaN 0xFFC00000 that path produces).  `stackSize` is the
 * reference's RTSTACK_MAXSIZE (raytraceStack.h:10; 6 as shipped) = depth + 1.
 *
 * All calls are blocking unless they take a `stream`; no call exits the
 * process.  Not re-entrant per context.
 */
#ifndef RTG_H
#define RTG_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTG_ABI_VERSION 1
#define RTG_MAX_STACK 16 /* largest supported RTSTACK_MAXSIZE */
/* Scenes hold fewer than RTG_MAX_SPHERES spheres (rtg_context_set_scene
 * rejects larger ones with RTG_ERR_INVALID): the kernel keeps material
 * indices in 22-bit fields and 32-bit table offsets. */
#define RTG_MAX_SPHERES (1u << 22)

/* vec.h:27-29 */
typedef struct rtg_vec { float x, y, z; } rtg_vec;
/* material.h:8-14 */
typedef struct rtg_material {
  rtg_vec matteColour;
  rtg_vec glossColour;
  float opacity;
  float refractiveIndex;
} rtg_material;
/* sphere.h:9-14 */
typedef struct rtg_sphere {
  rtg_vec pos;
  float radius;
  rtg_material material;
} rtg_sphere;
/* raytracer.h:20-25 */
typedef struct rtg_light { rtg_vec pos; rtg_vec col; } rtg_light;

/* Error codes (err_code.h:143-155 printed-and-exited; here they are returned). */
#define RTG_OK 0
#define RTG_ERR_INVALID (-1)   /* bad argument */
#define RTG_ERR_HIP (-2)       /* HIP runtime error; see rtg_last_error() */
#define RTG_ERR_NOMEM (-3)
#define RTG_ERR_NODEVICE (-4)
#define RTG_ERR_IO (-5)

/* Thread-local message for the last failing call ("" if none). */
const char* rtg_last_error(void);
int rtg_abi_version(void);

/* ---- device selection (device_picker.h:70-119, device_info.cpp:30-125) ---- */
int rtg_device_count(int* count);
/* Writes a one-line description ("name, CUs, clock, memory") into buf. */
int rtg_device_info(int device, char* buf, size_t buflen);

/* ---- one-shot drop-in for main.cpp:277-468 ----
 * Uploads the scene, renders the whole W x H frame on `device`, downloads
 * W*H rtg_vec into dstHost.  aliasFactor: the reference's kAliasFactor (3.f =
 * 3x3 supersampling); zoom: kZoom (-4.f). */
int rtg_render(int device, const rtg_sphere* spheres, unsigned sphNum,
               const rtg_light* lights, unsigned lgtNum, unsigned width,
               unsigned height, float zoom, float aliasFactor, int stackSize,
               rtg_vec* dstHost);

/* ---- multi-GPU one-shot: one process, nDevices GPUs ----
 * `devices` lists distinct device ids; devices[0] is the root.  Rows are dealt
 * row-cyclically in blocks of rowBlock (16 is a good default); every device
 * renders its shard on its own stream, ONE grouped RCCL gather (ncclGather)
 * brings the shards to the root over xGMI, the root restores row order
 * (rtg_assemble_shards_device) and W*H rtg_vec are copied to dstHost.
 * Bit-identical to rtg_render.  timingsMs (optional, 3 floats): slowest
 * device's render, gather + assemble on the root, wall time of the call. */
int rtg_render_multi(const int* devices, int nDevices, const rtg_sphere* spheres,
                     unsigned sphNum, const rtg_light* lights, unsigned lgtNum,
                     unsigned width, unsigned height, float zoom, float aliasFactor,
                     int stackSize, unsigned rowBlock, rtg_vec* dstHost, float* timingsMs);
/* The same with a persistent multi-device handle: the RCCL communicator
 * (ncclCommInitAll, ~0.5 s), the per-device contexts, streams and buffers
 * are kept across frames.  Not re-entrant per handle. */
typedef struct rtg_multi rtg_multi;
int rtg_multi_create(const int* devices, int nDevices, rtg_multi** out);
int rtg_multi_set_scene(rtg_multi* mg, const rtg_sphere* spheres, unsigned sphNum,
                        const rtg_light* lights, unsigned lgtNum);
int rtg_multi_render(rtg_multi* mg, unsigned width, unsigned height, float zoom,
                     float aliasFactor, int stackSize, unsigned rowBlock, rtg_vec* dstHost,
                     float* timingsMs);
int rtg_multi_destroy(rtg_multi* mg);
/* How rtg_multi_render brings the shards to the root:
 * RTG_GATHER_RCCL (default): one grouped ncclGather of the padded shards, then
 * the assemble kernel; RTG_GATHER_PEER_COPY (ablation): no collective, no
 * assemble — every device writes its shard's row blocks straight into the
 * root's frame with one strided peer copy (rtg_place_shard_device); needs
 * peer access to the root (enabled here, or RTG_ERR_HIP). */
#define RTG_GATHER_RCCL 0
#define RTG_GATHER_PEER_COPY 1
int rtg_multi_set_gather(rtg_multi* mg, int mode);

/* ---- persistent context: scene resident in HBM, caller-owned streams ----
 * A context may render on several streams; it orders its own scratch between
 * them with events (a launch on a stream other than the one its scratch slot
 * last ran on waits for that launch; hipStreamPerThread always waits).  A
 * stream handle that is destroyed and recreated while renders of the context
 * are still pending on it may come back with the same value: synchronise
 * such a stream (or the device) before destroying it. */
typedef struct rtg_context rtg_context;
int rtg_context_create(int device, rtg_context** out);
int rtg_context_destroy(rtg_context* ctx);
/* Copies the scene into device memory (kept until the next call / destroy). */
int rtg_context_set_scene(rtg_context* ctx, const rtg_sphere* spheres, unsigned sphNum,
                          const rtg_light* lights, unsigned lgtNum);

/* Cost of the last rtg_context_set_scene (end-to-end reporting, SURVEY.md
 * §8d): out4 = {host preparation ms (packed records, shadow / overlap / cone
 * masks, BVH build), upload ms (device allocation + H2D copies), device bytes
 * of the scene, BVH nodes}.  Zeros before the first scene. */
int rtg_context_scene_stats(rtg_context* ctx, double* out4);

/* Row sharding.  Rows are grouped in blocks of `rowBlock` rows; block b belongs
 * to shard (b % nShards) (row-cyclic).  A shard's rows are
 * packed in increasing row order.  nShards == 1 gives the whole frame in
 * row-major order.  Returns the number of rows of `shard` in *rows. */
int rtg_shard_rows(unsigned height, unsigned rowBlock, unsigned shard, unsigned nShards,
                   unsigned* rows);
/* Global row index of local row `localRow` of `shard`. */
unsigned rtg_shard_global_row(unsigned localRow, unsigned rowBlock, unsigned shard,
                              unsigned nShards);

/* Asynchronous render of shard `shard` of a W x H frame into device memory
 * dstDevice (rtg_shard_rows(...) * W rtg_vec) on `stream` (a hipStream_t, or
 * NULL for the null stream).  The camera uses global row indices, so the
 * shard's pixels are bit-identical to the same pixels of a 1-shard render. */
int rtg_render_device(rtg_context* ctx, unsigned width, unsigned height, float zoom,
                      float aliasFactor, int stackSize, unsigned rowBlock, unsigned shard,
                      unsigned nShards, rtg_vec* dstDevice, void* stream);

/* Restore row order after a gather of row-cyclic shards:
 * `gathered` holds nShards shard buffers of paddedRows x width rtg_vec each
 * (shard g's rows as rtg_render_device(..., rowBlock, g, nShards) packs them,
 * padded to paddedRows = ceil(ceil(H / rowBlock) / nShards) * rowBlock);
 * writes the height x width frame to `frame` on `stream`.  Device memory. */
int rtg_assemble_shards_device(rtg_context* ctx, const rtg_vec* gathered, unsigned nShards,
                               unsigned paddedRows, unsigned width, unsigned height,
                               unsigned rowBlock, rtg_vec* frame, void* stream);

/* The inverse placement without a gather buffer: copy shard `shardIdx`'s
 * packed rows (as rtg_render_device packs them) into their rows of the
 * height x width `frame` with one strided copy (hipMemcpy2DAsync; `frame` may
 * be another device's memory with peer access) plus one copy for a ragged
 * last block, on `stream`. */
int rtg_place_shard_device(rtg_context* ctx, const rtg_vec* shard, unsigned shardIdx,
                           unsigned nShards, unsigned width, unsigned height, unsigned rowBlock,
                           rtg_vec* frame, void* stream);

/* Render an explicit list of global rows (each < height) into dstDevice
 * (nRows * width rtg_vec, in list order); rowsDevice is device memory. */
int rtg_render_rows_device(rtg_context* ctx, unsigned width, unsigned height, float zoom,
                           float aliasFactor, int stackSize, const unsigned* rowsDevice,
                           unsigned nRows, rtg_vec* dstDevice, void* stream);
/* One-shot host version of the above (rows and dstHost in host memory). */
int rtg_render_rows(int device, const rtg_sphere* spheres, unsigned sphNum,
                    const rtg_light* lights, unsigned lgtNum, unsigned width, unsigned height,
                    float zoom, float aliasFactor, int stackSize, const unsigned* rows,
                    unsigned nRows, rtg_vec* dstHost);

/* Semantics of a context's renders.  RTG_SEMANTICS_CPU (default) is the
 * reference CPU path (raytracer.h), bit for bit.  RTG_SEMANTICS_OPENCL is the
 * reference's OpenCL kernel (raytrace_kernel.cl:641-867) under IEEE binary32:
 * f32 Fresnel (:399-432) and sinA1 (:507), the return register zeroed by the
 * reflection push (:835-845); pass stackSize 5 for the .cl's RTSTACK_MAXSIZE
 * (:58).  That kernel ran under OpenCL's relaxed division/sqrt, so its own
 * output (testPPM.ppm) is only approached, not reproduced bit for bit. */
#define RTG_SEMANTICS_CPU 0
#define RTG_SEMANTICS_OPENCL 1
int rtg_context_set_semantics(rtg_context* ctx, int semantics);

/* Launch-configuration knobs (performance only; results never change). */
typedef struct rtg_launch_opts {
  int variant;        /* 0 = default kernel; other values select A/B variants */
  int flags;          /* RTG_LAUNCH_* bits */
  int reserved[6];
} rtg_launch_opts;
int rtg_set_launch_opts(rtg_context* ctx, const rtg_launch_opts* opts);
/* Diagnostic variants (variant >= 100) sum per-wave s_memtime cycles spent in
 * {closest-hit queries, shadow queries, refraction, whole pixel} into 8
 * counters; read (and optionally zero) them.  Zeros for normal variants. */
int rtg_diag_read(rtg_context* ctx, unsigned long long* out8, int reset);
/* Executed-work counters of the counting build (variant 120: the default
 * kernel's control flow with per-unit counters): out[0 .. n/2)
 * wave-level executions of each unit (rtg_trace.h kCnt* / kU* slots), out[n/2
 * .. n) lane-level sums.  Copies min(cap, n) values, optionally zeroes them,
 * and returns n (cap <= 0: just returns n); negative on error. */
int rtg_diag_counts(rtg_context* ctx, unsigned long long* out, int cap, int reset);
#define RTG_LAUNCH_TIMELINE 1 /* record a per-wave timeline (rtg_diag_timeline) */
/* Compacted launches list pixel groups heaviest first, by the trace times the
 * previous launch of the same frame geometry measured (launch-order feedback:
 * a scheduling hint, the frame is the same either way).  This flag lists them
 * by primary-ray sphere count only (also env RTG_LAUNCH_ORDER=popcount). */
#define RTG_LAUNCH_NO_ORDER_FEEDBACK 2
/* Wave timeline of the last launch made with RTG_LAUNCH_TIMELINE: one record
 * per wave {start, end (s_memrealtime, 100 MHz, low 32 bits), HW_ID, XCC_ID | tag << 4}
 * (tag: the popcount of the wave's first group's sphere mask, 7 bits, then the
 * group's index, 21 bits; compacted launches only),
 * in launch order.  Copies min(cap, waves) records; *count = waves recorded.
 * Diagnostic only (occupancy analysis, tools/timeline.py). */
int rtg_diag_timeline(rtg_context* ctx, unsigned* out4, size_t cap, size_t* count);
/* The last compacted launch's pixel-group list (diagnostic; launch-order
 * studies, tools/cost_study.py): *groups = its pixel groups; cost[g] (cap
 * entries at most) the trace time of group g in s_memrealtime ticks (100 MHz)
 * as its cost table holds it (0 when the launch had none; a group not listed
 * keeps a stale value), list / sel (min(cap, groups) entries each) the listed
 * group indices and sphere masks in the order the trace kernel's waves take
 * them (runs[0] + ... + runs[3] entries), runs[4] the four run lengths summed
 * over the list's partitions.  Any output pointer may be null.
 * RTG_ERR_INVALID when the context has made no compacted launch. */
int rtg_diag_group_list(rtg_context* ctx, unsigned* cost, unsigned* list,
                        unsigned long long* sel, unsigned* runs, size_t cap, size_t* groups);

/* ---- output side ---- */
/* algebra.h:68-91 on the host. */
float rtg_max_colour(const rtg_vec* pixels, size_t n);
/* Same reduction on the device into *maxDevice (one float), on `stream`. */
int rtg_max_colour_device(rtg_context* ctx, const rtg_vec* pixelsDevice, size_t n,
                          float* maxDevice, void* stream);
/* main.cpp:66-81: 3 bytes per pixel, (unsigned char)(min(1,c)*255/max) with the
 * x86 truncating conversion (low byte of a 32-bit cvttss2si). */
void rtg_ppm_bytes(const rtg_vec* pixels, size_t n, float maxColourVal,
                   unsigned char* out);
/* Device version: reads *maxDevice, writes n*3 bytes to outDevice. */
int rtg_ppm_bytes_device(rtg_context* ctx, const rtg_vec* pixelsDevice, size_t n,
                         const float* maxDevice, unsigned char* outDevice, void* stream);
/* main.cpp:43-91: binary P6 writer. */
int rtg_save_ppm(const rtg_vec* pixels, const char* filename, int width, int height,
                 float maxColourVal);

/* ---- scene construction helpers (main.cpp:53-74, 113-168) ---- */
/* setMatOpacity + setMatteGlossBalance + setMatRefractivityIndex. */
void rtg_make_material(float opacity, float glossFactor, const rtg_vec* matte,
                       const rtg_vec* gloss, float refractiveIndex, rtg_material* out);
/* The reference's hard-coded 3-sphere / 2-light scene (main.cpp:104-168) when
 * sphNum<=3 && lgtNum<=2, extended by the seeded generator of SURVEY.md §8d.
 * seed 42 is the benchmark scene. */
int rtg_scene_generate(unsigned long long seed, unsigned sphNum, unsigned lgtNum,
                       rtg_sphere* spheres, rtg_light* lights);

/* ---- scene files (the reference hard-codes main.cpp:104-168) ----
 * Text format, one record per line ('#' starts a comment):
 *   material NAME opacity glossFactor mr mg mb gr gg gb refractiveIndex
 *   sphere x y z radius NAME
 *   sphere_raw x y z radius mr mg mb gr gg gb opacity refractiveIndex
 *   light x y z r g b
 * `material` builds the record with rtg_make_material (the reference's
 * setters).  Loads up to sphCap / lgtCap records and sets *sphNum / *lgtNum
 * to the file's totals (call with capacity 0 to size the arrays).  Errors
 * name the file and line.  rtg_scene_save writes sphere_raw / light records
 * that load back bit for bit. */
int rtg_scene_load(const char* path, rtg_sphere* spheres, unsigned sphCap, unsigned* sphNum,
                   rtg_light* lights, unsigned lgtCap, unsigned* lgtNum);
int rtg_scene_save(const char* path, const rtg_sphere* spheres, unsigned sphNum,
                   const rtg_light* lights, unsigned lgtNum);

#ifdef __cplusplus
}
#endif
#endif /* RTG_H */
