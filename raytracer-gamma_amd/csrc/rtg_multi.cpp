// rtg_multi.cpp — one process, several GPUs: the multi-GPU entry point of the
// C ABI (SURVEY.md §8b "rtg_render_multi", §8e).
//
// The frame's rows are dealt row-cyclically in blocks of `rowBlock` to the
// devices (shard g = blocks g, g + G, ...; rtg_render_device packs them), every
// device renders its shard on its own stream, and ONE grouped RCCL gather
// (ncclGather, rccl.h:745; root = devices[0]) moves the padded shards to the
// root over xGMI.  The root restores row order with the assemble kernel and
// copies the frame to the host.  The camera uses global rows, so the frame is
// bit-identical to rtg_render's.  Replaces the reference's single-device
// enqueue + readback (main.cpp:330-363, 456-468) for an 8-GPU node.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <vector>

#include "rtg.h"
#include "rtg_internal.h"

namespace {

struct Dev {
  int id = -1;
  rtg_context* ctx = nullptr;
  hipStream_t stream = nullptr;
  ncclComm_t comm = nullptr;
  rtg_vec* shard = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
};

}  // namespace

extern "C" int rtg_render_multi(const int* devices, int nDevices, const rtg_sphere* spheres,
                                unsigned sphNum, const rtg_light* lights, unsigned lgtNum,
                                unsigned width, unsigned height, float zoom, float aliasFactor,
                                int stackSize, unsigned rowBlock, rtg_vec* dstHost,
                                float* timingsMs) {
  rtg_clear_error();
  if (!devices || nDevices < 1 || !dstHost || rowBlock == 0 || width == 0 || height == 0 ||
      (sphNum && !spheres) || (lgtNum && !lights)) {
    rtg_set_error("rtg_render_multi: invalid arguments");
    return RTG_ERR_INVALID;
  }
  if (stackSize < 1 || stackSize > RTG_MAX_STACK) {
    rtg_set_error("stackSize %d outside [1, %d]", stackSize, RTG_MAX_STACK);
    return RTG_ERR_INVALID;
  }
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) {
    rtg_set_error("hipGetDeviceCount failed");
    return RTG_ERR_HIP;
  }
  for (int i = 0; i < nDevices; ++i) {
    if (devices[i] < 0 || devices[i] >= count) {
      rtg_set_error("rtg_render_multi: device %d not present (%d devices)", devices[i], count);
      return RTG_ERR_NODEVICE;
    }
    for (int j = 0; j < i; ++j)
      if (devices[j] == devices[i]) {
        rtg_set_error("rtg_render_multi: device %d listed twice", devices[i]);
        return RTG_ERR_INVALID;
      }
  }
  const auto t0 = std::chrono::steady_clock::now();
  const unsigned G = (unsigned)nDevices;
  const unsigned nb = (height + rowBlock - 1) / rowBlock;
  const unsigned Rmax = ((nb + G - 1) / G) * rowBlock;
  const size_t shardElems = (size_t)Rmax * width;  // rtg_vec per shard buffer
  std::vector<Dev> d(G);
  rtg_vec* gathered = nullptr;
  rtg_vec* frame = nullptr;
  int rc = RTG_OK;
  auto fail = [&](int code, const char* what, const char* detail) {
    if (rc == RTG_OK) {
      rtg_set_error("rtg_render_multi: %s%s%s", what, detail ? ": " : "", detail ? detail : "");
      rc = code;
    }
  };
  for (unsigned g = 0; g < G && rc == RTG_OK; ++g) {
    d[g].id = devices[g];
    int r = rtg_context_create(d[g].id, &d[g].ctx);
    if (r) { rc = r; break; }
    r = rtg_context_set_scene(d[g].ctx, spheres, sphNum, lights, lgtNum);
    if (r) { rc = r; break; }
    if (hipSetDevice(d[g].id) != hipSuccess ||
        hipStreamCreateWithFlags(&d[g].stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&d[g].e0) != hipSuccess || hipEventCreate(&d[g].e1) != hipSuccess)
      fail(RTG_ERR_HIP, "stream/event creation failed", nullptr);
    else if (hipMalloc(&d[g].shard, shardElems * sizeof(rtg_vec)) != hipSuccess)
      fail(RTG_ERR_NOMEM, "shard allocation failed", nullptr);
  }
  if (rc == RTG_OK) {
    if (hipSetDevice(d[0].id) != hipSuccess ||
        hipMalloc(&gathered, shardElems * G * sizeof(rtg_vec)) != hipSuccess ||
        hipMalloc(&frame, (size_t)width * height * sizeof(rtg_vec)) != hipSuccess)
      fail(RTG_ERR_NOMEM, "root buffers allocation failed", nullptr);
  }
  std::vector<ncclComm_t> comms(G, nullptr);
  if (rc == RTG_OK) {
    const ncclResult_t nr = ncclCommInitAll(comms.data(), nDevices, devices);
    if (nr != ncclSuccess) fail(RTG_ERR_HIP, "ncclCommInitAll failed", ncclGetErrorString(nr));
    for (unsigned g = 0; g < G; ++g) d[g].comm = comms[g];
  }
  // render every shard (asynchronous, one stream per device)
  for (unsigned g = 0; g < G && rc == RTG_OK; ++g) {
    (void)hipSetDevice(d[g].id);
    (void)hipEventRecord(d[g].e0, d[g].stream);
    const int r = rtg_render_device(d[g].ctx, width, height, zoom, aliasFactor, stackSize,
                                    rowBlock, g, G, d[g].shard, d[g].stream);
    if (r) rc = r;
    (void)hipEventRecord(d[g].e1, d[g].stream);
  }
  hipEvent_t g1 = nullptr;
  if (rc == RTG_OK) {  // ONE grouped gather of the padded shards to the root
    ncclResult_t nr = ncclGroupStart();
    for (unsigned g = 0; g < G && nr == ncclSuccess; ++g)
      nr = ncclGather(d[g].shard, g == 0 ? (void*)gathered : nullptr, shardElems * 3, ncclFloat,
                      0, d[g].comm, d[g].stream);
    const ncclResult_t ne = ncclGroupEnd();
    if (nr != ncclSuccess || ne != ncclSuccess)
      fail(RTG_ERR_HIP, "ncclGather failed", ncclGetErrorString(nr != ncclSuccess ? nr : ne));
  }
  if (rc == RTG_OK) {
    (void)hipSetDevice(d[0].id);
    const int r = rtg_assemble_shards_device(d[0].ctx, gathered, G, Rmax, width, height,
                                             rowBlock, frame, d[0].stream);
    if (r) rc = r;
    if (rc == RTG_OK && (hipEventCreate(&g1) != hipSuccess ||
                         hipEventRecord(g1, d[0].stream) != hipSuccess))
      fail(RTG_ERR_HIP, "event record failed", nullptr);
    if (rc == RTG_OK &&
        hipMemcpyAsync(dstHost, frame, (size_t)width * height * sizeof(rtg_vec),
                       hipMemcpyDeviceToHost, d[0].stream) != hipSuccess)
      fail(RTG_ERR_HIP, "frame readback failed", nullptr);
  }
  float renderMs = 0.f, gatherMs = 0.f;
  for (unsigned g = 0; g < G; ++g) {
    if (!d[g].stream) continue;
    (void)hipSetDevice(d[g].id);
    const hipError_t e = hipStreamSynchronize(d[g].stream);
    if (e != hipSuccess) fail(RTG_ERR_HIP, "device synchronisation failed", hipGetErrorString(e));
    float ms = 0.f;
    if (rc == RTG_OK && hipEventElapsedTime(&ms, d[g].e0, d[g].e1) == hipSuccess &&
        ms > renderMs)
      renderMs = ms;
  }
  if (rc == RTG_OK && g1) (void)hipEventElapsedTime(&gatherMs, d[0].e1, g1);
  if (timingsMs) {
    timingsMs[0] = renderMs;
    timingsMs[1] = gatherMs;
    timingsMs[2] = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0)
                       .count();
  }
  // teardown (also after a failure)
  for (unsigned g = 0; g < G; ++g)
    if (d[g].comm) (void)ncclCommDestroy(d[g].comm);
  if (g1) (void)hipEventDestroy(g1);
  if (G && d[0].id >= 0) {
    (void)hipSetDevice(d[0].id);
    (void)hipFree(gathered);
    (void)hipFree(frame);
  }
  for (unsigned g = 0; g < G; ++g) {
    if (d[g].id < 0) continue;
    (void)hipSetDevice(d[g].id);
    (void)hipFree(d[g].shard);
    if (d[g].e0) (void)hipEventDestroy(d[g].e0);
    if (d[g].e1) (void)hipEventDestroy(d[g].e1);
    if (d[g].stream) (void)hipStreamDestroy(d[g].stream);
    rtg_context_destroy(d[g].ctx);
  }
  return rc;
}
