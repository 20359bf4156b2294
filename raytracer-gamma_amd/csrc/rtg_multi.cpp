// rtg_multi.cpp — one process, several GPUs: the multi-GPU entry points of the
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
//
// rtg_multi_* keep the communicator, the per-device contexts, streams and
// buffers across frames (ncclCommInitAll costs ~0.5 s); rtg_render_multi is
// the one-shot form.
//
// Ablation (rtg_multi_set_gather(RTG_GATHER_PEER_COPY)): no
// collective and no assemble pass; each device places its shard's row blocks
// straight into the root's frame with ONE strided peer copy
// (rtg_place_shard_device, hipMemcpy2DAsync over xGMI), and the root waits for
// every device's copy before the read-back.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <string>
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
  size_t shardCap = 0;  // rtg_vec
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipEvent_t ec = nullptr;  // peer-copy mode: this device's copy into the root's frame is done
};

}  // namespace

struct rtg_multi {
  std::vector<Dev> d;
  int gather = RTG_GATHER_RCCL;  // RTG_GATHER_* (rtg_multi_set_gather)
  rtg_vec* gathered = nullptr;  // on devices[0]
  rtg_vec* frame = nullptr;
  size_t gatheredCap = 0, frameCap = 0;
  hipEvent_t g1 = nullptr;
  bool hasScene = false;
};

extern "C" {

int rtg_multi_destroy(rtg_multi* mg) {
  rtg::DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!mg) return RTG_OK;
  for (Dev& v : mg->d)
    if (v.comm) (void)ncclCommDestroy(v.comm);
  if (!mg->d.empty() && mg->d[0].id >= 0) {
    (void)hipSetDevice(mg->d[0].id);
    (void)hipFree(mg->gathered);
    (void)hipFree(mg->frame);
    if (mg->g1) (void)hipEventDestroy(mg->g1);
  }
  for (Dev& v : mg->d) {
    if (v.id < 0) continue;
    (void)hipSetDevice(v.id);
    (void)hipFree(v.shard);
    if (v.e0) (void)hipEventDestroy(v.e0);
    if (v.e1) (void)hipEventDestroy(v.e1);
    if (v.ec) (void)hipEventDestroy(v.ec);
    if (v.stream) (void)hipStreamDestroy(v.stream);
    rtg_context_destroy(v.ctx);
  }
  delete mg;
  return RTG_OK;
}

int rtg_multi_create(const int* devices, int nDevices, rtg_multi** out) {
  rtg::DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!out || !devices || nDevices < 1) {
    rtg_set_error("rtg_multi_create: invalid arguments");
    return RTG_ERR_INVALID;
  }
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) {
    rtg_set_error("hipGetDeviceCount failed");
    return RTG_ERR_HIP;
  }
  for (int i = 0; i < nDevices; ++i) {
    if (devices[i] < 0 || devices[i] >= count) {
      rtg_set_error("rtg_multi_create: device %d not present (%d devices)", devices[i], count);
      return RTG_ERR_NODEVICE;
    }
    for (int j = 0; j < i; ++j)
      if (devices[j] == devices[i]) {
        rtg_set_error("rtg_multi_create: device %d listed twice", devices[i]);
        return RTG_ERR_INVALID;
      }
  }
  rtg_multi* mg = new rtg_multi();
  mg->d.resize((size_t)nDevices);
  for (int g = 0; g < nDevices; ++g) {
    Dev& v = mg->d[(size_t)g];
    v.id = devices[g];
    const int r = rtg_context_create(v.id, &v.ctx);
    if (r) {
      rtg_multi_destroy(mg);
      return r;
    }
    if (hipSetDevice(v.id) != hipSuccess ||
        hipStreamCreateWithFlags(&v.stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&v.e0) != hipSuccess || hipEventCreate(&v.e1) != hipSuccess ||
        hipEventCreateWithFlags(&v.ec, hipEventDisableTiming) != hipSuccess) {
      rtg_multi_destroy(mg);
      rtg_set_error("rtg_multi_create: stream/event creation failed");
      return RTG_ERR_HIP;
    }
  }
  if (hipSetDevice(devices[0]) != hipSuccess || hipEventCreate(&mg->g1) != hipSuccess) {
    rtg_multi_destroy(mg);
    rtg_set_error("rtg_multi_create: event creation failed");
    return RTG_ERR_HIP;
  }
  std::vector<ncclComm_t> comms((size_t)nDevices, nullptr);
  const ncclResult_t nr = ncclCommInitAll(comms.data(), nDevices, devices);
  if (nr != ncclSuccess) {
    rtg_multi_destroy(mg);
    rtg_set_error("rtg_multi_create: ncclCommInitAll failed: %s", ncclGetErrorString(nr));
    return RTG_ERR_HIP;
  }
  for (int g = 0; g < nDevices; ++g) mg->d[(size_t)g].comm = comms[(size_t)g];
  *out = mg;
  return RTG_OK;
}

int rtg_multi_set_gather(rtg_multi* mg, int mode) {
  rtg::DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!mg || (mode != RTG_GATHER_RCCL && mode != RTG_GATHER_PEER_COPY)) {
    rtg_set_error("rtg_multi_set_gather: invalid arguments");
    return RTG_ERR_INVALID;
  }
  if (mode == RTG_GATHER_PEER_COPY) {  // the root's frame must be writable by every device
    const int root = mg->d[0].id;
    for (size_t g = 1; g < mg->d.size(); ++g) {
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, mg->d[g].id, root) != hipSuccess || !can) {
        rtg_set_error("rtg_multi_set_gather: device %d cannot access device %d", mg->d[g].id,
                      root);
        return RTG_ERR_HIP;
      }
      (void)hipSetDevice(mg->d[g].id);
      const hipError_t e = hipDeviceEnablePeerAccess(root, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
        rtg_set_error("rtg_multi_set_gather: peer access %d -> %d: %s", mg->d[g].id, root,
                      hipGetErrorString(e));
        return RTG_ERR_HIP;
      }
      (void)hipGetLastError();  // clear an "already enabled" status
    }
  }
  mg->gather = mode;
  return RTG_OK;
}

int rtg_multi_set_scene(rtg_multi* mg, const rtg_sphere* spheres, unsigned sphNum,
                        const rtg_light* lights, unsigned lgtNum) {
  rtg::DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!mg) {
    rtg_set_error("rtg_multi_set_scene: null handle");
    return RTG_ERR_INVALID;
  }
  mg->hasScene = false;
  for (Dev& v : mg->d) {
    const int r = rtg_context_set_scene(v.ctx, spheres, sphNum, lights, lgtNum);
    if (r) return r;
  }
  mg->hasScene = true;
  return RTG_OK;
}

int rtg_multi_render(rtg_multi* mg, unsigned width, unsigned height, float zoom,
                     float aliasFactor, int stackSize, unsigned rowBlock, rtg_vec* dstHost,
                     float* timingsMs) {
  rtg::DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!mg || !mg->hasScene || !dstHost || rowBlock == 0 || width == 0 || height == 0) {
    rtg_set_error("rtg_multi_render: invalid arguments (or no scene)");
    return RTG_ERR_INVALID;
  }
  if (stackSize < 1 || stackSize > RTG_MAX_STACK) {
    rtg_set_error("stackSize %d outside [1, %d]", stackSize, RTG_MAX_STACK);
    return RTG_ERR_INVALID;
  }
  const auto t0 = std::chrono::steady_clock::now();
  const unsigned G = (unsigned)mg->d.size();
  const unsigned nb = (height + rowBlock - 1) / rowBlock;
  const unsigned Rmax = ((nb + G - 1) / G) * rowBlock;
  const size_t shardElems = (size_t)Rmax * width;  // rtg_vec per shard buffer
  const size_t frameElems = (size_t)width * height;
  // buffers grow on demand and are kept for the next frame
  for (Dev& v : mg->d) {
    if (v.shardCap >= shardElems) continue;
    (void)hipSetDevice(v.id);
    (void)hipFree(v.shard);
    v.shard = nullptr;
    v.shardCap = 0;
    if (hipMalloc(&v.shard, shardElems * sizeof(rtg_vec)) != hipSuccess) {
      rtg_set_error("rtg_multi_render: shard allocation failed");
      return RTG_ERR_NOMEM;
    }
    v.shardCap = shardElems;
  }
  Dev& root = mg->d[0];
  (void)hipSetDevice(root.id);
  const bool peer = mg->gather == RTG_GATHER_PEER_COPY;
  if (!peer && mg->gatheredCap < shardElems * G) {
    (void)hipFree(mg->gathered);
    mg->gathered = nullptr;
    mg->gatheredCap = 0;
    if (hipMalloc(&mg->gathered, shardElems * G * sizeof(rtg_vec)) != hipSuccess) {
      rtg_set_error("rtg_multi_render: gather buffer allocation failed");
      return RTG_ERR_NOMEM;
    }
    mg->gatheredCap = shardElems * G;
  }
  if (mg->frameCap < frameElems) {
    (void)hipFree(mg->frame);
    mg->frame = nullptr;
    mg->frameCap = 0;
    if (hipMalloc(&mg->frame, frameElems * sizeof(rtg_vec)) != hipSuccess) {
      rtg_set_error("rtg_multi_render: frame allocation failed");
      return RTG_ERR_NOMEM;
    }
    mg->frameCap = frameElems;
  }
  int rc = RTG_OK;
  // render every shard (asynchronous, one stream per device)
  for (unsigned g = 0; g < G && rc == RTG_OK; ++g) {
    Dev& v = mg->d[g];
    (void)hipSetDevice(v.id);
    (void)hipEventRecord(v.e0, v.stream);
    rc = rtg_render_device(v.ctx, width, height, zoom, aliasFactor, stackSize, rowBlock, g, G,
                           v.shard, v.stream);
    (void)hipEventRecord(v.e1, v.stream);
    if (rc == RTG_OK && peer) {  // the shard's blocks straight into the root's frame
      rc = rtg_place_shard_device(v.ctx, v.shard, g, G, width, height, rowBlock, mg->frame,
                                  v.stream);
      if (rc == RTG_OK && g > 0 && hipEventRecord(v.ec, v.stream) == hipSuccess) {
        (void)hipSetDevice(root.id);  // the root's stream waits for this copy
        if (hipStreamWaitEvent(root.stream, v.ec, 0) != hipSuccess) {
          rtg_set_error("rtg_multi_render: stream wait failed");
          rc = RTG_ERR_HIP;
        }
      }
    }
  }
  if (rc == RTG_OK && peer) {
    (void)hipSetDevice(root.id);
    if (hipEventRecord(mg->g1, root.stream) != hipSuccess ||
        hipMemcpyAsync(dstHost, mg->frame, frameElems * sizeof(rtg_vec), hipMemcpyDeviceToHost,
                       root.stream) != hipSuccess) {
      rtg_set_error("rtg_multi_render: frame readback failed");
      rc = RTG_ERR_HIP;
    }
  }
  if (rc == RTG_OK && !peer) {  // ONE grouped gather of the padded shards to the root
    ncclResult_t nr = ncclGroupStart();
    for (unsigned g = 0; g < G && nr == ncclSuccess; ++g)
      nr = ncclGather(mg->d[g].shard, g == 0 ? (void*)mg->gathered : nullptr, shardElems * 3,
                      ncclFloat, 0, mg->d[g].comm, mg->d[g].stream);
    const ncclResult_t ne = ncclGroupEnd();
    if (nr != ncclSuccess || ne != ncclSuccess) {
      rtg_set_error("rtg_multi_render: ncclGather failed: %s",
                    ncclGetErrorString(nr != ncclSuccess ? nr : ne));
      rc = RTG_ERR_HIP;
    }
  }
  if (rc == RTG_OK && !peer) {
    (void)hipSetDevice(root.id);
    rc = rtg_assemble_shards_device(root.ctx, mg->gathered, G, Rmax, width, height, rowBlock,
                                    mg->frame, root.stream);
    if (rc == RTG_OK && (hipEventRecord(mg->g1, root.stream) != hipSuccess ||
                         hipMemcpyAsync(dstHost, mg->frame, frameElems * sizeof(rtg_vec),
                                        hipMemcpyDeviceToHost, root.stream) != hipSuccess)) {
      rtg_set_error("rtg_multi_render: frame readback failed");
      rc = RTG_ERR_HIP;
    }
  }
  float renderMs = 0.f, gatherMs = 0.f;
  for (Dev& v : mg->d) {
    (void)hipSetDevice(v.id);
    const hipError_t e = hipStreamSynchronize(v.stream);
    if (e != hipSuccess && rc == RTG_OK) {
      rtg_set_error("rtg_multi_render: device synchronisation failed: %s", hipGetErrorString(e));
      rc = RTG_ERR_HIP;
    }
    float ms = 0.f;
    if (rc == RTG_OK && hipEventElapsedTime(&ms, v.e0, v.e1) == hipSuccess && ms > renderMs)
      renderMs = ms;
  }
  if (rc == RTG_OK) (void)hipEventElapsedTime(&gatherMs, root.e1, mg->g1);
  if (timingsMs) {
    timingsMs[0] = renderMs;
    timingsMs[1] = gatherMs;
    timingsMs[2] =
        std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return rc;
}

int rtg_render_multi(const int* devices, int nDevices, const rtg_sphere* spheres,
                     unsigned sphNum, const rtg_light* lights, unsigned lgtNum, unsigned width,
                     unsigned height, float zoom, float aliasFactor, int stackSize,
                     unsigned rowBlock, rtg_vec* dstHost, float* timingsMs) {
  rtg_clear_error();
  if (!dstHost || rowBlock == 0 || width == 0 || height == 0 || (sphNum && !spheres) ||
      (lgtNum && !lights)) {
    rtg_set_error("rtg_render_multi: invalid arguments");
    return RTG_ERR_INVALID;
  }
  if (stackSize < 1 || stackSize > RTG_MAX_STACK) {
    rtg_set_error("stackSize %d outside [1, %d]", stackSize, RTG_MAX_STACK);
    return RTG_ERR_INVALID;
  }
  const auto t0 = std::chrono::steady_clock::now();
  rtg_multi* mg = nullptr;
  int rc = rtg_multi_create(devices, nDevices, &mg);
  if (!rc) rc = rtg_multi_set_scene(mg, spheres, sphNum, lights, lgtNum);
  if (!rc)
    rc = rtg_multi_render(mg, width, height, zoom, aliasFactor, stackSize, rowBlock, dstHost,
                          timingsMs);
  if (mg) {
    const std::string err = rc ? std::string(rtg_last_error()) : std::string();
    rtg_multi_destroy(mg);
    if (rc) rtg_set_error("%s", err.c_str());
  }
  if (!rc && timingsMs)
    timingsMs[2] =
        std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return rc;
}

}  // extern "C"
