// rtg_kernel.hip — launch code and the device half of the C ABI of librtg.so.
//
// Replaces the host orchestration of the OpenCL kernel `raytrace`
// (main.cpp:277-363, 456-468): scene upload into a persistent context, the
// trace launch (kernels in rtg_trace_kernels.h, one object per stack size),
// and the PPM helpers on the device (max colour, byte conversion).
//
// Launch geometry of the default (sample-parallel) kernel: one-wave
// workgroups, each wave floor(64 / nAA^2) consecutive pixels of the shard
// with one primary sample per lane (7 pixels x 9 samples at nAA = 3); the
// sphere loop index is wave-uniform, so sphere records are read with scalar
// loads into SGPRs.  See DESIGN.md §4.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <type_traits>
#include <vector>

#include "rtg.h"
#include "rtg_internal.h"
#include "rtg_trace_kernels.h"
#include "rtg_scene_pack.h"

#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) {                                                        \
      rtg_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                    __LINE__);                                                     \
      return RTG_ERR_HIP;                                                          \
    }                                                                              \
  } while (0)

namespace rtg {

// algebra.h:68-91 on the device: values are compared as floats (NaN never
// wins), the running max starts at +0 so only positive values can win, and a
// non-negative float orders like its bit pattern, so an integer atomicMax on
// the bits reduces across workgroups.
__global__ __launch_bounds__(256) void max_kernel(const float* __restrict__ c, size_t nval,
                                                  unsigned* __restrict__ out) {
  float mx = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nval;
       i += (size_t)gridDim.x * blockDim.x) {
    const float v = c[i];
    if (v > mx) mx = v;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const float o = __shfl_xor(mx, off);
    if (o > mx) mx = o;
  }
  __shared__ float part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; ++w)
      if (part[w] > mx) mx = part[w];
    atomicMax(out, __float_as_uint(mx));
  }
}

// Row-cyclic shards back to row order: grid.y = global row block gb (shard
// gb % G, local block gb / G), each block of rows is one contiguous copy.
template <class T>
__global__ __launch_bounds__(256) void assemble_kernel(const T* __restrict__ gathered,
                                                       T* __restrict__ frame, unsigned G,
                                                       unsigned Rmax, unsigned H, unsigned B,
                                                       size_t rowElems) {
  const unsigned gb = blockIdx.y;
  const unsigned g = gb % G, lb = gb / G;
  const unsigned row0 = gb * B;
  const unsigned rows = (H - row0 < B) ? (H - row0) : B;
  const size_t n = (size_t)rows * rowElems;
  const T* src = gathered + ((size_t)g * Rmax + (size_t)lb * B) * rowElems;
  T* dst = frame + (size_t)row0 * rowElems;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

__global__ void max_finish_kernel(unsigned* m) {
  if (__uint_as_float(*m) == 0.f) *m = __float_as_uint(1.f);
}

__global__ __launch_bounds__(256) void ppm_kernel(const float* __restrict__ c, size_t nval,
                                                  const float* __restrict__ mx,
                                                  unsigned char* __restrict__ out) {
  const float m = *mx;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nval;
       i += (size_t)gridDim.x * blockDim.x)
    out[i] = ppm_byte(c[i], m);
}

// Trivial-group pass of the compacted launch: one LANE per pixel group (the
// sample kernel's floor(64 / nAA^2) consecutive pixels).  The group's
// primary-ray bundle is bounded from primary_bounds of each of its pixels
// (the extremes of sample_dir's monotone float steps, as trace_group's cull)
// and tested against every sphere with primary_possible.  A group no
// sphere can be reached from is written +0 directly: every sample misses
// (closest_hit_sel over an empty set, raytracer.h:454-459), returns
// I (x) bgMaterial.matte = (1,1,1) (x) 0 = +0 (raytracer.h:544, the
// background matte is 0), and the pixel sum of +0 * inv is +0 in every
// channel.  The other groups are appended to groupList (one atomic per wave)
// for the trace kernel.  n <= 64 spheres.
// The spheres pixel group g can reach (the cull of trace_group): bit i set
// when primary_possible keeps sphere i for the group's bundle.
__device__ __forceinline__ uint64_t group_sel(const KernelArgs& a, size_t g, unsigned PPW,
                                              size_t total) {
  const size_t p0 = g * PPW;
  const unsigned nv = (unsigned)((total - p0 < PPW) ? (total - p0) : PPW);
  unsigned col, lr;
  divmod_u64(p0, a.W, a.invW, lr, col);
  float x0 = 3.0e38f, x1 = -3.0e38f, y0 = 3.0e38f, y1 = -3.0e38f;
  // one row: the first and last pixels bound the group (monotone float
  // steps, see trace_group); otherwise every pixel
  const bool oneRow = col + nv - 1 < a.W;
  for (unsigned k = 0; k < nv; ++k) {
    if (!oneRow || k == 0 || k == nv - 1) {
      const unsigned gy =
          a.rowList ? a.rowList[lr]
                    : shard_global_row_fast(lr, a.rowBlock, a.invRowBlock, a.shard, a.nShards);
      float bx0, bx1, by0, by1;
      primary_bounds(a.cam, col, gy, bx0, bx1, by0, by1);
      x0 = fminf(x0, bx0);
      x1 = fmaxf(x1, bx1);
      y0 = fminf(y0, by0);
      y1 = fmaxf(y1, by1);
    }
    if (++col == a.W) {
      col = 0;
      ++lr;
    }
  }
  const PrimBundle pb = primary_bundle(x0, x1, y0, y1, a.cam.zoom);
  const RTG_CONST float* geom = (const RTG_CONST float*)a.geom;
  const RTG_CONST float* pc = (const RTG_CONST float*)a.prim;
  uint64_t sel = 0;
  for (unsigned i = 0; i < a.n; ++i) {  // wave-uniform: scalar sphere records
    const RTG_CONST float* r = geom + 4 * i;
    const RTG_CONST float* k = pc + 4 * i;
    if (primary_possible(pb, v3(r[0], r[1], r[2]), k[0], k[1], k[2])) sel |= 1ull << i;
  }
  return sel;
}

// Launches of at most this many pixel groups list them in eight runs
// (KernelArgs::nRuns): a 1/8 or 1/4 C3 shard's chunks (~60 k, ~125 k), not a
// whole C2 frame (292 k).
#ifndef RTG_RUNS8_MAX_GROUPS
#define RTG_RUNS8_MAX_GROUPS 200000
#endif
constexpr size_t kRuns8MaxGroups = RTG_RUNS8_MAX_GROUPS;

// One launch's counter sets: the run lengths and the cost sums of all list
// partitions (KernelArgs::groupCount, costStat).
constexpr size_t kCountSet = (size_t)kListParts * kCountStride;
constexpr size_t kStatSet = (size_t)kListParts * kStatStride;

// A block takes 256 consecutive groups (one per lane) and appends its live
// ones with one atomic per run, in one of kListParts list partitions (block
// b: partition b % kListParts), each with its own run counters and cost sum
// on a cache line of its own.  Device-scope atomics on one address serialise
// (tools/cull_micro.hip, 1158 workgroups: one address 15.1 us, 8 lines 4.5,
// 32 lines 3.7, no atomic 3.7): with the whole list on one set of counters
// the C2 pass took 21 us, 11 of them queued atomics.  Once they no longer
// queue, one group per lane beats the 2 or 4 per lane that had kept the
// block count down (C3 pass 39 -> 31 us, C4 frame -1 %).
// The trace kernel's one-wave workgroups w take partition w % kListParts, so
// block b's groups are traced on the XCD that ran block b (both b mod 8) and
// find its list entries, cost-table reads and zero-filled lines in that XCD's
// L2.  Measured (profiles/r06/partition_map/): partition (b + b/16) % 16,
// which spreads a partition over all XCDs, C2 +4.5 %, C3 +6.5 %, C4 +4 %; a
// skew within each XCD's two partitions still +1.2-3.4 %.
// Each listed group's sphere mask goes to groupSel at the same list index:
// the trace kernel takes it as the wave's primary-ray subset (one scalar
// load) instead of recomputing the cull.
// Heavy groups first (longest-processing-time order): the trace kernel's
// waves take each partition's list in order (wave w: partition w % kListParts),
// and a launch ends with its last waves' tail (a wave traces a whole pixel
// group; durations spread 3x around the median), which dominates a short
// launch such as one GPU's shard of a multi-GPU frame.  A partition's groups
// are listed in four runs, heaviest first (KernelArgs::groupCount):
//  * with launch-order feedback (a.groupCost: the previous launch of the same
//    frame geometry wrote every listed group's trace time; a.costPrev: the
//    sums and counts of the times the previous cull pass read, whose mean is
//    mu), by that time: >= 2 mu, >= mu, >= mu / 2, the rest.  A group's cost
//    is a scheduling hint only: any value lists the group, so the frame is
//    the same whatever the hint (a group dead last time reads a stale value).
//    The pass also sums the times it reads into a.costStat, one atomic per
//    block on its partition's sum (the trace kernel's waves only store their
//    group's time: 10^5 atomics on one address from the trace waves cost a C3
//    frame 0.5 ms);
//  * otherwise (a geometry's first two launches, or feedback off) by the
//    sphere mask: >= a.lptMin spheres first.
// Partition p's region is [2 p cap, 2 (p + 1) cap) (cap = a.groupCap, the
// groups of the partition's blocks): run 0 fills its first half from the
// front, run 1 from the back, runs 2 and 3 the second half likewise.
template <unsigned kRuns>
__global__ __launch_bounds__(256) void cull_groups_kernel(const KernelArgs a, size_t nGroups,
                                                          unsigned* groupList,
                                                          unsigned long long* groupSel,
                                                          unsigned* groupCount) {
  static_assert(kRuns == 4 || kRuns == 8, "four or eight runs");
  __shared__ unsigned cnt[kRuns][4];
  __shared__ unsigned blockBase[kRuns];
  __shared__ unsigned long long waveCost[4];
  const unsigned lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const unsigned part = blockIdx.x % kListParts;
  const unsigned nAA = (unsigned)a.cam.nAA;
  const unsigned PPW = 64u / (nAA * nAA);
  const size_t total = (size_t)a.W * a.rowsLocal;
  const size_t g = (size_t)blockIdx.x * 256 + threadIdx.x;
  // the previous launch's mean group time (ticks), 0: no feedback
  float mu = 0.f;
  if (a.costPrev != nullptr) {
    unsigned long long st = 0;
#pragma unroll
    for (unsigned p = 0; p < kListParts; ++p) st += a.costPrev[p * kStatStride];
    const unsigned ng = (unsigned)(st >> 40);
    if (ng != 0u) mu = (float)(st & ((1ull << 40) - 1ull)) / (float)ng;
  }
  const uint64_t sel = g < nGroups ? group_sel(a, g, PPW, total) : 0ull;
  const unsigned pc = (unsigned)__builtin_popcountll(sel);
  // Zero-fill the pixels of all this wave's groups with coalesced stores
  // (the trace kernel, later on the same stream, overwrites the live ones).
  // Measured against writing only the empty groups from the trace kernel's
  // first or last waves: as fast on C2, slower on C3 (profiles/r05/cull).
  const size_t wg0 = g - lane;  // the wave's first group
  if (wg0 < nGroups) {
    const size_t q0 = wg0 * PPW * 3;
    size_t q1 = (wg0 + 64) * PPW * 3;
    if (q1 > total * 3) q1 = total * 3;
    for (size_t q = q0 + lane; q < q1; q += 64) a.dst[q] = 0.f;
  }
  unsigned cost = 0;
  unsigned long long costAcc = 0;  // this lane's listed group: time (low 40), count
  if (a.costStat != nullptr && a.groupCost != nullptr && pc != 0u) {
    cost = a.groupCost[g];
    costAcc = (1ull << 40) | (unsigned long long)cost;
  }
  unsigned run;
  if (mu > 0.f) {
    const float c = (float)cost;
    if constexpr (kRuns == 8)  // short launches (KernelArgs::nRuns): finer longest-first order
      run = c >= 3.f * mu ? 0u : c >= 2.f * mu ? 1u : c >= 1.5f * mu ? 2u : c >= mu ? 3u
          : c >= 0.75f * mu ? 4u : c >= 0.5f * mu ? 5u : c >= 0.25f * mu ? 6u : 7u;
    else
      run = c >= 2.f * mu ? 0u : c >= mu ? 1u : c >= 0.5f * mu ? 2u : 3u;
  } else {
    run = pc >= a.lptMin ? 0u : 1u;
  }
  uint64_t live[kRuns];
#pragma unroll
  for (unsigned c = 0; c < kRuns; ++c) {
    live[c] = __ballot(pc != 0u && run == c);
    if (lane == 0) cnt[c][wave] = (unsigned)__builtin_popcountll(live[c]);
  }
  if (a.costStat != nullptr) {  // the wave's sum (butterfly), for this launch's stat
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) costAcc += __shfl_xor(costAcc, off, 64);
    if (lane == 0) waveCost[wave] = costAcc;
  }
  __syncthreads();
  if (threadIdx.x < kRuns) {
    const unsigned c = threadIdx.x;
    const unsigned sum = cnt[c][0] + cnt[c][1] + cnt[c][2] + cnt[c][3];
    blockBase[c] = sum ? atomicAdd(&groupCount[part * kCountStride + c], sum) : 0u;
  } else if (threadIdx.x == 64 && a.costStat != nullptr) {
    const unsigned long long t = waveCost[0] + waveCost[1] + waveCost[2] + waveCost[3];
    if (t) atomicAdd(a.costStat + part * kStatStride, t);
  }
  __syncthreads();
  const unsigned cap = a.groupCap;
  // runs 2k and 2k + 1 share [k cap, (k + 1) cap): the even one from the
  // front, the odd one from the back
  const size_t region = (size_t)part * (kRuns / 2u) * cap;
#pragma unroll
  for (unsigned c = 0; c < kRuns; ++c) {
    const uint64_t m = live[c];
    if ((m >> lane) & 1ull) {
      unsigned off = blockBase[c];  // list order: (wave, lane)
      for (unsigned w = 0; w < wave; ++w) off += cnt[c][w];
      const unsigned r = off + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
      const unsigned at = (c >> 1) * cap + ((c & 1u) ? cap - 1u - r : r);
      groupList[region + at] = (unsigned)g;
      groupSel[region + at] = sel;
    }
  }
}

static TraceFn pick_trace(int S, bool lds, int variant, bool bvh, int list) {
  switch (S) {
#define RTG_CASE(k) case k: return trace_fn_s##k(lds, variant, bvh, list);
    RTG_CASE(1) RTG_CASE(2) RTG_CASE(3) RTG_CASE(4) RTG_CASE(5) RTG_CASE(6) RTG_CASE(7)
    RTG_CASE(8) RTG_CASE(9) RTG_CASE(10) RTG_CASE(11) RTG_CASE(12) RTG_CASE(13)
    RTG_CASE(14) RTG_CASE(15) RTG_CASE(16)
#undef RTG_CASE
    default: return nullptr;
  }
}

}  // namespace rtg

struct rtg_context {
  int device = 0;
  unsigned n = 0, m = 0, n4 = 0;
  float4* geom = nullptr;
  float* crad2 = nullptr;
  float* mats = nullptr;
  float* lights = nullptr;
  unsigned* smask = nullptr;  // shadow masks (null when the scene has none)
  unsigned* cone = nullptr;   // secondary-ray cone masks (null when none)
  float* prim = nullptr;      // primary-cull sphere constants
  float* bvhNodes = nullptr;  // BVH node records (null when the scene has none)
  float* capRec = nullptr;    // sphere lists of BVH scenes (null when none)
  unsigned* capOff = nullptr;
  float* ovRec = nullptr;
  unsigned* ovOff = nullptr;
  unsigned* maxScratch = nullptr;
  unsigned long long* diag = nullptr;  // probe counters of diagnostic variants
  unsigned long long* counts = nullptr;  // unit counters of the counting build (variant 120)
  uint4* timeline = nullptr;  // RTG_LAUNCH_TIMELINE records
  // Compacted-launch scratch: a ring of slots, so that renders of one
  // context on different streams can overlap; a slot is reused only after
  // the event recorded behind its last trace kernel (a wait skipped when that
  // launch was on the same stream: stream order covers it).
  // One event per launch, the slot's: created without the system-scope fence
  // (hipEventDisableSystemFence), as it only orders this device's streams
  // (a record with the fence wrote L2 back: ~2 us between launches on C2).
  // Its buffers are stream-ordered allocations (hipMallocAsync / hipFreeAsync
  // behind the slot's event), so growing them never blocks the host or other
  // streams.  count holds two sets of the four run lengths, used by
  // alternate launches: each launch's trace kernel zeroes the other set for
  // the next one (KernelArgs::zeroCount), so no memset precedes a cull pass.
  struct GroupSlot {
    unsigned* list = nullptr;  // listed pixel groups
    unsigned long long* sel = nullptr;  // their primary-ray sphere masks
    unsigned* count = nullptr;  // [2][4]
    unsigned parity = 0;
    size_t cap = 0;
    hipEvent_t done = nullptr;
    hipStream_t stream = nullptr;  // of its last launch
  };
  static constexpr int kSlots = 4;
  GroupSlot slots[kSlots];
  int nextSlot = 0;
  // Launch-order feedback (cull_groups_kernel): per frame geometry, the
  // groups' measured trace times of its last launch and the last two
  // launches' sums; a few geometries at once (multi-GPU chunks render
  // different row sets in turn), least recently used replaced.
  // An entry's buffers are stream-ordered allocations too: a replaced entry's
  // table is freed on the launching stream behind its last launch, never with
  // a device-wide synchronisation.  That launch's event is its slot's (`slot`):
  // recorded again only by later launches, so waiting on it is conservative.
  struct CostEntry {
    unsigned long long key = 0;
    unsigned* cost = nullptr;
    size_t cap = 0;
    unsigned long long* stat = nullptr;  // [2]
    int cur = 0;
    unsigned launches = 0;
    unsigned long long lastUse = 0;
    int slot = -1;                 // the slot of its last launch
    hipStream_t stream = nullptr;  // and that launch's stream
  };
  static constexpr int kCostEntries = 8;
  CostEntry costs[kCostEntries];
  unsigned long long costClock = 0;
  unsigned sceneGen = 0;  // bumped by rtg_context_set_scene (part of the geometry key)
  bool orderFeedback = true;  // false: RTG_LAUNCH_ORDER=popcount (A/B knob)
  int numCU = 256;
  int persistPerCU = 0;  // > 0: fixed persistent waves per CU (RTG_PERSIST_PER_CU A/B knob)
  int lptMin = 2;        // heavy-first listing threshold (cull_groups_kernel; RTG_LPT_MIN A/B knob)
  size_t timelineCap = 0, timelineCount = 0;
  // The last committed compacted launch (rtg_diag_group_list): its slot,
  // pixel groups, list partitions' capacity (KernelArgs::groupCap) and cost
  // entry (or -1), all set at the launch's commit point only.
  int lastSlot = -1;
  size_t lastGroups = 0;
  size_t lastPartCap = 0;
  unsigned lastRuns = 4;
  int lastCost = -1;
  rtg_launch_opts opts{};
  int semantics = RTG_SEMANTICS_CPU;
  bool hasScene = false;
  // the last rtg_context_set_scene: host preparation ms (records, masks,
  // cone masks, BVH), upload ms, device bytes, BVH nodes (rtg_context_scene_stats)
  double sceneStats[4] = {0, 0, 0, 0};
};

using namespace rtg;

static void free_scene(rtg_context* c) {
  (void)hipFree(c->geom);
  (void)hipFree(c->crad2);
  (void)hipFree(c->mats);
  (void)hipFree(c->lights);
  (void)hipFree(c->smask);
  (void)hipFree(c->cone);
  c->cone = nullptr;
  (void)hipFree(c->prim);
  c->prim = nullptr;
  (void)hipFree(c->bvhNodes);
  (void)hipFree(c->capRec);
  (void)hipFree(c->capOff);
  (void)hipFree(c->ovRec);
  (void)hipFree(c->ovOff);
  c->capRec = nullptr;
  c->capOff = nullptr;
  c->ovRec = nullptr;
  c->ovOff = nullptr;
  c->smask = nullptr;
  c->bvhNodes = nullptr;
  c->geom = nullptr;
  c->crad2 = nullptr;
  c->mats = nullptr;
  c->lights = nullptr;
  c->hasScene = false;
}

// Argument checks shared by the one-shot entry points (no HIP call made).
static int check_render_args(const rtg_sphere* spheres, unsigned sphNum, const rtg_light* lights,
                             unsigned lgtNum, unsigned width, unsigned height, float zoom,
                             float aliasFactor, int stackSize, const void* dst) {
  if (!dst) {
    rtg_set_error("render: null destination");
    return RTG_ERR_INVALID;
  }
  if ((sphNum && !spheres) || (lgtNum && !lights)) {
    rtg_set_error("render: null scene array");
    return RTG_ERR_INVALID;
  }
  if (stackSize < 1 || stackSize > RTG_MAX_STACK) {
    rtg_set_error("stackSize %d outside [1, %d]", stackSize, RTG_MAX_STACK);
    return RTG_ERR_INVALID;
  }
  Camera cam;
  return make_camera(width, height, zoom, aliasFactor, &cam);
}

extern "C" {

int rtg_device_count(int* count) {
  rtg_clear_error();
  if (!count) return RTG_ERR_INVALID;
  HIP_TRY(hipGetDeviceCount(count));
  return RTG_OK;
}

int rtg_device_info(int device, char* buf, size_t buflen) {
  rtg_clear_error();
  if (!buf || buflen == 0) return RTG_ERR_INVALID;
  hipDeviceProp_t p;
  HIP_TRY(hipGetDeviceProperties(&p, device));
  snprintf(buf, buflen, "%s (%s), %d CUs, %d MHz, %.1f GiB, LDS/block %zu KiB", p.name,
           p.gcnArchName, p.multiProcessorCount, p.clockRate / 1000,
           (double)p.totalGlobalMem / (1024.0 * 1024.0 * 1024.0),
           (size_t)p.sharedMemPerBlock / 1024);
  return RTG_OK;
}

int rtg_context_create(int device, rtg_context** out) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!out) return RTG_ERR_INVALID;
  *out = nullptr;
  int cnt = 0;
  HIP_TRY(hipGetDeviceCount(&cnt));
  if (device < 0 || device >= cnt) {
    rtg_set_error("device %d not present (%d devices)", device, cnt);
    return RTG_ERR_NODEVICE;
  }
  HIP_TRY(hipSetDevice(device));
  rtg_context* c = new rtg_context();
  c->device = device;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
      cus > 0)
    c->numCU = cus;
  if (const char* v = getenv("RTG_PERSIST_PER_CU")) {  // A/B knob (performance only)
    const int k = atoi(v);
    if (k >= 1 && k <= 4096) c->persistPerCU = k;
  }
  if (const char* v = getenv("RTG_LPT_MIN")) {  // A/B knob (performance only; 65 = off)
    const int k = atoi(v);
    if (k >= 1 && k <= 65) c->lptMin = k;
  }
  if (const char* v = getenv("RTG_LAUNCH_ORDER")) {  // A/B knob (performance only)
    if (strcmp(v, "popcount") == 0) c->orderFeedback = false;
  }
  if (const char* v = getenv("RTG_VARIANT")) {  // A/B knob
    char* end = nullptr;
    const long var = strtol(v, &end, 10);
    const VariantInfo* vi = (end != v && *end == '\0') ? variant_info((int)var) : nullptr;
    if (!vi || vi->semantic) {
      delete c;
      rtg_set_error("RTG_VARIANT=%s is not a launch variant", v);
      return RTG_ERR_INVALID;
    }
    c->opts.variant = (int)var;
  }
  if (hipMalloc(&c->maxScratch, 4) != hipSuccess) {
    delete c;
    rtg_set_error("hipMalloc failed");
    return RTG_ERR_NOMEM;
  }
  *out = c;
  return RTG_OK;
}

int rtg_context_destroy(rtg_context* ctx) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!ctx) return RTG_OK;
  (void)hipSetDevice(ctx->device);
  free_scene(ctx);
  (void)hipFree(ctx->maxScratch);
  (void)hipFree(ctx->diag);
  (void)hipFree(ctx->counts);
  (void)hipFree(ctx->timeline);
  // stream-ordered allocations (launch_trace): freed on the null stream after
  // all work of the device that may still read them
  (void)hipDeviceSynchronize();
  for (auto& sl : ctx->slots) {
    if (sl.list) (void)hipFreeAsync(sl.list, nullptr);
    if (sl.sel) (void)hipFreeAsync(sl.sel, nullptr);
    if (sl.count) (void)hipFreeAsync(sl.count, nullptr);
    if (sl.done) (void)hipEventDestroy(sl.done);
  }
  for (auto& ce : ctx->costs) {
    if (ce.cost) (void)hipFreeAsync(ce.cost, nullptr);
    if (ce.stat) (void)hipFreeAsync(ce.stat, nullptr);
  }
  (void)hipStreamSynchronize(nullptr);
  delete ctx;
  return RTG_OK;
}

int rtg_diag_read(rtg_context* ctx, unsigned long long* out, int reset) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!ctx || !out) return RTG_ERR_INVALID;
  if (!ctx->diag) {
    for (int k = 0; k < 8; ++k) out[k] = 0;
    return RTG_OK;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, ctx->diag, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  if (reset) HIP_TRY(hipMemset(ctx->diag, 0, 8 * sizeof(unsigned long long)));
  return RTG_OK;
}

int rtg_context_scene_stats(rtg_context* ctx, double* out4) {
  rtg_clear_error();
  if (!ctx || !out4) return RTG_ERR_INVALID;
  for (int k = 0; k < 4; ++k) out4[k] = ctx->hasScene ? ctx->sceneStats[k] : 0.0;
  return RTG_OK;
}

int rtg_diag_counts(rtg_context* ctx, unsigned long long* out, int cap, int reset) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!ctx || (cap > 0 && !out)) return RTG_ERR_INVALID;
  const int n = 2 * kCntSlots;
  if (cap <= 0) return n;
  const int k = cap < n ? cap : n;
  if (!ctx->counts) {
    for (int i = 0; i < k; ++i) out[i] = 0;
    return n;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, ctx->counts, (size_t)k * sizeof(unsigned long long),
                    hipMemcpyDeviceToHost));
  if (reset) HIP_TRY(hipMemset(ctx->counts, 0, (size_t)n * sizeof(unsigned long long)));
  return n;
}

int rtg_diag_timeline(rtg_context* ctx, unsigned* out4, size_t cap, size_t* count) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!ctx || (cap && !out4) || !count) return RTG_ERR_INVALID;
  *count = ctx->timelineCount;
  const size_t k = cap < ctx->timelineCount ? cap : ctx->timelineCount;
  if (k == 0) return RTG_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out4, ctx->timeline, k * sizeof(uint4), hipMemcpyDeviceToHost));
  return RTG_OK;
}

int rtg_diag_group_list(rtg_context* ctx, unsigned* cost, unsigned* list,
                        unsigned long long* sel, unsigned* runs, size_t cap, size_t* groups) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!ctx || !groups) return RTG_ERR_INVALID;
  if (ctx->lastSlot < 0) {
    rtg_set_error("rtg_diag_group_list: no compacted launch yet");
    return RTG_ERR_INVALID;
  }
  const rtg_context::GroupSlot& slot = ctx->slots[ctx->lastSlot];
  if (!slot.count || !slot.list) {
    rtg_set_error("rtg_diag_group_list: no compacted launch yet");
    return RTG_ERR_INVALID;
  }
  *groups = ctx->lastGroups;
  const size_t k = cap < ctx->lastGroups ? cap : ctx->lastGroups;
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipDeviceSynchronize());
  if (cost) {
    // the last launch's own entry (none: the feedback was off for it)
    const rtg_context::CostEntry* ce = ctx->lastCost >= 0 ? &ctx->costs[ctx->lastCost] : nullptr;
    if (ce && ce->cost && ce->cap >= k) HIP_TRY(hipMemcpy(cost, ce->cost, k * sizeof(unsigned), hipMemcpyDeviceToHost));
    else memset(cost, 0, k * sizeof(unsigned));
  }
  if (!list && !sel && !runs) return RTG_OK;
  // the set the last launch used (its trace kernel zeroed the other one)
  std::vector<unsigned> cnt(kCountSet);
  HIP_TRY(hipMemcpy(cnt.data(), slot.count + kCountSet * (1 - slot.parity),
                    kCountSet * sizeof(unsigned), hipMemcpyDeviceToHost));
  const unsigned nR = ctx->lastRuns;  // 4 or 8 runs (eight: reported in pairs)
  if (runs)
    for (unsigned c = 0; c < 4; ++c) {
      runs[c] = 0;
      for (unsigned p = 0; p < kListParts; ++p)
        for (unsigned k = c * nR / 4; k < (c + 1) * nR / 4; ++k) runs[c] += cnt[p * kCountStride + k];
    }
  if (!list && !sel) return RTG_OK;
  std::vector<unsigned> l(slot.cap);
  std::vector<unsigned long long> m(slot.cap);
  HIP_TRY(hipMemcpy(l.data(), slot.list, slot.cap * sizeof(unsigned), hipMemcpyDeviceToHost));
  HIP_TRY(hipMemcpy(m.data(), slot.sel, slot.cap * sizeof(unsigned long long),
                    hipMemcpyDeviceToHost));
  // the trace kernel's order: index t is partition t % kListParts's
  // run-order entry t / kListParts (trace_samples_body)
  const size_t pc = ctx->lastPartCap;
  size_t most = 0;
  unsigned tot[kListParts];
  for (unsigned p = 0; p < kListParts; ++p) {
    const unsigned* g = &cnt[p * kCountStride];
    tot[p] = 0;
    for (unsigned k = 0; k < nR; ++k) tot[p] += g[k];
    if (tot[p] > most) most = tot[p];
  }
  size_t out = 0;
  for (size_t t = 0; t < most * kListParts && out < k; ++t) {
    const unsigned p = (unsigned)(t % kListParts);
    const size_t j = t / kListParts;
    if (j >= tot[p]) continue;
    const unsigned* g = &cnt[p * kCountStride];
    size_t jr = j, c = 0;  // run c, its entry jr
    while (jr >= g[c]) jr -= g[c++];
    const size_t r = (c >> 1) * pc + ((c & 1) ? pc - 1 - jr : jr);
    const size_t at = (nR / 2) * pc * p + r;
    if (list) list[out] = l[at];
    if (sel) sel[out] = m[at];
    ++out;
  }
  return RTG_OK;
}

int rtg_context_set_semantics(rtg_context* ctx, int semantics) {
  rtg_clear_error();
  if (!ctx || (semantics != RTG_SEMANTICS_CPU && semantics != RTG_SEMANTICS_OPENCL)) {
    rtg_set_error("rtg_context_set_semantics: invalid arguments");
    return RTG_ERR_INVALID;
  }
  ctx->semantics = semantics;
  return RTG_OK;
}

int rtg_set_launch_opts(rtg_context* ctx, const rtg_launch_opts* opts) {
  rtg_clear_error();
  if (!ctx || !opts) return RTG_ERR_INVALID;
  const VariantInfo* vi = variant_info(opts->variant);
  if (!vi || vi->semantic) {  // semantic variants: rtg_context_set_semantics only
    rtg_set_error("rtg_set_launch_opts: unknown kernel variant %d", opts->variant);
    return RTG_ERR_INVALID;
  }
  if (opts->flags & ~(RTG_LAUNCH_TIMELINE | RTG_LAUNCH_NO_ORDER_FEEDBACK)) {
    rtg_set_error("rtg_set_launch_opts: unknown flags 0x%x", (unsigned)opts->flags);
    return RTG_ERR_INVALID;
  }
  ctx->opts = *opts;
  return RTG_OK;
}

int rtg_context_set_scene(rtg_context* ctx, const rtg_sphere* spheres, unsigned sphNum,
                          const rtg_light* lights, unsigned lgtNum) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!ctx || (sphNum && !spheres) || (lgtNum && !lights)) {
    rtg_set_error("rtg_context_set_scene: invalid arguments");
    return RTG_ERR_INVALID;
  }
  // Table limits of the kernel: a frame record keeps the refractive material
  // index in 22 bits (FrameC::meta, rm << 10), and scene tables are addressed
  // with 32-bit byte offsets (fidx / uidx).  For n < RTG_MAX_SPHERES the
  // per-sphere tables end below 2^32 bytes (the fused records at 80 n bytes);
  // the BVH's octant copies take about 1 KB per node (~3/4 n nodes), and
  // build_bvh refuses a tree past 2^32 bytes (the scene then takes the flat
  // queries); the sphere lists, which grow as O(m n^2), are capped
  // separately (kListMaxRecords, sphere_lists: over it a scene has no lists
  // and its queries take the BVH).
  if (sphNum >= RTG_MAX_SPHERES) {
    rtg_set_error("rtg_context_set_scene: %u spheres (at most %u)", sphNum, RTG_MAX_SPHERES - 1);
    return RTG_ERR_INVALID;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  free_scene(ctx);
  using clk = std::chrono::steady_clock;
  const auto tPack = clk::now();
  PackedScene ps;
  pack_scene(spheres, sphNum, lights, lgtNum, &ps);
  const auto tUp = clk::now();
  std::vector<float4> geom(ps.geom.size() / 4);
  memcpy(geom.data(), ps.geom.data(), ps.geom.size() * sizeof(float));
  const std::vector<float>& crad2 = ps.crad2;
  const std::vector<float>& mats = ps.mats;
  const std::vector<float>& lg = ps.lights;
  if (hipMalloc(&ctx->geom, geom.size() * sizeof(float4)) != hipSuccess ||
      hipMalloc(&ctx->crad2, crad2.size() * sizeof(float)) != hipSuccess ||
      hipMalloc(&ctx->mats, mats.size() * sizeof(float)) != hipSuccess ||
      hipMalloc(&ctx->lights, lg.size() * sizeof(float)) != hipSuccess) {
    free_scene(ctx);
    rtg_set_error("hipMalloc failed for scene");
    return RTG_ERR_NOMEM;
  }
  HIP_TRY(hipMemcpy(ctx->geom, geom.data(), geom.size() * sizeof(float4),
                    hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(ctx->crad2, crad2.data(), crad2.size() * sizeof(float),
                    hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(ctx->mats, mats.data(), mats.size() * sizeof(float),
                    hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(ctx->lights, lg.data(), lg.size() * sizeof(float), hipMemcpyHostToDevice));
  if (!ps.smask.empty()) {
    if (hipMalloc(&ctx->smask, ps.smask.size() * sizeof(unsigned)) != hipSuccess) {
      free_scene(ctx);
      rtg_set_error("hipMalloc failed for shadow masks");
      return RTG_ERR_NOMEM;
    }
    HIP_TRY(hipMemcpy(ctx->smask, ps.smask.data(), ps.smask.size() * sizeof(unsigned),
                      hipMemcpyHostToDevice));
  }
  if (hipMalloc(&ctx->prim, ps.prim.size() * sizeof(float)) != hipSuccess) {
    free_scene(ctx);
    rtg_set_error("hipMalloc failed for the primary-cull constants");
    return RTG_ERR_NOMEM;
  }
  HIP_TRY(hipMemcpy(ctx->prim, ps.prim.data(), ps.prim.size() * sizeof(float),
                    hipMemcpyHostToDevice));
  if (!ps.cone.empty()) {
    if (hipMalloc(&ctx->cone, ps.cone.size() * sizeof(unsigned)) != hipSuccess) {
      free_scene(ctx);
      rtg_set_error("hipMalloc failed for cone masks");
      return RTG_ERR_NOMEM;
    }
    HIP_TRY(hipMemcpy(ctx->cone, ps.cone.data(), ps.cone.size() * sizeof(unsigned),
                      hipMemcpyHostToDevice));
  }
  if (!ps.bvhNodes.empty()) {
    if (hipMalloc(&ctx->bvhNodes, ps.bvhNodes.size() * sizeof(float)) != hipSuccess) {
      free_scene(ctx);
      rtg_set_error("hipMalloc failed for the BVH");
      return RTG_ERR_NOMEM;
    }
    HIP_TRY(hipMemcpy(ctx->bvhNodes, ps.bvhNodes.data(), ps.bvhNodes.size() * sizeof(float),
                      hipMemcpyHostToDevice));
  }
  if (!ps.capOff.empty()) {
    if (hipMalloc(&ctx->capRec, (ps.capRec.size() + 4 * kCapWords) * sizeof(float)) != hipSuccess ||
        hipMalloc(&ctx->capOff, ps.capOff.size() * sizeof(unsigned)) != hipSuccess ||
        hipMalloc(&ctx->ovRec, (ps.ovRec.size() + kListWords) * sizeof(float)) != hipSuccess ||
        hipMalloc(&ctx->ovOff, ps.ovOff.size() * sizeof(unsigned)) != hipSuccess) {
      free_scene(ctx);
      rtg_set_error("hipMalloc failed for the sphere lists");
      return RTG_ERR_NOMEM;
    }
    HIP_TRY(hipMemcpy(ctx->capRec, ps.capRec.data(), ps.capRec.size() * sizeof(float),
                      hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(ctx->capOff, ps.capOff.data(), ps.capOff.size() * sizeof(unsigned),
                      hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(ctx->ovRec, ps.ovRec.data(), ps.ovRec.size() * sizeof(float),
                      hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(ctx->ovOff, ps.ovOff.data(), ps.ovOff.size() * sizeof(unsigned),
                      hipMemcpyHostToDevice));
  }
  ctx->n = sphNum;
  ctx->m = lgtNum;
  ctx->n4 = ps.n4;
  ctx->hasScene = true;
  ++ctx->sceneGen;  // new geometry keys: no launch-order feedback from the old scene
  const auto tEnd = clk::now();
  ctx->sceneStats[0] = std::chrono::duration<double, std::milli>(tUp - tPack).count();
  ctx->sceneStats[1] = std::chrono::duration<double, std::milli>(tEnd - tUp).count();
  ctx->sceneStats[2] = (double)((ps.geom.size() + ps.crad2.size() + ps.mats.size() +
                                 ps.lights.size() + ps.prim.size() + ps.bvhNodes.size() +
                                 ps.capRec.size() + ps.ovRec.size()) *
                                    sizeof(float) +
                                (ps.smask.size() + ps.cone.size() + ps.capOff.size() +
                                 ps.ovOff.size()) *
                                    sizeof(unsigned));
  ctx->sceneStats[3] = (double)(ps.bvhNodes.size() / (kBvhWords * kBvhCopies));
  return RTG_OK;
}

// The launch-order feedback's key of a frame geometry: everything that
// decides which pixel group an index names and what it costs (FNV-1a; a
// collision only mis-orders a launch, the frame is the same).
static unsigned long long geometry_key(unsigned width, unsigned height, float zoom,
                                       float aliasFactor, int stackSize, unsigned rowBlock,
                                       unsigned shard, unsigned nShards, const unsigned* rowList,
                                       unsigned nRowList, int variant, unsigned sceneGen) {
  unsigned long long h = 1469598103934665603ull;
  auto mix = [&h](unsigned long long v) {
    for (int k = 0; k < 8; ++k) {
      h ^= (v >> (8 * k)) & 0xFFu;
      h *= 1099511628211ull;
    }
  };
  unsigned zb, ab;
  memcpy(&zb, &zoom, 4);
  memcpy(&ab, &aliasFactor, 4);
  mix(((unsigned long long)width << 32) | height);
  mix(((unsigned long long)zb << 32) | ab);
  mix(((unsigned long long)(unsigned)stackSize << 32) | rowBlock);
  mix(((unsigned long long)shard << 32) | nShards);
  mix((unsigned long long)(uintptr_t)rowList);
  mix(((unsigned long long)nRowList << 32) | (unsigned)variant);
  mix(sceneGen);
  return h;
}

static int launch_trace(rtg_context* ctx, unsigned width, unsigned height, float zoom,
                        float aliasFactor, int stackSize, unsigned rowBlock, unsigned shard,
                        unsigned nShards, const unsigned* rowList, unsigned nRowList,
                        rtg_vec* dstDevice, void* stream) {
  if (!ctx || !ctx->hasScene) {
    rtg_set_error("render: no context/scene");
    return RTG_ERR_INVALID;
  }
  bool ldsMats = ctx->n + 1 <= kLdsMatMax;
  if (stackSize < 1 || stackSize > RTG_MAX_STACK) {  // before anything is launched
    rtg_set_error("no kernel for stackSize %d (valid: 1..%d)", stackSize, RTG_MAX_STACK);
    return RTG_ERR_INVALID;
  }
  KernelArgs a;
  int rc = make_camera(width, height, zoom, aliasFactor, &a.cam);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(ctx->device));  // before any allocation below
  int variant = ctx->opts.variant;
  if (ctx->semantics == RTG_SEMANTICS_OPENCL) variant = 50;  // results differ: not a knob
  const VariantInfo* vi = variant_info(variant);
  if (!vi) {
    rtg_set_error("render: unknown kernel variant %d", variant);
    return RTG_ERR_INVALID;
  }
  // sample-parallel kernels need all of a pixel's samples in one wave
  if (vi->kind == kVariantSample && (a.cam.nAA < 1 || a.cam.nAA > 8)) {
    variant = variant == 110 ? 100 : variant == 50 ? 59 : 9;
    vi = variant_info(variant);
  }
  const bool sampleKernel = vi->kind == kVariantSample;
  // the default sample kernel reads materials/geometry from global memory
  // (L1/L2-resident), not from a per-workgroup LDS copy (as do the shipped
  // tile kernels 9, 59, 100); only the A/B variants below stage it
  if (!(variant == 1 || variant == 2 || variant == 3 || variant == 4 || variant == 5 ||
        variant == 6 || variant == 8 || variant == 14 || variant == 104 || variant == 108))
    ldsMats = false;
  unsigned rows;
  if (rowList) {
    rows = nRowList;
  } else {
    if (rowBlock == 0 || nShards == 0 || shard >= nShards) {
      rtg_set_error("render: bad sharding %u/%u block %u", shard, nShards, rowBlock);
      return RTG_ERR_INVALID;
    }
    rows = shard_row_count(height, rowBlock, shard, nShards);
  }
  if (rows == 0) return RTG_OK;
  if ((double)width * rows >= 0x1p53) {  // divmod_u64's range (rtg_trace_kernels.h)
    rtg_set_error("render: frame too large (%u x %u)", width, rows);
    return RTG_ERR_INVALID;
  }
  if (!dstDevice) {
    rtg_set_error("render: null destination");
    return RTG_ERR_INVALID;
  }
  a.geom = ctx->geom;
  a.crad2 = ctx->crad2;
  a.mats = ctx->mats;
  a.lights = ctx->lights;
  a.smask = ctx->smask;
  a.cone = ctx->cone;
  a.prim = ctx->prim;
  a.bvhNodes = ctx->bvhNodes;
  a.capRec = ctx->capRec;
  a.capOff = ctx->capOff;
  a.ovRec = ctx->ovRec;
  a.ovOff = ctx->ovOff;
  a.n = ctx->n;
  a.m = ctx->m;
  a.n4 = ctx->n4;
  a.W = width;
  a.rowsLocal = rows;
  a.rowBlock = rowBlock ? rowBlock : 1;
  a.invW = 1.0 / (double)width;
  a.invRowBlock = 1.0 / (double)a.rowBlock;
  a.shard = shard;
  a.nShards = nShards ? nShards : 1;
  a.rowList = rowList;
  a.dst = reinterpret_cast<float*>(dstDevice);
  a.diag = nullptr;
  a.counts = nullptr;
  a.timeline = nullptr;
  a.groupList = nullptr;
  a.groupSel = nullptr;
  a.groupCount = nullptr;
  a.groupCap = 0;
  a.nRuns = 4;
  a.lptMin = (unsigned)ctx->lptMin;
  a.nPersist = 0;
  a.groupCost = nullptr;
  a.costStat = nullptr;
  a.costPrev = nullptr;
  a.zeroCount = nullptr;
  a.zeroStat = nullptr;
  rtg_context::CostEntry* costEntry = nullptr;  // the feedback entry of this launch
  if (variant == 120) {  // executed-work counting build
    if (!ctx->counts) {
      HIP_TRY(hipMalloc(&ctx->counts, 2 * kCntSlots * sizeof(unsigned long long)));
      HIP_TRY(hipMemset(ctx->counts, 0, 2 * kCntSlots * sizeof(unsigned long long)));
    }
    a.counts = ctx->counts;
  } else if (variant >= 100) {
    if (!ctx->diag) {
      HIP_TRY(hipMalloc(&ctx->diag, 8 * sizeof(unsigned long long)));
      HIP_TRY(hipMemset(ctx->diag, 0, 8 * sizeof(unsigned long long)));
    }
    a.diag = ctx->diag;
  }
  unsigned threads = (unsigned)kBlock;
  dim3 grid((width + 15u) / 16u, (rows + 15u) / 16u);
  rtg_context::GroupSlot* slot = nullptr;  // compacted launch scratch
  int slotIdx = -1;
  bool listed = false;                     // compacted launch (kList kernel)
  size_t cullGroups = 0;                   // pixel groups of the cull pass
  if (sampleKernel) {
    const unsigned ppw = 64u / (unsigned)(a.cam.nAA * a.cam.nAA);  // >= 1: nAA <= 8 here
    const size_t groupsPerWave = variant == 21 ? 4 : 1;
    const size_t groups = ((size_t)width * rows + ppw - 1) / ppw;
    const size_t waves = (groups + groupsPerWave - 1) / groupsPerWave;
    const unsigned tpb = variant == 14 ? 256u : 64u;
    const size_t blocks = (waves + tpb / 64 - 1) / (tpb / 64);
    threads = tpb;
    if (blocks > 0x7FFFFFFFu) {
      rtg_set_error("render: frame too large (%zu workgroups)", blocks);
      return RTG_ERR_INVALID;
    }
    grid = dim3((unsigned)blocks, 1);
    // Compacted launch (the default; variant 22 and the multi-wave-workgroup
    // variants launch one wave per group instead): a cull pass writes the
    // groups no primary ray can leave (+0) and lists the others; a grid of
    // one-wave workgroups traces the listed groups round-robin.
    const bool compact = tpb == 64 && variant != 21 && variant != 22;
    // each list partition's capacity: the groups of its cull-pass blocks
    const size_t cullBlocks = (groups + 255) / 256;
    const size_t partCap = (cullBlocks + kListParts - 1) / kListParts * 256;
    // short launches (a multi-GPU frame's shard chunks) list their groups in
    // eight longest-first runs, whole frames in four
    const unsigned nRuns = groups <= kRuns8MaxGroups ? 8u : 4u;
    const size_t listCap = (nRuns / 2) * kListParts * partCap;  // list entries (KernelArgs::groupCap)
    if (compact && ctx->n <= 64 && listCap < 0xFFFFFFFFull) {
      listed = true;
      const hipStream_t st = (hipStream_t)stream;
      slotIdx = ctx->nextSlot;  // the ring advances at the commit below
      slot = &ctx->slots[slotIdx];
      if (!slot->done)
        HIP_TRY(hipEventCreateWithFlags(&slot->done,
                                        hipEventDisableTiming | hipEventDisableSystemFence));
      else if (slot->stream != st || st == hipStreamPerThread)
        // the slot's last launch; the per-thread default stream's handle names
        // a different stream in each host thread, so it always waits (a
        // context must not span a stream handle destroyed and reused while
        // its launches are pending: rtg.h)
        HIP_TRY(hipStreamWaitEvent(st, slot->done, 0));
      if (slot->cap < listCap) {
        // stream-ordered: freed after the slot's last kernel (waited on above)
        if (slot->list) HIP_TRY(hipFreeAsync(slot->list, st));
        if (slot->sel) HIP_TRY(hipFreeAsync(slot->sel, st));
        slot->list = nullptr;
        slot->sel = nullptr;
        slot->cap = 0;
        // the partitions' two halves (the four runs, KernelArgs::groupCount)
        HIP_TRY(hipMallocAsync((void**)&slot->list, listCap * sizeof(unsigned), st));
        HIP_TRY(hipMallocAsync((void**)&slot->sel, listCap * sizeof(unsigned long long), st));
        slot->cap = listCap;
      }
      if (!slot->count) {
        HIP_TRY(hipMallocAsync((void**)&slot->count, 2 * kCountSet * sizeof(unsigned), st));
        HIP_TRY(hipMemsetAsync(slot->count, 0, 2 * kCountSet * sizeof(unsigned), st));
        slot->parity = 0;
      }
      if (ctx->orderFeedback && !(ctx->opts.flags & RTG_LAUNCH_NO_ORDER_FEEDBACK)) {
        // launch-order feedback: this frame geometry's entry (LRU)
        const unsigned long long key = geometry_key(width, height, zoom, aliasFactor, stackSize,
                                                    rowBlock, shard, nShards, rowList, nRowList,
                                                    variant, ctx->sceneGen);
        rtg_context::CostEntry* ce = nullptr;
        for (auto& e : ctx->costs)
          if (e.launches && e.key == key) ce = &e;
        if (!ce) {
          ce = &ctx->costs[0];
          for (auto& e : ctx->costs)
            if (e.lastUse < ce->lastUse) ce = &e;
          // the replaced entry's buffers may still be read by queued launches
          // (any stream): this stream waits for its last one
          if (ce->slot >= 0 && (ce->stream != st || st == hipStreamPerThread))
            HIP_TRY(hipStreamWaitEvent(st, ctx->slots[ce->slot].done, 0));
          ce->key = 0;
          ce->launches = 0;
          if (ce->cap < groups) {
            if (ce->cost) HIP_TRY(hipFreeAsync(ce->cost, st));
            ce->cost = nullptr;
            ce->cap = 0;
            HIP_TRY(hipMallocAsync((void**)&ce->cost, groups * sizeof(unsigned), st));
            ce->cap = groups;
          }
          if (!ce->stat)
            HIP_TRY(hipMallocAsync((void**)&ce->stat, 2 * kStatSet * sizeof(unsigned long long), st));
          HIP_TRY(hipMemsetAsync(ce->stat, 0, 2 * kStatSet * sizeof(unsigned long long), st));
          ce->cur = 0;
          ce->key = key;
        } else {
          // launches of this entry on other streams may still add to or zero
          // its sums: this stream waits for the last one
          if (ce->stream != st || st == hipStreamPerThread)
            HIP_TRY(hipStreamWaitEvent(st, ctx->slots[ce->slot].done, 0));
        }
        // the trace kernel writes groupCost every launch; the cull pass reads
        // it (and sums it into costStat) once a launch has written it, and
        // orders by it once a cull pass has summed it (costPrev).  The entry's
        // own state (cur, launches) advances only once nothing can fail
        // (commit below).
        a.groupCost = ce->cost;
        a.costStat = ce->launches >= 1 ? ce->stat + kStatSet * ce->cur : nullptr;
        a.costPrev = ce->launches >= 2 ? ce->stat + kStatSet * (1 - ce->cur) : nullptr;
        const unsigned nextCur = ce->launches >= 1 ? 1u - ce->cur : ce->cur;
        // the next launch's costStat, zeroed by this launch's trace kernel
        a.zeroStat = ce->stat + kStatSet * nextCur;
        costEntry = ce;
      }
      cullGroups = groups;  // the cull pass is enqueued below, after the last failure point
      // about one wave per listed group: the benchmark scenes list 13-17 % of
      // their groups; a wave past the count exits at once, and a scene that
      // lists more deals up to five groups to each wave
      size_t persist = groups / 5;
      if (persist < (size_t)ctx->numCU * 64) persist = (size_t)ctx->numCU * 64;
      if (ctx->persistPerCU > 0) persist = (size_t)ctx->numCU * ctx->persistPerCU;
      a.groupList = slot->list;
      a.groupSel = slot->sel;
      a.groupCount = slot->count + kCountSet * slot->parity;
      a.zeroCount = slot->count + kCountSet * (1 - slot->parity);  // parity flips at the commit
      a.groupCap = (unsigned)partCap;
      a.nRuns = nRuns;
      // a multiple of kListParts (wave w takes list partition w % kListParts)
      const size_t np = groups < persist ? groups : persist;
      a.nPersist = (unsigned)((np + kListParts - 1) / kListParts * kListParts);
      grid = dim3(a.nPersist, 1);
    }
  }
  // the compacted default kernel of a scene with shadow/overlap and cone masks
  // takes them as compile-time facts (kMasks)
  const int listKind = !listed ? 0 : (ctx->smask && ctx->cone) ? 2 : 1;
  TraceFn fn = pick_trace(stackSize, ldsMats, variant, ctx->bvhNodes != nullptr, listKind);
  if (!fn) {
    rtg_set_error("no kernel for stackSize %d (valid: 1..%d), variant %d", stackSize,
                  RTG_MAX_STACK, variant);
    return RTG_ERR_INVALID;
  }
  // the frame levels the chosen kernel keeps in LDS (its kBvh instantiation
  // keeps one fewer, LdsFramesTop)
  const bool bvhKernel = ctx->bvhNodes != nullptr && has_bvh_kernel(variant);
  const size_t frameLds = (size_t)frame_lds_levels(stackSize, bvhKernel) * threads * 16;
  const size_t lds = frameLds +
                     (ldsMats ? ((size_t)(ctx->n + 1) * 8 * sizeof(float) + (size_t)ctx->n4 * 16)
                              : 0) +
                     (ctx->bvhNodes ? (size_t)(threads / 64) * 64 * sizeof(int) : 0);
  if (ctx->opts.flags & RTG_LAUNCH_TIMELINE) {
    const size_t waves = (size_t)grid.x * grid.y * (threads / 64);
    if (ctx->timelineCap < waves) {
      (void)hipFree(ctx->timeline);
      ctx->timeline = nullptr;
      ctx->timelineCap = 0;
      HIP_TRY(hipMalloc(&ctx->timeline, waves * sizeof(uint4)));
      ctx->timelineCap = waves;
    }
    ctx->timelineCount = waves;
    a.timeline = ctx->timeline;
  }
  // Commit: nothing below fails before the launch, so the slot's counter set
  // and the cost entry advance only now (an earlier error return leaves both
  // as the previous launch left them: its trace kernel zeroed exactly the set
  // this launch would have used).
  if (slot) {
    slot->parity ^= 1u;
    ctx->nextSlot = (slotIdx + 1) % rtg_context::kSlots;
    ctx->lastSlot = slotIdx;
    ctx->lastGroups = cullGroups;
    ctx->lastPartCap = a.groupCap;
    ctx->lastRuns = a.nRuns;
    ctx->lastCost = costEntry ? (int)(costEntry - ctx->costs) : -1;
  }
  if (costEntry) {
    costEntry->slot = slotIdx;
    costEntry->stream = (hipStream_t)stream;
    costEntry->lastUse = ++ctx->costClock;
    if (costEntry->launches >= 1) costEntry->cur = 1 - costEntry->cur;
    ++costEntry->launches;
  }
  // Stream work starts here, after every check and allocation that can fail,
  // so an error never leaves a cull pass (which zero-fills dst and fills the
  // slot's list) in flight without the slot's event behind it.
  // No memset: the counters this cull pass adds to were zeroed by the
  // previous launch's trace kernel (KernelArgs::zeroCount / zeroStat).
  if (slot) {
    const hipStream_t st = (hipStream_t)stream;
    const dim3 cgrid((unsigned)((cullGroups + 255) / 256));
    unsigned* cnt = const_cast<unsigned*>(a.groupCount);
    if (a.nRuns == 8)
      hipLaunchKernelGGL(cull_groups_kernel<8>, cgrid, dim3(256), 0, st, a, cullGroups,
                         slot->list, slot->sel, cnt);
    else
      hipLaunchKernelGGL(cull_groups_kernel<4>, cgrid, dim3(256), 0, st, a, cullGroups,
                         slot->list, slot->sel, cnt);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) {
      hipLaunchKernelGGL(fn, grid, dim3(threads), lds, st, a);
      e = hipGetLastError();
    }
    if (e != hipSuccess) {  // no trace kernel zeroed the next launch's counters
      (void)hipMemsetAsync(a.zeroCount, 0, kCountSet * sizeof(unsigned), st);
      if (a.zeroStat)
        (void)hipMemsetAsync(a.zeroStat, 0, kStatSet * sizeof(unsigned long long), st);
    }
    (void)hipEventRecord(slot->done, st);  // on every path (the cost entry's too)
    slot->stream = st;
    HIP_TRY(e);
    return RTG_OK;
  }
  hipLaunchKernelGGL(fn, grid, dim3(threads), lds, (hipStream_t)stream, a);
  HIP_TRY(hipGetLastError());
  return RTG_OK;
}

int rtg_render_device(rtg_context* ctx, unsigned width, unsigned height, float zoom,
                      float aliasFactor, int stackSize, unsigned rowBlock, unsigned shard,
                      unsigned nShards, rtg_vec* dstDevice, void* stream) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  return launch_trace(ctx, width, height, zoom, aliasFactor, stackSize, rowBlock, shard,
                      nShards, nullptr, 0, dstDevice, stream);
}

int rtg_render_rows_device(rtg_context* ctx, unsigned width, unsigned height, float zoom,
                           float aliasFactor, int stackSize, const unsigned* rowsDevice,
                           unsigned nRows, rtg_vec* dstDevice, void* stream) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (nRows && !rowsDevice) {
    rtg_set_error("rtg_render_rows_device: null row list");
    return RTG_ERR_INVALID;
  }
  if (nRows == 0) return RTG_OK;
  return launch_trace(ctx, width, height, zoom, aliasFactor, stackSize, 1, 0, 1, rowsDevice,
                      nRows, dstDevice, stream);
}

int rtg_render_rows(int device, const rtg_sphere* spheres, unsigned sphNum,
                    const rtg_light* lights, unsigned lgtNum, unsigned width, unsigned height,
                    float zoom, float aliasFactor, int stackSize, const unsigned* rows,
                    unsigned nRows, rtg_vec* dstHost) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (nRows && (!rows || !dstHost)) {
    rtg_set_error("rtg_render_rows: null argument");
    return RTG_ERR_INVALID;
  }
  if (nRows) {
    int rc0 = check_render_args(spheres, sphNum, lights, lgtNum, width, height, zoom,
                                aliasFactor, stackSize, dstHost);
    if (rc0) return rc0;
  }
  for (unsigned k = 0; k < nRows; ++k)
    if (rows[k] >= height) {
      rtg_set_error("rtg_render_rows: row %u >= height %u", rows[k], height);
      return RTG_ERR_INVALID;
    }
  if (nRows == 0) return RTG_OK;
  rtg_context* ctx = nullptr;
  int rc = rtg_context_create(device, &ctx);
  if (rc) return rc;
  rtg_vec* d = nullptr;
  unsigned* drows = nullptr;
  const size_t bytes = (size_t)width * nRows * sizeof(rtg_vec);
  rc = rtg_context_set_scene(ctx, spheres, sphNum, lights, lgtNum);
  if (!rc && (hipMalloc(&d, bytes) != hipSuccess ||
              hipMalloc(&drows, nRows * sizeof(unsigned)) != hipSuccess)) {
    rtg_set_error("hipMalloc failed");
    rc = RTG_ERR_NOMEM;
  }
  if (!rc && hipMemcpy(drows, rows, nRows * sizeof(unsigned), hipMemcpyHostToDevice) !=
                 hipSuccess) {
    rtg_set_error("row list upload failed");
    rc = RTG_ERR_HIP;
  }
  if (!rc)
    rc = rtg_render_rows_device(ctx, width, height, zoom, aliasFactor, stackSize, drows, nRows,
                                d, nullptr);
  if (!rc) {
    hipError_t e = hipMemcpy(dstHost, d, bytes, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      rtg_set_error("kernel/readback failed: %s", hipGetErrorString(e));
      rc = RTG_ERR_HIP;
    }
  }
  (void)hipFree(d);
  (void)hipFree(drows);
  rtg_context_destroy(ctx);
  return rc;
}

int rtg_max_colour_device(rtg_context* ctx, const rtg_vec* pixelsDevice, size_t n,
                          float* maxDevice, void* stream) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!ctx || !maxDevice || (n && !pixelsDevice)) return RTG_ERR_INVALID;
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipMemsetAsync(maxDevice, 0, sizeof(float), s));
  if (n) {
    const size_t nval = n * 3;
    size_t blocks = (nval + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(max_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const float*)pixelsDevice, nval, (unsigned*)maxDevice);
    HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(max_finish_kernel, dim3(1), dim3(1), 0, s, (unsigned*)maxDevice);
  HIP_TRY(hipGetLastError());
  return RTG_OK;
}

int rtg_assemble_shards_device(rtg_context* ctx, const rtg_vec* gathered, unsigned nShards,
                               unsigned paddedRows, unsigned width, unsigned height,
                               unsigned rowBlock, rtg_vec* frame, void* stream) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!ctx || !gathered || !frame || nShards == 0 || rowBlock == 0 || width == 0 ||
      height == 0) {
    rtg_set_error("rtg_assemble_shards_device: invalid arguments");
    return RTG_ERR_INVALID;
  }
  const unsigned nb = (height + rowBlock - 1) / rowBlock;
  const unsigned need = ((nb + nShards - 1) / nShards) * rowBlock;
  if (paddedRows < need) {
    rtg_set_error("rtg_assemble_shards_device: paddedRows %u < %u", paddedRows, need);
    return RTG_ERR_INVALID;
  }
  if (nb > 65535u) {
    rtg_set_error("rtg_assemble_shards_device: %u row blocks (max 65535)", nb);
    return RTG_ERR_INVALID;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t rowBytes = (size_t)width * sizeof(rtg_vec);
  const size_t perBlock = rowBytes * rowBlock;
  unsigned gx = (unsigned)((perBlock / 16 + 255) / 256);
  if (gx > 64) gx = 64;
  if (gx == 0) gx = 1;
  const dim3 grid(gx, nb);
  const bool v16 = rowBytes % 16 == 0 && ((uintptr_t)gathered % 16 == 0) &&
                   ((uintptr_t)frame % 16 == 0);
  if (v16)
    hipLaunchKernelGGL(assemble_kernel<uint4>, grid, dim3(256), 0, st,
                       (const uint4*)gathered, (uint4*)frame, nShards, paddedRows, height,
                       rowBlock, rowBytes / 16);
  else
    hipLaunchKernelGGL(assemble_kernel<unsigned>, grid, dim3(256), 0, st,
                       (const unsigned*)gathered, (unsigned*)frame, nShards, paddedRows, height,
                       rowBlock, rowBytes / 4);
  HIP_TRY(hipGetLastError());
  return RTG_OK;
}

int rtg_place_shard_device(rtg_context* ctx, const rtg_vec* shard, unsigned shardIdx,
                           unsigned nShards, unsigned width, unsigned height, unsigned rowBlock,
                           rtg_vec* frame, void* stream) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!ctx || !shard || !frame || nShards == 0 || shardIdx >= nShards || rowBlock == 0 ||
      width == 0 || height == 0) {
    rtg_set_error("rtg_place_shard_device: invalid arguments");
    return RTG_ERR_INVALID;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  // shard block j holds global row block j G + g (rtg_shard_rows packing)
  const size_t nb = (height + rowBlock - 1) / rowBlock;
  const size_t rowBytes = (size_t)width * sizeof(rtg_vec);
  const size_t blockBytes = rowBytes * rowBlock;
  const size_t fullBlocks = height / rowBlock;  // global blocks of rowBlock rows
  size_t nFull = 0;                             // this shard's full blocks
  if (fullBlocks > shardIdx) nFull = (fullBlocks - shardIdx + nShards - 1) / nShards;
  hipStream_t st = (hipStream_t)stream;
  if (nFull > 0)
    HIP_TRY(hipMemcpy2DAsync((char*)frame + (size_t)shardIdx * blockBytes,
                             blockBytes * nShards, shard, blockBytes, blockBytes, nFull,
                             hipMemcpyDeviceToDevice, st));
  const size_t gb = nFull * nShards + shardIdx;  // a ragged last block of this shard
  if (gb < nb) {
    const size_t rows = height - gb * rowBlock;
    HIP_TRY(hipMemcpyAsync((char*)frame + gb * blockBytes, (const char*)shard + nFull * blockBytes,
                           rows * rowBytes, hipMemcpyDeviceToDevice, st));
  }
  return RTG_OK;
}

int rtg_ppm_bytes_device(rtg_context* ctx, const rtg_vec* pixelsDevice, size_t n,
                         const float* maxDevice, unsigned char* outDevice, void* stream) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  if (!ctx || !maxDevice || (n && (!pixelsDevice || !outDevice))) return RTG_ERR_INVALID;
  if (n == 0) return RTG_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  const size_t nval = n * 3;
  size_t blocks = (nval + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(ppm_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (const float*)pixelsDevice, nval, maxDevice, outDevice);
  HIP_TRY(hipGetLastError());
  return RTG_OK;
}

int rtg_render(int device, const rtg_sphere* spheres, unsigned sphNum, const rtg_light* lights,
               unsigned lgtNum, unsigned width, unsigned height, float zoom, float aliasFactor,
               int stackSize, rtg_vec* dstHost) {
  DeviceGuard deviceGuard;  // the caller's current device is restored on return
  rtg_clear_error();
  int rc0 = check_render_args(spheres, sphNum, lights, lgtNum, width, height, zoom, aliasFactor,
                              stackSize, dstHost);
  if (rc0) return rc0;
  rtg_context* ctx = nullptr;
  int rc = rtg_context_create(device, &ctx);
  if (rc) return rc;
  rtg_vec* d = nullptr;
  const size_t bytes = (size_t)width * height * sizeof(rtg_vec);
  rc = rtg_context_set_scene(ctx, spheres, sphNum, lights, lgtNum);
  if (!rc && hipMalloc(&d, bytes ? bytes : 4) != hipSuccess) {
    rtg_set_error("hipMalloc(%zu) failed", bytes);
    rc = RTG_ERR_NOMEM;
  }
  if (!rc)
    rc = rtg_render_device(ctx, width, height, zoom, aliasFactor, stackSize, 16, 0, 1, d,
                           nullptr);
  if (!rc) {
    hipError_t e = hipMemcpy(dstHost, d, bytes, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      rtg_set_error("kernel/readback failed: %s", hipGetErrorString(e));
      rc = RTG_ERR_HIP;
    }
  }
  (void)hipFree(d);
  rtg_context_destroy(ctx);
  return rc;
}

}  // extern "C"
