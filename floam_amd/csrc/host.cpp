// Host control of the MI355X-native FLOAM core + the C ABI (include/floam_c.h).
//
// floam_lp   = LaserProcessingClass   (include/laserProcessingClass.h:37-50)
// floam_odom = OdomEstimationClass    (include/odomEstimationClass.h:52-126, src/odomEstimationClass.cpp)
//
// All device work of one device is issued on one HIP stream.  Per updatePointsToMap call the host issues a fixed
// kernel sequence (downsample, [grid rebuild], optimization_count x {lm_init + correspondences, 5 x {LM evaluate,
// LM control}}) and synchronises once, to read the pose back — the reference exposes `odom` to its caller after
// every call (src/odomEstimationNode.cpp:242-244).  The keyframe decision and the map update follow on the host
// / device respectively.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "cloud_ops.hpp"
#include "fe.hpp"
#include "floam_common.hpp"
#include "formats.hpp"
#include "imu.hpp"
#include "mapmerge.hpp"
#include "mapping.hpp"
#include "odom_kernels.hpp"
#include "pose.hpp"
#include "voxel.hpp"
#include <unordered_map>

namespace floam {

// ----------------------------------------------------------------------------------------- device context
struct PendingTiming {
  std::string name;
  hipEvent_t e0, e1;
  double bytes;
};

struct DeviceCtx {
  int device = 0;
  hipStream_t stream = nullptr;
  VoxelScratch2 vs;           // standalone floam_voxel_grid
  DevBuf<int> zero;           // a device 0 (empty second job)
  DevBuf<int> ends;           // {count, front.time, back.time} read-back of the IMU pre-processing
  DevBuf<uint8_t> msg;        // staged PointCloud2 bytes (floam_cloud_from_pointcloud2)
  HostBuf<int> h_ends;
  int profile = 0;   // bitmask of FLOAM_PROF_* categories
  std::vector<PendingTiming> pending;
  std::vector<hipEvent_t> free_events;
  std::map<std::string, floam_kernel_timing> totals;
  // end-of-update events, recycled round-robin: one record per update serves every consumer of that point of the
  // stream (the host's collection, the next extraction into the update's clouds, the side stream's buffer reuse).
  // A record is a barrier packet that costs the stream several us, so it is issued once.  An event re-recorded by a
  // later update only makes a late waiter wait for a later point of the same stream (never too early); 64 updates
  // separate two records of one event (the deepest asynchronous ring is 16).
  hipEvent_t update_ev[64] = {};
  unsigned update_ev_next = 0;
  hipEvent_t next_update_event() {
    hipEvent_t& e = update_ev[update_ev_next++ % 64];
    if (!e) FLOAM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
  }

  hipEvent_t get_event() {
    if (!free_events.empty()) {
      hipEvent_t e = free_events.back();
      free_events.pop_back();
      return e;
    }
    hipEvent_t e;
    FLOAM_HIP(hipEventCreate(&e));
    return e;
  }
  void drain() {
    for (auto& p : pending) {
      float ms = 0.f;
      FLOAM_HIP(hipEventSynchronize(p.e1));
      FLOAM_HIP(hipEventElapsedTime(&ms, p.e0, p.e1));
      auto& t = totals[p.name];
      std::strncpy(t.name, p.name.c_str(), sizeof(t.name) - 1);
      t.launches += 1;
      t.total_ms += ms;
      t.algorithmic_bytes += p.bytes;
      free_events.push_back(p.e0);
      free_events.push_back(p.e1);
    }
    pending.clear();
  }
};

static std::mutex g_ctx_mu;
static std::map<int, std::unique_ptr<DeviceCtx>> g_ctx;

static void make_stream(hipStream_t* s, bool /*high*/) {
  FLOAM_HIP(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
}


static DeviceCtx& ctx_for(int device) {
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  auto it = g_ctx.find(device);
  if (it != g_ctx.end()) return *it->second;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
    throw Error(FLOAM_ERR_DEVICE, "no HIP device available (the floam_amd core needs an MI355X / gfx950 GPU)");
  if (device < 0 || device >= n) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "device index out of range");
  FLOAM_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  FLOAM_HIP(hipGetDeviceProperties(&prop, device));
  if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0)
    throw Error(FLOAM_ERR_DEVICE, std::string("device is ") + prop.gcnArchName + ", this build targets gfx950");
  auto c = std::make_unique<DeviceCtx>();
  c->device = device;
  make_stream(&c->stream, true);
  DeviceCtx& ref = *c;
  g_ctx[device] = std::move(c);
  return ref;
}

// Records HIP events around a launch sequence on the library stream when profiling is on.
struct ProfScope {
  DeviceCtx& c;
  const char* name;
  double bytes;
  hipEvent_t e0 = nullptr;
  hipStream_t s;
  ProfScope(DeviceCtx& ctx, const char* n, int category, double b = 0.0, hipStream_t stream = nullptr)
      : c(ctx), name(n), bytes(b), s(stream ? stream : ctx.stream) {
    if (c.profile & category) {
      e0 = c.get_event();
      FLOAM_HIP(hipEventRecord(e0, s));
    }
  }
  ~ProfScope() {
    if (e0) {
      hipEvent_t e1 = c.get_event();
      (void)hipEventRecord(e1, s);
      c.pending.push_back(PendingTiming{name, e0, e1, bytes});
    }
  }
};

// ----------------------------------------------------------------------------------------- cloud helpers
// Cross-stream ordering of the operations on a cloud.  The feature extraction runs on its handle's own stream (so
// the next scan's extraction overlaps the current scan's odometry, as the reference's laserProcessingNode runs beside
// odomEstimationNode); every other operation runs on the device stream.  Before an operation on stream s, s waits
// for the cloud's last operation if that ran on another stream: for the side stream the event was recorded right
// after its operation (cloud_publish), for the device stream it is recorded when needed (all of the stream's work
// issued so far, the cloud's last operation included).
static void cloud_on(const floam_cloud* cc, hipStream_t s) {
  auto* c = const_cast<floam_cloud*>(cc);
  const bool complete = c->done_ctr && *c->done_ctr >= c->done_seq;   // its last update has been collected
  if (c->last_stream && c->last_stream != s && !complete) {
    hipEvent_t e = c->ev_valid ? c->ext_ev : nullptr;
    if (!e) {
      if (!c->ev) FLOAM_HIP(hipEventCreateWithFlags(&c->ev, hipEventDisableTiming));
      if (!c->ev_valid) FLOAM_HIP(hipEventRecord(c->ev, c->last_stream));
      e = c->ev;
    }
    FLOAM_HIP(hipStreamWaitEvent(s, e, 0));
  }
  c->last_stream = s;
  c->ev_valid = false;
  c->ext_ev = nullptr;
  c->done_ctr.reset();
  if (c->clear_pending) {
    FLOAM_HIP(hipMemsetAsync(c->count.p, 0, sizeof(int), s));
    c->clear_pending = false;
  }
}
static void cloud_on_main(const floam_cloud* c) { cloud_on(c, ctx_for(c->device).stream); }
static void cloud_publish(const floam_cloud* cc, hipStream_t s) {   // after an operation on a side stream
  auto* c = const_cast<floam_cloud*>(cc);
  if (!c->ev) FLOAM_HIP(hipEventCreateWithFlags(&c->ev, hipEventDisableTiming));
  FLOAM_HIP(hipEventRecord(c->ev, s));
  c->last_stream = s;
  c->ev_valid = true;
  c->ext_ev = nullptr;
}
// after odometry update `seq` of a handle with collection counter ctr: a consumer on another stream skips the wait
// once the update has been collected; before that it waits on `recorded` (the update's end event) if there is one,
// else on an event recorded then on s (a later point of the same stream: correct, only later than needed)
static void cloud_publish_update(const floam_cloud* cc, hipStream_t s, hipEvent_t recorded,
                                 const std::shared_ptr<unsigned long long>& ctr, unsigned long long seq) {
  auto* c = const_cast<floam_cloud*>(cc);
  c->last_stream = s;
  c->ev_valid = recorded != nullptr;
  c->ext_ev = recorded;
  c->done_ctr = ctr;
  c->done_seq = seq;
}

static size_t cloud_count_sync(const floam_cloud* c) {
  if (c->host_count_valid) return c->host_count;
  cloud_on_main(c);
  DeviceCtx& ctx = ctx_for(c->device);
  int v = 0;
  FLOAM_HIP(hipMemcpyAsync(&v, c->count.p, sizeof(int), hipMemcpyDeviceToHost, ctx.stream));
  FLOAM_HIP(hipStreamSynchronize(ctx.stream));
  if (v < 0) throw Error(FLOAM_ERR_DEVICE, "device-side compaction failed (lookback timeout)");
  auto* mc = const_cast<floam_cloud*>(c);
  mc->host_count = (size_t)v;
  mc->host_count_valid = true;
  return mc->host_count;
}

// host upper bound of a cloud's size without synchronising (exact when the host knows the count)
static size_t cloud_ub(const floam_cloud* c) { return c->host_count_valid ? c->host_count : c->ub; }

// grow keeping the first `keep` points (stream-ordered copy, then the old buffer is freed after a sync)
static void cloud_reserve(floam_cloud* c, size_t n, size_t keep, hipStream_t st) {
  if (n <= c->pts.cap) return;
  const size_t cap = n < 4096 ? std::max<size_t>(n + n / 2, 1024) : std::max<size_t>(2 * n, (size_t)1 << 20);
  if (DevBuf<int>::alloc_log()) std::fprintf(stderr, "[floam alloc] cloud %zu pts (had %zu)\n", n, c->pts.cap);
  PointRec* p = nullptr;
  FLOAM_HIP(hipMalloc(&p, cap * sizeof(PointRec)));
  if (keep && c->pts.p) {
    FLOAM_HIP(hipMemcpyAsync(p, c->pts.p, keep * sizeof(PointRec), hipMemcpyDeviceToDevice, st));
    if (!capture_state().active) FLOAM_HIP(hipStreamSynchronize(st));
  }
  dev_free(c->pts.p);   // deferred while capturing (the copy above runs first)
  c->pts.p = p;
  c->pts.cap = cap;
}

static void cloud_init(floam_cloud* c, int device, size_t capacity) {
  c->device = device;
  c->count.reserve(1);
  DeviceCtx& ctx = ctx_for(device);
  FLOAM_HIP(hipMemsetAsync(c->count.p, 0, sizeof(int), ctx.stream));
  c->last_stream = ctx.stream;
  c->host_count = 0;
  c->host_count_valid = true;
  if (capacity) cloud_reserve(c, capacity, 0, ctx.stream);
}

// exchange the device storage of two clouds (stream-ordered users see the new contents after the swap)
static void cloud_swap(floam_cloud* a, floam_cloud* b) {
  std::swap(a->pts.p, b->pts.p);
  std::swap(a->pts.cap, b->pts.cap);
  std::swap(a->count.p, b->count.p);
  std::swap(a->count.cap, b->count.cap);
}

static bool g_keyframe_first = true;   // KeyFrameUpdate's function-static `first` (odomEstimationClass.cpp:323, Q6)

}  // namespace floam

using namespace floam;

// ============================================================================================ handles
struct floam_lp {
  int device = 0;
  FeParams prm{};
  FeScratch sc;
  DevBuf<int> status;
  HostBuf<int> h_out;   // edge count, surf count, status
  bool async = false;   // floam_lp_set_async: no synchronisation, counts stay on the device (upper bounds on host)
  hipStream_t stream = nullptr;   // the extraction's own stream (overlaps the odometry on the device stream)
  // floam_lp_feature_extraction_host: the device copies of the caller's cloud and of the two outputs
  std::unique_ptr<floam_cloud> h_in, h_edge, h_surf;
};

struct floam_odom {
  int device = 0;
  floam_lidar_params lp{};
  double map_resolution = 0.4;
  bool huber = false;
  float leafE = 0.4f, leafS = 0.8f;
  // local map (device) and host-known exact sizes (valid as of the last synchronisation)
  floam_cloud mapE, mapS;
  floam_cloud mapE_next, mapS_next;   // double buffers: the map update writes here, then the two swap
  // the maps' cell keys (mapmerge.hpp: the incremental map update), double-buffered with the maps: [map][buffer],
  // buffer mkcur the current one; mmeta: what the keys are worth (invalid after initMapWithPoints: a raw map)
  DevBuf<unsigned long long> mkeys[2][2];
  DevBuf<MapMeta> mmeta[2][2];
  int mkcur = 0;
  MapMergeScratch mms;
  bool map_merge = true;          // FLOAM_MAP_MERGE=0: the whole-map VoxelGrid of round 2 (A/B)
  bool map_force_full = false;    // FLOAM_MAP_FULL=1: the merge pipeline always takes its full-sort path (tests)
  int map_violate_mod = 0;        // FLOAM_MM_VIOLATE=n: every n-th merge reports its keys out of order (tests)
  size_t mapE_n = 0, mapS_n = 0;   // map sizes: exact after a synchronisation, else upper bounds
  // scratch
  DevBuf<PointRec> dE, dS, tmp;
  DevBuf<int> cnt;   // [0] dE count [1] dS count [2] tmp count
  VoxelScratch2 vs;
  Grid gE, gS;
  bool grid_dirty = true;
  CorrSet ce, cs;
  bool fp32 = false;                       // floam_odom_set_precision: fp32 residuals / Jacobians (C5 sweep)
  bool fp32_geom = false;                  // ... and fp32 line / plane fits (FLOAM_PRECISION_FP32_GEOMETRY)
  LMBuffers lmb;                           // the solves' scratch (lm.hip)
  DevBuf<unsigned long long> dbg_stamps;   // FLOAM_DEBUG_STAMPS=1: the resident solve's segment times (diagnostic)
  int qhint[2] = {0, 0};                   // recent downsampled edge / surf query counts (search grid sizing)
  // stage inspection (floam_odom_set_trace): one record per solve, and the last correspondence pass's queries
  int trace_cap = 0;
  DevBuf<double> trace;
  DevBuf<unsigned> trace_count;
  const PointRec* last_q[2] = {nullptr, nullptr};   // the last pass's query clouds (downsampled, sensor frame)
  const int* last_qn = nullptr;                     // their device counts
  bool last_traced = false;                         // that pass wrote neighbour indices / distances (tracing on)
  DevBuf<double> kf_io;                             // floam_odom_keyframe_update: pose in, flag out
  // keyframes_ (include/odomEstimationClass.h:116-117, 3 deep): the pose of every keyframe and, for the public
  // KeyFrameUpdate, device copies of the clouds it was given.  The updates' own keyframes keep the pose only (their
  // downsampled clouds are private in the reference and never read back); the decision itself reads the last
  // keyframe pose from the device state (OdomDev)
  struct Keyframe {
    Pose pose;
    floam_cloud* surf = nullptr;
    floam_cloud* edge = nullptr;
  };
  std::deque<Keyframe> keyframes;
  std::vector<floam_cloud*> kf_spare;               // clouds of dropped history entries, reused
  bool next_kf_first = false;                       // the update being issued consumed the process-wide `first`
  DevBuf<LMState> lm;
  // call 1 of a deskewed selector downsamples the edge cloud only (Q4), in the sensor frame: that VoxelGrid runs on a
  // side stream as soon as the scan's features exist, overlapped with the previous update (double-buffered by parity)
  hipStream_t side = nullptr;
  hipEvent_t side_ev[2] = {nullptr, nullptr};     // call-1 buffers of a parity consumed: the end of the update that
                                                  // used them (a shared end-of-update event, DeviceCtx::update_ev)
  hipEvent_t end_ev = nullptr;                    // the end-of-update event of the last issued update (if recorded)
  unsigned long long collected_seq = 0;           // serial number of the last collected update (updates complete in
                                                  // order: every update up to it is done); shared with the clouds
  std::shared_ptr<unsigned long long> done_ctr = std::make_shared<unsigned long long>(0);
  unsigned long long side_seq[2] = {0, 0};        // the update that last read each parity's call-1 buffers
  hipEvent_t pre_ev = nullptr;                    // the side stream's call-1 VoxelGrids done (both clouds' producers)
  bool side_ev_rec[2] = {false, false};
  DevBuf<PointRec> pE[2], pS[2];
  DevBuf<int> pcnt[2];
  VoxelScratch2 vs1;
  int pre_par = 0;
  int pre_valid = -1;                             // parity of the pre-downsampled call-1 clouds awaiting their update
  // clouds the main stream orders itself after only once the grid rebuild is issued (pre-downsampled call 1: the
  // rebuild reads neither cloud, so it runs while the side stream finishes)
  const floam_cloud* late_wait[2] = {nullptr, nullptr};
  // status slots, two per in-flight update (first / only call, second call of a deskewed selector)
  // written by the gather kernel straight into coherent pinned host memory (no copy launch on the stream); 32 slots
  // cover the deepest ring (depth 16), so the buffer never moves while updates are in flight
  HostBuf<UpdateStatus> h_ustat;
  DevBuf<OdomDev> ds;             // device-resident controller state (poses, keyframe)
  // updates issued but not yet collected (asynchronous mode keeps up to `depth` of them in flight)
  struct Pending {
    int ring;                     // status slots [2 ring, 2 ring + nslots)
    int nslots;
    int map_slot;                 // slot whose map counts precede this update's map update (-1: no map update)
    size_t addE, addS;            // upper bounds of the points the map update may add
    hipEvent_t ev;
    std::vector<void*> graveyard; // device buffers replaced while the update was captured (freed once it ran)
    bool kf_first;                // its keyframe decision took KeyFrameUpdate's `first` branch (no history trim)
    unsigned long long seq;       // its serial number (o->issued), stored last in each of its status slots
  };
  std::deque<Pending> inflight;
  int depth = 0;                  // floam_odom_set_async: 0 = every update synchronises (the reference's contract)
  unsigned long long issued = 0;
  size_t pendE = 0, pendS = 0;    // sum of addE / addS over the in-flight updates
  std::vector<double> collected;  // poses {q, t} of the updates collected since the last floam_odom_wait
  // each update is captured into a hipGraph and the executable graph of its kind updated in place
  // (hipGraphExecUpdate): one launch per update, and back-to-back kernel dispatch on the device
  bool use_graph = false;         // FLOAM_GRAPH=1 enables
  // [kind][k]: kind 0 updatePointsToMap, 1 deskewed selector; update i uses k = i % (depth + 1), so an executable
  // graph is never updated while a launch of it may still be in flight
  static constexpr int kExecRing = 17;
  hipGraphExec_t graph_exec[2][kExecRing] = {};
  DevBuf<unsigned long long> prof_bytes;
  DevBuf<unsigned long long> traffic_set;
  DevBuf<float4> knn_evict;   // FLOAM_KNN_STAGES (diagnostic): the L2 eviction buffer of knn_stage_launch
  bool prof_bytes_init = false;
  // host mirror of the controller poses, as of the last collected update
  Pose odom = pose_identity(), last_odom = pose_identity();
  int optimization_count = 2;
  // sharding
  int rank = 0, world = 1;
  ncclComm_t comm = nullptr;
  floam_allreduce_fn ar_fn = nullptr;   // host all-reduce (validation mode), used when comm is null
  void* ar_user = nullptr;
  HostBuf<double> h_sums;
  // peer sharding (floam_odom_set_shard_peers): this rank's exchange buffer, the ranks' buffers as mapped here, and
  // the IPC mappings to close
  unsigned long long* xbuf = nullptr;
  DevBuf<int> probe;   // the peer mapping probe's verdict (set_shard_peers)
  ShardPeers peers;
  std::vector<void*> xopened;
  bool peer = false;
  bool sharded() const { return world > 1 || comm != nullptr; }
  int coresident[16] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};   // lm_resident, per mode
  floam_odom_stats stats{};
  floam_status last_warning = FLOAM_OK;
  // a device failure of an update (a solve abandoned, a compaction lookback timed out) leaves the device controller
  // frozen (OdomDev::failed: no pose taken, no keyframe, no map update from then on): every later update of the
  // handle fails with the first failure's message instead of returning stale odometry
  std::string poisoned;
  // floam_odom_update_selector_host: device copies of the caller's clouds, and the Q5 write-back of the deskewed
  // records into the caller's arrays on a copy stream once deskew_bridge has run (overlapped with call 2)
  std::unique_ptr<floam_cloud> h_edge, h_surf;
  struct WriteBack {
    bool active = false;
    void* edge = nullptr;
    void* surf = nullptr;
    size_t ne = 0, ns = 0;
  } wb;
  hipStream_t copy = nullptr;
  hipEvent_t wb_ev = nullptr;
};

// dmapping::ImuHandler (include/dataHandler.h:31-66): the stamped orientation stream, host-side (AddMsg / Get /
// TimeContained are scalar look-ups) with an append-only HBM mirror for the pre-processing kernel.
struct floam_imu {
  int device = 0;
  std::vector<double> t;
  std::vector<Q4> q;
  double* d_t = nullptr;
  Q4* d_q = nullptr;
  size_t dcap = 0, uploaded = 0;
};

// LaserMappingClass (include/laserMappingClass.h:38-66): the cell map in HBM (cell-grouped records in getMap order),
// the cell table (absolute cell key, size) on the host.
struct floam_mapping {
  int device = 0;
  float leaf = 0.4f;
  floam_cloud map, next;                 // current map / the rebuild target (swapped per update)
  std::vector<unsigned long long> keys;  // cell keys, ascending
  std::vector<int> counts;               // points per cell
  // scratch
  DevBuf<PointRec> stage, sorted, vox;
  DevBuf<int> slot, hcnt, hrank, cellv, total;
  DevBuf<unsigned long long> hkeys;
  SortScratch ss;
  RadixScratch rs;
  VoxelScratch2 vs;
  HostBuf<unsigned long long> h_keys;
  HostBuf<int> h_cnt, h_cellv;
};

namespace {
thread_local std::string t_err;

floam_status fail(floam_status s, const std::string& m) {
  t_err = m;
  return s;
}

template <typename F>
floam_status guarded(F&& f) {
  try {
    return f();
  } catch (const Error& e) {
    return fail(e.status, e.what());
  } catch (const std::bad_alloc&) {
    return fail(FLOAM_ERR_OUT_OF_MEMORY, "host allocation failed");
  } catch (const std::exception& e) {
    return fail(FLOAM_ERR_DEVICE, e.what());
  }
}

// an ABI call made from inside another one: its failure propagates with its own status and message
void chk(floam_status s) {
  if (s != FLOAM_OK && s < 100) throw Error(s, t_err);
}

void check_params(const floam_lidar_params* p) {
  if (!p) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null lidar params");
  if (p->num_lines <= 0 || p->num_lines > 4096) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "num_lines out of range");
}

// ------------------------------------------------------------------------------------- odometry internals
// peer sharding off: close the IPC mappings of the other ranks' exchange buffers
void shard_peers_release(floam_odom* o) {
  if (!o->xopened.empty()) {
    (void)hipStreamSynchronize(ctx_for(o->device).stream);
    for (void* p : o->xopened) (void)hipIpcCloseMemHandle(p);
    o->xopened.clear();
  }
  o->peers = ShardPeers{};
  o->peer = false;
}

// the one collective of the sharded path: the 29 sums (cost, J^T J, J^T r, count) of an LM evaluation, summed over
// the ranks in place — RCCL on the library stream (no host synchronisation), or the validation callback
void allreduce_sums(floam_odom* o, DeviceCtx& ctx) {
  double* sums = o->lmb.sums.p;
  if (o->comm) {
    const ncclResult_t r = ncclAllReduce(sums, sums, LM_NSUM, ncclDouble, ncclSum, o->comm, ctx.stream);
    if (r != ncclSuccess) throw Error(FLOAM_ERR_COMM, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    return;
  }
  if (!o->ar_fn) throw Error(FLOAM_ERR_COMM, "sharded odometry without a communicator");
  o->h_sums.reserve(LM_NSUM);
  FLOAM_HIP(hipMemcpyAsync(o->h_sums.p, sums, sizeof(double) * LM_NSUM, hipMemcpyDeviceToHost, ctx.stream));
  FLOAM_HIP(hipStreamSynchronize(ctx.stream));
  if (o->ar_fn(o->h_sums.p, LM_NSUM, o->ar_user) != 0) throw Error(FLOAM_ERR_COMM, "host all-reduce callback failed");
  FLOAM_HIP(hipMemcpyAsync(sums, o->h_sums.p, sizeof(double) * LM_NSUM, hipMemcpyHostToDevice, ctx.stream));
  FLOAM_HIP(hipStreamSynchronize(ctx.stream));
}

// The resident solve needs its whole grid on the device at once (its blocks poll each other): checked once per mode
// from the kernel's occupancy (a partitioned or smaller device falls back to one launch per evaluation, the sharded
// path on one rank).  FLOAM_LM_PER_EVAL=1 forces the fallback (tests, diagnostic build).
bool lm_resident(floam_odom* o, int mode) {
  int& c = o->coresident[mode & 15];
  if (c < 0) {
    const char* f = FLOAM_DIAG_ENV("FLOAM_LM_PER_EVAL");
    c = (f && f[0] == '1') ? 0 : (lm_solve_coresident(mode, o->device) ? 1 : 0);
  }
  return c == 1;
}

// updatePointsToMap (src/odomEstimationClass.cpp:52-124) runs on the device end to end, the controller included:
//   odom_predict_launch  optimization_count (host), the constant-velocity prediction (:59-71; always taken, Q2)
//   odom_issue           downsample, [grid rebuild], optimization_count x {kNN + geometry, 5 LM steps}, and the
//                        status gather with the pose writeback (:114-116) and KeyFrameUpdate (:117-122, :320-343)
//   odom_map_update      addPointsToMap (:253-294), gated on the device by the keyframe decision
// then one device-to-host copy of the status slots; odom_collect reads them (errors, warnings, stats, poses, map
// sizes) — right away in synchronous mode, later in asynchronous mode.
// pre >= 0: the call's clouds were downsampled on the side stream into the parity-`pre` buffers (odom_prevoxel)
// predict: the update's prediction (odom_predict) is issued here — inside the grid rebuild's first launch when the
// maps changed, else as a launch of its own — before anything reads x0_dev
struct MapUpdatePlan {
  VoxelJob je, js;
  int ne_ub = 0, ns_ub = 0;
  VoxelFused vf;   // the bounding-box stage, run by the status gather before the update
  MapKeys ke, ks;  // the incremental merge (o->map_merge)
};

// downSamplingToMap's two VoxelGrids of one call (:137-142): edge cloud at the edge leaf, surf cloud at the surf leaf
void call_voxel_jobs(floam_odom* o, const floam_cloud* edge, const floam_cloud* surf, int ne_ub, int ns_ub, VoxelJob& je,
                     VoxelJob& js) {
  o->dE.reserve(std::max(ne_ub, 1));
  o->dS.reserve(std::max(ns_ub, 1));
  o->cnt.reserve(4);
  je.part0 = edge->pts.p; je.d_n0 = edge->count.p; je.n0_ub = ne_ub; je.leaf = o->leafE;
  je.out = o->dE.p; je.d_out = o->cnt.p + 0;
  js.part0 = surf->pts.p; js.d_n0 = surf->count.p; js.n0_ub = ns_ub; js.leaf = o->leafS;
  js.out = o->dS.p; js.d_out = o->cnt.p + 1;
}

// vox_fused: the call's VoxelGrids' bounding-box stage already ran (deskew_bridge); map: the map update that follows
// this call (its bounding-box stage and the next grid builds' clears run in the status gather)
void odom_issue(floam_odom* o, DeviceCtx& ctx, const floam_cloud* edge, const floam_cloud* surf, int ne_ub, int ns_ub,
                const double* x0_dev, int slot, int gather_mode, int pre = -1, bool predict = false,
                GatherArgs* defer_gather = nullptr, bool vox_fused = false, const MapUpdatePlan* map = nullptr) {
  hipStream_t st = ctx.stream;
  if (predict && !o->grid_dirty) odom_predict_launch(o->ds.p, st);
  o->dE.reserve(std::max(ne_ub, 1));
  o->dS.reserve(std::max(ns_ub, 1));
  o->cnt.reserve(4);
  PointRec* const dE = pre >= 0 ? o->pE[pre].p : o->dE.p;
  PointRec* const dS = pre >= 0 ? o->pS[pre].p : o->dS.p;
  int* const dcnt = pre >= 0 ? o->pcnt[pre].p : o->cnt.p;
  if (pre < 0) {
    ProfScope ps(ctx, "voxel_downsample", FLOAM_PROF_CLOUD);
    // VelToIntensityCopy + downSamplingToMap (:53-54, :75, :137-142): both grids in one pipeline
    VoxelJob je, js;
    call_voxel_jobs(o, edge, surf, ne_ub, ns_ub, je, js);
    voxel2_launch(o->vs, je, js, st, nullptr, vox_fused);
  }
  const int mE_ub = (int)o->mapE_n, mS_ub = (int)o->mapS_n;   // exact or upper bounds
  if (o->grid_dirty) {
    ProfScope ps(ctx, "grid_build", FLOAM_PROF_CLOUD);
    grid_build_launch(o->gE, o->mapE.pts.p, o->mapE.count.p, mE_ub, o->gS, o->mapS.pts.p, o->mapS.count.p, mS_ub, st,
                      predict ? o->ds.p : nullptr, true, o->mapE.pts.cap, o->mapS.pts.cap);
    o->grid_dirty = false;
  }
  if (o->late_wait[0]) {   // one wait orders the main stream after the side stream's VoxelGrids and, through them,
    FLOAM_HIP(hipStreamWaitEvent(st, o->pre_ev, 0));   // after both clouds' producers (odom_prevoxel)
    for (const floam_cloud*& c : o->late_wait) {
      if (!c) continue;
      auto* cc = const_cast<floam_cloud*>(c);
      cc->last_stream = st;
      cc->ev_valid = false;
      c = nullptr;
    }
  }
  o->lm.reserve(1);
  o->lmb.reserve(st);
  if (!o->dbg_stamps.p && FLOAM_DIAG_ENV("FLOAM_DEBUG_STAMPS")) {
    o->dbg_stamps.reserve(10);
    FLOAM_HIP(hipMemsetAsync(o->dbg_stamps.p, 0, sizeof(unsigned long long) * 10, st));
  }
  o->prof_bytes.reserve(2);
  if (!o->prof_bytes_init) {
    FLOAM_HIP(hipMemsetAsync(o->prof_bytes.p, 0, sizeof(unsigned long long) * 2, st));
    o->prof_bytes_init = true;
  }
  // the search grid is sized from the downsampled counts seen recently (the device count of this call is not
  // known on the host without a sync); the kernel grid-strides, so an underestimate only costs time
  QuerySet qe{dE, dcnt + 0, ne_ub};
  QuerySet qs{dS, dcnt + 1, ns_ub};
  if (o->qhint[0] > 0) qe.grid_hint = std::min(ne_ub, o->qhint[0] + o->qhint[0] / 4 + 256);
  if (o->qhint[1] > 0) qs.grid_hint = std::min(ns_ub, o->qhint[1] + o->qhint[1] / 4 + 256);
  o->ce.trace = o->cs.trace = o->trace_cap > 0;
  o->last_traced = o->ce.trace;   // the neighbour indices / distances of this pass are written only while tracing
  o->last_q[0] = dE;
  o->last_q[1] = dS;
  o->last_qn = dcnt;
  const bool sharded = o->sharded();
  const int mode = lm_mode(o->huber, o->fp32);
  const bool gram = (mode & LM_GRAM) != 0;
  const bool peer = o->peer && o->world > 1;   // peer sharding: the resident solve exchanges the ranks' sums itself
  if (peer && !lm_resident(o, mode))
    throw Error(FLOAM_ERR_UNSUPPORTED, "peer sharding needs the resident solve (its grid does not fit the device)");
  // (diagnostic, FLOAM_SHARD_SOLO=N on an unsharded handle: this GPU runs only rank 0's 1/N of the correspondence
  // queries and solves on them alone, no exchange — the per-rank compute of an N-rank sharded run)
  static const int solo = FLOAM_DIAG_ENV("FLOAM_SHARD_SOLO") ? std::atoi(FLOAM_DIAG_ENV("FLOAM_SHARD_SOLO")) : 0;
  const int qrank = o->rank, qworld = (solo > 1 && o->world == 1) ? std::min(solo, kMaxShardRanks) : o->world;
  for (int it = 0; it < o->optimization_count; ++it) {
    bool split = false;
    {
      ProfScope ps(ctx, "knn", FLOAM_PROF_KNN);   // the correspondence pass: search + geometry
      {
        static const bool stages = FLOAM_DIAG_ENV("FLOAM_KNN_STAGES") != nullptr;
        if (stages && (ctx.profile & FLOAM_PROF_KNN_BYTES))   // (replay only, before the timed scope)
          knn_stage_launch(o->lm.p, it == 0 ? x0_dev : nullptr, qe, o->gE, o->ce, qs, o->gS, o->cs, o->mapE.count.p,
                           o->mapS.count.p, qrank, qworld, o->knn_evict, st);
        ProfScope ps1(ctx, "knn_search_bracket", FLOAM_PROF_KNN_DETAIL);   // (events around the launch)
        // "knn_search": HIP events set by the launch itself to the kernel's start and end (rocprofv3's duration)
        hipEvent_t k0 = nullptr, k1 = nullptr;
        if (ctx.profile & FLOAM_PROF_KNN_DETAIL) {
          k0 = ctx.get_event();
          k1 = ctx.get_event();
        }
        // (also starts the solve: LM state reset, the first solve at the prediction)
        split = knn_geom_split_launch(o->lm.p, it == 0 ? x0_dev : nullptr, qe, o->gE, o->ce, qs, o->gS, o->cs,
                                      o->mapE.count.p, o->mapS.count.p, qrank, qworld, gram, o->fp32_geom, o->lmb,
                                      st, k0, k1);   // (diagnostic prototype; false in the product)
        if (!split)
          knn_launch(o->lm.p, it == 0 ? x0_dev : nullptr, qe, o->gE, o->ce, qs, o->gS, o->cs, o->mapE.count.p,
                     o->mapS.count.p, qrank, qworld, st, k0, k1);
        if (k0) ctx.pending.push_back(PendingTiming{"knn_search", k0, k1, 0.0});
      }
      ProfScope ps2(ctx, "knn_geometry", FLOAM_PROF_KNN_DETAIL);
      if (!split) geom_launch(o->lm.p, qe, o->ce, qs, o->cs, gram, o->fp32_geom, o->lmb, st);
    }
    if (ctx.profile & FLOAM_PROF_KNN_BYTES) {   // replay only: algorithmic bytes of the two launches above
      knn_traffic_launch(o->lm.p, qe, o->gE, o->ce, qrank, qworld, o->traffic_set, o->prof_bytes.p + 0, st);
      knn_traffic_launch(o->lm.p, qs, o->gS, o->cs, qrank, qworld, o->traffic_set, o->prof_bytes.p + 1, st);
    }
    // ceres::Solve: iteration zero + at most max_num_iterations = 4 candidates (odomEstimationClass.cpp:102)
    if ((!sharded || peer) && lm_resident(o, mode)) {
      ProfScope ps(ctx, "lm_solve", FLOAM_PROF_LM);
      lm_solve_launch(o->lm.p, o->ce, dcnt + 0, ne_ub, o->cs, dcnt + 1, ns_ub, mode, o->lmb, st, o->dbg_stamps.p,
                      peer ? &o->peers : nullptr);
    } else {   // one launch (+ one all-reduce of the 29 sums when sharded) per evaluation, all on the stream
      ProfScope ps(ctx, "lm_solve_sharded", FLOAM_PROF_LM);
      for (int ev = 0; ev < 5; ++ev) {
        lm_shard_eval_launch(ev, o->lm.p, o->ce, dcnt + 0, ne_ub, o->cs, dcnt + 1, ns_ub, mode, o->lmb, st);
        if (sharded) allreduce_sums(o, ctx);
      }
      lm_shard_final_launch(o->lm.p, o->lmb, st);
    }
    if (o->trace_cap > 0)
      lm_trace_launch(o->lm.p, dcnt, o->mapE.count.p, o->mapS.count.p, o->trace.p, o->trace_count.p, o->trace_cap, st);
  }
  if (o->optimization_count <= 0) lm_init_dev_launch(o->lm.p, x0_dev, st);
  const bool prof_knn = (ctx.profile & FLOAM_PROF_KNN_BYTES) != 0;
  if (defer_gather && !prof_knn && gather_mode == 0) {   // carried out by the next launch (deskew_bridge)
    *defer_gather = GatherArgs{dcnt, o->mapE.count.p, o->mapS.count.p, edge->fe_status, o->h_ustat.p + slot,
                               (unsigned)o->issued};
    return;
  }
  GridClearDev gc[2];
  if (map) {   // (the grids' last readers, this call's kNN launches, are issued: the tables may be resized now)
    gc[0] = grid_clear_prepare(o->gE, (int)o->mapE_n + map->ne_ub, st);
    gc[1] = grid_clear_prepare(o->gS, (int)o->mapS_n + map->ns_ub, st);
  }
  gather_status_launch(o->lm.p, dcnt, o->mapE.count.p, o->mapS.count.p, edge->fe_status,
                       prof_knn ? o->prof_bytes.p : nullptr, o->h_ustat.p + slot, o->ds.p, gather_mode,
                       (unsigned)o->issued, st,
                       map ? &map->vf : nullptr, map ? gc : nullptr);
  if (prof_knn) FLOAM_HIP(hipMemsetAsync(o->prof_bytes.p, 0, sizeof(unsigned long long) * 2, st));
}

// keyframes_.push_back + the history trim of KeyFrameUpdate (src/odomEstimationClass.cpp:326, 334-337): the `first`
// branch appends without trimming, the others keep the newest keyframe_history_ = 3
void keyframe_push(floam_odom* o, const floam_odom::Keyframe& k, bool first) {
  o->keyframes.push_back(k);
  if (!first && o->keyframes.size() > 3) {
    for (floam_cloud* c : {o->keyframes.front().surf, o->keyframes.front().edge})
      if (c) o->kf_spare.push_back(c);
    o->keyframes.pop_front();
  }
}

// stats and warning of one call from its status slot (the gate :77 and the warnings :112, :193, :248)
floam_status odom_call_status(floam_odom* o, const UpdateStatus& U) {
  const LMState& L = U.lm;
  const int* hc = U.counts;
  const bool gate = hc[2] > 10 && hc[3] > 50;
  floam_status w = FLOAM_OK;
  if (!gate) w = FLOAM_WARN_MAP_TOO_SMALL;
  else if (L.corr_edge < 20 || L.corr_surf < 20) w = FLOAM_WARN_FEW_CORRESPONDENCES;
  o->stats.optimization_count = o->optimization_count;
  o->stats.solves = gate ? o->optimization_count : 0;
  o->stats.edge_queries = hc[0];
  o->stats.surf_queries = hc[1];
  for (int k = 0; k < 2; ++k) o->qhint[k] = std::max(o->qhint[k] - o->qhint[k] / 8, hc[k]);   // decaying max
  o->stats.edge_correspondences = gate ? L.corr_edge : 0;
  o->stats.surf_correspondences = gate ? L.corr_surf : 0;
  o->stats.lm_iterations = gate ? L.iteration : 0;
  o->stats.final_cost = gate ? L.x_cost : 0.0;
  o->stats.map_updated = 0;
  o->stats.corner_map = (size_t)hc[2];
  o->stats.surf_map = (size_t)hc[3];
  return w;
}

// Wait until every status slot of update P carries its serial number (the gather kernels store it last, at system
// scope, into coherent pinned host memory).  A stream that went idle or failed without the number is a device error.
void wait_status(floam_odom* o, DeviceCtx& ctx, const floam_odom::Pending& P) {
  const UpdateStatus* slots = o->h_ustat.p + 2 * P.ring;
  const unsigned want = (unsigned)P.seq;
  auto done = [&] {
    for (int k = 0; k < P.nslots; ++k)
      if (__atomic_load_n(&slots[k].seq, __ATOMIC_ACQUIRE) != want) return false;
    return true;
  };
  static const bool query = !FLOAM_DIAG_ENV("FLOAM_NOQUERY");   // (diagnostic knob)
  for (long long spin = 0; !done(); ++spin) {
    if (query && (spin & 1023) == 1023) {   // now and then: has the stream stopped without the status?
      const hipError_t q = hipStreamQuery(ctx.stream);
      if (q == hipSuccess) {
        if (done()) break;
        throw Error(FLOAM_ERR_DEVICE, "the update's status gather did not run (stream idle)");
      }
      if (q != hipErrorNotReady) throw Error(FLOAM_ERR_DEVICE, std::string("HIP: ") + hipGetErrorString(q));
    }
    __builtin_ia32_pause();
  }
}

// Collect the oldest in-flight update: wait for its status copy, raise its device errors, take its warning, stats,
// poses and (exact) map sizes.  Returns the update's warning (the second call's, else the first call's).
floam_status odom_collect_one(floam_odom* o, DeviceCtx& ctx) {
  const floam_odom::Pending P = o->inflight.front();
  o->inflight.pop_front();
  o->pendE -= P.addE;
  o->pendS -= P.addS;
  if (P.ev) FLOAM_HIP(hipEventSynchronize(P.ev));   // (a recycled event: not destroyed)
  wait_status(o, ctx, P);
  static const bool mm_debug = FLOAM_DIAG_ENV("FLOAM_MM_DEBUG") != nullptr;   // (diagnostic: the merge's modes)
  if (mm_debug && o->map_merge && o->mms.ctl.p) {
    FLOAM_HIP(hipStreamSynchronize(ctx.stream));
    int c[kMergeCtlWords];
    FLOAM_HIP(hipMemcpy(c, o->mms.ctl.p, sizeof(c), hipMemcpyDeviceToHost));
    std::fprintf(stderr, "[floam mm] update %llu: set %d / %d, full %d / %d, overflow %d / %d\n", P.seq, c[0], c[1], c[2],
                 c[3], c[4], c[5]);
  }
  o->collected_seq = P.seq;
  *o->done_ctr = P.seq;
  for (void* b : P.graveyard) (void)hipFree(b);
  ctx.drain();
  const UpdateStatus* slots = o->h_ustat.p + 2 * P.ring;
  auto poison = [&](const char* m) {
    o->poisoned = m;
    throw Error(FLOAM_ERR_DEVICE, m);
  };
  for (int k = 0; k < P.nslots; ++k) {
    const UpdateStatus& U = slots[k];
    if (ctx.profile & FLOAM_PROF_KNN_BYTES) {
      floam_kernel_timing& t = ctx.totals["knn_search"];   // the search kernel's algorithmic bytes (knn_traffic)
      std::strncpy(t.name, "knn_search", sizeof(t.name) - 1);
      t.algorithmic_bytes += (double)U.prof[0] + (double)U.prof[1];
    }
    if (U.lm.n_res < 0 || U.lm.xfail) poison("an LM solve's hand-off timed out (blocks or peer ranks did not arrive)");
    if (U.counts[0] < 0 || U.counts[1] < 0 || U.counts[2] < 0 || U.counts[3] < 0)
      poison("voxel-grid compaction failed (lookback timeout)");
    if (U.fe_status & FE_STATUS_SECTOR_TOO_LONG)
      throw Error(FLOAM_ERR_UNSUPPORTED, "a ring sector had no feature scratch (internal error)");
    if (U.fe_status & FE_STATUS_BAD_RING)
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "point ring index >= num_lines (out of bounds in the reference)");
  }
  floam_status w = FLOAM_OK;
  for (int k = 0; k < P.nslots; ++k) {
    const floam_status wk = odom_call_status(o, slots[k]);
    if (wk != FLOAM_OK) w = wk;
  }
  const UpdateStatus& last = slots[P.nslots - 1];
  o->odom = last.odom;
  o->last_odom = last.last_odom;
  if (P.map_slot >= 0) {
    o->stats.map_updated = slots[P.map_slot].kf_flag;
    if (o->stats.map_updated) keyframe_push(o, floam_odom::Keyframe{slots[P.map_slot].odom}, P.kf_first);
  }
  // map sizes: exact before this update's map update, plus what the later in-flight updates may add
  const UpdateStatus& M = slots[P.map_slot >= 0 ? P.map_slot : P.nslots - 1];
  o->mapE_n = (size_t)M.counts[2] + P.addE + o->pendE;
  o->mapS_n = (size_t)M.counts[3] + P.addS + o->pendS;
  const bool exact = o->inflight.empty() && P.map_slot < 0;
  o->mapE.host_count_valid = o->mapS.host_count_valid = exact;
  o->mapE.host_count = o->mapE.ub = o->mapE_n;
  o->mapS.host_count = o->mapS.ub = o->mapS_n;
  if (o->depth > 0) {   // asynchronous mode: the poses wait for floam_odom_wait
    double q[4];
    mat_to_quat(o->odom.R, q);
    for (int i = 0; i < 4; ++i) o->collected.push_back(q[i]);
    for (int i = 0; i < 3; ++i) o->collected.push_back(o->odom.t[i]);
  }
  return w;
}

floam_status odom_collect(floam_odom* o, DeviceCtx& ctx, size_t max_pending) {
  floam_status w = FLOAM_OK;
  while (o->inflight.size() > max_pending) {
    const floam_status wk = odom_collect_one(o, ctx);
    if (wk != FLOAM_OK) w = wk;
  }
  return w;
}

// status slots for the next update (collecting the oldest in-flight update if the ring is full)
int odom_begin(floam_odom* o, DeviceCtx& ctx) {
  if (!o->poisoned.empty())
    throw Error(FLOAM_ERR_DEVICE, "an earlier update of this handle failed on the device (" + o->poisoned +
                                      "); its odometry is frozen: create a new handle");
  const int ring_n = std::max(o->depth, 1);
  if (o->inflight.size() >= (size_t)ring_n) {
    const floam_status w = odom_collect(o, ctx, (size_t)ring_n - 1);
    if (w != FLOAM_OK) o->last_warning = w;   // reported by the next floam_odom_wait
  }
  o->h_ustat.reserve(32, hipHostMallocCoherent);
  return (int)(o->issued++ % (unsigned long long)ring_n);
}

// Graph capture of one update (when enabled): odom_capture_begin before its first device operation,
// odom_capture_end after its last one instantiates or updates the executable graph of its kind and launches it.
// (not while the one-call host entry point's write-back is active: its copy stream would join the capture)
bool odom_capture_begin(floam_odom* o, DeviceCtx& ctx) {
  if (!o->use_graph || ctx.profile != 0 || o->sharded() || o->wb.active) return false;
  FLOAM_HIP(hipStreamBeginCapture(ctx.stream, hipStreamCaptureModeRelaxed));
  capture_state().active = true;
  return true;
}

void odom_capture_abort(DeviceCtx& ctx) {   // after an exception inside the captured region
  CaptureState& cs = capture_state();
  if (!cs.active) return;
  cs.active = false;
  hipGraph_t g = nullptr;
  (void)hipStreamEndCapture(ctx.stream, &g);
  if (g) (void)hipGraphDestroy(g);
}

void odom_capture_end(floam_odom* o, DeviceCtx& ctx, int kind) {
  CaptureState& cs = capture_state();
  cs.active = false;
  hipGraph_t g = nullptr;
  FLOAM_HIP(hipStreamEndCapture(ctx.stream, &g));
  hipGraphExec_t& ex = o->graph_exec[kind][(o->issued - 1) % (unsigned long long)(o->depth + 1)];
  bool ok = false;
  if (ex) {
    hipGraphNode_t err_node = nullptr;
    hipGraphExecUpdateResult res;
    ok = hipGraphExecUpdate(ex, g, &err_node, &res) == hipSuccess && res == hipGraphExecUpdateSuccess;
    if (!ok) {   // the topology changed (e.g. optimization_count): a fresh executable graph
      (void)hipGetLastError();
      FLOAM_HIP(hipGraphExecDestroy(ex));
      ex = nullptr;
    }
  }
  if (!ok) FLOAM_HIP(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  FLOAM_HIP(hipGraphDestroy(g));
  FLOAM_HIP(hipGraphLaunch(ex, ctx.stream));
}

// the end of an issued update (its status slots are written to pinned host memory by the gather kernel); synchronous
// mode collects it right away
floam_status odom_end(floam_odom* o, DeviceCtx& ctx, int ring, int nslots, int map_slot, size_t addE, size_t addS,
                      bool captured, int kind) {
  std::vector<void*> graveyard;
  if (captured) {
    graveyard.swap(capture_state().graveyard);
    odom_capture_end(o, ctx, kind);
  }
  // The host learns that an update is done by polling its status slots (their serial number is stored last), and
  // the consumers of its buffers on other streams check the collected serial number (cloud_on, odom_prevoxel), so
  // no event is recorded per update (profiles r03a/r03b: the device idled 30 us between two updates with four
  // records there, 14 us with one).  Only a ring deeper than 2 records one, for the side stream's buffer reuse (its
  // parity buffers may not be collected yet).
  hipEvent_t ev = nullptr;
  if (o->depth > 2 || captured) {
    ev = ctx.next_update_event();
    FLOAM_HIP(hipEventRecord(ev, ctx.stream));
  }
  o->end_ev = ev;
  o->inflight.push_back(floam_odom::Pending{ring, nslots, map_slot, addE, addS, ev, std::move(graveyard),
                                            o->next_kf_first, o->issued});
  o->next_kf_first = false;
  o->pendE += addE;
  o->pendS += addS;
  if (o->depth == 0) return odom_collect(o, ctx, 0);
  return FLOAM_OK;
}

int gather_keyframe_mode(floam_odom* o) {   // KeyFrameUpdate's process-wide `first` flag (Q6) is consumed here
  const int m = GATHER_KEYFRAME | (g_keyframe_first ? GATHER_KEYFRAME_FIRST : 0);
  o->next_kf_first = g_keyframe_first;
  g_keyframe_first = false;
  return m;
}

// addPointsToMap (:253-294), issued unconditionally and gated on the device by the keyframe decision (a skipped
// update copies the maps unchanged): transform + append + CropBox + VoxelGrid of both maps with the optimised pose
// (lm->x), one pipeline.  Returns the upper bounds of the points it may add.
MapUpdatePlan odom_map_plan(floam_odom* o, DeviceCtx& ctx, int ne_ub, int ns_ub) {
  hipStream_t st = ctx.stream;
  MapUpdatePlan P;
  P.ne_ub = ne_ub;
  P.ns_ub = ns_ub;
  const int ubS = (int)o->mapS_n + ns_ub, ubE = (int)o->mapE_n + ne_ub;
  cloud_reserve(&o->mapS_next, std::max(ubS, 1), 0, st);
  cloud_reserve(&o->mapE_next, std::max(ubE, 1), 0, st);
  o->dE.reserve(std::max(ne_ub, 1));
  o->dS.reserve(std::max(ns_ub, 1));
  o->cnt.reserve(4);
  o->lm.reserve(1);
  VoxelJob& je = P.je;
  VoxelJob& js = P.js;
  je.part0 = o->mapE.pts.p; je.d_n0 = o->mapE.count.p; je.n0_ub = (int)o->mapE_n;
  je.part1 = o->dE.p; je.d_n1 = o->cnt.p + 0; je.n1_ub = ne_ub;
  je.pose = o->lm.p->x; je.leaf = o->leafE; je.out = o->mapE_next.pts.p; je.d_out = o->mapE_next.count.p;
  js.part0 = o->mapS.pts.p; js.d_n0 = o->mapS.count.p; js.n0_ub = (int)o->mapS_n;
  js.part1 = o->dS.p; js.d_n1 = o->cnt.p + 1; js.n1_ub = ns_ub;
  js.pose = o->lm.p->x; js.leaf = o->leafS; js.out = o->mapS_next.pts.p; js.d_out = o->mapS_next.count.p;
  P.vf = voxel2_prepare(o->vs, je, js, st);
  if (o->map_merge) {
    const int cur = o->mkcur, nxt = cur ^ 1;
    for (int m = 0; m < 2; ++m) {
      o->mkeys[m][cur].reserve(std::max(m ? (int)o->mapS_n : (int)o->mapE_n, 1));
      o->mkeys[m][nxt].reserve(std::max(m ? ubS : ubE, 1));
      for (int b = 0; b < 2; ++b)
        if (!o->mmeta[m][b].p) {
          o->mmeta[m][b].reserve(1);
          FLOAM_HIP(hipMemsetAsync(o->mmeta[m][b].p, 0, sizeof(MapMeta), st));
        }
    }
    o->mms.reserve(1, st);
    P.ke = MapKeys{o->mkeys[0][cur].p, o->mmeta[0][cur].p, o->mkeys[0][nxt].p, o->mmeta[0][nxt].p};
    P.ks = MapKeys{o->mkeys[1][cur].p, o->mmeta[1][cur].p, o->mkeys[1][nxt].p, o->mmeta[1][nxt].p};
    P.vf.mc = merge_check(o->mms, (unsigned)o->issued);
  }
  return P;
}

// addPointsToMap (:253-294), issued unconditionally and gated on the device by the keyframe decision (a skipped
// update copies the maps unchanged): transform + append + CropBox + VoxelGrid of both maps with the optimised pose
// (lm->x), one pipeline whose bounding-box stage ran in the status gather (P.vf).  Returns the upper bounds of the
// points it may add.
void odom_map_update(floam_odom* o, DeviceCtx& ctx, const MapUpdatePlan& P, size_t& addE, size_t& addS) {
  hipStream_t st = ctx.stream;
  ProfScope ps(ctx, "map_update", FLOAM_PROF_CLOUD);
  const int ubS = (int)o->mapS_n + P.ns_ub, ubE = (int)o->mapE_n + P.ne_ub;
  if (o->map_merge) {   // the new scan voxels merged into the voxel-ordered maps (mapmerge.hip)
    map_merge_launch(o->vs, o->mms, P.je, P.js, P.ke, P.ks, &o->ds.p->kf_flag, (unsigned)o->issued,
                     o->map_force_full, o->map_violate_mod, st);
    o->mkcur ^= 1;
  } else {
    voxel2_launch(o->vs, P.je, P.js, st, &o->ds.p->kf_flag, true);
  }
  cloud_swap(&o->mapE, &o->mapE_next);
  cloud_swap(&o->mapS, &o->mapS_next);
  addE = (size_t)P.ne_ub;
  addS = (size_t)P.ns_ub;
  o->mapS_n = (size_t)ubS;   // upper bounds until the update is collected
  o->mapE_n = (size_t)ubE;
  o->mapS.host_count_valid = false;
  o->mapE.host_count_valid = false;
  o->mapS.ub = o->mapS_n;
  o->mapE.ub = o->mapE_n;
  o->grid_dirty = true;
}

// updatePointsToMap (src/odomEstimationClass.cpp:52-124), one call
floam_status odom_update(floam_odom* o, const floam_cloud* edge, const floam_cloud* surf, int type) {
  DeviceCtx& ctx = ctx_for(o->device);
  FLOAM_HIP(hipSetDevice(o->device));
  const int ring = odom_begin(o, ctx);
  const int ne_ub = (int)cloud_ub(edge), ns_ub = (int)cloud_ub(surf);
  const bool captured = odom_capture_begin(o, ctx);
  try {
    if (o->optimization_count > 2) o->optimization_count--;
    const bool update_map = type == FLOAM_VANILLA || type == FLOAM_REFINEMENT_AND_UPDATE;
    MapUpdatePlan mp;
    if (update_map) mp = odom_map_plan(o, ctx, ne_ub, ns_ub);
    odom_issue(o, ctx, edge, surf, ne_ub, ns_ub, o->ds.p->x0[0], 2 * ring,
               GATHER_FINISH | (update_map ? gather_keyframe_mode(o) : 0), -1, true, nullptr, false,
               update_map ? &mp : nullptr);
    size_t addE = 0, addS = 0;
    if (update_map) odom_map_update(o, ctx, mp, addE, addS);
    return odom_end(o, ctx, ring, 1, update_map ? 0 : -1, addE, addS, captured, 0);
  } catch (...) {
    odom_capture_abort(ctx);
    throw;
  }
}

// Call 1's VoxelGrids (edge cloud at the edge and the surf leaf, Q4) on the side stream, ordered after the cloud's
// producer (the feature extraction) and after the update that last used this parity's buffers; the main stream
// orders itself after it through the cloud (cloud_on_main).  Not used while an update is captured into a graph.
void odom_prevoxel(floam_odom* o, floam_cloud* edge, floam_cloud* surf) {
  if (o->use_graph) return;
  if (!o->side) {
    make_stream(&o->side, false);
    FLOAM_HIP(hipEventCreateWithFlags(&o->pre_ev, hipEventDisableTiming));
  }
  const int par = o->pre_par;
  o->pre_par ^= 1;
  const int ne_ub = (int)cloud_ub(edge);
  o->pE[par].reserve(std::max(ne_ub, 1));
  o->pS[par].reserve(std::max(ne_ub, 1));
  o->pcnt[par].reserve(2);
  if (o->side_ev_rec[par] && o->side_seq[par] > o->collected_seq) {   // the update that read them still runs
    hipEvent_t e = o->side_ev[par];
    if (!e) {   // (no end event was recorded for it: the main stream's tail, a later point)
      e = ctx_for(o->device).next_update_event();
      FLOAM_HIP(hipEventRecord(e, ctx_for(o->device).stream));
    }
    FLOAM_HIP(hipStreamWaitEvent(o->side, e, 0));
  }
  cloud_on(edge, o->side);
  cloud_on(surf, o->side);   // (not used here: so that one event below orders the main stream after both producers)
  VoxelJob je, js;
  je.part0 = edge->pts.p; je.d_n0 = edge->count.p; je.n0_ub = ne_ub; je.leaf = o->leafE;
  je.out = o->pE[par].p; je.d_out = o->pcnt[par].p + 0;
  js.part0 = edge->pts.p; js.d_n0 = edge->count.p; js.n0_ub = ne_ub; js.leaf = o->leafS;
  js.out = o->pS[par].p; js.d_out = o->pcnt[par].p + 1;
  voxel2_launch(o->vs1, je, js, o->side);
  FLOAM_HIP(hipEventRecord(o->pre_ev, o->side));
  o->pre_valid = par;
}

// UpdatePointsToMapSelector with deskew (src/odomEstimationClass.cpp:38-47): call 1 (edge, edge) INITIAL_ITERATION
// (Q4), GetVelocity + CompensateVelocity of both clouds in place (Q5), call 2 (edge, surf) REFINEMENT_AND_UPDATE,
// all issued without a host round trip (the velocity and the second prediction are formed by deskew_bridge).
floam_status odom_update_deskew(floam_odom* o, floam_cloud* edge, floam_cloud* surf) {
  const int pre = o->pre_valid;   // consumed by this update whatever happens
  o->pre_valid = -1;
  DeviceCtx& ctx = ctx_for(o->device);
  FLOAM_HIP(hipSetDevice(o->device));
  const int ring = odom_begin(o, ctx);
  const int ne_ub = (int)cloud_ub(edge), ns_ub = (int)cloud_ub(surf);
  const bool captured = odom_capture_begin(o, ctx);
  static const bool nop = FLOAM_DIAG_ENV("FLOAM_UPDATE_NOP") != nullptr;
  if (nop) update_nop_launch(ctx.stream);
  try {
    if (o->optimization_count > 2) o->optimization_count--;
    GatherArgs g1;
    odom_issue(o, ctx, edge, edge, ne_ub, ne_ub, o->ds.p->x0[0], 2 * ring, 0, pre, true, &g1);
    // the second call's VoxelGrids get their bounding boxes from deskew_bridge, which writes their input (distinct
    // clouds; aliased ones are shifted twice per point by one thread and keep the separate stage)
    const bool fuse = edge != surf;
    VoxelFused vf2{};
    if (fuse) {
      VoxelJob je, js;
      call_voxel_jobs(o, edge, surf, ne_ub, ns_ub, je, js);
      vf2 = voxel2_prepare(o->vs, je, js, ctx.stream);
    }
    {
      ProfScope ps(ctx, "deskew", FLOAM_PROF_CLOUD);
      deskew_bridge_launch(o->lm.p, o->ds.p, o->lp.scan_period, edge->pts.p, edge->count.p, ne_ub, surf->pts.p,
                           surf->count.p, ns_ub, ctx.stream, g1, fuse ? &vf2 : nullptr);
    }
    if (o->wb.active) {   // the clouds are final here (CompensateVelocity, Q5): the write-back may start
      if (!o->wb_ev) FLOAM_HIP(hipEventCreateWithFlags(&o->wb_ev, hipEventDisableTiming));
      FLOAM_HIP(hipEventRecord(o->wb_ev, ctx.stream));
    }
    if (o->optimization_count > 2) o->optimization_count--;
    MapUpdatePlan mp = odom_map_plan(o, ctx, ne_ub, ns_ub);
    odom_issue(o, ctx, edge, surf, ne_ub, ns_ub, o->ds.p->x0[1], 2 * ring + 1,
               GATHER_FINISH | GATHER_AFTER_MID | gather_keyframe_mode(o), -1, false, nullptr, fuse, &mp);
    size_t addE = 0, addS = 0;
    odom_map_update(o, ctx, mp, addE, addS);
    if (o->wb.active) {   // the whole update is issued: copy the deskewed records back while call 2 runs
      FLOAM_HIP(hipStreamWaitEvent(o->copy, o->wb_ev, 0));
      if (o->wb.ne)
        FLOAM_HIP(hipMemcpyAsync(o->wb.edge, edge->pts.p, o->wb.ne * sizeof(PointRec), hipMemcpyDeviceToHost, o->copy));
      if (o->wb.ns)
        FLOAM_HIP(hipMemcpyAsync(o->wb.surf, surf->pts.p, o->wb.ns * sizeof(PointRec), hipMemcpyDeviceToHost, o->copy));
    }
    const floam_status r = odom_end(o, ctx, ring, 2, 1, addE, addS, captured, 1);
    if (pre >= 0) {   // the side stream may refill this parity's buffers once this update has run (its end event)
      o->side_ev[pre] = o->end_ev;
      o->side_seq[pre] = o->issued;
      o->side_ev_rec[pre] = true;
    }
    return r;
  } catch (...) {
    odom_capture_abort(ctx);
    throw;
  }
}

// CompensateVelocity (src/dataHandler.cpp:82-92) with GetVelocity (include/odomEstimationClass.h:78)
void odom_velocity(const floam_odom* o, double v[3]) {
  for (int i = 0; i < 3; ++i) v[i] = (o->odom.t[i] - o->last_odom.t[i]) / o->lp.scan_period;
}

}  // namespace

namespace floam {
void set_last_error(const std::string& m) { t_err = m; }
}  // namespace floam

// ============================================================================================ C ABI
extern "C" {

const char* floam_last_error(void) { return t_err.c_str(); }
const char* floam_version(void) { return "floam_amd 0.4.0 (gfx950, ABI 3)"; }
int floam_abi_version(void) { return FLOAM_ABI_VERSION; }
void floam_reset_process_state(void) { g_keyframe_first = true; }

floam_status floam_device_synchronize(int device) {
  return guarded([&] {
    ctx_for(device);
    FLOAM_HIP(hipSetDevice(device));
    FLOAM_HIP(hipDeviceSynchronize());   // every stream (the feature extraction handles' included)
    return FLOAM_OK;
  });
}

floam_status floam_cloud_create(int device, size_t capacity, floam_cloud** out) {
  return guarded([&] {
    if (!out) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null out");
    auto c = std::make_unique<floam_cloud>();
    FLOAM_HIP(hipSetDevice(device));
    cloud_init(c.get(), device, capacity);
    *out = c.release();
    return FLOAM_OK;
  });
}

floam_status floam_cloud_destroy(floam_cloud* c) {
  return guarded([&] {
    if (c) {
      DeviceCtx& ctx = ctx_for(c->device);
      FLOAM_HIP(hipStreamSynchronize(ctx.stream));
      if (c->ev_valid && c->ext_ev) FLOAM_HIP(hipEventSynchronize(c->ext_ev));
      if (c->ev) {
        if (c->ev_valid && !c->ext_ev) FLOAM_HIP(hipEventSynchronize(c->ev));
        FLOAM_HIP(hipEventDestroy(c->ev));
      }
      delete c;
    }
    return FLOAM_OK;
  });
}

floam_status floam_cloud_upload(floam_cloud* c, const void* host, size_t n, size_t stride) {
  return guarded([&] {
    if (!c || (!host && n)) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null cloud / points");
    if (n > (size_t)INT32_MAX) throw Error(FLOAM_ERR_UNSUPPORTED, "cloud larger than 2^31 points");
    if (stride < 28) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "stride must cover the PointXYZIRT fields");
    DeviceCtx& ctx = ctx_for(c->device);
    FLOAM_HIP(hipSetDevice(c->device));
    cloud_on_main(c);
    FLOAM_HIP(hipStreamSynchronize(ctx.stream));
    cloud_reserve(c, std::max<size_t>(n, 1), 0, ctx.stream);
    if (stride == sizeof(PointRec)) {
      FLOAM_HIP(hipMemcpyAsync(c->pts.p, host, n * sizeof(PointRec), hipMemcpyHostToDevice, ctx.stream));
    } else {
      std::vector<PointRec> tmp(n);
      const char* b = static_cast<const char*>(host);
      for (size_t i = 0; i < n; ++i) std::memcpy(&tmp[i], b + i * stride, 28);
      FLOAM_HIP(hipMemcpyAsync(c->pts.p, tmp.data(), n * sizeof(PointRec), hipMemcpyHostToDevice, ctx.stream));
      FLOAM_HIP(hipStreamSynchronize(ctx.stream));
    }
    const int cnt = (int)n;
    FLOAM_HIP(hipMemcpyAsync(c->count.p, &cnt, sizeof(int), hipMemcpyHostToDevice, ctx.stream));
    FLOAM_HIP(hipStreamSynchronize(ctx.stream));
    c->host_count = n;
    c->host_count_valid = true;
    return FLOAM_OK;
  });
}

floam_status floam_cloud_size(const floam_cloud* c, size_t* n) {
  return guarded([&] {
    if (!c || !n) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    *n = cloud_count_sync(c);
    return FLOAM_OK;
  });
}

floam_status floam_cloud_download(const floam_cloud* c, void* host, size_t capacity, size_t* n_out) {
  return guarded([&] {
    if (!c) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null cloud");
    cloud_on_main(c);
    const size_t n = cloud_count_sync(c);
    if (n_out) *n_out = n;
    const size_t k = std::min(n, capacity);
    if (k) {
      if (!host) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null host buffer");
      DeviceCtx& ctx = ctx_for(c->device);
      FLOAM_HIP(hipMemcpyAsync(host, c->pts.p, k * sizeof(PointRec), hipMemcpyDeviceToHost, ctx.stream));
      FLOAM_HIP(hipStreamSynchronize(ctx.stream));
    }
    return FLOAM_OK;
  });
}

floam_status floam_cloud_clear(floam_cloud* c) {
  return guarded([&] {
    if (!c) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null cloud");
    // deferred to the cloud's next operation (cloud_on), so that clearing a feature buffer for the next scan does
    // not queue a fill on the odometry stream between two updates
    c->clear_pending = true;
    c->host_count = 0;
    c->host_count_valid = true;
    return FLOAM_OK;
  });
}

floam_status floam_cloud_copy(floam_cloud* dst, const floam_cloud* src) {
  return guarded([&] {
    if (!dst || !src) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null cloud");
    if (dst->device != src->device) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "clouds on different devices");
    DeviceCtx& ctx = ctx_for(dst->device);
    cloud_on_main(src);
    cloud_on_main(dst);
    const size_t n = cloud_count_sync(src);
    cloud_reserve(dst, std::max<size_t>(n, 1), 0, ctx.stream);
    if (n)
      FLOAM_HIP(hipMemcpyAsync(dst->pts.p, src->pts.p, n * sizeof(PointRec), hipMemcpyDeviceToDevice, ctx.stream));
    FLOAM_HIP(hipMemcpyAsync(dst->count.p, src->count.p, sizeof(int), hipMemcpyDeviceToDevice, ctx.stream));
    dst->host_count = n;
    dst->host_count_valid = true;
    return FLOAM_OK;
  });
}

void* floam_cloud_device_ptr(floam_cloud* c) { return c ? c->pts.p : nullptr; }

floam_status floam_voxel_grid(const floam_cloud* in, float leaf, floam_cloud* out) {
  return guarded([&] {
    if (!in || !out || in == out) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null or aliased cloud");
    if (in->device != out->device) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "clouds on different devices");
    if (!(leaf > 0.0f)) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "leaf size must be > 0");
    DeviceCtx& ctx = ctx_for(in->device);
    FLOAM_HIP(hipSetDevice(in->device));
    cloud_on_main(in);
    cloud_on_main(out);
    const size_t n = cloud_ub(in);
    if (n > (size_t)INT32_MAX / 2) throw Error(FLOAM_ERR_UNSUPPORTED, "cloud too large");
    cloud_reserve(out, std::max<size_t>(n, 1), 0, ctx.stream);
    if (!ctx.zero.p) {
      ctx.zero.reserve(2);
      FLOAM_HIP(hipMemsetAsync(ctx.zero.p, 0, sizeof(int) * 2, ctx.stream));
    }
    VoxelJob a, b;
    a.part0 = in->pts.p; a.d_n0 = in->count.p; a.n0_ub = (int)n; a.leaf = leaf;
    a.out = out->pts.p; a.d_out = out->count.p;
    b.part0 = in->pts.p; b.d_n0 = ctx.zero.p; b.n0_ub = 0; b.leaf = leaf;
    b.out = out->pts.p; b.d_out = ctx.zero.p + 1;   // the empty job's count lands in a scratch word
    ctx.vs.s.reserve(1);
    voxel2_launch(ctx.vs, a, b, ctx.stream);
    out->host_count_valid = false;
    out->ub = n;
    return FLOAM_OK;
  });
}

// ------------------------------------------------------------------------------------------ laser processing
floam_status floam_lp_create(const floam_lidar_params* p, int device, floam_lp** out) {
  return guarded([&] {
    check_params(p);
    if (!out) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null out");
    ctx_for(device);
    FLOAM_HIP(hipSetDevice(device));
    auto lp = std::make_unique<floam_lp>();
    lp->device = device;
    lp->prm.num_lines = p->num_lines;
    lp->prm.min_distance = p->min_distance;
    lp->prm.max_distance = p->max_distance;
    lp->status.reserve(1);
    lp->h_out.reserve(4);
    lp->sc.status = lp->status.p;
    make_stream(&lp->stream, false);
    *out = lp.release();
    return FLOAM_OK;
  });
}

floam_status floam_lp_set_async(floam_lp* lp, int async) {
  return guarded([&] {
    if (!lp) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    lp->async = async != 0;
    return FLOAM_OK;
  });
}

floam_status floam_lp_wait(floam_lp* lp) {
  return guarded([&] {
    if (!lp) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    FLOAM_HIP(hipMemcpyAsync(lp->h_out.p, lp->sc.out3.p, sizeof(int) * 3, hipMemcpyDeviceToHost, lp->stream));
    FLOAM_HIP(hipStreamSynchronize(lp->stream));
    const int status = lp->h_out.p[2];
    if (status & FE_STATUS_SECTOR_TOO_LONG)
      throw Error(FLOAM_ERR_UNSUPPORTED, "a ring sector had no feature scratch (internal error)");
    if (status & FE_STATUS_BAD_RING)
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "point ring index >= num_lines (out of bounds in the reference)");
    return FLOAM_OK;
  });
}

floam_status floam_lp_destroy(floam_lp* lp) {
  return guarded([&] {
    if (lp) {
      fe_stamps_print();
      if (lp->stream) {
        FLOAM_HIP(hipStreamSynchronize(lp->stream));
        FLOAM_HIP(hipStreamDestroy(lp->stream));
      }
      delete lp;
    }
    return FLOAM_OK;
  });
}

floam_status floam_lp_feature_extraction(floam_lp* lp, const floam_cloud* in, floam_cloud* edge, floam_cloud* surf) {
  return guarded([&] {
    if (!lp || !in || !edge || !surf) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    if (in->device != lp->device || edge->device != lp->device || surf->device != lp->device)
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "clouds and handle on different devices");
    if (edge == surf || in == edge || in == surf) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "clouds must be distinct");
    DeviceCtx& ctx = ctx_for(lp->device);
    hipStream_t st = lp->stream;
    FLOAM_HIP(hipSetDevice(lp->device));
    const size_t n = cloud_count_sync(in);
    const size_t ne0 = lp->async ? cloud_ub(edge) : cloud_count_sync(edge);
    const size_t ns0 = lp->async ? cloud_ub(surf) : cloud_count_sync(surf);
    const size_t ne_add = std::min(n, (size_t)lp->prm.num_lines * 6 * 20);
    cloud_on(in, st);
    // a pending clear of an output is folded into the extraction's kernels (no fill launch of its own)
    const int clear = n > 0 ? (edge->clear_pending ? 1 : 0) | (surf->clear_pending ? 2 : 0) : 0;
    if (clear & 1) edge->clear_pending = false;
    if (clear & 2) surf->clear_pending = false;
    cloud_on(edge, st);
    cloud_on(surf, st);
    cloud_reserve(edge, ne0 + ne_add + 1, ne0, st);
    cloud_reserve(surf, ns0 + n + 1, ns0, st);
    edge->fe_stat.reserve(1);
    surf->fe_stat.reserve(1);
    if (n > 0) {
      ProfScope ps(ctx, "feature_extraction", FLOAM_PROF_FE, 64.0 * (double)n, st);
      fe_launch(lp->sc, lp->prm, in->pts.p, (int)n, edge->pts.p, edge->count.p, surf->pts.p, surf->count.p, st,
                edge->fe_stat.p, surf->fe_stat.p, clear);
    }
    cloud_publish(in, st);
    cloud_publish(edge, st);
    cloud_publish(surf, st);
    if (lp->async && n > 0) {
      // counts stay on the device; the status flags travel with the clouds and are checked at the consumer's
      // synchronisation (odometry update) or by floam_lp_wait
      edge->host_count_valid = false;
      edge->ub = ne0 + ne_add;
      surf->host_count_valid = false;
      surf->ub = ns0 + n;
      edge->fe_status = edge->fe_stat.p;
      surf->fe_status = surf->fe_stat.p;
      return FLOAM_OK;
    }
    edge->fe_status = surf->fe_status = nullptr;
    if (n > 0) {
      FLOAM_HIP(hipMemcpyAsync(lp->h_out.p, lp->sc.out3.p, sizeof(int) * 3, hipMemcpyDeviceToHost, st));
      FLOAM_HIP(hipStreamSynchronize(st));
    } else {
      lp->h_out.p[0] = (int)ne0;
      lp->h_out.p[1] = (int)ns0;
      lp->h_out.p[2] = 0;
    }
    ctx.drain();
    edge->host_count = (size_t)lp->h_out.p[0];
    edge->host_count_valid = true;
    surf->host_count = (size_t)lp->h_out.p[1];
    surf->host_count_valid = true;
    const int status = lp->h_out.p[2];
    if (status & FE_STATUS_SECTOR_TOO_LONG)
      throw Error(FLOAM_ERR_UNSUPPORTED, "a ring sector had no feature scratch (internal error)");
    if (status & FE_STATUS_BAD_RING)
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "point ring index >= num_lines (out of bounds in the reference)");
    return FLOAM_OK;
  });
}

floam_status floam_lp_feature_extraction_host(floam_lp* lp, const void* in, size_t n, size_t stride, void* edge,
                                              size_t edge_cap, size_t* n_edge, void* surf, size_t surf_cap,
                                              size_t* n_surf) {
  return guarded([&] {
    if (!lp || (!in && n) || !n_edge || !n_surf) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    if (stride != sizeof(PointRec)) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "input must be 32-B PointXYZIRT records");
    if (n > (size_t)INT32_MAX) throw Error(FLOAM_ERR_UNSUPPORTED, "cloud larger than 2^31 points");
    hipStream_t st = lp->stream;
    FLOAM_HIP(hipSetDevice(lp->device));
    for (auto* c : {&lp->h_in, &lp->h_edge, &lp->h_surf})
      if (!*c) {
        *c = std::make_unique<floam_cloud>();
        cloud_init(c->get(), lp->device, 0);
      }
    floam_cloud *ci = lp->h_in.get(), *ce = lp->h_edge.get(), *cs = lp->h_surf.get();
    for (floam_cloud* c : {ci, ce, cs}) cloud_on(c, st);
    FLOAM_HIP(hipStreamSynchronize(st));
    *n_edge = *n_surf = 0;
    if (n == 0) return FLOAM_OK;
    const size_t ne_ub = std::min(n, (size_t)lp->prm.num_lines * 6 * 20);
    cloud_reserve(ci, n, 0, st);
    cloud_reserve(ce, ne_ub + 1, 0, st);
    cloud_reserve(cs, n + 1, 0, st);
    ce->fe_stat.reserve(1);
    cs->fe_stat.reserve(1);
    FLOAM_HIP(hipMemcpyAsync(ci->pts.p, in, n * sizeof(PointRec), hipMemcpyHostToDevice, st));
    FLOAM_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ci->count.p), (int)n, 1, st));
    // the outputs start empty: the clear is folded into the extraction's kernels
    fe_launch(lp->sc, lp->prm, ci->pts.p, (int)n, ce->pts.p, ce->count.p, cs->pts.p, cs->count.p, st, ce->fe_stat.p,
              cs->fe_stat.p, 3);
    FLOAM_HIP(hipMemcpyAsync(lp->h_out.p, lp->sc.out3.p, sizeof(int) * 3, hipMemcpyDeviceToHost, st));
    FLOAM_HIP(hipStreamSynchronize(st));
    const int status = lp->h_out.p[2];
    if (status & FE_STATUS_SECTOR_TOO_LONG)
      throw Error(FLOAM_ERR_UNSUPPORTED, "a ring sector had no feature scratch (internal error)");
    if (status & FE_STATUS_BAD_RING)
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "point ring index >= num_lines (out of bounds in the reference)");
    const size_t ne = (size_t)lp->h_out.p[0], ns = (size_t)lp->h_out.p[1];
    for (floam_cloud* c : {ce, cs}) {
      c->host_count = c == ce ? ne : ns;
      c->host_count_valid = true;
    }
    ci->host_count = n;
    ci->host_count_valid = true;
    if (ne > edge_cap || ns > surf_cap || (ne && !edge) || (ns && !surf))
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "output capacity too small for the extracted features");
    if (ne) FLOAM_HIP(hipMemcpyAsync(edge, ce->pts.p, ne * sizeof(PointRec), hipMemcpyDeviceToHost, st));
    if (ns) FLOAM_HIP(hipMemcpyAsync(surf, cs->pts.p, ns * sizeof(PointRec), hipMemcpyDeviceToHost, st));
    FLOAM_HIP(hipStreamSynchronize(st));
    *n_edge = ne;
    *n_surf = ns;
    return FLOAM_OK;
  });
}

// ------------------------------------------------------------------------------------------ odometry
floam_status floam_odom_create(const floam_lidar_params* p, double map_resolution, const char* loss, int device,
                               floam_odom** out) {
  return guarded([&] {
    check_params(p);
    if (!out) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null out");
    if (!(map_resolution > 0)) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "map_resolution must be > 0");
    ctx_for(device);
    FLOAM_HIP(hipSetDevice(device));
    auto o = std::make_unique<floam_odom>();
    o->device = device;
    o->lp = *p;
    o->map_resolution = map_resolution;
    if (const char* e = std::getenv("FLOAM_MAP_MERGE")) o->map_merge = e[0] != '0';
    if (const char* e = FLOAM_DIAG_ENV("FLOAM_MAP_FULL")) o->map_force_full = e[0] == '1';
    if (const char* e = FLOAM_DIAG_ENV("FLOAM_MM_VIOLATE")) o->map_violate_mod = std::atoi(e);
    if (const char* e = FLOAM_DIAG_ENV("FLOAM_LM_FAIL_TEST")) o->lmb.fail_test = std::atoi(e) != 0;
    if (const char* e = FLOAM_DIAG_ENV("FLOAM_PEER_DELAY_US")) o->lmb.peer_delay_us = std::atoi(e);
    std::string l = loss ? loss : "";
    std::transform(l.begin(), l.end(), l.begin(), [](unsigned char c) { return (char)std::tolower(c); });
    o->huber = (l == "huber");   // any other string: no robust loss (Q3)
    o->leafE = (float)map_resolution;          // downSizeFilterEdge.setLeafSize(r) (:13)
    o->leafS = (float)(map_resolution * 2);    // downSizeFilterSurf.setLeafSize(2r) (:14)
    cloud_init(&o->mapE, device, 1024);
    cloud_init(&o->mapS, device, 1024);
    cloud_init(&o->mapE_next, device, 1024);
    cloud_init(&o->mapS_next, device, 1024);
    o->cnt.reserve(4);
    DeviceCtx& ctx = ctx_for(device);
    FLOAM_HIP(hipMemsetAsync(o->cnt.p, 0, sizeof(int) * 4, ctx.stream));
    o->lm.reserve(1);
    FLOAM_HIP(hipMemsetAsync(o->lm.p, 0, sizeof(LMState), ctx.stream));
    o->ds.reserve(1);
    odom_dev_init_launch(o->ds.p, ctx.stream);
    const char* pg = std::getenv("FLOAM_GRAPH");   // measured slower than direct launches at C3: opt-in
    o->use_graph = pg && std::atoi(pg) != 0;
    FLOAM_HIP(hipStreamSynchronize(ctx.stream));
    *out = o.release();
    return FLOAM_OK;
  });
}

floam_status floam_odom_destroy(floam_odom* o) {
  return guarded([&] {
    if (o) {
      DeviceCtx& ctx = ctx_for(o->device);
      FLOAM_HIP(hipStreamSynchronize(ctx.stream));
      for (auto& P : o->inflight)
        for (void* b : P.graveyard) (void)hipFree(b);
      o->inflight.clear();
      for (auto& row : o->graph_exec)
        for (auto& ex : row)
          if (ex) FLOAM_HIP(hipGraphExecDestroy(ex));
      radix_stamps_print();
      vox_stamps_print();
      bucket_stamps_print();
      mm_stamps_print();
      geom_stamps_print();
      knn_waves_dump();
      lm_ctrl_stamps_print();
      if (o->dbg_stamps.p) {   // FLOAM_DEBUG_STAMPS: the resident solve's segments in block 0 (100 MHz ticks)
        unsigned long long h[10];
        FLOAM_HIP(hipMemcpy(h, o->dbg_stamps.p, sizeof(h), hipMemcpyDeviceToHost));
        const double n = h[4] ? (double)h[4] : 1.0;
        std::fprintf(stderr, "[floam stamps] %llu solves (block 0, per solve): evaluate + publish %.2f us, all-gather "
                     "%.2f us, reduce %.2f us, control step %.2f us; prologue %.2f us, block 0 first instruction to "
                     "state written %.2f us; inside the evaluations: wave 0's records %.2f us, wave 3's %.2f us\n",
                     h[4], h[0] / n / 100.0, h[1] / n / 100.0, h[2] / n / 100.0, h[3] / n / 100.0, h[5] / n / 100.0,
                     h[6] / n / 100.0, h[7] / n / 100.0, h[8] / n / 100.0);
      }
      if (o->copy) {
        (void)hipStreamSynchronize(o->copy);
        (void)hipStreamDestroy(o->copy);
      }
      if (o->wb_ev) (void)hipEventDestroy(o->wb_ev);
      if (o->side) {
        (void)hipStreamSynchronize(o->side);
        if (o->pre_ev) (void)hipEventDestroy(o->pre_ev);
        (void)hipStreamDestroy(o->side);
      }
      *o->done_ctr = ~0ull;   // (the stream is idle: clouds that still point here never wait)
      if (o->comm) ncclCommDestroy(o->comm);
      shard_peers_release(o);
      if (o->xbuf) (void)hipFree(o->xbuf);
      for (const auto& k : o->keyframes)
        for (floam_cloud* c : {k.surf, k.edge}) floam_cloud_destroy(c);
      for (floam_cloud* c : o->kf_spare) floam_cloud_destroy(c);
      delete o;
    }
    return FLOAM_OK;
  });
}

floam_status floam_odom_init_map(floam_odom* o, const floam_cloud* edge, const floam_cloud* surf) {
  return guarded([&] {
    if (!o || !edge || !surf) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    DeviceCtx& ctx = ctx_for(o->device);
    hipStream_t st = ctx.stream;
    odom_collect(o, ctx, 0);
    cloud_on_main(edge);
    cloud_on_main(surf);
    const size_t ne = cloud_count_sync(edge), ns = cloud_count_sync(surf);
    const size_t mE = cloud_count_sync(&o->mapE), mS = cloud_count_sync(&o->mapS);
    cloud_reserve(&o->mapE, mE + ne + 1, mE, st);
    cloud_reserve(&o->mapS, mS + ns + 1, mS, st);
    append_launch(o->mapE.pts.p, o->mapE.count.p, edge->pts.p, edge->count.p, (int)ne, true, st);
    append_launch(o->mapS.pts.p, o->mapS.count.p, surf->pts.p, surf->count.p, (int)ns, true, st);
    o->mapE_n = mE + ne;
    o->mapS_n = mS + ns;
    o->mapE.host_count = o->mapE_n; o->mapE.host_count_valid = true;
    o->mapS.host_count = o->mapS_n; o->mapS.host_count_valid = true;
    o->grid_dirty = true;
    for (int m = 0; m < 2; ++m) {   // a raw map (Q8): no cell keys until a map update has voxelised it
      o->mmeta[m][o->mkcur].reserve(1);
      FLOAM_HIP(hipMemsetAsync(o->mmeta[m][o->mkcur].p, 0, sizeof(MapMeta), st));
    }
    o->optimization_count = 12;   // (:31)
    FLOAM_HIP(hipStreamSynchronize(st));
    return FLOAM_OK;
  });
}

floam_status floam_odom_update(floam_odom* o, const floam_cloud* edge, const floam_cloud* surf, int type) {
  return guarded([&] {
    if (!o || !edge || !surf) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    if (type < 0 || type > 2) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "bad update type");
    cloud_on_main(edge);
    cloud_on_main(surf);
    return odom_update(o, edge, surf, type);
  });
}

namespace {
floam_status update_selector_impl(floam_odom* o, floam_cloud* edge, floam_cloud* surf, int deskew);
}

floam_status floam_odom_update_selector(floam_odom* o, floam_cloud* edge, floam_cloud* surf, int deskew) {
  return guarded([&] {
    if (!o || !edge || !surf) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    return update_selector_impl(o, edge, surf, deskew);
  });
}

floam_status floam_odom_update_selector_host(floam_odom* o, void* edge, size_t n_edge, void* surf, size_t n_surf,
                                             size_t stride, int deskew) {
  return guarded([&] {
    if (!o || (!edge && n_edge) || (!surf && n_surf)) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    if (stride != sizeof(PointRec))
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "host clouds must be 32-B PointXYZIRT / PointXYZI records");
    if (n_edge > (size_t)INT32_MAX || n_surf > (size_t)INT32_MAX)
      throw Error(FLOAM_ERR_UNSUPPORTED, "cloud larger than 2^31 points");
    DeviceCtx& ctx = ctx_for(o->device);
    FLOAM_HIP(hipSetDevice(o->device));
    odom_collect(o, ctx, 0);   // (a synchronous call: nothing of this handle stays in flight)
    for (auto* c : {&o->h_edge, &o->h_surf})
      if (!*c) {
        *c = std::make_unique<floam_cloud>();
        cloud_init(c->get(), o->device, 0);
      }
    floam_cloud* ce = o->h_edge.get();
    floam_cloud* cs = o->h_surf.get();
    cloud_on_main(ce);
    cloud_on_main(cs);
    FLOAM_HIP(hipStreamSynchronize(ctx.stream));   // (their previous users are done before the buffers are refilled)
    cloud_reserve(ce, std::max<size_t>(n_edge, 1), 0, ctx.stream);
    cloud_reserve(cs, std::max<size_t>(n_surf, 1), 0, ctx.stream);
    if (n_edge) FLOAM_HIP(hipMemcpyAsync(ce->pts.p, edge, n_edge * sizeof(PointRec), hipMemcpyHostToDevice, ctx.stream));
    if (n_surf) FLOAM_HIP(hipMemcpyAsync(cs->pts.p, surf, n_surf * sizeof(PointRec), hipMemcpyHostToDevice, ctx.stream));
    FLOAM_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ce->count.p), (int)n_edge, 1, ctx.stream));
    FLOAM_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(cs->count.p), (int)n_surf, 1, ctx.stream));
    ce->host_count = n_edge;
    cs->host_count = n_surf;
    ce->host_count_valid = cs->host_count_valid = true;
    ce->fe_status = cs->fe_status = nullptr;
    if (deskew && !o->copy) make_stream(&o->copy, false);
    const int depth = o->depth;   // synchronous whatever the streaming mode
    o->depth = 0;
    o->wb = floam_odom::WriteBack{deskew != 0, edge, surf, n_edge, n_surf};
    floam_status r = FLOAM_OK;
    try {
      r = update_selector_impl(o, ce, cs, deskew);
    } catch (...) {
      o->depth = depth;
      if (o->wb.active && o->copy) (void)hipStreamSynchronize(o->copy);
      o->wb.active = false;
      throw;
    }
    o->depth = depth;
    if (o->wb.active) FLOAM_HIP(hipStreamSynchronize(o->copy));
    o->wb.active = false;
    return r;
  });
}

namespace {
floam_status update_selector_impl(floam_odom* o, floam_cloud* edge, floam_cloud* surf, int deskew) {
  {
    if (deskew && edge != surf) odom_prevoxel(o, edge, surf);
    if (deskew && o->pre_valid >= 0) {   // ordered after the grid rebuild (odom_issue)
      o->late_wait[0] = edge;
      o->late_wait[1] = surf;
    } else {
      cloud_on_main(edge);
      cloud_on_main(surf);
    }
    floam_status r;
    try {
      r = deskew ? odom_update_deskew(o, edge, surf) : odom_update(o, edge, surf, FLOAM_VANILLA);
    } catch (...) {
      o->late_wait[0] = o->late_wait[1] = nullptr;
      throw;
    }
    if (!o->use_graph) {   // a later producer on another stream (the next extraction into these buffers) waits for
      hipStream_t st = ctx_for(o->device).stream;   // exactly this update, and not at all once it is collected
      cloud_publish_update(edge, st, o->end_ev, o->done_ctr, o->issued);
      if (surf != edge) cloud_publish_update(surf, st, o->end_ev, o->done_ctr, o->issued);
    }
    return r;
  }
}
}  // namespace

floam_status floam_odom_get_pose(const floam_odom* o, double q[4], double t[3]) {
  return guarded([&] {
    if (!o || !q || !t) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    mat_to_quat(o->odom.R, q);
    for (int i = 0; i < 3; ++i) t[i] = o->odom.t[i];
    return FLOAM_OK;
  });
}

floam_status floam_odom_get_last_pose(const floam_odom* o, double q[4], double t[3]) {
  return guarded([&] {
    if (!o || !q || !t) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    mat_to_quat(o->last_odom.R, q);
    for (int i = 0; i < 3; ++i) t[i] = o->last_odom.t[i];
    return FLOAM_OK;
  });
}

floam_status floam_odom_get_velocity(const floam_odom* o, double v[3]) {
  return guarded([&] {
    if (!o || !v) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    odom_velocity(o, v);
    return FLOAM_OK;
  });
}

floam_status floam_odom_get_map_sizes(floam_odom* o, size_t* corner, size_t* surf) {
  return guarded([&] {
    if (!o) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    odom_collect(o, ctx_for(o->device), 0);
    const size_t e = cloud_count_sync(&o->mapE), s = cloud_count_sync(&o->mapS);
    o->mapE_n = e;
    o->mapS_n = s;
    if (corner) *corner = e;
    if (surf) *surf = s;
    return FLOAM_OK;
  });
}

floam_status floam_odom_download_maps(floam_odom* o, void* corner, size_t ccap, void* surf, size_t scap) {
  return guarded([&] {
    if (!o) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    size_t n;
    floam_status s = floam_cloud_download(&o->mapE, corner, ccap, &n);
    if (s != FLOAM_OK) return s;
    return floam_cloud_download(&o->mapS, surf, scap, &n);
  });
}

floam_status floam_odom_get_map(floam_odom* o, floam_cloud* out) {
  return guarded([&] {
    if (!o || !out) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    DeviceCtx& ctx = ctx_for(o->device);
    odom_collect(o, ctx, 0);
    cloud_on_main(out);
    const size_t e = cloud_count_sync(&o->mapE), s = cloud_count_sync(&o->mapS), n0 = cloud_count_sync(out);
    cloud_reserve(out, n0 + e + s + 1, n0, ctx.stream);
    append_launch(out->pts.p, out->count.p, o->mapS.pts.p, o->mapS.count.p, (int)s, false, ctx.stream);
    append_launch(out->pts.p, out->count.p, o->mapE.pts.p, o->mapE.count.p, (int)e, false, ctx.stream);
    out->host_count = n0 + e + s;
    out->host_count_valid = true;
    return FLOAM_OK;
  });
}

floam_status floam_odom_get_stats(const floam_odom* o, floam_odom_stats* s) {
  return guarded([&] {
    if (!o || !s) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    *s = o->stats;
    return FLOAM_OK;
  });
}

floam_status floam_odom_set_async(floam_odom* o, int depth) {
  return guarded([&] {
    if (!o || depth < 0 || depth > 16) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null handle or depth not in [0, 16]");
    DeviceCtx& ctx = ctx_for(o->device);
    const floam_status w = odom_collect(o, ctx, 0);
    o->collected.clear();
    o->depth = depth;
    return w;
  });
}

floam_status floam_odom_wait(floam_odom* o, size_t max_pending, double* poses, size_t capacity, size_t* n_out) {
  return guarded([&] {
    if (!o) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null handle");
    DeviceCtx& ctx = ctx_for(o->device);
    floam_status w = odom_collect(o, ctx, max_pending);
    if (w == FLOAM_OK) w = o->last_warning;
    o->last_warning = FLOAM_OK;
    const size_t n = o->collected.size() / 7;
    if (n_out) *n_out = n;
    if (poses) std::memcpy(poses, o->collected.data(), sizeof(double) * 7 * std::min(n, capacity));
    o->collected.clear();
    return w;
  });
}

floam_status floam_comm_unique_id(void* id) {
  return guarded([&] {
    if (!id) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null id");
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id is 128 bytes");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) throw Error(FLOAM_ERR_COMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memcpy(id, &u, sizeof(u));
    return FLOAM_OK;
  });
}

floam_status floam_odom_set_shard(floam_odom* o, int rank, int world, const void* id) {
  return guarded([&] {
    if (!o || world < 1 || rank < 0 || rank >= world) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "bad rank / world");
    if (world > 1 && !id) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null unique id");
    odom_collect(o, ctx_for(o->device), 0);
    shard_peers_release(o);
    if (o->comm) {
      ncclCommDestroy(o->comm);
      o->comm = nullptr;
    }
    o->ar_fn = nullptr;
    o->rank = rank;
    o->world = world;
    if (id) {   // a communicator also for world = 1: the RCCL path of the sharded solve on one GPU
      FLOAM_HIP(hipSetDevice(o->device));
      ncclUniqueId u;
      std::memcpy(&u, id, sizeof(u));
      const ncclResult_t r = ncclCommInitRank(&o->comm, world, u, rank);
      if (r != ncclSuccess) throw Error(FLOAM_ERR_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    return FLOAM_OK;
  });
}

// peer sharding: this rank's exchange buffer (zeroed: the exchange tags are odd, lm.hip peer_exchange), allocated
// once.  Uncached device memory: the other ranks poll it over xGMI with system-scope loads, which are served from L2
// (MI355X_MICROARCH.md: sc1 / sc0 sc1 loads bypass L1 only), and coarse-grained memory of another GPU gives no
// cross-device coherence inside a kernel; uncached, every store and poll goes to this GPU's memory.  Without uncached
// memory peer sharding is refused (FLOAM_ERR_UNSUPPORTED: the caller takes the RCCL form) — a cached buffer would
// show up as sporadic 20-s hand-off timeouts, not as an error.
void shard_xbuf(floam_odom* o) {
  if (o->xbuf) return;
  FLOAM_HIP(hipSetDevice(o->device));
  const hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&o->xbuf),
                                             sizeof(unsigned long long) * kShardXchgWords, hipDeviceMallocUncached);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    o->xbuf = nullptr;
    throw Error(FLOAM_ERR_UNSUPPORTED, std::string("peer sharding needs uncached device memory: ") +
                                           hipGetErrorString(e));
  }
  FLOAM_HIP(hipMemset(o->xbuf, 0, sizeof(unsigned long long) * kShardXchgWords));
}

floam_status floam_odom_shard_exchange(floam_odom* o, void* ipc_handle_64, void** dev_ptr) {
  return guarded([&] {
    if (!o || (!ipc_handle_64 && !dev_ptr)) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null handle or outputs");
    shard_xbuf(o);
    if (ipc_handle_64) {
      hipIpcMemHandle_t h;
      FLOAM_HIP(hipIpcGetMemHandle(&h, o->xbuf));
      static_assert(sizeof(h) == 64, "hipIpcMemHandle_t is 64 bytes");
      std::memcpy(ipc_handle_64, &h, sizeof(h));
    }
    if (dev_ptr) *dev_ptr = o->xbuf;
    return FLOAM_OK;
  });
}

floam_status floam_odom_set_shard_peers(floam_odom* o, int rank, int world, const void* ipc_handles,
                                        void* const* dev_ptrs) {
  return guarded([&] {
    if (!o || world < 1 || world > kMaxShardRanks || rank < 0 || rank >= world)
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "bad rank / world (1 <= world <= 8)");
    if (world > 1 && (!ipc_handles == !dev_ptrs))
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "give exactly one of ipc_handles and dev_ptrs");
    DeviceCtx& ctx = ctx_for(o->device);
    odom_collect(o, ctx, 0);
    shard_xbuf(o);   // (may refuse: before the old configuration is torn down, so a refusal leaves it intact)
    if (o->comm) {
      ncclCommDestroy(o->comm);
      o->comm = nullptr;
    }
    o->ar_fn = nullptr;
    shard_peers_release(o);
    // from here on a failure leaves the handle unsharded (world 1), never half-configured
    o->rank = 0;
    o->world = 1;
    ShardPeers P;
    P.world = world;
    P.mine = o->xbuf;
    for (int r = 0; r < world && world > 1; ++r) {
      if (r == rank) {
        P.buf[r] = o->xbuf;
      } else if (dev_ptrs) {
        if (!dev_ptrs[r]) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null peer buffer");
        P.buf[r] = static_cast<const unsigned long long*>(dev_ptrs[r]);
      } else {
        hipIpcMemHandle_t h;
        std::memcpy(&h, static_cast<const char*>(ipc_handles) + 64 * r, sizeof(h));
        void* p = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
          shard_peers_release(o);
          throw Error(FLOAM_ERR_COMM, std::string("hipIpcOpenMemHandle (rank ") + std::to_string(r) +
                                          "): " + hipGetErrorString(e));
        }
        o->xopened.push_back(p);
        P.buf[r] = static_cast<const unsigned long long*>(p);
      }
    }
    // every rank starts a fresh exchange sequence: the counter (LMState::xseq) at zero and its own buffer zeroed, so
    // the tags of all ranks agree whatever each rank ran before (the ranks then meet at a barrier before updating)
    o->lm.reserve(1);
    FLOAM_HIP(hipMemsetAsync(reinterpret_cast<char*>(o->lm.p) + offsetof(LMState, xseq), 0, sizeof(unsigned),
                             ctx.stream));
    FLOAM_HIP(hipMemsetAsync(o->xbuf, 0, sizeof(unsigned long long) * kShardXchgWords, ctx.stream));
    if (world > 1) {   // every peer mapping answers before a solve relies on it (lm.hip peer_probe: <= 2 s)
      o->probe.reserve(1);
      peer_probe_launch(P, rank, o->probe.p, ctx.stream);
      int fail = 0;
      FLOAM_HIP(hipMemcpyAsync(&fail, o->probe.p, sizeof(int), hipMemcpyDeviceToHost, ctx.stream));
      FLOAM_HIP(hipStreamSynchronize(ctx.stream));
      if (fail) {
        shard_peers_release(o);
        std::string ranks;
        for (int r = 0; r < world; ++r)
          if ((fail >> r) & 1) ranks += (ranks.empty() ? "" : ", ") + std::to_string(r);
        throw Error(FLOAM_ERR_COMM, "peer exchange probe: no answer from rank(s) " + ranks +
                                        " within 2 s (the peer mapping does not work; use floam_odom_set_shard)");
      }
    }
    FLOAM_HIP(hipStreamSynchronize(ctx.stream));
    o->peers = P;
    o->rank = rank;
    o->world = world;
    o->peer = world > 1;
    return FLOAM_OK;
  });
}

floam_status floam_odom_set_shard_callback(floam_odom* o, int rank, int world, floam_allreduce_fn fn, void* user) {
  return guarded([&] {
    if (!o || world < 1 || rank < 0 || rank >= world) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "bad rank / world");
    if (world > 1 && !fn) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null all-reduce callback");
    odom_collect(o, ctx_for(o->device), 0);
    shard_peers_release(o);
    if (o->comm) {
      ncclCommDestroy(o->comm);
      o->comm = nullptr;
    }
    o->rank = rank;
    o->world = world;
    o->ar_fn = fn;
    o->ar_user = user;
    return FLOAM_OK;
  });
}

floam_status floam_odom_set_precision(floam_odom* o, int precision) {
  return guarded([&] {
    if (!o || (precision != FLOAM_PRECISION_FP64 && precision != FLOAM_PRECISION_FP32 &&
               precision != FLOAM_PRECISION_FP32_GEOMETRY))
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null handle or unknown precision");
    odom_collect(o, ctx_for(o->device), 0);
    o->fp32 = precision != FLOAM_PRECISION_FP64;
    o->fp32_geom = precision == FLOAM_PRECISION_FP32_GEOMETRY;
    return FLOAM_OK;
  });
}

floam_status floam_odom_set_trace(floam_odom* o, size_t capacity) {
  return guarded([&] {
    if (!o || capacity > (size_t)1 << 24) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null handle or capacity too large");
    DeviceCtx& ctx = ctx_for(o->device);
    odom_collect(o, ctx, 0);
    o->trace_cap = (int)capacity;
    if (capacity) {
      o->trace.reserve(capacity * kTraceWords);
      o->trace_count.reserve(1);
      FLOAM_HIP(hipMemsetAsync(o->trace_count.p, 0, sizeof(unsigned), ctx.stream));
      FLOAM_HIP(hipStreamSynchronize(ctx.stream));
    }
    return FLOAM_OK;
  });
}

floam_status floam_odom_get_traces(floam_odom* o, double* out, size_t capacity, size_t* n_out) {
  return guarded([&] {
    if (!o || o->trace_cap <= 0) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null handle or tracing off");
    DeviceCtx& ctx = ctx_for(o->device);
    odom_collect(o, ctx, 0);
    unsigned n = 0;
    FLOAM_HIP(hipMemcpyAsync(&n, o->trace_count.p, sizeof(unsigned), hipMemcpyDeviceToHost, ctx.stream));
    FLOAM_HIP(hipStreamSynchronize(ctx.stream));
    const size_t k = std::min({(size_t)n, capacity, (size_t)o->trace_cap});
    if (k) {
      if (!out) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null output");
      FLOAM_HIP(hipMemcpy(out, o->trace.p, k * kTraceWords * sizeof(double), hipMemcpyDeviceToHost));
    }
    if (n_out) *n_out = n;
    FLOAM_HIP(hipMemsetAsync(o->trace_count.p, 0, sizeof(unsigned), ctx.stream));
    FLOAM_HIP(hipStreamSynchronize(ctx.stream));
    return FLOAM_OK;
  });
}

floam_status floam_odom_find_correspondences(floam_odom* o, const floam_cloud* edge, const floam_cloud* surf,
                                             const double q[4], const double t[3]) {
  return guarded([&] {
    if (!o || !edge || !surf || !q || !t) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    if (o->trace_cap <= 0) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "tracing off (floam_odom_set_trace)");
    DeviceCtx& ctx = ctx_for(o->device);
    hipStream_t st = ctx.stream;
    FLOAM_HIP(hipSetDevice(o->device));
    odom_collect(o, ctx, 0);
    cloud_on_main(edge);
    cloud_on_main(surf);
    const int ne_ub = (int)cloud_ub(edge), ns_ub = (int)cloud_ub(surf);
    o->dE.reserve(std::max(ne_ub, 1));
    o->dS.reserve(std::max(ns_ub, 1));
    o->cnt.reserve(4);
    VoxelJob je, js;   // VelToIntensityCopy + downSamplingToMap (:53-54, :137-142)
    je.part0 = edge->pts.p; je.d_n0 = edge->count.p; je.n0_ub = ne_ub; je.leaf = o->leafE;
    je.out = o->dE.p; je.d_out = o->cnt.p + 0;
    js.part0 = surf->pts.p; js.d_n0 = surf->count.p; js.n0_ub = ns_ub; js.leaf = o->leafS;
    js.out = o->dS.p; js.d_out = o->cnt.p + 1;
    voxel2_launch(o->vs, je, js, st);
    if (o->grid_dirty) {
      grid_build_launch(o->gE, o->mapE.pts.p, o->mapE.count.p, (int)o->mapE_n, o->gS, o->mapS.pts.p,
                        o->mapS.count.p, (int)o->mapS_n, st, nullptr, false, o->mapE.pts.cap, o->mapS.pts.cap);
      o->grid_dirty = false;
    }
    o->lm.reserve(1);
    o->lmb.reserve(st);
    o->kf_io.reserve(16);
    const double x[7] = {q[0], q[1], q[2], q[3], t[0], t[1], t[2]};
    FLOAM_HIP(hipMemcpyAsync(o->kf_io.p, x, sizeof(x), hipMemcpyHostToDevice, st));
    o->ce.trace = o->cs.trace = true;
    o->last_traced = true;
    QuerySet qe{o->dE.p, o->cnt.p + 0, ne_ub}, qs{o->dS.p, o->cnt.p + 1, ns_ub};
    knn_launch(o->lm.p, o->kf_io.p, qe, o->gE, o->ce, qs, o->gS, o->cs, o->mapE.count.p, o->mapS.count.p, 0, 1, st);
    geom_launch(o->lm.p, qe, o->ce, qs, o->cs, false, o->fp32_geom, o->lmb, st);
    o->last_q[0] = o->dE.p;
    o->last_q[1] = o->dS.p;
    o->last_qn = o->cnt.p;
    FLOAM_HIP(hipStreamSynchronize(st));
    return FLOAM_OK;
  });
}

floam_status floam_odom_get_correspondences(floam_odom* o, int which, void* queries, uint8_t* flags, int* idx,
                                            float* sqd, double* records, size_t capacity, size_t* n_out) {
  return guarded([&] {
    if (!o || (which != 0 && which != 1)) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null handle or bad set");
    if (!o->last_qn) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "no correspondence pass yet");
    if ((idx || sqd) && !o->last_traced)   // (stale indices of an earlier traced pass are never returned)
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "the last correspondence pass ran untraced: no neighbour indices / "
                                              "distances (floam_odom_set_trace before the pass)");
    DeviceCtx& ctx = ctx_for(o->device);
    odom_collect(o, ctx, 0);
    FLOAM_HIP(hipStreamSynchronize(ctx.stream));
    int n = 0;
    FLOAM_HIP(hipMemcpy(&n, o->last_qn + which, sizeof(int), hipMemcpyDeviceToHost));
    const CorrSet& c = which ? o->cs : o->ce;
    n = std::min(n, c.cap);
    if (n_out) *n_out = (size_t)n;
    const size_t k = std::min((size_t)n, capacity);
    if (!k) return FLOAM_OK;
    if (queries)
      FLOAM_HIP(hipMemcpy(queries, o->last_q[which], k * sizeof(PointRec), hipMemcpyDeviceToHost));
    if (flags) FLOAM_HIP(hipMemcpy(flags, c.valid.p, k, hipMemcpyDeviceToHost));
    const int F = which ? SURF_FIELDS : EDGE_FIELDS;
    std::vector<double> rb;
    if (records) {   // SoA [field][cap] -> row-major [k][F]
      rb.resize((size_t)F * c.cap);
      FLOAM_HIP(hipMemcpy(rb.data(), c.rec.p, rb.size() * sizeof(double), hipMemcpyDeviceToHost));
      for (size_t i = 0; i < k; ++i)
        for (int f = 0; f < F; ++f) records[i * F + f] = rb[(size_t)f * c.cap + i];
    }
    if (idx || sqd) {   // k-major [5][cap] -> row-major [k][5]
      std::vector<int> ib((size_t)5 * c.cap);
      std::vector<float> sb((size_t)5 * c.cap);
      FLOAM_HIP(hipMemcpy(ib.data(), c.nnidx.p, ib.size() * sizeof(int), hipMemcpyDeviceToHost));
      FLOAM_HIP(hipMemcpy(sb.data(), c.nnsqd.p, sb.size() * sizeof(float), hipMemcpyDeviceToHost));
      for (size_t i = 0; i < k; ++i)
        for (int j = 0; j < 5; ++j) {
          if (idx) idx[i * 5 + j] = ib[(size_t)j * c.cap + i];
          if (sqd) sqd[i * 5 + j] = sb[(size_t)j * c.cap + i];
        }
    }
    return FLOAM_OK;
  });
}

floam_status floam_odom_keyframe_update(floam_odom* o, const floam_cloud* surf_cloud, const floam_cloud* edge_cloud,
                                        const double q[4], const double t[3], int* is_keyframe) {
  return guarded([&] {
    if (!o || !q || !t) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    for (const floam_cloud* c : {surf_cloud, edge_cloud})
      if (c && c->device != o->device) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "cloud on another device");
    DeviceCtx& ctx = ctx_for(o->device);
    FLOAM_HIP(hipSetDevice(o->device));
    odom_collect(o, ctx, 0);
    o->kf_io.reserve(16);
    const double x[7] = {q[0], q[1], q[2], q[3], t[0], t[1], t[2]};
    FLOAM_HIP(hipMemcpyAsync(o->kf_io.p, x, sizeof(x), hipMemcpyHostToDevice, ctx.stream));
    const bool first = g_keyframe_first;
    g_keyframe_first = false;
    keyframe_update_launch(o->ds.p, o->kf_io.p, first ? 1 : 0, reinterpret_cast<int*>(o->kf_io.p + 8), ctx.stream);
    int flag = 0;
    FLOAM_HIP(hipMemcpyAsync(&flag, o->kf_io.p + 8, sizeof(int), hipMemcpyDeviceToHost, ctx.stream));
    FLOAM_HIP(hipStreamSynchronize(ctx.stream));
    if (flag) {   // currentFrame{pose, edge_cloud, surf_cloud} joins the history (:322, :326, :334): the clouds are
      floam_odom::Keyframe k;   // copied on the device (the reference keeps the caller's shared pointers)
      k.pose = params_to_pose(x);
      floam_cloud** dst[2] = {&k.surf, &k.edge};
      const floam_cloud* src[2] = {surf_cloud, edge_cloud};
      for (int i = 0; i < 2; ++i) {
        if (!src[i]) continue;
        floam_cloud* c = nullptr;
        if (!o->kf_spare.empty()) {
          c = o->kf_spare.back();
          o->kf_spare.pop_back();
        } else {
          chk(floam_cloud_create(o->device, 0, &c));
        }
        *dst[i] = c;
        chk(floam_cloud_copy(c, src[i]));
      }
      keyframe_push(o, k, first);
    }
    if (is_keyframe) *is_keyframe = flag;
    return FLOAM_OK;
  });
}

floam_status floam_odom_get_keyframe(floam_odom* o, size_t index, double q[4], double t[3], floam_cloud* surf_out,
                                     floam_cloud* edge_out, size_t* n_keyframes) {
  return guarded([&] {
    if (!o) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null handle");
    DeviceCtx& ctx = ctx_for(o->device);
    odom_collect(o, ctx, 0);
    if (n_keyframes) *n_keyframes = o->keyframes.size();
    if (!q && !t && !surf_out && !edge_out) return FLOAM_OK;
    if (index >= o->keyframes.size()) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "keyframe index out of range");
    const floam_odom::Keyframe& k = o->keyframes[index];
    if (q) mat_to_quat(k.pose.R, q);
    if (t)
      for (int i = 0; i < 3; ++i) t[i] = k.pose.t[i];
    floam_cloud* outs[2] = {surf_out, edge_out};
    const floam_cloud* src[2] = {k.surf, k.edge};
    for (int i = 0; i < 2; ++i) {
      if (!outs[i]) continue;
      if (src[i]) chk(floam_cloud_copy(outs[i], src[i]));
      else chk(floam_cloud_clear(outs[i]));
    }
    return FLOAM_OK;
  });
}

floam_status floam_profile_enable(int device, int enable) {
  return guarded([&] {
    DeviceCtx& c = ctx_for(device);
    c.profile = enable;
    return FLOAM_OK;
  });
}

floam_status floam_profile_mark(int device, int id) {
  return guarded([&] {
    if (id < 0) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "marker id must be >= 0");
    DeviceCtx& c = ctx_for(device);
    FLOAM_HIP(hipSetDevice(device));
    profile_marker_launch(id, c.stream);
    return FLOAM_OK;
  });
}

floam_status floam_profile_reset(int device) {
  return guarded([&] {
    DeviceCtx& c = ctx_for(device);
    FLOAM_HIP(hipStreamSynchronize(c.stream));
    c.drain();
    c.totals.clear();
    return FLOAM_OK;
  });
}

floam_status floam_profile_read(int device, floam_kernel_timing* out, int max_entries, int* n_out) {
  return guarded([&] {
    DeviceCtx& c = ctx_for(device);
    FLOAM_HIP(hipStreamSynchronize(c.stream));
    c.drain();
    int k = 0;
    for (auto& kv : c.totals) {
      if (k < max_entries && out) out[k] = kv.second;
      ++k;
    }
    if (n_out) *n_out = k;
    return FLOAM_OK;
  });
}

}  // extern "C"

// ------------------------------------------------------------------------------------------ IMU pre-processing
namespace {
// pcl_conversions::fromPCL(stamp, ros::Time) (fromNSec(stamp * 1000)) + ros::Time::toSec()
double pcl_stamp_to_sec(uint64_t stamp_us) {
  const uint64_t ns = stamp_us * 1000ull;
  return (double)(uint32_t)(ns / 1000000000ull) + 1e-9 * (double)(uint32_t)(ns % 1000000000ull);
}
// ros::Time(double) (roscpp_core fromSec: floor, round-half-away nanoseconds, carry) + pcl_conversions::toPCL
// (toNSec() / 1000).  false where ros::Time throws (out of the dual 32-bit range): the stamp is then kept.
bool sec_to_pcl_stamp(double t, uint64_t* stamp_us) {
  const double fl = std::floor(t);
  if (!(fl >= 0.0) || fl > 4294967295.0) return false;
  uint32_t sec = (uint32_t)(int64_t)fl;
  uint32_t nsec = (uint32_t)std::round((t - (double)sec) * 1e9);
  sec += nsec / 1000000000ul;
  nsec %= 1000000000ul;
  *stamp_us = ((uint64_t)sec * 1000000000ull + (uint64_t)nsec) / 1000ull;
  return true;
}
size_t imu_lower_bound(const floam_imu* h, double ts) {   // std::lower_bound with dmapping::compare
  return (size_t)(std::lower_bound(h->t.begin(), h->t.end(), ts) - h->t.begin());
}
// ImuHandler::Get (src/dataHandler.cpp:48-75): the sample before the lower bound, or the zero orientation of a
// default-constructed sensor_msgs::Imu
bool imu_get(const floam_imu* h, double ts, Q4* out) {
  const size_t a = imu_lower_bound(h, ts);
  if (a != h->t.size() && a != 0 && a - 1 != 0) {
    *out = h->q[a - 1];
    return true;
  }
  *out = Q4{0.0, 0.0, 0.0, 0.0};
  return false;
}
bool imu_time_contained(const floam_imu* h, double ts) {   // ImuHandler::TimeContained (:76-81)
  return !h->t.empty() && ts >= h->t.front() && ts <= h->t.back();
}
bool imu_add(floam_imu* h, double stamp, const double* q) {   // ImuHandler::AddMsg (:23-38)
  if (!h->t.empty() && !(stamp - h->t.back() > 0.00001)) return false;
  h->t.push_back(stamp);
  h->q.push_back(Q4{q[0], q[1], q[2], q[3]});
  return true;
}
// bring the HBM mirror of the stream up to date (stream-ordered; the caller synchronises before returning)
void imu_upload(floam_imu* h, hipStream_t st) {
  const size_t n = h->t.size();
  if (n > h->dcap) {
    const size_t cap = std::max<size_t>(1024, n + n / 2);
    double* nt = nullptr;
    Q4* nq = nullptr;
    FLOAM_HIP(hipMalloc(&nt, cap * sizeof(double)));
    FLOAM_HIP(hipMalloc(&nq, cap * sizeof(Q4)));
    if (h->uploaded) {
      FLOAM_HIP(hipMemcpyAsync(nt, h->d_t, h->uploaded * sizeof(double), hipMemcpyDeviceToDevice, st));
      FLOAM_HIP(hipMemcpyAsync(nq, h->d_q, h->uploaded * sizeof(Q4), hipMemcpyDeviceToDevice, st));
      FLOAM_HIP(hipStreamSynchronize(st));
    }
    if (h->d_t) FLOAM_HIP(hipFree(h->d_t));
    if (h->d_q) FLOAM_HIP(hipFree(h->d_q));
    h->d_t = nt;
    h->d_q = nq;
    h->dcap = cap;
  }
  if (n > h->uploaded) {
    FLOAM_HIP(hipMemcpyAsync(h->d_t + h->uploaded, h->t.data() + h->uploaded, (n - h->uploaded) * sizeof(double),
                             hipMemcpyHostToDevice, st));
    FLOAM_HIP(hipMemcpyAsync(h->d_q + h->uploaded, h->q.data() + h->uploaded, (n - h->uploaded) * sizeof(Q4),
                             hipMemcpyHostToDevice, st));
    h->uploaded = n;
  }
}

// mode = OR of IMU_CENTER / IMU_COMPENSATE / IMU_ALIGN.  The scalar part (stamps, TimeContained, qInit, the LDS
// window) runs on the host from the cloud's front / back times (one 12-B read-back); the per-point part is one
// fused pass.  Returns false when Compensate would return false ("no imu data"); `in` is centred regardless.
bool imu_pre(int mode, floam_imu* h, floam_cloud* in, uint64_t* stamp_us, const double* extr, floam_cloud* out) {
  DeviceCtx& ctx = ctx_for(in->device);
  hipStream_t st = ctx.stream;
  FLOAM_HIP(hipSetDevice(in->device));
  cloud_on_main(in);
  if (out) cloud_on_main(out);
  if (mode & IMU_COMPENSATE) imu_upload(h, st);
  ctx.ends.reserve(3);
  ctx.h_ends.reserve(3);
  int* h_ends = ctx.h_ends.p;
  cloud_ends_launch(in->pts.p, in->count.p, ctx.ends.p, st);
  FLOAM_HIP(hipMemcpyAsync(h_ends, ctx.ends.p, sizeof(int) * 3, hipMemcpyDeviceToHost, st));
  FLOAM_HIP(hipStreamSynchronize(st));
  const int n = h_ends[0];
  in->host_count = (size_t)std::max(n, 0);
  in->host_count_valid = true;
  if (n <= 0) return false;
  float front, back;
  std::memcpy(&front, &h_ends[1], 4);
  std::memcpy(&back, &h_ends[2], 4);
  ImuPrepArgs a{};
  uint64_t stamp = *stamp_us;
  if (mode & IMU_CENTER) {   // CenterTime (src/laserProcessingNode.cpp:65-78)
    a.tScan = pcl_stamp_to_sec(stamp);
    const double tEnd = a.tScan + (double)back;
    const double tBegin = a.tScan + (double)front;
    a.tCenter = tBegin + (tEnd - tBegin) / 2.0;
    sec_to_pcl_stamp(a.tCenter, &stamp);
    front = (float)(((double)front + a.tScan) - a.tCenter);
    back = (float)(((double)back + a.tScan) - a.tCenter);
  }
  int launch_mode = mode;
  bool ok = true;
  if (mode & IMU_COMPENSATE) {   // dmapping::Compensate (src/dataHandler.cpp:93-122)
    a.tScan2 = pcl_stamp_to_sec(stamp);
    const double t0 = (double)front + a.tScan2, t1 = (double)back + a.tScan2;
    if (!imu_time_contained(h, t0) || !imu_time_contained(h, t1)) {
      ok = false;
      launch_mode = mode & IMU_CENTER;
    } else {
      a.extr = Q4{extr[0], extr[1], extr[2], extr[3]};
      Q4 qs;
      imu_get(h, a.tScan2, &qs);
      const Q4 qInit = q4_mul(qs, a.extr);
      a.qInitInv = q4_inverse(qInit);
      const double qv[4] = {qInit.x, qInit.y, qInit.z, qInit.w};
      const Mat3 R = quat_to_mat(qv);   // Eigen::Affine3d ImuNowT(q) (:109-110), translation 0
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) a.R[3 * r + c] = R.m[r][c];
      a.stamps = h->d_t;
      a.orient = h->d_q;
      a.n_imu = (int)h->t.size();
      const size_t lb0 = imu_lower_bound(h, std::min(t0, t1)), lb1 = imu_lower_bound(h, std::max(t0, t1));
      a.win_lo = (int)(lb0 > 0 ? lb0 - 1 : 0);
      a.win_hi = (int)std::min(h->t.size(), lb1 + 1);
      a.win_hi = std::min(a.win_hi, a.win_lo + kImuWindow);
    }
  }
  if (launch_mode & IMU_COMPENSATE) {
    cloud_reserve(out, (size_t)n, 0, st);
    ProfScope ps(ctx, "imu_preprocess", FLOAM_PROF_CLOUD, 68.0 * (double)n);
    imu_prep_launch(launch_mode, in->pts.p, out->pts.p, in->count.p, n, a, st);
    FLOAM_HIP(hipMemcpyAsync(out->count.p, in->count.p, sizeof(int), hipMemcpyDeviceToDevice, st));
    out->host_count = (size_t)n;
    out->host_count_valid = true;
  } else if (launch_mode & IMU_CENTER) {
    ProfScope ps(ctx, "center_time", FLOAM_PROF_CLOUD, 36.0 * (double)n);
    imu_prep_launch(IMU_CENTER, in->pts.p, nullptr, in->count.p, n, a, st);
  }
  *stamp_us = stamp;
  return ok;
}
}  // namespace

extern "C" {

floam_status floam_imu_create(int device, floam_imu** out) {
  return guarded([&] {
    if (!out) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null out");
    ctx_for(device);
    auto h = std::make_unique<floam_imu>();
    h->device = device;
    *out = h.release();
    return FLOAM_OK;
  });
}

floam_status floam_imu_destroy(floam_imu* h) {
  return guarded([&] {
    if (h) {
      FLOAM_HIP(hipStreamSynchronize(ctx_for(h->device).stream));
      if (h->d_t) FLOAM_HIP(hipFree(h->d_t));
      if (h->d_q) FLOAM_HIP(hipFree(h->d_q));
      delete h;
    }
    return FLOAM_OK;
  });
}

floam_status floam_imu_add_msg(floam_imu* h, double stamp, const double q_xyzw[4], int* added) {
  return guarded([&] {
    if (!h || !q_xyzw) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    const bool a = imu_add(h, stamp, q_xyzw);
    if (added) *added = a ? 1 : 0;
    return FLOAM_OK;
  });
}

floam_status floam_imu_add_msgs(floam_imu* h, const double* stamps, const double* q_xyzw, size_t n, size_t* added) {
  return guarded([&] {
    if (!h || (n && (!stamps || !q_xyzw))) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    size_t k = 0;
    for (size_t i = 0; i < n; ++i) k += imu_add(h, stamps[i], q_xyzw + 4 * i) ? 1 : 0;
    if (added) *added = k;
    return FLOAM_OK;
  });
}

floam_status floam_imu_size(const floam_imu* h, size_t* n) {
  return guarded([&] {
    if (!h || !n) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    *n = h->t.size();
    return FLOAM_OK;
  });
}

floam_status floam_imu_get(const floam_imu* h, double t, double q_xyzw[4], int* found) {
  return guarded([&] {
    if (!h || !q_xyzw) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    Q4 q;
    const bool f = imu_get(h, t, &q);
    q_xyzw[0] = q.x; q_xyzw[1] = q.y; q_xyzw[2] = q.z; q_xyzw[3] = q.w;
    if (found) *found = f ? 1 : 0;
    return FLOAM_OK;
  });
}

floam_status floam_imu_time_contained(const floam_imu* h, double t, int* contained) {
  return guarded([&] {
    if (!h || !contained) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    *contained = imu_time_contained(h, t) ? 1 : 0;
    return FLOAM_OK;
  });
}

floam_status floam_euler_to_quaternion(double roll, double pitch, double yaw, double q_xyzw[4]) {
  return guarded([&] {
    if (!q_xyzw) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    auto aa = [](double deg, int axis) {   // AngleAxisd(deg * M_PI / 180.0, Unit*()) -> Quaterniond
      const double ha = 0.5 * (deg * M_PI / 180.0);
      const double s = std::sin(ha);
      Q4 q{0.0 * s, 0.0 * s, 0.0 * s, std::cos(ha)};
      if (axis == 0) q.x = 1.0 * s;
      if (axis == 1) q.y = 1.0 * s;
      if (axis == 2) q.z = 1.0 * s;
      return q;
    };
    const Q4 q = q4_mul(q4_mul(aa(roll, 0), aa(yaw, 2)), aa(pitch, 1));   // rollAngle * yawAngle * pitchAngle
    q_xyzw[0] = q.x; q_xyzw[1] = q.y; q_xyzw[2] = q.z; q_xyzw[3] = q.w;
    return FLOAM_OK;
  });
}

floam_status floam_center_time(floam_cloud* cloud, uint64_t* stamp_us) {
  return guarded([&] {
    if (!cloud || !stamp_us) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    imu_pre(IMU_CENTER, nullptr, cloud, stamp_us, nullptr, nullptr);
    return FLOAM_OK;
  });
}

floam_status floam_imu_compensate(floam_imu* h, floam_cloud* in, uint64_t stamp_us, const double extr_xyzw[4],
                                  floam_cloud* compensated) {
  return guarded([&] {
    if (!h || !in || !extr_xyzw || !compensated) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    if (in == compensated) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "clouds must be distinct");
    if (in->device != h->device || compensated->device != h->device)
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "clouds and handle on different devices");
    uint64_t st = stamp_us;
    return imu_pre(IMU_COMPENSATE, h, in, &st, extr_xyzw, compensated) ? FLOAM_OK : FLOAM_WARN_NO_IMU_DATA;
  });
}

floam_status floam_imu_preprocess(floam_imu* h, floam_cloud* in, uint64_t* stamp_us, const double extr_xyzw[4],
                                  floam_cloud* aligned) {
  return guarded([&] {
    if (!h || !in || !stamp_us || !extr_xyzw || !aligned) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    if (in == aligned) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "clouds must be distinct");
    if (in->device != h->device || aligned->device != h->device)
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "clouds and handle on different devices");
    return imu_pre(IMU_CENTER | IMU_COMPENSATE | IMU_ALIGN, h, in, stamp_us, extr_xyzw, aligned)
               ? FLOAM_OK
               : FLOAM_WARN_NO_IMU_DATA;
  });
}

}  // extern "C"

// ------------------------------------------------------------------------------------------ wire formats
namespace {
struct FieldDesc {   // the registered fields of the point type (POINT_CLOUD_REGISTER_POINT_STRUCT order)
  const char* name;
  uint32_t offset;
  uint8_t datatype;
  uint32_t count;
};
// vel_point::PointXYZIRT (include/lidar.h:26-32) and pcl::PointXYZI
const FieldDesc kXYZIRT[] = {{"x", 0, 7, 1}, {"y", 4, 7, 1}, {"z", 8, 7, 1},
                             {"intensity", 16, 7, 1}, {"ring", 20, 4, 1}, {"time", 24, 7, 1}};
const FieldDesc kXYZI[] = {{"x", 0, 7, 1}, {"y", 4, 7, 1}, {"z", 8, 7, 1}, {"intensity", 16, 7, 1}};
size_t field_bytes(uint8_t dt) { return dt == 4 ? 2 : 4; }   // sizeof the struct member type (uint16 / float)
}  // namespace

extern "C" {

floam_status floam_pointcloud2_fields(int point_type, floam_pc2_field* out, size_t capacity, size_t* n_out,
                                      uint32_t* point_step) {
  return guarded([&] {
    if (point_type != FLOAM_POINT_XYZIRT && point_type != FLOAM_POINT_XYZI)
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "unknown point type");
    const FieldDesc* f = point_type == FLOAM_POINT_XYZIRT ? kXYZIRT : kXYZI;
    const size_t n = point_type == FLOAM_POINT_XYZIRT ? 6 : 4;
    for (size_t i = 0; i < n && i < capacity && out; ++i) {
      std::memset(&out[i], 0, sizeof(out[i]));
      std::strncpy(out[i].name, f[i].name, sizeof(out[i].name) - 1);
      out[i].offset = f[i].offset;
      out[i].datatype = f[i].datatype;
      out[i].count = f[i].count;
    }
    if (n_out) *n_out = n;
    if (point_step) *point_step = (uint32_t)sizeof(PointRec);
    return FLOAM_OK;
  });
}

floam_status floam_cloud_from_pointcloud2(floam_cloud* out, int point_type, const void* data, size_t data_size,
                                          uint32_t width, uint32_t height, uint32_t point_step, uint32_t row_step,
                                          const floam_pc2_field* fields, size_t nfields) {
  return guarded([&] {
    if (!out || (nfields && !fields)) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    if (point_type != FLOAM_POINT_XYZIRT && point_type != FLOAM_POINT_XYZI)
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "unknown point type");
    const size_t n = (size_t)width * height;
    if (n > (size_t)INT32_MAX) throw Error(FLOAM_ERR_UNSUPPORTED, "cloud larger than 2^31 points");
    if (n && !data) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null data");
    if (n && ((size_t)(height - 1) * row_step + (size_t)(width - 1) * point_step + point_step > data_size))
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "data smaller than height * row_step");
    // detail::FieldMapper (PCL 1.8.1 conversions.h): per registered field, the first message field with the same
    // name, datatype and count (count 0 accepted for scalars); missing fields only warn (#595)
    const FieldDesc* f = point_type == FLOAM_POINT_XYZIRT ? kXYZIRT : kXYZI;
    const size_t nf = point_type == FLOAM_POINT_XYZIRT ? 6 : 4;
    std::vector<Pc2Mapping> map;
    bool missing = false;
    for (size_t k = 0; k < nf; ++k) {
      bool found = false;
      for (size_t j = 0; j < nfields; ++j) {
        const floam_pc2_field& m = fields[j];
        if (std::strncmp(m.name, f[k].name, sizeof(m.name)) == 0 && m.datatype == f[k].datatype &&
            (m.count == 1 || m.count == 0)) {
          map.push_back(Pc2Mapping{(int)m.offset, (int)f[k].offset, (int)field_bytes(f[k].datatype)});
          found = true;
          break;
        }
      }
      if (!found) missing = true;
    }
    for (const auto& m : map)
      if ((size_t)m.serialized_offset + (size_t)m.size > point_step)
        throw Error(FLOAM_ERR_INVALID_ARGUMENT, "field extends past point_step");
    // coalesce adjacent fields with equal serialized / struct gaps (createMapping)
    std::sort(map.begin(), map.end(),
              [](const Pc2Mapping& a, const Pc2Mapping& b) { return a.serialized_offset < b.serialized_offset; });
    if (map.size() > 1) {
      size_t i = 0;
      for (size_t j = 1; j < map.size();) {
        if (map[j].serialized_offset - map[i].serialized_offset == map[j].struct_offset - map[i].struct_offset) {
          map[i].size += (map[j].struct_offset + map[j].size) - (map[i].struct_offset + map[i].size);
          map.erase(map.begin() + (long)j);
        } else {
          ++i;
          ++j;
        }
      }
    }
    Pc2Decode d{};
    d.row_step = row_step;
    d.point_step = (int)point_step;
    d.width = (int)width;
    d.height = (int)height;
    d.nmap = (int)map.size();
    for (size_t k = 0; k < map.size(); ++k) d.map[k] = map[k];
    d.whole = (map.size() == 1 && map[0].serialized_offset == 0 && map[0].struct_offset == 0 &&
               point_step == sizeof(PointRec)) ? 1 : 0;
    DeviceCtx& ctx = ctx_for(out->device);
    FLOAM_HIP(hipSetDevice(out->device));
    cloud_on_main(out);
    FLOAM_HIP(hipStreamSynchronize(ctx.stream));   // the staging buffer may still feed an earlier decode
    cloud_reserve(out, std::max<size_t>(n, 1), 0, ctx.stream);
    if (n) {
      const size_t bytes = (size_t)(height - 1) * row_step + (size_t)width * point_step;
      ctx.msg.reserve(bytes);
      FLOAM_HIP(hipMemcpyAsync(ctx.msg.p, data, bytes, hipMemcpyHostToDevice, ctx.stream));
      d.data = ctx.msg.p;
      ProfScope ps(ctx, "pc2_decode", FLOAM_PROF_CLOUD, (double)bytes + 32.0 * (double)n);
      pc2_decode_launch(d, out->pts.p, ctx.stream);
    }
    const int cnt = (int)n;
    FLOAM_HIP(hipMemcpyAsync(out->count.p, &cnt, sizeof(int), hipMemcpyHostToDevice, ctx.stream));
    FLOAM_HIP(hipStreamSynchronize(ctx.stream));   // pageable sources: the caller may reuse its buffers
    out->host_count = n;
    out->host_count_valid = true;
    return missing ? FLOAM_WARN_FIELD_MISSING : FLOAM_OK;
  });
}

floam_status floam_transform_cloud(const floam_cloud* in, const double m[16], floam_cloud* out) {
  return guarded([&] {
    if (!in || !m || !out) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    if (in->device != out->device) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "clouds on different devices");
    DeviceCtx& ctx = ctx_for(in->device);
    FLOAM_HIP(hipSetDevice(in->device));
    cloud_on_main(in);
    cloud_on_main(out);
    const size_t n = cloud_ub(in);
    if (in != out) cloud_reserve(out, std::max<size_t>(n, 1), 0, ctx.stream);
    const double m34[12] = {m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7], m[8], m[9], m[10], m[11]};
    if (n) {
      ProfScope ps(ctx, "transform_cloud", FLOAM_PROF_CLOUD, 64.0 * (double)n);
      transform_cloud_launch(in->pts.p, in->count.p, (int)n, m34, out->pts.p, ctx.stream);
    }
    if (in != out) {
      FLOAM_HIP(hipMemcpyAsync(out->count.p, in->count.p, sizeof(int), hipMemcpyDeviceToDevice, ctx.stream));
      out->host_count = in->host_count;
      out->host_count_valid = in->host_count_valid;
      out->ub = in->ub;
    }
    return FLOAM_OK;
  });
}

}  // extern "C"

// ------------------------------------------------------------------------------------------ global map
namespace {
void mapping_update(floam_mapping* m, const floam_cloud* in, const double* q, const double* t) {
  DeviceCtx& ctx = ctx_for(m->device);
  hipStream_t st = ctx.stream;
  FLOAM_HIP(hipSetDevice(m->device));
  cloud_on_main(in);
  const int n = (int)cloud_count_sync(in);
  // current_pose = Isometry3d::Identity().rotate(q).pretranslate(t) (src/laserMappingNode.cpp:108-110)
  const Mat3 R = quat_to_mat(q);
  auto cell_of = [](double v) { return (int)std::floor(v / 50.0 + 0.5); };
  const int px = cell_of(t[0]), py = cell_of(t[1]), pz = cell_of(t[2]);
  const int ncell_old = (int)m->keys.size();
  // 1. transform + cells of the new points, distinct cells counted
  std::unordered_map<unsigned long long, int> touched;   // key -> new points
  std::vector<int> slot_of;                              // touched cell -> hash slot
  if (n > 0) {
    m->stage.reserve(n);
    m->slot.reserve(n);
    m->hkeys.reserve(kMapHashSlots);
    m->hcnt.reserve(kMapHashSlots + 1);   // [kMapHashSlots] = overflow flag
    m->h_keys.reserve(kMapHashSlots);
    m->h_cnt.reserve(kMapHashSlots + 1);
    m->rs.reserve(n, st);
    FLOAM_HIP(hipMemsetAsync(m->hkeys.p, 0xFF, sizeof(unsigned long long) * kMapHashSlots, st));
    FLOAM_HIP(hipMemsetAsync(m->hcnt.p, 0, sizeof(int) * (kMapHashSlots + 1), st));
    MapPrepArgs a{};
    a.in = in->pts.p; a.d_n = in->count.p; a.n = n;
    for (int r = 0; r < 3; ++r) {   // pose_current.cast<float>() (src/laserMappingClass.cpp:157)
      for (int c = 0; c < 3; ++c) a.m[4 * r + c] = (float)R.m[r][c];
      a.m[4 * r + 3] = (float)t[r];
    }
    a.stage = m->stage.p; a.slot = m->slot.p; a.hkeys = m->hkeys.p; a.hcnt = m->hcnt.p;
    a.overflow = m->hcnt.p + kMapHashSlots; a.radix_ctl = m->rs.ctl.p;
    {
      ProfScope ps(ctx, "map_prep", FLOAM_PROF_CLOUD, 64.0 * n);
      map_prep_launch(a, st);
    }
    FLOAM_HIP(hipMemcpyAsync(m->h_keys.p, m->hkeys.p, sizeof(unsigned long long) * kMapHashSlots,
                             hipMemcpyDeviceToHost, st));
    FLOAM_HIP(hipMemcpyAsync(m->h_cnt.p, m->hcnt.p, sizeof(int) * (kMapHashSlots + 1), hipMemcpyDeviceToHost, st));
    FLOAM_HIP(hipStreamSynchronize(st));
    if (m->h_cnt.p[kMapHashSlots])
      throw Error(FLOAM_ERR_UNSUPPORTED, "one update touches more than 2048 map cells (100 km of 50-m cells)");
    for (int h = 0; h < kMapHashSlots; ++h)
      if (m->h_keys.p[h] != ~0ull) touched[m->h_keys.p[h]] = m->h_cnt.p[h];
  }
  // 2. the merged cell table; the neighbourhood of the pose is filtered (src/laserMappingClass.cpp:174-183)
  std::vector<unsigned long long> keys = m->keys;
  for (const auto& kv : touched)
    if (!std::binary_search(m->keys.begin(), m->keys.end(), kv.first)) keys.push_back(kv.first);
  std::sort(keys.begin(), keys.end());
  const int nc = (int)keys.size();
  // per cell: [0] old start, [1] old count, [2] new count, [3] new start, [4] voxel offset (-1: copied), [5] out count
  std::vector<int> old_start(nc, -1), seg(2 * nc, 0), new_start(nc, 0), vox_off(nc, -1), outcnt(nc, 0);
  {
    int os = 0, k = 0;
    for (int c = 0; c < nc; ++c) {
      if (k < ncell_old && m->keys[k] == keys[c]) {
        old_start[c] = os;
        seg[2 * c] = m->counts[k];
        os += m->counts[k];
        ++k;
      }
      auto it = touched.find(keys[c]);
      seg[2 * c + 1] = it == touched.end() ? 0 : it->second;
    }
  }
  int ns = 0, vs_total = 0;
  std::vector<int> filtered;
  for (int c = 0; c < nc; ++c) {
    new_start[c] = ns;
    ns += seg[2 * c + 1];
    int x, y, z;
    map_cell_coords(keys[c], x, y, z);
    const bool in_nb = std::abs(x - px) <= 2 && std::abs(y - py) <= 2 && std::abs(z - pz) <= 2;
    const int tot = seg[2 * c] + seg[2 * c + 1];
    outcnt[c] = tot;
    if (in_nb && tot > 0) {
      vox_off[c] = vs_total;
      vs_total += tot;
      filtered.push_back(c);
    }
  }
  const int total_ub = ns + (int)(m->map.host_count_valid ? m->map.host_count : m->map.ub);
  // device copies of the per-cell tables: [old_start | seg (2) | new_start | vox_off | outcnt | off (nc + 1)]
  m->cellv.reserve((size_t)7 * nc + 2);
  m->h_cellv.reserve((size_t)7 * nc + 2);
  int* hv = m->h_cellv.p;
  std::memcpy(hv, old_start.data(), sizeof(int) * nc);
  std::memcpy(hv + nc, seg.data(), sizeof(int) * 2 * nc);
  std::memcpy(hv + 3 * nc, new_start.data(), sizeof(int) * nc);
  std::memcpy(hv + 4 * nc, vox_off.data(), sizeof(int) * nc);
  std::memcpy(hv + 5 * nc, outcnt.data(), sizeof(int) * nc);
  FLOAM_HIP(hipMemcpyAsync(m->cellv.p, hv, sizeof(int) * 6 * nc, hipMemcpyHostToDevice, st));
  int* d_old_start = m->cellv.p;
  int* d_seg = m->cellv.p + nc;
  int* d_new_start = m->cellv.p + 3 * nc;
  int* d_vox_off = m->cellv.p + 4 * nc;
  int* d_outcnt = m->cellv.p + 5 * nc;
  int* d_off = m->cellv.p + 6 * nc;
  // 3. new points grouped by cell (stable radix sort by the cell's rank)
  if (n > 0) {
    m->hrank.reserve(kMapHashSlots);
    std::vector<int> hrank(kMapHashSlots, 0);
    for (int h = 0; h < kMapHashSlots; ++h)
      if (m->h_keys.p[h] != ~0ull)
        hrank[h] = (int)(std::lower_bound(keys.begin(), keys.end(), m->h_keys.p[h]) - keys.begin());
    FLOAM_HIP(hipMemcpyAsync(m->hrank.p, hrank.data(), sizeof(int) * kMapHashSlots, hipMemcpyHostToDevice, st));
    m->ss.reserve(n);
    m->sorted.reserve(n);
    map_rank_keys_launch(m->slot.p, m->hrank.p, n, m->ss.k0.p, m->ss.v0.p, m->rs.ctl.p, st);
    radix_sort_launch(m->rs, m->ss.k0.p, m->ss.v0.p, m->ss.k1.p, m->ss.v1.p, n, st);
    map_gather_launch(m->stage.p, m->ss.v0.p, n, m->sorted.p, st);
    FLOAM_HIP(hipStreamSynchronize(st));   // hrank is a pageable source
  }
  // 4. VoxelGrid of the neighbourhood's cells, two per pipeline launch
  m->vox.reserve(std::max(vs_total, 1));
  if (!ctx.zero.p) {
    ctx.zero.reserve(2);
    FLOAM_HIP(hipMemsetAsync(ctx.zero.p, 0, sizeof(int) * 2, st));
  }
  m->vs.s.reserve(1);
  for (size_t f = 0; f < filtered.size(); f += 2) {
    VoxelJob job[2];
    for (int u = 0; u < 2; ++u) {
      VoxelJob& J = job[u];
      J.leaf = m->leaf;
      if (f + u < filtered.size()) {
        const int c = filtered[f + u];
        J.part0 = m->map.pts.p + std::max(old_start[c], 0);
        J.d_n0 = d_seg + 2 * c;
        J.n0_ub = seg[2 * c];
        J.part1 = m->sorted.p + new_start[c];
        J.d_n1 = d_seg + 2 * c + 1;
        J.n1_ub = seg[2 * c + 1];
        J.out = m->vox.p + vox_off[c];
        J.d_out = d_outcnt + c;
      } else {   // empty second job
        J.part0 = m->vox.p; J.d_n0 = ctx.zero.p; J.n0_ub = 0;
        J.out = m->vox.p; J.d_out = ctx.zero.p + 1;
      }
    }
    ProfScope ps(ctx, "map_voxel", FLOAM_PROF_CLOUD, 0.0);
    voxel2_launch(m->vs, job[0], job[1], st);
  }
  // 5. the new map in cell order
  cloud_reserve(&m->next, std::max(total_ub, 1), 0, st);
  MapCopyArgs c{};
  c.ncell = nc; c.outcnt = d_outcnt; c.off = d_off; c.old_start = d_old_start; c.seg = d_seg;
  c.new_start = d_new_start; c.vox_off = d_vox_off; c.old_map = m->map.pts.p; c.new_pts = m->sorted.p;
  c.vox = m->vox.p; c.out = m->next.pts.p; c.d_total = m->next.count.p;
  {
    ProfScope ps(ctx, "map_rebuild", FLOAM_PROF_CLOUD, 64.0 * total_ub);
    map_rebuild_launch(c, total_ub, st);
  }
  FLOAM_HIP(hipMemcpyAsync(hv + 5 * nc, d_outcnt, sizeof(int) * (size_t)nc, hipMemcpyDeviceToHost, st));
  FLOAM_HIP(hipStreamSynchronize(st));
  m->keys.clear();
  m->counts.clear();
  size_t total = 0;
  for (int k = 0; k < nc; ++k) {
    const int v = hv[5 * nc + k];
    if (v < 0) throw Error(FLOAM_ERR_DEVICE, "voxel-grid compaction failed (lookback timeout)");
    if (v == 0) continue;   // empty cells contribute nothing to getMap
    m->keys.push_back(keys[k]);
    m->counts.push_back(v);
    total += (size_t)v;
  }
  cloud_swap(&m->map, &m->next);
  m->map.host_count = total;
  m->map.host_count_valid = true;
  m->map.last_stream = st;
}
}  // namespace

extern "C" {

floam_status floam_mapping_create(double map_resolution, int device, floam_mapping** out) {
  return guarded([&] {
    if (!out) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null out");
    if (!(map_resolution > 0.0)) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "map_resolution must be > 0");
    ctx_for(device);
    FLOAM_HIP(hipSetDevice(device));
    auto m = std::make_unique<floam_mapping>();
    m->device = device;
    m->leaf = (float)map_resolution;   // downSizeFilter.setLeafSize (src/laserMappingClass.cpp:31)
    cloud_init(&m->map, device, 0);
    cloud_init(&m->next, device, 0);
    *out = m.release();
    return FLOAM_OK;
  });
}

floam_status floam_mapping_destroy(floam_mapping* m) {
  return guarded([&] {
    if (m) {
      FLOAM_HIP(hipStreamSynchronize(ctx_for(m->device).stream));
      delete m;
    }
    return FLOAM_OK;
  });
}

floam_status floam_mapping_update(floam_mapping* m, const floam_cloud* in, const double q_xyzw[4], const double t[3]) {
  return guarded([&] {
    if (!m || !in || !q_xyzw || !t) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    if (in->device != m->device) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "cloud and handle on different devices");
    mapping_update(m, in, q_xyzw, t);
    return FLOAM_OK;
  });
}

floam_status floam_mapping_size(const floam_mapping* m, size_t* n) {
  return guarded([&] {
    if (!m || !n) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    *n = m->map.host_count;
    return FLOAM_OK;
  });
}

floam_status floam_mapping_get_map(floam_mapping* m, floam_cloud* out) {
  return guarded([&] {
    if (!m || !out) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    if (out->device != m->device) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "cloud and handle on different devices");
    DeviceCtx& ctx = ctx_for(m->device);
    cloud_on_main(out);
    const size_t n = m->map.host_count;
    cloud_reserve(out, std::max<size_t>(n, 1), 0, ctx.stream);
    if (n)
      FLOAM_HIP(hipMemcpyAsync(out->pts.p, m->map.pts.p, n * sizeof(PointRec), hipMemcpyDeviceToDevice, ctx.stream));
    FLOAM_HIP(hipMemcpyAsync(out->count.p, m->map.count.p, sizeof(int), hipMemcpyDeviceToDevice, ctx.stream));
    out->host_count = n;
    out->host_count_valid = true;
    return FLOAM_OK;
  });
}

}  // extern "C"
