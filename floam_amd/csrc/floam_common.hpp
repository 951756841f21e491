// Shared host/device definitions of the MI355X-native FLOAM core (gfx950, CDNA4).
#pragma once
#include <memory>
#include <hip/hip_runtime.h>

#include <cstddef>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

// Diagnostic, A/B and test hooks read from the environment exist only in the diagnostic build (-DFLOAM_DIAG:
// libfloam_amd_diag.so, which the tests that need a hook load); in the product library FLOAM_DIAG_ENV(name) is a null
// pointer and the name is not in the binary.  The product library reads two documented variables: FLOAM_GRAPH and
// FLOAM_MAP_MERGE.
#ifdef FLOAM_DIAG
#define FLOAM_DIAG_ENV(name) std::getenv(name)
#else
#define FLOAM_DIAG_ENV(name) (static_cast<const char*>(nullptr))
#endif

#include "../../include/floam_c.h"

namespace floam {

// 32-B record == vel_point::PointXYZIRT (include/lidar.h:14-32) == floam_point.  AoS in HBM for I/O clouds so a
// pcl::PointCloud's points.data() can be copied without repacking; 16-B aligned so one record is two dwordx4.
struct alignas(16) PointRec {
  float x, y, z, pad0;
  float intensity;
  uint16_t ring;
  uint16_t pad1;
  float time;
  float pad2;
};
static_assert(sizeof(PointRec) == 32, "point record must be 32 B");
static_assert(sizeof(PointRec) == sizeof(floam_point), "ABI");

// Error carried to the C-ABI as a status + message.
struct Error : std::runtime_error {
  floam_status status;
  Error(floam_status s, const std::string& m) : std::runtime_error(m), status(s) {}
};

#define FLOAM_HIP(call)                                                                                  \
  do {                                                                                                   \
    hipError_t _e = (call);                                                                              \
    if (_e != hipSuccess)                                                                                \
      throw ::floam::Error(_e == hipErrorOutOfMemory ? FLOAM_ERR_OUT_OF_MEMORY : FLOAM_ERR_DEVICE,      \
                           std::string(#call) + ": " + hipGetErrorString(_e) + " @" + __FILE__ + ":" +   \
                               std::to_string(__LINE__));                                                \
  } while (0)

#define FLOAM_LAUNCH_CHECK() FLOAM_HIP(hipGetLastError())

inline unsigned div_up(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

// ------------------------------------------------------------------------------------- device buffers
// Stream capture of an update into a hipGraph (host.cpp): while a capture is active, device memory replaced by a
// growing buffer is not freed (hipFree would synchronise) but kept until the captured work has run.
struct CaptureState {
  bool active = false;
  std::vector<void*> graveyard;
};
inline CaptureState& capture_state() {
  static thread_local CaptureState s;
  return s;
}
inline void dev_free(void* p) {
  if (!p) return;
  if (capture_state().active) capture_state().graveyard.push_back(p);
  else (void)hipFree(p);
}

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    dev_free(p);
    p = nullptr;
    cap = 0;
  }
  // grow-only; contents are not preserved
  void reserve(size_t n) {
    if (n <= cap) return;
    if (alloc_log()) std::fprintf(stderr, "[floam alloc] %zu x %zu B (had %zu)\n", n, sizeof(T), cap);
    release();
    // headroom: a reallocation (hipFree) stalls the whole device for 100-500 us, so the arrays that grow with the
    // map double and start at 1 M elements (HBM is plentiful; the steady state must not reallocate)
    size_t c = n < 1024 ? 1024 : (n < 4096 ? n + n / 2 : std::max(2 * n, (size_t)1 << 20));
    FLOAM_HIP(hipMalloc(&p, c * sizeof(T)));
    cap = c;
  }
  static bool alloc_log() {   // FLOAM_LOG_ALLOC=1: report device (re)allocations (diagnostic build)
    static const bool on = FLOAM_DIAG_ENV("FLOAM_LOG_ALLOC") != nullptr;
    return on;
  }
};

// Pinned host staging
template <typename T>
struct HostBuf {
  T* p = nullptr;
  size_t cap = 0;
  ~HostBuf() {
    if (p) (void)hipHostFree(p);
  }
  void reserve(size_t n, unsigned flags = hipHostMallocDefault) {
    if (n <= cap) return;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    FLOAM_HIP(hipHostMalloc(&p, n * sizeof(T), flags));
    cap = n;
  }
};

// Inclusive prefix sum over the 64 lanes of a wave by DPP lane moves: row_shr 1, 2, 4, 8 inside each row of 16 (lanes
// below the shift read 0), then row_bcast 15 (the row total into the next row, rows 1 and 3) and row_bcast 31 (rows
// 0 + 1 into rows 2 and 3) — six VALU steps where a __shfl_up loop takes six ds_bpermute round trips.  Every lane of
// the wave must be active (the callers run it in wave-uniform code).
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);
  return v;
}
__device__ __forceinline__ unsigned wave_incl_scan(unsigned v) { return (unsigned)wave_incl_scan((int)v); }

// Physical block p of the first `nactive` blocks -> logical block, so that the blocks with equal p % 8 (one XCD
// under the round-robin dispatch of MI355X_MICROARCH.md "Workgroup dispatch") get consecutive logical indices.
// A bijection on [0, nactive); placement only affects speed, never results.
__device__ __forceinline__ int xcd_block(int p, int nactive) {
  const int x = p & 7, r = p >> 3, base = nactive >> 3, rem = nactive & 7;
  return x * base + min(x, rem) + r;
}

}  // namespace floam

// Device-resident cloud behind the opaque floam_cloud handle.
struct floam_cloud {
  int device = 0;
  floam::DevBuf<floam::PointRec> pts;
  floam::DevBuf<int> count;    // count.p[0] = number of points (device-resident)
  size_t host_count = 0;       // last value the host knows (valid when host_count_valid)
  bool host_count_valid = true;
  size_t ub = 0;               // upper bound on the device count while host_count_valid is false
  const int* fe_status = nullptr;   // device status flags of the (asynchronous) feature extraction that filled it
  floam::DevBuf<int> fe_stat;       // ... stored here (per cloud: the next extraction cannot overwrite it)
  // cross-stream ordering: the stream of the last operation on the cloud, and an event marking its end
  hipStream_t last_stream = nullptr;
  hipEvent_t ev = nullptr;
  bool ev_valid = false;            // ev recorded after the last operation (else recorded lazily when needed)
  hipEvent_t ext_ev = nullptr;      // with ev_valid: a borrowed event (the end of an odometry update, shared with
                                    // the update's other consumers) used instead of ev
  // the last operation was odometry update `done_seq` of a handle whose collected serial number is *done_ctr: once
  // it has been collected the operation is complete and a consumer on another stream needs no wait at all
  std::shared_ptr<const unsigned long long> done_ctr;
  unsigned long long done_seq = 0;
  bool clear_pending = false;       // floam_cloud_clear: the device count is zeroed by the cloud's next operation,
                                    // on that operation's stream
};
