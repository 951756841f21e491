// Cloud operations on gfx950: map append (initMapWithPoints / getMap) and velocity deskew.
// CompensateVelocity: src/dataHandler.cpp:82-92.  VoxelGrid / CropBox live in voxel.hip.

#include "cloud_ops.hpp"

namespace floam {

void SortScratch::reserve(int n) {
  if ((size_t)n <= k0.cap) return;
  const size_t want = (size_t)n < 4096 ? 4096 : (size_t)n + (size_t)n / 4;
  k0.reserve(want); k1.reserve(want);
  v0.reserve(want); v1.reserve(want);
}

namespace {
constexpr int kTB = 256;

__global__ __launch_bounds__(kTB) void compensate(PointRec* __restrict__ pts, const int* __restrict__ d_n, int n_ub,
                                                  double vx, double vy, double vz) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ub || i >= *d_n) return;
  PointRec& p = pts[i];
  const double t = p.time;
  p.x = (float)((double)p.x + vx * t);
  p.y = (float)((double)p.y + vy * t);
  p.z = (float)((double)p.z + vz * t);
}
__global__ __launch_bounds__(kTB) void append_copy(PointRec* __restrict__ dst, const int* __restrict__ d_dst_count,
                                                   const PointRec* __restrict__ src, const int* __restrict__ d_src_count,
                                                   int src_ub, int xyzi) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= src_ub || i >= *d_src_count) return;
  PointRec p = src[i];
  if (xyzi) {
    p.pad0 = 1.0f;
    p.ring = 0; p.pad1 = 0; p.time = 0.0f; p.pad2 = 0.0f;
  }
  dst[*d_dst_count + i] = p;
}

__global__ void add_count(int* __restrict__ d_dst_count, const int* __restrict__ d_src_count) {
  if (threadIdx.x == 0) *d_dst_count += *d_src_count;
}

// a do-nothing dispatch whose name marks a point of the stream in a rocprofv3 kernel trace (floam_profile_mark)
__global__ void floam_profile_marker(int id) {
  if (id < 0) __builtin_trap();
}
// (diagnostic, FLOAM_UPDATE_NOP=1) a do-nothing dispatch at the start of every odometry update: whether the main
// stream's idle time before the update's first kernel belongs to that kernel or to the update boundary
__global__ void update_nop(int id) {
  if (id < 0) __builtin_trap();
}
}  // namespace

void update_nop_launch(hipStream_t st) {
  hipLaunchKernelGGL(update_nop, dim3(1), dim3(64), 0, st, 0);
  FLOAM_LAUNCH_CHECK();
}

void profile_marker_launch(int id, hipStream_t st) {
  hipLaunchKernelGGL(floam_profile_marker, dim3(1), dim3(64), 0, st, id);
  FLOAM_LAUNCH_CHECK();
}

void append_launch(PointRec* dst, int* d_dst_count, const PointRec* src, const int* d_src_count, int src_ub,
                   bool xyzi, hipStream_t st) {
  if (src_ub > 0) {
    hipLaunchKernelGGL(append_copy, dim3(div_up(src_ub, kTB)), dim3(kTB), 0, st, dst, d_dst_count, src, d_src_count,
                       src_ub, xyzi ? 1 : 0);
    FLOAM_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(add_count, dim3(1), dim3(64), 0, st, d_dst_count, d_src_count);
  FLOAM_LAUNCH_CHECK();
}

void compensate_velocity_launch(PointRec* pts, const int* d_n, int n_ub, double vx, double vy, double vz,
                                hipStream_t st) {
  if (n_ub <= 0) return;
  hipLaunchKernelGGL(compensate, dim3(div_up(n_ub, kTB)), dim3(kTB), 0, st, pts, d_n, n_ub, vx, vy, vz);
  FLOAM_LAUNCH_CHECK();
}

}  // namespace floam
