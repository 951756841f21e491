#pragma once
#include "floam_common.hpp"

namespace floam {

// pointAssociateToMap (src/odomEstimationClass.cpp:126-135): Eigen q*v (_transformVector) + t in double, float
// store.  pose = {qx, qy, qz, qw, tx, ty, tz} (include/odomEstimationClass.h:90-92).
__device__ __forceinline__ void associate_to_map(const double* __restrict__ pose, float x, float y, float z,
                                                 float& ox, float& oy, float& oz) {
  const double qx = pose[0], qy = pose[1], qz = pose[2], qw = pose[3];
  const double vx = x, vy = y, vz = z;
  double ux = qy * vz - qz * vy, uy = qz * vx - qx * vz, uz = qx * vy - qy * vx;
  ux = ux + ux; uy = uy + uy; uz = uz + uz;
  const double ax = vx + qw * ux, ay = vy + qw * uy, az = vz + qw * uz;
  const double cx = qy * uz - qz * uy, cy = qz * ux - qx * uz, cz = qx * uy - qy * ux;
  ox = (float)((ax + cx) + pose[4]);
  oy = (float)((ay + cy) + pose[5]);
  oz = (float)((az + cz) + pose[6]);
}

struct SortScratch {   // (key, value) ping-pong buffers of the voxel sort
  DevBuf<uint32_t> k0, k1;
  DevBuf<int> v0, v1;
  void reserve(int n);
};

// one marker dispatch (kernel floam_profile_marker) on the stream: tools/prof_summary.py slices traces by it
void profile_marker_launch(int id, hipStream_t st);
void update_nop_launch(hipStream_t st);   // FLOAM_UPDATE_NOP (diagnostic)

// dmapping::CompensateVelocity (src/dataHandler.cpp:82-92), in place
void compensate_velocity_launch(PointRec* pts, const int* d_n, int n_ub, double vx, double vy, double vz,
                                hipStream_t st);

// dst[*d_dst_count + i] = src[i] for i < *d_src_count, then *d_dst_count += *d_src_count.
// xyzi: VelToIntensityCopy semantics (src/odomEstimationClass.cpp:308-318): keep x, y, z, intensity only.
void append_launch(PointRec* dst, int* d_dst_count, const PointRec* src, const int* d_src_count, int src_ub,
                   bool xyzi, hipStream_t st);

__device__ __forceinline__ int f2ord(float f) {
  const int i = __float_as_int(f);
  return i >= 0 ? i : i ^ 0x7FFFFFFF;
}
__device__ __forceinline__ float ord2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7FFFFFFF); }

}  // namespace floam
