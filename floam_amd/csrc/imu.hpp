// IMU pre-processing of the laser-processing node on gfx950:
//   CenterTime                        src/laserProcessingNode.cpp:65-78
//   dmapping::Compensate              src/dataHandler.cpp:93-122 (ImuHandler::Get :48-75, TimeContained :76-81)
//   ImuNowT + pcl::transformPointCloud src/laserProcessingNode.cpp:109-113
// fused into one pass over the scan (32 B read + 32 B written per point, plus the 4-B time write-back of
// CenterTime, which mutates the caller's cloud).  The IMU stream lives in HBM (append-only stamps + orientations);
// each workgroup stages the window of stamps that covers the scan in LDS and binary-searches it.
#pragma once
#include "floam_common.hpp"

namespace floam {

struct Q4 {   // Eigen::Quaterniond coefficient order (x, y, z, w)
  double x, y, z, w;
};

// Eigen 3.3 Geometry_SSE.h quat_product<SSE, ..., double> (x86-64 SSE2, no SSE3: the reference has no -march)
__host__ __device__ inline Q4 q4_mul(const Q4& a, const Q4& b) {
  Q4 r;
  r.x = (a.w * b.x + a.y * b.z) - (a.z * b.y - a.x * b.w);
  r.y = (a.w * b.y + a.y * b.w) + (a.z * b.x - a.x * b.z);
  r.z = (a.w * b.z - a.y * b.x) + (a.z * b.w + a.x * b.y);
  r.w = (a.w * b.w - a.y * b.y) - (a.z * b.z + a.x * b.x);
  return r;
}
// QuaternionBase::inverse: conjugate / squaredNorm (2-lane packet reduction order), zero if the norm is not > 0
__host__ __device__ inline Q4 q4_inverse(const Q4& q) {
  const double n2 = (q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w);
  if (n2 > 0.0) return Q4{-q.x / n2, -q.y / n2, -q.z / n2, q.w / n2};
  return Q4{0.0, 0.0, 0.0, 0.0};
}

struct ImuPrepArgs {
  double tScan;       // CenterTime: stamp of the incoming cloud (s)
  double tCenter;     // CenterTime: centre of [front.time, back.time] + tScan
  double tScan2;      // Compensate: the centred stamp after the microsecond round trip through the PCL header
  Q4 qInitInv;        // (Imu2Orientation(Get(tScan2)) * extrinsics)^-1
  Q4 extr;            // extrinsics
  double R[9];        // rotation matrix of qInit (row-major), the IMU alignment ImuNowT
  const double* stamps;   // IMU stamps (strictly increasing, ImuHandler::AddMsg), n_imu of them
  const Q4* orient;       // IMU orientations
  int n_imu;
  int win_lo, win_hi;     // stamp window [win_lo, win_hi) staged in LDS (covers the scan's front/back times)
};

enum { IMU_CENTER = 1, IMU_COMPENSATE = 2, IMU_ALIGN = 4 };
constexpr int kImuWindow = 2048;   // stamps staged in LDS (16 KB); points outside it search the whole stream

// mode = OR of IMU_*; in is updated in place when IMU_CENTER (times), out written when IMU_COMPENSATE.
void imu_prep_launch(int mode, PointRec* in, PointRec* out, const int* d_n, int n_ub, const ImuPrepArgs& a,
                     hipStream_t st);
// {count, front.time, back.time} of a cloud into dst (3 words; the times as float bits), for the host's scalar part
void cloud_ends_launch(const PointRec* pts, const int* d_n, int* dst, hipStream_t st);

}  // namespace floam
