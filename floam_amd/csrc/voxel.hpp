// Batched pcl::VoxelGrid (+ the map-side half of addPointsToMap) — see voxel.hip.
#pragma once
#include "cloud_ops.hpp"
#include "floam_common.hpp"
#include "radix.hpp"

namespace floam {

// One cloud: the concatenation [part0 ; part1] (part1 optional).  With pose != null (device pointer to
// {qx,qy,qz,qw,tx,ty,tz}) part1 is transformed into the map frame (pointAssociateToMap) and both parts are cropped
// to t +- 100 (CropBox) before the voxel grid: addPointsToMap (src/odomEstimationClass.cpp:253-294).
// out must hold n0_ub + n1_ub points and must not alias part0 / part1.
struct VoxelJob {
  const PointRec* part0 = nullptr;
  const int* d_n0 = nullptr;
  int n0_ub = 0;
  const PointRec* part1 = nullptr;
  const int* d_n1 = nullptr;
  int n1_ub = 0;
  const double* pose = nullptr;
  float leaf = 1.0f;
  PointRec* out = nullptr;
  int* d_out = nullptr;
};

struct VoxelScratch2 {
  SortScratch s;
  DevBuf<float> partials;
  DevBuf<int> overflow;
  DevBuf<unsigned long long> status;
  DevBuf<unsigned> ticket;
  RadixScratch rs;
};

// Two independent voxel grids in one pipeline (3 kernels + the 4 radix passes).  *d_out of each job receives the
// voxel count (-1 if the single-pass compaction failed, never expected).  gate (device int, nullable): when it reads
// 0 the pipeline does nothing but copy each job's part0 to its output (a map update skipped on the device).
void voxel2_launch(VoxelScratch2& sc, const VoxelJob& a, const VoxelJob& b, hipStream_t st,
                   const int* gate = nullptr);

}  // namespace floam
