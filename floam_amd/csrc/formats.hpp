// Wire formats on gfx950: sensor_msgs/PointCloud2 -> PointXYZIRT / PointXYZI records
// (pcl::fromROSMsg = pcl_conversions::toPCL + pcl::fromPCLPointCloud2, PCL 1.8.1 conversions.h) and the dense
// pcl::transformPointCloud with a double Eigen::Affine3d (PCL 1.8.1 transforms.hpp), used by the odometry node's
// SaveMerged export (src/odomEstimationNode.cpp:66-96).
#pragma once
#include "floam_common.hpp"

namespace floam {

// One coalesced field mapping (detail::FieldMapping): `size` bytes from serialized_offset in the message point to
// struct_offset in the 32-B record.
struct Pc2Mapping {
  int serialized_offset, struct_offset, size;
};
struct Pc2Decode {
  const uint8_t* data;   // message bytes in HBM
  long long row_step;
  int point_step;
  int width, height;
  int nmap;              // <= 6
  Pc2Mapping map[6];
  int whole;             // the single-memcpy case: every point's first 32 bytes copied as they are
};
void pc2_decode_launch(const Pc2Decode& d, PointRec* out, hipStream_t st);

// x' = float(((m00 x + m01 y) + m02 z) + m03) etc. with a row-major double 3x4 matrix; all other fields copied.
void transform_cloud_launch(const PointRec* in, const int* d_n, int n_ub, const double* m34 /* host */,
                            PointRec* out, hipStream_t st);

}  // namespace floam
