// CPU ORACLE (test infrastructure) — wire formats of the odometry path, restated.
//
//   pcl::fromROSMsg -> pcl::fromPCLPointCloud2 with detail::FieldMapper / createMapping   (PCL 1.8.1 conversions.h)
//     call sites: src/laserProcessingNode.cpp:89, src/odomEstimationNode.cpp:205-206
//   pcl::transformPointCloud(in, out, Eigen::Affine3d)                                   (PCL 1.8.1 transforms.hpp)
//     call site: src/odomEstimationNode.cpp:72-76 (SaveMerged)
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "oracle.hpp"

namespace oracle {

namespace {
struct Reg {   // registered fields of the point type
  const char* name;
  uint32_t offset;
  uint8_t datatype;
  uint32_t size;   // sizeof the member type
};
const Reg kXYZIRT[] = {{"x", 0, 7, 4}, {"y", 4, 7, 4}, {"z", 8, 7, 4},
                       {"intensity", 16, 7, 4}, {"ring", 20, 4, 2}, {"time", 24, 7, 4}};
const Reg kXYZI[] = {{"x", 0, 7, 4}, {"y", 4, 7, 4}, {"z", 8, 7, 4}, {"intensity", 16, 7, 4}};
struct Mapping {
  uint32_t serialized_offset, struct_offset, size;
};
}  // namespace

// fromPCLPointCloud2: value-initialised points, per registered field the first message field matching name,
// datatype and count (0 or 1), mappings sorted by serialized offset and coalesced where the serialized and struct
// gaps agree, then either one memcpy of whole records (single mapping at 0/0 and point_step == 32) or per point
// per mapping.  Returns the number of registered fields without a match.
int from_pointcloud2(int point_type, const uint8_t* data, uint32_t width, uint32_t height, uint32_t point_step,
                     uint32_t row_step, const Pc2Field* fields, size_t nfields, Pt* out) {
  const Reg* r = point_type == 0 ? kXYZIRT : kXYZI;
  const size_t nr = point_type == 0 ? 6 : 4;
  std::vector<Mapping> map;
  int missing = 0;
  for (size_t k = 0; k < nr; ++k) {
    bool found = false;
    for (size_t j = 0; j < nfields; ++j) {
      if (std::string(fields[j].name) == r[k].name && fields[j].datatype == r[k].datatype &&
          (fields[j].count == 1 || fields[j].count == 0)) {
        map.push_back(Mapping{fields[j].offset, r[k].offset, r[k].size});
        found = true;
        break;
      }
    }
    if (!found) ++missing;
  }
  std::sort(map.begin(), map.end(),
            [](const Mapping& a, const Mapping& b) { return a.serialized_offset < b.serialized_offset; });
  if (map.size() > 1) {
    size_t i = 0, j = 1;
    while (j < map.size()) {
      if (map[j].serialized_offset - map[i].serialized_offset == map[j].struct_offset - map[i].struct_offset) {
        map[i].size += (map[j].struct_offset + map[j].size) - (map[i].struct_offset + map[i].size);
        map.erase(map.begin() + (long)j);
      } else {
        ++i;
        ++j;
      }
    }
  }
  const size_t n = (size_t)width * height;
  std::memset(out, 0, n * sizeof(Pt));
  uint8_t* cloud = reinterpret_cast<uint8_t*>(out);
  if (map.size() == 1 && map[0].serialized_offset == 0 && map[0].struct_offset == 0 && point_step == sizeof(Pt)) {
    const uint32_t cloud_row_step = (uint32_t)sizeof(Pt) * width;
    for (uint32_t row = 0; row < height; ++row)
      std::memcpy(cloud + (size_t)row * cloud_row_step, data + (size_t)row * row_step, cloud_row_step);
  } else {
    for (uint32_t row = 0; row < height; ++row)
      for (uint32_t col = 0; col < width; ++col) {
        const uint8_t* src = data + (size_t)row * row_step + (size_t)col * point_step;
        uint8_t* dst = cloud + ((size_t)row * width + col) * sizeof(Pt);
        for (const Mapping& m : map) std::memcpy(dst + m.struct_offset, src + m.serialized_offset, m.size);
      }
  }
  return missing;
}

// transformPointCloud, dense path, double transform: x' = float(((m00 x + m01 y) + m02 z) + m03)
void transform_cloud(const Pt* in, size_t n, const double m[16], Pt* out) {
  for (size_t i = 0; i < n; ++i) {
    const double x = in[i].x, y = in[i].y, z = in[i].z;
    Pt o = in[i];
    o.x = (float)(((m[0] * x + m[1] * y) + m[2] * z) + m[3]);
    o.y = (float)(((m[4] * x + m[5] * y) + m[6] * z) + m[7]);
    o.z = (float)(((m[8] * x + m[9] * y) + m[10] * z) + m[11]);
    out[i] = o;
  }
}

}  // namespace oracle
