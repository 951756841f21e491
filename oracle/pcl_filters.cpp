// CPU ORACLE (test infrastructure) — restatement of the PCL 1.8.1 filters on the path.
// VoxelGrid<PointXYZI>: call sites src/odomEstimationClass.cpp:13-14 (leaf r / 2r), :137-142 (scan downsample),
// :289-292 (map re-voxelisation).  CropBox<PointXYZI>: :270-287.  Parity unpinned (see oracle.hpp).
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdint>

#include "oracle.hpp"

namespace oracle {

namespace {
struct IdxPair {   // pcl::cloud_point_index_idx: operator< compares idx only
  unsigned int idx;
  unsigned int cloud_point_index;
  bool operator<(const IdxPair& o) const { return idx < o.idx; }
};
}  // namespace

void voxel_grid(const Pt* in, size_t n, float leaf, bool stable, std::vector<Pt>& out) {
  out.clear();
  if (n == 0) return;
  // setLeafSize(float) then inverse_leaf_size_ = 1 / leaf (float division)
  const float inv = 1.0f / leaf;
  // getMinMax3D over all points (is_dense cloud: no finiteness check)
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (size_t i = 0; i < n; ++i) {
    const float v[3] = {in[i].x, in[i].y, in[i].z};
    for (int d = 0; d < 3; ++d) {
      mn[d] = std::min(mn[d], v[d]);
      mx[d] = std::max(mx[d], v[d]);
    }
  }
  const int64_t dx = static_cast<int64_t>((mx[0] - mn[0]) * inv) + 1;
  const int64_t dy = static_cast<int64_t>((mx[1] - mn[1]) * inv) + 1;
  const int64_t dz = static_cast<int64_t>((mx[2] - mn[2]) * inv) + 1;
  if ((dx * dy * dz) > static_cast<int64_t>(INT32_MAX)) {   // "Leaf size is too small": output = input (Q9)
    out.assign(in, in + n);
    return;
  }
  int min_b[3], max_b[3], div_b[3];
  for (int d = 0; d < 3; ++d) {
    min_b[d] = static_cast<int>(std::floor(mn[d] * inv));
    max_b[d] = static_cast<int>(std::floor(mx[d] * inv));
    div_b[d] = max_b[d] - min_b[d] + 1;
  }
  const int divb_mul[3] = {1, div_b[0], div_b[0] * div_b[1]};
  std::vector<IdxPair> iv;
  iv.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    const int ijk0 = static_cast<int>(std::floor(in[i].x * inv) - static_cast<float>(min_b[0]));
    const int ijk1 = static_cast<int>(std::floor(in[i].y * inv) - static_cast<float>(min_b[1]));
    const int ijk2 = static_cast<int>(std::floor(in[i].z * inv) - static_cast<float>(min_b[2]));
    const int idx = ijk0 * divb_mul[0] + ijk1 * divb_mul[1] + ijk2 * divb_mul[2];
    iv.push_back(IdxPair{static_cast<unsigned int>(idx), static_cast<unsigned int>(i)});
  }
  if (stable) {
    std::stable_sort(iv.begin(), iv.end());
  } else {
    std::sort(iv.begin(), iv.end());
  }
  // third pass: voxel runs (min_points_per_voxel_ = 0); fourth pass: float centroid of x,y,z,intensity
  size_t index = 0;
  while (index < iv.size()) {
    size_t i = index + 1;
    while (i < iv.size() && iv[i].idx == iv[index].idx) ++i;
    const Pt& f = in[iv[index].cloud_point_index];
    float c[4] = {f.x, f.y, f.z, f.intensity};
    for (size_t k = index + 1; k < i; ++k) {
      const Pt& p = in[iv[k].cloud_point_index];
      c[0] += p.x; c[1] += p.y; c[2] += p.z; c[3] += p.intensity;
    }
    const float cnt = static_cast<float>(i - index);
    Pt o{};
    o.x = c[0] / cnt; o.y = c[1] / cnt; o.z = c[2] / cnt; o.pad0 = 1.0f;
    o.intensity = c[3] / cnt;
    out.push_back(o);
    index = i;
  }
}

void crop_box(const Pt* in, size_t n, const float mn[3], const float mx[3], std::vector<Pt>& out) {
  out.clear();
  for (size_t i = 0; i < n; ++i) {
    const Pt& p = in[i];
    if (p.x < mn[0] || p.y < mn[1] || p.z < mn[2] || p.x > mx[0] || p.y > mx[1] || p.z > mx[2]) continue;
    out.push_back(p);
  }
}

}  // namespace oracle
