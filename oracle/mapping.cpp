// CPU ORACLE (test infrastructure) — LaserMappingClass, the global cell map of the mapping node, restated
// (SURVEY.md §8 f-4).
//
//   LaserMappingClass::init                     src/laserMappingClass.cpp:7-32
//   LaserMappingClass::updateCurrentPointsToMap src/laserMappingClass.cpp:148-186 (checkPoints :107-145)
//   LaserMappingClass::getMap                   src/laserMappingClass.cpp:188-200
//   caller: src/laserMappingNode.cpp:101-117 (pose from /odom: Isometry3d::Identity().rotate(q).pretranslate(t))
//
// The reference keeps a dense, growing 3-D array of cell clouds (50 m cells, include/laserMappingClass.h:28-36)
// whose index origin shifts as it grows; what it outputs depends only on the absolute cell of each point, so the
// cells are kept here in a map ordered by absolute (x, y, z) — getMap's i, j, k loop order.  Cells created empty by
// checkPoints contribute nothing to getMap, so they need no representation.  Points landing outside the reference's
// allocated array (more than 2 cells = 100-125 m from the pose: out-of-bounds there) are kept in their cell here.
#include <array>
#include <cmath>
#include <map>
#include <vector>

#include "la.hpp"
#include "oracle.hpp"

namespace oracle {

struct MappingState {
  float leaf;
  bool stable;
  std::map<std::array<int, 3>, std::vector<Pt>> cells;
};

MappingState* mapping_create(double map_resolution, bool stable_voxel) {
  auto* m = new MappingState;
  m->leaf = (float)map_resolution;   // downSizeFilter.setLeafSize(double -> float) (:31)
  m->stable = stable_voxel;
  return m;
}
void mapping_destroy(MappingState* m) { delete m; }

// int(std::floor(v / LASER_CELL_WIDTH + 0.5)) (:150-152, :163-165), the double division of a float or double
static int cell_of(double v) { return (int)std::floor(v / 50.0 + 0.5); }

void mapping_update(MappingState* m, const Pt* in, size_t n, const double q_xyzw[4], const double t[3]) {
  // current_pose = Isometry3d::Identity(); rotate(q); pretranslate(t) (laserMappingNode.cpp:108-110)
  const M3 R = to_matrix(Quat{q_xyzw[0], q_xyzw[1], q_xyzw[2], q_xyzw[3]});
  const int cx = cell_of(t[0]), cy = cell_of(t[1]), cz = cell_of(t[2]);
  // pcl::transformPointCloud(*pc_in, *transformed, pose_current.cast<float>()) (:157): float matrix, float sums
  float mf[3][4];
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) mf[r][c] = (float)R.m[r][c];
    mf[r][3] = (float)t[r];
  }
  for (size_t i = 0; i < n; ++i) {
    const float x = in[i].x, y = in[i].y, z = in[i].z;
    Pt p{};
    p.x = ((mf[0][0] * x + mf[0][1] * y) + mf[0][2] * z) + mf[0][3];
    p.y = ((mf[1][0] * x + mf[1][1] * y) + mf[1][2] * z) + mf[1][3];
    p.z = ((mf[2][0] * x + mf[2][1] * y) + mf[2][2] * z) + mf[2][3];
    p.pad0 = 1.0f;
    // intensity = std::min(1.0, std::max(pc_in z + 2.0, 0.0) / 5) (:162), std::min/max argument order kept
    const double zz = (double)z + 2.0;
    const double mx = (zz < 0.0) ? 0.0 : zz;   // std::max(a, b) = (a < b) ? b : a
    const double v = mx / 5;
    p.intensity = (float)((v < 1.0) ? v : 1.0);   // std::min(a, b) = (b < a) ? b : a with a = 1.0
    m->cells[{cell_of(p.x), cell_of(p.y), cell_of(p.z)}].push_back(p);
  }
  // downSizeFilter over the 5 x 5 x 5 cells around the pose (:174-183), in place
  for (int i = cx - 2; i <= cx + 2; ++i)
    for (int j = cy - 2; j <= cy + 2; ++j)
      for (int k = cz - 2; k <= cz + 2; ++k) {
        auto it = m->cells.find({i, j, k});
        if (it == m->cells.end() || it->second.empty()) continue;
        std::vector<Pt> out;
        voxel_grid(it->second.data(), it->second.size(), m->leaf, m->stable, out);
        it->second.swap(out);
      }
}

size_t mapping_size(const MappingState* m) {
  size_t n = 0;
  for (const auto& kv : m->cells) n += kv.second.size();
  return n;
}

// getMap: every cell's cloud appended in (x, y, z) order
void mapping_get_map(const MappingState* m, Pt* out) {
  size_t k = 0;
  for (const auto& kv : m->cells)
    for (const Pt& p : kv.second) out[k++] = p;
}

}  // namespace oracle
