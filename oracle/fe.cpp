// CPU ORACLE (test infrastructure) — restatement of LaserProcessingClass::featureExtraction.
// Reference: src/laserProcessingClass.cpp:11-22 (RingExtractionVelodyne), :72-118 (featureExtraction),
// :121-231 (featureExtractionFromSector).  Parity unpinned (see oracle.hpp).
#include <algorithm>
#include <cmath>
#include <utility>

#include "oracle.hpp"

namespace oracle {
namespace {

struct Double2d {   // include/laserProcessingClass.h:22-27
  int id;
  double value;
};

// src/laserProcessingClass.cpp:11-22.  The xy range uses the float sum x*x+y*y and the float sqrt overload (the
// libstdc++ <math.h> wrapper pulled in through PCL/Eigen makes ::sqrt(float) the exact match); the comparison
// against min/max_distance is in double.  Input order is kept inside each ring (stable bucketing).
void ring_extraction(const LidarParams& lp, const Pt* in, size_t n, std::vector<std::vector<Pt>>& scans,
                     FeStats* st) {
  for (size_t i = 0; i < n; ++i) {
    const Pt& p = in[i];
    const int scanID = p.ring;
    const float d2 = p.x * p.x + p.y * p.y;
    const double distance = std::sqrt(d2);
    if (distance < lp.min_distance || distance > lp.max_distance) continue;
    if (scanID >= lp.num_lines) {   // reference: laserCloudScans[scanID] out of bounds (UB); dropped here
      if (st) st->out_of_range_rings++;
      continue;
    }
    Pt t{};
    t.x = p.x; t.y = p.y; t.z = p.z; t.pad0 = 1.0f;
    t.intensity = p.intensity; t.ring = p.ring; t.time = p.time;
    scans[scanID].push_back(t);
  }
}

// src/laserProcessingClass.cpp:121-231
void from_sector(const std::vector<Pt>& pc, std::vector<Double2d>& curv, std::vector<Pt>& edge,
                 std::vector<Pt>& surf, bool canonical) {
  if (canonical) {
    std::sort(curv.begin(), curv.end(), [](const Double2d& a, const Double2d& b) {
      return a.value < b.value || (a.value == b.value && a.id < b.id);
    });
  } else {
    std::sort(curv.begin(), curv.end(), [](const Double2d& a, const Double2d& b) { return a.value < b.value; });
  }
  int largestPickedNum = 0;
  std::vector<int> picked;
  for (int i = (int)curv.size() - 1; i >= 0; i--) {
    const int ind = curv[i].id;
    if (std::find(picked.begin(), picked.end(), ind) == picked.end()) {
      if (curv[i].value <= 0.1) break;                       // :136
      largestPickedNum++;
      picked.push_back(ind);
      if (largestPickedNum <= 20) {                          // :143 (21st pick: marked, not emitted, Q1)
        edge.push_back(pc[ind]);
      } else {
        break;
      }
      for (int k = 1; k <= 5; k++) {                         // :150-158
        const double dX = pc[ind + k].x - pc[ind + k - 1].x;
        const double dY = pc[ind + k].y - pc[ind + k - 1].y;
        const double dZ = pc[ind + k].z - pc[ind + k - 1].z;
        if (dX * dX + dY * dY + dZ * dZ > 0.05) break;
        picked.push_back(ind + k);
      }
      for (int k = -1; k >= -5; k--) {                       // :159-167
        const double dX = pc[ind + k].x - pc[ind + k + 1].x;
        const double dY = pc[ind + k].y - pc[ind + k + 1].y;
        const double dZ = pc[ind + k].z - pc[ind + k + 1].z;
        if (dX * dX + dY * dY + dZ * dZ > 0.05) break;
        picked.push_back(ind + k);
      }
    }
  }
  for (int i = 0; i <= (int)curv.size() - 1; i++) {          // :220-227 surf = unpicked, ascending curvature
    const int ind = curv[i].id;
    if (std::find(picked.begin(), picked.end(), ind) == picked.end()) surf.push_back(pc[ind]);
  }
}

}  // namespace

void feature_extraction(const LidarParams& lp, const Pt* in, size_t n, std::vector<Pt>& edge,
                        std::vector<Pt>& surf, bool canonical_sort, FeStats* st) {
  // :74-75 removeNaNFromPointCloud(*pc_in, indices) — indices discarded, the cloud is unchanged (Q7): no-op.
  const int N_SCANS = lp.num_lines;
  std::vector<std::vector<Pt>> scans(N_SCANS);
  ring_extraction(lp, in, n, scans, st);
  for (int i = 0; i < N_SCANS; i++) {
    const std::vector<Pt>& s = scans[i];
    if (s.size() < 131) continue;                            // :89
    std::vector<Double2d> curv;
    const int total_points = (int)s.size() - 10;
    for (int j = 5; j < (int)s.size() - 5; j++) {            // :95-101, float stencil in source order
      const float fx = s[j - 5].x + s[j - 4].x + s[j - 3].x + s[j - 2].x + s[j - 1].x - 10 * s[j].x + s[j + 1].x +
                       s[j + 2].x + s[j + 3].x + s[j + 4].x + s[j + 5].x;
      const float fy = s[j - 5].y + s[j - 4].y + s[j - 3].y + s[j - 2].y + s[j - 1].y - 10 * s[j].y + s[j + 1].y +
                       s[j + 2].y + s[j + 3].y + s[j + 4].y + s[j + 5].y;
      const float fz = s[j - 5].z + s[j - 4].z + s[j - 3].z + s[j - 2].z + s[j - 1].z - 10 * s[j].z + s[j + 1].z +
                       s[j + 2].z + s[j + 3].z + s[j + 4].z + s[j + 5].z;
      const double dX = fx, dY = fy, dZ = fz;
      curv.push_back(Double2d{j, dX * dX + dY * dY + dZ * dZ});
    }
    for (int j = 0; j < 6; j++) {                            // :103-114 (end exclusive: one entry never used)
      const int sector_length = total_points / 6;
      const int sector_start = sector_length * j;
      int sector_end = sector_length * (j + 1) - 1;
      if (j == 5) sector_end = total_points - 1;
      std::vector<Double2d> sub(curv.begin() + sector_start, curv.begin() + sector_end);
      if (st) {
        std::vector<double> v;
        for (auto& d : sub) v.push_back(d.value);
        std::sort(v.begin(), v.end());
        for (size_t k = 1; k < v.size(); ++k) st->sector_ties += (v[k] == v[k - 1]);
      }
      from_sector(s, sub, edge, surf, canonical_sort);
    }
  }
}

}  // namespace oracle
