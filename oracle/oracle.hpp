// CPU ORACLE — test infrastructure only, never shipped, never on the product path.
//
// A single-threaded C++ restatement of the FLOAM (dan11003/floam) scan-to-map odometry hot path, used by tests/
// (parity checker), __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Every function cites the reference
// file:line it follows (paths relative to the reference repo root).
//
// PARITY UNPINNED: the reference ships no tests, fixtures or golden outputs and cannot be compiled
// here (needs ROS Melodic, PCL, FLANN, Ceres, Eigen, Boost — none present, SURVEY.md §8 c).  The oracle is pinned
// instead by (1) independent numpy/scipy cross-checks of its sub-steps (tests/test_oracle_*.py), (2) known-answer
// tests (rigid-motion recovery, analytic-vs-numeric Jacobians) and (3) golden vectors it generated, committed under
// tests/golden/ for regression.
//
// Third-party semantics restated from their published algorithms (versions inferred from README.md:31-36, Ubuntu
// 18.04 / ROS Melodic; NOT pinned by the reference's build files): PCL 1.8.1 (VoxelGrid, CropBox, KdTreeFLANN),
// FLANN 1.9.1 (KDTreeSingleIndex leaf 15, L2_Simple<float>, KNNSimpleResultSet), Eigen 3.3.4
// (SelfAdjointEigenSolver<Matrix3d>, ColPivHouseholderQR, HouseholderQR, Quaternion/Isometry algebra),
// Ceres 1.13.0 (TrustRegionMinimizer + LevenbergMarquardtStrategy + DenseQRSolver + HuberLoss/Corrector).
// Eigen's SSE2 packet-reduction order is not reproduced (sums here are sequential): such differences are
// O(1e-16) relative and far below the 1e-3 pose tolerance.
#pragma once
#include <cstdint>
#include <cstddef>
#include <string>
#include <vector>

#include "la.hpp"

namespace oracle {

// vel_point::PointXYZIRT (include/lidar.h:14-32) — 32 B, EIGEN_ALIGN16.  pcl::PointXYZI has x,y,z,intensity at the
// same offsets and the same 32-B size, so one record serves both cloud types.
struct alignas(16) Pt {
  float x, y, z, pad0;
  float intensity;
  uint16_t ring;
  uint16_t pad1;
  float time;
  float pad2;
};
static_assert(sizeof(Pt) == 32, "point record must be 32 B");

// lidar::Lidar fields used on the path (include/lidar.h:53-85)
struct LidarParams {
  int num_lines;
  double scan_period;
  double min_distance;
  double max_distance;
};

// ---------------------------------------------------------------------------------------------- feature extraction
struct FeStats {
  size_t out_of_range_rings = 0;   // points with ring >= num_lines (UB in the reference, dropped here)
  size_t sector_ties = 0;          // adjacent equal curvature values inside a sector (breaks bit-exactness)
};
// LaserProcessingClass::featureExtraction (src/laserProcessingClass.cpp:72-118).  Appends to edge/surf.
// canonical_sort=false: std::sort exactly as the reference (:123-126, unstable); true: sort by (value, id),
// identical whenever a sector has no tied curvature values.
void feature_extraction(const LidarParams& lp, const Pt* in, size_t n, std::vector<Pt>& edge,
                        std::vector<Pt>& surf, bool canonical_sort, FeStats* stats);

// ---------------------------------------------------------------------------------------------- PCL filters
// pcl::VoxelGrid<PointXYZI>::applyFilter (PCL 1.8.1 voxel_grid.hpp) as used at src/odomEstimationClass.cpp:13-14,
// 137-142, 289-292.  stable=false: std::sort of (idx, i) like PCL (within-voxel order unspecified); stable=true:
// stable order (original index order within a voxel).
void voxel_grid(const Pt* in, size_t n, float leaf, bool stable, std::vector<Pt>& out);
// pcl::CropBox<PointXYZI> (PCL 1.8.1 crop_box.hpp) with identity transform, as at src/odomEstimationClass.cpp:270-287
void crop_box(const Pt* in, size_t n, const float mn[3], const float mx[3], std::vector<Pt>& out);

// ---------------------------------------------------------------------------------------------- FLANN KD-tree
class KdTree {
 public:
  void build(const Pt* pts, size_t n);                 // KdTreeFLANN::setInputCloud (odomEstimationClass.cpp:78-79)
  // nearestKSearch(k) (odomEstimationClass.cpp:153,206): ascending float sq-distances, FLANN tie semantics.
  int knn(const float q[3], int k, int* idx, float* sqd) const;
 private:
  struct Node { int left, right; int divfeat; float divlow, divhigh; int child1, child2; };
  struct Interval { float low, high; };
  int divide(int left, int right, Interval* bbox);
  void middle_split(int* ind, int count, int& index, int& cutfeat, float& cutval, const Interval* bbox);
  void plane_split(int* ind, int count, int cutfeat, float cutval, int& lim1, int& lim2);
  void min_max(const int* ind, int count, int dim, float& mn, float& mx) const;
  std::vector<float> data_;    // reordered xyz
  std::vector<int> vind_;
  std::vector<Node> nodes_;
  Interval root_bbox_[3];
  int root_ = -1;
  size_t n_ = 0;
};

// ---------------------------------------------------------------------------------------------- odometry
enum UpdateType { VANILLA = 0, INITIAL_ITERATION = 1, REFINEMENT_AND_UPDATE = 2 };  // odomEstimationClass.h:56

struct SolveTrace {            // one ceres::Solve (one outer iteration), for piecewise parity tests
  int n_edge_queries, n_surf_queries;
  int n_edge_corr, n_surf_corr;
  int iterations;              // trust-region iterations executed (<= 4)
  int successful;
  double initial_cost, final_cost;
  double x_in[7], x_out[7];
  double H0[21], g0[6];        // unscaled J^T J (upper, row-major) and J^T r at x_in
};

struct OdomState;
OdomState* odom_create(const LidarParams& lp, double map_resolution, const std::string& loss, bool stable_voxel);
void odom_destroy(OdomState*);
void odom_init_map(OdomState*, const Pt* edge, size_t ne, const Pt* surf, size_t ns);
void odom_update_selector(OdomState*, Pt* edge, size_t ne, Pt* surf, size_t ns, bool deskew);
void odom_update(OdomState*, const Pt* edge, size_t ne, const Pt* surf, size_t ns, UpdateType t);
void odom_get_pose(const OdomState*, double q_xyzw[4], double t[3]);
void odom_get_last_pose(const OdomState*, double q_xyzw[4], double t[3]);
void odom_get_velocity(const OdomState*, double v[3]);
size_t odom_map_size(const OdomState*, int which);                  // 0 = corner (edge), 1 = surf
const Pt* odom_map_data(const OdomState*, int which);
const std::vector<SolveTrace>& odom_traces(const OdomState*);
void odom_clear_traces(OdomState*);
int odom_optimization_count(const OdomState*);
void stage_correspondences(const Pt* map, size_t m, const Pt* q, size_t nq, const double* x, bool edge, int* idx,
                           float* sqd, unsigned char* flags, double* rec);
void stage_associate(const Pt* in, size_t n, const double* x, Pt* out);
void stage_solve(const double* erec, size_t ne, const double* srec, size_t ns, bool huber, double* x, double* trace);
// ---------------------------------------------------------------------------------------------- IMU pre-processing
// (oracle/imu.cpp).  Quat is Eigen's (x, y, z, w) order (la.hpp).
struct ImuHandler {                       // dmapping::ImuHandler (include/dataHandler.h:31-66), orientation only
  std::vector<double> t;
  std::vector<Quat> q;
  bool add_msg(double stamp, const Quat& orientation);
  size_t lower_bound(double ts) const;
  bool get(double ts, Quat* out) const;
  Quat get_or_zero(double ts) const;
  bool time_contained(double ts) const;
};
Quat qmul_sse2(const Quat& a, const Quat& b);
Quat qinverse(const Quat& q);
Quat euler_to_quaternion(double roll, double pitch, double yaw);
double pcl_stamp_to_sec(uint64_t stamp_us);
bool sec_to_pcl_stamp(double t, uint64_t* stamp_us);
void center_time(Pt* pts, size_t n, uint64_t* stamp_us);
bool compensate(const Pt* in, size_t n, uint64_t stamp_us, const ImuHandler& h, const Quat& extr, Pt* out);
void transform_by_quaternion(const Pt* in, size_t n, const Quat& q, Pt* out);
bool imu_preprocess(Pt* in, size_t n, uint64_t* stamp_us, const ImuHandler& h, const Quat& extr, Pt* out);

// ---------------------------------------------------------------------------------------------- wire formats
// (oracle/formats.cpp)
struct Pc2Field {   // sensor_msgs/PointField, the layout of floam_pc2_field
  char name[32];
  uint32_t offset;
  uint8_t datatype;
  uint32_t count;
};
int from_pointcloud2(int point_type, const uint8_t* data, uint32_t width, uint32_t height, uint32_t point_step,
                     uint32_t row_step, const Pc2Field* fields, size_t nfields, Pt* out);
void transform_cloud(const Pt* in, size_t n, const double m[16], Pt* out);

// ---------------------------------------------------------------------------------------------- global map
// LaserMappingClass (oracle/mapping.cpp)
struct MappingState;
MappingState* mapping_create(double map_resolution, bool stable_voxel);
void mapping_destroy(MappingState* m);
void mapping_update(MappingState* m, const Pt* in, size_t n, const double q_xyzw[4], const double t[3]);
size_t mapping_size(const MappingState* m);
void mapping_get_map(const MappingState* m, Pt* out);

void reset_process_statics();   // KeyFrameUpdate's function-static `first` (odomEstimationClass.cpp:323, Q6)
double test_edge_eval(const double cp[3], const double a[3], const double b[3], const double* x, double* J);
double test_surf_eval(const double cp[3], const double n[3], double d, const double* x, double* J);
void test_se3_plus(const double* x, const double* delta, double* out);

}  // namespace oracle
