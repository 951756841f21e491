// C++ consumer of the C ABI (include/floam_c.h), compiled with the host compiler against libfloam_amd.so the way a
// reference node or adapter would be: layout checks at compile time, then calls that need no GPU —
// argument validation, the loud failure of device calls on a host without a gfx950 device, the pure host helpers
// and the disk exporters (src/utils.cpp:3-106, src/odomEstimationNode.cpp:97-117).  Driven by tests/test_abi_cpp.py.
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

#include "floam_c.h"

// floam_point is byte-compatible with vel_point::PointXYZIRT (include/lidar.h:14-32) and pcl::PointXYZI
static_assert(sizeof(floam_point) == 32, "32-B point record");
static_assert(offsetof(floam_point, x) == 0 && offsetof(floam_point, y) == 4 && offsetof(floam_point, z) == 8,
              "xyz at PCL_ADD_POINT4D offsets");
static_assert(offsetof(floam_point, pad0) == 12, "PCL_ADD_POINT4D padding word");
static_assert(offsetof(floam_point, intensity) == 16, "intensity at 16 (PointXYZI / PointXYZIRT)");
static_assert(offsetof(floam_point, ring) == 20 && sizeof(((floam_point*)nullptr)->ring) == 2, "ring u16 at 20");
static_assert(offsetof(floam_point, time) == 24, "time at 24 (PointXYZIRT)");
static_assert(FLOAM_OK == 0 && FLOAM_ERR_INVALID_ARGUMENT == 1 && FLOAM_ERR_DEVICE == 2, "status codes");
static_assert(FLOAM_VANILLA == 0 && FLOAM_INITIAL_ITERATION == 1 && FLOAM_REFINEMENT_AND_UPDATE == 2,
              "OdomEstimationClass::UpdateType (include/odomEstimationClass.h:56)");

static int failures = 0;
#define CHECK(cond)                                                             \
  do {                                                                          \
    if (!(cond)) {                                                              \
      std::fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #cond);   \
      ++failures;                                                               \
    }                                                                           \
  } while (0)

static std::string slurp(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const bool expect_no_device = argc > 2 && std::strcmp(argv[2], "nodevice") == 0;

  CHECK(std::strstr(floam_version(), "gfx950") != nullptr);
  CHECK(floam_abi_version() == FLOAM_ABI_VERSION);
  {   // the one-call host entry points of the drop-in adapters (ABI 2): argument validation needs no device
    size_t ne = 7, ns = 7;
    CHECK(floam_lp_feature_extraction_host(nullptr, nullptr, 0, 32, nullptr, 0, &ne, nullptr, 0, &ns) ==
          FLOAM_ERR_INVALID_ARGUMENT);
    CHECK(floam_odom_update_selector_host(nullptr, nullptr, 0, nullptr, 0, 32, 1) == FLOAM_ERR_INVALID_ARGUMENT);
  }
  {   // peer sharding (ABI 3): validation before any device work
    char h[64];
    void* p = nullptr;
    CHECK(floam_odom_shard_exchange(nullptr, h, &p) == FLOAM_ERR_INVALID_ARGUMENT && p == nullptr);
    CHECK(floam_odom_set_shard_peers(nullptr, 0, 2, h, nullptr) == FLOAM_ERR_INVALID_ARGUMENT);
  }

  // null handles / arguments are rejected with a message, never dereferenced
  CHECK(floam_cloud_create(0, 0, nullptr) == FLOAM_ERR_INVALID_ARGUMENT);
  CHECK(std::strstr(floam_last_error(), "null") != nullptr);
  floam_lp* lp = nullptr;
  CHECK(floam_lp_create(nullptr, 0, &lp) == FLOAM_ERR_INVALID_ARGUMENT);
  double q[4], t[3];
  CHECK(floam_odom_get_pose(nullptr, q, t) == FLOAM_ERR_INVALID_ARGUMENT);
  CHECK(floam_odom_update_selector(nullptr, nullptr, nullptr, 1) == FLOAM_ERR_INVALID_ARGUMENT);
  CHECK(floam_odom_set_precision(nullptr, FLOAM_PRECISION_FP32) == FLOAM_ERR_INVALID_ARGUMENT);
  // KeyFrameUpdate(surf_cloud, edge_cloud, pose) (include/odomEstimationClass.h:80): the reference's argument order,
  // the clouds as device clouds (either may be null), the pose as (q, t)
  {
    floam_status (*kfu)(floam_odom*, const floam_cloud*, const floam_cloud*, const double*, const double*, int*) =
        &floam_odom_keyframe_update;
    int kf = -1;
    CHECK(kfu(nullptr, nullptr, nullptr, q, t, &kf) == FLOAM_ERR_INVALID_ARGUMENT && kf == -1);
    size_t nk = 7;
    CHECK(floam_odom_get_keyframe(nullptr, 0, q, t, nullptr, nullptr, &nk) == FLOAM_ERR_INVALID_ARGUMENT);
  }

  // device calls fail loudly without a gfx950 device (no CPU fallback)
  if (expect_no_device) {
    floam_cloud* c = nullptr;
    CHECK(floam_cloud_create(0, 16, &c) == FLOAM_ERR_DEVICE && c == nullptr);
    CHECK(std::strlen(floam_last_error()) > 0);
    floam_lidar_params p{64, 0.1, 2.0, 90.0, 0.5};
    floam_odom* o = nullptr;
    CHECK(floam_odom_create(&p, 0.1, "Cauchy", 0, &o) == FLOAM_ERR_DEVICE && o == nullptr);
  }

  // euler2Quaternion (src/lidar.cpp:8-16): a pure yaw of 90 deg
  CHECK(floam_euler_to_quaternion(0.0, 0.0, 90.0, q) == FLOAM_OK);
  CHECK(std::fabs(q[2] - std::sqrt(0.5)) < 1e-12 && std::fabs(q[3] - std::sqrt(0.5)) < 1e-12);

  // SavePosesHomogeneousBALM (src/odomEstimationNode.cpp:97-117): one pose row + one binary PCD
  floam_point pts[3];
  std::memset(pts, 0, sizeof(pts));
  for (int i = 0; i < 3; ++i) {
    pts[i].x = 1.0f + i;
    pts[i].y = 2.0f;
    pts[i].z = 3.0f;
    pts[i].pad0 = 1.0f;
    pts[i].intensity = 0.5f;
  }
  const double pose[16] = {1, 0, 0, 0.25, 0, 1, 0, 0.5, 0, 0, 1, 0.75, 0, 0, 0, 1};
  const double stamp = 12.5;
  const floam_point* clouds[1] = {pts};
  const size_t sizes[1] = {3};
  const std::string balm = dir + "/";
  CHECK(floam_save_poses_balm(balm.c_str(), pose, &stamp, clouds, sizes, 1) == FLOAM_OK);
  const std::string csv = slurp(balm + "alidarPose.csv");
  CHECK(!csv.empty() && csv.find("0.25") != std::string::npos);
  const std::string pcd = slurp(balm + "full0.pcd");
  CHECK(pcd.find("FIELDS x y z intensity") != std::string::npos && pcd.find("POINTS 3") != std::string::npos);
  CHECK(pcd.find("DATA binary") != std::string::npos);
  // the binary body: 3 points of 16 B (x y z intensity), after the header
  const size_t body = pcd.find("DATA binary\n");
  CHECK(body != std::string::npos && pcd.size() == body + std::strlen("DATA binary\n") + 3 * 16);
  CHECK(floam_save_pcd(nullptr, pts, 3) == FLOAM_ERR_INVALID_ARGUMENT);

  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("abi_check ok\n");
  return 0;
}
