// Disk exporters of the odometry node, callable from the C++ nodes through the C ABI:
//   SaveOdom / SavePosegraph (src/utils.cpp:3-106), SaveMerged / SavePosesHomogeneousBALM
//   (src/odomEstimationNode.cpp:66-117), pcl::io::savePCDFileBinary for pcl::PointXYZI (PCL 1.8.1 PCDWriter).
// Text goes through std::ostream exactly as the reference writes it (default precision 6, std::fixed for BALM) and
// Eigen's default matrix format; SaveMerged transforms and voxel-filters on the device (floam_transform_cloud,
// floam_voxel_grid).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "floam_common.hpp"
#include "pose.hpp"

namespace floam {
void set_last_error(const std::string& m);   // host.cpp: floam_last_error()'s thread-local message
}

namespace {

using floam::Error;

void make_dirs(const std::string& d) {
  std::error_code ec;
  std::filesystem::create_directories(d, ec);   // boost::filesystem::create_directories
  if (ec) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "cannot create " + d + ": " + ec.message());
}

// pcl::io::savePCDFileBinary(path, pcl::PointCloud<pcl::PointXYZI>): v0.7 header, x y z intensity packed (16 B)
void save_pcd_xyzi(const std::string& path, const floam_point* pts, size_t n) {
  std::ofstream f(path, std::ios::binary);
  if (!f) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "cannot write " + path);
  f << "# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z intensity\nSIZE 4 4 4 4\n"
       "TYPE F F F F\nCOUNT 1 1 1 1\nWIDTH "
    << n << "\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS " << n << "\nDATA binary\n";
  std::vector<float> packed(4 * n);
  for (size_t i = 0; i < n; ++i) {
    packed[4 * i + 0] = pts[i].x;
    packed[4 * i + 1] = pts[i].y;
    packed[4 * i + 2] = pts[i].z;
    packed[4 * i + 3] = pts[i].intensity;
  }
  f.write(reinterpret_cast<const char*>(packed.data()), (std::streamsize)(packed.size() * sizeof(float)));
}

// ros::Time(double) (roscpp_core fromSec: floor, rounded nanoseconds, carry)
void ros_time(double t, long long& sec, long long& nsec) {
  sec = (long long)std::floor(t);
  const double x = (t - (double)sec) * 1e9;
  nsec = x >= 0 ? (long long)std::floor(x + 0.5) : -(long long)std::floor(-x + 0.5);
  sec += nsec / 1000000000ll;
  nsec %= 1000000000ll;
}

// operator<<(ostream, Eigen::Matrix4d) with the default IOFormat: right-aligned to the widest coefficient
std::string eigen_str(const double* m, int rows, int cols) {
  std::vector<std::string> s((size_t)rows * cols);
  size_t w = 0;
  for (int i = 0; i < rows * cols; ++i) {
    std::ostringstream o;
    o << m[i];
    s[i] = o.str();
    w = std::max(w, s[i].size());
  }
  std::string out;
  for (int r = 0; r < rows; ++r) {
    for (int c = 0; c < cols; ++c) {
      if (c) out += ' ';
      out += std::string(w - s[(size_t)r * cols + c].size(), ' ') + s[(size_t)r * cols + c];
    }
    if (r + 1 < rows) out += '\n';
  }
  return out;
}

// Eigen::Quaterniond(Matrix3d) -> (x, y, z, w) of a row-major 4x4's rotation block
void quat_of(const double* T, double q[4]) {
  floam::Mat3 R;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R.m[i][j] = T[4 * i + j];
  floam::mat_to_quat(R, q);
}

// Eigen::Affine3d::inverse() (Affine mode: the linear block inverted by cofactors, t' = -A^-1 t), row-major 4x4
void affine_inverse(const double* T, double* out) {
  auto A = [&](int i, int j) { return T[4 * i + j]; };
  auto cof = [&](int i, int j) {
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return A(i1, j1) * A(i2, j2) - A(i1, j2) * A(i2, j1);
  };
  const double c0[3] = {cof(0, 0), cof(1, 0), cof(2, 0)};
  const double det = (c0[0] * A(0, 0) + c0[1] * A(1, 0)) + c0[2] * A(2, 0);
  const double inv = 1.0 / det;
  double Ai[3][3];
  for (int j = 0; j < 3; ++j) Ai[0][j] = c0[j] * inv;
  for (int j = 0; j < 3; ++j) Ai[1][j] = cof(j, 1) * inv;
  for (int j = 0; j < 3; ++j) Ai[2][j] = cof(j, 2) * inv;
  for (int i = 0; i < 16; ++i) out[i] = (i % 5 == 0) ? 1.0 : 0.0;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) out[4 * i + j] = Ai[i][j];
    out[4 * i + 3] = -((Ai[i][0] * T[3] + Ai[i][1] * T[7]) + Ai[i][2] * T[11]);
  }
}

void mat4_mul(const double* a, const double* b, double* o) {
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      double s = 0.0;
      for (int k = 0; k < 4; ++k) s += a[4 * i + k] * b[4 * k + j];
      o[4 * i + j] = s;
    }
}

template <typename F>
floam_status guarded_io(F&& f) {
  try {
    f();
    return FLOAM_OK;
  } catch (const Error& e) {
    floam::set_last_error(e.what());
    return e.status;
  } catch (const std::exception& e) {
    floam::set_last_error(e.what());
    return FLOAM_ERR_INVALID_ARGUMENT;
  }
}

void check_cloud_args(const floam_point* const* clouds, const size_t* sizes, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (sizes[i] && !clouds[i]) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null cloud");
}

}  // namespace

extern "C" {

floam_status floam_save_pcd(const char* path, const floam_point* points, size_t n) {
  return guarded_io([&] {
    if (!path || (n && !points)) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    save_pcd_xyzi(path, points, n);
  });
}

floam_status floam_save_odom(const char* dump_directory, const double* poses, const double* keyframe_stamps,
                             const floam_point* const* clouds, const size_t* cloud_sizes, size_t n) {
  return guarded_io([&] {
    if (!dump_directory || (n && (!poses || !keyframe_stamps || !clouds || !cloud_sizes)))
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    check_cloud_args(clouds, cloud_sizes, n);
    const std::string dir = dump_directory;
    make_dirs(dir);
    for (size_t i = 0; i < n; ++i) {
      long long sec, nsec;
      ros_time(keyframe_stamps[i], sec, nsec);
      const std::string base = dir + "/" + std::to_string(sec) + "_" + std::to_string(nsec);
      save_pcd_xyzi(base + ".pcd", clouds[i], cloud_sizes[i]);
      std::ofstream o(base + ".odom");
      const double* m = poses + 16 * i;
      for (int r = 0; r < 4; ++r)
        o << m[4 * r + 0] << " " << m[4 * r + 1] << " " << m[4 * r + 2] << " " << m[4 * r + 3] << std::endl;
    }
  });
}

floam_status floam_save_posegraph(const char* dump_directory, const double* poses, const double* keyframe_stamps,
                                  const floam_point* const* clouds, const size_t* cloud_sizes, size_t n) {
  return guarded_io([&] {
    if (!dump_directory || (n && (!poses || !keyframe_stamps))) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    if (n && (!clouds || !cloud_sizes)) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null clouds");
    check_cloud_args(clouds, cloud_sizes, n);
    const std::string dir = dump_directory;
    make_dirs(dir);
    std::ofstream g(dir + "/graph.g2o");
    for (size_t i = 0; i < n; ++i) {
      const double* T = poses + 16 * i;
      double q[4];
      quat_of(T, q);
      g << "VERTEX_SE3:QUAT " << i << " " << T[3] << " " << T[7] << " " << T[11] << " " << q[0] << " " << q[1] << " "
        << q[2] << " " << q[3] << "\n";
    }
    g << "FIX 0" << "\n";
    if (n <= 1) std::fprintf(stderr, "cannot save a pose graph with only 1 vertex\n");
    const double var[6] = {0.01, 0.01, 0.01, 0.001, 0.001, 0.001};
    for (size_t i = 0; i + 1 < n; ++i) {
      double inv[16], rel[16];
      affine_inverse(poses + 16 * i, inv);
      mat4_mul(inv, poses + 16 * (i + 1), rel);
      double q[4];
      quat_of(rel, q);
      g << "EDGE_SE3:QUAT " << i << " " << i + 1;
      g << " " << rel[3] << " " << rel[7] << " " << rel[11] << " " << q[0] << " " << q[1] << " " << q[2] << " " << q[3];
      for (int r = 0; r < 6; ++r)
        for (int c = r; c < 6; ++c) g << " " << (r == c ? var[r] : 0.0);
      g << "\n";
    }
    g.close();
    for (size_t i = 0; i < n; ++i) {
      char sub[32];
      std::snprintf(sub, sizeof(sub), "/%06zu", i);
      const std::string kd = dir + sub;
      make_dirs(kd);
      save_pcd_xyzi(kd + "/cloud.pcd", clouds[i], cloud_sizes[i]);
      long long sec, nsec;
      ros_time(keyframe_stamps[i], sec, nsec);
      std::ofstream d(kd + "/data");
      d << "stamp " << sec << " " << nsec << "\n";
      d << "estimate\n" << eigen_str(poses + 16 * i, 4, 4) << "\n";
      d << "odom\n" << eigen_str(poses + 16 * i, 4, 4) << "\n";
      d << "accum_distance -1" << "\n";
      d << "id " << i << "\n";
    }
  });
}

floam_status floam_save_poses_balm(const char* directory, const double* poses, const double* stamps,
                                   const floam_point* const* clouds, const size_t* cloud_sizes, size_t n) {
  return guarded_io([&] {
    if (!directory || (n && (!poses || !stamps || !clouds || !cloud_sizes)))
      throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    check_cloud_args(clouds, cloud_sizes, n);
    const std::string dir = directory;
    make_dirs(dir);
    std::fstream stream((dir + "alidarPose.csv").c_str(), std::fstream::out);
    for (size_t i = 0; i < n; ++i) {
      const double* m = poses + 16 * i;
      stream << std::fixed << m[0] << "," << m[1] << "," << m[2] << "," << m[3] << "," << std::endl
             << m[4] << "," << m[5] << "," << m[6] << "," << m[7] << "," << std::endl
             << m[8] << "," << m[9] << "," << m[10] << "," << m[11] << "," << std::endl
             << m[12] << "," << m[13] << "," << m[14] << "," << stamps[i] << "," << std::endl;
      save_pcd_xyzi(dir + "full" + std::to_string(i) + ".pcd", clouds[i], cloud_sizes[i]);
    }
  });
}

floam_status floam_save_merged(const char* directory, const double* poses, const floam_point* const* clouds,
                               const size_t* cloud_sizes, size_t n, double downsample_size, int device) {
  return guarded_io([&] {
    if (!directory || (n && (!poses || !clouds || !cloud_sizes))) throw Error(FLOAM_ERR_INVALID_ARGUMENT, "null argument");
    check_cloud_args(clouds, cloud_sizes, n);
    const std::string dir = directory;
    make_dirs(dir);
    std::vector<floam_point> merged;
    floam_cloud *in = nullptr, *out = nullptr;
    auto ok = [](floam_status s) {
      if (s != FLOAM_OK) throw Error(s, floam_last_error());
    };
    ok(floam_cloud_create(device, 0, &in));
    ok(floam_cloud_create(device, 0, &out));
    try {
      for (size_t i = 0; i < n; ++i) {   // pcl::transformPointCloud(*clouds[i], tmp, poses[i]); merged += tmp
        ok(floam_cloud_upload(in, clouds[i], cloud_sizes[i], sizeof(floam_point)));
        ok(floam_transform_cloud(in, poses + 16 * i, out));
        const size_t base = merged.size();
        merged.resize(base + cloud_sizes[i]);
        size_t got = 0;
        ok(floam_cloud_download(out, merged.data() + base, cloud_sizes[i], &got));
      }
      std::vector<floam_point> down;
      if (!merged.empty()) {   // pcl::VoxelGrid<PointXYZI> at downsample_size
        ok(floam_cloud_upload(in, merged.data(), merged.size(), sizeof(floam_point)));
        ok(floam_voxel_grid(in, (float)downsample_size, out));
        size_t m = 0;
        ok(floam_cloud_size(out, &m));
        down.resize(m);
        ok(floam_cloud_download(out, down.data(), m, &m));
      }
      save_pcd_xyzi(dir + "floam_merged.pcd", merged.data(), merged.size());
      if (!down.empty())
        save_pcd_xyzi(dir + "floam_merged_downsampled_leaf_" + std::to_string(downsample_size) + ".pcd", down.data(),
                      down.size());
      else
        std::printf("No downsampled point cloud saved - increase \"output_downsample_size\"\n");
    } catch (...) {
      floam_cloud_destroy(in);
      floam_cloud_destroy(out);
      throw;
    }
    floam_cloud_destroy(in);
    floam_cloud_destroy(out);
  });
}

}  // extern "C"
