// Rigid-transform algebra of the odometry controller (Eigen::Isometry3d / Quaterniond semantics as the reference
// uses them: src/odomEstimationClass.cpp:62-71, 114-116, 320-343).  Host and device share these definitions so the
// prediction the device forms between the two updatePointsToMap calls of a deskewed scan is bit-identical to the
// host's (both built with -ffp-contract=off; only +, *, / and sqrt, all correctly rounded in IEEE double).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

namespace floam {

struct Mat3 {
  double m[3][3];
};
struct Pose {   // rotation matrix + translation (Eigen::Isometry3d)
  Mat3 R;
  double t[3];
};

__host__ __device__ inline Mat3 mat_identity() {
  Mat3 r{};
  r.m[0][0] = r.m[1][1] = r.m[2][2] = 1.0;
  return r;
}
__host__ __device__ inline Pose pose_identity() {
  Pose p;
  p.R = mat_identity();
  p.t[0] = p.t[1] = p.t[2] = 0.0;
  return p;
}
__host__ __device__ inline Mat3 mat_mul(const Mat3& a, const Mat3& b) {
  Mat3 r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j];
  return r;
}
__host__ __device__ inline void mat_vec(const Mat3& a, const double v[3], double o[3]) {
  for (int i = 0; i < 3; ++i) o[i] = a.m[i][0] * v[0] + a.m[i][1] * v[1] + a.m[i][2] * v[2];
}
__host__ __device__ inline Pose pose_mul(const Pose& a, const Pose& b) {
  Pose r;
  r.R = mat_mul(a.R, b.R);
  double v[3];
  mat_vec(a.R, b.t, v);
  for (int i = 0; i < 3; ++i) r.t[i] = v[i] + a.t[i];
  return r;
}
__host__ __device__ inline Pose pose_inverse(const Pose& a) {
  Pose r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.R.m[i][j] = a.R.m[j][i];
  double v[3];
  mat_vec(r.R, a.t, v);
  for (int i = 0; i < 3; ++i) r.t[i] = -v[i];
  return r;
}
// Quaternion (x, y, z, w) -> rotation matrix (Eigen QuaternionBase::toRotationMatrix)
__host__ __device__ inline Mat3 quat_to_mat(const double q[4]) {
  const double x = q[0], y = q[1], z = q[2], w = q[3];
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  Mat3 r;
  r.m[0][0] = 1 - (tyy + tzz); r.m[0][1] = txy - twz; r.m[0][2] = txz + twy;
  r.m[1][0] = txy + twz; r.m[1][1] = 1 - (txx + tzz); r.m[1][2] = tyz - twx;
  r.m[2][0] = txz - twy; r.m[2][1] = tyz + twx; r.m[2][2] = 1 - (txx + tyy);
  return r;
}
// Shepperd's branch for the largest diagonal entry I (compile-time indices: a run-time index into the matrix made the
// device compiler keep it in scratch, 104 B per lane in every kernel that forms a pose)
template <int I>
__host__ __device__ inline void mat_to_quat_branch(const Mat3& a, double q[4]) {
  constexpr int J = (I + 1) % 3, K = (J + 1) % 3;
  double t = sqrt(a.m[I][I] - a.m[J][J] - a.m[K][K] + 1.0);
  double c[3];
  c[I] = 0.5 * t;
  t = 0.5 / t;
  q[3] = (a.m[K][J] - a.m[J][K]) * t;
  c[J] = (a.m[J][I] + a.m[I][J]) * t;
  c[K] = (a.m[K][I] + a.m[I][K]) * t;
  q[0] = c[0]; q[1] = c[1]; q[2] = c[2];
}
// Rotation matrix -> quaternion (x, y, z, w) (Eigen quaternionbase_assign_impl, Shepperd's method)
__host__ __device__ inline void mat_to_quat(const Mat3& a, double q[4]) {
  double t = a.m[0][0] + a.m[1][1] + a.m[2][2];
  if (t > 0) {
    t = sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (a.m[2][1] - a.m[1][2]) * t;
    q[1] = (a.m[0][2] - a.m[2][0]) * t;
    q[2] = (a.m[1][0] - a.m[0][1]) * t;
  } else {
    int i = 0;
    if (a.m[1][1] > a.m[0][0]) i = 1;
    if (a.m[2][2] > (i == 0 ? a.m[0][0] : a.m[1][1])) i = 2;
    if (i == 0) mat_to_quat_branch<0>(a, q);
    else if (i == 1) mat_to_quat_branch<1>(a, q);
    else mat_to_quat_branch<2>(a, q);
  }
}
// Eigen::AngleAxisd(R).angle()
__host__ __device__ inline double rotation_angle(const Mat3& R) {
  double q[4];
  mat_to_quat(R, q);
  const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
  if (n == 0) return 0.0;
  return 2.0 * atan2(n, fabs(q[3]));
}

// Eigen Quaterniond(odom.rotation()), odom.translation() -> parameters {qx, qy, qz, qw, tx, ty, tz}
__host__ __device__ inline void pose_to_params(const Pose& p, double x[7]) {
  mat_to_quat(p.R, x);
  x[4] = p.t[0];
  x[5] = p.t[1];
  x[6] = p.t[2];
}
// Isometry3d(q.toRotationMatrix(), t) from parameters
__host__ __device__ inline Pose params_to_pose(const double x[7]) {
  Pose p;
  p.R = quat_to_mat(x);
  p.t[0] = x[4];
  p.t[1] = x[5];
  p.t[2] = x[6];
  return p;
}

}  // namespace floam
