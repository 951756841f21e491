// CPU ORACLE (test infrastructure) — the small slice of Eigen 3.3 the reference path uses, restated.
// Quaternion storage order is Eigen's (x, y, z, w), matching `double parameters[7]` at
// include/odomEstimationClass.h:90-92.
#pragma once
#include <cmath>
#include <cstring>
#include <limits>
#include <utility>
#include <vector>

namespace oracle {

struct V3 {
  double x, y, z;
  double operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
  double& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator*(double s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline V3 operator/(V3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) {   // Eigen MatrixBase::cross (generic path)
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline double sqnorm(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
inline double norm(V3 a) { return std::sqrt(sqnorm(a)); }

struct M3 {
  double m[3][3];
  static M3 zero() { M3 r; std::memset(r.m, 0, sizeof(r.m)); return r; }
  static M3 identity() { M3 r = zero(); r.m[0][0] = r.m[1][1] = r.m[2][2] = 1; return r; }
};
inline M3 mul(const M3& a, const M3& b) {
  M3 r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j];
  return r;
}
inline V3 mul(const M3& a, V3 v) {
  return {a.m[0][0] * v.x + a.m[0][1] * v.y + a.m[0][2] * v.z, a.m[1][0] * v.x + a.m[1][1] * v.y + a.m[1][2] * v.z,
          a.m[2][0] * v.x + a.m[2][1] * v.y + a.m[2][2] * v.z};
}
inline M3 transpose(const M3& a) {
  M3 r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[j][i];
  return r;
}
// skew (src/lidarOptimization.cpp:142-152)
inline M3 skew(V3 v) {
  M3 s = M3::zero();
  s.m[0][1] = -v.z; s.m[0][2] = v.y; s.m[1][2] = -v.x;
  s.m[1][0] = v.z; s.m[2][0] = -v.y; s.m[2][1] = v.x;
  return s;
}

struct Quat {
  double x, y, z, w;
};
// Eigen QuaternionBase::_transformVector
inline V3 rotate(const Quat& q, V3 v) {
  const V3 qv{q.x, q.y, q.z};
  V3 uv = cross(qv, v);
  uv = uv + uv;
  const V3 a = v + q.w * uv;
  return a + cross(qv, uv);
}
// Eigen quat_product (generic form)
inline Quat qmul(const Quat& a, const Quat& b) {
  return {a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
          a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
// Eigen QuaternionBase::toRotationMatrix
inline M3 to_matrix(const Quat& q) {
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  M3 r;
  r.m[0][0] = 1 - (tyy + tzz); r.m[0][1] = txy - twz; r.m[0][2] = txz + twy;
  r.m[1][0] = txy + twz; r.m[1][1] = 1 - (txx + tzz); r.m[1][2] = tyz - twx;
  r.m[2][0] = txz - twy; r.m[2][1] = tyz + twx; r.m[2][2] = 1 - (txx + tyy);
  return r;
}
// Eigen quaternionbase_assign_impl<Matrix3>
inline Quat from_matrix(const M3& a) {
  Quat q;
  double t = a.m[0][0] + a.m[1][1] + a.m[2][2];
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    q.w = 0.5 * t;
    t = 0.5 / t;
    q.x = (a.m[2][1] - a.m[1][2]) * t;
    q.y = (a.m[0][2] - a.m[2][0]) * t;
    q.z = (a.m[1][0] - a.m[0][1]) * t;
  } else {
    int i = 0;
    if (a.m[1][1] > a.m[0][0]) i = 1;
    if (a.m[2][2] > a.m[i][i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(a.m[i][i] - a.m[j][j] - a.m[k][k] + 1.0);
    double c[3];
    c[i] = 0.5 * t;
    t = 0.5 / t;
    q.w = (a.m[k][j] - a.m[j][k]) * t;
    c[j] = (a.m[j][i] + a.m[i][j]) * t;
    c[k] = (a.m[k][i] + a.m[i][k]) * t;
    q.x = c[0]; q.y = c[1]; q.z = c[2];
  }
  return q;
}

// Eigen::Isometry3d (rotation part + translation)
struct Iso {
  M3 R;
  V3 t;
  static Iso identity() { return Iso{M3::identity(), V3{0, 0, 0}}; }
};
inline Iso mul(const Iso& a, const Iso& b) { return Iso{mul(a.R, b.R), mul(a.R, b.t) + a.t}; }
inline Iso inverse(const Iso& a) {   // Transform::inverse(Isometry)
  const M3 Rt = transpose(a.R);
  const V3 t = mul(Rt, a.t);
  return Iso{Rt, V3{-t.x, -t.y, -t.z}};
}
// AngleAxisd(R).angle() via quaternion (Eigen 3.3 AngleAxis::operator=(QuaternionBase))
inline double rotation_angle(const M3& R) {
  const Quat q = from_matrix(R);
  const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z);
  if (n == 0) return 0.0;
  return 2.0 * std::atan2(n, std::fabs(q.w));
}

// Eigen::numext::hypot (Eigen 3.3 hypot_impl)
inline double e_hypot(double x, double y) {
  const double ax = std::fabs(x), ay = std::fabs(y);
  double p, qp;
  if (ax > ay) { p = ax; qp = ay / p; } else { p = ay; qp = ax / p; }
  if (p == 0) return 0.0;
  return p * std::sqrt(1.0 + qp * qp);
}

// SelfAdjointEigenSolver<Matrix3d>::compute (Eigen 3.3: 3x3 closed-form tridiagonalisation,
// implicit-shift tridiagonal QR with Givens rotations, ascending sort).  Input: symmetric A.
// Output: eval ascending, evec column-major evec[col][row].
void eig_sym3(const M3& A, double eval[3], double evec[3][3]);

// ColPivHouseholderQR<Matrix<double,5,3>>::solve(b) (Eigen 3.3, incl. column-norm downdating)
void colpiv_qr_solve_5x3(const double A[5][3], const double b[5], double x[3]);

// HouseholderQR<MatrixXd>::solve for an (m x 6) column-major matrix (Ceres DenseQRSolver::SolveUsingEigen)
void householder_qr_solve(std::vector<double>& A_colmajor, int m, int n, const std::vector<double>& b, double* x);

}  // namespace oracle
