// CPU ORACLE (test infrastructure) — IMU pre-processing of the laser-processing node, restated.
//
//   dmapping::ImuHandler::AddMsg / Get / TimeContained      src/dataHandler.cpp:23-81
//   dmapping::Compensate                                    src/dataHandler.cpp:93-122
//   CenterTime                                              src/laserProcessingNode.cpp:65-78
//   ImuNowT + pcl::transformPointCloud (IMU alignment)      src/laserProcessingNode.cpp:109-113
//   euler2Quaternion                                        src/lidar.cpp:8-16
//
// Third-party arithmetic restated (versions as in oracle.hpp): ros::Time (roscpp_core 0.6, Melodic: fromSec with
// boost::math::round, toSec, fromNSec), pcl_conversions::fromPCL/toPCL (stamp in microseconds), Eigen 3.3.4 on
// x86-64 with SSE2 and no SSE3 (the reference has no -march, CMakeLists.txt:5-6): Quaterniond products use the
// packet kernel of Geometry_SSE.h (quat_product<SSE, ..., double>), squaredNorm the 2-lane packet reduction
// (x^2+z^2)+(y^2+w^2); PCL 1.8.1 transforms.hpp (dense path, double transform, left-to-right row sums).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "la.hpp"
#include "oracle.hpp"

namespace oracle {

// Eigen 3.3 Geometry_SSE.h, quat_product<Architecture::SSE, Derived, OtherDerived, double> without SSE3 (mask path)
Quat qmul_sse2(const Quat& a, const Quat& b) {
  Quat r;
  r.x = (a.w * b.x + a.y * b.z) - (a.z * b.y - a.x * b.w);
  r.y = (a.w * b.y + a.y * b.w) + (a.z * b.x - a.x * b.z);
  r.z = (a.w * b.z - a.y * b.x) + (a.z * b.w + a.x * b.y);
  r.w = (a.w * b.w - a.y * b.y) - (a.z * b.z + a.x * b.x);
  return r;
}

// QuaternionBase::inverse (Eigen 3.3 Quaternion.h): conjugate / squaredNorm, zero when the norm is not positive
Quat qinverse(const Quat& q) {
  const double n2 = (q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w);
  if (n2 > 0.0) return Quat{-q.x / n2, -q.y / n2, -q.z / n2, q.w / n2};
  return Quat{0.0, 0.0, 0.0, 0.0};
}

// euler2Quaternion (src/lidar.cpp:8-16): rollAngle * yawAngle * pitchAngle, each AngleAxisd -> Quaterniond
// (w = cos(angle/2), vec = sin(angle/2) * axis) and the products in that order.
Quat euler_to_quaternion(double roll, double pitch, double yaw) {
  auto aa = [](double deg, int axis) {
    const double ha = 0.5 * (deg * M_PI / 180.0);
    const double s = std::sin(ha);
    Quat q{0.0 * s, 0.0 * s, 0.0 * s, std::cos(ha)};
    if (axis == 0) q.x = 1.0 * s;
    if (axis == 1) q.y = 1.0 * s;
    if (axis == 2) q.z = 1.0 * s;
    return q;
  };
  return qmul_sse2(qmul_sse2(aa(roll, 0), aa(yaw, 2)), aa(pitch, 1));
}

// ------------------------------------------------------------------------------------------ ros::Time helpers
// pcl_conversions::fromPCL(uint64 stamp, ros::Time&) = fromNSec(stamp * 1000); ros::Time::toSec()
double pcl_stamp_to_sec(uint64_t stamp_us) {
  const uint64_t ns = stamp_us * 1000ull;
  const uint32_t sec = (uint32_t)(ns / 1000000000ull);
  const uint32_t nsec = (uint32_t)(ns % 1000000000ull);
  return (double)sec + 1e-9 * (double)nsec;
}
// ros::Time(double) (fromSec: floor, boost::math::round of the nanoseconds, carry) then pcl_conversions::toPCL
// (toNSec() / 1000).  Returns false where ros::Time throws ("Time is out of dual 32-bit range").
bool sec_to_pcl_stamp(double t, uint64_t* stamp_us) {
  const double fl = std::floor(t);
  if (!(fl >= 0.0) || fl > 4294967295.0) return false;
  const int64_t sec64 = (int64_t)fl;
  uint32_t sec = (uint32_t)sec64;
  uint32_t nsec = (uint32_t)std::round((t - (double)sec) * 1e9);   // boost::math::round: half away from zero
  sec += nsec / 1000000000ul;
  nsec %= 1000000000ul;
  *stamp_us = ((uint64_t)sec * 1000000000ull + (uint64_t)nsec) / 1000ull;
  return true;
}

// ------------------------------------------------------------------------------------------ ImuHandler
// ImuHandler::AddMsg (src/dataHandler.cpp:23-38): appended iff the handler is empty or the stamp is more than
// 1e-5 s after the last one (so the stamps stay strictly increasing).  Only the orientation is kept: it is the
// only field the path reads (Imu2Orientation, :7-9).
bool ImuHandler::add_msg(double stamp, const Quat& orientation) {
  if (!t.empty() && !(stamp - t.back() > 0.00001)) return false;
  t.push_back(stamp);
  q.push_back(orientation);
  return true;
}

// std::lower_bound with compare (:18-21): first sample whose stamp is not < ts
size_t ImuHandler::lower_bound(double ts) const {
  size_t first = 0, count = t.size();
  while (count > 0) {
    const size_t step = count / 2, it = first + step;
    if (t[it] < ts) {
      first = it + 1;
      count -= step + 1;
    } else {
      count = step;
    }
  }
  return first;
}

// ImuHandler::Get(t, data) (:48-69): the sample BEFORE the lower bound (Interpolate returns data1, :45-47), valid
// only when the lower bound is neither end() nor begin() and the sample before it is not begin().
bool ImuHandler::get(double ts, Quat* out) const {
  const size_t a = lower_bound(ts);
  if (a != t.size() && a != 0 && a - 1 != 0) {
    *out = q[a - 1];
    return true;
  }
  return false;
}
// ImuHandler::Get(t) (:71-75): a default-constructed sensor_msgs::Imu (orientation all zero) when not found
Quat ImuHandler::get_or_zero(double ts) const {
  Quat r{0.0, 0.0, 0.0, 0.0};
  get(ts, &r);
  return r;
}
// ImuHandler::TimeContained (:76-81)
bool ImuHandler::time_contained(double ts) const { return !t.empty() && ts >= t.front() && ts <= t.back(); }

// ------------------------------------------------------------------------------------------ node pre-processing
// CenterTime (src/laserProcessingNode.cpp:65-78): in place.  Empty clouds are left untouched (the reference reads
// points.back() of an empty vector, undefined).
void center_time(Pt* pts, size_t n, uint64_t* stamp_us) {
  if (n == 0) return;
  const double tScan = pcl_stamp_to_sec(*stamp_us);
  const double tEnd = tScan + (double)pts[n - 1].time;
  const double tBegin = tScan + (double)pts[0].time;
  const double tCenter = tBegin + (tEnd - tBegin) / 2.0;
  uint64_t st = 0;
  if (sec_to_pcl_stamp(tCenter, &st)) *stamp_us = st;
  for (size_t i = 0; i < n; ++i) pts[i].time = (float)(((double)pts[i].time + tScan) - tCenter);
}

// dmapping::Compensate (src/dataHandler.cpp:93-122): rotate every point by qInit^-1 * qNow (IMU orientations times
// the extrinsics) in double, store float.  Fields other than x, y, z are copied; the output's padding is canonical.
bool compensate(const Pt* in, size_t n, uint64_t stamp_us, const ImuHandler& h, const Quat& extr, Pt* out) {
  if (n == 0) return false;
  const double tScan = pcl_stamp_to_sec(stamp_us);
  const double t0 = (double)in[0].time + tScan;
  const double t1 = (double)in[n - 1].time + tScan;
  if (!h.time_contained(t0) || !h.time_contained(t1)) return false;   // "no imu data" (:101-104)
  const Quat qInit = qmul_sse2(h.get_or_zero(tScan), extr);
  const Quat qInitInv = qinverse(qInit);
  for (size_t i = 0; i < n; ++i) {
    const double timeCurrent = tScan + (double)in[i].time;
    const Quat qNow = qmul_sse2(h.get_or_zero(timeCurrent), extr);
    const Quat qDiff = qmul_sse2(qInitInv, qNow);
    const V3 p = rotate(qDiff, V3{(double)in[i].x, (double)in[i].y, (double)in[i].z});
    Pt o = in[i];
    o.x = (float)p.x; o.y = (float)p.y; o.z = (float)p.z;
    o.pad0 = 1.0f; o.pad1 = 0; o.pad2 = 0.0f;
    out[i] = o;
  }
  return true;
}

// Eigen::Affine3d ImuNowT(q) + pcl::transformPointCloud(in, out, ImuNowT) (PCL 1.8.1 transforms.hpp, dense path):
// x' = float(((m00 x + m01 y) + m02 z) + m03) with the double matrix of q (translation 0), all fields copied.
void transform_by_quaternion(const Pt* in, size_t n, const Quat& q, Pt* out) {
  const M3 R = to_matrix(q);
  for (size_t i = 0; i < n; ++i) {
    const double x = in[i].x, y = in[i].y, z = in[i].z;
    Pt o = in[i];
    o.x = (float)(((R.m[0][0] * x + R.m[0][1] * y) + R.m[0][2] * z) + 0.0);
    o.y = (float)(((R.m[1][0] * x + R.m[1][1] * y) + R.m[1][2] * z) + 0.0);
    o.z = (float)(((R.m[2][0] * x + R.m[2][1] * y) + R.m[2][2] * z) + 0.0);
    out[i] = o;
  }
}

// The laser-processing node's sequence before featureExtraction (src/laserProcessingNode.cpp:92-120): CenterTime,
// Compensate, then the IMU alignment with the orientation at the (centred) scan stamp.  Returns false where the
// node prints "cannot compensate - no IMU data" and skips the scan (:104-107); `in` is centred in either case.
bool imu_preprocess(Pt* in, size_t n, uint64_t* stamp_us, const ImuHandler& h, const Quat& extr, Pt* out) {
  center_time(in, n, stamp_us);
  std::vector<Pt> comp(n);
  if (!compensate(in, n, *stamp_us, h, extr, comp.data())) return false;
  const Quat q = qmul_sse2(h.get_or_zero(pcl_stamp_to_sec(*stamp_us)), extr);
  transform_by_quaternion(comp.data(), n, q, out);
  return true;
}

}  // namespace oracle
