// Residual blocks of the odometry solve on the device: EdgeAnalyticCostFunction / SurfNormAnalyticCostFunction
// (src/lidarOptimization.cpp:12-74) and their accumulation into the 29 sums of one LM evaluation (cost, J^T J upper,
// J^T r, count), shared by the resident solve (lm.hip) and the geometry launch (odom_kernels.hip), which evaluates the
// edge records of a solve's iteration zero while it builds them.
#pragma once
#include <cfloat>

#include "odom_kernels.hpp"

namespace floam {
namespace lmev {

template <typename R>
__device__ __forceinline__ R real_min() { return DBL_MIN; }
template <>
__device__ __forceinline__ float real_min<float>() { return FLT_MIN; }

// 1 / d for the dependent chains of the solve: v_rcp_f64 + two Newton steps (within an ulp of the division, a third of
// its instructions); the float variant is the plain division
__device__ __forceinline__ double recip(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}
__device__ __forceinline__ float recip(float d) { return 1.0f / d; }

// ===================================================================================== residuals (R = double | float)
// Eigen's q * v: uv = 2 q.vec x v; v + w uv + q.vec x uv
template <typename R>
__device__ __forceinline__ void rot(const R* x, R vx, R vy, R vz, R& ox, R& oy, R& oz) {
  const R qx = x[0], qy = x[1], qz = x[2], qw = x[3];
  R ux = qy * vz - qz * vy, uy = qz * vx - qx * vz, uz = qx * vy - qy * vx;
  ux = ux + ux; uy = uy + uy; uz = uz + uz;
  const R ax = vx + qw * ux, ay = vy + qw * uy, az = vz + qw * uz;
  ox = ax + (qy * uz - qz * uy);
  oy = ay + (qz * ux - qx * uz);
  oz = az + (qx * uy - qy * ux);
}

// EdgeAnalyticCostFunction::Evaluate (src/lidarOptimization.cpp:12-43): J = -(nu/|nu|)^T [de]x [-[lp]x, I] / |de|
// (the divisions by |nu| and |de| as products with their reciprocals: the same values to an ulp)
template <typename R>
__device__ __forceinline__ R edge_residual(const R* x, const R* r9, R J[6]) {
  R lx, ly, lz;
  rot(x, r9[0], r9[1], r9[2], lx, ly, lz);
  lx = lx + x[4]; ly = ly + x[5]; lz = lz + x[6];
  const R pax = lx - r9[3], pay = ly - r9[4], paz = lz - r9[5];
  const R pbx = lx - r9[6], pby = ly - r9[7], pbz = lz - r9[8];
  const R nux = pay * pbz - paz * pby, nuy = paz * pbx - pax * pbz, nuz = pax * pby - pay * pbx;
  const R dex = r9[3] - r9[6], dey = r9[4] - r9[7], dez = r9[5] - r9[8];
  const R de_norm = sqrt(dex * dex + dey * dey + dez * dez);
  const R nn = sqrt(nux * nux + nuy * nuy + nuz * nuz);
  const R ide = recip(de_norm), inn = recip(nn);   // one reciprocal each instead of ten divisions
  const R r = nn * ide;
  const R w0 = -nux * inn, w1 = -nuy * inn, w2 = -nuz * inn;
  // r1 = w * skew(de): skew(de) = [[0,-dz,dy],[dz,0,-dx],[-dy,dx,0]]
  const R r10 = w1 * dez + w2 * (-dey);
  const R r11 = w0 * (-dez) + w2 * dex;
  const R r12 = w0 * dey + w1 * (-dex);
  // dp = [-skew(lp), I]; -skew(lp) = [[0,lz,-ly],[-lz,0,lx],[ly,-lx,0]]
  J[0] = (r11 * (-lz) + r12 * ly) * ide;
  J[1] = (r10 * lz + r12 * (-lx)) * ide;
  J[2] = (r10 * (-ly) + r11 * lx) * ide;
  J[3] = r10 * ide;
  J[4] = r11 * ide;
  J[5] = r12 * ide;
  return r;
}

// SurfNormAnalyticCostFunction::Evaluate (src/lidarOptimization.cpp:51-74): J = n^T [-[pw]x, I]
template <typename R>
__device__ __forceinline__ R surf_residual(const R* x, const R* r7, R J[6]) {
  R px, py, pz;
  rot(x, r7[0], r7[1], r7[2], px, py, pz);
  px = px + x[4]; py = py + x[5]; pz = pz + x[6];
  const R nx = r7[3], ny = r7[4], nz = r7[5];
  const R r = (nx * px + ny * py + nz * pz) + r7[6];
  J[0] = ny * (-pz) + nz * py;
  J[1] = nx * pz + nz * (-px);
  J[2] = nx * (-py) + ny * px;
  J[3] = nx;
  J[4] = ny;
  J[5] = nz;
  return r;
}

// one residual (r, J) into the 29 sums (cost, J^T J upper, J^T r, count), with ceres::HuberLoss(0.1) + Corrector
// (rho'' <= 0 everywhere: residual scaling by sqrt(rho')) when HUBER (src/odomEstimationClass.cpp:84-87)
template <bool HUBER, typename R>
__device__ __forceinline__ void accumulate_residual(R (&acc)[LM_NSUM], R r, R (&J)[6]) {
  const R sq = r * r;
  if (HUBER) {
    R rho0, rho1;
    if (sq > R(0.01)) {
      const R rr = sqrt(sq);
      rho0 = R(2.0) * R(0.1) * rr - R(0.01);
      rho1 = fmax(real_min<R>(), R(0.1) / rr);
    } else {
      rho0 = sq;
      rho1 = R(1.0);
    }
    acc[0] += R(0.5) * rho0;
    const R sr = sqrt(rho1);
    r *= sr;
#pragma unroll
    for (int k = 0; k < 6; ++k) J[k] *= sr;
  } else {
    acc[0] += R(0.5) * sq;
  }
  int h = 1;
#pragma unroll
  for (int a = 0; a < 6; ++a)
#pragma unroll
    for (int b = a; b < 6; ++b) acc[h++] += J[a] * J[b];
#pragma unroll
  for (int a = 0; a < 6; ++a) acc[22 + a] += J[a] * r;
  acc[28] += R(1.0);
}


}  // namespace lmev
}  // namespace floam
