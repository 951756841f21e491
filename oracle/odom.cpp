// CPU ORACLE (test infrastructure) — restatement of OdomEstimationClass + the Ceres 1.13 trust-region LM solve.
// Reference: src/odomEstimationClass.cpp:7-343, include/odomEstimationClass.h:52-126,
// src/lidarOptimization.cpp:12-152, src/dataHandler.cpp:82-92.  Parity unpinned (see oracle.hpp).
//
// Deviation notes (all O(1e-15) on the pose, far below the 1e-3 tolerance):
//  * Eigen 3.3 Isometry3d::rotation() is an SVD polar decomposition; on the (orthonormal up to rounding) linear
//    part it is the identity map up to rounding, so the linear part is used directly.
//  * Eigen's SSE2 quaternion product / packet reductions are restated in scalar order.
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <limits>
#include <string>
#include <vector>

#include "la.hpp"
#include "oracle.hpp"

namespace oracle {

// ------------------------------------------------------------------------------------------ cost functions
namespace {

struct EdgeBlock { V3 cp, a, b; };          // EdgeAnalyticCostFunction (lidarOptimization.h)
struct SurfBlock { V3 cp, n; double d; };   // SurfNormAnalyticCostFunction

struct Problem {
  std::vector<EdgeBlock> edges;
  std::vector<SurfBlock> surfs;
  bool huber = false;
  int size() const { return (int)(edges.size() + surfs.size()); }
};

inline Quat q_of(const double* x) { return Quat{x[0], x[1], x[2], x[3]}; }
inline V3 t_of(const double* x) { return V3{x[4], x[5], x[6]}; }

// src/lidarOptimization.cpp:12-43
double edge_eval(const EdgeBlock& b, const double* x, double* J) {
  const V3 lp = rotate(q_of(x), b.cp) + t_of(x);
  const V3 nu = cross(lp - b.a, lp - b.b);
  const V3 de = b.a - b.b;
  const double de_norm = norm(de);
  const double r = norm(nu) / de_norm;
  if (J) {
    const M3 skew_lp = skew(lp);
    double dp[3][6];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        dp[i][j] = -skew_lp.m[i][j];
        dp[i][3 + j] = (i == j) ? 1.0 : 0.0;
      }
    const M3 skew_de = skew(de);
    const double nn = norm(nu);
    const double w[3] = {-nu.x / nn, -nu.y / nn, -nu.z / nn};
    double r1[3];
    for (int j = 0; j < 3; ++j) r1[j] = w[0] * skew_de.m[0][j] + w[1] * skew_de.m[1][j] + w[2] * skew_de.m[2][j];
    for (int k = 0; k < 6; ++k) J[k] = (r1[0] * dp[0][k] + r1[1] * dp[1][k] + r1[2] * dp[2][k]) / de_norm;
  }
  return r;
}

// src/lidarOptimization.cpp:51-74
double surf_eval(const SurfBlock& b, const double* x, double* J) {
  const V3 pw = rotate(q_of(x), b.cp) + t_of(x);
  const double r = dot(b.n, pw) + b.d;
  if (J) {
    const M3 s = skew(pw);
    double dp[3][6];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        dp[i][j] = -s.m[i][j];
        dp[i][3 + j] = (i == j) ? 1.0 : 0.0;
      }
    for (int k = 0; k < 6; ++k) J[k] = b.n.x * dp[0][k] + b.n.y * dp[1][k] + b.n.z * dp[2][k];
  }
  return r;
}

// PoseSE3Parameterization::Plus + getTransformFromSe3 (src/lidarOptimization.cpp:77-92, 103-140)
void se3_plus(const double* x, const double* delta, double* out) {
  const V3 omega{delta[0], delta[1], delta[2]};
  const V3 upsilon{delta[3], delta[4], delta[5]};
  const M3 Omega = skew(omega);
  const double theta = norm(omega);
  const double half_theta = 0.5 * theta;
  double imag_factor;
  const double real_factor = std::cos(half_theta);
  if (theta < 1e-10) {
    const double theta_sq = theta * theta;
    const double theta_po4 = theta_sq * theta_sq;
    imag_factor = 0.5 - 0.0208333 * theta_sq + 0.000260417 * theta_po4;
  } else {
    imag_factor = std::sin(half_theta) / theta;
  }
  const Quat dq{imag_factor * omega.x, imag_factor * omega.y, imag_factor * omega.z, real_factor};
  M3 Jm;
  if (theta < 1e-10) {
    Jm = to_matrix(dq);
  } else {
    const M3 Omega2 = mul(Omega, Omega);
    const double c1 = (1 - std::cos(theta)) / (theta * theta);
    const double c2 = (theta - std::sin(theta)) / std::pow(theta, 3);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Jm.m[i][j] = ((i == j) ? 1.0 : 0.0) + c1 * Omega.m[i][j] + c2 * Omega2.m[i][j];
  }
  const V3 dt = mul(Jm, upsilon);
  const Quat qp = qmul(dq, q_of(x));
  const V3 tp = rotate(dq, t_of(x)) + dt;
  out[0] = qp.x; out[1] = qp.y; out[2] = qp.z; out[3] = qp.w;
  out[4] = tp.x; out[5] = tp.y; out[6] = tp.z;
}

// ceres::HuberLoss(0.1)::Evaluate + Corrector (residual scaling only: rho'' <= 0 everywhere)
struct Loss {
  double rho0, rho1;
};
inline Loss huber(double s) {
  const double a = 0.1, b = 0.01;
  if (s > b) {
    const double r = std::sqrt(s);
    return Loss{2.0 * a * r - b, std::max(std::numeric_limits<double>::min(), a / r)};
  }
  return Loss{s, 1.0};
}

// ProgramEvaluator::Evaluate: cost = sum 0.5*rho(r^2); corrected residuals/Jacobian (local, first 6 columns);
// gradient = J^T r accumulated block by block.  J is column-major C x 6.
bool evaluate(const Problem& P, const double* x, double* cost, std::vector<double>* res, std::vector<double>* J,
              double* g) {
  const int C = P.size();
  double c = 0;
  if (g) std::fill(g, g + 6, 0.0);
  for (int i = 0; i < C; ++i) {
    double jr[6];
    const bool want_j = (J != nullptr) || (g != nullptr);
    double r = (i < (int)P.edges.size()) ? edge_eval(P.edges[i], x, want_j ? jr : nullptr)
                                          : surf_eval(P.surfs[i - P.edges.size()], x, want_j ? jr : nullptr);
    const double sq = r * r;
    if (!std::isfinite(r)) return false;
    if (P.huber) {
      const Loss L = huber(sq);
      c += 0.5 * L.rho0;
      const double sr = std::sqrt(L.rho1);
      r *= sr;
      if (want_j)
        for (int k = 0; k < 6; ++k) jr[k] *= sr;
    } else {
      c += 0.5 * sq;
    }
    if (want_j)
      for (int k = 0; k < 6; ++k)
        if (!std::isfinite(jr[k])) return false;
    if (res) (*res)[i] = r;
    if (J)
      for (int k = 0; k < 6; ++k) (*J)[(size_t)k * C + i] = jr[k];
    if (g)
      for (int k = 0; k < 6; ++k) g[k] += jr[k] * r;
  }
  *cost = c;
  return true;
}

double norm7(const double* a) {
  double s = 0;
  for (int i = 0; i < 7; ++i) s += a[i] * a[i];
  return std::sqrt(s);
}

struct SolveOut {
  int iterations = 0, successful = 0;
  double initial_cost = 0, final_cost = 0;
  double H0[21] = {0}, g0[6] = {0};
};

// ceres::Solve with LEVENBERG_MARQUARDT + DENSE_QR, max_num_iterations = 4, all other options default
// (src/odomEstimationClass.cpp:100-108; TrustRegionMinimizer / LevenbergMarquardtStrategy of Ceres 1.13).
SolveOut ceres_solve(const Problem& P, double* params) {
  SolveOut so;
  const int C = P.size();
  if (C == 0) return so;   // reduced program has no parameter blocks: parameters untouched
  const double kMinRelDecrease = 1e-3, kFuncTol = 1e-6, kGradTol = 1e-10, kParamTol = 1e-8;
  const double kMinDiag = 1e-6, kMaxDiag = 1e32, kMaxRadius = 1e16, kMinRadius = 1e-32;
  const int kMaxIter = 4, kMaxInvalid = 5;

  double x[7], cand[7];
  std::copy(params, params + 7, x);
  double x_norm = norm7(x);
  double minimum_cost = std::numeric_limits<double>::max();
  std::vector<double> r(C), J((size_t)C * 6);
  double g[6], scale[6], x_cost;

  auto grad_max_norm = [&](const double* xx, const double* gg) {
    double ng[6], proj[7];
    for (int k = 0; k < 6; ++k) ng[k] = -gg[k];
    se3_plus(xx, ng, proj);
    double m = 0;
    for (int i = 0; i < 7; ++i) m = std::max(m, std::fabs(xx[i] - proj[i]));
    return m;
  };
  auto col_sqnorm = [&](int k) {
    double s = 0;
    for (int i = 0; i < C; ++i) s += J[(size_t)k * C + i] * J[(size_t)k * C + i];
    return s;
  };

  // IterationZero
  if (!evaluate(P, x, &x_cost, &r, &J, g)) return so;
  for (int a = 0, idx = 0; a < 6; ++a)
    for (int b = a; b < 6; ++b, ++idx) {
      double s = 0;
      for (int i = 0; i < C; ++i) s += J[(size_t)a * C + i] * J[(size_t)b * C + i];
      so.H0[idx] = s;
    }
  std::copy(g, g + 6, so.g0);
  for (int k = 0; k < 6; ++k) scale[k] = 1.0 / (1.0 + std::sqrt(col_sqnorm(k)));
  auto scale_columns = [&]() {
    for (int k = 0; k < 6; ++k)
      for (int i = 0; i < C; ++i) J[(size_t)k * C + i] *= scale[k];
  };
  scale_columns();
  double gmax = grad_max_norm(x, g);
  so.initial_cost = x_cost;
  so.final_cost = x_cost;
  // Finalize(iteration 0): step_is_successful = true
  if (x_cost < minimum_cost) {
    minimum_cost = x_cost;
    std::copy(x, x + 7, params);
  }
  if (gmax <= kGradTol) return so;

  double radius = 1e4, dfac = 2.0;
  bool reuse = false;
  int num_invalid = 0;
  double diag[6];
  std::vector<double> A((size_t)(C + 6) * 6), rhs(C + 6);
  for (int iter = 1;; ++iter) {
    so.iterations = iter;
    bool success = false;
    // ComputeTrustRegionStep -> LevenbergMarquardtStrategy::ComputeStep
    if (!reuse) {
      for (int k = 0; k < 6; ++k) diag[k] = std::min(std::max(col_sqnorm(k), kMinDiag), kMaxDiag);
    }
    for (int k = 0; k < 6; ++k) {
      for (int i = 0; i < C; ++i) A[(size_t)k * (C + 6) + i] = J[(size_t)k * C + i];
      for (int i = 0; i < 6; ++i) A[(size_t)k * (C + 6) + C + i] = (i == k) ? std::sqrt(diag[k] / radius) : 0.0;
    }
    for (int i = 0; i < C; ++i) rhs[i] = r[i];
    for (int i = 0; i < 6; ++i) rhs[C + i] = 0.0;
    double step[6];
    householder_qr_solve(A, C + 6, 6, rhs, step);
    bool finite = true;
    for (int k = 0; k < 6; ++k) {
      finite = finite && std::isfinite(step[k]);
      step[k] = -step[k];
    }
    reuse = true;
    double mcc = -1;
    if (finite) {
      // model_cost_change = -(J s)'(r + J s / 2)
      mcc = 0;
      for (int i = 0; i < C; ++i) {
        double mr = 0;
        for (int k = 0; k < 6; ++k) mr += J[(size_t)k * C + i] * step[k];
        mcc += mr * (r[i] + mr / 2.0);
      }
      mcc = -mcc;
    }
    if (!(mcc > 0.0)) {
      // HandleInvalidStep -> StepIsInvalid -> StepRejected(0)
      if (++num_invalid >= kMaxInvalid) return so;
      radius = radius / dfac;
      dfac *= 2.0;
      reuse = true;
    } else {
      num_invalid = 0;
      double delta[6];
      for (int k = 0; k < 6; ++k) delta[k] = step[k] * scale[k];
      se3_plus(x, delta, cand);
      double cand_cost;
      if (!evaluate(P, cand, &cand_cost, nullptr, nullptr, nullptr)) cand_cost = std::numeric_limits<double>::max();
      // ParameterToleranceReached
      double sn = 0;
      for (int i = 0; i < 7; ++i) sn += (x[i] - cand[i]) * (x[i] - cand[i]);
      sn = std::sqrt(sn);
      if (sn <= kParamTol * (x_norm + kParamTol)) return so;
      // FunctionToleranceReached
      if (std::fabs(x_cost - cand_cost) <= kFuncTol * x_cost) return so;
      const double rho = (x_cost - cand_cost) / mcc;
      if (rho > kMinRelDecrease) {
        // HandleSuccessfulStep
        std::copy(cand, cand + 7, x);
        x_norm = norm7(x);
        if (!evaluate(P, x, &x_cost, &r, &J, g)) return so;
        scale_columns();
        gmax = grad_max_norm(x, g);
        radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * rho - 1.0, 3));
        radius = std::min(kMaxRadius, radius);
        dfac = 2.0;
        reuse = false;
        success = true;
        so.successful++;
      } else {
        radius = radius / dfac;
        dfac *= 2.0;
        reuse = true;
      }
    }
    // FinalizeIterationAndCheckIfMinimizerCanContinue
    if (success && x_cost < minimum_cost) {
      minimum_cost = x_cost;
      std::copy(x, x + 7, params);
      so.final_cost = x_cost;
    }
    if (iter >= kMaxIter) return so;
    if (radius < kMinRadius) return so;
    if (success && gmax <= kGradTol) return so;
  }
}

}  // namespace

// test hooks (capi.cpp): the cost functions and the manifold Plus, for Jacobian known-answer tests
double test_edge_eval(const double cp[3], const double a[3], const double b[3], const double* x, double* J) {
  return edge_eval(EdgeBlock{V3{cp[0], cp[1], cp[2]}, V3{a[0], a[1], a[2]}, V3{b[0], b[1], b[2]}}, x, J);
}
double test_surf_eval(const double cp[3], const double n[3], double d, const double* x, double* J) {
  return surf_eval(SurfBlock{V3{cp[0], cp[1], cp[2]}, V3{n[0], n[1], n[2]}, d}, x, J);
}
void test_se3_plus(const double* x, const double* delta, double* out) { se3_plus(x, delta, out); }

// ------------------------------------------------------------------------------------------ odometry state
struct OdomState {
  LidarParams lp;
  double map_resolution;
  std::string loss;
  bool stable_voxel;
  float leafE, leafS;
  std::vector<Pt> cornerMap, surfMap;
  Iso odom, last_odom;
  double parameters[7] = {0, 0, 0, 1, 0, 0, 0};
  int optimization_count;
  std::vector<Iso> keyframes;
  std::vector<SolveTrace> traces;
};

static bool g_keyframe_first = true;   // KeyFrameUpdate `static bool first` (odomEstimationClass.cpp:323, Q6)
void reset_process_statics() { g_keyframe_first = true; }

namespace {
Quat q_params(const OdomState* s) { return Quat{s->parameters[0], s->parameters[1], s->parameters[2], s->parameters[3]}; }
V3 t_params(const OdomState* s) { return V3{s->parameters[4], s->parameters[5], s->parameters[6]}; }

// pointAssociateToMap (odomEstimationClass.cpp:126-135): double math, float result
Pt associate(const OdomState* s, const Pt& pi) {
  const V3 pc{pi.x, pi.y, pi.z};
  const V3 w = rotate(q_params(s), pc) + t_params(s);
  Pt po{};
  po.x = (float)w.x; po.y = (float)w.y; po.z = (float)w.z; po.pad0 = 1.0f;
  po.intensity = pi.intensity;
  return po;
}

// addEdgeCostFactor's per-query geometry (odomEstimationClass.cpp:156-189): line through the 5 neighbours, kept iff
// the largest eigenvalue exceeds 3x the middle one
bool edge_factor(const std::vector<Pt>& map, const int (&ind)[5], const Pt& p, EdgeBlock* out) {
  V3 near[5];
  V3 center{0, 0, 0};
  for (int j = 0; j < 5; ++j) {
    near[j] = V3{map[ind[j]].x, map[ind[j]].y, map[ind[j]].z};
    center = center + near[j];
  }
  center = center / 5.0;
  M3 cov = M3::zero();
  for (int j = 0; j < 5; ++j) {
    const V3 z = near[j] - center;
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) cov.m[a][b] = cov.m[a][b] + z[a] * z[b];
  }
  double ev[3], evec[3][3];
  eig_sym3(cov, ev, evec);
  const V3 u{evec[2][0], evec[2][1], evec[2][2]};
  if (!(ev[2] > 3 * ev[1])) return false;
  *out = EdgeBlock{V3{p.x, p.y, p.z}, 0.1 * u + center, -0.1 * u + center};
  return true;
}

// addSurfCostFactor's per-query geometry (odomEstimationClass.cpp:208-243): least-squares plane n.x + 1 = 0 through
// the 5 neighbours (ColPivHouseholderQR), kept iff every neighbour is within 0.2 of it
bool surf_factor(const std::vector<Pt>& map, const int (&ind)[5], const Pt& p, SurfBlock* out) {
  double A[5][3], b[5];
  for (int j = 0; j < 5; ++j) {
    A[j][0] = map[ind[j]].x;
    A[j][1] = map[ind[j]].y;
    A[j][2] = map[ind[j]].z;
    b[j] = -1.0;
  }
  double nv[3];
  colpiv_qr_solve_5x3(A, b, nv);
  V3 n{nv[0], nv[1], nv[2]};
  const double z = sqnorm(n);
  const double negative_OA_dot_norm = 1 / std::sqrt(z);
  if (z > 0) n = n / std::sqrt(z);   // Eigen normalize()
  for (int j = 0; j < 5; ++j)
    if (std::fabs(n.x * map[ind[j]].x + n.y * map[ind[j]].y + n.z * map[ind[j]].z + negative_OA_dot_norm) > 0.2)
      return false;
  *out = SurfBlock{V3{p.x, p.y, p.z}, n, negative_OA_dot_norm};
  return true;
}

// addEdgeCostFactor (odomEstimationClass.cpp:144-196)
void add_edge(OdomState* s, const std::vector<Pt>& pc, const std::vector<Pt>& map, const KdTree& kd, Problem& P) {
  for (size_t i = 0; i < pc.size(); ++i) {
    const Pt pt = associate(s, pc[i]);
    const float q[3] = {pt.x, pt.y, pt.z};
    int ind[5];
    float sqd[5];
    kd.knn(q, 5, ind, sqd);
    EdgeBlock e;
    if (sqd[4] < 1.0 && edge_factor(map, ind, pc[i], &e)) P.edges.push_back(e);
  }
}

// addSurfCostFactor (odomEstimationClass.cpp:198-251)
void add_surf(OdomState* s, const std::vector<Pt>& pc, const std::vector<Pt>& map, const KdTree& kd, Problem& P) {
  for (size_t i = 0; i < pc.size(); ++i) {
    const Pt pt = associate(s, pc[i]);
    const float q[3] = {pt.x, pt.y, pt.z};
    int ind[5];
    float sqd[5];
    kd.knn(q, 5, ind, sqd);
    SurfBlock f;
    if (sqd[4] < 1.0 && surf_factor(map, ind, pc[i], &f)) P.surfs.push_back(f);
  }
}

std::vector<Pt> vel_to_intensity(const Pt* in, size_t n) {   // VelToIntensityCopy (:308-318)
  std::vector<Pt> out(n);
  for (size_t i = 0; i < n; ++i) {
    Pt p{};
    p.x = in[i].x; p.y = in[i].y; p.z = in[i].z; p.pad0 = 1.0f;
    p.intensity = in[i].intensity;
    out[i] = p;
  }
  return out;
}

// KeyFrameUpdate (:320-343)
bool keyframe_update(OdomState* s, const Iso& pose) {
  if (g_keyframe_first || s->keyframes.empty()) {
    g_keyframe_first = false;
    s->keyframes.push_back(pose);
    return true;
  }
  const Iso delta = mul(inverse(s->keyframes.back()), pose);
  const double dm = norm(delta.t);
  const double dr = rotation_angle(delta.R);
  if (dm > 0.07 || dr > 2 * M_PI / 180.0) {
    s->keyframes.push_back(pose);
    if (s->keyframes.size() > 3) s->keyframes.erase(s->keyframes.begin());
    return true;
  }
  return false;
}

// addPointsToMap (:253-294)
void add_points_to_map(OdomState* s, const std::vector<Pt>& dE, const std::vector<Pt>& dS) {
  for (const Pt& p : dE) s->cornerMap.push_back(associate(s, p));
  for (const Pt& p : dS) s->surfMap.push_back(associate(s, p));
  const V3 t = s->odom.t;
  const float mn[3] = {(float)(t.x - 100), (float)(t.y - 100), (float)(t.z - 100)};
  const float mx[3] = {(float)(t.x + 100), (float)(t.y + 100), (float)(t.z + 100)};
  std::vector<Pt> tmpCorner, tmpSurf;
  crop_box(s->surfMap.data(), s->surfMap.size(), mn, mx, tmpSurf);
  crop_box(s->cornerMap.data(), s->cornerMap.size(), mn, mx, tmpCorner);
  voxel_grid(tmpSurf.data(), tmpSurf.size(), s->leafS, s->stable_voxel, s->surfMap);
  voxel_grid(tmpCorner.data(), tmpCorner.size(), s->leafE, s->stable_voxel, s->cornerMap);
}
}  // namespace

OdomState* odom_create(const LidarParams& lp, double map_resolution, const std::string& loss, bool stable_voxel) {
  OdomState* s = new OdomState();
  s->lp = lp;
  s->map_resolution = map_resolution;
  s->loss = loss;
  std::transform(s->loss.begin(), s->loss.end(), s->loss.begin(), [](unsigned char c) { return std::tolower(c); });
  s->stable_voxel = stable_voxel;
  s->leafE = (float)map_resolution;
  s->leafS = (float)(map_resolution * 2);
  s->odom = Iso::identity();
  s->last_odom = Iso::identity();
  s->optimization_count = 2;
  return s;
}

void odom_destroy(OdomState* s) { delete s; }

void odom_init_map(OdomState* s, const Pt* edge, size_t ne, const Pt* surf, size_t ns) {
  s->cornerMap.insert(s->cornerMap.end(), edge, edge + ne);
  s->surfMap.insert(s->surfMap.end(), surf, surf + ns);
  s->optimization_count = 12;
}

void odom_update(OdomState* s, const Pt* edge_in, size_t ne, const Pt* surf_in, size_t ns, UpdateType type) {
  const std::vector<Pt> edge = vel_to_intensity(edge_in, ne);
  const std::vector<Pt> surf = vel_to_intensity(surf_in, ns);
  if (s->optimization_count > 2) s->optimization_count--;
  const Iso pred = mul(s->odom, mul(inverse(s->last_odom), s->odom));
  // `update_type == VANILLA || UpdateType::INITIAL_ITERATION` is always true (Q2)
  s->last_odom = s->odom;
  s->odom = pred;
  const Quat q = from_matrix(s->odom.R);
  s->parameters[0] = q.x; s->parameters[1] = q.y; s->parameters[2] = q.z; s->parameters[3] = q.w;
  s->parameters[4] = s->odom.t.x; s->parameters[5] = s->odom.t.y; s->parameters[6] = s->odom.t.z;

  std::vector<Pt> dE, dS;
  voxel_grid(edge.data(), edge.size(), s->leafE, s->stable_voxel, dE);
  voxel_grid(surf.data(), surf.size(), s->leafS, s->stable_voxel, dS);
  if (s->cornerMap.size() > 10 && s->surfMap.size() > 50) {
    KdTree kdE, kdS;
    kdE.build(s->cornerMap.data(), s->cornerMap.size());
    kdS.build(s->surfMap.data(), s->surfMap.size());
    for (int it = 0; it < s->optimization_count; ++it) {
      Problem P;
      P.huber = (s->loss == "huber");   // any other string: no loss (Q3)
      SolveTrace tr{};
      std::copy(s->parameters, s->parameters + 7, tr.x_in);
      add_edge(s, dE, s->cornerMap, kdE, P);
      add_surf(s, dS, s->surfMap, kdS, P);
      const SolveOut so = ceres_solve(P, s->parameters);
      tr.n_edge_queries = (int)dE.size();
      tr.n_surf_queries = (int)dS.size();
      tr.n_edge_corr = (int)P.edges.size();
      tr.n_surf_corr = (int)P.surfs.size();
      tr.iterations = so.iterations;
      tr.successful = so.successful;
      tr.initial_cost = so.initial_cost;
      tr.final_cost = so.final_cost;
      std::copy(so.H0, so.H0 + 21, tr.H0);
      std::copy(so.g0, so.g0 + 6, tr.g0);
      std::copy(s->parameters, s->parameters + 7, tr.x_out);
      s->traces.push_back(tr);
    }
  }
  s->odom.R = to_matrix(q_params(s));
  s->odom.t = t_params(s);
  if (type == VANILLA || type == REFINEMENT_AND_UPDATE) {
    if (keyframe_update(s, s->odom)) add_points_to_map(s, dE, dS);
  }
}

// CompensateVelocity (src/dataHandler.cpp:82-92): in place, double math, float store (Q5)
static void compensate_velocity(Pt* pts, size_t n, const V3& v) {
  for (size_t i = 0; i < n; ++i) {
    const double tp = pts[i].time;
    const V3 pos{pts[i].x, pts[i].y, pts[i].z};
    const V3 err = tp * v;   // Eigen: velocity * tPoint
    const V3 c = pos + err;
    pts[i].x = (float)c.x; pts[i].y = (float)c.y; pts[i].z = (float)c.z;
  }
}

void odom_update_selector(OdomState* s, Pt* edge, size_t ne, Pt* surf, size_t ns, bool deskew) {
  if (!deskew) {
    odom_update(s, edge, ne, surf, ns, VANILLA);
  } else {
    odom_update(s, edge, ne, edge, ne, INITIAL_ITERATION);   // Q4: edge cloud as the surf input
    V3 v;
    odom_get_velocity(s, &v.x);
    compensate_velocity(edge, ne, v);
    compensate_velocity(surf, ns, v);
    odom_update(s, edge, ne, surf, ns, REFINEMENT_AND_UPDATE);
  }
}

void odom_get_pose(const OdomState* s, double q[4], double t[3]) {
  const Quat qq = from_matrix(s->odom.R);
  q[0] = qq.x; q[1] = qq.y; q[2] = qq.z; q[3] = qq.w;
  t[0] = s->odom.t.x; t[1] = s->odom.t.y; t[2] = s->odom.t.z;
}
void odom_get_last_pose(const OdomState* s, double q[4], double t[3]) {
  const Quat qq = from_matrix(s->last_odom.R);
  q[0] = qq.x; q[1] = qq.y; q[2] = qq.z; q[3] = qq.w;
  t[0] = s->last_odom.t.x; t[1] = s->last_odom.t.y; t[2] = s->last_odom.t.z;
}
// GetVelocity (include/odomEstimationClass.h:78)
void odom_get_velocity(const OdomState* s, double v[3]) {
  const V3 d = s->odom.t - s->last_odom.t;
  v[0] = d.x / s->lp.scan_period;
  v[1] = d.y / s->lp.scan_period;
  v[2] = d.z / s->lp.scan_period;
}
size_t odom_map_size(const OdomState* s, int which) { return which == 0 ? s->cornerMap.size() : s->surfMap.size(); }
const Pt* odom_map_data(const OdomState* s, int which) {
  return which == 0 ? s->cornerMap.data() : s->surfMap.data();
}
const std::vector<SolveTrace>& odom_traces(const OdomState* s) { return s->traces; }
void odom_clear_traces(OdomState* s) { s->traces.clear(); }
int odom_optimization_count(const OdomState* s) { return s->optimization_count; }

// stage hooks (capi.cpp): one correspondence pass — pointAssociateToMap at parameters x, the KD-tree 5-NN, the
// sqd[4] < 1 gate and the factor geometry, per query: neighbours (index, float sq-distance), flags (bit 0 factor
// kept, bit 2 gate passed) and the record (edge cp, a, b; surf cp, n, d)
void stage_correspondences(const Pt* map, size_t m, const Pt* q, size_t nq, const double* x, bool edge, int* idx,
                           float* sqd, unsigned char* flags, double* rec) {
  OdomState s{};
  std::copy(x, x + 7, s.parameters);
  const std::vector<Pt> mp(map, map + m);
  KdTree kd;
  kd.build(mp.data(), mp.size());
  for (size_t i = 0; i < nq; ++i) {
    const Pt pt = associate(&s, q[i]);
    const float qq[3] = {pt.x, pt.y, pt.z};
    int* ind = idx + 5 * i;
    float* d = sqd + 5 * i;
    kd.knn(qq, 5, ind, d);
    flags[i] = 0;
    if (!(d[4] < 1.0)) continue;
    flags[i] = 4;
    int ii[5] = {ind[0], ind[1], ind[2], ind[3], ind[4]};
    if (edge) {
      EdgeBlock e;
      if (edge_factor(mp, ii, q[i], &e)) {
        flags[i] |= 1;
        const double r[9] = {e.cp.x, e.cp.y, e.cp.z, e.a.x, e.a.y, e.a.z, e.b.x, e.b.y, e.b.z};
        std::copy(r, r + 9, rec + 9 * i);
      }
    } else {
      SurfBlock f;
      if (surf_factor(mp, ii, q[i], &f)) {
        flags[i] |= 1;
        const double r[7] = {f.cp.x, f.cp.y, f.cp.z, f.n.x, f.n.y, f.n.z, f.d};
        std::copy(r, r + 7, rec + 7 * i);
      }
    }
  }
}

// pointAssociateToMap (odomEstimationClass.cpp:126-135) of n points at parameters x
void stage_associate(const Pt* in, size_t n, const double* x, Pt* out) {
  OdomState s{};
  std::copy(x, x + 7, s.parameters);
  for (size_t i = 0; i < n; ++i) out[i] = associate(&s, in[i]);
}

// ceres::Solve on given factor records (edge: 9 doubles, surf: 7) from parameters x (in: x_in, out: the solution);
// trace: the SolveTrace layout (49 doubles)
void stage_solve(const double* erec, size_t ne, const double* srec, size_t ns, bool huber, double* x, double* trace) {
  Problem P;
  P.huber = huber;
  for (size_t i = 0; i < ne; ++i) {
    const double* r = erec + 9 * i;
    P.edges.push_back(EdgeBlock{V3{r[0], r[1], r[2]}, V3{r[3], r[4], r[5]}, V3{r[6], r[7], r[8]}});
  }
  for (size_t i = 0; i < ns; ++i) {
    const double* r = srec + 7 * i;
    P.surfs.push_back(SurfBlock{V3{r[0], r[1], r[2]}, V3{r[3], r[4], r[5]}, r[6]});
  }
  double x_in[7];
  std::copy(x, x + 7, x_in);
  const SolveOut so = ceres_solve(P, x);
  int k = 0;
  trace[k++] = 0; trace[k++] = 0; trace[k++] = (double)ne; trace[k++] = (double)ns;
  trace[k++] = so.iterations; trace[k++] = so.successful; trace[k++] = so.initial_cost; trace[k++] = so.final_cost;
  for (int j = 0; j < 7; ++j) trace[k++] = x_in[j];
  for (int j = 0; j < 7; ++j) trace[k++] = x[j];
  for (int j = 0; j < 21; ++j) trace[k++] = so.H0[j];
  for (int j = 0; j < 6; ++j) trace[k++] = so.g0[j];
}

}  // namespace oracle
