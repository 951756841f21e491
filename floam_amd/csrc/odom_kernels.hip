// Scan-to-map registration on gfx950: spatial-hash kNN correspondence search + fp64 line / plane geometry +
// analytic residuals / Jacobians + normal-equation reduction + on-device Levenberg-Marquardt control.
//
// Reference: src/odomEstimationClass.cpp:78-110 (kd-tree, Ceres problem), :126-135 (pointAssociateToMap),
// :144-196 (addEdgeCostFactor), :198-251 (addSurfCostFactor); src/lidarOptimization.cpp:12-140 (cost functions,
// SE3 Plus).  Ceres 1.13 TrustRegionMinimizer + LevenbergMarquardtStrategy semantics are restated in lm_control
// (see SURVEY.md §8 a-12 and oracle/odom.cpp for the CPU restatement).
#include <cfloat>
#include <climits>

#include "odom_kernels.hpp"
#include "primitives.hpp"

namespace floam {

namespace {
constexpr int kTB = 256;
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

// ===================================================================================== hash grid build
__global__ void grid_setup(const int* __restrict__ mm, const int* __restrict__ d_m, int shift, unsigned mask,
                           GridParams* __restrict__ gp) {
  if (threadIdx.x != 0) return;
  const int m = *d_m;
  GridParams p;
  p.shift = shift;
  p.mask = mask;
  p.n = m;
  if (m <= 0) {
    p.ox = p.oy = p.oz = 0.0;
    p.c = 1.0;
    p.nx = p.ny = p.nz = 1;
    *gp = p;
    return;
  }
  double o[3], mx[3];
  for (int d = 0; d < 3; ++d) {
    o[d] = floor((double)ord2f(mm[d]));
    mx[d] = (double)ord2f(mm[3 + d]);
  }
  double c = 1.0;
  int n[3];
  for (;;) {
    for (int d = 0; d < 3; ++d) n[d] = (int)floor((mx[d] - o[d]) / c) + 1;
    if ((double)n[0] * (double)n[1] * (double)n[2] < 2147483000.0) break;
    c *= 2.0;
  }
  p.ox = o[0]; p.oy = o[1]; p.oz = o[2];
  p.c = c;
  p.nx = n[0]; p.ny = n[1]; p.nz = n[2];
  *gp = p;
}

__device__ __forceinline__ int cell_of(double v, double o, double inv_c, int n) {
  int c = (int)floor((v - o) * inv_c);
  return c < 0 ? 0 : (c >= n ? n - 1 : c);
}

__global__ __launch_bounds__(kTB) void grid_keys(const PointRec* __restrict__ map, const int* __restrict__ d_m, int m_ub,
                                                 const GridParams* __restrict__ gp, uint32_t* __restrict__ keys,
                                                 int* __restrict__ vals) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m_ub) return;
  uint32_t key = kEmpty;
  if (i < *d_m) {
    const GridParams p = *gp;
    const double inv = 1.0 / p.c;
    const float4 q = *reinterpret_cast<const float4*>(&map[i].x);
    const int cx = cell_of(q.x, p.ox, inv, p.nx), cy = cell_of(q.y, p.oy, inv, p.ny), cz = cell_of(q.z, p.oz, inv, p.nz);
    key = (uint32_t)cx + (uint32_t)p.nx * ((uint32_t)cy + (uint32_t)p.ny * (uint32_t)cz);
  }
  keys[i] = key;
  vals[i] = i;
}

__device__ __forceinline__ uint32_t hash_slot(uint32_t key, int shift) { return (key * 0x9E3779B1u) >> shift; }

__global__ __launch_bounds__(kTB) void grid_fill(const PointRec* __restrict__ map, const int* __restrict__ d_m,
                                                 const uint32_t* __restrict__ keys, const int* __restrict__ vals,
                                                 const GridParams* __restrict__ gp, float4* __restrict__ pts,
                                                 uint32_t* __restrict__ tkey, int2* __restrict__ tval) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int m = *d_m;
  if (i >= m) return;
  const int j = vals[i];
  const float4 q = *reinterpret_cast<const float4*>(&map[j].x);
  pts[i] = make_float4(q.x, q.y, q.z, __int_as_float(j));
  const uint32_t k = keys[i];
  if (i == 0 || keys[i - 1] != k) {
    int e = i + 1;
    while (e < m && keys[e] == k) ++e;
    const GridParams p = *gp;
    uint32_t h = hash_slot(k, p.shift);
    for (;;) {
      const uint32_t prev = atomicCAS(&tkey[h], kEmpty, k);
      if (prev == kEmpty) {
        tval[h] = make_int2(i, e - i);
        break;
      }
      h = (h + 1) & p.mask;
    }
  }
}

// ===================================================================================== geometry (fp64)
// Eigen 3.3 SelfAdjointEigenSolver<Matrix3d>::compute restated for the device (same algorithm and operation
// order as oracle/eigen_solvers.cpp: scaled lower triangle, closed-form 3x3 tridiagonalisation, implicit
// Wilkinson-shift QR with Givens rotations, ascending selection sort).
__device__ __forceinline__ double e_hypot(double x, double y) {
  const double ax = fabs(x), ay = fabs(y);
  double p, qp;
  if (ax > ay) { p = ax; qp = ay / p; } else { p = ay; qp = ax / p; }
  if (p == 0.0) return 0.0;
  return p * sqrt(1.0 + qp * qp);
}

__device__ void eig_sym3(const double A[3][3], double ev[3], double u_top[3]) {
  double mat[3][3];
  double scale = 0.0;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c <= r; ++c) {
      mat[r][c] = A[r][c];
      scale = fmax(scale, fabs(A[r][c]));
    }
  if (scale == 0.0) scale = 1.0;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c <= r; ++c) mat[r][c] /= scale;
  double diag[3], sub[2], Q[3][3];   // Q[col][row]
  diag[0] = mat[0][0];
  const double v1norm2 = mat[2][0] * mat[2][0];
  if (v1norm2 <= DBL_MIN) {
    diag[1] = mat[1][1];
    diag[2] = mat[2][2];
    sub[0] = mat[1][0];
    sub[1] = mat[2][1];
    for (int c = 0; c < 3; ++c)
      for (int r = 0; r < 3; ++r) Q[c][r] = (c == r) ? 1.0 : 0.0;
  } else {
    const double beta = sqrt(mat[1][0] * mat[1][0] + v1norm2);
    const double invBeta = 1.0 / beta;
    const double m01 = mat[1][0] * invBeta;
    const double m02 = mat[2][0] * invBeta;
    const double q = 2.0 * m01 * mat[2][1] + m02 * (mat[2][2] - mat[1][1]);
    diag[1] = mat[1][1] + m02 * q;
    diag[2] = mat[2][2] - m02 * q;
    sub[0] = beta;
    sub[1] = mat[2][1] - m01 * q;
    Q[0][0] = 1; Q[0][1] = 0; Q[0][2] = 0;
    Q[1][0] = 0; Q[1][1] = m01; Q[1][2] = m02;
    Q[2][0] = 0; Q[2][1] = m02; Q[2][2] = -m01;
  }
  const double precision = 2.0 * DBL_EPSILON;
  int end = 2, start = 0, iter = 0;
  while (end > 0) {
    for (int i = start; i < end; ++i)
      if (fabs(sub[i]) <= (fabs(diag[i]) + fabs(diag[i + 1])) * precision || fabs(sub[i]) <= DBL_MIN) sub[i] = 0.0;
    while (end > 0 && sub[end - 1] == 0.0) end--;
    if (end <= 0) break;
    if (++iter > 90) break;
    start = end - 1;
    while (start > 0 && sub[start - 1] != 0.0) start--;
    // tridiagonal_qr_step
    const double td = (diag[end - 1] - diag[end]) * 0.5;
    const double e = sub[end - 1];
    double mu = diag[end];
    if (td == 0.0) {
      mu -= fabs(e);
    } else {
      const double e2 = sub[end - 1] * sub[end - 1];
      const double h = e_hypot(td, e);
      if (e2 == 0.0) mu -= (e / (td + (td > 0.0 ? 1.0 : -1.0))) * (e / h);
      else mu -= e2 / (td + (td > 0.0 ? h : -h));
    }
    double x = diag[start] - mu;
    double z = sub[start];
    for (int k = start; k < end; ++k) {
      double c, s;
      if (z == 0.0) {
        c = x < 0.0 ? -1.0 : 1.0;
        s = 0.0;
      } else if (x == 0.0) {
        c = 0.0;
        s = z < 0.0 ? 1.0 : -1.0;
      } else if (fabs(x) > fabs(z)) {
        const double t = z / x;
        double uu = sqrt(1.0 + t * t);
        if (x < 0.0) uu = -uu;
        c = 1.0 / uu;
        s = -t * c;
      } else {
        const double t = x / z;
        double uu = sqrt(1.0 + t * t);
        if (z < 0.0) uu = -uu;
        s = -1.0 / uu;
        c = -t * s;
      }
      const double sdk = s * diag[k] + c * sub[k];
      const double dkp1 = s * sub[k] + c * diag[k + 1];
      diag[k] = c * (c * diag[k] - s * sub[k]) - s * (c * sub[k] - s * diag[k + 1]);
      diag[k + 1] = s * sdk + c * dkp1;
      sub[k] = c * sdk - s * dkp1;
      if (k > start) sub[k - 1] = c * sub[k - 1] - s * z;
      x = sub[k];
      if (k < end - 1) {
        z = -s * sub[k + 1];
        sub[k + 1] = c * sub[k + 1];
      }
      for (int i = 0; i < 3; ++i) {
        const double xi = Q[k][i], yi = Q[k + 1][i];
        Q[k][i] = c * xi - s * yi;
        Q[k + 1][i] = s * xi + c * yi;
      }
    }
  }
  for (int i = 0; i < 2; ++i) {
    int k = i;
    for (int j = i + 1; j < 3; ++j)
      if (diag[j] < diag[k]) k = j;
    if (k != i) {
      const double t = diag[i]; diag[i] = diag[k]; diag[k] = t;
      for (int r = 0; r < 3; ++r) { const double q = Q[i][r]; Q[i][r] = Q[k][r]; Q[k][r] = q; }
    }
  }
  for (int i = 0; i < 3; ++i) ev[i] = diag[i] * scale;
  u_top[0] = Q[2][0]; u_top[1] = Q[2][1]; u_top[2] = Q[2][2];
}

// Eigen 3.3 ColPivHouseholderQR<Matrix<double,5,3>>::solve(-1) restated for the device.
__device__ void householder(double* v, int len, double& tau, double& beta) {
  double tail = 0.0;
  for (int i = 1; i < len; ++i) tail += v[i] * v[i];
  const double c0 = v[0];
  if (tail <= DBL_MIN) {
    tau = 0.0;
    beta = c0;
    for (int i = 1; i < len; ++i) v[i] = 0.0;
  } else {
    beta = sqrt(c0 * c0 + tail);
    if (c0 >= 0.0) beta = -beta;
    for (int i = 1; i < len; ++i) v[i] = v[i] / (c0 - beta);
    tau = (beta - c0) / beta;
  }
}

__device__ void plane_solve(const double A[5][3], double x[3]) {
  double qr[3][5];
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 5; ++r) qr[c][r] = A[r][c];
  double hc[3], nu[3], nd[3];
  int tr[3], perm[3] = {0, 1, 2};
  for (int k = 0; k < 3; ++k) {
    double s = 0.0;
    for (int r = 0; r < 5; ++r) s += qr[k][r] * qr[k][r];
    nd[k] = sqrt(s);
    nu[k] = nd[k];
  }
  const double maxn = fmax(nu[0], fmax(nu[1], nu[2]));
  const double threshold_helper = (maxn * DBL_EPSILON) * (maxn * DBL_EPSILON) / 5;
  const double norm_downdate_threshold = sqrt(DBL_EPSILON);
  int nz = 3;
  for (int k = 0; k < 3; ++k) {
    int big = k;
    for (int j = k + 1; j < 3; ++j)
      if (nu[j] > nu[big]) big = j;
    if (nz == 3 && nu[big] * nu[big] < threshold_helper * (5 - k)) nz = k;
    tr[k] = big;
    if (k != big) {
      for (int r = 0; r < 5; ++r) { const double t = qr[k][r]; qr[k][r] = qr[big][r]; qr[big][r] = t; }
      double t = nu[k]; nu[k] = nu[big]; nu[big] = t;
      t = nd[k]; nd[k] = nd[big]; nd[big] = t;
    }
    double beta;
    householder(&qr[k][k], 5 - k, hc[k], beta);
    qr[k][k] = beta;
    if (hc[k] != 0.0) {
      for (int j = k + 1; j < 3; ++j) {
        double tmp = 0.0;
        for (int r = k + 1; r < 5; ++r) tmp += qr[k][r] * qr[j][r];
        tmp += qr[j][k];
        qr[j][k] -= hc[k] * tmp;
        for (int r = k + 1; r < 5; ++r) qr[j][r] -= hc[k] * qr[k][r] * tmp;
      }
    }
    for (int j = k + 1; j < 3; ++j) {
      if (nu[j] != 0.0) {
        double temp = fabs(qr[j][k]) / nu[j];
        temp = (1.0 + temp) * (1.0 - temp);
        temp = temp < 0.0 ? 0.0 : temp;
        const double ratio = nu[j] / nd[j];
        const double temp2 = temp * ratio * ratio;
        if (temp2 <= norm_downdate_threshold) {
          double s = 0.0;
          for (int r = k + 1; r < 5; ++r) s += qr[j][r] * qr[j][r];
          nd[j] = sqrt(s);
          nu[j] = nd[j];
        } else {
          nu[j] *= sqrt(temp);
        }
      }
    }
  }
  for (int k = 0; k < 3; ++k) {
    const int t = perm[k]; perm[k] = perm[tr[k]]; perm[tr[k]] = t;
  }
  x[0] = x[1] = x[2] = 0.0;
  if (nz == 0) return;
  double c[5] = {-1.0, -1.0, -1.0, -1.0, -1.0};
  for (int k = 0; k < nz; ++k) {
    if (hc[k] == 0.0) continue;
    double tmp = c[k];
    for (int r = k + 1; r < 5; ++r) tmp += qr[k][r] * c[r];
    c[k] -= hc[k] * tmp;
    for (int r = k + 1; r < 5; ++r) c[r] -= hc[k] * qr[k][r] * tmp;
  }
  for (int i = nz - 1; i >= 0; --i) {
    double s = c[i];
    for (int j = i + 1; j < nz; ++j) s -= qr[j][i] * c[j];
    c[i] = s / qr[i][i];
  }
  double out[3] = {0.0, 0.0, 0.0};
  for (int i = 0; i < nz; ++i) out[perm[i]] = c[i];
  x[0] = out[0]; x[1] = out[1]; x[2] = out[2];
}

// ===================================================================================== correspondence search
struct Top5 {
  float d[5];
  int i[5];     // map index (tie-break, = FLANN index order)
  int pos[5];   // position in the cell-sorted array (coordinates)
  int cnt;
};

__device__ __forceinline__ void top5_insert(Top5& t, float d, int idx, int pos) {
  // keep the 5 smallest (d, idx) in ascending order; ties broken by map index
  if (!(d < t.d[4] || (d == t.d[4] && idx < t.i[4]))) return;
  int k = 4;
  while (k > 0 && (d < t.d[k - 1] || (d == t.d[k - 1] && idx < t.i[k - 1]))) {
    t.d[k] = t.d[k - 1];
    t.i[k] = t.i[k - 1];
    t.pos[k] = t.pos[k - 1];
    --k;
  }
  t.d[k] = d;
  t.i[k] = idx;
  t.pos[k] = pos;
}

__device__ __forceinline__ int2 grid_lookup(const uint32_t* __restrict__ tkey, const int2* __restrict__ tval,
                                            uint32_t key, int shift, unsigned mask) {
  uint32_t h = hash_slot(key, shift);
  for (;;) {
    const uint32_t k = tkey[h];
    if (k == key) return tval[h];
    if (k == kEmpty) return make_int2(0, 0);
    h = (h + 1) & mask;
  }
}

// Exact fixed-radius 5-NN: every map point with float sqd < 1 (FLANN L2_Simple order: ((0+dx^2)+dy^2)+dz^2)
// is visited; the 5 smallest are kept.  valid <=> at least 5 such points  <=>  KD-tree sqd[4] < 1.
__device__ __forceinline__ void knn5(const GridParams& p, const float4* __restrict__ pts,
                                     const uint32_t* __restrict__ tkey, const int2* __restrict__ tval, float qx,
                                     float qy, float qz, Top5& t) {
  for (int k = 0; k < 5; ++k) { t.d[k] = FLT_MAX; t.i[k] = INT_MAX; t.pos[k] = 0; }
  t.cnt = 0;
  const double inv = 1.0 / p.c;
  // |p - q| < 1 along each axis => cell in [floor((q-o-1)/c), floor((q-o+1)/c)]  (exact: c is a power of two)
  const int x0 = max(0, (int)floor(((double)qx - p.ox - 1.0) * inv)), x1 = min(p.nx - 1, (int)floor(((double)qx - p.ox + 1.0) * inv));
  const int y0 = max(0, (int)floor(((double)qy - p.oy - 1.0) * inv)), y1 = min(p.ny - 1, (int)floor(((double)qy - p.oy + 1.0) * inv));
  const int z0 = max(0, (int)floor(((double)qz - p.oz - 1.0) * inv)), z1 = min(p.nz - 1, (int)floor(((double)qz - p.oz + 1.0) * inv));
  for (int cz = z0; cz <= z1; ++cz)
    for (int cy = y0; cy <= y1; ++cy)
      for (int cx = x0; cx <= x1; ++cx) {
        const uint32_t key = (uint32_t)cx + (uint32_t)p.nx * ((uint32_t)cy + (uint32_t)p.ny * (uint32_t)cz);
        const int2 se = grid_lookup(tkey, tval, key, p.shift, p.mask);
        for (int j = se.x; j < se.x + se.y; ++j) {
          const float4 m = pts[j];
          float dd = 0.0f;
          float df = qx - m.x;
          dd += df * df;
          df = qy - m.y;
          dd += df * df;
          df = qz - m.z;
          dd += df * df;
          if (dd < 1.0f) {
            t.cnt++;
            top5_insert(t, dd, __float_as_int(m.w), j);
          }
        }
      }
}

template <bool EDGE>
__global__ __launch_bounds__(kTB) void corr_kernel(LMState* __restrict__ st, const PointRec* __restrict__ q,
                                                   const int* __restrict__ d_n, int n_ub,
                                                   const GridParams* __restrict__ gp, const float4* __restrict__ gpts,
                                                   const uint32_t* __restrict__ tkey, const int2* __restrict__ tval,
                                                   const int* __restrict__ d_me, const int* __restrict__ d_ms,
                                                   double* __restrict__ rec, uint8_t* __restrict__ valid, int cap,
                                                   int rank, int world) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ub) return;
  const int n = *d_n;
  const int lo = (int)(((long long)n * rank) / world), hi = (int)(((long long)n * (rank + 1)) / world);
  bool ok = false;
  if (i >= lo && i < hi && *d_me > 10 && *d_ms > 50) {   // map-size gate (odomEstimationClass.cpp:77)
    const PointRec pr = q[i];
    float wx, wy, wz;
    associate_to_map(st->x, pr.x, pr.y, pr.z, wx, wy, wz);
    const GridParams p = *gp;
    Top5 t;
    knn5(p, gpts, tkey, tval, wx, wy, wz, t);
    if (t.cnt >= 5) {
      // the 5 neighbours in ascending distance order (Eigen::Vector3d of the map's float coordinates)
      double P[5][3];
      for (int j = 0; j < 5; ++j) {
        const float4 mp = gpts[t.pos[j]];
        P[j][0] = mp.x; P[j][1] = mp.y; P[j][2] = mp.z;
      }
      const double cpx = pr.x, cpy = pr.y, cpz = pr.z;
      if (EDGE) {
        // addEdgeCostFactor geometry (odomEstimationClass.cpp:156-189)
        double c[3] = {0.0, 0.0, 0.0};
        for (int j = 0; j < 5; ++j)
          for (int d = 0; d < 3; ++d) c[d] = c[d] + P[j][d];
        for (int d = 0; d < 3; ++d) c[d] = c[d] / 5.0;
        double cov[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
        for (int j = 0; j < 5; ++j) {
          const double z[3] = {P[j][0] - c[0], P[j][1] - c[1], P[j][2] - c[2]};
          for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) cov[a][b] = cov[a][b] + z[a] * z[b];
        }
        double ev[3], u[3];
        eig_sym3(cov, ev, u);
        if (ev[2] > 3 * ev[1]) {
          ok = true;
          rec[0 * cap + i] = cpx; rec[1 * cap + i] = cpy; rec[2 * cap + i] = cpz;
          rec[3 * cap + i] = 0.1 * u[0] + c[0]; rec[4 * cap + i] = 0.1 * u[1] + c[1]; rec[5 * cap + i] = 0.1 * u[2] + c[2];
          rec[6 * cap + i] = -0.1 * u[0] + c[0]; rec[7 * cap + i] = -0.1 * u[1] + c[1]; rec[8 * cap + i] = -0.1 * u[2] + c[2];
        }
      } else {
        // addSurfCostFactor geometry (odomEstimationClass.cpp:208-243)
        double nv[3];
        plane_solve(P, nv);
        const double z = nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2];
        const double d = 1 / sqrt(z);
        if (z > 0.0) {
          const double sz = sqrt(z);
          nv[0] = nv[0] / sz; nv[1] = nv[1] / sz; nv[2] = nv[2] / sz;
        }
        bool planeValid = true;
        for (int j = 0; j < 5; ++j)
          if (fabs(nv[0] * P[j][0] + nv[1] * P[j][1] + nv[2] * P[j][2] + d) > 0.2) { planeValid = false; break; }
        if (planeValid) {
          ok = true;
          rec[0 * cap + i] = cpx; rec[1 * cap + i] = cpy; rec[2 * cap + i] = cpz;
          rec[3 * cap + i] = nv[0]; rec[4 * cap + i] = nv[1]; rec[5 * cap + i] = nv[2];
          rec[6 * cap + i] = d;
        }
      }
    }
  }
  valid[i] = ok ? 1 : 0;
  const unsigned long long b = __ballot(ok);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(EDGE ? &st->corr_edge : &st->corr_surf, __popcll(b));
}

__global__ void lm_init(LMState* st) {
  if (threadIdx.x != 0) return;
  st->phase = 0;
  st->done = 0;
  st->iteration = 0;
  st->reuse = 0;
  st->invalid = 0;
  st->successful = 0;
  st->n_res = 0;
  st->corr_edge = 0;
  st->corr_surf = 0;
  st->radius = 1e4;
  st->dfac = 2.0;
}

// ===================================================================================== residuals + reduction
__device__ __forceinline__ void rot(const double* x, double vx, double vy, double vz, double& ox, double& oy, double& oz) {
  const double qx = x[0], qy = x[1], qz = x[2], qw = x[3];
  double ux = qy * vz - qz * vy, uy = qz * vx - qx * vz, uz = qx * vy - qy * vx;
  ux = ux + ux; uy = uy + uy; uz = uz + uz;
  const double ax = vx + qw * ux, ay = vy + qw * uy, az = vz + qw * uz;
  ox = ax + (qy * uz - qz * uy);
  oy = ay + (qz * ux - qx * uz);
  oz = az + (qx * uy - qy * ux);
}

// EdgeAnalyticCostFunction::Evaluate (src/lidarOptimization.cpp:12-43): J = -(nu/|nu|)^T [de]x [-[lp]x, I] / |de|
__device__ __forceinline__ double edge_residual(const double* x, const double* r9, double J[6]) {
  double lx, ly, lz;
  rot(x, r9[0], r9[1], r9[2], lx, ly, lz);
  lx = lx + x[4]; ly = ly + x[5]; lz = lz + x[6];
  const double pax = lx - r9[3], pay = ly - r9[4], paz = lz - r9[5];
  const double pbx = lx - r9[6], pby = ly - r9[7], pbz = lz - r9[8];
  const double nux = pay * pbz - paz * pby, nuy = paz * pbx - pax * pbz, nuz = pax * pby - pay * pbx;
  const double dex = r9[3] - r9[6], dey = r9[4] - r9[7], dez = r9[5] - r9[8];
  const double de_norm = sqrt(dex * dex + dey * dey + dez * dez);
  const double nn = sqrt(nux * nux + nuy * nuy + nuz * nuz);
  const double r = nn / de_norm;
  const double w0 = -nux / nn, w1 = -nuy / nn, w2 = -nuz / nn;
  // r1 = w * skew(de): skew(de) = [[0,-dz,dy],[dz,0,-dx],[-dy,dx,0]]
  const double r10 = w1 * dez + w2 * (-dey);
  const double r11 = w0 * (-dez) + w2 * dex;
  const double r12 = w0 * dey + w1 * (-dex);
  // dp = [-skew(lp), I]; -skew(lp) = [[0,lz,-ly],[-lz,0,lx],[ly,-lx,0]]
  J[0] = (r11 * (-lz) + r12 * ly) / de_norm;
  J[1] = (r10 * lz + r12 * (-lx)) / de_norm;
  J[2] = (r10 * (-ly) + r11 * lx) / de_norm;
  J[3] = r10 / de_norm;
  J[4] = r11 / de_norm;
  J[5] = r12 / de_norm;
  return r;
}

// SurfNormAnalyticCostFunction::Evaluate (src/lidarOptimization.cpp:51-74): J = n^T [-[pw]x, I]
__device__ __forceinline__ double surf_residual(const double* x, const double* r7, double J[6]) {
  double px, py, pz;
  rot(x, r7[0], r7[1], r7[2], px, py, pz);
  px = px + x[4]; py = py + x[5]; pz = pz + x[6];
  const double nx = r7[3], ny = r7[4], nz = r7[5];
  const double r = (nx * px + ny * py + nz * pz) + r7[6];
  J[0] = ny * (-pz) + nz * py;
  J[1] = nx * pz + nz * (-px);
  J[2] = nx * (-py) + ny * px;
  J[3] = nx;
  J[4] = ny;
  J[5] = nz;
  return r;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}

__global__ __launch_bounds__(kTB) void lm_eval(const LMState* __restrict__ st, const double* __restrict__ erec,
                                               const uint8_t* __restrict__ evalid, int ecap, int ne_ub,
                                               const double* __restrict__ srec, const uint8_t* __restrict__ svalid,
                                               int scap, int ns_ub, int huber, double* __restrict__ partials) {
  if (st->done) return;
  double x[7];
  const double* px = st->phase == 0 ? st->x : st->cand;
  for (int k = 0; k < 7; ++k) x[k] = px[k];
  double acc[LM_NSUM];
#pragma unroll
  for (int k = 0; k < LM_NSUM; ++k) acc[k] = 0.0;
  const int total = ne_ub + ns_ub;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    double J[6], r;
    if (idx < ne_ub) {
      if (!evalid[idx]) continue;
      double f[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) f[k] = erec[k * ecap + idx];
      r = edge_residual(x, f, J);
    } else {
      const int s = idx - ne_ub;
      if (!svalid[s]) continue;
      double f[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) f[k] = srec[k * scap + s];
      r = surf_residual(x, f, J);
    }
    const double sq = r * r;
    if (huber) {   // ceres::HuberLoss(0.1) + Corrector (rho'' <= 0: residual scaling sqrt(rho'))
      double rho0, rho1;
      if (sq > 0.01) {
        const double rr = sqrt(sq);
        rho0 = 2.0 * 0.1 * rr - 0.01;
        rho1 = fmax(DBL_MIN, 0.1 / rr);
      } else {
        rho0 = sq;
        rho1 = 1.0;
      }
      acc[0] += 0.5 * rho0;
      const double sr = sqrt(rho1);
      r *= sr;
#pragma unroll
      for (int k = 0; k < 6; ++k) J[k] *= sr;
    } else {
      acc[0] += 0.5 * sq;
    }
    int h = 1;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = a; b < 6; ++b) acc[h++] += J[a] * J[b];
#pragma unroll
    for (int a = 0; a < 6; ++a) acc[22 + a] += J[a] * r;
    acc[28] += 1.0;
  }
  __shared__ double red[LM_NSUM][kTB / 64];
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < LM_NSUM; ++k) {
    const double v = wave_sum(acc[k]);
    if ((threadIdx.x & 63) == 0) red[k][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < LM_NSUM) {
    double v = 0.0;
    for (int k = 0; k < kTB / 64; ++k) v += red[threadIdx.x][k];
    partials[threadIdx.x * gridDim.x + blockIdx.x] = v;
  }
}

__device__ void reduce_partials_block(const double* __restrict__ partials, int nblk, double* sums /* shared */) {
  double acc[LM_NSUM];
  for (int k = 0; k < LM_NSUM; ++k) acc[k] = 0.0;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x)
    for (int k = 0; k < LM_NSUM; ++k) acc[k] += partials[k * nblk + b];
  __shared__ double red[LM_NSUM][kTB / 64];
  const int w = threadIdx.x >> 6;
  for (int k = 0; k < LM_NSUM; ++k) {
    const double v = wave_sum(acc[k]);
    if ((threadIdx.x & 63) == 0) red[k][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < LM_NSUM) {
    double v = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) v += red[threadIdx.x][k];
    sums[threadIdx.x] = v;
  }
  __syncthreads();
}

// ===================================================================================== LM control (Ceres 1.13)
// PoseSE3Parameterization::Plus + getTransformFromSe3 (src/lidarOptimization.cpp:77-140)
__device__ void se3_plus(const double* x, const double* d, double* out) {
  const double wx = d[0], wy = d[1], wz = d[2];
  const double theta = sqrt(wx * wx + wy * wy + wz * wz);
  const double half = 0.5 * theta;
  const double real_factor = cos(half);
  double imag;
  if (theta < 1e-10) {
    const double t2 = theta * theta, t4 = t2 * t2;
    imag = 0.5 - 0.0208333 * t2 + 0.000260417 * t4;
  } else {
    imag = sin(half) / theta;
  }
  const double dq[4] = {imag * wx, imag * wy, imag * wz, real_factor};   // x, y, z, w
  double Jm[3][3];
  if (theta < 1e-10) {
    const double tx = 2 * dq[0], ty = 2 * dq[1], tz = 2 * dq[2];
    const double twx = tx * dq[3], twy = ty * dq[3], twz = tz * dq[3];
    const double txx = tx * dq[0], txy = ty * dq[0], txz = tz * dq[0];
    const double tyy = ty * dq[1], tyz = tz * dq[1], tzz = tz * dq[2];
    Jm[0][0] = 1 - (tyy + tzz); Jm[0][1] = txy - twz; Jm[0][2] = txz + twy;
    Jm[1][0] = txy + twz; Jm[1][1] = 1 - (txx + tzz); Jm[1][2] = tyz - twx;
    Jm[2][0] = txz - twy; Jm[2][1] = tyz + twx; Jm[2][2] = 1 - (txx + tyy);
  } else {
    const double O[3][3] = {{0, -wz, wy}, {wz, 0, -wx}, {-wy, wx, 0}};
    double O2[3][3];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) O2[i][j] = O[i][0] * O[0][j] + O[i][1] * O[1][j] + O[i][2] * O[2][j];
    const double c1 = (1 - cos(theta)) / (theta * theta);
    const double c2 = (theta - sin(theta)) / pow(theta, 3.0);
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Jm[i][j] = ((i == j) ? 1.0 : 0.0) + c1 * O[i][j] + c2 * O2[i][j];
  }
  const double dtx = Jm[0][0] * d[3] + Jm[0][1] * d[4] + Jm[0][2] * d[5];
  const double dty = Jm[1][0] * d[3] + Jm[1][1] * d[4] + Jm[1][2] * d[5];
  const double dtz = Jm[2][0] * d[3] + Jm[2][1] * d[4] + Jm[2][2] * d[5];
  // q+ = dq * q
  const double ax = dq[0], ay = dq[1], az = dq[2], aw = dq[3];
  const double bx = x[0], by = x[1], bz = x[2], bw = x[3];
  out[0] = aw * bx + ax * bw + ay * bz - az * by;
  out[1] = aw * by + ay * bw + az * bx - ax * bz;
  out[2] = aw * bz + az * bw + ax * by - ay * bx;
  out[3] = aw * bw - ax * bx - ay * by - az * bz;
  double tx, ty, tz;
  rot(dq, x[4], x[5], x[6], tx, ty, tz);
  out[4] = tx + dtx;
  out[5] = ty + dty;
  out[6] = tz + dtz;
}

__device__ double grad_max_norm(const double* x, const double* g) {
  double ng[6], pr[7];
  for (int k = 0; k < 6; ++k) ng[k] = -g[k];
  se3_plus(x, ng, pr);
  double m = 0.0;
  for (int i = 0; i < 7; ++i) m = fmax(m, fabs(x[i] - pr[i]));
  return m;
}

__device__ __forceinline__ int hidx(int a, int b) {   // upper-triangle row-major index, a <= b
  return a * 6 - a * (a - 1) / 2 + (b - a);
}

// LevenbergMarquardtStrategy::ComputeStep in normal-equation form on the Jacobi-scaled system:
// (Hs + diag(Hs)/radius) y = gs, step = -y; then TrustRegionMinimizer::ComputeTrustRegionStep's model cost change.
__device__ bool compute_step(LMState* s) {
  double Hs[6][6], gs[6];
  for (int a = 0; a < 6; ++a) {
    gs[a] = s->scale[a] * s->g[a];
    for (int b = 0; b < 6; ++b) {
      const int i = a <= b ? hidx(a, b) : hidx(b, a);
      Hs[a][b] = s->scale[a] * s->H[i] * s->scale[b];
    }
  }
  if (!s->reuse)
    for (int k = 0; k < 6; ++k) s->diag[k] = fmin(fmax(Hs[k][k], 1e-6), 1e32);
  s->reuse = 1;
  double A[6][6];
  for (int a = 0; a < 6; ++a)
    for (int b = 0; b < 6; ++b) A[a][b] = Hs[a][b] + (a == b ? s->diag[a] / s->radius : 0.0);
  // Cholesky A = L L^T
  double L[6][6];
  for (int j = 0; j < 6; ++j) {
    double d = A[j][j];
    for (int k = 0; k < j; ++k) d -= L[j][k] * L[j][k];
    if (!(d > 0.0)) return false;
    L[j][j] = sqrt(d);
    for (int i = j + 1; i < 6; ++i) {
      double v = A[i][j];
      for (int k = 0; k < j; ++k) v -= L[i][k] * L[j][k];
      L[i][j] = v / L[j][j];
    }
  }
  double y[6];
  for (int i = 0; i < 6; ++i) {
    double v = gs[i];
    for (int k = 0; k < i; ++k) v -= L[i][k] * y[k];
    y[i] = v / L[i][i];
  }
  for (int i = 5; i >= 0; --i) {
    double v = y[i];
    for (int k = i + 1; k < 6; ++k) v -= L[k][i] * y[k];
    y[i] = v / L[i][i];
  }
  double step[6];
  bool finite = true;
  for (int k = 0; k < 6; ++k) {
    step[k] = -y[k];
    finite = finite && isfinite(step[k]);
  }
  if (!finite) return false;
  double sg = 0.0, sHs = 0.0;
  for (int a = 0; a < 6; ++a) {
    sg += step[a] * gs[a];
    double hv = 0.0;
    for (int b = 0; b < 6; ++b) hv += Hs[a][b] * step[b];
    sHs += step[a] * hv;
  }
  const double mcc = -(sg + 0.5 * sHs);
  if (!(mcc > 0.0)) return false;
  s->mcc = mcc;
  double delta[6];
  for (int k = 0; k < 6; ++k) delta[k] = step[k] * s->scale[k];
  se3_plus(s->x, delta, s->cand);
  return true;
}

__device__ void next_step(LMState* s) {
  for (;;) {
    s->iteration++;
    if (compute_step(s)) {
      s->invalid = 0;
      return;   // candidate pending evaluation
    }
    // HandleInvalidStep -> StepIsInvalid -> StepRejected(0)
    if (++s->invalid >= 5) { s->done = 1; return; }
    s->radius /= s->dfac;
    s->dfac *= 2.0;
    s->reuse = 1;
    if (s->iteration >= 4 || s->radius < 1e-32) { s->done = 1; return; }
  }
}

__device__ double norm7(const double* a) {
  double v = 0.0;
  for (int i = 0; i < 7; ++i) v += a[i] * a[i];
  return sqrt(v);
}

__device__ void lm_logic(LMState* s, const double* sums) {
  if (s->phase == 0) {   // IterationZero
    s->n_res = (int)sums[28];
    if (s->n_res == 0) { s->done = 1; return; }   // no residual blocks: parameters untouched
    s->x_cost = sums[0];
    if (!isfinite(s->x_cost)) { s->done = 1; return; }
    for (int k = 0; k < 21; ++k) s->H[k] = sums[1 + k];
    for (int k = 0; k < 6; ++k) s->g[k] = sums[22 + k];
    s->initial_cost = s->x_cost;
    for (int k = 0; k < 6; ++k) s->scale[k] = 1.0 / (1.0 + sqrt(s->H[hidx(k, k)]));
    s->x_norm = norm7(s->x);
    s->gmax = grad_max_norm(s->x, s->g);
    s->radius = 1e4;
    s->dfac = 2.0;
    s->reuse = 0;
    s->invalid = 0;
    s->iteration = 0;
    s->phase = 1;
    if (s->gmax <= 1e-10) { s->done = 1; return; }
    next_step(s);
    return;
  }
  double cand_cost = sums[0];
  if (!isfinite(cand_cost)) cand_cost = DBL_MAX;
  // ParameterToleranceReached (candidate not applied)
  double sn = 0.0;
  for (int i = 0; i < 7; ++i) sn += (s->x[i] - s->cand[i]) * (s->x[i] - s->cand[i]);
  sn = sqrt(sn);
  if (sn <= 1e-8 * (s->x_norm + 1e-8)) { s->done = 1; return; }
  // FunctionToleranceReached
  if (fabs(s->x_cost - cand_cost) <= 1e-6 * s->x_cost) { s->done = 1; return; }
  const double rho = (s->x_cost - cand_cost) / s->mcc;
  bool success = false;
  if (rho > 1e-3) {
    for (int i = 0; i < 7; ++i) s->x[i] = s->cand[i];
    s->x_norm = norm7(s->x);
    s->x_cost = cand_cost;
    for (int k = 0; k < 21; ++k) s->H[k] = sums[1 + k];
    for (int k = 0; k < 6; ++k) s->g[k] = sums[22 + k];
    s->gmax = grad_max_norm(s->x, s->g);
    const double t = 2.0 * rho - 1.0;
    s->radius = fmin(1e16, s->radius / fmax(1.0 / 3.0, 1.0 - t * t * t));
    s->dfac = 2.0;
    s->reuse = 0;
    s->successful++;
    success = true;
  } else {
    s->radius /= s->dfac;
    s->dfac *= 2.0;
    s->reuse = 1;
  }
  if (s->iteration >= 4 || s->radius < 1e-32 || (success && s->gmax <= 1e-10)) { s->done = 1; return; }
  next_step(s);
}

__global__ __launch_bounds__(kTB) void lm_control(LMState* __restrict__ st, const double* __restrict__ partials, int nblk) {
  __shared__ double sums[LM_NSUM];
  if (st->done) return;
  if (nblk > 0) {
    reduce_partials_block(partials, nblk, sums);
  } else {
    if (threadIdx.x < LM_NSUM) sums[threadIdx.x] = partials[threadIdx.x];
    __syncthreads();
  }
  if (threadIdx.x == 0) lm_logic(st, sums);
}

__global__ __launch_bounds__(kTB) void lm_reduce(const double* __restrict__ partials, int nblk, double* __restrict__ out) {
  __shared__ double sums[LM_NSUM];
  reduce_partials_block(partials, nblk, sums);
  if (threadIdx.x < LM_NSUM) out[threadIdx.x] = sums[threadIdx.x];
}

}  // namespace

// ===================================================================================== launchers
void grid_build_launch(Grid& g, GridScratch& sc, const PointRec* map, const int* d_m, int m_ub, hipStream_t st) {
  g.params.reserve(1);
  sc.mm.reserve(8);
  const int ub = m_ub > 0 ? m_ub : 1;
  sc.s.reserve(ub);
  g.pts.reserve(ub);
  int tsize = 1024, shift = 32 - 10;
  while (tsize < 2 * ub) { tsize <<= 1; --shift; }
  g.tkey.reserve(tsize);
  g.tval.reserve(tsize);
  g.table_size = tsize;
  g.shift = shift;
  FLOAM_HIP(hipMemsetAsync(g.tkey.p, 0xFF, sizeof(uint32_t) * tsize, st));
  minmax_launch(map, d_m, ub, sc.mm.p, st);
  hipLaunchKernelGGL(grid_setup, dim3(1), dim3(64), 0, st, sc.mm.p, d_m, shift, (unsigned)(tsize - 1), g.params.p);
  FLOAM_LAUNCH_CHECK();
  const unsigned gb = div_up(ub, kTB);
  hipLaunchKernelGGL(grid_keys, dim3(gb), dim3(kTB), 0, st, map, d_m, ub, g.params.p, sc.s.k0.p, sc.s.v0.p);
  FLOAM_LAUNCH_CHECK();
  sort_pairs_u32(sc.s.temp.p, sc.s.temp_bytes, sc.s.k0.p, sc.s.k1.p, sc.s.v0.p, sc.s.v1.p, ub, 32, st);
  hipLaunchKernelGGL(grid_fill, dim3(gb), dim3(kTB), 0, st, map, d_m, sc.s.k1.p, sc.s.v1.p, g.params.p, g.pts.p,
                     g.tkey.p, g.tval.p);
  FLOAM_LAUNCH_CHECK();
}

void corr_launch(LMState* d_st, const QuerySet& qe, const Grid& ge, const int* d_me, const QuerySet& qs,
                 const Grid& gs, const int* d_ms, CorrSet& ce, CorrSet& cs, int rank, int world, hipStream_t st) {
  hipLaunchKernelGGL(lm_init, dim3(1), dim3(64), 0, st, d_st);
  FLOAM_LAUNCH_CHECK();
  ce.reserve(std::max(qe.n_ub, 1), EDGE_FIELDS);
  cs.reserve(std::max(qs.n_ub, 1), SURF_FIELDS);
  if (qe.n_ub > 0) {
    hipLaunchKernelGGL(corr_kernel<true>, dim3(div_up(qe.n_ub, kTB)), dim3(kTB), 0, st, d_st, qe.pts, qe.d_n,
                       qe.n_ub, ge.params.p, ge.pts.p, ge.tkey.p, ge.tval.p, d_me, d_ms, ce.rec.p,
                       ce.valid.p, ce.cap, rank, world);
    FLOAM_LAUNCH_CHECK();
  }
  if (qs.n_ub > 0) {
    hipLaunchKernelGGL(corr_kernel<false>, dim3(div_up(qs.n_ub, kTB)), dim3(kTB), 0, st, d_st, qs.pts, qs.d_n,
                       qs.n_ub, gs.params.p, gs.pts.p, gs.tkey.p, gs.tval.p, d_me, d_ms, cs.rec.p,
                       cs.valid.p, cs.cap, rank, world);
    FLOAM_LAUNCH_CHECK();
  }
}

int lm_eval_launch(const LMState* d_st, const CorrSet& ce, int ne_ub, const CorrSet& cs, int ns_ub, bool huber,
                   double* partials, hipStream_t st) {
  const int total = std::max(ne_ub + ns_ub, 1);
  const int nblk = (int)std::min<unsigned>(div_up(total, kTB), 512u);
  hipLaunchKernelGGL(lm_eval, dim3(nblk), dim3(kTB), 0, st, d_st, ce.rec.p, ce.valid.p, ce.cap, ne_ub, cs.rec.p,
                     cs.valid.p, cs.cap, ns_ub, huber ? 1 : 0, partials);
  FLOAM_LAUNCH_CHECK();
  return nblk;
}

void lm_control_launch(LMState* d_st, const double* partials, int nblk, hipStream_t st) {
  hipLaunchKernelGGL(lm_control, dim3(1), dim3(kTB), 0, st, d_st, partials, nblk);
  FLOAM_LAUNCH_CHECK();
}

void lm_reduce_launch(const double* partials, int nblk, double* sums, hipStream_t st) {
  hipLaunchKernelGGL(lm_reduce, dim3(1), dim3(kTB), 0, st, partials, nblk, sums);
  FLOAM_LAUNCH_CHECK();
}

}  // namespace floam
