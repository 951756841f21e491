// CPU ORACLE (test infrastructure) — Eigen 3.3 dense solvers used on the path, restated.
// Call sites: SelfAdjointEigenSolver<Matrix3d> src/odomEstimationClass.cpp:175; colPivHouseholderQr().solve
// :220; Ceres DENSE_QR (HouseholderQR) :101.  Parity unpinned (see oracle.hpp).
#include <algorithm>
#include <cmath>
#include <limits>

#include "la.hpp"

namespace oracle {

namespace {
struct Givens {
  double c, s;
};
// JacobiRotation<double>::makeGivens (real case)
Givens make_givens(double p, double q) {
  Givens g;
  if (q == 0) {
    g.c = p < 0 ? -1.0 : 1.0;
    g.s = 0;
  } else if (p == 0) {
    g.c = 0;
    g.s = q < 0 ? 1.0 : -1.0;
  } else if (std::fabs(p) > std::fabs(q)) {
    const double t = q / p;
    double u = std::sqrt(1.0 + t * t);
    if (p < 0) u = -u;
    g.c = 1.0 / u;
    g.s = -t * g.c;
  } else {
    const double t = p / q;
    double u = std::sqrt(1.0 + t * t);
    if (q < 0) u = -u;
    g.s = -1.0 / u;
    g.c = -t * g.s;
  }
  return g;
}

// internal::tridiagonal_qr_step (column-major Q, n = 3)
void tridiagonal_qr_step(double* diag, double* subdiag, int start, int end, double Q[3][3]) {
  const double td = (diag[end - 1] - diag[end]) * 0.5;
  const double e = subdiag[end - 1];
  double mu = diag[end];
  if (td == 0) {
    mu -= std::fabs(e);
  } else {
    const double e2 = subdiag[end - 1] * subdiag[end - 1];
    const double h = e_hypot(td, e);
    if (e2 == 0)
      mu -= (e / (td + (td > 0 ? 1.0 : -1.0))) * (e / h);
    else
      mu -= e2 / (td + (td > 0 ? h : -h));
  }
  double x = diag[start] - mu;
  double z = subdiag[start];
  for (int k = start; k < end; ++k) {
    const Givens rot = make_givens(x, z);
    const double sdk = rot.s * diag[k] + rot.c * subdiag[k];
    const double dkp1 = rot.s * subdiag[k] + rot.c * diag[k + 1];
    diag[k] = rot.c * (rot.c * diag[k] - rot.s * subdiag[k]) - rot.s * (rot.c * subdiag[k] - rot.s * diag[k + 1]);
    diag[k + 1] = rot.s * sdk + rot.c * dkp1;
    subdiag[k] = rot.c * sdk - rot.s * dkp1;
    if (k > start) subdiag[k - 1] = rot.c * subdiag[k - 1] - rot.s * z;
    x = subdiag[k];
    if (k < end - 1) {
      z = -rot.s * subdiag[k + 1];
      subdiag[k + 1] = rot.c * subdiag[k + 1];
    }
    // Q = Q * G : applyOnTheRight(k, k+1, rot) -> x' = c x - s y, y' = s x + c y over columns k, k+1
    for (int i = 0; i < 3; ++i) {
      const double xi = Q[k][i], yi = Q[k + 1][i];
      Q[k][i] = rot.c * xi - rot.s * yi;
      Q[k + 1][i] = rot.s * xi + rot.c * yi;
    }
  }
}
}  // namespace

void eig_sym3(const M3& A, double eval[3], double evec[3][3]) {
  // mat = lower triangle of A, scaled to [-1, 1]
  double mat[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};   // row-major mat[r][c], lower part used
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c <= r; ++c) mat[r][c] = A.m[r][c];
  double scale = 0;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c <= r; ++c) scale = std::max(scale, std::fabs(mat[r][c]));
  if (scale == 0) scale = 1;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c <= r; ++c) mat[r][c] /= scale;
  // tridiagonalization_inplace_selector<MatrixType,3,false>
  double diag[3], sub[2];
  double Q[3][3];   // column-major Q[col][row]
  const double tol = std::numeric_limits<double>::min();
  diag[0] = mat[0][0];
  const double v1norm2 = mat[2][0] * mat[2][0];
  if (v1norm2 <= tol) {
    diag[1] = mat[1][1];
    diag[2] = mat[2][2];
    sub[0] = mat[1][0];
    sub[1] = mat[2][1];
    for (int c = 0; c < 3; ++c)
      for (int r = 0; r < 3; ++r) Q[c][r] = (c == r);
  } else {
    const double beta = std::sqrt(mat[1][0] * mat[1][0] + v1norm2);
    const double invBeta = 1.0 / beta;
    const double m01 = mat[1][0] * invBeta;
    const double m02 = mat[2][0] * invBeta;
    const double q = 2.0 * m01 * mat[2][1] + m02 * (mat[2][2] - mat[1][1]);
    diag[1] = mat[1][1] + m02 * q;
    diag[2] = mat[2][2] - m02 * q;
    sub[0] = beta;
    sub[1] = mat[2][1] - m01 * q;
    // mat << 1,0,0, 0,m01,m02, 0,m02,-m01  (row-major listing) -> column-major storage
    const double rm[3][3] = {{1, 0, 0}, {0, m01, m02}, {0, m02, -m01}};
    for (int c = 0; c < 3; ++c)
      for (int r = 0; r < 3; ++r) Q[c][r] = rm[r][c];
  }
  // computeFromTridiagonal_impl
  const int n = 3;
  int end = n - 1, start = 0, iter = 0;
  const double considerAsZero = std::numeric_limits<double>::min();
  const double precision = 2.0 * std::numeric_limits<double>::epsilon();
  const int maxIterations = 30;
  while (end > 0) {
    for (int i = start; i < end; ++i)
      if (std::fabs(sub[i]) <= (std::fabs(diag[i]) + std::fabs(diag[i + 1])) * precision ||
          std::fabs(sub[i]) <= considerAsZero)
        sub[i] = 0;
    while (end > 0 && sub[end - 1] == 0) end--;
    if (end <= 0) break;
    iter++;
    if (iter > maxIterations * n) break;
    start = end - 1;
    while (start > 0 && sub[start - 1] != 0) start--;
    tridiagonal_qr_step(diag, sub, start, end, Q);
  }
  // sort ascending (selection by minCoeff, first minimum)
  for (int i = 0; i < n - 1; ++i) {
    int k = i;
    for (int j = i + 1; j < n; ++j)
      if (diag[j] < diag[k]) k = j;
    if (k != i) {
      std::swap(diag[i], diag[k]);
      for (int r = 0; r < 3; ++r) std::swap(Q[i][r], Q[k][r]);
    }
  }
  for (int i = 0; i < 3; ++i) {
    eval[i] = diag[i] * scale;
    for (int r = 0; r < 3; ++r) evec[i][r] = Q[i][r];
  }
}

namespace {
// MatrixBase::makeHouseholder on v[0..len): returns tau, beta; essential part written to v[1..]
void make_householder(double* v, int len, int stride, double& tau, double& beta) {
  double tailSqNorm = 0;
  for (int i = 1; i < len; ++i) tailSqNorm += v[i * stride] * v[i * stride];
  const double c0 = v[0];
  const double tol = std::numeric_limits<double>::min();
  if (tailSqNorm <= tol) {
    tau = 0;
    beta = c0;
    for (int i = 1; i < len; ++i) v[i * stride] = 0;
  } else {
    beta = std::sqrt(c0 * c0 + tailSqNorm);
    if (c0 >= 0) beta = -beta;
    for (int i = 1; i < len; ++i) v[i * stride] = v[i * stride] / (c0 - beta);
    tau = (beta - c0) / beta;
  }
}
}  // namespace

void colpiv_qr_solve_5x3(const double A[5][3], const double b[5], double x[3]) {
  const int rows = 5, cols = 3, size = 3;
  double qr[3][5];                       // column-major qr[col][row]
  for (int c = 0; c < cols; ++c)
    for (int r = 0; r < rows; ++r) qr[c][r] = A[r][c];
  double hc[3];
  int transp[3];
  double normsUpd[3], normsDir[3];
  int perm[3] = {0, 1, 2};
  for (int k = 0; k < cols; ++k) {
    double s = 0;
    for (int r = 0; r < rows; ++r) s += qr[k][r] * qr[k][r];
    normsDir[k] = std::sqrt(s);
    normsUpd[k] = normsDir[k];
  }
  double maxn = std::max(normsUpd[0], std::max(normsUpd[1], normsUpd[2]));
  const double eps = std::numeric_limits<double>::epsilon();
  const double threshold_helper = (maxn * eps) * (maxn * eps) / rows;
  const double norm_downdate_threshold = std::sqrt(eps);
  int nonzero_pivots = size;
  for (int k = 0; k < size; ++k) {
    int big = k;
    for (int j = k + 1; j < cols; ++j)
      if (normsUpd[j] > normsUpd[big]) big = j;
    const double big_sq = normsUpd[big] * normsUpd[big];
    if (nonzero_pivots == size && big_sq < threshold_helper * (rows - k)) nonzero_pivots = k;
    transp[k] = big;
    if (k != big) {
      for (int r = 0; r < rows; ++r) std::swap(qr[k][r], qr[big][r]);
      std::swap(normsUpd[k], normsUpd[big]);
      std::swap(normsDir[k], normsDir[big]);
    }
    double beta;
    make_householder(&qr[k][k], rows - k, 1, hc[k], beta);
    qr[k][k] = beta;
    // applyHouseholderOnTheLeft to bottomRightCorner(rows-k, cols-k-1) with essential qr[k][k+1..]
    if (hc[k] != 0) {
      for (int j = k + 1; j < cols; ++j) {
        double tmp = 0;
        for (int r = k + 1; r < rows; ++r) tmp += qr[k][r] * qr[j][r];
        tmp += qr[j][k];
        qr[j][k] -= hc[k] * tmp;
        for (int r = k + 1; r < rows; ++r) qr[j][r] -= hc[k] * qr[k][r] * tmp;
      }
    }
    for (int j = k + 1; j < cols; ++j) {
      if (normsUpd[j] != 0) {
        double temp = std::fabs(qr[j][k]) / normsUpd[j];
        temp = (1.0 + temp) * (1.0 - temp);
        temp = temp < 0 ? 0 : temp;
        const double ratio = normsUpd[j] / normsDir[j];
        const double temp2 = temp * ratio * ratio;
        if (temp2 <= norm_downdate_threshold) {
          double s = 0;
          for (int r = k + 1; r < rows; ++r) s += qr[j][r] * qr[j][r];
          normsDir[j] = std::sqrt(s);
          normsUpd[j] = normsDir[j];
        } else {
          normsUpd[j] *= std::sqrt(temp);
        }
      }
    }
  }
  for (int k = 0; k < size; ++k) std::swap(perm[k], perm[transp[k]]);
  if (nonzero_pivots == 0) {
    x[0] = x[1] = x[2] = 0;
    return;
  }
  double c[5];
  for (int r = 0; r < rows; ++r) c[r] = b[r];
  // apply H_0 ... H_{np-1} (transpose of the householder sequence) to c
  for (int k = 0; k < nonzero_pivots; ++k) {
    if (hc[k] == 0) continue;
    double tmp = c[k];
    for (int r = k + 1; r < rows; ++r) tmp += qr[k][r] * c[r];
    c[k] -= hc[k] * tmp;
    for (int r = k + 1; r < rows; ++r) c[r] -= hc[k] * qr[k][r] * tmp;
  }
  // back substitution with the upper triangle
  for (int i = nonzero_pivots - 1; i >= 0; --i) {
    double s = c[i];
    for (int j = i + 1; j < nonzero_pivots; ++j) s -= qr[j][i] * c[j];
    c[i] = s / qr[i][i];
  }
  double out[3] = {0, 0, 0};
  for (int i = 0; i < nonzero_pivots; ++i) out[perm[i]] = c[i];
  x[0] = out[0]; x[1] = out[1]; x[2] = out[2];
}

void householder_qr_solve(std::vector<double>& A, int m, int n, const std::vector<double>& b, double* x) {
  // householder_qr_inplace_unblocked (n <= 48: a single block)
  std::vector<double> hc(n);
  for (int k = 0; k < n; ++k) {
    double* col = &A[(size_t)k * m];
    double beta;
    make_householder(col + k, m - k, 1, hc[k], beta);
    col[k] = beta;
    if (hc[k] != 0) {
      for (int j = k + 1; j < n; ++j) {
        double* cj = &A[(size_t)j * m];
        double tmp = 0;
        for (int r = k + 1; r < m; ++r) tmp += col[r] * cj[r];
        tmp += cj[k];
        cj[k] -= hc[k] * tmp;
        for (int r = k + 1; r < m; ++r) cj[r] -= hc[k] * col[r] * tmp;
      }
    }
  }
  std::vector<double> c(b);
  for (int k = 0; k < n; ++k) {
    if (hc[k] == 0) continue;
    const double* col = &A[(size_t)k * m];
    double tmp = c[k];
    for (int r = k + 1; r < m; ++r) tmp += col[r] * c[r];
    c[k] -= hc[k] * tmp;
    for (int r = k + 1; r < m; ++r) c[r] -= hc[k] * col[r] * tmp;
  }
  for (int i = n - 1; i >= 0; --i) {
    double s = c[i];
    for (int j = i + 1; j < n; ++j) s -= A[(size_t)j * m + i] * c[j];
    c[i] = s / A[(size_t)i * m + i];
  }
  for (int i = 0; i < n; ++i) x[i] = c[i];
}

}  // namespace oracle
