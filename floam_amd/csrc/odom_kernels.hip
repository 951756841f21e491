// Scan-to-map correspondences on gfx950: spatial-hash kNN correspondence search + line / plane geometry (fp64, or
// fp32 for the C5 precision sweep) + the device-resident odometry controller (prediction, deskew bridge, status
// gather, KeyFrameUpdate).  The LM solve itself is lm.hip.
//
// Reference: src/odomEstimationClass.cpp:78-79 (kd-tree), :126-135 (pointAssociateToMap), :144-196
// (addEdgeCostFactor), :198-251 (addSurfCostFactor), :57-124 (updatePointsToMap control), :320-343 (KeyFrameUpdate).
#include <cfloat>
#include <chrono>
#include <cstring>
#include <thread>
#include <cstdlib>
#include <climits>

#include <hip/hip_ext.h>

#include "grid.hpp"
#include "lm_eval.hpp"
#include "odom_kernels.hpp"

namespace floam {

namespace {
constexpr int kTB = 256;

// ===================================================================================== geometry (R = double | float)
// Eigen 3.3 SelfAdjointEigenSolver<Matrix3d>::compute and ColPivHouseholderQR<Matrix<double,5,3>>::solve restated
// for the device with the same algorithm and operation order as oracle/eigen_solvers.cpp.  Every array index is a
// compile-time constant (templates / full unrolling) so the solvers stay in VGPRs instead of scratch.  R = double is
// the reference's precision; R = float is the C5 sweep's fp32 variant (the same algorithm with float's epsilon/min).
template <typename R>
struct Lim {
  static __device__ __forceinline__ R eps() { return DBL_EPSILON; }
  static __device__ __forceinline__ R min() { return DBL_MIN; }
};
template <>
struct Lim<float> {
  static __device__ __forceinline__ float eps() { return FLT_EPSILON; }
  static __device__ __forceinline__ float min() { return FLT_MIN; }
};

template <typename R>
__device__ __forceinline__ R e_hypot(R x, R y) {
  const R ax = fabs(x), ay = fabs(y);
  const bool xb = ax > ay;   // (one division for both orders: lanes of a wave may take either)
  const R p = xb ? ax : ay, qp = (xb ? ay : ax) / p;
  if (p == R(0)) return R(0);
  return p * sqrt(R(1) + qp * qp);
}

// JacobiRotation<double>::makeGivens (real case)
template <typename R>
__device__ __forceinline__ void make_givens(R p, R q, R& c, R& s) {
  if (q == R(0)) {
    c = p < R(0) ? R(-1) : R(1);
    s = R(0);
  } else if (p == R(0)) {
    c = R(0);
    s = q < R(0) ? R(1) : R(-1);
  } else {   // |p| > |q|: t = q / p, c = 1 / u, s = -t c; else t = p / q, s = -1 / u, c = -t s (one division, one
    // square root and one reciprocal for both cases: lanes of a wave may take either)
    const bool pb = fabs(p) > fabs(q);
    const R t = (pb ? q : p) / (pb ? p : q);
    R u = sqrt(R(1) + t * t);
    if ((pb ? p : q) < R(0)) u = -u;
    const R r = (pb ? R(1) : R(-1)) / u;
    c = pb ? r : -t * r;
    s = pb ? -t * r : r;
  }
}

// internal::tridiagonal_qr_step on rows/cols [S, E] of a 3x3 tridiagonal (Q column-major: Q[col][row])
template <int S, int E, typename R>
__device__ __forceinline__ void tridiag_qr_step(R (&d)[3], R (&e)[2], R (&Q)[3][3]) {
  const R td = (d[E - 1] - d[E]) * R(0.5);
  const R ee = e[E - 1];
  R mu = d[E];
  if (td == R(0)) {
    mu -= fabs(ee);
  } else {
    const R e2 = e[E - 1] * e[E - 1];
    const R h = e_hypot(td, ee);
    if (e2 == R(0)) mu -= (ee / (td + (td > R(0) ? R(1) : R(-1)))) * (ee / h);
    else mu -= e2 / (td + (td > R(0) ? h : -h));
  }
  R x = d[S] - mu;
  R z = e[S];
#pragma unroll
  for (int k = S; k < E; ++k) {
    R c, s;
    make_givens(x, z, c, s);
    const R sdk = s * d[k] + c * e[k];
    const R dkp1 = s * e[k] + c * d[k + 1];
    d[k] = c * (c * d[k] - s * e[k]) - s * (c * e[k] - s * d[k + 1]);
    d[k + 1] = s * sdk + c * dkp1;
    e[k] = c * sdk - s * dkp1;
    if (k > S) e[k - 1] = c * e[k - 1] - s * z;
    x = e[k];
    if (k < E - 1) {
      z = -s * e[k + 1];
      e[k + 1] = c * e[k + 1];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const R xi = Q[k][i], yi = Q[k + 1][i];
      Q[k][i] = c * xi - s * yi;
      Q[k + 1][i] = s * xi + c * yi;
    }
  }
}

// The three variants above as ONE instruction stream: lanes of a wave whose matrices need different variants
// (<0, 2>, <1, 2>, <0, 1> by their deflation state) would otherwise run all three bodies one after the other every
// iteration.  Operands are selected, not recomputed: every value is the same expression of the same inputs as in
// the variant the lane needs (bit-identical); the second rotation of <0, 2> runs only when a lane needs it.
template <typename R>
__device__ __forceinline__ void tridiag_qr_step_any(R (&d)[3], R (&e)[2], R (&Q)[3][3], int end, int start) {
  const bool two = end == 2 && start == 0;   // <0, 2>
  const bool hi = end == 2 && start == 1;    // <1, 2>: the rotation acts on rows 1..2 (else rows 0..1)
  const bool lo_tail = end == 1;             // <0, 1>: the shift from rows 0..1 (else rows 1..2)
  const R t0 = lo_tail ? d[0] : d[1], t1 = lo_tail ? d[1] : d[2], ee = lo_tail ? e[0] : e[1];
  const R td = (t0 - t1) * R(0.5);
  R mu = t1;
  if (td == R(0)) {
    mu -= fabs(ee);
  } else {
    const R e2 = ee * ee;
    const R h = e_hypot(td, ee);
    if (e2 == R(0)) mu -= (ee / (td + (td > R(0) ? R(1) : R(-1)))) * (ee / h);
    else mu -= e2 / (td + (td > R(0) ? h : -h));
  }
  // rotation k = S on rows (a, b) = (d[S], d[S + 1]), off-diagonal ek = e[S]
  const R a = hi ? d[1] : d[0], b = hi ? d[2] : d[1], ek = hi ? e[1] : e[0];
  R c, s;
  make_givens(a - mu, ek, c, s);
  const R sdk = s * a + c * ek;
  const R dkp1 = s * ek + c * b;
  const R na = c * (c * a - s * ek) - s * (c * ek - s * b);
  const R nb = s * sdk + c * dkp1;
  const R nek = c * sdk - s * dkp1;
  if (hi) { d[1] = na; d[2] = nb; e[1] = nek; } else { d[0] = na; d[1] = nb; e[0] = nek; }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const R xi = hi ? Q[1][i] : Q[0][i], yi = hi ? Q[2][i] : Q[1][i];
    const R qa = c * xi - s * yi, qb = s * xi + c * yi;
    if (hi) { Q[1][i] = qa; Q[2][i] = qb; } else { Q[0][i] = qa; Q[1][i] = qb; }
  }
  if (two) {   // <0, 2>: the bulge chased to rows 1..2
    const R z = -s * e[1];
    e[1] = c * e[1];
    R c2, s2;
    make_givens(e[0], z, c2, s2);
    const R sdk2 = s2 * d[1] + c2 * e[1];
    const R dkp12 = s2 * e[1] + c2 * d[2];
    d[1] = c2 * (c2 * d[1] - s2 * e[1]) - s2 * (c2 * e[1] - s2 * d[2]);
    d[2] = s2 * sdk2 + c2 * dkp12;
    e[1] = c2 * sdk2 - s2 * dkp12;
    e[0] = c2 * e[0] - s2 * z;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const R xi = Q[1][i], yi = Q[2][i];
      Q[1][i] = c2 * xi - s2 * yi;
      Q[2][i] = s2 * xi + c2 * yi;
    }
  }
}

template <typename R>
__device__ __forceinline__ void swap_r(R& a, R& b) {
  const R t = a;
  a = b;
  b = t;
}

// eigenvalues ascending in ev; u_top = eigenvector of the largest eigenvalue
template <typename R>
__device__ void eig_sym3(const R (&A)[3][3], R (&ev)[3], R (&u_top)[3]) {
  R m00 = A[0][0], m10 = A[1][0], m11 = A[1][1], m20 = A[2][0], m21 = A[2][1], m22 = A[2][2];
  R scale = fabs(m00);
  scale = fmax(scale, fabs(m10));
  scale = fmax(scale, fabs(m11));
  scale = fmax(scale, fabs(m20));
  scale = fmax(scale, fabs(m21));
  scale = fmax(scale, fabs(m22));
  if (scale == R(0)) scale = R(1);
  m00 /= scale; m10 /= scale; m11 /= scale; m20 /= scale; m21 /= scale; m22 /= scale;
  R d[3], e[2], Q[3][3];
  d[0] = m00;
  const R v1norm2 = m20 * m20;
  if (v1norm2 <= Lim<R>::min()) {
    d[1] = m11; d[2] = m22; e[0] = m10; e[1] = m21;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int r = 0; r < 3; ++r) Q[c][r] = (c == r) ? R(1) : R(0);
  } else {
    const R beta = sqrt(m10 * m10 + v1norm2);
    const R invBeta = R(1) / beta;
    const R m01 = m10 * invBeta;
    const R m02 = m20 * invBeta;
    const R q = R(2) * m01 * m21 + m02 * (m22 - m11);
    d[1] = m11 + m02 * q;
    d[2] = m22 - m02 * q;
    e[0] = beta;
    e[1] = m21 - m01 * q;
    Q[0][0] = 1; Q[0][1] = 0; Q[0][2] = 0;
    Q[1][0] = 0; Q[1][1] = m01; Q[1][2] = m02;
    Q[2][0] = 0; Q[2][1] = m02; Q[2][2] = -m01;
  }
  const R precision = R(2) * Lim<R>::eps();
  int end = 2, start = 0, iter = 0;
  while (end > 0) {
    if (start <= 0 && 0 < end)
      if (fabs(e[0]) <= (fabs(d[0]) + fabs(d[1])) * precision || fabs(e[0]) <= Lim<R>::min()) e[0] = R(0);
    if (start <= 1 && 1 < end)
      if (fabs(e[1]) <= (fabs(d[1]) + fabs(d[2])) * precision || fabs(e[1]) <= Lim<R>::min()) e[1] = R(0);
    if (end == 2 && e[1] == R(0)) end = 1;
    if (end == 1 && e[0] == R(0)) end = 0;
    if (end <= 0) break;
    if (++iter > 90) break;
    start = (end == 2 && e[0] != R(0)) ? 0 : end - 1;
#ifdef FLOAM_EIG_VARIANTS   // (A/B and bit-identity checks: the three variants as separate bodies)
    if (end == 2) {
      if (start == 0) tridiag_qr_step<0, 2>(d, e, Q);
      else tridiag_qr_step<1, 2>(d, e, Q);
    } else {
      tridiag_qr_step<0, 1>(d, e, Q);
    }
#else
    tridiag_qr_step_any(d, e, Q, end, start);
#endif
  }
  // ascending selection sort (first minimum), swapping eigenvector columns
  int k = 0;
  if (d[1] < d[k]) k = 1;
  if (d[2] < d[k]) k = 2;
  if (k == 1) {
    swap_r(d[0], d[1]);
#pragma unroll
    for (int r = 0; r < 3; ++r) swap_r(Q[0][r], Q[1][r]);
  } else if (k == 2) {
    swap_r(d[0], d[2]);
#pragma unroll
    for (int r = 0; r < 3; ++r) swap_r(Q[0][r], Q[2][r]);
  }
  if (d[2] < d[1]) {
    swap_r(d[1], d[2]);
#pragma unroll
    for (int r = 0; r < 3; ++r) swap_r(Q[1][r], Q[2][r]);
  }
  ev[0] = d[0] * scale; ev[1] = d[1] * scale; ev[2] = d[2] * scale;
  u_top[0] = Q[2][0]; u_top[1] = Q[2][1]; u_top[2] = Q[2][2];
}

// Householder on column K of a column-major 5x3 (qr[col][row]): makeHouseholderInPlace + apply to columns > K
template <int K, typename R>
__device__ __forceinline__ void plane_hh(R (&qr)[3][5], R (&hc)[3]) {
  R tail = R(0);
#pragma unroll
  for (int i = K + 1; i < 5; ++i) tail += qr[K][i] * qr[K][i];
  const R c0 = qr[K][K];
  R tau, beta;
  if (tail <= Lim<R>::min()) {
    tau = R(0);
    beta = c0;
#pragma unroll
    for (int i = K + 1; i < 5; ++i) qr[K][i] = R(0);
  } else {
    beta = sqrt(c0 * c0 + tail);
    if (c0 >= R(0)) beta = -beta;
#pragma unroll
    for (int i = K + 1; i < 5; ++i) qr[K][i] = qr[K][i] / (c0 - beta);
    tau = (beta - c0) / beta;
  }
  hc[K] = tau;
  qr[K][K] = beta;
  if (tau != R(0)) {
#pragma unroll
    for (int j = K + 1; j < 3; ++j) {
      R tmp = R(0);
#pragma unroll
      for (int r = K + 1; r < 5; ++r) tmp += qr[K][r] * qr[j][r];
      tmp += qr[j][K];
      qr[j][K] -= tau * tmp;
#pragma unroll
      for (int r = K + 1; r < 5; ++r) qr[j][r] -= tau * qr[K][r] * tmp;
    }
  }
}

template <int K, typename R>
__device__ __forceinline__ void plane_pivot_step(R (&qr)[3][5], R (&hc)[3], R (&nu)[3], R (&nd)[3], int (&tr)[3],
                                                 int& nz, R threshold_helper) {
  int big = K;
#pragma unroll
  for (int j = K + 1; j < 3; ++j)
    if (nu[j] > nu[big == 0 ? 0 : (big == 1 ? 1 : 2)]) big = j;
  R nb = nu[K];
#pragma unroll
  for (int j = K + 1; j < 3; ++j)
    if (big == j) nb = nu[j];
  if (nz == 3 && nb * nb < threshold_helper * R(5 - K)) nz = K;
  tr[K] = big;
#pragma unroll
  for (int j = K + 1; j < 3; ++j) {
    if (big == j) {
#pragma unroll
      for (int r = 0; r < 5; ++r) swap_r(qr[K][r], qr[j][r]);
      swap_r(nu[K], nu[j]);
      swap_r(nd[K], nd[j]);
    }
  }
  plane_hh<K>(qr, hc);
  const R nrm_thr = sqrt(Lim<R>::eps());
#pragma unroll
  for (int j = K + 1; j < 3; ++j) {
    if (nu[j] != R(0)) {
      R temp = fabs(qr[j][K]) / nu[j];
      temp = (R(1) + temp) * (R(1) - temp);
      temp = temp < R(0) ? R(0) : temp;
      const R ratio = nu[j] / nd[j];
      const R temp2 = temp * ratio * ratio;
      if (temp2 <= nrm_thr) {
        R s = R(0);
#pragma unroll
        for (int r = K + 1; r < 5; ++r) s += qr[j][r] * qr[j][r];
        nd[j] = sqrt(s);
        nu[j] = nd[j];
      } else {
        nu[j] *= sqrt(temp);
      }
    }
  }
}

// least-squares plane n: min || A n + 1 || (odomEstimationClass.cpp:220), A = the 5 neighbours (rows)
template <typename R>
__device__ void plane_solve(const R (&A)[5][3], R (&x)[3]) {
  R qr[3][5];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 5; ++r) qr[c][r] = A[r][c];
  R hc[3] = {R(0), R(0), R(0)}, nu[3], nd[3];
  int tr[3] = {0, 1, 2};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    R s = R(0);
#pragma unroll
    for (int r = 0; r < 5; ++r) s += qr[k][r] * qr[k][r];
    nd[k] = sqrt(s);
    nu[k] = nd[k];
  }
  const R maxn = fmax(nu[0], fmax(nu[1], nu[2]));
  const R threshold_helper = (maxn * Lim<R>::eps()) * (maxn * Lim<R>::eps()) / R(5);
  int nz = 3;
  plane_pivot_step<0>(qr, hc, nu, nd, tr, nz, threshold_helper);
  plane_pivot_step<1>(qr, hc, nu, nd, tr, nz, threshold_helper);
  plane_pivot_step<2>(qr, hc, nu, nd, tr, nz, threshold_helper);
  // column permutation: perm = identity, then swap(perm[k], perm[tr[k]]) for k = 0..2
  int perm[3] = {0, 1, 2};
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      if (j != k && tr[k] == j) {
        const int t = perm[k];
        perm[k] = perm[j];
        perm[j] = t;
      }
  x[0] = x[1] = x[2] = R(0);
  if (nz == 0) return;
  R c[5] = {R(-1), R(-1), R(-1), R(-1), R(-1)};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k < nz && hc[k] != R(0)) {
      R tmp = c[k];
#pragma unroll
      for (int r = k + 1; r < 5; ++r) tmp += qr[k][r] * c[r];
      c[k] -= hc[k] * tmp;
#pragma unroll
      for (int r = k + 1; r < 5; ++r) c[r] -= hc[k] * qr[k][r] * tmp;
    }
  }
#pragma unroll
  for (int i = 2; i >= 0; --i) {
    if (i < nz) {
      R s = c[i];
#pragma unroll
      for (int j = i + 1; j < 3; ++j)
        if (j < nz) s -= qr[j][i] * c[j];
      c[i] = s / qr[i][i];
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (i < nz) {
#pragma unroll
      for (int j = 0; j < 3; ++j)
        if (perm[i] == j) x[j] = c[i];
    }
}


// LM state at the start of a solve (the former lm_init launch)
__device__ __forceinline__ void lm_reset(LMState* st, const X7& x0) {
  if (x0.set)
#pragma unroll
    for (int k = 0; k < 7; ++k) st->x[k] = x0.v[k];
  st->phase = 0;
  st->done = 0;
  st->iteration = 0;
  st->reuse = 0;
  st->invalid = 0;
  st->successful = 0;
  st->n_res = 0;
  st->corr_edge = 0;
  st->corr_surf = 0;
  st->tpend = 0;
  st->tdone = 0;
  st->radius = 1e4;
  st->dfac = 2.0;
  st->epoch += 8u;   // fresh hand-off tags for this solve's granules (lm.hip)
}

// ===================================================================================== correspondence search
// One query per group of kGroup lanes.  The group looks up the (<= 27) stencil cells of its query in parallel
// (one 16-B hash probe per cell), scans their counts into an exclusive prefix held in LDS, and then walks the
// FLATTENED candidate list: candidate t of the query lives in cell c with pre[c] <= t < pre[c+1], so the lanes
// take t = lane, lane + 16, ... with a forward-only cursor and kUnroll independent 16-B loads in flight per lane
// (coalesced within a cell, since cells are contiguous runs of the cell-sorted map).  Each lane keeps a sorted
// top-5 of 64-bit keys (float sq-distance bits << 32 | map index: ascending distance, ties by map index) and a
// butterfly merge over the group gives the exact 5-NN; lane 0 then runs the fp64 line / plane geometry.
constexpr int kGroupDefault = 16;   // lanes per query (template parameter G below)
constexpr int kUnrollDefault = 2;   // candidate loads in flight per lane (U; 2 beat 4 and 8 at C3)

// (start, count) of a coarse cell, or (0, 0): the entry's {key, start, total} head (one 16-B load)
template <typename Cell>
__device__ __forceinline__ int2 grid_lookup(const Cell* __restrict__ tab, unsigned long long key, int bits,
                                            unsigned mask) {
  unsigned h = coarse_slot(key, bits);
  for (;;) {
    const int4 e = *reinterpret_cast<const int4*>(&tab[h]);
    const unsigned long long k = ((unsigned long long)(unsigned)e.y << 32) | (unsigned)e.x;
    if (k == key) return make_int2(e.z, e.w);
    if (k == kEmptyKey) return make_int2(0, 0);
    h = (h + 1) & mask;
  }
}

// points in the fine (0.5-m) cell (fx, fy, fz): its sub-cell count in the entry of the coarse cell that holds it
__device__ __forceinline__ int fine_count(const struct CorrArgs& A, int fx, int fy, int fz);

__device__ __forceinline__ void cswap(unsigned long long& a, unsigned long long& b) {
  const unsigned long long lo = a < b ? a : b, hi = a < b ? b : a;
  a = lo;
  b = hi;
}

struct Top5 {
  unsigned long long k[5];
};

__device__ __forceinline__ void top5_insert(Top5& t, unsigned long long key) {
  if (key >= t.k[4]) return;
  t.k[4] = key;
  cswap(t.k[3], t.k[4]);
  cswap(t.k[2], t.k[3]);
  cswap(t.k[1], t.k[2]);
  cswap(t.k[0], t.k[1]);
}

// 5 smallest of two ascending 5-lists: bitonic split min(a[i], b[4-i]), then a 5-input sorting network
__device__ __forceinline__ void top5_merge(Top5& a, const Top5& b) {
  unsigned long long m[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) m[i] = a.k[i] < b.k[4 - i] ? a.k[i] : b.k[4 - i];
  cswap(m[0], m[1]); cswap(m[3], m[4]); cswap(m[2], m[4]); cswap(m[2], m[3]); cswap(m[0], m[3]);
  cswap(m[0], m[2]); cswap(m[1], m[4]); cswap(m[1], m[3]); cswap(m[1], m[2]);
#pragma unroll
  for (int i = 0; i < 5; ++i) a.k[i] = m[i];
}

template <int G>
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int m) {
  const int lo = __shfl_xor((int)(v & 0xFFFFFFFFull), m, G);
  const int hi = __shfl_xor((int)(v >> 32), m, G);
  return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}

template <int G>
__device__ __forceinline__ int group_incl_scan(int v, int lane) {
  if constexpr (G == 16) {   // one DPP row: row_shr 1, 2, 4, 8 (lanes below the shift get 0: bound_ctrl)
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);
    return v;
  }
#pragma unroll
  for (int o = 1; o < G; o <<= 1) {
    const int u = __shfl_up(v, o, G);
    if (lane >= o) v += u;
  }
  return v;
}

// LDS written by some lanes of a wave and read by others of the same wave: DS ops of one wave execute in order,
// so only the compiler has to be kept from reordering.
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// agent-scope relaxed 8-B store / load (global_store / global_load ... sc1): the hand-off forms of the Gram reduction
__device__ __forceinline__ void sc1_store(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double sc1_load(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

struct CorrArgs {
  const PointRec* q;       // downsampled scan points (sensor frame)
  const int* d_n;          // device count
  int n_ub;
  const float4* gpts;      // the map grouped by cell: {x, y, z, map index bits}
  const CoarseCell* coarse;
  int bits;                // table size 1 << bits (both tables)
  unsigned mask;
  const float4* map;       // the map's coordinates in its own order (neighbour coordinates by map index)
  int map_stride;          // float4s per map index: 1 (the grid's xyz copy) or 2 (FLOAM_GRID_NOXYZ: the records)
  double* rec;
  uint8_t* valid;
  float* nnxyz;
  int* nnidx;              // stage inspection (tracing only, else null): neighbour map indices, k-major
  float* nnsqd;            // ... and their float squared distances
  int cap;
};

// a neighbour's coordinates in A.map: the grid's xyz copy (product), or the map records (FLOAM_GRID_NOXYZ, diagnostic)
__device__ __forceinline__ size_t knn_map_index(const CorrArgs& A, unsigned idx) {
#ifdef FLOAM_DIAG
  return (size_t)A.map_stride * idx;
#else
  return idx;
#endif
}

__device__ __forceinline__ int fine_count(const CorrArgs& A, int fx, int fy, int fz) {
  const unsigned long long key = cell_key(fx >> 1, fy >> 1, fz >> 1);
  unsigned h = coarse_slot(key, A.bits);
  for (;;) {
    const CoarseCell& c = A.coarse[h];
    if (c.key == key) return c.sub[(fx & 1) | ((fy & 1) << 1) | ((fz & 1) << 2)];
    if (c.key == kEmptyKey) return 0;
    h = (h + 1) & A.mask;
  }
}

// Scan a block of up to 3 x 3 x 3 cells of one table into the lane-local top-5 (keys: float sq-distance bits << 32
// | position in the cell-sorted array, so ties go to the lower position).  Lane l looks up a contiguous run of the
// block's cells (all first probes issued before any is waited on), the group scans the counts into an exclusive
// prefix in LDS (cell order), and the lanes walk the flattened candidate list t = lane, lane + G, ... with a forward
// cursor and U independent 16-B loads in flight (coalesced within a cell).
constexpr int kMaxStencil = 27;

// Fine 3x3x3 block (stage 1) without a fine-cell table: the block's 27 fine cells lie in exactly 2x2x2 coarse cells
// (three consecutive fine indices halve to two consecutive coarse indices), whose entries carry the coarse range
// start and the point count of each of their 8 fine sub-cells (sub-cells are consecutive inside the range, in sub
// order: grid.hip).  Lanes 0..7 probe the 8 coarse cells (head and sub counts of a slot in one round trip) into LDS
// (s_cc[8][9]: start, 8 counts), then every fine cell's range is start + the counts of the sub-cells before it.
// NB = 2: the 2x2x2 fine block with low corner (lx, ly, lz) (the query's cell and its nearer neighbour per axis),
// whose cells lie in 1 or 2 coarse cells per axis (only those are probed).
template <int G, int NB = 3>
__device__ __forceinline__ void fine_block_ranges(const CorrArgs& A, int lx, int ly, int lz, int lane,
                                                  int* __restrict__ s_pre, int* __restrict__ s_start,
                                                  int* __restrict__ s_cc) {
  static_assert(G >= 8, "one coarse probe per lane");
  const int cx0 = lx >> 1, cy0 = ly >> 1, cz0 = lz >> 1;   // floor division by 2
  // (NB = 3: three consecutive fine indices always span two coarse indices; NB = 2: two when lx is odd)
  const bool need = NB == 3 || (((lane & 1) == 0 || (lx & 1)) && (((lane >> 1) & 1) == 0 || (ly & 1)) &&
                                ((lane >> 2) == 0 || (lz & 1)));
  if (lane < 8 && !need) {
    int* cc = s_cc + 9 * lane;
#pragma unroll
    for (int k = 0; k < 9; ++k) cc[k] = 0;
  }
  if (lane < 8 && need) {
    const unsigned long long key = cell_key(cx0 + (lane & 1), cy0 + ((lane >> 1) & 1), cz0 + (lane >> 2));
    unsigned slot = coarse_slot(key, A.bits);
    const int4* e = reinterpret_cast<const int4*>(&A.coarse[slot]);
    int4 h = e[0], s0 = e[1], s1 = e[2];
    unsigned long long k = ((unsigned long long)(unsigned)h.y << 32) | (unsigned)h.x;
    while (k != key && k != kEmptyKey) {   // collision chain (rare)
      slot = (slot + 1) & A.mask;
      e = reinterpret_cast<const int4*>(&A.coarse[slot]);
      h = e[0];
      s0 = e[1];
      s1 = e[2];
      k = ((unsigned long long)(unsigned)h.y << 32) | (unsigned)h.x;
    }
    const bool hit = k == key;
    int* cc = s_cc + 9 * lane;
    cc[0] = hit ? h.z : 0;
    cc[1] = hit ? s0.x : 0; cc[2] = hit ? s0.y : 0; cc[3] = hit ? s0.z : 0; cc[4] = hit ? s0.w : 0;
    cc[5] = hit ? s1.x : 0; cc[6] = hit ? s1.y : 0; cc[7] = hit ? s1.z : 0; cc[8] = hit ? s1.w : 0;
  }
  wave_lds_order();
  constexpr int NC = NB * NB * NB;
  constexpr int P = (NC + G - 1) / G;   // fine cells per lane
  const int cb = min(NC, lane * P), ce = min(NC, cb + P);
  int local = 0;
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const int c = cb + j;
    if (c < ce) {
      const int fx = lx + c % NB, fy = ly + (c / NB) % NB, fz = lz + c / (NB * NB);
      const int ci = ((fx >> 1) - cx0) | (((fy >> 1) - cy0) << 1) | (((fz >> 1) - cz0) << 2);
      const int sub = (fx & 1) | ((fy & 1) << 1) | ((fz & 1) << 2);
      const int* cc = s_cc + 9 * ci;
      int start = cc[0];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < sub) start += cc[1 + k];
      s_start[c] = start;
      s_pre[c] = local;
      local += cc[1 + sub];
    }
  }
  const int incl = group_incl_scan<G>(local, lane);
  const int excl = incl - local;
#pragma unroll
  for (int j = 0; j < P; ++j)
    if (cb + j < ce) s_pre[cb + j] += excl;
  if (lane == G - 1) s_pre[NC] = incl;
  wave_lds_order();
}

template <int G, int U, bool COARSE, int NB = 3>
__device__ __forceinline__ void stencil_scan(const CorrArgs& A, int x0, int x1, int y0, int y1, int z0, int z1,
                                             float wx, float wy, float wz, int lane, int* __restrict__ s_pre,
                                             int* __restrict__ s_start, Top5& t, int& cnt,
                                             int* __restrict__ s_cc = nullptr) {
  constexpr int P = (kMaxStencil + G - 1) / G;   // cells per lane
  const int nxr = x1 - x0 + 1, nyr = y1 - y0 + 1, nzr = z1 - z0 + 1;
  const int ncell = nxr * nyr * nzr;
  int tot;
  if constexpr (!COARSE) {   // the fine block with low corner (x0, y0, z0), ranges from the coarse entries
    fine_block_ranges<G, NB>(A, x0, y0, z0, lane, s_pre, s_start, s_cc);
    tot = s_pre[NB * NB * NB];
  } else {
  const int per = (ncell + G - 1) / G;
  const int cb = min(ncell, lane * per), ce = min(ncell, cb + per);
  unsigned long long key[P];
  unsigned slot[P];
  int4 e[P];
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const int c = cb + j;
    key[j] = kEmptyKey;
    e[j] = make_int4(-1, -1, 0, 0);
    if (c < ce) {
      key[j] = cell_key(x0 + c % nxr, y0 + (c / nxr) % nyr, z0 + c / (nxr * nyr));
      slot[j] = coarse_slot(key[j], A.bits);
      e[j] = *reinterpret_cast<const int4*>(&A.coarse[slot[j]]);
    }
  }
  int local = 0;
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const int c = cb + j;
    if (c < ce) {
      unsigned long long k = ((unsigned long long)(unsigned)e[j].y << 32) | (unsigned)e[j].x;
      while (k != key[j] && k != kEmptyKey) {   // collision chain (rare)
        slot[j] = (slot[j] + 1) & A.mask;
        e[j] = *reinterpret_cast<const int4*>(&A.coarse[slot[j]]);
        k = ((unsigned long long)(unsigned)e[j].y << 32) | (unsigned)e[j].x;
      }
      const bool hit = k == key[j];
      s_start[c] = hit ? e[j].z : 0;
      s_pre[c] = local;
      local += hit ? e[j].w : 0;
    }
  }
  const int incl = group_incl_scan<G>(local, lane);
  const int excl = incl - local;
#pragma unroll
  for (int j = 0; j < P; ++j)
    if (cb + j < ce) s_pre[cb + j] += excl;
  tot = __shfl(incl, G - 1, G);
  if (lane == 0) s_pre[ncell] = tot;
  wave_lds_order();
  }
  int c = 0, c_lo = 0, c_hi = s_pre[1], c_start = s_start[0];   // cursor: cell c = [c_lo, c_hi)
  for (int tb = 0; tb < tot; tb += G * U) {
    float4 m[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tt = tb + u * G + lane;
      if (tt < tot) {
        while (tt >= c_hi) {
          ++c;
          c_lo = c_hi;
          c_hi = s_pre[c + 1];
          c_start = s_start[c];
        }
        m[u] = A.gpts[c_start + (tt - c_lo)];
      } else {
        m[u] = make_float4(1e30f, 1e30f, 1e30f, 0.0f);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float dd = 0.0f;   // flann::L2_Simple<float>: ((0 + dx*dx) + dy*dy) + dz*dz
      float df = wx - m[u].x;
      dd += df * df;
      df = wy - m[u].y;
      dd += df * df;
      df = wz - m[u].z;
      dd += df * df;
      if (dd < 1.0f) {
        ++cnt;
        top5_insert(t, ((unsigned long long)__float_as_uint(dd) << 32) | (unsigned)__float_as_int(m[u].w));
      }
    }
  }
  wave_lds_order();   // the group's LDS slot is rewritten by its next scan
}

// one merge step with the partner lane given by a DPP control (a VALU lane move within a row of 16: no LDS crossbar
// round trip, which ds_bpermute — __shfl_xor — costs for each of the 11 words)
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
template <int CTRL>
__device__ __forceinline__ void merge_step_dpp(Top5& t, int& cnt) {
  Top5 o;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int lo = dpp_i32<CTRL>((int)(t.k[k] & 0xFFFFFFFFull)), hi = dpp_i32<CTRL>((int)(t.k[k] >> 32));
    o.k[k] = ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
  }
  top5_merge(t, o);
  cnt += dpp_i32<CTRL>(cnt);
}

// group-wide top-5 (every lane ends with the merged list) and count.  The merge of two top-5 lists is the top 5 of
// their union (keys are distinct), so any pairing that leaves every lane of the group with the whole union gives
// the same list: for G = 16 (one DPP row) quad_perm xor 1, quad_perm xor 2, then the half-row and the row mirrored
// (lane i with 7 - i, then with 15 - i), each step pairing two groups that are already uniform
template <int G>
__device__ __forceinline__ void group_merge(Top5& t, int& cnt) {
  if constexpr (G == 16) {
    merge_step_dpp<0xB1>(t, cnt);    // quad_perm [1, 0, 3, 2]
    merge_step_dpp<0x4E>(t, cnt);    // quad_perm [2, 3, 0, 1]
    merge_step_dpp<0x141>(t, cnt);   // row_half_mirror
    merge_step_dpp<0x140>(t, cnt);   // row_mirror
  } else {
#pragma unroll
    for (int mm = G / 2; mm > 0; mm >>= 1) {
      Top5 o;
#pragma unroll
      for (int k = 0; k < 5; ++k) o.k[k] = shfl_xor_u64<G>(t.k[k], mm);
      top5_merge(t, o);
      cnt += __shfl_xor(cnt, mm, G);
    }
  }
}


// Pass 1: exact 5-NN of every query (no fp64 geometry here, so the kernel stays small and at high occupancy).
// The reference keeps a correspondence iff the 5th-nearest float sq-distance is < 1 (:154, :210), so only map
// points within 1 m matter.  Stage 1 scans the 3x3x3 FINE cells (edge 0.5 m) around the query's cell: every point
// outside that block is at least 0.5 m away along some axis, so its float sq-distance is >= 0.25 (exact: the cell
// bounds are exact and fl(dx) >= 0.5 by monotone rounding); if 5 points with sq-distance < 0.25 were found they are
// the exact 5-NN.  Otherwise stage 2 scans the COARSE cells (1 m) spanning [q - r, q + r] on every axis (<= 3x3x3):
// r = 1 m (every point within 1 m) unless stage 1 already found 5 points within 1 m, then r = sqrt(d5) (1 + 1e-6) with
// d5 their 5th float sq-distance (the ball that holds the 5-NN and every tie with the 5th; see knn_group).  Ties at
// equal float distance go to the lower map index (FLANN's own order depends on its tree traversal; tie-free data is
// identical).
// Output: valid bit 0 = 5 neighbours within sqd < 1 (their coordinates in nnxyz), bit 1 = stage 2 was needed.
// Low fine corner of a query's stage-1 block: nb = 3, the cells around the query's (qx, qy, qz); nb = 2, the
// query's cell and the neighbour on the nearer side per axis (2 w - f is exact: f = floor(2 w) and 2 w are floats
// within a factor 2)
__device__ __forceinline__ void knn_block_corner(int nb, float wx, float wy, float wz, int qx, int qy, int qz, int& lx,
                                                 int& ly, int& lz) {
  lx = qx - 1;
  ly = qy - 1;
  lz = qz - 1;
  if (nb == 2) {
    if (2.0f * wx - (float)qx >= 0.5f) ++lx;
    if (2.0f * wy - (float)qy >= 0.5f) ++ly;
    if (2.0f * wz - (float)qz >= 0.5f) ++lz;
  }
}

template <bool EDGE, typename R>
__device__ __forceinline__ bool geom_fit(const R (&P)[5][3], float4 pq, double* __restrict__ rec, int cap, int i,
                                         double* __restrict__ w, const double* o);

// STOP (diagnostic, FLOAM_KNN_STAGES: the per-round-trip read attribution of DESIGN.md §3) ends each query after
// its first STOP dependent memory round trips — 1: the query load and transform; 2: + the coarse probes of the fine
// block; 3: + stage 1's candidate loads; 4: + stage 2 — and writes only a flag derived from what it loaded
template <int G, int U, int NB, int STOP = 0>
__device__ __forceinline__ void knn_group(const double (&pose)[7], const CorrArgs& A, int gid, int ngroups,
                                          int lane, bool gate, int rank, int world, int* __restrict__ s_pre,
                                          int* __restrict__ s_start, int* __restrict__ s_cc) {
  const int n = min(*A.d_n, A.n_ub);
  const int lo = (int)(((long long)n * rank) / world), hi = (int)(((long long)n * (rank + 1)) / world);
  // grid-stride over the queries the device holds (the host only knows an upper bound)
  for (int i0 = 0; i0 < n; i0 += ngroups) {
    const int i = i0 + gid;   // query
    if (i >= n) break;
    int flags = 0;
    if (i >= lo && i < hi && gate) {
      const float4 pq = *reinterpret_cast<const float4*>(&A.q[i].x);
      float wx, wy, wz;
      associate_to_map(pose, pq.x, pq.y, pq.z, wx, wy, wz);   // pointAssociateToMap (:126-135)
      int qx, qy, qz;
      fine_cell(wx, wy, wz, qx, qy, qz);
      if constexpr (STOP == 1) {
        if (lane == 0) A.valid[i] = (uint8_t)(qx ^ qy ^ qz);
        continue;
      }
      Top5 t;
#pragma unroll
      for (int k = 0; k < 5; ++k) t.k[k] = ~0ull;
      int cnt = 0;
      int lx, ly, lz;
      knn_block_corner(NB, wx, wy, wz, qx, qy, qz, lx, ly, lz);
      if constexpr (STOP == 2) {
        fine_block_ranges<G, NB>(A, lx, ly, lz, lane, s_pre, s_start, s_cc);
        if (lane == 0) A.valid[i] = (uint8_t)s_pre[NB * NB * NB];
        wave_lds_order();
        continue;
      }
      stencil_scan<G, U, false, NB>(A, lx, lx + NB - 1, ly, ly + NB - 1, lz, lz + NB - 1, wx, wy, wz, lane, s_pre,
                                    s_start, t, cnt, s_cc);
      group_merge<G>(t, cnt);
      // exact early exit: a map point outside the fine block [lo, hi) (lo = l / 2, hi = (l + NB) / 2 per axis, exact
      // in float) lies beyond a face, so on that axis |fl(q - p)| >= fl(q - lo) or fl(hi - q) (monotone rounding)
      // and its float sq-distance is >= fl(b^2), b the query's smallest face distance (>= 0.5 for NB = 3, >= 0.25
      // for NB = 2)
      const float b = fminf(fminf(fminf(wx - 0.5f * (float)lx, 0.5f * (float)(lx + NB) - wx),
                                  fminf(wy - 0.5f * (float)ly, 0.5f * (float)(ly + NB) - wy)),
                            fminf(wz - 0.5f * (float)lz, 0.5f * (float)(lz + NB) - wz));
      const bool complete = cnt >= 5 && __uint_as_float((unsigned)(t.k[4] >> 32)) < b * b;
      if constexpr (STOP == 3) {
        if (lane == 0) A.valid[i] = (uint8_t)(cnt + (complete ? 1 : 0) + (int)(t.k[4] & 0xFF));
        continue;
      }
      if (!complete) {
        // coarse cells floor(q - r) .. floor(q + r) per axis (exact in double).  r = 1 (every point within 1 m)
        // unless stage 1 already holds 5 points within 1 m: then the 5-NN and every point tied with the 5th lie in
        // the ball of its float sq-distance d5, and r = sqrt(d5) (1 + 1e-6) covers that ball with margin — a point
        // outside the box is more than r away along one axis, so its float sq-distance is >= r^2 (1 - 2^-24)^5 > d5
        // (monotone rounding of the 3 squares and 2 adds) and it can neither enter nor tie the top-5
        double r = 1.0;
        if (cnt >= 5) r = fmin(1.0, sqrt((double)__uint_as_float((unsigned)(t.k[4] >> 32))) * (1.0 + 1e-6));
#pragma unroll
        for (int k = 0; k < 5; ++k) t.k[k] = ~0ull;
        cnt = 0;
        stencil_scan<G, U, true>(A, (int)floor((double)wx - r), (int)floor((double)wx + r),
                                 (int)floor((double)wy - r), (int)floor((double)wy + r),
                                 (int)floor((double)wz - r), (int)floor((double)wz + r), wx, wy, wz, lane, s_pre,
                                 s_start, t, cnt);
        group_merge<G>(t, cnt);
        flags |= 2;
      }
      if constexpr (STOP == 4) {
        if (lane == 0) A.valid[i] = (uint8_t)(flags + cnt + (int)(t.k[4] & 0xFF));
        continue;
      }
      if (cnt >= 5) {   // sqd[4] < 1 (:154, :210)
        flags |= 1;
        if (lane < 5) {   // lane k writes the coordinates of neighbour k
          unsigned long long kk = t.k[0];
#pragma unroll
          for (int k = 1; k < 5; ++k)
            if (lane == k) kk = t.k[k];
          const float4 m = A.map[knn_map_index(A, (unsigned)(kk & 0xFFFFFFFFull))];
          A.nnxyz[(3 * lane + 0) * A.cap + i] = m.x;
          A.nnxyz[(3 * lane + 1) * A.cap + i] = m.y;
          A.nnxyz[(3 * lane + 2) * A.cap + i] = m.z;
          if (A.nnidx) {   // stage inspection: the neighbour's map index and float squared distance
            A.nnidx[lane * A.cap + i] = (int)(kk & 0xFFFFFFFFull);
            A.nnsqd[lane * A.cap + i] = __uint_as_float((unsigned)(kk >> 32));
          }
        }
      }
    }
    if (lane == 0) A.valid[i] = (uint8_t)flags;
  }
}

// -DFLOAM_KNN_WAVES (a scratch diagnostic build, tools/gpu_knn_waves.sh): every wave of the latest search launch
// records its start and end (s_memrealtime, 100 MHz) and its block's role; dumped by knn_waves_dump at handle close
#ifdef FLOAM_KNN_WAVES
constexpr int kKnnWaveRows = 16384;
__device__ unsigned long long g_knn_waves[kKnnWaveRows][2];
#endif

// Edge and surf kNN in one launch: blocks [0, nbE) run edge groups, the others surf groups.  The launch also starts
// the solve (lm_init folded in): block 0 resets the LM state and, for the first solve of an update, stores the
// prediction x0 that every block uses for its transforms (the others never read st->x in that case).
// (the search of logical block blk: knn_kernel's, and the search role of the role-split prototype below)
template <int G, int U, int NB, int STOP = 0>
__device__ __forceinline__ void knn_block(LMState* __restrict__ st, const double* __restrict__ x0_dev,
                                          const CorrArgs& E, const CorrArgs& S, int nbE, int nblocks, int blk,
                                          const int* __restrict__ d_me, const int* __restrict__ d_ms, int rank,
                                          int world) {
#ifdef FLOAM_KNN_WAVES
  const unsigned long long kw0 = __builtin_amdgcn_s_memrealtime();
#endif
  __shared__ int s_pre[kTB / G][kMaxStencil + 1];
  __shared__ int s_start[kTB / G][kMaxStencil];
  __shared__ int s_cc[kTB / G][8 * 9];
  const int lane = threadIdx.x & (G - 1);
  const int g = threadIdx.x / G;
  double pose[7];   // wave-uniform: kept in SGPRs (readfirstlane), not in 14 VGPRs of every lane
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const long long b = __double_as_longlong(x0_dev ? x0_dev[k] : st->x[k]);
    const int lo = __builtin_amdgcn_readfirstlane((int)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    pose[k] = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  }
  if (blk == 0 && threadIdx.x == 0) {
    X7 xs;
    xs.set = x0_dev ? 1 : 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) xs.v[k] = pose[k];
    lm_reset(st, xs);
  }
  const bool gate = *d_me > 10 && *d_ms > 50;   // map-size gate (odomEstimationClass.cpp:77)
  // XCD-aware placement: the blocks that hold queries are renumbered so that the blocks sharing an XCD (physical
  // index mod 8 under round-robin dispatch) take consecutive query ranges.  The queries are in voxel order, so each
  // XCD then works on a compact slab of the scene and its L2 holds that slab's map cells instead of all of them.
  const bool edge = blk < nbE;
  const CorrArgs& A = edge ? E : S;
  const int nb = edge ? nbE : nblocks - nbE;
  int p = edge ? blk : blk - nbE;
  const int nq = min(*A.d_n, A.n_ub);
  const int nact = min(nb, (int)(((long long)nq * G + kTB - 1) / kTB));
  if (p < nact) p = xcd_block(p, nact);
  knn_group<G, U, NB, STOP>(pose, A, (p * kTB + (int)threadIdx.x) / G, nb * (kTB / G), lane, gate, rank, world,
                            s_pre[g], s_start[g], s_cc[g]);
#ifdef FLOAM_KNN_WAVES
  {   // start | edge << 62 | holds queries << 61 | XCC id << 56 (HW_REG_XCC_ID), end; vector stores by lane 0
    const unsigned long long kw1 = __builtin_amdgcn_s_memrealtime();
    const unsigned xcc = (unsigned)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;
    const int w = blk * (kTB / 64) + (int)threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0 && w < kKnnWaveRows) {
      g_knn_waves[w][0] = (kw0 & ((1ull << 56) - 1)) | ((unsigned long long)(edge ? 1 : 0) << 62) |
                          ((unsigned long long)(p < nact ? 1 : 0) << 61) | ((unsigned long long)xcc << 56);
      g_knn_waves[w][1] = kw1;
    }
  }
#endif
}

template <int G, int U, int W, int NB, int STOP = 0>
__global__ __launch_bounds__(kTB, W) void knn_kernel(LMState* __restrict__ st, const double* __restrict__ x0_dev,
                                                  CorrArgs E, CorrArgs S, int nbE,
                                                  const int* __restrict__ d_me, const int* __restrict__ d_ms,
                                                  int rank, int world) {
  knn_block<G, U, NB, STOP>(st, x0_dev, E, S, nbE, (int)gridDim.x, (int)blockIdx.x, d_me, d_ms, rank, world);
}

#ifdef FLOAM_DIAG
// ----------------------------------------------------------------------------------- LDS-staged stage 1
// The north star's "LDS-staged spatial-hash grid", re-measured against the search above (diagnostic build:
// FLOAM_KNN_LDS=1).  A block's 16 queries (one per 16-lane group, as knn_kernel) are consecutive in voxel order, so
// their 3 x 3 x 3 fine blocks overlap: the block takes the bounding box of the 16 fine blocks (fine cells, <= kLdsCells),
// probes the coarse entries that cover it once (one thread per coarse cell, <= kLdsCoarse), lays the box's fine cells
// out in LDS order (a block scan of their counts) and copies their points into LDS with one flattened, coalesced load
// round (<= kLdsPts points); each group then scans its query's 27 fine cells from LDS — the same candidates, float
// distances and (distance, map index) keys as the global scan, so the same top-5.  Stage 2 and the outputs are the
// search's own.  A block whose box or points do not fit takes the global stage 1 (fine_block_ranges + stencil_scan).
constexpr int kLdsCells = 512;
constexpr int kLdsCoarse = 256;
constexpr int kLdsPts = 1536;

template <int G, int U>
__device__ __forceinline__ void knn_group_lds(const double (&pose)[7], const CorrArgs& A, int gbase, int ngroups,
                                              int lane, int g, bool gate, int rank, int world, int* __restrict__ s_pre,
                                              int* __restrict__ s_start, int* __restrict__ s_cc) {
  constexpr int NB = 3;
  __shared__ int s_box[6];                 // fine-corner min x, y, z, max x, y, z of the active queries
  __shared__ int s_cs[kLdsCoarse][9];      // coarse entries over the box: start, 8 sub-cell counts
  __shared__ int s_fs[kLdsCells];          // fine cells of the box: start in the cell-grouped map
  __shared__ int s_fo[kLdsCells + 1];      // ... and their offset in s_pts (exclusive scan of the counts)
  __shared__ float4 s_pts[kLdsPts];
  __shared__ int s_ws[kTB / 64];
  const int t = (int)threadIdx.x;
  const int n = min(*A.d_n, A.n_ub);
  const int lo = (int)(((long long)n * rank) / world), hi = (int)(((long long)n * (rank + 1)) / world);
  for (int i0 = 0; i0 < n; i0 += ngroups) {   // block-uniform trip count (every group of the block in each round)
    const int i = i0 + gbase + g;
    const bool act = i < n && i >= lo && i < hi && gate;
    float wx = 0.f, wy = 0.f, wz = 0.f;
    int lx = 0, ly = 0, lz = 0;
    if (act) {
      const float4 pq = *reinterpret_cast<const float4*>(&A.q[i].x);
      associate_to_map(pose, pq.x, pq.y, pq.z, wx, wy, wz);   // pointAssociateToMap (:126-135)
      int qx, qy, qz;
      fine_cell(wx, wy, wz, qx, qy, qz);
      knn_block_corner(NB, wx, wy, wz, qx, qy, qz, lx, ly, lz);
    }
    // the block's box of fine blocks
    if (t < 6) s_box[t] = t < 3 ? INT_MAX : INT_MIN;
    __syncthreads();
    if (act && lane == 0) {
      atomicMin(&s_box[0], lx); atomicMin(&s_box[1], ly); atomicMin(&s_box[2], lz);
      atomicMax(&s_box[3], lx); atomicMax(&s_box[4], ly); atomicMax(&s_box[5], lz);
    }
    __syncthreads();
    const int bx0 = s_box[0], by0 = s_box[1], bz0 = s_box[2];
    const bool any = bx0 != INT_MAX;
    const int DX = any ? s_box[3] - bx0 + NB : 0, DY = any ? s_box[4] - by0 + NB : 0, DZ = any ? s_box[5] - bz0 + NB : 0;
    const long long nfc = (long long)DX * DY * DZ;
    const int cx0 = bx0 >> 1, cy0 = by0 >> 1, cz0 = bz0 >> 1;   // coarse box (floor halves)
    const int CX = any ? ((bx0 + DX - 1) >> 1) - cx0 + 1 : 0, CY = any ? ((by0 + DY - 1) >> 1) - cy0 + 1 : 0,
              CZ = any ? ((bz0 + DZ - 1) >> 1) - cz0 + 1 : 0;
    const long long ncc = (long long)CX * CY * CZ;
    bool staged = any && nfc <= kLdsCells && ncc <= kLdsCoarse;   // (block-uniform)
    if (staged) {
      if (t < ncc) {   // one coarse probe per thread (head + sub counts: 48 B of the 64-B entry)
        const int ax = t % CX, ay = (t / CX) % CY, az = t / (CX * CY);
        const unsigned long long key = cell_key(cx0 + ax, cy0 + ay, cz0 + az);
        unsigned slot = coarse_slot(key, A.bits);
        const int4* e = reinterpret_cast<const int4*>(&A.coarse[slot]);
        int4 h = e[0], s0 = e[1], s1 = e[2];
        unsigned long long k = ((unsigned long long)(unsigned)h.y << 32) | (unsigned)h.x;
        while (k != key && k != kEmptyKey) {   // collision chain (rare)
          slot = (slot + 1) & A.mask;
          e = reinterpret_cast<const int4*>(&A.coarse[slot]);
          h = e[0]; s0 = e[1]; s1 = e[2];
          k = ((unsigned long long)(unsigned)h.y << 32) | (unsigned)h.x;
        }
        const bool hit = k == key;
        int* cc = s_cs[t];
        cc[0] = hit ? h.z : 0;
        cc[1] = hit ? s0.x : 0; cc[2] = hit ? s0.y : 0; cc[3] = hit ? s0.z : 0; cc[4] = hit ? s0.w : 0;
        cc[5] = hit ? s1.x : 0; cc[6] = hit ? s1.y : 0; cc[7] = hit ? s1.z : 0; cc[8] = hit ? s1.w : 0;
      }
      __syncthreads();
      // fine cells c = 2 t, 2 t + 1 (box order, x fastest): start and count, then the block's exclusive scan
      int cnt2[2] = {0, 0};
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = 2 * t + u;
        if (c < nfc) {
          const int fx = bx0 + c % DX, fy = by0 + (c / DX) % DY, fz = bz0 + c / (DX * DY);
          const int ci = ((fx >> 1) - cx0) + CX * (((fy >> 1) - cy0) + CY * ((fz >> 1) - cz0));
          const int sub = (fx & 1) | ((fy & 1) << 1) | ((fz & 1) << 2);
          const int* cc = s_cs[ci];
          int start = cc[0];
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (k < sub) start += cc[1 + k];
          s_fs[c] = start;
          cnt2[u] = cc[1 + sub];
        }
      }
      const int mine = cnt2[0] + cnt2[1];
      const int incl = wave_incl_scan(mine);
      if ((t & 63) == 63) s_ws[t >> 6] = incl;
      __syncthreads();
      int wb = 0, tot = 0;
#pragma unroll
      for (int k = 0; k < kTB / 64; ++k) {
        if (k < (t >> 6)) wb += s_ws[k];
        tot += s_ws[k];
      }
      const int ex = wb + incl - mine;
      if (2 * t < nfc) s_fo[2 * t] = ex;
      if (2 * t + 1 < nfc) s_fo[2 * t + 1] = ex + cnt2[0];
      if (t == 0) s_fo[nfc] = tot;
      staged = tot <= kLdsPts;   // (block-uniform)
      __syncthreads();
      if (staged) {   // the box's points into LDS: element q of the flattened list, cell by binary search
        constexpr int kR = (kLdsPts + kTB - 1) / kTB;
        int src[kR];   // every element's source first (LDS binary searches, fixed 9 steps), then all loads in flight
#pragma unroll
        for (int r = 0; r < kR; ++r) {
          const int q = r * kTB + t;
          int a = 0;   // last cell with s_fo[cell] <= q
#pragma unroll
          for (int step = kLdsCells / 2; step > 0; step >>= 1)
            if (a + step < nfc && s_fo[a + step] <= q) a += step;
          src[r] = q < tot ? s_fs[a] + (q - s_fo[a]) : -1;
        }
        float4 m[kR];
#pragma unroll
        for (int r = 0; r < kR; ++r) m[r] = src[r] >= 0 ? A.gpts[src[r]] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int r = 0; r < kR; ++r)
          if (r * kTB + t < tot) s_pts[r * kTB + t] = m[r];
        __syncthreads();
      }
    }
    int flags = 0;
    Top5 tp;
#pragma unroll
    for (int k = 0; k < 5; ++k) tp.k[k] = ~0ull;
    int cnt = 0;
    if (act) {
      if (staged) {   // the query's 27 fine cells from LDS: lane l takes cells 2 l, 2 l + 1 (a group scan of counts)
        constexpr int NC = NB * NB * NB;
        int lc[2], lo2[2], ln[2];
        int local = 0;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int c = 2 * lane + u;
          lc[u] = 0; lo2[u] = 0; ln[u] = 0;
          if (c < NC) {
            const int fx = lx + c % NB, fy = ly + (c / NB) % NB, fz = lz + c / (NB * NB);
            const int bc = (fx - bx0) + DX * ((fy - by0) + DY * (fz - bz0));
            lo2[u] = s_fo[bc];
            ln[u] = s_fo[bc + 1] - lo2[u];
            lc[u] = local;
            local += ln[u];
          }
        }
        const int inc = group_incl_scan<G>(local, lane);
        const int ex = inc - local;
        const int tot = __shfl(inc, G - 1, G);
        int* pre = s_pre;   // this group's: [c] prefix, and s_start[c] its LDS offset
#pragma unroll
        for (int u = 0; u < 2; ++u)
          if (2 * lane + u < NC) {
            pre[2 * lane + u] = ex + lc[u];
            s_start[2 * lane + u] = lo2[u];
          }
        if (lane == 0) pre[NC] = tot;
        wave_lds_order();
        int c = 0, c_lo = 0, c_hi = pre[1], c_start = s_start[0];
        for (int tt = lane; tt < tot; tt += G) {
          while (tt >= c_hi) {
            ++c;
            c_lo = c_hi;
            c_hi = pre[c + 1];
            c_start = s_start[c];
          }
          const float4 mm = s_pts[c_start + (tt - c_lo)];
          float dd = 0.0f;   // flann::L2_Simple<float>: ((0 + dx*dx) + dy*dy) + dz*dz
          float df = wx - mm.x;
          dd += df * df;
          df = wy - mm.y;
          dd += df * df;
          df = wz - mm.z;
          dd += df * df;
          if (dd < 1.0f) {
            ++cnt;
            top5_insert(tp, ((unsigned long long)__float_as_uint(dd) << 32) | (unsigned)__float_as_int(mm.w));
          }
        }
        wave_lds_order();
      } else {
        stencil_scan<G, U, false, NB>(A, lx, lx + NB - 1, ly, ly + NB - 1, lz, lz + NB - 1, wx, wy, wz, lane, s_pre,
                                      s_start, tp, cnt, s_cc);
      }
      group_merge<G>(tp, cnt);
      const float b = fminf(fminf(fminf(wx - 0.5f * (float)lx, 0.5f * (float)(lx + NB) - wx),
                                  fminf(wy - 0.5f * (float)ly, 0.5f * (float)(ly + NB) - wy)),
                            fminf(wz - 0.5f * (float)lz, 0.5f * (float)(lz + NB) - wz));
      const bool complete = cnt >= 5 && __uint_as_float((unsigned)(tp.k[4] >> 32)) < b * b;
      if (!complete) {   // stage 2 exactly as knn_group
        double r = 1.0;
        if (cnt >= 5) r = fmin(1.0, sqrt((double)__uint_as_float((unsigned)(tp.k[4] >> 32))) * (1.0 + 1e-6));
#pragma unroll
        for (int k = 0; k < 5; ++k) tp.k[k] = ~0ull;
        cnt = 0;
        stencil_scan<G, U, true>(A, (int)floor((double)wx - r), (int)floor((double)wx + r),
                                 (int)floor((double)wy - r), (int)floor((double)wy + r),
                                 (int)floor((double)wz - r), (int)floor((double)wz + r), wx, wy, wz, lane, s_pre,
                                 s_start, tp, cnt);
        group_merge<G>(tp, cnt);
        flags |= 2;
      }
      if (cnt >= 5) {   // sqd[4] < 1 (:154, :210)
        flags |= 1;
        if (lane < 5) {   // lane k writes the coordinates of neighbour k
          unsigned long long kk = tp.k[0];
#pragma unroll
          for (int k = 1; k < 5; ++k)
            if (lane == k) kk = tp.k[k];
          const float4 mm = A.map[knn_map_index(A, (unsigned)(kk & 0xFFFFFFFFull))];
          A.nnxyz[(3 * lane + 0) * A.cap + i] = mm.x;
          A.nnxyz[(3 * lane + 1) * A.cap + i] = mm.y;
          A.nnxyz[(3 * lane + 2) * A.cap + i] = mm.z;
          if (A.nnidx) {
            A.nnidx[lane * A.cap + i] = (int)(kk & 0xFFFFFFFFull);
            A.nnsqd[lane * A.cap + i] = __uint_as_float((unsigned)(kk >> 32));
          }
        }
      }
    }
    if (i < n && lane == 0) A.valid[i] = (uint8_t)flags;
    __syncthreads();   // (the staging arrays are rewritten next round)
  }
}

template <int G, int U>
__global__ __launch_bounds__(kTB) void knn_kernel_lds(LMState* __restrict__ st, const double* __restrict__ x0_dev,
                                                       CorrArgs E, CorrArgs S, int nbE, const int* __restrict__ d_me,
                                                       const int* __restrict__ d_ms, int rank, int world) {
  __shared__ int s_pre[kTB / G][kMaxStencil + 1];
  __shared__ int s_start[kTB / G][kMaxStencil];
  __shared__ int s_cc[kTB / G][8 * 9];
  const int lane = threadIdx.x & (G - 1);
  const int g = threadIdx.x / G;
  double pose[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const long long b = __double_as_longlong(x0_dev ? x0_dev[k] : st->x[k]);
    const int lo = __builtin_amdgcn_readfirstlane((int)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    pose[k] = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    X7 xs;
    xs.set = x0_dev ? 1 : 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) xs.v[k] = pose[k];
    lm_reset(st, xs);
  }
  const bool gate = *d_me > 10 && *d_ms > 50;
  const bool edge = (int)blockIdx.x < nbE;
  const CorrArgs& A = edge ? E : S;
  const int nb = edge ? nbE : (int)gridDim.x - nbE;
  int p = edge ? (int)blockIdx.x : (int)blockIdx.x - nbE;
  const int nq = min(*A.d_n, A.n_ub);
  const int nact = min(nb, (int)(((long long)nq * G + kTB - 1) / kTB));
  if (p < nact) p = xcd_block(p, nact);
  knn_group_lds<G, U>(pose, A, p * (kTB / G), nb * (kTB / G), lane, g, gate, rank, world, s_pre[g], s_start[g],
                      s_cc[g]);
}
#endif

// Pass 2: line / plane geometry, one query per lane (all 64 lanes busy), in R = double (the reference's precision)
// or float (the C5 sweep's fp32 variant; records are stored as the doubles of the float results).
// Surf record i as the 13-vector w = [n (x) p (9), n (3), d + n.o] (p the sensor-frame point, n the unit normal,
// d the plane offset, o the solve's starting translation): every surf residual and Jacobian entry is linear in w
// (see lm.hip surf_sums_from_gram), so the surf half of each squared-loss LM evaluation needs only sum(w w^T).
// EDGE with w != null: the record's 9 values are also returned in w (the iteration-zero edge sums).  Returns whether
// the query produced a record.
// the line / plane fit of query i from its 5 neighbours P and its sensor-frame point pq: the record at rec[. * cap + i]
// (and w, below); returns whether the fit produced a record
template <bool EDGE, typename R>
__device__ __forceinline__ bool geom_fit(const R (&P)[5][3], float4 pq, double* __restrict__ rec, int cap, int i,
                                         double* __restrict__ w, const double* o) {
  bool ok = false;
  {
    const double cpx = pq.x, cpy = pq.y, cpz = pq.z;
    if (EDGE) {
      // addEdgeCostFactor geometry (odomEstimationClass.cpp:156-189)
      R cc[3] = {R(0), R(0), R(0)};
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        cc[0] = cc[0] + P[j][0]; cc[1] = cc[1] + P[j][1]; cc[2] = cc[2] + P[j][2];
      }
      cc[0] = cc[0] / R(5); cc[1] = cc[1] / R(5); cc[2] = cc[2] / R(5);
      R cov[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const R z[3] = {P[j][0] - cc[0], P[j][1] - cc[1], P[j][2] - cc[2]};
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
          for (int b = 0; b < 3; ++b) cov[a][b] = cov[a][b] + z[a] * z[b];
      }
      R ev[3], u[3];
      eig_sym3(cov, ev, u);
      if (ev[2] > R(3) * ev[1]) {
        ok = true;
        rec[0 * cap + i] = cpx; rec[1 * cap + i] = cpy; rec[2 * cap + i] = cpz;
        rec[3 * cap + i] = R(0.1) * u[0] + cc[0]; rec[4 * cap + i] = R(0.1) * u[1] + cc[1];
        rec[5 * cap + i] = R(0.1) * u[2] + cc[2];
        rec[6 * cap + i] = R(-0.1) * u[0] + cc[0]; rec[7 * cap + i] = R(-0.1) * u[1] + cc[1];
        rec[8 * cap + i] = R(-0.1) * u[2] + cc[2];
        if (w) {   // (the same values as stored)
          w[0] = cpx; w[1] = cpy; w[2] = cpz;
          w[3] = (double)(R(0.1) * u[0] + cc[0]); w[4] = (double)(R(0.1) * u[1] + cc[1]);
          w[5] = (double)(R(0.1) * u[2] + cc[2]);
          w[6] = (double)(R(-0.1) * u[0] + cc[0]); w[7] = (double)(R(-0.1) * u[1] + cc[1]);
          w[8] = (double)(R(-0.1) * u[2] + cc[2]);
        }
      }
    } else {
      // addSurfCostFactor geometry (odomEstimationClass.cpp:208-243)
      R nv[3];
      plane_solve(P, nv);
      const R z = nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2];
      const R d = R(1) / sqrt(z);
      if (z > R(0)) {
        const R sz = sqrt(z);
        nv[0] = nv[0] / sz; nv[1] = nv[1] / sz; nv[2] = nv[2] / sz;
      }
      bool planeValid = true;
#pragma unroll
      for (int j = 0; j < 5; ++j)
        if (fabs(nv[0] * P[j][0] + nv[1] * P[j][1] + nv[2] * P[j][2] + d) > R(0.2)) planeValid = false;
      if (planeValid) {
        ok = true;
        rec[0 * cap + i] = cpx; rec[1 * cap + i] = cpy; rec[2 * cap + i] = cpz;
        rec[3 * cap + i] = nv[0]; rec[4 * cap + i] = nv[1]; rec[5 * cap + i] = nv[2];
        rec[6 * cap + i] = d;
        if (w) {   // (double only: the Gram path is the fp64 squared-loss solve)
          const double nd[3] = {(double)nv[0], (double)nv[1], (double)nv[2]};
          const double pp[3] = {cpx, cpy, cpz};
#pragma unroll
          for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int e = 0; e < 3; ++e) w[3 * a + e] = nd[a] * pp[e];
          w[9] = nd[0]; w[10] = nd[1]; w[11] = nd[2];
          w[12] = (double)d + ((nd[0] * o[0] + nd[1] * o[1]) + nd[2] * o[2]);
        }
      }
    }
  }
  return ok;
}

// -DFLOAM_GEOM_STAMPS (diagnostic build): geom_kernel's phase times per block of the latest launches (s_memrealtime,
// 100 MHz), stored by thread 0 with plain stores into the block's own row (no shared counters: atomics on shared
// words would queue behind each other and inflate what they measure): [0] start, [1] query loads done (flags
// known), [2] fit done, [3] edge sums / Gram done, [4] hand-off done (surf), [5] end, [6] role (0 edge, 1 surf,
// 2 surf with the group reduce); printed by geom_stamps_print for the blocks of the newest launch
#ifdef FLOAM_GEOM_STAMPS
constexpr int kGeomStampBlocks = 4096;
__device__ unsigned long long g_geom_blk[kGeomStampBlocks][8];
__device__ __forceinline__ unsigned long long geom_now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void geom_row(unsigned long long t0, unsigned long long ta, unsigned long long tb,
                                         unsigned long long tg, unsigned long long th, int role) {
  if (threadIdx.x != 0 || blockIdx.x >= (unsigned)kGeomStampBlocks) return;
  unsigned long long* r = g_geom_blk[blockIdx.x];
  r[0] = t0; r[1] = ta; r[2] = tb; r[3] = tg; r[4] = th; r[5] = geom_now(); r[6] = (unsigned long long)role;
}
#define GEOM_STAMP(v, dep)                  \
  asm volatile("" ::"v"((int)(dep)));       \
  const unsigned long long v = geom_now()
#else
#define GEOM_STAMP(v, dep)
#endif

template <bool EDGE, typename R>
__device__ __forceinline__ bool geom_query(LMState* __restrict__ st, const CorrArgs& A, int i,
                                           double* __restrict__ w = nullptr, const double* o = nullptr,
                                           unsigned long long* tst = nullptr) {
  // the flag, the neighbours and the query loaded speculatively for every slot inside the arrays (i < n_ub <= cap),
  // beside the device count: one memory round trip before the fit instead of three dependent ones (count -> flag ->
  // coordinates); slots without a search result are read but never used
  R P[5][3];
  float4 pq = make_float4(0.f, 0.f, 0.f, 0.f);
  int flags0 = 0;
  if (i < A.n_ub) {
    flags0 = A.valid[i];
#pragma unroll
    for (int j = 0; j < 5; ++j)
#pragma unroll
      for (int a = 0; a < 3; ++a) P[j][a] = A.nnxyz[(3 * j + a) * A.cap + i];
    pq = *reinterpret_cast<const float4*>(&A.q[i].x);
  }
  const int n = min(*A.d_n, A.n_ub);
  bool ok = false;
  const int flags = i < n ? flags0 : 0;
  GEOM_STAMP(ta, flags + (int)P[4][2] + (int)pq.x);
  if (flags & 1) {
    ok = geom_fit<EDGE, R>(P, pq, A.rec, A.cap, i, w, o);
    A.valid[i] = (uint8_t)((flags & 2) | (ok ? 1 : 0) | 4);   // bit 2: the search found 5 neighbours
  }
#ifdef FLOAM_GEOM_STAMPS
  GEOM_STAMP(tb, ok);
  if (tst) { tst[0] = ta; tst[1] = tb; }
#endif
  const unsigned long long b = __ballot(ok);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(EDGE ? &st->corr_edge : &st->corr_surf, __popcll(b));
  return ok;
}

__device__ __forceinline__ void gram_pair(int e, int& i, int& j) {   // upper-triangle entry e -> (i, j), i <= j
  i = 0;
  while (e >= kGramW - i) {
    e -= kGramW - i;
    ++i;
  }
  j = i + e;
}

// Edge blocks: one query per lane.  Surf blocks (fixed grid, grid-stride): one query per lane, and the block's
// partial Gram matrix of its accepted surf records (waves stage w in LDS, lane e sums entry e over the wave's 64
// records in lane order, waves combined in order) into gpart[block][91].
template <typename R>
__device__ __forceinline__ void geom_block(LMState* __restrict__ st, const CorrArgs& E, const CorrArgs& S, int nbE,
                                           int blk, double* __restrict__ gpart, double* __restrict__ gmat,
                                           unsigned* __restrict__ gcnt) {
#ifdef FLOAM_GEOM_STAMPS
  GEOM_STAMP(t0, 0);
  unsigned long long tq[2] = {t0, t0};
#define GEOM_TQ , tq
#else
#define GEOM_TQ
#endif
  if (blk < nbE) {
    geom_query<true, R>(st, E, blk * (int)blockDim.x + (int)threadIdx.x, nullptr, nullptr GEOM_TQ);
#ifdef FLOAM_GEOM_STAMPS
    geom_row(t0, tq[0], tq[1], tq[1], tq[1], 0);
#endif
    return;
  }
  const int sb = blk - nbE;
  const int ns = min(*S.d_n, S.n_ub);   // the device count bounds the grid-stride loops (block-uniform)
  if (!gpart) {
    for (int i0 = sb * kTB; i0 < ns; i0 += kSurfGeomBlocks * kTB) geom_query<false, R>(st, S, i0 + threadIdx.x);
    return;
  }
  __shared__ double s_w[kTB / 64][kGramW][65];   // padded rows: lanes reading different rows hit different banks
  __shared__ double s_part[kTB / 64][kGram];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double o[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) o[k] = st->x[4 + k];
  int ei0, ej0, ei1 = 0, ej1 = 0;
  gram_pair(lane, ei0, ej0);
  if (lane + 64 < kGram) gram_pair(lane + 64, ei1, ej1);
  double g0 = 0.0, g1 = 0.0;
#ifdef FLOAM_GEOM_STAMPS
  unsigned long long sl = 0ull, sf = 0ull, sg = 0ull;
#endif
  for (int i0 = sb * kTB; i0 < ns; i0 += kSurfGeomBlocks * kTB) {   // wave-uniform trip count
#ifdef FLOAM_GEOM_STAMPS
    GEOM_STAMP(ti, 0);
#endif
    double w[kGramW];
#pragma unroll
    for (int k = 0; k < kGramW; ++k) w[k] = 0.0;
    geom_query<false, R>(st, S, i0 + threadIdx.x, w, o GEOM_TQ);
#pragma unroll
    for (int k = 0; k < kGramW; ++k) s_w[wv][k][lane] = w[k];
    wave_lds_order();
    double a0 = 0.0, a1 = 0.0;
#pragma unroll 16
    for (int r = 0; r < 64; ++r) {
      a0 += s_w[wv][ei0][r] * s_w[wv][ej0][r];
      a1 += s_w[wv][ei1][r] * s_w[wv][ej1][r];
    }
    g0 += a0;
    g1 += a1;
    wave_lds_order();
#ifdef FLOAM_GEOM_STAMPS
    GEOM_STAMP(tg, __double_as_longlong(g0) & 1);
    sl += tq[0] - ti;
    sf += tq[1] - tq[0];
    sg += tg - tq[1];
#endif
  }
  s_part[wv][lane] = g0;
  if (lane + 64 < kGram) s_part[wv][lane + 64] = g1;
  __syncthreads();
  if (threadIdx.x < kGram) {
    double v = s_part[0][threadIdx.x];
#pragma unroll
    for (int k = 1; k < kTB / 64; ++k) v += s_part[k][threadIdx.x];
    sc1_store(&gpart[sb * kGram + threadIdx.x], v);
  }
  // G of the solve, reduced by the last-arriving block of each group (fixed order: the 32 blocks of a group here; the
  // 8 groups in the solve's prologue, gram_load),
  // without agent fences (MI355X_MICROARCH.md "Hand-offs measured with sc1 loads in place of the acquire", first
  // row): every partial is stored sc1 and loaded sc1; each storing wave drains its stores (vmcnt(0)) before the
  // block barrier behind which one lane adds to the group's ticket; the block whose add comes last reads the group
  // after its add has returned (its other waves after the barrier).  (Two release / acquire fence pairs on the
  // chain cost ~1.7 us each.)
  constexpr int per = kSurfGeomBlocks / kGramGroups;
  __shared__ int s_last;
  const int grp = sb / per;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(&gcnt[grp], 1u) == (unsigned)(per - 1);
  __syncthreads();
#ifdef FLOAM_GEOM_STAMPS
  GEOM_STAMP(t4, s_last);
  if (!s_last) geom_row(t0, t0 + sl, t0 + sl + sf, t0 + sl + sf + sg, t4, 1);
#endif
  if (!s_last) return;
  if (threadIdx.x < kGram) {   // the group's partial of G into gmat[grp] (the solve adds the groups, gram_load)
    double v = 0.0;
    double gp[per];   // all loads in flight before the in-order sum
#pragma unroll
    for (int k = 0; k < per; ++k) gp[k] = sc1_load(&gpart[(grp * per + k) * kGram + threadIdx.x]);
#pragma unroll
    for (int k = 0; k < per; ++k) v += gp[k];
    gmat[grp * kGram + threadIdx.x] = v;
  } else if (grp == 0 && threadIdx.x < kGram + 3) {
    gmat[kGramGroups * kGram + threadIdx.x - kGram] = o[threadIdx.x - kGram];   // the origin the records use
  }
  if (threadIdx.x == 0) gcnt[grp] = 0u;   // every block of the group has arrived (next launch: kernel boundary)
#ifdef FLOAM_GEOM_STAMPS
  geom_row(t0, t0 + sl, t0 + sl + sf, t0 + sl + sf + sg, t4, 2);
#endif
}
#undef GEOM_TQ

template <typename R>
__global__ __launch_bounds__(kTB) void geom_kernel(LMState* __restrict__ st, CorrArgs E, CorrArgs S, int nbE,
                                                   double* __restrict__ gpart, double* __restrict__ gmat,
                                                   unsigned* __restrict__ gcnt) {
  geom_block<R>(st, E, S, nbE, (int)blockIdx.x, gpart, gmat, gcnt);
}

#ifdef FLOAM_DIAG
// ----------------------------------------------------------------------------------- role-split prototype (r05 item 2)
// The search and the geometry fits in ONE launch (diagnostic build, FLOAM_KNN_SPLIT=1): every block takes a ticket
// at its start; tickets [0, nbK) run the search blocks of knn_kernel, the later ones the geometry blocks of
// geom_kernel, each after polling the completion count of the 256 queries it fits (sctl[kSplitChunk0 + chunk]: edge chunks
// first, then surf).  A geometry block only waits on search blocks with smaller tickets, which are already running,
// so the launch cannot deadlock (the lookbacks' argument).  Hand-off (MI355X_MICROARCH.md, valid forms):
// the search block's plain stores -> every wave's vmcnt(0) -> barrier -> one lane's agent release fence -> vmcnt(0) ->
// relaxed agent adds to the chunk counters; the geometry block: relaxed polls -> agent acquire -> vmcnt(0) -> barrier.
// The LM reset of ticket 0 is published the same way (sctl[kSplitResetWord] = epoch) before any geometry block counts
// correspondences.  The kernel is allocated the geometry's registers, so the search runs at the occupancy those allow.
// sctl: [0] the ticket, [32] the reset word, [64 + chunk] the completion counts — each on lines of its own, and every
// access atomic (agent scope: sc1).  A plain store or load of one of these lines leaves it in that XCD's L2, where the
// sc1 polls of that XCD's blocks then keep reading the stale copy (the first form of this prototype did so, saw no
// completion and went on with the fits of stale flags).
constexpr int kSplitResetWord = 32;
constexpr int kSplitChunk0 = 64;
template <typename R>
__global__ __launch_bounds__(kTB) void knn_geom_split(LMState* __restrict__ st, const double* __restrict__ x0_dev,
                                                      CorrArgs E, CorrArgs S, int nbE, int nbK, int gE,
                                                      const int* __restrict__ d_me, const int* __restrict__ d_ms,
                                                      int rank, int world, double* __restrict__ gpart,
                                                      double* __restrict__ gmat, unsigned* __restrict__ gcnt,
                                                      unsigned* __restrict__ sctl, unsigned epoch,
                                                      unsigned* __restrict__ watch) {
  constexpr int G = kGroupDefault;
  auto wadd = [&](int k, unsigned v) {   // (watch: host-pinned progress counters, system scope)
    if (watch) __hip_atomic_fetch_add(&watch[k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  };
  __shared__ int s_t;
  if (threadIdx.x == 0) s_t = (int)atomicAdd(&sctl[0], 1u);
  __syncthreads();
  const int t = s_t;
  if (t == (int)gridDim.x - 1 && threadIdx.x == 0)   // every ticket taken: ready for the next launch
    __hip_atomic_store(&sctl[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t < nbK) {
    knn_block<G, kUnrollDefault, 3>(st, x0_dev, E, S, nbE, nbK, t, d_me, d_ms, rank, world);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (t == 0) __hip_atomic_store(&sctl[kSplitResetWord], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // the chunks this block's rounds covered (knn_block's query mapping)
      const bool edge = t < nbE;
      const CorrArgs& A = edge ? E : S;
      const int nb = edge ? nbE : nbK - nbE;
      int p = edge ? t : t - nbE;
      const int nq = min(*A.d_n, A.n_ub);
      const int nact = min(nb, (int)(((long long)nq * G + kTB - 1) / kTB));
      if (p < nact) p = xcd_block(p, nact);
      const int ngroups = nb * (kTB / G);
      for (int i0 = 0; i0 < nq; i0 += ngroups) {
        const int q = i0 + p * (kTB / G);
        if (q >= nq) break;
        atomicAdd(&sctl[kSplitChunk0 + (edge ? 0 : gE) + q / kTB], 1u);
        wadd(1, 1u);
      }
      wadd(0, 1u);
    }
    return;
  }
  const int gb = t - nbK;   // geometry block
  const bool edge = gb < gE;
  const CorrArgs& A = edge ? E : S;
  const int nq = min(*A.d_n, A.n_ub);
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    wadd(2, 1u);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool ok = true;
    while (__hip_atomic_load(&sctl[kSplitResetWord], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) { ok = false; break; }   // 1 s (never expected)
      __builtin_amdgcn_s_sleep(2);
    }
    // the chunks of this block: edge chunk gb; surf chunks sb, sb + kSurfGeomBlocks, ...
    const int c0 = edge ? gb : gb - gE;
    for (int c = c0; ok && c < (nq + kTB - 1) / kTB; c += edge ? (nq + kTB - 1) / kTB : kSurfGeomBlocks) {
      const unsigned need = (unsigned)((min(nq, (c + 1) * kTB) - c * kTB + G - 1) / G);
      unsigned* w = &sctl[kSplitChunk0 + (edge ? 0 : gE) + c];
      while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) { ok = false; break; }
        __builtin_amdgcn_s_sleep(2);
      }
      // (the only consumer: zero for the next launch, ordered by the kernel boundary)
      __hip_atomic_store(w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!ok) atomicOr(&sctl[kSplitResetWord + 1], 1u);   // (a wait timed out: never expected; the fits are skipped)
    wadd(ok ? 3 : 4, 1u);
    if (!ok && watch) {
      watch[5] = __hip_atomic_load(&sctl[kSplitResetWord], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      watch[6] = epoch;
      watch[7] = (unsigned)gb;
      const int c = edge ? gb : gb - gE;
      if (c < (nq + kTB - 1) / kTB) watch[8] = __hip_atomic_load(&sctl[kSplitChunk0 + (edge ? 0 : gE) + c], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
      watch[9] = (unsigned)nq;
    }
    s_ok = ok;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (!s_ok) return;   // (block-uniform; never on stale neighbours)
  geom_block<R>(st, E, S, gE, gb, gpart, gmat, gcnt);
}
#endif

// Algorithmic traffic of one launch of the search kernel (knn_kernel; SURVEY.md §8 d): every map
// cell any query scans is streamed once (16 B per map point: the union over queries of the fine 3x3x3 block around
// the query's cell — level 0 — and of the coarse +-1 m stencil for the queries whose bit 1 says they needed stage 2
// — level 1), every query is read once (16 B) and writes its flag (1 B) and, with 5 neighbours, their coordinates
// (60 B) (counted at level 0).  Runs untimed, on a replay, only when profiling.
//
// The radius of a query's stage 2 (knn_group): 1, or with 5 points within 1 m in the fine block around the query's
// block (nb^3 fine cells), sqrt of the 5th-smallest float sq-distance among them times (1 + 1e-6) — recomputed here
// serially over the same fine cells with the same float arithmetic
__device__ double stage2_radius(const CorrArgs& A, int nb, float wx, float wy, float wz) {
  int qx, qy, qz, lx, ly, lz;
  fine_cell(wx, wy, wz, qx, qy, qz);
  knn_block_corner(nb, wx, wy, wz, qx, qy, qz, lx, ly, lz);
  float best[5] = {2.f, 2.f, 2.f, 2.f, 2.f};   // ascending
  int cnt = 0;
  for (int fz = lz; fz < lz + nb; ++fz)
    for (int fy = ly; fy < ly + nb; ++fy)
      for (int fx = lx; fx < lx + nb; ++fx) {
        const unsigned long long key = cell_key(fx >> 1, fy >> 1, fz >> 1);
        unsigned h = coarse_slot(key, A.bits);
        while (A.coarse[h].key != key && A.coarse[h].key != kEmptyKey) h = (h + 1) & A.mask;
        const CoarseCell& c = A.coarse[h];
        if (c.key != key) continue;
        const int sub = (fx & 1) | ((fy & 1) << 1) | ((fz & 1) << 2);
        int start = c.start;
        for (int k = 0; k < sub; ++k) start += c.sub[k];
        for (int j = 0; j < c.sub[sub]; ++j) {
          const float4 m = A.gpts[start + j];
          float dd = 0.0f, df = wx - m.x;
          dd += df * df;
          df = wy - m.y;
          dd += df * df;
          df = wz - m.z;
          dd += df * df;
          if (!(dd < 1.0f)) continue;
          ++cnt;
          for (int k = 0; k < 5; ++k)
            if (dd < best[k]) {
              const float tmp = best[k];
              best[k] = dd;
              dd = tmp;
            }
        }
      }
  return cnt >= 5 ? fmin(1.0, sqrt((double)best[4]) * (1.0 + 1e-6)) : 1.0;
}

__global__ __launch_bounds__(kTB) void knn_traffic(const LMState* __restrict__ st, CorrArgs A, int rank,
                                                   int world, int level, int nb,
                                                   unsigned long long* __restrict__ set,
                                                   unsigned set_mask, int set_bits,
                                                   unsigned long long* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= A.n_ub) return;
  const int n = *A.d_n;
  const int lo = (int)(((long long)n * rank) / world), hi = (int)(((long long)n * (rank + 1)) / world);
  if (i < lo || i >= hi) return;
  const int f = A.valid[i];
  if (level == 1 && !(f & 2)) return;
  const PointRec pr = A.q[i];
  float wx, wy, wz;
  associate_to_map(st->x, pr.x, pr.y, pr.z, wx, wy, wz);
  // the search kernel's own bytes: query (16 B) + flag (1 B) + the neighbours' coordinates it hands to the
  // geometry pass (5 x 12 B, for the queries with 5 neighbours: bit 2 after the geometry pass)
  unsigned long long bytes = level ? 0ull : 16ull + 1ull + ((f & 4) ? 60ull : 0ull);
  int x0, y0, z0, x1, y1, z1;
  if (level) {
    const double r = stage2_radius(A, nb, wx, wy, wz);
    x0 = (int)floor((double)wx - r); x1 = (int)floor((double)wx + r);
    y0 = (int)floor((double)wy - r); y1 = (int)floor((double)wy + r);
    z0 = (int)floor((double)wz - r); z1 = (int)floor((double)wz + r);
  } else {
    int qx, qy, qz;
    fine_cell(wx, wy, wz, qx, qy, qz);
    knn_block_corner(nb, wx, wy, wz, qx, qy, qz, x0, y0, z0);
    x1 = x0 + nb - 1; y1 = y0 + nb - 1; z1 = z0 + nb - 1;
  }
  for (int z = z0; z <= z1; ++z)
    for (int y = y0; y <= y1; ++y)
      for (int x = x0; x <= x1; ++x) {
        const unsigned long long k = cell_key(x, y, z);
        const int cnt = level ? grid_lookup(A.coarse, k, A.bits, A.mask).y : fine_count(A, x, y, z);
        if (cnt == 0) continue;
        unsigned h = hash_slot64(k, set_bits);
        for (;;) {
          const unsigned long long prev = atomicCAS(&set[h], kEmptyKey, k);
          if (prev == kEmptyKey) { bytes += 16ull * (unsigned long long)cnt; break; }
          if (prev == k) break;
          h = (h + 1) & set_mask;
        }
      }
  if (bytes) atomicAdd(out, bytes);
}


__global__ void lm_init_dev(LMState* st, X7 x0, const double* __restrict__ x0_dev) {
  if (threadIdx.x != 0) return;
  if (x0_dev) {
    x0.set = 1;
#pragma unroll
    for (int k = 0; k < 7; ++k) x0.v[k] = x0_dev[k];
  }
  lm_reset(st, x0);
}

}  // namespace
__device__ __forceinline__ void gather_block(const LMState* __restrict__ lm, const int* __restrict__ dcnt,
                                             const int* __restrict__ mapE_count, const int* __restrict__ mapS_count,
                                             const int* __restrict__ fe_status,
                                             const unsigned long long* __restrict__ prof,
                                             UpdateStatus* __restrict__ out, OdomDev* __restrict__ s, int mode,
                                             unsigned seq);
namespace {

__global__ __launch_bounds__(kTB) void deskew_bridge(const LMState* __restrict__ st, OdomDev* __restrict__ s,
                                                     double period, PointRec* __restrict__ edge,
                                                     const int* __restrict__ d_ne, int ne_ub,
                                                     PointRec* __restrict__ surf, const int* __restrict__ d_ns,
                                                     int ns_ub, int aliased, GatherArgs g, float* __restrict__ vpart,
                                                     unsigned* __restrict__ vctl) {
  const bool lead = blockIdx.x == 0 && blockIdx.y == 0;
  if (g.out && lead) gather_block(st, g.dcnt, g.mapE_count, g.mapS_count, g.fe_status, nullptr, g.out, s, 0, g.seq);
  double x1[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) x1[k] = st->x[k];
  const double* t0 = s->last_odom.t;   // the pose before the first call (read-only in this launch)
  // GetVelocity (include/odomEstimationClass.h:78): (odom.translation() - last_odom.translation()) / scan_period
  const double vx = (x1[4] - t0[0]) / period, vy = (x1[5] - t0[1]) / period, vz = (x1[6] - t0[2]) / period;
  const int ne = min(*d_ne, ne_ub);
  if (vpart) {
    // fused with the next VoxelGrids' bounding-box stage: blockIdx.y = the cloud (0 edge, 1 surf), partial
    // blockIdx.x of its min / max over the compensated coordinates (edge != surf)
    // (the edge cloud over blocks 1 .. n-1: block (0, 0) publishes call 1's status and forms the prediction, and
    // stores an empty box into the edge cloud's partial slot n-1)
    const int job = (int)blockIdx.y;
    PointRec* __restrict__ c = job ? surf : edge;
    const int n = job ? min(*d_ns, ns_ub) : ne;
    const int nb = job ? (int)gridDim.x : (int)gridDim.x - 1;
    const int bx = job ? (int)blockIdx.x : (int)blockIdx.x - 1;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = bx * blockDim.x + threadIdx.x; bx >= 0 && i < n; i += nb * blockDim.x) {
      PointRec& p = c[i];   // CompensateVelocity: p += v * time, double -> float
      const double t = p.time;
      const float x = (float)((double)p.x + vx * t), y = (float)((double)p.y + vy * t), z = (float)((double)p.z + vz * t);
      p.x = x;
      p.y = y;
      p.z = z;
      mn[0] = fminf(mn[0], x); mn[1] = fminf(mn[1], y); mn[2] = fminf(mn[2], z);
      mx[0] = fmaxf(mx[0], x); mx[1] = fmaxf(mx[1], y); mx[2] = fmaxf(mx[2], z);
    }
    vox_partial_store(mn, mx, job, bx >= 0 ? bx : nb, vpart);
    if (lead) radix_ctl_zero(vctl, threadIdx.x, blockDim.x);
  } else {
    // aliased (edge and surf are one cloud): the reference's two CompensateVelocity calls (src/odomEstimationClass.cpp:
    // 42-43) shift every point twice, one after the other, so one thread applies both shifts to its point
    const int ns = aliased ? 0 : min(*d_ns, ns_ub);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ne + ns; i += gridDim.x * blockDim.x) {
      PointRec& p = i < ne ? edge[i] : surf[i - ne];   // CompensateVelocity: p += v * time, double -> float
      const double t = p.time;
      float x = (float)((double)p.x + vx * t), y = (float)((double)p.y + vy * t), z = (float)((double)p.z + vz * t);
      if (aliased) {
        x = (float)((double)x + vx * t);
        y = (float)((double)y + vy * t);
        z = (float)((double)z + vz * t);
      }
      p.x = x;
      p.y = y;
      p.z = z;
    }
  }
  if (lead && threadIdx.x == 0) {
    // the first call's writeback (:114-116) and the second call's prediction (:62-71): odom1 (last^-1 odom1)
    const Pose odom1 = params_to_pose(x1);
    const Pose pred = pose_mul(odom1, pose_mul(pose_inverse(s->last_odom), odom1));
    s->mid = odom1;
    pose_to_params(pred, s->x0[1]);
  }
}

__global__ void odom_dev_init(OdomDev* s) {
  if (threadIdx.x != 0) return;
  s->odom = pose_identity();
  s->last_odom = pose_identity();
  s->mid = pose_identity();
  s->kf = pose_identity();
  s->kf_count = 0;
  s->kf_flag = 0;
  s->failed = 0;
  pose_to_params(pose_identity(), s->x0[0]);
  pose_to_params(pose_identity(), s->x0[1]);
}

__global__ void odom_predict(OdomDev* s) {
  if (threadIdx.x == 0) odom_predict_step(s);
}

}  // namespace

// ===================================================================================== launchers
void deskew_bridge_launch(const LMState* d_st, OdomDev* s, double scan_period, PointRec* edge, const int* d_ne,
                          int ne_ub, PointRec* surf, const int* d_ns, int ns_ub, hipStream_t stream,
                          const GatherArgs& gather, const VoxelFused* vf) {
  const int aliased = edge == surf ? 1 : 0;
  if (vf && !aliased) {
    hipLaunchKernelGGL(deskew_bridge, dim3(kVoxMinMaxBlocks, 2), dim3(kTB), 0, stream, d_st, s, scan_period, edge, d_ne,
                       ne_ub, surf, d_ns, ns_ub, 0, gather, vf->partials, vf->ctl);
  } else {
    const unsigned nb = std::max(1u, std::min(div_up(std::max(ne_ub + ns_ub, 1), kTB), 1024u));
    hipLaunchKernelGGL(deskew_bridge, dim3(nb), dim3(kTB), 0, stream, d_st, s, scan_period, edge, d_ne, ne_ub, surf,
                       d_ns, ns_ub, aliased, gather, nullptr, nullptr);
  }
  FLOAM_LAUNCH_CHECK();
}

// KeyFrameUpdate(pose) (odomEstimationClass.cpp:320-343): a keyframe iff it is the process-wide first call (`first`,
// Q6), there is no keyframe yet, or the pose moved > 0.07 m or turned > 2 deg from the last keyframe; the last three
// keyframes are kept (only the last is ever read).  The result also gates the device map update (kf_flag).
__device__ __forceinline__ bool keyframe_decide(OdomDev* __restrict__ s, const Pose& pose, bool first) {
  bool key = true;
  if (!first && s->kf_count > 0) {
    const Pose delta = pose_mul(pose_inverse(s->kf), pose);
    const double dm = sqrt(delta.t[0] * delta.t[0] + delta.t[1] * delta.t[1] + delta.t[2] * delta.t[2]);
    const double dr = rotation_angle(delta.R);
    key = dm > 0.07 || dr > 2 * M_PI / 180.0;
  }
  if (key) {
    s->kf = pose;
    s->kf_count = min(s->kf_count + 1, 3);
  }
  s->kf_flag = key ? 1 : 0;
  return key;
}

// One D2H per update: LM state + query / map counts (+ profiling bytes) gathered into one block.
// Called by every thread of one block.
__device__ __forceinline__ void gather_block(const LMState* __restrict__ lm, const int* __restrict__ dcnt,
                                             const int* __restrict__ mapE_count, const int* __restrict__ mapS_count,
                                             const int* __restrict__ fe_status,
                                             const unsigned long long* __restrict__ prof,
                                             UpdateStatus* __restrict__ out, OdomDev* __restrict__ s, int mode,
                                             unsigned seq) {
  constexpr int kWords = kStateWords;
  const unsigned* src = reinterpret_cast<const unsigned*>(lm);
  unsigned* dst = reinterpret_cast<unsigned*>(&out->lm);
  for (int w = threadIdx.x; w < kWords; w += blockDim.x) dst[w] = src[w];
  if (threadIdx.x == 0) {
    out->counts[0] = dcnt[0];
    out->counts[1] = dcnt[1];
    out->counts[2] = *mapE_count;
    out->counts[3] = *mapS_count;
    out->fe_status = fe_status ? *fe_status : 0;
    out->prof[0] = prof ? prof[0] : 0ull;
    out->prof[1] = prof ? prof[1] : 0ull;
    out->kf_flag = 0;
    s->kf_flag = 0;   // (the map update's gate)
    if (lm->n_res < 0 || lm->xfail) s->failed = 1;   // an abandoned solve: its pose is not taken, no keyframe, no
    if (!s->failed) {                   // map update — for this update and every later one; the host raises it
      if (mode & GATHER_FINISH) {
        if (mode & GATHER_AFTER_MID) s->last_odom = s->mid;
        s->odom = params_to_pose(lm->x);   // x == the prediction when the solve did not run (gate, no residuals)
      }
      if (mode & GATHER_KEYFRAME) out->kf_flag = keyframe_decide(s, s->odom, (mode & GATHER_KEYFRAME_FIRST) != 0);
    }
    out->odom = s->odom;
    out->last_odom = s->last_odom;
  }
  // the serial number last, after every other word of the slot is visible to the host: the host polls it instead
  // of waiting on an event (an event record is a barrier packet that costs the stream ~10 us per update)
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(&out->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void gather_status(const LMState* __restrict__ lm, const int* __restrict__ dcnt,
                              const int* __restrict__ mapE_count, const int* __restrict__ mapS_count,
                              const int* __restrict__ fe_status, const unsigned long long* __restrict__ prof,
                              UpdateStatus* __restrict__ out, OdomDev* __restrict__ s, int mode, unsigned seq,
                              VoxelJobDev A,
                              VoxelJobDev B, float* __restrict__ vpart, unsigned* __restrict__ vctl,
                              GridClearDev gcE, GridClearDev gcS, MergeCheck mc) {
  const bool lead = blockIdx.x == 0 && blockIdx.y == 0;
  if (lead) gather_block(lm, dcnt, mapE_count, mapS_count, fe_status, prof, out, s, mode, seq);
  if (!vpart) return;
  if (blockIdx.y < 2) {   // the map update's bounding-box stage (its keyframe gate is applied by the launches after)
    if (lead) {
      radix_ctl_zero(vctl, threadIdx.x, blockDim.x);
      if (mc.ctl && threadIdx.x < kMergeCtlWords) mc.ctl[threadIdx.x] = 0;
    }
    // job A's points over blocks 1 .. n-1 only: block (0, 0) publishes the status (host memory, system-scope fence)
    // and would finish last with a share of points on top; it stores an empty box into the partial slot n-1
    const int job = (int)blockIdx.y;
    const int nb = job == 0 ? (int)gridDim.x - 1 : (int)gridDim.x;
    const int b = job == 0 ? (int)blockIdx.x - 1 : (int)blockIdx.x;
    if (b < 0) {
      float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
      vox_partial_store(mn, mx, 0, nb, vpart);
    } else if (mc.flags) {   // + the incremental merge's checks (mapmerge.hip)
      mm_minmax_block(job == 0 ? A : B, job, b, nb, vpart, mc);
    } else {
      vox_minmax_block(job == 0 ? A : B, job, b, nb, vpart);
    }
  } else if (gcE.coarse) {   // blocks of their own: the next grid builds' clears (this update's kNN launches are done)
    grid_clear_part(blockIdx.y == 2 ? gcE : gcS, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x,
                    blockIdx.x == 0 && threadIdx.x == 0);
  }
}

void gather_status_launch(const LMState* lm, const int* dcnt, const int* mapE_count, const int* mapS_count,
                          const int* fe_status, const unsigned long long* prof, UpdateStatus* out, OdomDev* s,
                          int mode, unsigned seq, hipStream_t st, const VoxelFused* vf, const GridClearDev* gc) {
  const GridClearDev none{};
  if (vf) {
    hipLaunchKernelGGL(gather_status, dim3(kVoxMinMaxBlocks, gc ? 4 : 2), dim3(256), 0, st, lm, dcnt, mapE_count, mapS_count,
                       fe_status, prof, out, s, mode, seq, vf->A, vf->B, vf->partials, vf->ctl, gc ? gc[0] : none,
                       gc ? gc[1] : none, vf->mc);
  } else {
    hipLaunchKernelGGL(gather_status, dim3(1), dim3(256), 0, st, lm, dcnt, mapE_count, mapS_count, fe_status, prof,
                       out, s, mode, seq, VoxelJobDev{}, VoxelJobDev{}, nullptr, nullptr, none, none, MergeCheck{});
  }
  FLOAM_LAUNCH_CHECK();
}

void odom_dev_init_launch(OdomDev* s, hipStream_t st) {
  hipLaunchKernelGGL(odom_dev_init, dim3(1), dim3(64), 0, st, s);
  FLOAM_LAUNCH_CHECK();
}

void odom_predict_launch(OdomDev* s, hipStream_t st) {
  hipLaunchKernelGGL(odom_predict, dim3(1), dim3(64), 0, st, s);
  FLOAM_LAUNCH_CHECK();
}

void lm_init_dev_launch(LMState* d_st, const double* x0_dev, hipStream_t st) {
  hipLaunchKernelGGL(lm_init_dev, dim3(1), dim3(64), 0, st, d_st, X7{}, x0_dev);
  FLOAM_LAUNCH_CHECK();
}

// KeyFrameUpdate(pose) (src/odomEstimationClass.cpp:320-343) standalone: the method of the reference's public header
// (include/odomEstimationClass.h:80) on an explicit pose
__global__ void keyframe_update_kernel(OdomDev* __restrict__ s, const double* __restrict__ x, int first,
                                       int* __restrict__ flag) {
  if (threadIdx.x != 0) return;
  *flag = keyframe_decide(s, params_to_pose(x), first != 0) ? 1 : 0;
}

void keyframe_update_launch(OdomDev* s, const double* x_dev, int first, int* flag, hipStream_t st) {
  hipLaunchKernelGGL(keyframe_update_kernel, dim3(1), dim3(64), 0, st, s, x_dev, first, flag);
  FLOAM_LAUNCH_CHECK();
}

static void corr_args(const QuerySet& qe, const Grid& ge, CorrSet& ce, const QuerySet& qs, const Grid& gs,
                      CorrSet& cs, CorrArgs& E, CorrArgs& S) {
  ce.reserve(std::max(qe.n_ub, 1), EDGE_FIELDS);
  cs.reserve(std::max(qs.n_ub, 1), SURF_FIELDS);
  const bool rec = grid_noxyz();   // (diagnostic: neighbour coordinates from the map records, 2 float4s each)
  E = CorrArgs{qe.pts, qe.d_n, qe.n_ub, ge.pts.p, ge.coarse.p, ge.bits, ge.mask,
               rec ? reinterpret_cast<const float4*>(ge.src) : ge.xyz.p, rec ? 2 : 1, ce.rec.p,
               ce.valid.p, ce.nnxyz.p, ce.trace ? ce.nnidx.p : nullptr, ce.trace ? ce.nnsqd.p : nullptr, ce.cap};
  S = CorrArgs{qs.pts, qs.d_n, qs.n_ub, gs.pts.p, gs.coarse.p, gs.bits, gs.mask,
               rec ? reinterpret_cast<const float4*>(gs.src) : gs.xyz.p, rec ? 2 : 1, cs.rec.p,
               cs.valid.p, cs.nnxyz.p, cs.trace ? cs.nnidx.p : nullptr, cs.trace ? cs.nnsqd.p : nullptr, cs.cap};
}

void knn_launch(LMState* d_st, const double* x0_dev, const QuerySet& qe, const Grid& ge, CorrSet& ce,
                const QuerySet& qs, const Grid& gs, CorrSet& cs, const int* d_me, const int* d_ms, int rank, int world,
                hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
  CorrArgs E, S;
  corr_args(qe, ge, ce, qs, gs, cs, E, S);
  if (qe.n_ub <= 0 && qs.n_ub <= 0) {   // nothing to search: still start the solve
    hipLaunchKernelGGL(lm_init_dev, dim3(1), dim3(64), 0, st, d_st, X7{}, x0_dev);
    FLOAM_LAUNCH_CHECK();
    return;
  }
  constexpr int G = kGroupDefault;
  const int nE = qe.grid_hint > 0 ? std::min(qe.grid_hint, qe.n_ub) : qe.n_ub;
  const int nS = qs.grid_hint > 0 ? std::min(qs.grid_hint, qs.n_ub) : qs.n_ub;
  const unsigned nbE = std::min(div_up((size_t)std::max(nE, 1) * G, kTB), 4096u);
  const unsigned nbS = std::min(div_up((size_t)std::max(nS, 1) * G, kTB), 8192u);
  // (diagnostic, FLOAM_KNN_LDS_PAD=bytes: dynamic LDS that caps the blocks per CU — the search at the occupancy a
  // launch that also ran the geometry fits would have: 118 VGPRs -> 4 waves per SIMD = 40 KB of LDS a block)
  static const unsigned pad = FLOAM_DIAG_ENV("FLOAM_KNN_LDS_PAD") ? (unsigned)std::atoi(FLOAM_DIAG_ENV("FLOAM_KNN_LDS_PAD")) : 0u;
#ifdef FLOAM_DIAG
  static const bool lds = FLOAM_DIAG_ENV("FLOAM_KNN_LDS") != nullptr;   // (the LDS-staged stage 1, profiles/r06c)
  if (lds)
    hipExtLaunchKernelGGL((knn_kernel_lds<G, kUnrollDefault>), dim3(nbE + nbS), dim3(kTB), 0, st, ev0, ev1, 0,
                          d_st, x0_dev, E, S, (int)nbE, d_me, d_ms, rank, world);
  else
#endif
  if (ev0 || ev1)
    hipExtLaunchKernelGGL((knn_kernel<G, kUnrollDefault, 6, 3>), dim3(nbE + nbS), dim3(kTB), pad, st, ev0, ev1, 0,
                          d_st, x0_dev, E, S, (int)nbE, d_me, d_ms, rank, world);
  else
    hipLaunchKernelGGL((knn_kernel<G, kUnrollDefault, 6, 3>), dim3(nbE + nbS), dim3(kTB), pad, st, d_st, x0_dev, E, S,
                       (int)nbE, d_me, d_ms, rank, world);
  FLOAM_LAUNCH_CHECK();
}

bool knn_geom_split_launch(LMState* d_st, const double* x0_dev, const QuerySet& qe, const Grid& ge, CorrSet& ce,
                           const QuerySet& qs, const Grid& gs, CorrSet& cs, const int* d_me, const int* d_ms,
                           int rank, int world, bool gram, bool fp32, LMBuffers& b, hipStream_t st, hipEvent_t ev0,
                           hipEvent_t ev1) {
#ifdef FLOAM_DIAG
  static const bool on = FLOAM_DIAG_ENV("FLOAM_KNN_SPLIT") != nullptr;
  if (!on || fp32 || qe.n_ub <= 0 || qs.n_ub <= 0) return false;
  constexpr int G = kGroupDefault;
  CorrArgs E, S;
  corr_args(qe, ge, ce, qs, gs, cs, E, S);
  const int nE = qe.grid_hint > 0 ? std::min(qe.grid_hint, qe.n_ub) : qe.n_ub;
  const int nS = qs.grid_hint > 0 ? std::min(qs.grid_hint, qs.n_ub) : qs.n_ub;
  const unsigned nbE = std::min(div_up((size_t)std::max(nE, 1) * G, kTB), 4096u);
  const unsigned nbS = std::min(div_up((size_t)std::max(nS, 1) * G, kTB), 8192u);
  const unsigned gE = div_up(std::max(qe.n_ub, 1), kTB);
  const int chunks = 2 + (int)gE + (int)div_up(std::max(qs.n_ub, 1), kTB);
  static DevBuf<unsigned> sctl;   // (one prototype launch in flight per process: the diagnostic measurements)
  static unsigned epoch = 0;
  if ((size_t)(kSplitChunk0 + chunks) > sctl.cap) {
    sctl.reserve((size_t)(kSplitChunk0 + chunks));
    FLOAM_HIP(hipMemsetAsync(sctl.p, 0, sizeof(unsigned) * sctl.cap, st));
  }
  if (gram) b.reserve(st);
  // (FLOAM_SPLIT_WATCH=1: host-pinned progress counters, printed every 2 s by a watcher thread — kNN blocks published,
  // chunk adds, geometry blocks started / passed / timed out, and the words a timed-out block saw)
  static unsigned* watch = [] {
    if (!FLOAM_DIAG_ENV("FLOAM_SPLIT_WATCH")) return (unsigned*)nullptr;
    unsigned* w = nullptr;
    FLOAM_HIP(hipHostMalloc(reinterpret_cast<void**>(&w), 64 * sizeof(unsigned), hipHostMallocCoherent));
    std::memset(w, 0, 64 * sizeof(unsigned));
    std::thread([w] {
      for (;;) {
        std::this_thread::sleep_for(std::chrono::seconds(2));
        std::fprintf(stderr, "[split watch] knn published %u, chunk adds %u, geometry started %u passed %u timed out %u; "
                     "last timeout: reset word %u epoch %u block %u count %u nq %u\n", w[0], w[1], w[2], w[3], w[4],
                     w[5], w[6], w[7], w[8], w[9]);
      }
    }).detach();
    return w;
  }();
  hipExtLaunchKernelGGL(knn_geom_split<double>, dim3(nbE + nbS + gE + kSurfGeomBlocks), dim3(kTB), 0, st, ev0, ev1, 0,
                        d_st, x0_dev, E, S, (int)nbE, (int)(nbE + nbS), (int)gE, d_me, d_ms, rank, world,
                        gram ? b.gpart.p : nullptr, gram ? b.gmat.p : nullptr, b.gcnt.p, sctl.p, ++epoch, watch);
  FLOAM_LAUNCH_CHECK();
  return true;
#else
  (void)d_st; (void)x0_dev; (void)qe; (void)ge; (void)ce; (void)qs; (void)gs; (void)cs; (void)d_me; (void)d_ms;
  (void)rank; (void)world; (void)gram; (void)fp32; (void)b; (void)st; (void)ev0; (void)ev1;
  return false;
#endif
}

void geom_launch(LMState* d_st, const QuerySet& qe, CorrSet& ce, const QuerySet& qs, CorrSet& cs, bool gram,
                 bool fp32, LMBuffers& b, hipStream_t st) {
  if (qe.n_ub <= 0 && qs.n_ub <= 0) return;
  if (gram) b.reserve(st);
  Grid none;
  CorrArgs E, S;
  corr_args(qe, none, ce, qs, none, cs, E, S);
  const unsigned gE = div_up(std::max(qe.n_ub, 1), kTB);
  double* gpart = gram ? b.gpart.p : nullptr;
  double* gmat = gram ? b.gmat.p : nullptr;
  if (fp32)
    hipLaunchKernelGGL(geom_kernel<float>, dim3(gE + kSurfGeomBlocks), dim3(kTB), 0, st, d_st, E, S, (int)gE,
                       gpart, gmat, b.gcnt.p);
  else
    hipLaunchKernelGGL(geom_kernel<double>, dim3(gE + kSurfGeomBlocks), dim3(kTB), 0, st, d_st, E, S, (int)gE,
                       gpart, gmat, b.gcnt.p);
  FLOAM_LAUNCH_CHECK();
}

// (diagnostic) every XCD's L2 refilled with other lines: a grid-stride read of a buffer 16x the size of one XCD's
// L2 by every block, so that the next launch finds none of its lines cached (FETCH_SIZE then counts its cold fetches)
__global__ __launch_bounds__(kTB) void l2_evict(const float4* __restrict__ buf, size_t n, float* __restrict__ sink) {
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * kTB + threadIdx.x; i < n; i += (size_t)gridDim.x * kTB) acc += buf[i].x;
  if (acc == 1234.5f) sink[0] = acc;   // (never: keeps the loads)
}

void knn_waves_dump() {
#ifdef FLOAM_KNN_WAVES
  const char* path = std::getenv("FLOAM_KNN_WAVES");
  if (!path) return;
  static unsigned long long h[kKnnWaveRows][2];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_knn_waves), sizeof(h)) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  if (FILE* f = std::fopen(path, "wb")) {
    std::fwrite(h, sizeof(h), 1, f);
    std::fclose(f);
  }
#endif
}

void geom_stamps_print() {
#ifdef FLOAM_GEOM_STAMPS
  static unsigned long long h[kGeomStampBlocks][8];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_geom_blk), sizeof(h)) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  unsigned long long last = 0;   // the newest launch: rows that started within 50 us of the latest start
  for (int b = 0; b < kGeomStampBlocks; ++b) last = std::max(last, h[b][0]);
  unsigned long long t_min = ~0ull, t_end = 0;
  double sum[3][6] = {}, mx[3][6] = {};
  int n[3] = {0, 0, 0};
  for (int b = 0; b < kGeomStampBlocks; ++b) {
    if (!h[b][0] || h[b][0] + 5000 < last) continue;
    t_min = std::min(t_min, h[b][0]);
  }
  for (int b = 0; b < kGeomStampBlocks; ++b) {
    if (!h[b][0] || h[b][0] + 5000 < last) continue;
    const int r = (int)h[b][6];
    if (r < 0 || r > 2) continue;
    ++n[r];
    t_end = std::max(t_end, h[b][5]);
    const double v[6] = {(double)(h[b][0] - t_min), (double)(h[b][1] - h[b][0]), (double)(h[b][2] - h[b][1]),
                         (double)(h[b][3] - h[b][2]), (double)(h[b][4] - h[b][3]), (double)(h[b][5] - h[b][4])};
    for (int k = 0; k < 6; ++k) {
      sum[r][k] += v[k];
      mx[r][k] = std::max(mx[r][k], v[k]);
    }
  }
  const char* names[3] = {"edge", "surf", "surf (group reduce)"};
  for (int r = 0; r < 3; ++r) {
    if (!n[r]) continue;
    std::fprintf(stderr, "[geom stamps] %s, %d blocks, avg (max) us: start after the first %.2f (%.2f), loads %.2f (%.2f), "
                 "fit %.2f (%.2f), sums / Gram %.2f (%.2f), hand-off %.2f (%.2f), tail %.2f (%.2f)\n", names[r], n[r],
                 sum[r][0] / n[r] / 100, mx[r][0] / 100, sum[r][1] / n[r] / 100, mx[r][1] / 100, sum[r][2] / n[r] / 100,
                 mx[r][2] / 100, sum[r][3] / n[r] / 100, mx[r][3] / 100, sum[r][4] / n[r] / 100, mx[r][4] / 100,
                 sum[r][5] / n[r] / 100, mx[r][5] / 100);
  }
  std::fprintf(stderr, "[geom stamps] newest launch: first block start -> last block end %.2f us\n",
               t_end > t_min ? (double)(t_end - t_min) / 100 : 0.0);
#endif
}

void knn_stage_launch(LMState* d_st, const double* x0_dev, const QuerySet& qe, const Grid& ge, CorrSet& ce,
                      const QuerySet& qs, const Grid& gs, CorrSet& cs, const int* d_me, const int* d_ms, int rank,
                      int world, DevBuf<float4>& evict, hipStream_t st) {
  if (qe.n_ub <= 0 && qs.n_ub <= 0) return;
  constexpr size_t kEvict = (size_t)64 << 20;   // bytes
  if (!evict.p) {
    evict.reserve(kEvict / sizeof(float4) + 1);
    FLOAM_HIP(hipMemsetAsync(evict.p, 0, kEvict, st));
  }
  CorrArgs E, S;
  corr_args(qe, ge, ce, qs, gs, cs, E, S);
  constexpr int G = kGroupDefault;
  const int nE = qe.grid_hint > 0 ? std::min(qe.grid_hint, qe.n_ub) : qe.n_ub;
  const int nS = qs.grid_hint > 0 ? std::min(qs.grid_hint, qs.n_ub) : qs.n_ub;
  const unsigned nbE = std::min(div_up((size_t)std::max(nE, 1) * G, kTB), 4096u);
  const unsigned nbS = std::min(div_up((size_t)std::max(nS, 1) * G, kTB), 8192u);
  const dim3 g(nbE + nbS);
  auto flush = [&] {
    hipLaunchKernelGGL(l2_evict, dim3(2048), dim3(kTB), 0, st, evict.p, kEvict / sizeof(float4),
                       reinterpret_cast<float*>(evict.p) + kEvict / sizeof(float));
    FLOAM_LAUNCH_CHECK();
  };
  flush();
  hipLaunchKernelGGL((knn_kernel<G, kUnrollDefault, 6, 3, 1>), g, dim3(kTB), 0, st, d_st, x0_dev, E, S, (int)nbE,
                     d_me, d_ms, rank, world);
  flush();
  hipLaunchKernelGGL((knn_kernel<G, kUnrollDefault, 6, 3, 2>), g, dim3(kTB), 0, st, d_st, x0_dev, E, S, (int)nbE,
                     d_me, d_ms, rank, world);
  flush();
  hipLaunchKernelGGL((knn_kernel<G, kUnrollDefault, 6, 3, 3>), g, dim3(kTB), 0, st, d_st, x0_dev, E, S, (int)nbE,
                     d_me, d_ms, rank, world);
  flush();
  hipLaunchKernelGGL((knn_kernel<G, kUnrollDefault, 6, 3, 4>), g, dim3(kTB), 0, st, d_st, x0_dev, E, S, (int)nbE,
                     d_me, d_ms, rank, world);
  flush();   // (the real search follows, cold as well)
  FLOAM_LAUNCH_CHECK();
}

void knn_traffic_launch(const LMState* d_st, const QuerySet& q, const Grid& g, CorrSet& c, int rank, int world,
                        DevBuf<unsigned long long>& set, unsigned long long* d_bytes, hipStream_t st) {
  if (q.n_ub <= 0) return;
  int bits = 10;
  while ((1 << bits) < 64 * q.n_ub) ++bits;   // distinct occupied cells scanned (<= 27 per query)
  set.reserve((size_t)1 << bits);
  CorrArgs A, B;
  corr_args(q, g, c, q, g, c, A, B);
  for (int level = 0; level < 2; ++level) {
    FLOAM_HIP(hipMemsetAsync(set.p, 0xFF, sizeof(unsigned long long) << bits, st));
    hipLaunchKernelGGL(knn_traffic, dim3(div_up(q.n_ub, kTB)), dim3(kTB), 0, st, d_st, A, rank, world,
                       level, 3, set.p, (1u << bits) - 1u, bits, d_bytes);
    FLOAM_LAUNCH_CHECK();
  }
}

}  // namespace floam
