// Scan-to-map registration on gfx950: spatial-hash kNN correspondence search + fp64 line / plane geometry +
// analytic residuals / Jacobians + normal-equation reduction + on-device Levenberg-Marquardt control.
//
// Reference: src/odomEstimationClass.cpp:78-110 (kd-tree, Ceres problem), :126-135 (pointAssociateToMap),
// :144-196 (addEdgeCostFactor), :198-251 (addSurfCostFactor); src/lidarOptimization.cpp:12-140 (cost functions,
// SE3 Plus).  Ceres 1.13 TrustRegionMinimizer + LevenbergMarquardtStrategy semantics are restated in lm_control
// (see SURVEY.md §8 a-12 and oracle/odom.cpp for the CPU restatement).
#include <cfloat>
#include <cstdlib>
#include <climits>

#include "grid.hpp"
#include "odom_kernels.hpp"

namespace floam {

namespace {
constexpr int kTB = 256;
constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr unsigned kEvalBlocks = 128;   // LM evaluation grid (grid-stride over the device-resident slots)

// ===================================================================================== geometry (fp64)
// Eigen 3.3 SelfAdjointEigenSolver<Matrix3d>::compute and ColPivHouseholderQR<Matrix<double,5,3>>::solve restated
// for the device with the same algorithm and operation order as oracle/eigen_solvers.cpp.  Every array index is a
// compile-time constant (templates / full unrolling) so the solvers stay in VGPRs instead of scratch.
__device__ __forceinline__ double e_hypot(double x, double y) {
  const double ax = fabs(x), ay = fabs(y);
  double p, qp;
  if (ax > ay) { p = ax; qp = ay / p; } else { p = ay; qp = ax / p; }
  if (p == 0.0) return 0.0;
  return p * sqrt(1.0 + qp * qp);
}

// JacobiRotation<double>::makeGivens (real case)
__device__ __forceinline__ void make_givens(double p, double q, double& c, double& s) {
  if (q == 0.0) {
    c = p < 0.0 ? -1.0 : 1.0;
    s = 0.0;
  } else if (p == 0.0) {
    c = 0.0;
    s = q < 0.0 ? 1.0 : -1.0;
  } else if (fabs(p) > fabs(q)) {
    const double t = q / p;
    double u = sqrt(1.0 + t * t);
    if (p < 0.0) u = -u;
    c = 1.0 / u;
    s = -t * c;
  } else {
    const double t = p / q;
    double u = sqrt(1.0 + t * t);
    if (q < 0.0) u = -u;
    s = -1.0 / u;
    c = -t * s;
  }
}

// internal::tridiagonal_qr_step on rows/cols [S, E] of a 3x3 tridiagonal (Q column-major: Q[col][row])
template <int S, int E>
__device__ __forceinline__ void tridiag_qr_step(double (&d)[3], double (&e)[2], double (&Q)[3][3]) {
  const double td = (d[E - 1] - d[E]) * 0.5;
  const double ee = e[E - 1];
  double mu = d[E];
  if (td == 0.0) {
    mu -= fabs(ee);
  } else {
    const double e2 = e[E - 1] * e[E - 1];
    const double h = e_hypot(td, ee);
    if (e2 == 0.0) mu -= (ee / (td + (td > 0.0 ? 1.0 : -1.0))) * (ee / h);
    else mu -= e2 / (td + (td > 0.0 ? h : -h));
  }
  double x = d[S] - mu;
  double z = e[S];
#pragma unroll
  for (int k = S; k < E; ++k) {
    double c, s;
    make_givens(x, z, c, s);
    const double sdk = s * d[k] + c * e[k];
    const double dkp1 = s * e[k] + c * d[k + 1];
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
      const double xi = Q[k][i], yi = Q[k + 1][i];
      Q[k][i] = c * xi - s * yi;
      Q[k + 1][i] = s * xi + c * yi;
    }
  }
}

__device__ __forceinline__ void swap_d(double& a, double& b) {
  const double t = a;
  a = b;
  b = t;
}

// eigenvalues ascending in ev; u_top = eigenvector of the largest eigenvalue
__device__ void eig_sym3(const double (&A)[3][3], double (&ev)[3], double (&u_top)[3]) {
  double m00 = A[0][0], m10 = A[1][0], m11 = A[1][1], m20 = A[2][0], m21 = A[2][1], m22 = A[2][2];
  double scale = fabs(m00);
  scale = fmax(scale, fabs(m10));
  scale = fmax(scale, fabs(m11));
  scale = fmax(scale, fabs(m20));
  scale = fmax(scale, fabs(m21));
  scale = fmax(scale, fabs(m22));
  if (scale == 0.0) scale = 1.0;
  m00 /= scale; m10 /= scale; m11 /= scale; m20 /= scale; m21 /= scale; m22 /= scale;
  double d[3], e[2], Q[3][3];
  d[0] = m00;
  const double v1norm2 = m20 * m20;
  if (v1norm2 <= DBL_MIN) {
    d[1] = m11; d[2] = m22; e[0] = m10; e[1] = m21;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int r = 0; r < 3; ++r) Q[c][r] = (c == r) ? 1.0 : 0.0;
  } else {
    const double beta = sqrt(m10 * m10 + v1norm2);
    const double invBeta = 1.0 / beta;
    const double m01 = m10 * invBeta;
    const double m02 = m20 * invBeta;
    const double q = 2.0 * m01 * m21 + m02 * (m22 - m11);
    d[1] = m11 + m02 * q;
    d[2] = m22 - m02 * q;
    e[0] = beta;
    e[1] = m21 - m01 * q;
    Q[0][0] = 1; Q[0][1] = 0; Q[0][2] = 0;
    Q[1][0] = 0; Q[1][1] = m01; Q[1][2] = m02;
    Q[2][0] = 0; Q[2][1] = m02; Q[2][2] = -m01;
  }
  const double precision = 2.0 * DBL_EPSILON;
  int end = 2, start = 0, iter = 0;
  while (end > 0) {
    if (start <= 0 && 0 < end)
      if (fabs(e[0]) <= (fabs(d[0]) + fabs(d[1])) * precision || fabs(e[0]) <= DBL_MIN) e[0] = 0.0;
    if (start <= 1 && 1 < end)
      if (fabs(e[1]) <= (fabs(d[1]) + fabs(d[2])) * precision || fabs(e[1]) <= DBL_MIN) e[1] = 0.0;
    if (end == 2 && e[1] == 0.0) end = 1;
    if (end == 1 && e[0] == 0.0) end = 0;
    if (end <= 0) break;
    if (++iter > 90) break;
    start = (end == 2 && e[0] != 0.0) ? 0 : end - 1;
    if (end == 2) {
      if (start == 0) tridiag_qr_step<0, 2>(d, e, Q);
      else tridiag_qr_step<1, 2>(d, e, Q);
    } else {
      tridiag_qr_step<0, 1>(d, e, Q);
    }
  }
  // ascending selection sort (first minimum), swapping eigenvector columns
  int k = 0;
  if (d[1] < d[k]) k = 1;
  if (d[2] < d[k]) k = 2;
  if (k == 1) {
    swap_d(d[0], d[1]);
#pragma unroll
    for (int r = 0; r < 3; ++r) swap_d(Q[0][r], Q[1][r]);
  } else if (k == 2) {
    swap_d(d[0], d[2]);
#pragma unroll
    for (int r = 0; r < 3; ++r) swap_d(Q[0][r], Q[2][r]);
  }
  if (d[2] < d[1]) {
    swap_d(d[1], d[2]);
#pragma unroll
    for (int r = 0; r < 3; ++r) swap_d(Q[1][r], Q[2][r]);
  }
  ev[0] = d[0] * scale; ev[1] = d[1] * scale; ev[2] = d[2] * scale;
  u_top[0] = Q[2][0]; u_top[1] = Q[2][1]; u_top[2] = Q[2][2];
}

// Householder on column K of a column-major 5x3 (qr[col][row]): makeHouseholderInPlace + apply to columns > K
template <int K>
__device__ __forceinline__ void plane_hh(double (&qr)[3][5], double (&hc)[3]) {
  double tail = 0.0;
#pragma unroll
  for (int i = K + 1; i < 5; ++i) tail += qr[K][i] * qr[K][i];
  const double c0 = qr[K][K];
  double tau, beta;
  if (tail <= DBL_MIN) {
    tau = 0.0;
    beta = c0;
#pragma unroll
    for (int i = K + 1; i < 5; ++i) qr[K][i] = 0.0;
  } else {
    beta = sqrt(c0 * c0 + tail);
    if (c0 >= 0.0) beta = -beta;
#pragma unroll
    for (int i = K + 1; i < 5; ++i) qr[K][i] = qr[K][i] / (c0 - beta);
    tau = (beta - c0) / beta;
  }
  hc[K] = tau;
  qr[K][K] = beta;
  if (tau != 0.0) {
#pragma unroll
    for (int j = K + 1; j < 3; ++j) {
      double tmp = 0.0;
#pragma unroll
      for (int r = K + 1; r < 5; ++r) tmp += qr[K][r] * qr[j][r];
      tmp += qr[j][K];
      qr[j][K] -= tau * tmp;
#pragma unroll
      for (int r = K + 1; r < 5; ++r) qr[j][r] -= tau * qr[K][r] * tmp;
    }
  }
}

template <int K>
__device__ __forceinline__ void plane_pivot_step(double (&qr)[3][5], double (&hc)[3], double (&nu)[3], double (&nd)[3],
                                                 int (&tr)[3], int& nz, double threshold_helper) {
  int big = K;
#pragma unroll
  for (int j = K + 1; j < 3; ++j)
    if (nu[j] > nu[big == 0 ? 0 : (big == 1 ? 1 : 2)]) big = j;
  double nb = nu[K];
#pragma unroll
  for (int j = K + 1; j < 3; ++j)
    if (big == j) nb = nu[j];
  if (nz == 3 && nb * nb < threshold_helper * (5 - K)) nz = K;
  tr[K] = big;
#pragma unroll
  for (int j = K + 1; j < 3; ++j) {
    if (big == j) {
#pragma unroll
      for (int r = 0; r < 5; ++r) swap_d(qr[K][r], qr[j][r]);
      swap_d(nu[K], nu[j]);
      swap_d(nd[K], nd[j]);
    }
  }
  plane_hh<K>(qr, hc);
  const double nrm_thr = sqrt(DBL_EPSILON);
#pragma unroll
  for (int j = K + 1; j < 3; ++j) {
    if (nu[j] != 0.0) {
      double temp = fabs(qr[j][K]) / nu[j];
      temp = (1.0 + temp) * (1.0 - temp);
      temp = temp < 0.0 ? 0.0 : temp;
      const double ratio = nu[j] / nd[j];
      const double temp2 = temp * ratio * ratio;
      if (temp2 <= nrm_thr) {
        double s = 0.0;
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
__device__ void plane_solve(const double (&A)[5][3], double (&x)[3]) {
  double qr[3][5];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 5; ++r) qr[c][r] = A[r][c];
  double hc[3] = {0.0, 0.0, 0.0}, nu[3], nd[3];
  int tr[3] = {0, 1, 2};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < 5; ++r) s += qr[k][r] * qr[k][r];
    nd[k] = sqrt(s);
    nu[k] = nd[k];
  }
  const double maxn = fmax(nu[0], fmax(nu[1], nu[2]));
  const double threshold_helper = (maxn * DBL_EPSILON) * (maxn * DBL_EPSILON) / 5;
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
  x[0] = x[1] = x[2] = 0.0;
  if (nz == 0) return;
  double c[5] = {-1.0, -1.0, -1.0, -1.0, -1.0};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (k < nz && hc[k] != 0.0) {
      double tmp = c[k];
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
      double s = c[i];
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
  st->radius = 1e4;
  st->dfac = 2.0;
  st->go = 0ull;
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
constexpr int kUnrollDefault = 4;   // candidate loads in flight per lane (U)

// (start, count) of a coarse cell, or (0, 0): the entry's {key, start, total} head (one 16-B load)
template <typename Cell>
__device__ __forceinline__ int2 grid_lookup(const Cell* __restrict__ tab, unsigned long long key, int bits,
                                            unsigned mask) {
  unsigned h = hash_slot64(key, bits);
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

struct CorrArgs {
  const PointRec* q;       // downsampled scan points (sensor frame)
  const int* d_n;          // device count
  int n_ub;
  const float4* gpts;      // the map grouped by cell: {x, y, z, map index bits}
  const CoarseCell* coarse;
  int bits;                // table size 1 << bits (both tables)
  unsigned mask;
  const float4* map;       // the map's coordinates in its own order (neighbour coordinates by map index)
  double* rec;
  uint8_t* valid;
  float* nnxyz;
  int cap;
  unsigned long long* dbg;   // FLOAM_DEBUG_STAMPS: per-phase latency sums (diagnostic, normally null)
};

__device__ __forceinline__ int fine_count(const CorrArgs& A, int fx, int fy, int fz) {
  const unsigned long long key = cell_key(fx >> 1, fy >> 1, fz >> 1);
  unsigned h = hash_slot64(key, A.bits);
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
template <int G>
__device__ __forceinline__ void fine_block_ranges(const CorrArgs& A, int qx, int qy, int qz, int lane,
                                                  int* __restrict__ s_pre, int* __restrict__ s_start,
                                                  int* __restrict__ s_cc) {
  static_assert(G >= 8, "one coarse probe per lane");
  const int cx0 = (qx - 1) >> 1, cy0 = (qy - 1) >> 1, cz0 = (qz - 1) >> 1;   // floor division by 2
  if (lane < 8) {
    const unsigned long long key = cell_key(cx0 + (lane & 1), cy0 + ((lane >> 1) & 1), cz0 + (lane >> 2));
    unsigned slot = hash_slot64(key, A.bits);
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
  constexpr int P = (kMaxStencil + G - 1) / G;   // fine cells per lane
  const int cb = min(kMaxStencil, lane * P), ce = min(kMaxStencil, cb + P);
  int local = 0;
#pragma unroll
  for (int j = 0; j < P; ++j) {
    const int c = cb + j;
    if (c < ce) {
      const int fx = qx - 1 + c % 3, fy = qy - 1 + (c / 3) % 3, fz = qz - 1 + c / 9;
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
  if (lane == G - 1) s_pre[kMaxStencil] = incl;
  wave_lds_order();
}

template <int G, int U, bool COARSE>
__device__ __forceinline__ void stencil_scan(const CorrArgs& A, int x0, int x1, int y0, int y1, int z0, int z1,
                                             float wx, float wy, float wz, int lane, int* __restrict__ s_pre,
                                             int* __restrict__ s_start, Top5& t, int& cnt,
                                             int* __restrict__ s_cc = nullptr) {
  constexpr int P = (kMaxStencil + G - 1) / G;   // cells per lane
  const int nxr = x1 - x0 + 1, nyr = y1 - y0 + 1, nzr = z1 - z0 + 1;
  const int ncell = nxr * nyr * nzr;
  int tot;
  if constexpr (!COARSE) {   // the fine block around (x0 + 1, y0 + 1, z0 + 1), ranges from the coarse entries
    fine_block_ranges<G>(A, x0 + 1, y0 + 1, z0 + 1, lane, s_pre, s_start, s_cc);
    tot = s_pre[kMaxStencil];
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
      slot[j] = hash_slot64(key[j], A.bits);
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

// group-wide top-5 (every lane ends with the merged list) and count
template <int G>
__device__ __forceinline__ void group_merge(Top5& t, int& cnt) {
#pragma unroll
  for (int mm = G / 2; mm > 0; mm >>= 1) {
    Top5 o;
#pragma unroll
    for (int k = 0; k < 5; ++k) o.k[k] = shfl_xor_u64<G>(t.k[k], mm);
    top5_merge(t, o);
    cnt += __shfl_xor(cnt, mm, G);
  }
}

// Physical block p of the first `nactive` blocks -> logical block, so that the blocks with equal p % 8 (one XCD
// under the round-robin dispatch of MI355X_MICROARCH.md "Workgroup dispatch") get consecutive logical indices.
// A bijection on [0, nactive); placement only affects speed, never results.
__device__ __forceinline__ int xcd_block(int p, int nactive) {
  const int x = p & 7, r = p >> 3, base = nactive >> 3, rem = nactive & 7;
  return x * base + min(x, rem) + r;
}

// Pass 1: exact 5-NN of every query (no fp64 geometry here, so the kernel stays small and at high occupancy).
// The reference keeps a correspondence iff the 5th-nearest float sq-distance is < 1 (:154, :210), so only map
// points within 1 m matter.  Stage 1 scans the 3x3x3 FINE cells (edge 0.5 m) around the query's cell: every point
// outside that block is at least 0.5 m away along some axis, so its float sq-distance is >= 0.25 (exact: the cell
// bounds are exact and fl(dx) >= 0.5 by monotone rounding); if 5 points with sq-distance < 0.25 were found they are
// the exact 5-NN.  Otherwise stage 2 scans the COARSE cells (1 m) spanning [q-1, q+1] on every axis (<= 3x3x3),
// which contain every point within 1 m.  Ties at equal float distance go to the lower map index (FLANN's own order
// depends on its tree traversal; tie-free data is identical).
// Output: valid bit 0 = 5 neighbours within sqd < 1 (their coordinates in nnxyz), bit 1 = stage 2 was needed.
template <int G, int U>
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
      Top5 t;
#pragma unroll
      for (int k = 0; k < 5; ++k) t.k[k] = ~0ull;
      int cnt = 0;
      stencil_scan<G, U, false>(A, qx - 1, qx + 1, qy - 1, qy + 1, qz - 1, qz + 1, wx, wy, wz, lane, s_pre, s_start,
                                t, cnt, s_cc);
      group_merge<G>(t, cnt);
      const bool complete = cnt >= 5 && __uint_as_float((unsigned)(t.k[4] >> 32)) < 0.25f;
      if (!complete) {   // coarse cells floor(q - 1) .. floor(q + 1) per axis (exact in double)
#pragma unroll
        for (int k = 0; k < 5; ++k) t.k[k] = ~0ull;
        cnt = 0;
        stencil_scan<G, U, true>(A, (int)floor((double)wx - 1.0), (int)floor((double)wx + 1.0),
                                 (int)floor((double)wy - 1.0), (int)floor((double)wy + 1.0),
                                 (int)floor((double)wz - 1.0), (int)floor((double)wz + 1.0), wx, wy, wz, lane, s_pre,
                                 s_start, t, cnt);
        group_merge<G>(t, cnt);
        flags |= 2;
      }
      if (cnt >= 5) {   // sqd[4] < 1 (:154, :210)
        flags |= 1;
        if (lane < 5) {   // lane k writes the coordinates of neighbour k
          unsigned long long kk = t.k[0];
#pragma unroll
          for (int k = 1; k < 5; ++k)
            if (lane == k) kk = t.k[k];
          const float4 m = A.map[(int)(kk & 0xFFFFFFFFull)];
          A.nnxyz[(3 * lane + 0) * A.cap + i] = m.x;
          A.nnxyz[(3 * lane + 1) * A.cap + i] = m.y;
          A.nnxyz[(3 * lane + 2) * A.cap + i] = m.z;
        }
      }
    }
    if (lane == 0) A.valid[i] = (uint8_t)flags;
  }
}

// Edge and surf kNN in one launch: blocks [0, nbE) run edge groups, the others surf groups.  The launch also starts
// the solve (lm_init folded in): block 0 resets the LM state and, for the first solve of an update, stores the
// prediction x0 that every block uses for its transforms (the others never read st->x in that case).
template <int G, int U, int W>
__global__ __launch_bounds__(kTB, W) void knn_kernel(LMState* __restrict__ st, X7 x0, const double* __restrict__ x0_dev,
                                                  CorrArgs E, CorrArgs S, int nbE,
                                                  const int* __restrict__ d_me, const int* __restrict__ d_ms,
                                                  int rank, int world) {
  __shared__ int s_pre[kTB / G][kMaxStencil + 1];
  __shared__ int s_start[kTB / G][kMaxStencil];
  __shared__ int s_cc[kTB / G][8 * 9];
  const int lane = threadIdx.x & (G - 1);
  const int g = threadIdx.x / G;
  double pose[7];   // wave-uniform: kept in SGPRs (readfirstlane), not in 14 VGPRs of every lane
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const long long b = __double_as_longlong(x0_dev ? x0_dev[k] : (x0.set ? x0.v[k] : st->x[k]));
    const int lo = __builtin_amdgcn_readfirstlane((int)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    pose[k] = __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    X7 xs;
    xs.set = (x0_dev || x0.set) ? 1 : 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) xs.v[k] = pose[k];
    lm_reset(st, xs);
  }
  const bool gate = *d_me > 10 && *d_ms > 50;   // map-size gate (odomEstimationClass.cpp:77)
  // XCD-aware placement: the blocks that hold queries are renumbered so that the blocks sharing an XCD (physical
  // index mod 8 under round-robin dispatch) take consecutive query ranges.  The queries are in voxel order, so each
  // XCD then works on a compact slab of the scene and its L2 holds that slab's map cells instead of all of them.
  const bool edge = (int)blockIdx.x < nbE;
  const CorrArgs& A = edge ? E : S;
  const int nb = edge ? nbE : (int)gridDim.x - nbE;
  int p = edge ? (int)blockIdx.x : (int)blockIdx.x - nbE;
  const int nq = min(*A.d_n, A.n_ub);
  const int nact = min(nb, (int)(((long long)nq * G + kTB - 1) / kTB));
  const unsigned long long t_start = E.dbg ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const bool had = p < nact;
  if (p < nact) p = xcd_block(p, nact);
  knn_group<G, U>(pose, A, (p * kTB + (int)threadIdx.x) / G, nb * (kTB / G), lane, gate, rank, world, s_pre[g],
                  s_start[g], s_cc[g]);
  if (E.dbg && (threadIdx.x & 63) == 0) {   // FLOAM_KNN_TRACE: per-wave (start, end) of the launch (diagnostic)
    const unsigned w = blockIdx.x * (kTB / 64) + (threadIdx.x >> 6);
    if (w < (1u << 16)) {
      E.dbg[2 * w] = t_start | (had ? (1ull << 63) : 0ull);
      E.dbg[2 * w + 1] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

// Pass 2: fp64 line / plane geometry, one query per lane (all 64 lanes busy).
// Surf record i as the 13-vector w = [n (x) p (9), n (3), d + n.o] (p the sensor-frame point, n the unit normal,
// d the plane offset, o the solve's starting translation): every surf residual and Jacobian entry is linear in w
// (see surf_sums_from_gram), so the surf half of each LM evaluation needs only the Gram matrix sum(w w^T).
constexpr int kGramW = 13;
constexpr int kGram = kGramW * (kGramW + 1) / 2;   // 91 unique entries (upper triangle, row-major)
constexpr int kSurfGeomBlocks = 256;               // fixed surf geometry grid: fixed Gram reduction order

template <bool EDGE>
__device__ __forceinline__ void geom_query(LMState* __restrict__ st, const CorrArgs& A, int i,
                                           double* __restrict__ w = nullptr, const double* o = nullptr) {
  const int n = min(*A.d_n, A.n_ub);
  bool ok = false;
  const int flags = i < n ? A.valid[i] : 0;
  if (flags & 1) {
    double P[5][3];
#pragma unroll
    for (int j = 0; j < 5; ++j)
#pragma unroll
      for (int a = 0; a < 3; ++a) P[j][a] = A.nnxyz[(3 * j + a) * A.cap + i];
    const float4 pq = *reinterpret_cast<const float4*>(&A.q[i].x);
    const double cpx = pq.x, cpy = pq.y, cpz = pq.z;
    double* rec = A.rec;
    const int cap = A.cap;
    if (EDGE) {
      // addEdgeCostFactor geometry (odomEstimationClass.cpp:156-189)
      double cc[3] = {0.0, 0.0, 0.0};
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        cc[0] = cc[0] + P[j][0]; cc[1] = cc[1] + P[j][1]; cc[2] = cc[2] + P[j][2];
      }
      cc[0] = cc[0] / 5.0; cc[1] = cc[1] / 5.0; cc[2] = cc[2] / 5.0;
      double cov[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const double z[3] = {P[j][0] - cc[0], P[j][1] - cc[1], P[j][2] - cc[2]};
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
          for (int b = 0; b < 3; ++b) cov[a][b] = cov[a][b] + z[a] * z[b];
      }
      double ev[3], u[3];
      eig_sym3(cov, ev, u);
      if (ev[2] > 3 * ev[1]) {
        ok = true;
        rec[0 * cap + i] = cpx; rec[1 * cap + i] = cpy; rec[2 * cap + i] = cpz;
        rec[3 * cap + i] = 0.1 * u[0] + cc[0]; rec[4 * cap + i] = 0.1 * u[1] + cc[1];
        rec[5 * cap + i] = 0.1 * u[2] + cc[2];
        rec[6 * cap + i] = -0.1 * u[0] + cc[0]; rec[7 * cap + i] = -0.1 * u[1] + cc[1];
        rec[8 * cap + i] = -0.1 * u[2] + cc[2];
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
#pragma unroll
      for (int j = 0; j < 5; ++j)
        if (fabs(nv[0] * P[j][0] + nv[1] * P[j][1] + nv[2] * P[j][2] + d) > 0.2) planeValid = false;
      if (planeValid) {
        ok = true;
        rec[0 * cap + i] = cpx; rec[1 * cap + i] = cpy; rec[2 * cap + i] = cpz;
        rec[3 * cap + i] = nv[0]; rec[4 * cap + i] = nv[1]; rec[5 * cap + i] = nv[2];
        rec[6 * cap + i] = d;
        if (w) {
          const double pp[3] = {cpx, cpy, cpz};
#pragma unroll
          for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int e = 0; e < 3; ++e) w[3 * a + e] = nv[a] * pp[e];
          w[9] = nv[0]; w[10] = nv[1]; w[11] = nv[2];
          w[12] = d + ((nv[0] * o[0] + nv[1] * o[1]) + nv[2] * o[2]);
        }
      }
    }
    A.valid[i] = (uint8_t)((flags & 2) | (ok ? 1 : 0) | 4);   // bit 2: the search found 5 neighbours
  }
  const unsigned long long b = __ballot(ok);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(EDGE ? &st->corr_edge : &st->corr_surf, __popcll(b));
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
constexpr int kGramGroups = 8;   // the surf blocks' partials are reduced in 8 groups of 32, then the groups

__global__ __launch_bounds__(kTB) void geom_kernel(LMState* __restrict__ st, CorrArgs E, CorrArgs S, int nbE,
                                                   double* __restrict__ gpart, double* __restrict__ gmat,
                                                   unsigned* __restrict__ gcnt) {
  if ((int)blockIdx.x < nbE) {
    geom_query<true>(st, E, blockIdx.x * blockDim.x + threadIdx.x);
    return;
  }
  const int sb = (int)blockIdx.x - nbE;
  const int ns = min(*S.d_n, S.n_ub);   // the device count bounds the grid-stride loops (block-uniform)
  if (!gpart) {
    for (int i0 = sb * kTB; i0 < ns; i0 += kSurfGeomBlocks * kTB) geom_query<false>(st, S, i0 + threadIdx.x);
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
  for (int i0 = sb * kTB; i0 < ns; i0 += kSurfGeomBlocks * kTB) {   // wave-uniform trip count
    double w[kGramW];
#pragma unroll
    for (int k = 0; k < kGramW; ++k) w[k] = 0.0;
    geom_query<false>(st, S, i0 + threadIdx.x, w, o);
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
  }
  s_part[wv][lane] = g0;
  if (lane + 64 < kGram) s_part[wv][lane + 64] = g1;
  __syncthreads();
  if (threadIdx.x < kGram) {
    double v = s_part[0][threadIdx.x];
#pragma unroll
    for (int k = 1; k < kTB / 64; ++k) v += s_part[k][threadIdx.x];
    gpart[sb * kGram + threadIdx.x] = v;
  }
  // G of the solve, reduced by the last-arriving blocks (fixed order: the 32 blocks of a group, then the 8 groups):
  // producer stores -> vmcnt(0) -> barrier -> agent release -> ticket; the block whose ticket is last acquires
  constexpr int per = kSurfGeomBlocks / kGramGroups;
  __shared__ int s_last;
  const int grp = sb / per;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    s_last = atomicAdd(&gcnt[grp], 1u) == (unsigned)(per - 1);
    if (s_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  if (!s_last) return;
  double* gpart2 = gpart + kSurfGeomBlocks * kGram;   // [8][91] group partials
  if (threadIdx.x < kGram) {
    double v = 0.0;
    double gp[per];   // all loads in flight before the in-order sum
#pragma unroll
    for (int k = 0; k < per; ++k) gp[k] = gpart[(grp * per + k) * kGram + threadIdx.x];
#pragma unroll
    for (int k = 0; k < per; ++k) v += gp[k];
    gpart2[grp * kGram + threadIdx.x] = v;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    gcnt[grp] = 0u;   // every block of the group has arrived (next launch: kernel boundary)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    s_last = atomicAdd(&gcnt[kGramGroups], 1u) == (unsigned)(kGramGroups - 1);
    if (s_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x < kGram) {
    double v = gpart2[threadIdx.x];
    for (int k = 1; k < kGramGroups; ++k) v += gpart2[k * kGram + threadIdx.x];
    gmat[threadIdx.x] = v;
  } else if (threadIdx.x < kGram + 3) {
    gmat[threadIdx.x] = o[threadIdx.x - kGram];   // the origin the records were recentred on
  }
  if (threadIdx.x == 0) gcnt[kGramGroups] = 0u;
}

// Algorithmic traffic of one launch of the search kernel (knn_kernel; SURVEY.md §8 d): every map
// cell any query scans is streamed once (16 B per map point: the union over queries of the fine 3x3x3 block around
// the query's cell — level 0 — and of the coarse +-1 m stencil for the queries whose bit 1 says they needed stage 2
// — level 1), every query is read once (16 B) and writes its flag (1 B) and, with 5 neighbours, their coordinates
// (60 B) (counted at level 0).  Runs untimed, on a replay, only when profiling.
__global__ __launch_bounds__(kTB) void knn_traffic(const LMState* __restrict__ st, CorrArgs A, int rank,
                                                   int world, int level, unsigned long long* __restrict__ set,
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
    x0 = (int)floor((double)wx - 1.0); x1 = (int)floor((double)wx + 1.0);
    y0 = (int)floor((double)wy - 1.0); y1 = (int)floor((double)wy + 1.0);
    z0 = (int)floor((double)wz - 1.0); z1 = (int)floor((double)wz + 1.0);
  } else {
    fine_cell(wx, wy, wz, x0, y0, z0);
    --x0; --y0; --z0;
    x1 = x0 + 2; y1 = y0 + 2; z1 = z0 + 2;
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


__global__ void lm_init(LMState* st, X7 x0) {
  if (threadIdx.x == 0) lm_reset(st, x0);
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
                                             UpdateStatus* __restrict__ out, OdomDev* __restrict__ s, int mode);
namespace {

__global__ __launch_bounds__(kTB) void deskew_bridge(const LMState* __restrict__ st, OdomDev* __restrict__ s,
                                                     double period, PointRec* __restrict__ edge,
                                                     const int* __restrict__ d_ne, int ne_ub,
                                                     PointRec* __restrict__ surf, const int* __restrict__ d_ns,
                                                     int ns_ub, GatherArgs g) {
  if (g.out && blockIdx.x == 0) gather_block(st, g.dcnt, g.mapE_count, g.mapS_count, g.fe_status, nullptr, g.out, s, 0);
  double x1[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) x1[k] = st->x[k];
  const double* t0 = s->last_odom.t;   // the pose before the first call (read-only in this launch)
  // GetVelocity (include/odomEstimationClass.h:78): (odom.translation() - last_odom.translation()) / scan_period
  const double vx = (x1[4] - t0[0]) / period, vy = (x1[5] - t0[1]) / period, vz = (x1[6] - t0[2]) / period;
  const int ne = min(*d_ne, ne_ub), ns = min(*d_ns, ns_ub);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ne + ns; i += gridDim.x * blockDim.x) {
    PointRec& p = i < ne ? edge[i] : surf[i - ne];   // CompensateVelocity: p += v * time, double -> float
    const double t = p.time;
    p.x = (float)((double)p.x + vx * t);
    p.y = (float)((double)p.y + vy * t);
    p.z = (float)((double)p.z + vz * t);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
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
  pose_to_params(pose_identity(), s->x0[0]);
  pose_to_params(pose_identity(), s->x0[1]);
}

__global__ void odom_predict(OdomDev* s) {
  if (threadIdx.x == 0) odom_predict_step(s);
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

// Per-block partial sums (cost, J^T J upper, J^T r, count) of one LM evaluation over the device-resident
// correspondence slots [0, *d_ne) and [0, *d_ns).  Evaluated at x (phase 0, iteration zero) or at the candidate.
// Stores / loads of words handed between blocks of one launch without fences: agent-scope relaxed atomics compile
// to sc1 (L2-coherent) accesses, so the consumer needs no cache invalidation (MI355X_MICROARCH.md "Valid forms":
// sc1 stores drained with vmcnt(0) before the flag, sc1 loads after it).
__device__ __forceinline__ void store_sc1(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_sc1(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

template <bool SC1>
__device__ void eval_block_at(const double (&x)[7], const double* __restrict__ erec,
                              const uint8_t* __restrict__ evalid, int ecap, int ne, const double* __restrict__ srec,
                              const uint8_t* __restrict__ svalid, int scap, int ns, int huber,
                              double* __restrict__ partials, int blk, int nblk);

template <bool SC1>
__device__ void eval_block(const LMState* __restrict__ st, const double* __restrict__ erec,
                           const uint8_t* __restrict__ evalid, int ecap, int ne, const double* __restrict__ srec,
                           const uint8_t* __restrict__ svalid, int scap, int ns, int huber, double* __restrict__ partials,
                           int blk, int nblk) {
  // x and cand are adjacent in LMState: load both with the phase in one round trip, then select
  double xa[7], xc[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) { xa[k] = st->x[k]; xc[k] = st->cand[k]; }
  const bool at_x = st->phase == 0;
  double x[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) x[k] = at_x ? xa[k] : xc[k];
  eval_block_at<SC1>(x, erec, evalid, ecap, ne, srec, svalid, scap, ns, huber, partials, blk, nblk);
}

// one residual (r, J) into the 29 sums (cost, J^T J upper, J^T r, count), with the Huber corrector if asked
__device__ __forceinline__ void accumulate_residual(double (&acc)[LM_NSUM], double r, double (&J)[6], int huber) {
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

// fixed-order block reduction through LDS: [component][thread] -> 8 strips of 32 per component -> 8 partials
template <bool SC1>
__device__ void store_block_partials(const double (&acc)[LM_NSUM], double* __restrict__ partials, int blk, int nblk) {
  __shared__ double red[LM_NSUM][kTB];
  __shared__ double strip[LM_NSUM][8];
#pragma unroll
  for (int k = 0; k < LM_NSUM; ++k) red[k][threadIdx.x] = acc[k];
  __syncthreads();
  if (threadIdx.x < LM_NSUM * 8) {
    const int c = threadIdx.x >> 3, p = threadIdx.x & 7;
    double v = 0.0;
#pragma unroll
    for (int j = 0; j < kTB / 8; ++j) v += red[c][p * (kTB / 8) + j];
    strip[c][p] = v;
  }
  __syncthreads();
  if (threadIdx.x < LM_NSUM) {
    double v = 0.0;
    for (int p = 0; p < 8; ++p) v += strip[threadIdx.x][p];
    if (SC1) store_sc1(&partials[threadIdx.x * nblk + blk], v);
    else partials[threadIdx.x * nblk + blk] = v;
  }
}

template <bool SC1>
__device__ void eval_block_at(const double (&x)[7], const double* __restrict__ erec,
                              const uint8_t* __restrict__ evalid, int ecap, int ne, const double* __restrict__ srec,
                              const uint8_t* __restrict__ svalid, int scap, int ns, int huber,
                              double* __restrict__ partials, int blk, int nblk) {
  double acc[LM_NSUM];
#pragma unroll
  for (int k = 0; k < LM_NSUM; ++k) acc[k] = 0.0;
  const int total = ne + ns;
  for (int idx = blk * blockDim.x + threadIdx.x; idx < total; idx += nblk * blockDim.x) {
    double J[6], r;
    if (idx < ne) {
      if (!(evalid[idx] & 1)) continue;
      double f[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) f[k] = erec[k * ecap + idx];
      r = edge_residual(x, f, J);
    } else {
      const int s = idx - ne;
      if (!(svalid[s] & 1)) continue;
      double f[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) f[k] = srec[k * scap + s];
      r = surf_residual(x, f, J);
    }
    accumulate_residual(acc, r, J, huber);
  }
  store_block_partials<SC1>(acc, partials, blk, nblk);
}

__global__ __launch_bounds__(kTB) void lm_eval(const LMState* __restrict__ st, const double* __restrict__ erec,
                                               const uint8_t* __restrict__ evalid, int ecap, const int* __restrict__ d_ne,
                                               int ne_ub, const double* __restrict__ srec,
                                               const uint8_t* __restrict__ svalid, int scap,
                                               const int* __restrict__ d_ns, int ns_ub, int huber,
                                               double* __restrict__ partials) {
  if (st->done) return;
  eval_block<false>(st, erec, evalid, ecap, min(*d_ne, ne_ub), srec, svalid, scap, min(*d_ns, ns_ub), huber,
                    partials, blockIdx.x, gridDim.x);
}

template <bool SC1 = false>
__device__ void reduce_partials_block(const double* __restrict__ partials, int nblk, double* sums /* shared */) {
  // component c = t / 8 sums its 8 block strips in order, then thread c sums the 8 strip totals (fixed order)
  __shared__ double strip[LM_NSUM][8];
  if (threadIdx.x < LM_NSUM * 8) {
    const int c = threadIdx.x >> 3, p = threadIdx.x & 7;
    const int per = (nblk + 7) / 8;
    const int b0 = p * per, b1 = min(nblk, b0 + per);
    double v = 0.0;
    int bb = b0;
    for (; bb + 8 <= b1; bb += 8) {   // 8 loads in flight, then added in order
      double t[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) t[k] = SC1 ? load_sc1(&partials[c * nblk + bb + k]) : partials[c * nblk + bb + k];
#pragma unroll
      for (int k = 0; k < 8; ++k) v += t[k];
    }
    {
      double t[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        t[k] = bb + k < b1 ? (SC1 ? load_sc1(&partials[c * nblk + bb + k]) : partials[c * nblk + bb + k]) : 0.0;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (bb + k < b1) v += t[k];
    }
    strip[c][p] = v;
  }
  __syncthreads();
  if (threadIdx.x < LM_NSUM) {
    double v = 0.0;
    for (int p = 0; p < 8; ++p) v += strip[threadIdx.x][p];
    sums[threadIdx.x] = v;
  }
  __syncthreads();
}

// ===================================================================================== LM control (Ceres 1.13)
// The control step is serial fp64 code, so its cost is its dependent instruction count (every fp64 VALU op is at
// least 4 cycles for a wave).  It runs on one wave whose 64 lanes all hold the same LM state in registers (the
// uniform part costs the same on 64 lanes as on one); the two SE(3) exponentials of a step — the candidate
// x [+] delta and the gradient projection x [+] -g of the gradient-norm test — run side by side in lanes 0 and 1 of
// the same instruction stream; the 6x6 Cholesky divides by each pivot once (reciprocals).  Loops are fully unrolled
// with constant indices so nothing leaves registers.

// PoseSE3Parameterization::Plus + getTransformFromSe3 (src/lidarOptimization.cpp:77-140).  theta^3 is formed by
// multiplication where the reference calls pow(theta, 3) (<= 1 ulp apart).
__device__ __forceinline__ void se3_plus(const double (&x)[7], const double (&d)[6], double (&out)[7]) {
  const double wx = d[0], wy = d[1], wz = d[2];
  const double theta = sqrt(wx * wx + wy * wy + wz * wz);
  const double half = 0.5 * theta;
  double sh, ch;
  sincos(half, &sh, &ch);
  const double real_factor = ch;
  double imag;
  const bool small = theta < 1e-10;
  if (small) {
    const double t2 = theta * theta, t4 = t2 * t2;
    imag = 0.5 - 0.0208333 * t2 + 0.000260417 * t4;
  } else {
    imag = sh / theta;
  }
  const double dq[4] = {imag * wx, imag * wy, imag * wz, real_factor};   // x, y, z, w
  double Jm[3][3];
  if (small) {
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
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) O2[i][j] = O[i][0] * O[0][j] + O[i][1] * O[1][j] + O[i][2] * O[2][j];
    double st, ct;
    sincos(theta, &st, &ct);
    const double c1 = (1 - ct) / (theta * theta);
    const double c2 = (theta - st) / (theta * theta * theta);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
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

__host__ __device__ constexpr int hidx(int a, int b) {   // upper-triangle row-major index, a <= b
  return a * 6 - a * (a - 1) / 2 + (b - a);
}

// LevenbergMarquardtStrategy::ComputeStep in normal-equation form on the Jacobi-scaled system:
// (Hs + diag(Hs)/radius) y = gs, step = -y; then TrustRegionMinimizer::ComputeTrustRegionStep's model cost change.
// (The oracle solves the equivalent [J; sqrt(D/radius)] least-squares problem by Householder QR like Ceres'
// DENSE_QR; the two agree to ~cond * eps.)  Returns false for an invalid step; delta = scaled step.
__device__ __forceinline__ bool solve_step(LMState& s, double (&delta)[6]) {
  // every field the step reads is loaded once into registers up front (one LDS round trip), the two LDS writes
  // (diag, reuse) go out at the end: no store-to-load waits on the state inside the dependent fp64 chain
  double sc[6], gs[6], Hu[21], dg[6];
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    sc[a] = s.scale[a];
    dg[a] = s.diag[a];
  }
#pragma unroll
  for (int k = 0; k < 21; ++k) Hu[k] = s.H[k];
#pragma unroll
  for (int a = 0; a < 6; ++a) gs[a] = sc[a] * s.g[a];
  const int reuse = s.reuse;
  const double inv_radius = 1.0 / s.radius;
  // packed lower triangle (row-major, l(i,j) = i(i+1)/2 + j): Hs = S H S, then A = Hs + diag/radius factored in place
  double Hs[21], A[21];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      Hs[i * (i + 1) / 2 + j] = sc[i] * Hu[hidx(j, i)] * sc[j];
      A[i * (i + 1) / 2 + j] = Hs[i * (i + 1) / 2 + j];
    }
  if (!reuse) {
#pragma unroll
    for (int k = 0; k < 6; ++k) dg[k] = fmin(fmax(Hs[k * (k + 1) / 2 + k], 1e-6), 1e32);
#pragma unroll
    for (int k = 0; k < 6; ++k) s.diag[k] = dg[k];
  }
  s.reuse = 1;
  // LDL^T of A = Hs + diag / radius (no square roots on the dependent chain; one reciprocal per pivot): W[i][j] =
  // L[i][j] D[j] is kept beside L, packed lower like A
#pragma unroll
  for (int k = 0; k < 6; ++k) A[k * (k + 1) / 2 + k] += dg[k] * inv_radius;
  double W[21], rD[6];
  bool pd = true;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double d = A[j * (j + 1) / 2 + j];
#pragma unroll
    for (int k = 0; k < j; ++k) d -= A[j * (j + 1) / 2 + k] * W[j * (j + 1) / 2 + k];
    pd = pd && (d > 0.0);
    rD[j] = 1.0 / d;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double v = A[i * (i + 1) / 2 + j];
#pragma unroll
      for (int k = 0; k < j; ++k) v -= A[i * (i + 1) / 2 + k] * W[j * (j + 1) / 2 + k];
      W[i * (i + 1) / 2 + j] = v;            // L[i][j] D[j]
      A[i * (i + 1) / 2 + j] = v * rD[j];    // L[i][j]
    }
  }
  if (!pd) return false;
  double y[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {   // L z = gs
    double v = gs[i];
#pragma unroll
    for (int k = 0; k < i; ++k) v -= A[i * (i + 1) / 2 + k] * y[k];
    y[i] = v;
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {   // L^T y = D^-1 z
    double v = y[i] * rD[i];
#pragma unroll
    for (int k = i + 1; k < 6; ++k) v -= A[k * (k + 1) / 2 + i] * y[k];
    y[i] = v;
  }
  bool finite = true;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    y[k] = -y[k];   // the step
    finite = finite && isfinite(y[k]);
  }
  if (!finite) return false;
  // model cost change -(step^T gs + step^T Hs step / 2)
  double sg = 0.0, sHs = 0.0;
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    sg += y[a] * gs[a];
    double hv = 0.0;
#pragma unroll
    for (int b = 0; b < 6; ++b) hv += Hs[a >= b ? a * (a + 1) / 2 + b : b * (b + 1) / 2 + a] * y[b];
    sHs += y[a] * hv;
  }
  const double mcc = -(sg + 0.5 * sHs);
  if (!(mcc > 0.0)) return false;
  s.mcc = mcc;
#pragma unroll
  for (int k = 0; k < 6; ++k) delta[k] = y[k] * sc[k];
  return true;
}

// value of lane src (a compile-time / wave-uniform lane) to every lane: two v_readlane (no LDS round trip)
__device__ __forceinline__ double bcast(double v, int src) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, src);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), src);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// NextStep with the gradient-norm test folded in: ComputeTrustRegionStep (+ HandleInvalidStep retries) and, when
// check_gmax, the projected-gradient max norm at x (lane 1) computed alongside the candidate (lane 0).  If the
// gradient test ends the solve the step is discarded, as in the sequential order (test first, then step).
#ifdef FLOAM_CTRL_STAMPS
__device__ unsigned long long g_ctrl_stamps[8];
#define CTRL_STAMP(i, t)                                                        \
  do {                                                                          \
    const unsigned long long tn_ = __builtin_amdgcn_s_memrealtime();            \
    if (lane == 0) atomicAdd(&g_ctrl_stamps[i], tn_ - (t));                      \
    (t) = tn_;                                                                  \
  } while (0)
#else
#define CTRL_STAMP(i, t) (void)0
#endif
__device__ __forceinline__ void next_step_wave(LMState& s, bool check_gmax, int lane) {
  for (;;) {
#ifdef FLOAM_CTRL_STAMPS
    unsigned long long ts = __builtin_amdgcn_s_memrealtime();
#endif
    double delta[6];
    const bool valid = solve_step(s, delta);
    CTRL_STAMP(0, ts);
    double d[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) d[k] = lane == 1 ? -s.g[k] : (valid ? delta[k] : 0.0);
    double out[7];
    se3_plus(s.x, d, out);
    CTRL_STAMP(1, ts);
    if (check_gmax) {
      double m = 0.0;
#pragma unroll
      for (int i = 0; i < 7; ++i) m = fmax(m, fabs(s.x[i] - bcast(out[i], 1)));
      s.gmax = m;
      check_gmax = false;
      if (s.gmax <= 1e-10) { s.done = 1; return; }   // (phase 0: before any step; phase 1: success && gmax)
    }
    CTRL_STAMP(5, ts);
    s.iteration++;
    if (valid) {
#pragma unroll
      for (int i = 0; i < 7; ++i) s.cand[i] = bcast(out[i], 0);
      s.invalid = 0;
      return;   // candidate pending evaluation
    }
    // HandleInvalidStep -> StepIsInvalid -> StepRejected(0)
    if (++s.invalid >= 5) { s.done = 1; return; }
    s.radius /= s.dfac;
    s.dfac *= 2.0;
    s.reuse = 1;
    if (s.iteration >= 4 || s.radius < 1e-32) { s.done = 1; return; }
  }
}

__device__ __forceinline__ double norm7(const double (&a)[7]) {
  double v = 0.0;
#pragma unroll
  for (int i = 0; i < 7; ++i) v += a[i] * a[i];
  return sqrt(v);
}

// One Ceres control step after an evaluation (sums = cost, J^T J, J^T r, count at x in phase 0, else at cand).
// Called by all 64 lanes of one wave with identical s and sums; every lane ends with the same s.
__device__ __forceinline__ void lm_logic(LMState& s, const double (&sums)[LM_NSUM], int lane) {
#ifdef FLOAM_CTRL_STAMPS
  unsigned long long ts = __builtin_amdgcn_s_memrealtime();
#endif
  if (s.phase == 0) {   // IterationZero
    s.n_res = (int)sums[28];
    if (s.n_res == 0) { s.done = 1; return; }   // no residual blocks: parameters untouched
    s.x_cost = sums[0];
    if (!isfinite(s.x_cost)) { s.done = 1; return; }
#pragma unroll
    for (int k = 0; k < 21; ++k) s.H[k] = sums[1 + k];
#pragma unroll
    for (int k = 0; k < 6; ++k) s.g[k] = sums[22 + k];
    s.initial_cost = s.x_cost;
#pragma unroll
    for (int k = 0; k < 6; ++k) s.scale[k] = 1.0 / (1.0 + sqrt(s.H[hidx(k, k)]));
    s.x_norm = norm7(s.x);
    s.radius = 1e4;
    s.dfac = 2.0;
    s.reuse = 0;
    s.invalid = 0;
    s.iteration = 0;
    s.phase = 1;
    CTRL_STAMP(4, ts);
    next_step_wave(s, true, lane);
    return;
  }
  double cand_cost = sums[0];
  if (!isfinite(cand_cost)) cand_cost = DBL_MAX;
  // ParameterToleranceReached (candidate not applied)
  double sn = 0.0;
#pragma unroll
  for (int i = 0; i < 7; ++i) sn += (s.x[i] - s.cand[i]) * (s.x[i] - s.cand[i]);
  sn = sqrt(sn);
  if (sn <= 1e-8 * (s.x_norm + 1e-8)) { s.done = 1; return; }
  // FunctionToleranceReached
  if (fabs(s.x_cost - cand_cost) <= 1e-6 * s.x_cost) { s.done = 1; return; }
  const double rho = (s.x_cost - cand_cost) / s.mcc;
  bool success = false;
  if (rho > 1e-3) {
#pragma unroll
    for (int i = 0; i < 7; ++i) s.x[i] = s.cand[i];
    s.x_norm = norm7(s.x);
    s.x_cost = cand_cost;
#pragma unroll
    for (int k = 0; k < 21; ++k) s.H[k] = sums[1 + k];
#pragma unroll
    for (int k = 0; k < 6; ++k) s.g[k] = sums[22 + k];
    const double t = 2.0 * rho - 1.0;
    s.radius = fmin(1e16, s.radius / fmax(1.0 / 3.0, 1.0 - t * t * t));
    s.dfac = 2.0;
    s.reuse = 0;
    s.successful++;
    success = true;
  } else {
    s.radius /= s.dfac;
    s.dfac *= 2.0;
    s.reuse = 1;
  }
  if (s.iteration >= 4 || s.radius < 1e-32) { s.done = 1; return; }
  CTRL_STAMP(6, ts);
  next_step_wave(s, success, lane);
}

// Wave 0 of the block runs the control step in place on the LM state staged in LDS (sst): all 64 lanes read the
// same fields (LDS broadcast) and store identical values, so the state never has to fit in registers.
__device__ __forceinline__ void lm_logic_wave0(LMState& sst, const double* sums_lds) {
  if (threadIdx.x < 64) {
#ifdef FLOAM_CTRL_STAMPS
    const int lane = threadIdx.x;
    unsigned long long ts = __builtin_amdgcn_s_memrealtime();
#endif
    double sm[LM_NSUM];
#pragma unroll
    for (int k = 0; k < LM_NSUM; ++k) sm[k] = sums_lds[k];
    lm_logic(sst, sm, (int)threadIdx.x);
    CTRL_STAMP(2, ts);
#ifdef FLOAM_CTRL_STAMPS
    if (lane == 0) atomicAdd(&g_ctrl_stamps[3], 1ull);
#endif
  }
}

__device__ __forceinline__ void lm_logic_lds(LMState* __restrict__ st, const double* sums) {
  __shared__ LMState sst;
  constexpr int kWords = kStateWords;
  static_assert(sizeof(LMState) % sizeof(unsigned) == 0, "LMState must be a whole number of dwords");
  const unsigned* gsrc = reinterpret_cast<const unsigned*>(st);
  unsigned* ldst = reinterpret_cast<unsigned*>(&sst);
  for (int w = threadIdx.x; w < kWords; w += blockDim.x) ldst[w] = gsrc[w];
  __syncthreads();
  lm_logic_wave0(sst, sums);
  __syncthreads();
  unsigned* gdst = reinterpret_cast<unsigned*>(st);
  for (int w = threadIdx.x; w < kWords; w += blockDim.x) gdst[w] = ldst[w];
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
  lm_logic_lds(st, sums);
}

// One LM iteration in one launch (single-GPU path).  Block 0 is the control block; blocks 1..nblk evaluate.
// Block 0 stages the LM state while the others evaluate, waits for them (bounded spin on a device-scope arrival
// counter), reduces the partials in fixed block order and runs the control step on its first wave.
// Hand-off per MI355X_MICROARCH.md "Valid forms": plain stores -> s_waitcnt vmcnt(0) -> barrier -> lane-0 agent
// release -> s_waitcnt -> atomic; block 0: poll (agent-scope atomic load) -> agent acquire -> barrier -> plain loads.
__global__ __launch_bounds__(kTB) void lm_step(LMState* __restrict__ st, const double* __restrict__ erec,
                                               const uint8_t* __restrict__ evalid, int ecap, const int* __restrict__ d_ne,
                                               int ne_ub, const double* __restrict__ srec,
                                               const uint8_t* __restrict__ svalid, int scap,
                                               const int* __restrict__ d_ns, int ns_ub, int huber,
                                               double* __restrict__ partials, unsigned* __restrict__ counter,
                                               unsigned long long* __restrict__ dbg) {
  const int nblk = (int)gridDim.x - 1;
  if (blockIdx.x > 0) {
    if (st->done) return;
    eval_block<true>(st, erec, evalid, ecap, min(*d_ne, ne_ub), srec, svalid, scap, min(*d_ns, ns_ub), huber,
                     partials, blockIdx.x - 1, nblk);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the sc1 partials have reached L2-coherent memory
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  __shared__ LMState sst;
  __shared__ double sums[LM_NSUM];
  __shared__ int s_timeout;
  constexpr int kWords = kStateWords;
  static_assert(sizeof(LMState) % sizeof(unsigned) == 0, "LMState must be a whole number of dwords");
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  {
    const unsigned* gsrc = reinterpret_cast<const unsigned*>(st);
    unsigned* ldst = reinterpret_cast<unsigned*>(&sst);
    for (int w = threadIdx.x; w < kWords; w += blockDim.x) ldst[w] = gsrc[w];
  }
  __syncthreads();
  if (sst.done) return;
  unsigned long long t1 = 0, t2 = 0, t3 = 0;
  if (threadIdx.x == 0) {
    t1 = __builtin_amdgcn_s_memrealtime();
    int timeout = 1;   // bounded wait (~1 s)
    for (long long it = 0; it < (1ll << 24); ++it) {
      if (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)nblk) {
        timeout = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    s_timeout = timeout;
    t2 = __builtin_amdgcn_s_memrealtime();
  }
  __syncthreads();
  if (s_timeout) {   // never expected: give up on this solve instead of hanging the device
    if (threadIdx.x == 0) {
      st->done = 1;
      st->n_res = -1;
      *counter = 0u;
    }
    return;
  }
  reduce_partials_block<true>(partials, nblk, sums);   // sc1 loads: no invalidation needed
  t3 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) *counter = 0u;   // ready for the next launch (kernel boundary orders it)
  lm_logic_wave0(sst, sums);
  __syncthreads();
  {
    unsigned* gdst = reinterpret_cast<unsigned*>(st);
    const unsigned* lsrc = reinterpret_cast<const unsigned*>(&sst);
    for (int w = threadIdx.x; w < kWords; w += blockDim.x) gdst[w] = lsrc[w];
  }
  if (dbg && threadIdx.x == 0) {   // diagnostic stamps (100 MHz): stage, wait, reduce, control step + store
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const unsigned long long t4 = __builtin_amdgcn_s_memrealtime();
    atomicAdd(&dbg[0], t1 - t0);
    atomicAdd(&dbg[1], t2 - t1);
    atomicAdd(&dbg[2], t3 - t2);
    atomicAdd(&dbg[3], t4 - t3);
    atomicAdd(&dbg[4], 1ull);
  }
}

// ================================================================= LM step with the surf half from a Gram matrix
// With the squared loss (the launch default: "Cauchy" means no robust loss, Q3) a surf residual and its Jacobian are
// LINEAR in the record vector w of geom_kernel: with M the matrix of Eigen's q * v (M = I + 2 w [u]x + 2 [u]x^2,
// u = q.vec) and t' = t - o,
//   r      = c^T w,     c   = [M (row-major a,e) | t' | 1]     (w[12] = d + n.o absorbs the origin)
//   J[3+a] = n_a        = e_{9+a}^T w
//   J[i]   = (lp x n)_i = K_i^T w,  K_i[3c+e] = sum_b eps_ibc M_be,  K_i[9+c] = sum_b eps_ibc t_b,  K_i[12] = 0
// so the surf part of J^T J, J^T r and the cost are quadratic forms of the Gram matrix G = sum w w^T (reduced once
// per solve).  The edge records are still evaluated per record (EdgeAnalyticCostFunction's J has the direction
// nu/|nu|, which depends on the pose).  The residuals cancel inside G c (terms ~|p|^2 per record); recentring c on o
// keeps those terms independent of how far the pose is from the map origin.  Same function values as the
// per-residual evaluation in exact arithmetic; the rounding differs (~|G| eps in c^T G c, ~1e-9 of the cost at C3;
// poses agree with the per-record path to ~1e-14).
constexpr unsigned kEdgeEvalBlocks = 32;   // edge-only evaluation grid (fixed: fixed reduction order)
constexpr int kGramWords = kGram + 3;      // G (upper triangle) + the origin o it was built on

// G (LDS, full symmetric) -> the 29 surf sums at x (LDS out).  Called by the whole block (256 threads).
__device__ void surf_sums_from_gram(const double (&x)[7], const double* o /* shared [3] */,
                                    const double (*G)[kGramW] /* shared */, double n_surf, double* out /* shared */) {
  __shared__ double V[7][kGramW];   // K_0..K_5, c
  __shared__ double Y[7][kGramW];   // G V
  const int t = threadIdx.x;
  if (t < kGramW) {   // lanes 0..12 build one component of all 7 vectors
    const double qx = x[0], qy = x[1], qz = x[2], qw = x[3];
    const double U[3][3] = {{0, -qz, qy}, {qz, 0, -qx}, {-qy, qx, 0}};
    double Mm[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const double u2 = U[a][0] * U[0][b] + U[a][1] * U[1][b] + U[a][2] * U[2][b];
        Mm[a][b] = ((a == b) ? 1.0 : 0.0) + 2.0 * qw * U[a][b] + 2.0 * u2;
      }
    const double tp[3] = {x[4] - o[0], x[5] - o[1], x[6] - o[2]};   // c: recentred (d absorbed n.o)
    const double tf[3] = {x[4], x[5], x[6]};                        // K: the Jacobian's lp = M p + t itself
    const int m = t;   // component of w
    // register-resident selects instead of run-time array indexing (no scratch)
    auto Msel = [&](int r, int c) {
      double v = 0.0;
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b)
          if (a == r && b == c) v = Mm[a][b];
      return v;
    };
    auto vsel = [&](const double (&vv)[3], int k) { return k == 0 ? vv[0] : (k == 1 ? vv[1] : vv[2]); };
    double cm = 1.0;
    if (m < 9) cm = Msel(m / 3, m % 3);
    else if (m < 12) cm = vsel(tp, m - 9);
    V[6][m] = cm;
#pragma unroll
    for (int i = 0; i < 3; ++i) {   // K_i for i = 0..2 (lp x n)
      const int b1 = (i + 1) % 3, b2 = (i + 2) % 3;   // eps_{i b1 b2} = +1, eps_{i b2 b1} = -1
      double km = 0.0;
      if (m < 9) {
        const int c = m / 3, e = m % 3;   // w index 3c + e: sum_b eps_{ibc} M_be
        if (c == b2) km = Msel(b1, e);
        else if (c == b1) km = -Msel(b2, e);
      } else if (m < 12) {
        const int c = m - 9;              // sum_b eps_{ibc} t_b
        if (c == b2) km = vsel(tf, b1);
        else if (c == b1) km = -vsel(tf, b2);
      }
      V[i][m] = km;
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) V[3 + a][m] = (m == 9 + a) ? 1.0 : 0.0;   // K_{3+a} = e_{9+a}
  }
  __syncthreads();
  if (t < 7 * kGramW) {   // Y = G V
    const int v = t / kGramW, i = t % kGramW;
    double a = 0.0;
#pragma unroll
    for (int j = 0; j < kGramW; ++j) a += G[i][j] * V[v][j];
    Y[v][i] = a;
  }
  __syncthreads();
  if (t < LM_NSUM) {   // cost, J^T J upper (row-major), J^T r, count
    double s;
    if (t == 0) {
      double a = 0.0;
#pragma unroll
      for (int i = 0; i < kGramW; ++i) a += V[6][i] * Y[6][i];
      s = 0.5 * a;
    } else if (t < 22) {
      int hh = t - 1, ja = 0;
      while (hh >= 6 - ja) { hh -= 6 - ja; ++ja; }
      const int jb = ja + hh;
      double a = 0.0;
#pragma unroll
      for (int i = 0; i < kGramW; ++i) a += V[ja][i] * Y[jb][i];
      s = a;
    } else if (t < 28) {
      double a = 0.0;
#pragma unroll
      for (int i = 0; i < kGramW; ++i) a += V[t - 22][i] * Y[6][i];
      s = a;
    } else {
      s = n_surf;
    }
    out[t] = s;
  }
  __syncthreads();
}

// G of this solve into LDS: either reduced from the surf geometry blocks' partials (first evaluation of the solve;
// fixed order: 8 strips of 32 blocks, then the strips) and published to gmat with the origin o = x (no step has been
// taken yet), or unpacked from gv = gmat[t] (loaded by the caller together with the LM state).
__device__ void gram_load(const double* __restrict__ gpart, double* __restrict__ gmat, bool reduce, double gv,
                          const LMState& sst, double (*G)[kGramW], double* o) {
  __shared__ double s_gp[kGram][8];
  const int t = threadIdx.x;
  if (reduce) {
    for (int q = t; q < kGram * 8; q += blockDim.x) {
      const int e = q >> 3, p = q & 7;
      constexpr int per = kSurfGeomBlocks / 8;
      double v[per];
#pragma unroll
      for (int k = 0; k < per; ++k) v[k] = gpart[(p * per + k) * kGram + e];
      double a = 0.0;
#pragma unroll
      for (int k = 0; k < per; ++k) a += v[k];
      s_gp[e][p] = a;
    }
    __syncthreads();
  }
  if (t < kGram) {
    double a = gv;
    if (reduce) {
      a = s_gp[t][0];
#pragma unroll
      for (int p = 1; p < 8; ++p) a += s_gp[t][p];
      gmat[t] = a;
    }
    int i, j;
    gram_pair(t, i, j);
    G[i][j] = a;
    G[j][i] = a;
  } else if (t < kGramWords) {
    const int k = t - kGram;
    const double v = reduce ? sst.x[4 + k] : gv;
    if (reduce) gmat[t] = v;
    o[k] = v;
  }
  __syncthreads();
}

// One LM iteration in one launch, surf half from G.  Block 0 (control) stages the state and G and computes the
// surf sums at the evaluation point while blocks 1..nblk evaluate the edge records; then it waits for them (same
// hand-off as lm_step), adds the edge sums and runs the control step.
__global__ __launch_bounds__(kTB) void lm_step_gram(LMState* __restrict__ st, const double* __restrict__ erec,
                                                    const uint8_t* __restrict__ evalid, int ecap,
                                                    const int* __restrict__ d_ne, int ne_ub,
                                                    const double* __restrict__ gpart, double* __restrict__ gmat,
                                                    int reduce_g, double* __restrict__ partials,
                                                    unsigned* __restrict__ counter, unsigned long long* __restrict__ dbg) {
  const int nblk = (int)gridDim.x - 1;
  if (blockIdx.x > 0) {
    const unsigned long long e0 = __builtin_amdgcn_s_memrealtime();
    if (st->done) return;
    eval_block<true>(st, erec, evalid, ecap, min(*d_ne, ne_ub), nullptr, nullptr, 0, 0, 0, partials, blockIdx.x - 1,
                     nblk);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the sc1 partials have reached L2-coherent memory
    __syncthreads();
    if (threadIdx.x == 0) {
      if (dbg) {   // evaluation block window: first start, last arrival, summed duration
        const unsigned long long e1 = __builtin_amdgcn_s_memrealtime();
        atomicMin(&dbg[25], e0);
        atomicMax(&dbg[26], e1);
        atomicAdd(&dbg[5], e1 - e0);
        atomicAdd(&dbg[6], 1ull);
      }
      __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  __shared__ LMState sst;
  __shared__ double G[kGramW][kGramW];
  __shared__ double o[3];
  __shared__ double ssum[LM_NSUM];
  __shared__ double sums[LM_NSUM];
  __shared__ int s_timeout;
  constexpr int kWords = kStateWords;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  double gv = 0.0;
  {   // the LM state and (after the first evaluation of the solve) G + o, in one round trip
    const unsigned* gsrc = reinterpret_cast<const unsigned*>(st);
    unsigned* ldst = reinterpret_cast<unsigned*>(&sst);
    if (!reduce_g && threadIdx.x < kGramWords) gv = gmat[threadIdx.x];
    for (int w = threadIdx.x; w < kWords; w += blockDim.x) ldst[w] = gsrc[w];
  }
  __syncthreads();
  if (sst.done) return;
  gram_load(gpart, gmat, reduce_g != 0, gv, sst, G, o);
  {
    double x[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) x[k] = sst.phase == 0 ? sst.x[k] : sst.cand[k];
    surf_sums_from_gram(x, o, G, (double)sst.corr_surf, ssum);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime(), t2 = 0, t3 = 0;
  if (threadIdx.x == 0) {
    int timeout = 1;   // bounded wait (~1 s)
    for (long long it = 0; it < (1ll << 24); ++it) {
      if (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)nblk) {
        timeout = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    s_timeout = timeout;
    t2 = __builtin_amdgcn_s_memrealtime();
  }
  __syncthreads();
  if (s_timeout) {   // never expected: give up on this solve instead of hanging the device
    if (threadIdx.x == 0) {
      st->done = 1;
      st->n_res = -1;
      *counter = 0u;
    }
    return;
  }
  reduce_partials_block<true>(partials, nblk, sums);
  if (threadIdx.x < LM_NSUM) sums[threadIdx.x] = sums[threadIdx.x] + ssum[threadIdx.x];   // edge + surf
  __syncthreads();
  t3 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) *counter = 0u;   // ready for the next launch (kernel boundary orders it)
  lm_logic_wave0(sst, sums);
  __syncthreads();
  {
    unsigned* gdst = reinterpret_cast<unsigned*>(st);
    const unsigned* lsrc = reinterpret_cast<const unsigned*>(&sst);
    for (int w = threadIdx.x; w < kWords; w += blockDim.x) gdst[w] = lsrc[w];
  }
  if (dbg && threadIdx.x == 0) {   // stamps (100 MHz): stage + G + surf sums, wait, reduce, control step + store
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    const unsigned long long t4 = __builtin_amdgcn_s_memrealtime();
    atomicAdd(&dbg[0], t1 - t0);
    atomicAdd(&dbg[1], t2 - t1);
    atomicAdd(&dbg[2], t3 - t2);
    atomicAdd(&dbg[3], t4 - t3);
    atomicAdd(&dbg[4], 1ull);
    const unsigned long long first = dbg[25], last = dbg[26];
    atomicAdd(&dbg[7], first > t0 ? first - t0 : 0ull);   // control start -> first evaluation block start
    atomicAdd(&dbg[27], last > t0 ? last - t0 : 0ull);    // control start -> last arrival
    dbg[25] = ~0ull;
    dbg[26] = 0ull;
  }
}

// A whole Ceres solve in one launch (single GPU, squared loss): block 0 is the control block, blocks 1..nblk
// evaluate the edge records; the surf half of every evaluation comes from G (reduced once, at the start, by the
// control block while the evaluation blocks run iteration zero).  The blocks stay resident across the up to 5
// evaluations and hand off without cache invalidations (sc1 words, MI355X_MICROARCH.md "Valid forms"):
//   evaluation -> control: the block's 29 partial sums stored sc1, drained, then one agent-scope add on `cnt`;
//   control -> evaluation: the next point (7 doubles) stored sc1 into `point`, drained, then the word
//        go = (done << 7) | evaluations released.  go and cnt are zero at the launch (the kNN launch of the solve
//        clears go; the control block leaves cnt at zero).
// All 1 + nblk blocks must be co-resident (33 blocks); every wait is bounded (~1 s) and a timeout ends the solve
// with st->n_res = -1, which the host reports as an error.
__device__ __forceinline__ bool wait_u32_geq(unsigned* p, unsigned target) {
  for (long long it = 0; it < (1ll << 24); ++it) {
    if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}

__global__ __launch_bounds__(kTB) void lm_solve_gram(LMState* __restrict__ st, const double* __restrict__ erec,
                                                     const uint8_t* __restrict__ evalid, int ecap,
                                                     const int* __restrict__ d_ne, int ne_ub,
                                                     const double* __restrict__ gpart, double* __restrict__ gmat,
                                                     double* __restrict__ partials, unsigned* __restrict__ cnt,
                                                     unsigned long long* __restrict__ dbg) {
  const int nblk = (int)gridDim.x - 1;
  unsigned long long* go = &st->go;
  double* point = st->point;
  __shared__ int s_flag;
  if (blockIdx.x > 0) {
    const int ne = min(*d_ne, ne_ub);
    __shared__ double s_x[7];
    // the thread's first edge record stays in registers across the evaluations (all of them at C3: ne <= 8192)
    const int blk = blockIdx.x - 1, stride = nblk * kTB, i0 = blk * kTB + threadIdx.x;
    double f0[9];
    const bool has0 = i0 < ne && (evalid[i0] & 1);
#pragma unroll
    for (int k = 0; k < 9; ++k) f0[k] = has0 ? erec[k * ecap + i0] : 0.0;
    for (int it = 0; it < 5; ++it) {
      if (it == 0) {   // iteration zero evaluates at x (set by the kNN launch; kernel boundary)
        if (threadIdx.x == 0) s_flag = st->done ? 1 : 0;
        if (threadIdx.x < 7) s_x[threadIdx.x] = st->x[threadIdx.x];
      } else {         // wait for the control step of evaluation it - 1, then read the point it released
        if (threadIdx.x == 0) {
          int f = 2;   // 0: go, 1: done, 2: timeout
          for (long long k = 0; k < (1ll << 24); ++k) {
            const unsigned long long g = __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (g & 0x80ull) { f = 1; break; }
            if ((int)(g & 0x7F) >= it) { f = 0; break; }
            __builtin_amdgcn_s_sleep(1);
          }
          s_flag = f;
        }
        __syncthreads();
        if (threadIdx.x < 7) s_x[threadIdx.x] = load_sc1(&point[threadIdx.x]);
      }
      __syncthreads();
      if (s_flag) return;
      double x[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) x[k] = s_x[k];
      double acc[LM_NSUM];
#pragma unroll
      for (int k = 0; k < LM_NSUM; ++k) acc[k] = 0.0;
      if (has0) {
        double J[6];
        const double r = edge_residual(x, f0, J);
        accumulate_residual(acc, r, J, 0);
      }
      for (int idx = i0 + stride; idx < ne; idx += stride) {   // beyond one record per thread
        if (!(evalid[idx] & 1)) continue;
        double f[9], J[6];
#pragma unroll
        for (int k = 0; k < 9; ++k) f[k] = erec[k * ecap + idx];
        const double r = edge_residual(x, f, J);
        accumulate_residual(acc, r, J, 0);
      }
      store_block_partials<true>(acc, partials, blk, nblk);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the sc1 partials have reached L2-coherent memory
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  // control block
  __shared__ LMState sst;
  __shared__ double G[kGramW][kGramW];
  __shared__ double o[3];
  __shared__ double ssum[LM_NSUM];
  __shared__ double sums[LM_NSUM];
  constexpr int kWords = kStateWords;
  {
    const unsigned* gsrc = reinterpret_cast<const unsigned*>(st);
    unsigned* ldst = reinterpret_cast<unsigned*>(&sst);
    for (int w = threadIdx.x; w < kWords; w += blockDim.x) ldst[w] = gsrc[w];
  }
  __syncthreads();
  if (sst.done) return;   // (the evaluation blocks saw st->done too)
  {
    const double gv = threadIdx.x < kGramWords ? gmat[threadIdx.x] : 0.0;
    gram_load(gpart, gmat, false, gv, sst, G, o);
  }
  unsigned long long t_surf = 0, t_wait = 0, t_reduce = 0, t_ctrl = 0, n_it = 0;
  int it = 0;
  bool failed = false;
  for (; it < 5 && !sst.done; ++it) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    {   // the surf half at this evaluation's point, while the evaluation blocks work
      double x[7];
#pragma unroll
      for (int k = 0; k < 7; ++k) x[k] = sst.phase == 0 ? sst.x[k] : sst.cand[k];
      surf_sums_from_gram(x, o, G, (double)sst.corr_surf, ssum);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) s_flag = wait_u32_geq(cnt, (unsigned)(nblk * (it + 1))) ? 0 : 1;
    __syncthreads();
    if (s_flag) {
      failed = true;
      break;
    }
    const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    reduce_partials_block<true>(partials, nblk, sums);
    if (threadIdx.x < LM_NSUM) sums[threadIdx.x] = sums[threadIdx.x] + ssum[threadIdx.x];   // edge + surf
    __syncthreads();
    const unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    lm_logic_wave0(sst, sums);
    __syncthreads();
    if (threadIdx.x == 0) {   // release the next evaluation point (cand after a step; x never changes here)
      if (!sst.done) {
#pragma unroll
        for (int k = 0; k < 7; ++k) store_sc1(&point[k], sst.phase == 0 ? sst.x[k] : sst.cand[k]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __hip_atomic_store(go, (sst.done ? 0x80ull : 0ull) | (unsigned long long)(it + 1), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    const unsigned long long t4 = __builtin_amdgcn_s_memrealtime();
    t_surf += t1 - t0;
    t_wait += t2 - t1;
    t_reduce += t3 - t2;
    t_ctrl += t4 - t3;
    ++n_it;
  }
  __syncthreads();
  {   // the final state for the host gather / the next launches (kernel boundary makes it visible)
    unsigned* gdst = reinterpret_cast<unsigned*>(st);
    const unsigned* lsrc = reinterpret_cast<const unsigned*>(&sst);
    for (int w = threadIdx.x; w < kWords; w += blockDim.x) gdst[w] = lsrc[w];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (failed) {   // never expected: end the solve, release the evaluation blocks, report through n_res
      st->done = 1;
      st->n_res = -1;
      __hip_atomic_store(go, 0x80ull | 0x7Full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (it == 0) {   // done before the first evaluation: let any waiting evaluation block go
      __hip_atomic_store(go, 0x80ull | 0x7Full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *cnt = 0u;   // every evaluation block has arrived for the last released evaluation (kernel boundary orders it)
    if (dbg && n_it) {   // diagnostic stamps (100 MHz): surf sums, wait, reduce, control step + publish
      atomicAdd(&dbg[0], t_surf);
      atomicAdd(&dbg[1], t_wait);
      atomicAdd(&dbg[2], t_reduce);
      atomicAdd(&dbg[3], t_ctrl);
      atomicAdd(&dbg[4], n_it);
    }
  }
}

__global__ __launch_bounds__(kTB) void lm_reduce(const double* __restrict__ partials, int nblk, double* __restrict__ out) {
  __shared__ double sums[LM_NSUM];
  reduce_partials_block(partials, nblk, sums);
  if (threadIdx.x < LM_NSUM) out[threadIdx.x] = sums[threadIdx.x];
}

}  // namespace

// ===================================================================================== launchers
void deskew_bridge_launch(const LMState* d_st, OdomDev* s, double scan_period, PointRec* edge, const int* d_ne,
                          int ne_ub, PointRec* surf, const int* d_ns, int ns_ub, hipStream_t stream,
                          const GatherArgs& gather) {
  const unsigned nb = std::max(1u, std::min(div_up(std::max(ne_ub + ns_ub, 1), kTB), 1024u));
  hipLaunchKernelGGL(deskew_bridge, dim3(nb), dim3(kTB), 0, stream, d_st, s, scan_period, edge, d_ne, ne_ub, surf,
                     d_ns, ns_ub, gather);
  FLOAM_LAUNCH_CHECK();
}

void lm_init_launch(LMState* d_st, const double* x0, hipStream_t st) {
  X7 x{};
  if (x0) {
    for (int k = 0; k < 7; ++k) x.v[k] = x0[k];
    x.set = 1;
  }
  hipLaunchKernelGGL(lm_init, dim3(1), dim3(64), 0, st, d_st, x);
  FLOAM_LAUNCH_CHECK();
}

// One D2H per update: LM state + query / map counts (+ profiling bytes) gathered into one block.
// Called by every thread of one block.
__device__ __forceinline__ void gather_block(const LMState* __restrict__ lm, const int* __restrict__ dcnt,
                                             const int* __restrict__ mapE_count, const int* __restrict__ mapS_count,
                                             const int* __restrict__ fe_status,
                                             const unsigned long long* __restrict__ prof,
                                             UpdateStatus* __restrict__ out, OdomDev* __restrict__ s, int mode) {
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
    if (mode & GATHER_FINISH) {
      if (mode & GATHER_AFTER_MID) s->last_odom = s->mid;
      s->odom = params_to_pose(lm->x);   // x == the prediction when the solve did not run (gate, no residuals)
    }
    if (mode & GATHER_KEYFRAME) {   // KeyFrameUpdate (odomEstimationClass.cpp:320-343)
      bool key = true;
      if (!(mode & GATHER_KEYFRAME_FIRST) && s->kf_count > 0) {
        const Pose delta = pose_mul(pose_inverse(s->kf), s->odom);
        const double dm = sqrt(delta.t[0] * delta.t[0] + delta.t[1] * delta.t[1] + delta.t[2] * delta.t[2]);
        const double dr = rotation_angle(delta.R);
        key = dm > 0.07 || dr > 2 * M_PI / 180.0;
      }
      if (key) {
        s->kf = s->odom;
        s->kf_count = min(s->kf_count + 1, 3);
      }
      s->kf_flag = key ? 1 : 0;
      out->kf_flag = s->kf_flag;
    }
    out->odom = s->odom;
    out->last_odom = s->last_odom;
  }
}

__global__ void gather_status(const LMState* __restrict__ lm, const int* __restrict__ dcnt,
                              const int* __restrict__ mapE_count, const int* __restrict__ mapS_count,
                              const int* __restrict__ fe_status, const unsigned long long* __restrict__ prof,
                              UpdateStatus* __restrict__ out, OdomDev* __restrict__ s, int mode) {
  gather_block(lm, dcnt, mapE_count, mapS_count, fe_status, prof, out, s, mode);
}

void gather_status_launch(const LMState* lm, const int* dcnt, const int* mapE_count, const int* mapS_count,
                          const int* fe_status, const unsigned long long* prof, UpdateStatus* out, OdomDev* s,
                          int mode, hipStream_t st) {
  hipLaunchKernelGGL(gather_status, dim3(1), dim3(256), 0, st, lm, dcnt, mapE_count, mapS_count, fe_status, prof,
                     out, s, mode);
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

static void corr_args(const QuerySet& qe, const Grid& ge, const PointRec* mapE, CorrSet& ce, const QuerySet& qs,
                      const Grid& gs, const PointRec* mapS, CorrSet& cs, unsigned long long* dbg, CorrArgs& E,
                      CorrArgs& S) {
  ce.reserve(std::max(qe.n_ub, 1), EDGE_FIELDS);
  cs.reserve(std::max(qs.n_ub, 1), SURF_FIELDS);
  (void)mapE;
  (void)mapS;
  E = CorrArgs{qe.pts, qe.d_n, qe.n_ub, ge.pts.p, ge.coarse.p, ge.bits, ge.mask, ge.xyz.p, ce.rec.p,
               ce.valid.p, ce.nnxyz.p, ce.cap, dbg};
  S = CorrArgs{qs.pts, qs.d_n, qs.n_ub, gs.pts.p, gs.coarse.p, gs.bits, gs.mask, gs.xyz.p, cs.rec.p,
               cs.valid.p, cs.nnxyz.p, cs.cap, dbg ? dbg + 8 : nullptr};
}

template <int G, int U, int W = 1>
static void knn_launch_t(LMState* d_st, const X7& x0, const double* x0_dev, const QuerySet& qe, const QuerySet& qs, const CorrArgs& E,
                         const CorrArgs& S, const int* d_me, const int* d_ms, int rank, int world, hipStream_t st) {
  static const unsigned cap = [] {   // FLOAM_KNN_MAXBLOCKS: grid cap per query set (tuning only)
    const char* v = std::getenv("FLOAM_KNN_MAXBLOCKS");
    return v ? (unsigned)std::atoi(v) : 8192u;
  }();
  const int nE = qe.grid_hint > 0 ? std::min(qe.grid_hint, qe.n_ub) : qe.n_ub;
  const int nS = qs.grid_hint > 0 ? std::min(qs.grid_hint, qs.n_ub) : qs.n_ub;
  const unsigned nbE = std::min(div_up((size_t)std::max(nE, 1) * G, kTB), std::min(cap, 4096u));
  const unsigned nbS = std::min(div_up((size_t)std::max(nS, 1) * G, kTB), cap);
  hipLaunchKernelGGL((knn_kernel<G, U, W>), dim3(nbE + nbS), dim3(kTB), 0, st, d_st, x0, x0_dev, E, S, (int)nbE, d_me,
                     d_ms, rank, world);
  FLOAM_LAUNCH_CHECK();
}

void knn_launch(LMState* d_st, const double* x0, const double* x0_dev, const QuerySet& qe, const Grid& ge, const PointRec* mapE,
                CorrSet& ce, const QuerySet& qs, const Grid& gs, const PointRec* mapS, CorrSet& cs, const int* d_me,
                const int* d_ms, int rank, int world, hipStream_t st, unsigned long long* dbg) {
  CorrArgs E, S;
  corr_args(qe, ge, mapE, ce, qs, gs, mapS, cs, dbg, E, S);
  X7 x{};
  if (x0) {
    for (int k = 0; k < 7; ++k) x.v[k] = x0[k];
    x.set = 1;
  }
  if (qe.n_ub <= 0 && qs.n_ub <= 0) {   // nothing to search: still start the solve
    hipLaunchKernelGGL(lm_init_dev, dim3(1), dim3(64), 0, st, d_st, x, x0_dev);
    FLOAM_LAUNCH_CHECK();
    return;
  }
  static const int variant = [] {   // FLOAM_KNN_VARIANT: lanes per query x loads in flight (tuning only)
    const char* v = std::getenv("FLOAM_KNN_VARIANT");
    return v ? std::atoi(v) : 0;
  }();
  switch (variant) {
    case 1: knn_launch_t<8, 4>(d_st, x, x0_dev, qe, qs, E, S, d_me, d_ms, rank, world, st); break;
    case 2: knn_launch_t<8, 2>(d_st, x, x0_dev, qe, qs, E, S, d_me, d_ms, rank, world, st); break;
    case 3: knn_launch_t<32, 2>(d_st, x, x0_dev, qe, qs, E, S, d_me, d_ms, rank, world, st); break;
    case 4: knn_launch_t<16, 2>(d_st, x, x0_dev, qe, qs, E, S, d_me, d_ms, rank, world, st); break;
    case 6: knn_launch_t<16, 4, 6>(d_st, x, x0_dev, qe, qs, E, S, d_me, d_ms, rank, world, st); break;
    case 7: knn_launch_t<16, 2, 6>(d_st, x, x0_dev, qe, qs, E, S, d_me, d_ms, rank, world, st); break;
    case 8: knn_launch_t<16, 2, 8>(d_st, x, x0_dev, qe, qs, E, S, d_me, d_ms, rank, world, st); break;
    default: knn_launch_t<kGroupDefault, kUnrollDefault, 6>(d_st, x, x0_dev, qe, qs, E, S, d_me, d_ms, rank, world, st); break;
  }
}

void geom_launch(LMState* d_st, const QuerySet& qe, const Grid& ge, const PointRec* mapE, CorrSet& ce,
                 const QuerySet& qs, const Grid& gs, const PointRec* mapS, CorrSet& cs, double* gpart, double* gmat,
                 unsigned* gcnt, hipStream_t st) {
  CorrArgs E, S;
  corr_args(qe, ge, mapE, ce, qs, gs, mapS, cs, nullptr, E, S);
  if (qe.n_ub <= 0 && qs.n_ub <= 0) return;
  const unsigned gE = div_up(std::max(qe.n_ub, 1), kTB);
  hipLaunchKernelGGL(geom_kernel, dim3(gE + kSurfGeomBlocks), dim3(kTB), 0, st, d_st, E, S, (int)gE, gpart, gmat,
                     gcnt);
  FLOAM_LAUNCH_CHECK();
}

void knn_traffic_launch(const LMState* d_st, const QuerySet& q, const Grid& g, const PointRec* map, CorrSet& c,
                        int rank, int world, DevBuf<unsigned long long>& set,
                        unsigned long long* d_bytes, hipStream_t st) {
  if (q.n_ub <= 0) return;
  int bits = 10;
  while ((1 << bits) < 64 * q.n_ub) ++bits;   // distinct occupied cells scanned (<= 27 per query)
  set.reserve((size_t)1 << bits);
  CorrArgs A, B;
  corr_args(q, g, map, c, q, g, map, c, nullptr, A, B);
  for (int level = 0; level < 2; ++level) {
    FLOAM_HIP(hipMemsetAsync(set.p, 0xFF, sizeof(unsigned long long) << bits, st));
    hipLaunchKernelGGL(knn_traffic, dim3(div_up(q.n_ub, kTB)), dim3(kTB), 0, st, d_st, A, rank, world,
                       level, set.p, (1u << bits) - 1u, bits, d_bytes);
    FLOAM_LAUNCH_CHECK();
  }
}

int lm_eval_launch(const LMState* d_st, const CorrSet& ce, const int* d_ne, int ne_ub, const CorrSet& cs,
                   const int* d_ns, int ns_ub, bool huber, double* partials, hipStream_t st) {
  // a fixed evaluation grid: the partition of the records over blocks (hence the fixed reduction order) must not
  // depend on the host's upper bounds, only on the device counts
  const int nblk = (int)kEvalBlocks;
  (void)ne_ub;
  (void)ns_ub;
  hipLaunchKernelGGL(lm_eval, dim3(nblk), dim3(kTB), 0, st, d_st, ce.rec.p, ce.valid.p, ce.cap, d_ne, ne_ub,
                     cs.rec.p, cs.valid.p, cs.cap, d_ns, ns_ub, huber ? 1 : 0, partials);
  FLOAM_LAUNCH_CHECK();
  return nblk;
}

void lm_step_launch(LMState* d_st, const CorrSet& ce, const int* d_ne, int ne_ub, const CorrSet& cs,
                    const int* d_ns, int ns_ub, bool huber, double* partials, unsigned* counter, hipStream_t st,
                    unsigned long long* dbg) {
  // a fixed evaluation grid: the partition of the records over blocks (hence the fixed reduction order) must not
  // depend on the host's upper bounds, only on the device counts
  const int nblk = (int)kEvalBlocks;
  (void)ne_ub;
  (void)ns_ub;
  hipLaunchKernelGGL(lm_step, dim3(nblk + 1), dim3(kTB), 0, st, d_st, ce.rec.p, ce.valid.p, ce.cap, d_ne, ne_ub,
                     cs.rec.p, cs.valid.p, cs.cap, d_ns, ns_ub, huber ? 1 : 0, partials, counter, dbg);
  FLOAM_LAUNCH_CHECK();
}

void lm_solve_gram_launch(LMState* d_st, const CorrSet& ce, const int* d_ne, int ne_ub, const double* gpart,
                          double* gmat, double* partials, unsigned* cnt, hipStream_t st, unsigned long long* dbg) {
  hipLaunchKernelGGL(lm_solve_gram, dim3(kEdgeEvalBlocks + 1), dim3(kTB), 0, st, d_st, ce.rec.p, ce.valid.p, ce.cap,
                     d_ne, ne_ub, gpart, gmat, partials, cnt, dbg);
  FLOAM_LAUNCH_CHECK();
}

void ctrl_stamps_print() {
#ifdef FLOAM_CTRL_STAMPS
  unsigned long long h[8];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_ctrl_stamps), sizeof(h)) == hipSuccess && h[3])
    std::fprintf(stderr, "[floam ctrl] %llu control steps: solve_step %.2f us, se3_plus %.2f us (per step), whole %.2f us\n",
                 h[3], h[0] / (double)h[3] / 100.0, h[1] / (double)h[3] / 100.0, h[2] / (double)h[3] / 100.0);
#endif
}

bool lm_gram_supported(bool huber) { return !huber; }
size_t lm_gram_partials() { return (size_t)(kSurfGeomBlocks + kGramGroups) * kGram; }
int lm_gram_counters() { return kGramGroups + 1; }
size_t lm_gram_words() { return (size_t)kGramWords; }

void lm_step_gram_launch(LMState* d_st, const CorrSet& ce, const int* d_ne, int ne_ub, const double* gpart,
                         double* gmat, bool first, double* partials, unsigned* counter, hipStream_t st,
                         unsigned long long* dbg) {
  hipLaunchKernelGGL(lm_step_gram, dim3(kEdgeEvalBlocks + 1), dim3(kTB), 0, st, d_st, ce.rec.p, ce.valid.p, ce.cap,
                     d_ne, ne_ub, gpart, gmat, first ? 1 : 0, partials, counter, dbg);
  FLOAM_LAUNCH_CHECK();
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
