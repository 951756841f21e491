// The Levenberg-Marquardt solve of updatePointsToMap on gfx950: ceres::Solve with LEVENBERG_MARQUARDT, DENSE_QR and
// max_num_iterations = 4 (src/odomEstimationClass.cpp:95-108) over the residual blocks of src/lidarOptimization.cpp
// (EdgeAnalyticCostFunction :12-43, SurfNormAnalyticCostFunction :51-74, PoseSE3Parameterization :77-140).  The
// Ceres 1.13 TrustRegionMinimizer + LevenbergMarquardtStrategy control is restated in control_step / lm_step
// (oracle/odom.cpp ceres_solve is the CPU restatement).
//
// Single GPU — lm_solve, ONE launch per solve, no control block.  Every active block (256 threads) keeps its records
// in registers across the up to five evaluations, evaluates them at the current point, publishes its 29 partial sums
// as data-tagged 8-byte granules (MI355X_MICROARCH.md "handoff-1to1": one sc1 store per granule, {tag, 32 data
// bits}; the consumer polls until every granule carries the tag it expects; no flags, counters or drains), then
// gathers every active block's granules, summing them in a fixed order as they arrive (gather_blocks), and runs the
// Ceres control step on its wave 0 over the LM state in LDS.  All blocks compute the same bits, so the next point is
// known everywhere without a control -> evaluation hop: one hand-off per evaluation.  Tags are epoch + evaluation
// index, with the epoch advanced by 8 at every solve (lm_reset), so a granule of an earlier evaluation or solve never
// matches and nothing is ever cleared.  Every poll is bounded (~0.3 s); a timeout ends the solve with n_res = -1
// (FLOAM_ERR_DEVICE on the host).
//
// Modes (LM_*): GRAM — squared loss (the launch default, Q3): the surf half of every evaluation comes from the Gram
// matrix of the surf records (exact in real arithmetic, see surf_sums_wave), formed by wave 3 of every block beside
// the edge records of waves 0..2; otherwise (Huber, fp32) all 4 waves evaluate records of both kinds.  FP32:
// residuals, Jacobians and the per-thread sums in float (the C5 precision sweep, BASELINE.json configs[4]);
// reductions and control in double.
//
// Multi-GPU — lm_shard_eval: one launch per evaluation, the control step of the previous evaluation (on the
// all-reduced sums) run redundantly by every block, then this rank's block partials reduced in fixed order by the
// last-arriving block into the 29 sums the host all-reduces (RCCL) between the launches.
//
// Fixed reduction orders throughout (thread -> 8 strips -> block; blocks -> 8 strips -> total), so the result
// does not depend on timing.  The sharded path on one rank agrees with the resident solve to a few ulps (lm.o is built
// with FMA contraction, and the compiler may contract the two kernels' evaluations differently); its LM decisions are
// identical.
#include <cfloat>
#include <cstdio>
#include <climits>

#include "lm_eval.hpp"
#include "odom_kernels.hpp"

namespace floam {

namespace {
using namespace lmev;
constexpr int kTB = 256;     // solve blocks: 4 waves, one per SIMD (the control wave keeps the LM state in 512 registers)
constexpr int kStrips = 8;   // block_sums strips
constexpr long long kSpin = 1ll << 23;   // bounded polls (s_sleep 1 each): ~0.3 s

// LDS written by some lanes of a wave and read by others of the same wave: DS ops of one wave execute in order, so
// only the compiler has to be kept from reordering
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// record slot (edge: 9 fields, surf: 7) of the device-resident correspondence arrays, converted to R
template <typename R, int N>
__device__ __forceinline__ void load_rec(const double* __restrict__ rec, int cap, int i, R (&f)[9]) {
#pragma unroll
  for (int k = 0; k < 9; ++k) f[k] = k < N ? (R)rec[k * cap + i] : R(0);
}

// thread sums of the record threads [0, NR) -> the block's 29 sums, fixed order: strip p of component c (8 strips,
// 29 x 8 = 232 threads) adds threads p, p + 8, p + 16, ... (the strip threads read consecutive LDS words: no bank
// conflicts), then the 8 strips are added in order.  Returns, to thread t < 58, the sum of component t >> 1 (the
// caller publishes it in two halves); no barrier after the last LDS read of `strip`.
template <int NR>
constexpr int red_stride() { return NR + 1; }   // odd row stride (in doubles): the 8 rows a wave reads hit 8 bank sets

// the 8 strip sums of component c live in lanes 8c .. 8c + 7 of one wave: a fixed butterfly gives every one of them
// the same total (each step adds two values, commutatively, so all eight lanes compute the same bits)
// (DPP lane moves, no LDS crossbar round trip: quad_perm xor 1, quad_perm xor 2, then the half-row mirrored — lane i
// with 7 - i pairs the two uniform quads exactly as xor 4 did, so the bits are those of the xor butterfly)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
__device__ __forceinline__ double strip8_total(double v) {
  v += dpp_f64<0xB1>(v);
  v += dpp_f64<0x4E>(v);
  v += dpp_f64<0x141>(v);
  return v;
}

// thread sums of the record threads [0, NR) -> the block's 29 sums, fixed order: strip p of component c (8 strips,
// threads 8c + p) adds threads p, p + 8, p + 16, ... (the strip threads read consecutive LDS words: no bank
// conflicts), then the 8 strips by strip8_total.  Returns, to threads 8c and 8c + 1 (c < 29), the sum of component c
// (the caller publishes it in two halves); one block barrier.
template <int NR>
__device__ __forceinline__ double block_sums(const double (&acc)[LM_NSUM], double* red /* LDS [LM_NSUM][NR + 1] */) {
  static_assert(NR % kStrips == 0 && LM_NSUM * kStrips <= kTB && kStrips == 8, "strip layout");
  constexpr int RS = red_stride<NR>();
  const int t = threadIdx.x;
  if (t < NR)
#pragma unroll
    for (int k = 0; k < LM_NSUM; ++k) red[k * RS + t] = acc[k];
  __syncthreads();
  double v = 0.0;
  if (t < LM_NSUM * kStrips) {
    const int c = t / kStrips, p = t % kStrips;
#pragma unroll 4
    for (int j = 0; j < NR / kStrips; ++j) v += red[c * RS + j * kStrips + p];
  }
  return strip8_total(v);   // (threads >= 232 hold zeros)
}

// block partials P(c, b) (c < 29, b < nblk) -> 29 sums in out (LDS), fixed order: component c sums 8 strips of
// consecutive blocks in block order, then the strip totals by strip8_total; + add[c] when add is given (the surf half)
template <typename Load>
__device__ __forceinline__ void reduce_blocks(Load P, int nblk, double* out /* LDS [LM_NSUM] */,
                                              const double* add = nullptr /* LDS [LM_NSUM] */) {
  const int t = threadIdx.x;
  double v = 0.0;
  if (t < LM_NSUM * 8) {
    const int c = t >> 3, p = t & 7;
    const int per = (nblk + 7) / 8;
    const int b0 = p * per, b1 = min(nblk, b0 + per);
    for (int b = b0; b < b1; ++b) v += P(c, b);
  }
  v = strip8_total(v);
  if (t < LM_NSUM * 8 && (t & 7) == 0) out[t >> 3] = add ? v + add[t >> 3] : v;
  __syncthreads();
}

// This block's share of one evaluation at x: every thread's records (the first one held in registers by the caller),
// summed per thread in R, then reduced in double.  Record index space: edge slots [0, ne), then surf slots.
template <bool HUBER, typename R>
__device__ __forceinline__ void eval_records(const R (&x)[7], bool has0, bool edge0, const R (&f0)[9], int i1,
                                             int stride, int ne, int total, const double* __restrict__ erec,
                                             const uint8_t* __restrict__ evalid, int ecap,
                                             const double* __restrict__ srec, const uint8_t* __restrict__ svalid,
                                             int scap, double (&accd)[LM_NSUM]) {
  R acc[LM_NSUM];
#pragma unroll
  for (int k = 0; k < LM_NSUM; ++k) acc[k] = R(0);
  if (has0) {
    R J[6];
    const R r = edge0 ? edge_residual<R>(x, f0, J) : surf_residual<R>(x, f0, J);
    accumulate_residual<HUBER, R>(acc, r, J);
  }
  for (int idx = i1; idx < total; idx += stride) {   // beyond the record held in registers
    R f[9], J[6], r;
    if (idx < ne) {
      if (!(evalid[idx] & 1)) continue;
      load_rec<R, EDGE_FIELDS>(erec, ecap, idx, f);
      r = edge_residual<R>(x, f, J);
    } else {
      const int s = idx - ne;
      if (!(svalid[s] & 1)) continue;
      load_rec<R, SURF_FIELDS>(srec, scap, s, f);
      r = surf_residual<R>(x, f, J);
    }
    accumulate_residual<HUBER, R>(acc, r, J);
  }
#pragma unroll
  for (int k = 0; k < LM_NSUM; ++k) accd[k] = (double)acc[k];
}

// ===================================================================================== surf half from G
// With the squared loss a surf residual and its Jacobian are LINEAR in the record vector w of geom_kernel: with M the
// matrix of Eigen's q * v (M = I + 2 w [u]x + 2 [u]x^2, u = q.vec) and t' = t - o,
//   r      = c^T w,     c   = [M (row-major a,e) | t' | 1]     (w[12] = d + n.o absorbs the origin)
//   J[3+a] = n_a        = e_{9+a}^T w
//   J[i]   = (lp x n)_i = K_i^T w,  K_i[3c+e] = sum_b eps_ibc M_be,  K_i[9+c] = sum_b eps_ibc t_b,  K_i[12] = 0
// so the surf part of J^T J, J^T r and the cost are quadratic forms of G = sum w w^T (reduced once per solve by the
// geometry launch).  The edge records are evaluated per record (EdgeAnalyticCostFunction's J has the direction
// nu/|nu|, which depends on the pose).  Recentring c on o keeps the cancellation inside G c independent of how far the
// pose is from the map origin.  Same function values as the per-residual evaluation in exact arithmetic; the rounding
// differs (~|G| eps in c^T G c, ~1e-9 of the cost at C3; poses agree with the per-record path to ~1e-14).
// One wave (lane = 0..63) computes the surf half; the other waves of the block are not involved (no block barrier).
// Lane 0 forms M and the translations (LDS); V = [K_0..K_5, c] is filled branch-free from a constant table (entry =
// sign x one of M, t', t, 1); only Y = G [K_0, K_1, K_2, c] is formed, because K_3..K_5 are the unit vectors
// e_9..e_11: every output is one 13-term dot product of two rows of V, Y or G (a row of G for G K_{3+a} = G e_{9+a},
// G symmetric) — the same products and sums, in the same order, as the full quadratic forms (the unit vectors only
// contribute exact zeros).
struct SurfTable {
  signed char sgn[7][kGramW];   // -1, 0, +1
  unsigned char idx[7][kGramW]; // into Mt: M (0..8), t' (9..11), t (12..14), 1 (15)
  unsigned char ra[LM_NSUM], rb[LM_NSUM];   // output rows: 0..6 V, 7..10 Y(K_0, K_1, K_2, c), 11..23 G
};
constexpr SurfTable make_surf_table() {
  SurfTable T{};
  for (int m = 0; m < kGramW; ++m) {   // c = [M, t', 1]
    T.sgn[6][m] = 1;
    T.idx[6][m] = (unsigned char)(m < 12 ? m : 15);
  }
  for (int i = 0; i < 3; ++i) {        // K_i: sum_b eps_ibc M_be (w index 3c + e), sum_b eps_ibc t_b
    const int b1 = (i + 1) % 3, b2 = (i + 2) % 3;
    for (int m = 0; m < kGramW; ++m) {
      if (m < 9) {
        const int c = m / 3, e = m % 3;
        if (c == b2) { T.sgn[i][m] = 1; T.idx[i][m] = (unsigned char)(3 * b1 + e); }
        else if (c == b1) { T.sgn[i][m] = -1; T.idx[i][m] = (unsigned char)(3 * b2 + e); }
      } else if (m < 12) {
        const int c = m - 9;
        if (c == b2) { T.sgn[i][m] = 1; T.idx[i][m] = (unsigned char)(12 + b1); }
        else if (c == b1) { T.sgn[i][m] = -1; T.idx[i][m] = (unsigned char)(12 + b2); }
      }
    }
  }
  for (int a = 0; a < 3; ++a) { T.sgn[3 + a][9 + a] = 1; T.idx[3 + a][9 + a] = 15; }   // K_{3+a} = e_{9+a}
  // outputs: cost = c.Gc; J^T J (a <= b): a, b < 3: K_a.(G K_b); a < 3 <= b: K_a.(row 9+b-3 of G);
  // 3 <= a, b: e_{9+a-3}.(row 9+b-3 of G); J^T r: a < 3: K_a.(G c); a >= 3: e_{9+a-3}.(G c)
  auto yrow = [](int v) { return v < 3 ? 7 + v : 10; };   // Y row of K_v (v < 3) or c (v = 6)
  T.ra[0] = 6; T.rb[0] = 10;
  int h = 1;
  for (int a = 0; a < 6; ++a)
    for (int b = a; b < 6; ++b, ++h) {
      T.ra[h] = (unsigned char)a;   // V row K_a (the unit vectors for a >= 3)
      T.rb[h] = (unsigned char)(b < 3 ? yrow(b) : 11 + 9 + b - 3);
    }
  for (int a = 0; a < 6; ++a) { T.ra[22 + a] = (unsigned char)a; T.rb[22 + a] = 10; }
  T.ra[28] = 6; T.rb[28] = 6;   // (count: not a dot product)
  return T;
}

// How each of the 29 outputs follows from Y = G [K_0, K_1, K_2, c] (G symmetric, the products commute, so every
// shortcut below is the very sum the full quadratic form computes, in the same order): a 13-term dot of one of
// K_0, K_1, K_2, c with a row of Y; a single entry of Y (K_a . row r of G = (G K_a)_r, e_{9+a} . row of Y); a single
// entry of G (e_{9+a} . row of G); or the count
struct SurfOut {
  signed char kind[LM_NSUM];   // 0 dot, 1 Y entry, 2 G entry, 3 count
  signed char a[LM_NSUM];      // dot: A row (0..2 K_a, 3 c); entry: row
  signed char b[LM_NSUM];      // dot: Y row; entry: column
};
constexpr SurfOut make_surf_out() {
  const SurfTable T = make_surf_table();
  SurfOut S{};
  for (int t = 0; t < LM_NSUM; ++t) {
    const int ra = T.ra[t], rb = T.rb[t];
    if (t == 28) { S.kind[t] = 3; continue; }
    if (rb >= 7 && rb < 11) {   // with a row of Y
      if (ra < 3 || ra == 6) { S.kind[t] = 0; S.a[t] = (signed char)(ra == 6 ? 3 : ra); S.b[t] = (signed char)(rb - 7); }
      else { S.kind[t] = 1; S.a[t] = (signed char)(rb - 7); S.b[t] = (signed char)(9 + ra - 3); }
    } else {                    // with row rb - 11 of G
      if (ra < 3) { S.kind[t] = 1; S.a[t] = (signed char)ra; S.b[t] = (signed char)(rb - 11); }
      else { S.kind[t] = 2; S.a[t] = (signed char)(rb - 11); S.b[t] = (signed char)(9 + ra - 3); }
    }
  }
  return S;
}
__constant__ SurfOut c_surf_out = make_surf_out();

// lane t's output of surf_sums_wave (kind, a, b of c_surf_out), read from constant memory once per launch: inside
// the evaluation loop the three byte loads were a memory round trip on the surf half's path every evaluation
struct SurfRole {
  int kind, ra, rb;
};
__device__ __forceinline__ SurfRole surf_role(int t) {
  SurfRole r{3, 0, 0};
  if (t < LM_NSUM) r = SurfRole{c_surf_out.kind[t], c_surf_out.a[t], c_surf_out.b[t]};
  return r;
}

// Two LDS phases: every lane forms M and the translations itself (the wave-uniform values lane 0 used to publish;
// the V rows are compile-time selections of them), lanes 0..12 form row i of Y from row i of G; then lane t < 29
// forms output t.  Bit-identical to the four-phase form (same products, same summation orders).
__device__ void surf_sums_wave(const SurfRole& role, const double* x /* LDS [7] */, const double* o /* LDS [3] */,
                               const double (*G)[kGramW] /* LDS */, double n_surf, double* out /* LDS [29] */,
                               int t /* lane */) {
  __shared__ double Yl[4][kGramW];   // G K_0, G K_1, G K_2, G c
  constexpr SurfTable T = make_surf_table();
  double g[kGramW];
  if (t < kGramW) {
#pragma unroll
    for (int j = 0; j < kGramW; ++j) g[j] = G[t][j];
  }
  double Mt[16];
  {
    const double qx = x[0], qy = x[1], qz = x[2], qw = x[3];
    const double U[3][3] = {{0, -qz, qy}, {qz, 0, -qx}, {-qy, qx, 0}};
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const double u2 = U[a][0] * U[0][b] + U[a][1] * U[1][b] + U[a][2] * U[2][b];
        Mt[3 * a + b] = ((a == b) ? 1.0 : 0.0) + 2.0 * qw * U[a][b] + 2.0 * u2;
      }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      Mt[9 + k] = x[4 + k] - o[k];   // c: recentred (d absorbed n.o)
      Mt[12 + k] = x[4 + k];         // K: the Jacobian's lp = M p + t itself
    }
    Mt[15] = 1.0;
  }
  auto V = [&](int v, int m) -> double {   // (v, m compile-time after unrolling)
    const int sg = T.sgn[v][m];
    const double mv = Mt[T.idx[v][m]];
    return sg > 0 ? mv : (sg < 0 ? -mv : 0.0);
  };
  if (t < kGramW) {   // Y[v][t] = row t of G . V row (K_0, K_1, K_2, c)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      double a = 0.0;
#pragma unroll
      for (int j = 0; j < kGramW; ++j) a += g[j] * V(v == 3 ? 6 : v, j);
      Yl[v][t] = a;
    }
  }
  wave_lds_order();
  if (t < LM_NSUM) {
    const int kind = role.kind, ra = role.ra, rb = role.rb;
    double r;
    if (kind == 0) {   // the four candidate dots in independent chains, then the lane's own
      double d0 = 0.0, d1 = 0.0, d2 = 0.0, d3 = 0.0;
#pragma unroll
      for (int m = 0; m < kGramW; ++m) {
        const double y = Yl[rb][m];
        d0 += V(0, m) * y;
        d1 += V(1, m) * y;
        d2 += V(2, m) * y;
        d3 += V(6, m) * y;
      }
      r = ra == 0 ? d0 : (ra == 1 ? d1 : (ra == 2 ? d2 : d3));
    } else if (kind == 1) {
      r = Yl[ra][rb];
    } else if (kind == 2) {
      r = G[ra][rb];
    } else {
      r = n_surf;
    }
    out[t] = t == 0 ? 0.5 * r : r;
  }
  wave_lds_order();
}

__device__ __forceinline__ void gram_pair(int e, int& i, int& j) {   // upper-triangle entry e -> (i, j), i <= j
  i = 0;
  while (e >= kGramW - i) {
    e -= kGramW - i;
    ++i;
  }
  j = i + e;
}

// G (full symmetric) and its origin o into LDS from the geometry launch's gmat (gv = gram_load(gmat, threadIdx.x))
__device__ __forceinline__ void gram_unpack(double gv, double (*G)[kGramW], double* o) {
  const int t = threadIdx.x;
  if (t < kGram) {
    int i, j;
    gram_pair(t, i, j);
    G[i][j] = gv;
    G[j][i] = gv;
  } else if (t < kGramWords) {
    o[t - kGram] = gv;
  }
  __syncthreads();
}

// ===================================================================================== LM control (Ceres 1.13)
// The control step is serial fp64 code, so its cost is its dependent instruction count.  It runs on one wave whose 64
// lanes all hold the same LM state in REGISTERS for the whole solve (loaded once, stored once); the two SE(3)
// exponentials of a step — the candidate x [+] delta and the gradient projection x [+] -g of the gradient-norm test —
// run side by side in lanes 0 and 1 of the same instruction stream; the 6x6 LDL^T divides by each pivot once.
// Loops are fully unrolled with constant indices so nothing leaves registers.

// sin and cos of |x| <= pi / 4 by fdlibm's kernel polynomials (__kernel_sin / __kernel_cos, < 1 ulp): the two
// 6-term chains interleave, one dependent chain instead of the library sincos's range reduction and branches (the
// control step is one wave's serial fp64 instruction stream).  Larger |x| (a huge step, or the gradient projection of
// the iteration-zero test) takes the library's sincos.
__device__ __forceinline__ void sincos_small(double x, double* s, double* c) {
#ifdef FLOAM_LM_LIBSINCOS   // (A/B builds only: the library's sincos for every angle)
  sincos(x, s, c);
  return;
#endif
  if (!(fabs(x) <= 0.78125)) {
    sincos(x, s, c);
    return;
  }
  const double z = x * x, v = z * x;
  const double rs = 8.33333333332248946124e-03 +
                    z * (-1.98412698298579493134e-04 +
                         z * (2.75573137070700676789e-06 + z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)));
  const double rc = z * (4.16666666666666019037e-02 +
                         z * (-1.38888888888741095749e-03 +
                              z * (2.48015872894767294178e-05 +
                                   z * (-2.75573143513906633035e-07 +
                                        z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
  *s = x + v * (-1.66666666666666324348e-01 + z * rs);
  if (fabs(x) < 0.3) {
    *c = 1.0 - (0.5 * z - z * rc);
  } else {   // fdlibm's split of 1 - z / 2 for 0.3 <= |x| <= 0.78125: qx = |x| / 4 with its low word cleared
    const long long hb = __double_as_longlong(fabs(x)) - (0x00200000ll << 32);
    const double qx = __longlong_as_double(hb & (long long)0xFFFFFFFF00000000ull);
    const double hz = 0.5 * z - qx, a = 1.0 - qx;
    *c = a - (hz - z * rc);
  }
}

// PoseSE3Parameterization::Plus + getTransformFromSe3 (src/lidarOptimization.cpp:77-140).  theta^3 is formed by
// multiplication where the reference calls pow(theta, 3) (<= 1 ulp apart).
__device__ __forceinline__ void se3_plus(const double (&x)[7], const double (&d)[6], double (&out)[7]) {
  const double wx = d[0], wy = d[1], wz = d[2];
  const double theta = sqrt(wx * wx + wy * wy + wz * wz);
  const double half = 0.5 * theta;
  double sh, ch;
  sincos_small(half, &sh, &ch);
  const double real_factor = ch;
  double imag;
  const bool small = theta < 1e-10;
  const double rt = recip(theta);   // beside the sincos, off the dependent chain
  if (small) {
    const double t2 = theta * theta, t4 = t2 * t2;
    imag = 0.5 - 0.0208333 * t2 + 0.000260417 * t4;
  } else {
    imag = sh * rt;
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
    // sin(theta), 1 - cos(theta) from the half angle (one sincos per exponential instead of two: the control step is
    // a single wave's fp64 instruction stream, 4 cycles an instruction)
    const double st = 2.0 * sh * ch, omc = 2.0 * sh * sh;
    const double c1 = omc * (rt * rt);
    const double c2 = (theta - st) * (rt * rt * rt);
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
  rot<double>(dq, x[4], x[5], x[6], tx, ty, tz);
  out[4] = tx + dtx;
  out[5] = ty + dty;
  out[6] = tz + dtz;
}

__host__ __device__ constexpr int hidx(int a, int b) {   // upper-triangle row-major index, a <= b
  return a * 6 - a * (a - 1) / 2 + (b - a);
}

// LevenbergMarquardtStrategy::ComputeStep in normal-equation form + TrustRegionMinimizer::ComputeTrustRegionStep's
// model cost change, on the UNSCALED system.  Ceres solves the Jacobi-scaled system (S H S + D / radius) y = S g with
// S = diag(scale) and D = clamp(diag(S H S), 1e-6, 1e32), and steps by delta = -S y.  With z = S y that is
// (H + E / radius) z = g, delta = -z, where E = D S^-2 = clamp(diag(H), 1e-6 S^-2, 1e32 S^-2) (bounds fixed with S
// at iteration zero: LMState::dlo, dhi), and the model cost change (y.Sg + y.D y / radius) / 2 = (z.g + z.E z /
// radius) / 2 — the same step in exact arithmetic without the 54 products of the scaling; the rounding differs at
// ~cond * eps, as the oracle's Householder QR of [J; sqrt(D / radius)] (Ceres' DENSE_QR) differs from both.
// LDL^T by rows (W = L D of the current row only, one reciprocal per pivot).  Returns false for an invalid step.
__device__ __forceinline__ bool lm_step(const double (&H)[21], const double (&g)[6], const double (&E)[6],
                                        double inv_r, double (&z)[6], double& mcc) {
  double L[15], rD[6];   // L strictly lower, packed by rows: l(i, j) = i (i - 1) / 2 + j
  bool pd = true;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    double W[6];
#pragma unroll
    for (int j = 0; j < i; ++j) {
      double w = H[hidx(j, i)];
#pragma unroll
      for (int k = 0; k < j; ++k) w -= W[k] * L[j * (j - 1) / 2 + k];
      W[j] = w;                            // L[i][j] D[j]
      L[i * (i - 1) / 2 + j] = w * rD[j];
    }
    double d = fma(E[i], inv_r, H[hidx(i, i)]);
#pragma unroll
    for (int k = 0; k < i; ++k) d -= W[k] * L[i * (i - 1) / 2 + k];
    pd = pd && (d > 0.0);
    rD[i] = recip(d);
  }
  if (!pd) return false;
  double y[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {   // L u = g
    double v = g[i];
#pragma unroll
    for (int k = 0; k < i; ++k) v -= L[i * (i - 1) / 2 + k] * y[k];
    y[i] = v;
  }
#pragma unroll
  for (int i = 5; i >= 0; --i) {   // L^T z = D^-1 u
    double v = y[i] * rD[i];
#pragma unroll
    for (int k = 5; k > i; --k) v -= L[k * (k - 1) / 2 + i] * z[k];
    z[i] = v;
  }
  bool finite = true;
#pragma unroll
  for (int k = 0; k < 6; ++k) finite = finite && isfinite(z[k]);
  if (!finite) return false;
  double zg = 0.0, zEz = 0.0;
#pragma unroll
  for (int a = 0; a < 6; ++a) {
    zg += z[a] * g[a];
    zEz += (z[a] * z[a]) * E[a];
  }
  mcc = 0.5 * (zg + zEz * inv_r);
  return mcc > 0.0;
}

// -DFLOAM_CTRL_STAMPS (diagnostic build): block 0's control-step segments, s_memrealtime (100 MHz), accumulated by
// lane 0: [0] steps, [1] bookkeeping before the step, [2] solve_step, [3] se3_plus, [4] the candidate hand-over
// broadcast, [5] whole step; printed by lm_ctrl_stamps_print
#ifdef FLOAM_CTRL_STAMPS
__device__ unsigned long long g_ctrl_stamps[8];
#define CTRL_T(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime()
#define CTRL_ADD(k, d)                                                          \
  do {                                                                          \
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_ctrl_stamps[k], d);   \
  } while (0)
#else
#define CTRL_T(v)
#define CTRL_ADD(k, d) \
  do {                 \
  } while (0)
#endif

// the resident solve's segment stamps (FLOAM_DEBUG_STAMPS): read only by the diagnostic build — in the product
// library the clock reads are gone from the evaluation loop altogether (each one is a scalar-memory message whose
// return the next LDS wait also waits for)
#ifdef FLOAM_DIAG
#define LM_NOW() __builtin_amdgcn_s_memrealtime()
#else
#define LM_NOW() 0ull
#endif

// value of lane src (a compile-time / wave-uniform lane) to every lane: two v_readlane (no LDS round trip)
__device__ __forceinline__ double bcast(double v, int src) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, src);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), src);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// The gradient-norm test (at iteration zero and after a successful step) only asks whether
// max_i |x_i - (x [+] -g)_i| <= 1e-10; lane 1 forms the projection x [+] -g beside lane 0's candidate, in the same
// instruction stream.  If the test ends the solve the step is discarded, as in the sequential order (test first, then
// step).  A rotation of angle th moves the unit quaternion by |dq - 1| = 2 |sin(th / 4)| in the 2-norm (the product
// with q preserves it), so some component by at least |sin(th / 4)|: when th / 4 is more than 1e-6 from every multiple
// of pi (a two-constant reduction, exact far beyond any gradient) the test fails without the projection.  Large
// gradients are the rule before convergence, and their angle would send lane 1 through the library sincos's range
// reduction while lane 0 waits (one wave).
__device__ __forceinline__ bool gradient_step_far(const double (&g)[6]) {
  const double th = sqrt(g[0] * g[0] + g[1] * g[1] + g[2] * g[2]);
  if (!(th > 1.5625 && th < 1e15)) return false;   // (small angles take sincos_small anyway)
  const double u = 0.25 * th;
  const double k = rint(u * 0.31830988618379067154);
  double r = fma(-k, 3.141592653589793116, u);
  r = fma(-k, 1.2246467991473532072e-16, r);
  return fabs(r) > 1e-6 && fabs(r) < 3.1415916;
}

// H[21] followed by g[6] (H0 by g0), the layout of sums[1..27]: the 27 words, one a lane
static_assert(offsetof(LMState, g) == offsetof(LMState, H) + 21 * sizeof(double) &&
              offsetof(LMState, g0) == offsetof(LMState, H0) + 21 * sizeof(double), "H, g contiguous");
__device__ __forceinline__ double* state_words(LMState& S, size_t off) {
  return reinterpret_cast<double*>(reinterpret_cast<char*>(&S) + off);
}

__device__ __forceinline__ double norm7(const double (&a)[7]) {
  double v = 0.0;
#pragma unroll
  for (int i = 0; i < 7; ++i) v += a[i] * a[i];
  return sqrt(v);
}

// the values are taken as written here (an empty asm that "changes" them): their loads cannot sink below this point
template <int N>
__device__ __forceinline__ void pin(double (&v)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k) asm volatile("" : "+v"(v[k]));
}

// The tests of a candidate that read nothing of its evaluation — the gradient-norm test due with the step
// (max_i |x_i - (x [+] -g)_i| <= 1e-10, the projection in S.proj) and ParameterToleranceReached (|x - cand| <= 1e-8
// (|x| + 1e-8)) — and |cand|, run by one wave while the candidate is being evaluated instead of between the step and
// the evaluation (resident solve: wave 0, between its publish and its polls; the per-evaluation launches: at the start
// of the next control step).  When one ends the solve, the candidate's evaluation is discarded, as if it had not been
// made (the sequential order skips it; nothing of it enters the state).  Same operands, same order, same bits as the
// tests inline.
__device__ __forceinline__ void deferred_tests(LMState& S, int lane) {
  const int tp = S.tpend;   // (wave-uniform)
  if (!tp) return;
  double x[7], c[7], p[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    x[k] = S.x[k];
    c[k] = S.cand[k];
    p[k] = S.proj[k];
  }
  double gm = S.gmax;
  const double x_norm = S.x_norm;
  int verdict = 0;
  if (tp & 2) {
    double ml = 0.0;
#pragma unroll
    for (int i = 0; i < 7; ++i) ml = fmax(ml, fabs(x[i] - p[i]));
    gm = ml;
    if (gm <= 1e-10) verdict = 2;
  }
  if (!verdict && (tp & 1)) {
    double sn2 = 0.0;
#pragma unroll
    for (int i = 0; i < 7; ++i) sn2 += (x[i] - c[i]) * (x[i] - c[i]);
    const double ptol = 1e-8 * (x_norm + 1e-8);
    if (sn2 <= ptol * ptol) verdict = 1;
  }
  const double cn = norm7(c);
  if (lane == 0) {
    S.gmax = gm;
    S.cand_norm = cn;
    S.tdone = verdict;
    S.tpend = 0;
  }
  wave_lds_order();
}

// One Ceres control step after an evaluation (sums: cost, J^T J, J^T r, count at x in phase 0, else at cand), run by
// the 64 lanes of one wave on the LM state in LDS.  Every lane reads the same words (LDS broadcast) and computes the
// same values — but lane 1, which forms the gradient projection of the gradient-norm test beside lane 0's candidate —
// so every branch is wave-uniform; vector copies (x_in, H0 / g0, H / g on a successful step, the clamp bounds) go one
// element a lane, and lane 0 writes the scalars back once at the end.  Nothing of the state stays in registers
// between steps: the evaluation's registers and the step's do not compete (the register-resident form spent a third
// of its instructions moving the state through the accumulation registers).  The next point is S.cand (every block's
// evaluation reads it there); S.done ends the solve.  The step itself is NextStep: ComputeTrustRegionStep (lm_step)
// with HandleInvalidStep's retries, the gradient-norm test folded in.
// tests: the candidate's deferred tests are still to run (the per-evaluation launches; the resident solve ran them
// during the evaluation).
__device__ __forceinline__ void control_step(LMState& S, const double* __restrict__ sums, int lane, bool tests) {
  CTRL_T(t0);
  if (tests) deferred_tests(S, lane);
  // every word the decisions read, loaded together and pinned where they are loaded: one LDS round trip (the compiler
  // otherwise sinks each load into the branch that uses it, a round trip per branch)
  double x[7], c[7], sm[28], lo[6], hi[6];   // sm: cost, H[21], g[6]; lo, hi: the diagonal's clamp bounds
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    x[k] = S.x[k];
    c[k] = S.cand[k];
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    lo[k] = S.dlo[k];
    hi[k] = S.dhi[k];
  }
#pragma unroll
  for (int k = 0; k < 28; ++k) sm[k] = sums[k];
  double x_cost = S.x_cost, radius = S.radius, dfac = S.dfac, mcc = S.mcc, x_norm = S.x_norm, gmax = S.gmax;
  const double cand_norm = S.cand_norm;
  int iteration = S.iteration, reuse = S.reuse, invalid = S.invalid, successful = S.successful;
  int phase = S.phase;
  const int tdone = S.tdone;
  pin(x);
  pin(c);
  pin(sm);
  pin(lo);
  pin(hi);
  const double cost = sm[0];
  int done = 0;
  bool fresh = false;        // H, g (and E) from this evaluation's sums
  bool check_gmax = false;   // the gradient-norm test is due: at iteration zero and after a successful step
  bool moved = false;        // x <- cand
  if (phase == 0) {   // IterationZero
    if (lane < 7) S.x_in[lane] = S.x[lane];                // the trace of iteration zero
    if (lane < 27) state_words(S, offsetof(LMState, H0))[lane] = sums[1 + lane];   // H0, g0
    const int n_res = (int)sums[28];
    if (lane == 0) {
      S.n_res = n_res;
      S.initial_cost = cost;
    }
    x_cost = cost;
    if (n_res == 0 || !isfinite(cost)) {   // no residual blocks (parameters untouched), or a non-finite cost
      done = 1;
    } else {
      if (lane < 6) {   // Jacobi scaling 1 / (1 + sqrt(H_kk)), as the bounds of the unscaled diagonal (lm_step)
        const double r = 1.0 + sqrt(sums[1 + hidx(lane, lane)]);
        S.dlo[lane] = 1e-6 * (r * r);
        S.dhi[lane] = 1e32 * (r * r);
      }
      wave_lds_order();
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        lo[k] = S.dlo[k];
        hi[k] = S.dhi[k];
      }
      x_norm = norm7(x);
      radius = 1e4;
      dfac = 2.0;
      reuse = 0;
      invalid = 0;
      iteration = 0;
      phase = 1;
      fresh = true;
      check_gmax = true;
    }
  } else if (tdone) {   // a deferred test of the candidate ended the solve: its evaluation is discarded
    done = 1;
    if (tdone == 2) --iteration;   // (the gradient-norm test comes before the step: the step is not counted)
  } else {
    const double cand_cost = isfinite(cost) ? cost : DBL_MAX;
    if (fabs(x_cost - cand_cost) <= 1e-6 * x_cost) {   // FunctionToleranceReached
      done = 1;
    } else {
      // rho = decrease / mcc > 1e-3 decided without the reciprocal (mcc > 0); rho itself only for the radius update
      const double dec = x_cost - cand_cost;
      moved = dec > 1e-3 * mcc;   // success
      const double rho = dec * recip(mcc);   // (within an ulp of the division)
      const double t = 2.0 * rho - 1.0;
      const double up = fmin(1e16, radius * recip(fmax(1.0 / 3.0, 1.0 - t * t * t)));
      const double down = radius * recip(dfac);   // (dfac a power of two: exact)
#pragma unroll
      for (int i = 0; i < 7; ++i) x[i] = moved ? c[i] : x[i];
      x_norm = moved ? cand_norm : x_norm;   // (norm7 of the candidate, formed with it)
      x_cost = moved ? cand_cost : x_cost;
      radius = moved ? up : down;
      dfac = moved ? 2.0 : 2.0 * dfac;
      reuse = moved ? 0 : 1;
      successful += moved ? 1 : 0;
      fresh = moved;
      check_gmax = moved;
      if (iteration >= 4 || radius < 1e-32) done = 1;
    }
  }
  if (fresh && !done && lane < 27) state_words(S, offsetof(LMState, H))[lane] = sums[1 + lane];   // H, g
  CTRL_T(t1);
  CTRL_ADD(1, t1 - t0);
  bool have_cand = false;
  int tp = 0;   // the candidate's deferred tests (LMState::tpend)
  double out[7];
  if (!done) {
    double H[21], g[6], E[6];
    if (fresh) {
#pragma unroll
      for (int k = 0; k < 21; ++k) H[k] = sm[1 + k];
#pragma unroll
      for (int k = 0; k < 6; ++k) g[k] = sm[22 + k];
    } else {   // (a rejected step: J^T J and J^T r of x, kept in the state)
      const double* Hp = state_words(S, offsetof(LMState, H));   // H, then g
#pragma unroll
      for (int k = 0; k < 21; ++k) H[k] = Hp[k];
#pragma unroll
      for (int k = 0; k < 6; ++k) g[k] = Hp[21 + k];
    }
    if (!reuse) {
#pragma unroll
      for (int k = 0; k < 6; ++k) E[k] = fmin(fmax(H[hidx(k, k)], lo[k]), hi[k]);
    } else {
#pragma unroll
      for (int k = 0; k < 6; ++k) E[k] = S.diag[k];
    }
    const bool new_diag = !reuse;
    reuse = 1;
    for (;;) {
      CTRL_T(ta);
      double z[6], m = 0.0;
      const bool valid = lm_step(H, g, E, recip(radius), z, m);
      CTRL_T(tb);
      // lane 1: the gradient projection x [+] -g, when the test is due and cannot be decided from the angle alone
      const bool far = check_gmax && gradient_step_far(g);
      double d[6];
#pragma unroll
      for (int k = 0; k < 6; ++k)   // (lane 1 without a projection to compute follows lane 0: no divergent branch)
        d[k] = (lane == 1 && check_gmax && !far) ? -g[k] : (valid ? -z[k] : 0.0);
      se3_plus(x, d, out);
      CTRL_T(tc);
      CTRL_ADD(2, tb - ta);
      CTRL_ADD(3, tc - tb);
      if (valid) {   // the candidate goes to its evaluation now, its tests with it (deferred_tests)
        if (check_gmax) {
          if (far) gmax = HUGE_VAL;   // (the test fails: only the comparison with the tolerance is used)
          else tp |= 2;               // lane 1's projection, written with the candidate
          check_gmax = false;
        }
        tp |= 1;
        iteration++;
        mcc = m;
        invalid = 0;
        have_cand = true;
        CTRL_T(td);
        CTRL_ADD(4, td - tc);
        break;   // candidate pending evaluation
      }
      // an invalid step: the gradient-norm test inline, then HandleInvalidStep.  (Wave-uniform) lane 1 computed the
      // projection: it measures its own distance to x, which is read from it (one read-lane pair)
      if (check_gmax) {
        double gm = HUGE_VAL;   // (far: the test fails; only the comparison with the tolerance is used)
        if (!far) {
          double ml = 0.0;
#pragma unroll
          for (int i = 0; i < 7; ++i) ml = fmax(ml, fabs(x[i] - out[i]));
          gm = bcast(ml, 1);
        }
        gmax = gm;
        check_gmax = false;
        if (gmax <= 1e-10) {   // (phase 0: before any step; phase 1: success && gmax)
          done = 1;
          break;
        }
      }
      iteration++;
      // HandleInvalidStep -> StepIsInvalid -> StepRejected(0)
      if (++invalid >= 5) {
        done = 1;
        break;
      }
      radius *= recip(dfac);   // (dfac a power of two: exact)
      dfac *= 2.0;
      if (iteration >= 4 || radius < 1e-32) {
        done = 1;
        break;
      }
    }
    if (new_diag && lane == 0) {
#pragma unroll
      for (int k = 0; k < 6; ++k) S.diag[k] = E[k];
    }
  }
  if (lane == 1 && (tp & 2)) {   // the projection x [+] -g (lane 1's se3_plus)
#pragma unroll
    for (int k = 0; k < 7; ++k) S.proj[k] = out[k];
  }
  if (lane == 0) {
    if (moved) {
#pragma unroll
      for (int k = 0; k < 7; ++k) S.x[k] = x[k];
    }
    if (have_cand) {
#pragma unroll
      for (int k = 0; k < 7; ++k) S.cand[k] = out[k];
    }
    S.tpend = tp;
    S.x_cost = x_cost; S.radius = radius; S.dfac = dfac; S.mcc = mcc; S.x_norm = x_norm; S.gmax = gmax;
    S.iteration = iteration; S.reuse = reuse; S.invalid = invalid; S.successful = successful;
    S.phase = phase;
    S.done = done;
  }
  wave_lds_order();
  CTRL_T(t2);
  CTRL_ADD(5, t2 - t0);
  CTRL_ADD(0, 1ull);
}

__device__ __forceinline__ void stage_state(const LMState* __restrict__ st, LMState& sst) {
  const unsigned* src = reinterpret_cast<const unsigned*>(st);
  unsigned* dst = reinterpret_cast<unsigned*>(&sst);
  for (int w = threadIdx.x; w < kStateWords; w += blockDim.x) dst[w] = src[w];
}
// (every word but xfail, which only a block reporting a timed-out hand-off writes)
__device__ __forceinline__ void publish_state(const LMState& sst, LMState* __restrict__ st) {
  const unsigned* src = reinterpret_cast<const unsigned*>(&sst);
  unsigned* dst = reinterpret_cast<unsigned*>(st);
  for (int w = threadIdx.x; w < kPublishWords; w += blockDim.x) dst[w] = src[w];
}

__device__ __forceinline__ unsigned long long granule(unsigned tag, unsigned data) {
  return ((unsigned long long)tag << 32) | data;
}
__device__ __forceinline__ void put_granule(unsigned long long* p, unsigned long long g) {
  __hip_atomic_store(p, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The all-gather and the block reduction in one pass, straight from the granules: thread t < 232 (component
// c = t >> 3, strip p = t & 7) polls the two halves of component c from the blocks of its strip (consecutive blocks,
// in block order: reduce_blocks' partition) and adds them in block order; the 8 strips by strip8_total — the bits of
// reduce_blocks over the gathered table, without the table (no LDS write and read, no barrier between them).
// Every poll loop is bounded (kSpin); bad = a granule never arrived.  Called by every thread; returns, to the threads with
// (t & 7) == 0 and t < 232, the sum of component t >> 3.
constexpr int kGatherChunk = 4;   // blocks polled together by a thread (8 granule loads in flight)
__device__ __forceinline__ double gather_blocks(const unsigned long long* __restrict__ slot, int nact, unsigned tag,
                                                bool& bad) {
  const int t = threadIdx.x;
  const int c = t >> 3, p = t & 7;
  const int per = (nact + 7) / 8;
  const int b0 = min(nact, p * per), nb = t < LM_NSUM * 8 ? min(nact, b0 + per) - b0 : 0;
  double v = 0.0;
  bad = false;
  for (int k0 = 0; k0 < nb; k0 += kGatherChunk) {   // chunks in block order
    const unsigned long long* g = slot + (size_t)(b0 + k0) * 2 * LM_NSUM + 2 * c;
    const int nk = min(kGatherChunk, nb - k0);
    unsigned lo[kGatherChunk], hi[kGatherChunk];
    unsigned pend = 0;   // bit 2k: block k's low half, 2k + 1 its high half
#pragma unroll
    for (int k = 0; k < kGatherChunk; ++k) {
      lo[k] = 0u;
      hi[k] = 0u;
      if (k < nk) pend |= 3u << (2 * k);
    }
    for (long long it = 0; it < kSpin && pend; ++it) {
      unsigned long long w[2 * kGatherChunk];
#pragma unroll
      for (int q = 0; q < 2 * kGatherChunk; ++q)   // all loads of the round issued before any is examined
        w[q] = (pend >> q) & 1u ? __hip_atomic_load(&g[(q >> 1) * 2 * LM_NSUM + (q & 1)], __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)
                                : 0ull;
#pragma unroll
      for (int q = 0; q < 2 * kGatherChunk; ++q)
        if (((pend >> q) & 1u) && (unsigned)(w[q] >> 32) == tag) {
          if (q & 1) hi[q >> 1] = (unsigned)w[q]; else lo[q >> 1] = (unsigned)w[q];
          pend &= ~(1u << q);
        }
      if (pend) __builtin_amdgcn_s_sleep(1);
    }
    if (pend) {
      bad = true;
      break;
    }
#pragma unroll
    for (int k = 0; k < kGatherChunk; ++k)
      if (k < nk) v += __longlong_as_double((long long)(((unsigned long long)hi[k] << 32) | lo[k]));
  }
  return strip8_total(v);
}

// evaluation blocks that hold records: one record slot per record thread while they fit, at most nblk (a function of
// the device count only, so the partition and the reduction order never depend on the host's upper bounds)
template <int NR>
__device__ __forceinline__ int active_blocks(int total, int nblk) {
  return max(1, min(nblk, (total + NR - 1) / NR));
}

// record threads of a solve block: GRAM — waves 0..2 hold edge records and wave 3 forms the surf half from G;
// otherwise every thread holds records
template <bool GRAM>
constexpr int rec_threads() { return GRAM ? kTB - 64 : kTB; }

struct LMArgs {
  LMState* st;
  const double* erec;
  const uint8_t* evalid;
  int ecap;
  const int* d_ne;
  int ne_ub;
  const double* srec;
  const uint8_t* svalid;
  int scap;
  const int* d_ns;
  int ns_ub;
  const double* gmat;              // GRAM: G + origin (kGramWords)
  unsigned long long* part;        // [2][kRecEvalBlocks][2 * LM_NSUM] partial granules (by evaluation parity)
  double* partials;                // sharded: [LM_NSUM][nblk]
  double* sums;                    // sharded: 29 sums (all-reduced in place between launches)
  unsigned* ticket;                // sharded: arrival ticket
  unsigned long long* dbg;         // FLOAM_DEBUG_STAMPS: block 0's segment times (diagnostic, normally null)
  int fail_test;                   // LMBuffers::fail_test: report the first hand-off as timed out (tests)
  // peer sharding (world > 1): this rank's exchange granules [2][2 * LM_NSUM] and every rank's, peer-mapped, rank order
  int world;
  unsigned long long* xme;
  const unsigned long long* xpeer[kMaxShardRanks];
  unsigned peer_delay;             // (diagnostic build, tests) 100-MHz ticks the non-zero blocks wait before a peer poll
};

// Peer sharding: after a block has its rank's 29 sums (block partials + the surf half), block 0 publishes them as
// tagged granules in this rank's exchange buffer and every block gathers all ranks' granules (system scope: the buffers
// of the other ranks are on other GPUs, read through xGMI) and sums them in rank order — every block of every rank the
// same bits, so every rank takes the same LM decisions.
// Slot and tag come from the exchange counter xs (LMState::xseq): the evaluations exchanged since
// floam_odom_set_shard_peers reset it on every rank, continued across solves — the same sequence on every rank, since
// every rank takes the same decisions.  Slot xs & 1, tag 2 xs + 1 (odd: the zeroed buffer never matches).  Reuse: a
// rank overwrites the slot of exchange xs only at xs + 2, after it has read every rank's granules of xs + 1, and a rank
// publishes xs + 1 only after each of its blocks has finished reading xs — inside a solve because the block all-gather
// of the evaluation behind xs + 1 waits for every block of the rank, across solves because the next solve is a later
// launch on the rank's stream.  (A per-solve counter broke the second case: after a solve that ended on an even
// evaluation the next solve's first exchange reused slot 0 while a late block of another rank could still be polling
// it for the old tag.)  The wait is bounded in time (~20 s: ranks in other processes may be far apart at the first
// solve), not in polls.
__device__ __forceinline__ bool peer_exchange(const LMArgs& a, unsigned xs, double* s_sums, unsigned* s_x) {
  constexpr int kG = 2 * LM_NSUM;   // granules per rank and slot
  static_assert(kMaxShardRanks * kG <= 2 * kTB, "every rank's granules: at most two per thread");
  static_assert(2 * kG <= kShardXchgWords, "two slots in the exchange buffer");
  const int tid = (int)threadIdx.x;
  const int slot = (int)(xs & 1u) * kG;
  const unsigned tag = 2u * xs + 1u;
  if (blockIdx.x == 0 && tid < kG) {
    const int c = tid >> 1, h = tid & 1;
    const unsigned long long b = (unsigned long long)__double_as_longlong(s_sums[c]);
    __hip_atomic_store(&a.xme[slot + tid], granule(tag, h ? (unsigned)(b >> 32) : (unsigned)b), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
#ifdef FLOAM_DIAG
  if (a.peer_delay && blockIdx.x != 0) {   // (tests: a late block, the case the slot reuse argument must cover)
    const unsigned long long d0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - d0 < a.peer_delay) __builtin_amdgcn_s_sleep(8);
  }
#endif
  // granules j = tid and tid + kTB of the world x kG (rank r's granule j - r kG)
  const int n = a.world * kG;
  const unsigned long long* src[2] = {nullptr, nullptr};
  unsigned pend = 0;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = tid + u * kTB;
    if (j < n) {
      const int r = j / kG;
      const unsigned long long* base = a.xpeer[0];
#pragma unroll
      for (int q = 1; q < kMaxShardRanks; ++q)   // (selected, not indexed: the argument array stays in registers)
        if (q == r) base = a.xpeer[q];
      src[u] = base + slot + (j - r * kG);
      pend |= 1u << u;
    }
  }
  bool ok = true;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (pend) {
    unsigned long long v[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)   // both loads in flight before either is examined
      v[u] = (pend >> u) & 1u ? __hip_atomic_load(src[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull;
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (((pend >> u) & 1u) && (unsigned)(v[u] >> 32) == tag) {
        s_x[tid + u * kTB] = (unsigned)v[u];
        pend &= ~(1u << u);
      }
    if (!pend) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull) {   // 100 MHz: 20 s
      ok = false;
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  if (__syncthreads_or(!ok)) return false;
  if (tid < LM_NSUM) {
    double v = 0.0;
    for (int r = 0; r < a.world; ++r) {
      const int g = r * kG + 2 * tid;
      v += __longlong_as_double((long long)(((unsigned long long)s_x[g + 1] << 32) | s_x[g]));
    }
    s_sums[tid] = v;
  }
  __syncthreads();
  return true;
}

// the block's first record (the one kept in registers across the evaluations) of record thread i0
template <typename R>
__device__ __forceinline__ void first_record(const LMArgs& a, int i0, int ne, int total, R (&f0)[9], bool& has0,
                                             bool& edge0) {
#pragma unroll
  for (int k = 0; k < 9; ++k) f0[k] = R(0);
  has0 = false;
  edge0 = true;
  if (i0 < ne) {
    has0 = a.evalid[i0] & 1;
    if (has0) load_rec<R, EDGE_FIELDS>(a.erec, a.ecap, i0, f0);
  } else if (i0 < total) {
    edge0 = false;
    has0 = a.svalid[i0 - ne] & 1;
    if (has0) load_rec<R, SURF_FIELDS>(a.srec, a.scap, i0 - ne, f0);
  }
}

// ===================================================================================== the resident solve
// Every active block runs the whole solve: it evaluates its records at the current point, publishes its 29 partial
// sums as tagged granules, gathers every active block's granules (all-gather: one hand-off per evaluation, no
// control -> evaluation release hop), reduces them in a fixed block order and runs the Ceres control step on wave 0
// — every block computes the same bits, so every block knows the next point and whether the solve ended.  Block 0
// writes the state back.  Granule slots alternate with the evaluation's parity: a block overwrites its slot of
// evaluation k only in evaluation k + 2, after it has seen every block's granule of evaluation k + 1, which each block
// publishes only after it has seen every granule of evaluation k.
template <bool GRAM, bool HUBER, typename R>
__global__ __launch_bounds__(kTB) void lm_solve(LMArgs a) {
  constexpr int NR = rec_threads<GRAM>();
  __shared__ double s_buf[LM_NSUM * red_stride<NR>()];   // thread sums
  __shared__ double s_sums[LM_NSUM];
  __shared__ double s_ssum[LM_NSUM];
  __shared__ LMState sst;
  __shared__ double G[kGramW][kGramW];
  __shared__ double o[3];
  const int nblk = (int)gridDim.x, blk = (int)blockIdx.x, tid = (int)threadIdx.x, lane = tid & 63;
  const unsigned long long t_start = LM_NOW();
  // the counts, the LM state, G and (GRAM) this thread's edge record — speculatively, for i0 < ne_ub, which is
  // inside the record arrays — all issued before any is waited on: one memory round trip before the first evaluation
  static_assert(kStateWords <= kTB, "one state word per thread");
  const int i0 = blk * NR + tid;
  const int ne_dev = *a.d_ne;
  const int ns_dev = GRAM ? 0 : *a.d_ns;
  const unsigned sw = tid < kStateWords ? reinterpret_cast<const unsigned*>(a.st)[tid] : 0u;
  const double gv = GRAM ? gram_load(a.gmat, tid) : 0.0;
  const SurfRole srole = GRAM && tid >= NR ? surf_role(lane) : SurfRole{3, 0, 0};   // (wave 3: the surf half)
  R f0[9];
  bool has0 = false, edge0 = true;
  uint8_t v0 = 0;
  if (GRAM) {
#pragma unroll
    for (int k = 0; k < 9; ++k) f0[k] = R(0);
    if (tid < NR && i0 < a.ne_ub) {
      v0 = a.evalid[i0];
      load_rec<R, EDGE_FIELDS>(a.erec, a.ecap, i0, f0);
    }
  }
  const int ne = min(ne_dev, a.ne_ub);
  const int total = ne + (GRAM ? 0 : min(ns_dev, a.ns_ub));
  const int nact = active_blocks<NR>(total, nblk);
  if (blk >= nact) return;   // no records: nobody waits for this block
  if (tid < kStateWords) reinterpret_cast<unsigned*>(&sst)[tid] = sw;
  const int stride = nact * NR;
  if (GRAM) has0 = tid < NR && i0 < ne && (v0 & 1);
  else if (tid < NR) first_record<R>(a, i0, ne, total, f0, has0, edge0);
  __syncthreads();
  if (sst.done) return;   // (never after lm_reset)
  if (GRAM) gram_unpack(gv, G, o);
  const unsigned ep = sst.epoch;
  const unsigned xs0 = sst.xseq;   // peer sharding: this solve's first exchange
  // every evaluation is at sst.cand: iteration zero's at x (set by the kNN launch; kernel boundary)
  if (tid < 7 && sst.phase == 0) sst.cand[tid] = sst.x[tid];
  unsigned long long tm[4] = {0, 0, 0, 0};
  __shared__ unsigned s_xch[kMaxShardRanks * 2 * LM_NSUM];   // peer sharding: every rank's sums (u32 halves)
  const bool peers = a.world > 1;
  unsigned nx = 0;   // evaluations exchanged with the other ranks in this solve
  const unsigned long long t_loop = LM_NOW();
  int failed_at = -1;   // evaluation whose granules never arrived (never expected)
  for (int it = 0; it < 5; ++it) {
    const unsigned long long t0 = LM_NOW();
    __syncthreads();   // the point and done flag of this evaluation
    if (sst.done) break;
    const unsigned long long tw = LM_NOW();   // (this wave's start of the evaluation)
    unsigned long long t1 = t0, t2 = t0;
    unsigned tag = ep + (unsigned)it;
    {
      double acc[LM_NSUM];
      if (tid < NR) {
        R x[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) x[k] = (R)sst.cand[k];
        eval_records<HUBER, R>(x, has0, edge0, f0, i0 + stride, stride, ne, total, a.erec, a.evalid, a.ecap, a.srec,
                               a.svalid, a.scap, acc);
      } else {
#pragma unroll
        for (int k = 0; k < LM_NSUM; ++k) acc[k] = 0.0;
        if (GRAM) surf_sums_wave(srole, sst.cand, o, G, (double)sst.corr_surf, s_ssum, lane);   // beside the edges
      }
#ifdef FLOAM_DIAG
      // block 0's wave 0 (edge records) and wave 3 (GRAM: the surf half) from the evaluation's start to their sums
      if (a.dbg && blk == 0 && (tid == 0 || tid == 3 * 64)) atomicAdd(&a.dbg[tid ? 8 : 7], LM_NOW() - tw);
#endif
      const double v = block_sums<NR>(acc, s_buf);
      unsigned long long* slot = a.part + (size_t)(it & 1) * kRecEvalBlocks * 2 * LM_NSUM;
      if (tid < LM_NSUM * kStrips && (tid & 7) < 2) {   // 58 granules: component c in 32-bit halves (lanes 8c, 8c + 1)
        const int c = tid >> 3, h = tid & 1;
        const unsigned long long b = (unsigned long long)__double_as_longlong(v);
        put_granule(&slot[blk * 2 * LM_NSUM + 2 * c + h], granule(tag, h ? (unsigned)(b >> 32) : (unsigned)b));
      }
      t1 = LM_NOW();
      // the candidate's tests while the granules travel (wave 0, between its publish and its polls; the control step
      // reads the verdict after the gather's barrier)
      if (tid < 64) deferred_tests(sst, lane);
      // every active block's granules of this evaluation (this block's own included), summed in block order as they
      // are gathered
      bool bad = false;
      const double vs = gather_blocks(slot, nact, tag, bad);
      if (__syncthreads_or(bad || a.fail_test)) {
        failed_at = it;
        break;
      }
      t2 = LM_NOW();
      if (tid < LM_NSUM * 8 && (tid & 7) == 0) s_sums[tid >> 3] = GRAM ? vs + s_ssum[tid >> 3] : vs;   // edge + surf
      __syncthreads();
    }
    // (one call site each for the exchange and the control step: a second inlined copy of the control step doubled
    // the kernel's code, 16k instructions against 8k, past what the instruction cache holds)
    if (peers) {
      if (!peer_exchange(a, xs0 + nx, s_sums, s_xch)) {
        failed_at = it;
        break;
      }
      ++nx;
    }
    const unsigned long long t3 = LM_NOW();
    if (tid < 64) control_step(sst, s_sums, lane, false);   // the next point (if the solve goes on)
    if (a.dbg && blk == 0) {
      const unsigned long long t4 = LM_NOW();
      tm[0] += t1 - t0; tm[1] += t2 - t1; tm[2] += t3 - t2; tm[3] += t4 - t3;
    }
  }
  // a timed-out hand-off in ANY block fails the update: xfail, which the state write-back never overwrites, is read
  // by the status gather (the solve's pose is not taken, the handle is poisoned on the host)
  if (failed_at >= 0 && tid == 0) __hip_atomic_store(&a.st->xfail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (blk != 0) return;
  __syncthreads();   // (wave 0's last control step)
  if (tid == 0) {
    if (failed_at >= 0) {   // end the solve, report through n_res
      sst.done = 1;
      sst.n_res = -1;
    }
    sst.xseq = xs0 + nx;
  }
  __syncthreads();
  publish_state(sst, a.st);
  if (a.dbg && tid == 0) {   // diagnostic stamps (100 MHz): evaluate + publish, all-gather, reduce, control step,
    atomicAdd(&a.dbg[0], tm[0]);   // then the prologue (first instruction -> loop) and the write-back
    atomicAdd(&a.dbg[1], tm[1]);
    atomicAdd(&a.dbg[2], tm[2]);
    atomicAdd(&a.dbg[3], tm[3]);
    atomicAdd(&a.dbg[4], 1ull);
    atomicAdd(&a.dbg[5], t_loop - t_start);
    atomicAdd(&a.dbg[6], LM_NOW() - t_start);
  }
}

// ===================================================================================== the sharded evaluation
// Launch k: every block stages the state, runs the control step of evaluation k - 1 on the all-reduced sums (all
// blocks compute the same state), evaluates its records at the resulting point with the resident solve's partition
// and reduction order, and the last-arriving block reduces the block partials (fixed order) + the surf half into
// a.sums for the all-reduce and writes the state (on one rank: the resident solve's bits).
template <bool GRAM, bool HUBER, typename R>
__global__ __launch_bounds__(kTB) void lm_shard_eval(LMArgs a, int k) {
  constexpr int NR = rec_threads<GRAM>();
  __shared__ double s_buf[LM_NSUM * red_stride<NR>()];
  __shared__ double s_sums[LM_NSUM];
  __shared__ double s_ssum[LM_NSUM];
  __shared__ LMState sst;
  __shared__ int s_last;
  const int nblk = (int)gridDim.x, blk = (int)blockIdx.x, tid = (int)threadIdx.x, lane = tid & 63;
  stage_state(a.st, sst);
  if (k > 0 && tid < LM_NSUM) s_sums[tid] = a.sums[tid];   // all-reduced (kernel boundary)
  __syncthreads();
  if (tid < 64) {
    if (k > 0 && !sst.done) control_step(sst, s_sums, lane, true);
    else if (tid < 7 && sst.phase == 0) sst.cand[tid] = sst.x[tid];   // iteration zero evaluates at x
  }
  __syncthreads();
  const bool done = sst.done != 0;
  const int ne = min(*a.d_ne, a.ne_ub);
  const int total = ne + (GRAM ? 0 : min(*a.d_ns, a.ns_ub));
  const int nact = active_blocks<NR>(total, nblk);
  if (!done && blk < nact) {   // block-uniform
    double acc[LM_NSUM];
    if (tid < NR) {
      R x[7];
#pragma unroll
      for (int q = 0; q < 7; ++q) x[q] = (R)sst.cand[q];
      const int stride = nact * NR, i0 = blk * NR + tid;
      R f0[9];
      bool has0, edge0;
      first_record<R>(a, i0, ne, total, f0, has0, edge0);
      eval_records<HUBER, R>(x, has0, edge0, f0, i0 + stride, stride, ne, total, a.erec, a.evalid, a.ecap, a.srec,
                             a.svalid, a.scap, acc);
    } else {
#pragma unroll
      for (int q = 0; q < LM_NSUM; ++q) acc[q] = 0.0;
    }
    const double v = block_sums<NR>(acc, s_buf);
    if (tid < LM_NSUM * kStrips && (tid & 7) == 0)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(&a.partials[(tid >> 3) * nact + blk]),
                         (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // arrival without agent fences (MI355X_MICROARCH.md, sc1 hand-off, first row): sc1 partial stores -> every wave's
  // vmcnt(0) -> barrier -> one lane's ticket add; the block whose add comes last loads the partials sc1
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) s_last = atomicAdd(a.ticket, 1u) == (unsigned)(nblk - 1);
  __syncthreads();
  if (!s_last) return;
  if (!done) {
    reduce_blocks([&](int c, int b) {
      return __longlong_as_double((long long)__hip_atomic_load(
          reinterpret_cast<const unsigned long long*>(&a.partials[c * nact + b]), __ATOMIC_RELAXED,
          __HIP_MEMORY_SCOPE_AGENT));
    }, nact, s_sums);
    if (GRAM) {
      __shared__ double G[kGramW][kGramW];
      __shared__ double o[3];
      gram_unpack(gram_load(a.gmat, tid), G, o);
      if (tid < 64) surf_sums_wave(surf_role(lane), sst.cand, o, G, (double)sst.corr_surf, s_ssum, lane);
      __syncthreads();
      if (tid < LM_NSUM) s_sums[tid] = s_sums[tid] + s_ssum[tid];
      __syncthreads();
    }
    if (tid < LM_NSUM) a.sums[tid] = s_sums[tid];
  } else if (tid < LM_NSUM) {
    a.sums[tid] = 0.0;   // nothing evaluated: the all-reduce still runs on every rank (the same decision everywhere)
  }
  if (tid == 0) *a.ticket = 0u;   // every block has arrived (next launch: kernel boundary)
  __syncthreads();
  publish_state(sst, a.st);
}

// the control step after the last evaluation of a sharded solve
__global__ __launch_bounds__(64) void lm_shard_final(LMState* __restrict__ st, const double* __restrict__ sums) {
  __shared__ LMState sst;
  __shared__ double s_sums[LM_NSUM];
  stage_state(st, sst);
  if (threadIdx.x < LM_NSUM) s_sums[threadIdx.x] = sums[threadIdx.x];
  __syncthreads();
  if (!sst.done) control_step(sst, s_sums, threadIdx.x, true);
  __syncthreads();
  publish_state(sst, st);
}

__global__ void lm_trace(const LMState* __restrict__ st, const int* __restrict__ dcnt, const int* __restrict__ d_me,
                         const int* __restrict__ d_ms, double* __restrict__ trace, unsigned* __restrict__ count,
                         int cap) {
  if (threadIdx.x != 0) return;
  if (!(*d_me > 10 && *d_ms > 50)) return;   // the map-size gate (:77): no solve ran
  const unsigned i = *count;
  *count = i + 1;   // counts every solve: a count above the capacity tells the reader that records were dropped
  if ((int)i >= cap) return;
  double* o = trace + (size_t)i * kTraceWords;
  int k = 0;
  o[k++] = dcnt[0]; o[k++] = dcnt[1]; o[k++] = st->corr_edge; o[k++] = st->corr_surf;
  o[k++] = st->iteration; o[k++] = st->successful; o[k++] = st->initial_cost; o[k++] = st->x_cost;
  for (int j = 0; j < 7; ++j) o[k++] = st->x_in[j];
  for (int j = 0; j < 7; ++j) o[k++] = st->x[j];
  for (int j = 0; j < 21; ++j) o[k++] = st->H0[j];
  for (int j = 0; j < 6; ++j) o[k++] = st->g0[j];
}

LMArgs make_args(LMState* d_st, const CorrSet& ce, const int* d_ne, int ne_ub, const CorrSet& cs, const int* d_ns,
                 int ns_ub, LMBuffers& b, unsigned long long* dbg, const ShardPeers* peers = nullptr) {
  LMArgs a{d_st, ce.rec.p, ce.valid.p, ce.cap, d_ne, std::max(ne_ub, 0), cs.rec.p, cs.valid.p, cs.cap, d_ns,
           std::max(ns_ub, 0), b.gmat.p, b.part.p, b.partials.p, b.sums.p, b.ticket.p, dbg, b.fail_test, 1, nullptr,
           {}, (unsigned)std::max(b.peer_delay_us, 0) * 100u};
  if (peers && peers->world > 1) {
    a.world = peers->world;
    a.xme = peers->mine;
    for (int r = 0; r < peers->world; ++r) a.xpeer[r] = peers->buf[r];
  }
  return a;
}
}  // namespace

void lm_ctrl_stamps_print() {
#ifdef FLOAM_CTRL_STAMPS
  unsigned long long h[8];
  FLOAM_HIP(hipDeviceSynchronize());
  FLOAM_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_ctrl_stamps), sizeof(h)));
  const double n = h[0] ? (double)h[0] : 1.0;
  std::fprintf(stderr, "[floam ctrl] %llu phase-1 control steps (block 0): bookkeeping %.3f us, solve_step %.3f us, "
               "se3_plus %.3f us, candidate hand-over %.3f us; whole step %.3f us\n", h[0], h[1] / n / 100.0,
               h[2] / n / 100.0, h[3] / n / 100.0, h[4] / n / 100.0, h[5] / n / 100.0);
#endif
}

void LMBuffers::reserve(hipStream_t st) {
  if (part.p) return;
  part.reserve((size_t)2 * kRecEvalBlocks * 2 * LM_NSUM);
  partials.reserve((size_t)kRecEvalBlocks * LM_NSUM);
  sums.reserve(LM_NSUM);
  ticket.reserve(1);
  gpart.reserve((size_t)kSurfGeomBlocks * kGram);
  gmat.reserve(kGramMatWords);
  gcnt.reserve(kGramGroups + 1);
  // tag 0 never matches (epochs start at 8), counters start at zero
  FLOAM_HIP(hipMemsetAsync(part.p, 0, sizeof(unsigned long long) * part.cap, st));
  FLOAM_HIP(hipMemsetAsync(ticket.p, 0, sizeof(unsigned), st));
  FLOAM_HIP(hipMemsetAsync(gcnt.p, 0, sizeof(unsigned) * gcnt.cap, st));
  FLOAM_HIP(hipMemsetAsync(gmat.p, 0, sizeof(double) * gmat.cap, st));
}

// Peer mapping probe (floam_odom_set_shard_peers): every rank stores a fixed word at kShardProbeWord of its own
// exchange buffer (system scope) and reads every rank's through the peer mappings until each carries its rank's word or
// kShardProbeTicks have passed.  *fail = the mask of the ranks not seen.  The ranks call set_shard_peers together (they
// have just gathered each other's handles), so a working xGMI mapping answers in microseconds; a mapping that does not
// work fails the peering in seconds — and the caller takes the RCCL form — instead of the first solve's ~20-s wait.
__device__ __forceinline__ unsigned long long probe_word(int r) { return (0x9E3779B9ull << 32) | (unsigned)(r + 1); }

__global__ void peer_probe(ShardPeers P, int rank, int* __restrict__ fail) {
  const int lane = (int)threadIdx.x;
  if (lane == 0)
    __hip_atomic_store(&P.mine[kShardProbeWord], probe_word(rank), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  bool seen = lane >= P.world;
  const unsigned long long* src = P.buf[0];
#pragma unroll
  for (int q = 1; q < kMaxShardRanks; ++q)   // (selected, not indexed: the argument array stays in registers)
    if (q == lane) src = P.buf[q];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (!seen) {
    seen = __hip_atomic_load(&src[kShardProbeWord], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == probe_word(lane);
    if (seen || __builtin_amdgcn_s_memrealtime() - t0 > kShardProbeTicks) break;
    __builtin_amdgcn_s_sleep(8);
  }
  const unsigned long long missing = __ballot(!seen);
  if (lane == 0) *fail = (int)(unsigned)missing;
}

void peer_probe_launch(const ShardPeers& P, int rank, int* d_fail, hipStream_t st) {
  hipLaunchKernelGGL(peer_probe, dim3(1), dim3(64), 0, st, P, rank, d_fail);
  FLOAM_LAUNCH_CHECK();
}

void lm_solve_launch(LMState* d_st, const CorrSet& ce, const int* d_ne, int ne_ub, const CorrSet& cs,
                     const int* d_ns, int ns_ub, int mode, LMBuffers& b, hipStream_t st, unsigned long long* dbg,
                     const ShardPeers* peers) {
  b.reserve(st);
  const LMArgs a = make_args(d_st, ce, d_ne, ne_ub, cs, d_ns, ns_ub, b, dbg, peers);
  // the active blocks (at most 64 or 128 blocks of 256 threads on 256 CUs) are co-resident: checked by the caller
  // through lm_solve_coresident before it chooses this path
  if (mode & LM_GRAM) {
    hipLaunchKernelGGL((lm_solve<true, false, double>), dim3(kEdgeEvalBlocks), dim3(kTB), 0, st, a);
  } else {
    const dim3 g(kRecEvalBlocks);
    switch (mode & (LM_HUBER | LM_FP32)) {
      case LM_HUBER: hipLaunchKernelGGL((lm_solve<false, true, double>), g, dim3(kTB), 0, st, a); break;
      case LM_FP32: hipLaunchKernelGGL((lm_solve<false, false, float>), g, dim3(kTB), 0, st, a); break;
      case LM_HUBER | LM_FP32: hipLaunchKernelGGL((lm_solve<false, true, float>), g, dim3(kTB), 0, st, a); break;
      default: hipLaunchKernelGGL((lm_solve<false, false, double>), g, dim3(kTB), 0, st, a); break;
    }
  }
  FLOAM_LAUNCH_CHECK();
}

template <typename K>
static bool fits(K kernel, int blocks, int device) {
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kTB, 0) != hipSuccess) return false;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return false;
  return (long long)per_cu * cus >= blocks;
}

bool lm_solve_coresident(int mode, int device) {
  if (mode & LM_GRAM) return fits(lm_solve<true, false, double>, kEdgeEvalBlocks, device);
  switch (mode & (LM_HUBER | LM_FP32)) {
    case LM_HUBER: return fits(lm_solve<false, true, double>, kRecEvalBlocks, device);
    case LM_FP32: return fits(lm_solve<false, false, float>, kRecEvalBlocks, device);
    case LM_HUBER | LM_FP32: return fits(lm_solve<false, true, float>, kRecEvalBlocks, device);
    default: return fits(lm_solve<false, false, double>, kRecEvalBlocks, device);
  }
}

void lm_shard_eval_launch(int k, LMState* d_st, const CorrSet& ce, const int* d_ne, int ne_ub, const CorrSet& cs,
                          const int* d_ns, int ns_ub, int mode, LMBuffers& b, hipStream_t st) {
  b.reserve(st);
  const LMArgs a = make_args(d_st, ce, d_ne, ne_ub, cs, d_ns, ns_ub, b, nullptr);
  if (mode & LM_GRAM) {
    hipLaunchKernelGGL((lm_shard_eval<true, false, double>), dim3(kEdgeEvalBlocks), dim3(kTB), 0, st, a, k);
  } else {
    const dim3 g(kRecEvalBlocks);
    switch (mode & (LM_HUBER | LM_FP32)) {
      case LM_HUBER: hipLaunchKernelGGL((lm_shard_eval<false, true, double>), g, dim3(kTB), 0, st, a, k); break;
      case LM_FP32: hipLaunchKernelGGL((lm_shard_eval<false, false, float>), g, dim3(kTB), 0, st, a, k); break;
      case LM_HUBER | LM_FP32: hipLaunchKernelGGL((lm_shard_eval<false, true, float>), g, dim3(kTB), 0, st, a, k); break;
      default: hipLaunchKernelGGL((lm_shard_eval<false, false, double>), g, dim3(kTB), 0, st, a, k); break;
    }
  }
  FLOAM_LAUNCH_CHECK();
}

void lm_shard_final_launch(LMState* d_st, LMBuffers& b, hipStream_t st) {
  hipLaunchKernelGGL(lm_shard_final, dim3(1), dim3(64), 0, st, d_st, b.sums.p);
  FLOAM_LAUNCH_CHECK();
}

void lm_trace_launch(const LMState* d_st, const int* dcnt, const int* d_me, const int* d_ms, double* trace,
                     unsigned* count, int cap, hipStream_t st) {
  hipLaunchKernelGGL(lm_trace, dim3(1), dim3(64), 0, st, d_st, dcnt, d_me, d_ms, trace, count, cap);
  FLOAM_LAUNCH_CHECK();
}

}  // namespace floam
