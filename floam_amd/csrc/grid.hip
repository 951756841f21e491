// Sort-free two-level hash grid over the local maps (the kd-tree replacement of SURVEY.md §8 a-8).
//
// Reference: src/odomEstimationClass.cpp:78-79 rebuilds pcl::KdTreeFLANN over both maps on every
// updatePointsToMap call; here the grids are rebuilt only when the maps changed (a keyframe, :117-122), both maps in
// the same four launches:
//   grid_clear   empty the table entries the previous build occupied (its slot lists; everything after a resize) —
//                run inside the status gather before the build (grid_clear_prepare)
//   grid_count   per point: insert its coarse cell (1 m, absolute coordinates -> 64-bit key; new cells appended to
//                the occupied list), count it in its fine sub-cell (0.5 m) and keep its rank there
//   grid_alloc   per occupied coarse cell (from the list): a contiguous range of the cell-grouped array (one atomic
//                per block on a bump cursor), fine sub-cells consecutive inside it
//   grid_scatter per point: its slot = coarse start + preceding sub-cells + rank
// No bounding box, no sort: O(M) work, every step one launch.
// Incremental variants measured against this rebuild (round 5) and not kept:
//  * a fine-cell table whose cells keep their pool ranges across builds (one counting launch + a relocation fix-up,
//    no alloc / scatter pass): build 23.7 + 12.1 us and the kNN 22 -> 36 us (27 probes per query, cells scattered
//    through the pool) — profiles/r05b_proto_fine_cells (prototype.patch);
//  * this table with persistent cells (keys kept, counts reset; plain-load probes, CAS only for new cells) and
//    XCD-local point ranges: count 14.1, alloc 5.3, scatter 6.3 us against 13.5, 5.1, 5.1 — profiles/r05c_proto_persistent_cells.
#include "floam_common.hpp"
#include "grid.hpp"
#include "odom_kernels.hpp"

namespace floam {

namespace {
constexpr int kTB = 256;

struct GridJob {
  const PointRec* map;
  const int* d_m;
  int m_ub;
  int spec_ub;      // speculative loads of the first stride: below the map's and the slot words' buffer sizes
  float4* pts;
  CoarseCell* coarse;
  uint2* where;
  float4* xyz;      // the map's coordinates by map index (the kNN's neighbour gathers)
  int* clist_new;   // appended by this build
  const int* clist_old;   // cleared by this build
  int* counters;    // [0] cursor, [1 + parity] coarse list size
  int parity;
  int full_clear;
  int bits;
  unsigned mask;
};

__device__ __forceinline__ CoarseCell empty_coarse() {
  CoarseCell c;
  c.key = kEmptyKey;
  c.start = 0;
  c.total = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) c.sub[k] = 0;
  return c;
}

__global__ __launch_bounds__(kTB) void grid_clear(GridClearDev E, GridClearDev S) {
  grid_clear_part(blockIdx.y == 0 ? E : S, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x,
                  blockIdx.x == 0 && threadIdx.x == 0);
}

__host__ __device__ inline GridCountDev count_dev(const GridJob& J) {
  return GridCountDev{J.coarse, J.where, J.clist_new, J.counters, J.parity, J.bits, J.mask};
}

// (grid_count_point, grid.hpp)
__global__ __launch_bounds__(kTB) void grid_count(GridJob E, GridJob S, OdomDev* __restrict__ predict) {
  const GridJob& J = blockIdx.y == 0 ? E : S;
  if (predict && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) odom_predict_step(predict);
  // the first stride's point loaded speculatively beside the device count (inside the map's buffer), so the
  // inserts start one memory round trip earlier; the load is used only when i < m
  const int i_first = blockIdx.x * blockDim.x + threadIdx.x;
  float4 p_first = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i_first < J.spec_ub) p_first = *reinterpret_cast<const float4*>(&J.map[i_first].x);
  const int m = min(*J.d_m, J.m_ub);
  const GridCountDev C = count_dev(J);
  for (int i0 = blockIdx.x * blockDim.x; i0 < m; i0 += gridDim.x * blockDim.x) {   // wave-uniform trip count
    const int i = i0 + threadIdx.x;
    const bool valid = i < m;
    float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
    if (valid) p = i == i_first ? p_first : *reinterpret_cast<const float4*>(&J.map[i].x);
    grid_count_point(C, i, valid, p.x, p.y, p.z);
  }
}

__global__ __launch_bounds__(kTB) void grid_alloc(GridJob E, GridJob S) {
  const GridJob& J = blockIdx.y == 0 ? E : S;
  // the first stride's list entry loaded speculatively beside the list size (t <= mask: inside the list's buffer;
  // entries past the size are stale and never used)
  const int t_first = blockIdx.x * blockDim.x + threadIdx.x;
  const int slot_first = t_first <= (int)J.mask ? J.clist_new[t_first] : 0;
  const int nc = J.counters[1 + J.parity];
  __shared__ int s_wave[kTB / 64];
  __shared__ int s_base;
  for (int t0 = blockIdx.x * blockDim.x; t0 < nc; t0 += gridDim.x * blockDim.x) {   // block-uniform trip count
    const int t = t0 + threadIdx.x;
    CoarseCell c;
    int total = 0, slot = 0;
    if (t < nc) {
      slot = t == t_first ? slot_first : J.clist_new[t];
      c = J.coarse[slot];
#pragma unroll
      for (int k = 0; k < 8; ++k) total += c.sub[k];
    }
    // block exclusive scan of the totals: wave inclusive scan, then the wave totals
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl = total;
    incl = wave_incl_scan(incl);   // (DPP, floam_common.hpp)
    if (lane == 63) s_wave[w] = incl;
    __syncthreads();
    int wbase = 0, btotal = 0;
#pragma unroll
    for (int k = 0; k < kTB / 64; ++k) {
      if (k < w) wbase += s_wave[k];
      btotal += s_wave[k];
    }
    if (threadIdx.x == 0) s_base = btotal ? atomicAdd(&J.counters[0], btotal) : 0;
    __syncthreads();
    if (t < nc) {
      J.coarse[slot].start = s_base + wbase + incl - total;
      J.coarse[slot].total = total;
    }
    __syncthreads();   // s_wave / s_base reuse
  }
}

__global__ __launch_bounds__(kTB) void grid_scatter(GridJob E, GridJob S) {
  const GridJob& J = blockIdx.y == 0 ? E : S;
  // the first stride's slot word and point loaded speculatively beside the device count (inside both buffers)
  const int i_first = blockIdx.x * blockDim.x + threadIdx.x;
  uint2 wr_first = make_uint2(0u, 0u);
  float4 p_first = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i_first < J.spec_ub) {
    wr_first = J.where[i_first];
    p_first = *reinterpret_cast<const float4*>(&J.map[i_first].x);
  }
  const int m = min(*J.d_m, J.m_ub);
  for (int i = i_first; i < m; i += gridDim.x * blockDim.x) {
    const uint2 wr = i == i_first ? wr_first : J.where[i];
    const int sub = (int)(wr.y >> 28), rank = (int)(wr.y & 0x0FFFFFFFu);
    const CoarseCell& c = J.coarse[wr.x];
    int pos = c.start + rank;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < sub) pos += c.sub[k];
    const float4 p = i == i_first ? p_first : *reinterpret_cast<const float4*>(&J.map[i].x);
    J.pts[pos] = make_float4(p.x, p.y, p.z, __int_as_float(i));
    if (J.xyz) J.xyz[i] = make_float4(p.x, p.y, p.z, 0.0f);
  }
}

void reserve_grid(Grid& g, int ub) {
  g.pts.reserve(ub);
  g.where.reserve(ub);
  g.xyz.reserve(ub);
  g.counters.reserve(8);
  int bits = 10;
  // capacity >= 2 x points >= 2 x cells: the load never exceeds 1/2, so every insert and every probe of an absent
  // cell (the kNN's lookups) reaches an empty slot and terminates, even when every point has a cell of its own
  while ((1 << bits) < 2 * ub) ++bits;
  bits = std::max(bits, kDirectBits);   // (the direct-indexed table's minimum, grid.hpp coarse_slot)
  if (bits > g.bits) {   // (reserve keeps the arrays when their capacity already covers the larger table)
    g.coarse.reserve((size_t)1 << bits);
    for (int k = 0; k < 2; ++k) g.clist[k].reserve((size_t)1 << bits);
    g.bits = bits;
    g.mask = (1u << bits) - 1u;
    g.fresh = true;
  }
}

GridClearDev clear_job(const Grid& g) {
  return GridClearDev{g.coarse.p, g.clist[g.parity ^ 1].p, g.counters.p, g.parity, g.fresh ? 1 : 0, g.mask};
}

GridJob make_job(Grid& g, const PointRec* map, const int* d_m, int m_ub, size_t map_cap = 0) {
  const int p = g.parity;
  const int spec = (int)std::min<size_t>({(size_t)m_ub, map_cap, g.where.cap});
  g.src = map;
  return GridJob{map, d_m, m_ub, spec, g.pts.p, g.coarse.p, g.where.p, grid_noxyz() ? nullptr : g.xyz.p,
                 g.clist[p].p, g.clist[p ^ 1].p, g.counters.p, p, g.fresh ? 1 : 0, g.bits, g.mask};
}
}  // namespace

bool grid_noxyz() {
  static const bool on = FLOAM_DIAG_ENV("FLOAM_GRID_NOXYZ") != nullptr;
  return on;
}

GridClearDev grid_clear_prepare(Grid& g, int ub, hipStream_t st) {
  reserve_grid(g, std::max(ub, 1));
  if (g.fresh) FLOAM_HIP(hipMemsetAsync(g.counters.p, 0, sizeof(int) * 8, st));
  const GridClearDev c = clear_job(g);
  g.fresh = false;
  g.precleared = true;
  return c;
}

void grid_build_launch(Grid& gE, const PointRec* mapE, const int* d_mE, int mE_ub, Grid& gS, const PointRec* mapS,
                       const int* d_mS, int mS_ub, hipStream_t st, OdomDev* predict, bool precleared,
                       size_t mE_cap, size_t mS_cap) {
  mE_ub = std::max(mE_ub, 1);
  mS_ub = std::max(mS_ub, 1);
  // a build cleared in advance was sized for at least this map (the upper bounds only shrink once the update that
  // added the points is collected); otherwise the clear runs here (again: clearing the same entries is idempotent)
  precleared = precleared && gE.precleared && gS.precleared && (1 << gE.bits) >= 2 * mE_ub &&
               (1 << gS.bits) >= 2 * mS_ub;
  if (!precleared) {
    reserve_grid(gE, mE_ub);
    reserve_grid(gS, mS_ub);
    if (gE.fresh) FLOAM_HIP(hipMemsetAsync(gE.counters.p, 0, sizeof(int) * 8, st));
    if (gS.fresh) FLOAM_HIP(hipMemsetAsync(gS.counters.p, 0, sizeof(int) * 8, st));
  }
  const GridJob E = make_job(gE, mapE, d_mE, mE_ub, mE_cap), S = make_job(gS, mapS, d_mS, mS_ub, mS_cap);
  if (!precleared) {
    const bool full = gE.fresh || gS.fresh;
    const int tmax = (int)std::max(gE.mask, gS.mask) + 1;
    const unsigned tb = full ? std::min(div_up(tmax, kTB), 2048u) : std::min(div_up(std::max(mE_ub, mS_ub), kTB), 512u);
    hipLaunchKernelGGL(grid_clear, dim3(tb, 2), dim3(kTB), 0, st, clear_job(gE), clear_job(gS));
    FLOAM_LAUNCH_CHECK();
  }
  const unsigned pb = std::min(div_up(std::max(mE_ub, mS_ub), kTB), 2048u);
  hipLaunchKernelGGL(grid_count, dim3(pb, 2), dim3(kTB), 0, st, E, S, predict);
  FLOAM_LAUNCH_CHECK();
  hipLaunchKernelGGL(grid_alloc, dim3(std::min(pb, 512u), 2), dim3(kTB), 0, st, E, S);
  FLOAM_LAUNCH_CHECK();
  hipLaunchKernelGGL(grid_scatter, dim3(pb, 2), dim3(kTB), 0, st, E, S);
  FLOAM_LAUNCH_CHECK();
  for (Grid* g : {&gE, &gS}) {
    g->fresh = false;
    g->precleared = false;
    g->parity ^= 1;
  }
}

}  // namespace floam
