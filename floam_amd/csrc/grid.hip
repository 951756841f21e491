// Sort-free two-level hash grid over the local maps (the kd-tree replacement of SURVEY.md §8 a-8).
//
// Reference: src/odomEstimationClass.cpp:78-79 rebuilds pcl::KdTreeFLANN over both maps on every
// updatePointsToMap call; here the grids are rebuilt only when the maps changed (a keyframe, :117-122), both maps in
// the same four launches:
//   grid_clear   empty both tables of both maps
//   grid_count   per point: insert its coarse cell (1 m, absolute coordinates -> 64-bit key), count it in its fine
//                sub-cell (0.5 m) and keep its rank there
//   grid_alloc   per occupied coarse cell: a contiguous range of the cell-grouped array (one atomic per block on a
//                bump cursor), fine sub-cells consecutive inside it, fine cells inserted into the fine table
//   grid_scatter per point: its slot = coarse start + preceding sub-cells + rank
// No bounding box, no sort: O(M) work, every step one launch.
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
  float4* pts;
  FineCell* fine;
  CoarseCell* coarse;
  uint2* where;
  int* cursor;
  int bits;
  unsigned mask;
};

__global__ __launch_bounds__(kTB) void grid_clear(GridJob E, GridJob S) {
  const GridJob& J = blockIdx.y == 0 ? E : S;
  const int size = (int)J.mask + 1;
  const int stride = gridDim.x * blockDim.x;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < size; t += stride) {
    J.fine[t].key = kEmptyKey;
    CoarseCell c;
    c.key = kEmptyKey;
    c.start = 0;
    c.total = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) c.sub[k] = 0;
    J.coarse[t] = c;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *J.cursor = 0;
}

__global__ __launch_bounds__(kTB) void grid_count(GridJob E, GridJob S) {
  const GridJob& J = blockIdx.y == 0 ? E : S;
  const int m = min(*J.d_m, J.m_ub);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
    const float4 p = *reinterpret_cast<const float4*>(&J.map[i].x);
    int fx, fy, fz;
    fine_cell(p.x, p.y, p.z, fx, fy, fz);
    const unsigned long long key = cell_key(fx >> 1, fy >> 1, fz >> 1);
    const int sub = (fx & 1) | ((fy & 1) << 1) | ((fz & 1) << 2);
    unsigned h = hash_slot64(key, J.bits);
    for (;;) {
      const unsigned long long prev = atomicCAS(&J.coarse[h].key, kEmptyKey, key);
      if (prev == kEmptyKey || prev == key) break;
      h = (h + 1) & J.mask;
    }
    const int rank = atomicAdd(&J.coarse[h].sub[sub], 1);
    J.where[i] = make_uint2(h, ((unsigned)sub << 28) | (unsigned)rank);
  }
}

__global__ __launch_bounds__(kTB) void grid_alloc(GridJob E, GridJob S) {
  const GridJob& J = blockIdx.y == 0 ? E : S;
  const int size = (int)J.mask + 1;
  __shared__ int s_wave[kTB / 64];
  __shared__ int s_base;
  for (int t0 = blockIdx.x * blockDim.x; t0 < size; t0 += gridDim.x * blockDim.x) {   // block-uniform trip count
    const int t = t0 + threadIdx.x;
    CoarseCell c;
    int total = 0;
    if (t < size) {
      c = J.coarse[t];
      if (c.key != kEmptyKey)
#pragma unroll
        for (int k = 0; k < 8; ++k) total += c.sub[k];
    }
    // block exclusive scan of the totals: wave inclusive scan, then the wave totals
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int incl = total;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) s_wave[w] = incl;
    __syncthreads();
    int wbase = 0, btotal = 0;
#pragma unroll
    for (int k = 0; k < kTB / 64; ++k) {
      if (k < w) wbase += s_wave[k];
      btotal += s_wave[k];
    }
    if (threadIdx.x == 0) s_base = btotal ? atomicAdd(J.cursor, btotal) : 0;
    __syncthreads();
    if (t < size && total > 0) {
      const int start = s_base + wbase + incl - total;
      J.coarse[t].start = start;
      J.coarse[t].total = total;
      const int cx = key_x(c.key), cy = key_y(c.key), cz = key_z(c.key);
      int off = start;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (c.sub[k] > 0) {
          const unsigned long long fk = cell_key(2 * cx + (k & 1), 2 * cy + ((k >> 1) & 1), 2 * cz + (k >> 2));
          unsigned h = hash_slot64(fk, J.bits);
          for (;;) {
            const unsigned long long prev = atomicCAS(&J.fine[h].key, kEmptyKey, fk);
            if (prev == kEmptyKey) break;
            h = (h + 1) & J.mask;
          }
          J.fine[h].start = off;
          J.fine[h].count = c.sub[k];
        }
        off += c.sub[k];
      }
    }
    __syncthreads();   // s_wave / s_base reuse
  }
}

__global__ __launch_bounds__(kTB) void grid_scatter(GridJob E, GridJob S) {
  const GridJob& J = blockIdx.y == 0 ? E : S;
  const int m = min(*J.d_m, J.m_ub);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
    const uint2 wr = J.where[i];
    const int sub = (int)(wr.y >> 28), rank = (int)(wr.y & 0x0FFFFFFFu);
    const CoarseCell& c = J.coarse[wr.x];
    int pos = c.start + rank;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < sub) pos += c.sub[k];
    const float4 p = *reinterpret_cast<const float4*>(&J.map[i].x);
    J.pts[pos] = make_float4(p.x, p.y, p.z, __int_as_float(i));
  }
}

void reserve_grid(Grid& g, int ub) {
  g.pts.reserve(ub);
  g.where.reserve(ub);
  g.cursor.reserve(1);
  int bits = 10;
  while ((1 << bits) < 2 * ub) ++bits;   // load <= 1/2 (cells <= points)
  g.fine.reserve((size_t)1 << bits);
  g.coarse.reserve((size_t)1 << bits);
  g.bits = bits;
  g.mask = (1u << bits) - 1u;
}
}  // namespace

void grid_build_launch(Grid& gE, const PointRec* mapE, const int* d_mE, int mE_ub, Grid& gS, const PointRec* mapS,
                       const int* d_mS, int mS_ub, hipStream_t st) {
  mE_ub = std::max(mE_ub, 1);
  mS_ub = std::max(mS_ub, 1);
  reserve_grid(gE, mE_ub);
  reserve_grid(gS, mS_ub);
  const GridJob E{mapE, d_mE, mE_ub, gE.pts.p, gE.fine.p, gE.coarse.p, gE.where.p, gE.cursor.p, gE.bits, gE.mask};
  const GridJob S{mapS, d_mS, mS_ub, gS.pts.p, gS.fine.p, gS.coarse.p, gS.where.p, gS.cursor.p, gS.bits, gS.mask};
  const int tmax = (int)std::max(gE.mask, gS.mask) + 1;
  const unsigned tb = std::min(div_up(tmax, kTB), 2048u);
  const unsigned pb = std::min(div_up(std::max(mE_ub, mS_ub), kTB), 2048u);
  hipLaunchKernelGGL(grid_clear, dim3(tb, 2), dim3(kTB), 0, st, E, S);
  FLOAM_LAUNCH_CHECK();
  hipLaunchKernelGGL(grid_count, dim3(pb, 2), dim3(kTB), 0, st, E, S);
  FLOAM_LAUNCH_CHECK();
  hipLaunchKernelGGL(grid_alloc, dim3(tb, 2), dim3(kTB), 0, st, E, S);
  FLOAM_LAUNCH_CHECK();
  hipLaunchKernelGGL(grid_scatter, dim3(pb, 2), dim3(kTB), 0, st, E, S);
  FLOAM_LAUNCH_CHECK();
}

}  // namespace floam
