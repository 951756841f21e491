// The kNN grid over the local maps (the kd-tree replacement of SURVEY.md §8 a-8), updated incrementally.
//
// Reference: src/odomEstimationClass.cpp:78-79 rebuilds pcl::KdTreeFLANN over both maps on every updatePointsToMap
// call; here the grids are rebuilt only when the maps changed (a keyframe, :117-122, after addPointsToMap :253-294),
// and a rebuild keeps what the map update did not change: the table of fine cells and the pool range of every cell
// persist from build to build (odom_kernels.hpp, Grid).  Per build, both maps in the same launches:
//   (clear)      in the status gather before it (grid_clear_part): every listed cell's fill reset
//   grid_fill    per point: find its cell (a new cell is inserted with capacity 0), add it to the cell's fill, write it
//                at start + rank inside the capacity, else record an overflow entry
//   grid_fixup   per overflow entry: relocate the cell to a fresh pool range sized 2 fill + 8 (the first of its entries
//                allocates and copies the old range; no block ever waits on a block that has not started), then write
//                the point at new start + rank
// No bounding box, no sort, no allocation pass over all cells: a keyframe that leaves most cells within their
// capacity costs one counting launch and a light fix-up.  Tables and pools are sized for the map's upper bound; a
// table holding too many stale cells or a pool nearly used up is reset by the clear (the next build relocates every
// cell, as the first one does).
#include "floam_common.hpp"
#include "grid.hpp"
#include "odom_kernels.hpp"

namespace floam {

namespace {
constexpr int kTB = 256;
constexpr int kFillRounds = 2;     // points per thread and grid stride whose memory round trips are issued together
constexpr int kRelocFailed = -2;   // a relocation that did not fit the pool (or a lost lock holder)

struct FillJob {
  GridDev G;
  const PointRec* map;
  const int* d_m;
  int m_ub;
  int spec_ub;   // speculative loads of the first stride: below the map's buffer size
};

__global__ __launch_bounds__(kTB) void grid_clear(GridClearDev E, GridClearDev S) {
  grid_clear_part(blockIdx.y == 0 ? E : S, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x,
                  blockIdx.x == 0 && threadIdx.x == 0);
}

// wave-aggregated append: lanes with take get consecutive slots of list[*count ...]; returns the lane's slot
__device__ __forceinline__ int wave_append(int* __restrict__ count, bool take) {
  const unsigned long long b = __ballot(take);
  if (!b) return -1;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)b) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(count, __popcll(b));
  base = __shfl(base, leader, 64);
  return take ? base + __popcll(b & ((1ull << lane) - 1ull)) : -1;
}

// R rounds of points at once (valid[r]: the lane has map point i[r] = p[r]); called by all 64 lanes of a wave.  Map
// points are in voxel order, so a wave's points fall in a handful of fine cells: the lanes are grouped by cell
// (ballots), one leader per cell finds or inserts it and adds the group to its fill, ranks in lane order.
template <int R>
__device__ __forceinline__ void fill_points(const GridDev& G, const int* i, const bool* valid, const float4* p) {
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  unsigned long long key[R], grp[R];
  int leader[R];
  unsigned h[R];
  bool look[R], fresh[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    key[r] = kEmptyKey;
    h[r] = 0u;
    if (valid[r]) {
      int fx, fy, fz;
      fine_cell(p[r].x, p[r].y, p[r].z, fx, fy, fz);
      key[r] = cell_key(fx, fy, fz);
      h[r] = cell_slot(fx, fy, fz, G.bits);
    }
    unsigned long long pending = __ballot(valid[r]);
    grp[r] = 0ull;
    while (pending) {   // lanes grouped by key: grp = the lanes sharing my cell
      const int l = __ffsll((long long)pending) - 1;
      const unsigned lo = (unsigned)__shfl((int)(unsigned)key[r], l, 64);
      const unsigned hi = (unsigned)__shfl((int)(unsigned)(key[r] >> 32), l, 64);
      const unsigned long long g = __ballot(valid[r] && key[r] == (((unsigned long long)hi << 32) | lo)) & pending;
      if ((g >> lane) & 1ull) grp[r] = g;
      pending &= ~g;
    }
    leader[r] = valid[r] ? __ffsll((long long)grp[r]) - 1 : lane;
    look[r] = valid[r] && leader[r] == lane;
    fresh[r] = false;
  }
  // the leaders' lookups: every round's probe issued together (plain loads: the table was last written by earlier
  // launches); an empty slot is claimed by CAS, a slot of another key continues the probe
  for (;;) {
    unsigned long long k[R];
#pragma unroll
    for (int r = 0; r < R; ++r) k[r] = look[r] ? G.head[h[r]].key : key[r];
    bool more = false;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!look[r]) continue;
      if (k[r] == kEmptyKey) {
        const unsigned long long prev = atomicCAS(&G.head[h[r]].key, kEmptyKey, key[r]);
        if (prev == kEmptyKey) {
          fresh[r] = true;
          look[r] = false;
          continue;
        }
        k[r] = prev;   // (another wave inserted a cell here just now: maybe this one)
      }
      if (k[r] == key[r]) {
        look[r] = false;
      } else {
        h[r] = (h[r] + 1) & G.mask;
        more = true;
      }
    }
    if (!__any(more)) break;
  }
  // one fill add per (cell, wave) and the cell's range: all rounds issued together
  int rank0[R], start[R], cap[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const bool lead = valid[r] && leader[r] == lane;
    rank0[r] = lead ? atomicAdd(&G.head[h[r]].fill, __popcll(grp[r])) : 0;
    start[r] = lead ? G.head[h[r]].start : 0;   // (a cell new in this build: start 0, capacity 0)
    cap[r] = lead ? G.aux[h[r]].cap : 0;
  }
  bool over[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int rank = __shfl(rank0[r], leader[r], 64) + __popcll(grp[r] & below);
    const int st = __shfl(start[r], leader[r], 64), cp = __shfl(cap[r], leader[r], 64);
    const int hs = __shfl((int)h[r], leader[r], 64);
    over[r] = valid[r] && rank >= cp;
    if (valid[r] && !over[r]) G.pool[st + rank] = make_float4(p[r].x, p[r].y, p[r].z, __int_as_float(i[r]));
    const int o = wave_append(&G.ctr[2], over[r]);
    if (over[r]) {
      G.ovf[o] = make_int4(hs, i[r], rank, 0);
      G.ovf_pt[o] = make_float4(p[r].x, p[r].y, p[r].z, __int_as_float(i[r]));
    }
    const int c = wave_append(&G.ctr[1], fresh[r]);
    if (fresh[r]) G.cells[c] = (int)h[r];
  }
}

__global__ __launch_bounds__(kTB) void grid_fill(FillJob E, FillJob S, OdomDev* __restrict__ predict) {
  const FillJob& J = blockIdx.y == 0 ? E : S;
  if (predict && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) odom_predict_step(predict);
  // the first stride's points loaded speculatively beside the device count (inside the map's buffer), so the
  // lookups start one memory round trip earlier; a load is used only when its index is below the count
  const int stride = (int)(gridDim.x * blockDim.x) * kFillRounds;
  const int i_first = (int)(blockIdx.x * blockDim.x * kFillRounds + threadIdx.x);
  float4 p_first[kFillRounds];
#pragma unroll
  for (int r = 0; r < kFillRounds; ++r) {
    const int i = i_first + r * kTB;
    p_first[r] = i < J.spec_ub ? *reinterpret_cast<const float4*>(&J.map[i].x) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const int m = min(*J.d_m, J.m_ub);
  for (int i0 = i_first; i0 - (int)threadIdx.x < m; i0 += stride) {   // (wave-uniform trip count)
    int i[kFillRounds];
    bool valid[kFillRounds];
    float4 p[kFillRounds];
#pragma unroll
    for (int r = 0; r < kFillRounds; ++r) {
      i[r] = i0 + r * kTB;
      valid[r] = i[r] < m;
      p[r] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (valid[r]) p[r] = i0 == i_first ? p_first[r] : *reinterpret_cast<const float4*>(&J.map[i[r]].x);
      if (valid[r]) J.G.xyz[i[r]] = make_float4(p[r].x, p[r].y, p[r].z, 0.0f);
    }
    fill_points<kFillRounds>(J.G, i, valid, p);
  }
}

// The overflow entries: the first entry of a cell to take its lock relocates it (new range of 2 fill + 8 from the
// pool cursor, the points already in the old range copied, head and capacity updated, the new start published); the
// others retry until it is published.  Every lane retries inside one loop that all lanes of the wave run, so the lane
// holding the lock is never masked off behind a spinning one.
__global__ __launch_bounds__(kTB) void grid_fixup(GridDev E, GridDev S) {
  const GridDev& G = blockIdx.y == 0 ? E : S;
  const int n = G.ctr[2];
  for (int o0 = blockIdx.x * blockDim.x; o0 < n; o0 += gridDim.x * blockDim.x) {   // (block-uniform trip count)
    const int o = o0 + (int)threadIdx.x;
    const bool has = o < n;
    int4 e = make_int4(0, 0, 0, 0);
    float4 pt = make_float4(0.f, 0.f, 0.f, 0.f);
    if (has) {
      e = G.ovf[o];
      pt = G.ovf_pt[o];
    }
    const int slot = e.x;
    int ns = -1;
    bool done = !has;
    for (long long spin = 0; __any(!done); ++spin) {
      if (!done) {
        ns = __hip_atomic_load(&G.aux[slot].nstart, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        done = ns != -1;
      }
      if (!done && atomicCAS(&G.aux[slot].lock, 0, 1) == 0) {
        const int fill = G.head[slot].fill, ostart = G.head[slot].start, ocap = G.aux[slot].cap;
        const int ncap = 2 * fill + 8;
        ns = atomicAdd(&G.ctr[0], ncap);
        if (ns + ncap > G.pool_cap) {   // (the clear keeps room for one build's relocations: never expected)
          ns = kRelocFailed;
        } else {
          const int keep = min(ocap, fill);   // ranks below the old capacity were written into the old range
          for (int j = 0; j < keep; ++j) G.pool[ns + j] = G.pool[ostart + j];
          G.head[slot].start = ns;
          G.aux[slot].cap = ncap;
        }
        __hip_atomic_store(&G.aux[slot].nstart, ns, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        done = true;
      }
      if (!done && spin > (1ll << 22)) {   // (the lock holder never published: never expected)
        ns = kRelocFailed;
        done = true;
      }
      if (__any(!done)) __builtin_amdgcn_s_sleep(1);
    }
    if (has && ns == kRelocFailed) {   // reported through the status gather (the update fails, the handle is poisoned)
      atomicOr(&G.ctr[3], 1);
      if (G.err) atomicOr(G.err, 1);
      G.head[slot].fill = 0;
    }
    if (has && ns >= 0) G.pool[ns + e.z] = pt;
  }
}

GridDev make_dev(Grid& g, int* err) {
  return GridDev{g.head.p, g.aux.p, g.pool.p, g.xyz.p, g.cells.p, g.ovf.p, g.ovf_pt.p, grid_ctr(g, g.parity), err,
                 g.bits, g.mask, (int)std::min<size_t>(g.pool.cap, (size_t)INT32_MAX)};
}

// room for the relocations of one build: each moved cell takes 2 fill + 8, at most 2 ub + 8 ub over all cells
constexpr int kPoolBuilds = 12;   // pool = 12 ub: a full reset once the cursor is past 2 ub

void reserve_grid(Grid& g, int ub, hipStream_t st) {
  ub = std::max(ub, 1);
  g.xyz.reserve(ub);
  g.ovf.reserve(ub);
  g.ovf_pt.reserve(ub);
  if (!g.ctr.p) {
    g.ctr.reserve(2 * kGridCtrWords);
    FLOAM_HIP(hipMemsetAsync(g.ctr.p, 0, sizeof(int) * 2 * kGridCtrWords, st));
  }
  int bits = 10;
  // capacity >= 2 x points: after a clear the table holds at most a quarter stale cells plus one build's new cells
  // (<= points), so every insert and every probe of an absent cell (the kNN's lookups) reaches an empty slot
  while ((1 << bits) < 2 * ub) ++bits;
  if (bits > g.bits) {   // (reserve keeps the arrays when their capacity already covers the larger table)
    g.head.reserve((size_t)1 << bits);
    g.aux.reserve((size_t)1 << bits);
    g.cells.reserve((size_t)1 << bits);
    g.bits = bits;
    g.mask = (1u << bits) - 1u;
    g.fresh = true;
  }
  const size_t pool = (size_t)kPoolBuilds * (size_t)ub + 64;
  if (pool > g.pool.cap) {
    g.pool.reserve(pool);
    g.fresh = true;   // (cell ranges point into the old pool)
  }
  g.ub = std::max(g.ub, ub);
}

GridClearDev clear_job(Grid& g) {
  const long long room = 10ll * g.ub;
  const long long gc = (long long)std::min<size_t>(g.pool.cap, (size_t)INT32_MAX) - room;
  return GridClearDev{g.head.p, g.aux.p, g.cells.p, grid_ctr(g, g.parity ^ 1), grid_ctr(g, g.parity),
                      g.fresh ? 1 : 0, g.mask, (int)((g.mask + 1) / 4), (int)std::max(0ll, gc)};
}
}  // namespace

GridClearDev grid_clear_prepare(Grid& g, int ub, hipStream_t st) {
  reserve_grid(g, ub, st);
  const GridClearDev c = clear_job(g);
  g.fresh = false;
  g.precleared = true;
  return c;
}

void grid_build_launch(Grid& gE, const PointRec* mapE, const int* d_mE, int mE_ub, Grid& gS, const PointRec* mapS,
                       const int* d_mS, int mS_ub, hipStream_t st, OdomDev* predict, bool precleared,
                       size_t mE_cap, size_t mS_cap, int* err) {
  mE_ub = std::max(mE_ub, 1);
  mS_ub = std::max(mS_ub, 1);
  // a build cleared in advance was sized for at least this map (the upper bounds only shrink once the update that
  // added the points is collected); otherwise the clear runs here
  precleared = precleared && gE.precleared && gS.precleared && gE.ub >= mE_ub && gS.ub >= mS_ub;
  if (!precleared) {
    reserve_grid(gE, mE_ub, st);
    reserve_grid(gS, mS_ub, st);
    const GridClearDev cE = clear_job(gE), cS = clear_job(gS);
    const bool full = gE.fresh || gS.fresh;
    const int tmax = (int)std::max(gE.mask, gS.mask) + 1;
    const unsigned tb = full ? std::min(div_up(tmax, kTB), 2048u) : std::min(div_up(std::max(mE_ub, mS_ub), kTB), 512u);
    hipLaunchKernelGGL(grid_clear, dim3(tb, 2), dim3(kTB), 0, st, cE, cS);
    FLOAM_LAUNCH_CHECK();
    gE.fresh = gS.fresh = false;
  }
  const auto job = [err](Grid& g, const PointRec* map, const int* d_m, int m_ub, size_t cap) {
    return FillJob{make_dev(g, err), map, d_m, m_ub, (int)std::min<size_t>((size_t)m_ub, cap ? cap : (size_t)m_ub)};
  };
  const FillJob E = job(gE, mapE, d_mE, mE_ub, mE_cap), S = job(gS, mapS, d_mS, mS_ub, mS_cap);
  const unsigned pb = std::min(div_up(std::max(mE_ub, mS_ub), kTB * kFillRounds), 2048u);
  hipLaunchKernelGGL(grid_fill, dim3(pb, 2), dim3(kTB), 0, st, E, S, predict);
  FLOAM_LAUNCH_CHECK();
  // the fix-up's grid: the overflow entries are a device count (all points at the first build, few afterwards);
  // blocks past it leave at once
  const unsigned fb = std::min(div_up(std::max(mE_ub, mS_ub), kTB), 512u);
  hipLaunchKernelGGL(grid_fixup, dim3(fb, 2), dim3(kTB), 0, st, E.G, S.G);
  FLOAM_LAUNCH_CHECK();
  for (Grid* g : {&gE, &gS}) {
    g->precleared = false;
    g->parity ^= 1;
  }
}

}  // namespace floam
