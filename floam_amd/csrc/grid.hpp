// Cell coordinates and 64-bit keys of the two-level hash grid (device helpers shared by grid.hip and the kNN).
#pragma once
#include "floam_common.hpp"

namespace floam {

// fine cell (edge 0.5 m) of a float point: floor(v / 0.5) in double is exact (v is a float, the division is a
// power-of-two scaling), so cell bounds are exact and the kNN's distance bounds hold exactly
__device__ __forceinline__ void fine_cell(float x, float y, float z, int& fx, int& fy, int& fz) {
  fx = (int)floor((double)x * 2.0);
  fy = (int)floor((double)y * 2.0);
  fz = (int)floor((double)z * 2.0);
}

// 21 bits per axis, offset 2^20 (cells within +-2^20 of the origin: +-524 km for fine cells); clamped
__device__ __forceinline__ unsigned long long cell_key(int x, int y, int z) {
  const int lim = (1 << 20) - 1;
  x = min(max(x, -lim), lim);
  y = min(max(y, -lim), lim);
  z = min(max(z, -lim), lim);
  return ((unsigned long long)(unsigned)(z + (1 << 20)) << 42) | ((unsigned long long)(unsigned)(y + (1 << 20)) << 21) |
         (unsigned long long)(unsigned)(x + (1 << 20));
}
__device__ __forceinline__ int key_x(unsigned long long k) { return (int)(k & 0x1FFFFFull) - (1 << 20); }
__device__ __forceinline__ int key_y(unsigned long long k) { return (int)((k >> 21) & 0x1FFFFFull) - (1 << 20); }
__device__ __forceinline__ int key_z(unsigned long long k) { return (int)(k >> 42) - (1 << 20); }

__device__ __forceinline__ unsigned hash_slot64(unsigned long long key, int bits) {
  return (unsigned)((key * 0x9E3779B97F4A7C15ull) >> (64 - bits));
}

// Initial slot of a coarse cell in the open-addressing table: direct-indexed.  The 2x2x2 block of coarse cells that
// holds it (its "super-cell", coordinates halved) has a bucket of 8 consecutive entries (512 B: 4 cache lines) and the
// cell's position in the block picks the entry; the bucket index is the super-cell's coordinates wrapped to
// 128 x 128 x 2^(bits - 17), x fastest (the table has at least 2^kDirectBits entries, reserve_grid).  Every coarse cell
// of a 256 m x 256 m x 2^(bits - 16) m window (64 m at the minimum size) has a slot of its own — the cropped map (the
// CropBox is 200 m wide) never collides in x and y — and neighbouring super-cells sit side by side, so the 8 coarse
// cells a query's fine block spans sit in 1 to 8 neighbouring buckets.  Cells a window apart share a home slot and
// probe linearly (+1), so every insert and lookup terminates for any map.  Against the former hashed buckets
// (profiles/r05g_direct, the same kernels otherwise): grid build -1.8 us, the status gather's clear -1.9 us, kNN
// -0.15 us per pass, at 2 x 256 MB of table (one full clear when first sized).
constexpr int kDirectBits = 22;
__device__ __forceinline__ unsigned coarse_slot(unsigned long long key, int bits) {
  const int x = (int)(key & 0x1FFFFFull) - (1 << 20), y = (int)((key >> 21) & 0x1FFFFFull) - (1 << 20),
            z = (int)(key >> 42) - (1 << 20);
  const unsigned sub = (unsigned)((x & 1) | ((y & 1) << 1) | ((z & 1) << 2));
  const unsigned sx = (unsigned)(x >> 1) & 127u, sy = (unsigned)(y >> 1) & 127u,
                 sz = (unsigned)(z >> 1) & ((1u << (bits - 17)) - 1u);
  return (((sz << 14) | (sy << 7) | sx) << 3) | sub;
}

constexpr double kFineCell = 0.5;

struct alignas(64) CoarseCell {   // 64 B, one per half cache line: a probe never straddles two lines
  unsigned long long key;
  int start, total;
  int sub[8];                // points per fine sub-cell (x bit 0, y bit 1, z bit 2)
  int pad[4];
};
constexpr unsigned long long kEmptyKey = ~0ull;

// The per-point step of a grid build (grid.hip): the point's coarse cell inserted (new cells appended to the build's
// slot list), its fine sub-cell counted and its rank there kept in where[i].
struct GridCountDev {
  CoarseCell* coarse;
  uint2* where;
  int* clist_new;   // appended by this build
  int* counters;    // [0] cursor, [1 + parity] coarse list size
  int parity;
  int bits;
  unsigned mask;
};

// wave-aggregated append of `slot` (lanes with take) to list[*count ...]
__device__ __forceinline__ void grid_list_append(int* __restrict__ list, int* __restrict__ count, bool take, int slot) {
  const unsigned long long b = __ballot(take);
  if (!b) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)b) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(count, __popcll(b));
  base = __shfl(base, leader, 64);
  if (take) list[base + __popcll(b & ((1ull << lane) - 1ull))] = slot;
}

// Called by all 64 lanes of a wave together, for R rounds of points at once (valid[r]: the lane has point i[r] at
// (x, y, z)[r]; the rounds' atomics are issued together, so R rounds cost the memory round trips of one).  Map points
// are in voxel order, so a wave's 64 points fall in a handful of coarse cells: the wave groups its lanes by cell key
// (ballots, no memory traffic), one leader per cell inserts it, and one leader per (cell, sub-cell) adds the group's
// count — a few atomics per wave on each cache line instead of two per point.  Ranks inside a group follow lane
// order (the order inside a cell is not deterministic across waves either way; the kNN breaks distance ties by map
// index).
template <int R>
__device__ __forceinline__ void grid_count_points(const GridCountDev& J, const int* i, const bool* valid,
                                                  const float* x, const float* y, const float* z) {
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  unsigned long long key[R], my_grp[R];
  int sub[R], leader[R];
  unsigned h[R];
  bool ins[R], fresh[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    key[r] = kEmptyKey;
    sub[r] = 0;
    if (valid[r]) {
      int fx, fy, fz;
      fine_cell(x[r], y[r], z[r], fx, fy, fz);
      key[r] = cell_key(fx >> 1, fy >> 1, fz >> 1);
      sub[r] = (fx & 1) | ((fy & 1) << 1) | ((fz & 1) << 2);
    }
    // lanes grouped by key: my_grp = the lanes sharing my cell, leader = its lowest lane
    unsigned long long pending = __ballot(valid[r]);
    my_grp[r] = 0ull;
    while (pending) {
      const int l = __ffsll((long long)pending) - 1;
      const unsigned lo = (unsigned)__shfl((int)(unsigned)key[r], l, 64);
      const unsigned hi = (unsigned)__shfl((int)(unsigned)(key[r] >> 32), l, 64);
      const unsigned long long grp = __ballot(valid[r] && key[r] == (((unsigned long long)hi << 32) | lo)) & pending;
      if ((grp >> lane) & 1ull) my_grp[r] = grp;
      pending &= ~grp;
    }
    leader[r] = valid[r] ? __ffsll((long long)my_grp[r]) - 1 : lane;
    ins[r] = valid[r] && leader[r] == lane;
    fresh[r] = false;
    h[r] = ins[r] ? coarse_slot(key[r], J.bits) : 0u;
  }
  // the leaders' inserts: every round's probe issued together, until each found its cell or an empty slot
  for (;;) {
    unsigned long long prev[R];
#pragma unroll
    for (int r = 0; r < R; ++r) prev[r] = ins[r] ? atomicCAS(&J.coarse[h[r]].key, kEmptyKey, key[r]) : key[r];
    bool more = false;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (!ins[r]) continue;
      if (prev[r] == kEmptyKey) fresh[r] = true;
      if (prev[r] == kEmptyKey || prev[r] == key[r]) {
        ins[r] = false;
      } else {
        h[r] = (h[r] + 1) & J.mask;
        more = true;
      }
    }
    if (!more) break;
  }
  int leader2[R], base[R];
  unsigned long long sub_grp[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    h[r] = (unsigned)__shfl((int)h[r], leader[r], 64);
    // lanes of my cell with my sub-cell: one add per (cell, sub-cell) group, ranks in lane order
    sub_grp[r] = 0ull;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const unsigned long long b = __ballot(valid[r] && sub[r] == s);
      if (sub[r] == s) sub_grp[r] = b & my_grp[r];
    }
    leader2[r] = valid[r] ? __ffsll((long long)sub_grp[r]) - 1 : lane;
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
    base[r] = valid[r] && leader2[r] == lane ? atomicAdd(&J.coarse[h[r]].sub[sub[r]], __popcll(sub_grp[r])) : 0;
  // the new cells of all rounds appended to the slot list with one atomic
  unsigned long long fb[R];
  int nfresh = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    fb[r] = __ballot(fresh[r]);
    nfresh += __popcll(fb[r]);
  }
  int lbase = 0;
  if (nfresh && lane == 0) lbase = atomicAdd(&J.counters[1 + J.parity], nfresh);
  lbase = __shfl(lbase, 0, 64);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int b = __shfl(base[r], leader2[r], 64);
    if (valid[r]) J.where[i[r]] = make_uint2(h[r], ((unsigned)sub[r] << 28) | (unsigned)(b + __popcll(sub_grp[r] & below)));
    if (fresh[r]) J.clist_new[lbase + __popcll(fb[r] & below)] = (int)h[r];
    lbase += __popcll(fb[r]);
  }
}

__device__ __forceinline__ void grid_count_point(const GridCountDev& J, int i, bool valid, float x, float y, float z) {
  grid_count_points<1>(J, &i, &valid, &x, &y, &z);
}

}  // namespace floam
