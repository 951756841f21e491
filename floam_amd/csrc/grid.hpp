// Fine cells and the persistent hash table of the kNN grid (device helpers shared by grid.hip and the kNN).
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

__device__ __forceinline__ unsigned hash_slot64(unsigned long long key, int bits) {
  return (unsigned)((key * 0x9E3779B97F4A7C15ull) >> (64 - bits));
}

// Initial slot of a fine cell in the open-addressing table: the 2x2x2 block of fine cells that holds it (its
// "super-cell", coordinates halved) picks a bucket of 8 consecutive heads (8 x 16 B: one 128-B line) and the cell's
// position in the block picks the head, so the 27 fine cells of a query's 3x3x3 block lie in 8 buckets, 8 lines.
// Collisions probe linearly (+1), so every insert and lookup terminates while the table has an empty slot.
__device__ __forceinline__ unsigned cell_slot(int x, int y, int z, int bits) {
  const unsigned sub = (unsigned)((x & 1) | ((y & 1) << 1) | ((z & 1) << 2));
  return (hash_slot64(cell_key(x >> 1, y >> 1, z >> 1), bits - 3) << 3) | sub;
}

// The kNN grid of one map (grid.hip): a PERSISTENT open-addressing table of fine cells, each owning a range of a
// point pool.  A build (one per keyframe) only re-counts: every point adds itself to its cell's fill and lands at
// start + rank when its rank is inside the cell's reserved capacity; cells that outgrew their range (and cells new in
// this build, capacity 0) are moved to a fresh range by a second launch.  Cells and ranges survive from build to
// build, so a keyframe that changes few cells moves few points through the second launch.
struct alignas(16) CellHead {   // what the kNN reads: one 16-B load per probe
  unsigned long long key;
  int start;                    // the cell's points are pool[start, start + fill)
  int fill;                     // this build's point count
};
struct alignas(16) CellAux {    // the build's bookkeeping, beside the heads
  int cap;                      // reserved range length
  int lock;                     // this build's relocation: taken by the first of the cell's overflow entries
  int nstart;                   // this build's new range start (-1: not relocated yet)
  int pad;
};
constexpr unsigned long long kEmptyKey = ~0ull;

// Per-build counters, double-buffered by build parity (a build's clear reads the previous build's words and writes
// its own, so no reader races the reset): [0] pool cursor, [1] cells in the persistent list, [2] overflow entries,
// [3] error (a relocation that did not fit the pool: never expected)
constexpr int kGridCtrWords = 8;

struct GridDev {   // one grid as the kernels see it
  CellHead* head;
  CellAux* aux;
  float4* pool;        // {x, y, z, map index bits}, grouped by cell
  float4* xyz;         // {x, y, z, 0} by map index (the kNN's neighbour gathers)
  int* cells;          // persistent list of occupied slots (appended on insert)
  int4* ovf;           // overflow entries {slot, map index, rank, 0}
  float4* ovf_pt;      // their points
  int* ctr;            // this build's counters (kGridCtrWords)
  int* err;            // OdomDev::grid_err of the owning handle (null: none)
  int bits;
  unsigned mask;
  int pool_cap;
};

}  // namespace floam
