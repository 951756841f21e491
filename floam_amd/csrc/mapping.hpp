// LaserMappingClass (the mapping node's global cell map) on gfx950 — see mapping.hip.
#pragma once
#include "floam_common.hpp"
#include "radix.hpp"

namespace floam {

constexpr int kMapHashSlots = 4096;   // distinct cells one update may touch: <= kMapHashSlots / 2

// Packed absolute cell key: (x + 2^20) << 42 | (y + 2^20) << 21 | (z + 2^20); unsigned order = getMap's (x, y, z)
// loop order (src/laserMappingClass.cpp:188-200).
__host__ __device__ inline unsigned long long map_cell_key(int x, int y, int z) {
  return ((unsigned long long)(x + (1 << 20)) << 42) | ((unsigned long long)(y + (1 << 20)) << 21) |
         (unsigned long long)(z + (1 << 20));
}
inline void map_cell_coords(unsigned long long k, int& x, int& y, int& z) {
  x = (int)((k >> 42) & 0x1FFFFF) - (1 << 20);
  y = (int)((k >> 21) & 0x1FFFFF) - (1 << 20);
  z = (int)(k & 0x1FFFFF) - (1 << 20);
}

struct MapPrepArgs {
  const PointRec* in;
  const int* d_n;
  int n;
  float m[12];                 // pose_current.cast<float>() rows (3 x 4)
  PointRec* stage;             // transformed points, input order
  int* slot;                   // per point: its cell's hash slot
  unsigned long long* hkeys;   // [kMapHashSlots] cell keys (~0 = empty)
  int* hcnt;                   // [kMapHashSlots] points per cell
  int* overflow;               // set when the table fills up
  unsigned* radix_ctl;         // zeroed here for the rank sort that follows
};
// transform + intensity + cell of every point, distinct cells counted in the hash table (cleared by the caller)
void map_prep_launch(const MapPrepArgs& a, hipStream_t st);
// rank keys (per point: rank of its cell, from hrank[slot]) + the rank sort's digit histograms
void map_rank_keys_launch(const int* slot, const int* hrank, int n, uint32_t* keys, int* vals, unsigned* radix_ctl,
                          hipStream_t st);
// dst[j] = src[perm[j]]
void map_gather_launch(const PointRec* src, const int* perm, int n, PointRec* dst, hipStream_t st);

struct MapCopyArgs {
  int ncell;
  const int* outcnt;        // [ncell] points of each cell after the update (voxel jobs wrote theirs)
  int* off;                 // [ncell + 1] exclusive scan of outcnt (written by map_offsets)
  const int* old_start;     // [ncell] cell's first point in the old map (or -1 if new)
  const int* seg;           // [2 * ncell] old count, new count
  const int* new_start;     // [ncell] cell's first point among the cell-sorted new points
  const int* vox_off;       // [ncell] filtered cells: first output slot in the voxel scratch, else -1
  const PointRec* old_map;
  const PointRec* new_pts;
  const PointRec* vox;
  PointRec* out;
  int* d_total;             // map size after the update
};
// offsets (one block) and the copy of every cell's final points into the new map, in cell order
void map_rebuild_launch(const MapCopyArgs& a, int total_ub, hipStream_t st);

}  // namespace floam
