// Incremental map update of addPointsToMap (src/odomEstimationClass.cpp:253-294): merge the sorted new scan voxels
// into the voxel-ordered map instead of re-sorting the whole map — see mapmerge.hip.
#pragma once
#include "bucket.hpp"
#include "grid.hpp"
#include "voxel.hpp"

namespace floam {

struct MapMergeScratch {
  DevBuf<unsigned long long> status;   // [2][tiles_cap] lookback words of the merge (one array per map)
  DevBuf<int> ctl;                     // [kMergeCtlWords]
  DevBuf<unsigned> flags;              // [2]
  // the scan-voxel sort's splitters: the map merge's own (its keys are map-frame cells of the new scan; the call's
  // VoxelGrids, whose scratch the merge otherwise shares, sort sensor-frame cells — each pipeline's quantiles predict
  // only its own next sort)
  BucketScratch bs;
  int tiles_cap = 0;
  void reserve(int tiles_per_job, hipStream_t st);
};

// What a map's stored cell keys are worth (device, beside the keys): written by the merge that produced the map.
// The keys can be merged against when valid and the producer found them strictly increasing (violation != seq).
struct MapMeta {
  int valid;          // 0: no keys (a raw initMapWithPoints map, Q8)
  unsigned seq;       // serial number of the update whose merge wrote them
  unsigned violation; // == seq: that merge found a centroid outside its voxel (rounded across a cell face), a key
                      // out of range, or an index overflow (its output is then not in voxel order)
  int pad;
};

// One map of the update: its current records (part0 of the VoxelJob) with their stored cell keys and meta, and
// where the new map's keys / meta go (beside J.out / J.d_out).
struct MapKeys {
  const unsigned long long* in = nullptr;
  const MapMeta* meta_in = nullptr;
  unsigned long long* out = nullptr;
  MapMeta* meta_out = nullptr;
};

// the bounding-box stage's checks for map_merge_launch (VoxelFused::mc of the status gather that precedes it)
MergeCheck merge_check(MapMergeScratch& ms, unsigned seq);

// The map update of both maps (jobs a = corner, b = surf; part1 = the downsampled scan, pose != null): the
// bounding-box stage already ran with merge_check(ms, seq) (the status gather).  Per map, when its stored keys are
// clean (MapMeta), the scan is finite and the index range does not overflow, only the scan's cropped voxels are
// sorted (one 32-bit radix sort of the scan points of both maps) and merged into the map; otherwise the map's points
// join the sort (the full VoxelGrid of map + scan, PCL semantics incl. the overflow pass-through).  gate: as
// voxel2_launch (0 = no keyframe: the maps, keys and metas are copied unchanged).  Test knobs (diagnostic build): force_full:
// always the full sort; violate_mod > 0: the merges of updates seq % violate_mod == 0 report their keys out of order
// (the next update then takes the full sort).
void map_merge_launch(VoxelScratch2& vs, MapMergeScratch& ms, const VoxelJob& a, const VoxelJob& b, const MapKeys& ka,
                      const MapKeys& kb, const int* gate, unsigned seq, bool force_full, int violate_mod,
                      hipStream_t st);

void mm_stamps_print();   // FLOAM_MM_STAMPS (diagnostic)

}  // namespace floam
