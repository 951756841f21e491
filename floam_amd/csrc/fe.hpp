#pragma once
#include "floam_common.hpp"
#include "radix.hpp"

namespace floam {

enum : int { FE_STATUS_BAD_RING = 1, FE_STATUS_SECTOR_TOO_LONG = 2 };

struct FeParams {
  int num_lines;
  double min_distance, max_distance;
};

struct FeScratch {
  DevBuf<uint32_t> keys, keys2;   // ring keys of the bucketing sort (and its ping-pong buffer)
  DevBuf<int> vals;               // input indices before the sort
  RadixScratch rs;                // the sort's control block (this extraction's own: it runs on its own stream)
  DevBuf<int> ring_count, ring_idx, sec_edge_cnt, sec_surf_cnt, sec_edge_pos, surf_pos;
  // the scan staged ring-major once, by the bucketing pass: the sectors stream contiguous coordinates and records
  DevBuf<float4> ring_xyz;
  DevBuf<PointRec> ring_pts;
  DevBuf<int> out3;        // edge count, surf count, status after the call (one D2H)
  DevBuf<unsigned> ticket; // fe_output's arrival counter (its last block commits)
  DevBuf<int> long_sec;    // [0] count, [1..] sectors longer than 1024 entries (fe_sector -> fe_sector_long)
  // sectors beyond 4096 entries (fe_sector_huge): curvature keys, entries, picked / gap flags, two halves each
  DevBuf<unsigned long long> huge_k;
  DevBuf<int> huge_i;
  DevBuf<uint8_t> huge_b;
  int* status = nullptr;   // device int, owned by the caller
  bool zeroed = false;
  int zeroed_lines = 0;
};

// FLOAM_FE_STAMPS=1: print fe_sector's in-kernel phase times (diagnostic; synchronises the device)
void fe_stamps_print();

// Appends edge/surf features of d_in[0, n) to edge_out/surf_out at their device counts (which are advanced).
// clear: bit 0 / bit 1 — the edge / surf output counts are taken as 0 (a pending floam_cloud_clear, folded in).
void fe_launch(FeScratch& sc, const FeParams& prm, const PointRec* d_in, int n, PointRec* edge_out, int* edge_count,
               PointRec* surf_out, int* surf_count, hipStream_t st, int* stat_edge = nullptr,
               int* stat_surf = nullptr, int clear = 0);

}  // namespace floam
