// Incremental map update: addPointsToMap (src/odomEstimationClass.cpp:253-294) without re-sorting the whole map.
//
// The reference re-voxelises map + transformed scan every keyframe: CropBox [t +- 100] of both, then PCL 1.8.1
// VoxelGrid — a sort of all points by voxel index, one centroid per voxel in ascending index.  The previous map is
// itself a VoxelGrid output, so it is already in ascending voxel order, and the order of voxel indices does not depend
// on the grid's min_b (idx = i + j dx + k dx dy with ijk = floor(p inv) - min_b orders points exactly as the cell
// (floor(z inv), floor(y inv), floor(x inv)) does); CropBox keeps the order.  So the stable sort of [map ; scan] by
// voxel is the merge of the map (in order) with the stably sorted scan, the map's point first within a voxel.
//
// Each map point keeps its cell key (mm_cell_key of its own coordinates — what the next VoxelGrid computes).  The
// merge that writes a map checks that every centroid lies in the voxel of its own run (then the keys are strictly
// increasing: one output per voxel, in voxel order; a centroid rounded across a cell face breaks it) and records the
// verdict in the map's MapMeta.  The next update merges against the map when the verdict
// is clean, the scan is finite and the index range does not overflow; otherwise it takes the full sort (the map's
// points join the sort set: PCL's VoxelGrid of map + scan, the overflow pass-through included).
//
// Launches per update (both maps at once): mm_keys (the sort set's 32-bit voxel keys + digit histograms, the
// VoxelGrid's own key arithmetic), the four radix passes (radix.hip) — over the scan voxels only on the merge path —
// and mm_merge (merge-path tiles: partition by a 128-ary search of the two index sequences, the tile's elements
// merged in LDS, runs -> centroids, decoupled-lookback output positions, the new map's cell keys and verdict).
// Merge comparisons run on voxel indices: the set's sort keys, and the map's stored cell keys mapped into the same
// grid — a cropped map point may lie outside it and is saturated to the first / last cell of its row, plane or grid,
// which keeps the order (it takes part in the order only: a cropped point adds nothing to a centroid).
#include <cfloat>
#include <climits>

#include "cloud_ops.hpp"
#include "lookback.hpp"
#include "mapmerge.hpp"
#include "profwb.hpp"
#include "radix.hpp"

namespace floam {

namespace {
constexpr int kTB = 256;
constexpr int kMergePer = 4;   // merged elements per thread: 1024-element tiles (512 measured the same)
constexpr unsigned long long kNone = ~0ull;   // no element (never an index or a sort key: both < 2^32)

__global__ __launch_bounds__(kTB) void mm_keys(VoxelJobDev A, VoxelJobDev B, const float* __restrict__ partials,
                                               uint32_t* __restrict__ keys, int* __restrict__ vals,
                                               unsigned long long* __restrict__ mstatus, int status_words,
                                               unsigned* __restrict__ radix_ctl, const int* __restrict__ gate,
                                               int* __restrict__ n_dev, int* __restrict__ ctl,
                                               const MapMeta* __restrict__ metaA, const MapMeta* __restrict__ metaB,
                                               const unsigned* __restrict__ flags, unsigned seq, int force_full,
                                               BucketDev bd) {
  // the prologue's loads are all issued before any is waited on (one round trip instead of four in a row): the gate,
  // the bounding-box partials, the metas, the flags, the counts and — for the merge path, where element e is scan
  // point e — this thread's first scan record and the pose (the host bound n1_ub keeps the load inside the array), and
  // this thread's splitter
  const int job = blockIdx.y;
  const int gv = gate ? *gate : 1;
  const MapMeta mA = *metaA, mB = *metaB;
  const unsigned flA = flags[0], flB = flags[1];
  const int dA0 = *A.d_n0, dA1 = *A.d_n1, dB0 = *B.d_n0, dB1 = *B.d_n1;
  float pv[2][kVoxMinMaxBlocks / 32];
#pragma unroll
  for (int h = 0; h < 2; ++h) {   // partial q = threadIdx.x + 256 h of the 384 (2 jobs x 6 components x 32 lanes)
    const int q = threadIdx.x + kTB * h;
    const int jb = q / 192, c = (q / 32) % 6, l = q & 31;
#pragma unroll
    for (int u = 0; u < kVoxMinMaxBlocks / 32; ++u)
      pv[h][u] = q < 2 * 6 * 32 ? partials[(jb * kVoxMinMaxBlocks + l + 32 * u) * 6 + c] : 0.f;
  }
  const VoxelJobDev& J0 = job ? B : A;
  // this thread's first element: a chunk of kTB x kAppendR per block with the bucket append, else a grid stride
  const int e0 = blockIdx.x * blockDim.x * (bd.split ? kAppendR : 1) + threadIdx.x;
  // (the bucket append: all kAppendR scan records of this thread's first chunk, element e0 + r kTB)
  float4 sp[kAppendR];
#pragma unroll
  for (int r = 0; r < kAppendR; ++r) {
    const int e = e0 + r * kTB;
    sp[r] = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((r == 0 || bd.split) && e < J0.n1_ub) sp[r] = *reinterpret_cast<const float4*>(&J0.part1[e].x);
  }
  double pose0[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) pose0[k] = J0.pose[k];
  const unsigned long long sp_t = bucket_split_prefetch(bd.split);   // (the splitters, bucket_keys_lds)
  if (!gv) return;
  __shared__ float s_mm[2][6];
  __shared__ unsigned s_hist[kRadixHistWords];
  __shared__ int s_kept;
  radix_hist_begin(s_hist);   // (bd.split: the bucket histogram in its first 256 words)
  if (threadIdx.x == 0) s_kept = 0;
  // both maps' bounding boxes (job B's elements are packed after job A's, whose count depends on A's mode)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int q = threadIdx.x + kTB * h;
    if (q >= 2 * 6 * 32) continue;   // (wave-uniform: 384 = 6 waves)
    const int jb = q / 192, c = (q / 32) % 6, l = q & 31;
    const bool is_min = c < 3;
    float v = is_min ? FLT_MAX : -FLT_MAX;
#pragma unroll
    for (int u = 0; u < kVoxMinMaxBlocks / 32; ++u) v = is_min ? fminf(v, pv[h][u]) : fmaxf(v, pv[h][u]);
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      const float w = __shfl_xor(v, o, 64);
      v = is_min ? fminf(v, w) : fmaxf(v, w);
    }
    if (l == 0) s_mm[jb][c] = v;
  }
  for (int t = (job * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x; t < status_words;
       t += 2 * gridDim.x * blockDim.x)
    mstatus[t] = 0ull;   // lookback state of mm_merge
  __syncthreads();
  VoxelGeom gA, gB;
  int dzA, dzB;
  {
    const float mn[3] = {s_mm[0][0], s_mm[0][1], s_mm[0][2]}, mx[3] = {s_mm[0][3], s_mm[0][4], s_mm[0][5]};
    gA = voxel_geom(mn, mx, A.inv);
    dzA = (int)floorf(mx[2] * A.inv) - gA.min_b[2] + 1;
  }
  {
    const float mn[3] = {s_mm[1][0], s_mm[1][1], s_mm[1][2]}, mx[3] = {s_mm[1][3], s_mm[1][4], s_mm[1][5]};
    gB = voxel_geom(mn, mx, B.inv);
    dzB = (int)floorf(mx[2] * B.inv) - gB.min_b[2] + 1;
  }
  // the full sort if forced, the map's keys are absent or out of order, a scan point is not finite, or overflow
  const bool fullA = force_full || !mA.valid || mA.violation == mA.seq || flA == seq || gA.overflow;
  const bool fullB = force_full || !mB.valid || mB.violation == mB.seq || flB == seq || gB.overflow;
  const int nA0 = min(dA0, A.n0_ub), nA1 = min(dA1, A.n1_ub);
  const int nB0 = min(dB0, B.n0_ub), nB1 = min(dB1, B.n1_ub);
  const int sizeA = (fullA ? nA0 : 0) + nA1, sizeB = (fullB ? nB0 : 0) + nB1;
  if (job == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
    *n_dev = sizeA + sizeB;
    ctl[2] = fullA; ctl[3] = fullB;
    ctl[4] = gA.overflow; ctl[5] = gB.overflow;
    for (int d = 0; d < 3; ++d) {   // the grids: min_b, then dx, dy, dz
      ctl[6 + d] = gA.min_b[d];
      ctl[12 + d] = gB.min_b[d];
    }
    ctl[9] = gA.divb_mul[1];
    ctl[10] = gA.divb_mul[1] ? gA.divb_mul[2] / gA.divb_mul[1] : 0;
    ctl[11] = dzA;
    ctl[15] = gB.divb_mul[1];
    ctl[16] = gB.divb_mul[1] ? gB.divb_mul[2] / gB.divb_mul[1] : 0;
    ctl[17] = dzB;
  }
  const VoxelJobDev& J = job ? B : A;
  const bool full = job ? fullB : fullA;
  VoxelGeom G;   // (a copy selected field by field: a reference to one of the two kept both in scratch)
  for (int d = 0; d < 3; ++d) {
    G.min_b[d] = job ? gB.min_b[d] : gA.min_b[d];
    G.divb_mul[d] = job ? gB.divb_mul[d] : gA.divb_mul[d];
  }
  G.overflow = job ? gB.overflow : gA.overflow;
  const int n0 = job ? nB0 : nA0, n1 = job ? nB1 : nA1;
  const int start = full ? 0 : n0, count = job ? sizeB : sizeA, base = job ? sizeA : 0;
  __shared__ uint32_t s_spl[kBuckets];
  const bool bucket = vox_bucket_begin(bd, sp_t, job, G, job ? s_mm[1][5] : s_mm[0][5], J.inv, s_spl);
  int kept = 0;
  // sort key of element e of the job's set (0xFFFFFFFF: cropped); pre: its scan record prefetched (the merge path)
  auto key_of = [&](int e, bool pre, float4 spr) {
    const int i = start + e;   // index into the job's [map ; scan] concatenation
    float4 q;   // (x, y, z, intensity: no PointRec temporary, which stays a private array in this kernel)
    bool in;
    if (!full && pre) {   // the prefetched scan record: vox_fetch's transform and CropBox, on registers
      float x, y, z;
      associate_to_map(pose0, spr.x, spr.y, spr.z, x, y, z);
      q = make_float4(x, y, z, 0.f);
      const float mnx = (float)(pose0[4] - 100), mny = (float)(pose0[5] - 100), mnz = (float)(pose0[6] - 100);
      const float mxx = (float)(pose0[4] + 100), mxy = (float)(pose0[5] + 100), mxz = (float)(pose0[6] + 100);
      in = !(x < mnx || y < mny || z < mnz || x > mxx || y > mxy || z > mxz);
    } else {
      in = vox_fetch4(J, n0, n1, i, q);
    }
    if (!in) return 0xFFFFFFFFu;
    ++kept;
    return ((uint32_t)job << 31) | (G.overflow ? (uint32_t)i : voxel_idx(G, J.inv, q.x, q.y, q.z));
  };
  if (bucket) {   // appended to the buckets' regions: no keys array, no scatter pass
    for (int c0 = blockIdx.x * blockDim.x * kAppendR; c0 < count; c0 += gridDim.x * blockDim.x * kAppendR) {
      uint32_t key[kAppendR];
      int val[kAppendR];
#pragma unroll
      for (int r = 0; r < kAppendR; ++r) {
        const int e = c0 + r * kTB + (int)threadIdx.x;
        key[r] = e < count ? key_of(e, e == e0 + r * kTB && e < J0.n1_ub, sp[r]) : 0xFFFFFFFFu;
        val[r] = start + e;
      }
      bucket_append<kAppendR>(bd, radix_ctl, s_spl, key, val, s_hist, reinterpret_cast<int*>(s_hist + kBuckets),
                              reinterpret_cast<int*>(s_hist + 2 * kBuckets));
    }
    if (kept) atomicAdd(&s_kept, kept);
    __syncthreads();
  } else {
    for (int e = e0; e < count; e += gridDim.x * blockDim.x) {
      const uint32_t key = key_of(e, e == e0 && e < J0.n1_ub, sp[0]);
      keys[base + e] = key;
      vals[base + e] = start + e;
      radix_hist_add(s_hist, key);
    }
    if (kept) atomicAdd(&s_kept, kept);
    radix_hist_end(s_hist, radix_ctl);   // (its barrier orders s_kept)
  }
  if (threadIdx.x == 0 && s_kept) atomicAdd(&ctl[job], s_kept);
}

// ---------------------------------------------------------------------------------------------- merge tiles
struct MergeView {   // one map of the update as mm_merge sees it
  VoxelJobDev J;
  MapKeys K;
  int n0, n1;        // map points, scan points (device counts)
  int nset, base;    // the job's sort-set elements (not cropped) and their first position in the sorted arrays
  bool full, ovf;
  long long mb[3], dx, dy, dz;   // the VoxelGrid's min_b and dimensions
  const uint32_t* skeys;
  const int* svals;
};

// the record of concatenation element i (kept: in the crop box)
__device__ __forceinline__ bool mv_fetch4(const MergeView& V, int i, float4& q) { return vox_fetch4(V.J, V.n0, V.n1, i, q); }

// ov[nout++] = v with nout in registers: every slot a compare-select (a dynamically indexed array is private memory)
template <int PER>
__device__ __forceinline__ void put_out(float4 (&ov)[PER], int& nout, float4 v) {
#pragma unroll
  for (int q = 0; q < PER; ++q)
    if (q == nout) ov[q] = v;
  ++nout;
}

// voxel index of sort-set element j (its sort key without the cloud bit)
__device__ __forceinline__ unsigned long long set_idx(const MergeView& V, int j) {
  return (unsigned long long)(V.skeys[V.base + j] & 0x7FFFFFFFu);
}

// voxel index of map element i from its stored cell key; a cell outside the grid (a point the crop removes) is
// saturated in lexicographic order: below the grid -> its first cell, beyond -> its last, likewise per plane and row
__device__ __forceinline__ unsigned long long map_idx(const MergeView& V, int i) {
  const unsigned long long k = V.K.in[i];
  const long long cx = (long long)(k & 0x1FFFFFull) - (1 << 20) - V.mb[0];
  const long long cy = (long long)((k >> 21) & 0x1FFFFFull) - (1 << 20) - V.mb[1];
  const long long cz = (long long)(k >> 42) - (1 << 20) - V.mb[2];
  const long long plane = V.dx * V.dy;
  if (cz < 0) return 0ull;
  if (cz >= V.dz) return (unsigned long long)(plane * V.dz - 1);
  if (cy < 0) return (unsigned long long)(cz * plane);
  if (cy >= V.dy) return (unsigned long long)(cz * plane + plane - 1);
  if (cx < 0) return (unsigned long long)(cz * plane + cy * V.dx);
  if (cx >= V.dx) return (unsigned long long)(cz * plane + cy * V.dx + V.dx - 1);
  return (unsigned long long)(cz * plane + cy * V.dx + cx);
}

// Merge-path split of merged position d: the number of map elements among the first d merged elements (map element
// i precedes set element j iff idx_i <= idx_j: a map point comes first within its voxel).  Called by all 256
// threads: the two halves (h = 0, 1) search for their own d together, 128 threads each; every round tests 128 evenly
// spaced candidates of the remaining range (the predicate is true, then false, along it), so a range of R closes in
// log_128 R rounds of one memory round trip each.
__device__ __forceinline__ int merge_split(const MergeView& V, int d, int lane128, int half, int* s_first,
                                           int* s_open) {
  int lo = max(0, d - V.nset), hi = min(d, V.n0);   // answer in [lo, hi]; pred(hi) is false
  for (;;) {
    const bool open = lo < hi;
    if (lane128 == 0) s_open[half] = open;
    if (lane128 == 0) s_first[half] = INT_MAX;
    __syncthreads();
    if (!s_open[0] && !s_open[1]) break;
    const int range = hi - lo;
    const int c = lo + (int)(((long long)range * lane128) / 128);
    if (open) {   // pred(c): map element c precedes set element d - c - 1
      const bool pred = c < V.n0 && d - c - 1 >= 0 && map_idx(V, c) <= set_idx(V, d - c - 1);
      if (!pred) atomicMin(&s_first[half], lane128);
    }
    __syncthreads();
    if (open) {
      const int f = s_first[half];
      if (f == 0) {
        hi = lo;
      } else if (f == INT_MAX) {
        lo = lo + (int)(((long long)range * 127) / 128) + 1;
      } else {
        const int cprev = lo + (int)(((long long)range * (f - 1)) / 128);
        hi = lo + (int)(((long long)range * f) / 128);
        lo = cprev + 1;
      }
    }
    __syncthreads();   // (s_first / s_open are rewritten next round)
  }
  return lo;
}

// the voxel index of a point in the update's grid (voxel_idx's arithmetic): an output keeps its place in the map's
// order exactly when its centroid lies in its own run's voxel (a centroid rounded across a face does not)
__device__ __forceinline__ unsigned long long mv_idx(const MergeView& V, float x, float y, float z) {
  const float inv = V.J.inv;
  const int i0 = (int)(floorf(x * inv) - (float)V.mb[0]);
  const int i1 = (int)(floorf(y * inv) - (float)V.mb[1]);
  const int i2 = (int)(floorf(z * inv) - (float)V.mb[2]);
  if (i0 < 0 || i1 < 0 || i2 < 0 || i0 >= V.dx || i1 >= V.dy || i2 >= V.dz) return kNone;
  return (unsigned long long)i0 + (unsigned long long)i1 * V.dx + (unsigned long long)i2 * V.dx * V.dy;
}


// One job's tile (the kernel below calls it with the job's own kernel arguments: selecting the argument structs by a
// run-time job index made the compiler copy both into scratch and load every field from there — 144-176 B / lane of
// private memory traffic per launch)
// FLOAM_MM_STAMPS=1 (diagnostic): per-tile phase times of the last merge (start, split, LDS merge, runs, lookback,
// stores), printed by mm_stamps_print
constexpr int kMmStampTiles = 512;
__device__ unsigned g_mm_st[2][kMmStampTiles][6];
__device__ __forceinline__ unsigned long long mm_now(int on) { return on ? __builtin_amdgcn_s_memrealtime() : 0ull; }

template <int PER>
__device__ __forceinline__ void mm_merge_job(const VoxelJobDev& JJ, const MapKeys& KK, int job,
                                             const uint32_t* __restrict__ skeys, const int* __restrict__ svals,
                                             int* __restrict__ ctl, unsigned long long* __restrict__ mstatus,
                                             int tiles_cap, int tilesA,
                                             const unsigned* __restrict__ radix_ctl, const int* __restrict__ gate,
                                             unsigned seq, int violate_mod,
                                             int stamps) {
  const unsigned long long T0 = mm_now(stamps);
  // prologue loads first, so they travel with the ticket: the counts, the gate and the status gather's verdict words
  // (none depends on the tile; on the gated-off path the verdict words are read but unused)
  MergeView V;
  V.J = JJ;
  V.K = KK;
  V.n0 = min(*V.J.d_n0, V.J.n0_ub);
  V.n1 = min(*V.J.d_n1, V.J.n1_ub);
  const bool gated_off = gate && !*gate;
  V.full = ctl[2 + job] != 0;
  V.ovf = ctl[4 + job] != 0;
  V.nset = ctl[job];
  V.base = job ? ctl[0] : 0;
  for (int d = 0; d < 3; ++d) V.mb[d] = ctl[6 + 6 * job + d];
  V.dx = ctl[9 + 6 * job];
  V.dy = ctl[10 + 6 * job];
  V.dz = ctl[11 + 6 * job];
  // the tile within the job is the block's ticket (ctl[kMergeTicketWord + 32 job], zeroed by the status gather): a
  // tile's lookback only waits on tiles that are already running (HIP promises no dispatch order)
  __shared__ int s_tile;
  if (threadIdx.x == 0)
    s_tile = atomicAdd(&ctl[kMergeTicketWord + 32 * job], 1);
  const int njb = job ? (int)gridDim.x - tilesA : tilesA;   // this job's blocks
  const int t = threadIdx.x;
  __syncthreads();
  const int tile = s_tile;
  if (gated_off) {   // no keyframe: the map, its keys and their verdict stay as they are (no lookback: by index)
    const int tile = job ? (int)blockIdx.x - tilesA : (int)blockIdx.x;
    for (int i0 = tile * kTB; i0 < V.n0; i0 += njb * kTB) {   // (wave-uniform trip count: the grid count)
      const int i = i0 + t;
      if (i < V.n0) {
        const float4* q = reinterpret_cast<const float4*>(V.J.part0 + i);
        float4* o = reinterpret_cast<float4*>(V.J.out + i);
        o[0] = q[0];
        o[1] = q[1];
        V.K.out[i] = V.K.in[i];
      }
    }
    if (tile == 0 && t == 0) {
      *V.J.d_out = V.n0;
      *V.K.meta_out = *V.K.meta_in;
    }
    return;
  }
  V.skeys = skeys;
  V.svals = svals;
  const int L = V.full ? V.nset : V.n0 + V.nset;   // merged elements
  const int ntiles = (L + (PER * kTB) - 1) / (PER * kTB);
  if (tile >= ntiles) {   // (block-uniform; nobody waits on a tile beyond the last)
    if (tile == 0 && t == 0) {
      *V.J.d_out = 0;
      V.K.meta_out->valid = 1;
      V.K.meta_out->seq = seq;
    }
    return;
  }
  const int d0 = tile * (PER * kTB), d1 = min(L, d0 + (PER * kTB)), cnt = d1 - d0;
  // the tile's merged elements in LDS: key (s_key[k + 1] for element k; s_key[0] the previous element, s_key[cnt + 1]
  // the next one), point, source index (concatenation), kept flag
  __shared__ unsigned long long s_key[(PER * kTB) + 2];
  __shared__ float4 s_pt[(PER * kTB)];
  __shared__ int s_src[(PER * kTB)];
  __shared__ unsigned char s_live[(PER * kTB)];
  __shared__ int s_split[2], s_first[2], s_open[2];
  __shared__ int s_has_cross;   // a run of this tile continues past it (finished cooperatively below)
  unsigned long long T1 = 0ull;
  int j1 = d1;       // first set element after the tile (sorted order)
  int i1m = V.n0;    // first map element after the tile (the merge path; none on the full path: the map is in the set)
  if (t == 0) s_has_cross = 0;
  if (V.full) {
    for (int k = t; k < cnt; k += kTB) {
      const int pos = V.base + d0 + k;
      const int src = svals[pos];
      float4 q;
      mv_fetch4(V, src, q);
      s_key[k + 1] = skeys[pos];
      s_pt[k] = q;
      s_src[k] = src;
      s_live[k] = 1;
    }
    if (t == 0) s_key[0] = d0 > 0 ? skeys[V.base + d0 - 1] : kNone;
    if (t == 1) s_key[cnt + 1] = d1 < L ? skeys[V.base + d1] : kNone;
  } else {
    int i0, i1, j0;
    {
      const int half = t >> 7, lane128 = t & 127;
      const int sp = merge_split(V, half ? d1 : d0, lane128, half, s_first, s_open);
      if (lane128 == 0) s_split[half] = sp;
      __syncthreads();
      i0 = s_split[0];
      i1 = s_split[1];
      j0 = d0 - i0;
      j1 = d1 - i1;
      i1m = i1;
    }
    T1 = mm_now(stamps);
    const int na = i1 - i0, nb = j1 - j0;
    // the two runs' indices in LDS (points, sources, kept flags stay in registers: element k = t + r kTB)
    __shared__ unsigned long long s_ak[(PER * kTB)], s_bk[(PER * kTB)];
    float4 rp[PER];
    int rs[PER];
    bool rl[PER];
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const int k = t + r * kTB;
      rs[r] = 0;
      rl[r] = false;
      rp[r] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k >= na + nb) continue;
      float4 q;
      if (k < na) {
        const int i = i0 + k;
        rl[r] = mv_fetch4(V, i, q);
        rs[r] = i;
        s_ak[k] = map_idx(V, i);
      } else {
        const int j = j0 + k - na;
        rs[r] = svals[V.base + j];
        rl[r] = true;
        mv_fetch4(V, rs[r], q);
        s_bk[k - na] = set_idx(V, j);
      }
      rp[r] = q;
    }
    if (t == 0) {   // the merged element before the tile: the later of map[i0 - 1] and set[j0 - 1]
      unsigned long long prev = kNone;
      const bool hm = i0 > 0, hs = j0 > 0;
      const unsigned long long km = hm ? map_idx(V, i0 - 1) : 0ull, ks = hs ? set_idx(V, j0 - 1) : 0ull;
      if (hm && hs) prev = km > ks ? km : ks;
      else if (hm) prev = km;
      else if (hs) prev = ks;
      s_key[0] = prev;
    }
    if (t == 1) {   // the merged element after the tile: the earlier of map[i1] and set[j1] (the map first on ties)
      unsigned long long next = kNone;
      const bool hm = i1 < V.n0, hs = j1 < V.nset;
      const unsigned long long km = hm ? map_idx(V, i1) : 0ull, ks = hs ? set_idx(V, j1) : 0ull;
      if (hm && hs) next = km <= ks ? km : ks;
      else if (hm) next = km;
      else if (hs) next = ks;
      s_key[cnt + 1] = next;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < PER; ++r) {   // merged position: own rank + the other run's elements before it
      const int k = t + r * kTB;
      if (k >= na + nb) continue;
      int pos;
      unsigned long long key;
      if (k < na) {
        key = s_ak[k];
        int lo = 0, hi = nb;   // set elements with idx < idx (strictly: the map first within a voxel)
        while (lo < hi) {
          const int m = (lo + hi) >> 1;
          if (s_bk[m] < key) lo = m + 1; else hi = m;
        }
        pos = k + lo;
      } else {
        const int b = k - na;
        key = s_bk[b];
        int lo = 0, hi = na;   // map elements with idx <= idx
        while (lo < hi) {
          const int m = (lo + hi) >> 1;
          if (s_ak[m] <= key) lo = m + 1; else hi = m;
        }
        pos = b + lo;
      }
      s_key[pos + 1] = key;
      s_pt[pos] = rp[r];
      s_src[pos] = rs[r];
      s_live[pos] = rl[r] ? 1 : 0;
    }
  }
  __syncthreads();
  const unsigned long long T2 = mm_now(stamps);
  // runs: element k heads a run when its key differs from the previous element's; a run is output when one of its
  // elements is kept (a cropped map point takes part in the order only); its centroid sums the kept points in merged
  // order.  A run that continues past the tile is finished by the whole block: its continuation is the merged
  // sequence after the tile — map elements first (within a voxel the map precedes the scan; cropped map points that
  // map_idx saturated into this voxel among them, summed only when kept), then set elements (all kept)
  const unsigned long long next_key = s_key[cnt + 1];
  int nout = 0;
  // the new map's keys are strictly increasing when every centroid lies in its run's voxel; on an index overflow the
  // map leaves voxel order altogether (both: the next update takes the full sort)
  bool bad = V.ovf;
  float4 ov[PER];      // this thread's outputs: centroid (or, on overflow, the source index in ov.x's bits)
  int cross_u = -1;     // which of them continues past the tile (summed so far into s_cross*)
  __shared__ float s_cross[4];
  __shared__ int s_cross_n, s_cross_local;
  __shared__ unsigned long long s_cross_key;
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    ov[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int k = t * PER + u;
    if (k >= cnt || s_key[k + 1] == s_key[k]) continue;
    const unsigned long long key = s_key[k + 1];
    int e = k + 1;
    while (e < cnt && s_key[e + 1] == key) ++e;
    const bool crosses = e == cnt && next_key == key;
    if (V.ovf) {   // index overflow: every point is returned unchanged (Q9; identity keys: runs of one)
      put_out(ov, nout, make_float4(__int_as_float(s_src[k]), 0.f, 0.f, 0.f));
      continue;
    }
    float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
    int n = 0;
    for (int j = k; j < e; ++j) {   // sequential sum in merged (= the reference's stable) order, kept points only
      if (!s_live[j]) continue;
      const float4 p = s_pt[j];
      if (n == 0) { c0 = p.x; c1 = p.y; c2 = p.z; c3 = p.w; }
      else { c0 += p.x; c1 += p.y; c2 += p.z; c3 += p.w; }
      ++n;
    }
    if (crosses) {   // finished cooperatively below (output only if a kept point is found)
      s_cross[0] = c0; s_cross[1] = c1; s_cross[2] = c2; s_cross[3] = c3;
      s_cross_n = n;
      s_cross_key = key;
      s_has_cross = 1;
      cross_u = nout;
      continue;
    }
    if (n == 0) continue;   // only cropped map points
    const float cn = (float)n;
    put_out(ov, nout, make_float4(c0 / cn, c1 / cn, c2 / cn, c3 / cn));
    if (mv_idx(V, c0 / cn, c1 / cn, c2 / cn) != (key & 0x7FFFFFFFull)) bad = true;
  }
  __syncthreads();
  if (s_has_cross) {   // block-uniform: the crossing run's continuation, chunk by chunk
    const unsigned long long key = s_cross_key;
    __shared__ int s_done;
    __shared__ float4 s_cp[kTB];
    __shared__ unsigned char s_cl[kTB];
    // part 0: map elements i1m.. with the run's index (a prefix of each chunk: map indices never decrease); part 1:
    // set elements j1.. (likewise a prefix)
    for (int part = 0; part < 2; ++part) {
      int jn = part ? j1 : i1m;
      const int jend = part ? (V.full ? L : V.nset) : V.n0;
      for (;;) {
        const int j = jn + t;
        bool in = false, live = false;
        float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
        if (j < jend) {
          float4 pq = make_float4(0.f, 0.f, 0.f, 0.f);
          if (part == 0) {
            in = map_idx(V, j) == key;
            if (in) live = mv_fetch4(V, j, pq);
          } else {
            in = (V.full ? (unsigned long long)skeys[V.base + j] : set_idx(V, j)) == key;
            if (in) {
              mv_fetch4(V, svals[V.base + j], pq);
              live = true;
            }
          }
          if (live) q = pq;
        }
        s_cp[t] = q;
        s_cl[t] = live ? 1 : 0;
        const int nin = __syncthreads_count(in);   // the run is a prefix of the chunk
        if (t == 0) {
          float c0 = s_cross[0], c1 = s_cross[1], c2 = s_cross[2], c3 = s_cross[3];
          int n = s_cross_n;
          for (int r = 0; r < nin; ++r) {
            if (!s_cl[r]) continue;
            const float4 p = s_cp[r];
            if (n == 0) { c0 = p.x; c1 = p.y; c2 = p.z; c3 = p.w; }
            else { c0 += p.x; c1 += p.y; c2 += p.z; c3 += p.w; }
            ++n;
          }
          s_cross[0] = c0; s_cross[1] = c1; s_cross[2] = c2; s_cross[3] = c3;
          s_cross_n = n;
          s_done = nin < kTB;
        }
        __syncthreads();
        jn += nin;
        if (s_done) break;
      }
    }
    if (cross_u >= 0) {
      if (s_cross_n > 0) ++nout;   // (cross_u == the old nout: the crossing run is this thread's last)
      else cross_u = -1;            // only cropped map points: no output (as a run inside a tile)
    }
  }
  const unsigned long long T3 = mm_now(stamps);
  if (t == 0) s_cross_local = -1;
  // the tile's output order: block exclusive scan of the per-thread counts
  __shared__ int s_w[kTB / 64];
  const int lane = t & 63, w = t >> 6;
  int inc = nout;
  inc = wave_incl_scan(inc);   // (DPP, floam_common.hpp)
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  int wb = 0, nloc = 0;
#pragma unroll
  for (int k = 0; k < kTB / 64; ++k) {
    if (k < w) wb += s_w[k];
    nloc += s_w[k];
  }
  const int lbase = wb + inc - nout;   // this thread's first output in the tile
  if (cross_u >= 0) s_cross_local = lbase + cross_u;
  __syncthreads();
  // stage the outputs in tile order (s_pt, s_src are free now) and their cell keys (s_key)
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    if (u >= nout || u == cross_u) continue;
    s_pt[lbase + u] = ov[u];
  }
  if (t == 0 && s_cross_local >= 0) {
    const float cn = (float)s_cross_n;
    const float4 c = make_float4(s_cross[0] / cn, s_cross[1] / cn, s_cross[2] / cn, s_cross[3] / cn);
    s_pt[s_cross_local] = c;
    if (mv_idx(V, c.x, c.y, c.z) != (s_cross_key & 0x7FFFFFFFull)) bad = true;
  }
  __syncthreads();
  for (int k = t; k < nloc; k += kTB) {
    const float4 c = s_pt[k];
    float x = c.x, y = c.y, z = c.z;
    if (V.ovf) {
      float4 q;
      mv_fetch4(V, __float_as_int(c.x), q);
      x = q.x; y = q.y; z = q.z;
    }
    bool ok;
    s_key[k] = mm_cell_key(x, y, z, V.J.inv, ok);
    bad = bad || !ok;
  }
  const Prefix2 pre = lookback_prefix(mstatus + (size_t)job * tiles_cap, tile, Prefix2{nloc, 0});
  if (pre.a < 0) {   // lookback timed out (never expected)
    if (t == 0) *V.J.d_out = -1;
    return;
  }
  const unsigned long long T4 = mm_now(stamps);
  if (violate_mod > 0 && seq % (unsigned)violate_mod == 0) bad = true;   // (test knob: exercise the fallback)
  if (__syncthreads_or(bad) && t == 0) V.K.meta_out->violation = seq;
#pragma unroll
  for (int r = 0; r < PER; ++r) {   // (nloc <= (PER * kTB): every output in one of the PER rounds)
    const int k = r * kTB + t;
    if (k < nloc) {
      const float4 c = s_pt[k];
      float4 lo, hi;   // (the record as two halves: no PointRec temporary)
      if (V.ovf) {
        vox_fetch_halves(V.J, V.n0, V.n1, __float_as_int(c.x), lo, hi);
      } else {   // VoxelGrid's output record of a centroid: x, y, z, 1 | intensity, ring 0, time 0, 0
        lo = make_float4(c.x, c.y, c.z, 1.0f);
        hi = make_float4(c.w, 0.0f, 0.0f, 0.0f);
      }
      float4* o = reinterpret_cast<float4*>(V.J.out + pre.a + k);
      o[0] = lo;
      o[1] = hi;
      V.K.out[pre.a + k] = s_key[k];
    }
  }
  if (stamps && tile < kMmStampTiles) {   // plain per-tile records
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      unsigned* q = g_mm_st[job][tile];
      q[0] = (unsigned)T0; q[1] = (unsigned)(T1 ? T1 - T0 : 0ull); q[2] = (unsigned)(T2 - (T1 ? T1 : T0));
      q[3] = (unsigned)(T3 - T2); q[4] = (unsigned)(T4 - T3); q[5] = (unsigned)(mm_now(1) - T4);
    }
  }
  if (tile == ntiles - 1 && t == 0) {
    const bool sort_failed = radix_ctl[kRadixErrorWord] != 0u;   // a sort lookback timed out (never expected)
    *V.J.d_out = sort_failed ? -1 : pre.a + nloc;
    V.K.meta_out->valid = 1;
    V.K.meta_out->seq = seq;
  }
}

template <int PER>
__global__ __launch_bounds__(kTB) void mm_merge(VoxelJobDev A, VoxelJobDev B, MapKeys KA, MapKeys KB,
                                                const uint32_t* __restrict__ skeys, const int* __restrict__ svals,
                                                int* __restrict__ ctl, unsigned long long* __restrict__ mstatus,
                                                int tiles_cap, int tilesA,
                                                const unsigned* __restrict__ radix_ctl, const int* __restrict__ gate,
                                                unsigned seq, int violate_mod, int stamps) {
  if ((int)blockIdx.x < tilesA)   // (block-uniform)
    mm_merge_job<PER>(A, KA, 0, skeys, svals, ctl, mstatus, tiles_cap, tilesA, radix_ctl, gate, seq, violate_mod,
                      stamps);
  else
    mm_merge_job<PER>(B, KB, 1, skeys, svals, ctl, mstatus, tiles_cap, tilesA, radix_ctl, gate, seq, violate_mod,
                      stamps);
}

}  // namespace

void MapMergeScratch::reserve(int tiles_per_job, hipStream_t st) {
  ctl.reserve(kMergeCtlWords);
  if (!flags.p) {
    flags.reserve(2);
    FLOAM_HIP(hipMemsetAsync(flags.p, 0, sizeof(unsigned) * 2, st));   // seq 0 is never an update's serial
  }
  if (tiles_per_job > tiles_cap) {
    const int cap = std::max(tiles_per_job + tiles_per_job / 4 + 4, 256);
    status.release();
    status.reserve((size_t)2 * cap);
    tiles_cap = cap;
  }
}

MergeCheck merge_check(MapMergeScratch& ms, unsigned seq) {
  MergeCheck mc;
  mc.flags = ms.flags.p;
  mc.ctl = ms.ctl.p;
  mc.seq = seq;
  return mc;
}

void mm_stamps_print() {
  if (!FLOAM_DIAG_ENV("FLOAM_MM_STAMPS")) return;
  static unsigned q[2][kMmStampTiles][6];
  FLOAM_HIP(hipDeviceSynchronize());
  FLOAM_HIP(hipMemcpyFromSymbol(q, HIP_SYMBOL(g_mm_st), sizeof(q)));
  // (tiles beyond the last merge's count keep older records: only those started within 200 us of the latest start)
  unsigned tmax = 0;
  for (int j = 0; j < 2; ++j)
    for (int t = 0; t < kMmStampTiles; ++t)
      if (q[j][t][0] && (int)(q[j][t][0] - tmax) > 0) tmax = q[j][t][0];
  const unsigned t00 = tmax - 20000u;
  int nt = 0, smin = 1 << 30, smax = 0, emax = 0;
  double ph[5] = {0, 0, 0, 0, 0}, mx[5] = {0, 0, 0, 0, 0};
  for (int j = 0; j < 2; ++j)
    for (int t = 0; t < kMmStampTiles; ++t) {
      const unsigned* r = q[j][t];
      if (r[0] == 0 || (int)(r[0] - t00) < 0) continue;
      ++nt;
      int len = 0;
      for (int k = 0; k < 5; ++k) {
        ph[k] += r[1 + k];
        mx[k] = std::max(mx[k], (double)r[1 + k]);
        len += (int)r[1 + k];
      }
      const int st = (int)(r[0] - t00);
      smin = std::min(smin, st);
      smax = std::max(smax, st);
      emax = std::max(emax, st + len);
    }
  if (!nt) return;
  std::fprintf(stderr, "[mm stamps] last merge, %d tiles: split %.2f (max %.2f), LDS merge %.2f (max %.2f), runs %.2f "
               "(max %.2f), lookback %.2f (max %.2f), stores %.2f (max %.2f) us; tile starts spread %.2f us; first start "
               "-> last end %.2f us\n", nt, ph[0] / nt / 100.0, mx[0] / 100.0, ph[1] / nt / 100.0, mx[1] / 100.0,
               ph[2] / nt / 100.0, mx[2] / 100.0, ph[3] / nt / 100.0, mx[3] / 100.0, ph[4] / nt / 100.0, mx[4] / 100.0,
               (smax - smin) / 100.0, (emax - smin) / 100.0);
}

void map_merge_launch(VoxelScratch2& vs, MapMergeScratch& ms, const VoxelJob& a, const VoxelJob& b, const MapKeys& ka,
                      const MapKeys& kb, const int* gate, unsigned seq, bool force_full, int violate_mod,
                      hipStream_t st) {
  const VoxelJobDev A = to_dev(a, 0);
  const VoxelJobDev B = to_dev(b, a.n0_ub + a.n1_ub);
  const int nA = a.n0_ub + a.n1_ub, nB = b.n0_ub + b.n1_ub, n = std::max(nA + nB, 1);
  // (diagnostic, FLOAM_MM_PER=2: 512-element tiles — twice the tile edges for the tests' runs to cross)
  static const int per = FLOAM_DIAG_ENV("FLOAM_MM_PER") && std::atoi(FLOAM_DIAG_ENV("FLOAM_MM_PER")) == 2 ? 2 : kMergePer;
  const int tile = kTB * per;
  const int tilesA = std::max(1, (int)div_up(std::max(nA, 1), tile));
  const int tilesB = std::max(1, (int)div_up(std::max(nB, 1), tile));
  ms.reserve(std::max(tilesA, tilesB), st);
  vs.s.reserve(n);
  vs.partials.reserve(2 * kVoxMinMaxBlocks * 6);
  vs.overflow.reserve(3);
  vs.rs.reserve(n, st);
  // the sort set is the scan's points on the merge path: a grid for them (a full-sort update loops over more)
  const int nset_ub = std::max(a.n1_ub, b.n1_ub);
  // the bucket sort once its splitters are seeded (bucket.hip); the first sort takes the digit passes and seeds them
  const bool bucket = bucket_sort_enabled(1), use_bucket = bucket && ms.bs.seeded;
  BucketDev bd{};
  if (bucket) bd = bucket_dev(ms.bs, n, st);
  // the bucket append: one chunk of kTB x kAppendR elements per block (a full-sort update loops over more); the digit
  // histograms: few blocks (one global atomic per non-zero bin and block)
  const unsigned kblocks = use_bucket ? std::max(1u, std::min(div_up(std::max(nset_ub, 1), kTB * kAppendR), 512u))
                                      : std::max(1u, std::min(div_up(std::max(nset_ub, 1), 4 * kTB), 64u));
  hipLaunchKernelGGL(mm_keys, dim3(kblocks, 2), dim3(kTB), 0, st, A, B, vs.partials.p, vs.s.k0.p, vs.s.v0.p,
                     ms.status.p, 2 * ms.tiles_cap, vs.rs.ctl.p, gate, vs.overflow.p + 2, ms.ctl.p, ka.meta_in,
                     kb.meta_in, ms.flags.p, seq, force_full ? 1 : 0, bd);
  FLOAM_LAUNCH_CHECK();
  if (use_bucket) {
    bucket_sort_launch(ms.bs, vs.rs, vs.s.k0.p, vs.s.v0.p, vs.s.k1.p, vs.s.v1.p, n, st, gate);
  } else {
    radix_sort_launch(vs.rs, vs.s.k0.p, vs.s.v0.p, vs.s.k1.p, vs.s.v1.p, n, st, gate, vs.overflow.p + 2);
    if (bucket) bucket_seed_launch(ms.bs, vs.s.k0.p, vs.overflow.p + 2, n, st, gate);
  }
  const bool wb = prof_wb_enabled();   // (diagnostic: the merge's own write bytes, profwb.hpp)
  static const int stamps = FLOAM_DIAG_ENV("FLOAM_MM_STAMPS") ? 1 : 0;
  if (wb) prof_l2_writeback(st);
#ifdef FLOAM_DIAG
  if (per == 2)
    hipLaunchKernelGGL(mm_merge<2>, dim3(tilesA + tilesB), dim3(kTB), 0, st, A, B, ka, kb, vs.s.k0.p, vs.s.v0.p,
                       ms.ctl.p, ms.status.p, ms.tiles_cap, tilesA, vs.rs.ctl.p, gate, seq, violate_mod, stamps);
  else
#endif
  hipLaunchKernelGGL(mm_merge<kMergePer>, dim3(tilesA + tilesB), dim3(kTB), 0, st, A, B, ka, kb, vs.s.k0.p, vs.s.v0.p,
                       ms.ctl.p, ms.status.p, ms.tiles_cap, tilesA, vs.rs.ctl.p, gate, seq, violate_mod,
                       stamps);
  FLOAM_LAUNCH_CHECK();
  if (wb) prof_l2_writeback(st);
}

}  // namespace floam
