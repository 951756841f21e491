// pcl::VoxelGrid (PCL 1.8.1 semantics) for two independent clouds per call, optionally fused with the map-side
// half of addPointsToMap (transform + concatenation + CropBox).
//
// Reference call sites: src/odomEstimationClass.cpp:137-142 (downSamplingToMap: edge leaf r, surf leaf 2r, both in
// one updatePointsToMap call) and :253-294 (addPointsToMap: transform the downsampled scan into the map frame,
// append it to the map, CropBox [t-100, t+100], VoxelGrid — for the corner and the surf map).
//
// PCL's VoxelGrid: min/max over the input, leaf index ijk = floor(p * inv) - min_b (float), idx = i + j*dx + k*dx*dy,
// input returned unchanged if dx*dy*dz > INT_MAX, std::sort of (idx, point) pairs, one centroid (float sums of
// x, y, z, intensity in sorted order / float(count)) per voxel in ascending idx.  Here the within-voxel order is
// the stable (input) order; PCL's unstable std::sort can only change a centroid's float summation order.
//
// Launches per call (both clouds): vox_minmax (block partials), vox_keys (reduce partials -> 32-bit keys with the
// cloud in bit 31, dropped points -> 0xFFFFFFFF, + the sort's digit histograms), the four single-pass digit launches
// of a stable radix sort (radix.hip), vox_compact (run heads + single-pass decoupled-lookback positions for both
// clouds at once + centroids).
#include <cfloat>
#include <climits>

#include "cloud_ops.hpp"
#include "lookback.hpp"
#include "radix.hpp"
#include "voxel.hpp"

namespace floam {

// FLOAM_VOX_STAMPS=1 (diagnostic): vox_compact's per-tile phase times of the last launch over >= 32 tiles (10-ns
// ticks): [0] start (low bits), [1] keys staged, [2] points gathered + heads, [3] lookback done, [4] end (drained),
// [5] the longest run with its head in the tile
__device__ unsigned g_vox_st[1024][6];

namespace {
constexpr int kTB = 256;
constexpr int kMinMaxBlocks = kVoxMinMaxBlocks;   // partials per cloud
constexpr int kPerThread = 4;
constexpr int kTile = kTB * kPerThread;   // elements per compaction tile

__global__ __launch_bounds__(kTB) void vox_minmax(VoxelJobDev A, VoxelJobDev B, float* __restrict__ partials,
                                                  unsigned* __restrict__ radix_ctl, const int* __restrict__ gate) {
  if (gate && !*gate) return;
  if (blockIdx.x == 0 && blockIdx.y == 0) radix_ctl_zero(radix_ctl, threadIdx.x, blockDim.x);   // for vox_keys
  vox_minmax_block(blockIdx.y == 0 ? A : B, (int)blockIdx.y, (int)blockIdx.x, (int)gridDim.x, partials);
}

__global__ __launch_bounds__(kTB) void vox_keys(VoxelJobDev A, VoxelJobDev B, const float* __restrict__ partials,
                                                uint32_t* __restrict__ keys, int* __restrict__ vals,
                                                int* __restrict__ overflow, unsigned long long* __restrict__ status,
                                                int ntiles, unsigned* __restrict__ ticket,
                                                unsigned* __restrict__ radix_ctl, const int* __restrict__ gate,
                                                int* __restrict__ n_dev, BucketDev bd) {
  // the prologue's loads are issued together (one round trip instead of three in a row): the gate, the partials,
  // the counts, this thread's first record of the first part (inside the array by the host bound n0_ub) and its splitter
  const int job = blockIdx.y;
  const VoxelJobDev& J = job == 0 ? A : B;
  const int gv = gate ? *gate : 1;
  const int dA0 = *A.d_n0, dA1 = A.d_n1 ? *A.d_n1 : 0, dB0 = *B.d_n0, dB1 = B.d_n1 ? *B.d_n1 : 0;
  const int c = threadIdx.x >> 5, l = threadIdx.x & 31;   // component c = t / 32 (two per wave), 32 lanes
  float pv[kMinMaxBlocks / 32];
#pragma unroll
  for (int u = 0; u < kMinMaxBlocks / 32; ++u)
    pv[u] = threadIdx.x < 6 * 32 ? partials[(job * kMinMaxBlocks + l + 32 * u) * 6 + c] : 0.f;
  // the first element of this thread: a chunk of kTB x kAppendR per block with the bucket append, else a grid stride
  const int i0 = blockIdx.x * blockDim.x * (bd.split ? kAppendR : 1) + threadIdx.x;
  // (the bucket append: the kAppendR first-part records of this thread's first chunk, element i0 + r kTB)
  float4 p0[kAppendR];
#pragma unroll
  for (int r = 0; r < kAppendR; ++r) {
    const int i = i0 + r * kTB;
    p0[r] = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((r == 0 || bd.split) && i < J.n0_ub) p0[r] = *reinterpret_cast<const float4*>(&J.part0[i].x);
  }
  const unsigned long long sp_t = bucket_split_prefetch(bd.split);   // (the splitters, bucket_keys_lds)
  if (!gv) return;
  __shared__ float s_mm[6];
  __shared__ unsigned s_hist[kRadixHistWords];
  // bd.split: the bucket append's per-bucket words in s_hist (bucket_append), else the four digit histograms
  radix_hist_begin(s_hist);
  if (threadIdx.x < 6 * 32) {   // the partials' min / max per component: 32 lanes, then a 32-lane reduction
    const bool is_min = c < 3;
    float v = is_min ? FLT_MAX : -FLT_MAX;
#pragma unroll
    for (int u = 0; u < kMinMaxBlocks / 32; ++u) v = is_min ? fminf(v, pv[u]) : fmaxf(v, pv[u]);
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      const float w = __shfl_xor(v, o, 64);
      v = is_min ? fminf(v, w) : fmaxf(v, w);
    }
    if (l == 0) s_mm[c] = v;
  }
  // lookback state of the compaction launch that follows this one
  for (int t = (job * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x; t < ntiles; t += 2 * gridDim.x * blockDim.x)
    status[t] = 0ull;
  if (job == 0 && blockIdx.x == 0 && threadIdx.x == 0) *ticket = 0u;
  __syncthreads();
  const float mn[3] = {s_mm[0], s_mm[1], s_mm[2]}, mx[3] = {s_mm[3], s_mm[4], s_mm[5]};
  const VoxelGeom g = voxel_geom(mn, mx, J.inv);
  if (blockIdx.x == 0 && threadIdx.x == 0) overflow[job] = g.overflow ? 1 : 0;
  // the elements the device holds, packed: cloud A at [0, nA), cloud B at [nA, nA + nB) (no upper-bound padding)
  const int nA0 = min(dA0, A.n0_ub), nA1 = A.d_n1 ? min(dA1, A.n1_ub) : 0;
  const int nB0 = min(dB0, B.n0_ub), nB1 = B.d_n1 ? min(dB1, B.n1_ub) : 0;
  const int n0 = job ? nB0 : nA0, n1 = job ? nB1 : nA1;
  const int base = job ? nA0 + nA1 : 0;
  if (job == 0 && blockIdx.x == 0 && threadIdx.x == 0) *n_dev = nA0 + nA1 + nB0 + nB1;
  __shared__ uint32_t s_spl[kBuckets];
  const bool bucket = vox_bucket_begin(bd, sp_t, job, g, mx[2], J.inv, s_spl);
  // element i's sort key (0xFFFFFFFF: none / dropped); pre: its first-part record prefetched
  auto key_of = [&](int i, bool pre, float4 pr) {
    float4 q;   // (x, y, z, intensity: no PointRec temporary)
    bool in;
    if (pre && i < n0 && !J.pose) {   // the prefetched record (no transform, no crop: vox_fetch's first part)
      q = pr;
      in = true;
    } else {
      in = vox_fetch4(J, n0, n1, i, q);
    }
    if (!in) return 0xFFFFFFFFu;
    // index overflow: output = input unchanged (Q9): identity order, one "voxel" per point
    const uint32_t idx = g.overflow ? (uint32_t)i : voxel_idx(g, J.inv, q.x, q.y, q.z);
    return ((uint32_t)job << 31) | idx;
  };
  if (bucket) {   // appended to the buckets' regions: no keys array, no scatter pass
    for (int c0 = blockIdx.x * blockDim.x * kAppendR; c0 < n0 + n1; c0 += gridDim.x * blockDim.x * kAppendR) {
      uint32_t key[kAppendR];
      int val[kAppendR];
#pragma unroll
      for (int r = 0; r < kAppendR; ++r) {
        const int i = c0 + r * kTB + (int)threadIdx.x;
        key[r] = i < n0 + n1 ? key_of(i, i == i0 + r * kTB, p0[r]) : 0xFFFFFFFFu;
        val[r] = i;
      }
      bucket_append<kAppendR>(bd, radix_ctl, s_spl, key, val, s_hist, reinterpret_cast<int*>(s_hist + kBuckets),
                              reinterpret_cast<int*>(s_hist + 2 * kBuckets));
    }
    return;
  }
  for (int i = i0; i < n0 + n1; i += gridDim.x * blockDim.x) {
    const uint32_t key = key_of(i, i == i0, p0[0]);
    keys[base + i] = key;
    vals[base + i] = i;
    radix_hist_add(s_hist, key);
  }
  radix_hist_end(s_hist, radix_ctl);
}

// Run heads of the sorted keys -> output slot per cloud (decoupled lookback over tiles) -> centroid of the run.
__global__ __launch_bounds__(kTB) void vox_compact(VoxelJobDev A, VoxelJobDev B, const uint32_t* __restrict__ keys,
                                                   const int* __restrict__ vals, const int* __restrict__ overflow,
                                                   const int* __restrict__ n_dev, unsigned long long* __restrict__ status,
                                                   unsigned* __restrict__ ticket, const unsigned* __restrict__ radix_ctl,
                                                   const int* __restrict__ gate, int n_cap, int stamps) {
  const unsigned long long T0 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // the prologue's loads are issued together (one round trip instead of four in a row): the gate, the device
  // counts, and the tile's keys and values up to the host bound n_cap (allocated; entries past the device count are
  // masked below)
  // the tile is the block's ticket (zeroed by vox_keys): a tile only waits on tiles that are already running (HIP
  // promises no dispatch order); the tile-independent loads in flight beside the ticket
  __shared__ int s_tile;
  if (threadIdx.x == 0) s_tile = (int)atomicAdd(ticket, 1u);
  const int gv = gate ? *gate : 1;
  const int total_d = *n_dev;   // packed elements (vox_keys)
  const int nA0 = *A.d_n0, nA1 = A.d_n1 ? *A.d_n1 : 0, nB0 = *B.d_n0, nB1 = B.d_n1 ? *B.d_n1 : 0;
  const int ovf[2] = {overflow[0], overflow[1]};
  __syncthreads();
  const int tile = s_tile;
  const int t0 = tile * kTile;
  // s_key[k] = key of element t0 - 1 + k, k in [0, kTile + 1 + kHalo]: the rounds of the prologue's key loads
  // also cover kHalo elements past the tile (the continuation of a run that crosses the tile end, usually short)
  constexpr int kRounds = (kTile + 2 + kTB - 1) / kTB;
  constexpr int kHalo = kRounds * kTB - (kTile + 2);
  __shared__ uint32_t s_key[kTile + 2 + kHalo];
  uint32_t kr[kRounds];
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int k = r * kTB + threadIdx.x;
    const int i = t0 - 1 + k;
    kr[r] = (i >= 0 && i < n_cap) ? keys[i] : 0xFFFFFFFFu;
  }
  const int vh = threadIdx.x < kHalo && t0 + kTile + (int)threadIdx.x < n_cap ? vals[t0 + kTile + threadIdx.x] : 0;
  const int4* __restrict__ vals4 = reinterpret_cast<const int4*>(vals);
  const int k0 = threadIdx.x * kPerThread;
  int v[kPerThread];
  if (t0 + k0 + kPerThread <= n_cap) {
    const int4 vv = vals4[(t0 + k0) / kPerThread];
    v[0] = vv.x; v[1] = vv.y; v[2] = vv.z; v[3] = vv.w;
  } else {
#pragma unroll
    for (int u = 0; u < kPerThread; ++u) v[u] = t0 + k0 + u < n_cap ? vals[t0 + k0 + u] : 0;
  }
  if (!gv) {   // gated off (no keyframe): the output is the unchanged first part (the map)
    for (int job = 0; job < 2; ++job) {
      const VoxelJobDev& J = job == 0 ? A : B;
      const int n0 = job ? nB0 : nA0;
      for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n0; i += gridDim.x * blockDim.x) J.out[i] = J.part0[i];
      if (blockIdx.x == 0 && threadIdx.x == 0) *J.d_out = n0;
    }
    return;
  }
  const int total = total_d;
  const int ntiles = (total + kTile - 1) / kTile;
  if (tile >= ntiles) {   // beyond the device's elements (the grid is sized by the host's upper bounds)
    if (tile == 0 && threadIdx.x == 0) { *A.d_out = 0; *B.d_out = 0; }   // no elements at all
    return;
  }
#pragma unroll
  for (int r = 0; r < kRounds; ++r) {
    const int k = r * kTB + threadIdx.x;
    const int i = t0 - 1 + k;
    s_key[k] = i < total ? kr[r] : 0xFFFFFFFFu;
  }
  __syncthreads();
  const unsigned long long T1 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // run tails of the tile as a bitmask: bit k set if element t0 + k is the last of its run
  __shared__ unsigned s_tail[kTile / 32];
  {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < kTile / kTB; ++r) {
      const int k = r * kTB + threadIdx.x;
      const unsigned long long b = __ballot(s_key[k + 1] != s_key[k + 2]);
      if (lane == 0) {
        s_tail[(r * kTB + w * 64) / 32] = (unsigned)b;
        s_tail[(r * kTB + w * 64) / 32 + 1] = (unsigned)(b >> 32);
      }
    }
  }
  // gather every element's point (x, y, z, intensity) of the tile into LDS: one parallel round trip, issued
  // before the lookback wait so the two latencies overlap; the runs are then summed from LDS
  __shared__ float4 s_pt[kTile];
  {
#pragma unroll
    for (int u = 0; u < kPerThread; ++u) {
      const uint32_t key = s_key[k0 + u + 1];
      float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
      if (key != 0xFFFFFFFFu) {
        PointRec p;
        if (key >> 31) vox_fetch(B, nB0, nB1, v[u], p);
        else vox_fetch(A, nA0, nA1, v[u], p);
        q = make_float4(p.x, p.y, p.z, p.intensity);
      }
      s_pt[k0 + u] = q;
    }
  }
  // ... and the halo elements that continue the tile's last run (sorted: the elements equal to it are contiguous)
  __shared__ float4 s_halo[kHalo];
  if (threadIdx.x < kHalo) {
    const uint32_t key = s_key[kTile + 1 + threadIdx.x];   // element t0 + kTile + threadIdx.x
    if (key != 0xFFFFFFFFu && key == s_key[kTile]) {
      PointRec p;
      if (key >> 31) vox_fetch(B, nB0, nB1, vh, p);
      else vox_fetch(A, nA0, nA1, vh, p);
      s_halo[threadIdx.x] = make_float4(p.x, p.y, p.z, p.intensity);
    }
  }
  // heads in this thread's 4 consecutive elements
  int cnt[2] = {0, 0};
  unsigned headmask = 0;
#pragma unroll
  for (int u = 0; u < kPerThread; ++u) {
    const int k = threadIdx.x * kPerThread + u;   // element t0 + k, previous key at s_key[k]
    const uint32_t key = s_key[k + 1];
    if (key != 0xFFFFFFFFu && (t0 + k == 0 || key != s_key[k])) {
      headmask |= 1u << u;
      ++cnt[key >> 31];
    }
  }
  // block exclusive scan of (cnt0, cnt1)
  __shared__ int s_w[2][kTB / 64];
  int inc[2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    int v = cnt[c];
    v = wave_incl_scan(v);   // (DPP, floam_common.hpp)
    inc[c] = v;
    if (lane == 63) s_w[c][w] = v;
  }
  __syncthreads();
  int wb[2] = {0, 0}, agg[2] = {0, 0};
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int k = 0; k < kTB / 64; ++k) {
      if (k < w) wb[c] += s_w[c][k];
      agg[c] += s_w[c][k];
    }
  unsigned long long T2 = 0ull;
  if (stamps) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    T2 = __builtin_amdgcn_s_memrealtime();
  }
  const Prefix2 pre = lookback_prefix(status, tile, Prefix2{agg[0], agg[1]});
  const unsigned long long T3 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  if (pre.a < 0) {   // lookback timed out (never expected): report through the output counts
    if (threadIdx.x == 0) { *A.d_out = -1; *B.d_out = -1; }
    return;
  }
  int pos[2] = {pre.a + wb[0] + inc[0] - cnt[0], pre.b + wb[1] + inc[1] - cnt[1]};
  // the run that crosses the tile end (at most one): its head's partial sums, finished cooperatively below
  __shared__ float s_cross[4];
  __shared__ int s_cross_pos, s_cross_head, s_cross_job;
  __shared__ int s_maxrun;
  if (threadIdx.x == 0) { s_cross_head = -1; s_maxrun = 0; }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kPerThread; ++u) {
    if (!(headmask & (1u << u))) continue;
    const int k = threadIdx.x * kPerThread + u;
    const int i = t0 + k;
    const uint32_t key = s_key[k + 1];
    const int job = (int)(key >> 31);
    const VoxelJobDev& J = job == 0 ? A : B;
    if (ovf[job]) {   // input returned unchanged: the whole record
      PointRec o;
      vox_fetch(J, job ? nB0 : nA0, job ? nB1 : nA1, v[u], o);
      J.out[pos[job]++] = o;
      continue;
    }
    // run end: the next tail at or after k (bitmask search), or the tile end
    int end = kTile;
    for (int wd = k >> 5; wd < kTile / 32; ++wd) {
      unsigned m = s_tail[wd];
      if (wd == (k >> 5)) m &= ~0u << (k & 31);
      if (m) {
        end = wd * 32 + __ffs(m);   // one past the tail
        break;
      }
    }
    if (stamps) s_maxrun = max(s_maxrun, end - k);   // (diagnostic; racy max is fine)
    const float4 f = s_pt[k];
    float c0 = f.x, c1 = f.y, c2 = f.z, c3 = f.w;
    // sequential sum in sorted (= input) order; a long run (dense near-range voxels: tens to hundreds of points)
    // reads 8 points per LDS round trip, the additions staying in order
    int j = k + 1;
    for (; j + 8 <= end; j += 8) {
      float4 p[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) p[q] = s_pt[j + q];
#pragma unroll
      for (int q = 0; q < 8; ++q) { c0 += p[q].x; c1 += p[q].y; c2 += p[q].z; c3 += p[q].w; }
    }
    for (; j < end; ++j) {
      const float4 p = s_pt[j];
      c0 += p.x; c1 += p.y; c2 += p.z; c3 += p.w;
    }
    const bool crosses = end == kTile && t0 + kTile < total && s_key[kTile + 1] == key;
    if (crosses) {   // its continuation in the halo, in order (elements past the count read 0xFFFFFFFF)
      int h = 0;
      while (h < kHalo && s_key[kTile + 1 + h] == key) {
        const float4 p = s_halo[h];
        c0 += p.x; c1 += p.y; c2 += p.z; c3 += p.w;
        ++h;
      }
      if (h < kHalo) {   // it ends there
        const float cn = (float)(t0 + kTile + h - i);
        PointRec o;
        o.x = c0 / cn; o.y = c1 / cn; o.z = c2 / cn; o.pad0 = 1.0f;
        o.intensity = c3 / cn;
        o.ring = 0; o.pad1 = 0; o.time = 0.0f; o.pad2 = 0.0f;
        J.out[pos[job]++] = o;
        continue;
      }
      // longer than the halo: finished cooperatively below, from element t0 + kTile + kHalo
      s_cross[0] = c0; s_cross[1] = c1; s_cross[2] = c2; s_cross[3] = c3;
      s_cross_pos = pos[job]++;
      s_cross_head = i;
      s_cross_job = job;
      continue;
    }
    const float cn = (float)(t0 + end - i);
    PointRec o;
    o.x = c0 / cn; o.y = c1 / cn; o.z = c2 / cn; o.pad0 = 1.0f;
    o.intensity = c3 / cn;
    o.ring = 0; o.pad1 = 0; o.time = 0.0f; o.pad2 = 0.0f;
    J.out[pos[job]++] = o;
  }
  __syncthreads();
  const unsigned long long T3b = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const bool had_cross = s_cross_head >= 0;
  if (s_cross_head >= 0) {   // block-uniform: gather the run's continuation chunk by chunk, thread 0 sums in order
    const int job = s_cross_job;
    const VoxelJobDev& J = job == 0 ? A : B;
    const uint32_t key = s_key[kTile];   // the tile's last element belongs to the crossing run
    const int n0 = job ? nB0 : nA0, n1 = job ? nB1 : nA1;
    __shared__ int s_done;
    int j0 = t0 + kTile + kHalo;
    for (;;) {
      const int j = j0 + threadIdx.x;
      const bool in = j < total && keys[j] == key;
      float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
      if (in) {
        PointRec p;
        vox_fetch(J, n0, n1, vals[j], p);
        q = make_float4(p.x, p.y, p.z, p.intensity);
      }
      s_pt[threadIdx.x] = q;
      const int nin = __syncthreads_count(in);   // the run is a prefix of the chunk
      if (threadIdx.x == 0) {
        float c0 = s_cross[0], c1 = s_cross[1], c2 = s_cross[2], c3 = s_cross[3];
        for (int r = 0; r < nin; ++r) {
          const float4 p = s_pt[r];
          c0 += p.x; c1 += p.y; c2 += p.z; c3 += p.w;
        }
        s_cross[0] = c0; s_cross[1] = c1; s_cross[2] = c2; s_cross[3] = c3;
        s_done = nin < (int)blockDim.x;
      }
      __syncthreads();
      j0 += nin;
      if (s_done) break;
    }
    if (threadIdx.x == 0) {
      const float cn = (float)(j0 - s_cross_head);
      PointRec o;
      o.x = s_cross[0] / cn; o.y = s_cross[1] / cn; o.z = s_cross[2] / cn; o.pad0 = 1.0f;
      o.intensity = s_cross[3] / cn;
      o.ring = 0; o.pad1 = 0; o.time = 0.0f; o.pad2 = 0.0f;
      J.out[s_cross_pos] = o;
    }
  }
  if (tile == ntiles - 1 && threadIdx.x == 0) {
    const bool sort_failed = radix_ctl[kRadixErrorWord] != 0u;   // a sort lookback timed out (never expected)
    *A.d_out = sort_failed ? -1 : pre.a + agg[0];
    *B.d_out = sort_failed ? -1 : pre.b + agg[1];
  }
  if (stamps && ntiles >= 32 && tile < 1024) {   // plain per-tile records (no shared atomics: they would queue)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long T4 = __builtin_amdgcn_s_memrealtime();
      unsigned* q = g_vox_st[tile];
      q[0] = (unsigned)T0; q[1] = (unsigned)(T1 - T0); q[2] = (unsigned)(T2 - T1); q[3] = (unsigned)(T3 - T2);
      q[4] = (unsigned)(T4 - T3); q[5] = (unsigned)s_maxrun | (unsigned)(T3b - T3) << 16 | (had_cross ? 1u << 31 : 0u);
    }
  }
}

}  // namespace

static int vox_stamps_on() {
  static const int on = FLOAM_DIAG_ENV("FLOAM_VOX_STAMPS") ? 1 : 0;
  return on;
}

void vox_stamps_print() {
  if (!vox_stamps_on()) return;
  static unsigned q[1024][6];
  FLOAM_HIP(hipDeviceSynchronize());
  FLOAM_HIP(hipMemcpyFromSymbol(q, HIP_SYMBOL(g_vox_st), sizeof(q)));
  int nt = 0;
  double ph[4] = {0, 0, 0, 0};
  int smin = 0, emax = 0;   // relative to tile 0's start
  for (int t = 0; t < 1024; ++t) {
    if (q[t][1] == 0 && q[t][4] == 0) continue;
    ++nt;
    for (int k = 0; k < 4; ++k) ph[k] += q[t][1 + k];
    const int st = (int)(q[t][0] - q[0][0]);
    smin = std::min(smin, st);
    emax = std::max(emax, st + (int)(q[t][1] + q[t][2] + q[t][3] + q[t][4]));
  }
  const int last_end = emax - smin;
  if (!nt) return;
  std::fprintf(stderr, "[vox stamps] last launch, %d tiles: keys staged %.2f, gather + heads %.2f, lookback %.2f, "
               "sums + stores + drain %.2f us per tile; first start -> last end %.2f us\n", nt, ph[0] / nt / 100.0,
               ph[1] / nt / 100.0, ph[2] / nt / 100.0, ph[3] / nt / 100.0, last_end / 100.0);
  for (int t = 0; t < nt; t += std::max(1, nt / 8))
    std::fprintf(stderr, "[vox tile %4d] start +%.2f: %.2f %.2f %.2f %.2f us (heads %.2f us%s), longest run %u\n", t,
                 (int)(q[t][0] - q[0][0]) / 100.0, q[t][1] / 100.0, q[t][2] / 100.0, q[t][3] / 100.0, q[t][4] / 100.0,
                 ((q[t][5] >> 16) & 0x7FFF) / 100.0, (q[t][5] >> 31) ? ", deferred crossing run" : "", q[t][5] & 0xFFFF);
}

VoxelJobDev to_dev(const VoxelJob& j, int base) {
  return VoxelJobDev{j.part0, j.d_n0, j.n0_ub, j.part1, j.d_n1, j.part1 ? j.n1_ub : 0, j.pose, 1.0f / j.leaf,
                     j.out, j.d_out, base};
}

VoxelFused voxel2_prepare(VoxelScratch2& sc, const VoxelJob& a, const VoxelJob& b, hipStream_t st) {
  const int total = a.n0_ub + (a.part1 ? a.n1_ub : 0) + b.n0_ub + (b.part1 ? b.n1_ub : 0);
  sc.partials.reserve(2 * kMinMaxBlocks * 6);
  sc.rs.reserve(std::max(total, 1), st);
  return VoxelFused{to_dev(a, 0), to_dev(b, a.n0_ub + (a.part1 ? a.n1_ub : 0)), sc.partials.p, sc.rs.ctl.p};
}

void voxel2_launch(VoxelScratch2& sc, const VoxelJob& a, const VoxelJob& b, hipStream_t st, const int* gate,
                   bool minmax_done) {
  const VoxelJobDev A = to_dev(a, 0);
  const VoxelJobDev B = to_dev(b, a.n0_ub + (a.part1 ? a.n1_ub : 0));
  const int total = B.base + b.n0_ub + (b.part1 ? b.n1_ub : 0);
  if (total == 0) {   // both clouds empty
    FLOAM_HIP(hipMemsetAsync(a.d_out, 0, sizeof(int), st));
    FLOAM_HIP(hipMemsetAsync(b.d_out, 0, sizeof(int), st));
    return;
  }
  const int n = total;
  sc.s.reserve(n);
  sc.partials.reserve(2 * kMinMaxBlocks * 6);
  sc.overflow.reserve(3);   // [0, 1] index overflow per cloud, [2] packed element count
  const bool bucket = bucket_sort_enabled(0);
  const int ntiles = (int)div_up(n, kTile);
  const int nstatus = bucket ? std::max(ntiles, kBuckets) : ntiles;   // the compaction's lookback words
  sc.status.reserve(nstatus);
  sc.ticket.reserve(1);
  const int umax = std::max(A.n0_ub + A.n1_ub, b.n0_ub + (b.part1 ? b.n1_ub : 0));
  sc.rs.reserve(n, st);
  if (!minmax_done) {   // else the producer of the clouds ran the stage (voxel2_prepare)
    hipLaunchKernelGGL(vox_minmax, dim3(kMinMaxBlocks, 2), dim3(kTB), 0, st, A, B, sc.partials.p, sc.rs.ctl.p, gate);
    FLOAM_LAUNCH_CHECK();
  }
  // the bucket sort once its splitters are seeded; the first sort of the pipeline takes the digit passes and seeds them
  const bool use_bucket = bucket && sc.bs.seeded;
  BucketDev bd{};
  if (bucket) bd = bucket_dev(sc.bs, n, st);
  // the digit histograms: few blocks (each folds its LDS histograms into the global ones with one atomic per non-zero
  // bin); the bucket append: one chunk of kTB x kAppendR elements per block
  const unsigned kb = use_bucket ? std::max(1u, std::min(div_up(std::max(umax, 1), kTB * kAppendR), 1024u))
                                 : std::max(1u, std::min(div_up(std::max(umax, 1), kTB), 64u));
  hipLaunchKernelGGL(vox_keys, dim3(kb, 2), dim3(kTB), 0, st, A, B, sc.partials.p, sc.s.k0.p, sc.s.v0.p,
                     sc.overflow.p, sc.status.p, nstatus, sc.ticket.p, sc.rs.ctl.p, gate, sc.overflow.p + 2, bd);
  FLOAM_LAUNCH_CHECK();
  if (use_bucket) {   // scatter by bucket, and one block per bucket that sorts it and emits its voxels
    bucket_voxel_launch(sc.bs, sc.rs, A, B, sc.s.k0.p, sc.s.v0.p, sc.s.k1.p, sc.s.v1.p, n, sc.overflow.p,
                        sc.status.p, sc.ticket.p, st, gate, sc.overflow.p + 2);
    return;
  }
  // sorted pairs in k0 / v0; the passes and the compaction work on the packed device count
  radix_sort_launch(sc.rs, sc.s.k0.p, sc.s.v0.p, sc.s.k1.p, sc.s.v1.p, n, st, gate, sc.overflow.p + 2);
  if (bucket) bucket_seed_launch(sc.bs, sc.s.k0.p, sc.overflow.p + 2, n, st, gate);
  hipLaunchKernelGGL(vox_compact, dim3(ntiles), dim3(kTB), 0, st, A, B, sc.s.k0.p, sc.s.v0.p, sc.overflow.p,
                     sc.overflow.p + 2, sc.status.p, sc.ticket.p, sc.rs.ctl.p, gate, n, vox_stamps_on());
  FLOAM_LAUNCH_CHECK();
}

}  // namespace floam
