// Batched pcl::VoxelGrid (+ the map-side half of addPointsToMap) — see voxel.hip.
#pragma once
#include <cfloat>
#include <climits>

#include "bucket.hpp"
#include "cloud_ops.hpp"
#include "floam_common.hpp"
#include "radix.hpp"

namespace floam {

// One cloud: the concatenation [part0 ; part1] (part1 optional).  With pose != null (device pointer to
// {qx,qy,qz,qw,tx,ty,tz}) part1 is transformed into the map frame (pointAssociateToMap) and both parts are cropped
// to t +- 100 (CropBox) before the voxel grid: addPointsToMap (src/odomEstimationClass.cpp:253-294).
// out must hold n0_ub + n1_ub points and must not alias part0 / part1.
struct VoxelJob {
  const PointRec* part0 = nullptr;
  const int* d_n0 = nullptr;
  int n0_ub = 0;
  const PointRec* part1 = nullptr;
  const int* d_n1 = nullptr;
  int n1_ub = 0;
  const double* pose = nullptr;
  float leaf = 1.0f;
  PointRec* out = nullptr;
  int* d_out = nullptr;
};

// ---- device side of the pipeline, shared with kernels that produce a voxel grid's input (stage fusion)

// the device view of a VoxelJob (base: first element of this cloud in the combined key array)
struct VoxelJobDev {
  const PointRec* part0;
  const int* d_n0;
  int n0_ub;
  const PointRec* part1;
  const int* d_n1;
  int n1_ub;
  const double* pose;   // non-null: part1 -> map frame, CropBox(t +- 100) over both parts
  float inv;
  PointRec* out;
  int* d_out;
  int base;             // first element of this cloud in the combined key array
};

// element i of the (virtual) concatenation; false if it does not exist or is cropped away
__device__ __forceinline__ bool vox_fetch(const VoxelJobDev& J, int n0, int n1, int i, PointRec& p) {
  if (i < n0) {
    p = J.part0[i];
  } else if (i < n0 + n1) {
    const PointRec s = J.part1[i - n0];
    if (J.pose) {   // pointAssociateToMap (:126-135) into an XYZI record
      float x, y, z;
      associate_to_map(J.pose, s.x, s.y, s.z, x, y, z);
      p.x = x; p.y = y; p.z = z; p.pad0 = 1.0f;
      p.intensity = s.intensity;
      p.ring = 0; p.pad1 = 0; p.time = 0.0f; p.pad2 = 0.0f;
    } else {
      p = s;
    }
  } else {
    return false;
  }
  if (J.pose) {   // CropBox min/max = Vector4f(t -+ 100) (double -> float), inclusive (:270-287)
    const double* t = J.pose + 4;
    const float mnx = (float)(t[0] - 100), mny = (float)(t[1] - 100), mnz = (float)(t[2] - 100);
    const float mxx = (float)(t[0] + 100), mxy = (float)(t[1] + 100), mxz = (float)(t[2] + 100);
    if (p.x < mnx || p.y < mny || p.z < mnz || p.x > mxx || p.y > mxy || p.z > mxz) return false;
  }
  return true;
}

// The same element as two 16-B halves — lo = {x, y, z, pad0}, hi = {intensity, ring | pad1, time, pad2} — without a
// PointRec temporary (a struct with 16-bit fields copied along conditional paths stays a private array in some
// kernels: mm_merge's scratch).  xyzi only: vox_fetch4.
__device__ __forceinline__ bool vox_fetch_halves(const VoxelJobDev& J, int n0, int n1, int i, float4& lo, float4& hi) {
  const PointRec* src;
  bool to_map = false;
  if (i < n0) {
    src = J.part0 + i;
  } else if (i < n0 + n1) {
    src = J.part1 + (i - n0);
    to_map = J.pose != nullptr;
  } else {
    return false;
  }
  const float4* q = reinterpret_cast<const float4*>(src);
  lo = q[0];
  hi = q[1];
  if (to_map) {   // pointAssociateToMap (:126-135) into an XYZI record
    float x, y, z;
    associate_to_map(J.pose, lo.x, lo.y, lo.z, x, y, z);
    lo = make_float4(x, y, z, 1.0f);
    hi = make_float4(hi.x, 0.0f, 0.0f, 0.0f);   // intensity; ring = pad1 = 0 (bits), time = pad2 = 0
  }
  if (J.pose) {   // CropBox min/max = Vector4f(t -+ 100) (double -> float), inclusive (:270-287)
    const double* t = J.pose + 4;
    const float mnx = (float)(t[0] - 100), mny = (float)(t[1] - 100), mnz = (float)(t[2] - 100);
    const float mxx = (float)(t[0] + 100), mxy = (float)(t[1] + 100), mxz = (float)(t[2] + 100);
    if (lo.x < mnx || lo.y < mny || lo.z < mnz || lo.x > mxx || lo.y > mxy || lo.z > mxz) return false;
  }
  return true;
}
__device__ __forceinline__ bool vox_fetch4(const VoxelJobDev& J, int n0, int n1, int i, float4& xyzi) {
  float4 lo, hi;
  const bool kept = vox_fetch_halves(J, n0, n1, i, lo, hi);
  xyzi = make_float4(lo.x, lo.y, lo.z, hi.x);
  return kept;
}

constexpr int kVoxMinMaxBlocks = 64;   // bounding-box partials per cloud

struct VoxelGeom {
  int min_b[3];
  int divb_mul[3];
  bool overflow;
};

// PCL 1.8.1 VoxelGrid::applyFilter index arithmetic (float leaf inverse, int min/max boxes)
__device__ __forceinline__ VoxelGeom voxel_geom(const float (&mn)[3], const float (&mx)[3], float inv) {
  VoxelGeom g;
  const long long dx = (long long)((mx[0] - mn[0]) * inv) + 1;
  const long long dy = (long long)((mx[1] - mn[1]) * inv) + 1;
  const long long dz = (long long)((mx[2] - mn[2]) * inv) + 1;
  g.overflow = (dx * dy * dz) > (long long)INT_MAX;
  int div_b[3];
  for (int d = 0; d < 3; ++d) {
    g.min_b[d] = (int)floorf(mn[d] * inv);
    const int max_b = (int)floorf(mx[d] * inv);
    div_b[d] = max_b - g.min_b[d] + 1;
  }
  g.divb_mul[0] = 1;
  g.divb_mul[1] = div_b[0];
  g.divb_mul[2] = div_b[0] * div_b[1];
  return g;
}

// the voxel index of a point inside the grid's box (vox_keys; 32 bits with the cloud in bit 31)
__device__ __forceinline__ uint32_t voxel_idx(const VoxelGeom& g, float inv, float x, float y, float z) {
  const int ijk0 = (int)(floorf(x * inv) - (float)g.min_b[0]);
  const int ijk1 = (int)(floorf(y * inv) - (float)g.min_b[1]);
  const int ijk2 = (int)(floorf(z * inv) - (float)g.min_b[2]);
  return (uint32_t)(ijk0 * g.divb_mul[0] + ijk1 * g.divb_mul[1] + ijk2 * g.divb_mul[2]);
}
__device__ __forceinline__ uint32_t voxel_idx(const VoxelGeom& g, float inv, const PointRec& p) {
  return voxel_idx(g, inv, p.x, p.y, p.z);
}

// The bounding-box stage for one cloud: min / max over the elements i = b * blockDim.x + threadIdx.x (+ k * nblocks *
// blockDim.x) that vox_fetch keeps, reduced over the block and stored as partial b of cloud `job`.  Called by every
// thread of a block; blocks b = 0 .. nblocks - 1 (nblocks = kVoxMinMaxBlocks) of each job must all run.
__device__ __forceinline__ void vox_partial_store(float (&mn)[3], float (&mx)[3], int job, int b,
                                                  float* __restrict__ partials) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      mn[d] = fminf(mn[d], __shfl_down(mn[d], o, 64));
      mx[d] = fmaxf(mx[d], __shfl_down(mx[d], o, 64));
    }
  __shared__ float s[6][16];
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int d = 0; d < 3; ++d) { s[d][w] = mn[d]; s[3 + d][w] = mx[d]; }
  __syncthreads();
  if (threadIdx.x < 6) {
    float v = s[threadIdx.x][0];
    for (int k = 1; k < nw; ++k) v = threadIdx.x < 3 ? fminf(v, s[threadIdx.x][k]) : fmaxf(v, s[threadIdx.x][k]);
    partials[(job * kVoxMinMaxBlocks + b) * 6 + threadIdx.x] = v;
  }
}

__device__ __forceinline__ void vox_minmax_block(const VoxelJobDev& J, int job, int b, int nblocks,
                                                 float* __restrict__ partials) {
  const int n0 = *J.d_n0, n1 = J.d_n1 ? *J.d_n1 : 0;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int i = b * blockDim.x + threadIdx.x; i < n0 + n1; i += nblocks * blockDim.x) {
    PointRec p;
    if (!vox_fetch(J, n0, n1, i, p)) continue;
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  }
  vox_partial_store(mn, mx, job, b, partials);
}

// The map's voxel order key: the cell (floor(z inv), floor(y inv), floor(x inv)) packed lexicographically, 21 bits a
// component (offset 2^20).  For points inside a VoxelGrid's bounding box this orders exactly as PCL's
// idx = i + j dx + k dx dy (ijk = floor(p inv) - min_b: a translation), whatever min_b is.  ok = false for
// non-finite coordinates or cells beyond +-2^20 (the merge then falls back to the full sort).
__device__ __forceinline__ unsigned long long mm_cell_key(float x, float y, float z, float inv, bool& ok) {
  const float fx = floorf(x * inv), fy = floorf(y * inv), fz = floorf(z * inv);
  constexpr float kLim = 1048575.0f;   // 2^20 - 1
  ok = fabsf(fx) <= kLim && fabsf(fy) <= kLim && fabsf(fz) <= kLim;   // (false for NaN)
  if (!ok) return ~0ull;
  const unsigned long long cx = (unsigned long long)((int)fx + (1 << 20));
  const unsigned long long cy = (unsigned long long)((int)fy + (1 << 20));
  const unsigned long long cz = (unsigned long long)((int)fz + (1 << 20));
  return (cz << 42) | (cy << 21) | cx;
}

// What the map update's bounding-box stage (run inside the status gather) checks for the merge: a non-finite scan
// point (part1) of job j stores `seq` into flags[j] (the update then takes the full sort; the map's own points are
// covered by its stored cell keys, mapmerge.hip).  ctl: the merge's per-update words, zeroed by the same launch.
struct MergeCheck {
  unsigned* flags = nullptr;   // [2]
  int* ctl = nullptr;          // [kMergeCtlWords]
  unsigned seq = 0;
};
// [0, 1] kept set elements of job A / B, [2, 3] mode (1 full), [4, 5] overflow, [6 + 6j .. 11 + 6j] job j's min_b[3],
// div_b[3]
// ... [32], [64]: mm_merge's tile tickets per job, each on a 128-B line of its own (every block reads [0, 18) at its
// start: beside the tickets' atomics those reads would queue behind them — +7 us per merge, r04i)
constexpr int kMergeCtlWords = 96;
constexpr int kMergeTicketWord = 32;   // + 32 * job

// bounding box of one cloud (as vox_minmax_block) + the MergeCheck test of its scan points
__device__ __forceinline__ void mm_minmax_block(const VoxelJobDev& J, int job, int b, int nblocks,
                                                float* __restrict__ partials, const MergeCheck& mc) {
  const int n0 = *J.d_n0, n1 = J.d_n1 ? *J.d_n1 : 0;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  bool bad = false;
  for (int i = b * blockDim.x + threadIdx.x; i < n0 + n1; i += nblocks * blockDim.x) {
    PointRec p;
    const bool kept = vox_fetch(J, n0, n1, i, p);
    if (i >= n0 && !(isfinite(p.x) && isfinite(p.y) && isfinite(p.z))) bad = true;   // (cropped ones too)
    if (!kept) continue;
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) mc.flags[job] = mc.seq;
  vox_partial_store(mn, mx, job, b, partials);
}

// What a producer kernel needs to run the bounding-box stage of a voxel2_launch issued after it (minmax_done):
// both clouds' device jobs, the partials, and the sort's control words, which block (0, 0) zeroes
// (radix_ctl_zero) once its previous sort is complete in stream order.
struct VoxelFused {
  VoxelJobDev A, B;
  float* partials;
  unsigned* ctl;
  MergeCheck mc;   // the map update (mapmerge.hpp): the merge's checks run in the same stage (mc.flags != null)
};

struct VoxelScratch2 {
  SortScratch s;
  DevBuf<float> partials;
  DevBuf<int> overflow;
  DevBuf<unsigned long long> status;
  DevBuf<unsigned> ticket;
  RadixScratch rs;
  BucketScratch bs;   // the bucket sort (bucket.hip), the default; FLOAM_SORT=radix: the four digit passes of rs
};

// dy and dz of a VoxelGrid's box (dx = divb_mul[1]) from its geometry and the box's max z
__device__ __forceinline__ void voxel_dims(const VoxelGeom& g, float mx_z, float inv, long long& dx, long long& dy,
                                           long long& dz) {
  dx = g.divb_mul[1];
  dy = g.divb_mul[1] ? g.divb_mul[2] / g.divb_mul[1] : 0;
  dz = (long long)floorf(mx_z * inv) - g.min_b[2] + 1;
}

// The key producer's bucket stage (bucket.hip), called by every thread of a block whose cloud is `job`: the grid's
// splitters into s_spl (LDS, 256; sp_t = bucket_split_prefetch(bd.split) from the prologue), the grid for the next splitters (block 0 of the job).  Returns whether the
// bucket sort runs (else the producer builds digit histograms for the radix passes).
__device__ __forceinline__ bool vox_bucket_begin(const BucketDev& bd, unsigned long long sp_t, int job,
                                                 const VoxelGeom& g, float mx_z, float inv, uint32_t* s_spl) {
  long long dx, dy, dz;
  voxel_dims(g, mx_z, inv, dx, dy, dz);
  if (bd.geo && blockIdx.x == 0 && threadIdx.x == 0) bucket_geo_store(bd.geo, job, g.min_b, (int)dx, (int)dy, g.overflow);
  if (!bd.split) return false;
  bucket_keys_lds(bd.split, sp_t, job, g.min_b, dx, dy, dz, g.overflow, s_spl);
  return true;
}

// Two independent voxel grids in one pipeline (3 kernels + the 4 radix passes).  *d_out of each job receives the
// voxel count (-1 if the single-pass compaction failed, never expected).  gate (device int, nullable): when it reads
// 0 the pipeline does nothing but copy each job's part0 to its output (a map update skipped on the device).
// minmax_done: a producer kernel already ran the bounding-box stage with voxel2_prepare's VoxelFused (same jobs).
// FLOAM_VOX_STAMPS=1: print vox_compact's in-kernel phase times (diagnostic; synchronises the device)
void vox_stamps_print();

// The sort + compaction half of the pipeline with the bucket sort (bucket.hip): plan, bucket scatter, and one block
// per bucket that sorts it and emits its voxels (output slots by lookback over the 256 buckets: status must hold >= 256
// zeroed words, ticket a zeroed counter: vox_keys zeroes both).  k0 / v0 hold the keys from vox_keys (with the
// bucket histogram); the outputs land in A.out / B.out.
void bucket_voxel_launch(BucketScratch& bs, RadixScratch& rs, const VoxelJobDev& A, const VoxelJobDev& B, uint32_t* k0,
                         int* v0, uint32_t* k1, int* v1, int n, const int* overflow, unsigned long long* status,
                         unsigned* ticket, hipStream_t st, const int* gate, const int* n_dev);

void voxel2_launch(VoxelScratch2& sc, const VoxelJob& a, const VoxelJob& b, hipStream_t st,
                   const int* gate = nullptr, bool minmax_done = false);
// reserves the scratch of a voxel2_launch of the same jobs and returns the producer's view of it
VoxelFused voxel2_prepare(VoxelScratch2& sc, const VoxelJob& a, const VoxelJob& b, hipStream_t st);
VoxelJobDev to_dev(const VoxelJob& j, int base);

}  // namespace floam
