// Cloud operations on gfx950: PCL 1.8.1 VoxelGrid / CropBox semantics, map append, velocity deskew.
// VoxelGrid call sites: src/odomEstimationClass.cpp:13-14, 137-142, 289-292.  CropBox: :270-287.
// CompensateVelocity: src/dataHandler.cpp:82-92.
//
// VoxelGrid pipeline (all sizes device-resident; grids sized by a host upper bound):
//   minmax -> voxel keys (PCL's idx = i + j*dx + k*dx*dy over floor(p*inv) - min_b) -> stable radix sort of
//   (idx, i) -> run heads -> exclusive scan -> one thread per voxel sums x,y,z,intensity in float in sorted
//   (= original) order and divides by float(count).  PCL sorts with the unstable std::sort, whose within-voxel
//   order is unspecified; the stable order used here can differ from it only in the float summation order
//   inside a voxel (a centroid may differ in its last bit), see DESIGN.md.
#include <cfloat>
#include <climits>

#include "cloud_ops.hpp"
#include "primitives.hpp"

namespace floam {

void SortScratch::reserve(int n) {
  if ((size_t)n <= k0.cap && temp_bytes > 0) return;
  const size_t want = (size_t)n < 4096 ? 4096 : (size_t)n + (size_t)n / 4;
  k0.reserve(want); k1.reserve(want);
  v0.reserve(want); v1.reserve(want);
  flags.reserve(want); pos.reserve(want);
  const size_t tb = std::max(sort_pairs_temp_bytes((int)k0.cap), scan_temp_bytes((int)k0.cap));
  if (tb > temp.cap) temp.reserve(tb);
  temp_bytes = temp.cap;
}

namespace {
constexpr int kTB = 256;

__global__ void mm_init(int* mm) {
  if (threadIdx.x < 3) mm[threadIdx.x] = f2ord(FLT_MAX);
  else if (threadIdx.x < 6) mm[threadIdx.x] = f2ord(-FLT_MAX);
}

__global__ __launch_bounds__(kTB) void mm_reduce(const PointRec* __restrict__ in, const int* __restrict__ d_n,
                                                 int* __restrict__ mm) {
  const int n = *d_n;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float4 p = *reinterpret_cast<const float4*>(&in[i].x);
    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      mn[d] = fminf(mn[d], __shfl_down(mn[d], o, 64));
      mx[d] = fmaxf(mx[d], __shfl_down(mx[d], o, 64));
    }
  __shared__ float s[6][kTB / 64];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
    for (int d = 0; d < 3; ++d) { s[d][w] = mn[d]; s[3 + d][w] = mx[d]; }
  __syncthreads();
  if (threadIdx.x < 6) {
    float v = s[threadIdx.x][0];
    for (int k = 1; k < kTB / 64; ++k) v = threadIdx.x < 3 ? fminf(v, s[threadIdx.x][k]) : fmaxf(v, s[threadIdx.x][k]);
    if (threadIdx.x < 3) atomicMin(&mm[threadIdx.x], f2ord(v));
    else atomicMax(&mm[threadIdx.x], f2ord(v));
  }
}

struct VoxelGeom {
  int min_b[3];
  int divb_mul[3];
  bool overflow;
};

__device__ __forceinline__ VoxelGeom voxel_geom(const int* mm, float inv) {
  VoxelGeom g;
  float mn[3], mx[3];
  for (int d = 0; d < 3; ++d) { mn[d] = ord2f(mm[d]); mx[d] = ord2f(mm[3 + d]); }
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

__global__ __launch_bounds__(kTB) void vg_keys(const PointRec* __restrict__ in, const int* __restrict__ d_n, int n_ub,
                                               const int* __restrict__ mm, float inv, uint32_t* __restrict__ keys,
                                               int* __restrict__ vals) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ub) return;
  const int n = *d_n;
  uint32_t key = 0xFFFFFFFFu;
  if (i < n) {
    const VoxelGeom g = voxel_geom(mm, inv);
    if (g.overflow) {
      key = (uint32_t)i;   // output = input unchanged (Q9): identity order, one "voxel" per point
    } else {
      const float4 p = *reinterpret_cast<const float4*>(&in[i].x);
      const int ijk0 = (int)(floorf(p.x * inv) - (float)g.min_b[0]);
      const int ijk1 = (int)(floorf(p.y * inv) - (float)g.min_b[1]);
      const int ijk2 = (int)(floorf(p.z * inv) - (float)g.min_b[2]);
      key = (uint32_t)(ijk0 * g.divb_mul[0] + ijk1 * g.divb_mul[1] + ijk2 * g.divb_mul[2]);
    }
  }
  keys[i] = key;
  vals[i] = i;
}

__global__ __launch_bounds__(kTB) void run_heads(const uint32_t* __restrict__ keys, const int* __restrict__ d_n, int n_ub,
                                                 int* __restrict__ flags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ub) return;
  const int n = *d_n;
  flags[i] = (i < n) && (i == 0 || keys[i] != keys[i - 1]);
}

__global__ __launch_bounds__(kTB) void vg_reduce(const PointRec* __restrict__ in, const int* __restrict__ d_n, int n_ub,
                                                 const uint32_t* __restrict__ keys, const int* __restrict__ vals,
                                                 const int* __restrict__ flags, const int* __restrict__ pos,
                                                 const int* __restrict__ mm, float inv, PointRec* __restrict__ out,
                                                 int* __restrict__ d_out_count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = *d_n;
  if (i == 0 && n == 0) *d_out_count = 0;
  if (i >= n) return;
  if (i == n - 1) *d_out_count = pos[i] + flags[i];
  if (!flags[i]) return;
  const uint32_t k = keys[i];
  const PointRec f = in[vals[i]];
  PointRec o;
  const VoxelGeom g = voxel_geom(mm, inv);
  if (g.overflow) {
    o = f;
  } else {
    float c0 = f.x, c1 = f.y, c2 = f.z, c3 = f.intensity;
    int j = i + 1;
    for (; j < n && keys[j] == k; ++j) {
      const PointRec p = in[vals[j]];
      c0 += p.x; c1 += p.y; c2 += p.z; c3 += p.intensity;
    }
    const float cnt = (float)(j - i);
    o.x = c0 / cnt; o.y = c1 / cnt; o.z = c2 / cnt; o.pad0 = 1.0f;
    o.intensity = c3 / cnt;
    o.ring = 0; o.pad1 = 0; o.time = 0.0f; o.pad2 = 0.0f;
  }
  out[pos[i]] = o;
}

__device__ __forceinline__ bool cc_point(const PointRec* __restrict__ old, int n_old, const PointRec* __restrict__ neu,
                                         int n_new, const double* __restrict__ pose, int i, PointRec& p) {
  if (i < n_old) {
    p = old[i];
    return true;
  }
  if (i < n_old + n_new) {
    const PointRec s = neu[i - n_old];
    float x, y, z;
    associate_to_map(pose, s.x, s.y, s.z, x, y, z);
    p.x = x; p.y = y; p.z = z; p.pad0 = 1.0f;
    p.intensity = s.intensity;
    p.ring = 0; p.pad1 = 0; p.time = 0.0f; p.pad2 = 0.0f;
    return true;
  }
  return false;
}

// CropBox with min/max = Vector4f(t -+ 100) (double -> float), inclusive, order preserving
__device__ __forceinline__ bool in_box(const PointRec& p, const double* __restrict__ pose) {
  const float mnx = (float)(pose[4] - 100), mny = (float)(pose[5] - 100), mnz = (float)(pose[6] - 100);
  const float mxx = (float)(pose[4] + 100), mxy = (float)(pose[5] + 100), mxz = (float)(pose[6] + 100);
  return !(p.x < mnx || p.y < mny || p.z < mnz || p.x > mxx || p.y > mxy || p.z > mxz);
}

__global__ __launch_bounds__(kTB) void cc_flags(const PointRec* __restrict__ old, const int* __restrict__ d_old,
                                                const PointRec* __restrict__ neu, const int* __restrict__ d_new,
                                                int ub, const double* __restrict__ pose, int* __restrict__ flags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ub) return;
  PointRec p;
  const bool have = cc_point(old, *d_old, neu, *d_new, pose, i, p);
  flags[i] = have && in_box(p, pose);
}

__global__ __launch_bounds__(kTB) void cc_scatter(const PointRec* __restrict__ old, const int* __restrict__ d_old,
                                                  const PointRec* __restrict__ neu, const int* __restrict__ d_new,
                                                  int ub, const double* __restrict__ pose,
                                                  const int* __restrict__ flags, const int* __restrict__ pos,
                                                  PointRec* __restrict__ out, int* __restrict__ d_out_count) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = *d_old + *d_new;
  if (i == 0 && total == 0) *d_out_count = 0;
  if (i >= ub || i >= total) return;
  if (i == total - 1) *d_out_count = pos[i] + flags[i];
  if (!flags[i]) return;
  PointRec p;
  cc_point(old, *d_old, neu, *d_new, pose, i, p);
  out[pos[i]] = p;
}

__global__ __launch_bounds__(kTB) void compensate(PointRec* __restrict__ pts, const int* __restrict__ d_n, int n_ub,
                                                  double vx, double vy, double vz) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_ub || i >= *d_n) return;
  PointRec& p = pts[i];
  const double t = p.time;
  p.x = (float)((double)p.x + vx * t);
  p.y = (float)((double)p.y + vy * t);
  p.z = (float)((double)p.z + vz * t);
}
__global__ __launch_bounds__(kTB) void append_copy(PointRec* __restrict__ dst, const int* __restrict__ d_dst_count,
                                                   const PointRec* __restrict__ src, const int* __restrict__ d_src_count,
                                                   int src_ub, int xyzi) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= src_ub || i >= *d_src_count) return;
  PointRec p = src[i];
  if (xyzi) {
    p.pad0 = 1.0f;
    p.ring = 0; p.pad1 = 0; p.time = 0.0f; p.pad2 = 0.0f;
  }
  dst[*d_dst_count + i] = p;
}

__global__ void add_count(int* __restrict__ d_dst_count, const int* __restrict__ d_src_count) {
  if (threadIdx.x == 0) *d_dst_count += *d_src_count;
}
}  // namespace

void append_launch(PointRec* dst, int* d_dst_count, const PointRec* src, const int* d_src_count, int src_ub,
                   bool xyzi, hipStream_t st) {
  if (src_ub > 0) {
    hipLaunchKernelGGL(append_copy, dim3(div_up(src_ub, kTB)), dim3(kTB), 0, st, dst, d_dst_count, src, d_src_count,
                       src_ub, xyzi ? 1 : 0);
    FLOAM_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(add_count, dim3(1), dim3(64), 0, st, d_dst_count, d_src_count);
  FLOAM_LAUNCH_CHECK();
}

void minmax_launch(const PointRec* in, const int* d_n, int n_ub, int* d_mm, hipStream_t st) {
  hipLaunchKernelGGL(mm_init, dim3(1), dim3(64), 0, st, d_mm);
  FLOAM_LAUNCH_CHECK();
  const unsigned blocks = std::max(1u, std::min(div_up(n_ub, kTB), 1024u));
  hipLaunchKernelGGL(mm_reduce, dim3(blocks), dim3(kTB), 0, st, in, d_n, d_mm);
  FLOAM_LAUNCH_CHECK();
}

void voxel_launch(VoxelScratch& sc, const PointRec* in, const int* d_n, int n_ub, float leaf, PointRec* out,
                  int* d_out_count, hipStream_t st) {
  if (n_ub <= 0) {
    FLOAM_HIP(hipMemsetAsync(d_out_count, 0, sizeof(int), st));
    return;
  }
  sc.mm.reserve(8);
  sc.s.reserve(n_ub);
  const float inv = 1.0f / leaf;   // PCL: inverse_leaf_size_ = 1 / leaf_size_ (float)
  minmax_launch(in, d_n, n_ub, sc.mm.p, st);
  const unsigned g = div_up(n_ub, kTB);
  hipLaunchKernelGGL(vg_keys, dim3(g), dim3(kTB), 0, st, in, d_n, n_ub, sc.mm.p, inv, sc.s.k0.p, sc.s.v0.p);
  FLOAM_LAUNCH_CHECK();
  sort_pairs_u32(sc.s.temp.p, sc.s.temp_bytes, sc.s.k0.p, sc.s.k1.p, sc.s.v0.p, sc.s.v1.p, n_ub, 32, st);
  hipLaunchKernelGGL(run_heads, dim3(g), dim3(kTB), 0, st, sc.s.k1.p, d_n, n_ub, sc.s.flags.p);
  FLOAM_LAUNCH_CHECK();
  exclusive_scan_i32(sc.s.temp.p, sc.s.temp_bytes, sc.s.flags.p, sc.s.pos.p, n_ub, st);
  hipLaunchKernelGGL(vg_reduce, dim3(g), dim3(kTB), 0, st, in, d_n, n_ub, sc.s.k1.p, sc.s.v1.p, sc.s.flags.p,
                     sc.s.pos.p, sc.mm.p, inv, out, d_out_count);
  FLOAM_LAUNCH_CHECK();
}

void crop_concat_launch(SortScratch& sc, const PointRec* old, const int* d_old, int old_ub, const PointRec* neu,
                        const int* d_new, int new_ub, const double* d_pose, PointRec* out, int* d_out_count,
                        hipStream_t st) {
  const int ub = old_ub + new_ub;
  if (ub <= 0) {
    FLOAM_HIP(hipMemsetAsync(d_out_count, 0, sizeof(int), st));
    return;
  }
  sc.reserve(ub);
  const unsigned g = div_up(ub, kTB);
  hipLaunchKernelGGL(cc_flags, dim3(g), dim3(kTB), 0, st, old, d_old, neu, d_new, ub, d_pose, sc.flags.p);
  FLOAM_LAUNCH_CHECK();
  exclusive_scan_i32(sc.temp.p, sc.temp_bytes, sc.flags.p, sc.pos.p, ub, st);
  hipLaunchKernelGGL(cc_scatter, dim3(g), dim3(kTB), 0, st, old, d_old, neu, d_new, ub, d_pose, sc.flags.p, sc.pos.p,
                     out, d_out_count);
  FLOAM_LAUNCH_CHECK();
}

void compensate_velocity_launch(PointRec* pts, const int* d_n, int n_ub, double vx, double vy, double vz,
                                hipStream_t st) {
  if (n_ub <= 0) return;
  hipLaunchKernelGGL(compensate, dim3(div_up(n_ub, kTB)), dim3(kTB), 0, st, pts, d_n, n_ub, vx, vy, vz);
  FLOAM_LAUNCH_CHECK();
}

}  // namespace floam
