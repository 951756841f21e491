// LaserMappingClass::updateCurrentPointsToMap on gfx950 (src/laserMappingClass.cpp:148-186).
//
// The map lives in HBM as one array of 32-B XYZI records grouped by 50-m cell in getMap order (absolute (x, y, z)),
// with the cell table (key, count) on the host.  One update:
//   map_prep       per input point: pose_current.cast<float>() transform (float sums, PCL 1.8.1 transforms.hpp),
//                  intensity min(1, max(z + 2, 0) / 5) from the untransformed z, cell index, and its cell counted in
//                  an open-addressing table of the cells this scan touches
//   (host)         reads the touched cells, merges them into the cell table, ranks them
//   map_rank_keys  per point: its cell's rank as a radix key (+ histograms); the stable radix sort (radix.hip) and
//   map_gather     group the new points by cell, input order kept inside a cell (push_back order)
//   voxel2         pcl::VoxelGrid of every non-empty cell of the 5 x 5 x 5 neighbourhood of the pose, over
//                  [old points of the cell ; its new points] — the cell's cloud after the push_backs (voxel.hip)
//   map_offsets    exclusive scan of the per-cell sizes (one block)
//   map_copy       every point of the new map from its source: the cell's voxel output, or (cells outside the
//                  neighbourhood) its old points then its new points
// Two synchronisations per update: the touched-cell table and the final per-cell sizes.
#include "mapping.hpp"

namespace floam {

namespace {
constexpr int kTB = 256;

__device__ __forceinline__ unsigned map_hash(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  return (unsigned)k;
}

__device__ __forceinline__ int cell_of(double v) { return (int)floor(v / 50.0 + 0.5); }

__global__ __launch_bounds__(kTB) void map_prep(MapPrepArgs a) {
  if (blockIdx.x == 0) radix_ctl_zero(a.radix_ctl, threadIdx.x, blockDim.x);
  const int i = blockIdx.x * kTB + threadIdx.x;
  const int n = min(*a.d_n, a.n);
  if (i >= n) return;
  const PointRec s = a.in[i];
  PointRec p;
  p.x = ((a.m[0] * s.x + a.m[1] * s.y) + a.m[2] * s.z) + a.m[3];
  p.y = ((a.m[4] * s.x + a.m[5] * s.y) + a.m[6] * s.z) + a.m[7];
  p.z = ((a.m[8] * s.x + a.m[9] * s.y) + a.m[10] * s.z) + a.m[11];
  p.pad0 = 1.0f;
  const double zz = (double)s.z + 2.0;
  const double mx = (zz < 0.0) ? 0.0 : zz;   // std::max(z + 2.0, 0.0)
  const double v = mx / 5;
  p.intensity = (float)((v < 1.0) ? v : 1.0);   // std::min(1.0, .)
  p.ring = 0; p.pad1 = 0; p.time = 0.0f; p.pad2 = 0.0f;
  a.stage[i] = p;
  const unsigned long long key = map_cell_key(cell_of(p.x), cell_of(p.y), cell_of(p.z));
  unsigned h = map_hash(key) & (kMapHashSlots - 1);
  for (int probe = 0; probe < kMapHashSlots / 2; ++probe) {
    const unsigned long long prev = atomicCAS(&a.hkeys[h], ~0ull, key);
    if (prev == ~0ull || prev == key) {
      atomicAdd(&a.hcnt[h], 1);
      a.slot[i] = (int)h;
      return;
    }
    h = (h + 1) & (kMapHashSlots - 1);
  }
  *a.overflow = 1;
  a.slot[i] = -1;
}

__global__ __launch_bounds__(kTB) void map_rank_keys(const int* __restrict__ slot, const int* __restrict__ hrank,
                                                     int n, uint32_t* __restrict__ keys, int* __restrict__ vals,
                                                     unsigned* __restrict__ radix_ctl) {
  __shared__ unsigned s_hist[kRadixHistWords];
  radix_hist_begin(s_hist);
  for (int i = blockIdx.x * kTB + threadIdx.x; i < n; i += gridDim.x * kTB) {
    const int sl = slot[i];
    const uint32_t k = sl >= 0 ? (uint32_t)hrank[sl] : 0xFFFFFFFFu;
    keys[i] = k;
    vals[i] = i;
    radix_hist_add(s_hist, k);
  }
  radix_hist_end(s_hist, radix_ctl);
}

__global__ __launch_bounds__(kTB) void map_gather(const PointRec* __restrict__ src, const int* __restrict__ perm, int n,
                                                  PointRec* __restrict__ dst) {
  const int j = blockIdx.x * kTB + threadIdx.x;
  if (j < n) dst[j] = src[perm[j]];
}

// exclusive scan of outcnt -> off (one block, chunks of 1024 cells)
__global__ __launch_bounds__(1024) void map_offsets(MapCopyArgs a) {
  __shared__ int s[1024];
  __shared__ int s_carry;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (int c0 = 0; c0 < a.ncell; c0 += 1024) {
    const int c = c0 + (int)threadIdx.x;
    const int v = c < a.ncell ? max(a.outcnt[c], 0) : 0;   // -1: a failed compaction (reported by the host)
    s[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {   // Hillis-Steele inclusive scan
      const int t = threadIdx.x >= (unsigned)o ? s[threadIdx.x - o] : 0;
      __syncthreads();
      s[threadIdx.x] += t;
      __syncthreads();
    }
    if (c < a.ncell) a.off[c] = s_carry + s[threadIdx.x] - v;
    __syncthreads();
    if (threadIdx.x == 1023) s_carry += s[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.off[a.ncell] = s_carry;
    *a.d_total = s_carry;
  }
}

__global__ __launch_bounds__(kTB) void map_copy(MapCopyArgs a) {
  const int j = blockIdx.x * kTB + threadIdx.x;
  if (j >= a.off[a.ncell]) return;
  int lo = 0, hi = a.ncell;   // last cell with off[c] <= j
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (a.off[mid] <= j) lo = mid;
    else hi = mid;
  }
  const int c = lo, local = j - a.off[c];
  PointRec p;
  if (a.vox_off[c] >= 0) {
    p = a.vox[a.vox_off[c] + local];
  } else {
    const int nold = a.seg[2 * c];
    p = local < nold ? a.old_map[a.old_start[c] + local] : a.new_pts[a.new_start[c] + local - nold];
  }
  a.out[j] = p;
}
}  // namespace

void map_prep_launch(const MapPrepArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(map_prep, dim3(div_up(std::max(a.n, 1), kTB)), dim3(kTB), 0, st, a);
  FLOAM_LAUNCH_CHECK();
}

void map_rank_keys_launch(const int* slot, const int* hrank, int n, uint32_t* keys, int* vals, unsigned* radix_ctl,
                          hipStream_t st) {
  const unsigned nb = std::max(1u, std::min(div_up(std::max(n, 1), kTB), 64u));
  hipLaunchKernelGGL(map_rank_keys, dim3(nb), dim3(kTB), 0, st, slot, hrank, n, keys, vals, radix_ctl);
  FLOAM_LAUNCH_CHECK();
}

void map_gather_launch(const PointRec* src, const int* perm, int n, PointRec* dst, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(map_gather, dim3(div_up(n, kTB)), dim3(kTB), 0, st, src, perm, n, dst);
  FLOAM_LAUNCH_CHECK();
}

void map_rebuild_launch(const MapCopyArgs& a, int total_ub, hipStream_t st) {
  hipLaunchKernelGGL(map_offsets, dim3(1), dim3(1024), 0, st, a);
  FLOAM_LAUNCH_CHECK();
  if (total_ub > 0) {
    hipLaunchKernelGGL(map_copy, dim3(div_up(total_ub, kTB)), dim3(kTB), 0, st, a);
    FLOAM_LAUNCH_CHECK();
  }
}

}  // namespace floam
