// Stable sort of the VoxelGrid pipelines' (u32 key, i32 value) pairs in ONE launch after the key producer —
// see bucket.hip.  Keys carry the cloud in bit 31 (vox_keys / mm_keys); 0xFFFFFFFF marks a dropped element and
// sorts last.
#pragma once
#include "floam_common.hpp"
#include "radix.hpp"

namespace floam {

constexpr int kBuckets = 256;     // buckets 0..254 hold keys (254 splitters), 255 the dropped elements (never stored)
constexpr int kSplitters = kBuckets - 2;
constexpr int kBucketCap = 4096;  // sorted in registers by one block; a larger bucket streams through global memory
constexpr int kGeoWords = 16;     // per job j: geo[8 j + 0..2] min_b, +3 dx, +4 dy, +5 index overflow (Q9)
constexpr int kAppendR = 4;       // elements per thread and chunk of a producer's bucket append
// the sort's control words (RadixScratch::ctl, zeroed per sort by radix_ctl_zero): [0, 256) the bucket cursors (the
// appended count of each bucket: its size once the producer is done), and the overflow list's length
constexpr int kBucketOvfWord = kRadixHistWords;

struct BucketScratch {
  DevBuf<unsigned long long> split;   // [kSplitters] (job << 63 | cell key) at the quantiles of the previous sort
  DevBuf<int> geo;                    // [kGeoWords] the key producer's grids (cell key <-> voxel index)
  DevBuf<unsigned long long> reg;     // [kBuckets][cap] the producer's appends: (key << 32 | value) per element
  DevBuf<unsigned long long> ovf;     // [n] appends past a bucket's region (stale splitters), ...
  DevBuf<uint8_t> ovf_b;              // ... and their buckets
  DevBuf<unsigned long long> gath;    // [n] an overflowed bucket's elements gathered at its output range
  int cap = 0;                        // region capacity per bucket (bucket_cap(n))
  bool seeded = false;                // host: split holds quantiles (else this sort takes the digit passes and seeds)
  void reserve(int n, hipStream_t st);
};

// Region capacity per bucket for a sort of up to n elements: twice the mean bucket, so only splitters gone stale
// (a new distribution) overflow into the list
inline int bucket_cap(int n) { return std::max(512, ((2 * std::max(n, 1) / (kBuckets - 1) + 64 + 63) / 64) * 64); }

// The key producer's view (split null: the four digit passes of radix.hip follow instead)
struct BucketDev {
  const unsigned long long* split;
  int* geo;
  unsigned long long* reg;
  unsigned long long* ovf;
  uint8_t* ovf_b;
  int cap;
  int ovf_cap;
};

// Producer side.  bucket_keys_lds: the splitters as 32-bit sort keys of the calling block's cloud `job` (its grid: min_b,
// dx, dy, dz, overflow), in LDS s[256] (ascending; the other cloud's splitters collapse to 0 below / ~0 above):
// a splitter cell outside the grid saturates to the grid's first / last cell of its row, plane or grid, which keeps the
// order.  All threads call it (it ends with a barrier).  bucket_of: the bucket of a sort key.
// sp_t: split[threadIdx.x], loaded by the caller in its prologue (bucket_split_prefetch) so the splitters do not add a
// memory round trip after the bounding box
__device__ __forceinline__ unsigned long long bucket_split_prefetch(const unsigned long long* __restrict__ split) {
  return split && (int)threadIdx.x < kSplitters ? split[threadIdx.x] : 0ull;
}
__device__ __forceinline__ void bucket_keys_lds(const unsigned long long* __restrict__ split, unsigned long long sp_t,
                                                int job, const int (&mb)[3], long long dx, long long dy, long long dz,
                                                bool ovf, uint32_t* s) {
  const int t = threadIdx.x;
  for (int m = t; m < kBuckets; m += blockDim.x) {
    uint32_t v = 0xFFFFFFFFu;
    if (m < kSplitters) {
      const unsigned long long sp = m == t ? sp_t : split[m];
      const int sj = (int)(sp >> 63);
      if (sj < job) {
        v = 0u;
      } else if (sj == job) {
        if (ovf) {
          v = ((uint32_t)job << 31) | 0x7FFFFFFFu;   // identity keys (Q9): the whole cloud in one bucket
        } else {
          const unsigned long long ck = sp & 0x7FFFFFFFFFFFFFFFull;
          const long long cx = (long long)(ck & 0x1FFFFFull) - (1 << 20) - mb[0];
          const long long cy = (long long)((ck >> 21) & 0x1FFFFFull) - (1 << 20) - mb[1];
          const long long cz = (long long)((ck >> 42) & 0x1FFFFFull) - (1 << 20) - mb[2];
          const long long plane = dx * dy;
          long long idx;
          if (cz < 0) idx = 0;
          else if (cz >= dz) idx = plane * dz - 1;
          else if (cy < 0) idx = cz * plane;
          else if (cy >= dy) idx = cz * plane + plane - 1;
          else if (cx < 0) idx = cz * plane + cy * dx;
          else if (cx >= dx) idx = cz * plane + cy * dx + dx - 1;
          else idx = cz * plane + cy * dx + cx;
          idx = idx < 0 ? 0 : (idx > 0x7FFFFFFEll ? 0x7FFFFFFEll : idx);
          v = ((uint32_t)job << 31) | (uint32_t)idx;
        }
      }
    }
    s[m] = v;
  }
  __syncthreads();
}

__device__ __forceinline__ unsigned bucket_of(const uint32_t* s, uint32_t key) {
  if (key == 0xFFFFFFFFu) return kBuckets - 1;
  unsigned b = 0;   // splitters <= key among s[0 .. 253] (s[254], s[255] = ~0 never count)
#pragma unroll
  for (int step = 128; step > 0; step >>= 1)
    if (s[b + step - 1] <= key) b += step;
  return b;
}

// Producer-side bucket append (the stable scatter pass it replaces cost a launch, ~9 us, on every sort): every thread
// holds R elements of the block's chunk; each valid key (not 0xFFFFFFFF) takes its rank among the chunk's elements of
// its bucket (LDS atomic), thread b reserves bucket b's slots for the whole chunk with one atomic on the bucket's
// cursor, and every element is stored as (key << 32 | value) at its slot of the bucket's region — or, past the
// region's capacity, in the overflow list with its bucket.  Slots inside a bucket are in no particular order: the
// consumer sorts by (key, value), and the values are the elements' input positions, so that order is the stable one.
// Called by all threads of the block (kTB == kBuckets); s_cnt [kBuckets] zero on entry and on return, s_off / s_ovf
// [kBuckets] scratch; cursor = the sort's control words (kBucketOvfWord: the list's length).  Contains barriers.
template <int R>
__device__ __forceinline__ void bucket_append(const BucketDev& bd, unsigned* __restrict__ cursor, const uint32_t* s_spl,
                                              const uint32_t (&key)[R], const int (&val)[R], unsigned* s_cnt,
                                              int* s_off, int* s_ovf) {
  unsigned b[R], rk[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    b[r] = kBuckets - 1;
    rk[r] = 0u;
    if (key[r] != 0xFFFFFFFFu) {
      b[r] = bucket_of(s_spl, key[r]);
      rk[r] = atomicAdd(&s_cnt[b[r]], 1u);
    }
  }
  __syncthreads();
  const int t = threadIdx.x;
  const unsigned c = s_cnt[t];
  if (c) {
    const unsigned base = atomicAdd(&cursor[t], c);
    s_off[t] = (int)base;
    const unsigned cap = (unsigned)bd.cap;
    if (base + c > cap) {   // overflow: ranks past the capacity go to the list, in rank order
      const unsigned first = base > cap ? base : cap;
      const unsigned o = atomicAdd(&cursor[kBucketOvfWord], base + c - first);
      s_ovf[t] = (int)o + (int)base - (int)first;   // list position of rank 0 (only ranks >= first - base use it)
    }
    s_cnt[t] = 0u;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (key[r] == 0xFFFFFFFFu) continue;
    const unsigned long long ent = ((unsigned long long)key[r] << 32) | (unsigned)val[r];
    const int slot = s_off[b[r]] + (int)rk[r];
    if (slot < bd.cap) {
      bd.reg[(size_t)b[r] * bd.cap + slot] = ent;
    } else {
      const int o = s_ovf[b[r]] + (int)rk[r];
      if (o < bd.ovf_cap) {
        bd.ovf[o] = ent;
        bd.ovf_b[o] = (uint8_t)b[r];
      }
    }
  }
}

// the producer's grid of cloud `job` for the next splitters (block 0 of the job, one thread)
__device__ __forceinline__ void bucket_geo_store(int* geo, int job, const int (&mb)[3], int dx, int dy, bool ovf) {
  int* g = geo + 8 * job;
  g[0] = mb[0]; g[1] = mb[1]; g[2] = mb[2];
  g[3] = dx; g[4] = dy; g[5] = ovf ? 1 : 0;
}

// Sort-only form (the map merge, mapmerge.hip): one block per bucket sorts the elements the producer appended to it
// (bucket_append, with the BucketDev of bs: bs.seeded) into k0 / v0 at the bucket's output range and writes the next
// splitters; k1 / v1 are the scratch of a bucket that streams.  Before seeding, use radix_sort_launch followed by
// bucket_seed_launch.
void bucket_sort_launch(BucketScratch& bs, RadixScratch& rs, uint32_t* k0, int* v0, uint32_t* k1, int* v1, int n,
                        hipStream_t st, const int* gate);

// After a digit-pass sort of the same pipeline (sorted keys in k0, n_dev elements): the first splitters, from its
// quantiles (one block)
void bucket_seed_launch(BucketScratch& bs, const uint32_t* k0, const int* n_dev, int n, hipStream_t st,
                        const int* gate);

// The producer's view of bs for a sort of up to n elements (reserves it; split null unless seeded)
BucketDev bucket_dev(BucketScratch& bs, int n, hipStream_t st);

// pipeline 0: the VoxelGrids (voxel2_launch), 1: the map merge (map_merge_launch).  FLOAM_SORT=radix|bucket|merge
// (read once per process; default bucket: both pipelines)
bool bucket_sort_enabled(int pipeline);

void bucket_stamps_print();   // FLOAM_BC_STAMPS (diagnostic)

}  // namespace floam
