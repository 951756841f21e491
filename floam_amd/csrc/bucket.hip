// Stable (key, value) sort for the VoxelGrid pipelines (pcl::VoxelGrid's std::sort of (idx, point) pairs,
// src/odomEstimationClass.cpp:137-142 and :278-292 via PCL 1.8.1) in ONE launch after the key producer, instead of
// four 8-bit digit passes (radix.hip: ~9 us each at the scan's sizes whatever the size — each is a device-wide
// ranking + decoupled lookback + scatter, bound by its latency).
//
// Sample sort with the previous sort's quantiles as splitters:
//   * the key producer (vox_keys / mm_keys) puts every key into one of 255 buckets — contiguous key ranges cut at 254
//     splitters — by a binary search in LDS, and appends it with its value to the bucket's region (bucket_append,
//     bucket.hpp: one atomic per block and bucket reserves the block's slots; past the region's capacity the element
//     goes to an overflow list).  Round 5 scattered the keys by bucket with a stable digit pass instead: a launch of
//     ~9 us on each of the two main-stream sorts of a scan;
//   * one block per bucket sorts its elements by (key, value) — the values are the input positions, so that is the
//     stable order whatever order the appends landed in — with a register bitonic network — every stride a compile-time constant, lane exchanges by ds_swizzle / ds_bpermute, LDS
//     only for strides that cross waves — and either writes them out (the map merge) or, for a VoxelGrid, emits its
//     voxels' centroids itself (a voxel's points share one key, so they never straddle two buckets; output slots by
//     decoupled lookback over the buckets in key order).  A bucket beyond 4096 elements (stale splitters) is sorted
//     by the same block through global memory, chunk by chunk — slower, same result.
// The splitters are cell keys (the map's (z, y, x) cell order, 21 bits a component, mapmerge.hpp), which do not depend
// on a grid's min_b: every sort writes the cell keys at its own 254 quantiles for the next one, and the next sort
// converts them into its own grid's voxel indices.  Consecutive scans (sensor frame) or scan voxels (map frame) have
// nearly the same distribution, so the buckets stay balanced (C3 surf cloud: largest bucket 541 of 113.5k keys, mean
// 445).  The first sort of a pipeline takes the digit passes and seeds the splitters from its output.  Any splitters
// give the same result: they only decide which block sorts which key range.
#include <cfloat>
#include <climits>
#include <cstdlib>
#include <type_traits>

#include "bucket.hpp"
#include "lookback.hpp"
#include "voxel.hpp"

namespace floam {

namespace {
constexpr int kTB = 256;
constexpr int kW = kTB / 64;
static_assert(kTB == kBuckets, "bucket_range: one histogram word per thread");

// ---------------------------------------------------------------------------------------------- next splitters
// the cell key of sort key k (job bit + voxel index of the producer's grid) for the splitters
__device__ __forceinline__ unsigned long long split_key(uint32_t k, const int* __restrict__ geo) {
  const int job = (int)(k >> 31);
  const int* g = geo + 8 * job;
  if (g[5]) return ((unsigned long long)job << 63) | 0x7FFFFFFFFFFFFFFFull;   // identity keys (Q9): no cells
  const long long idx = (long long)(k & 0x7FFFFFFFu);
  const long long dx = g[3] > 0 ? g[3] : 1, dy = g[4] > 0 ? g[4] : 1;
  const long long i = idx % dx, j = (idx / dx) % dy, kk = idx / (dx * dy);
  auto comp = [](long long c) {
    c += (1 << 20);
    return (unsigned long long)(c < 0 ? 0 : (c > 0x1FFFFF ? 0x1FFFFF : c));
  };
  return ((unsigned long long)job << 63) | (comp(kk + g[2]) << 42) | (comp(j + g[1]) << 21) | comp(i + g[0]);
}

// the quantile ranks r_m = (m + 1) kept / 255 that fall in [lo, lo + cnt): split[m] from the sorted key at r_m
template <typename KeyAt>
__device__ __forceinline__ void write_splitters(unsigned long long* __restrict__ split, const int* __restrict__ geo,
                                                int kept, int lo, int cnt, KeyAt key_at) {
  for (int m = threadIdx.x; m < kSplitters; m += blockDim.x) {
    const int r = (int)(((long long)(m + 1) * kept) / (kSplitters + 1));
    if (r >= lo && r < lo + cnt && r < kept) split[m] = split_key(key_at(r - lo), geo);
  }
}

// bucket b's start and size from the producer's bucket histogram (256 words): every block scans it.  c = hist[t],
// loaded by the caller in its prologue (it does not depend on b, so it travels with the ticket / gate loads)
struct BucketRange {
  int start, size, kept;
};
__device__ __forceinline__ BucketRange bucket_range(unsigned c, int b, unsigned* s_tmp) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  unsigned inc = c;
  inc = wave_incl_scan(inc);   // (DPP, floam_common.hpp)
  if (lane == 63) s_tmp[w] = inc;
  __syncthreads();
  unsigned add = 0;
#pragma unroll
  for (int k = 0; k < kW; ++k)
    if (k < w) add += s_tmp[k];
  __shared__ int s_r[3];
  if (t == b) { s_r[0] = (int)(add + inc - c); s_r[1] = (int)c; }
  if (t == kBuckets - 1) s_r[2] = (int)(add + inc - c);   // keys before the dropped bucket
  __syncthreads();
  return BucketRange{s_r[0], s_r[1], s_r[2]};
}

// ---------------------------------------------------------------------------------------------- bucket source
struct BucketSrc {   // the consumer's view of the producer's appends (BucketDev)
  const unsigned long long* reg;
  const unsigned long long* ovf;
  const uint8_t* ovf_b;
  unsigned long long* gath;
  int cap;
};

BucketSrc bucket_src(const BucketScratch& bs) { return BucketSrc{bs.reg.p, bs.ovf.p, bs.ovf_b.p, bs.gath.p, bs.cap}; }

// Bucket b's `size` elements as (key << 32 | value) words: its region, or — when the appends overflowed it — the
// region's words and the bucket's entries of the overflow list (novf long) gathered to gath[start, start + size).
// Called by all threads (block-uniform arguments); contains barriers.
__device__ __forceinline__ const unsigned long long* bucket_source(const BucketSrc& S, int b, int start, int size,
                                                                   int novf) {
  const unsigned long long* reg = S.reg + (size_t)b * S.cap;
  if (size <= S.cap) return reg;
  unsigned long long* g = S.gath + start;
  __shared__ int s_n;
  const int t = threadIdx.x;
  for (int e = t; e < S.cap; e += kTB) g[e] = reg[e];
  if (t == 0) s_n = S.cap;
  __syncthreads();
  for (int o0 = 0; o0 < novf; o0 += kTB) {   // (block-uniform trip count)
    const int o = o0 + t;
    if (o < novf && S.ovf_b[o] == (uint8_t)b) g[atomicAdd(&s_n, 1)] = S.ovf[o];
  }
  __syncthreads();
  return g;
}

// ---------------------------------------------------------------------------------------------- bitonic network
// E 64-bit words per thread (position p = E t + e), N = kTB E; a stage's stride is a compile-time constant
template <int M>
__device__ __forceinline__ unsigned long long xor_lane64(unsigned long long v) {
  int lo = (int)(unsigned)v, hi = (int)(unsigned)(v >> 32);
  if constexpr (M < 32) {
    lo = __builtin_amdgcn_ds_swizzle(lo, (M << 10) | 0x1F);   // bitmask mode: lane ^ M within 32
    hi = __builtin_amdgcn_ds_swizzle(hi, (M << 10) | 0x1F);
  } else {
    const int a = (((int)threadIdx.x & 63) ^ M) << 2;
    lo = __builtin_amdgcn_ds_bpermute(a, lo);
    hi = __builtin_amdgcn_ds_bpermute(a, hi);
  }
  return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}

template <int E, int SIZE, int STRIDE>
__device__ __forceinline__ void bitonic_stage64(unsigned long long (&k)[E], unsigned long long* s_x) {
  const int t = threadIdx.x;
  unsigned long long ok[E];
  if constexpr (STRIDE < E) {
#pragma unroll
    for (int e = 0; e < E; ++e) ok[e] = k[e ^ STRIDE];
  } else if constexpr (STRIDE < 64 * E) {
#pragma unroll
    for (int e = 0; e < E; ++e) ok[e] = xor_lane64<STRIDE / E>(k[e]);
  } else {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) s_x[E * t + e] = k[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) ok[e] = s_x[(E * t + e) ^ STRIDE];
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int pp = E * t + e;
    const bool lower = (pp & STRIDE) == 0, asc = (pp & SIZE) == 0;
    const unsigned long long a = k[e], b = ok[e];
    k[e] = (asc == lower) ? (a < b ? a : b) : (a < b ? b : a);
  }
}
template <int E, int SIZE, int STRIDE>
__device__ __forceinline__ void bitonic_strides64(unsigned long long (&k)[E], unsigned long long* s_x) {
  bitonic_stage64<E, SIZE, STRIDE>(k, s_x);
  if constexpr (STRIDE > 1) bitonic_strides64<E, SIZE, STRIDE / 2>(k, s_x);
}
template <int E, int SIZE>
__device__ __forceinline__ void bitonic_sizes64(unsigned long long (&k)[E], unsigned long long* s_x) {
  bitonic_strides64<E, SIZE, SIZE / 2>(k, s_x);
  if constexpr (SIZE < kTB * E) bitonic_sizes64<E, SIZE * 2>(k, s_x);
}

// The bucket's `size` (<= kTB E) (key << 32 | value) words src[0, size) sorted: keys and values into s_k / s_v[0,
// size).  Contains barriers.
template <int E>
__device__ __forceinline__ void bucket_bitonic(const unsigned long long* __restrict__ src, int size,
                                               unsigned long long* s_x, uint32_t* s_k, int* s_v) {
  const int t = threadIdx.x;
  unsigned long long k[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int q = E * t + e;
    k[e] = q < size ? src[q] : ~0ull;
  }
  bitonic_sizes64<E, 2>(k, s_x);
  __syncthreads();   // (s_x's last reads, when s_k / s_v share its storage)
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int p = E * t + e;
    if (p < size) {
      s_k[p] = (uint32_t)(k[e] >> 32);
      s_v[p] = (int)(unsigned)k[e];
    }
  }
  __syncthreads();
}

template <typename F>
__device__ __forceinline__ void by_size(int size, F f) {   // the smallest network that holds the bucket
  if (size <= kTB) f(std::integral_constant<int, 1>{});
  else if (size <= 2 * kTB) f(std::integral_constant<int, 2>{});
  else if (size <= 4 * kTB) f(std::integral_constant<int, 4>{});
  else if (size <= 8 * kTB) f(std::integral_constant<int, 8>{});
  else f(std::integral_constant<int, 16>{});
}

// ---------------------------------------------------------------------------------------------- streamed bucket
// A bucket beyond kBucketCap (stale splitters): stable LSD passes through global memory, chunk by chunk of
// kStreamChunk (ping-pong between ka / va and kb / vb; the result lands in kb / vb) — first over the values' range,
// then over the keys' range, so the result is in (key, value) order whatever the input order.
constexpr int kStreamR = 8;
constexpr int kStreamChunk = kTB * kStreamR;

__device__ __forceinline__ unsigned long long match_digit8(unsigned d, bool valid) {
  unsigned long long m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const bool bit = (d >> b) & 1u;
    const unsigned long long v = __ballot(bit);
    m &= bit ? v : ~v;
  }
  return m;
}

struct StreamLds {
  unsigned cnt[kW][256];
  unsigned off[257];
  unsigned ws[4];
  unsigned run[256];
  unsigned base[256];
  uint32_t red[2][kW];
};

// one stable 8-bit counting step over a chunk held in registers, element e = w 64 R + r 64 + lane: pos = rank by
// (digit, e) among the nvalid elements; L.off = the chunk's digit starts
__device__ __forceinline__ void chunk_rank(const unsigned (&dig)[kStreamR], int nvalid, unsigned (&pos)[kStreamR],
                                           StreamLds& L) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  for (int k = t; k < kW * 256; k += kTB) (&L.cnt[0][0])[k] = 0u;
  __syncthreads();
  const unsigned long long lt = (1ull << lane) - 1ull;
  unsigned rank[kStreamR];
#pragma unroll
  for (int r = 0; r < kStreamR; ++r) {
    const int e = w * 64 * kStreamR + r * 64 + lane;
    const bool valid = e < nvalid;
    const unsigned long long peers = match_digit8(dig[r], valid);
    const unsigned before = L.cnt[w][dig[r]];
    rank[r] = before + (unsigned)__popcll(peers & lt);
    if (valid && lane == 63 - __clzll((long long)peers)) L.cnt[w][dig[r]] = before + (unsigned)__popcll(peers);
  }
  __syncthreads();
  unsigned tot = 0, inc = 0;
#pragma unroll
  for (int k = 0; k < kW; ++k) {   // thread t = digit t
    const unsigned v = L.cnt[k][t];
    L.cnt[k][t] = tot;
    tot += v;
  }
  inc = tot;
  inc = wave_incl_scan(inc);   // (DPP, floam_common.hpp)
  if (lane == 63) L.ws[w] = inc;
  __syncthreads();
  unsigned add = 0;
#pragma unroll
  for (int k = 0; k < kW; ++k)
    if (k < w) add += L.ws[k];
  L.off[t] = add + inc - tot;
  if (t == 255) L.off[256] = add + inc;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kStreamR; ++r) pos[r] = L.off[dig[r]] + L.cnt[w][dig[r]] + rank[r];
}

__device__ void stream_sort(uint32_t* __restrict__ ka, int* __restrict__ va, uint32_t* __restrict__ kb,
                            int* __restrict__ vb, int size, StreamLds& L) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t mn[2] = {0xFFFFFFFFu, 0xFFFFFFFFu}, mx[2] = {0u, 0u};   // [0] keys, [1] values
  for (int e = t; e < size; e += kTB) {
    const uint32_t k = ka[e], v = (uint32_t)va[e];
    mn[0] = min(mn[0], k);
    mx[0] = max(mx[0], k);
    mn[1] = min(mn[1], v);
    mx[1] = max(mx[1], v);
  }
  uint32_t lo[2], hi[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      mn[j] = min(mn[j], (uint32_t)__shfl_xor((int)mn[j], o, 64));
      mx[j] = max(mx[j], (uint32_t)__shfl_xor((int)mx[j], o, 64));
    }
    __syncthreads();
    if (lane == 0) { L.red[0][w] = mn[j]; L.red[1][w] = mx[j]; }
    __syncthreads();
    lo[j] = L.red[0][0];
    hi[j] = L.red[1][0];
#pragma unroll
    for (int k = 1; k < kW; ++k) {
      lo[j] = min(lo[j], L.red[0][k]);
      hi[j] = max(hi[j], L.red[1][k]);
    }
  }
  const uint32_t krange = hi[0] - lo[0], vrange = hi[1] - lo[1];
  const int nkey = krange ? (32 - __clz((int)krange) + 7) / 8 : 0;
  const int nval = vrange ? (32 - __clz((int)vrange) + 7) / 8 : 0;
  const int npass = nval + nkey;
  uint32_t *ks = ka, *kd = kb;
  int *vs = va, *vd = vb;
  for (int p = 0; p < npass; ++p) {
    const bool by_val = p < nval;   // (block-uniform)
    const int sh = 8 * (by_val ? p : p - nval);
    const uint32_t base = by_val ? lo[1] : lo[0];
    auto digit = [&](uint32_t k, int v) { return (((by_val ? (uint32_t)v : k) - base) >> sh) & 255u; };
    L.run[t] = 0u;
    __syncthreads();
    for (int e = t; e < size; e += kTB) atomicAdd(&L.run[digit(ks[e], vs[e])], 1u);
    __syncthreads();
    const unsigned c = L.run[t];
    unsigned inc = c;
    inc = wave_incl_scan(inc);   // (DPP, floam_common.hpp)
    if (lane == 63) L.ws[w] = inc;
    __syncthreads();
    unsigned add = 0;
    for (int k = 0; k < w; ++k) add += L.ws[k];
    L.base[t] = add + inc - c;
    L.run[t] = 0u;
    __syncthreads();
    for (int c0 = 0; c0 < size; c0 += kStreamChunk) {
      const int nc = min(kStreamChunk, size - c0);
      uint32_t key[kStreamR];
      int val[kStreamR];
      unsigned dig[kStreamR], pos[kStreamR];
#pragma unroll
      for (int r = 0; r < kStreamR; ++r) {
        const int e = w * 64 * kStreamR + r * 64 + lane;
        key[r] = e < nc ? ks[c0 + e] : 0u;
        val[r] = e < nc ? vs[c0 + e] : 0;
        dig[r] = digit(key[r], val[r]);
      }
      chunk_rank(dig, nc, pos, L);
#pragma unroll
      for (int r = 0; r < kStreamR; ++r) {
        const int e = w * 64 * kStreamR + r * 64 + lane;
        if (e >= nc) continue;
        const unsigned d = dig[r];
        const unsigned dst = L.base[d] + L.run[d] + (pos[r] - L.off[d]);
        kd[dst] = key[r];
        vd[dst] = val[r];
      }
      __syncthreads();
      L.run[t] += L.off[t + 1] - L.off[t];
      __syncthreads();
    }
    uint32_t* tk = ks; ks = kd; kd = tk;
    int* tv = vs; vs = vd; vd = tv;
  }
  if (ks != kb) {   // an even number of passes (or none): the sorted elements are in the scatter's region
    for (int e = t; e < size; e += kTB) {
      kb[e] = ks[e];
      vb[e] = vs[e];
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------- sort-only (merge)
struct SortLds {
  unsigned long long x[kBucketCap];   // bitonic exchanges across waves
  uint32_t k[kBucketCap];
  int v[kBucketCap];
  unsigned tmp[kW];
};

// a streamed bucket's elements unpacked into separate keys / values (stream_sort's layout)
__device__ __forceinline__ void unpack_bucket(const unsigned long long* __restrict__ src, int size,
                                              uint32_t* __restrict__ k, int* __restrict__ v) {
  for (int e = threadIdx.x; e < size; e += kTB) {
    const unsigned long long x = src[e];
    k[e] = (uint32_t)(x >> 32);
    v[e] = (int)(unsigned)x;
  }
  __syncthreads();
}

// kscr / vscr: scratch of a streamed bucket (at the bucket's output range)
__global__ __launch_bounds__(kTB) void bucket_sort(BucketSrc S, uint32_t* __restrict__ kscr, int* __restrict__ vscr,
                                                   uint32_t* __restrict__ kout, int* __restrict__ vout,
                                                   const unsigned* __restrict__ hist, const int* __restrict__ gate,
                                                   unsigned long long* __restrict__ split, const int* __restrict__ geo) {
  const int b = blockIdx.x, t = threadIdx.x;
  const unsigned hc = hist[t];   // (kTB == kBuckets; issued with the gate load)
  const int novf = (int)hist[kBucketOvfWord];
  const int gv = gate ? *gate : 1;
  if (!gv) return;
  __shared__ union {
    SortLds s;
    StreamLds st;
  } L;
  const BucketRange R = bucket_range(hc, b, L.s.tmp);
  const int start = R.start, size = R.size;
  if (size == 0) return;   // (bucket 255, the dropped elements, is never appended to)
  const unsigned long long* src = bucket_source(S, b, start, size, novf);
  if (size > kBucketCap) {
    unpack_bucket(src, size, kscr + start, vscr + start);
    stream_sort(kscr + start, vscr + start, kout + start, vout + start, size, L.st);
    write_splitters(split, geo, R.kept, start, size, [&](int q) { return kout[start + q]; });
    return;
  }
  by_size(size, [&](auto EC) {
    constexpr int E = decltype(EC)::value;
    bucket_bitonic<E>(src, size, L.s.x, L.s.k, L.s.v);
  });
  for (int e = t; e < size; e += kTB) {
    kout[start + e] = L.s.k[e];
    vout[start + e] = L.s.v[e];
  }
  write_splitters(split, geo, R.kept, start, size, [&](int q) { return L.s.k[q]; });
}

// ---------------------------------------------------------------------------------------------- VoxelGrid
constexpr int kRunPad = 16;   // the emit loop's look-ahead reads up to 15 elements past the chunk (values unused)
struct CompactLds {
  union {
    unsigned long long x[kBucketCap];
    float4 pt[kBucketCap + kRunPad];
  } u;   // the network's exchanges, then the points (staged after the sort)
  uint32_t k[kBucketCap + kRunPad];
  int v[kBucketCap];
  unsigned tmp[kW];
  unsigned hw[2][kW];
  float carry[4];
  int carry_n, carry_pos, carry_job;
  uint32_t carry_key, prev_key;
};

__device__ __forceinline__ PointRec centroid_out(float c0, float c1, float c2, float c3, int n) {
  const float cn = (float)n;
  PointRec o;
  o.x = c0 / cn; o.y = c1 / cn; o.z = c2 / cn; o.pad0 = 1.0f;
  o.intensity = c3 / cn;
  o.ring = 0; o.pad1 = 0; o.time = 0.0f; o.pad2 = 0.0f;
  return o;
}

// this thread's elements of a chunk of nc: the contiguous range [e0, e1) (outputs are numbered in element order)
__device__ __forceinline__ void thread_range(int nc, int& e0, int& e1) {
  const int per = (nc + kTB - 1) / kTB;
  e0 = min(nc, (int)threadIdx.x * per);
  e1 = min(nc, e0 + per);
}

// heads (first element of a key run) among the sorted keys k[0, nc) of a chunk, per cloud, in this thread's range;
// prev = the key before the chunk, first = the chunk starts the bucket
__device__ __forceinline__ void chunk_heads(const uint32_t* k, int nc, uint32_t prev, bool first, int (&c)[2]) {
  c[0] = c[1] = 0;
  int e0, e1;
  thread_range(nc, e0, e1);
  for (int e = e0; e < e1; ++e) {
    const uint32_t kp = e ? k[e - 1] : prev;
    if ((e == 0 && first) || k[e] != kp) {   // (no dynamic index into c: it would be private memory)
      const int j = (int)(k[e] >> 31);
      c[0] += 1 - j;
      c[1] += j;
    }
  }
}

// block sum of two counters (every thread gets the totals); contains barriers
__device__ __forceinline__ void block_sum2(int (&c)[2], unsigned (*hw)[kW]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int v = c[j];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) hw[j][w] = (unsigned)v;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    int v = 0;
#pragma unroll
    for (int k = 0; k < kW; ++k) v += (int)hw[j][k];
    c[j] = v;
  }
  __syncthreads();
}

// FLOAM_BC_STAMPS=1 (diagnostic): per-bucket phase times of the last two bucket_compact launches (slot = launch
// parity: call 1's VoxelGrids on the side stream, then call 2's on the main stream), printed by bucket_stamps_print
__device__ unsigned g_bc_st[2][kBuckets][8];

// kin / vin: scratch of a streamed bucket (its keys and values unpacked at the bucket's range), kout / vout: the
// streamed sort's output
__global__ __launch_bounds__(kTB) void bucket_compact(VoxelJobDev A, VoxelJobDev B, BucketSrc S,
                                                      uint32_t* __restrict__ kin,
                                                      int* __restrict__ vin, uint32_t* __restrict__ kout,
                                                      int* __restrict__ vout, const unsigned* __restrict__ hist,
                                                      const int* __restrict__ overflow,
                                                      unsigned long long* __restrict__ status,
                                                      const unsigned* __restrict__ radix_ctl,
                                                      const int* __restrict__ gate,
                                                      unsigned long long* __restrict__ split,
                                                      const int* __restrict__ geo, unsigned* __restrict__ ticket,
                                                      int stamps) {
  const unsigned long long T0 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // the bucket is the block's ticket (zeroed by vox_keys): a bucket's lookback only waits on buckets that are already
  // running (HIP promises no dispatch order).  Prologue loads together with it: gate, the clouds' counts, the
  // overflow flags and this thread's histogram word (bucket_range)
  __shared__ int s_b;
  if (t == 0) s_b = (int)atomicAdd(ticket, 1u);
  const int gv = gate ? *gate : 1;
  const int nA0 = *A.d_n0, nA1 = A.d_n1 ? *A.d_n1 : 0, nB0 = *B.d_n0, nB1 = B.d_n1 ? *B.d_n1 : 0;
  const int ovf0 = overflow[0], ovf1 = overflow[1];   // (no two-element arrays indexed by a run-time job: scratch)
  const unsigned hw0 = hist[t];                        // (kTB == kBuckets)
  const int novf = (int)hist[kBucketOvfWord];
  __syncthreads();
  const int b = s_b;
  if (!gv) {   // gated off (no keyframe): the output is the unchanged first part (the map).  By block index: no
    // lookback here, and the ticket counter is zeroed only by an ungated vox_keys
    const int bi = (int)blockIdx.x;
    for (int job = 0; job < 2; ++job) {
      const VoxelJobDev& J = job == 0 ? A : B;
      const int n0 = job ? nB0 : nA0;
      for (int i = bi * kTB + t; i < n0; i += gridDim.x * kTB) J.out[i] = J.part0[i];
      if (bi == 0 && t == 0) *J.d_out = n0;
    }
    return;
  }
  __shared__ union {
    CompactLds c;
    StreamLds st;
  } U;
  CompactLds& L = U.c;
  const BucketRange R = bucket_range(hw0, b, L.tmp);
  const int start = R.start, size = R.size;
  if (b == kBuckets - 1 || size == 0) {   // nothing to emit: publish zero; the last bucket ends the outputs
    const Prefix2 pre = lookback_prefix(status, b, Prefix2{0, 0});
    if (b == kBuckets - 1 && t == 0) {
      const bool failed = pre.a < 0 || radix_ctl[kRadixErrorWord] != 0u;   // a lookback timed out (never)
      *A.d_out = failed ? -1 : pre.a;
      *B.d_out = failed ? -1 : pre.b;
    }
    return;
  }
  const bool streamed = size > kBucketCap;   // (block-uniform)
  const unsigned long long* src = bucket_source(S, b, start, size, novf);
  if (streamed) {
    unpack_bucket(src, size, kin + start, vin + start);
    stream_sort(kin + start, vin + start, kout + start, vout + start, size, U.st);
  } else {
    by_size(size, [&](auto EC) {
      constexpr int E = decltype(EC)::value;
      bucket_bitonic<E>(src, size, L.u.x, L.k, L.v);
    });
  }
  const unsigned long long T1 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // the bucket's heads per cloud -> its output range (lookback over the buckets)
  int hc[2];
  if (!streamed) {
    chunk_heads(L.k, size, 0u, true, hc);
  } else {
    hc[0] = hc[1] = 0;
    for (int e = t; e < size; e += kTB) {
      const uint32_t k = kout[start + e];
      if (e == 0 || k != kout[start + e - 1]) {
        const int j = (int)(k >> 31);
        hc[0] += 1 - j;
        hc[1] += j;
      }
    }
  }
  block_sum2(hc, L.hw);
  const unsigned long long T2 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const Prefix2 pre = lookback_prefix(status, b, Prefix2{hc[0], hc[1]});
  if (pre.a < 0) return;   // (timed out, never expected: bucket 255 reports it)
  const unsigned long long T3 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  unsigned long long Tg = T3, Th = T3, Te = T3;   // (stamps: gather done, heads scanned, emit loop done)
  if (streamed) write_splitters(split, geo, R.kept, start, size, [&](int q) { return kout[start + q]; });
  else write_splitters(split, geo, R.kept, start, size, [&](int q) { return L.k[q]; });
  int run_base[2] = {pre.a, pre.b};   // output slot of the next head, per cloud
  if (t == 0) L.carry_pos = -1;
  for (int c0 = 0; c0 < size; c0 += kBucketCap) {
    const int nc = min(kBucketCap, size - c0);
    __syncthreads();
    if (streamed) {
      for (int e = t; e < nc; e += kTB) {
        L.k[e] = kout[start + c0 + e];
        L.v[e] = vout[start + c0 + e];
      }
      __syncthreads();
    }
    // every element's point: kGather elements per thread with all their loads in flight before any is used (one
    // memory round trip for a bucket of up to kGather x 256, not one per 256)
    constexpr int kGather = 4;
    for (int g0 = 0; g0 < nc; g0 += kGather * kTB) {
      float4 lo[kGather], hi[kGather];
#pragma unroll
      for (int u = 0; u < kGather; ++u) {
        const int e = g0 + u * kTB + t;
        lo[u] = hi[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < nc) {
          if (L.k[e] >> 31) vox_fetch_halves(B, nB0, nB1, L.v[e], lo[u], hi[u]);
          else vox_fetch_halves(A, nA0, nA1, L.v[e], lo[u], hi[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < kGather; ++u) {
        const int e = g0 + u * kTB + t;
        if (e < nc) L.u.pt[e] = make_float4(lo[u].x, lo[u].y, lo[u].z, hi[u].x);   // x, y, z, intensity
      }
    }
    const uint32_t prev = c0 ? L.prev_key : 0u;
    __syncthreads();
    // the run carried over from the previous chunk (streamed buckets only), continued in order by thread 0
    if (t == 0 && L.carry_pos >= 0) {
      float s0 = L.carry[0], s1 = L.carry[1], s2 = L.carry[2], s3 = L.carry[3];
      int n = L.carry_n, e = 0;
      for (; e < nc && L.k[e] == L.carry_key; ++e) {
        const float4 q = L.u.pt[e];
        s0 += q.x; s1 += q.y; s2 += q.z; s3 += q.w;
        ++n;
      }
      if (e < nc) {   // it ends here
        (L.carry_job ? B : A).out[L.carry_pos] = centroid_out(s0, s1, s2, s3, n);
        L.carry_pos = -1;
      } else {
        L.carry[0] = s0; L.carry[1] = s1; L.carry[2] = s2; L.carry[3] = s3;
        L.carry_n = n;
      }
    }
    if (stamps) Tg = __builtin_amdgcn_s_memrealtime();   // (gather + carry done)
    // this thread's heads in its contiguous range; slots by a block scan of the per-thread counts (element order)
    int c[2];
    chunk_heads(L.k, nc, prev, c0 == 0, c);
    int inc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      int v = c[j];
      v = wave_incl_scan(v);   // (DPP, floam_common.hpp)
      inc[j] = v;
    }
    __syncthreads();   // (the carry above is done before a head below may start a new one)
    if (lane == 63) { L.hw[0][w] = (unsigned)inc[0]; L.hw[1][w] = (unsigned)inc[1]; }
    __syncthreads();
    int pos[2] = {run_base[0], run_base[1]}, tot[2] = {0, 0};
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int k = 0; k < kW; ++k) {
        if (k < w) pos[j] += (int)L.hw[j][k];
        tot[j] += (int)L.hw[j][k];
      }
    pos[0] += inc[0] - c[0];
    pos[1] += inc[1] - c[1];
    int pos0 = pos[0], pos1 = pos[1];   // the next output slot per cloud (selected by job below, never indexed)
    int e0, e1;
    thread_range(nc, e0, e1);
    if (stamps) Th = __builtin_amdgcn_s_memrealtime();
    for (int e = e0; e < e1; ++e) {
      const uint32_t key = L.k[e];
      const uint32_t kp = e ? L.k[e - 1] : prev;
      if (!((e == 0 && c0 == 0) || key != kp)) continue;
      const int job = (int)(key >> 31);
      const VoxelJobDev& J = job ? B : A;
      const int slot = job ? pos1 : pos0;
      if (job) ++pos1; else ++pos0;
      if (job ? ovf1 : ovf0) {   // index overflow: the input returned unchanged (Q9; identity keys: runs of one)
        PointRec o;
        vox_fetch(J, job ? nB0 : nA0, job ? nB1 : nA1, L.v[e], o);
        J.out[slot] = o;
        continue;
      }
      const float4 f = L.u.pt[e];
      float s0 = f.x, s1 = f.y, s2 = f.z, s3 = f.w;
      int j = e + 1;
      // The run's points in groups of 8 keys + 8 points per LDS round trip, double-buffered: the next group's loads are
      // issued before this group's additions, so long runs (dense voxels near the sensor) stream at the rate of the
      // in-order adds, not of one LDS round trip per group.  Keys ascend within the chunk, so a group whose last key is
      // still this voxel's is the voxel's throughout: its 8 additions run without a test or a select (the dependent
      // adds alone); only the run's last group tests each key.  Look-ahead reads past the chunk's end land in the
      // arrays' padding (kRunPad) and are never used.  (Two buffers unrolled by hand: no register moves per group.)
      constexpr int G = 8;
      static_assert(2 * G - 1 <= kRunPad, "the look-ahead (up to 2 G - 1 past a run end <= nc) stays in the padding");
      uint32_t ka[G], kb[G];
      float4 pa[G], pb[G];
      auto load = [&](uint32_t(&kk)[G], float4(&pp)[G], int at) {
#pragma unroll
        for (int q = 0; q < G; ++q) {
          kk[q] = L.k[at + q];
          pp[q] = L.u.pt[at + q];
        }
      };
      auto add_full = [&](const float4(&pp)[G]) {
#pragma unroll
        for (int q = 0; q < G; ++q) {
          s0 += pp[q].x; s1 += pp[q].y; s2 += pp[q].z; s3 += pp[q].w;
        }
        j += G;
      };
      auto add_tail = [&](const uint32_t(&kk)[G], const float4(&pp)[G]) {
        bool more = true;
#pragma unroll
        for (int q = 0; q < G; ++q) {
          if (more && j < nc && kk[q] == key) {
            s0 += pp[q].x; s1 += pp[q].y; s2 += pp[q].z; s3 += pp[q].w;
            ++j;
          } else {
            more = false;
          }
        }
      };
      load(ka, pa, j);
      for (;;) {
        load(kb, pb, j + G);
        if (!(j + G <= nc && ka[G - 1] == key)) { add_tail(ka, pa); break; }
        add_full(pa);
        load(ka, pa, j + G);
        if (!(j + G <= nc && kb[G - 1] == key)) { add_tail(kb, pb); break; }
        add_full(pb);
      }
      if (j == nc && streamed && c0 + nc < size) {   // reaches the chunk end of a streamed bucket: carried over
        L.carry[0] = s0; L.carry[1] = s1; L.carry[2] = s2; L.carry[3] = s3;
        L.carry_n = j - e;
        L.carry_pos = slot;
        L.carry_job = job;
        L.carry_key = key;
        continue;
      }
      {   // VoxelGrid's output record as two 16-B stores: x, y, z, 1 | intensity, ring 0 + pad, time 0, 0
        const float cn = (float)(j - e);
        float4* o = reinterpret_cast<float4*>(J.out + slot);
        o[0] = make_float4(s0 / cn, s1 / cn, s2 / cn, 1.0f);
        o[1] = make_float4(s3 / cn, 0.0f, 0.0f, 0.0f);
      }
    }
    run_base[0] += tot[0];
    run_base[1] += tot[1];
    __syncthreads();
    if (stamps) Te = __builtin_amdgcn_s_memrealtime();
    if (t == 0) L.prev_key = L.k[nc - 1];
  }
  __syncthreads();
  if (t == 0 && L.carry_pos >= 0)   // (a streamed bucket whose last run reached its end)
    (L.carry_job ? B : A).out[L.carry_pos] = centroid_out(L.carry[0], L.carry[1], L.carry[2], L.carry[3], L.carry_n);
  if (stamps) {   // plain per-bucket records (start, sort, heads + sum, lookback, gather + emit + drain)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      unsigned* q = g_bc_st[stamps - 1][b];
      q[0] = (unsigned)T0; q[1] = (unsigned)(T1 - T0); q[2] = (unsigned)(T2 - T1); q[3] = (unsigned)(T3 - T2);
      q[4] = (unsigned)(__builtin_amdgcn_s_memrealtime() - T3);
      q[5] = (unsigned)(Tg - T3); q[6] = (unsigned)(Th - Tg); q[7] = (unsigned)(Te - Th);
    }
  }
}

// ---------------------------------------------------------------------------------------------- seeding
// the first splitters of a pipeline from a digit-pass sort's output (sorted keys, dropped ones last)
__global__ __launch_bounds__(kTB) void bucket_seed(const uint32_t* __restrict__ k0, const int* __restrict__ n_dev,
                                                   int n_host, const int* __restrict__ gate,
                                                   unsigned long long* __restrict__ split,
                                                   const int* __restrict__ geo) {
  if (gate && !*gate) return;
  const int n = n_dev ? min(*n_dev, n_host) : n_host;
  __shared__ int s_kept;   // the first dropped key's position (binary search, one thread)
  if (threadIdx.x == 0) {
    int lo = 0, hi = n;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (k0[mid] != 0xFFFFFFFFu) lo = mid + 1; else hi = mid;
    }
    s_kept = lo;
  }
  __syncthreads();
  write_splitters(split, geo, s_kept, 0, s_kept, [&](int q) { return k0[q]; });
}

}  // namespace

void BucketScratch::reserve(int n, hipStream_t st) {
  if (!split.p) {
    split.reserve(kSplitters);
    geo.reserve(kGeoWords);
    FLOAM_HIP(hipMemsetAsync(geo.p, 0, sizeof(int) * kGeoWords, st));
  }
  n = std::max(n, 1);
  cap = std::max(cap, bucket_cap(n));   // (only grows: a region sized for more elements serves fewer)
  reg.reserve((size_t)kBuckets * cap);
  ovf.reserve((size_t)n);
  ovf_b.reserve((size_t)n);
  gath.reserve((size_t)n);
}

BucketDev bucket_dev(BucketScratch& bs, int n, hipStream_t st) {
  bs.reserve(n, st);
  return BucketDev{bs.seeded ? bs.split.p : nullptr, bs.geo.p, bs.reg.p, bs.ovf.p, bs.ovf_b.p, bs.cap,
                   (int)std::min<size_t>(bs.ovf.cap, (size_t)INT_MAX)};
}

bool bucket_sort_enabled(int pipeline) {
  // FLOAM_SORT: radix (the four digit passes everywhere), merge (the bucket sort in the map merge only), bucket (both
  // pipelines; the default: r4d, 1914-1918 scans/s against 1800 merge-only and 1691-1706 radix, one box)
  static const int mask = [] {
    const char* e = FLOAM_DIAG_ENV("FLOAM_SORT");
    if (e && e[0] == 'r') return 0;
    if (e && e[0] == 'm') return 2;
    return 3;
  }();
  return (mask >> pipeline) & 1;
}

void bucket_voxel_launch(BucketScratch& bs, RadixScratch& rs, const VoxelJobDev& A, const VoxelJobDev& B, uint32_t* k0,
                         int* v0, uint32_t* k1, int* v1, int n, const int* overflow, unsigned long long* status,
                         unsigned* ticket, hipStream_t st, const int* gate, const int* n_dev) {
  if (n <= 0) return;
  bs.reserve(n, st);
  rs.reserve(n, st);
  static const bool stamps = FLOAM_DIAG_ENV("FLOAM_BC_STAMPS") != nullptr;
  static unsigned launches = 0;
  hipLaunchKernelGGL(bucket_compact, dim3(kBuckets), dim3(kTB), 0, st, A, B, bucket_src(bs), k1, v1, k0, v0, rs.ctl.p,
                     overflow,
                     status, rs.ctl.p, gate, bs.split.p, bs.geo.p, ticket,
                     stamps ? (int)(launches++ & 1u) + 1 : 0);
  FLOAM_LAUNCH_CHECK();
}

void bucket_stamps_print() {
  if (!FLOAM_DIAG_ENV("FLOAM_BC_STAMPS")) return;
  static unsigned q[2][kBuckets][8];
  FLOAM_HIP(hipDeviceSynchronize());
  FLOAM_HIP(hipMemcpyFromSymbol(q, HIP_SYMBOL(g_bc_st), sizeof(q)));
  for (int sl = 0; sl < 2; ++sl) {
    int nb = 0, smin = 0, emax = 0, worst = 0, worst_end = 0;
    double ph[4] = {0, 0, 0, 0}, mx[4] = {0, 0, 0, 0}, sub[3] = {0, 0, 0};
    for (int b = 0; b < kBuckets; ++b) {
      if (q[sl][b][1] == 0 && q[sl][b][4] == 0) continue;
      ++nb;
      for (int k = 0; k < 3; ++k) sub[k] += q[sl][b][5 + k];
      for (int k = 0; k < 4; ++k) {
        ph[k] += q[sl][b][1 + k];
        mx[k] = std::max(mx[k], (double)q[sl][b][1 + k]);
      }
      const int st = (int)(q[sl][b][0] - q[sl][0][0]);
      const int end = st + (int)(q[sl][b][1] + q[sl][b][2] + q[sl][b][3] + q[sl][b][4]);
      smin = std::min(smin, st);
      if (end > emax) { emax = end; worst = b; worst_end = end; }
    }
    if (!nb) continue;
    std::fprintf(stderr, "[bc stamps] launch slot %d (%s), %d buckets: sort %.2f (max %.2f), heads + sum %.2f (max "
                 "%.2f), lookback %.2f (max %.2f), gather + emit + drain %.2f (max %.2f) us; first start -> last end "
                 "%.2f us (bucket %d: start +%.2f)\n", sl, sl ? "call 2, main stream" : "call 1, side stream", nb,
                 ph[0] / nb / 100.0, mx[0] / 100.0, ph[1] / nb / 100.0, mx[1] / 100.0, ph[2] / nb / 100.0, mx[2] / 100.0,
                 ph[3] / nb / 100.0, mx[3] / 100.0, (emax - smin) / 100.0, worst,
                 (int)(q[sl][worst][0] - q[sl][0][0]) / 100.0);
    (void)worst_end;
    std::fprintf(stderr, "[bc stamps]   slot %d gather + emit: gather %.2f, heads + scans %.2f, emit loop + barrier %.2f, "
                 "drain %.2f us (means)\n", sl, sub[0] / nb / 100.0, sub[1] / nb / 100.0, sub[2] / nb / 100.0,
                 (ph[3] - sub[0] - sub[1] - sub[2]) / nb / 100.0);
  }
}

void bucket_sort_launch(BucketScratch& bs, RadixScratch& rs, uint32_t* k0, int* v0, uint32_t* k1, int* v1, int n,
                        hipStream_t st, const int* gate) {
  if (n <= 0) return;
  bs.reserve(n, st);
  rs.reserve(n, st);
  hipLaunchKernelGGL(bucket_sort, dim3(kBuckets), dim3(kTB), 0, st, bucket_src(bs), k1, v1, k0, v0, rs.ctl.p, gate,
                     bs.split.p, bs.geo.p);
  FLOAM_LAUNCH_CHECK();
}

void bucket_seed_launch(BucketScratch& bs, const uint32_t* k0, const int* n_dev, int n, hipStream_t st,
                        const int* gate) {
  if (n <= 0) return;
  hipLaunchKernelGGL(bucket_seed, dim3(1), dim3(kTB), 0, st, k0, n_dev, n, gate, bs.split.p, bs.geo.p);
  FLOAM_LAUNCH_CHECK();
  bs.seeded = true;
}

}  // namespace floam
