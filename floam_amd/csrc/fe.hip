// Feature extraction on gfx950: LaserProcessingClass::featureExtraction (src/laserProcessingClass.cpp:72-231).
//
// Kernels (one scan, P points, R rings):
//   fe_keys     grid over P     range filter + ring key + per-ring histogram + the radix digit histograms
//   radix_pass  grid over P     stable bucketing by ring: ONE digit pass of the onesweep radix sort (radix.hip) for
//                               R <= 255 rings, O(P), which stages the scan ring-major as it goes: every point's
//                               coordinates (16 B) and record (32 B) written once to its ring-major slot (more rings:
//                               two key-only passes, then fe_stage gathers by the ring-ordered indices)
//   fe_sector   one WG / sector curvature stencil over the contiguous ring-major coordinates, LDS bitonic
//                               sort (block barriers only around the strides that cross waves), wave-parallel
//                               greedy edge pick, surf compaction
//   fe_output   one WG / sector copy the 32-B ring-major records of edges / surfs to their sector-major slots; the
//                               last block to finish advances the output counts (the commit)
// Arithmetic follows the reference bit for bit: float stencil sums in source order, double squares, no FMA
// contraction (built with -ffp-contract=off).  Sorting is by (value, ring index), which equals the reference's
// unstable std::sort whenever a sector has no tied curvature values (SURVEY.md §7 "Hard parts").
#include <vector>

#include "floam_common.hpp"
#include "fe.hpp"
#include "profwb.hpp"
#include "radix.hpp"

namespace floam {

// FLOAM_FE_STAMPS=1 (diagnostic): fe_sector's per-block phase times (100 MHz ticks): [0] staging, [1] curvature +
// sort, [2] greedy pick, [3] surf compaction + writes, [4] blocks, [5] sum of launch spans, [6] launches
__device__ unsigned long long g_fe_stamps[8 + 3 * 1024];   // + per launch: first start, last start, last end
__device__ unsigned g_fe_sec[1024][12];   // per sector, the last launch: m, phases (10-ns ticks), start vs first

namespace {

constexpr int kSectorThreads = 256;   // fe_output
// fe_sector's block (128 threads measured slower: 32 vs 25 us from the first block's start to the last one's end)
constexpr int kSortThreads = 256;
constexpr int kMaxEdgesPerSector = 20;

__device__ __forceinline__ PointRec make_out(const PointRec& p) {
  PointRec o;
  o.x = p.x; o.y = p.y; o.z = p.z; o.pad0 = 1.0f;
  o.intensity = p.intensity;
  o.ring = p.ring; o.pad1 = 0;
  o.time = p.time; o.pad2 = 0.0f;
  return o;
}

// RingExtractionVelodyne (src/laserProcessingClass.cpp:11-22): float x*x+y*y, float sqrt, double compare.  Keys for
// the stable bucketing sort: the ring, or 0xFFFF for a dropped point (sorted after every ring); values: the index.
// ONE_DIGIT (R <= 255 rings, one bucketing pass): the per-ring counts ARE the pass's digit histogram (a dropped
// point's low digit 0xFF is no ring), so one 256-bin LDS histogram serves both; otherwise the ring histogram and
// the four digit histograms separately.
template <bool ONE_DIGIT>
__global__ void fe_keys(const PointRec* __restrict__ in, int n, int num_lines, double min_d, double max_d,
                        uint32_t* __restrict__ keys, int* __restrict__ vals, int* __restrict__ ring_count,
                        int* __restrict__ status, unsigned* __restrict__ radix_ctl) {
  extern __shared__ int hist[];
  __shared__ unsigned s_rhist[ONE_DIGIT ? kRadixDigits : kRadixHistWords];
  if (ONE_DIGIT) {
    for (int k = threadIdx.x; k < kRadixDigits; k += blockDim.x) s_rhist[k] = 0u;
    __syncthreads();
  } else {
    for (int r = threadIdx.x; r < num_lines; r += blockDim.x) hist[r] = 0;
    radix_hist_begin(s_rhist);
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float2 xy = *reinterpret_cast<const float2*>(&in[i].x);
    const uint16_t ring = in[i].ring;
    const float d2 = xy.x * xy.x + xy.y * xy.y;
    const double d = (double)sqrtf(d2);
    bool keep = !(d < min_d || d > max_d);
    if (keep && ring >= num_lines) {   // reference: vector index out of bounds (UB)
      atomicOr(status, FE_STATUS_BAD_RING);
      keep = false;
    }
    const uint32_t key = keep ? ring : 0xFFFFu;
    keys[i] = key;
    if (ONE_DIGIT) {
      atomicAdd(&s_rhist[key & 255u], 1u);
    } else {
      vals[i] = i;
      radix_hist_add(s_rhist, key);
      if (keep) atomicAdd(&hist[ring], 1);
    }
  }
  if (ONE_DIGIT) {
    __syncthreads();
    for (int k = threadIdx.x; k < kRadixDigits; k += blockDim.x) {
      const unsigned v = s_rhist[k];
      if (v) {
        atomicAdd(&radix_ctl[k], v);   // pass 0's digit histogram
        if (k < num_lines) atomicAdd(&ring_count[k], (int)v);
      }
    }
  } else {
    radix_hist_end(s_rhist, radix_ctl);
    __syncthreads();
    for (int r = threadIdx.x; r < num_lines; r += blockDim.x)
      if (hist[r]) atomicAdd(&ring_count[r], hist[r]);
  }
}

__device__ __forceinline__ int block_exclusive_scan_1024(int v, int* smem /* >= 32 ints */, int* total) {
  // wave-level inclusive scan then cross-wave scan; blockDim.x <= 1024, wave = 64
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) smem[wid] = x;
  __syncthreads();
  const int nw = (blockDim.x + 63) >> 6;
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int w = 0; w < nw; ++w) {
      const int t = smem[w];
      smem[w] = acc;
      acc += t;
    }
    smem[32] = acc;
  }
  __syncthreads();
  const int excl = smem[wid] + x - v;
  *total = smem[32];
  __syncthreads();
  return excl;
}

// points in rings [0, r): the first wave loads the counts together (one round trip, not one per ring) and sums
// them in a fixed order; called by every thread, the result in every thread (one block barrier)
__device__ __forceinline__ int ring_offset(const int* ring_count, int r, int* s_red) {
  if (threadIdx.x < 64) {
    int v = 0;
    for (int k = threadIdx.x; k < r; k += 64) v += ring_count[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (threadIdx.x == 0) *s_red = v;
  }
  __syncthreads();
  return *s_red;
}

__device__ __forceinline__ void sector_range(int n_r, int s, int& a, int& b) {
  // src/laserProcessingClass.cpp:103-110: T = n - 10, L = T / 6, [L*s, L*(s+1) - 1), last: [5L, T - 1)
  const int T = n_r - 10;
  const int L = T / 6;
  a = L * s;
  b = (s == 5) ? T - 1 : L * (s + 1) - 1;
}

// ---- register bitonic sort of a sector's entries by (curvature, entry): the network sorts one 32-bit word per entry,
// the top 21 bits of the curvature's bit pattern above the 11-bit entry (unique words: a compare-exchange is one
// min / max), N = kSortThreads E words, E per thread (position p = E t + e), every stage's stride a compile-time
// constant, so a lane exchange inside a wave is one ds_swizzle (xor of the lane bits, no memory) or, across the wave
// halves, one ds_bpermute; only strides >= 64 E go through LDS.  Entries whose prefixes tie are then re-ordered by
// their full value (rare, short runs).
template <int M>
__device__ __forceinline__ unsigned xor_lane(unsigned v) {
  if constexpr (M < 32) return (unsigned)__builtin_amdgcn_ds_swizzle((int)v, (M << 10) | 0x1F);   // bitmask mode
  else return (unsigned)__builtin_amdgcn_ds_bpermute((int)((((threadIdx.x & 63) ^ M)) << 2), (int)v);
}

// one stage (size, stride) of the network on the thread's E words
template <int E, int SIZE, int STRIDE>
__device__ __forceinline__ void bitonic_stage(unsigned (&k)[E], unsigned* s_pk) {
  const int t = threadIdx.x;
  unsigned ok[E];
  if constexpr (STRIDE < E) {
#pragma unroll
    for (int e = 0; e < E; ++e) ok[e] = k[e ^ STRIDE];
  } else if constexpr (STRIDE < 64 * E) {
#pragma unroll
    for (int e = 0; e < E; ++e) ok[e] = xor_lane<STRIDE / E>(k[e]);
  } else {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) s_pk[E * t + e] = k[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E; ++e) ok[e] = s_pk[(E * t + e) ^ STRIDE];
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int pp = E * t + e;
    const bool lower = (pp & STRIDE) == 0, asc = (pp & SIZE) == 0;
    // the lower slot of an ascending pair keeps the smaller, and so on
    k[e] = asc == lower ? min(k[e], ok[e]) : max(k[e], ok[e]);
  }
}
template <int E, int SIZE, int STRIDE>
__device__ __forceinline__ void bitonic_strides(unsigned (&k)[E], unsigned* s_pk) {
  bitonic_stage<E, SIZE, STRIDE>(k, s_pk);
  if constexpr (STRIDE > 1) bitonic_strides<E, SIZE, STRIDE / 2>(k, s_pk);
}
template <int E, int SIZE>
__device__ __forceinline__ void bitonic_sizes(unsigned (&k)[E], unsigned* s_pk) {
  bitonic_strides<E, SIZE, SIZE / 2>(k, s_pk);
  if constexpr (SIZE < kSortThreads * E) bitonic_sizes<E, SIZE * 2>(k, s_pk);
}
// the m curvature values (entries 0..m-1 <= 1024): s_key[q] = the value of entry q, s_id = the entries in ascending
// (value, entry) order
template <int E, typename Curv>
__device__ __forceinline__ void sector_sort(int m, Curv curvature, unsigned long long* s_key, uint16_t* s_id,
                                            unsigned* s_pk) {
  unsigned k[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int q = E * threadIdx.x + e;
    if (q < m) {
      const unsigned long long v = curvature(q);   // v >= +0 (bit 63 clear): 21 bits below it
      s_key[q] = v;
      k[e] = (unsigned)(v >> 42) << 11 | (unsigned)q;   // < 0xFFFFFFFF: the padding sorts last
    } else {
      k[e] = ~0u;
    }
  }
  bitonic_sizes<E, 2>(k, s_pk);
  __syncthreads();
#pragma unroll
  for (int e = 0; e < E; ++e) s_pk[E * threadIdx.x + e] = k[e];
  __syncthreads();
  // a position that starts a prefix (its predecessor's differs) writes its entry; if its successors share the
  // prefix, it orders that run by (value, entry) — insertion sort, a run of tied prefixes being short and rare
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int p = E * threadIdx.x + e;
    if (p >= m) continue;
    const unsigned pre = k[e] >> 11;
    if (p > 0 && (s_pk[p - 1] >> 11) == pre) continue;   // inside a run: its first position orders it
    if (p + 1 < m && (s_pk[p + 1] >> 11) == pre) {
      int end = p + 2;
      while (end < m && (s_pk[end] >> 11) == pre) ++end;
      for (int i = p; i < end; ++i) {
        const int q = (int)(s_pk[i] & 0x7FFu);
        const unsigned long long v = s_key[q];
        int j = i;
        while (j > p) {
          const int qj = s_id[j - 1];
          const unsigned long long vj = s_key[qj];
          if (vj < v || (vj == v && qj < q)) break;
          s_id[j] = (uint16_t)qj;
          --j;
        }
        s_id[j] = (uint16_t)q;
      }
    } else {
      s_id[p] = (uint16_t)(k[e] & 0x7FFu);
    }
  }
}

// Sectors with MINSEC < m <= MAXSEC are processed; the small-LDS instantiation runs first and the large one only
// picks up the (rare) longer sectors, so the common case keeps several workgroups per CU.
template <int MINSEC, int MAXSEC, bool LAST>
__device__ __forceinline__ void fe_sector_body(int sec, const int* __restrict__ ring_count,
                                               const float4* __restrict__ ring_xyz, int* __restrict__ sec_edge_cnt,
                                               int* __restrict__ sec_edge_pos, int* __restrict__ sec_surf_cnt,
                                               int* __restrict__ surf_pos, int* __restrict__ status, int stamps,
                                               int* __restrict__ long_list, int* __restrict__ long_count) {
  const unsigned long long T0 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  constexpr int kPts = MAXSEC + 10;
  __shared__ unsigned long long s_key[MAXSEC];
  __shared__ uint16_t s_id[MAXSEC];      // ring index - a - 5 (the curvature entry offset)
  __shared__ unsigned s_pk[MAXSEC <= 1024 ? MAXSEC : 1];   // the register network's LDS exchanges
  __shared__ float s_x[kPts], s_y[kPts], s_z[kPts];
  __shared__ uint8_t s_picked[kPts];
  __shared__ unsigned s_gapw[(kPts + 63) / 64 * 2];   // bit j: points j and j + 1 farther apart than 0.05 (sq.)
  __shared__ int s_edges[kMaxEdgesPerSector];
  __shared__ int s_nedge;
  __shared__ int smem[33];
  __shared__ int s_off;

  const int r = sec / 6, s = sec % 6;
  const int n_r = ring_count[r];
  if (n_r < 131) {                                    // :89
    if (MINSEC == 0 && threadIdx.x == 0) { sec_edge_cnt[sec] = 0; sec_surf_cnt[sec] = 0; }
    return;
  }
  int a, b;
  sector_range(n_r, s, a, b);
  const int m = b - a;
  if (m <= MINSEC) return;
  if (m > MAXSEC) {
    if (LAST && threadIdx.x == 0) {
      atomicOr(status, FE_STATUS_SECTOR_TOO_LONG);
      sec_edge_cnt[sec] = 0;
      sec_surf_cnt[sec] = 0;
    }
    if (!LAST && long_list && threadIdx.x == 0) long_list[atomicAdd(long_count, 1)] = sec;   // for fe_sector_long
    return;
  }
  const int off = ring_offset(ring_count, r, &s_off);
  // stage ring points [a, b + 10) (= ids a..b+9: stencils of entries a..b-1 and all suppression neighbours)
  const int npts = m + 10;
  for (int k = threadIdx.x; k < npts; k += blockDim.x) {   // contiguous ring-major coordinates
    const float4 p = ring_xyz[off + a + k];
    s_x[k] = p.x; s_y[k] = p.y; s_z[k] = p.z;
    s_picked[k] = 0;
  }
  __syncthreads();
  const unsigned long long T1 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // the reference's neighbour test (:151-166) between consecutive points, once per pair, as a bitmask: float
  // differences, double squares (the left-side test of a pair computes the same numbers negated: the same result)
  for (int j0 = (threadIdx.x & ~63); j0 < npts; j0 += blockDim.x) {   // (wave-uniform: a word pair per wave)
    const int j = j0 + (threadIdx.x & 63);
    bool gap = false;
    if (j + 1 < npts) {
      const double dX = s_x[j + 1] - s_x[j];
      const double dY = s_y[j + 1] - s_y[j];
      const double dZ = s_z[j + 1] - s_z[j];
      gap = dX * dX + dY * dY + dZ * dZ > 0.05;
    }
    const unsigned long long b = __ballot(gap);
    if ((threadIdx.x & 63) == 0) {
      s_gapw[j0 >> 5] = (unsigned)b;
      s_gapw[(j0 >> 5) + 1] = (unsigned)(b >> 32);
    }
  }
  // curvature (src/laserProcessingClass.cpp:95-101), entry e = a + k, point j = e + 5 -> local k + 5
  auto curvature = [&](int k) -> unsigned long long {
    const int c = k + 5;
    const float fx = s_x[c - 5] + s_x[c - 4] + s_x[c - 3] + s_x[c - 2] + s_x[c - 1] - 10 * s_x[c] + s_x[c + 1] +
                     s_x[c + 2] + s_x[c + 3] + s_x[c + 4] + s_x[c + 5];
    const float fy = s_y[c - 5] + s_y[c - 4] + s_y[c - 3] + s_y[c - 2] + s_y[c - 1] - 10 * s_y[c] + s_y[c + 1] +
                     s_y[c + 2] + s_y[c + 3] + s_y[c + 4] + s_y[c + 5];
    const float fz = s_z[c - 5] + s_z[c - 4] + s_z[c - 3] + s_z[c - 2] + s_z[c - 1] - 10 * s_z[c] + s_z[c + 1] +
                     s_z[c + 2] + s_z[c + 3] + s_z[c + 4] + s_z[c + 5];
    const double dX = fx, dY = fy, dZ = fz;
    const double v = dX * dX + dY * dY + dZ * dZ;
    return (unsigned long long)__double_as_longlong(v);   // v >= +0: the bit pattern is order-preserving
  };
  // s_key by entry (the register network) or by sorted position (the LDS network)
  const bool by_entry = MAXSEC <= 1024 && m <= 1024;
  if (by_entry) {   // (block-uniform) the register network, E = 1, 2 or 4 entries a thread
    if (m <= kSortThreads) sector_sort<1>(m, curvature, s_key, s_id, s_pk);
    else if (m <= 2 * kSortThreads) sector_sort<2>(m, curvature, s_key, s_id, s_pk);
    else sector_sort<4>(m, curvature, s_key, s_id, s_pk);
  } else {   // longer sectors (the 4096 instantiation): the network in LDS
    int P2 = 1;
    while (P2 < m) P2 <<= 1;
    for (int k = threadIdx.x; k < P2; k += blockDim.x) {
      if (k < m) {
        s_key[k] = curvature(k);
        s_id[k] = (uint16_t)k;
      } else {
        s_key[k] = ~0ull;
        s_id[k] = 0xFFFF;
      }
    }
    __syncthreads();
    // bitonic sort ascending by (key, id).  A stage with stride <= 64 pairs positions inside one 128-entry chunk,
    // and every chunk belongs to one wave (thread t's pairs lie in chunk t / 64 and t / 64 + 4, ...): those stages
    // need only the wave's own LDS ordering; block barriers surround the stages with longer strides
    for (int size = 2; size <= P2; size <<= 1) {
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        if (stride >= 128) __syncthreads();
        for (int t = threadIdx.x; t < (P2 >> 1); t += blockDim.x) {
          const int lo = 2 * t - (t & (stride - 1));
          const int hi = lo + stride;
          const bool up = ((lo & size) == 0);
          const unsigned long long ka = s_key[lo], kb = s_key[hi];
          const uint16_t ia = s_id[lo], ib = s_id[hi];
          const bool gt = (ka > kb) || (ka == kb && ia > ib);
          if (gt == up) {
            s_key[lo] = kb; s_key[hi] = ka;
            s_id[lo] = ib; s_id[hi] = ia;
          }
        }
        if (stride >= 128) {   // (its pairs crossed chunks: the next stage's chunks were written by other waves)
          __syncthreads();
        } else {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
    }
  }
  __syncthreads();
  const unsigned long long T2 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // greedy edge pick (src/laserProcessingClass.cpp:129-170) by wave 0: the candidates in descending order, 64 at a
  // time (lane order = the reference's order).  Per chunk every lane reads whether its point was picked by an earlier
  // chunk; then, pick by pick, the first unsuppressed lane is the next candidate the reference examines (the ones
  // before it are skipped as picked): its curvature ends the loop at <= 0.1, otherwise it is picked, its +-5
  // neighbour runs (every lane's, from the pair-gap bitmask at the chunk's start: one read-lane on the pick's chain),
  // and its picked run is marked in LDS and in the chunk's suppression mask.  One step per pick, not per candidate.
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int picked_num = 0, nedge = 0;
    bool stop = false;
    for (int c0 = m - 1; c0 >= 0 && !stop; c0 -= 64) {   // (wave-uniform)
      const int i = c0 - lane;
      const bool valid = i >= 0;
      int ind = 0;
      bool over = false;   // not curvature <= 0.1 (the reference's loop continues)
      if (valid) {
        ind = s_id[i] + 5;   // local point index
        over = !(__longlong_as_double((long long)s_key[by_entry ? ind - 5 : i]) <= 0.1);
      }
      bool supp = !valid || s_picked[ind];
      // each lane's suppression run if its point is picked, from the pair-gap bitmask: right, pairs
      // (ind + k - 1, ind + k) = bits ind .. ind + 4; left, pairs (ind - k, ind - k + 1) = bits ind - 1 down to ind - 5
      int run = 0;   // ind | rr << 16 | ll << 20
      if (valid) {
        const int wb = (ind - 5) >> 5;
        const unsigned long long win = (unsigned long long)s_gapw[wb] | ((unsigned long long)s_gapw[wb + 1] << 32);
        const unsigned bits10 = (unsigned)(win >> ((ind - 5) & 31)) & 0x3FFu;   // bits ind - 5 .. ind + 4
        const unsigned gr = bits10 >> 5, gl = bits10 & 0x1Fu;
        const int rr = gr ? __builtin_ctz(gr) : 5;              // neighbours marked to the right
        const int ll = gl ? 4 - (31 - __builtin_clz(gl)) : 5;   // and to the left
        run = ind | rr << 16 | ll << 20;
      }
      const unsigned long long ends = __ballot(valid && !over);   // candidates that end the loop
      unsigned long long pending = __ballot(valid);
      for (;;) {
        const unsigned long long cand = __ballot(!supp) & pending;
        if (!cand) break;   // the rest of the chunk was picked: the next chunk
        const int l = __ffsll((long long)cand) - 1;
        if ((ends >> l) & 1ull) { stop = true; break; }
        const int rl = __builtin_amdgcn_readlane(run, l);
        const int il = rl & 0xFFFF;
        ++picked_num;
        if (picked_num > 20) {   // picked, not kept, and the loop ends
          if (lane == 0) s_picked[il] = 1;
          stop = true;
          break;
        }
        if (lane == 0) s_edges[nedge] = il;
        ++nedge;
        const int rr = (rl >> 16) & 0xF, ll = rl >> 20;
        if (lane <= rr + ll) s_picked[il - ll + lane] = 1;
        supp = supp || (valid && ind >= il - ll && ind <= il + rr);
        pending &= ~((2ull << l) - 1ull);   // candidates up to l examined
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // (this wave's picked marks: the next chunk's reads)
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0) s_nedge = nedge;
  }
  __syncthreads();
  const unsigned long long T3 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const int nedge = s_nedge;
  if (threadIdx.x < nedge) sec_edge_pos[sec * kMaxEdgesPerSector + threadIdx.x] = off + a + s_edges[threadIdx.x];
  // surf = unpicked entries in ascending order (src/laserProcessingClass.cpp:220-227): contiguous chunk per thread
  const int per = (m + blockDim.x - 1) / blockDim.x;
  const int i0 = threadIdx.x * per, i1 = min(m, i0 + per);
  int c = 0;
  for (int i = i0; i < i1; ++i) c += !s_picked[s_id[i] + 5];
  int total;
  const unsigned long long T3a = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  int pos = block_exclusive_scan_1024(c, smem, &total);
  const unsigned long long T3b = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // the sector's surf positions are one contiguous range: staged in LDS (the curvature keys are free now), then
  // written as whole lines
  int* s_out = reinterpret_cast<int*>(s_key);
  for (int i = i0; i < i1; ++i) {
    const int ind = s_id[i] + 5;
    if (!s_picked[ind]) s_out[pos++] = off + a + ind;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < total; k += blockDim.x) surf_pos[off + a + k] = s_out[k];
  const unsigned long long T3c = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  if (threadIdx.x == 0) {
    sec_edge_cnt[sec] = nedge;
    sec_surf_cnt[sec] = total;
  }
  if (stamps) {
    const unsigned long long T3d = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    const unsigned long long T3e = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) {
      const unsigned long long T4 = __builtin_amdgcn_s_memrealtime();
      if (sec < 1024) g_fe_sec[sec][11] = (unsigned)(((T3e - T3d) & 0xFFFF) | ((T4 - T3e) << 16));
      // (plain per-sector records only: 384 blocks' atomics on a few shared words would queue behind one another
      // and delay the stores being timed)
      if (sec < 1024) {
        unsigned* q = g_fe_sec[sec];
        q[0] = (unsigned)m; q[1] = (unsigned)(T1 - T0); q[2] = (unsigned)(T2 - T1); q[3] = (unsigned)(T3 - T2);
        q[4] = (unsigned)(T4 - T3); q[5] = (unsigned)(T0 & 0xFFFFFFFFu); q[6] = (unsigned)r;
        q[7] = (unsigned)(((T3a - T3) & 0x3FF) | (((T3b - T3a) & 0x3FF) << 10) | (((T3c - T3b) & 0x3FF) << 20));
        q[8] = (unsigned)nedge; q[9] = (unsigned)total; q[10] = (unsigned)(off + a);
      }
    }
  }
}

// one sector per block; with long_list: a sector longer than MAXSEC is listed for fe_sector_long
template <int MINSEC, int MAXSEC, bool LAST>
__global__ __launch_bounds__(kSortThreads) void fe_sector(const int* __restrict__ ring_count,
                                                          const float4* __restrict__ ring_xyz,
                                                          int* __restrict__ sec_edge_cnt, int* __restrict__ sec_edge_pos,
                                                          int* __restrict__ sec_surf_cnt, int* __restrict__ surf_pos,
                                                          int* __restrict__ status, int stamps,
                                                          int* __restrict__ long_list, int* __restrict__ long_count) {
  fe_sector_body<MINSEC, MAXSEC, LAST>((int)blockIdx.x, ring_count, ring_xyz, sec_edge_cnt, sec_edge_pos, sec_surf_cnt,
                                       surf_pos, status, stamps, long_list, long_count);
}

// ---- sectors beyond 4096 entries (a ring of more than ~24.6k points: e.g. a cloud whose ring field is all zero,
// which PCL produces when the field is absent): the sector of src/laserProcessingClass.cpp:88-231 through global
// memory by one block — curvature keys, a stable LSD sort of the 64-bit keys in entry order (ties keep ascending
// entries: the (value, entry) order of the LDS networks), the reference's serial greedy pick (:129-170) by one thread,
// the surf compaction (:220-227).  Slow; for inputs the fast path cannot hold.
// Concurrent huge sectors (several blocks) keep apart: keys and entries at the sector's ring-major position off + a
// (n each), the per-point flags at off + a + 10 sec (its m + 10 staged points; n + 60 R each).
struct HugeScratch {
  unsigned long long *k0, *k1;   // curvature keys (ping-pong)
  int *i0, *i1;                  // entries
  uint8_t *picked, *gap;         // per staged point: picked; far from the next point (the suppression test)
};

__device__ __forceinline__ unsigned long long match8(unsigned d, bool valid) {
  unsigned long long m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const bool bit = (d >> b) & 1u;
    const unsigned long long v = __ballot(bit);
    m &= bit ? v : ~v;
  }
  return m;
}

__device__ void fe_sector_huge(int sec, const int* __restrict__ ring_count, const float4* __restrict__ ring_xyz,
                               int* __restrict__ sec_edge_cnt, int* __restrict__ sec_edge_pos,
                               int* __restrict__ sec_surf_cnt, int* __restrict__ surf_pos, int* __restrict__ status,
                               const HugeScratch& H) {
  constexpr int TB = kSortThreads, R8 = 8, CH = TB * R8, NW = TB / 64;
  __shared__ int s_off;
  __shared__ unsigned s_cnt[NW][256], s_base[256], s_run[256], s_off8[257], s_ws[NW];
  __shared__ unsigned long long s_mm[2][NW];
  __shared__ int s_edges[kMaxEdgesPerSector], s_nedge, smem[33];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int r = sec / 6, s = sec % 6;
  const int n_r = ring_count[r];
  int a, b;
  sector_range(n_r, s, a, b);
  const int m = b - a, npts = m + 10;
  const int off = ring_offset(ring_count, r, &s_off);
  if (!H.k0) {   // (fe_launch reserves the scratch whenever a sector can exceed 4096 entries: never expected)
    if (t == 0) { atomicOr(status, FE_STATUS_SECTOR_TOO_LONG); sec_edge_cnt[sec] = 0; sec_surf_cnt[sec] = 0; }
    return;
  }
  const float4* P = ring_xyz + off + a;   // staged points [0, m + 10): entry k's stencil is points k .. k + 10
  unsigned long long* const K0 = H.k0 + off + a;
  unsigned long long* const K1 = H.k1 + off + a;
  int* const I0 = H.i0 + off + a;
  int* const I1 = H.i1 + off + a;
  uint8_t* const PK = H.picked + off + a + 10 * sec;
  uint8_t* const GP = H.gap + off + a + 10 * sec;
  unsigned long long mn = ~0ull, mx = 0ull;
  for (int k = t; k < m; k += TB) {   // curvature (:95-101) in the float summation order, double squares
    const int c = k + 5;
    float4 q[11];
#pragma unroll
    for (int j = 0; j < 11; ++j) q[j] = P[c - 5 + j];
    const float fx = q[0].x + q[1].x + q[2].x + q[3].x + q[4].x - 10 * q[5].x + q[6].x + q[7].x + q[8].x + q[9].x + q[10].x;
    const float fy = q[0].y + q[1].y + q[2].y + q[3].y + q[4].y - 10 * q[5].y + q[6].y + q[7].y + q[8].y + q[9].y + q[10].y;
    const float fz = q[0].z + q[1].z + q[2].z + q[3].z + q[4].z - 10 * q[5].z + q[6].z + q[7].z + q[8].z + q[9].z + q[10].z;
    const double dX = fx, dY = fy, dZ = fz;
    const unsigned long long v = (unsigned long long)__double_as_longlong(dX * dX + dY * dY + dZ * dZ);
    K0[k] = v;
    I0[k] = k;
    mn = v < mn ? v : mn;
    mx = v > mx ? v : mx;
  }
  for (int j = t; j < npts; j += TB) {   // the neighbour test (:151-166) between consecutive points, once per pair
    bool gap = false;
    if (j + 1 < npts) {
      const float4 p0 = P[j], p1 = P[j + 1];
      const double dX = p1.x - p0.x, dY = p1.y - p0.y, dZ = p1.z - p0.z;
      gap = dX * dX + dY * dY + dZ * dZ > 0.05;
    }
    GP[j] = gap ? 1 : 0;
    PK[j] = 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long a2 = __shfl_xor(mn, o, 64), b2 = __shfl_xor(mx, o, 64);
    mn = a2 < mn ? a2 : mn;
    mx = b2 > mx ? b2 : mx;
  }
  if (lane == 0) { s_mm[0][w] = mn; s_mm[1][w] = mx; }
  __syncthreads();
  unsigned long long kmin = s_mm[0][0], kmax = s_mm[1][0];
  for (int k = 1; k < NW; ++k) {
    kmin = s_mm[0][k] < kmin ? s_mm[0][k] : kmin;
    kmax = s_mm[1][k] > kmax ? s_mm[1][k] : kmax;
  }
  const unsigned long long range = kmax - kmin;
  const int npass = range ? (64 - __clzll((long long)range) + 7) / 8 : 0;
  unsigned long long *ks = K0, *kd = K1;
  int *is = I0, *id = I1;
  for (int p = 0; p < npass; ++p) {   // stable LSD passes over the keys' varying bytes
    const int sh = 8 * p;
    s_run[t] = 0u;
    __syncthreads();
    for (int e = t; e < m; e += TB) atomicAdd(&s_run[((ks[e] - kmin) >> sh) & 255u], 1u);
    __syncthreads();
    {
      const unsigned c = s_run[t];
      unsigned inc = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned u = __shfl_up(inc, o, 64);
        if (lane >= o) inc += u;
      }
      if (lane == 63) s_ws[w] = inc;
      __syncthreads();
      unsigned add = 0;
      for (int k = 0; k < w; ++k) add += s_ws[k];
      s_base[t] = add + inc - c;
      s_run[t] = 0u;
      __syncthreads();
    }
    for (int c0 = 0; c0 < m; c0 += CH) {   // chunks in order; within a chunk a stable rank by wave ballots
      const int nc = min(CH, m - c0);
      unsigned long long key[R8];
      int val[R8];
      unsigned dig[R8], rank[R8];
      for (int k = t; k < NW * 256; k += TB) (&s_cnt[0][0])[k] = 0u;
#pragma unroll
      for (int rr = 0; rr < R8; ++rr) {
        const int e = w * 64 * R8 + rr * 64 + lane;
        key[rr] = e < nc ? ks[c0 + e] : 0ull;
        val[rr] = e < nc ? is[c0 + e] : 0;
        dig[rr] = (unsigned)(((key[rr] - kmin) >> sh) & 255u);
      }
      __syncthreads();
      const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
      for (int rr = 0; rr < R8; ++rr) {
        const int e = w * 64 * R8 + rr * 64 + lane;
        const bool valid = e < nc;
        const unsigned long long peers = match8(dig[rr], valid);
        const unsigned before = s_cnt[w][dig[rr]];
        rank[rr] = before + (unsigned)__popcll(peers & lt);
        if (valid && lane == 63 - __clzll((long long)peers)) s_cnt[w][dig[rr]] = before + (unsigned)__popcll(peers);
      }
      __syncthreads();
      unsigned tot = 0;
      for (int k = 0; k < NW; ++k) {   // thread t = digit t: offsets of the waves within the chunk's digit
        const unsigned v = s_cnt[k][t];
        s_cnt[k][t] = tot;
        tot += v;
      }
      s_off8[t] = tot;   // the chunk's count of digit t
      __syncthreads();
#pragma unroll
      for (int rr = 0; rr < R8; ++rr) {
        const int e = w * 64 * R8 + rr * 64 + lane;
        if (e >= nc) continue;
        const unsigned d = dig[rr];
        const unsigned dst = s_base[d] + s_run[d] + s_cnt[w][d] + rank[rr];
        kd[dst] = key[rr];
        id[dst] = val[rr];
      }
      __syncthreads();
      s_run[t] += s_off8[t];
      __syncthreads();
    }
    unsigned long long* tk = ks; ks = kd; kd = tk;
    int* ti = is; is = id; id = ti;
  }
  __threadfence_block();
  __syncthreads();
  // greedy edge pick (:129-170): the entries in descending (value, entry) order, the reference's loop, one thread
  if (t == 0) {
    int picked_num = 0, nedge = 0;
    for (int i = m - 1; i >= 0; --i) {
      const int ind = is[i] + 5;
      if (PK[ind]) continue;
      if (__longlong_as_double((long long)ks[i]) <= 0.1) break;
      ++picked_num;
      if (picked_num > 20) {   // picked, not kept (Q1), and the loop ends
        PK[ind] = 1;
        break;
      }
      s_edges[nedge++] = ind;
      PK[ind] = 1;
      for (int k = 1; k <= 5 && !GP[ind + k - 1]; ++k) PK[ind + k] = 1;   // pairs (ind+k-1, ind+k)
      for (int k = 1; k <= 5 && !GP[ind - k]; ++k) PK[ind - k] = 1;       // pairs (ind-k, ind-k+1)
    }
    s_nedge = nedge;
  }
  __threadfence_block();
  __syncthreads();
  const int nedge = s_nedge;
  if (t < nedge) sec_edge_pos[sec * kMaxEdgesPerSector + t] = off + a + s_edges[t];
  // surf = unpicked entries in ascending order (:220-227): contiguous chunk per thread, block scan, then in order
  const int per = (m + TB - 1) / TB;
  const int j0 = t * per, j1 = min(m, j0 + per);
  int c = 0;
  for (int i = j0; i < j1; ++i) c += !PK[is[i] + 5];
  int total;
  int pos = block_exclusive_scan_1024(c, smem, &total);
  for (int i = j0; i < j1; ++i) {
    const int ind = is[i] + 5;
    if (!PK[ind]) surf_pos[off + a + pos++] = off + a + ind;
  }
  if (t == 0) {
    sec_edge_cnt[sec] = nedge;
    sec_surf_cnt[sec] = total;
  }
}

// the listed long sectors (m > 1024), a few blocks looping over the list (a grid of one block per sector would cost
// a launch of 6 R blocks that nearly all find nothing to do): up to 4096 entries in LDS, longer ones through global
// memory (fe_sector_huge)
__global__ __launch_bounds__(kSortThreads) void fe_sector_long(const int* __restrict__ ring_count,
                                                               const float4* __restrict__ ring_xyz,
                                                               int* __restrict__ sec_edge_cnt,
                                                               int* __restrict__ sec_edge_pos,
                                                               int* __restrict__ sec_surf_cnt,
                                                               int* __restrict__ surf_pos, int* __restrict__ status,
                                                               const int* __restrict__ long_list,
                                                               const int* __restrict__ long_count, HugeScratch H) {
  const int nl = *long_count;
  for (int j = blockIdx.x; j < nl; j += gridDim.x) {
    const int sec = long_list[j];
    const int n_r = ring_count[sec / 6];
    int a, b;
    sector_range(n_r, sec % 6, a, b);
    if (b - a > 4096) {   // (block-uniform)
      fe_sector_huge(sec, ring_count, ring_xyz, sec_edge_cnt, sec_edge_pos, sec_surf_cnt, surf_pos, status, H);
    } else {
      fe_sector_body<1024, 4096, true>(sec, ring_count, ring_xyz, sec_edge_cnt, sec_edge_pos, sec_surf_cnt, surf_pos,
                                       status, 0, nullptr, nullptr);
    }
    __syncthreads();   // (the body's LDS is reused by the next listed sector)
  }
}

// Advances the output counts, publishes (edge count, surf count, status) for one D2H copy and re-zeroes the
// per-call counters for the next call (so no memset nodes are needed).  Run by the last block of fe_output to
// arrive (every other block has read the counts and ring sizes it needs), not as a launch of its own.
__device__ __forceinline__ void fe_commit_block(int* __restrict__ long_count, int n_sectors, const int* __restrict__ sec_edge_cnt, const int* __restrict__ sec_surf_cnt,
                          int* __restrict__ edge_count, int* __restrict__ surf_count, int* __restrict__ ring_count,
                          int num_lines, int* __restrict__ status, int* __restrict__ out3,
                          int* __restrict__ stat_edge, int* __restrict__ stat_surf, unsigned* __restrict__ radix_ctl,
                          int clear) {
  radix_ctl_zero(radix_ctl, threadIdx.x, blockDim.x);   // the next call's bucketing sort (its histograms, epoch)
  __shared__ int red[2][4];
  int pe = 0, ps = 0;
  for (int k = threadIdx.x; k < n_sectors; k += blockDim.x) {
    pe += sec_edge_cnt[k];
    ps += sec_surf_cnt[k];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    pe += __shfl_down(pe, o, 64);
    ps += __shfl_down(ps, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = pe;
    red[1][threadIdx.x >> 6] = ps;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int te = 0, ts = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { te += red[0][w]; ts += red[1][w]; }
    edge_count[0] = ((clear & 1) ? 0 : edge_count[0]) + te;   // clear: the outputs were emptied before this call
    surf_count[0] = ((clear & 2) ? 0 : surf_count[0]) + ts;    // (floam_cloud_clear, folded in: no fill launch)
    out3[0] = edge_count[0];
    out3[1] = surf_count[0];
    const int sv = *status;
    out3[2] = sv;
    if (stat_edge) *stat_edge = sv;   // the status travels with the output clouds (asynchronous consumers)
    if (stat_surf) *stat_surf = sv;
    *status = 0;
  }
  for (int r = threadIdx.x; r < num_lines; r += blockDim.x) ring_count[r] = 0;
  if (threadIdx.x == 0) *long_count = 0;   // fe_sector's long-sector list, for the next call
}

__global__ __launch_bounds__(kSectorThreads) void fe_output(const PointRec* __restrict__ ring_pts,
                                                            const int* __restrict__ ring_count,
                                                            const int* __restrict__ sec_edge_cnt,
                                                            const int* __restrict__ sec_edge_pos,
                                                            const int* __restrict__ sec_surf_cnt,
                                                            const int* __restrict__ surf_pos,
                                                            PointRec* __restrict__ edge_out, int* __restrict__ edge_count,
                                                            PointRec* __restrict__ surf_out, int* __restrict__ surf_count,
                                                            int clear, int* __restrict__ ring_count_w, int num_lines,
                                                            int* __restrict__ status, int* __restrict__ out3,
                                                            int* __restrict__ stat_edge, int* __restrict__ stat_surf,
                                                            unsigned* __restrict__ radix_ctl,
                                                            unsigned* __restrict__ ticket, int* __restrict__ long_count) {
  __shared__ int red[2][kSectorThreads / 64];
  __shared__ int s_off;
  const int sec = blockIdx.x;
  const int r = sec / 6, s = sec % 6;
  int pe = 0, ps = 0;
  for (int k = threadIdx.x; k < sec; k += blockDim.x) {
    pe += sec_edge_cnt[k];
    ps += sec_surf_cnt[k];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    pe += __shfl_down(pe, o, 64);
    ps += __shfl_down(ps, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = pe;
    red[1][threadIdx.x >> 6] = ps;
  }
  const int roff = ring_offset(ring_count, r, &s_off);   // (its barrier also orders red[][])
  int edge_prefix = 0, surf_prefix = 0;
  for (int w = 0; w < kSectorThreads / 64; ++w) {
    edge_prefix += red[0][w];
    surf_prefix += red[1][w];
  }
  const int ne = sec_edge_cnt[sec], ns = sec_surf_cnt[sec];
  const int be = ((clear & 1) ? 0 : edge_count[0]) + edge_prefix, bs = ((clear & 2) ? 0 : surf_count[0]) + surf_prefix;
  if ((int)threadIdx.x < ne) edge_out[be + threadIdx.x] = make_out(ring_pts[sec_edge_pos[sec * kMaxEdgesPerSector + threadIdx.x]]);
  if (ns > 0) {
    int a, b;
    sector_range(ring_count[r], s, a, b);
    const int base = roff + a;
    for (int k = threadIdx.x; k < ns; k += blockDim.x) surf_out[bs + k] = make_out(ring_pts[surf_pos[base + k]]);
  }
  // the commit by the last block to arrive (its add returns nblocks - 1: every block has read what it needs)
  __shared__ int s_last;
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  fe_commit_block(long_count, (int)gridDim.x, sec_edge_cnt, sec_surf_cnt, edge_count, surf_count, ring_count_w, num_lines, status,
                  out3, stat_edge, stat_surf, radix_ctl, clear);
  if (threadIdx.x == 0) *ticket = 0u;
}

// more than 255 rings: the ring-major staging by the ring-ordered input indices (the key-only passes' output)
__global__ void fe_stage(const PointRec* __restrict__ in, const int* __restrict__ ring_idx, int n,
                         float4* __restrict__ ring_xyz, PointRec* __restrict__ ring_pts) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const PointRec p = in[ring_idx[i]];
    ring_xyz[i] = make_float4(p.x, p.y, p.z, 0.0f);
    ring_pts[i] = p;
  }
}

}  // namespace

static int fe_stamps_on() {
  static const int on = FLOAM_DIAG_ENV("FLOAM_FE_STAMPS") ? 1 : 0;
  static unsigned launches = 0;
  static bool init = false;
  if (on && !init) {
    init = true;
    static unsigned long long h[8 + 3 * 1024];
    for (int k = 0; k < 8 + 3 * 1024; ++k) h[k] = (k >= 8 && (k - 8) % 3 == 0) ? ~0ull : 0ull;
    FLOAM_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_fe_stamps), h, sizeof(h)));
  }
  return on ? (int)(launches++ % 1024u) + 1 : 0;   // per launch: its slot + 1
}

void fe_stamps_print() {
  if (!FLOAM_DIAG_ENV("FLOAM_FE_STAMPS")) return;
  static unsigned long long h[8 + 3 * 1024];
  FLOAM_HIP(hipDeviceSynchronize());
  FLOAM_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_fe_stamps), sizeof(h)));
  {
    static unsigned q[1024][12];
    FLOAM_HIP(hipMemcpyFromSymbol(q, HIP_SYMBOL(g_fe_sec), sizeof(q)));
    unsigned t0 = ~0u;
    for (int k = 0; k < 1024; ++k)
      if (q[k][0]) t0 = std::min(t0, q[k][5]);
    std::vector<std::pair<unsigned, int>> d;
    double ph[4] = {0, 0, 0, 0};
    unsigned tend = 0;
    for (int k = 0; k < 1024; ++k)
      if (q[k][0]) {
        d.push_back({q[k][1] + q[k][2] + q[k][3] + q[k][4], k});
        for (int j = 0; j < 4; ++j) ph[j] += q[k][1 + j];
        tend = std::max(tend, q[k][5] - t0 + q[k][1] + q[k][2] + q[k][3] + q[k][4]);
      }
    std::sort(d.begin(), d.end());
    const int nd = (int)d.size();
    if (nd)
      std::fprintf(stderr, "[fe stamps] last launch, %d sector blocks: staging %.2f, curvature + sort %.2f, greedy "
                   "pick %.2f, compaction %.2f us per block; first start -> last end %.2f us\n", nd,
                   ph[0] / nd / 100.0, ph[1] / nd / 100.0, ph[2] / nd / 100.0, ph[3] / nd / 100.0, tend / 100.0);
    for (int j = 0; j < nd; ++j) {
      if (j >= 6 && j < nd - 10) continue;   // the fastest and the slowest blocks of the last launch
      const unsigned* x = q[d[j].second];
      std::fprintf(stderr, "[fe sector %3d ring %2u] m %4u start +%.2f us: staging %.2f sort %.2f pick %.2f "
                   "compaction %.2f us (count %.2f, scan %.2f, writes %.2f, drain %.2f: barrier %.2f, stores %.2f) edges %u surf %u "
                   "at %u\n",
                   d[j].second, x[6], x[0],
                   (x[5] - t0) / 100.0, x[1] / 100.0, x[2] / 100.0, x[3] / 100.0, x[4] / 100.0,
                   (x[7] & 0x3FF) / 100.0, ((x[7] >> 10) & 0x3FF) / 100.0, ((x[7] >> 20) & 0x3FF) / 100.0,
                   (x[4] - (x[7] & 0x3FF) - ((x[7] >> 10) & 0x3FF) - ((x[7] >> 20) & 0x3FF)) / 100.0,
                   (x[11] & 0xFFFF) / 100.0, (x[11] >> 16) / 100.0, x[8], x[9], x[10]);
    }
  }
}

void fe_launch(FeScratch& sc, const FeParams& prm, const PointRec* d_in, int n, PointRec* edge_out,
               int* edge_count, PointRec* surf_out, int* surf_count, hipStream_t st, int* stat_edge,
               int* stat_surf, int clear) {
  const int R = prm.num_lines;
  sc.keys.reserve(n);
  sc.keys2.reserve(n);
  sc.vals.reserve(n);
  sc.ring_idx.reserve(n + 16);
  sc.ring_xyz.reserve(n + 16);
  sc.ring_pts.reserve(n + 16);
  if (sc.ring_count.cap < (size_t)R) sc.zeroed = false;
  sc.ring_count.reserve(R);
  sc.out3.reserve(4);
  sc.sec_edge_cnt.reserve(6 * R);
  sc.sec_surf_cnt.reserve(6 * R);
  sc.sec_edge_pos.reserve(6 * R * kMaxEdgesPerSector);
  sc.surf_pos.reserve(n + 16);
  sc.rs.reserve(n, st);   // (a fresh control block is zeroed by the allocation)
  if (!sc.ticket.p) {
    sc.ticket.reserve(1);
    FLOAM_HIP(hipMemsetAsync(sc.ticket.p, 0, sizeof(unsigned), st));   // (reset by the last block of every call)
  }
  if (sc.long_sec.cap < (size_t)(6 * R + 1)) {   // [0] count (reset by the commit), [1..] long sectors
    sc.long_sec.release();
    sc.long_sec.reserve(6 * R + 1);
    FLOAM_HIP(hipMemsetAsync(sc.long_sec.p, 0, sizeof(int), st));
  }
  if (!sc.zeroed || sc.zeroed_lines < R) {   // the commit re-zeroes the counters at the end of every call
    FLOAM_HIP(hipMemsetAsync(sc.ring_count.p, 0, sizeof(int) * sc.ring_count.cap, st));
    FLOAM_HIP(hipMemsetAsync(sc.status, 0, sizeof(int), st));
    sc.zeroed = true;
    sc.zeroed_lines = R;
  }
  const int tb = 256;
  if (R <= 255) {   // few blocks, 4+ points per thread: each block folds <= 256 bins with global atomics
    hipLaunchKernelGGL(fe_keys<true>, dim3(std::max(1u, std::min(div_up(n, 4 * tb), 256u))), dim3(tb), 0, st, d_in,
                       n, R, prm.min_distance, prm.max_distance, sc.keys.p, sc.vals.p, sc.ring_count.p, sc.status,
                       sc.rs.ctl.p);
  } else {
    hipLaunchKernelGGL(fe_keys<false>, dim3(std::min(div_up(n, tb), 512u)), dim3(tb), sizeof(int) * R, st, d_in, n,
                       R, prm.min_distance, prm.max_distance, sc.keys.p, sc.vals.p, sc.ring_count.p, sc.status,
                       sc.rs.ctl.p);
  }
  FLOAM_LAUNCH_CHECK();
  // stable bucketing by ring: rings < 255 differ in the low digit only (dropped points: 0xFFFF, last); the pass
  // stages the scan ring-major
  if (R <= 255) {
    const bool wb = prof_wb_enabled();   // (diagnostic: the pass's own write bytes, profwb.hpp)
    if (wb) prof_l2_writeback(st);
    radix_pass_payload_launch(sc.rs, sc.keys.p, nullptr, nullptr, n, d_in, sc.ring_xyz.p, sc.ring_pts.p, st);
    if (wb) prof_l2_writeback(st);
  } else {
    radix_pass_launch(sc.rs, sc.keys.p, sc.vals.p, sc.keys2.p, sc.surf_pos.p, n, 0, st);
    radix_pass_launch(sc.rs, sc.keys2.p, sc.surf_pos.p, sc.keys.p, sc.ring_idx.p, n, 1, st);
    hipLaunchKernelGGL(fe_stage, dim3(std::min(div_up(n, 256u), 1024u)), dim3(256), 0, st, d_in, sc.ring_idx.p, n,
                       sc.ring_xyz.p, sc.ring_pts.p);
    FLOAM_LAUNCH_CHECK();
  }
  // the longest possible sector is (max ring size - 10) / 6 <= n / 6: the 4096 pass is only needed beyond 1024
  const bool big = n / 6 + 8 > 1024;
  if (big) {   // sectors beyond 1024 entries (rare) are listed by the first launch and run by a small second one
    hipLaunchKernelGGL((fe_sector<0, 1024, false>), dim3(6 * R), dim3(kSortThreads), 0, st, sc.ring_count.p,
                       sc.ring_xyz.p, sc.sec_edge_cnt.p, sc.sec_edge_pos.p, sc.sec_surf_cnt.p, sc.surf_pos.p,
                       sc.status, fe_stamps_on(), sc.long_sec.p + 1, sc.long_sec.p + 0);
    FLOAM_LAUNCH_CHECK();
    // sectors beyond 4096 entries (a sector holds at most n / 6) run through the global scratch of fe_sector_huge
    HugeScratch H{};
    if (n / 6 + 8 > 4096) {
      const size_t nb = (size_t)n + 60 * (size_t)R + 16;
      sc.huge_k.reserve(2 * (size_t)n);
      sc.huge_i.reserve(2 * (size_t)n);
      sc.huge_b.reserve(2 * nb);
      H = HugeScratch{sc.huge_k.p, sc.huge_k.p + n, sc.huge_i.p, sc.huge_i.p + n, sc.huge_b.p, sc.huge_b.p + nb};
    }
    hipLaunchKernelGGL(fe_sector_long, dim3(16), dim3(kSortThreads), 0, st, sc.ring_count.p, sc.ring_xyz.p,
                       sc.sec_edge_cnt.p, sc.sec_edge_pos.p, sc.sec_surf_cnt.p, sc.surf_pos.p, sc.status,
                       sc.long_sec.p + 1, sc.long_sec.p + 0, H);
  } else {
    hipLaunchKernelGGL((fe_sector<0, 1024, true>), dim3(6 * R), dim3(kSortThreads), 0, st, sc.ring_count.p,
                       sc.ring_xyz.p, sc.sec_edge_cnt.p, sc.sec_edge_pos.p, sc.sec_surf_cnt.p, sc.surf_pos.p,
                       sc.status, fe_stamps_on(), nullptr, nullptr);
  }
  FLOAM_LAUNCH_CHECK();
  hipLaunchKernelGGL(fe_output, dim3(6 * R), dim3(kSectorThreads), 0, st, sc.ring_pts.p, sc.ring_count.p,
                     sc.sec_edge_cnt.p, sc.sec_edge_pos.p, sc.sec_surf_cnt.p, sc.surf_pos.p, edge_out, edge_count,
                     surf_out, surf_count, clear, sc.ring_count.p, R, sc.status, sc.out3.p, stat_edge, stat_surf,
                     sc.rs.ctl.p, sc.ticket.p, sc.long_sec.p + 0);
  FLOAM_LAUNCH_CHECK();

}

}  // namespace floam
