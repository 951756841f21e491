// Stable LSD radix sort, one single-pass launch per 8-bit digit (see radix.hpp).
//
// A launch sorts by one digit.  Each block is a tile (256 threads x kItems consecutive elements; tile = the block's
// ticket, the order blocks start in, so a tile only ever waits on tiles that are already running: HIP promises no
// dispatch order, and a tile taken by block index can wait on a block that never gets a CU — MI355X_MICROARCH.md
// "Workgroup dispatch"; observed with two processes' kernels on one GPU) and
//   1. loads its elements: wave w owns the 64 * kItems elements [w * 64 * kItems, ...), lane l element r * 64 + l in
//      round r, so (round, lane) order is input order;
//   2. ranks them stably: per round, the lanes holding the same digit find each other with 8 ballots, each takes
//      its position among them, and the highest of them advances the wave's counter of that digit (LDS; one wave
//      reads and writes its own counters in program order);
//   3. thread d (one per digit): the wave offsets of digit d, the tile's count of d published to the lookback
//      word (tile, d), the exclusive prefix of d over the earlier tiles by walking back to an inclusive word, and
//      the digit's bucket start (exclusive scan of the global histogram);
//   4. scatters every element to bucket start + tile prefix + wave offset + rank.
// Lookback words are 64 bits — epoch (30) | flag (2) | count (32) — stored and loaded with agent-scope atomics,
// so no array has to be cleared between sorts: a word from an older sort carries an older epoch.
#include "radix.hpp"

namespace floam {

// FLOAM_RADIX_STAMPS=1 (diagnostic): per-block phase times of every pass (100 MHz ticks) and per-launch first block
// start / last block end, printed by radix_stamps_print
constexpr int kStampSlots = 4096;
__device__ unsigned long long g_radix_stamps[8 + 2 * kStampSlots];

namespace {
constexpr int kTB = 256;
constexpr int kItems = 8;
constexpr int kTile = kTB * kItems;
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr unsigned long long kFlagAgg = 1ull << 32, kFlagInc = 2ull << 32;

__device__ __forceinline__ unsigned long long lb_word(unsigned epoch, unsigned long long flag, unsigned v) {
  return ((unsigned long long)epoch << 34) | flag | (unsigned long long)v;
}

__device__ __forceinline__ unsigned long long match_digit(unsigned d, bool valid) {
  unsigned long long m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const bool bit = (d >> b) & 1u;
    const unsigned long long v = __ballot(bit);
    m &= bit ? v : ~v;
  }
  return m;
}

// PAYLOAD: the values are the element positions (a first pass over the original order), and each element's
// record pin[i] travels with it: its 16-B coordinates to pxyz[dst], the whole 32-B record to prec[dst] (loaded
// coalesced with the keys, written where the element lands); the sorted keys / values only if kout != null
template <bool PAYLOAD>
__global__ __launch_bounds__(kTB) void radix_pass(const uint32_t* __restrict__ kin, const int* __restrict__ vin,
                                                  uint32_t* __restrict__ kout, int* __restrict__ vout, int n,
                                                  int pass, unsigned* __restrict__ ctl,
                                                  unsigned long long* __restrict__ status,
                                                  const int* __restrict__ gate, const int* __restrict__ n_dev,
                                                  int stamps, const PointRec* __restrict__ pin,
                                                  float4* __restrict__ pxyz, PointRec* __restrict__ prec) {
  const unsigned long long ts0 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // every load of the prologue is issued at once (one memory round trip, not three in a row): the gate, the epoch,
  // the device count, this digit's histogram count and the tile's elements up to the host bound n (allocated; the
  // ones past the device count are dropped below)
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // the ticket (zeroed per sort with the histograms) with the tile-independent loads in flight beside it
  __shared__ int s_tile;
  if (t == 0) s_tile = (int)atomicAdd(&ctl[kRadixTicketWord + pass], 1u);
  const int gv = gate ? *gate : 1;
  const unsigned epoch = ctl[kRadixEpochWord];
  const int nd = n_dev ? *n_dev : n;
  const unsigned h = ctl[pass * kRadixDigits + t];   // digit t's histogram count
  __syncthreads();
  const int tile = s_tile;
  const int base = tile * kTile + w * 64 * kItems;
  uint32_t key[kItems];
  int val[kItems];
  unsigned dig[kItems];
#pragma unroll
  for (int r = 0; r < kItems; ++r) {
    const int i = base + r * 64 + lane;
    key[r] = i < n ? kin[i] : 0u;
    val[r] = PAYLOAD ? i : (i < n ? vin[i] : 0);
    dig[r] = (key[r] >> (8 * pass)) & 255u;
  }
  // PAYLOAD: the tile's records into LDS in input order as 16-B chunks, thread t chunk t + 256 k (every load
  // instruction covers whole contiguous lines once; a lane loading both halves of its own record made each 128-B line
  // two requests of two instructions); the scatter reads them back by input position
  __shared__ v4i s_nat[PAYLOAD ? 2 * kTile : 1];
  if (PAYLOAD) {
    const v4i* q = reinterpret_cast<const v4i*>(pin + (size_t)tile * kTile);
    const int nchunk = 2 * (min(n, (tile + 1) * kTile) - tile * kTile);   // (host bound: allocated)
#pragma unroll
    for (int k = 0; k < 2 * kItems; ++k) {
      const int c = t + k * kTB;
      if (c < nchunk) s_nat[c] = q[c];
    }
  }
  if (!gv) return;
  n = min(n, nd);
  if (tile * kTile >= n) return;   // beyond the elements (block-uniform); nobody waits on a later tile
  __shared__ unsigned s_wcnt[kTB / 64][kRadixDigits];
  __shared__ unsigned s_off[kRadixDigits];
  __shared__ unsigned s_wsum[kTB / 64];
#pragma unroll
  for (int k = 0; k < kTB / 64; ++k) s_wcnt[k][t] = 0u;
  __syncthreads();
  // 2. stable rank within (wave, digit)
  unsigned rank[kItems];
  const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int r = 0; r < kItems; ++r) {
    const bool valid = base + r * 64 + lane < n;
    const unsigned d = dig[r];
    const unsigned long long peers = match_digit(d, valid);
    const unsigned before = s_wcnt[w][d];
    rank[r] = before + (unsigned)__popcll(peers & lt);
    if (valid && lane == 63 - __clzll((long long)peers)) s_wcnt[w][d] = before + (unsigned)__popcll(peers);
  }
  __syncthreads();
  const unsigned long long ts1 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // 3. thread t = digit t: wave offsets, tile count, bucket start, lookback over the earlier tiles
  unsigned c[kTB / 64], cnt = 0;
#pragma unroll
  for (int k = 0; k < kTB / 64; ++k) {
    c[k] = s_wcnt[k][t];
    s_wcnt[k][t] = cnt;   // exclusive over the waves
    cnt += c[k];
  }
  unsigned long long* st = status;   // this pass's [tiles][256] region is passed in
  __hip_atomic_store(&st[(size_t)tile * kRadixDigits + t], lb_word(epoch, tile == 0 ? kFlagInc : kFlagAgg, cnt),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // bucket start of digit t: exclusive scan of the pass histogram (wave scan + wave totals)
  unsigned incl = h;
  incl = wave_incl_scan(incl);   // (DPP, floam_common.hpp)
  if (lane == 63) s_wsum[w] = incl;
  // PAYLOAD: the tile-local start of digit t (exclusive scan of the tile's digit counts) for the LDS staging
  __shared__ unsigned s_twsum[kTB / 64];
  unsigned tincl = cnt;
  if (PAYLOAD) {
    tincl = wave_incl_scan(tincl);   // (DPP, floam_common.hpp)
    if (lane == 63) s_twsum[w] = tincl;
  }
  unsigned prefix = 0;
  if (tile > 0) {
    // windowed lookback: the words of the kLbWin nearest unconsumed predecessors are loaded together (one round
    // trip per window instead of one per predecessor), then consumed in order up to the first inclusive prefix
    // or the first word not yet published (the walk resumes there)
    constexpr int kLbWin = 8;
    bool failed = false;
    long long polls = 0;
    for (int j = tile - 1; j >= 0;) {
      unsigned long long x[kLbWin];
#pragma unroll
      for (int k = 0; k < kLbWin; ++k)
        x[k] = j - k >= 0 ? __hip_atomic_load(&st[(size_t)(j - k) * kRadixDigits + t], __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT)
                          : 0ull;
      int consumed = 0;
      bool done = false, stall = false;
#pragma unroll
      for (int k = 0; k < kLbWin; ++k) {
        if (done || stall || j - k < 0) continue;
        const unsigned long long flag = x[k] & (3ull << 32);
        if ((unsigned)(x[k] >> 34) != (epoch & 0x3FFFFFFFu) || flag == 0) {
          stall = true;
          continue;
        }
        prefix += (unsigned)(x[k] & 0xFFFFFFFFull);
        ++consumed;
        if (flag == kFlagInc) done = true;
      }
      if (done) break;
      j -= consumed;
      if (stall) {
        if (++polls > (1ll << 22)) { failed = true; break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (failed) atomicOr(&ctl[kRadixErrorWord], 1u);
    __hip_atomic_store(&st[(size_t)tile * kRadixDigits + t], lb_word(epoch, kFlagInc, prefix + cnt), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  unsigned wb = 0;
#pragma unroll
  for (int k = 0; k < kTB / 64; ++k)
    if (k < w) wb += s_wsum[k];
  s_off[t] = wb + incl - h + prefix;
  __shared__ unsigned s_tstart[PAYLOAD ? kRadixDigits : 1];
  if (PAYLOAD) {
    unsigned twb = 0;
#pragma unroll
    for (int k = 0; k < kTB / 64; ++k)
      if (k < w) twb += s_twsum[k];
    s_tstart[t] = twb + tincl - cnt;
  }
  __syncthreads();
  const unsigned long long ts2 = stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // 4. scatter
  if (PAYLOAD) {   // keys / values as below; the records through LDS in tile-sorted order, then written as runs
    __shared__ unsigned short s_src[PAYLOAD ? kTile : 1];   // input position in the tile, by tile-sorted slot
    __shared__ unsigned char s_dig[PAYLOAD ? kTile : 1];
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
      if (base + r * 64 + lane < n) {
        const unsigned d = dig[r];
        const unsigned loc = s_tstart[d] + s_wcnt[w][d] + rank[r];
        s_src[loc] = (unsigned short)(w * 64 * kItems + r * 64 + lane);
        s_dig[loc] = (unsigned char)d;
        if (kout) {
          const unsigned dst = s_off[d] + s_wcnt[w][d] + rank[r];
          kout[dst] = key[r];
          vout[dst] = val[r];
        }
      }
    }
    __syncthreads();
    const int nloc = min(kTile, n - tile * kTile);
    for (int j = t; j < nloc; j += kTB) {   // consecutive j of one digit land on consecutive slots
      const unsigned d = s_dig[j];
      const unsigned dst = s_off[d] + ((unsigned)j - s_tstart[d]);
      const int src = s_src[j];
      const v4i lo = s_nat[2 * src], hi = s_nat[2 * src + 1];
      v4i* o = reinterpret_cast<v4i*>(prec + dst);
      o[0] = lo;
      o[1] = hi;
      pxyz[dst] = make_float4(__int_as_float(lo.x), __int_as_float(lo.y), __int_as_float(lo.z), 0.0f);
    }
  } else {
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
      if (base + r * 64 + lane < n) {
        const unsigned d = dig[r];
        const unsigned dst = s_off[d] + s_wcnt[w][d] + rank[r];
        kout[dst] = key[r];
        vout[dst] = val[r];
      }
    }
  }
  if (stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      const unsigned long long ts3 = __builtin_amdgcn_s_memrealtime();
      atomicAdd(&g_radix_stamps[0], ts1 - ts0);
      atomicAdd(&g_radix_stamps[1], ts2 - ts1);
      atomicAdd(&g_radix_stamps[2], ts3 - ts2);
      atomicAdd(&g_radix_stamps[3], 1ull);
      const int slot = stamps - 1;   // the host's launch counter
      atomicMin(&g_radix_stamps[8 + 2 * slot], ts0);
      atomicMax(&g_radix_stamps[8 + 2 * slot + 1], ts3);
    }
  }
}

}  // namespace

static int stamps_on() {
  static unsigned launches = 0;
  static const int on = FLOAM_DIAG_ENV("FLOAM_RADIX_STAMPS") ? 1 : 0;
  static bool init = false;
  if (on && !init) {
    init = true;
    static unsigned long long h[8 + 2 * kStampSlots];
    for (int k = 0; k < 8 + 2 * kStampSlots; ++k) h[k] = (k >= 8 && (k & 1) == 0) ? ~0ull : 0ull;
    FLOAM_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_radix_stamps), h, sizeof(h)));
  }
  return on ? (int)(launches++ % (unsigned)kStampSlots) + 1 : 0;   // per launch: its slot + 1
}

void radix_stamps_print() {
  if (!FLOAM_DIAG_ENV("FLOAM_RADIX_STAMPS")) return;
  static unsigned long long h[8 + 2 * kStampSlots];
  FLOAM_HIP(hipDeviceSynchronize());
  FLOAM_HIP(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_radix_stamps), sizeof(h)));
  const double nb = h[3] ? (double)h[3] : 1.0;
  double span = 0.0;
  int nl = 0;
  for (int k = 0; k < kStampSlots; ++k)
    if (h[8 + 2 * k + 1] != 0ull) {
      span += (double)(h[8 + 2 * k + 1] - h[8 + 2 * k]);
      ++nl;
    }
  std::fprintf(stderr, "[radix stamps] %llu blocks: load + rank %.2f us, lookback %.2f us, scatter + drain %.2f us per "
               "block; %d launches: first block start -> last block end %.2f us\n", h[3], h[0] / nb / 100.0,
               h[1] / nb / 100.0, h[2] / nb / 100.0, nl, nl ? span / nl / 100.0 : 0.0);
}

void RadixScratch::reserve(int n, hipStream_t st) {
  if (!ctl.p) {
    ctl.reserve(kRadixCtlWords);
    FLOAM_HIP(hipMemsetAsync(ctl.p, 0, sizeof(unsigned) * kRadixCtlWords, st));
  }
  const int tiles = (int)div_up((unsigned)std::max(n, 1), (unsigned)kTile);
  if (tiles > tiles_cap) {
    const int cap = std::max(tiles + tiles / 4 + 4, 1024);   // 2 M elements before a reallocation (device stall)
    status.release();
    status.reserve((size_t)kRadixPasses * cap * kRadixDigits);
    // a fresh array: make every word's epoch field differ from the next epochs
    FLOAM_HIP(hipMemsetAsync(status.p, 0xFF, sizeof(unsigned long long) * kRadixPasses * cap * kRadixDigits, st));
    tiles_cap = cap;
  }
}

void radix_pass_launch(RadixScratch& sc, const uint32_t* kin, const int* vin, uint32_t* kout, int* vout, int n,
                       int pass, hipStream_t st) {
  if (n <= 0) return;
  sc.reserve(n, st);
  const int tiles = (int)div_up((unsigned)n, (unsigned)kTile);
  hipLaunchKernelGGL(radix_pass<false>, dim3(tiles), dim3(kTB), 0, st, kin, vin, kout, vout, n, pass, sc.ctl.p,
                     sc.status.p + (size_t)pass * sc.tiles_cap * kRadixDigits, nullptr, nullptr, stamps_on(), nullptr,
                     nullptr, nullptr);
  FLOAM_LAUNCH_CHECK();
}

void radix_pass_payload_launch(RadixScratch& sc, const uint32_t* kin, uint32_t* kout, int* vout, int n,
                               const PointRec* pin, float4* pxyz, PointRec* prec, hipStream_t st) {
  if (n <= 0) return;
  sc.reserve(n, st);
  const int tiles = (int)div_up((unsigned)n, (unsigned)kTile);
  hipLaunchKernelGGL(radix_pass<true>, dim3(tiles), dim3(kTB), 0, st, kin, nullptr, kout, vout, n, 0, sc.ctl.p,
                     sc.status.p, nullptr, nullptr, stamps_on(), pin, pxyz, prec);
  FLOAM_LAUNCH_CHECK();
}

void radix_sort_launch(RadixScratch& sc, uint32_t* k0, int* v0, uint32_t* k1, int* v1, int n, hipStream_t st,
                       const int* gate, const int* n_dev) {
  if (n <= 0) return;
  sc.reserve(n, st);
  const int tiles = (int)div_up((unsigned)n, (unsigned)kTile);
  for (int p = 0; p < kRadixPasses; ++p) {
    const bool even = (p & 1) == 0;
    hipLaunchKernelGGL(radix_pass<false>, dim3(tiles), dim3(kTB), 0, st, even ? k0 : k1, even ? v0 : v1,
                       even ? k1 : k0, even ? v1 : v0, n, p, sc.ctl.p,
                       sc.status.p + (size_t)p * sc.tiles_cap * kRadixDigits, gate, n_dev, stamps_on(), nullptr,
                       nullptr, nullptr);
    FLOAM_LAUNCH_CHECK();
  }
}

}  // namespace floam
