// Single-pass decoupled-lookback prefix over tiles, for two independent counters at once (device helper).
//
// Each tile of a launch takes a ticket (its logical index, so a tile only ever waits on tiles that were already
// running), publishes its aggregate, walks back over its predecessors' published words until one carries an
// inclusive prefix, and publishes its own inclusive prefix.  A status word is 64 bits: flag (2) | b (31) | a (31),
// stored and loaded with agent-scope atomics, so payload and flag travel together.  The status array and the ticket
// counter must be zero before the launch.
#pragma once
#include "floam_common.hpp"

namespace floam {

struct Prefix2 {
  int a, b;
};

constexpr unsigned long long kLbAggregate = 1ull << 62, kLbInclusive = 2ull << 62;

__device__ __forceinline__ unsigned long long lb_pack(unsigned long long flag, int a, int b) {
  return flag | ((unsigned long long)(unsigned)b << 31) | (unsigned long long)(unsigned)a;
}

// Called by ALL threads of the block (contains barriers).  Returns the tile's exclusive prefix; tile = ticket.
// Wave 0 looks back over a window of 64 predecessors at once (one status word per lane): the nearest inclusive
// prefix in the window ends the walk, otherwise the whole window's aggregates are added and the window moves back.
// The wait on a predecessor is bounded (~1 s); on timeout the prefix comes back with a = -1 (caller reports it).
__device__ __forceinline__ Prefix2 lookback_prefix(unsigned long long* __restrict__ status, int tile, Prefix2 agg) {
  __shared__ Prefix2 s_prefix;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    if (tile == 0) {
      if (lane == 0) {
        __hip_atomic_store(&status[0], lb_pack(kLbInclusive, agg.a, agg.b), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        s_prefix = Prefix2{0, 0};
      }
    } else {
      if (lane == 0)
        __hip_atomic_store(&status[tile], lb_pack(kLbAggregate, agg.a, agg.b), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      long long pa = 0, pb = 0;
      bool failed = false;
      long long polls = 0;
      for (int hi = tile - 1; hi >= 0;) {   // window [hi - 63, hi]; lane k reads tile hi - k
        const int j = hi - lane;
        unsigned long long w = kLbInclusive;   // beyond tile 0: acts as an inclusive zero
        if (j >= 0) w = __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long flag = w & (3ull << 62);
        const unsigned long long incl = __ballot(flag == kLbInclusive);
        const int stop = incl ? __ffsll((long long)incl) - 1 : 63;   // nearest inclusive lane (or whole window)
        const unsigned long long notready = __ballot(flag == 0) & ((stop == 63) ? ~0ull : ((2ull << stop) - 1ull));
        if (notready) {
          if (++polls > (1ll << 24)) { failed = true; break; }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        long long va = (lane <= stop && j >= 0) ? (long long)(w & 0x7FFFFFFFull) : 0;
        long long vb = (lane <= stop && j >= 0) ? (long long)((w >> 31) & 0x7FFFFFFFull) : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          va += __shfl_xor(va, o, 64);
          vb += __shfl_xor(vb, o, 64);
        }
        pa += va;
        pb += vb;
        if (incl) break;
        hi -= 64;
      }
      if (lane == 0) {
        if (failed) {
          s_prefix = Prefix2{-1, 0};
        } else {
          __hip_atomic_store(&status[tile], lb_pack(kLbInclusive, (int)pa + agg.a, (int)pb + agg.b),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_prefix = Prefix2{(int)pa, (int)pb};
        }
      }
    }
  }
  __syncthreads();
  const Prefix2 r = s_prefix;
  __syncthreads();
  return r;
}

// The block's ticket (logical tile index), taken by thread 0 and broadcast.
__device__ __forceinline__ int lookback_ticket(unsigned* __restrict__ counter) {
  __shared__ int s_tile;
  if (threadIdx.x == 0) s_tile = (int)atomicAdd(counter, 1u);
  __syncthreads();
  const int t = s_tile;
  __syncthreads();
  return t;
}

}  // namespace floam
