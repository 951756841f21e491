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
// The wait on a predecessor is bounded (~1 s); on timeout the prefix comes back with a = -1 (caller reports it).
__device__ __forceinline__ Prefix2 lookback_prefix(unsigned long long* __restrict__ status, int tile, Prefix2 agg) {
  __shared__ Prefix2 s_prefix;
  if (threadIdx.x == 0) {
    Prefix2 pre{0, 0};
    if (tile == 0) {
      __hip_atomic_store(&status[0], lb_pack(kLbInclusive, agg.a, agg.b), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_store(&status[tile], lb_pack(kLbAggregate, agg.a, agg.b), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      long long polls = 0;
      for (int j = tile - 1; j >= 0;) {
        const unsigned long long w = __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long flag = w & (3ull << 62);
        if (flag == 0) {
          if (++polls > (1ll << 24)) {
            pre.a = -1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        pre.a += (int)(w & 0x7FFFFFFFull);
        pre.b += (int)((w >> 31) & 0x7FFFFFFFull);
        if (flag == kLbInclusive) break;
        --j;
      }
      if (pre.a >= 0)
        __hip_atomic_store(&status[tile], lb_pack(kLbInclusive, pre.a + agg.a, pre.b + agg.b), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    s_prefix = pre;
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
