// Stable LSD radix sort of (u32 key, i32 value) pairs for the VoxelGrid pipeline (voxel.hip): 8-bit digits, one
// single-pass ("onesweep") launch per digit — tile ranking by wave-level digit matching, per-digit decoupled
// lookback across tiles, scatter — with the four digit histograms accumulated by the key-producing kernel.
#pragma once
#include "floam_common.hpp"

namespace floam {

constexpr int kRadixDigits = 256;
constexpr int kRadixPasses = 4;
constexpr int kRadixHistWords = kRadixPasses * kRadixDigits;   // followed by 4 spare words + 1 error word
constexpr int kRadixErrorWord = kRadixHistWords + 4;            // != 0: a lookback timed out
constexpr int kRadixZeroWords = kRadixHistWords + 5;            // zeroed per sort
constexpr int kRadixEpochWord = kRadixHistWords + 5;            // sort counter (tags the lookback words)
// [pass]: the pass's tile tickets, on a 128-B line of their own (the every-block reads of the epoch and the
// histograms would otherwise queue behind the tickets' atomics), zeroed per sort with the words above
constexpr int kRadixTicketWord = kRadixHistWords + 32;
constexpr int kRadixCtlWords = kRadixHistWords + 64;

struct RadixScratch {
  DevBuf<unsigned> ctl;                  // [4][256] digit histograms, [4] tickets, [1] error (zeroed per sort),
                                         // [1] the sort counter (advanced per sort on the device)
  DevBuf<unsigned long long> status;     // [4][tiles][256] lookback words, tagged with the sort's epoch
  int tiles_cap = 0;
  void reserve(int n, hipStream_t st);
};

// Producer side (inside the kernel that writes the keys; all threads of the block call both):
//   radix_hist_begin(s_hist)            zero a [1024] LDS histogram
//   radix_hist_add(s_hist, key)         per key (LDS atomics)
//   radix_hist_end(s_hist, ctl)         fold the block's histogram into ctl (global atomics, non-zero bins)
// ctl must be zero before the producer runs (radix_ctl_zero, e.g. from an earlier kernel of the same stream).
__device__ __forceinline__ void radix_hist_begin(unsigned* s_hist) {
  for (int k = threadIdx.x; k < kRadixHistWords; k += blockDim.x) s_hist[k] = 0u;
  __syncthreads();
}
__device__ __forceinline__ void radix_hist_add(unsigned* s_hist, uint32_t key) {
#pragma unroll
  for (int p = 0; p < kRadixPasses; ++p) atomicAdd(&s_hist[p * kRadixDigits + ((key >> (8 * p)) & 255u)], 1u);
}
__device__ __forceinline__ void radix_hist_end(const unsigned* s_hist, unsigned* ctl) {
  __syncthreads();
  for (int k = threadIdx.x; k < kRadixHistWords; k += blockDim.x) {
    const unsigned v = s_hist[k];
    if (v) atomicAdd(&ctl[k], v);
  }
}
// zero the per-sort words and advance the sort counter (epoch 0x3FFFFFFF is the fresh-array pattern: skipped)
__device__ __forceinline__ void radix_ctl_zero(unsigned* ctl, int t, int stride) {
  for (int k = t; k < kRadixZeroWords; k += stride) ctl[k] = 0u;
  for (int k = t; k < kRadixPasses; k += stride) ctl[kRadixTicketWord + k] = 0u;
  if (t == 0) {
    unsigned e = (ctl[kRadixEpochWord] + 1u) & 0x3FFFFFFFu;
    if (e == 0x3FFFFFFFu) e = 0u;
    ctl[kRadixEpochWord] = e;
  }
}

// The four passes: (k0, v0) -> (k1, v1) -> (k0, v0) -> (k1, v1) -> (k0, v0); the sorted pairs end in k0 / v0.
// n must be the element count the histograms were built over; radix_ctl_zero must have run since the last sort.  ctl[1028] != 0 afterwards if a lookback timed out
// (never expected; the consumer reports it).
// gate (device int, nullable): the passes do nothing when it reads 0.
// n_dev (device int, nullable): the element count actually sorted (<= n, which sizes the grid).
void radix_sort_launch(RadixScratch& sc, uint32_t* k0, int* v0, uint32_t* k1, int* v1, int n, hipStream_t st,
                       const int* gate = nullptr, const int* n_dev = nullptr);

// One digit pass (pass p sorts by bits [8p, 8p + 8)) of the same sort, for keys whose high digits are known to be
// equal (e.g. the feature extraction's ring keys: one pass for <= 255 rings)
// The first digit pass (pass 0) over elements in their original order (values = positions, not read) carrying each
// element's record: its coordinates to pxyz[dst] and the record to prec[dst] (the feature extraction's ring-major
// staging of the scan); kout / vout (nullable): the sorted keys and positions
void radix_pass_payload_launch(RadixScratch& sc, const uint32_t* kin, uint32_t* kout, int* vout, int n,
                               const PointRec* pin, float4* pxyz, PointRec* prec, hipStream_t st);

// FLOAM_RADIX_STAMPS=1: print the passes' in-kernel phase times (diagnostic; synchronises the device)
void radix_stamps_print();

void radix_pass_launch(RadixScratch& sc, const uint32_t* kin, const int* vin, uint32_t* kout, int* vout, int n,
                       int pass, hipStream_t st);

}  // namespace floam
