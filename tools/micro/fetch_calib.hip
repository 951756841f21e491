// Calibration of rocprofv3's FETCH_SIZE for the access patterns of the kNN search (MI355X_MICROARCH.md § HBM: the
// x2 correction is measured for wide coalesced 16-B/lane streams only; "other access widths are uncalibrated").
//
// Every kernel reads a known number of bytes from a 1-GiB array (4x the 256-MiB Infinity Cache, fresh lines each
// kernel, so the reads reach the memory-side counters) and writes one float per thread:
//   stream    coalesced float4 per lane, consecutive                         bytes = threads * 16
//   gather1   one float4 per lane at a random 128-B line (lane-independent)  bytes = threads * 16, lines = threads
//   gather16  16-lane groups read 16 consecutive float4 (256 B) at a random 256-B-aligned base (the kNN's candidate
//             rows of a cell)                                              bytes = threads * 16, lines = threads / 8
// Usage (GPU box): rocprofv3 --pmc FETCH_SIZE --kernel-trace -d OUT -- ./fetch_calib; FETCH_SIZE (KiB) per kernel
// against the byte counts printed here.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

constexpr size_t kArrayBytes = size_t(1) << 30;
constexpr size_t kF4 = kArrayBytes / 16;   // float4 elements
constexpr int kThreads = 1 << 20;          // per kernel: 16 MiB requested

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__global__ void stream(const float4* __restrict__ a, size_t base, float* __restrict__ out) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  const float4 v = a[base + t];
  out[t] = v.x + v.y + v.z + v.w;
}

__global__ void gather1(const float4* __restrict__ a, unsigned seed, float* __restrict__ out) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  const size_t line = hash32(t ^ seed) % (kArrayBytes / 128);
  const float4 v = a[line * 8 + (t & 7)];
  out[t] = v.x + v.y + v.z + v.w;
}

__global__ void gather16(const float4* __restrict__ a, unsigned seed, float* __restrict__ out) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  const size_t row = hash32((t >> 4) ^ seed) % (kArrayBytes / 256);
  const float4 v = a[row * 16 + (t & 15)];
  out[t] = v.x + v.y + v.z + v.w;
}

int main() {
  float4* a;
  float* out;
  CHECK(hipMalloc(&a, kArrayBytes));
  CHECK(hipMalloc(&out, sizeof(float) * kThreads));
  CHECK(hipMemset(a, 0, kArrayBytes));
  CHECK(hipDeviceSynchronize());
  const dim3 g(kThreads / 256), b(256);
  for (int rep = 0; rep < 3; ++rep) {
    // each kernel touches a region no earlier kernel of this process touched since the cache was last swept
    hipLaunchKernelGGL(stream, g, b, 0, 0, a, (size_t)(rep % 3) * (kF4 / 3), out);
    hipLaunchKernelGGL(gather1, g, b, 0, 0, a, 0x1234u + 7u * rep, out);
    hipLaunchKernelGGL(gather16, g, b, 0, 0, a, 0x9876u + 13u * rep, out);
    CHECK(hipDeviceSynchronize());
  }
  std::printf("threads per kernel %d: requested bytes %zu (16 B per lane); stream lines %zu, gather1 lines %d "
              "(128 B each), gather16 rows %d (256 B each)\n",
              kThreads, (size_t)kThreads * 16, (size_t)kThreads * 16 / 128, kThreads, kThreads / 16);
  CHECK(hipFree(a));
  CHECK(hipFree(out));
  return 0;
}
