// Latency of the LM control step (lm_logic_wave0) and of the Gram surf sums (surf_sums_from_gram) inside one block,
// measured with s_memrealtime (100 MHz) over repeated calls on a synthetic, well-conditioned state (diagnostic).
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I floam_amd/csrc tools/micro/lm_ctrl.hip
#include "../../floam_amd/csrc/odom_kernels.hip"

#include <cstdio>

namespace floam {
__global__ __launch_bounds__(256) void ctrl_bench(unsigned long long* out, double* sink) {
  __shared__ LMState sst;
  __shared__ double sums[LM_NSUM];
  __shared__ double G[kGramW][kGramW];
  __shared__ double o[3];
  __shared__ double ssum[LM_NSUM];
  const int t = threadIdx.x;
  unsigned long long acc[4] = {0, 0, 0, 0};
  for (int rep = 0; rep < 64; ++rep) {
    if (t == 0) {
      LMState s{};
      s.x[3] = 1.0;
      s.x[4] = 0.1 + 1e-3 * rep;
      sst = s;
    }
    if (t < LM_NSUM) {   // cost, H (diagonally dominant), g, count
      double v;
      if (t == 0) v = 50.0;
      else if (t < 22) {
        int hh = t - 1, a = 0;
        while (hh >= 6 - a) { hh -= 6 - a; ++a; }
        v = hh == 0 ? 1000.0 + 10.0 * a : 3.0 + 0.1 * (a + hh);
      } else if (t < 28) v = 1.0 + 0.3 * (t - 22);
      else v = 20000.0;
      sums[t] = v;
    }
    if (t < kGramW * kGramW) G[t / kGramW][t % kGramW] = (t / kGramW == t % kGramW) ? 100.0 : 0.5;
    if (t < 3) o[t] = 0.0;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    lm_logic_wave0(sst, sums);   // IterationZero + the first step
    __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (t < LM_NSUM) sums[t] = t == 0 ? 49.0 : sums[t];
    __syncthreads();
    unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    lm_logic_wave0(sst, sums);   // candidate accepted + the next step
    __syncthreads();
    unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    double x[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) x[k] = sst.x[k];
    surf_sums_from_gram(x, o, G, 20000.0, ssum);
    unsigned long long t4 = __builtin_amdgcn_s_memrealtime();
    acc[0] += t1 - t0;
    acc[1] += t3 - t2;
    acc[2] += t4 - t3;
    acc[3] += sst.iteration;
    if (t == 0) sink[rep] = sst.cand[4] + ssum[3];
    __syncthreads();
  }
  if (t == 0)
    for (int k = 0; k < 4; ++k) out[k] = acc[k];
}
}  // namespace floam

int main() {
  unsigned long long* d;
  double* sink;
  hipMalloc(&d, 32);
  hipMalloc(&sink, 64 * sizeof(double));
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(floam::ctrl_bench, dim3(1), dim3(256), 0, 0, d, sink);
    hipDeviceSynchronize();
  }
  unsigned long long h[4];
  hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
#ifdef FLOAM_CTRL_STAMPS
  unsigned long long c[8];
  hipMemcpyFromSymbol(c, HIP_SYMBOL(floam::g_ctrl_stamps), sizeof(c));
  const double n = c[3] ? (double)c[3] : 1.0;
  std::printf("control stamps over %llu steps: solve_step %.2f us, se3_plus %.2f us, gmax+cand %.2f us, whole step %.2f us;"
              " per phase-0 prologue %.2f us, per phase-1 prologue %.2f us\n", c[3], c[0] / n / 100.0, c[1] / n / 100.0,
              c[5] / n / 100.0, c[2] / n / 100.0, c[4] / (n / 2) / 100.0, c[6] / (n / 2) / 100.0);
#endif
  std::printf("control step: iteration zero + step %.2f us, accept + step %.2f us; surf sums from G %.2f us "
              "(iterations %llu)\n", h[0] / 64.0 / 100.0, h[1] / 64.0 / 100.0, h[2] / 64.0 / 100.0, h[3]);
  return 0;
}
