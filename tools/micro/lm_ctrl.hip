// Latency of the pieces of one resident-solve evaluation (lm.hip), inside one 256-thread block, measured with
// s_memrealtime (100 MHz) over repeated calls on a synthetic, well-conditioned state (diagnostic):
//   control step (iteration zero + step; accepted candidate + step), solve_step, se3_plus, the surf half from G
//   (one wave), one edge record's residual + Jacobian + accumulation, block_sums over 192 record threads.
// Build + run (GPU box): hipcc -O3 -std=c++17 -ffp-contract=fast --offload-arch=gfx950 tools/micro/lm_ctrl.hip
//                        -o /tmp/lm_ctrl && /tmp/lm_ctrl
#include "../../floam_amd/csrc/lm.hip"

#include <cstdio>

namespace floam {
namespace {
__global__ __launch_bounds__(256) void ctrl_bench(unsigned long long* out, double* sink) {
  __shared__ LMState sst;
  __shared__ double sums[LM_NSUM];
  __shared__ double G[kGramW][kGramW];
  __shared__ double o[3];
  __shared__ double ssum[LM_NSUM];
  __shared__ double red[LM_NSUM * 193];
  __shared__ double pt[7];
  const int t = threadIdx.x, lane = t & 63;
  unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
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
    LMState s;
    if (t < 64) s = sst;
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (t < 64) control_step(s, sst, sums, lane);   // IterationZero + the first step
    __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (t < LM_NSUM) sums[t] = t == 0 ? 49.0 : sums[t];
    __syncthreads();
    unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    if (t < 64) control_step(s, sst, sums, lane);   // candidate accepted + the next step
    __syncthreads();
    unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    if (t < 7) pt[t] = s.x[t];
    __syncthreads();
    unsigned long long t4 = __builtin_amdgcn_s_memrealtime();
    if (t < 64) surf_sums_wave(pt, o, G, 20000.0, ssum, lane);
    __syncthreads();
    unsigned long long t5 = __builtin_amdgcn_s_memrealtime();
    double delta[6];
    bool ok = false;
    if (t < 64) ok = solve_step(s, delta);
    __syncthreads();
    unsigned long long t6 = __builtin_amdgcn_s_memrealtime();
    double xo[7];
    if (t < 64) {
      double d[6];
#pragma unroll
      for (int k = 0; k < 6; ++k) d[k] = ok ? delta[k] : 1e-3 * (k + 1);
      se3_plus(s.x, d, xo);
    }
    __syncthreads();
    unsigned long long t7 = __builtin_amdgcn_s_memrealtime();
    double accd[LM_NSUM];
    {
      double x[7], f[9];
#pragma unroll
      for (int k = 0; k < 7; ++k) x[k] = pt[k];
#pragma unroll
      for (int k = 0; k < 9; ++k) f[k] = 0.3 * k + 0.01 * t + (k == 3 ? 1.0 : 0.0);
      eval_records<false, double>(x, true, true, f, 1 << 30, 1, 0, 0, nullptr, nullptr, 0, nullptr, nullptr, 0, accd);
    }
    __syncthreads();
    unsigned long long t8 = __builtin_amdgcn_s_memrealtime();
    const double v = block_sums<192>(accd, red);
    __syncthreads();
    unsigned long long t9 = __builtin_amdgcn_s_memrealtime();
    acc[0] += t1 - t0;
    acc[1] += t3 - t2;
    acc[2] += t5 - t4;
    acc[3] += t6 - t5;
    acc[4] += t7 - t6;
    acc[5] += t8 - t7;
    acc[6] += t9 - t8;
    acc[7] += s.iteration;
    if (t < 58) sink[rep * 64 + t] = s.cand[4] + ssum[3] + xo[t % 7] + v;
    __syncthreads();
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    for (int k = 0; k < 8; ++k) out[k] = acc[k];
    out[8] = c1 - c0;
    out[9] = r1 - r0;
  }
}
}  // namespace
}  // namespace floam

int main() {
  unsigned long long* d;
  double* sink;
  hipMalloc(&d, 80);
  hipMalloc(&sink, 64 * 64 * sizeof(double));
  for (int r = 0; r < 3; ++r) {
    hipLaunchKernelGGL(floam::ctrl_bench, dim3(1), dim3(256), 0, 0, d, sink);
    hipDeviceSynchronize();
  }
  unsigned long long h[10];
  hipMemcpy(h, d, 80, hipMemcpyDeviceToHost);
  std::printf("shader clock during the run: %.0f MHz (s_memtime / s_memrealtime)\n", 100.0 * h[8] / (double)h[9]);
  const char* names[7] = {"control step (iteration zero + step)", "control step (accept + step)", "surf half (one wave)",
                          "solve_step", "se3_plus", "edge record eval + accumulate", "block_sums<192>"};
  for (int k = 0; k < 7; ++k) std::printf("%-40s %6.2f us\n", names[k], h[k] / 64.0 / 100.0);
  std::printf("(iterations %llu)\n", h[7]);
  return 0;
}
