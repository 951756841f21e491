// Reduced reproducer of the LLVM exec-mask pattern that corrupted lm_solve once (profiles/r05m).
//
// Source shape: a divergent if (t < 64) whose body ends with a nested divergent if (t == 0) — the control step's
// lane-0 write-back inside the wave-0 branch of lm_solve.  Both ifs end at the same point.  With LLVM's default
// -amdgpu-remove-redundant-endcf=true the inner if's exec restore is removed as "redundant" with the outer one's, so
// the inner if lowers to `s_and_b64 exec, exec, vcc` (the mask narrowed WITHOUT saving it) and only the outer restore
// remains.  Any instruction the register allocator later places at the top of the shared join block (in lm_solve:
// accumulation-register restores) then runs under the inner mask, for lane 0 only.  Nothing in the source is a
// divergence hazard: the inner branch has no barrier, no cross-lane operation, no early exit.
//
// tests/test_codegen.py compiles this file twice and checks that the default pipeline emits the unsaved narrowing
// and that -mllvm -amdgpu-remove-redundant-endcf=false (floam_amd/csrc/Makefile) does not: the pattern is the
// compiler's, and the flag is what removes it.
#include <hip/hip_runtime.h>

__global__ void endcf_repro(double* out, const double* in, int n) {
  __shared__ double s[256];
  const int t = threadIdx.x;
  const double acc = in[t];
  s[t] = acc;
  __syncthreads();
  if (t < 64) {   // the outer divergent if (lm_solve: wave 0 runs the control step)
    double v = s[t] * 2.0 + s[(t + 1) & 255];
    for (int i = 0; i < n; ++i) v = v * 1.0001 + s[(t + i) & 255];
    if (t == 0) out[blockIdx.x] = v;   // the nested if ending with it (lm_solve: lane 0's state write-back)
  }
  out[gridDim.x + blockIdx.x * 256 + t] = acc;
}
