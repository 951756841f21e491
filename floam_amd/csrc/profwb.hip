// See profwb.hpp.
#include "profwb.hpp"

#include <cstdlib>

#include "floam_common.hpp"

namespace floam {
namespace {
// every block's first wave issues a system-scope release: the L2 of its XCD writes back its dirty lines.  64 blocks
// reach all eight XCDs under round-robin dispatch (MI355X_MICROARCH.md "Workgroup dispatch").
__global__ void l2_writeback() {
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}
}  // namespace

bool prof_wb_enabled() {
  static const bool on = [] {
    const char* e = FLOAM_DIAG_ENV("FLOAM_PROF_WB");
    return e && e[0] == '1';
  }();
  return on;
}

void prof_l2_writeback(hipStream_t st) {
  hipLaunchKernelGGL(l2_writeback, dim3(64), dim3(64), 0, st);
  FLOAM_LAUNCH_CHECK();
}
}  // namespace floam
