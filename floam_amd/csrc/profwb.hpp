// Diagnostic (FLOAM_PROF_WB=1, profiling runs only): an L2 write-back dispatch bracketing the kernels whose HBM write
// counters are being attributed.  WRITE_SIZE counts the L2's write-backs to the fabric during a
// dispatch, whoever dirtied the lines: with every XCD's L2 written back just before a kernel, nothing it evicts is an
// earlier kernel's, and the lines it leaves dirty are written back by the dispatch after it — so its own write bytes
// are WRITE_SIZE(kernel) + WRITE_SIZE(the write-back after it).
#pragma once
#include <hip/hip_runtime.h>

namespace floam {
bool prof_wb_enabled();                    // FLOAM_PROF_WB=1, read once
void prof_l2_writeback(hipStream_t st);    // one system-scope release per XCD (buffer_wbl2), no memory traffic of its own
}  // namespace floam
