// Device-wide sort / scan primitives (rocPRIM, header-only, ROCm 7.2).  Isolated in one translation unit so the
// template-heavy instantiations compile once; everything else in the core is hand-written HIP.
#include <cstring>  // rocprim/iterator/texture_cache_iterator.hpp uses memset without including it

#include <rocprim/rocprim.hpp>

#include "floam_common.hpp"
#include "primitives.hpp"

namespace floam {

size_t sort_pairs_temp_bytes(int n) {
  size_t bytes = 0;
  FLOAM_HIP(rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                      (const int*)nullptr, (int*)nullptr, (size_t)n, 0, 32));
  return bytes;
}

size_t scan_temp_bytes(int n) {
  size_t bytes = 0;
  FLOAM_HIP(rocprim::exclusive_scan(nullptr, bytes, (const int*)nullptr, (int*)nullptr, 0, (size_t)n,
                                    rocprim::plus<int>()));
  return bytes;
}

void sort_pairs_u32(void* temp, size_t temp_bytes, const uint32_t* kin, uint32_t* kout, const int* vin, int* vout,
                    int n, int end_bit, hipStream_t st) {
  if (n <= 0) return;
  size_t b = temp_bytes;
  FLOAM_HIP(rocprim::radix_sort_pairs(temp, b, kin, kout, vin, vout, (size_t)n, 0, end_bit, st));
}

void exclusive_scan_i32(void* temp, size_t temp_bytes, const int* in, int* out, int n, hipStream_t st) {
  if (n <= 0) return;
  size_t b = temp_bytes;
  FLOAM_HIP(rocprim::exclusive_scan(temp, b, in, out, 0, (size_t)n, rocprim::plus<int>(), st));
}

}  // namespace floam
