#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace floam {
size_t sort_pairs_temp_bytes(int n);
size_t scan_temp_bytes(int n);
// stable LSD radix sort of (key, value) pairs on bits [0, end_bit)
void sort_pairs_u32(void* temp, size_t temp_bytes, const uint32_t* kin, uint32_t* kout, const int* vin, int* vout,
                    int n, int end_bit, hipStream_t st);
void exclusive_scan_i32(void* temp, size_t temp_bytes, const int* in, int* out, int n, hipStream_t st);
}  // namespace floam
