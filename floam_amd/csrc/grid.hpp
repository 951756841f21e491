// Cell coordinates and 64-bit keys of the two-level hash grid (device helpers shared by grid.hip and the kNN).
#pragma once
#include "floam_common.hpp"

namespace floam {

// fine cell (edge 0.5 m) of a float point: floor(v / 0.5) in double is exact (v is a float, the division is a
// power-of-two scaling), so cell bounds are exact and the kNN's distance bounds hold exactly
__device__ __forceinline__ void fine_cell(float x, float y, float z, int& fx, int& fy, int& fz) {
  fx = (int)floor((double)x * 2.0);
  fy = (int)floor((double)y * 2.0);
  fz = (int)floor((double)z * 2.0);
}

// 21 bits per axis, offset 2^20 (cells within +-2^20 of the origin: +-524 km for fine cells); clamped
__device__ __forceinline__ unsigned long long cell_key(int x, int y, int z) {
  const int lim = (1 << 20) - 1;
  x = min(max(x, -lim), lim);
  y = min(max(y, -lim), lim);
  z = min(max(z, -lim), lim);
  return ((unsigned long long)(unsigned)(z + (1 << 20)) << 42) | ((unsigned long long)(unsigned)(y + (1 << 20)) << 21) |
         (unsigned long long)(unsigned)(x + (1 << 20));
}
__device__ __forceinline__ int key_x(unsigned long long k) { return (int)(k & 0x1FFFFFull) - (1 << 20); }
__device__ __forceinline__ int key_y(unsigned long long k) { return (int)((k >> 21) & 0x1FFFFFull) - (1 << 20); }
__device__ __forceinline__ int key_z(unsigned long long k) { return (int)(k >> 42) - (1 << 20); }

__device__ __forceinline__ unsigned hash_slot64(unsigned long long key, int bits) {
  return (unsigned)((key * 0x9E3779B97F4A7C15ull) >> (64 - bits));
}

}  // namespace floam
