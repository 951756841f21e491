// PointCloud2 decoding and the dense double-affine cloud transform on gfx950 (see formats.hpp).
//
// pc2_decode: one 64-lane wave per 64 points.  A point's record is assembled in registers as eight dwords: every
// mapped byte range is copied byte by byte from the message (field offsets need not be aligned, point_step need
// not be a multiple of 4), unmapped bytes stay zero (pcl::PointCloud::resize value-initialises the points), and
// the record is written with two 16-B stores.  The message is read once (the bytes of a wave's 64 points are
// contiguous, so the byte loads of a wave fall in a few cache lines and are served by L1/L2 after the first).
#include "formats.hpp"

namespace floam {
namespace {
constexpr int kTB = 256;

__global__ __launch_bounds__(kTB) void pc2_decode(Pc2Decode d, PointRec* __restrict__ out) {
  const long long n = (long long)d.width * d.height;
  const long long i = (long long)blockIdx.x * kTB + threadIdx.x;
  if (i >= n) return;
  const int row = (int)(i / d.width), col = (int)(i - (long long)row * d.width);
  const uint8_t* __restrict__ src = d.data + row * d.row_step + (long long)col * d.point_step;
  uint32_t w[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  if (d.whole) {
#pragma unroll 8
    for (int b = 0; b < 32; ++b) w[b >> 2] |= (uint32_t)src[b] << (8 * (b & 3));
  } else {
    for (int m = 0; m < d.nmap; ++m) {
      const Pc2Mapping mp = d.map[m];
      for (int b = 0; b < mp.size; ++b) {
        const int o = mp.struct_offset + b;
        w[o >> 2] |= (uint32_t)src[mp.serialized_offset + b] << (8 * (o & 3));
      }
    }
  }
  uint4* dst = reinterpret_cast<uint4*>(out + i);
  dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
  dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

__global__ __launch_bounds__(kTB) void transform_cloud(const PointRec* __restrict__ in, const int* __restrict__ d_n,
                                                       int n_ub, PointRec* __restrict__ out, double m00, double m01,
                                                       double m02, double m03, double m10, double m11, double m12,
                                                       double m13, double m20, double m21, double m22, double m23) {
  const int i = blockIdx.x * kTB + threadIdx.x;
  if (i >= n_ub || i >= *d_n) return;
  PointRec p = in[i];
  const double x = p.x, y = p.y, z = p.z;
  p.x = (float)(((m00 * x + m01 * y) + m02 * z) + m03);
  p.y = (float)(((m10 * x + m11 * y) + m12 * z) + m13);
  p.z = (float)(((m20 * x + m21 * y) + m22 * z) + m23);
  out[i] = p;
}
}  // namespace

void pc2_decode_launch(const Pc2Decode& d, PointRec* out, hipStream_t st) {
  const long long n = (long long)d.width * d.height;
  if (n <= 0) return;
  hipLaunchKernelGGL(pc2_decode, dim3(div_up((size_t)n, kTB)), dim3(kTB), 0, st, d, out);
  FLOAM_LAUNCH_CHECK();
}

void transform_cloud_launch(const PointRec* in, const int* d_n, int n_ub, const double* m, PointRec* out,
                            hipStream_t st) {
  if (n_ub <= 0) return;
  hipLaunchKernelGGL(transform_cloud, dim3(div_up(n_ub, kTB)), dim3(kTB), 0, st, in, d_n, n_ub, out, m[0], m[1],
                     m[2], m[3], m[4], m[5], m[6], m[7], m[8], m[9], m[10], m[11]);
  FLOAM_LAUNCH_CHECK();
}

}  // namespace floam
