// IMU pre-processing kernel (CenterTime + dmapping::Compensate + IMU alignment), gfx950.  See imu.hpp.
//
// One thread per point, 256-thread workgroups.  Per point: the 32-B record is read once (two dwordx4 loads,
// coalesced), the centred time is written back into the caller's cloud (CenterTime mutates it), the IMU sample
// is found by a binary search over the LDS-staged stamp window (ImuHandler::Get's lower_bound, the sample before
// it), the orientation is read from HBM (a handful of distinct 32-B rows per workgroup: L1/L2 hits), and the
// rotated record is written once.  All arithmetic is double with float stores, operation order as the reference
// (built with -ffp-contract=off), so the output is bit-identical to the CPU oracle.
#include "imu.hpp"

namespace floam {
namespace {
constexpr int kTB = 256;

// std::lower_bound over stamps[lo, lo + count)
__device__ __forceinline__ int lower_bound_range(const double* __restrict__ s, int lo, int count, double t) {
  int first = lo;
  while (count > 0) {
    const int step = count >> 1, it = first + step;
    if (s[it] < t) {
      first = it + 1;
      count -= step + 1;
    } else {
      count = step;
    }
  }
  return first;
}

template <int MODE>
__global__ __launch_bounds__(kTB) void imu_prep(PointRec* __restrict__ in, PointRec* __restrict__ out,
                                                const int* __restrict__ d_n, int n_ub, ImuPrepArgs a) {
  __shared__ double win[kImuWindow];
  const int n = min(*d_n, n_ub);
  const int wn = a.win_hi - a.win_lo;
  if (MODE & IMU_COMPENSATE) {
    for (int k = threadIdx.x; k < wn; k += kTB) win[k] = a.stamps[a.win_lo + k];
    __syncthreads();
  }
  const int i = blockIdx.x * kTB + threadIdx.x;
  if (i >= n) return;
  PointRec p = in[i];
  float tc = p.time;
  if (MODE & IMU_CENTER) {
    tc = (float)(((double)p.time + a.tScan) - a.tCenter);   // pnt.time + tScan - tCenter
    in[i].time = tc;
  }
  if (MODE & IMU_COMPENSATE) {
    const double tcur = a.tScan2 + (double)tc;
    int idx;
    if (wn > 0 && tcur > win[0] && tcur <= win[wn - 1])
      idx = a.win_lo + lower_bound_range(win, 0, wn, tcur);   // the window decides: lower bound in (lo, hi - 1]
    else
      idx = lower_bound_range(a.stamps, 0, a.n_imu, tcur);
    Q4 qs{0.0, 0.0, 0.0, 0.0};   // default-constructed sensor_msgs::Imu when Get fails
    if (idx != a.n_imu && idx != 0 && idx - 1 != 0) qs = a.orient[idx - 1];
    const Q4 qNow = q4_mul(qs, a.extr);
    const Q4 q = q4_mul(a.qInitInv, qNow);
    // Eigen _transformVector: uv = q.vec x v; uv += uv; v + w * uv + q.vec x uv
    const double vx = p.x, vy = p.y, vz = p.z;
    double ux = q.y * vz - q.z * vy, uy = q.z * vx - q.x * vz, uz = q.x * vy - q.y * vx;
    ux = ux + ux; uy = uy + uy; uz = uz + uz;
    const double ax = vx + q.w * ux, ay = vy + q.w * uy, az = vz + q.w * uz;
    float cx = (float)(ax + (q.y * uz - q.z * uy));
    float cy = (float)(ay + (q.z * ux - q.x * uz));
    float cz = (float)(az + (q.x * uy - q.y * ux));
    if (MODE & IMU_ALIGN) {
      const double px = cx, py = cy, pz = cz;
      const double* R = a.R;
      cx = (float)(((R[0] * px + R[1] * py) + R[2] * pz) + 0.0);
      cy = (float)(((R[3] * px + R[4] * py) + R[5] * pz) + 0.0);
      cz = (float)(((R[6] * px + R[7] * py) + R[8] * pz) + 0.0);
    }
    PointRec o;
    o.x = cx; o.y = cy; o.z = cz; o.pad0 = 1.0f;
    o.intensity = p.intensity; o.ring = p.ring; o.pad1 = 0; o.time = tc; o.pad2 = 0.0f;
    out[i] = o;
  }
}

__global__ void cloud_ends(const PointRec* __restrict__ pts, const int* __restrict__ d_n, int* __restrict__ dst) {
  if (threadIdx.x != 0) return;
  const int n = *d_n;
  dst[0] = n;
  dst[1] = n > 0 ? __float_as_int(pts[0].time) : 0;
  dst[2] = n > 0 ? __float_as_int(pts[n - 1].time) : 0;
}
}  // namespace

void imu_prep_launch(int mode, PointRec* in, PointRec* out, const int* d_n, int n_ub, const ImuPrepArgs& a,
                     hipStream_t st) {
  if (n_ub <= 0) return;
  if (a.win_hi - a.win_lo > kImuWindow || a.win_lo < 0 || a.win_hi > a.n_imu)
    throw Error(FLOAM_ERR_INVALID_ARGUMENT, "IMU stamp window out of range");
  const dim3 g(div_up(n_ub, kTB)), b(kTB);
  switch (mode) {
    case IMU_CENTER: hipLaunchKernelGGL(imu_prep<IMU_CENTER>, g, b, 0, st, in, out, d_n, n_ub, a); break;
    case IMU_COMPENSATE: hipLaunchKernelGGL(imu_prep<IMU_COMPENSATE>, g, b, 0, st, in, out, d_n, n_ub, a); break;
    case IMU_COMPENSATE | IMU_ALIGN:
      hipLaunchKernelGGL((imu_prep<IMU_COMPENSATE | IMU_ALIGN>), g, b, 0, st, in, out, d_n, n_ub, a);
      break;
    case IMU_CENTER | IMU_COMPENSATE | IMU_ALIGN:
      hipLaunchKernelGGL((imu_prep<IMU_CENTER | IMU_COMPENSATE | IMU_ALIGN>), g, b, 0, st, in, out, d_n, n_ub, a);
      break;
    default: throw Error(FLOAM_ERR_INVALID_ARGUMENT, "unsupported IMU pre-processing mode");
  }
  FLOAM_LAUNCH_CHECK();
}

void cloud_ends_launch(const PointRec* pts, const int* d_n, int* dst, hipStream_t st) {
  hipLaunchKernelGGL(cloud_ends, dim3(1), dim3(64), 0, st, pts, d_n, dst);
  FLOAM_LAUNCH_CHECK();
}

}  // namespace floam
