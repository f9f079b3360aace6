// LiDAR BEV voxelisation: the sweep-to-current-ego transform
// (dataset.py:319-340 -> utils.transform_points, utils.py:27-33) fused with the height-sliced
// intensity scatter-max of utils.create_intentnet_lidar_bev (utils.py:62-106).
//
// One thread per point, blockIdx.y = sweep. The transform and the binning follow the
// reference's operation order and precision (see bin_point); no implicit FMA contraction:
// every product / sum / quotient rounds as numpy's does. The scatter-max is a signed-int atomicMax on the f32 bit pattern: the
// raster starts at +0 (np.zeros) and only intensities > 0 can raise a cell, and for
// non-negative IEEE floats integer order == float order; NaN intensities store a canonical +NaN
// (np.maximum propagates NaN and nothing replaces it). HBM-bound on the caller's zero fill; the
// scatter itself is ~12 B per point.
#include "ivit_common.h"

#pragma clang fp contract(off)

namespace {

// Binning precision C follows numpy's promotion in the reference: points that went through
// transform_points are f64 (dataset path), and f64 input stays f64; f32 points handed in
// directly are binned in f32 (f32 array op Python float -> f32 under both legacy value-based
// casting and NEP 50), including the z < Z_MAX test against f32(3.8).
template <typename C>
IVIT_DEV bool bin_point(C x, C y, C z, int H, int W, int HC, double voxel, double offx, double offy, double zmin,
                        double zmax, double zrange, long& fy_out, long& fx_out, long& hz_out) {
  const C fx = floor((C)offx + y / (C)voxel);  // utils.py:80
  const C fy = floor((C)offy - x / (C)voxel);  // utils.py:81
  if (!(fx >= (C)0 && fx < (C)W && fy >= (C)0 && fy < (C)H && z >= (C)zmin && z < (C)zmax)) return false;
  long hz = (long)floor((z - (C)zmin) / (C)zrange * (C)HC);  // utils.py:95-96
  hz_out = hz < 0 ? 0 : (hz > HC - 1 ? HC - 1 : hz);
  fy_out = (long)fy;
  fx_out = (long)fx;
  return true;
}

template <typename P>
__global__ void lidar_bev_kernel(const P* __restrict__ pts, long ld, const float* __restrict__ inten,
                                 const long* __restrict__ start, const double* __restrict__ tf,
                                 const int* __restrict__ plane, float* __restrict__ bev, int H, int W, int HC,
                                 double voxel, double offx, double offy, double zmin, double zmax, double zrange) {
  const int s = blockIdx.y;
  const long p = start[s] + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= start[s + 1]) return;
  const P* q = pts + p * ld;
  long fy, fx, hz;
  bool in;
  if (tf) {  // transform_points: (T @ [x y z 1]^T)[:3], row-major 4x4, f64
    // numpy's f64 matmul (BLAS dgemm) accumulates k = 0..3 as an FMA chain from t0*x; this order
    // reproduces it bit for bit (checked against the reference's transform_points in
    // oracle/make_golden.py; a plain mul+add chain differs in ~50% of the coordinates by 1 ulp).
    const double* t = tf + (long)s * 16;
    const double x = (double)q[0], y = (double)q[1], z = (double)q[2];
    const double xe = fma(t[2], z, fma(t[1], y, t[0] * x)) + t[3];
    const double ye = fma(t[6], z, fma(t[5], y, t[4] * x)) + t[7];
    const double ze = fma(t[10], z, fma(t[9], y, t[8] * x)) + t[11];
    in = bin_point<double>(xe, ye, ze, H, W, HC, voxel, offx, offy, zmin, zmax, zrange, fy, fx, hz);
  } else {
    in = bin_point<P>(q[0], q[1], q[2], H, W, HC, voxel, offx, offy, zmin, zmax, zrange, fy, fx, hz);
  }
  if (!in) return;
  const float v = inten[p];
  if (!(v > 0.f) && v == v) return;  // max(cell, v) == cell for v <= 0 (cells start at +0)
  const long cell = ((long)(plane[s] + hz) * H + fy) * W + fx;
  const int bits = v == v ? __float_as_int(v) : 0x7fc00000;
  atomicMax((int*)bev + cell, bits);
}

}  // namespace

extern "C" int ivit_lidar_bev(const void* points, int points_f64, long ld, const float* intensity,
                              const long* sweep_start, long n_sweeps, long max_points, const double* sweep_tf,
                              const int* sweep_plane, float* bev, long H, long W, long height_channels,
                              double voxel, double off_x, double off_y, double z_min, double z_max,
                              double z_range, void* stream) {
  if (n_sweeps <= 0 || max_points <= 0) return 0;
  IVIT_CHECK_ARG(ld >= 3, "ivit_lidar_bev: point rows need x, y, z (ld=%ld)", ld);
  IVIT_CHECK_ARG(n_sweeps < 65536, "ivit_lidar_bev: too many sweeps (%ld)", n_sweeps);
  IVIT_CHECK_ARG(H > 0 && W > 0 && height_channels > 0 && voxel > 0.0 && z_range > 0.0,
                 "ivit_lidar_bev: bad grid (H=%ld W=%ld C=%ld)", H, W, height_channels);
  dim3 g(ivit_cdiv(max_points, 256), n_sweeps);
  if (points_f64)
    hipLaunchKernelGGL(lidar_bev_kernel<double>, g, dim3(256), 0, ivit_stream(stream), (const double*)points, ld,
                       intensity, sweep_start, sweep_tf, sweep_plane, bev, (int)H, (int)W, (int)height_channels,
                       voxel, off_x, off_y, z_min, z_max, z_range);
  else
    hipLaunchKernelGGL(lidar_bev_kernel<float>, g, dim3(256), 0, ivit_stream(stream), (const float*)points, ld,
                       intensity, sweep_start, sweep_tf, sweep_plane, bev, (int)H, (int)W, (int)height_channels,
                       voxel, off_x, off_y, z_min, z_max, z_range);
  IVIT_LAUNCH_CHECK();
  return 0;
}
