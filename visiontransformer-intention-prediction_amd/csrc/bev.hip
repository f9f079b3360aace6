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

// ------------------------------------------------------------------------------------------
// BEV augmentation passes (utils.py:394-517). One launch runs one pass
// for every [C, H, W] stack of a batch (LiDAR and map stacks of all samples; blockIdx.z =
// pass entry). Each thread owns one output pixel: it derives its source taps and weights once
// (the same for every plane) and then streams CPB planes, so the map arithmetic is amortised
// and the pass is a read + write of the stack (HBM-bound). Tiles are 64 x 4 pixels (16 x 16 for
// the rotation, whose per-wave source footprint is sheared).
//   op 0: copy (np.flip / dropout only), op 1: cv2.warpAffine INTER_LINEAR BORDER_CONSTANT 0
//   (1/32-pixel fixed-point source coordinates, exact bilinear table), op 2: cv2.resize
//   INTER_LINEAR to (new_w, new_h) then the centre crop / zero pad of random_scale_bev.
// The f32 sums keep OpenCV's scalar order, unfused (fp contract off above); the oracle
// (oracle/ivit_oracle.py cv2_*) restates the same arithmetic.
namespace {

struct BevPass {
  unsigned long long src, dst;
  int C, op, flip, n_rect;
  double m[6];
  double scale_x, scale_y;
  int new_w, new_h, off_x, off_y;
  int rect[5][4];
};
static_assert(sizeof(BevPass) == 192, "ivit_bev_pass layout");

constexpr int kBevTileW = 64, kBevTileH = 4, kBevCPB = 16;

// resizeGeneric's per-axis source index and weights (f32 data): the f64 source position is
// rounded to f32, floored, clamped at both ends (weight 0), and from sx >= n - 1 on the
// horizontal pass copies S[sx] instead of interpolating.
IVIT_DEV void resize_axis(int d, int n_src, double scale, int& s0, int& s1, float& a0, float& a1, bool& copy) {
  float f = (float)(((double)d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f = f - (float)s;
  if (s < 0) { f = 0.f; s = 0; }
  copy = s >= n_src - 1;
  if (copy) { f = 0.f; s = n_src - 1; }
  s0 = s;
  s1 = min(s + 1, n_src - 1);
  a0 = 1.f - f;
  a1 = f;
}

using gcfloat = const __attribute__((address_space(1))) float;
using gfloat = __attribute__((address_space(1))) float;

// One pixel's source taps (plane offsets), weights and flags: MODE 0 copies tap 0; MODE 1 sums
// ((v0 w0 + v1 w1) + v2 w2) + v3 w3 with taps outside the image reading 0 (ok); MODE 2 is the
// separable resize, h_r = cpx ? v_r0 : v_r0 w0 + v_r1 w1 (rows r = taps 0-1 / 2-3), out =
// h_0 w2 + h_1 w3; MODE 3 writes zeros.
struct Taps {
  unsigned i[4];  // unsigned 32-bit offsets: the loads take the uniform base in SGPRs (saddr)
  bool ok[4];
  float w[4];
  bool cpx;
};

// N planes of one pixel: every load is issued before the first store, so a thread keeps 4N
// loads in flight (the planes are independent; src and dst never alias).
template <int MODE, int N>
IVIT_DEV void bev_planes(gcfloat* __restrict__ s, gfloat* __restrict__ d, unsigned HW, unsigned o, const Taps& t) {
  if constexpr (MODE == 3) {
#pragma unroll
    for (unsigned c = 0; c < N; ++c) d[c * HW + o] = 0.f;
  } else if constexpr (MODE == 0) {
    float v[N];
#pragma unroll
    for (unsigned c = 0; c < N; ++c) v[c] = s[c * HW + t.i[0]];
#pragma unroll
    for (unsigned c = 0; c < N; ++c) d[c * HW + o] = v[c];
  } else {
    float v[N][4];
#pragma unroll
    for (unsigned c = 0; c < N; ++c)
#pragma unroll
      for (int k = 0; k < 4; ++k) v[c][k] = s[c * HW + t.i[k]];
#pragma unroll
    for (unsigned c = 0; c < N; ++c) {
      float r;
      if constexpr (MODE == 1) {
        const float v0 = t.ok[0] ? v[c][0] : 0.f, v1 = t.ok[1] ? v[c][1] : 0.f;
        const float v2 = t.ok[2] ? v[c][2] : 0.f, v3 = t.ok[3] ? v[c][3] : 0.f;
        r = ((v0 * t.w[0] + v1 * t.w[1]) + v2 * t.w[2]) + v3 * t.w[3];
      } else {
        const float h0 = t.cpx ? v[c][0] : v[c][0] * t.w[0] + v[c][1] * t.w[1];
        const float h1 = t.cpx ? v[c][2] : v[c][2] * t.w[0] + v[c][3] * t.w[1];
        r = h0 * t.w[2] + h1 * t.w[3];
      }
      d[c * HW + o] = r;
    }
  }
}

template <int MODE>
IVIT_DEV void bev_run(gcfloat* s, gfloat* d, unsigned HW, unsigned o, int cn, const Taps& t) {
  if (cn == kBevCPB) {
    bev_planes<MODE, kBevCPB>(s, d, HW, o, t);
  } else {
    for (int c = 0; c < cn; ++c) bev_planes<MODE, 1>(s + (long)c * HW, d + (long)c * HW, HW, o, t);
  }
}

__global__ __launch_bounds__(256) void bev_pass_kernel(const BevPass* __restrict__ passes, int H, int W) {
  const BevPass& P = passes[blockIdx.z];  // uniform: scalar loads, all read before the first store
  const int c0 = blockIdx.y * kBevCPB;
  if (c0 >= P.C) return;
  const int op = P.op;
  // XCD-aware tile order: gridDim.x is a multiple of 8 and workgroups go round-robin over the 8
  // XCDs, so XCD k runs the contiguous tile range [k * per, (k + 1) * per): neighbouring tiles,
  // which share source cache lines and the rows below, hit one L2.
  const int per = gridDim.x >> 3;
  const int tile = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  int x, y;
  if (op == 1) {  // rotation: 16 x 16 tiles (a wave = 16 x 4 pixels), so one gather instruction's
                  // sheared source footprint spans ~8 rows instead of the ~17 of a 64-pixel row
    const int tw = (W + 15) / 16;
    x = (tile % tw) * 16 + (threadIdx.x & 15);
    y = (tile / tw) * 16 + (threadIdx.x >> 4);
  } else {  // 64 x 4 tiles: 256-B row segments per wave
    const int tw = (W + kBevTileW - 1) / kBevTileW;
    x = (tile % tw) * kBevTileW + (threadIdx.x & (kBevTileW - 1));
    y = (tile / tw) * kBevTileH + threadIdx.x / kBevTileW;
  }
  if (x >= W || y >= H) return;
  const unsigned HW = H * W, o = y * W + x;  // 32-bit plane offsets (launcher: kBevCPB * H * W < 2^31)
  gcfloat* src = reinterpret_cast<gcfloat*>(P.src) + (long)c0 * HW;  // uniform bases: saddr loads / stores
  gfloat* dst = reinterpret_cast<gfloat*>(P.dst) + (long)c0 * HW;
  const int cn = min(kBevCPB, P.C - c0);

  bool zero = false;
  for (int r = 0; r < P.n_rect; ++r)
    zero |= y >= P.rect[r][0] && y < P.rect[r][0] + P.rect[r][2] && x >= P.rect[r][1] && x < P.rect[r][1] + P.rect[r][3];
  if (!zero && op == 2) {
    const int ry = y + P.off_y, rx = x + P.off_x;
    zero = ry < 0 || ry >= P.new_h || rx < 0 || rx >= P.new_w;
  }
  if (zero) return bev_run<3>(src, dst, HW, o, cn, Taps{});
  const bool flip = P.flip;
  auto col = [&](int c) { return flip ? W - 1 - c : c; };
  Taps t{};
  if (op == 0) {
    t.i[0] = (unsigned)(y * W + col(x));
    return bev_run<0>(src, dst, HW, o, cn, t);
  }
  if (op == 1) {
    const double* m = P.m;
    const int rd = (1 << 10) / 32 / 2;
    const int adx = (int)rint(m[0] * (double)x * 1024.0), bdx = (int)rint(m[3] * (double)x * 1024.0);
    const int X0 = (int)rint((m[1] * (double)y + m[2]) * 1024.0) + rd;
    const int Y0 = (int)rint((m[4] * (double)y + m[5]) * 1024.0) + rd;
    const int X = (X0 + adx) >> 5, Y = (Y0 + bdx) >> 5;
    const int sx = min(max(X >> 5, -32768), 32767), sy = min(max(Y >> 5, -32768), 32767);
    const float tx = (float)(X & 31) * (1.f / 32.f), ty = (float)(Y & 31) * (1.f / 32.f);
    t.w[0] = (1.f - ty) * (1.f - tx);
    t.w[1] = (1.f - ty) * tx;
    t.w[2] = ty * (1.f - tx);
    t.w[3] = ty * tx;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int cx = sx + (k & 1), cy = sy + (k >> 1);
      t.ok[k] = cx >= 0 && cx < W && cy >= 0 && cy < H;
      t.i[k] = t.ok[k] ? (unsigned)(cy * W + col(cx)) : 0u;  // an in-bounds address; the value is replaced by 0
    }
    return bev_run<1>(src, dst, HW, o, cn, t);
  }
  // op 2: resize (then centre crop / pad: out(y, x) = resized(y + off_y, x + off_x))
  int sx0, sx1, sy0, sy1;
  bool cpy;
  resize_axis(x + P.off_x, W, P.scale_x, sx0, sx1, t.w[0], t.w[1], t.cpx);
  resize_axis(y + P.off_y, H, P.scale_y, sy0, sy1, t.w[2], t.w[3], cpy);
  t.i[0] = (unsigned)(sy0 * W + col(sx0));
  t.i[1] = (unsigned)(sy0 * W + col(sx1));
  t.i[2] = (unsigned)(sy1 * W + col(sx0));
  t.i[3] = (unsigned)(sy1 * W + col(sx1));
  bev_run<2>(src, dst, HW, o, cn, t);
}

}  // namespace

extern "C" int ivit_bev_augment(const void* passes, long n_passes, long H, long W, long max_planes, void* stream) {
  if (n_passes <= 0 || max_planes <= 0) return 0;
  IVIT_CHECK_ARG(passes != nullptr, "ivit_bev_augment: null pass table");
  IVIT_CHECK_ARG(n_passes < 65536, "ivit_bev_augment: too many passes (%ld)", n_passes);
  IVIT_CHECK_ARG(H > 1 && W > 1 && kBevCPB * H * W < (1L << 31) && H < 32768 && W < 32768,
                 "ivit_bev_augment: bad plane size %ldx%ld", H, W);
  long tiles = std::max(ivit_cdiv(W, kBevTileW) * ivit_cdiv(H, kBevTileH), ivit_cdiv(W, 16) * ivit_cdiv(H, 16));
  tiles = ivit_cdiv(tiles, 8) * 8;  // the kernel's XCD tile order needs a multiple of 8
  dim3 g((unsigned)tiles, (unsigned)ivit_cdiv(max_planes, kBevCPB), (unsigned)n_passes);
  hipLaunchKernelGGL(bev_pass_kernel, g, dim3(256), 0, ivit_stream(stream), (const BevPass*)passes, (int)H,
                     (int)W);
  IVIT_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------- HD-map rasterisation
// rasterize_map_ego_centric (utils.py:108-182): cv2.polylines / cv2.fillPoly (LINE_8, thickness
// 1, shift 0, colour 1) into zero-initialised f32 planes, as two launches over host-built tables:
//   segments: every open-polyline segment and every polygon edge (cv::fillPoly draws each edge
//             with cv::Line) — one thread walks cv::LineIterator's 8-connected pixels
//             (leftToRight, err = major - 2 minor, step the minor axis when err < 0);
//   fill rows: one thread per (polygon, scanline y): the x of every edge active at y
//             (y0 <= y < y1) in 16.16 fixed point, x = x_top + (y - y0) * dx (the exact value
//             FillEdgeCollection's per-scanline x += dx reaches), sorted, spans
//             [x_2k >> 16, x_2k+1 >> 16] filled (delta 0 for LINE_8), clipped to the image.
// Every write stores 1.0f: concurrent writers of one pixel agree, no atomics.
namespace {
constexpr int kMapMaxEdges = 256;

IVIT_DEV void map_put(float* img, long HW, int mask, long off) {
#pragma unroll 1
  for (int c = 0; mask; ++c, mask >>= 1)
    if (mask & 1) img[c * HW + off] = 1.0f;
}

__global__ void map_segments_kernel(const int* __restrict__ seg, long n, const long* __restrict__ base, int H,
                                    int W, float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int* s = seg + i * 5;  // x0, y0, x1, y1, plane mask
  int x0 = s[0], y0 = s[1], x1 = s[2], y1 = s[3];
  const int mask = s[4];
  float* img = out + base[i];
  const long HW = (long)H * W;
  int dx = x1 - x0, dy = y1 - y0;
  if (dx < 0) {  // leftToRight
    dx = -dx;
    dy = -dy;
    x0 = x1;
    y0 = y1;
  }
  int sy = 1;
  if (dy < 0) {
    dy = -dy;
    sy = -1;
  }
  const bool vert = dy > dx;
  const int major = vert ? dy : dx, minor = vert ? dx : dy;
  int err = major - 2 * minor;
  int x = x0, y = y0;
  for (int k = 0; k <= major; ++k) {
    if (x >= 0 && x < W && y >= 0 && y < H) map_put(img, HW, mask, (long)y * W + x);
    const bool step = err < 0;
    err += -2 * minor + (step ? 2 * major : 0);
    if (vert) {
      y += sy;
      x += step ? 1 : 0;
    } else {
      x += 1;
      y += step ? sy : 0;
    }
  }
}

__global__ void map_fill_kernel(const long* __restrict__ edges, const int* __restrict__ polys,
                                const int* __restrict__ rows, long n_rows, const long* __restrict__ base, int H,
                                int W, float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rows) return;
  const int p = rows[2 * i], y = rows[2 * i + 1];
  const int e0 = polys[3 * p], ne = polys[3 * p + 1], mask = polys[3 * p + 2];
  long xs[kMapMaxEdges];
  int n = 0;
  for (int e = 0; e < ne; ++e) {  // edge: y0, y1, x_top (16.16), dx (16.16)
    const long* E = edges + 4 * (long)(e0 + e);
    if (E[0] <= y && y < E[1]) {
      const long x = E[2] + (long)(y - E[0]) * E[3];
      int j = n++;
      while (j > 0 && xs[j - 1] > x) {  // insertion sort
        xs[j] = xs[j - 1];
        --j;
      }
      xs[j] = x;
    }
  }
  float* img = out + base[p];
  const long HW = (long)H * W;
  for (int k = 0; k + 1 < n; k += 2) {
    int x1 = (int)(xs[k] >> 16), x2 = (int)(xs[k + 1] >> 16);
    if (x1 < W && x2 >= 0) {
      x1 = x1 < 0 ? 0 : x1;
      x2 = x2 >= W ? W - 1 : x2;
      for (int x = x1; x <= x2; ++x) map_put(img, HW, mask, (long)y * W + x);
    }
  }
}
}  // namespace

extern "C" int ivit_map_raster(const int* seg, long n_seg, const long* seg_base, const long* edges,
                               const int* polys, long n_polys, const long* poly_base, const int* rows, long n_rows,
                               long max_edges, long H, long W, float* out, void* stream) {
  IVIT_CHECK_ARG(H > 0 && W > 0 && H < 65536 && W < 65536, "ivit_map_raster: bad plane size %ldx%ld", H, W);
  IVIT_CHECK_ARG(max_edges <= kMapMaxEdges, "ivit_map_raster: a polygon has %ld edges (max %d)", max_edges,
                 kMapMaxEdges);
  IVIT_CHECK_ARG(n_seg == 0 || (seg && seg_base), "ivit_map_raster: null segment table");
  IVIT_CHECK_ARG(n_rows == 0 || (edges && polys && poly_base && rows), "ivit_map_raster: null fill tables");
  (void)n_polys;
  hipStream_t st = ivit_stream(stream);
  if (n_seg > 0)
    hipLaunchKernelGGL(map_segments_kernel, dim3(ivit_cdiv(n_seg, 256)), dim3(256), 0, st, seg, n_seg, seg_base,
                       (int)H, (int)W, out);
  if (n_rows > 0)
    hipLaunchKernelGGL(map_fill_kernel, dim3(ivit_cdiv(n_rows, 256)), dim3(256), 0, st, edges, polys, rows, n_rows,
                       poly_base, (int)H, (int)W, out);
  IVIT_LAUNCH_CHECK();
  return 0;
}
