// Box geometry device functions shared by the loss and the eval kernels (utils.py).
// Bit-exactness with the reference's f32 tensor arithmetic requires no FMA contraction:
// every file including this header compiles with `#pragma clang fp contract(off)`.
#pragma once
#include "ivit_common.h"

#pragma clang fp contract(off)

namespace ivit {

// utils.py:276-292 compute_axis_aligned_iou (cx, cy, w, h): corners by /2, inter via
// clamp(min=0), union = (a1 + a2) - inter, iou = inter / (union + 1e-7).
IVIT_DEV float axis_iou(const float* a, const float* b) {
  const float ax1 = a[0] - a[2] / 2.f, ay1 = a[1] - a[3] / 2.f, ax2 = a[0] + a[2] / 2.f, ay2 = a[1] + a[3] / 2.f;
  const float bx1 = b[0] - b[2] / 2.f, by1 = b[1] - b[3] / 2.f, bx2 = b[0] + b[2] / 2.f, by2 = b[1] + b[3] / 2.f;
  const float iw = fmaxf(fminf(ax2, bx2) - fmaxf(ax1, bx1), 0.f);
  const float ih = fmaxf(fminf(ay2, by2) - fmaxf(ay1, by1), 0.f);
  const float inter = iw * ih;
  const float a1 = a[2] * a[3], a2 = b[2] * b[3];
  const float uni = (a1 + a2) - inter;
  return inter / (uni + 1e-7f);
}

// ---- rotated IoU (utils.py:295-392): rectangle corners [-w/2,-l/2],[w/2,-l/2],[w/2,l/2],
// [-w/2,l/2] rotated by yaw about (cx, cy); convex clipping in double (GEOS computes in double).
struct Poly {
  int n;
  double x[12], y[12];
};

IVIT_DEV void rect_poly(const float* b, Poly& p) {
  const double cx = b[0], cy = b[1], hw = (double)b[2] / 2.0, hl = (double)b[3] / 2.0, a = b[4];
  const double c = cos(a), s = sin(a);
  const double lx[4] = {-hw, hw, hw, -hw}, ly[4] = {-hl, -hl, hl, hl};
  p.n = 4;
  for (int i = 0; i < 4; ++i) {
    p.x[i] = lx[i] * c - ly[i] * s + cx;
    p.y[i] = lx[i] * s + ly[i] * c + cy;
  }
}

IVIT_DEV double poly_area_signed(const Poly& p) {
  double s = 0.0;
  for (int i = 0; i < p.n; ++i) {
    const int j = (i + 1) % p.n;
    s += p.x[i] * p.y[j] - p.y[i] * p.x[j];
  }
  return 0.5 * s;
}

IVIT_DEV void make_ccw(Poly& p) {
  if (poly_area_signed(p) < 0.0) {
    for (int i = 0; i < p.n / 2; ++i) {
      const int j = p.n - 1 - i;
      double t = p.x[i]; p.x[i] = p.x[j]; p.x[j] = t;
      t = p.y[i]; p.y[i] = p.y[j]; p.y[j] = t;
    }
  }
}

// Sutherland-Hodgman: clip P (ccw) by convex Q (ccw); result in P.
IVIT_DEV void clip_poly(Poly& P, const Poly& Q) {
  Poly out;
  for (int e = 0; e < Q.n && P.n > 0; ++e) {
    const double ax = Q.x[e], ay = Q.y[e], bx = Q.x[(e + 1) % Q.n], by = Q.y[(e + 1) % Q.n];
    const double ex = bx - ax, ey = by - ay;
    out.n = 0;
    for (int j = 0; j < P.n; ++j) {
      const int pj = (j + P.n - 1) % P.n;
      const double cxp = P.x[j], cyp = P.y[j], pxp = P.x[pj], pyp = P.y[pj];
      const double sc = ex * (cyp - ay) - ey * (cxp - ax);
      const double sp = ex * (pyp - ay) - ey * (pxp - ax);
      if (sc >= 0.0) {
        if (sp < 0.0 && out.n < 12) {
          const double t = sp / (sp - sc);
          out.x[out.n] = pxp + t * (cxp - pxp);
          out.y[out.n] = pyp + t * (cyp - pyp);
          ++out.n;
        }
        if (out.n < 12) { out.x[out.n] = cxp; out.y[out.n] = cyp; ++out.n; }
      } else if (sp >= 0.0 && out.n < 12) {
        const double t = sp / (sp - sc);
        out.x[out.n] = pxp + t * (cxp - pxp);
        out.y[out.n] = pyp + t * (cyp - pyp);
        ++out.n;
      }
    }
    P = out;
  }
}

IVIT_DEV float rotated_iou(const float* a, const float* b) {
  Poly pa, pb;
  rect_poly(a, pa);
  rect_poly(b, pb);
  const double A1 = fabs(poly_area_signed(pa)), A2 = fabs(poly_area_signed(pb));
  if (A1 < 1e-6 || A2 < 1e-6) return 0.f;
  make_ccw(pa);
  make_ccw(pb);
  clip_poly(pa, pb);
  const double inter = pa.n >= 3 ? fabs(poly_area_signed(pa)) : 0.0;
  if (!(inter > 1e-7)) return 0.f;
  const double u = A1 + A2 - inter;
  if (!(u > 1e-6)) return 0.f;
  return (float)(inter / u);
}

}  // namespace ivit
