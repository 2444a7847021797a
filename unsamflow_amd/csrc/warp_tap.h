// The warp's per-pixel tap: the reference coordinate chain of flow_warp
// (utils/warp_utils.py:97-106 + ATen grid_sampler_2d bilinear, see warp.hip)
// evaluated once per output pixel. Shared by warp.hip and photo.hip.
#pragma once
#include "usf_common.h"

namespace usf {

struct Tap {
  int xw, yn;                   // integer north-west corner (before masking)
  int o_nw, o_ne, o_sw, o_se;   // offsets within a channel plane
  bool m_nw, m_ne, m_sw, m_se;  // corner inside the image
  float n, s, w, e;             // distances (see header)
  float mx, my;                 // d(ix)/d(gx), d(iy)/d(gy) incl. clamp mask
};

__device__ __forceinline__ inline Tap make_tap(float u, float v, int x, int y, int H, int W,
                                        bool border) {
  // Every step of the coordinate chain is rounded separately, as in the
  // reference: hipcc's default -ffp-contract=fast would otherwise fuse
  // w = ix - floor(ix) into fma(sx, gx+1, -floor) on the unrounded product,
  // which moves the sample point by up to 1 ulp of the coordinate (6e-5 px
  // at W=832) and the output by ~3e-5.
#pragma clang fp contract(off)
  Tap t;
  const float wm1 = (float)(W - 1), hm1 = (float)(H - 1);
  // norm_grid: 2.0 * v / (W - 1) - 1.0  (fp32, true division as in torch CPU)
  const float gx = 2.0f * ((float)x + u) / wm1 - 1.0f;
  const float gy = 2.0f * ((float)y + v) / hm1 - 1.0f;
  // grid_sampler unnormalise, align_corners=True
  const float sx = wm1 / 2.0f, sy = hm1 / 2.0f;
  float ix = (gx + 1.0f) * sx;
  float iy = (gy + 1.0f) * sy;
  t.mx = sx;
  t.my = sy;
  if (border) {
    // clip_coordinates + its gradient: borders count as out of bounds
    if (!(ix > 0.f)) { ix = 0.f; t.mx = 0.f; }
    else if (ix >= wm1) { ix = wm1; t.mx = 0.f; }
    if (!(iy > 0.f)) { iy = 0.f; t.my = 0.f; }
    else if (iy >= hm1) { iy = hm1; t.my = 0.f; }
  }
  const float fx = floorf(ix), fy = floorf(iy);
  t.w = ix - fx;
  t.e = 1.0f - t.w;
  t.n = iy - fy;
  t.s = 1.0f - t.n;
  const int xw = (int)fx, yn = (int)fy;
  const int xe = xw + 1, ys = yn + 1;
  t.xw = xw;
  t.yn = yn;
  const bool vxw = (unsigned)xw < (unsigned)W, vxe = (unsigned)xe < (unsigned)W;
  const bool vyn = (unsigned)yn < (unsigned)H, vys = (unsigned)ys < (unsigned)H;
  t.m_nw = vxw && vyn;
  t.m_ne = vxe && vyn;
  t.m_sw = vxw && vys;
  t.m_se = vxe && vys;
  // offsets only used when the mask is set; clamp to 0 otherwise
  t.o_nw = t.m_nw ? yn * W + xw : 0;
  t.o_ne = t.m_ne ? yn * W + xe : 0;
  t.o_sw = t.m_sw ? ys * W + xw : 0;
  t.o_se = t.m_se ? ys * W + xe : 0;
  return t;
}

}  // namespace usf
