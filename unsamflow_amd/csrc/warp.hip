// Bilinear backward warp (flow_warp) forward / backward for gfx950.
//
// Semantics: utils/warp_utils.py:97-106 — mesh_grid (:7-13) + flow, the
// normalisation of norm_grid (:16-23), then grid_sample(bilinear,
// align_corners=True, padding_mode in {border, zeros}). The sampler itself is
// third-party ATen code (grid_sampler_2d, torch 2.10); the coordinate chain is
// restated exactly as the reference computes it so the fp32 round trip
// normalise -> unnormalise is reproduced:
//   gx  = 2*(x+u)/(W-1) - 1            (warp_utils.py:21)
//   ix  = (gx + 1) * ((W-1)/2)          (align_corners unnormalise)
//   ix  = clamp(ix, 0, W-1)             (border only)
//   x_w = floor(ix); w = ix - x_w; e = 1 - w   (and n/s for y)
//   out = v_nw*s*e + v_ne*s*w + v_sw*n*e + v_se*n*w   (out-of-image corners = 0)
// Backward: grad_x gets w*g scattered to the 4 corners; the coordinate grad is
//   dix = sum_c g*((v_ne-v_nw)*s + (v_se-v_sw)*n),
//   diy = sum_c g*((v_sw-v_nw)*e + (v_se-v_ne)*w),
// times (W-1)/2 (zero where the border clamp is active: ix<=0 or ix>=W-1),
// then through norm_grid's autograd: du = (dgx/(W-1))*2.
//
// Layout: one lane per output pixel (consecutive lanes = consecutive x, so
// flow/out/gout accesses are coalesced), channels looped inside the lane with
// the 4 corner offsets and weights computed once per pixel. grad_x uses fp32
// global atomics (global_atomic_add_f32, no CAS loop); grad_flow is a
// per-lane reduction over channels, written once (deterministic).
#include "usf_common.h"

namespace usf {
namespace {

struct Tap {
  int o_nw, o_ne, o_sw, o_se;   // offsets within a channel plane
  bool m_nw, m_ne, m_sw, m_se;  // corner inside the image
  float n, s, w, e;             // distances (see header)
  float mx, my;                 // d(ix)/d(gx), d(iy)/d(gy) incl. clamp mask
};

__device__ __forceinline__ Tap make_tap(float u, float v, int x, int y, int H, int W,
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

template <bool BORDER>
__global__ __launch_bounds__(256) void warp_fwd_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ flow,
                                                       long long fbs, float* __restrict__ out,
                                                       int B, int C, int H, int W) {
  const int HW = H * W;
  const int p = blockIdx.x * 256 + threadIdx.x;  // pixel within the sample
  const int b = blockIdx.y;
  if (p >= HW) return;
  const int y = p / W, xx = p - y * W;
  const float* fb = flow + b * fbs;
  const Tap t = make_tap(fb[p], fb[HW + p], xx, y, H, W, BORDER);
  const float wnw = t.s * t.e, wne = t.s * t.w, wsw = t.n * t.e, wse = t.n * t.w;
  const float* xb = x + (size_t)b * C * HW;
  float* ob = out + (size_t)b * C * HW + p;
#pragma unroll 4
  for (int c = 0; c < C; ++c) {
    const float* xc = xb + (size_t)c * HW;
    const float vnw = t.m_nw ? xc[t.o_nw] : 0.f;
    const float vne = t.m_ne ? xc[t.o_ne] : 0.f;
    const float vsw = t.m_sw ? xc[t.o_sw] : 0.f;
    const float vse = t.m_se ? xc[t.o_se] : 0.f;
    ob[(size_t)c * HW] = vnw * wnw + vne * wne + vsw * wsw + vse * wse;
  }
}

template <bool BORDER, bool WANT_GX, bool WANT_GF>
__global__ __launch_bounds__(256) void warp_bwd_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ flow,
                                                       long long fbs,
                                                       const float* __restrict__ gout,
                                                       float* __restrict__ gx,
                                                       float* __restrict__ gflow, int B, int C,
                                                       int H, int W) {
  const int HW = H * W;
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (p >= HW) return;
  const int y = p / W, xx = p - y * W;
  const float* fb = flow + b * fbs;
  const Tap t = make_tap(fb[p], fb[HW + p], xx, y, H, W, BORDER);
  const float wnw = t.s * t.e, wne = t.s * t.w, wsw = t.n * t.e, wse = t.n * t.w;
  const float* xb = x + (size_t)b * C * HW;
  const float* gb = gout + (size_t)b * C * HW + p;
  float* gxb = WANT_GX ? gx + (size_t)b * C * HW : nullptr;
  float dix = 0.f, diy = 0.f;
#pragma unroll 4
  for (int c = 0; c < C; ++c) {
    const float go = gb[(size_t)c * HW];
    if (WANT_GX) {
      float* gc = gxb + (size_t)c * HW;
      if (t.m_nw) atomicAdd(gc + t.o_nw, go * wnw);
      if (t.m_ne) atomicAdd(gc + t.o_ne, go * wne);
      if (t.m_sw) atomicAdd(gc + t.o_sw, go * wsw);
      if (t.m_se) atomicAdd(gc + t.o_se, go * wse);
    }
    if (WANT_GF) {
      const float* xc = xb + (size_t)c * HW;
      const float vnw = t.m_nw ? xc[t.o_nw] : 0.f;
      const float vne = t.m_ne ? xc[t.o_ne] : 0.f;
      const float vsw = t.m_sw ? xc[t.o_sw] : 0.f;
      const float vse = t.m_se ? xc[t.o_se] : 0.f;
      dix += ((vne - vnw) * t.s + (vse - vsw) * t.n) * go;
      diy += ((vsw - vnw) * t.e + (vse - vne) * t.w) * go;
    }
  }
  if (WANT_GF) {
    // grid grad, then norm_grid's autograd (DivBackward by (W-1), MulBackward by 2)
    const float ggx = dix * t.mx, ggy = diy * t.my;
    float* gf = gflow + (size_t)b * 2 * HW + p;
    gf[0] = (ggx / (float)(W - 1)) * 2.0f;
    gf[HW] = (ggy / (float)(H - 1)) * 2.0f;
  }
}

template <bool BORDER>
hipError_t bwd_launch_pad(const float* x, const float* flow, long long fbs, const float* gout,
                          float* gx, float* gflow, int B, int C, int H, int W, hipStream_t s) {
  const dim3 grid((unsigned)((H * W + 255) / 256), (unsigned)B), block(256);
  if (gx && gflow)
    hipLaunchKernelGGL((warp_bwd_kernel<BORDER, true, true>), grid, block, 0, s, x, flow, fbs,
                       gout, gx, gflow, B, C, H, W);
  else if (gx)
    hipLaunchKernelGGL((warp_bwd_kernel<BORDER, true, false>), grid, block, 0, s, x, flow, fbs,
                       gout, gx, gflow, B, C, H, W);
  else if (gflow)
    hipLaunchKernelGGL((warp_bwd_kernel<BORDER, false, true>), grid, block, 0, s, x, flow, fbs,
                       gout, gx, gflow, B, C, H, W);
  return hipGetLastError();
}

}  // namespace

hipError_t warp_fwd_launch(const float* x, const float* flow, long long fbs, float* out, int B,
                           int C, int H, int W, int pad_mode, hipStream_t s) {
  const dim3 grid((unsigned)((H * W + 255) / 256), (unsigned)B), block(256);
  if (pad_mode == 1)
    hipLaunchKernelGGL((warp_fwd_kernel<true>), grid, block, 0, s, x, flow, fbs, out, B, C, H, W);
  else
    hipLaunchKernelGGL((warp_fwd_kernel<false>), grid, block, 0, s, x, flow, fbs, out, B, C, H,
                       W);
  return hipGetLastError();
}

hipError_t warp_bwd_launch(const float* x, const float* flow, long long fbs, const float* gout,
                           float* gx, float* gflow, int B, int C, int H, int W, int pad_mode,
                           hipStream_t s) {
  if (!gx && !gflow) return hipSuccess;
  if (pad_mode == 1) return bwd_launch_pad<true>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s);
  return bwd_launch_pad<false>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s);
}

}  // namespace usf
