// Fused occlusion-aware photometric loss of unFlowLoss for gfx950 (CDNA4):
// the per-scale, per-direction term of losses/flow_loss.py:127-148 with
// loss_photomatric (:33-50) and SSIM (losses/loss_blocks.py:53-72):
//
//   rec  = flow_warp(src, flow, pad)                      (warp_utils.py:97-106)
//   x    = rec * m,  y = tgt * m                          (SSIM arguments, :40)
//   L    = ( w_l1 * mean_{b,c,p} |tgt - rec| * m
//          + w_ssim * mean_{b,c,q} S_q ) / (mean_{b,p} m + 1e-6)
//   S_q  = clamp((1 - n/d) / 2, 0, 1) over every valid 3x3 window q
//          (avg_pool2d(3, 1, 0)): mu = E[.], sig_x = E[x^2] - mu_x^2,
//          sig_xy = E[xy] - mu_x mu_y, n = (2 mu_x mu_y + C1)(2 sig_xy + C2),
//          d = (mu_x^2 + mu_y^2 + C1)(sig_x + sig_y + C2), C1 = 0.01^2, C2 = 0.03^2
//
// The mask m and tgt carry no gradient (the reference thresholds the mask);
// only the flow does. Forward: one kernel per (16x16 tile, sample) warps the
// source for the tile + 2-pixel halo straight into LDS, sums the L1, SSIM and
// mask terms and writes per-block partials; a one-block kernel combines them
// in a fixed order (fp64) into the loss and the two backward coefficients.
// Backward: dS_q/dx_p = alpha_q + beta_q x_p + gamma_q y_p (closed form below),
// so one kernel per tile stages x/y for the tile + 2-pixel halo, the window
// coefficients for the tile + 1-pixel halo, sums the 9 windows around each
// pixel, adds the L1 sign term and folds dL/drec through the bilinear
// coordinate derivative into grad_flow -- the warp's grad_flow path of
// warp.hip, without materialising rec, the SSIM maps or dL/drec in HBM.
#include <cstdint>

#include "usf_common.h"
#include "warp_tap.h"

namespace usf {
namespace {

constexpr int kTile = 16;              // 16x16 output pixels per workgroup (256 threads)
constexpr int kMaxC = 3;               // image channels per pixel (RGB; LDS is sized for 3)
constexpr float kC1 = 0.01f * 0.01f;   // torch casts the python scalars to fp32
constexpr float kC2 = 0.03f * 0.03f;

// bilinear sample of the C channels of src at pixel (px, py) displaced by the
// flow, with the reference's coordinate chain (warp_tap.h); also returns the tap
__device__ __forceinline__ void sample_px(const float* __restrict__ srcb, const float* __restrict__ fb,
                                          int px, int py, int H, int W, int C, bool border,
                                          float (&out)[kMaxC], Tap& tp) {
#pragma clang fp contract(off)
  const int HW = H * W;
  const int p = py * W + px;
  tp = make_tap(fb[p], fb[HW + p], px, py, H, W, border);
  const float wnw = tp.s * tp.e, wne = tp.s * tp.w, wsw = tp.n * tp.e, wse = tp.n * tp.w;
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) {
    if (c >= C) break;
    const float* sc = srcb + (size_t)c * HW;
    const float vnw = tp.m_nw ? sc[tp.o_nw] : 0.f;
    const float vne = tp.m_ne ? sc[tp.o_ne] : 0.f;
    const float vsw = tp.m_sw ? sc[tp.o_sw] : 0.f;
    const float vse = tp.m_se ? sc[tp.o_se] : 0.f;
    out[c] = vnw * wnw + vne * wne + vsw * wsw + vse * wse;  // ATen's order
  }
}

// tile and sample of this workgroup: grid = (tiles, B), XCD-aware order so that
// neighbouring tiles (shared halos and gather footprints) run on one L2
__device__ __forceinline__ void photo_work(int tiles_x, int& ty0, int& tx0, int& b) {
  const int ntiles = gridDim.x;
  const int w = xcd_remap(linear_block(), ntiles * gridDim.y);
  const int tile = w % ntiles;
  b = w / ntiles;
  ty0 = (tile / tiles_x) * kTile;
  tx0 = (tile % tiles_x) * kTile;
}

// block-wide sum of 3 values in a fixed order (deterministic)
__device__ __forceinline__ void block_sum3(float a, float b, float c, float* red, float* out3) {
  const int t = threadIdx.x;
  red[t] = a;
  red[256 + t] = b;
  red[512 + t] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) {
      red[t] += red[t + s];
      red[256 + t] += red[256 + t + s];
      red[512 + t] += red[512 + t + s];
    }
    __syncthreads();
  }
  if (t == 0) {
    out3[0] = red[0];
    out3[1] = red[256];
    out3[2] = red[512];
  }
}

// ---------------------------------------------------------------- forward --
template <bool BORDER>
__global__ __launch_bounds__(256) void photo_fwd_kernel(const float* __restrict__ src,
                                                        const float* __restrict__ tgt,
                                                        const float* __restrict__ mask,
                                                        const float* __restrict__ flow, long long fbs,
                                                        float* __restrict__ partials, int C, int H,
                                                        int W, int tiles_x) {
#pragma clang fp contract(off)
  constexpr int R = kTile + 2;  // windows starting in the tile read 2 more rows / cols
  __shared__ float xs[kMaxC][R][R + 1], ys[kMaxC][R][R + 1];
  __shared__ float red[768];
  const int t = threadIdx.x;
  int ty0, tx0, b;
  photo_work(tiles_x, ty0, tx0, b);
  const int HW = H * W;
  const float* srcb = src + (size_t)b * C * HW;
  const float* tgtb = tgt + (size_t)b * C * HW;
  const float* mb = mask + (size_t)b * HW;
  const float* fb = flow + b * fbs;

  float l1 = 0.f, msum = 0.f;
  for (int e = t; e < R * R; e += 256) {
    const int ry = e / R, rx = e - ry * R;
    const int py = ty0 + ry, px = tx0 + rx;
    float rec[kMaxC] = {};
    float m = 0.f;
    const bool in = py < H && px < W;
    if (in) {
      Tap tp;
      sample_px(srcb, fb, px, py, H, W, C, BORDER, rec, tp);
      m = mb[py * W + px];
    }
    const bool own = in && ry < kTile && rx < kTile;  // this tile's pixel: L1 + mask terms
    if (own) msum += m;
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) {
      if (c >= C) break;
      const float tv = in ? tgtb[(size_t)c * HW + py * W + px] : 0.f;
      if (own) l1 += fabsf(tv - rec[c]) * m;
      xs[c][ry][rx] = rec[c] * m;
      ys[c][ry][rx] = tv * m;
    }
  }
  __syncthreads();
  // the 3x3 window whose top-left is this thread's pixel
  float ssim = 0.f;
  const int wy = t / kTile, wx = t % kTile;
  const int qy = ty0 + wy, qx = tx0 + wx;
  if (qy <= H - 3 && qx <= W - 3) {
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) {
      if (c >= C) break;
      float sx = 0.f, sy = 0.f, sxx = 0.f, syy = 0.f, sxy = 0.f;
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const float a = xs[c][wy + i][wx + j], v = ys[c][wy + i][wx + j];
          sx += a;
          sy += v;
          sxx += a * a;
          syy += v * v;
          sxy += a * v;
        }
      const float mx = sx / 9.f, my = sy / 9.f;
      const float mxy = mx * my, mx2 = mx * mx, my2 = my * my;
      const float sig_x = sxx / 9.f - mx2, sig_y = syy / 9.f - my2, sig_xy = sxy / 9.f - mxy;
      const float n = (2.f * mxy + kC1) * (2.f * sig_xy + kC2);
      const float d = (mx2 + my2 + kC1) * (sig_x + sig_y + kC2);
      ssim += fminf(fmaxf((1.f - n / d) / 2.f, 0.f), 1.f);
    }
  }
  const int blk = b * gridDim.x + (ty0 / kTile) * tiles_x + tx0 / kTile;  // fixed slot per tile
  block_sum3(l1, ssim, msum, red, partials + 3 * blk);
}

// One block: fixed-order fp64 sum of the partials -> out = {loss, c_l1, c_ssim}
// with c_* the backward coefficients w_* / (N_* * (mean(m) + 1e-6)).
__global__ __launch_bounds__(256) void photo_final_kernel(const float* __restrict__ partials,
                                                          int nblk, float* __restrict__ out,
                                                          double n1, double n2, double n3, float w_l1,
                                                          float w_ssim) {
  __shared__ double red[3][256];
  const int t = threadIdx.x;
  double a = 0, b = 0, c = 0;
  for (int i = t; i < nblk; i += 256) {
    a += partials[3 * i];
    b += partials[3 * i + 1];
    c += partials[3 * i + 2];
  }
  red[0][t] = a;
  red[1][t] = b;
  red[2][t] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) {
      red[0][t] += red[0][t + s];
      red[1][t] += red[1][t + s];
      red[2][t] += red[2][t + s];
    }
    __syncthreads();
  }
  if (t == 0) {
    const double den = red[2][0] / n3 + 1e-6;
    const double l1 = n1 > 0 ? red[0][0] / n1 : 0.0, ss = n2 > 0 ? red[1][0] / n2 : 0.0;
    out[0] = (float)((w_l1 * l1 + w_ssim * ss) / den);
    out[1] = n1 > 0 ? (float)(w_l1 / (n1 * den)) : 0.f;
    out[2] = n2 > 0 ? (float)(w_ssim / (n2 * den)) : 0.f;
  }
}

// --------------------------------------------------------------- backward --
// d S_q / d x_p for a pixel p of window q (x = rec * m, y = tgt * m):
//   A1 = 2 mx my + C1, A2 = 2 sig_xy + C2, B1 = mx^2 + my^2 + C1, B2 = sig_x + sig_y + C2,
//   n = A1 A2, d = B1 B2, r = n / d, S = (1 - r) / 2 (clamped to [0, 1]):
//   dS/dx_p = -(1 / (9 d)) [ my (A2 - A1) - r mx (B2 - B1) + A1 y_p - r B1 x_p ]
//           = alpha + beta x_p + gamma y_p,  zero where the clamp is active
//   (torch.clamp passes the gradient for 0 <= raw <= 1).
template <bool BORDER>
__global__ __launch_bounds__(256) void photo_bwd_kernel(const float* __restrict__ src,
                                                        const float* __restrict__ tgt,
                                                        const float* __restrict__ mask,
                                                        const float* __restrict__ flow, long long fbs,
                                                        const float* __restrict__ coef,
                                                        const float* __restrict__ gloss,
                                                        float* __restrict__ gflow, int C, int H,
                                                        int W, int tiles_x) {
#pragma clang fp contract(off)
  constexpr int RI = kTile + 4;  // x / y region: rows ty0-2 .. ty0+TH+1
  constexpr int RW = kTile + 2;  // windows: top-left rows ty0-2 .. ty0+TH-1
  __shared__ float xs[kMaxC][RI][RI + 1], ys[kMaxC][RI][RI + 1];
  __shared__ float al[kMaxC][RW][RW + 1], be[kMaxC][RW][RW + 1], ga[kMaxC][RW][RW + 1];
  __shared__ float corners[kMaxC][4][kTile * kTile];  // own pixels' source corners
  const int t = threadIdx.x;
  int ty0, tx0, b;
  photo_work(tiles_x, ty0, tx0, b);
  const int HW = H * W;
  const float* srcb = src + (size_t)b * C * HW;
  const float* tgtb = tgt + (size_t)b * C * HW;
  const float* mb = mask + (size_t)b * HW;
  const float* fb = flow + b * fbs;

  for (int e = t; e < RI * RI; e += 256) {
    const int ry = e / RI, rx = e - ry * RI;
    const int py = ty0 - 2 + ry, px = tx0 - 2 + rx;
    float m = 0.f;
    const bool in = py >= 0 && px >= 0 && py < H && px < W;
    const bool own = ry >= 2 && rx >= 2 && ry < kTile + 2 && rx < kTile + 2;
    const int o = (ry - 2) * kTile + (rx - 2);
    Tap tp;
    if (in) {
      tp = make_tap(fb[py * W + px], fb[HW + py * W + px], px, py, H, W, BORDER);
      m = mb[py * W + px];
    }
    // one channel at a time: gather the 4 corners, keep them in LDS for the
    // owned pixels (the coordinate derivative below needs them), store x and y
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) {
      if (c >= C) break;
      float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f, r = 0.f;
      if (in) {
        const float* sc = srcb + (size_t)c * HW;
        v0 = tp.m_nw ? sc[tp.o_nw] : 0.f;
        v1 = tp.m_ne ? sc[tp.o_ne] : 0.f;
        v2 = tp.m_sw ? sc[tp.o_sw] : 0.f;
        v3 = tp.m_se ? sc[tp.o_se] : 0.f;
        r = v0 * (tp.s * tp.e) + v1 * (tp.s * tp.w) + v2 * (tp.n * tp.e) + v3 * (tp.n * tp.w);
      }
      xs[c][ry][rx] = r * m;
      ys[c][ry][rx] = in ? tgtb[(size_t)c * HW + py * W + px] * m : 0.f;
      if (own) {
        corners[c][0][o] = v0;
        corners[c][1][o] = v1;
        corners[c][2][o] = v2;
        corners[c][3][o] = v3;
      }
    }
  }
  __syncthreads();
  for (int e = t; e < RW * RW; e += 256) {
    const int wy = e / RW, wx = e - wy * RW;
    const int qy = ty0 - 2 + wy, qx = tx0 - 2 + wx;
    const bool valid = qy >= 0 && qx >= 0 && qy <= H - 3 && qx <= W - 3;
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) {
      if (c >= C) break;
      float a = 0.f, bb = 0.f, g = 0.f;
      if (valid) {
        float sx = 0.f, sy = 0.f, sxx = 0.f, syy = 0.f, sxy = 0.f;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const float u = xs[c][wy + i][wx + j], v = ys[c][wy + i][wx + j];
            sx += u;
            sy += v;
            sxx += u * u;
            syy += v * v;
            sxy += u * v;
          }
        const float mx = sx / 9.f, my = sy / 9.f;
        const float mxy = mx * my, mx2 = mx * mx, my2 = my * my;
        const float sig_x = sxx / 9.f - mx2, sig_y = syy / 9.f - my2, sig_xy = sxy / 9.f - mxy;
        const float A1 = 2.f * mxy + kC1, A2 = 2.f * sig_xy + kC2;
        const float B1 = mx2 + my2 + kC1, B2 = sig_x + sig_y + kC2;
        const float n = A1 * A2, d = B1 * B2;
        const float r = n / d;
        const float raw = (1.f - r) / 2.f;
        if (raw >= 0.f && raw <= 1.f) {
          const float k = -1.f / (9.f * d);
          a = k * (my * (A2 - A1) - r * mx * (B2 - B1));
          bb = k * (-r * B1);
          g = k * A1;
        }
      }
      al[c][wy][wx] = a;
      be[c][wy][wx] = bb;
      ga[c][wy][wx] = g;
    }
  }
  __syncthreads();
  const int ly = t / kTile, lx = t % kTile;
  const int py = ty0 + ly, px = tx0 + lx;
  if (py >= H || px >= W) return;
  const float gl = *gloss;
  const float c_l1 = coef[1] * gl, c_ss = coef[2] * gl;
  const int HWp = py * W + px;
  const Tap tp = make_tap(fb[HWp], fb[HW + HWp], px, py, H, W, BORDER);  // weights + masks only
  const float m = mb[HWp];
  float dix = 0.f, diy = 0.f;
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) {
    if (c >= C) break;
    // windows covering p have top-left (py - i, px - j), i, j in 0..2 -> local (ly + 2 - i, lx + 2 - j)
    float sa = 0.f, sb = 0.f, sg = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        sa += al[c][ly + 2 - i][lx + 2 - j];
        sb += be[c][ly + 2 - i][lx + 2 - j];
        sg += ga[c][ly + 2 - i][lx + 2 - j];
      }
    const float xp = xs[c][ly + 2][lx + 2], yp = ys[c][ly + 2][lx + 2];
    const float tv = tgtb[(size_t)c * HW + py * W + px];
    const float vnw = corners[c][0][t], vne = corners[c][1][t];
    const float vsw = corners[c][2][t], vse = corners[c][3][t];
    const float rec = vnw * (tp.s * tp.e) + vne * (tp.s * tp.w) + vsw * (tp.n * tp.e) + vse * (tp.n * tp.w);
    const float diff = rec - tv;
    const float sgn = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
    const float g = (c_l1 * sgn + c_ss * (sa + sb * xp + sg * yp)) * m;  // dL / d rec_c
    dix += ((vne - vnw) * tp.s + (vse - vsw) * tp.n) * g;
    diy += ((vsw - vnw) * tp.e + (vse - vne) * tp.w) * g;
  }
  // grid grad, then norm_grid's autograd (warp.hip, warp_bwd_kernel)
  const float ggx = dix * tp.mx, ggy = diy * tp.my;
  float* gf = gflow + (size_t)b * 2 * HW + py * W + px;
  gf[0] = (ggx / (float)(W - 1)) * 2.0f;
  gf[HW] = (ggy / (float)(H - 1)) * 2.0f;
}

}  // namespace

int photo_partials(int B, int H, int W) {
  return 3 * B * ((H + kTile - 1) / kTile) * ((W + kTile - 1) / kTile);
}

hipError_t photo_fwd_launch(const float* src, const float* tgt, const float* mask, const float* flow,
                            long long fbs, float* partials, float* out, int B, int C, int H, int W,
                            int pad_mode, float w_l1, float w_ssim, hipStream_t s) {
  const int tiles_x = (W + kTile - 1) / kTile, tiles_y = (H + kTile - 1) / kTile;
  const dim3 grid((unsigned)(tiles_x * tiles_y), (unsigned)B);
  if (pad_mode == 1)
    hipLaunchKernelGGL(photo_fwd_kernel<true>, grid, dim3(256), 0, s, src, tgt, mask, flow, fbs,
                       partials, C, H, W, tiles_x);
  else
    hipLaunchKernelGGL(photo_fwd_kernel<false>, grid, dim3(256), 0, s, src, tgt, mask, flow, fbs,
                       partials, C, H, W, tiles_x);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const double n1 = (double)B * C * H * W;
  const double n2 = (H >= 3 && W >= 3) ? (double)B * C * (H - 2) * (W - 2) : 0.0;
  const double n3 = (double)B * H * W;
  hipLaunchKernelGGL(photo_final_kernel, dim3(1), dim3(256), 0, s, partials, tiles_x * tiles_y * B,
                     out, n1, n2, n3, w_l1, w_ssim);
  return hipGetLastError();
}

hipError_t photo_bwd_launch(const float* src, const float* tgt, const float* mask, const float* flow,
                            long long fbs, const float* coef, const float* gloss, float* gflow,
                            int B, int C, int H, int W, int pad_mode, hipStream_t s) {
  const int tiles_x = (W + kTile - 1) / kTile, tiles_y = (H + kTile - 1) / kTile;
  const dim3 grid((unsigned)(tiles_x * tiles_y), (unsigned)B);
  if (pad_mode == 1)
    hipLaunchKernelGGL(photo_bwd_kernel<true>, grid, dim3(256), 0, s, src, tgt, mask, flow, fbs,
                       coef, gloss, gflow, C, H, W, tiles_x);
  else
    hipLaunchKernelGGL(photo_bwd_kernel<false>, grid, dim3(256), 0, s, src, tgt, mask, flow, fbs,
                       coef, gloss, gflow, C, H, W, tiles_x);
  return hipGetLastError();
}

}  // namespace usf
