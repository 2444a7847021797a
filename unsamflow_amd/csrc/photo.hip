// Fused occlusion-aware photometric loss of unFlowLoss for gfx950 (CDNA4):
// the per-scale term of losses/flow_loss.py:127-148 with loss_photomatric
// (:33-50) and SSIM (losses/loss_blocks.py:53-72), for one flow direction or
// for both directions of a with_bk scale in one launch:
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
// only the flow does, and L is linear in its two normalised sums, so
//   dL/dflow_p = c_l1 * A_p + c_ssim * S'_p
// with the per-pixel vectors (dI/dflow = the bilinear tap's coordinate
// derivative incl. norm_grid and the border clip, as in warp.hip)
//   A_p  = m_p * sum_c sign(rec_pc - tgt_pc) * dI_pc/dflow
//   S'_p = m_p * sum_c (sum_{q ∋ p} dS_q/dx_pc) * dI_pc/dflow
// and the scalars c_l1 = w_l1 / (N_l1 (mean m + 1e-6)), c_ssim likewise, which
// are known only after the global reduction. So ONE pass does all the work:
// photo_fwd_kernel<GRAD> warps the source for a 32x16 tile + 2-pixel halo
// straight into LDS (x, y), sums the L1, SSIM and mask terms into per-tile
// partials and, when the flow needs a gradient, also evaluates the closed form
// dS_q/dx_p = alpha_q + beta_q x_p + gamma_q y_p per window, box-sums it around
// every pixel and writes the 4-float basis {A_p, S'_p} (16 B/pixel). A one-block
// (per direction) kernel combines the partials in a fixed fp64 order into
// {L, c_l1, c_ssim}; the backward is then a dense 24 B/pixel pass,
// gflow = g (c_l1 A + c_ssim S'). Nothing is recomputed between forward and
// backward and no warped image, SSIM map or dL/drec reaches HBM.
// Deterministic: fixed-order sums, no atomics.
//
// Work split (256 threads): the owner thread stages its two vertically
// adjacent pixels and keeps their tap derivatives in registers (no second
// flow / image read); the 208-pixel halo ring is one more staging pass. All
// global loads of the staging are issued before their first use
// (unconditional loads at clamped in-bounds offsets), so a workgroup pays the
// flow -> gather latency chain once. Windows are evaluated column-wise, three
// stacked windows per thread from five horizontal row sums (one pass over the
// 34 x 18 window grid); the pixel box sums reuse the overlap of the owner's two
// pixels. Window statistics use FMAs and a hardware reciprocal (the loss is
// checked against the reference at a stated tolerance); the warp coordinate
// chain keeps the reference rounding (warp_tap.h).
#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "usf_common.h"
#include "warp_tap.h"

namespace usf {
namespace {

constexpr int kTW = 32, kTH = 16;              // own tile: 32 x 16 pixels, 2 per thread
constexpr int kRW = kTW + 4, kRH = kTH + 4;    // x / y region: 2-pixel halo
constexpr int kWW = kTW + 2, kWH = kTH + 2;    // windows (top-left) the tile's pixels touch
constexpr int kXS = kRW + 1;                   // LDS row strides
constexpr int kAS = kWW + 1;
constexpr int kHalo = kRW * kRH - kTW * kTH;   // 208 halo pixels
constexpr int kWG = 3;                         // stacked windows per thread (window phase)
constexpr int kWItems = kWW * (kWH / kWG);     // 204 column items
constexpr int kNT = 256;
constexpr int kMaxC = 3;                       // image channels per pixel (RGB; LDS is sized for 3)
constexpr float kC1 = 0.01f * 0.01f;           // torch casts the python scalars to fp32
constexpr float kC2 = 0.03f * 0.03f;
static_assert(kHalo <= kNT && kWItems <= kNT && kWH % kWG == 0, "one pass per phase");

// one flow direction: rec = warp(src, flow), compared with tgt under mask
struct PhotoDir {
  const float* src;
  const float* tgt;
  const float* mask;
  const float* flow;  // [2,H,W] block per sample at flow + b * fbs
  float* basis;       // 4 planes per sample at basis + b * bbs, or null (forward only)
};
struct PhotoArgs {
  PhotoDir dir[2];
  long long fbs, bbs;  // flow / basis batch strides (elements)
  int B, C, H, W, tiles_x;
};

// region coordinates of halo element h (top 2 rows, bottom 2 rows, left 2 cols, right 2 cols)
__device__ __forceinline__ void halo_coord(int h, int& ry, int& rx) {
  if (h < 2 * kRW) {
    ry = h / kRW; rx = h - ry * kRW;
  } else if (h < 4 * kRW) {
    h -= 2 * kRW; ry = kRH - 2 + h / kRW; rx = h % kRW;
  } else if (h < 4 * kRW + 2 * kTH) {
    h -= 4 * kRW; ry = 2 + (h >> 1); rx = h & 1;
  } else {
    h -= 4 * kRW + 2 * kTH; ry = 2 + (h >> 1); rx = kRW - 2 + (h & 1);
  }
}

// One staged pixel: the reference coordinate chain (warp_tap.h), the 4 corner
// gathers of every channel and the target, all loads unconditional at
// clamped in-bounds offsets so they issue back to back.
struct Px {
  Tap tp;
  float m;
  float v[kMaxC][4];  // corners nw, ne, sw, se (0 where masked)
  float t[kMaxC];     // target
  bool in;
};

template <bool BORDER>
__device__ __forceinline__ void stage_load(Px& p, const float* __restrict__ srcb,
                                           const float* __restrict__ tgtb,
                                           const float* __restrict__ mb,
                                           const float* __restrict__ fb, int py, int px, int H,
                                           int W, int C) {
  const int HW = H * W;
  p.in = py >= 0 && px >= 0 && py < H && px < W;
  const int cy = min(max(py, 0), H - 1), cx = min(max(px, 0), W - 1);
  const int o = cy * W + cx;
  p.tp = make_tap(fb[o], fb[HW + o], cx, cy, H, W, BORDER);
  p.m = mb[o];
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) {
    if (c >= C) break;
    const float* sc = srcb + (size_t)c * HW;
    p.v[c][0] = sc[p.tp.o_nw];
    p.v[c][1] = sc[p.tp.o_ne];
    p.v[c][2] = sc[p.tp.o_sw];
    p.v[c][3] = sc[p.tp.o_se];
    p.t[c] = tgtb[(size_t)c * HW + o];
  }
}

// masks applied after the loads landed; rec in ATen's order; x, y to LDS
// (x, y) of one region pixel: one 8-byte LDS slot, so a window row's six
// values are three ds_read_b64 and the window statistics run on packed pairs
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void stage_finish(Px& p, int C, f2 (*xy)[kRH][kXS], int ry, int rx,
                                             float (&rec)[kMaxC]) {
#pragma clang fp contract(off)
  const Tap& tp = p.tp;
  const float wnw = tp.s * tp.e, wne = tp.s * tp.w, wsw = tp.n * tp.e, wse = tp.n * tp.w;
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) {
    if (c >= C) break;
    p.v[c][0] = tp.m_nw ? p.v[c][0] : 0.f;
    p.v[c][1] = tp.m_ne ? p.v[c][1] : 0.f;
    p.v[c][2] = tp.m_sw ? p.v[c][2] : 0.f;
    p.v[c][3] = tp.m_se ? p.v[c][3] : 0.f;
    rec[c] = p.v[c][0] * wnw + p.v[c][1] * wne + p.v[c][2] * wsw + p.v[c][3] * wse;
    xy[c][ry][rx] = f2{p.in ? rec[c] * p.m : 0.f, p.in ? p.t[c] * p.m : 0.f};
  }
}

// deterministic block sum of 3 values: wave butterflies, then waves in order
__device__ __forceinline__ void block_sum3(float a, float b, float c, float* red, float* out3) {
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    a += __shfl_xor(a, s);
    b += __shfl_xor(b, s);
    c += __shfl_xor(c, s);
  }
  const int t = threadIdx.x, wv = t >> 6;
  if ((t & 63) == 0) {
    red[3 * wv] = a;
    red[3 * wv + 1] = b;
    red[3 * wv + 2] = c;
  }
  __syncthreads();
  if (t == 0) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int w = 0; w < kNT / 64; ++w) {
      s0 += red[3 * w];
      s1 += red[3 * w + 1];
      s2 += red[3 * w + 2];
    }
    out3[0] = s0;
    out3[1] = s1;
    out3[2] = s2;
  }
}

// sums over 3 columns of one region row: {x, y}, {x^2, y^2}, xy (the pairs
// as packed fp32: the same per-component operations as the scalar forms)
struct Row5 {
  f2 s, ss;
  float sxy;
};
__device__ __forceinline__ Row5 row5(const f2* r3) {
  Row5 r;
  const f2 v0 = r3[0], v1 = r3[1], v2 = r3[2];
  r.s = v0 + v1 + v2;
  r.ss = __builtin_elementwise_fma(v2, v2, __builtin_elementwise_fma(v1, v1, v0 * v0));
  r.sxy = fmaf(v2.x, v2.y, fmaf(v1.x, v1.y, v0.x * v0.y));
  return r;
}

// SSIM of one window from its three row sums; with GRAD also the coefficients
// of dS/dx_p = alpha + beta x_p + gamma y_p (zero where the clamp is active:
// torch.clamp passes the gradient for 0 <= raw <= 1):
//   A1 = 2 mx my + C1, A2 = 2 sig_xy + C2, B1 = mx^2 + my^2 + C1, B2 = sig_x + sig_y + C2,
//   dS/dx_p = -(1 / (9 d)) [ my (A2 - A1) - r mx (B2 - B1) + A1 y_p - r B1 x_p ],  r = n / d
template <bool GRAD>
__device__ __forceinline__ float ssim_window(const Row5& r0, const Row5& r1, const Row5& r2,
                                             float& al, float& be, float& ga) {
  constexpr float k9 = 1.0f / 9.0f;
  const f2 m = (r0.s + r1.s + r2.s) * k9;     // mx, my
  const f2 e = (r0.ss + r1.ss + r2.ss) * k9;  // exx, eyy
  const float mx = m.x, my = m.y;
  const float exy = (r0.sxy + r1.sxy + r2.sxy) * k9;
  const float mxy = mx * my;
  const f2 m2 = m * m;   // mx^2, my^2
  const f2 sg = e - m2;  // sig_x, sig_y
  const float A1 = 2.f * mxy + kC1, A2 = 2.f * (exy - mxy) + kC2;
  const float B1 = m2.x + m2.y + kC1, B2 = sg.x + sg.y + kC2;
  const float d = B1 * B2;
  const float rd = __builtin_amdgcn_rcpf(d);
  const float r = (A1 * A2) * rd;
  const float raw = 0.5f - 0.5f * r;
  if constexpr (GRAD) {
    al = be = ga = 0.f;
    if (raw >= 0.f && raw <= 1.f) {
      const float k = -k9 * rd;
      al = k * (my * (A2 - A1) - r * mx * (B2 - B1));
      be = k * (-r * B1);
      ga = k * A1;
    }
  }
  return fminf(fmaxf(raw, 0.f), 1.f);
}

// ---------------------------------------------------------------- forward --
// grid = (tiles, B, ndir); XCD-aware order so that neighbouring tiles (shared
// halos and gather footprints) of one sample run on one L2
template <bool BORDER, bool GRAD>
__global__ __launch_bounds__(kNT) void photo_fwd_kernel(PhotoArgs a, float* __restrict__ partials) {
  __shared__ f2 xy[kMaxC][kRH][kXS];
  __shared__ float al[GRAD ? kMaxC : 1][GRAD ? kWH : 1][GRAD ? kAS : 1];
  __shared__ float be[GRAD ? kMaxC : 1][GRAD ? kWH : 1][GRAD ? kAS : 1];
  __shared__ float ga[GRAD ? kMaxC : 1][GRAD ? kWH : 1][GRAD ? kAS : 1];
  __shared__ float red[3 * kNT / 64];
  const int t = threadIdx.x;
  const int ntiles = gridDim.x;
  const int w = xcd_remap(linear_block(), ntiles * gridDim.y * gridDim.z);
  const int tile = w % ntiles;
  const int bd = w / ntiles;  // dir * B + b
  const int dirn = bd / a.B, b = bd - dirn * a.B;
  const int ty0 = (tile / a.tiles_x) * kTH, tx0 = (tile % a.tiles_x) * kTW;
  const PhotoDir& dr = a.dir[dirn];
  const int C = a.C, H = a.H, W = a.W, HW = H * W;
  const float* srcb = dr.src + (size_t)b * C * HW;
  const float* tgtb = dr.tgt + (size_t)b * C * HW;
  const float* mb = dr.mask + (size_t)b * HW;
  const float* fb = dr.flow + b * a.fbs;

  // ---- staging: own pixels (lx, ly0) and (lx, ly0 + 1), then one halo pixel
  const int lx = t & (kTW - 1), ly0 = 2 * (t / kTW);
  const bool has_halo = t < kHalo;
  int hy = 0, hx = 0;
  halo_coord(has_halo ? t : 0, hy, hx);
  Px own[2], hp;
#pragma unroll
  for (int k = 0; k < 2; ++k)
    stage_load<BORDER>(own[k], srcb, tgtb, mb, fb, ty0 + ly0 + k, tx0 + lx, H, W, C);
  stage_load<BORDER>(hp, srcb, tgtb, mb, fb, ty0 - 2 + hy, tx0 - 2 + hx, H, W, C);

  float l1 = 0.f, msum = 0.f;
  // per own pixel: dI_c/d(ix), dI_c/d(iy) (before the coordinate factors), sign(rec - tgt)
  float dix[2][kMaxC], diy[2][kMaxC], sg[2][kMaxC];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    float rec[kMaxC];
    stage_finish(own[k], C, xy, ly0 + k + 2, lx + 2, rec);
    const Px& p = own[k];
    if (p.in) msum += p.m;
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) {
      if (c >= C) break;
      if (p.in) l1 += fabsf(p.t[c] - rec[c]) * p.m;
      if constexpr (GRAD) {
        const float* v = p.v[c];
        dix[k][c] = (v[1] - v[0]) * p.tp.s + (v[3] - v[2]) * p.tp.n;
        diy[k][c] = (v[2] - v[0]) * p.tp.e + (v[3] - v[1]) * p.tp.w;
        const float diff = rec[c] - p.t[c];
        sg[k][c] = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
      }
    }
  }
  if (has_halo) {
    float rec[kMaxC];
    stage_finish(hp, C, xy, hy, hx, rec);
  }
  __syncthreads();

  // ---- windows, column-wise: item (g, wx) evaluates windows (kWG g + r, wx),
  // r < kWG, from kWG + 2 horizontal row sums. Without GRAD only the tile's
  // own windows (window rows / cols >= 2) are needed.
  float ssim = 0.f;
  if (t < kWItems) {
    const int g = t / kWW, wx = t - g * kWW;
    const int wy0 = kWG * g;
    const int qx = tx0 - 2 + wx;
    const bool col_ok = qx >= 0 && qx <= W - 3;
    const bool col_own = wx >= 2;
    if (GRAD || (col_own && wy0 + kWG > 2)) {
#pragma unroll
      for (int c = 0; c < kMaxC; ++c) {
        if (c >= C) break;
        Row5 rs[kWG + 2];
#pragma unroll
        for (int i = 0; i < kWG + 2; ++i) rs[i] = row5(&xy[c][wy0 + i][wx]);
#pragma unroll
        for (int r = 0; r < kWG; ++r) {
          const int wy = wy0 + r, qy = ty0 - 2 + wy;
          const bool valid = col_ok && qy >= 0 && qy <= H - 3;
          float a1 = 0.f, b1 = 0.f, g1 = 0.f;
          const float s = ssim_window<GRAD>(rs[r], rs[r + 1], rs[r + 2], a1, b1, g1);
          if (valid && col_own && wy >= 2) ssim += s;
          if constexpr (GRAD) {
            al[c][wy][wx] = valid ? a1 : 0.f;
            be[c][wy][wx] = valid ? b1 : 0.f;
            ga[c][wy][wx] = valid ? g1 : 0.f;
          }
        }
      }
    }
  }
  const int blk = bd * ntiles + tile;  // fixed slot per (direction, sample, tile)
  block_sum3(l1, ssim, msum, red, partials + 3 * blk);  // (its barrier also orders al/be/ga)
  if constexpr (!GRAD) return;

  // ---- gradient basis of the own pixels: box sums of the 9 windows around each;
  // the two pixels share 2 of their 3 window rows (window rows ly0 .. ly0 + 3)
  float ax[2] = {0.f, 0.f}, ay[2] = {0.f, 0.f}, bx[2] = {0.f, 0.f}, by[2] = {0.f, 0.f};
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) {
    if (c >= C) break;
    float ra[4], rb[4], rg[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float* pa = &al[c][ly0 + i][lx];
      const float* pb = &be[c][ly0 + i][lx];
      const float* pg = &ga[c][ly0 + i][lx];
      ra[i] = pa[0] + pa[1] + pa[2];
      rb[i] = pb[0] + pb[1] + pb[2];
      rg[i] = pg[0] + pg[1] + pg[2];
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const float sa = ra[k] + ra[k + 1] + ra[k + 2];
      const float sb = rb[k] + rb[k + 1] + rb[k + 2];
      const float sgm = rg[k] + rg[k + 1] + rg[k + 2];
      const f2 pxy = xy[c][ly0 + k + 2][lx + 2];
      const float xp = pxy.x, yp = pxy.y;
      const float ds = sa + sb * xp + sgm * yp;  // sum_q dS_q / dx_pc
      ax[k] += sg[k][c] * dix[k][c];
      ay[k] += sg[k][c] * diy[k][c];
      bx[k] += ds * dix[k][c];
      by[k] += ds * diy[k][c];
    }
  }
  // dL/drec_pc carries the mask m (x = rec m); grid grad -> norm_grid autograd
  const float fxs = 2.0f / (float)(W - 1), fys = 2.0f / (float)(H - 1);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const Px& p = own[k];
    if (!p.in) continue;
    const float kx = p.m * p.tp.mx * fxs, ky = p.m * p.tp.my * fys;
    float* o = dr.basis + (size_t)b * a.bbs + (ty0 + ly0 + k) * W + tx0 + lx;
    o[0] = ax[k] * kx;
    o[HW] = ay[k] * ky;
    o[2 * HW] = bx[k] * kx;
    o[3 * HW] = by[k] * ky;
  }
}

// One block per direction: fixed-order fp64 sum of its partials ->
// out[3 dir ..] = {loss, c_l1, c_ssim}, c_* = w_* / (N_* * (mean(m) + 1e-6)).
constexpr int kFinNT = 512;
__global__ __launch_bounds__(kFinNT) void photo_final_kernel(const float* __restrict__ partials,
                                                             int nblk, float* __restrict__ out,
                                                             double n1, double n2, double n3,
                                                             float w_l1, float w_ssim) {
  __shared__ double red[3][kFinNT / 64];
  const int t = threadIdx.x, dirn = blockIdx.x;
  const float* p = partials + (size_t)3 * nblk * dirn;
  double a = 0, b = 0, c = 0;
  int i = t;
  // 4 slots in flight per thread, summed in slot order (fixed)
  for (; i + 3 * kFinNT < nblk; i += 4 * kFinNT) {
    float v[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 3; ++q) v[j][q] = p[3 * (i + j * kFinNT) + q];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a += v[j][0];
      b += v[j][1];
      c += v[j][2];
    }
  }
  for (; i < nblk; i += kFinNT) {
    a += p[3 * i];
    b += p[3 * i + 1];
    c += p[3 * i + 2];
  }
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    a += __shfl_xor(a, s);
    b += __shfl_xor(b, s);
    c += __shfl_xor(c, s);
  }
  if ((t & 63) == 0) {
    red[0][t >> 6] = a;
    red[1][t >> 6] = b;
    red[2][t >> 6] = c;
  }
  __syncthreads();
  if (t == 0) {
    double s0 = 0, s1 = 0, s2 = 0;
    for (int w = 0; w < kFinNT / 64; ++w) {
      s0 += red[0][w];
      s1 += red[1][w];
      s2 += red[2][w];
    }
    const double den = s2 / n3 + 1e-6;
    const double l1 = n1 > 0 ? s0 / n1 : 0.0, ss = n2 > 0 ? s1 / n2 : 0.0;
    float* o = out + 3 * dirn;
    o[0] = (float)((w_l1 * l1 + w_ssim * ss) / den);
    o[1] = n1 > 0 ? (float)(w_l1 / (n1 * den)) : 0.f;
    o[2] = n2 > 0 ? (float)(w_ssim / (n2 * den)) : 0.f;
  }
}

// --------------------------------------------------------------- backward --
// gflow[b, 2 dir + j, p] = g_dir (c_l1 basis[b, 4 dir + j, p] + c_ssim basis[b, 4 dir + 2 + j, p])
__global__ __launch_bounds__(256) void photo_bwd_kernel(const float* __restrict__ basis,
                                                        const float* __restrict__ coef,
                                                        const float* __restrict__ gloss,
                                                        float* __restrict__ gflow, int HW, int ndir) {
  const int dirn = blockIdx.z, b = blockIdx.y;
  const float gl = gloss[dirn];
  const float k1 = coef[3 * dirn + 1] * gl, k2 = coef[3 * dirn + 2] * gl;
  const float* a = basis + ((size_t)b * ndir + dirn) * 4 * HW;
  float* o = gflow + ((size_t)b * ndir + dirn) * 2 * HW;
  const int i = (blockIdx.x * 256 + threadIdx.x) * 4;
  if ((HW & 3) == 0) {
    if (i >= HW) return;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float4 u = *reinterpret_cast<const float4*>(a + j * HW + i);
      const float4 v = *reinterpret_cast<const float4*>(a + (2 + j) * HW + i);
      *reinterpret_cast<float4*>(o + j * HW + i) =
          make_float4(k1 * u.x + k2 * v.x, k1 * u.y + k2 * v.y, k1 * u.z + k2 * v.z, k1 * u.w + k2 * v.w);
    }
  } else {
    for (int e = i; e < i + 4 && e < HW; ++e)
#pragma unroll
      for (int j = 0; j < 2; ++j) o[j * HW + e] = k1 * a[j * HW + e] + k2 * a[(2 + j) * HW + e];
  }
}

// ------------------------------------------------------- strip (row-stream) --
// photo_strip_kernel: the same per-direction result as photo_fwd_kernel,
// organised for gfx950's wave instead of a workgroup tile. One WAVE owns a
// strip of 64 staged columns (lanes; the 60 middle ones are its own pixels)
// by R own rows and streams down it, one staged row per step:
//   stage row r   -> lane l holds x = rec*m, y = tgt*m of column x0-2+l (C channels)
//   row sums      -> 3-column sums of x, y, x^2, y^2, xy by two DPP adds each
//                    (v_add_f32_dpp wave_shl:1: lane l reads lane l+1)
//   window r-2    -> the three latest row sums (kept in registers) give the 3x3
//                    window whose top-left row is r-2: SSIM, and with GRAD the
//                    coefficients alpha, beta, gamma of its pixel derivative
//   pixel row r-2 -> the 3x3 box sums of alpha/beta/gamma around each pixel
//                    (vertical in registers, horizontal by DPP wave_shr:1)
//                    complete its gradient basis.
// No LDS, no barriers: the waves of a workgroup are independent (4 per
// workgroup only to fill CUs in fewer dispatches). Each staged pixel is
// warped once; the halo is 2 rows above and below each strip (R chosen per
// shape, strip_plan) and 2 columns either side. The next row's flow, mask and
// target loads are issued one step ahead. Work items are (sample, strip,
// direction) with the direction fastest, so both directions of a strip run
// side by side on one CU and share the two frames' lines in L1/L2.
#ifndef USF_PHOTO_WAVES
#define USF_PHOTO_WAVES 2  // waves per SIMD the strip kernel's registers are sized for
#endif
constexpr int kSL = 64;        // lanes of a strip = staged columns
constexpr int kSO = kSL - 4;   // own columns per strip (lanes 2 .. 61)
constexpr int kOffNone = 0x7FFFFFF0;  // buffer offset past num_records: reads 0
constexpr int kRsrcWord3 = 0x00020000;

struct StripArgs {
  PhotoDir dir[2];
  long long fbs, bbs;
  int B, H, W, R, nsx, nsy, ndir, nitems;
};

// lane l reads lane l+1 / l-1 of the wave (DPP wave_shl:1 / wave_shr:1;
// the missing neighbour of lane 63 / 0 reads 0). Every lane must be active.
// mov_dpp with bound_ctrl (no "old" operand to materialise), so the compiler
// folds it into the add that consumes it (v_add_f32_dpp).
__device__ __forceinline__ float from_next(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true));
}
__device__ __forceinline__ float from_prev(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float hsum_next(float v) { return v + from_next(v + from_next(v)); }  // v[l]+v[l+1]+v[l+2]
__device__ __forceinline__ float hsum_prev(float v) { return v + from_prev(v + from_prev(v)); }  // v[l]+v[l-1]+v[l-2]

struct Sums {   // window statistics need only x, y, x^2 + y^2 and xy
  float x, y, q, xy;
};

// SSIM of one window from its sums over the 9 pixels, and with GRAD the
// coefficients of dS/dx_p = alpha + beta x_p + gamma y_p (see ssim_window)
template <bool GRAD>
__device__ __forceinline__ float ssim_sums(const Sums& s, float& al, float& be, float& ga) {
  constexpr float k9 = 1.0f / 9.0f;
  const float mx = s.x * k9, my = s.y * k9;
  const float exy = s.xy * k9;
  const float mxy = mx * my;
  const float m2 = fmaf(mx, mx, my * my);                  // mx^2 + my^2
  const float A1 = fmaf(2.f, mxy, kC1), A2 = fmaf(2.f, exy - mxy, kC2);
  const float B1 = m2 + kC1;
  const float B2 = fmaf(s.q, k9, -m2) + kC2;              // sig_x + sig_y + C2
  const float rd = __builtin_amdgcn_rcpf(B1 * B2);
  const float r = (A1 * A2) * rd;
  const float raw = fmaf(-0.5f, r, 0.5f);
  const float cl = __builtin_amdgcn_fmed3f(raw, 0.f, 1.f);
  if constexpr (GRAD) {
    const bool pass = cl == raw;  // torch.clamp passes the gradient for 0 <= raw <= 1
    const float k = pass ? -k9 * rd : 0.f;
    al = k * fmaf(-r * mx, B2 - B1, my * (A2 - A1));
    be = (k * -r) * B1;
    ga = k * A1;
  }
  return cl;
}

// The warp tap of warp_tap.h (same rounding, same results) with the border
// clip as selects instead of branches, and the four corner byte offsets for
// buffer loads: a masked corner gets an offset past num_records, which the
// hardware reads as 0 (no value selects after the loads).
struct TapB {
  int onw, one, osw, ose;
  float n, s, w, e, mx, my;
};
template <bool BORDER>
__device__ __forceinline__ TapB make_tap_b(float u, float v, int x, int y, int H, int W) {
#pragma clang fp contract(off)
  TapB t;
  const float wm1 = (float)(W - 1), hm1 = (float)(H - 1);
  const float gx = 2.0f * ((float)x + u) / wm1 - 1.0f;
  const float gy = 2.0f * ((float)y + v) / hm1 - 1.0f;
  const float sx = wm1 / 2.0f, sy = hm1 / 2.0f;
  float ix = (gx + 1.0f) * sx;
  float iy = (gy + 1.0f) * sy;
  t.mx = sx;
  t.my = sy;
  if (BORDER) {
    const bool xlo = !(ix > 0.f), xhi = ix >= wm1, ylo = !(iy > 0.f), yhi = iy >= hm1;
    ix = xlo ? 0.f : (xhi ? wm1 : ix);
    iy = ylo ? 0.f : (yhi ? hm1 : iy);
    t.mx = (xlo || xhi) ? 0.f : sx;
    t.my = (ylo || yhi) ? 0.f : sy;
  }
  const float fx = floorf(ix), fy = floorf(iy);
  t.w = ix - fx;
  t.e = 1.0f - t.w;
  t.n = iy - fy;
  t.s = 1.0f - t.n;
  const int xw = (int)fx, yn = (int)fy;
  const bool vxw = (unsigned)xw < (unsigned)W, vxe = (unsigned)(xw + 1) < (unsigned)W;
  const bool vyn = (unsigned)yn < (unsigned)H, vys = (unsigned)(yn + 1) < (unsigned)H;
  const int o = 4 * (yn * W + xw);
  t.onw = vxw && vyn ? o : kOffNone;
  t.one = vxe && vyn ? o + 4 : kOffNone;
  t.osw = vxw && vys ? o + 4 * W : kOffNone;
  t.ose = vxe && vys ? o + 4 * W + 4 : kOffNone;
  return t;
}

// One wave's strip, as a stream of staged rows. Every ring (loads of rows r
// and r+1, row sums of rows r-2..r, window coefficients of window rows
// q-2..q, pixel state of rows r-2..r) has period 3, and step<PH> handles the
// rows with r = y0 - 2 + i, i = PH mod 3, so all ring slots are compile-time
// registers: no copies between steps.
template <bool BORDER, bool GRAD, int C>
struct Strip {
  // per-wave constants: buffer resources of the sample's source planes (gathers),
  // flow, mask, target (row loads) and basis (stores); 32-bit byte offsets
  __amdgpu_buffer_rsrc_t rs[C], rflow, rmask, rtgt, rbas;
  int H, W, HW, y0, rown, col, cc, lane;
  bool col_in, lane_own, wcol;
  float fxs, fys;
  // rings (period 3). The memory work of a row runs ahead of its arithmetic:
  // its flow is loaded two steps early, its tap evaluated and its gathers,
  // target and mask loads issued one step early, so a wave's gather latency
  // overlaps the previous row's window and basis work.
  float fu[3], fv[3];                        // flow of a row
  float gv[3][C][4], tt[3][C], mm[3];        // gathered corners (nw, ne, sw, se), target, mask
  float tn[3], tw[3], tmx[3], tmy[3];        // tap distances (s = 1 - n, e = 1 - w) and coordinate factors
  Sums sm[3][C];                             // row sums of x, y, x^2 + y^2, xy
  float ca[3][C], cb[3][C], cg[3][C];        // window coefficients alpha, beta, gamma
  // pixel state from its staging to the completion of its basis two steps later
  // ({dix*kx, diy*ky, x, y} per channel, 12 floats packed in 3 float4s): in LDS,
  // this wave's own planes [slot][chunk][lane] (16-byte lanes, conflict-free),
  // which keeps the kernel at 3 waves per SIMD
  float4* pend;
  float l1, ssum, msum;

  // Every memory instruction of a step is issued on every path: rows outside
  // the image or past the strip, and lanes that own no output, use a byte
  // offset past num_records (loads read 0, stores are dropped) instead of a
  // branch. The compiler's s_waitcnt then counts the same instructions on all
  // paths and can wait for row r's gathers without waiting for row r+1's (a
  // branch around a load made it wait for everything, vmcnt(0)).
  __device__ __forceinline__ static float ld(__amdgpu_buffer_rsrc_t r, int off, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, soff, 0));
  }
  __device__ __forceinline__ void st(float v, int off, int soff) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), rbas, off, soff, 0);
  }
  __device__ __forceinline__ int row_off(int r, bool ok) const {
    return ok && r >= 0 && r < H ? 4 * (r * W + cc) : kOffNone;
  }
  template <int slot>
  __device__ __forceinline__ void load_flow(int r, bool ok) {
    const int o = row_off(r, ok);
    fu[slot] = ld(rflow, o, 0);
    fv[slot] = ld(rflow, o, 4 * HW);
  }
  // the row's tap, then its gathers and its target / mask loads (not waited for)
  template <int slot>
  __device__ __forceinline__ void issue(int r, bool ok) {
    const TapB tp = make_tap_b<BORDER>(fu[slot], fv[slot], cc, r, H, W);
    const int o = row_off(r, ok);
    const bool in = o != kOffNone;
    const int onw = in ? tp.onw : kOffNone, one = in ? tp.one : kOffNone;
    const int osw = in ? tp.osw : kOffNone, ose = in ? tp.ose : kOffNone;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      gv[slot][c][0] = ld(rs[c], onw, 0);
      gv[slot][c][1] = ld(rs[c], one, 0);
      gv[slot][c][2] = ld(rs[c], osw, 0);
      gv[slot][c][3] = ld(rs[c], ose, 0);
      tt[slot][c] = ld(rtgt, o, 4 * c * HW);
    }
    mm[slot] = ld(rmask, o, 0);
    tn[slot] = tp.n;
    tw[slot] = tp.w;
    tmx[slot] = tp.mx;
    tmy[slot] = tp.my;
  }

  // ST / WIN / BAS: whether row r is an own row (staged with its gradient
  // state), window row r - 2 is computed, pixel row r - 2's basis completes:
  // 0 = never, 1 = always, 2 = decided at run time. The strip's interior steps
  // run with all three known true (no branches, no value merges); the first
  // four and the last two to four steps decide at run time.
  template <int PH, int ST = 2, int WIN = 2, int BAS = 2>
  __device__ __forceinline__ void step(int i, int nsteps) {
    constexpr int S0 = PH, S1 = (PH + 2) % 3, S2 = (PH + 1) % 3;  // slots of rows r, r-1, r-2
    const int r = y0 - 2 + i;
    // rows r+2 and r+1 reuse the memory-side slots of rows r-1 and r-2
    load_flow<S1>(r + 2, i + 2 < nsteps);
    issue<S2>(r + 1, i + 1 < nsteps);

    // ---- stage row r: x = rec * m, y = tgt * m (all loads read 0 outside the image)
    const bool own_row = ST == 2 ? (i >= 2 && i < rown + 2) : ST == 1;  // wave-uniform
    float x[C], y[C];
    const float n = tn[S0], w = tw[S0];
    float s, e;
    {
#pragma clang fp contract(off)
      s = 1.0f - n;  // as make_tap_b computes them
      e = 1.0f - w;
    }
    const float (&v)[C][4] = gv[S0];
    const float m = mm[S0];
    const float me = col_in ? m : 0.f;
    float rec[C];
    {
#pragma clang fp contract(off)
      const float wnw = s * e, wne = s * w, wsw = n * e, wse = n * w;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        rec[c] = v[c][0] * wnw + v[c][1] * wne + v[c][2] * wsw + v[c][3] * wse;
        x[c] = rec[c] * me;
        y[c] = tt[S0][c] * me;
      }
    }
    float ax = 0.f, ay = 0.f, kx = 0.f, ky = 0.f;
    float pk[4 * C];
#pragma unroll
    for (int k = 0; k < 4 * C; ++k) pk[k] = 0.f;
    if (own_row) {  // compute only
      const float mo = lane_own ? m : 0.f;  // L1 / mask sums: own pixels only
      kx = m * tmx[S0] * fxs;
      ky = m * tmy[S0] * fys;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float diff = rec[c] - tt[S0][c];
        l1 += fabsf(diff) * mo;
        if constexpr (GRAD) {
          const float dix = (v[c][1] - v[c][0]) * s + (v[c][3] - v[c][2]) * n;
          const float diy = (v[c][2] - v[c][0]) * e + (v[c][3] - v[c][1]) * w;
          const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
          ax += sg * dix;
          ay += sg * diy;
          pk[4 * c] = dix * kx;
          pk[4 * c + 1] = diy * ky;
          pk[4 * c + 2] = x[c];
          pk[4 * c + 3] = y[c];
        }
      }
      msum += mo;
    }
    if constexpr (GRAD) {
#pragma unroll
      for (int k = 0; k < C; ++k)
        pend[(S0 * C + k) * 64 + lane] = make_float4(pk[4 * k], pk[4 * k + 1], pk[4 * k + 2], pk[4 * k + 3]);
      const int o = own_row && lane_own ? 4 * (r * W + col) : kOffNone;
      st(ax * kx, o, 0);
      st(ay * ky, o, 4 * HW);
    }

    // ---- row sums of row r
#pragma unroll
    for (int c = 0; c < C; ++c)
      sm[S0][c] = Sums{hsum_next(x[c]), hsum_next(y[c]), hsum_next(fmaf(x[c], x[c], y[c] * y[c])),
                       hsum_next(x[c] * y[c])};

    // ---- window with top-left row q = r - 2, then pixel row q's gradient basis
    const int q = r - 2;
    const bool qown = BAS == 2 ? i >= 4 : BAS == 1;  // q is an own row of this strip (wave-uniform)
    float4 pq[C];              // pixel row q's state
    if constexpr (GRAD) {
#pragma unroll
      for (int k = 0; k < C; ++k) pq[k] = pend[(S2 * C + k) * 64 + lane];
    }
    float bx = 0.f, by = 0.f;
    if (WIN == 2 ? i >= 2 : WIN == 1) {  // compute only
      // (in interior steps q is an own row, so 0 <= q <= H - 3 holds)
      const bool wrow = WIN == 1 || (q >= 0 && q <= H - 3);  // wave-uniform
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float al = 0.f, be = 0.f, ga = 0.f;
        if (wrow) {
          const Sums& a2 = sm[S2][c];
          const Sums& a1 = sm[S1][c];
          const Sums& a0 = sm[S0][c];
          const Sums w{a2.x + a1.x + a0.x, a2.y + a1.y + a0.y, a2.q + a1.q + a0.q, a2.xy + a1.xy + a0.xy};
          const float s = ssim_sums<GRAD>(w, al, be, ga);
          ssum += qown && lane_own && wcol ? s : 0.f;
          if (!wcol) al = be = ga = 0.f;
        }
        if constexpr (GRAD) {
          ca[S0][c] = al;
          cb[S0][c] = be;
          cg[S0][c] = ga;
          if (qown) {
            const float ha = hsum_prev(ca[S2][c] + ca[S1][c] + al);
            const float hb = hsum_prev(cb[S2][c] + cb[S1][c] + be);
            const float hg = hsum_prev(cg[S2][c] + cg[S1][c] + ga);
            const float ds = fmaf(hg, pq[c].w, fmaf(hb, pq[c].z, ha));  // sum over windows q' of p
            bx = fmaf(ds, pq[c].x, bx);
            by = fmaf(ds, pq[c].y, by);
          }
        }
      }
    }
    if constexpr (GRAD) {
      const int o = qown && lane_own ? 4 * (q * W + col) : kOffNone;
      st(bx, o, 8 * HW);
      st(by, o, 12 * HW);
    }
  }
};

template <bool BORDER, bool GRAD, int C>
__global__ __launch_bounds__(256, USF_PHOTO_WAVES) void photo_strip_kernel(StripArgs a, float* __restrict__ partials) {
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6));
  if (wid >= a.nitems) return;
  int rest = wid;
  int dirn = 0;
  if (a.ndir == 2) {
    dirn = rest & 1;
    rest >>= 1;
  }
  const int sx = rest % a.nsx;
  rest /= a.nsx;
  const int sy = rest % a.nsy;
  const int b = rest / a.nsy;
  const PhotoDir dr = a.dir[dirn];
  __shared__ float4 pend_lds[GRAD ? 4 * 3 * C * 64 : 1];
  Strip<BORDER, GRAD, C> st;
  st.pend = pend_lds + (threadIdx.x >> 6) * (3 * C * 64);
  st.H = a.H;
  st.W = a.W;
  st.HW = a.H * a.W;
  const int x0 = sx * kSO;
  // balanced strips: heights H / nsy rounded down or up
  st.y0 = (int)((long long)sy * a.H / a.nsy);
  st.rown = (int)((long long)(sy + 1) * a.H / a.nsy) - st.y0;
  st.lane = lane;
  st.col = x0 - 2 + lane;
  st.cc = min(max(st.col, 0), a.W - 1);
  st.col_in = st.col >= 0 && st.col < a.W;
  st.lane_own = lane >= 2 && lane < 2 + kSO && st.col < a.W;
  st.wcol = st.col >= 0 && st.col <= a.W - 3;  // window with top-left column col is valid
  const size_t HW = (size_t)st.HW;
  const float* srcb = dr.src + (size_t)b * C * HW;
  const int pb = st.HW * 4;  // plane bytes (< 2^31, capi.cpp)
#pragma unroll
  for (int c = 0; c < C; ++c)
    st.rs[c] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(srcb + (size_t)c * HW), 0, pb, kRsrcWord3);
  st.rtgt = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dr.tgt + (size_t)b * C * HW), 0, C * pb, kRsrcWord3);
  st.rmask = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dr.mask + (size_t)b * HW), 0, pb, kRsrcWord3);
  st.rflow = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dr.flow + b * a.fbs), 0, 2 * pb, kRsrcWord3);
  if constexpr (GRAD)
    st.rbas = __builtin_amdgcn_make_buffer_rsrc(dr.basis + b * a.bbs, 0, 4 * pb, kRsrcWord3);
  st.fxs = 2.0f / (float)(a.W - 1);
  st.fys = 2.0f / (float)(a.H - 1);
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int c = 0; c < C; ++c) {
      st.sm[k][c] = Sums{0.f, 0.f, 0.f, 0.f};
      st.ca[k][c] = st.cb[k][c] = st.cg[k][c] = 0.f;
    }
  st.l1 = st.ssum = st.msum = 0.f;
  const int nsteps = st.rown + 4;
  st.template load_flow<0>(st.y0 - 2, true);
  st.template load_flow<1>(st.y0 - 1, true);
  st.template issue<0>(st.y0 - 2, true);
  // steps 0-3: the two halo rows above, then own rows y0, y0 + 1 (if the
  // strip has them) with the windows above them; no basis completes yet
  st.template step<0, 0, 0, 0>(0, nsteps);
  st.template step<1, 0, 0, 0>(1, nsteps);
  st.template step<2, 2, 2, 0>(2, nsteps);
  st.template step<0, 2, 2, 0>(3, nsteps);
  // interior: own row staged, window and basis of the row two above
  int i = 4;
  for (; i + 3 <= st.rown + 2; i += 3) {
    st.template step<1, 1, 1, 1>(i, nsteps);
    st.template step<2, 1, 1, 1>(i + 1, nsteps);
    st.template step<0, 1, 1, 1>(i + 2, nsteps);
  }
  // tail: up to two interior steps left, then the two halo rows below (at most 4)
  if (i < nsteps) st.template step<1>(i, nsteps);
  if (i + 1 < nsteps) st.template step<2>(i + 1, nsteps);
  if (i + 2 < nsteps) st.template step<0>(i + 2, nsteps);
  if (i + 3 < nsteps) st.template step<1>(i + 3, nsteps);

  // ---- wave partials (fixed-order butterflies), one slot per (direction, sample, strip)
  float l1 = st.l1, ssum = st.ssum, msum = st.msum;
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    l1 += __shfl_xor(l1, s);
    ssum += __shfl_xor(ssum, s);
    msum += __shfl_xor(msum, s);
  }
  if (lane == 0) {
    float* o = partials + 3 * (((size_t)dirn * a.B + b) * a.nsy * a.nsx + (size_t)sy * a.nsx + sx);
    o[0] = l1;
    o[1] = ssum;
    o[2] = msum;
  }
}

// ------------------------------------------------ producer / consumer pair --
// photo_pc_kernel: the strip stream of photo_strip_kernel split over a PAIR of
// waves, so each holds half the state and twice as many waves share a SIMD.
// The producer stages rows (flow, tap, gathers, x = rec m, y = tgt m, the L1
// and mask sums, its own pixels' dI/dflow and the A basis) and hands each row's
// x, y and {dix kx, diy ky} to the consumer through an LDS ring; the consumer
// turns them into row sums, windows (SSIM and its coefficients) and the S
// basis, one row behind. One workgroup barrier per step: the producer writes
// row t while the consumer reads rows t-1 (new) and t-3 (the pixel row whose
// basis completes), so a ring of 4 rows suffices. Both pairs of a workgroup
// stream the same strip rows (the two directions, or two neighbouring strips),
// so they take the same number of steps and barriers.
constexpr int kRing = 4;

template <bool BORDER, bool GRAD, int C>
struct PairCommon {
  __amdgpu_buffer_rsrc_t rbas;
  int H, W, HW, y0, rown, col, cc, lane;
  bool col_in, lane_own, wcol;
  float* xy;  // this pair's LDS ring: [kRing][C][2][64] (x, y planes)
  float* pd;  // [kRing][C][2][64] (dix kx, diy ky planes)
  __device__ __forceinline__ void st(float v, int off, int soff) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(int, v), rbas, off, soff, 0);
  }
  __device__ __forceinline__ int ring(int slot, int c, int k) const { return ((slot * C + c) * 2 + k) * 64 + lane; }
};

template <bool BORDER, bool GRAD, int C>
struct Producer : PairCommon<BORDER, GRAD, C> {
  using B_ = PairCommon<BORDER, GRAD, C>;
  __amdgpu_buffer_rsrc_t rs[C], rflow, rmask, rtgt;
  float fxs, fys;
  float fu[3], fv[3];
  float gv[3][C][4], tt[3][C], mm[3];
  float tn[3], tw[3], tmx[3], tmy[3];
  float l1, msum;

  __device__ __forceinline__ static float ld(__amdgpu_buffer_rsrc_t r, int off, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, soff, 0));
  }
  __device__ __forceinline__ int row_off(int r, bool ok) const {
    return ok && r >= 0 && r < this->H ? 4 * (r * this->W + this->cc) : kOffNone;
  }
  template <int slot>
  __device__ __forceinline__ void load_flow(int r, bool ok) {
    const int o = row_off(r, ok);
    fu[slot] = ld(rflow, o, 0);
    fv[slot] = ld(rflow, o, 4 * this->HW);
  }
  template <int slot>
  __device__ __forceinline__ void issue(int r, bool ok) {
    const TapB tp = make_tap_b<BORDER>(fu[slot], fv[slot], this->cc, r, this->H, this->W);
    const int o = row_off(r, ok);
    const bool in = o != kOffNone;
    const int onw = in ? tp.onw : kOffNone, one = in ? tp.one : kOffNone;
    const int osw = in ? tp.osw : kOffNone, ose = in ? tp.ose : kOffNone;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      gv[slot][c][0] = ld(rs[c], onw, 0);
      gv[slot][c][1] = ld(rs[c], one, 0);
      gv[slot][c][2] = ld(rs[c], osw, 0);
      gv[slot][c][3] = ld(rs[c], ose, 0);
      tt[slot][c] = ld(rtgt, o, 4 * c * this->HW);
    }
    mm[slot] = ld(rmask, o, 0);
    tn[slot] = tp.n;
    tw[slot] = tp.w;
    tmx[slot] = tp.mx;
    tmy[slot] = tp.my;
  }
  // row r = y0 - 2 + i; ST: own row (0 / 1 / 2 = run time); ends with the step's barrier
  template <int PH, int ST>
  __device__ __forceinline__ void step(int i, int nsteps) {
    constexpr int S0 = PH, S1 = (PH + 2) % 3, S2 = (PH + 1) % 3;
    const int r = this->y0 - 2 + i;
    load_flow<S1>(r + 2, i + 2 < nsteps);
    issue<S2>(r + 1, i + 1 < nsteps);
    const bool own_row = ST == 2 ? (i >= 2 && i < this->rown + 2) : ST == 1;
    const float n = tn[S0], w = tw[S0];
    float s, e;
    {
#pragma clang fp contract(off)
      s = 1.0f - n;
      e = 1.0f - w;
    }
    const float (&v)[C][4] = gv[S0];
    const float m = mm[S0];
    const float me = this->col_in ? m : 0.f;
    float rec[C], x[C], y[C];
    {
#pragma clang fp contract(off)
      const float wnw = s * e, wne = s * w, wsw = n * e, wse = n * w;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        rec[c] = v[c][0] * wnw + v[c][1] * wne + v[c][2] * wsw + v[c][3] * wse;
        x[c] = rec[c] * me;
        y[c] = tt[S0][c] * me;
      }
    }
    float ax = 0.f, ay = 0.f, kx = 0.f, ky = 0.f;
    float dk[C][2];
#pragma unroll
    for (int c = 0; c < C; ++c) dk[c][0] = dk[c][1] = 0.f;
    if (own_row) {
      const float mo = this->lane_own ? m : 0.f;
      kx = m * tmx[S0] * fxs;
      ky = m * tmy[S0] * fys;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float diff = rec[c] - tt[S0][c];
        l1 += fabsf(diff) * mo;
        if constexpr (GRAD) {
          const float dix = (v[c][1] - v[c][0]) * s + (v[c][3] - v[c][2]) * n;
          const float diy = (v[c][2] - v[c][0]) * e + (v[c][3] - v[c][1]) * w;
          const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
          ax += sg * dix;
          ay += sg * diy;
          dk[c][0] = dix * kx;
          dk[c][1] = diy * ky;
        }
      }
      msum += mo;
    }
    const int slot = i & (kRing - 1);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      this->xy[this->ring(slot, c, 0)] = x[c];
      this->xy[this->ring(slot, c, 1)] = y[c];
      if constexpr (GRAD) {
        this->pd[this->ring(slot, c, 0)] = dk[c][0];
        this->pd[this->ring(slot, c, 1)] = dk[c][1];
      }
    }
    if constexpr (GRAD) {
      const int o = own_row && this->lane_own ? 4 * (r * this->W + this->col) : kOffNone;
      this->st(ax * kx, o, 0);
      this->st(ay * ky, o, 4 * this->HW);
    }
    __syncthreads();
  }
};

template <bool BORDER, bool GRAD, int C>
struct Consumer : PairCommon<BORDER, GRAD, C> {
  Sums sm[3][C];
  float ca[3][C], cb[3][C], cg[3][C];
  float ssum;
  // row j of the strip (r = y0 - 2 + j), written by the producer one step
  // earlier; WIN: window row r - 2; BAS: pixel row r - 2's basis (0 / 1 / 2 =
  // run time); ends with the step's barrier
  template <int PH, int WIN, int BAS>
  __device__ __forceinline__ void step(int j) {
    constexpr int S0 = PH, S1 = (PH + 2) % 3, S2 = (PH + 1) % 3;
    const int r = this->y0 - 2 + j;
    const int slot = j & (kRing - 1), slot2 = (j - 2) & (kRing - 1);
    float x[C], y[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      x[c] = this->xy[this->ring(slot, c, 0)];
      y[c] = this->xy[this->ring(slot, c, 1)];
    }
#pragma unroll
    for (int c = 0; c < C; ++c)
      sm[S0][c] = Sums{hsum_next(x[c]), hsum_next(y[c]), hsum_next(fmaf(x[c], x[c], y[c] * y[c])),
                       hsum_next(x[c] * y[c])};
    const int q = r - 2;
    const bool qown = BAS == 2 ? j >= 4 : BAS == 1;
    float px[C], py[C], dx[C], dy[C];  // pixel row q: x, y and its gradient state
    if constexpr (GRAD) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        px[c] = this->xy[this->ring(slot2, c, 0)];
        py[c] = this->xy[this->ring(slot2, c, 1)];
        dx[c] = this->pd[this->ring(slot2, c, 0)];
        dy[c] = this->pd[this->ring(slot2, c, 1)];
      }
    }
    float bx = 0.f, by = 0.f;
    if (WIN == 2 ? j >= 2 : WIN == 1) {
      const bool wrow = WIN == 1 || (q >= 0 && q <= this->H - 3);
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float al = 0.f, be = 0.f, ga = 0.f;
        if (wrow) {
          const Sums& a2 = sm[S2][c];
          const Sums& a1 = sm[S1][c];
          const Sums& a0 = sm[S0][c];
          const Sums w{a2.x + a1.x + a0.x, a2.y + a1.y + a0.y, a2.q + a1.q + a0.q, a2.xy + a1.xy + a0.xy};
          const float s = ssim_sums<GRAD>(w, al, be, ga);
          ssum += qown && this->lane_own && this->wcol ? s : 0.f;
          if (!this->wcol) al = be = ga = 0.f;
        }
        if constexpr (GRAD) {
          ca[S0][c] = al;
          cb[S0][c] = be;
          cg[S0][c] = ga;
          if (qown) {
            const float ha = hsum_prev(ca[S2][c] + ca[S1][c] + al);
            const float hb = hsum_prev(cb[S2][c] + cb[S1][c] + be);
            const float hg = hsum_prev(cg[S2][c] + cg[S1][c] + ga);
            const float ds = fmaf(hg, py[c], fmaf(hb, px[c], ha));
            bx = fmaf(ds, dx[c], bx);
            by = fmaf(ds, dy[c], by);
          }
        }
      }
    }
    if constexpr (GRAD) {
      const int o = qown && this->lane_own ? 4 * (q * this->W + this->col) : kOffNone;
      this->st(bx, o, 8 * this->HW);
      this->st(by, o, 12 * this->HW);
    }
    __syncthreads();
  }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s);
  return v;
}

template <bool BORDER, bool GRAD, int C>
__global__ __launch_bounds__(256) void photo_pc_kernel(StripArgs a, float* __restrict__ partials) {
  __shared__ float lds[2][2][kRing * C * 2 * 64];  // [pair][x,y | gradient state]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pair = wave >> 1;
  const bool prod = (wave & 1) == 0;
  // workgroup -> (sample, strip row, pair of strip items sharing that row)
  const int npx = a.ndir == 2 ? a.nsx : (a.nsx + 1) / 2;  // workgroups per strip row
  const int g = xcd_remap(blockIdx.x, gridDim.x);
  const int gx = g % npx, rest = g / npx;
  const int sy = rest % a.nsy, b = rest / a.nsy;
  const int dirn = a.ndir == 2 ? pair : 0;
  const int sx = a.ndir == 2 ? gx : 2 * gx + pair;
  const bool valid = sx < a.nsx;  // wave-uniform
  const int H = a.H, W = a.W;
  const int y0 = (int)((long long)sy * H / a.nsy);
  const int rown = (int)((long long)(sy + 1) * H / a.nsy) - y0;
  const int nsteps = rown + 4;  // the same for both pairs (same strip row)
  if (!valid) {  // keep the barrier count of the other pair
    for (int i = 0; i <= nsteps; ++i) __syncthreads();
    return;
  }
  const PhotoDir dr = a.dir[dirn];
  const int HW = H * W;
  const size_t HWs = (size_t)HW;
  const int x0 = sx * kSO;
  auto init = [&](PairCommon<BORDER, GRAD, C>& p) {
    p.H = H;
    p.W = W;
    p.HW = HW;
    p.y0 = y0;
    p.rown = rown;
    p.lane = lane;
    p.col = x0 - 2 + lane;
    p.cc = min(max(p.col, 0), W - 1);
    p.col_in = p.col >= 0 && p.col < W;
    p.lane_own = lane >= 2 && lane < 2 + kSO && p.col < W;
    p.wcol = p.col >= 0 && p.col <= W - 3;
    p.xy = lds[pair][0];
    p.pd = lds[pair][1];
    if constexpr (GRAD) p.rbas = __builtin_amdgcn_make_buffer_rsrc(dr.basis + b * a.bbs, 0, 16 * HW, kRsrcWord3);
  };
  float* po = partials + 3 * (((size_t)dirn * a.B + b) * a.nsy * a.nsx + (size_t)sy * a.nsx + sx);
  if (prod) {
    Producer<BORDER, GRAD, C> P;
    init(P);
    const float* srcb = dr.src + (size_t)b * C * HWs;
#pragma unroll
    for (int c = 0; c < C; ++c)
      P.rs[c] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(srcb + c * HWs), 0, 4 * HW, kRsrcWord3);
    P.rtgt = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dr.tgt + (size_t)b * C * HWs), 0, 4 * C * HW,
                                               kRsrcWord3);
    P.rmask = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dr.mask + (size_t)b * HWs), 0, 4 * HW, kRsrcWord3);
    P.rflow = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dr.flow + b * a.fbs), 0, 8 * HW, kRsrcWord3);
    P.fxs = 2.0f / (float)(W - 1);
    P.fys = 2.0f / (float)(H - 1);
    P.l1 = P.msum = 0.f;
    P.template load_flow<0>(y0 - 2, true);
    P.template load_flow<1>(y0 - 1, true);
    P.template issue<0>(y0 - 2, true);
    P.template step<0, 0>(0, nsteps);
    P.template step<1, 0>(1, nsteps);
    int i = 2;
    for (; i + 3 <= rown + 2; i += 3) {
      P.template step<2, 1>(i, nsteps);
      P.template step<0, 1>(i + 1, nsteps);
      P.template step<1, 1>(i + 2, nsteps);
    }
    if (i < nsteps) P.template step<2, 2>(i, nsteps);
    if (i + 1 < nsteps) P.template step<0, 2>(i + 1, nsteps);
    if (i + 2 < nsteps) P.template step<1, 2>(i + 2, nsteps);
    if (i + 3 < nsteps) P.template step<2, 2>(i + 3, nsteps);
    __syncthreads();  // the consumer's last step
    const float l1 = wave_sum(P.l1), ms = wave_sum(P.msum);
    if (lane == 0) {
      po[0] = l1;
      po[2] = ms;
    }
  } else {
    Consumer<BORDER, GRAD, C> Q;
    init(Q);
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int c = 0; c < C; ++c) {
        Q.sm[k][c] = Sums{0.f, 0.f, 0.f, 0.f};
        Q.ca[k][c] = Q.cb[k][c] = Q.cg[k][c] = 0.f;
      }
    Q.ssum = 0.f;
    __syncthreads();  // the producer's first row
    Q.template step<0, 0, 0>(0);
    Q.template step<1, 0, 0>(1);
    Q.template step<2, 2, 0>(2);
    Q.template step<0, 2, 0>(3);
    int j = 4;
    for (; j + 3 <= rown + 2; j += 3) {
      Q.template step<1, 1, 1>(j);
      Q.template step<2, 1, 1>(j + 1);
      Q.template step<0, 1, 1>(j + 2);
    }
    if (j < nsteps) Q.template step<1, 2, 2>(j);
    if (j + 1 < nsteps) Q.template step<2, 2, 2>(j + 1);
    if (j + 2 < nsteps) Q.template step<0, 2, 2>(j + 2);
    if (j + 3 < nsteps) Q.template step<1, 2, 2>(j + 3);
    const float ss = wave_sum(Q.ssum);
    if (lane == 0) po[1] = ss;
  }
}

// Strip heights. Every wave streams R + 4 rows, so a launch takes about
// (R + 4) steps times the rounds of waves the chip holds: USF_PHOTO_WAVES per
// SIMD (the kernel's registers), 1024 SIMDs. A step of a wave alone on its
// SIMD takes ~0.76 of a step with a second wave beside it (measured,
// profiles/r03_photo_rows.json), so below one wave per SIMD fewer, taller
// strips do not help. The strips of a column are balanced (heights differ by
// at most one row); the cheapest count wins, ties to fewer strips.
constexpr int kSimds = 1024;  // 256 CUs x 4 SIMDs
constexpr int kMinStripRows = 4;  // the partials buffer holds ceil(H / 4) strips per column

struct StripPlan {
  int R, nsy;
};

StripPlan strip_plan(int B, int H, int W, int ndir) {
  static const int forced = [] {  // USF_PHOTO_ROWS=R: tuning override (tools/photoab.py)
    const char* v = getenv("USF_PHOTO_ROWS");
    return v ? atoi(v) : 0;
  }();
  if (forced >= kMinStripRows) return {forced, (H + forced - 1) / forced};
  const long long cols = (long long)ndir * B * ((W + kSO - 1) / kSO);
  StripPlan best{H, 1};
  double best_cost = -1.0;
  for (int nsy = 1; nsy <= (H + kMinStripRows - 1) / kMinStripRows; ++nsy) {
    const int R = (H + nsy - 1) / nsy;
    if ((H + R - 1) / R != nsy) continue;  // the same R as a smaller count
    const long long waves = cols * nsy;
    const long long rounds = (waves + (long long)USF_PHOTO_WAVES * kSimds - 1) / ((long long)USF_PHOTO_WAVES * kSimds);
    const double cost = (double)rounds * (R + 4) * (waves > kSimds ? 1.0 : 0.76);
    if (best_cost < 0 || cost < best_cost) {
      best_cost = cost;
      best = {R, nsy};
    }
  }
  return best;
}

template <bool BORDER, bool GRAD>
hipError_t strip_launch_c(const StripArgs& sa, int C, dim3 grid, float* partials, hipStream_t s) {
  if (C == 3)
    hipLaunchKernelGGL((photo_strip_kernel<BORDER, GRAD, 3>), grid, dim3(256), 0, s, sa, partials);
  else if (C == 2)
    hipLaunchKernelGGL((photo_strip_kernel<BORDER, GRAD, 2>), grid, dim3(256), 0, s, sa, partials);
  else
    hipLaunchKernelGGL((photo_strip_kernel<BORDER, GRAD, 1>), grid, dim3(256), 0, s, sa, partials);
  return hipGetLastError();
}
template <bool BORDER, bool GRAD>
hipError_t pc_launch_c(const StripArgs& sa, int C, dim3 grid, float* partials, hipStream_t s) {
  if (C == 3)
    hipLaunchKernelGGL((photo_pc_kernel<BORDER, GRAD, 3>), grid, dim3(256), 0, s, sa, partials);
  else if (C == 2)
    hipLaunchKernelGGL((photo_pc_kernel<BORDER, GRAD, 2>), grid, dim3(256), 0, s, sa, partials);
  else
    hipLaunchKernelGGL((photo_pc_kernel<BORDER, GRAD, 1>), grid, dim3(256), 0, s, sa, partials);
  return hipGetLastError();
}

hipError_t photo_strip_launch(const PhotoArgs& a, int ndir, int pad_mode, float* partials, float* out,
                              float w_l1, float w_ssim, hipStream_t s) {
  StripArgs sa{};
  sa.dir[0] = a.dir[0];
  sa.dir[1] = a.dir[1];
  sa.fbs = a.fbs;
  sa.bbs = a.bbs;
  sa.B = a.B;
  sa.H = a.H;
  sa.W = a.W;
  const StripPlan plan = strip_plan(a.B, a.H, a.W, ndir);
  sa.R = plan.R;
  sa.nsx = (a.W + kSO - 1) / kSO;
  sa.nsy = plan.nsy;
  sa.ndir = ndir;
  sa.nitems = ndir * a.B * sa.nsx * sa.nsy;
  const bool grad = a.dir[0].basis != nullptr;
  hipError_t e;
  if (variant_override(3) == 2) {  // one wave per strip
    const dim3 grid((unsigned)((sa.nitems + 3) / 4));
    if (pad_mode == 1)
      e = grad ? strip_launch_c<true, true>(sa, a.C, grid, partials, s) : strip_launch_c<true, false>(sa, a.C, grid, partials, s);
    else
      e = grad ? strip_launch_c<false, true>(sa, a.C, grid, partials, s) : strip_launch_c<false, false>(sa, a.C, grid, partials, s);
  } else {  // a producer / consumer pair of waves per strip, two strips per workgroup
    const int npx = ndir == 2 ? sa.nsx : (sa.nsx + 1) / 2;
    const dim3 grid((unsigned)(a.B * sa.nsy * npx));
    if (pad_mode == 1)
      e = grad ? pc_launch_c<true, true>(sa, a.C, grid, partials, s) : pc_launch_c<true, false>(sa, a.C, grid, partials, s);
    else
      e = grad ? pc_launch_c<false, true>(sa, a.C, grid, partials, s) : pc_launch_c<false, false>(sa, a.C, grid, partials, s);
  }
  if (e != hipSuccess) return e;
  const double n1 = (double)a.B * a.C * a.H * a.W;
  const double n2 = (a.H >= 3 && a.W >= 3) ? (double)a.B * a.C * (a.H - 2) * (a.W - 2) : 0.0;
  const double n3 = (double)a.B * a.H * a.W;
  hipLaunchKernelGGL(photo_final_kernel, dim3((unsigned)ndir), dim3(kFinNT), 0, s, partials,
                     a.B * sa.nsx * sa.nsy, out, n1, n2, n3, w_l1, w_ssim);
  return hipGetLastError();
}

hipError_t photo_launch(const PhotoArgs& a, int ndir, int pad_mode, float* partials, float* out,
                        float w_l1, float w_ssim, hipStream_t s) {
  if (variant_override(3) != 1) return photo_strip_launch(a, ndir, pad_mode, partials, out, w_l1, w_ssim, s);
  const int tiles_y = (a.H + kTH - 1) / kTH;
  const int ntiles = a.tiles_x * tiles_y;
  const dim3 grid((unsigned)ntiles, (unsigned)a.B, (unsigned)ndir);
  const bool grad = a.dir[0].basis != nullptr;
  if (pad_mode == 1) {
    if (grad)
      hipLaunchKernelGGL((photo_fwd_kernel<true, true>), grid, dim3(kNT), 0, s, a, partials);
    else
      hipLaunchKernelGGL((photo_fwd_kernel<true, false>), grid, dim3(kNT), 0, s, a, partials);
  } else {
    if (grad)
      hipLaunchKernelGGL((photo_fwd_kernel<false, true>), grid, dim3(kNT), 0, s, a, partials);
    else
      hipLaunchKernelGGL((photo_fwd_kernel<false, false>), grid, dim3(kNT), 0, s, a, partials);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const double n1 = (double)a.B * a.C * a.H * a.W;
  const double n2 = (a.H >= 3 && a.W >= 3) ? (double)a.B * a.C * (a.H - 2) * (a.W - 2) : 0.0;
  const double n3 = (double)a.B * a.H * a.W;
  hipLaunchKernelGGL(photo_final_kernel, dim3((unsigned)ndir), dim3(kFinNT), 0, s, partials,
                     ntiles * a.B, out, n1, n2, n3, w_l1, w_ssim);
  return hipGetLastError();
}

}  // namespace

int photo_partials(int B, int H, int W) {
  // either kernel, any strip height (the smallest R has the most strips)
  const int tile = 3 * B * ((H + kTH - 1) / kTH) * ((W + kTW - 1) / kTW);
  const int strip = 3 * B * ((H + kMinStripRows - 1) / kMinStripRows) * ((W + kSO - 1) / kSO);
  return std::max(tile, strip);
}

hipError_t photo_fwd_launch(const float* src, const float* tgt, const float* mask, const float* flow,
                            long long fbs, float* partials, float* out, float* basis, int B, int C,
                            int H, int W, int pad_mode, float w_l1, float w_ssim, hipStream_t s) {
  PhotoArgs a{};
  a.dir[0] = PhotoDir{src, tgt, mask, flow, basis};
  a.dir[1] = a.dir[0];
  a.fbs = fbs;
  a.bbs = 4LL * H * W;
  a.B = B; a.C = C; a.H = H; a.W = W;
  a.tiles_x = (W + kTW - 1) / kTW;
  return photo_launch(a, 1, pad_mode, partials, out, w_l1, w_ssim, s);
}

// both directions of a with_bk scale: dir 0 warps im2 by flow[:, 0:2] onto im1
// (mask1), dir 1 warps im1 by flow[:, 2:4] onto im2 (mask2) (flow_loss.py:130-131).
// basis: [B, 2, 4, H, W] (= [B,8,H,W]) or null.
hipError_t photo_pair_fwd_launch(const float* im1, const float* im2, const float* mask1,
                                 const float* mask2, const float* flow, long long fbs,
                                 float* partials, float* out, float* basis, int B, int C, int H,
                                 int W, int pad_mode, float w_l1, float w_ssim, hipStream_t s) {
  PhotoArgs a{};
  const size_t HW = (size_t)H * W;
  // basis block of (sample b, direction d) at basis + (2 b + d) * 4HW
  a.dir[0] = PhotoDir{im2, im1, mask1, flow, basis};
  a.dir[1] = PhotoDir{im1, im2, mask2, flow + 2 * HW, basis ? basis + 4 * HW : nullptr};
  a.fbs = fbs;
  a.bbs = 8LL * H * W;
  a.B = B; a.C = C; a.H = H; a.W = W;
  a.tiles_x = (W + kTW - 1) / kTW;
  return photo_launch(a, 2, pad_mode, partials, out, w_l1, w_ssim, s);
}

hipError_t photo_bwd_launch(const float* basis, const float* coef, const float* gloss, float* gflow,
                            int B, int H, int W, int ndir, hipStream_t s) {
  const int HW = H * W;
  const dim3 grid((unsigned)((HW + 1023) / 1024), (unsigned)B, (unsigned)ndir);
  hipLaunchKernelGGL(photo_bwd_kernel, grid, dim3(256), 0, s, basis, coef, gloss, gflow, HW, ndir);
  return hipGetLastError();
}

}  // namespace usf
