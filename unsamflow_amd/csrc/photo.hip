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
// are known only after the global reduction. So ONE forward pass does all
// the work: it warps the source, sums the L1, SSIM and mask terms into
// per-strip partials and, when the flow needs a gradient, evaluates the closed
// form dS_q/dx_p = alpha_q + beta_q x_p + gamma_q y_p per window, box-sums it
// around every pixel and writes the 4-float basis {A_p, S'_p} (16 B/pixel). A
// one-block (per direction) kernel combines the partials in a fixed fp64 order
// into {L, c_l1, c_ssim}; the backward is then a dense 24 B/pixel pass,
// gflow = g (c_l1 A + c_ssim S'). Nothing is recomputed between forward and
// backward and no warped image, SSIM map or dL/drec reaches HBM.
// Deterministic: fixed-order sums, no atomics.
//
// The forward (photo_pc_kernel, below) streams column strips down the image,
// one staged row per step, split over a producer / consumer pair of waves.
// Two earlier forms -- a 32x16 workgroup tile with a 2-pixel halo ring, and
// one wave per strip -- were measured slower and removed.
#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "usf_common.h"
#include "warp_tap.h"

namespace usf {
namespace {

constexpr float kC1 = 0.01f * 0.01f;           // torch casts the python scalars to fp32
constexpr float kC2 = 0.03f * 0.03f;

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
  int B, C, H, W;
};


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
// A strip is 64 staged columns (lanes; the 60 middle ones are its own pixels)
// by R own rows, streamed down one staged row per step:
//   stage row r   -> lane l holds x = rec*m, y = tgt*m of column x0-2+l (C channels)
//   row sums      -> 3-column sums of x, y, x^2, y^2, xy by two DPP adds each
//                    (v_add_f32_dpp wave_shl:1: lane l reads lane l+1)
//   window r-2    -> the three latest row sums (kept in registers) give the 3x3
//                    window whose top-left row is r-2: SSIM, and with GRAD the
//                    coefficients alpha, beta, gamma of its pixel derivative
//   pixel row r-2 -> the 3x3 box sums of alpha/beta/gamma around each pixel
//                    (vertical in registers, horizontal by DPP wave_shr:1)
//                    complete its gradient basis.
// Each staged pixel is warped once; the halo is 2 rows above and below each
// strip (R chosen per shape, strip_plan) and 2 columns either side.
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


// ------------------------------------------------ producer / consumer pair --
// photo_pc_kernel: the strip stream above split over a PAIR of
// waves, so each holds half the state and twice as many waves share a SIMD.
// The producer stages rows (flow, tap, gathers, x = rec m, y = tgt m, the L1
// and mask sums, its own pixels' dI/dflow and the A basis) and hands each row's
// x, y and {dix kx, diy ky} to the consumer through an LDS ring; the consumer
// turns them into row sums, windows (SSIM and its coefficients) and the S
// basis, one row behind. One workgroup barrier per step: the producer writes
// row t while the consumer reads rows t-1 (new) and t-3 (the pixel row whose
// basis completes), so a ring of 4 rows suffices. With two pairs per
// workgroup (USF_PHOTO_PAIRS=2) both stream the same strip rows (the two
// directions, or two neighbouring strips), so they take the same number of
// steps and barriers.
constexpr int kRing = 4;
// (Round 5 built the pair without a workgroup barrier per step: two step
// counters in LDS and a six-row ring, so the producer could run three rows
// ahead. Full resolution with the gradient basis: 55.6-56.0 vs 55.4-56.3 us,
// smaller scales 0.3-0.6 us slower; forward only 35.3 vs 37.7 us.
// profiles/ab_r05/photo_flags.json; not kept: the step is not set by the
// barrier handshake.)
// producer/consumer pairs per workgroup. One: each pair's barrier waits for its
// own two waves only. Two pairs per 256-thread workgroup (round 3) kept both
// pairs in step; one pair measured 0.3-1.3 us faster at every loss scale
// (profiles/ab_r04/photo_pairs_per_wg.json; USF_PHOTO_PAIRS=2 for A/B).
// Occupancy target of the pair kernel, waves per SIMD (A/B knob). 4: 111
// VGPRs with the gradient basis at C = 3, no spills.
#ifndef USF_PHOTO_EU
#define USF_PHOTO_EU 4
#endif
#ifndef USF_PHOTO_PAIRS
#define USF_PHOTO_PAIRS 1
#endif
constexpr int kPairs = USF_PHOTO_PAIRS;

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

// The strip stream of one scale's workgroup blk of nblk (photo_pc_kernel: the
// whole grid; photo_pyr_kernel: that scale's range of a multi-scale grid).
template <bool BORDER, bool GRAD, int C>
__device__ __forceinline__ void pc_body(const StripArgs& a, float* __restrict__ partials, int blk, int nblk) {
  __shared__ float lds[kPairs][2][kRing * C * 2 * 64];  // [pair][x,y | gradient state]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pair = wave >> 1;
  const bool prod = (wave & 1) == 0;
  // workgroup -> (sample, strip row, pair of strip items sharing that row)
  const int npx = kPairs == 1 ? a.ndir * a.nsx : a.ndir == 2 ? a.nsx : (a.nsx + 1) / 2;  // workgroups per strip row
  const int g = xcd_remap(blk, nblk);
  const int gx = g % npx, rest = g / npx;
  const int sy = rest % a.nsy, b = rest / a.nsy;
  const int dirn = kPairs == 1 ? gx % a.ndir : a.ndir == 2 ? pair : 0;
  const int sx = kPairs == 1 ? gx / a.ndir : a.ndir == 2 ? gx : 2 * gx + pair;
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

template <bool BORDER, bool GRAD, int C>
__global__ __launch_bounds__(128 * kPairs) __attribute__((amdgpu_waves_per_eu(USF_PHOTO_EU))) void photo_pc_kernel(StripArgs a, float* __restrict__ partials) {
  pc_body<BORDER, GRAD, C>(a, partials, blockIdx.x, gridDim.x);
}

// The loss scales of a with_bk step in ONE launch (usf_photo_loss_pyramid_fwd_f32):
// scale s owns workgroups [start[s], start[s + 1]) -- the largest scale first,
// so the small scales' few strips fill the chip's tail instead of each paying a
// launch and a drain of their own.
constexpr int kMaxScales = 4;
struct StripPyr {
  StripArgs sc[kMaxScales];
  float* part[kMaxScales];
  int start[kMaxScales + 1];
};

template <bool BORDER, bool GRAD, int C>
__global__ __launch_bounds__(128 * kPairs) __attribute__((amdgpu_waves_per_eu(USF_PHOTO_EU))) void photo_pyr_kernel(StripPyr m) {
  const int blk = blockIdx.x;
  const int s = (blk >= m.start[1]) + (blk >= m.start[2]) + (blk >= m.start[3]);  // unused scales: start = total
  pc_body<BORDER, GRAD, C>(m.sc[s], m.part[s], blk - m.start[s], m.start[s + 1] - m.start[s]);
}

// One block per (direction, scale): photo_final_kernel's fixed-order reduction.
struct FinPyr {
  const float* part[kMaxScales];
  int nblk[kMaxScales];
  double n1[kMaxScales], n2[kMaxScales], n3[kMaxScales];
};
__global__ __launch_bounds__(kFinNT) void photo_pyr_final_kernel(FinPyr f, float* __restrict__ out, float w_l1,
                                                                 float w_ssim) {
  const int s = blockIdx.y;
  // the same code as the single-scale reduction, on this scale's partials (one
  // block per direction: blockIdx.x) and outputs out[6 s ..]
  __shared__ double red[3][kFinNT / 64];
  const int t = threadIdx.x, dirn = blockIdx.x, nblk = f.nblk[s];
  const float* p = f.part[s] + (size_t)3 * nblk * dirn;
  double a = 0, b = 0, c = 0;
  int i = t;
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
  for (int sh = 32; sh > 0; sh >>= 1) {
    a += __shfl_xor(a, sh);
    b += __shfl_xor(b, sh);
    c += __shfl_xor(c, sh);
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
    const double n1 = f.n1[s], n2 = f.n2[s], n3 = f.n3[s];
    const double den = s2 / n3 + 1e-6;
    const double l1 = n1 > 0 ? s0 / n1 : 0.0, ss = n2 > 0 ? s1 / n2 : 0.0;
    float* o = out + 6 * s + 3 * dirn;
    o[0] = (float)((w_l1 * l1 + w_ssim * ss) / den);
    o[1] = n1 > 0 ? (float)(w_l1 / (n1 * den)) : 0.f;
    o[2] = n2 > 0 ? (float)(w_ssim / (n2 * den)) : 0.f;
  }
}

// The backward of every scale in one launch: blockIdx.z = 2 s + direction.
struct BwdPyr {
  const float* basis[kMaxScales];
  float* gflow[kMaxScales];
  int HW[kMaxScales];
};
__global__ __launch_bounds__(256) void photo_pyr_bwd_kernel(BwdPyr m, const float* __restrict__ coef,
                                                            const float* __restrict__ gloss) {
  const int s = blockIdx.z >> 1, dirn = blockIdx.z & 1, b = blockIdx.y;
  const int HW = m.HW[s];
  const int i = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= HW) return;
  const float gl = gloss[2 * s + dirn];
  const float k1 = coef[6 * s + 3 * dirn + 1] * gl, k2 = coef[6 * s + 3 * dirn + 2] * gl;
  const float* a = m.basis[s] + ((size_t)b * 2 + dirn) * 4 * HW;
  float* o = m.gflow[s] + ((size_t)b * 2 + dirn) * 2 * HW;
  if ((HW & 3) == 0) {
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

// Strip heights. Every wave streams R + 4 rows, so a launch takes about
// (R + 4) steps times the rounds of strips the chip holds: USF_PHOTO_EU / 2
// wave pairs per SIMD (the pair kernel's registers), 1024 SIMDs. A step of a wave alone on its
// SIMD takes ~0.76 of a step with a second wave beside it (measured,
// profiles/r03_photo_rows.json), so below one wave per SIMD fewer, taller
// strips do not help. The strips of a column are balanced (heights differ by
// at most one row); the cheapest count wins, ties to fewer strips.
constexpr int kSimds = 1024;  // 256 CUs x 4 SIMDs
constexpr int kMinStripRows = 4;  // the partials buffer holds ceil(H / 4) strips per column
constexpr long long kPairSlots = (long long)USF_PHOTO_EU * kSimds / 2;  // resident strips

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
    const long long rounds = (waves + kPairSlots - 1) / kPairSlots;
    const double cost = (double)rounds * (R + 4) * (waves > kSimds ? 1.0 : 0.76);
    if (best_cost < 0 || cost < best_cost) {
      best_cost = cost;
      best = {R, nsy};
    }
  }
  return best;
}

template <bool BORDER, bool GRAD>
hipError_t pc_launch_c(const StripArgs& sa, int C, dim3 grid, float* partials, hipStream_t s) {
  if (C == 3)
    hipLaunchKernelGGL((photo_pc_kernel<BORDER, GRAD, 3>), grid, dim3(128 * kPairs), 0, s, sa, partials);
  else if (C == 2)
    hipLaunchKernelGGL((photo_pc_kernel<BORDER, GRAD, 2>), grid, dim3(128 * kPairs), 0, s, sa, partials);
  else
    hipLaunchKernelGGL((photo_pc_kernel<BORDER, GRAD, 1>), grid, dim3(128 * kPairs), 0, s, sa, partials);
  return hipGetLastError();
}

// StripArgs of one launch (one scale, ndir directions) and its workgroup count.
StripArgs strip_args(const PhotoArgs& a, int ndir, unsigned& nwg) {
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
  const int npx = kPairs == 1 ? ndir * sa.nsx : ndir == 2 ? sa.nsx : (sa.nsx + 1) / 2;
  nwg = (unsigned)(a.B * sa.nsy * npx);
  return sa;
}

template <bool BORDER, bool GRAD>
hipError_t pyr_launch_c(const StripPyr& m, int C, dim3 grid, hipStream_t s) {
  if (C == 3)
    hipLaunchKernelGGL((photo_pyr_kernel<BORDER, GRAD, 3>), grid, dim3(128 * kPairs), 0, s, m);
  else if (C == 2)
    hipLaunchKernelGGL((photo_pyr_kernel<BORDER, GRAD, 2>), grid, dim3(128 * kPairs), 0, s, m);
  else
    hipLaunchKernelGGL((photo_pyr_kernel<BORDER, GRAD, 1>), grid, dim3(128 * kPairs), 0, s, m);
  return hipGetLastError();
}

hipError_t photo_launch(const PhotoArgs& a, int ndir, int pad_mode, float* partials, float* out,
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
  // a producer / consumer pair of waves per strip, two strips per workgroup
  const int npx = kPairs == 1 ? ndir * sa.nsx : ndir == 2 ? sa.nsx : (sa.nsx + 1) / 2;
  const dim3 grid((unsigned)(a.B * sa.nsy * npx));
  hipError_t e;
  if (pad_mode == 1)
    e = grad ? pc_launch_c<true, true>(sa, a.C, grid, partials, s) : pc_launch_c<true, false>(sa, a.C, grid, partials, s);
  else
    e = grad ? pc_launch_c<false, true>(sa, a.C, grid, partials, s) : pc_launch_c<false, false>(sa, a.C, grid, partials, s);
  if (e != hipSuccess) return e;
  const double n1 = (double)a.B * a.C * a.H * a.W;
  const double n2 = (a.H >= 3 && a.W >= 3) ? (double)a.B * a.C * (a.H - 2) * (a.W - 2) : 0.0;
  const double n3 = (double)a.B * a.H * a.W;
  hipLaunchKernelGGL(photo_final_kernel, dim3((unsigned)ndir), dim3(kFinNT), 0, s, partials,
                     a.B * sa.nsx * sa.nsy, out, n1, n2, n3, w_l1, w_ssim);
  return hipGetLastError();
}

}  // namespace

int photo_partials(int B, int H, int W) {
  // any strip height (the smallest R has the most strips)
  return 3 * B * ((H + kMinStripRows - 1) / kMinStripRows) * ((W + kSO - 1) / kSO);
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
  return photo_launch(a, 2, pad_mode, partials, out, w_l1, w_ssim, s);
}

hipError_t photo_pyr_fwd_launch(int nscale, const float* const* im1, const float* const* im2,
                                const float* const* mask1, const float* const* mask2, const float* const* flow,
                                const long long* fbs, const int* H, const int* W, float* partials, float* out,
                                float* const* basis, int B, int C, int pad_mode, float w_l1, float w_ssim,
                                hipStream_t s) {
  if (nscale < 1 || nscale > kMaxScales) return hipErrorInvalidValue;
  StripPyr m{};
  FinPyr f{};
  bool grad = false;
  unsigned total = 0;
  long long poff = 0;
  for (int k = 0; k < nscale; ++k) {
    PhotoArgs a{};
    const size_t HW = (size_t)H[k] * W[k];
    float* bk = basis ? basis[k] : nullptr;
    a.dir[0] = PhotoDir{im2[k], im1[k], mask1[k], flow[k], bk};
    a.dir[1] = PhotoDir{im1[k], im2[k], mask2[k], flow[k] + 2 * HW, bk ? bk + 4 * HW : nullptr};
    a.fbs = fbs[k];
    a.bbs = 8LL * H[k] * W[k];
    a.B = B; a.C = C; a.H = H[k]; a.W = W[k];
    grad = grad || bk != nullptr;
    unsigned nwg = 0;
    m.sc[k] = strip_args(a, 2, nwg);
    m.part[k] = partials + poff;
    m.start[k] = (int)total;
    total += nwg;
    f.part[k] = partials + poff;
    f.nblk[k] = B * m.sc[k].nsx * m.sc[k].nsy;
    f.n1[k] = (double)B * C * H[k] * W[k];
    f.n2[k] = (H[k] >= 3 && W[k] >= 3) ? (double)B * C * (H[k] - 2) * (W[k] - 2) : 0.0;
    f.n3[k] = (double)B * H[k] * W[k];
    poff += 2LL * photo_partials(B, H[k], W[k]);
  }
  for (int k = nscale; k <= kMaxScales; ++k) m.start[k] = (int)total;
  for (int k = nscale; k < kMaxScales; ++k) m.sc[k] = m.sc[0];  // never selected (start[k] = total)
  hipError_t e;
  const dim3 grid(total);
  if (pad_mode == 1)
    e = grad ? pyr_launch_c<true, true>(m, C, grid, s) : pyr_launch_c<true, false>(m, C, grid, s);
  else
    e = grad ? pyr_launch_c<false, true>(m, C, grid, s) : pyr_launch_c<false, false>(m, C, grid, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(photo_pyr_final_kernel, dim3(2, (unsigned)nscale), dim3(kFinNT), 0, s, f, out, w_l1, w_ssim);
  return hipGetLastError();
}

hipError_t photo_pyr_bwd_launch(int nscale, const float* const* basis, const float* coef, const float* gloss,
                                float* const* gflow, const int* H, const int* W, int B, hipStream_t s) {
  if (nscale < 1 || nscale > kMaxScales) return hipErrorInvalidValue;
  BwdPyr m{};
  int hwmax = 0;
  for (int k = 0; k < nscale; ++k) {
    m.basis[k] = basis[k];
    m.gflow[k] = gflow[k];
    m.HW[k] = H[k] * W[k];
    hwmax = std::max(hwmax, m.HW[k]);
  }
  const dim3 grid((unsigned)((hwmax + 1023) / 1024), (unsigned)B, (unsigned)(2 * nscale));
  hipLaunchKernelGGL(photo_pyr_bwd_kernel, grid, dim3(256), 0, s, m, coef, gloss);
  return hipGetLastError();
}

hipError_t photo_bwd_launch(const float* basis, const float* coef, const float* gloss, float* gflow,
                            int B, int H, int W, int ndir, hipStream_t s) {
  const int HW = H * W;
  const dim3 grid((unsigned)((HW + 1023) / 1024), (unsigned)B, (unsigned)ndir);
  hipLaunchKernelGGL(photo_bwd_kernel, grid, dim3(256), 0, s, basis, coef, gloss, gflow, HW, ndir);
  return hipGetLastError();
}

}  // namespace usf
