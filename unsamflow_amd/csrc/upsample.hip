// Decoder flow upsampling for gfx950:
//   F.interpolate(flow * k, scale_factor=k, mode="bilinear", align_corners=True)
// (models/pwclite.py:299-301 between pyramid levels with k = 2, and the x4
// output flows). Semantics of ATen's upsample_bilinear2d with
// align_corners=True (third-party, torch 2.10): with the scale factor given,
// the source scale is still (in - 1) / (out - 1) in fp32; src = scale * dst;
// i0 = floor(src), i1 = i0 + (i0 < in - 1), l1 = src - i0, l0 = 1 - l1;
// out = l0_y (l0_x v00 + l1_x v01) + l1_y (l0_x v10 + l1_x v11) with v = k * flow.
// Forward: one lane per output element (coalesced writes, gathers from a
// 4x smaller input). Backward: deterministic gather form -- each input element
// sums the weights of the few output rows / columns whose taps reach it
// (ATen scatters with atomics), times k.
//
// Also the loss's image pyramid (flow_loss.py:128-129 of the reference's
// unFlowLoss: F.interpolate(im, (H >> s, W >> s), mode="area") per scale s):
// adaptive_avg_pool2d with exact 2^s blocks = the block's elements summed in
// row-major order, then / k / k (torch's CPU order, bit-exact; the divisions
// are by powers of two). One thread reads an 8x8 block once (16 float4 loads)
// and writes all three coarser scales.
#include <algorithm>
#include <cmath>

#include "interp_tap.h"
#include "usf_common.h"

namespace usf {
namespace {

__global__ __launch_bounds__(256) void upsample_fwd_kernel(const float* __restrict__ x,
                                                           float* __restrict__ out, long long planes,
                                                           int H, int W, int Ho, int Wo, float sy,
                                                           float sx, float k) {
#pragma clang fp contract(off)
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long n = planes * Ho * Wo;
  if (i >= n) return;
  const int ox = (int)(i % Wo);
  const int oy = (int)((i / Wo) % Ho);
  const long long pl = i / ((long long)Ho * Wo);
  const float* xp = x + pl * H * W;
  out[i] = up_bilinear(xp, W, lin_tap(oy, sy, H), lin_tap(ox, sx, W), k);
}

// total weight output index `o` (tap t) gives input index `in_i` along one axis
__device__ __forceinline__ float axis_weight(const Lin& t, int in_i) {
  float w = 0.f;
  if (t.i0 == in_i) w += t.l0;
  if (t.i1 == in_i) w += t.l1;
  return w;
}

// output rows whose taps can touch input row i: src in (i - 1, i + 1] (a
// generous window, filtered exactly by axis_weight)
__device__ __forceinline__ void tap_window(int i, float s, int out, int& o0, int& o1) {
  o0 = s > 0.f ? max(0, (int)floorf((i - 1) / s) - 1) : 0;
  o1 = s > 0.f ? min(out - 1, (int)ceilf((i + 1) / s) + 1) : out - 1;
}

// NWIN > 0: every window fits NWIN rows / columns (checked on the host), so
// the weights are computed once per axis and all loads are issued
// unconditionally at clamped offsets (zero weights outside the window: adding
// 0 * g leaves the sums unchanged). NWIN == 0: the generic loop.
// TWO: the output gradient is gout + gout2 (the decoder's upsampled flow gets
// one gradient from the warp and one from its other uses; summed here per
// element, the same number as a separate add)
template <int NWIN, bool TWO = false>
__global__ __launch_bounds__(256) void upsample_bwd_kernel(const float* __restrict__ gout,
                                                           float* __restrict__ gx, long long planes,
                                                           int H, int W, int Ho, int Wo, float sy,
                                                           float sx, float k,
                                                           const float* __restrict__ gout2 = nullptr) {
#pragma clang fp contract(off)
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long n = planes * H * W;
  if (i >= n) return;
  const int ix = (int)(i % W);
  const int iy = (int)((i / W) % H);
  const long long pl = i / ((long long)H * W);
  const float* gp = gout + pl * Ho * Wo;
  const float* gp2 = TWO ? gout2 + pl * Ho * Wo : gp;
  auto g = [&](int o) { return TWO ? gp[o] + gp2[o] : gp[o]; };
  int oy0, oy1, ox0, ox1;
  tap_window(iy, sy, Ho, oy0, oy1);
  tap_window(ix, sx, Wo, ox0, ox1);
  float acc = 0.f;
  if constexpr (NWIN > 0) {
    float wx[NWIN];
    int cx[NWIN];
#pragma unroll
    for (int j = 0; j < NWIN; ++j) {
      const int ox = ox0 + j;
      wx[j] = ox <= ox1 ? axis_weight(lin_tap(ox, sx, W), ix) : 0.f;
      cx[j] = min(ox, Wo - 1);
    }
#pragma unroll
    for (int r = 0; r < NWIN; ++r) {
      const int oy = oy0 + r;
      const float wy = oy <= oy1 ? axis_weight(lin_tap(oy, sy, H), iy) : 0.f;
      const int ro = min(oy, Ho - 1) * Wo;
      float row = 0.f;
#pragma unroll
      for (int j = 0; j < NWIN; ++j) row += wx[j] * g(ro + cx[j]);
      acc += wy * row;
    }
  } else {
    for (int oy = oy0; oy <= oy1; ++oy) {
      const float wy = axis_weight(lin_tap(oy, sy, H), iy);
      if (wy == 0.f) continue;
      float row = 0.f;
      for (int ox = ox0; ox <= ox1; ++ox) {
        const float wx = axis_weight(lin_tap(ox, sx, W), ix);
        if (wx != 0.f) row += wx * g(oy * Wo + ox);
      }
      acc += wy * row;
    }
  }
  gx[i] = acc * k;
}

// planes x (H/8) x (W/8) threads; H % 8 == 0, W % 8 == 0 (checked by the caller)
__global__ __launch_bounds__(256) void area_pyramid_kernel(const float* __restrict__ x,
                                                           float* __restrict__ o1,
                                                           float* __restrict__ o2,
                                                           float* __restrict__ o3, long long planes,
                                                           int H, int W) {
#pragma clang fp contract(off)
  const int bw = W >> 3, bh = H >> 3;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= planes * bh * bw) return;
  const int bx = (int)(i % bw);
  const int by = (int)((i / bw) % bh);
  const long long pl = i / ((long long)bh * bw);
  const float* xp = x + pl * H * W + (by * 8) * W + bx * 8;
  float v[8][8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const float4 a = reinterpret_cast<const float4*>(xp + r * W)[0];
    const float4 b = reinterpret_cast<const float4*>(xp + r * W)[1];
    v[r][0] = a.x; v[r][1] = a.y; v[r][2] = a.z; v[r][3] = a.w;
    v[r][4] = b.x; v[r][5] = b.y; v[r][6] = b.z; v[r][7] = b.w;
  }
  // block sum of a k x k block at (r0, c0), row-major sequential from 0 (torch's order)
  auto bsum = [&](int r0, int c0, int k) {
    float s = 0.f;
    for (int r = 0; r < k; ++r)
      for (int c = 0; c < k; ++c) s += v[r0 + r][c0 + c];
    return s;
  };
  const int W1 = W >> 1, W2 = W >> 2, W3 = W >> 3;
  float* p1 = o1 + pl * (H >> 1) * W1 + (by * 4) * W1 + bx * 4;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float q[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) q[c] = bsum(2 * r, 2 * c, 2) / 2.f / 2.f;
    reinterpret_cast<float4*>(p1 + r * W1)[0] = make_float4(q[0], q[1], q[2], q[3]);
  }
  float* p2 = o2 + pl * (H >> 2) * W2 + (by * 2) * W2 + bx * 2;
#pragma unroll
  for (int r = 0; r < 2; ++r)
    reinterpret_cast<float2*>(p2 + r * W2)[0] =
        make_float2(bsum(4 * r, 0, 4) / 4.f / 4.f, bsum(4 * r, 4, 4) / 4.f / 4.f);
  o3[pl * (H >> 3) * W3 + by * W3 + bx] = bsum(0, 0, 8) / 8.f / 8.f;
}

}  // namespace

hipError_t upsample_fwd_launch(const float* x, float* out, int B, int C, int H, int W, int k,
                               hipStream_t s) {
  const int Ho = H * k, Wo = W * k;
  const long long planes = (long long)B * C;
  const long long n = planes * Ho * Wo;
  hipLaunchKernelGGL(upsample_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, out,
                     planes, H, W, Ho, Wo, ac_scale(H, Ho), ac_scale(W, Wo), (float)k);
  return hipGetLastError();
}

// widest tap window over all input indices of one axis (host mirror of tap_window)
static int max_window(int in, int out) {
  const float s = ac_scale(in, out);
  if (!(s > 0.f)) return out;
  int m = 0;
  for (int i = 0; i < in; ++i) {
    const int o0 = std::max(0, (int)std::floor((i - 1) / s) - 1);
    const int o1 = std::min(out - 1, (int)std::ceil((i + 1) / s) + 1);
    m = std::max(m, o1 - o0 + 1);
  }
  return m;
}

hipError_t upsample_bwd_launch(const float* gout, float* gx, int B, int C, int H, int W, int k,
                               hipStream_t s, const float* gout2) {
  const int Ho = H * k, Wo = W * k;
  const long long planes = (long long)B * C;
  const long long n = planes * H * W;
  const dim3 grid((unsigned)((n + 255) / 256));
  const float sy = ac_scale(H, Ho), sx = ac_scale(W, Wo);
  const int win = std::max(max_window(H, Ho), max_window(W, Wo));
  if (win <= 8 && gout2)
    hipLaunchKernelGGL((upsample_bwd_kernel<8, true>), grid, dim3(256), 0, s, gout, gx, planes, H, W, Ho, Wo, sy,
                       sx, (float)k, gout2);
  else if (win <= 8)
    hipLaunchKernelGGL((upsample_bwd_kernel<8, false>), grid, dim3(256), 0, s, gout, gx, planes, H, W, Ho, Wo, sy,
                       sx, (float)k, nullptr);
  else if (gout2)
    hipLaunchKernelGGL((upsample_bwd_kernel<0, true>), grid, dim3(256), 0, s, gout, gx, planes, H, W, Ho, Wo, sy,
                       sx, (float)k, gout2);
  else
    hipLaunchKernelGGL((upsample_bwd_kernel<0, false>), grid, dim3(256), 0, s, gout, gx, planes, H, W, Ho, Wo, sy,
                       sx, (float)k, nullptr);
  return hipGetLastError();
}

hipError_t area_pyramid_launch(const float* x, float* o1, float* o2, float* o3, long long planes,
                               int H, int W, hipStream_t s) {
  const long long n = planes * (H / 8) * (W / 8);
  hipLaunchKernelGGL(area_pyramid_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, o1, o2,
                     o3, planes, H, W);
  return hipGetLastError();
}

}  // namespace usf
