// Learned (convex) flow upsampling for gfx950 -- SURVEY.md §8f row 4, the
// RAFT-style upsampler of the reference's UpFlowNetwork (models/pwclite.py:
// 140-166; kitti_base.json / sintel_base.json set learned_upsampler = true, so
// it runs on every decoder level of both directions):
//
//   up_mask = 0.25 * convs(feat)                              (:163-165)
//   w       = softmax(up_mask.view(N, 1, 9, S, S, H, W), dim=2) (:151-153)
//   patches = unfold(S * flow, 3x3, padding=1)                (:155-156)
//   up[n, c, S y + i, S x + j] = sum_k w[n, k, i, j, y, x] * patches[n, c, k, y, x]
//                                                             (:158-160)
// with k = 3 ky + kx over the neighbour (y + ky - 1, x + kx - 1) (zero outside).
//
// torch runs this as ~8 passes over a [N,2,9,S,S,H,W] intermediate (softmax,
// unfold, broadcast multiply, sum, permute + reshape copy) forward and as many
// backward. Here the forward is one pass: read the mask (9 S^2 planes) and the
// flow once, write the S x S output blocks. Work item: 64 consecutive low-res
// pixels x S sub-rows; wave i of the workgroup owns sub-row i, so every mask
// load is one coalesced 256-byte wave access and every output write one
// contiguous 16-byte run per lane (S = 4). The 0.25 mask scale and the factor
// S on the flow are folded in (both powers of two: exact, as in torch).
//
// Backward, with G = grad_up and p = w:
//   dp_k = sum_c G_c v_ck;  grad_mask_k = mask_scale * p_k (dp_k - sum_l p_l dp_l)
//   grad_v_ck (per pixel) = sum_ij p_k G_c            -> scratch [N, 2*9, H, W]
//   grad_flow[c, q] = S * sum_k grad_v_ck(q - offset_k)  (unfold's backward,
//   a fixed-order 9-tap gather in a second kernel; no atomics, deterministic).
// The S sub-row waves of a workgroup combine their grad_v partials through LDS
// in sub-row order.
#include "usf_common.h"

namespace usf {
namespace {

template <int S>
struct ConvexTile {
  static constexpr int NT = 64 * S;
  static constexpr int SS = S * S;
};

// the 3x3 zero-padded neighbourhood of (y, x), times S: unfold(S * flow)
__device__ __forceinline__ void convex_patches(const float* __restrict__ fb, int y, int x, int H,
                                               int W, float s, float (&v)[2][9]) {
  const int HW = H * W;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      const int yy = y + ky - 1, xx = x + kx - 1;
      const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      const int o = ok ? yy * W + xx : 0;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float f = fb[c * HW + o];
        v[c][ky * 3 + kx] = ok ? s * f : 0.f;
      }
    }
  }
}

// softmax over the 9 neighbours (max-shifted, then * 1/sum as torch's CPU kernel)
__device__ __forceinline__ void softmax9(float (&m)[9]) {
  float mx = m[0];
#pragma unroll
  for (int k = 1; k < 9; ++k) mx = fmaxf(mx, m[k]);
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    m[k] = expf(m[k] - mx);
    sum += m[k];
  }
  const float inv = 1.f / sum;
#pragma unroll
  for (int k = 0; k < 9; ++k) m[k] *= inv;
}

template <int S>
__device__ __forceinline__ void store_run(float* __restrict__ dst, const float (&o)[S]) {
  if constexpr (S % 4 == 0) {
#pragma unroll
    for (int j = 0; j < S; j += 4)
      reinterpret_cast<float4*>(dst)[j / 4] = make_float4(o[j], o[j + 1], o[j + 2], o[j + 3]);
  } else if constexpr (S % 2 == 0) {
#pragma unroll
    for (int j = 0; j < S; j += 2) reinterpret_cast<float2*>(dst)[j / 2] = make_float2(o[j], o[j + 1]);
  } else {
#pragma unroll
    for (int j = 0; j < S; ++j) dst[j] = o[j];
  }
}

template <int S>
__device__ __forceinline__ void load_run(const float* __restrict__ src, float (&o)[S]) {
  if constexpr (S % 4 == 0) {
#pragma unroll
    for (int j = 0; j < S; j += 4) {
      const float4 t = reinterpret_cast<const float4*>(src)[j / 4];
      o[j] = t.x; o[j + 1] = t.y; o[j + 2] = t.z; o[j + 3] = t.w;
    }
  } else if constexpr (S % 2 == 0) {
#pragma unroll
    for (int j = 0; j < S; j += 2) {
      const float2 t = reinterpret_cast<const float2*>(src)[j / 2];
      o[j] = t.x; o[j + 1] = t.y;
    }
  } else {
#pragma unroll
    for (int j = 0; j < S; ++j) o[j] = src[j];
  }
}

template <int S>
__device__ __forceinline__ void convex_fwd_body(const float* __restrict__ flow, const float* __restrict__ mask,
                                                float* __restrict__ out, int H, int W, float mask_scale, int blk,
                                                int b) {
  constexpr int SS = S * S;
  const int lane = threadIdx.x & 63;
  const int i = threadIdx.x >> 6;  // sub-row of this wave
  const int HW = H * W;
  const int p = blk * 64 + lane;
  if (p >= HW) return;
  const int y = p / W, x = p - y * W;
  float v[2][9];
  convex_patches(flow + (size_t)b * 2 * HW, y, x, H, W, (float)S, v);
  const float* mb = mask + ((size_t)b * 9 * SS + i * S) * HW + p;
  float o[2][S];
#pragma unroll
  for (int j = 0; j < S; ++j) {
    float m[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) m[k] = mask_scale * mb[(size_t)(k * SS + j) * HW];
    softmax9(m);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
#pragma clang fp contract(off)
      float acc = m[0] * v[c][0];
#pragma unroll
      for (int k = 1; k < 9; ++k) acc += m[k] * v[c][k];
      o[c][j] = acc;
    }
  }
  const int Wo = S * W;
#pragma unroll
  for (int c = 0; c < 2; ++c)
    store_run<S>(out + ((size_t)(b * 2 + c) * S * H + S * y + i) * Wo + S * x, o[c]);
}

template <int S>
__global__ __launch_bounds__(64 * S) void convex_up_fwd_kernel(const float* __restrict__ flow,
                                                               const float* __restrict__ mask,
                                                               float* __restrict__ out, int H, int W,
                                                               float mask_scale) {
  convex_fwd_body<S>(flow, mask, out, H, W, mask_scale, blockIdx.x, blockIdx.y);
}

template <int S>
__device__ __forceinline__ void convex_bwd_body(const float* __restrict__ flow, const float* __restrict__ mask,
                                                const float* __restrict__ gout, float* __restrict__ gmask,
                                                float* __restrict__ gv, int H, int W, float mask_scale, int blk,
                                                int b) {
  constexpr int SS = S * S;
  __shared__ float red[S - 1][18][64];
  const int lane = threadIdx.x & 63;
  const int i = threadIdx.x >> 6;
  const int HW = H * W;
  const int p = blk * 64 + lane;
  const bool live = p < HW;  // no early return: the waves meet at a barrier
  const int pc = live ? p : HW - 1;
  const int y = pc / W, x = pc - y * W;
  float v[2][9];
  convex_patches(flow + (size_t)b * 2 * HW, y, x, H, W, (float)S, v);
  const int Wo = S * W;
  float g[2][S];
#pragma unroll
  for (int c = 0; c < 2; ++c) load_run<S>(gout + ((size_t)(b * 2 + c) * S * H + S * y + i) * Wo + S * x, g[c]);
  const float* mb = mask + ((size_t)b * 9 * SS + i * S) * HW + pc;
  float* gmb = gmask ? gmask + ((size_t)b * 9 * SS + i * S) * HW + pc : nullptr;
  float acc[2][9];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int k = 0; k < 9; ++k) acc[c][k] = 0.f;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    float m[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) m[k] = mask_scale * mb[(size_t)(k * SS + j) * HW];
    softmax9(m);
    if (gmb) {
      float dp[9];
      float dot = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        dp[k] = g[0][j] * v[0][k] + g[1][j] * v[1][k];
        dot += m[k] * dp[k];
      }
      if (live) {
#pragma unroll
        for (int k = 0; k < 9; ++k) gmb[(size_t)(k * SS + j) * HW] = mask_scale * (m[k] * (dp[k] - dot));
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int k = 0; k < 9; ++k) acc[c][k] = fmaf(m[k], g[c][j], acc[c][k]);
  }
  if (!gv) return;  // uniform over the launch
  if (i > 0) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int k = 0; k < 9; ++k) red[i - 1][c * 9 + k][lane] = acc[c][k];
  }
  __syncthreads();
  if (i == 0 && live) {
    // sub-rows combined in order 0, 1, ..., S-1; times S (d(S * flow) / d flow)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        float s = acc[c][k];
#pragma unroll
        for (int r = 0; r < S - 1; ++r) s += red[r][c * 9 + k][lane];
        gv[((size_t)b * 18 + c * 9 + k) * HW + p] = (float)S * s;
      }
  }
}

template <int S>
__global__ __launch_bounds__(64 * S) void convex_up_bwd_kernel(
    const float* __restrict__ flow, const float* __restrict__ mask, const float* __restrict__ gout,
    float* __restrict__ gmask, float* __restrict__ gv, int H, int W, float mask_scale) {
  convex_bwd_body<S>(flow, mask, gout, gmask, gv, H, W, mask_scale, blockIdx.x, blockIdx.y);
}

// grad_flow[b, c, q] = sum_k gv[b, c, k, q - offset_k]: unfold's backward (col2im)
// as a fixed-order gather over the 9 taps.
__device__ __forceinline__ void convex_gather_body(const float* __restrict__ gv, float* __restrict__ gflow, int B,
                                                   int H, int W, long long t) {
  const int HW = H * W;
  if (t >= (long long)B * 2 * HW) return;
  const int q = (int)(t % HW);
  const int bc = (int)(t / HW);  // b * 2 + c
  const int y = q / W, x = q - y * W;
  const float* src = gv + (size_t)bc * 9 * HW;
  float s = 0.f;
#pragma unroll
  for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      // pixel (y - ky + 1, x - kx + 1) saw q as its neighbour k = 3 ky + kx
      const int yy = y - ky + 1, xx = x - kx + 1;
      const bool ok = (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      const float g = src[(size_t)(ky * 3 + kx) * HW + (ok ? yy * W + xx : 0)];
      s += ok ? g : 0.f;
    }
  }
  gflow[t] = s;
}

__global__ __launch_bounds__(256) void convex_up_gather_kernel(const float* __restrict__ gv,
                                                               float* __restrict__ gflow, int B, int H,
                                                               int W) {
  convex_gather_body(gv, gflow, B, H, W, (long long)blockIdx.x * 256 + threadIdx.x);
}

// The decoder's output flows of every level in ONE launch each way
// (usf_convex_upsample_pyramid_{f32,bwd_f32}): level l owns blocks
// [start[l], start[l + 1]) of the grid, the largest level first. The levels'
// upsampled flows are independent of each other (only the loss reads them),
// so PWCLite defers them to the end of the decoder.
constexpr int kMaxLevels = 6;
struct ConvexPyr {
  const float* flow[kMaxLevels];
  const float* mask[kMaxLevels];
  const float* gout[kMaxLevels];
  float* out[kMaxLevels];    // forward output / backward grad_flow
  float* gmask[kMaxLevels];  // backward
  float* gv[kMaxLevels];     // backward scratch of the level
  int H[kMaxLevels], W[kMaxLevels];
  int start[kMaxLevels + 1];
  int n;
};

__device__ __forceinline__ int pyr_level(const ConvexPyr& m, int blk) {
  int l = 0;
#pragma unroll
  for (int k = 1; k < kMaxLevels; ++k) l += blk >= m.start[k];
  return l;
}

template <int S>
__global__ __launch_bounds__(64 * S) void convex_pyr_fwd_kernel(ConvexPyr m, float mask_scale) {
  const int l = pyr_level(m, blockIdx.x);
  convex_fwd_body<S>(m.flow[l], m.mask[l], m.out[l], m.H[l], m.W[l], mask_scale, blockIdx.x - m.start[l],
                     blockIdx.y);
}

template <int S>
__global__ __launch_bounds__(64 * S) void convex_pyr_bwd_kernel(ConvexPyr m, float mask_scale) {
  const int l = pyr_level(m, blockIdx.x);
  convex_bwd_body<S>(m.flow[l], m.mask[l], m.gout[l], m.gmask[l], m.out[l] ? m.gv[l] : nullptr, m.H[l], m.W[l],
                     mask_scale, blockIdx.x - m.start[l], blockIdx.y);
}

// start[] in 256-element blocks of each level's B * 2 * H * W outputs
__global__ __launch_bounds__(256) void convex_pyr_gather_kernel(ConvexPyr m, int B) {
  const int l = pyr_level(m, blockIdx.x);
  convex_gather_body(m.gv[l], m.out[l], B, m.H[l], m.W[l], (long long)(blockIdx.x - m.start[l]) * 256 + threadIdx.x);
}

template <int S>
hipError_t convex_fwd_s(const float* flow, const float* mask, float* out, int B, int H, int W,
                        float mask_scale, hipStream_t s) {
  const dim3 grid((unsigned)((H * W + 63) / 64), (unsigned)B);
  hipLaunchKernelGGL(convex_up_fwd_kernel<S>, grid, dim3(64 * S), 0, s, flow, mask, out, H, W,
                     mask_scale);
  return hipGetLastError();
}

template <int S>
hipError_t convex_bwd_s(const float* flow, const float* mask, const float* gout, float* gflow,
                        float* gmask, float* scratch, int B, int H, int W, float mask_scale,
                        hipStream_t s) {
  const dim3 grid((unsigned)((H * W + 63) / 64), (unsigned)B);
  hipLaunchKernelGGL(convex_up_bwd_kernel<S>, grid, dim3(64 * S), 0, s, flow, mask, gout, gmask,
                     gflow ? scratch : nullptr, H, W, mask_scale);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !gflow) return e;
  const long long n = (long long)B * 2 * H * W;
  hipLaunchKernelGGL(convex_up_gather_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     scratch, gflow, B, H, W);
  return hipGetLastError();
}

template <int S>
hipError_t convex_pyr_fwd_s(ConvexPyr m, int B, float mask_scale, hipStream_t s) {
  int total = 0;
  for (int l = 0; l < m.n; ++l) {
    m.start[l] = total;
    total += (m.H[l] * m.W[l] + 63) / 64;
  }
  for (int l = m.n; l <= kMaxLevels; ++l) m.start[l] = total;
  hipLaunchKernelGGL(convex_pyr_fwd_kernel<S>, dim3((unsigned)total, (unsigned)B), dim3(64 * S), 0, s, m,
                     mask_scale);
  return hipGetLastError();
}

template <int S>
hipError_t convex_pyr_bwd_s(ConvexPyr m, int B, float mask_scale, bool want_flow, hipStream_t s) {
  int total = 0;
  for (int l = 0; l < m.n; ++l) {
    m.start[l] = total;
    total += (m.H[l] * m.W[l] + 63) / 64;
  }
  for (int l = m.n; l <= kMaxLevels; ++l) m.start[l] = total;
  hipLaunchKernelGGL(convex_pyr_bwd_kernel<S>, dim3((unsigned)total, (unsigned)B), dim3(64 * S), 0, s, m,
                     mask_scale);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !want_flow) return e;
  total = 0;
  for (int l = 0; l < m.n; ++l) {
    m.start[l] = total;
    total += (int)((2LL * B * m.H[l] * m.W[l] + 255) / 256);
  }
  for (int l = m.n; l <= kMaxLevels; ++l) m.start[l] = total;
  hipLaunchKernelGGL(convex_pyr_gather_kernel, dim3((unsigned)total), dim3(256), 0, s, m, B);
  return hipGetLastError();
}

}  // namespace

bool convex_factor_ok(int factor) { return factor == 2 || factor == 4 || factor == 8; }

int convex_pyramid_max_levels() { return kMaxLevels; }

// largest level first (the launch order of the blocks)
hipError_t convex_pyr_fwd_launch(int n, const float* const* flow, const float* const* mask, float* const* out,
                                 const int* H, const int* W, int B, int factor, float mask_scale, hipStream_t s) {
  if (n < 1 || n > kMaxLevels || factor != 4) return hipErrorInvalidValue;
  ConvexPyr m{};
  m.n = n;
  for (int l = 0; l < n; ++l) {
    m.flow[l] = flow[l];
    m.mask[l] = mask[l];
    m.out[l] = out[l];
    m.H[l] = H[l];
    m.W[l] = W[l];
  }
  return convex_pyr_fwd_s<4>(m, B, mask_scale, s);
}

hipError_t convex_pyr_bwd_launch(int n, const float* const* flow, const float* const* mask,
                                 const float* const* gout, float* const* gflow, float* const* gmask, float* scratch,
                                 const int* H, const int* W, int B, int factor, float mask_scale, hipStream_t s) {
  if (n < 1 || n > kMaxLevels || factor != 4) return hipErrorInvalidValue;
  ConvexPyr m{};
  m.n = n;
  long long off = 0;
  for (int l = 0; l < n; ++l) {
    m.flow[l] = flow[l];
    m.mask[l] = mask[l];
    m.gout[l] = gout[l];
    m.out[l] = gflow ? gflow[l] : nullptr;
    m.gmask[l] = gmask ? gmask[l] : nullptr;
    m.gv[l] = gflow ? scratch + off : nullptr;
    m.H[l] = H[l];
    m.W[l] = W[l];
    off += convex_bwd_scratch(B, H[l], W[l]);
  }
  return convex_pyr_bwd_s<4>(m, B, mask_scale, gflow != nullptr, s);
}

long long convex_bwd_scratch(int B, int H, int W) { return 18LL * B * H * W; }

hipError_t convex_fwd_launch(const float* flow, const float* mask, float* out, int B, int H, int W,
                             int factor, float mask_scale, hipStream_t s) {
  switch (factor) {
    case 2: return convex_fwd_s<2>(flow, mask, out, B, H, W, mask_scale, s);
    case 4: return convex_fwd_s<4>(flow, mask, out, B, H, W, mask_scale, s);
    case 8: return convex_fwd_s<8>(flow, mask, out, B, H, W, mask_scale, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t convex_bwd_launch(const float* flow, const float* mask, const float* gout, float* gflow,
                             float* gmask, float* scratch, int B, int H, int W, int factor,
                             float mask_scale, hipStream_t s) {
  switch (factor) {
    case 2: return convex_bwd_s<2>(flow, mask, gout, gflow, gmask, scratch, B, H, W, mask_scale, s);
    case 4: return convex_bwd_s<4>(flow, mask, gout, gflow, gmask, scratch, B, H, W, mask_scale, s);
    case 8: return convex_bwd_s<8>(flow, mask, gout, gflow, gmask, scratch, B, H, W, mask_scale, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace usf
