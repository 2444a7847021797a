// Local correlation (cost volume) forward / backward for gfx950 (CDNA4).
//
// Semantics (fp32, NCHW, displacement radius d, K = 2d+1, KK = K*K):
//   out[b, dy*K+dx, y, x] = (1/C) sum_c x1[b,c,y,x] * X2(b,c, y+dy-d, x+dx-d)
//   gx1[b,c,y,x] = (1/C) sum_k g[b,k,y,x] * X2(b,c, y+dy_k-d, x+dx_k-d)
//   gx2[b,c,y,x] = (1/C) sum_k G(b,k, y-dy_k+d, x-dx_k+d) * X1(b,c, y-dy_k+d, x-dx_k+d)
// with X*, G = 0 outside [0,H)x[0,W). This is correlation_native.py:13-23
// (zero pad :16, 81 slice-products :18-21, channel mean :21, concat order :23)
// and the CUDA plugin's correlation_forward / correlation_backward_input{1,2}
// (correlation_cuda_kernel.cu:41-114, :116-207, :209-300) restricted to
// kernel_size=1, stride1=stride2=1, pad=d, which is what pwclite.py:208-215 uses.
//
// Design (MI355X-first, not a translation of the CUDA kernels):
//  * Forward: one workgroup = one output tile (TH rows x TW cols) x NDY
//    displacement rows. Wave w owns displacement row dyb+w; lane l owns PX
//    consecutive output pixels (row l/SEGX, segment l%SEGX). A channel stage of
//    CC channels of the x1 tile and the (TH+NDY-1) x (TW+2d) x2 halo is staged
//    in LDS (coalesced dword loads, zero fill = the zero padding), then each
//    lane keeps K*PX accumulators in VGPRs and reads one x1 segment and one
//    x2 window (PX+2d floats) per channel with ds_read_b128: K*PX FMAs per
//    (2*PX+2d) LDS floats. No cross-lane reduction (the channel sum is a
//    per-lane FMA chain), so no shared prod_sum/serial reduction as in the
//    reference (.cu:84-109).
//  * Backward: deterministic gather form, no atomics. gx1 and gx2 are the
//    same kernel (G2 template flag): the output channel is independent, so a
//    workgroup owns one tile x CC channels; wave w owns displacement rows
//    w, w+NW, ...; per displacement row the lane loads its K*PX slice of g
//    (coalesced along x) once and streams CC channels of the staged x halo
//    from LDS. The NW per-wave partial sums are combined through LDS (which
//    aliases the staging buffer) and written once, coalesced.
#include "usf_common.h"

namespace usf {
namespace {

// ---------------------------------------------------------------- forward --
template <int D, int PX, int SEGX, int NDY, int CC>
struct FwdCfg {
  static constexpr int K = 2 * D + 1;
  static constexpr int TW = SEGX * PX;          // tile width (pixels)
  static constexpr int TH = 64 / SEGX;          // tile height (rows)
  static constexpr int NT = 64 * NDY;           // threads per workgroup
  static constexpr int NDYG = (K + NDY - 1) / NDY;
  static constexpr int R2 = TH + NDY - 1;       // staged x2 rows
  static constexpr int C2 = TW + 2 * D;         // staged x2 cols
  static constexpr int WIN = round_up(PX + 2 * D, 4);
  static constexpr int XS = round_up(C2, 4) + 4;  // LDS row stride (floats)
  static constexpr int N1 = CC * TH * TW;         // staged x1 elements per stage
  static constexpr int N2 = CC * R2 * C2;         // staged x2 elements per stage
  static constexpr int L1 = (N1 + NT - 1) / NT;   // per-thread staging registers
  static constexpr int L2 = (N2 + NT - 1) / NT;
  static constexpr int S1N = N1;
  static constexpr int S2N = CC * R2 * XS + WIN;  // + tail pad for window over-read
  static_assert(PX % 4 == 0, "PX must be a multiple of 4 (ds_read_b128)");
  static_assert(64 % SEGX == 0, "SEGX must divide 64");
};

// Staging: every global load of a stage is issued before the first LDS write
// (unconditional loads from clamped addresses, zero selected afterwards —
// a per-element "load or 0" branch would make hipcc wait for each load in
// turn), and the next stage's loads are in flight while the current stage is
// computed (register double-buffering, one LDS image).
template <int D, int PX, int SEGX, int NDY, int CC>
__global__ __launch_bounds__(64 * NDY) void corr_fwd_kernel(const float* __restrict__ x1,
                                                            const float* __restrict__ x2,
                                                            float* __restrict__ out, int C,
                                                            int H, int W, int tiles_x) {
  using F = FwdCfg<D, PX, SEGX, NDY, CC>;
  constexpr int K = F::K, TW = F::TW, TH = F::TH, NT = F::NT, R2 = F::R2, C2 = F::C2;
  constexpr int WIN = F::WIN, XS = F::XS, N1 = F::N1, N2 = F::N2, L1 = F::L1, L2 = F::L2;
  __shared__ __attribute__((aligned(16))) float s1[F::S1N];
  __shared__ __attribute__((aligned(16))) float s2[F::S2N];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int dyb = blockIdx.x * NDY;
  const int tile = blockIdx.y;
  const int b = blockIdx.z;
  const int ty = tile / tiles_x;
  const int tx = tile - ty * tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  const int r = lane / SEGX, q = lane % SEGX;
  const int dy = dyb + wave;
  const bool active = dy < K;

  const int HW = H * W;
  const float* x1b = x1 + (size_t)b * C * HW;
  const float* x2b = x2 + (size_t)b * C * HW;
  const int gy2 = y0 + dyb - D;  // image row of staged x2 row 0
  const int gx2 = x0 - D;        // image col of staged x2 col 0

  float r1[L1], r2[L2];
  auto fetch = [&](int c0) {
#pragma unroll
    for (int k = 0; k < L1; ++k) {
      const int e = tid + k * NT;
      const int c = e / (TH * TW);
      const int rem = e - c * (TH * TW);
      const int rr = rem / TW, cc = rem - (rem / TW) * TW;
      const bool ok = e < N1 && c0 + c < C && y0 + rr < H && x0 + cc < W;
      const float v = x1b[ok ? (c0 + c) * HW + (y0 + rr) * W + x0 + cc : 0];
      r1[k] = ok ? v : 0.f;
    }
#pragma unroll
    for (int k = 0; k < L2; ++k) {
      const int e = tid + k * NT;
      const int c = e / (R2 * C2);
      const int rem = e - c * (R2 * C2);
      const int rr = rem / C2, cc = rem - (rem / C2) * C2;
      const int gy = gy2 + rr, gx = gx2 + cc;
      const bool ok = e < N2 && c0 + c < C && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
      const float v = x2b[ok ? (c0 + c) * HW + gy * W + gx : 0];
      r2[k] = ok ? v : 0.f;
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int k = 0; k < L1; ++k) {
      const int e = tid + k * NT;
      if (e < N1) s1[e] = r1[k];
    }
#pragma unroll
    for (int k = 0; k < L2; ++k) {
      const int e = tid + k * NT;
      const int c = e / (R2 * C2);
      const int rem = e - c * (R2 * C2);
      const int rr = rem / C2, cc = rem - (rem / C2) * C2;
      if (e < N2) s2[c * (R2 * XS) + rr * XS + cc] = r2[k];
    }
  };

  float acc[K][PX];
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int i = 0; i < PX; ++i) acc[j][i] = 0.f;

  fetch(0);
  stash();
  __syncthreads();
  for (int c0 = 0; c0 < C; c0 += CC) {
    const bool more = c0 + CC < C;
    if (more) fetch(c0 + CC);  // in flight during this stage's FMAs
    if (active) {
#pragma unroll 2
      for (int c = 0; c < CC; ++c) {
        float a[PX], w[WIN];
        const float4* p1 =
            reinterpret_cast<const float4*>(s1 + c * (TH * TW) + r * TW + q * PX);
#pragma unroll
        for (int i = 0; i < PX / 4; ++i) {
          const float4 t = p1[i];
          a[4 * i] = t.x; a[4 * i + 1] = t.y; a[4 * i + 2] = t.z; a[4 * i + 3] = t.w;
        }
        const float4* p2 =
            reinterpret_cast<const float4*>(s2 + c * (R2 * XS) + (r + wave) * XS + q * PX);
#pragma unroll
        for (int i = 0; i < WIN / 4; ++i) {
          const float4 t = p2[i];
          w[4 * i] = t.x; w[4 * i + 1] = t.y; w[4 * i + 2] = t.z; w[4 * i + 3] = t.w;
        }
#pragma unroll
        for (int dx = 0; dx < K; ++dx)
#pragma unroll
          for (int i = 0; i < PX; ++i) acc[dx][i] = fmaf(a[i], w[i + dx], acc[dx][i]);
      }
    }
    __syncthreads();
    if (more) {
      stash();
      __syncthreads();
    }
  }

  if (!active) return;
  const int y = y0 + r;
  if (y >= H) return;
  const int xb = x0 + q * PX;
  const float cf = (float)C;
  float* ob = out + ((size_t)b * K * K + (size_t)dy * K) * HW + y * W + xb;
  const bool vec = ((W & 3) == 0) && (xb + PX <= W);
#pragma unroll
  for (int dx = 0; dx < K; ++dx) {
    float* o = ob + dx * HW;
    if (vec) {
#pragma unroll
      for (int i = 0; i < PX / 4; ++i)
        reinterpret_cast<float4*>(o)[i] =
            make_float4(acc[dx][4 * i] / cf, acc[dx][4 * i + 1] / cf, acc[dx][4 * i + 2] / cf,
                        acc[dx][4 * i + 3] / cf);
    } else {
#pragma unroll
      for (int i = 0; i < PX; ++i)
        if (xb + i < W) o[i] = acc[dx][i] / cf;
    }
  }
}

template <int D, int PX, int SEGX, int NDY, int CC>
hipError_t launch_fwd(const float* x1, const float* x2, float* out, int B, int C, int H, int W,
                      hipStream_t s) {
  using F = FwdCfg<D, PX, SEGX, NDY, CC>;
  const int tiles_x = (W + F::TW - 1) / F::TW;
  const int tiles_y = (H + F::TH - 1) / F::TH;
  dim3 grid(F::NDYG, tiles_x * tiles_y, B);
  hipLaunchKernelGGL((corr_fwd_kernel<D, PX, SEGX, NDY, CC>), grid, dim3(F::NT), 0, s, x1, x2,
                     out, C, H, W, tiles_x);
  return hipGetLastError();
}

// Tuning hook: usf_set_variant(op, i) forces candidate i for d=4
// (tools/kbench.py sweeps them on the GPU); -1 = the shape heuristic below.

hipError_t fwd_candidate_d4(int i, const float* x1, const float* x2, float* out, int B, int C,
                            int H, int W, hipStream_t s) {
  switch (i) {
    case 0: return launch_fwd<4, 8, 8, 9, 4>(x1, x2, out, B, C, H, W, s);
    case 1: return launch_fwd<4, 4, 8, 9, 8>(x1, x2, out, B, C, H, W, s);
    case 2: return launch_fwd<4, 4, 8, 3, 8>(x1, x2, out, B, C, H, W, s);
    case 3: return launch_fwd<4, 8, 8, 3, 4>(x1, x2, out, B, C, H, W, s);
    case 4: return launch_fwd<4, 4, 16, 3, 8>(x1, x2, out, B, C, H, W, s);
    case 5: return launch_fwd<4, 4, 16, 9, 8>(x1, x2, out, B, C, H, W, s);
    case 6: return launch_fwd<4, 8, 8, 1, 8>(x1, x2, out, B, C, H, W, s);
    case 7: return launch_fwd<4, 4, 8, 1, 8>(x1, x2, out, B, C, H, W, s);
    case 8: return launch_fwd<4, 4, 4, 3, 8>(x1, x2, out, B, C, H, W, s);
    case 9: return launch_fwd<4, 4, 8, 3, 16>(x1, x2, out, B, C, H, W, s);
    default: return hipErrorInvalidValue;
  }
}
constexpr int kFwdCandidates = 10;

template <int D>
hipError_t fwd_dispatch(const float* x1, const float* x2, float* out, int B, int C, int H,
                        int W, hipStream_t s) {
  constexpr int K = 2 * D + 1;
  if (D == 4) {
    const int forced = variant_override(0);
    if (forced >= 0) return fwd_candidate_d4(forced, x1, x2, out, B, C, H, W, s);
  }
  // Prefer the big tile (8 px/lane, one workgroup covers every displacement
  // row: x1/x2 staged once); fall back to smaller tiles / split displacement
  // rows when that would leave most of the 256 CUs idle.
  const long big = (long)B * ((W + 63) / 64) * ((H + 7) / 8);
  if (big >= 256) return launch_fwd<D, 8, 8, K, 4>(x1, x2, out, B, C, H, W, s);
  const long mid = (long)B * ((W + 31) / 32) * ((H + 7) / 8);
  if (mid >= 256) return launch_fwd<D, 4, 8, K, 8>(x1, x2, out, B, C, H, W, s);
  return launch_fwd<D, 4, 8, 3, 8>(x1, x2, out, B, C, H, W, s);
}

// --------------------------------------------------------------- backward --
template <int D, int PX, int SEGX, int NW, int CC>
struct BwdCfg {
  static constexpr int K = 2 * D + 1;
  static constexpr int TW = SEGX * PX;
  static constexpr int TH = 64 / SEGX;
  static constexpr int NT = 64 * NW;
  static constexpr int R = TH + 2 * D;           // staged rows
  static constexpr int C2 = TW + 2 * D;          // staged cols
  static constexpr int WIN = round_up(PX + 2 * D, 4);
  static constexpr int XS = round_up(C2, 4) + 4;
  static constexpr int SN = CC * R * XS + WIN;   // staging image
  static constexpr int RN = NW * CC * TH * TW;   // per-wave partial sums (aliases staging)
  static constexpr int SMN = SN > RN ? SN : RN;
  static_assert(PX % 4 == 0, "PX must be a multiple of 4");
};

// G2 == false: gx1 from (g, x2).  G2 == true: gx2 from (g, x1).
template <int D, int PX, int SEGX, int NW, int CC, bool G2>
__global__ __launch_bounds__(64 * NW) void corr_bwd_kernel(const float* __restrict__ xs,
                                                           const float* __restrict__ g,
                                                           float* __restrict__ gx, int C, int H,
                                                           int W, int tiles_x) {
  using F = BwdCfg<D, PX, SEGX, NW, CC>;
  constexpr int K = F::K, TW = F::TW, TH = F::TH, NT = F::NT, R = F::R, C2 = F::C2;
  constexpr int WIN = F::WIN, XS = F::XS;
  __shared__ __attribute__((aligned(16))) float sm[F::SMN];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int tile = blockIdx.x;
  const int c0 = blockIdx.y * CC;
  const int b = blockIdx.z;
  const int ty = tile / tiles_x;
  const int tx = tile - ty * tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  const int r = lane / SEGX, q = lane % SEGX;
  const int y = y0 + r;
  const int xb = x0 + q * PX;

  const int HW = H * W;
  const float* xsb = xs + (size_t)b * C * HW;
  const float* gb = g + (size_t)b * K * K * HW;

  // stage xs rows [y0-D, y0+TH+D) x cols [x0-D, x0+TW+D) for CC channels:
  // all loads in flight first (clamped unconditional loads), then LDS writes
  {
    constexpr int N = CC * R * C2, L = (N + NT - 1) / NT;
    constexpr int CH = 16;  // loads in flight per batch (caps the staging registers)
#pragma unroll 1
    for (int k0 = 0; k0 < L; k0 += CH) {
      float v[CH];
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int e = tid + (k0 + j) * NT;
        const int c = e / (R * C2);
        const int rem = e - c * (R * C2);
        const int rr = rem / C2, cc = rem - (rem / C2) * C2;
        const int gy = y0 - D + rr, gxx = x0 - D + cc;
        const bool ok = e < N && c0 + c < C && (unsigned)gy < (unsigned)H && (unsigned)gxx < (unsigned)W;
        const float t = xsb[ok ? (c0 + c) * HW + gy * W + gxx : 0];
        v[j] = ok ? t : 0.f;
      }
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int e = tid + (k0 + j) * NT;
        const int c = e / (R * C2);
        const int rem = e - c * (R * C2);
        const int rr = rem / C2, cc = rem - (rem / C2) * C2;
        if (e < N) sm[c * (R * XS) + rr * XS + cc] = v[j];
      }
    }
  }
  __syncthreads();

  float acc[CC][PX];
#pragma unroll
  for (int c = 0; c < CC; ++c)
#pragma unroll
    for (int i = 0; i < PX; ++i) acc[c][i] = 0.f;

  for (int dy = wave; dy < K; dy += NW) {
    float gv[K][PX];
    if (!G2) {
      // g at the output pixels themselves: g[b, dy*K+dx, y, xb+i]
      const bool rowok = y < H;
#pragma unroll
      for (int dx = 0; dx < K; ++dx) {
        const float* gp = gb + (dy * K + dx) * HW + y * W + xb;
#pragma unroll
        for (int i = 0; i < PX; ++i) {
          const bool ok = rowok && xb + i < W;
          const float t = gp[ok ? i : 0 - (y * W + xb)];  // clamped to the plane start
          gv[dx][i] = ok ? t : 0.f;
        }
      }
    } else {
      // g at the source pixels: g[b, dy*K+dx, y-(dy-D), xb+i-(dx-D)]
      const int yy = y - dy + D;
      const bool rowok = (unsigned)yy < (unsigned)H;
#pragma unroll
      for (int dx = 0; dx < K; ++dx) {
        const int xx0 = xb - dx + D;
        const float* gp = gb + (dy * K + dx) * HW + yy * W + xx0;
#pragma unroll
        for (int i = 0; i < PX; ++i) {
          const bool ok = rowok && (unsigned)(xx0 + i) < (unsigned)W;
          const float t = gp[ok ? i : 0 - (yy * W + xx0)];  // clamped to the plane start
          gv[dx][i] = ok ? t : 0.f;
        }
      }
    }
    const int rs = G2 ? (2 * D - dy) : dy;
    const float* srow = sm + (r + rs) * XS + q * PX;
#pragma unroll
    for (int c = 0; c < CC; ++c) {
      float w[WIN];
      const float4* p = reinterpret_cast<const float4*>(srow + c * (R * XS));
#pragma unroll
      for (int i = 0; i < WIN / 4; ++i) {
        const float4 t = p[i];
        w[4 * i] = t.x; w[4 * i + 1] = t.y; w[4 * i + 2] = t.z; w[4 * i + 3] = t.w;
      }
#pragma unroll
      for (int dx = 0; dx < K; ++dx) {
        const int cs = G2 ? (2 * D - dx) : dx;
#pragma unroll
        for (int i = 0; i < PX; ++i) acc[c][i] = fmaf(gv[dx][i], w[i + cs], acc[c][i]);
      }
    }
  }
  __syncthreads();  // every wave is done reading the staging image

  float* rp = sm + wave * (CC * TH * TW) + r * TW + q * PX;
#pragma unroll
  for (int c = 0; c < CC; ++c)
#pragma unroll
    for (int i = 0; i < PX / 4; ++i)
      reinterpret_cast<float4*>(rp + c * (TH * TW))[i] =
          make_float4(acc[c][4 * i], acc[c][4 * i + 1], acc[c][4 * i + 2], acc[c][4 * i + 3]);
  __syncthreads();

  const float cf = (float)C;
  float* gxb = gx + (size_t)b * C * HW;
  for (int o = tid; o < CC * TH * TW; o += NT) {
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) sum += sm[w * (CC * TH * TW) + o];
    const int c = o / (TH * TW);
    const int pix = o - c * (TH * TW);
    const int yy = y0 + pix / TW;
    const int xx = x0 + pix % TW;
    if (c0 + c < C && yy < H && xx < W) gxb[(c0 + c) * HW + yy * W + xx] = sum / cf;
  }
}

template <int D, bool G2, int PX = 4, int SEGX = 8, int NW = 3, int CC = 16>
hipError_t launch_bwd(const float* xs, const float* g, float* gx, int B, int C, int H, int W,
                      hipStream_t s) {
  using F = BwdCfg<D, PX, SEGX, NW, CC>;
  const int tiles_x = (W + F::TW - 1) / F::TW;
  const int tiles_y = (H + F::TH - 1) / F::TH;
  dim3 grid(tiles_x * tiles_y, (C + CC - 1) / CC, B);
  hipLaunchKernelGGL((corr_bwd_kernel<D, PX, SEGX, NW, CC, G2>), grid, dim3(F::NT), 0, s, xs, g,
                     gx, C, H, W, tiles_x);
  return hipGetLastError();
}

template <bool G2>
hipError_t bwd_candidate_d4(int i, const float* xs, const float* g, float* gx, int B, int C, int H,
                            int W, hipStream_t s) {
  switch (i) {
    case 0: return launch_bwd<4, G2, 4, 8, 3, 16>(xs, g, gx, B, C, H, W, s);
    case 1: return launch_bwd<4, G2, 4, 8, 3, 8>(xs, g, gx, B, C, H, W, s);
    case 2: return launch_bwd<4, G2, 4, 16, 3, 16>(xs, g, gx, B, C, H, W, s);
    case 3: return launch_bwd<4, G2, 4, 4, 3, 16>(xs, g, gx, B, C, H, W, s);
    case 4: return launch_bwd<4, G2, 4, 8, 9, 8>(xs, g, gx, B, C, H, W, s);
    case 5: return launch_bwd<4, G2, 4, 8, 1, 16>(xs, g, gx, B, C, H, W, s);
    default: return hipErrorInvalidValue;
  }
}
constexpr int kBwdCandidates = 6;

template <int D>
hipError_t bwd_dispatch(const float* x1, const float* x2, const float* g, float* gx1, float* gx2,
                        int B, int C, int H, int W, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (D == 4) {
    const int forced = variant_override(1);
    if (forced >= 0) {
      if (gx1) e = bwd_candidate_d4<false>(forced, x2, g, gx1, B, C, H, W, s);
      if (e == hipSuccess && gx2) e = bwd_candidate_d4<true>(forced, x1, g, gx2, B, C, H, W, s);
      return e;
    }
  }
  if (gx1) e = launch_bwd<D, false>(x2, g, gx1, B, C, H, W, s);
  if (e == hipSuccess && gx2) e = launch_bwd<D, true>(x1, g, gx2, B, C, H, W, s);
  return e;
}

}  // namespace

static int g_variant[2] = {-1, -1};
int variant_override(int op) { return __atomic_load_n(&g_variant[op], __ATOMIC_RELAXED); }
int variant_count(int op) { return op == 0 ? kFwdCandidates : kBwdCandidates; }
void set_variant_override(int op, int index) { __atomic_store_n(&g_variant[op], index, __ATOMIC_RELAXED); }

hipError_t corr_fwd_launch(const float* x1, const float* x2, float* out, int B, int C, int H,
                           int W, int d, hipStream_t s) {
  switch (d) {
    case 1: return fwd_dispatch<1>(x1, x2, out, B, C, H, W, s);
    case 2: return fwd_dispatch<2>(x1, x2, out, B, C, H, W, s);
    case 3: return fwd_dispatch<3>(x1, x2, out, B, C, H, W, s);
    case 4: return fwd_dispatch<4>(x1, x2, out, B, C, H, W, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t corr_bwd_launch(const float* x1, const float* x2, const float* gout, float* gx1,
                           float* gx2, int B, int C, int H, int W, int d, hipStream_t s) {
  switch (d) {
    case 1: return bwd_dispatch<1>(x1, x2, gout, gx1, gx2, B, C, H, W, s);
    case 2: return bwd_dispatch<2>(x1, x2, gout, gx1, gx2, B, C, H, W, s);
    case 3: return bwd_dispatch<3>(x1, x2, gout, gx1, gx2, B, C, H, W, s);
    case 4: return bwd_dispatch<4>(x1, x2, gout, gx1, gx2, B, C, H, W, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace usf
