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
//  * Staging is LDS-DMA (buffer_load_dword ... lds): a stage of CC channels is
//    copied HBM->LDS by one wave-instruction per 64 consecutive elements of a
//    channel's tile image, with no VGPR round trip and no per-element index
//    math. Each chunk gets a buffer descriptor covering exactly one channel
//    plane, so the zero padding outside the image (and the channel tail) is
//    the hardware's out-of-range zero fill: off-image lanes carry an offset
//    past num_records, channels >= C carry num_records = 0. The per-lane
//    offsets are stage-invariant and computed once. Two LDS images: the DMA
//    of stage s+1 is in flight while stage s is computed.
//  * Forward: one workgroup = one output tile (TH rows x TW cols) x NDY
//    displacement rows; wave w owns displacement row dyb+w, lane l owns PX
//    consecutive pixels (row l/SEGX, segment l%SEGX) and keeps K*PX
//    accumulators in VGPRs; per channel it reads an x1 segment and a PX+2d
//    x2 window with ds_read_b128 (K*PX FMAs per 2*PX+2d LDS floats). The
//    channel sum is a per-lane FMA chain: no cross-lane reduction.
//  * Backward: deterministic gather form, no atomics. gx1 and gx2 are the same
//    kernel (G2 flag, mirrored indices). A workgroup owns one tile x a channel
//    group; wave w owns DYW displacement rows and keeps its DYW*K*PX slice of g
//    in VGPRs for the whole channel loop (g read once per workgroup); per
//    channel the DYW partial rows are summed in registers, the NW per-wave
//    partials are added through LDS in a fixed order and written once.
#include <cstdint>

#include "usf_common.h"

namespace usf {
namespace {

// gfx950 buffer descriptor word 3 for raw 32-bit loads (MI355X guide T8).
constexpr int kRsrcFlags = 0x00020000;
// a byte offset past any plane's num_records (planes are < 2 GiB, checked in capi.cpp)
constexpr int kOffImage = 0x7FFFFFF0;

using lds_void_t = __attribute__((address_space(3))) void;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const float* plane, bool valid,
                                                           int plane_bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(plane), (short)0,
                                           valid ? plane_bytes : 0, kRsrcFlags);
}

// One wave-instruction: 64 consecutive floats of LDS at `dst` (wave-uniform)
// from per-lane byte offsets `voff` of the plane described by `rsrc`.
__device__ __forceinline__ void dma64(__amdgpu_buffer_rsrc_t rsrc, float* dst, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_t*)dst, 4, voff, 0, 0, 0);
}

__device__ __forceinline__ void dma_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// LDS read of N consecutive floats with ds_read_b64 (B64) or ds_read_b128.
template <bool B64, int N>
__device__ __forceinline__ void lds_read(const float* p, float (&v)[N]) {
  if constexpr (B64) {
    static_assert(N % 2 == 0, "b64 reads");
#pragma unroll
    for (int i = 0; i < N / 2; ++i) {
      const float2 t = reinterpret_cast<const float2*>(p)[i];
      v[2 * i] = t.x; v[2 * i + 1] = t.y;
    }
  } else {
    static_assert(N % 4 == 0, "b128 reads");
#pragma unroll
    for (int i = 0; i < N / 4; ++i) {
      const float4 t = reinterpret_cast<const float4*>(p)[i];
      v[4 * i] = t.x; v[4 * i + 1] = t.y; v[4 * i + 2] = t.z; v[4 * i + 3] = t.w;
    }
  }
}

using f2v = __attribute__((ext_vector_type(2))) float;

// LDS byte address of a pointer into __shared__ memory.
__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)p;
}

// x1 segment (8 floats at pa) + x2 window (16 floats at pw) with twelve
// ds_read_b64 in ONE asm statement that also waits for them: hipcc would
// otherwise fuse adjacent b64 reads into ds_read2_b64, whose 16-lane groups
// bank mod 32 and conflict on the stride-74 image (measured with
// tools/probes/lds_probe.hip + SQ_LDS_BANK_CONFLICT).
__device__ __forceinline__ void lds_read_px8(const float* pa, const float* pw, float (&a)[8],
                                             float (&w)[16]) {
  f2v a0, a1, a2, a3, w0, w1, w2, w3, w4, w5, w6, w7;
  asm volatile(
      "ds_read_b64 %0, %12\n\t"
      "ds_read_b64 %1, %12 offset:8\n\t"
      "ds_read_b64 %2, %12 offset:16\n\t"
      "ds_read_b64 %3, %12 offset:24\n\t"
      "ds_read_b64 %4, %13\n\t"
      "ds_read_b64 %5, %13 offset:8\n\t"
      "ds_read_b64 %6, %13 offset:16\n\t"
      "ds_read_b64 %7, %13 offset:24\n\t"
      "ds_read_b64 %8, %13 offset:32\n\t"
      "ds_read_b64 %9, %13 offset:40\n\t"
      "ds_read_b64 %10, %13 offset:48\n\t"
      "ds_read_b64 %11, %13 offset:56\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(a0), "=&v"(a1), "=&v"(a2), "=&v"(a3), "=&v"(w0), "=&v"(w1), "=&v"(w2), "=&v"(w3),
        "=&v"(w4), "=&v"(w5), "=&v"(w6), "=&v"(w7)
      : "v"(lds_addr(pa)), "v"(lds_addr(pw))
      : "memory");
  a[0] = a0.x; a[1] = a0.y; a[2] = a1.x; a[3] = a1.y; a[4] = a2.x; a[5] = a2.y; a[6] = a3.x; a[7] = a3.y;
  w[0] = w0.x; w[1] = w0.y; w[2] = w1.x; w[3] = w1.y; w[4] = w2.x; w[5] = w2.y; w[6] = w3.x; w[7] = w3.y;
  w[8] = w4.x; w[9] = w4.y; w[10] = w5.x; w[11] = w5.y; w[12] = w6.x; w[13] = w6.y; w[14] = w7.x; w[15] = w7.y;
}

// LDS layout policy, chosen with a model of gfx950's ds_read lane groups
// (MI355X_MICROARCH.md §LDS; tools/lds_banks.py) so every window/segment read
// is bank-conflict free:
//  * PX == 8: lanes row-major (r = l / SEGX), ds_read_b64, row stride = TW+10
//    floats (74 at TW=64): each 32-lane group of a b64 read covers all 64
//    banks once.
//  * PX == 4: lanes column-major (q = l / TH, r = l % TH), ds_read_b128, row
//    stride = round_up(TW+2d, 16) + 8 (48 at TW=32).
// Pad columns of an LDS row are DMA'd as out-of-range zeros.
template <int PX, int SEGX, int D>
struct Layout {
  static constexpr int TW = SEGX * PX, TH = 64 / SEGX;
  static constexpr bool B64 = PX == 8;
  static constexpr bool COLMAJOR = PX != 8;
  static constexpr int S = B64 ? TW + 10 : round_up(TW + 2 * D, 16) + 8;
  static_assert(S >= TW + 2 * D, "row stride must hold the halo row");
  __device__ static int row(int lane) { return COLMAJOR ? lane % TH : lane / SEGX; }
  __device__ static int seg(int lane) { return COLMAJOR ? lane / TH : lane % SEGX; }
};

// ---------------------------------------------------------------- forward --
template <int D, int PX, int SEGX, int NDY, int CC>
struct FwdCfg {
  static constexpr int K = 2 * D + 1;
  static constexpr int TW = SEGX * PX;              // tile width (pixels)
  static constexpr int TH = 64 / SEGX;              // tile height (rows)
  static constexpr int NT = 64 * NDY;               // threads per workgroup
  static constexpr int NDYG = (K + NDY - 1) / NDY;  // workgroups per tile
  using L = Layout<PX, SEGX, D>;
  static constexpr int R2 = TH + NDY - 1;           // staged x2 rows
  static constexpr int C2 = TW + 2 * D;             // staged x2 cols
  static constexpr int S = L::S;                    // LDS row stride (x1 and x2 images)
  static constexpr int P1 = round_up(TH * S, 64);   // x1 plane image (floats)
  static constexpr int P2 = round_up(R2 * S, 64);   // x2 plane image
  static constexpr int CH1 = P1 / 64, CH2 = P2 / 64;  // 64-float chunks per plane
  static constexpr int J1 = (CH1 + NDY - 1) / NDY;  // chunks per wave per plane
  static constexpr int J2 = (CH2 + NDY - 1) / NDY;
  static constexpr int WIN = round_up(PX + 2 * D, 4);
  static constexpr int STAGE = CC * (P1 + P2);
  static constexpr int LDSN = 2 * STAGE + WIN;      // two images + window over-read pad
  static_assert(PX % 4 == 0, "PX must be a multiple of 4 (ds_read_b128)");
  static_assert(64 % SEGX == 0, "SEGX must divide 64");
};

template <int D, int PX, int SEGX, int NDY, int CC>
__global__ __launch_bounds__(64 * NDY) void corr_fwd_kernel(const float* __restrict__ x1,
                                                            const float* __restrict__ x2,
                                                            float* __restrict__ out, int C,
                                                            int H, int W, int tiles_x) {
  using F = FwdCfg<D, PX, SEGX, NDY, CC>;
  constexpr int K = F::K, TW = F::TW, TH = F::TH, C2 = F::C2, S = F::S, P1 = F::P1, P2 = F::P2;
  constexpr int WIN = F::WIN, STAGE = F::STAGE;
  constexpr bool B64 = F::L::B64;
  __shared__ __attribute__((aligned(16))) float sm[F::LDSN];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int dyb = blockIdx.x * NDY;
  const int tile = blockIdx.y;
  const int b = blockIdx.z;
  const int ty = tile / tiles_x;
  const int tx = tile - ty * tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  const int r = F::L::row(lane), q = F::L::seg(lane);
  const int dy = dyb + wave;
  const bool active = dy < K;

  const int HW = H * W;
  const float* x1b = x1 + (size_t)b * C * HW;
  const float* x2b = x2 + (size_t)b * C * HW;

  // stage-invariant per-lane byte offsets of this wave's chunks (row stride S;
  // pad columns and off-image pixels read as zeros)
  int vo1[F::J1], vo2[F::J2];
#pragma unroll
  for (int t = 0; t < F::J1; ++t) {
    const int e = (wave + t * NDY) * 64 + lane;
    const int rr = e / S, cc = e % S;
    const int gy = y0 + rr, gx = x0 + cc;
    const bool ok = rr < TH && cc < TW && gy < H && gx < W;
    vo1[t] = ok ? (gy * W + gx) * 4 : kOffImage;
  }
#pragma unroll
  for (int t = 0; t < F::J2; ++t) {
    const int e = (wave + t * NDY) * 64 + lane;
    const int rr = e / S, cc = e % S;
    const int gy = y0 + dyb - D + rr, gx = x0 - D + cc;
    const bool ok = rr < F::R2 && cc < C2 && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
    vo2[t] = ok ? (gy * W + gx) * 4 : kOffImage;
  }
  auto dma_stage = [&](int c0, float* img) {
#pragma unroll
    for (int c = 0; c < CC; ++c) {
      const bool cv = c0 + c < C;
      const auto r1 = plane_rsrc(x1b + (size_t)(c0 + c) * HW, cv, HW * 4);
      const auto r2 = plane_rsrc(x2b + (size_t)(c0 + c) * HW, cv, HW * 4);
#pragma unroll
      for (int t = 0; t < F::J1; ++t)
        if (wave + t * NDY < F::CH1) dma64(r1, img + c * P1 + (wave + t * NDY) * 64, vo1[t]);
#pragma unroll
      for (int t = 0; t < F::J2; ++t)
        if (wave + t * NDY < F::CH2)
          dma64(r2, img + CC * P1 + c * P2 + (wave + t * NDY) * 64, vo2[t]);
    }
  };

  float acc[K][PX];
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int i = 0; i < PX; ++i) acc[j][i] = 0.f;

  dma_stage(0, sm);
  dma_wait_all();
  __syncthreads();
  int st = 0;
  for (int c0 = 0; c0 < C; c0 += CC, ++st) {
    const float* cur = sm + (st & 1) * STAGE;
    if (c0 + CC < C) dma_stage(c0 + CC, sm + ((st + 1) & 1) * STAGE);  // in flight during FMAs
    if (active) {
      const float* p1 = cur + r * S + q * PX;
      const float* p2 = cur + CC * P1 + (r + wave) * S + q * PX;
#pragma unroll 2
      for (int c = 0; c < CC; ++c) {
        float a[PX], w[WIN];
        if constexpr (B64 && PX == 8 && WIN == 16) {
          lds_read_px8(p1 + c * P1, p2 + c * P2, a, w);
        } else {
          lds_read<B64>(p1 + c * P1, a);
          lds_read<B64>(p2 + c * P2, w);
        }
#pragma unroll
        for (int dx = 0; dx < K; ++dx)
#pragma unroll
          for (int i = 0; i < PX; ++i) acc[dx][i] = fmaf(a[i], w[i + dx], acc[dx][i]);
      }
    }
    dma_wait_all();
    __syncthreads();
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

// Tuning hook: usf_set_variant(0, i) forces candidate i for d=4
// (tools/kbench.py sweeps them on the GPU); -1 = the shape heuristic below.
hipError_t fwd_candidate_d4(int i, const float* x1, const float* x2, float* out, int B, int C,
                            int H, int W, hipStream_t s) {
  switch (i) {
    case 0: return launch_fwd<4, 8, 8, 9, 8>(x1, x2, out, B, C, H, W, s);
    case 1: return launch_fwd<4, 8, 8, 9, 4>(x1, x2, out, B, C, H, W, s);
    case 2: return launch_fwd<4, 4, 8, 9, 8>(x1, x2, out, B, C, H, W, s);
    case 3: return launch_fwd<4, 4, 8, 9, 4>(x1, x2, out, B, C, H, W, s);
    case 4: return launch_fwd<4, 4, 8, 3, 8>(x1, x2, out, B, C, H, W, s);
    case 5: return launch_fwd<4, 4, 8, 3, 4>(x1, x2, out, B, C, H, W, s);
    case 6: return launch_fwd<4, 8, 8, 3, 4>(x1, x2, out, B, C, H, W, s);
    case 7: return launch_fwd<4, 4, 8, 1, 8>(x1, x2, out, B, C, H, W, s);
    default: return hipErrorInvalidValue;
  }
}
constexpr int kFwdCandidates = 8;

template <int D>
hipError_t fwd_dispatch(const float* x1, const float* x2, float* out, int B, int C, int H,
                        int W, hipStream_t s) {
  constexpr int K = 2 * D + 1;
  if (D == 4) {
    const int forced = variant_override(0);
    if (forced >= 0) return fwd_candidate_d4(forced, x1, x2, out, B, C, H, W, s);
  }
  // Prefer the big tile (8 px/lane, all displacement rows in one workgroup:
  // x1/x2 staged once); fall back to smaller tiles / split displacement rows
  // when that would leave most of the 256 CUs idle.
  const long big = (long)B * ((W + 63) / 64) * ((H + 7) / 8);
  if (big >= 256) return launch_fwd<D, 8, 8, K, 8>(x1, x2, out, B, C, H, W, s);
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
  static constexpr int DYW = (K + NW - 1) / NW;      // displacement rows per wave
  using L = Layout<PX, SEGX, D>;
  static constexpr int R = TH + 2 * D;               // staged rows
  static constexpr int C2 = TW + 2 * D;              // staged cols
  static constexpr int S = L::S;                     // LDS row stride
  static constexpr int P = round_up(R * S, 64);      // plane image (floats)
  static constexpr int CH = P / 64;
  static constexpr int J = (CH + NW - 1) / NW;       // chunks per wave per plane
  static constexpr int WIN = round_up(PX + 2 * D, 4);
  static constexpr int XIMG = CC * P;
  static constexpr int RED = NW * CC * TH * TW;      // per-wave partial sums
  static constexpr int LDSN = 2 * XIMG + WIN + RED;
  static_assert(PX % 4 == 0, "PX must be a multiple of 4");
};

// G2 == false: gx1 from (g, x2).  G2 == true: gx2 from (g, x1).
template <int D, int PX, int SEGX, int NW, int CC, bool G2>
__global__ __launch_bounds__(64 * NW) void corr_bwd_kernel(const float* __restrict__ xs,
                                                           const float* __restrict__ g,
                                                           float* __restrict__ gx, int C, int H,
                                                           int W, int tiles_x, int cg) {
  using F = BwdCfg<D, PX, SEGX, NW, CC>;
  constexpr int K = F::K, TW = F::TW, TH = F::TH, NT = F::NT, C2 = F::C2, S = F::S, P = F::P;
  constexpr int WIN = F::WIN, DYW = F::DYW, XIMG = F::XIMG;
  constexpr bool B64 = F::L::B64;
  __shared__ __attribute__((aligned(16))) float sm[F::LDSN];
  float* red = sm + 2 * XIMG + WIN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tile = blockIdx.x;
  const int cbeg = blockIdx.y * cg;
  const int cend = min(C, cbeg + cg);
  const int b = blockIdx.z;
  const int ty = tile / tiles_x;
  const int tx = tile - ty * tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  const int r = F::L::row(lane), q = F::L::seg(lane);
  const int y = y0 + r;
  const int xb = x0 + q * PX;

  const int HW = H * W;
  const float* xsb = xs + (size_t)b * C * HW;
  const float* gb = g + (size_t)b * K * K * HW;

  // this wave's DYW rows of g for its PX pixels, read once (clamped unconditional loads)
  float gv[DYW][K][PX];
#pragma unroll
  for (int t = 0; t < DYW; ++t) {
    const int dy = wave * DYW + t;
#pragma unroll
    for (int dx = 0; dx < K; ++dx) {
      const int k = min(dy, K - 1) * K + dx;
      const int yy = G2 ? y - dy + D : y;
#pragma unroll
      for (int i = 0; i < PX; ++i) {
        const int xx = G2 ? xb + i - dx + D : xb + i;
        const bool ok = dy < K && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
        const float v = gb[k * HW + (ok ? yy * W + xx : 0)];
        gv[t][dx][i] = ok ? v : 0.f;
      }
    }
  }

  int vo[F::J];
#pragma unroll
  for (int t = 0; t < F::J; ++t) {
    const int e = (wave + t * NW) * 64 + lane;
    const int rr = e / S, cc = e % S;
    const int gy = y0 - D + rr, gxx = x0 - D + cc;
    const bool ok = rr < F::R && cc < C2 && (unsigned)gy < (unsigned)H && (unsigned)gxx < (unsigned)W;
    vo[t] = ok ? (gy * W + gxx) * 4 : kOffImage;
  }
  auto dma_stage = [&](int c0, float* img) {
#pragma unroll
    for (int c = 0; c < CC; ++c) {
      const auto rs = plane_rsrc(xsb + (size_t)(c0 + c) * HW, c0 + c < cend, HW * 4);
#pragma unroll
      for (int t = 0; t < F::J; ++t)
        if (wave + t * NW < F::CH) dma64(rs, img + c * P + (wave + t * NW) * 64, vo[t]);
    }
  };

  const float cf = (float)C;
  float* gxb = gx + (size_t)b * C * HW;
  dma_stage(cbeg, sm);
  dma_wait_all();
  __syncthreads();
  int st = 0;
  for (int c0 = cbeg; c0 < cend; c0 += CC, ++st) {
    const float* cur = sm + (st & 1) * XIMG;
    if (c0 + CC < cend) dma_stage(c0 + CC, sm + ((st + 1) & 1) * XIMG);
    // partials stored lane-linear (lane*PX): conflict-free ds_write_b128
    float* rp = red + wave * (CC * TH * TW) + lane * PX;
#pragma unroll 2
    for (int c = 0; c < CC; ++c) {
      float acc[PX];
#pragma unroll
      for (int i = 0; i < PX; ++i) acc[i] = 0.f;
#pragma unroll
      for (int t = 0; t < DYW; ++t) {
        const int dy = wave * DYW + t;
        if (dy < K) {
          const int rs = G2 ? (2 * D - dy) : dy;
          float w[WIN];
          lds_read<B64>(cur + c * P + (r + rs) * S + q * PX, w);
#pragma unroll
          for (int dx = 0; dx < K; ++dx) {
            const int cs = G2 ? (2 * D - dx) : dx;
#pragma unroll
            for (int i = 0; i < PX; ++i) acc[i] = fmaf(gv[t][dx][i], w[i + cs], acc[i]);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < PX / 4; ++i)
        reinterpret_cast<float4*>(rp + c * (TH * TW))[i] =
            make_float4(acc[4 * i], acc[4 * i + 1], acc[4 * i + 2], acc[4 * i + 3]);
    }
    dma_wait_all();
    __syncthreads();  // partials complete; next stage's image landed
    for (int o = tid; o < CC * TH * TW; o += NT) {
      const int c = o / (TH * TW);
      const int pix = o - c * (TH * TW);
      const int py = pix / TW, pxo = pix % TW;
      // lane that owns pixel (py, pxo) under the layout's lane mapping
      const int ol = F::L::COLMAJOR ? (pxo / PX) * TH + py : py * SEGX + pxo / PX;
      const int ridx = c * (TH * TW) + ol * PX + pxo % PX;
      float sum = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < NW; ++w2) sum += red[w2 * (CC * TH * TW) + ridx];  // fixed order
      const int yy = y0 + py, xx = x0 + pxo;
      if (c0 + c < cend && yy < H && xx < W) gxb[(c0 + c) * HW + yy * W + xx] = sum / cf;
    }
    __syncthreads();  // partial slices free for the next stage
  }
}

template <int D, bool G2, int PX = 4, int SEGX = 8, int NW = 3, int CC = 4>
hipError_t launch_bwd(const float* xs, const float* g, float* gx, int B, int C, int H, int W,
                      hipStream_t s) {
  using F = BwdCfg<D, PX, SEGX, NW, CC>;
  const int tiles_x = (W + F::TW - 1) / F::TW;
  const int tiles_y = (H + F::TH - 1) / F::TH;
  const long tiles = (long)tiles_x * tiles_y * B;
  // channel group per workgroup: g is re-read once per group, so use as few
  // groups as still give ~512 workgroups
  int groups = (int)((512 + tiles - 1) / tiles);
  groups = max(1, min(groups, (C + CC - 1) / CC));
  const int cg = round_up((C + groups - 1) / groups, CC);
  dim3 grid(tiles_x * tiles_y, (C + cg - 1) / cg, B);
  hipLaunchKernelGGL((corr_bwd_kernel<D, PX, SEGX, NW, CC, G2>), grid, dim3(F::NT), 0, s, xs, g,
                     gx, C, H, W, tiles_x, cg);
  return hipGetLastError();
}

template <bool G2>
hipError_t bwd_candidate_d4(int i, const float* xs, const float* g, float* gx, int B, int C, int H,
                            int W, hipStream_t s) {
  switch (i) {
    case 0: return launch_bwd<4, G2, 4, 8, 3, 4>(xs, g, gx, B, C, H, W, s);
    case 1: return launch_bwd<4, G2, 4, 8, 3, 8>(xs, g, gx, B, C, H, W, s);
    case 2: return launch_bwd<4, G2, 4, 8, 9, 4>(xs, g, gx, B, C, H, W, s);
    case 3: return launch_bwd<4, G2, 4, 8, 9, 8>(xs, g, gx, B, C, H, W, s);
    default: return hipErrorInvalidValue;
  }
}
constexpr int kBwdCandidates = 4;

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

static int g_variant[3] = {-1, -1, -1};
int variant_override(int op) { return __atomic_load_n(&g_variant[op], __ATOMIC_RELAXED); }
int variant_count(int op) { return op == 0 ? kFwdCandidates : op == 1 ? kBwdCandidates : 2; }
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
