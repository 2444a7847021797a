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
#include <algorithm>
#include <cstdint>

#include "usf_common.h"

namespace usf {
namespace {

// gfx950 buffer descriptor word 3 for raw 32-bit loads (MI355X guide T8).
constexpr int kRsrcFlags = 0x00020000;
// a byte offset past any plane's num_records (planes are < 2 GiB, checked in capi.cpp)
constexpr int kOffImage = 0x7FFFFFF0;

#ifdef USF_TRACE
// Probe builds only (tools/probes/corr_trace.hip includes this file with
// USF_TRACE defined): lane 0 of every wave stores s_memrealtime (100 MHz) at
// phase boundaries, plus its HW_ID/XCC_ID, into g_trace[wave][kTraceSlots].
constexpr int kTraceSlots = 128;
__device__ unsigned long long* g_trace;
__device__ __forceinline__ unsigned trace_wave_id() {
  return ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * (blockDim.x >> 6) +
         (threadIdx.x >> 6);
}
#define USF_TRACE_AT(slot)                                                                   \
  do {                                                                                      \
    if ((threadIdx.x & 63) == 0 && g_trace && (slot) < kTraceSlots - 1)                     \
      g_trace[(size_t)trace_wave_id() * kTraceSlots + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define USF_TRACE_HWID()                                                                     \
  do {                                                                                      \
    if ((threadIdx.x & 63) == 0 && g_trace)                                                 \
      g_trace[(size_t)trace_wave_id() * kTraceSlots + kTraceSlots - 1] =                    \
          ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |          \
          (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);                              \
  } while (0)
#define USF_TRACE_VMWAIT() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#else
#define USF_TRACE_AT(slot) \
  do {                     \
  } while (0)
#define USF_TRACE_HWID() \
  do {                   \
  } while (0)
#define USF_TRACE_VMWAIT() \
  do {                     \
  } while (0)
#endif

using lds_void_t = __attribute__((address_space(3))) void;
using rsrc_t = int __attribute__((ext_vector_type(4)));

// Raw buffer descriptor of one channel plane (stride 0, num_records in bytes;
// 0 records for a channel past C so its whole stage reads as zeros).
__device__ __forceinline__ rsrc_t plane_rsrc(const float* plane, bool valid, int plane_bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(plane);
  rsrc_t r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) & 0xFFFF);
  r.z = __builtin_amdgcn_readfirstlane(valid ? plane_bytes : 0);
  r.w = kRsrcFlags;
  return r;
}

// One wave-instruction: 64*V consecutive floats of LDS at `dst` (wave-uniform;
// lane l fills floats [V*l, V*l+V)) from per-lane byte offsets `voff` of the
// plane described by `rsrc`. V = 4 is buffer_load_dwordx4 ... lds (1 KiB per
// instruction, about the issue cost of a 256-B dword DMA).
// Issued as inline asm on purpose: with the builtin, the compiler cannot tell
// the in-flight DMA into the other LDS image from the ds_reads of the current
// one and puts an s_waitcnt vmcnt(0) in front of every ds_read, serialising
// the prefetch with the FMAs. Completion is awaited explicitly (dma_wait_all +
// barrier at the end of each stage). M0 holds the LDS destination (an asm
// input, so the compiler materialises it). hipcc pads no hazard inside an asm
// statement, so the string opens with s_nop 4: the descriptor SGPRs may come
// straight from a VALU write (v_readfirstlane, or a v_readlane reloading a
// spilled SGPR), which a VMEM read needs 5 wait states behind
// (cdna_hip_programming.md 5.7 item 2); it also covers the M0 write.
template <int V>
__device__ __forceinline__ void dma(const rsrc_t& rsrc, float* dst, int voff) {
  static_assert(V == 1 || V == 4, "dword or dwordx4 LDS-DMA");
  // low 32 bits of a generic LDS pointer = the LDS byte address (no null check)
  const int m0 = __builtin_amdgcn_readfirstlane((int)(uint32_t)reinterpret_cast<uintptr_t>(dst));
  if constexpr (V == 4)
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
                 :
                 : "{m0}"(m0), "v"(voff), "s"(rsrc)
                 : "memory");
  else
    asm volatile("s_nop 4\n\tbuffer_load_dword %1, %2, 0 offen lds"
                 :
                 : "{m0}"(m0), "v"(voff), "s"(rsrc)
                 : "memory");
}

__device__ __forceinline__ void dma_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Buffer resource over `bytes` bytes at `p` (raw, stride 0) and a 16-byte load
// through it at a byte offset: the address is one 32-bit VGPR.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_buf(const float* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, bytes, kRsrcFlags);
}
__device__ __forceinline__ float buf_load1(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}
using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
using f32x4 = float __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 buf_load4(__amdgpu_buffer_rsrc_t r, int byte_off) {
  // explicitly typed: with `auto` and per-element bit casts this hipcc emitted ONE
  // buffer_load_dword and splatted it into all four lanes (caught by the parity tests)
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0);
  const f32x4 f = __builtin_bit_cast(f32x4, v);
  return make_float4(f.x, f.y, f.z, f.w);
}

__device__ __forceinline__ unsigned long long buf_load8(__amdgpu_buffer_rsrc_t r, int byte_off) {
  using u32x2 = unsigned int __attribute__((ext_vector_type(2)));
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, 0);
  return (unsigned long long)v.x | ((unsigned long long)v.y << 32);
}

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
//    stride = round_up(TW+2d, 16) (48 at TW=32): conflict-free, where 56 would
//    cost a 2-way conflict on every window read (tools/lds_banks.py).
// Pad columns of an LDS row are DMA'd as out-of-range zeros (never read).
// 16-byte DMA lanes (V = 4) need a row stride that is a multiple of 4 floats
// and image columns that start 4-aligned: the PX == 4 layout at d == 4 with
// W % 4 == 0 (every 4-float group is then wholly inside or outside the image).
template <int PX, int SEGX, int D>
struct Layout {
  static constexpr int TW = SEGX * PX, TH = 64 / SEGX;
  static constexpr bool B64 = PX == 8;
  static constexpr bool COLMAJOR = PX != 8;
  static constexpr int S = B64 ? TW + 10 : round_up(TW + 2 * D, 16);
  static_assert(S >= TW + 2 * D, "row stride must hold the halo row");
  static constexpr bool X4 = !B64 && S % 4 == 0 && D % 4 == 0;
  __device__ static int row(int lane) { return COLMAJOR ? lane % TH : lane / SEGX; }
  __device__ static int seg(int lane) { return COLMAJOR ? lane / TH : lane % SEGX; }
};

// One stage of CC channel planes staged HBM -> LDS: plane c of the stage is
// a ROWS x S image (row stride S, COLS valid columns from global column gx0,
// rows from gy0) at LDS offset c * PL, PL = ROWS * S rounded up to whole DMA
// chunks of 64*V floats, filled by CHP chunks per plane spread over NWAVE
// waves. The per-lane byte offsets are channel- and stage-invariant (one
// descriptor spans the whole sample; the channel base is added per plane), so
// each lane keeps only J of them. Lanes outside the image and planes past
// cend carry kOffImage (hardware zero fill); kOffImage + a channel base stays
// past num_records (< 2^31, capi.cpp).
template <int ROWS, int COLS, int S, int CC, int V, int NWAVE>
struct StageImg {
  static constexpr int CHUNK = 64 * V;
  static constexpr int PL = round_up(ROWS * S, CHUNK);  // LDS floats per plane
  static constexpr int CHP = PL / CHUNK;                // DMA chunks per plane
  static constexpr int J = (CHP + NWAVE - 1) / NWAVE;   // chunks per wave per plane
  static constexpr int N = CC * PL;                     // floats per stage image
  unsigned off[J];

  __device__ __forceinline__ void init(int wave, int lane, int gy0, int gx0, int H, int W) {
#pragma unroll
    for (int t = 0; t < J; ++t) {
      const int e = (wave + t * NWAVE) * CHUNK + lane * V;
      const int rr = e / S, cc = e - (e / S) * S;
      const int gy = gy0 + rr, gx = gx0 + cc;
      const bool ok = rr < ROWS && cc < COLS && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W;
      off[t] = ok ? (unsigned)((gy * W + gx) * 4) : (unsigned)kOffImage;
    }
  }
  // channels [c0, c0 + CC) of the sample; channels >= cend read as zeros
  __device__ __forceinline__ void load(const rsrc_t& rs, float* img, int wave, int c0, int cend,
                                       int HW) const {
#pragma unroll
    for (int c = 0; c < CC; ++c) {
      const bool cv = c0 + c < cend;
      const unsigned base = (unsigned)(c0 + c) * (unsigned)HW * 4u;
#pragma unroll
      for (int t = 0; t < J; ++t)
        if (wave + t * NWAVE < CHP)
          dma<V>(rs, img + c * PL + (wave + t * NWAVE) * CHUNK,
                 cv ? (int)(off[t] + base) : kOffImage);
    }
  }
};

// ---------------------------------------------------------------- forward --
// CS: channel slices inside one workgroup. With CS > 1 the workgroup has
// NDY * CS waves; all of them stage each CC-channel stage, and wave group h
// sums channels [h CC / CS, (h + 1) CC / CS) of it, so the stage buffers are
// shared (no extra LDS) while CS times as many waves hide the per-channel LDS
// latency (SURVEY config 2: 1152 waves for 1024 SIMDs at CS = 1). The slices'
// sums are added through LDS once at the end, in slice order.
template <int D, int PX, int SEGX, int NDY, int CC, int V, int CS = 1>
struct FwdCfg {
  static constexpr int K = 2 * D + 1;
  static constexpr int TW = SEGX * PX;              // tile width (pixels)
  static constexpr int TH = 64 / SEGX;              // tile height (rows)
  static constexpr int NW = NDY * CS;               // waves per workgroup
  static constexpr int NT = 64 * NW;                // threads per workgroup
  static constexpr int NDYG = (K + NDY - 1) / NDY;  // workgroups per tile
  using L = Layout<PX, SEGX, D>;
  static constexpr int R2 = TH + NDY - 1;           // staged x2 rows
  static constexpr int C2 = TW + 2 * D;             // staged x2 cols
  static constexpr int S = L::S;                    // LDS row stride (x1 and x2 images)
  using X1 = StageImg<TH, TW, S, CC, V, NW>;         // x1 tile, CC planes
  using X2 = StageImg<R2, C2, S, CC, V, NW>;         // x2 halo window, CC planes
  static constexpr int WIN = round_up(PX + 2 * D, 4);
  static constexpr int STAGE = X1::N + X2::N;
  static constexpr int LDSN = 2 * STAGE + WIN;      // two images + window over-read pad
  static_assert(CC % CS == 0, "whole channels per slice");
  static_assert(CS == 1 || 2 * STAGE >= (CS - 1) * NDY * K * PX * 64, "slice sums fit the stage buffers");
  static_assert(PX % 4 == 0, "PX must be a multiple of 4 (ds_read_b128)");
  static_assert(64 % SEGX == 0, "SEGX must divide 64");
  static_assert(V == 1 || L::X4, "16-byte DMA needs the 4-aligned layout");
};

// 1: partial-column tiles are dispatched last (corr_fwd_kernel); 0: the
// XCD-contiguous order for every grid
#ifndef USF_FWD_EDGE_LAST
#define USF_FWD_EDGE_LAST 1
#endif
#ifndef USF_FWD_EDGE_XCD
#define USF_FWD_EDGE_XCD 1
#endif
#ifndef USF_FWD_EDGE_CHUNK
#define USF_FWD_EDGE_CHUNK 8
#endif
// ... for grids of at least this many workgroups (smaller ones fit one round,
// where the reorder measured slower: config 2 23.1 -> 26.3 us warm)
#ifndef USF_FWD_EDGE_MIN
#define USF_FWD_EDGE_MIN 512
#endif

template <int N>
__device__ __forceinline__ void dma_wait_le() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }

template <int D, int PX, int SEGX, int NDY, int CC, int V, int CS = 1>
__global__ __launch_bounds__(64 * NDY * CS) void corr_fwd_kernel(const float* __restrict__ x1,
                                                                 const float* __restrict__ x2,
                                                                 float* __restrict__ out, int C,
                                                                 int H, int W, int tiles_x, FwdEpi ep) {
  using F = FwdCfg<D, PX, SEGX, NDY, CC, V, CS>;
  constexpr int K = F::K, TW = F::TW, TH = F::TH, S = F::S;
  constexpr int P1 = F::X1::PL, P2 = F::X2::PL, N1 = F::X1::N;
  constexpr int WIN = F::WIN, STAGE = F::STAGE;
  constexpr bool B64 = F::L::B64;
  __shared__ __attribute__((aligned(16))) float sm[F::LDSN];

  USF_TRACE_AT(0);
  USF_TRACE_HWID();
  const int lane = threadIdx.x & 63;
  const int wall = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // 0 .. NW-1 (DMA share)
  const int slice = wall / NDY;                                      // channel slice (uniform)
  const int wave = wall - slice * NDY;                               // displacement row in the group
  // work item: displacement-row group fastest, then tile, then (sample, channel group)
  const int nitems = gridDim.x * gridDim.y * gridDim.z;
  int dyb, tile, bz;
  const int tiles_y = gridDim.y / tiles_x;
  if (USF_FWD_EDGE_LAST && (W % TW) != 0 && tiles_x > 1 && nitems >= USF_FWD_EDGE_MIN) {
    // Partial-column tiles (the image's right edge, about half the work of a
    // full tile) are dispatched LAST, in chunks of consecutive items per XCD
    // (xcd_chunk keeps dispatch order at chunk granularity): when the grid is a
    // little over one resident round (KITTI L4 at batch 16: 896 workgroups for
    // 768 slots, 128 of them edge tiles), the second round is the cheap one.
    const int tf = tiles_y * (tiles_x - 1);     // full-column tiles per (sample, group)
    const int nfull = (int)(gridDim.z) * tf;
    // Within each phase every XCD takes one contiguous run of items (xcd_remap):
    // vertically neighbouring tiles, whose x2 halo rows overlap by 8 of 16, then
    // share an L2. Round 4 dealt 8-item chunks round-robin instead, which put
    // those neighbours on different XCDs: PMC fetch 57.6 -> 87.4 MB per L4
    // launch (1.03x -> 1.26x of algorithmic). USF_FWD_EDGE_XCD=0
    // restores the chunked deal (tools/ab_build.py).
    const int lin = linear_block(), nf = nfull * F::NDYG;
    const int u = !USF_FWD_EDGE_XCD ? xcd_chunk(lin, nitems, USF_FWD_EDGE_CHUNK)
                  : lin < nf        ? xcd_remap(lin, nf)
                                    : nf + xcd_remap(lin - nf, nitems - nf);
    const int g = u % F::NDYG, pi = u / F::NDYG;
    int tx, ty;
    if (pi < nfull) {
      bz = pi / tf;
      const int t = pi - bz * tf;
      ty = t / (tiles_x - 1);
      tx = t - ty * (tiles_x - 1);
    } else {
      const int e = pi - nfull;
      bz = e / tiles_y;
      ty = e - bz * tiles_y;
      tx = tiles_x - 1;
    }
    dyb = g * NDY;
    tile = ty * tiles_x + tx;
  } else {
    const int w = xcd_remap(linear_block(), nitems);
    dyb = (w % F::NDYG) * NDY;
    tile = (w / F::NDYG) % gridDim.y;
    bz = w / (F::NDYG * gridDim.y);
  }
  const int G = ep.groups;
  const int b = bz / G, grp = bz - b * G;
  // channel range of this workgroup (whole C without a split)
  const int cg = G > 1 ? round_up((C + G - 1) / G, CC) : C;
  const int cbeg = grp * cg, cend = min(C, cbeg + cg);
  const int ty = tile / tiles_x;
  const int tx = tile - ty * tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  const int r = F::L::row(lane), q = F::L::seg(lane);
  const int dy = dyb + wave;
  const bool active = dy < K;

  const int HW = H * W;
  // stage-invariant per-lane DMA offsets (pad columns / off-image pixels: zeros)
  typename F::X1 s1;
  typename F::X2 s2;
  s1.init(wall, lane, y0, x0, H, W);
  s2.init(wall, lane, y0 + dyb - D, x0 - D, H, W);
  const rsrc_t r1 = plane_rsrc(x1 + (size_t)b * C * HW, true, C * HW * 4);
  const rsrc_t r2 = plane_rsrc(x2 + (size_t)b * C * HW, true, C * HW * 4);
  auto dma_stage = [&](int c0, float* img) {
    s1.load(r1, img, wall, c0, cend, HW);
    s2.load(r2, img + N1, wall, c0, cend, HW);
  };

  float acc[K][PX];
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int i = 0; i < PX; ++i) acc[j][i] = 0.f;

  // Two stage images: each iteration waits for stage st, then (after the
  // barrier: every wave is done with stage st - 1's image) refills that image
  // with stage st + 1, in flight while stage st is summed. (A deeper ring, NB - 1
  // stages in flight, was slower at every shape in rounds 3 and 4: §4.2.)
  const int nst = (cend - cbeg + CC - 1) / CC;
  dma_stage(cbeg, sm);
  USF_TRACE_AT(1);
  for (int st = 0; st < nst; ++st) {
    USF_TRACE_AT(2 + 4 * st);
    dma_wait_all();
    USF_TRACE_AT(3 + 4 * st);
    __syncthreads();
    if (st + 1 < nst) dma_stage(cbeg + (st + 1) * CC, sm + ((st + 1) & 1) * STAGE);  // in flight during FMAs
    const float* cur = sm + (st & 1) * STAGE;
    USF_TRACE_AT(4 + 4 * st);
    if (active) {
      const float* p1 = cur + r * S + q * PX;
      const float* p2 = cur + N1 + (r + wave) * S + q * PX;
#pragma unroll 2
      for (int c = slice * (CC / CS); c < (slice + 1) * (CC / CS); ++c) {
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
    USF_TRACE_AT(5 + 4 * st);
  }

  if (G > 1 && ep.act && ep.mask) {
    // split forward: zero the sign mask here (every thread of the grid takes
    // part); corr_fwd_reduce_kernel, launched after this kernel, ORs its bits in
    const long long nw = (long long)(gridDim.z / G) * K * H * ((W + 3) >> 2);
    const long long nt = (long long)gridDim.x * gridDim.y * gridDim.z * blockDim.x;
    for (long long i = (long long)linear_block() * blockDim.x + threadIdx.x; i < nw; i += nt) ep.mask[i] = 0ull;
  }
  if constexpr (CS > 1) {
    // slices 1.. hand their sums to slice 0 through the stage buffers (idle
    // after this barrier); slice 0 adds them in slice order and runs the epilogue
    __syncthreads();
    float* xa = sm + (wave * K * PX) * 64 + lane;
    if (slice > 0 && active) {
#pragma unroll
      for (int j = 0; j < K; ++j)
#pragma unroll
        for (int i = 0; i < PX; ++i) xa[((slice - 1) * NDY * K * PX + j * PX + i) * 64] = acc[j][i];
    }
    __syncthreads();
    if (slice > 0) return;
    if (active) {
#pragma unroll
      for (int h = 1; h < CS; ++h)
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
          for (int i = 0; i < PX; ++i) acc[j][i] += xa[((h - 1) * NDY * K * PX + j * PX + i) * 64];
    }
  }
  if (!active) return;
  const int y = y0 + r;
  if (y >= H) return;
  const int xb = x0 + q * PX;
  if (G > 1) {  // raw channel-group partials [g][b][k][p]; corr_fwd_reduce_kernel finishes
    const int Bn = gridDim.z / G;

    float* pb = ep.part + ((size_t)(grp * Bn + b) * K * K + (size_t)dy * K) * HW + y * W + xb;
    const bool pvec = ((W & 3) == 0) && (xb + PX <= W);
#pragma unroll
    for (int dx = 0; dx < K; ++dx) {
      if (pvec) {
#pragma unroll
        for (int i = 0; i < PX / 4; ++i)
          reinterpret_cast<float4*>(pb + dx * HW)[i] =
              make_float4(acc[dx][4 * i], acc[dx][4 * i + 1], acc[dx][4 * i + 2], acc[dx][4 * i + 3]);
      } else {
#pragma unroll
        for (int i = 0; i < PX; ++i)
          if (xb + i < W) pb[dx * HW + i] = acc[dx][i];
      }
    }
    return;
  }
  const float cf = (float)C;
  // output planes of sample b start at b * ep.out_bstride (a channel slice of a
  // concat buffer, or the dense [B,K*K,H,W] tensor); LeakyReLU epilogue on request
  float* ob = out + (size_t)b * ep.out_bstride + (size_t)dy * K * HW + y * W + xb;
  const bool leaky = ep.act != 0;
  const float slope = ep.slope;
  // The channel mean v = acc / C as the reference rounds it. For a power-of-two C
  // (KITTI L1, L3, L4) the product with 1/C is the same number (exact scaling, one
  // rounding) without the IEEE division sequence. The branch is uniform; each
  // path is the whole epilogue (stores, then the sign mask).
  auto epilogue = [&](auto mean, auto pos) {
    auto epi = [&](float a) {
      const float v = mean(a);
      return leaky ? (v > 0.f ? v : v * slope) : v;
    };
    const bool vec = ((W & 3) == 0) && ((ep.out_bstride & 3) == 0) && (xb + PX <= W);
#pragma unroll
    for (int dx = 0; dx < K; ++dx) {
      float* o = ob + dx * HW;
      if (vec) {
#pragma unroll
        for (int i = 0; i < PX / 4; ++i)
          reinterpret_cast<float4*>(o)[i] = make_float4(epi(acc[dx][4 * i]), epi(acc[dx][4 * i + 1]),
                                                        epi(acc[dx][4 * i + 2]), epi(acc[dx][4 * i + 3]));
      } else {
#pragma unroll
        for (int i = 0; i < PX; ++i)
          if (xb + i < W) o[i] = epi(acc[dx][i]);
      }
    }
    if (leaky && ep.mask && xb < W) {
      // sign bits of this lane's activated outputs, one word per 4-pixel quad
      // (the epilogue's test v = mean(acc) > 0, as pos()); bits past W stay 0
      unsigned long long* mw = ep.mask + ((size_t)(b * K + dy) * H + y) * ((W + 3) >> 2) + (xb >> 2);
      // one bit per dx nibble, replicated: masks the columns past W of a partial quad
      constexpr unsigned long long kRep = [] {
        unsigned long long r = 0;
        for (int dx = 0; dx < K; ++dx) r |= 1ull << (4 * dx);
        return r;
      }();
#pragma unroll
      for (int j = 0; j < PX / 4; ++j) {
        unsigned long long bits = 0;
#pragma unroll
        for (int dx = 0; dx < K; ++dx)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            bits |= (unsigned long long)pos(acc[dx][4 * j + i]) << (4 * dx + i);
        const int nv = W - (xb + 4 * j);  // valid columns of this quad (> 0 for quads in the row)
        if (nv > 0) mw[j] = nv >= 4 ? bits : bits & (kRep * ((1ull << nv) - 1));
      }
    }
  };
  if ((C & (C - 1)) == 0) {
    // C = 2^k: v = RN(a 2^-k) > 0 exactly when a > 2^(k-150) (below that the
    // product rounds to zero), so the sign test needs no second product
    const float inv = 1.0f / cf;
    const float thr = C > 1 ? (cf * 0x1p-75f) * 0x1p-75f : 0.f;  // 2^(k-150), exact for k >= 1
    epilogue([&](float a) { return a * inv; }, [&](float a) { return a > thr; });
  } else {
    epilogue([&](float a) { return a / cf; }, [&](float a) { return a / cf > 0.f; });
  }
}

// out[b * obs + k * HW + p] = epilogue(sum_g part[g][b][k][p] / C), g in order.
// With the sign mask (zeroed by the split forward kernel before this one
// runs): each positive activated output ORs its bit 4 dx + x % 4 into word
// (b, dy, y, x / 4) -- the same words the unsplit forward's epilogue writes.
__device__ __forceinline__ void mask_or(const FwdEpi& ep, long long i, int KHW, int K, int H, int W) {
  const int HW = H * W;
  const long long b = i / KHW;
  const int r = (int)(i - b * KHW), k = r / HW, pp = r - k * HW;
  const int dy = k / K, dx = k - dy * K, y = pp / W, x = pp - y * W;
  atomicOr(ep.mask + ((b * K + dy) * H + y) * ((W + 3) >> 2) + (x >> 2), 1ull << (4 * dx + (x & 3)));
}
__global__ __launch_bounds__(256) void corr_fwd_reduce_kernel(const float* __restrict__ part,
                                                              float* __restrict__ out, FwdEpi ep,
                                                              int G, int B, int KHW, int C, int K,
                                                              int H, int W) {
  const long long per = (long long)B * KHW;
  const long long i0 = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i0 >= per) return;
  const float cf = (float)C;
  auto fin = [&](float s) {
    const float v = s / cf;
    return ep.act ? (v > 0.f ? v : v * ep.slope) : v;
  };
  const bool bits = ep.act && ep.mask;
  if ((KHW & 3) == 0 && (ep.out_bstride & 3) == 0) {
    float4 s = *reinterpret_cast<const float4*>(part + i0);
    for (int g = 1; g < G; ++g) {
      const float4 v = *reinterpret_cast<const float4*>(part + g * per + i0);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    const long long b = i0 / KHW, r = i0 - b * KHW;
    const float4 o = make_float4(fin(s.x), fin(s.y), fin(s.z), fin(s.w));
    *reinterpret_cast<float4*>(out + b * ep.out_bstride + r) = o;
    if (bits) {
      if (o.x > 0.f) mask_or(ep, i0, KHW, K, H, W);
      if (o.y > 0.f) mask_or(ep, i0 + 1, KHW, K, H, W);
      if (o.z > 0.f) mask_or(ep, i0 + 2, KHW, K, H, W);
      if (o.w > 0.f) mask_or(ep, i0 + 3, KHW, K, H, W);
    }
  } else {
    for (long long i = i0; i < i0 + 4 && i < per; ++i) {
      float s = part[i];
      for (int g = 1; g < G; ++g) s += part[g * per + i];
      const long long b = i / KHW, r = i - b * KHW;
      const float o = fin(s);
      out[b * ep.out_bstride + r] = o;
      if (bits && o > 0.f) mask_or(ep, i, KHW, K, H, W);
    }
  }
}

template <int D, int PX, int SEGX, int NDY, int CC, int V, int CS = 1>
hipError_t launch_fwd_v(const float* x1, const float* x2, float* out, int B, int C, int H, int W,
                        hipStream_t s, FwdEpi ep) {
  using F = FwdCfg<D, PX, SEGX, NDY, CC, V, CS>;
  const int tiles_x = (W + F::TW - 1) / F::TW;
  const int tiles_y = (H + F::TH - 1) / F::TH;
  dim3 grid(F::NDYG, tiles_x * tiles_y, B * ep.groups);
  hipLaunchKernelGGL((corr_fwd_kernel<D, PX, SEGX, NDY, CC, V, CS>), grid, dim3(F::NT), 0, s, x1,
                     x2, out, C, H, W, tiles_x, ep);
  if (ep.groups > 1) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int KHW = F::K * F::K * H * W;
    const long long per = (long long)B * KHW;
    // the element-wise reduce also ORs the sign bits into the mask (a
    // thread-per-word reduce was 4x slower at L0/L1: 36 x G dependent loads)
    hipLaunchKernelGGL(corr_fwd_reduce_kernel, dim3((unsigned)((per + 1023) / 1024)), dim3(256), 0, s,
                       ep.part, out, ep, ep.groups, B, KHW, C, F::K, H, W);
  }
  return hipGetLastError();
}

// 16-byte DMA staging whenever the layout and W allow it (see Layout).
template <int D, int PX, int SEGX, int NDY, int CC, int CS = 1>
hipError_t launch_fwd(const float* x1, const float* x2, float* out, int B, int C, int H, int W,
                      hipStream_t s, FwdEpi ep) {
  if constexpr (Layout<PX, SEGX, D>::X4) {
    if (W % 4 == 0) return launch_fwd_v<D, PX, SEGX, NDY, CC, 4, CS>(x1, x2, out, B, C, H, W, s, ep);
  }
  return launch_fwd_v<D, PX, SEGX, NDY, CC, 1, CS>(x1, x2, out, B, C, H, W, s, ep);
}

// ------------------------------------------------------ small-image forward --
// KITTI L0 / L1 (16 x {192x4x13, 128x8x26} in the decoder): the tiled kernel
// launches 48 workgroups there and walks 16-24 channel stages, each a full
// LDS-DMA round trip, so it splits the channel loop over workgroups and adds
// the partials in a second kernel (two launches, ~17 us). Here one workgroup
// owns (sample, displacement row dy, image row y) and stages ALL channels
// of its x1 row and of the x2 row y + dy - d (with the column halo as
// zeros) at once: one load round trip, one barrier. Thread t computes quad
// t % Q (4 pixels of one row, all K dx) over the channel slice t / Q; the
// slices are added through LDS in a fixed order (four interleaved chains,
// then pairwise: deterministic), and the same workgroup applies the mean, the
// LeakyReLU epilogue and writes the sign-mask words of its row.
// Staging is plain buffer loads + ds_write: W = 13, 26 rows are not 16-byte
// aligned, and the dword LDS-DMA form moved 64 KB per workgroup at a few
// bytes per clock (measured: L1 37 us with it vs 18.6 us for the split pair).
template <int D>
struct SmallFwdCfg {
  static constexpr int K = 2 * D + 1;
  static constexpr int WIN = round_up(4 + 2 * D, 4);  // x2 window of a quad
  static constexpr int HALO = round_up(2 * D, 4);     // x2 row = 4 W4 + HALO floats
  static constexpr int NT = 256;
  static constexpr int LDSN = 8192;                   // 32 KB: 5 workgroups per CU
  static constexpr int U = 36;                        // loads in flight per thread
};

// LDS image [C][S] of image row gy, columns gx0 .. gx0 + S - 1, all C
// channels of one sample, filled by NT2 threads (t = 0 .. NT2-1): element
// e = t + NT2 u, its column and offset advanced by NT2 with one carry (no
// divisions in the loop); off-image elements load as zeros (offset past
// num_records). The workgroup's x1 and x2 images are staged by different
// waves (descriptors stay wave-uniform), so both are in flight at once.
// V = 2 (even W, so every column pair is 8-byte aligned and wholly on or off
// the image): elements are column pairs, one 8-byte load each.
template <int NT2, int U, int V>
__device__ __forceinline__ void small_stage(__amdgpu_buffer_rsrc_t rs, float* img, int C, int S, int gy, int gx0,
                                            int H, int W, int t) {
  static_assert(V == 1 || V == 2, "dword or dwordx2 elements");
  const int SV = S / V, n = C * SV, HW = H * W;
  const int c0 = t / SV;
  int j = t - c0 * SV;                           // element column (units of V floats)
  int off = c0 * HW + gy * W + gx0 + V * j;      // float offset (used only on the image)
  const int dc = NT2 / SV, dj = NT2 - dc * SV;
  const bool rowok = (unsigned)gy < (unsigned)H;
  for (int e0 = 0; e0 < n; e0 += NT2 * U) {
    float v[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = rowok && e0 + u * NT2 + t < n && (unsigned)(gx0 + V * j) < (unsigned)W;
      if constexpr (V == 1) {
        v[u][0] = buf_load1(rs, ok ? off * 4 : kOffImage);
      } else {
        const unsigned long long w2 = buf_load8(rs, ok ? off * 4 : kOffImage);
        v[u][0] = __uint_as_float((unsigned)w2);
        v[u][1] = __uint_as_float((unsigned)(w2 >> 32));
      }
      j += dj;
      off += dc * HW + V * dj;
      if (j >= SV) { j -= SV; off += HW - S; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * NT2 + t;
      if (e < n) {
        if constexpr (V == 1)
          img[e] = v[u][0];
        else
          reinterpret_cast<float2*>(img)[e] = make_float2(v[u][0], v[u][1]);
      }
    }
  }
}

template <int D>
__global__ __launch_bounds__(256) void corr_fwd_small_kernel(const float* __restrict__ x1,
                                                             const float* __restrict__ x2,
                                                             float* __restrict__ out, int C, int H,
                                                             int W, FwdEpi ep) {
  using F = SmallFwdCfg<D>;
  constexpr int K = F::K, WIN = F::WIN, NT = F::NT;
  __shared__ __attribute__((aligned(16))) float sm[F::LDSN];
  // work item: dy fastest, then row, then sample; the K items of a row (same
  // x1 row, overlapping x2 rows) run on one XCD
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int dy = w % K;
  const int y = (w / K) % H;
  const int b = w / (K * H);
  const int W4 = (W + 3) >> 2, S1 = 4 * W4, S2 = 4 * W4 + F::HALO;
  const int n1 = C * S1;  // x1 image [C][S1], then x2 image [C][S2]
  const int tid = threadIdx.x;
  const int HW = H * W;
  const auto r1 = plane_buf(x1 + (size_t)b * C * HW, C * HW * 4);
  const auto r2 = plane_buf(x2 + (size_t)b * C * HW, C * HW * 4);
  if ((W & 1) == 0 && (D & 1) == 0) {  // 8-byte column pairs (x2's halo starts at -D)
    if (tid < NT / 2)
      small_stage<NT / 2, F::U / 2, 2>(r1, sm, C, S1, y, 0, H, W, tid);
    else
      small_stage<NT / 2, F::U / 2, 2>(r2, sm + n1, C, S2, y + dy - D, -D, H, W, tid - NT / 2);
  } else {
    if (tid < NT / 2)
      small_stage<NT / 2, F::U, 1>(r1, sm, C, S1, y, 0, H, W, tid);
    else
      small_stage<NT / 2, F::U, 1>(r2, sm + n1, C, S2, y + dy - D, -D, H, W, tid - NT / 2);
  }
  __syncthreads();

  const int Q = W4;  // quads of the row (<= 64, host-checked)
  // channel slices: as many as the threads allow and whose partials fit the stage
  const int NS = min(NT / Q, F::LDSN / (K * 4 * Q));
  const int cs = (C + NS - 1) / NS;
  const int ns = (C + cs - 1) / cs;  // slices that own channels
  const int qd = tid % Q, s = tid / Q;
  float acc[K][4];
#pragma unroll
  for (int dx = 0; dx < K; ++dx)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[dx][i] = 0.f;
  if (s < ns) {
    const int c1 = min(C, (s + 1) * cs);
    const float* p1 = sm + 4 * qd;
    const float* p2 = sm + n1 + 4 * qd;
#pragma unroll 2
    for (int c = s * cs; c < c1; ++c) {
      float a[4], wv[WIN];
      lds_read<false>(p1 + c * S1, a);
      lds_read<false>(p2 + c * S2, wv);
#pragma unroll
      for (int dx = 0; dx < K; ++dx)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[dx][i] = fmaf(a[i], wv[i + dx], acc[dx][i]);
    }
  }
  __syncthreads();  // staging images free: slice partials [s][dx * 4 + i][Q]
  float* red = sm;
  if (s < ns) {
#pragma unroll
    for (int dx = 0; dx < K; ++dx)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(s * (K * 4) + dx * 4 + i) * Q + qd] = acc[dx][i];
  }
  __syncthreads();

  const float cf = (float)C, inv = 1.f / cf;
  const bool pow2 = (C & (C - 1)) == 0;  // acc * (1/C) is then the same number as acc / C
  const bool leaky = ep.act != 0;
  const int ss = K * 4 * Q;  // slice stride of the partials
  for (int o = tid; o < K * S1; o += NT) {
    const int dx = o / S1, x = o - dx * S1;
    const int idx = (dx * 4 + (x & 3)) * Q + (x >> 2);
    // slices added in a fixed order: four interleaved chains, then (0+1)+(2+3)
    float t[4] = {0.f, 0.f, 0.f, 0.f};
    int s2 = 0;
    for (; s2 + 4 <= ns; s2 += 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k) t[k] += red[(s2 + k) * ss + idx];
    }
    for (int k = 0; s2 < ns; ++s2, ++k) t[k] += red[s2 * ss + idx];
    const float sum = (t[0] + t[1]) + (t[2] + t[3]);
    const float m = pow2 ? sum * inv : sum / cf;
    const float v = leaky ? (m > 0.f ? m : m * ep.slope) : m;
    // the sign mask tests the mean m > 0, as the tiled epilogue and the split
    // reduce do (the same bit as leaky(m) > 0 for slope >= 0; this thread is
    // the only reader of idx)
    red[idx] = m;
    if (x < W) out[(size_t)b * ep.out_bstride + (size_t)(dy * K + dx) * HW + y * W + x] = v;
  }
  if (!(leaky && ep.mask)) return;
  __syncthreads();
  if (tid < Q) {
    // all K * 4 reads issued at once (a per-element column test here made them
    // a dependent chain: ~2-3 us of the kernel), then the columns past W masked
    float v[K * 4];
#pragma unroll
    for (int k = 0; k < K * 4; ++k) v[k] = red[k * Q + tid];
    unsigned long long bits = 0;
#pragma unroll
    for (int k = 0; k < K * 4; ++k) bits |= (unsigned long long)(v[k] > 0.f) << (4 * (k >> 2) + (k & 3));
    constexpr unsigned long long kRep = [] {
      unsigned long long r = 0;
      for (int dx = 0; dx < K; ++dx) r |= 1ull << (4 * dx);
      return r;
    }();
    const int nv = W - 4 * tid;  // valid columns of the quad (> 0)
    ep.mask[((size_t)(b * K + dy) * H + y) * W4 + tid] = nv >= 4 ? bits : bits & (kRep * ((1ull << nv) - 1));
  }
}

// The small-image forward applies where one row of all channels (x1 [C][4 W4]
// + x2 [C][4 W4 + halo]) fits the 32 KB stage and every slice has a partial slot.
template <int D>
bool small_fwd_fits(int C, int H, int W) {
  using F = SmallFwdCfg<D>;
  const long W4 = (W + 3) / 4;
  return (long)C * (8 * W4 + F::HALO) <= F::LDSN && W4 <= 64 && H >= 1;
}

template <int D>
hipError_t launch_fwd_small(const float* x1, const float* x2, float* out, int B, int C, int H, int W,
                            hipStream_t s, FwdEpi ep) {
  if (!small_fwd_fits<D>(C, H, W)) return hipErrorInvalidValue;
  ep.groups = 1;
  ep.part = nullptr;
  hipLaunchKernelGGL((corr_fwd_small_kernel<D>), dim3((unsigned)(B * H * (2 * D + 1))),
                     dim3(SmallFwdCfg<D>::NT), 0, s, x1, x2, out, C, H, W, ep);
  return hipGetLastError();
}

// Tuning hook: usf_set_variant(0, i) forces candidate i for d=4
// (tools/kbench.py sweeps them on the GPU); -1 = the shape heuristic below.
hipError_t fwd_candidate_d4(int i, const float* x1, const float* x2, float* out, int B, int C,
                            int H, int W, hipStream_t s, FwdEpi ep) {
  switch (i) {
    case 0: return launch_fwd<4, 8, 8, 9, 8>(x1, x2, out, B, C, H, W, s, ep);
    case 1: return launch_fwd<4, 8, 8, 9, 4>(x1, x2, out, B, C, H, W, s, ep);
    case 2: return launch_fwd<4, 4, 8, 9, 8>(x1, x2, out, B, C, H, W, s, ep);
    case 3: return launch_fwd<4, 4, 8, 9, 4>(x1, x2, out, B, C, H, W, s, ep);
    case 4: return launch_fwd<4, 4, 8, 3, 8>(x1, x2, out, B, C, H, W, s, ep);
    case 5: return launch_fwd<4, 4, 8, 3, 4>(x1, x2, out, B, C, H, W, s, ep);
    case 6: return launch_fwd<4, 8, 8, 3, 4>(x1, x2, out, B, C, H, W, s, ep);
    case 7: return launch_fwd<4, 4, 8, 1, 8>(x1, x2, out, B, C, H, W, s, ep);
    case 8: return launch_fwd<4, 4, 8, 3, 8, 2>(x1, x2, out, B, C, H, W, s, ep);
    case 9: return launch_fwd<4, 4, 8, 3, 4, 2>(x1, x2, out, B, C, H, W, s, ep);
    case 10: return launch_fwd<4, 4, 8, 1, 8, 2>(x1, x2, out, B, C, H, W, s, ep);
    case 11: return launch_fwd<4, 4, 8, 1, 8, 4>(x1, x2, out, B, C, H, W, s, ep);
    case 12: return launch_fwd_small<4>(x1, x2, out, B, C, H, W, s, ep);
    default: return hipErrorInvalidValue;
  }
}
constexpr int kFwdCandidates = 13;

// Shape heuristic: all displacement rows in one workgroup (x1/x2 staged once)
// when that still fills the 256 CUs; else split displacement rows across
// workgroups (profiles/r01_v4_kbench.json: <4,8,9,4> is the fastest d=4
// candidate at the 64x208 level, <4,8,3,8> at 32x104 and below). Small levels
// (KITTI L0-L2: 24-96 workgroups, 12-24 serial channel stages of ~2 us DMA
// round trip each) also split the channel loop over `groups` workgroups
// (>= 2 stages each) when the caller provides the workspace for the partials.
struct FwdPlan {
  int cfg;     // 0: <4,8,K,4>, 1: <4,8,K,8>, 2: <4,8,3,8>, 3: small-image kernel
  int groups;  // channel groups
};
// the small-image kernel replaces the channel split wherever its rows fit
// (tools/ab_build.py -DUSF_FWD_SMALL=0: the split + reduce pair)
#ifndef USF_FWD_SMALL
#define USF_FWD_SMALL 1
#endif
template <int D>
FwdPlan fwd_plan(int B, int C, int H, int W) {
  constexpr int K = 2 * D + 1;
  const long tiles32 = (long)((W + 31) / 32) * ((H + 7) / 8);
  FwdPlan p{2, 1};
  const long big = (long)B * ((W + 63) / 64) * ((H + 7) / 8);
  if (big >= 256) p.cfg = 0;
  else if ((long)B * tiles32 >= 256) p.cfg = 1;
// split below 192 workgroups into ~384: at batch 16 splitting more (L2 into
// 2-6 groups) is slower, 22-26 vs 18.4 us (profiles/ab_r01/fwd_split_b16.json)
#ifndef USF_FWD_SPLIT_BELOW
#define USF_FWD_SPLIT_BELOW 192
#endif
#ifndef USF_FWD_SPLIT_TARGET
#define USF_FWD_SPLIT_TARGET 384
#endif
  if (p.cfg == 2) {
    const long wgs = (long)B * tiles32 * ((K + 2) / 3);
    if (wgs < USF_FWD_SPLIT_BELOW) {
      const int CC = 8;
      int g = (int)((USF_FWD_SPLIT_TARGET + wgs - 1) / wgs);
      p.groups = std::max(1, std::min(g, C / (2 * CC)));
      if (USF_FWD_SMALL && small_fwd_fits<D>(C, H, W)) p = FwdPlan{3, 1};
    }
  }
  return p;
}

template <int D>
hipError_t fwd_dispatch(const float* x1, const float* x2, float* out, int B, int C, int H,
                        int W, hipStream_t s, FwdEpi ep, float* ws, long long ws_floats) {
  constexpr int K = 2 * D + 1;
  if (D == 4) {
    const int forced = variant_override(0);
    if (forced >= 0) return fwd_candidate_d4(forced, x1, x2, out, B, C, H, W, s, ep);
  }
  const FwdPlan p = fwd_plan<D>(B, C, H, W);
  if (p.cfg == 3) return launch_fwd_small<D>(x1, x2, out, B, C, H, W, s, ep);
  if (p.cfg == 0) return launch_fwd<D, 4, 8, K, 4>(x1, x2, out, B, C, H, W, s, ep);
  if (p.cfg == 1) return launch_fwd<D, 4, 8, K, 8>(x1, x2, out, B, C, H, W, s, ep);
  const long long need = (long long)p.groups * B * K * K * H * W;
  if (p.groups > 1 && ws && ws_floats >= need) {
    ep.part = ws;
    ep.groups = p.groups;
    return launch_fwd<D, 4, 8, 3, 8>(x1, x2, out, B, C, H, W, s, ep);
  }
  // unsplit mid-size grids: two channel slices per workgroup on shared stages
  // (profiles/ab_r02/fwd_slices.json: KITTI L2 18.3 -> 14.6 us, SURVEY config 1
  // 9.3 -> 8.2 us with CC = 8). At C >= 128 (only SURVEY config 2 reaches this
  // path) one slice with CC = 8: from cold caches 28.0 vs 33.1 us (two slices
  // of CC = 4), warm 25.4 vs 23.9 us (profiles/ab_r05/corr_fwd_variants.json);
  // the cold figure is the HBM-honest one.
  if (C >= 128) return launch_fwd<D, 4, 8, 3, 8>(x1, x2, out, B, C, H, W, s, ep);
  return launch_fwd<D, 4, 8, 3, 8, 2>(x1, x2, out, B, C, H, W, s, ep);
}

// --------------------------------------------------------------- backward --
// 16-byte g loads in the backward prologue (tools/ab_build.py -DUSF_BWD_VECG=0: dword loads)
#ifndef USF_BWD_VECG
#define USF_BWD_VECG 1
#endif
template <int D, int PX, int SEGX, int NW, int CC, int V, int NB = 2>
struct BwdCfg {
  static constexpr int K = 2 * D + 1;
  static constexpr int TW = SEGX * PX;
  static constexpr int TH = 64 / SEGX;
  static constexpr int NT = 64 * NW;
  static constexpr int NW_ = NW;
  static constexpr int DYW = (K + NW - 1) / NW;      // displacement rows per wave
  using L = Layout<PX, SEGX, D>;
  static constexpr int R = TH + 2 * D;               // staged rows
  static constexpr int C2 = TW + 2 * D;              // staged cols
  static constexpr int S = L::S;                     // LDS row stride
  using X = StageImg<R, C2, S, CC, V, NW>;          // x halo window, CC planes
  static constexpr int P = X::PL;                    // plane image (floats)
  static constexpr int WIN = round_up(PX + 2 * D, 4);
  static constexpr int XIMG = X::N;
  static constexpr int RED = NW * CC * TH * TW;      // per-wave partial sums
  // <4,4,8,3,4>: 36 KB, so four workgroups fit the 160 KB LDS of a CU.
  // NB x image buffers in a ring: the DMA of stages s + 1 .. s + NB - 1 is in
  // flight during stage s. At L4 a third buffer (48 KB: 3 workgroups per CU)
  // was slower, 76.2 vs 67.8 us (profiles/ab_r02/bwd_nbuf.json); four buffers
  // pay on small grids, whose channel loops are short (bwd_dispatch).
  static constexpr int LDSN = NB * XIMG + RED;
  static constexpr int CC_ = CC;
  // resident workgroups per CU the LDS allows (at most the 3 the VGPRs allow)
  static constexpr int PER_CU = (160 * 1024 / (LDSN * 4)) < 3 ? (160 * 1024 / (LDSN * 4)) : 3;
  static_assert(PX % 4 == 0, "PX must be a multiple of 4");
  static_assert(V == 1 || L::X4, "16-byte DMA needs the 4-aligned layout");
};

// 1: the backward's stage-0 x DMA goes out before the g slice and the first
// barrier waits only for it (corr_bwd_tile); 0: both waited for (vmcnt(0)).
#ifndef USF_BWD_EARLY
#define USF_BWD_EARLY 1
#endif
// Occupancy target of the backward kernels (see corr_bwd_kernel).
#ifndef USF_BWD_WAVES_PER_EU
#define USF_BWD_WAVES_PER_EU 3
#endif
// Work items per XCD chunk of the backward's block order (see corr_bwd_kernel).
#ifndef USF_BWD_CHUNK
#define USF_BWD_CHUNK 14
#endif
// g prologue of one wave: its DYW displacement rows of g for its PX pixels,
// read once per workgroup. gx1 (G2 == false) takes g at the lane's own pixels;
// gx2 (G2 == true) takes, for displacement k, g at pixel - delta_k. All loads
// are unconditional at clamped in-bounds offsets (no branch, so no wait, inside
// the burst). With W % 4 == 0 (V == 4) each 4-pixel run is ONE 16-byte load:
// the dword form made every wave-instruction touch 8 cache lines for 32 of
// their 128 bytes, 4 times over. gx2's runs start at xb - dx + d (dword
// aligned): the load is clamped into the row and the lanes at the image edge
// pick their elements out of it by index. AM: the LeakyReLU derivative from
// the forward's sign mask, applied inside the loads.
template <int D, int PX, int SEGX, int NW, int CC, int V, bool G2, bool AM, int DYW, int K>
__device__ __forceinline__ void bwd_load_g(float (&gv)[DYW][K][PX], const float* __restrict__ gb,
                                           const BwdEpi& ep, int b, int wave, int y, int xb, int H,
                                           int W) {
  static_assert(DYW == BwdCfg<D, PX, SEGX, NW, CC, V>::DYW && K == 2 * D + 1, "g slice shape");
  const int HW = H * W;
  // raw buffer descriptors over this sample's K*K planes: 16-byte loads with a
  // 32-bit offset (one VGPR per address instead of a 64-bit pointer pair)
  const auto grs = plane_buf(gb, K * K * HW * 4);
  // AM: the forward's LeakyReLU sign mask of sample b ([dy][y][ceil(W/4)] words)
  const int W4 = (W + 3) >> 2;
  const auto mrs = AM ? __builtin_amdgcn_make_buffer_rsrc(
                            const_cast<unsigned long long*>(ep.mask + (size_t)b * K * H * W4), 0,
                            K * H * W4 * 8, kRsrcFlags)
                      : grs;
  // the mask words cover pixels xb - 4 .. xb + 7 (mw[0..2]), i.e. ei in [-d, 3 + d] for d <= 4
  static_assert(!AM || (PX == 4 && D <= 4), "sign-mask derivative: 4-pixel runs, d <= 4");
#pragma unroll
  for (int t = 0; t < DYW; ++t) {
    const int dy = wave * DYW + t;
    // AM: sign words of this row -- gx1: the lane's own quad; gx2: its runs
    // start at xb - dx + d, so the quads left of, at and right of xb
    unsigned long long mw[3] = {0, 0, 0};
    if constexpr (AM) {
      const int yy = G2 ? y - dy + D : y;
      const bool rowok = dy < K && (unsigned)yy < (unsigned)H;
      const int mrow = (min(dy, K - 1) * H + (rowok ? yy : 0)) * W4;
      const int q0 = xb >> 2;
#pragma unroll
      for (int o = G2 ? -1 : 0; o <= (G2 ? 1 : 0); ++o) {
        const int qq = min(max(q0 + o, 0), W4 - 1);
        mw[o + 1] = buf_load8(mrs, (mrow + qq) * 8);
      }
    }
#pragma unroll
    for (int dx = 0; dx < K; ++dx) {
      const int k = min(dy, K - 1) * K + dx;
      const int yy = G2 ? y - dy + D : y;
      const bool rowok = dy < K && (unsigned)yy < (unsigned)H;
      if constexpr (USF_BWD_VECG && V == 4 && PX % 4 == 0) {
        const unsigned ro = (unsigned)(k * HW + (rowok ? yy : 0) * W);
#pragma unroll
        for (int i4 = 0; i4 < PX; i4 += 4) {
          const int xs = G2 ? xb + i4 - dx + D : xb + i4;
          const int xc = min(max(xs, 0), W - 4);
          const float4 v = buf_load4(grs, (int)((ro + (unsigned)xc) * 4u));
          const int shift = xs - xc;  // 0 inside the image
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int xx = xs + i;
            const bool ok = rowok && (unsigned)xx < (unsigned)W;
            // gx2's edge lanes pick their element by index; gx1 runs are aligned, never shifted
            const int idx = G2 ? i + shift : i;
            float e = idx <= 0 ? v.x : idx == 1 ? v.y : idx == 2 ? v.z : v.w;
            if constexpr (AM) {
              // LeakyReLU derivative (on the result, as the in-place module):
              // pixel xb + ei of the row, ei in [-d, 3 + d]; compile-time word and bit
              const int ei = G2 ? i4 + i - dx + D : i4 + i;
              const unsigned long long wd = mw[(ei + 4) >> 2];
              const bool pos = (wd >> (4 * dx + (ei & 3))) & 1ull;
              e = pos ? e : e * ep.slope;
            }
            gv[t][dx][i4 + i] = ok ? e : 0.f;
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < PX; ++i) {
          const int xx = G2 ? xb + i - dx + D : xb + i;
          const bool ok = rowok && (unsigned)xx < (unsigned)W;
          float v = buf_load1(grs, (k * HW + (ok ? yy * W + xx : 0)) * 4);
          if constexpr (AM) {  // as in the 16-byte path: pixel xb + ei, compile-time word and bit
            const int ei = G2 ? i - dx + D : i;
            const bool pos = (mw[(ei + 4) >> 2] >> (4 * dx + (ei & 3))) & 1ull;
            v = pos ? v : v * ep.slope;
          }
          gv[t][dx][i] = ok ? v : 0.f;
        }
      }
    }
  }
}

// VMEM instructions bwd_load_g issues per wave, after the stage DMAs that the
// backward's first wait counts past (bwd_wait_stages' EXTRA): per displacement
// row its sign-mask words (AM: 1 for gx1, 3 for gx2) and one load per (dx,
// 4-pixel run) on the 16-byte path, per (dx, pixel) on the dword path. Every
// one is a separate buffer load at a runtime offset, so none can be merged.
// The first wait leaves at most this many younger loads outstanding; a smaller
// count would let the FMAs read a partly landed stage 0 (advisor r04).
template <int D, int PX, int V, bool G2, bool AM, int DYW>
constexpr int bwd_g_loads() {
  constexpr int K = 2 * D + 1;
  constexpr int per_dx = (USF_BWD_VECG && V == 4 && PX % 4 == 0) ? PX / 4 : PX;
  return DYW * ((AM ? (G2 ? 3 : 1) : 0) + K * per_dx);
}

// One stage of CC channels for one wave: its DYW displacement rows summed in
// registers per channel, the partial written lane-linear (lane*PX:
// conflict-free ds_write_b128) to rp + c * TH * TW.
template <int D, int PX, int SEGX, int NW, int CC, int V, bool G2, int DYW, int K>
__device__ __forceinline__ void bwd_stage(const float (&gv)[DYW][K][PX], const float* cur, float* rp,
                                          int wave, int r, int q, const BwdEpi& ep) {
  using F = BwdCfg<D, PX, SEGX, NW, CC, V>;
  constexpr int TW = F::TW, TH = F::TH, S = F::S, P = F::P;
  constexpr int WIN = F::WIN;
  constexpr bool B64 = F::L::B64;
#pragma unroll 2
  for (int c = 0; c < CC; ++c) {
    float acc[PX];
#pragma unroll
    for (int i = 0; i < PX; ++i) acc[i] = 0.f;
#pragma unroll
    for (int t = 0; t < DYW; ++t) {
      const int dy = wave * DYW + t;
      // compile-time true when the waves' rows tile K exactly (NW * DYW == K):
      // no per-row branch, so the compiler overlaps one row's ds_reads with the
      // previous row's FMAs (L4 75.4 -> 70.6 us, profiles/ab_r02)
      if (NW * DYW == K || dy < K) {
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
}

#ifndef USF_BWD_RCP
#define USF_BWD_RCP 1
#endif
// Combine the NW wave partials of one direction (red: [NW][CC][TH*TW]) in a
// fixed order, 4 pixels per thread (a lane's PX pixels are contiguous in its
// partial slot), and write channels [c0, c0 + CC) of the tile, divided by C.
template <int D, int PX, int SEGX, int NW, int CC, int V>
__device__ __forceinline__ void bwd_combine(const float* red, float* gxb, int t1, int nthr, int c0,
                                            int cend, int y0, int x0, int H, int W, float cf, float fc,
                                            bool pow2) {
  using F = BwdCfg<D, PX, SEGX, NW, CC, V>;
  constexpr int TW = F::TW, TH = F::TH;
  const int HW = H * W;
  const bool vec_out = (W & 3) == 0;
  // items in partial-slot order (consecutive threads read consecutive 16-byte
  // slots: conflict-free ds_read_b128; the pixel-order walk this replaces put
  // 2-4 lanes of each 16-lane group on one bank set under the column-major
  // lane layout); a 64-thread run still writes whole 128-byte
  // row pieces of the tile.
  for (int o = t1; o < CC * TH * TW / 4; o += nthr) {
    const int c = o / (TH * TW / 4);
    const int slot = (o - c * (TH * TW / 4)) * 4;  // = ol * PX + j
    const int ol = slot / PX, j = slot % PX;
    // pixel of lane ol's j-th 4-pixel run under the layout's lane mapping
    const int py = F::L::COLMAJOR ? ol % TH : ol / SEGX;
    const int pxo = (F::L::COLMAJOR ? ol / TH : ol % SEGX) * PX + j;
    const int ridx = c * (TH * TW) + slot;
    float4 sum = *reinterpret_cast<const float4*>(red + ridx);
#pragma unroll
    for (int w2 = 1; w2 < NW; ++w2) {
      const float4 v = *reinterpret_cast<const float4*>(red + w2 * (CC * TH * TW) + ridx);
      sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
    }
    const int yy = y0 + py, xx = x0 + pxo;
    if (c0 + c < cend && yy < H) {
      float* o4 = gxb + (size_t)(c0 + c) * HW + yy * W + xx;
      // the channel mean: for power-of-two C a multiply by 1/C, which is the
      // same number as the division (scaling by 2^-k rounds once); for other C
      // the IEEE division the reference does (correlation_cuda_kernel.cu:204,
      // 297; ~10 VALU instructions per element, only at those levels)
      if (USF_BWD_RCP && pow2) {
        sum.x *= cf; sum.y *= cf; sum.z *= cf; sum.w *= cf;
      } else {
        sum.x /= fc; sum.y /= fc; sum.z /= fc; sum.w /= fc;
      }
      if (vec_out && xx + 3 < W) {
        *reinterpret_cast<float4*>(o4) = sum;
      } else {
        if (xx < W) o4[0] = sum.x;
        if (xx + 1 < W) o4[1] = sum.y;
        if (xx + 2 < W) o4[2] = sum.z;
        if (xx + 3 < W) o4[3] = sum.w;
      }
    }
  }
}

// Wait until at most KS stages of this wave's x DMA plus EXTRA younger loads
// are outstanding. A wave owns the J-th chunk slot of the image or not
// (StageImg::load), so it issues one of two per-stage counts.
template <class F, int KS, int EXTRA>
__device__ __forceinline__ void bwd_wait_stages(int wave) {
  constexpr int J = F::X::J, CC = F::CC_;
  static_assert(KS * CC * J + EXTRA <= 63, "vmcnt holds 6 bits");
  if (wave + (J - 1) * F::NW_ < F::X::CHP) dma_wait_le<KS * CC * J + EXTRA>();
  else dma_wait_le<KS * CC * (J - 1) + EXTRA>();
}

// One (tile, channel group) of gx1 (G2 == false: from g and x2) or gx2
// (G2 == true: from g and x1; mirrored indices).
template <int D, int PX, int SEGX, int NW, int CC, int V, bool G2, bool AM, int NB>
__device__ __forceinline__ void corr_bwd_tile(float* sm, const float* __restrict__ xs,
                                              const float* __restrict__ g,
                                              float* __restrict__ gx, int tile, int group, int b,
                                              int C, int H, int W, int tiles_x, int cg,
                                              const BwdEpi& ep) {
  using F = BwdCfg<D, PX, SEGX, NW, CC, V, NB>;
  constexpr int K = F::K, TW = F::TW, TH = F::TH, NT = F::NT;
  constexpr int DYW = F::DYW, XIMG = F::XIMG;
  (void)K;
  float* red = sm + NB * XIMG;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cbeg = group * cg;
  const int cend = min(C, cbeg + cg);
  const int ty = tile / tiles_x;
  const int tx = tile - ty * tiles_x;
  const int y0 = ty * TH, x0 = tx * TW;
  const int r = F::L::row(lane), q = F::L::seg(lane);
  const int y = y0 + r;
  const int xb = x0 + q * PX;

  const int HW = H * W;
  const float* xsb = xs + (size_t)b * C * HW;
  typename F::X sx;
  sx.init(wave, lane, y0 - D, x0 - D, H, W);
  const rsrc_t rx = plane_rsrc(xsb, true, C * HW * 4);
  auto dma_stage = [&](int c0, float* img) { sx.load(rx, img, wave, c0, cend, HW); };

  const float cf = 1.f / (float)C, fc = (float)C;  // bwd_combine's scale (exact: power-of-two C only)
  const bool pow2 = (C & (C - 1)) == 0;
  float* gxb = gx + (size_t)b * C * HW;
  // The x DMA of stages 0 .. NB-2 goes out before the g slice, and the first
  // barrier waits only for stage 0: vmcnt leaves the younger stages and the
  // DYW * K g loads in flight, so the FMAs of displacement row t wait only for
  // that row's g loads (hipcc's per-register waits) and the slice's HBM burst
  // overlaps the first stage.
  const int nst = (cend - cbeg + CC - 1) / CC;
#pragma unroll
  for (int i = 0; i < NB - 1; ++i)
    if (i < nst) dma_stage(cbeg + i * CC, sm + i * XIMG);
  // g of sample b at b * ep.g_bstride: a channel slice of the concat gradient,
  // or the dense [B,K*K,H,W] tensor
  float gv[DYW][2 * D + 1][PX];
  bwd_load_g<D, PX, SEGX, NW, CC, V, G2, AM>(gv, g + (size_t)b * ep.g_bstride, ep, b, wave, y, xb, H, W);
  USF_TRACE_VMWAIT();
  USF_TRACE_AT(1);
  // ring: stage st in slot st % NB. The first barrier waits for stage 0 only;
  // then each iteration refills the slot of stage st - 1 (every wave is past
  // the barrier that follows its last read of it) with stage st + NB - 1 and
  // sums stage st. Two placements of the wait for the next stage, each the
  // faster one where it is used (profiles/ab_r04/corr_bwd_ring.json):
  //  * NB == 2: after the FMAs, BEFORE the combine. vmcnt also counts the
  //    combine's global stores (gfx9 has no separate store counter), and a wait
  //    placed after them puts their write latency on every stage (in the step
  //    L3 49 -> 57 us, L4 73 -> 76 us);
  //  * NB == 4 (small grids, 2-6 stages): at the top of the next iteration,
  //    after the combine (L0/L1 16.0 -> 13.9 / 15.6 -> 13.6 us replayed).
  // Stage 0's wait is peeled in front of the loop for the 16-byte-DMA two-image
  // loop (L3/L4: 74.2 -> 72.4 us, same-box A/B) and stays inside it otherwise:
  // peeled, NB == 4 measured 2 us slower at L1 and the dword-DMA two-image
  // instantiation spilled a register.
  constexpr bool TOPWAIT = NB > 2;
  constexpr bool PEEL = !TOPWAIT && V == 4;
  // the first wait's EXTRA: the g slice loads issued after the stage DMAs (a lower bound)
  constexpr int GL = DYW * K;
  static_assert(GL <= bwd_g_loads<D, PX, V, G2, AM, DYW>(), "first wait counts past more loads than bwd_load_g issues");
  if constexpr (PEEL) {
    if (USF_BWD_EARLY) bwd_wait_stages<F, 0, GL>(wave);
    else dma_wait_all();
    __syncthreads();  // stage 0 landed
  }
  for (int st = 0; st < nst; ++st) {
    // ring slots of the stage read and of the one refilled (NB is 2 or 4: masks)
    const int rd = st % NB, wr = (st + NB - 1) % NB;
    if (!PEEL && (TOPWAIT || st == 0)) {
      // stage st; the stages issued after it (st + 1 .. st + NB - 2) and, at st = 0,
      // the g slice may stay in flight
      if (st == 0 && USF_BWD_EARLY) {
        if (NB == 2 || nst >= NB - 1) bwd_wait_stages<F, NB - 2, GL>(wave);
        else dma_wait_all();
      } else if (TOPWAIT && st + NB - 2 < nst) {
        bwd_wait_stages<F, NB - 2, 0>(wave);
      } else {
        dma_wait_all();
      }
      __syncthreads();  // stage st landed; partial slices free
    }
    USF_TRACE_AT(3 + 5 * st);
    if (st + NB - 1 < nst) dma_stage(cbeg + (st + NB - 1) * CC, sm + wr * XIMG);
    const float* cur = sm + rd * XIMG;
    USF_TRACE_AT(4 + 5 * st);
    bwd_stage<D, PX, SEGX, NW, CC, V, G2>(gv, cur, red + wave * (CC * TH * TW) + lane * PX, wave, r, q, ep);
    USF_TRACE_AT(5 + 5 * st);
    if (!TOPWAIT) dma_wait_all();  // stage st + 1 (NB == 2: nothing else in flight)
    USF_TRACE_AT(6 + 5 * st);
    __syncthreads();  // partials complete (NB == 2: and stage st + 1 landed)
    USF_TRACE_AT(7 + 5 * st);
    bwd_combine<D, PX, SEGX, NW, CC, V>(red, gxb, tid, NT, cbeg + st * CC, cend, y0, x0, H, W, cf, fc, pow2);
    if (!TOPWAIT) __syncthreads();  // partial slices free for the next stage
  }
}

// MODE 1: gx1 only, 2: gx2 only, 3: both (blockIdx.z in [0, 2B): gx1 first).
// One launch for both directions keeps the whole chip busy through the tail
// of either half and halves the launch count; the two inlined bodies still
// fit 3 waves/SIMD at <4,8,3,4> (tools/kernel_resources.py).
// Budget (tests/test_kernel_resources.py): <4,8,3,4> within 168 VGPRs and
// 40 KB LDS, i.e. 3 waves/SIMD = 4 resident workgroups of 3 waves per CU.
// amdgpu_waves_per_eu(3) pins the VGPR target: without it, allocation for the
// two inlined direction bodies flips between 163 and 231 on unrelated edits.
template <int D, int PX, int SEGX, int NW, int CC, int V, int MODE, bool AM, int NB>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(USF_BWD_WAVES_PER_EU))) void corr_bwd_kernel(const float* __restrict__ x1,
                                                           const float* __restrict__ x2,
                                                           const float* __restrict__ g,
                                                           float* __restrict__ gx1,
                                                           float* __restrict__ gx2, int B, int C,
                                                           int H, int W, int tiles_x, int cg,
                                                           BwdEpi ep) {
  __shared__ __attribute__((aligned(16))) float sm[BwdCfg<D, PX, SEGX, NW, CC, V, NB>::LDSN];
  USF_TRACE_AT(0);
  USF_TRACE_HWID();
  // work item: channel group fastest (the groups of a tile share its g planes),
  // then tile, then (direction, sample); grid = (tiles, groups, B * dirs).
  // Whole-sample XCD orders were measured slower on the box (tools/ab_build.py):
  // remapping this order (L4 85 vs 59 us) and a direction-fastest order dealt
  // to the XCDs in contiguous chunks (L4 84 vs 59 us, L3 51 vs 43 us), although
  // they cut the FETCH traffic (2.6x -> 1.4x of algorithmic). Short chunks
  // (below) keep both.
  int w = linear_block();
#ifndef USF_BWD_GROUP_XCD
#define USF_BWD_GROUP_XCD 1
#endif
#ifndef USF_BWD_SAMPLE_RING
#define USF_BWD_SAMPLE_RING 1
#endif
  // (A direction-fastest order -- a tile's gx1 and gx2 items neighbours in one
  // XCD chunk, so the second read of its g slice hits L2 -- cut FETCH 215.6 ->
  // 157.9 MB per L4 launch at the same replayed time but ran 6 us slower in the
  // step, profiles/ab_r02/bwd_dirfast_pmc.json and r02_v3_*; removed in round 6.)
  const int nitems = gridDim.x * gridDim.y * gridDim.z;
  const int per_sample = gridDim.x * gridDim.y;  // work items of one (sample, direction)
  if (NB > 2 && USF_BWD_SAMPLE_RING && nitems >= 8 * per_sample) {
    // small (four-image ring) grids: every item of a (sample, direction) -- its
    // tiles, whose x halo rows overlap, and their channel groups, which all
    // load the tile's g slice -- on one XCD (USF_BWD_SAMPLE_RING; KITTI L2 PMC
    // traffic 2.13x -> 1.02x, 25.5 -> 23.7 us, profiles/ab_r05/corr_bwd_sample_xcd.json)
    w = xcd_chunk(w, nitems, per_sample);
  } else if (USF_BWD_CHUNK > 0 && gridDim.x >= 16) {
    // Q consecutive work items per XCD, chunks dealt round-robin over the 8
    // XCDs (block lin runs on XCD lin % 8; it gets item Q (8 m + x) + j): a few
    // neighbouring tiles share their halo lines in one L2 while every XCD still
    // gets a mix of samples and directions. L4 59.5 -> 54.5 us, L3 43 -> 40 us
    // (profiles/ab_r01/bwd_chunk_*.json); whole-sample chunks (xcd_remap) are
    // slower (84 us) and so are levels with < 16 tiles (L1 11.6 -> 13.5 us).
    w = xcd_chunk(w, gridDim.x * gridDim.y * gridDim.z, USF_BWD_CHUNK);
  } else if (USF_BWD_GROUP_XCD && gridDim.y > 1) {
    // Otherwise small grids that split a tile's channels over gridDim.y groups
    // (each loads the tile's whole g slice): one XCD chunk per tile's groups. In
    // the linear order they were consecutive blocks on different XCDs, every
    // group missing its own L2 (L0 1.89x -> 1.17x, L1 2.06x -> 1.06x,
    // profiles/ab_r05/corr_bwd_group_xcd.json).
    w = xcd_chunk(w, nitems, gridDim.y);
  }
  const int group = w % gridDim.y;
  const int tile = (w / gridDim.y) % gridDim.x;
  const int b = w / (gridDim.x * gridDim.y);
  if constexpr (MODE == 1) {
    corr_bwd_tile<D, PX, SEGX, NW, CC, V, false, AM, NB>(sm, x2, g, gx1, tile, group, b, C, H, W, tiles_x, cg, ep);
  } else if constexpr (MODE == 2) {
    corr_bwd_tile<D, PX, SEGX, NW, CC, V, true, AM, NB>(sm, x1, g, gx2, tile, group, b, C, H, W, tiles_x, cg, ep);
  } else {
    if (b >= B)
      corr_bwd_tile<D, PX, SEGX, NW, CC, V, true, AM, NB>(sm, x1, g, gx2, tile, group, b - B, C, H, W,
                                                      tiles_x, cg, ep);
    else
      corr_bwd_tile<D, PX, SEGX, NW, CC, V, false, AM, NB>(sm, x2, g, gx1, tile, group, b, C, H, W,
                                                       tiles_x, cg, ep);
  }
}

// Workgroups a backward launch aims for (both directions together): enough to
// fill the 256 CUs at 3-4 resident workgroups each, and no more -- every
// extra channel group re-reads its tile's slice of g (81 planes).
#ifndef USF_BWD_TARGET_WG
#define USF_BWD_TARGET_WG 768
#endif
constexpr int kBwdTargetWorkgroups = USF_BWD_TARGET_WG;

template <int D, int PX, int SEGX, int NW, int CC, int V, int MODE, int NB>
hipError_t launch_bwd_mode(const float* x1, const float* x2, const float* g, float* gx1,
                           float* gx2, int B, int C, int H, int W, hipStream_t s, BwdEpi ep) {
  using F = BwdCfg<D, PX, SEGX, NW, CC, V, NB>;
  const int dirs = MODE == 3 ? 2 : 1;
  const int tiles_x = (W + F::TW - 1) / F::TW;
  const int tiles_y = (H + F::TH - 1) / F::TH;
  const long units = (long)tiles_x * tiles_y * B * dirs;
  // one resident round: 768 at 3 workgroups per CU, fewer for a deeper ring
  const long target = (long)kBwdTargetWorkgroups * F::PER_CU / 3;
  int groups = (int)((target + units - 1) / units);
  groups = max(1, min(groups, (C + CC - 1) / CC));
  const int cg = round_up((C + groups - 1) / groups, CC);
  dim3 grid(tiles_x * tiles_y, (C + cg - 1) / cg, B * dirs);
  if constexpr (PX == 4) {
    if (ep.mask) {
      hipLaunchKernelGGL((corr_bwd_kernel<D, PX, SEGX, NW, CC, V, MODE, true, NB>), grid, dim3(F::NT), 0, s,
                         x1, x2, g, gx1, gx2, B, C, H, W, tiles_x, cg, ep);
      return hipGetLastError();
    }
  }
  if (ep.mask) return hipErrorInvalidValue;  // 4-pixel runs only
  hipLaunchKernelGGL((corr_bwd_kernel<D, PX, SEGX, NW, CC, V, MODE, false, NB>), grid, dim3(F::NT), 0, s, x1,
                     x2, g, gx1, gx2, B, C, H, W, tiles_x, cg, ep);
  return hipGetLastError();
}

template <int D, int PX, int SEGX, int NW, int CC, int V, int NB>
hipError_t launch_bwd_v(const float* x1, const float* x2, const float* g, float* gx1, float* gx2,
                        int B, int C, int H, int W, hipStream_t s, BwdEpi ep) {
  if (gx1 && gx2)
    return launch_bwd_mode<D, PX, SEGX, NW, CC, V, 3, NB>(x1, x2, g, gx1, gx2, B, C, H, W, s, ep);
  hipError_t e = hipSuccess;
  if (gx1) e = launch_bwd_mode<D, PX, SEGX, NW, CC, V, 1, NB>(x1, x2, g, gx1, gx2, B, C, H, W, s, ep);
  if (e == hipSuccess && gx2)
    e = launch_bwd_mode<D, PX, SEGX, NW, CC, V, 2, NB>(x1, x2, g, gx1, gx2, B, C, H, W, s, ep);
  return e;
}

template <int D, int PX = 4, int SEGX = 8, int NW = 3, int CC = 4, int NB = 2>
hipError_t launch_bwd(const float* x1, const float* x2, const float* g, float* gx1, float* gx2,
                      int B, int C, int H, int W, hipStream_t s, BwdEpi ep) {
  if constexpr (Layout<PX, SEGX, D>::X4) {
    if (W % 4 == 0)
      return launch_bwd_v<D, PX, SEGX, NW, CC, 4, NB>(x1, x2, g, gx1, gx2, B, C, H, W, s, ep);
  }
  return launch_bwd_v<D, PX, SEGX, NW, CC, 1, NB>(x1, x2, g, gx1, gx2, B, C, H, W, s, ep);
}

// Tuning hook: usf_set_variant(1, i) forces candidate i for d=4: 0 = the
// two-image tile (the tile-rich levels' default), 1 = the four-image ring (the
// small grids' default). (CC = 8 and nine-wave forms were measured slower in
// rounds 1-4 -- profiles/ab_r01/bwd_variants_b16.txt -- and removed in round 6.)
hipError_t bwd_candidate_d4(int i, const float* x1, const float* x2, const float* g, float* gx1,
                            float* gx2, int B, int C, int H, int W, hipStream_t s, BwdEpi ep) {
  switch (i) {
    case 0: return launch_bwd<4, 4, 8, 3, 4>(x1, x2, g, gx1, gx2, B, C, H, W, s, ep);
    case 1: return launch_bwd<4, 4, 8, 3, 4, 4>(x1, x2, g, gx1, gx2, B, C, H, W, s, ep);
    default: return hipErrorInvalidValue;
  }
}
constexpr int kBwdCandidates = 2;

// Small grids take the 4-image ring: at most this many (tile, direction, sample)
// units. There every workgroup's channel loop is short (2-6 stages), and with
// three stages in flight behind the g slice the loop is one load round trip
// instead of a round trip per stage. Two runs at batch 16
// (profiles/ab_r04/corr_bwd_ring.json, warm / cold us): L0 19.0 -> 13.9 / 24.9
// -> 18.7, L1 18.7 -> 13.6 / 24.0 -> 17.2, L2 28.8 -> 25.4 / 32.9 -> 30.0,
// config 1 18.7 -> 14.4, config 2 41.1 -> 40.4. From L3 up (512 units and more)
// the ring's 60 KB cost a resident workgroup per CU: L3 38.9 -> 43.7, L4 74 -> 88.
// SURVEY config 2 (exactly 256 units) is faster on the two-image tile with 4
// channel groups: 39.0 / 43.6 vs 40.8 / 45.5 us warm / cold (round 6,
// profiles/ab_r06/corr_variants.json), so the ring takes fewer than 256.
#ifndef USF_BWD_RING_UNITS
#define USF_BWD_RING_UNITS 192
#endif

template <int D>
hipError_t bwd_dispatch(const float* x1, const float* x2, const float* g, float* gx1, float* gx2,
                        int B, int C, int H, int W, hipStream_t s, BwdEpi ep) {
  if (D == 4) {
    const int forced = variant_override(1);
    if (forced >= 0) return bwd_candidate_d4(forced, x1, x2, g, gx1, gx2, B, C, H, W, s, ep);
  }
  using T = BwdCfg<D, 4, 8, 3, 4, 1>;  // the default tile (32 x 8)
  const long units = (long)((W + T::TW - 1) / T::TW) * ((H + T::TH - 1) / T::TH) * B * ((gx1 && gx2) ? 2 : 1);
  if (units <= USF_BWD_RING_UNITS) return launch_bwd<D, 4, 8, 3, 4, 4>(x1, x2, g, gx1, gx2, B, C, H, W, s, ep);
  return launch_bwd<D>(x1, x2, g, gx1, gx2, B, C, H, W, s, ep);
}

// g_eff[b, k, p] = g[b * g_bstride + k * HW + p] * (act[...] > 0 ? 1 : slope):
// torch's leaky_relu_backward on the result (the in-place module's form), read
// from the concat-gradient slice and written dense for the backward kernel.
__global__ __launch_bounds__(256) void leaky_bwd_gather_kernel(const float* __restrict__ g,
                                                               const float* __restrict__ act,
                                                               long long gbs, float slope,
                                                               float* __restrict__ out, int K2,
                                                               int HW) {
  const long long per = (long long)K2 * HW;
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  const int b = blockIdx.y;
  if (i >= per) return;
  const float* gb = g + (size_t)b * gbs;
  const float* ab = act + (size_t)b * gbs;
  float* ob = out + (size_t)b * per;
  if (i + 3 < per && (gbs & 3) == 0) {
    const float4 gv = *reinterpret_cast<const float4*>(gb + i);
    const float4 av = *reinterpret_cast<const float4*>(ab + i);
    *reinterpret_cast<float4*>(ob + i) =
        make_float4(av.x > 0.f ? gv.x : gv.x * slope, av.y > 0.f ? gv.y : gv.y * slope,
                    av.z > 0.f ? gv.z : gv.z * slope, av.w > 0.f ? gv.w : gv.w * slope);
  } else {
    for (long long j = i; j < per && j < i + 4; ++j) ob[j] = ab[j] > 0.f ? gb[j] : gb[j] * slope;
  }
}

}  // namespace

hipError_t leaky_bwd_gather_launch(const float* g, const float* act, long long g_bstride, float slope,
                                   float* out, int B, int K2, int H, int W, hipStream_t s) {
  const long long per = (long long)K2 * H * W;
  const dim3 grid((unsigned)((per + 1023) / 1024), (unsigned)B);
  hipLaunchKernelGGL(leaky_bwd_gather_kernel, grid, dim3(256), 0, s, g, act, g_bstride, slope, out,
                     K2, H * W);
  return hipGetLastError();
}

namespace {
}  // namespace

static int g_variant[4] = {-1, -1, -1, -1};
int variant_override(int op) { return __atomic_load_n(&g_variant[op], __ATOMIC_RELAXED); }
int variant_count(int op) { return op == 0 ? kFwdCandidates : op == 1 ? kBwdCandidates : op == 2 ? 3 : 1; }
void set_variant_override(int op, int index) { __atomic_store_n(&g_variant[op], index, __ATOMIC_RELAXED); }

hipError_t corr_fwd_launch(const float* x1, const float* x2, float* out, int B, int C, int H,
                           int W, int d, hipStream_t s, FwdEpi ep, float* ws, long long ws_floats) {
  ep.part = nullptr;
  ep.groups = 1;
  switch (d) {
    case 1: return fwd_dispatch<1>(x1, x2, out, B, C, H, W, s, ep, ws, ws_floats);
    case 2: return fwd_dispatch<2>(x1, x2, out, B, C, H, W, s, ep, ws, ws_floats);
    case 3: return fwd_dispatch<3>(x1, x2, out, B, C, H, W, s, ep, ws, ws_floats);
    case 4: return fwd_dispatch<4>(x1, x2, out, B, C, H, W, s, ep, ws, ws_floats);
    default: return hipErrorInvalidValue;
  }
}

long long corr_fwd_workspace(int B, int C, int H, int W, int d) {
  FwdPlan p{2, 1};
  switch (d) {
    case 1: p = fwd_plan<1>(B, C, H, W); break;
    case 2: p = fwd_plan<2>(B, C, H, W); break;
    case 3: p = fwd_plan<3>(B, C, H, W); break;
    case 4: p = fwd_plan<4>(B, C, H, W); break;
    default: return 0;
  }
  if (p.groups <= 1) return 0;
  const long long K = 2 * d + 1;
  return (long long)p.groups * B * K * K * H * W;
}

// With act_out (no sign mask) the LeakyReLU derivative is a separate dense pass
// (leaky_bwd_gather_kernel): loading the activated output itself next to g in
// the prologue spilled 250-600 bytes past the 168-VGPR budget of the
// 3-waves/SIMD backward. The forward's sign mask (BwdEpi::mask, 6-18 extra
// VGPRs) is the fused form.

long long corr_act_mask_words(int B, int H, int W, int d) {
  if (d < 1 || d > 4) return 0;
  return (long long)B * (2 * d + 1) * H * ((W + 3) / 4);
}

hipError_t corr_bwd_launch(const float* x1, const float* x2, const float* gout, float* gx1,
                           float* gx2, int B, int C, int H, int W, int d, hipStream_t s, BwdEpi ep) {
  switch (d) {
    case 1: return bwd_dispatch<1>(x1, x2, gout, gx1, gx2, B, C, H, W, s, ep);
    case 2: return bwd_dispatch<2>(x1, x2, gout, gx1, gx2, B, C, H, W, s, ep);
    case 3: return bwd_dispatch<3>(x1, x2, gout, gx1, gx2, B, C, H, W, s, ep);
    case 4: return bwd_dispatch<4>(x1, x2, gout, gx1, gx2, B, C, H, W, s, ep);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace usf
