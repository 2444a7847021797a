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
// Layout: one lane per (output pixel, channel slice); consecutive lanes =
// consecutive x, so flow/out/gout accesses are coalesced; the 4 corner offsets
// and weights are computed once per lane and reused over its channels. grad_x uses fp32
// global atomics (global_atomic_add_f32, no CAS loop); grad_flow is a
// per-lane reduction over channels, written once (deterministic).
#include <algorithm>
#include <climits>

#include "interp_tap.h"
#include "usf_common.h"
#include "warp_tap.h"

namespace usf {
namespace {

// Work split: a 256-thread workgroup covers PXB = 256/CS consecutive pixels x
// CS channel slices (thread t: pixel t % PXB, channels t/PXB, t/PXB + CS, ...),
// so consecutive lanes stay on consecutive pixels (coalesced flow/out/gout and
// near-contiguous corner gathers / atomics) while small, channel-heavy pyramid
// levels still spread over many workgroups instead of looping C channels per
// lane.
// (pixel block, sample) of this workgroup; with USF_WARP_CHUNK > 0 runs of
// neighbouring pixel blocks (shared source rows / scatter targets) go to one XCD.
// 16 blocks per chunk: warp forward L4 14.3 -> 12.6 us, L2 8.7 -> 7.9 us; the
// backward and the splat are unchanged (profiles/ab_r01/warp_chunk_*.json)
#ifndef USF_WARP_CHUNK
#define USF_WARP_CHUNK 16
#endif
__device__ __forceinline__ void warp_block(int& bx, int& b) {
  if (USF_WARP_CHUNK > 0) {
    const int w = xcd_chunk(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y, USF_WARP_CHUNK);
    bx = w % gridDim.x;
    b = w / gridDim.x;
  } else {
    bx = blockIdx.x;
    b = blockIdx.y;
  }
}

#ifndef USF_WARP_FWD_PAIR
#define USF_WARP_FWD_PAIR 1  // forward L4 23.9 -> 13.1 us, L2 11.8 -> 7.5 us (profiles/ab_r04/warp_corner_pairs.json)
#endif
constexpr int kWarpOffNone = 0x7FFFFFF0;  // buffer offset past num_records: reads 0

// A corner row's two taps are neighbours in memory, so each row is ONE 8-byte
// load per channel (2 gathers per pixel and channel instead of 4: these
// gathers are bound by address processing, not bytes). The pair starts at
// lo = clamp(xw, 0, W - 2), so it never leaves the row where a corner is valid;
// at xw = -1 / W - 1 the valid corner is the pair's other half (swp). A row off
// the image gets an offset past num_records (reads 0; adding a channel base
// keeps it past). Needs W >= 2. Values of masked corners are zeroed, as before.
struct PairTap {
  unsigned on, os;  // byte offsets of the north / south pairs in a channel plane
  bool swp;
};
__device__ __forceinline__ PairTap pair_tap(const Tap& tp, int W) {
  PairTap q;
  const int lo = min(max(tp.xw, 0), W - 2);
  q.swp = tp.xw != lo;
  q.on = tp.m_nw || tp.m_ne ? 4u * (unsigned)(tp.yn * W + lo) : (unsigned)kWarpOffNone;
  q.os = tp.m_sw || tp.m_se ? 4u * (unsigned)((tp.yn + 1) * W + lo) : (unsigned)kWarpOffNone;
  return q;
}
__device__ __forceinline__ void pair_corners(__amdgpu_buffer_rsrc_t rs, const PairTap& q, const Tap& tp, unsigned cb,
                                             float& vnw, float& vne, float& vsw, float& vse) {
  using u32x2 = unsigned int __attribute__((ext_vector_type(2)));
  const u32x2 pn = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(q.on + cb), 0, 0);
  const u32x2 ps = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(q.os + cb), 0, 0);
  const float n0 = __uint_as_float(pn.x), n1 = __uint_as_float(pn.y);
  const float s0 = __uint_as_float(ps.x), s1 = __uint_as_float(ps.y);
  vnw = tp.m_nw ? (q.swp ? n1 : n0) : 0.f;
  vne = tp.m_ne ? (q.swp ? n0 : n1) : 0.f;
  vsw = tp.m_sw ? (q.swp ? s1 : s0) : 0.f;
  vse = tp.m_se ? (q.swp ? s0 : s1) : 0.f;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sample_rsrc(const float* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, bytes, 0x00020000);
}

// UP: the flow is the decoder's x2 upsampling of a coarse [B,2,H/2,W/2] flow
// (pwclite.py:299-302: flow = F.interpolate(flow * 2, ...), then
// flow_warp(x2, flow)), formed per pixel as upsample_fwd_kernel forms it
// (interp_tap.h: the same numbers) and written once to `up` ([B,2,H,W], by the
// first channel slice) beside the warp: one launch instead of two.
struct UpArgs {
  const float* coarse = nullptr;  // [B,2,h,w] dense
  float* up = nullptr;            // [B,2,H,W] dense
  int h = 0, w = 0;
  float sy = 0.f, sx = 0.f;       // ac_scale(h, H), ac_scale(w, W)
};
template <bool BORDER, int CS, bool UP = false>
__global__ __launch_bounds__(256) void warp_fwd_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ flow,
                                                       long long fbs, float* __restrict__ out,
                                                       int B, int C, int H, int W, UpArgs ua = {}) {
  constexpr int PXB = 256 / CS;
  const int HW = H * W;
  const int t = threadIdx.x;
  const int slice = t / PXB;
  int bx, b;
  warp_block(bx, b);
  const int p = bx * PXB + (t - slice * PXB);
  if (p >= HW) return;
  const int y = p / W, xx = p - y * W;
  float u, v;
  if constexpr (UP) {
    const Lin ty = lin_tap(y, ua.sy, ua.h), tx = lin_tap(xx, ua.sx, ua.w);
    const float* cb = ua.coarse + (size_t)b * 2 * ua.h * ua.w;
    u = up_bilinear(cb, ua.w, ty, tx, 2.f);
    v = up_bilinear(cb + ua.h * ua.w, ua.w, ty, tx, 2.f);
    if (slice == 0) {
      ua.up[(size_t)b * 2 * HW + p] = u;
      ua.up[(size_t)b * 2 * HW + HW + p] = v;
    }
  } else {
    const float* fb = flow + b * fbs;
    u = fb[p];
    v = fb[HW + p];
  }
  const Tap tp = make_tap(u, v, xx, y, H, W, BORDER);
  const float wnw = tp.s * tp.e, wne = tp.s * tp.w, wsw = tp.n * tp.e, wse = tp.n * tp.w;
  float* ob = out + (size_t)b * C * HW + p;
  if (USF_WARP_FWD_PAIR && W >= 2) {  // corner pairs (pair_tap)
    const PairTap q = pair_tap(tp, W);
    const auto rs = sample_rsrc(x + (size_t)b * C * HW, 4 * C * HW);
#pragma unroll 4
    for (int c = slice; c < C; c += CS) {
      float vnw, vne, vsw, vse;
      pair_corners(rs, q, tp, 4u * (unsigned)(c * HW), vnw, vne, vsw, vse);
      ob[(size_t)c * HW] = vnw * wnw + vne * wne + vsw * wsw + vse * wse;
    }
    return;
  }
  const float* xb = x + (size_t)b * C * HW;
#pragma unroll 4
  for (int c = slice; c < C; c += CS) {
    const float* xc = xb + (size_t)c * HW;
    const float vnw = xc[tp.o_nw], vne = xc[tp.o_ne], vsw = xc[tp.o_sw], vse = xc[tp.o_se];
    ob[(size_t)c * HW] = (tp.m_nw ? vnw : 0.f) * wnw + (tp.m_ne ? vne : 0.f) * wne +
                         (tp.m_sw ? vsw : 0.f) * wsw + (tp.m_se ? vse : 0.f) * wse;
  }
}

// grad_x scatter of one corner row (north: nw/ne, or south: sw/se) as a
// wave-level reduce-by-key. Consecutive lanes are consecutive pixels, so along
// a wave the target cells of a row are (nearly) monotone: lanes whose west
// corner hits the same cell (the flow compresses, or floor() of a coordinate
// that round-trips a hair below an integer) form a RUN, and a run's east cell
// is usually the next run's west cell. Each run is summed onto its last lane
// (log-step segmented scan over shuffles; the bound is the longest run in the
// wave, channel-invariant, so the common no-collision case costs 2 shuffles),
// the next run's head adds the previous run's east total into its west value,
// and only run tails issue atomics: ~1 global atomic per cell and channel, and
// no two lanes of one atomic instruction on the same address (those serialise).
struct RowRuns {
  int pos;      // lane's distance from its run head
  int maxlen;   // longest run in the wave (wave-uniform)
  bool tail;    // last lane of its run: issues the run's atomics
  bool take;    // run head that adds the previous run's east total (cells chain)
  bool give;    // run tail whose east total the next run's head takes
};

// key: row * (W + 1) + west column + 1, or a lane-unique negative value when the
// row is outside the image (no atomics); has_left/has_right: the neighbour lane
// exists and belongs to the same channel slice.
__device__ __forceinline__ RowRuns row_runs(int key, bool m_w, bool m_e, bool has_left,
                                            bool has_right) {
  const int lane = threadIdx.x & 63;
  const int kl = __shfl_up(key, 1);
  const bool left_me = __shfl_up(m_e ? 1 : 0, 1) != 0;
  const bool head = !(has_left && kl == key);
  const unsigned long long heads = __ballot(head);
  const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
  RowRuns r;
  r.pos = lane - (63 - __clzll(heads & upto));
  r.tail = lane == 63 || ((heads >> (lane + 1)) & 1ull) != 0;
  int m = r.pos;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o));
  r.maxlen = m + 1;
  r.take = head && has_left && m_w && left_me && kl + 1 == key;
  // every cross-lane read executes in all lanes (never behind a short-circuit:
  // a ds_bpermute from an inactive lane returns garbage)
  const bool right_takes = __shfl_down(r.take ? 1 : 0, 1) != 0;
  r.give = r.tail && has_right && right_takes;
  return r;
}

// segmented inclusive scan: lane l ends with the sum over [its run head, l]
__device__ __forceinline__ float run_sum(float v, const RowRuns& r) {
  for (int d = 1; d < r.maxlen; d <<= 1) {
    const float u = __shfl_up(v, d);
    if (r.pos >= d) v += u;
  }
  return v;
}

__device__ __forceinline__ void scatter_row(float* gc, int o_w, int o_e, bool m_w, bool m_e,
                                            float vw, float ve, const RowRuns& r) {
  const float se = run_sum(ve, r);
  const float lt = __shfl_up(se, 1);
  const float sw = run_sum(vw + (r.take ? lt : 0.f), r);
  if (r.tail) {
    if (m_w) atomicAdd(gc + o_w, sw);
    if (m_e && !r.give) atomicAdd(gc + o_e, se);
  }
}

// grad_x scatter over vertically adjacent PIXEL PAIRS: lane = (x, rows 2j and
// 2j + 1). When both pixels hit the same west column and consecutive corner
// rows (smooth flow), the first pixel's south row and the second's north row
// are the same cells: the lane adds the two contributions before the wave's
// reduce-by-key, so a pair scatters 3 corner rows instead of 4 (1.5 atomics per
// pixel and channel instead of 2). Lanes whose pixels do not line up keep a
// fourth row (issued only when some lane of the wave needs it).
__device__ __forceinline__ int row_key(bool ok, int row, int xw, int H, int W, int lane) {
  // keys alias nothing only for west columns in [-1, W-1]; elsewhere both cells are off-image
  return ok && xw >= -1 && xw < W && (unsigned)row < (unsigned)H ? row * (W + 1) + xw + 1 : -(lane + 2);
}

template <bool BORDER, bool WANT_GF, int CS>
__global__ __launch_bounds__(256) void warp_bwd_pair_kernel(const float* __restrict__ x,
                                                            const float* __restrict__ flow,
                                                            long long fbs,
                                                            const float* __restrict__ gout,
                                                            float* __restrict__ gx,
                                                            float* __restrict__ gflow, int B, int C,
                                                            int H, int W) {
  constexpr int PXB = 256 / CS;
  __shared__ float red[4][256];
  const int HW = H * W, H2 = (H + 1) >> 1;
  const int t = threadIdx.x;
  const int slice = t / PXB;
  const int pl = t - slice * PXB;
  const int lane = t & 63;
  int bx, b;
  warp_block(bx, b);
  const int pp = bx * PXB + pl;  // pair index over W x ceil(H / 2)
  const bool v0 = pp < W * H2;
  const int px = v0 ? pp % W : 0, py = v0 ? 2 * (pp / W) : 0;
  const bool v1 = v0 && py + 1 < H;
  const int p0 = py * W + px, p1 = v1 ? p0 + W : p0;
  const float* fb = flow + b * fbs;
  Tap t0{}, t1{};
  if (v0) t0 = make_tap(fb[p0], fb[HW + p0], px, py, H, W, BORDER);
  if (v1) t1 = make_tap(fb[p1], fb[HW + p1], px, py + 1, H, W, BORDER);
  if (!v0) t0.m_nw = t0.m_ne = t0.m_sw = t0.m_se = false;
  if (!v1) t1.m_nw = t1.m_ne = t1.m_sw = t1.m_se = false;
  const bool merged = v1 && t0.xw == t1.xw && t0.yn + 1 == t1.yn;
  const bool split = __any(v1 && !merged);  // wave-uniform
  const bool has_left = pl > 0 && lane != 0;
  const bool has_right = pl + 1 < PXB && lane != 63;
  const RowRuns r0 = row_runs(row_key(v0, t0.yn, t0.xw, H, W, lane), t0.m_nw, t0.m_ne, has_left, has_right);
  const RowRuns r1 = row_runs(row_key(v0, t0.yn + 1, t0.xw, H, W, lane), t0.m_sw, t0.m_se, has_left, has_right);
  const RowRuns r2 = row_runs(row_key(v1, t1.yn + 1, t1.xw, H, W, lane), t1.m_sw, t1.m_se, has_left, has_right);
  const bool n1 = v1 && !merged;  // the second pixel's north row on its own
  RowRuns r3{};
  if (split) r3 = row_runs(row_key(n1, t1.yn, t1.xw, H, W, lane), t1.m_nw && n1, t1.m_ne && n1, has_left, has_right);
  const float wnw0 = t0.s * t0.e, wne0 = t0.s * t0.w, wsw0 = t0.n * t0.e, wse0 = t0.n * t0.w;
  const float wnw1 = t1.s * t1.e, wne1 = t1.s * t1.w, wsw1 = t1.n * t1.e, wse1 = t1.n * t1.w;
  float dix0 = 0.f, diy0 = 0.f, dix1 = 0.f, diy1 = 0.f;
  const float* xb = x + (size_t)b * C * HW;
  const float* gb = gout + (size_t)b * C * HW;
  float* gxb = gx + (size_t)b * C * HW;
#pragma unroll 2
  for (int c = slice; c < C; c += CS) {
    const float go0 = v0 ? gb[(size_t)c * HW + p0] : 0.f;
    const float go1 = v1 ? gb[(size_t)c * HW + p1] : 0.f;
    float* gc = gxb + (size_t)c * HW;
    scatter_row(gc, t0.o_nw, t0.o_ne, t0.m_nw, t0.m_ne, go0 * wnw0, go0 * wne0, r0);
    const float vw = merged ? go0 * wsw0 + go1 * wnw1 : go0 * wsw0;
    const float ve = merged ? go0 * wse0 + go1 * wne1 : go0 * wse0;
    scatter_row(gc, t0.o_sw, t0.o_se, t0.m_sw, t0.m_se, vw, ve, r1);
    scatter_row(gc, t1.o_sw, t1.o_se, t1.m_sw, t1.m_se, go1 * wsw1, go1 * wse1, r2);
    if (split) scatter_row(gc, t1.o_nw, t1.o_ne, t1.m_nw && n1, t1.m_ne && n1, go1 * wnw1, go1 * wne1, r3);
    if (WANT_GF) {
      const float* xc = xb + (size_t)c * HW;
      if (v0) {
        const float a = t0.m_nw ? xc[t0.o_nw] : 0.f, e = t0.m_ne ? xc[t0.o_ne] : 0.f;
        const float s = t0.m_sw ? xc[t0.o_sw] : 0.f, d = t0.m_se ? xc[t0.o_se] : 0.f;
        dix0 += ((e - a) * t0.s + (d - s) * t0.n) * go0;
        diy0 += ((s - a) * t0.e + (d - e) * t0.w) * go0;
      }
      if (v1) {
        const float a = t1.m_nw ? xc[t1.o_nw] : 0.f, e = t1.m_ne ? xc[t1.o_ne] : 0.f;
        const float s = t1.m_sw ? xc[t1.o_sw] : 0.f, d = t1.m_se ? xc[t1.o_se] : 0.f;
        dix1 += ((e - a) * t1.s + (d - s) * t1.n) * go1;
        diy1 += ((s - a) * t1.e + (d - e) * t1.w) * go1;
      }
    }
  }
  if (!WANT_GF) return;
  if (CS > 1) {  // channel slices combined in a fixed order (deterministic)
    red[0][t] = dix0;
    red[1][t] = diy0;
    red[2][t] = dix1;
    red[3][t] = diy1;
    __syncthreads();
    if (slice != 0) return;
#pragma unroll
    for (int k = 1; k < CS; ++k) {
      dix0 += red[0][pl + k * PXB];
      diy0 += red[1][pl + k * PXB];
      dix1 += red[2][pl + k * PXB];
      diy1 += red[3][pl + k * PXB];
    }
  }
  float* gf = gflow + (size_t)b * 2 * HW;
  if (v0) {
    gf[p0] = ((dix0 * t0.mx) / (float)(W - 1)) * 2.0f;
    gf[HW + p0] = ((diy0 * t0.my) / (float)(H - 1)) * 2.0f;
  }
  if (v1) {
    gf[p1] = ((dix1 * t1.mx) / (float)(W - 1)) * 2.0f;
    gf[HW + p1] = ((diy1 * t1.my) / (float)(H - 1)) * 2.0f;
  }
}

// grad_x by a binned gather (the default with a caller workspace,
// usf_warp_bwd_ex_f32). Each source pixel p is filed, by the first pass, under
// its north-west corner cell nw(p) (a cell grid extended by one row and column
// above / left of the image, so corners at -1 are addressable): up to kBinSlots
// pixels per cell, the rest on an overflow list. The gather pass then gives
// every target cell q exactly the pixels filed under q, q - (0,1), q - (1,0)
// and q - (1,1) -- those whose NW, NE, SW or SE corner is q -- in a fixed order
// (corner, then pixel index), and writes gx[c][q] once: no float atomics, no
// zero fill, deterministic. Overflow pixels (more than kBinSlots sharing one
// cell: strongly compressive flow, or border clamping) are listed and added
// afterwards with float atomics.
constexpr int kBinSlots = 4;
constexpr int kBinTW = 32, kBinTH = 8;
// A parity word of the persistent workspace, read with a VECTOR buffer load:
// it then waits in vmcnt beside the kernel's first data loads instead of a
// scalar load that the kernel-argument wait serialises in front of them.
__device__ __forceinline__ int hdr_word(const int* hdr, int i) {
  const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(hdr), 0, 8, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b32(r, 4 * i, 0, 0);
}
// the parity at its use: kept in a VGPR (the asm hides its uniformity, so no
// v_readfirstlane is hoisted to the load), the wait sits here
__device__ __forceinline__ int at_use(int v) {
  asm volatile("" : "+v"(v));
  return v;
}  // target tile of the gather pass (warp_gx_bins_kernel)
struct BinArgs {
  int* cnt = nullptr;      // [B][(H+1)(W+1)] pixels filed per cell
  int* bins = nullptr;     // [B][(H+1)(W+1)][kBinSlots] source pixel (py << 16 | px)
  float* wbin = nullptr;   // [4][B (H+1)(W+1)][kBinSlots] slot weights per corner k (nw, ne, sw, se), 0 off-image:
                           // a target cell's gather reads one float4 (its 4 slots) per corner
  long long ncell = 0;     // B (H+1)(W+1)
  int* ovf = nullptr;      // [B * HW] overflow list: b * HW + p
  int* novf = nullptr;     // overflow list length
  int ovf_cap = 0;         // list capacity (B * HW): a pixel is listed at most once per call
  // Persistent workspace (BIN >= 2, usf_warp_bwd_persist_f32; see bwd_bins_persist):
  // two count buffers chosen by a parity word; overflow pixels either scattered
  // into a dense [B][C][H][W] buffer that the gather adds and re-zeroes per dirty
  // tile (BIN == 2), or listed for the overflow pass with two list lengths chosen
  // by the same parity (BIN == 3, the list form).
  int* hdr = nullptr;          // [0]: parity the filing pass reads, [1]: the gather's, [2 + par]: list lengths
  int* cnt2 = nullptr;         // 2 x [B (H+1)(W+1)] count buffers
  float* ovfgx = nullptr;      // [B][C][H][W] overflow contributions (zero between calls)
  unsigned* dirty = nullptr;   // [B][tiles]: bit g = channel group g of the gather has overflow to add
  unsigned dmask = 0;          // all groups' bits
  int tiles_x = 0, ntiles = 0; // the gather's 32 x 8 target tiles
};

// The per-pixel backward of one (pixel block bx, sample b): warp_bwd_kernel's
// body, also run by the small-level fused kernel (warp_bwd_fused_small_kernel)
template <bool BORDER, bool WANT_GX, bool WANT_GF, int CS, int BIN>
__device__ __forceinline__ void warp_bwd_body(const float* __restrict__ x, const float* __restrict__ flow,
                                              long long fbs, const float* __restrict__ gout,
                                              float* __restrict__ gx, float* __restrict__ gflow, int B, int C,
                                              int H, int W, const BinArgs& ba, int bx, int b) {
  constexpr int PXB = 256 / CS;
  __shared__ float red[2][256];
  // BIN >= 2: this call's count-buffer parity, loaded first so its latency
  // overlaps the flow loads (the filing atomics need both)
  const int par = BIN >= 2 ? hdr_word(ba.hdr, 0) : 0;
  const int HW = H * W;
  const int t = threadIdx.x;
  const int slice = t / PXB;
  const int pl = t - slice * PXB;
  const int p = bx * PXB + pl;
  bool valid = p < HW;
  float dix = 0.f, diy = 0.f;
  Tap tp{};
  if (valid) {
    const int y = p / W, xx = p - y * W;
    const float* fb = flow + b * fbs;
    const float u = fb[p], v = fb[HW + p];
    tp = make_tap(u, v, xx, y, H, W, BORDER);
  }
  if (!valid) tp.m_nw = tp.m_ne = tp.m_sw = tp.m_se = false;
  bool ovf = false;  // BIN == 2: p did not get a slot; its contributions go to ba.ovfgx
  if (BIN && slice == 0 && valid) {
    // file p under its north-west corner cell (see BinArgs); weights as the scatter forms them
    if (tp.m_nw || tp.m_ne || tp.m_sw || tp.m_se) {  // then xw in [-1, W), yn in [-1, H)
      const size_t cell = (size_t)b * (H + 1) * (W + 1) + (size_t)(tp.yn + 1) * (W + 1) + (tp.xw + 1);
      // BIN >= 2: this call's count buffer, the one the parity selects
      int* cnt = BIN >= 2 ? ba.cnt2 + (size_t)at_use(par) * ba.ncell : ba.cnt;
      const int slot = atomicAdd(cnt + cell, 1);
      if (slot < kBinSlots) {
        ba.bins[cell * kBinSlots + slot] = (p / W) << 16 | (p % W);  // (py, px): sorts as p
        float* wb = ba.wbin + cell * kBinSlots + slot;
        const size_t ks = (size_t)ba.ncell * kBinSlots;  // corner plane stride
        wb[0] = tp.m_nw ? tp.s * tp.e : 0.f;
        wb[ks] = tp.m_ne ? tp.s * tp.w : 0.f;
        wb[2 * ks] = tp.m_sw ? tp.n * tp.e : 0.f;
        wb[3 * ks] = tp.m_se ? tp.n * tp.w : 0.f;
      } else if (BIN == 1 || BIN == 3) {
        // scattered by the overflow pass; the capacity test only matters if the
        // per-call zero fill of novf / counts did not run (every pixel lists once).
        // BIN == 3: the list length the parity selects (the gather zeroes the other)
        const int o = atomicAdd(BIN == 3 ? ba.hdr + 2 + at_use(par) : ba.novf, 1);
        if (o < ba.ovf_cap) ba.ovf[o] = b * HW + p;
      } else {
        // persistent form: scattered below into ba.ovfgx; every gather workgroup of
        // the target tiles its corners touch adds that buffer (and re-zeroes it)
        ovf = true;
        const int qy[2] = {tp.yn, tp.yn + 1}, qx[2] = {tp.xw, tp.xw + 1};
        const bool mk[4] = {tp.m_nw, tp.m_ne, tp.m_sw, tp.m_se};
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (mk[k])
            ba.dirty[(size_t)b * ba.ntiles + (qy[k >> 1] / kBinTH) * ba.tiles_x + qx[k & 1] / kBinTW] = ba.dmask;
      }
    }
  }
  // handed to the gather, which flips hdr[0] for the next call (one writer: a
  // same-address store from every workgroup would queue on one L2 line)
  if (BIN >= 2 && t == 0 && linear_block() == 0) ba.hdr[1] = at_use(par);
  // grad_x: reduce-by-key over the wave per corner row (see scatter_row)
  RowRuns rn{}, rs{};
  if (WANT_GX) {
    const int lane = t & 63;
    const bool has_left = pl > 0 && lane != 0;
    const bool has_right = pl + 1 < PXB && lane != 63;
    // keys alias nothing only for west columns in [-1, W-1] (zeros padding can
    // put xw anywhere; outside that range both corners of the row are off-image)
    const bool vx = tp.xw >= -1 && tp.xw < W;
    const bool vyn = valid && vx && (unsigned)tp.yn < (unsigned)H;
    const bool vys = valid && vx && (unsigned)(tp.yn + 1) < (unsigned)H;
    const int kn = vyn ? tp.yn * (W + 1) + tp.xw + 1 : -(lane + 2);
    const int ks = vys ? (tp.yn + 1) * (W + 1) + tp.xw + 1 : -(lane + 2);
    rn = row_runs(kn, tp.m_nw, tp.m_ne, has_left, has_right);
    rs = row_runs(ks, tp.m_sw, tp.m_se, has_left, has_right);
  }
  {
    const float wnw = tp.s * tp.e, wne = tp.s * tp.w, wsw = tp.n * tp.e, wse = tp.n * tp.w;
    const float* xb = x + (size_t)b * C * HW;
    const float* gb = gout + (size_t)b * C * HW + (valid ? p : 0);
    float* gxb = WANT_GX ? gx + (size_t)b * C * HW : nullptr;
    // (corner-pair loads as in the forward measured no faster here: L4 56.9 vs
    // 54.5 us, profiles/ab_r04/warp_corner_pairs.json; the filing pass is not
    // gather-bound, so the build-time option was removed in round 5)
#pragma unroll 2
    for (int c = slice; c < C; c += CS) {
      const float go = valid ? gb[(size_t)c * HW] : 0.f;
      if (WANT_GX) {
        float* gc = gxb + (size_t)c * HW;
        scatter_row(gc, tp.o_nw, tp.o_ne, tp.m_nw, tp.m_ne, go * wnw, go * wne, rn);
        scatter_row(gc, tp.o_sw, tp.o_se, tp.m_sw, tp.m_se, go * wsw, go * wse, rs);
      }
      if (WANT_GF && valid) {
        const float* xc = xb + (size_t)c * HW;
        const float vnw = tp.m_nw ? xc[tp.o_nw] : 0.f;
        const float vne = tp.m_ne ? xc[tp.o_ne] : 0.f;
        const float vsw = tp.m_sw ? xc[tp.o_sw] : 0.f;
        const float vse = tp.m_se ? xc[tp.o_se] : 0.f;
        dix += ((vne - vnw) * tp.s + (vse - vsw) * tp.n) * go;
        diy += ((vsw - vnw) * tp.e + (vse - vne) * tp.w) * go;
      }
    }
  }
  if (BIN == 2) {
    // Overflow pixels (rare: strongly compressive flow, border piles) go to
    // ba.ovfgx with the reduce-by-key atomics. Only the filing lane knows its
    // pixel overflowed; the barrier sits after the channel loop, so no slice
    // ever waits for the filing atomics, and each slice then scatters its own
    // channels with its loads batched (no load round trip per channel).
    __shared__ unsigned char ovf_s[PXB];
    if (slice == 0) ovf_s[pl] = ovf;
    __syncthreads();
    const bool po = ovf_s[pl] != 0;
    if (__any(po)) {  // wave-uniform: every lane takes part in the shuffles
      const int lane = t & 63;
      const bool has_left = pl > 0 && lane != 0, has_right = pl + 1 < PXB && lane != 63;
      const bool vx = po && tp.xw >= -1 && tp.xw < W;
      const bool vyn = vx && (unsigned)tp.yn < (unsigned)H, vys = vx && (unsigned)(tp.yn + 1) < (unsigned)H;
      const RowRuns ron = row_runs(vyn ? tp.yn * (W + 1) + tp.xw + 1 : -(lane + 2), po && tp.m_nw, po && tp.m_ne,
                                   has_left, has_right);
      const RowRuns ros = row_runs(vys ? (tp.yn + 1) * (W + 1) + tp.xw + 1 : -(lane + 2), po && tp.m_sw,
                                   po && tp.m_se, has_left, has_right);
      const float wnw = tp.s * tp.e, wne = tp.s * tp.w, wsw = tp.n * tp.e, wse = tp.n * tp.w;
      const float* gp = gout + (size_t)b * C * HW + (po ? p : 0);
      // a wave-uniform loop (a wave may hold several slices): lane channel
      // c = base + slice + j * CS, masked past C, so every lane runs every shuffle
      constexpr int NB8 = 8;
      for (int base = 0; base < C; base += NB8 * CS) {
        float go[NB8];
#pragma unroll
        for (int j = 0; j < NB8; ++j) {
          const int c = base + slice + j * CS;
          go[j] = po && c < C ? gp[(size_t)c * HW] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < NB8; ++j) {
          const int c = base + slice + j * CS;
          const bool cv = po && c < C;
          float* oc = ba.ovfgx + ((size_t)b * C + min(c, C - 1)) * HW;
          scatter_row(oc, tp.o_nw, tp.o_ne, cv && tp.m_nw, cv && tp.m_ne, go[j] * wnw, go[j] * wne, ron);
          scatter_row(oc, tp.o_sw, tp.o_se, cv && tp.m_sw, cv && tp.m_se, go[j] * wsw, go[j] * wse, ros);
        }
      }
    }
  }
  if (WANT_GF) {
    if (CS > 1) {  // combine the channel slices in a fixed order (deterministic)
      red[0][t] = dix;
      red[1][t] = diy;
      __syncthreads();
      if (slice != 0) return;
#pragma unroll
      for (int k = 1; k < CS; ++k) {
        dix += red[0][pl + k * PXB];
        diy += red[1][pl + k * PXB];
      }
    }
    if (!valid) return;
    // grid grad, then norm_grid's autograd (DivBackward by (W-1), MulBackward by 2)
    const float ggx = dix * tp.mx, ggy = diy * tp.my;
    float* gf = gflow + (size_t)b * 2 * HW + p;
    gf[0] = (ggx / (float)(W - 1)) * 2.0f;
    gf[HW] = (ggy / (float)(H - 1)) * 2.0f;
  }
}

template <bool BORDER, bool WANT_GX, bool WANT_GF, int CS, int BIN = 0>
__global__ __launch_bounds__(256) void warp_bwd_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ flow,
                                                       long long fbs,
                                                       const float* __restrict__ gout,
                                                       float* __restrict__ gx,
                                                       float* __restrict__ gflow, int B, int C,
                                                       int H, int W, BinArgs ba = {}) {
  int bx, b;
  warp_block(bx, b);
  warp_bwd_body<BORDER, WANT_GX, WANT_GF, CS, BIN>(x, flow, fbs, gout, gx, gflow, B, C, H, W, ba, bx, b);
}

// The gather pass of the binned grad_x: thread = target cell q, channels
// [c0, c0 + cper) of sample b. For corner k (0 NW, 1 NE, 2 SW, 3 SE) the
// pixels filed under q - (k / 2, k % 2) are sorted by index (at most
// kBinSlots), and each channel sums weight * gout over them in that order.
// Slot loops run to the wave's largest count (uniform), so every register
// index is static.
constexpr int kGatherCH = 8;  // channels per pass of the binned gather
__device__ __forceinline__ void cswap(int& a, int& b) {
  const int lo = min(a, b), hi = max(a, b);
  a = lo;
  b = hi;
}
// Target tile of the gather pass: 32 x 8 cells (thread t: column t % 32, row
// t / 32); the box of all its source pixels (one per entry) is staged in LDS
// per pass of kGatherCH channels when it holds at most kBoxCap pixels
// (smooth flows: the tile shifted by the local flow, plus its spread), else
// the sources are read from global memory directly.
constexpr int kBoxW = 64, kBoxH = 16;  // staged box: rows of kBoxW floats (lane = column)

constexpr int kBoxCap = kBoxW * kBoxH;
// PM: 0 per-call workspace, 1 persistent with the dense overflow buffer, 2
// persistent list form (the overflow pass follows)
template <int PM = 0>
__global__ __launch_bounds__(256) void warp_gx_bins_kernel(const float* __restrict__ gout, BinArgs ba,
                                                           float* __restrict__ gx, int C, int H, int W,
                                                           int tiles_x, int cper) {
  static_assert(kBinSlots == 4, "sorting network for 4 slots");
  __shared__ float box[kGatherCH * kBoxCap];
  __shared__ int bb[4];  // source box: y min, y max, x min, x max
  const int HW = H * W, W1 = W + 1, E = (H + 1) * W1;
  const int t = threadIdx.x;
  const int ty0 = (blockIdx.x / tiles_x) * kBinTH, tx0 = (blockIdx.x % tiles_x) * kBinTW;
  const int qy = ty0 + t / kBinTW, qx = tx0 + t % kBinTW;
  const int b = blockIdx.y;
  const int c0 = blockIdx.z * cper, c1 = min(C, c0 + cper);
  const bool valid = qy < H && qx < W;
  const int qq = valid ? qy * W + qx : 0;
  // PERSIST: this call's count buffer is the one the filing pass's parity
  // selects; both buffers' counts are loaded beside the parity (no dependent
  // load before the gather's own), and the other buffer is zeroed at the end
  // for the next call, which reads the flipped parity
  constexpr bool PERSIST = PM > 0;
  const int par = PERSIST ? hdr_word(ba.hdr, 1) : 0;
  // both count buffers (2 x ncell ints < 2 GiB: capi.cpp bounds the shapes)
  const auto crs = __builtin_amdgcn_make_buffer_rsrc(PERSIST ? ba.cnt2 : ba.cnt, 0,
                                                     (int)(PERSIST ? 8 * ba.ncell : 4), 0x00020000);
  const unsigned dword = PM == 1 ? ba.dirty[(size_t)b * ba.ntiles + blockIdx.x] : 0u;
  if (t == 0) {
    bb[0] = INT_MAX; bb[1] = INT_MIN; bb[2] = INT_MAX; bb[3] = INT_MIN;
  }
  // entries: packed (py << 16 | px) of the sources filed under the four cells
  int pk[4][kBinSlots];
  float wk[4][kBinSlots];
  int nmax[4];
  int ylo = INT_MAX, yhi = INT_MIN, xlo = INT_MAX, xhi = INT_MIN;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const size_t cell = (size_t)b * E + (size_t)(qy - (k >> 1) + 1) * W1 + (qx - (k & 1) + 1);
    // count, slots and the slots' weights load together (slots 0 and 1
    // unconditionally: most cells hold at most two pixels)
    const size_t ce = valid ? cell : 0;
    int cn;
    if (PERSIST) {
      // both buffers' counts by buffer-load intrinsics: the compiler cannot fold
      // the parity select into one load's address (a load behind the parity load)
      const int ca = __builtin_amdgcn_raw_buffer_load_b32(crs, (int)(4 * ce), 0, 0);
      const int cb = __builtin_amdgcn_raw_buffer_load_b32(crs, (int)(4 * (ba.ncell + ce)), 0, 0);
      cn = at_use(par) ? cb : ca;
    } else {
      cn = ba.cnt[ce];
    }
    const int n = valid ? min(cn, kBinSlots) : 0;
    const int4 e4 = *reinterpret_cast<const int4*>(ba.bins + ce * kBinSlots);
    // the 4 slots' weights for this corner: one 16-byte load (corner-major layout)
    const float4 w4 = *reinterpret_cast<const float4*>(ba.wbin + ((size_t)k * ba.ncell + ce) * kBinSlots);
    float wv[kBinSlots] = {n > 0 ? w4.x : 0.f, n > 1 ? w4.y : 0.f, n > 2 ? w4.z : 0.f, n > 3 ? w4.w : 0.f};
    pk[k][0] = n > 0 ? e4.x : INT_MAX;
    pk[k][1] = n > 1 ? e4.y : INT_MAX;
    pk[k][2] = n > 2 ? e4.z : INT_MAX;
    pk[k][3] = n > 3 ? e4.w : INT_MAX;
    // sort the (pixel, weight) pairs by pixel: the summation order is fixed
    auto cs2 = [&](int i, int j) {
      const bool sw = pk[k][j] < pk[k][i];
      const int pi = pk[k][i], pj = pk[k][j];
      const float wi = wv[i], wj = wv[j];
      pk[k][i] = sw ? pj : pi; pk[k][j] = sw ? pi : pj;
      wv[i] = sw ? wj : wi; wv[j] = sw ? wi : wj;
    };
    cs2(0, 1); cs2(2, 3); cs2(0, 2); cs2(1, 3); cs2(1, 2);
#pragma unroll
    for (int j = 0; j < kBinSlots; ++j) {
      const bool has = j < n;
      const int py = pk[k][j] >> 16, px = pk[k][j] & 0xFFFF;
      wk[k][j] = wv[j];
      pk[k][j] = has ? (py << 16) | px : -1;  // empty slot: weight 0 at offset 0 (below)
      if (has) {
        ylo = min(ylo, py); yhi = max(yhi, py); xlo = min(xlo, px); xhi = max(xhi, px);
      }
    }
    int m = n;  // the wave's largest count for this corner
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o));
    nmax[k] = m;
  }
  // the workgroup's source box: wave reduction, then one LDS atomic per wave
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ylo = min(ylo, __shfl_xor(ylo, o)); yhi = max(yhi, __shfl_xor(yhi, o));
    xlo = min(xlo, __shfl_xor(xlo, o)); xhi = max(xhi, __shfl_xor(xhi, o));
  }
  __syncthreads();  // bb initialised
  if ((t & 63) == 0 && ylo <= yhi) {
    atomicMin(&bb[0], ylo); atomicMax(&bb[1], yhi); atomicMin(&bb[2], xlo); atomicMax(&bb[3], xhi);
  }
  __syncthreads();
  // box columns start on a 4-float boundary when rows are 16-byte aligned
  // (W % 4 == 0): every box quad is then one aligned 16-byte load inside its row
  const bool w4 = (W & 3) == 0;
  const int by0 = bb[0], bx0 = w4 ? bb[2] & ~3 : bb[2];
  const bool any = bb[0] <= bb[1];  // no entry in the workgroup: bb keeps INT_MAX / INT_MIN
  const int bh = any ? bb[1] - by0 + 1 : 0, bw = any ? bb[3] - bx0 + 1 : 0;  // (no signed overflow)
  const bool staged = any && bh <= kBoxH && bw <= kBoxW;  // workgroup-uniform
  const float* gb = gout + (size_t)b * C * HW;
  float* gq = gx + (size_t)b * C * HW + qq;
  // per entry: offset into the staged box, or the plane offset
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int j = 0; j < kBinSlots; ++j) {
      // empty slots read element 0 (always staged, finite) with weight 0: the
      // box is written only where sources lie, so anything else may be stale LDS
      const int py = pk[k][j] >> 16, px = pk[k][j] & 0xFFFF;
      pk[k][j] = pk[k][j] < 0 ? 0 : staged ? (py - by0) * kBoxW + (px - bx0) : py * W + px;
    }
  // kGatherCH channels per pass with independent accumulators
  // thread = (box row t / 16, column quad t % 16): kBoxH x kBoxW = 256 quads,
  // so each thread stages at most one quad per channel, all loads in flight together
  static_assert(kBoxH * kBoxW == 4 * 256, "one quad per thread and channel");
  const int ry = t >> 4, rx = (t & 15) * 4;
  const bool stager = staged && ry < bh && rx < bw;
  const float* ssrc = gb + (size_t)(by0 + ry) * W + bx0 + rx;
  auto stage_loads = [&](int c, float4 (&v)[kGatherCH]) {
    if (w4) {
#pragma unroll
      for (int u = 0; u < kGatherCH; ++u)
        v[u] = c + u < c1 ? *reinterpret_cast<const float4*>(ssrc + (size_t)(c + u) * HW)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
    } else {  // unaligned rows: dword loads, none past the row
      const int nv = min(4, W - (bx0 + rx));
#pragma unroll
      for (int u = 0; u < kGatherCH; ++u) {
        const float* sc = ssrc + (size_t)min(c + u, c1 - 1) * HW;
        const bool ok = c + u < c1;
        v[u] = make_float4(ok ? sc[0] : 0.f, ok && nv > 1 ? sc[1] : 0.f, ok && nv > 2 ? sc[2] : 0.f,
                           ok && nv > 3 ? sc[3] : 0.f);
      }
    }
  };
  // (Loading the next pass's quads into registers before this pass's sums --
  // round 6 -- took the kernel from 116 to 144 VGPRs, 4 to 3 workgroups per CU:
  // KITTI L4 in-step 64.9 vs 57.4 us, profiles/ab_r06/warp_gather_prefetch.json.)
  for (int c = c0; c < c1; c += kGatherCH) {
    float acc[kGatherCH];
#pragma unroll
    for (int u = 0; u < kGatherCH; ++u) acc[u] = 0.f;
    if (staged) {
      __syncthreads();  // the previous pass is done with the box
      if (stager) {
        float4 v[kGatherCH];
        stage_loads(c, v);
#pragma unroll
        for (int u = 0; u < kGatherCH; ++u) *reinterpret_cast<float4*>(&box[u * kBoxCap + ry * kBoxW + rx]) = v[u];
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int j = 0; j < kBinSlots; ++j)
          if (j < nmax[k]) {
#pragma unroll
            for (int u = 0; u < kGatherCH; ++u) acc[u] = fmaf(wk[k][j], box[u * kBoxCap + pk[k][j]], acc[u]);
          }
    } else {
      int co[kGatherCH];  // channel offsets, clamped into the group (extra lanes load, never store)
#pragma unroll
      for (int u = 0; u < kGatherCH; ++u) co[u] = min(c + u, c1 - 1) * HW;
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int j = 0; j < kBinSlots; ++j)
          if (j < nmax[k]) {
            const float* src = gb + pk[k][j];
#pragma unroll
            for (int u = 0; u < kGatherCH; ++u) acc[u] = fmaf(wk[k][j], src[co[u]], acc[u]);
          }
    }
    const bool dirty = PM == 1 && ((dword >> blockIdx.z) & 1u);  // overflow to add for this channel group
    if (dirty && valid) {
      // the overflow pixels' contributions (scattered by the filing pass), then
      // re-zeroed: this workgroup is their only reader
      float* oq = ba.ovfgx + (size_t)b * C * HW + qq;
#pragma unroll
      for (int u = 0; u < kGatherCH; ++u)
        if (c + u < c1) {
          acc[u] += oq[(size_t)(c + u) * HW];
          oq[(size_t)(c + u) * HW] = 0.f;
        }
    }
    if (valid) {
#pragma unroll
      for (int u = 0; u < kGatherCH; ++u)
        if (c + u < c1) gq[(size_t)(c + u) * HW] = acc[u];
    }
  }
  if (PERSIST) {
    if (PM == 1 && ((dword >> blockIdx.z) & 1u) && t == 0)
      atomicAnd(ba.dirty + (size_t)b * ba.ntiles + blockIdx.x, ~(1u << blockIdx.z));
    const int pv = at_use(par);  // (a VGPR: no scalar copy of the parity is hoisted to its load)
    int* other = ba.cnt2 + (size_t)(1 - pv) * ba.ncell;
    const long long nth = (long long)gridDim.x * gridDim.y * gridDim.z * 256;
    for (long long i = (long long)linear_block() * 256 + t; i < ba.ncell; i += nth) other[i] = 0;
    if (linear_block() == 0 && t == 0) {
      ba.hdr[0] = 1 - pv;
      // list form: the next call's list length (this call's overflow pass reads hdr[2 + pv])
      if (PM == 2) ba.hdr[2 + (1 - pv)] = 0;
    }
  }
}

// Small levels (H*W <= kSmallPx, (H+1)(W+1) <= kSmallCells: KITTI L1,
// Sintel L1): the whole backward in ONE launch with no workspace. Workgroups
// [0, B*GA) each bin their sample's source pixels in LDS -- counts per
// north-west cell (LDS atomics), an exclusive scan, placement, then every
// cell's pixels sorted by index -- and gather grad_x for their channel group
// (every target cell sums its four corner cells' pixels in that fixed order:
// the binned gather's numbers wherever a cell holds at most kBinSlots pixels,
// and deterministic beyond, with no overflow atomics). The remaining
// workgroups run the filing pass's grad_flow (warp_bwd_body, the same channel
// slices as bin_pass picks, so the same numbers) without the filing.
// (At 832 pixels -- KITTI L2 -- the per-workgroup binning and the longer gather
// loop made it slower than the two-launch form: 33.6 vs 22.7 us in the step,
// while L1 went 19.3 -> 14.7 us; profiles/ab_r06/warp_small_fused.json.)
constexpr int kSmallPx = 512, kSmallCells = 768, kSmallCH = 8;
template <bool BORDER>
__device__ void warp_gx_small(const float* __restrict__ flow, long long fbs, const float* __restrict__ gout,
                              float* __restrict__ gx, int C, int H, int W, int b, int c0, int c1) {
  __shared__ float s_w[kSmallPx], s_n[kSmallPx];
  __shared__ int s_cell[kSmallPx], s_list[kSmallPx];
  __shared__ unsigned char s_m[kSmallPx];
  __shared__ int s_start[kSmallCells + 1], s_fill[kSmallCells];
  __shared__ int s_part[256];
  const int HW = H * W, W1 = W + 1, E = (H + 1) * W1;
  const int t = threadIdx.x, lane = t & 63;
  for (int i = t; i <= E; i += 256) s_start[i] = 0;
  __syncthreads();
  // taps of every source pixel of sample b; count per north-west cell
  const float* fb = flow + (size_t)b * fbs;
  for (int p = t; p < HW; p += 256) {
    const int y = p / W, xx = p - y * W;
    const Tap tp = make_tap(fb[p], fb[HW + p], xx, y, H, W, BORDER);
    s_w[p] = tp.w;
    s_n[p] = tp.n;
    s_m[p] = (unsigned char)((tp.m_nw ? 1 : 0) | (tp.m_ne ? 2 : 0) | (tp.m_sw ? 4 : 0) | (tp.m_se ? 8 : 0));
    int cell = -1;
    if (tp.m_nw || tp.m_ne || tp.m_sw || tp.m_se) {  // then xw in [-1, W), yn in [-1, H)
      cell = (tp.yn + 1) * W1 + tp.xw + 1;
      atomicAdd(&s_start[cell], 1);
    }
    s_cell[p] = cell;
  }
  __syncthreads();
  // exclusive scan of the counts: K consecutive cells per thread, the 256
  // thread totals scanned by wave 0 (4 per lane)
  const int K = (E + 255) / 256;
  const int i0 = min(E, t * K), i1 = min(E, i0 + K);
  int loc = 0;
  for (int i = i0; i < i1; ++i) loc += s_start[i];
  s_part[t] = loc;
  __syncthreads();
  if (t < 64) {
    const int a0 = s_part[4 * t], a1 = s_part[4 * t + 1], a2 = s_part[4 * t + 2], a3 = s_part[4 * t + 3];
    const int sum = a0 + a1 + a2 + a3;
    int inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(inc, o);
      if (lane >= o) inc += v;
    }
    const int ex = inc - sum;
    s_part[4 * t] = ex;
    s_part[4 * t + 1] = ex + a0;
    s_part[4 * t + 2] = ex + a0 + a1;
    s_part[4 * t + 3] = ex + a0 + a1 + a2;
  }
  __syncthreads();
  int run = s_part[t];
  for (int i = i0; i < i1; ++i) {
    const int c = s_start[i];
    s_start[i] = run;
    s_fill[i] = run;
    run += c;
  }
  if (i0 < i1 && i1 == E) s_start[E] = run;  // the thread holding the last cell
  __syncthreads();
  for (int p = t; p < HW; p += 256) {
    const int cell = s_cell[p];
    if (cell >= 0) s_list[atomicAdd(&s_fill[cell], 1)] = p;
  }
  __syncthreads();
  // each cell's pixels in index order (placement order is the atomics')
  for (int c = t; c < E; c += 256) {
    const int a = s_start[c], z = s_start[c + 1];
    for (int i = a + 1; i < z; ++i) {
      const int v = s_list[i];
      int j = i - 1;
      while (j >= a && s_list[j] > v) {
        s_list[j + 1] = s_list[j];
        --j;
      }
      s_list[j + 1] = v;
    }
  }
  __syncthreads();
  const float* gb = gout + (size_t)b * C * HW;
  float* gxb = gx + (size_t)b * C * HW;
  for (int q = t; q < HW; q += 256) {
    const int qy = q / W, qx = q - qy * W;
    for (int c = c0; c < c1; c += kSmallCH) {
      float acc[kSmallCH];
#pragma unroll
      for (int u = 0; u < kSmallCH; ++u) acc[u] = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int cell = (qy - (k >> 1) + 1) * W1 + (qx - (k & 1) + 1);
        const int a = s_start[cell], z = s_start[cell + 1];
        for (int i = a; i < z; ++i) {
          const int p = s_list[i];
          const int m = s_m[p];
          const float w = s_w[p], n = s_n[p];
          const float e = 1.0f - w, sn = 1.0f - n;  // as make_tap forms them
          // corner k's weight as the filing pass writes it (BinArgs::wbin)
          const float wt = k == 0 ? ((m & 1) ? sn * e : 0.f)
                           : k == 1 ? ((m & 2) ? sn * w : 0.f)
                           : k == 2 ? ((m & 4) ? n * e : 0.f)
                                    : ((m & 8) ? n * w : 0.f);
          const float* src = gb + p;
#pragma unroll
          for (int u = 0; u < kSmallCH; ++u)
            acc[u] = fmaf(wt, src[(size_t)min(c + u, c1 - 1) * HW], acc[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < kSmallCH; ++u)
        if (c + u < c1) gxb[(size_t)(c + u) * HW + q] = acc[u];
    }
  }
}

template <bool BORDER, int CS, bool WANT_GF>
__global__ __launch_bounds__(256) void warp_bwd_fused_small_kernel(const float* __restrict__ x,
                                                                   const float* __restrict__ flow, long long fbs,
                                                                   const float* __restrict__ gout,
                                                                   float* __restrict__ gx, float* __restrict__ gflow,
                                                                   int B, int C, int H, int W, int GA, int cper,
                                                                   int nbx) {
  const int i = blockIdx.x;
  const int nA = B * GA;
  if (i < nA) {
    const int b = i / GA, g = i - (i / GA) * GA;
    warp_gx_small<BORDER>(flow, fbs, gout, gx, C, H, W, b, g * cper, min(C, (g + 1) * cper));
    return;
  }
  if constexpr (WANT_GF) {
    const int j = i - nA;
    warp_bwd_body<BORDER, false, true, CS, 0>(x, flow, fbs, gout, nullptr, gflow, B, C, H, W, BinArgs{}, j % nbx,
                                              j / nbx);
  }
}

// Overflow pixels of the binned grad_x add their four corner contributions
// with float atomics after the gather pass. A wave takes 64 consecutive list
// entries (lane = entry) x kOvfCh channels: consecutive entries mostly share
// their cell (the list fills in pixel order, and a border-clamped strip piles
// onto one edge cell per row), so runs of lanes with the same cell are summed
// by a segmented shuffle scan (row_runs / run_sum, as the scatter does) and
// only run tails issue the atomics. With one atomic per (entry, channel,
// corner) the large-shift field took 111 us at L4 on same-address atomics.
// The loop bound is the device-side list length: nothing overflowed, nothing runs.
constexpr int kOvfCh = 4;

// Device-side error flags of this code object (usf_device_errors() reads and
// clears them; USF_SYNC_CHECK=1 reports them after every launch). A list
// length past its capacity can only come from stale per-call state (the
// capacity is one entry per pixel); the pass then stops at the capacity and
// raises USF_DEVERR_WARP_OVERFLOW instead of silently dropping entries.
__device__ int g_dev_errors = 0;

template <bool BORDER>
__global__ __launch_bounds__(256) void warp_gx_ovf_kernel(const float* __restrict__ flow, long long fbs,
                                                          const float* __restrict__ gout, BinArgs ba,
                                                          float* __restrict__ gx, int C, int H, int W) {
  const int HW = H * W;
  // list form: the length this call's filing pass counted (parity hdr[1])
  const int listed = ba.hdr ? ba.hdr[2 + (ba.hdr[1] & 1)] : *ba.novf;
  const int n = min(listed, ba.ovf_cap);
  const int lane = threadIdx.x & 63;
  if ((listed < 0 || listed > ba.ovf_cap) && blockIdx.x == 0 && threadIdx.x == 0)
    atomicOr(&g_dev_errors, USF_DEVERR_WARP_OVERFLOW);
  const int ngrp = (C + kOvfCh - 1) / kOvfCh;
  const long long units = (long long)((n + 63) / 64) * ngrp;  // (64-entry chunk, channel group)
  const long long nw = (long long)gridDim.x * (blockDim.x >> 6);
  for (long long u = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); u < units; u += nw) {
    const int chunk = (int)(u / ngrp), grp = (int)(u - (long long)chunk * ngrp);
    const int e = chunk * 64 + lane;
    const bool valid = e < n;
    const int ent = valid ? ba.ovf[e] : 0;
    const int b = ent / HW, p = ent - b * HW;
    const int y = p / W, xx = p - y * W;
    const float* fb = flow + b * fbs;
    Tap tp = make_tap(fb[p], fb[HW + p], xx, y, H, W, BORDER);
    if (!valid) tp.m_nw = tp.m_ne = tp.m_sw = tp.m_se = false;
    // run key: the entry's north-west cell (same cell = same four corners and masks)
    const bool any = tp.m_nw || tp.m_ne || tp.m_sw || tp.m_se;
    const int key = any ? (int)(((long long)b * (H + 1) + tp.yn + 1) * (W + 1) + tp.xw + 1) : -(lane + 2);
    const int kl = __shfl_up(key, 1);
    const bool head = lane == 0 || kl != key;
    const unsigned long long heads = __ballot(head);
    const unsigned long long upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    RowRuns r;
    r.pos = lane - (63 - __clzll(heads & upto));
    r.tail = lane == 63 || ((heads >> (lane + 1)) & 1ull) != 0;
    int m = r.pos;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o));
    r.maxlen = m + 1;
    const float wv[4] = {tp.s * tp.e, tp.s * tp.w, tp.n * tp.e, tp.n * tp.w};
    const bool mk[4] = {tp.m_nw, tp.m_ne, tp.m_sw, tp.m_se};
    const int ok[4] = {tp.o_nw, tp.o_ne, tp.o_sw, tp.o_se};
    const int c0 = grp * kOvfCh;
    float go[kOvfCh];  // all of the group's loads in flight together
#pragma unroll
    for (int j = 0; j < kOvfCh; ++j)
      go[j] = valid && c0 + j < C ? gout[((size_t)b * C + c0 + j) * HW + p] : 0.f;
#pragma unroll
    for (int j = 0; j < kOvfCh; ++j) {
      const size_t bs = ((size_t)b * C + c0 + j) * HW;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float v = run_sum(go[j] * wv[k], r);  // every lane takes part (shuffles)
        if (r.tail && mk[k] && c0 + j < C) atomicAdd(gx + bs + ok[k], v);
      }
    }
  }
}

// Channel slices per workgroup: the smallest CS in {1,4,16,64} giving >= 1024
// workgroups (8 XCDs x 32 CUs x 4), capped by C.
inline int pick_cs(int B, int C, int HW) {
  const int opts[4] = {1, 4, 16, 64};
  for (int i = 0; i < 4; ++i) {
    const int cs = opts[i];
    const long blocks = (long)B * ((HW + 256 / cs - 1) / (256 / cs));
    if (blocks >= 1024 || cs >= C || i == 3) return cs;
  }
  return 64;
}

template <bool BORDER, int CS, bool UP>
void fwd_launch_cs(const float* x, const float* flow, long long fbs, float* out, int B, int C,
                   int H, int W, hipStream_t s, const UpArgs& ua) {
  const dim3 grid((unsigned)((H * W + 256 / CS - 1) / (256 / CS)), (unsigned)B), block(256);
  hipLaunchKernelGGL((warp_fwd_kernel<BORDER, CS, UP>), grid, block, 0, s, x, flow, fbs, out, B, C, H,
                     W, ua);
}

template <bool BORDER, bool UP = false>
void fwd_launch_pad(const float* x, const float* flow, long long fbs, float* out, int B, int C,
                    int H, int W, hipStream_t s, const UpArgs& ua = {}) {
  switch (pick_cs(B, C, H * W)) {
    case 1: fwd_launch_cs<BORDER, 1, UP>(x, flow, fbs, out, B, C, H, W, s, ua); break;
    case 4: fwd_launch_cs<BORDER, 4, UP>(x, flow, fbs, out, B, C, H, W, s, ua); break;
    case 16: fwd_launch_cs<BORDER, 16, UP>(x, flow, fbs, out, B, C, H, W, s, ua); break;
    default: fwd_launch_cs<BORDER, 64, UP>(x, flow, fbs, out, B, C, H, W, s, ua); break;
  }
}

template <bool BORDER, int CS>
void bwd_launch_cs(const float* x, const float* flow, long long fbs, const float* gout, float* gx,
                   float* gflow, int B, int C, int H, int W, hipStream_t s) {
  const dim3 grid((unsigned)((H * W + 256 / CS - 1) / (256 / CS)), (unsigned)B), block(256);
  if (gx && gflow)
    hipLaunchKernelGGL((warp_bwd_kernel<BORDER, true, true, CS>), grid, block, 0, s, x, flow, fbs, gout, gx, gflow,
                       B, C, H, W);
  else if (gx)
    hipLaunchKernelGGL((warp_bwd_kernel<BORDER, true, false, CS>), grid, block, 0, s, x, flow, fbs, gout, gx, gflow,
                       B, C, H, W);
  else
    hipLaunchKernelGGL((warp_bwd_kernel<BORDER, false, true, CS>), grid, block, 0, s, x, flow, fbs, gout, gx, gflow,
                       B, C, H, W);
}

template <bool BORDER, int CS>
void bwd_pair_cs(const float* x, const float* flow, long long fbs, const float* gout, float* gx,
                 float* gflow, int B, int C, int H, int W, hipStream_t s) {
  const int pairs = W * ((H + 1) / 2);
  const dim3 grid((unsigned)((pairs + 256 / CS - 1) / (256 / CS)), (unsigned)B), block(256);
  if (gflow)
    hipLaunchKernelGGL((warp_bwd_pair_kernel<BORDER, true, CS>), grid, block, 0, s, x, flow, fbs, gout, gx,
                       gflow, B, C, H, W);
  else
    hipLaunchKernelGGL((warp_bwd_pair_kernel<BORDER, false, CS>), grid, block, 0, s, x, flow, fbs, gout, gx,
                       gflow, B, C, H, W);
}

// Binned-gather workspace: overflow count and cell counts (zeroed per call),
// cell slots with their weights, overflow list.
// Zero fill as a kernel on the launch stream. Under stream capture a
// hipMemsetAsync here raced the kernel launched after it on graph replay (the
// binned backward's cell counts were still stale when the filing pass began:
// tests/test_gpu_graph_replay.py), so every fill the library needs is this
// launch, ordered like its other kernels in eager and captured streams alike.
// p 16-byte aligned (torch allocations, the workspace layout), bytes % 4 == 0.
// 16-byte stores from the first 16-byte boundary on; the dwords before it (a
// caller pointer through the C ABI need only be 4-byte aligned) and the tail
// are stored singly.
__global__ __launch_bounds__(256) void zero_fill_kernel(unsigned* __restrict__ p, long long n, int head) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  if (t < head && t < n) p[t] = 0u;
  unsigned* q = p + head;
  const long long m = n - head;
  const long long stride = (long long)gridDim.x * 256 * 4;
  for (long long i = t * 4; i < m; i += stride) {
    if (i + 4 <= m) {
      *reinterpret_cast<uint4*>(q + i) = make_uint4(0u, 0u, 0u, 0u);
    } else {
      for (long long j = i; j < m; ++j) q[j] = 0u;
    }
  }
}

hipError_t zero_fill(void* p, size_t bytes, hipStream_t s) {
  const long long n = (long long)(bytes / 4);
  if (n <= 0) return hipSuccess;
  const int head = (int)std::min<long long>(((16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15) / 4, n);
  const long long blocks = std::min<long long>((n + 1023) / 1024, 4096);
  hipLaunchKernelGGL(zero_fill_kernel, dim3((unsigned)blocks), dim3(256), 0, s, static_cast<unsigned*>(p), n,
                     head);
  return hipGetLastError();
}

struct BinLayout {
  long long novf_off, cnt_off, bins_off, wbin_off, ovf_off, total;
};
inline BinLayout bin_layout(int B, int H, int W) {
  auto al = [](long long v) { return (v + 255) & ~255LL; };
  const long long E = (long long)B * (H + 1) * (W + 1), P = (long long)B * H * W;
  BinLayout L;
  L.novf_off = 0;
  L.cnt_off = 256;
  L.bins_off = al(L.cnt_off + 4 * E);
  L.wbin_off = al(L.bins_off + 4 * E * kBinSlots);
  L.ovf_off = al(L.wbin_off + 16 * E * kBinSlots);
  L.total = al(L.ovf_off + 4 * P);
  return L;
}

template <bool BORDER, int CS, int BINM>
void bin_pass_cs(const float* x, const float* flow, long long fbs, const float* gout, float* gflow, int B,
                 int C, int H, int W, BinArgs ba, hipStream_t s) {
  const dim3 grid((unsigned)((H * W + 256 / CS - 1) / (256 / CS)), (unsigned)B), block(256);
  if (gflow)
    hipLaunchKernelGGL((warp_bwd_kernel<BORDER, false, true, CS, BINM>), grid, block, 0, s, x, flow, fbs,
                       gout, nullptr, gflow, B, C, H, W, ba);
  else
    hipLaunchKernelGGL((warp_bwd_kernel<BORDER, false, false, CS, BINM>), grid, block, 0, s, x, flow,
                       fbs, gout, nullptr, nullptr, B, C, H, W, ba);
}

// The gather pass's grid: 32 x 8 target tiles x B x channel groups (multiples
// of kGatherCH) until ~512 workgroups. Round 2 chose ~1024 against ~2048 by
// warm replay (L3: 43.3 -> 38.3 us, profiles/ab_r02/warp_bins_ab.json); round
// 6 compared 512 / 1024 / 2048 by in-step time inside the training step
// (tools/instep_ab.py, profiles/ab_r06/instep_knobs.json): at KITTI L4 (896
// tiles x samples) one group of 32 channels instead of two of 16 reads each
// cell's metadata once: 58.3 vs 62.8 us; L1-L3 within the run-to-run spread.
#ifndef USF_BIN_WGS
#define USF_BIN_WGS 512
#endif
struct GatherGrid {
  int tiles_x, ntiles, cper, zg;
};
inline GatherGrid gather_grid(int B, int C, int H, int W) {
  GatherGrid g;
  g.tiles_x = (W + kBinTW - 1) / kBinTW;
  g.ntiles = g.tiles_x * ((H + kBinTH - 1) / kBinTH);
  const long units = (long)g.ntiles * B;
  const int chunks = (C + kGatherCH - 1) / kGatherCH;
  const int want = (int)std::min<long>(chunks, std::max<long>(1, (USF_BIN_WGS + units - 1) / units));
  g.cper = ((chunks + want - 1) / want) * kGatherCH;
  g.zg = (C + g.cper - 1) / g.cper;
  return g;
}

// filing pass, with grad_flow's channel slices chosen as for the scatter: the
// smallest slice count in {4, 16, 64} that still gives >= 768 workgroups
// (profiles/ab_r02/warp_bins_ab.json: L2 31.5 -> 26.7 us with 16 instead of 4;
// L3/L4 keep 4, L1 64)
inline int bin_cs(int B, int C, int H, int W) {
  int cs = 64;
  for (const int o : {4, 16}) {
    if ((long)B * ((H * W + 256 / o - 1) / (256 / o)) >= 768) {
      cs = o;
      break;
    }
  }
  while (cs > 4 && cs > C) cs >>= 2;  // no more slices than channels (4 at least)
  return cs;
}

template <bool BORDER, int BINM>
void bin_pass(const float* x, const float* flow, long long fbs, const float* gout, float* gflow, int B, int C,
              int H, int W, BinArgs ba, hipStream_t s) {
  int cs = bin_cs(B, C, H, W);
#ifdef USF_BIN_CS
  cs = USF_BIN_CS;  // A/B builds only
#endif
  switch (cs) {
    case 1: bin_pass_cs<BORDER, 1, BINM>(x, flow, fbs, gout, gflow, B, C, H, W, ba, s); break;
    case 4: bin_pass_cs<BORDER, 4, BINM>(x, flow, fbs, gout, gflow, B, C, H, W, ba, s); break;
    case 16: bin_pass_cs<BORDER, 16, BINM>(x, flow, fbs, gout, gflow, B, C, H, W, ba, s); break;
    default: bin_pass_cs<BORDER, 64, BINM>(x, flow, fbs, gout, gflow, B, C, H, W, ba, s); break;
  }
}

// The small-level fused backward (warp_bwd_fused_small_kernel): false when the
// shape is not small enough (or grad_x is not wanted).
template <bool BORDER, int CS>
void small_fused_cs(const float* x, const float* flow, long long fbs, const float* gout, float* gx, float* gflow,
                    int B, int C, int H, int W, hipStream_t s) {
  const int HW = H * W;
  const int GA = (C + kSmallCH - 1) / kSmallCH;
  const int nbx = (HW + 256 / CS - 1) / (256 / CS);
  const unsigned nblk = (unsigned)(B * GA + (gflow ? B * nbx : 0));
  if (gflow)
    hipLaunchKernelGGL((warp_bwd_fused_small_kernel<BORDER, CS, true>), dim3(nblk), dim3(256), 0, s, x, flow, fbs,
                       gout, gx, gflow, B, C, H, W, GA, kSmallCH, nbx);
  else
    hipLaunchKernelGGL((warp_bwd_fused_small_kernel<BORDER, CS, false>), dim3(nblk), dim3(256), 0, s, x, flow, fbs,
                       gout, gx, gflow, B, C, H, W, GA, kSmallCH, nbx);
}
#ifndef USF_WARP_SMALL_FUSED
#define USF_WARP_SMALL_FUSED 1
#endif
template <bool BORDER>
bool bwd_small_fused(const float* x, const float* flow, long long fbs, const float* gout, float* gx, float* gflow,
                     int B, int C, int H, int W, hipStream_t s) {
  if (!USF_WARP_SMALL_FUSED || !gx || H * W > kSmallPx || (long long)(H + 1) * (W + 1) > kSmallCells) return false;
  switch (bin_cs(B, C, H, W)) {  // grad_flow's slices as the filing pass picks them (the same numbers)
    case 4: small_fused_cs<BORDER, 4>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s); break;
    case 16: small_fused_cs<BORDER, 16>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s); break;
    default: small_fused_cs<BORDER, 64>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s); break;
  }
  return true;
}

// grad_x by the binned gather (+ grad_flow in the filing pass); see BinArgs.
template <bool BORDER>
void bwd_bins(const float* x, const float* flow, long long fbs, const float* gout, float* gx, float* gflow, int B,
              int C, int H, int W, void* ws, hipStream_t s) {
  const BinLayout L = bin_layout(B, H, W);
  char* w = static_cast<char*>(ws);
  BinArgs ba;
  ba.cnt = reinterpret_cast<int*>(w + L.cnt_off);
  ba.bins = reinterpret_cast<int*>(w + L.bins_off);
  ba.wbin = reinterpret_cast<float*>(w + L.wbin_off);
  ba.ncell = (long long)B * (H + 1) * (W + 1);
  ba.ovf = reinterpret_cast<int*>(w + L.ovf_off);
  ba.novf = reinterpret_cast<int*>(w + L.novf_off);
  ba.ovf_cap = B * H * W;
  (void)zero_fill(w, (size_t)(L.cnt_off + 4LL * B * (H + 1) * (W + 1)), s);  // novf + counts
  bin_pass<BORDER, 1>(x, flow, fbs, gout, gflow, B, C, H, W, ba, s);
  const GatherGrid gg = gather_grid(B, C, H, W);
  hipLaunchKernelGGL(warp_gx_bins_kernel<0>, dim3((unsigned)gg.ntiles, (unsigned)B, (unsigned)gg.zg), dim3(256),
                     0, s, gout, ba, gx, C, H, W, gg.tiles_x, gg.cper);
  // overflow pixels (few or none for smooth flows): listed, scattered with atomics
  hipLaunchKernelGGL((warp_gx_ovf_kernel<BORDER>), dim3(256), dim3(256), 0, s, flow, fbs, gout, ba, gx, C, H, W);
}

// Persistent-workspace form (usf_warp_bwd_persist_f32): TWO launches, no fill
// and no overflow pass. The workspace is zero when first handed over and is
// left reusable: the filing pass counts into the buffer the parity word
// selects, the gather zeroes the other one and flips the parity for the next
// call (each word has one writer kernel and is read by the other, so launch
// order on the stream is the only synchronisation: graph-replay safe).
// Overflow pixels (more than kBinSlots per cell) are scattered by the filing
// pass into a dense [B][C][H][W] buffer with the same reduce-by-key atomics as
// the old overflow pass, and every target tile they touch is marked dirty for
// each gather channel group; that group's workgroup adds the buffer into its
// sums and zeroes it again (its only reader). The summation order of a cell
// is the bins' (fixed), then the overflow sum, as in the four-launch form.
//
// List form (levels above USF_PERSIST_LIST_PIXELS pixels): THREE launches, the
// overflow handled as in the four-launch form -- listed by the filing pass and
// added by warp_gx_ovf_kernel after the gather -- with the list length kept
// under the same parity as the counts (hdr[2 + par]; the gather zeroes the
// other one), so no zero fill runs. At KITTI L4 (64 x 208) the dense buffer's
// overflow path cost the filing pass and the gather ~7 us each for 48 overflow
// pixels of the training step's own flow (tools/warp_flow_capture.py +
// tools/warp_form_prof.py: 24.3 + 27.7 us vs 17.3 + 21.0 + 6.0 + 4.8 us for the
// four-launch form), while the four-launch form paid its zero fill.
#ifndef USF_PERSIST_LIST_PIXELS
#define USF_PERSIST_LIST_PIXELS 8192
#endif
inline bool persist_list(int H, int W) { return (long long)H * W > USF_PERSIST_LIST_PIXELS; }
struct BinLayout2 {
  long long hdr_off, cnt_off, bins_off, wbin_off, dirty_off, ovfgx_off, ovf_off, total;
  bool list;
};
inline BinLayout2 bin_layout2(int B, int C, int H, int W) {
  auto al = [](long long v) { return (v + 255) & ~255LL; };
  const long long E = (long long)B * (H + 1) * (W + 1);
  const GatherGrid gg = gather_grid(B, C, H, W);
  BinLayout2 L;
  L.list = persist_list(H, W);
  L.hdr_off = 0;
  L.cnt_off = 256;
  L.bins_off = al(L.cnt_off + 2 * 4 * E);
  L.wbin_off = al(L.bins_off + 4 * E * kBinSlots);
  if (L.list) {  // the overflow list (one entry per pixel at most)
    L.dirty_off = L.ovfgx_off = -1;
    L.ovf_off = al(L.wbin_off + 16 * E * kBinSlots);
    L.total = al(L.ovf_off + 4LL * B * H * W);
  } else {
    L.ovf_off = -1;
    L.dirty_off = al(L.wbin_off + 16 * E * kBinSlots);
    L.ovfgx_off = al(L.dirty_off + 4LL * B * gg.ntiles);
    L.total = al(L.ovfgx_off + 4LL * B * C * H * W);
  }
  return L;
}

template <bool BORDER>
void bwd_bins_persist(const float* x, const float* flow, long long fbs, const float* gout, float* gx, float* gflow,
                      int B, int C, int H, int W, void* ws, hipStream_t s) {
  const BinLayout2 L = bin_layout2(B, C, H, W);
  const GatherGrid gg = gather_grid(B, C, H, W);
  char* w = static_cast<char*>(ws);
  BinArgs ba;
  ba.hdr = reinterpret_cast<int*>(w + L.hdr_off);
  ba.cnt2 = reinterpret_cast<int*>(w + L.cnt_off);
  ba.bins = reinterpret_cast<int*>(w + L.bins_off);
  ba.wbin = reinterpret_cast<float*>(w + L.wbin_off);
  ba.ncell = (long long)B * (H + 1) * (W + 1);
  ba.tiles_x = gg.tiles_x;
  ba.ntiles = gg.ntiles;
  const dim3 ggrid((unsigned)gg.ntiles, (unsigned)B, (unsigned)gg.zg);
  if (L.list) {
    ba.ovf = reinterpret_cast<int*>(w + L.ovf_off);
    ba.ovf_cap = B * H * W;
    bin_pass<BORDER, 3>(x, flow, fbs, gout, gflow, B, C, H, W, ba, s);
    hipLaunchKernelGGL(warp_gx_bins_kernel<2>, ggrid, dim3(256), 0, s, gout, ba, gx, C, H, W, gg.tiles_x, gg.cper);
    hipLaunchKernelGGL((warp_gx_ovf_kernel<BORDER>), dim3(256), dim3(256), 0, s, flow, fbs, gout, ba, gx, C, H, W);
    return;
  }
  ba.dirty = reinterpret_cast<unsigned*>(w + L.dirty_off);
  ba.ovfgx = reinterpret_cast<float*>(w + L.ovfgx_off);
  ba.dmask = gg.zg >= 32 ? ~0u : (1u << gg.zg) - 1u;
  bin_pass<BORDER, 2>(x, flow, fbs, gout, gflow, B, C, H, W, ba, s);
  hipLaunchKernelGGL(warp_gx_bins_kernel<1>, ggrid, dim3(256), 0, s, gout, ba, gx, C, H, W, gg.tiles_x, gg.cper);
}

// grad_x paths (usf_set_variant(2, v), benchmarking only): 0 = the lane-merged
// scatter (fp32 atomics, one lane per pixel), 1 = the same over vertically
// adjacent pixel pairs, 2 = the binned gather (needs a workspace); -1 = the
// built-in choice: with a workspace the binned gather (persistent or per
// call), without one the pair scatter at large levels and the per-pixel
// scatter elsewhere. (Round 6 removed the measured-slower paths that no default
// took: the LDS-aggregated tile scatter, the small-radius gather with its
// outlier scatter, the small-image one-launch kernel and the forced channel
// splits -- docs/EXPERIMENTS.md keeps their measurements.)
template <bool BORDER>
void bwd_launch_pad(const float* x, const float* flow, long long fbs, const float* gout,
                    float* gx, float* gflow, int B, int C, int H, int W, hipStream_t s,
                    void* ws = nullptr, long long ws_bytes = 0, bool persist = false) {
  const int v = variant_override(2);
  // small levels: one launch, no workspace (the persistent one stays untouched)
  if ((v < 0 || v == 2) && bwd_small_fused<BORDER>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s)) return;
  if (persist) {  // usf_warp_bwd_persist_f32 (capi.cpp checked the workspace size and C)
    if (gx && (v < 0 || v == 2)) {
      bwd_bins_persist<BORDER>(x, flow, fbs, gout, gx, gflow, B, C, H, W, ws, s);
      return;
    }
    // grad_flow only, or a forced scatter: the per-call dispatch WITHOUT the
    // workspace (its layout differs; the persistent state stays untouched)
    ws = nullptr;
    ws_bytes = 0;
  }
  // binned gather (default with a workspace; usf_set_variant(2, 2) requires one)
  // (bin entries pack (py, px) into 16-bit halves)
  if (gx && ws && ws_bytes >= bin_layout(B, H, W).total && (v < 0 || v == 2) && H < 32768 && W < 65536) {
    bwd_bins<BORDER>(x, flow, fbs, gout, gx, gflow, B, C, H, W, ws, s);
    return;
  }
  // the scatters accumulate into gx: zero it first (gx is overwritten either way)
  if (gx) (void)zero_fill(gx, sizeof(float) * (size_t)B * C * H * W, s);
  // pixel-pair scatter: variant 1, and the default for large levels. Measured at
  // batch 16 (profiles/ab_r01/warp_pairs.json, grad_x + grad_flow): L4 67 vs
  // 82 us (zero flow), 50 vs 60 (constant sub-pixel), equal for +-2 / +-8 px
  // fields; at L2 it halves the workgroups and is slower (52 vs 31 us).
  const bool pair_default = v < 0 && (long)W * ((H + 1) / 2) >= 4096 && C >= 4;
  if (gx && (v == 1 || pair_default)) {
    const long runs64p = (long)B * ((W * ((H + 1) / 2) + 63) / 64);
    const int csp = (runs64p >= 96 && C >= 4) ? 4 : pick_cs(B, C, W * ((H + 1) / 2));
    switch (csp) {
      case 1: bwd_pair_cs<BORDER, 1>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s); break;
      case 4: bwd_pair_cs<BORDER, 4>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s); break;
      case 16: bwd_pair_cs<BORDER, 16>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s); break;
      default: bwd_pair_cs<BORDER, 64>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s); break;
    }
    return;
  }
  // Per-pixel scatter: CS = 4 (each wave one 64-pixel run of one channel, so an
  // atomic wave-instruction covers one contiguous row piece) whenever that still
  // gives ~100 workgroups; narrower pixel runs (CS 16/64) only for the tiny
  // levels. tools/wbench.py: L3 48 vs 61 us, L2 35 vs 57 us (CS 4 vs 16); L1
  // (8x26, 32 workgroups at CS 4) 26 us at CS 64 vs 44 us.
  const long runs64 = (long)B * ((H * W + 63) / 64);
  const int cs = (runs64 >= 96 && C >= 4) ? 4 : pick_cs(B, C, H * W);
  switch (cs) {
    case 1: bwd_launch_cs<BORDER, 1>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s); break;
    case 4: bwd_launch_cs<BORDER, 4>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s); break;
    case 16: bwd_launch_cs<BORDER, 16>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s); break;
    default: bwd_launch_cs<BORDER, 64>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s); break;
  }
}

// ----------------------------------------------------------- occlusion --
// Forward bilinear splat of unit mass (warp_utils.py:26-94 get_corresponding_map,
// used by get_occu_mask_backward :120-126): source pixel p of sample b lands at
// (x, y) = (px + u, py + v) (ABS: (u, v) are absolute coordinates already) and
// adds (1-|x-cx|)(1-|y-cy|) to each of its 4 integer neighbours (cx, cy) that
// lies inside the image, with cx in {x0 = floor(x), x0 + 1}, computed in the
// reference's fp32 order (contraction off). Same reduce-by-key scatter as the
// warp's grad_x (lanes = consecutive source pixels): ~2 atomics per pixel.
template <bool ABS>
__global__ __launch_bounds__(256) void splat_kernel(const float* __restrict__ flow, long long fbs,
                                                    float* __restrict__ map, int H, int W) {
#pragma clang fp contract(off)
  const int HW = H * W;
  const int t = threadIdx.x;
  const int lane = t & 63;
  int bx, b;
  warp_block(bx, b);
  const int p = bx * 256 + t;
  const bool valid = p < HW;
  float x = 0.f, y = 0.f;
  if (valid) {
    const float* fb = flow + b * fbs;
    const int py = p / W, px = p - py * W;
    x = ABS ? fb[p] : (float)px + fb[p];
    y = ABS ? fb[HW + p] : (float)py + fb[HW + p];
  }
  const float fx = floorf(x), fy = floorf(y);
  const float fx1 = fx + 1.f, fy1 = fy + 1.f;
  const float wm1 = (float)(W - 1), hm1 = (float)(H - 1);
  // corner inside the image <=> clamp(c, 0, size-1) == c (the reference's test)
  const bool vx0 = fx >= 0.f && fx <= wm1, vx1 = fx1 >= 0.f && fx1 <= wm1;
  const bool vy0 = valid && fy >= 0.f && fy <= hm1, vy1 = valid && fy1 >= 0.f && fy1 <= hm1;
  const float ax0 = 1.f - fabsf(x - fx), ax1 = 1.f - fabsf(x - fx1);
  const float ay0 = 1.f - fabsf(y - fy), ay1 = 1.f - fabsf(y - fy1);
  // integer corner indices, saturated so far-away targets cannot overflow
  const int xi = fx < -1.f ? -2 : (fx > wm1 ? W : (int)fx);
  const int yi = fy < -1.f ? -2 : (fy > hm1 ? H : (int)fy);
  const bool kx = xi >= -1 && xi < W;  // keys alias nothing only for x0 in [-1, W-1]
  const int kn = (vy0 && kx) ? yi * (W + 1) + xi + 1 : -(lane + 2);
  const int ks = (vy1 && kx) ? (yi + 1) * (W + 1) + xi + 1 : -(lane + 2);
  const bool has_left = lane != 0, has_right = lane != 63;
  const bool m_nw = vx0 && vy0, m_ne = vx1 && vy0, m_sw = vx0 && vy1, m_se = vx1 && vy1;
  const RowRuns rn = row_runs(kn, m_nw, m_ne, has_left, has_right);
  const RowRuns rs = row_runs(ks, m_sw, m_se, has_left, has_right);
  const int o_nw = m_nw || m_ne ? yi * W + xi : 0;
  const int o_sw = m_sw || m_se ? (yi + 1) * W + xi : 0;
  float* mb = map + (size_t)b * HW;
  scatter_row(mb, o_nw, o_nw + 1, m_nw, m_ne, ax0 * ay0, ax1 * ay0, rn);
  scatter_row(mb, o_sw, o_sw + 1, m_sw, m_se, ax0 * ay1, ax1 * ay1, rs);
}

// The splat over vertically adjacent pixel pairs (as warp_bwd_pair_kernel): a
// lane owns rows 2j and 2j + 1 of one column; when both land on the same west
// column and consecutive (unsaturated) corner rows, the shared row's four
// weights are added in the lane and the pair scatters 3 rows instead of 4.
struct SplatTap {
  int xi, yi;
  bool m_nw, m_ne, m_sw, m_se, kx, ky;  // ky: yi in [-1, H-1] (not saturated)
  float ax0, ax1, ay0, ay1;
};
template <bool ABS>
__device__ __forceinline__ SplatTap splat_tap(const float* __restrict__ fb, int p, int px, int py, bool valid,
                                              int H, int W) {
#pragma clang fp contract(off)
  const int HW = H * W;
  float x = 0.f, y = 0.f;
  if (valid) {
    x = ABS ? fb[p] : (float)px + fb[p];
    y = ABS ? fb[HW + p] : (float)py + fb[HW + p];
  }
  SplatTap s;
  const float fx = floorf(x), fy = floorf(y);
  const float fx1 = fx + 1.f, fy1 = fy + 1.f;
  const float wm1 = (float)(W - 1), hm1 = (float)(H - 1);
  const bool vx0 = fx >= 0.f && fx <= wm1, vx1 = fx1 >= 0.f && fx1 <= wm1;
  const bool vy0 = valid && fy >= 0.f && fy <= hm1, vy1 = valid && fy1 >= 0.f && fy1 <= hm1;
  s.ax0 = 1.f - fabsf(x - fx);
  s.ax1 = 1.f - fabsf(x - fx1);
  s.ay0 = 1.f - fabsf(y - fy);
  s.ay1 = 1.f - fabsf(y - fy1);
  s.xi = fx < -1.f ? -2 : (fx > wm1 ? W : (int)fx);
  s.yi = fy < -1.f ? -2 : (fy > hm1 ? H : (int)fy);
  s.kx = s.xi >= -1 && s.xi < W;
  s.ky = valid && s.yi >= -1 && s.yi < H;
  s.m_nw = vx0 && vy0;
  s.m_ne = vx1 && vy0;
  s.m_sw = vx0 && vy1;
  s.m_se = vx1 && vy1;
  return s;
}

template <bool ABS>
__global__ __launch_bounds__(256) void splat_pair_kernel(const float* __restrict__ flow, long long fbs,
                                                         float* __restrict__ map, int H, int W) {
#pragma clang fp contract(off)
  const int HW = H * W, H2 = (H + 1) >> 1;
  const int t = threadIdx.x;
  const int lane = t & 63;
  int bx, b;
  warp_block(bx, b);
  const int pp = bx * 256 + t;
  const bool v0 = pp < W * H2;
  const int px = v0 ? pp % W : 0, py = v0 ? 2 * (pp / W) : 0;
  const bool v1 = v0 && py + 1 < H;
  const float* fb = flow + b * fbs;
  const int p0 = py * W + px;
  const SplatTap s0 = splat_tap<ABS>(fb, p0, px, py, v0, H, W);
  const SplatTap s1 = splat_tap<ABS>(fb, v1 ? p0 + W : p0, px, py + 1, v1, H, W);
  const bool merged = v1 && s0.kx && s0.ky && s1.ky && s0.xi == s1.xi && s0.yi + 1 == s1.yi;
  const bool split = __any(v1 && !merged);
  const bool has_left = lane != 0, has_right = lane != 63;
  auto key = [&](const SplatTap& s, int row, bool rowok) {
    return rowok && s.kx ? row * (W + 1) + s.xi + 1 : -(lane + 2);
  };
  // rows: yi (north, valid iff its corners' row is in the image) and yi + 1
  const RowRuns r0 = row_runs(key(s0, s0.yi, v0 && s0.yi >= 0 && s0.yi < H), s0.m_nw, s0.m_ne, has_left, has_right);
  const RowRuns r1 = row_runs(key(s0, s0.yi + 1, v0 && s0.yi + 1 >= 0 && s0.yi + 1 < H), s0.m_sw, s0.m_se,
                              has_left, has_right);
  const RowRuns r2 = row_runs(key(s1, s1.yi + 1, v1 && s1.yi + 1 >= 0 && s1.yi + 1 < H), s1.m_sw, s1.m_se,
                              has_left, has_right);
  const bool own1 = v1 && !merged;
  RowRuns r3{};
  if (split)
    r3 = row_runs(key(s1, s1.yi, own1 && s1.yi >= 0 && s1.yi < H), s1.m_nw && own1, s1.m_ne && own1,
                  has_left, has_right);
  float* mb = map + (size_t)b * HW;
  const int o0 = s0.yi * W + s0.xi, o1 = s1.yi * W + s1.xi;
  const int on0 = s0.m_nw || s0.m_ne ? o0 : 0, os0 = s0.m_sw || s0.m_se ? o0 + W : 0;
  const int on1 = s1.m_nw || s1.m_ne ? o1 : 0, os1 = s1.m_sw || s1.m_se ? o1 + W : 0;
  scatter_row(mb, on0, on0 + 1, s0.m_nw, s0.m_ne, s0.ax0 * s0.ay0, s0.ax1 * s0.ay0, r0);
  const float vw = merged ? s0.ax0 * s0.ay1 + s1.ax0 * s1.ay0 : s0.ax0 * s0.ay1;
  const float ve = merged ? s0.ax1 * s0.ay1 + s1.ax1 * s1.ay0 : s0.ax1 * s0.ay1;
  scatter_row(mb, os0, os0 + 1, s0.m_sw, s0.m_se, vw, ve, r1);
  scatter_row(mb, os1, os1 + 1, s1.m_sw, s1.m_se, s1.ax0 * s1.ay1, s1.ax1 * s1.ay1, r2);
  if (split) scatter_row(mb, on1, on1 + 1, s1.m_nw && own1, s1.m_ne && own1, s1.ax0 * s1.ay0, s1.ax1 * s1.ay0, r3);
}

// occ = clamp(map, 0, 1) < th ? 1 : 0 (get_occu_mask_backward :124-126); in
// place (occ == map), or (REZERO) from a persistent map that is zeroed as read
template <bool REZERO>
__global__ __launch_bounds__(256) void occ_threshold_kernel(float* m, float* occ, long long n, float th) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float v = m[i];
  if (REZERO) m[i] = 0.f;
  occ[i] = fminf(fmaxf(v, 0.f), 1.f) < th ? 1.f : 0.f;
}

// Both directions of a with_bk loss at once (usf_occ_vis_pair_persist_f32):
// the splat map is interleaved [B][2][H][W] (half j = 0: the splat of
// flow12 = top[:, :2], j = 1: of flow21 = top[:, 2:]), and the threshold pass
// writes the visibility masks the loss uses, 1 - occ, direction-major:
// vis[0][b] = 1 - occ(flow21) (flow_loss.py:102 vis_mask1), vis[1][b] =
// 1 - occ(flow12) (:103 vis_mask2), each a contiguous [B,1,H,W]; the map is
// re-zeroed as read (its only reader).
__global__ __launch_bounds__(256) void occ_vis_pair_kernel(float* __restrict__ m, float* __restrict__ vis, int HW,
                                                           int B, float th) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long n = 2LL * B * HW;
  if (i >= n) return;
  const int b2 = (int)(i / HW), p = (int)(i - (long long)b2 * HW);
  const int b = b2 >> 1, j = b2 & 1;
  const float v = m[i];
  m[i] = 0.f;
  const float occ = fminf(fmaxf(v, 0.f), 1.f) < th ? 1.f : 0.f;
  vis[((long long)(1 - j) * B + b) * HW + p] = 1.f - occ;
}

}  // namespace

int device_errors(hipStream_t s, bool clear) {
  int v = 0;
  if (hipStreamSynchronize(s) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_dev_errors), sizeof(int)) != hipSuccess) return -1;
  if (clear && v != 0) {
    const int z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dev_errors), &z, sizeof(int)) != hipSuccess) return -1;
  }
  return v;
}

hipError_t warp_fwd_launch(const float* x, const float* flow, long long fbs, float* out, int B,
                           int C, int H, int W, int pad_mode, hipStream_t s) {
  if (pad_mode == 1)
    fwd_launch_pad<true>(x, flow, fbs, out, B, C, H, W, s);
  else
    fwd_launch_pad<false>(x, flow, fbs, out, B, C, H, W, s);
  return hipGetLastError();
}

hipError_t warp_fwd_up_launch(const float* x, const float* coarse, float* up, float* out, int B, int C, int H, int W,
                              int pad_mode, hipStream_t s) {
  UpArgs ua;
  ua.coarse = coarse;
  ua.up = up;
  ua.h = H / 2;
  ua.w = W / 2;
  ua.sy = ac_scale(ua.h, H);
  ua.sx = ac_scale(ua.w, W);
  if (pad_mode == 1)
    fwd_launch_pad<true, true>(x, nullptr, 0, out, B, C, H, W, s, ua);
  else
    fwd_launch_pad<false, true>(x, nullptr, 0, out, B, C, H, W, s, ua);
  return hipGetLastError();
}

hipError_t warp_bwd_launch(const float* x, const float* flow, long long fbs, const float* gout,
                           float* gx, float* gflow, int B, int C, int H, int W, int pad_mode,
                           hipStream_t s, void* ws, long long ws_bytes, bool persist) {
  if (!gx && !gflow) return hipSuccess;
  if (pad_mode == 1)
    bwd_launch_pad<true>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s, ws, ws_bytes, persist);
  else
    bwd_launch_pad<false>(x, flow, fbs, gout, gx, gflow, B, C, H, W, s, ws, ws_bytes, persist);
  return hipGetLastError();
}

namespace {
// Persistent-workspace audit (USF_SYNC_CHECK=1 only, after the call's own
// launches): any nonzero word where the next call expects zero raises
// USF_DEVERR_WORKSPACE_DIRTY, so a faulted or interrupted call cannot
// silently poison the calls of that shape that follow.
__global__ __launch_bounds__(256) void zero_check_kernel(const unsigned* __restrict__ p, long long n) {
  bool bad = false;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    bad |= p[i] != 0u;
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(&g_dev_errors, USF_DEVERR_WORKSPACE_DIRTY);
}
// the warp backward's next count buffer is the one the parity word selects
__global__ __launch_bounds__(256) void cnt_check_kernel(const int* __restrict__ hdr, const unsigned* __restrict__ cnt2,
                                                        long long ncell, bool list) {
  const int par = hdr[0];
  bool bad = par != 0 && par != 1;
  if (list && blockIdx.x == 0 && threadIdx.x == 0) bad |= hdr[2 + (par & 1)] != 0;  // the next list length
  const unsigned* c = cnt2 + (size_t)(par & 1) * ncell;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < ncell; i += (long long)gridDim.x * 256)
    bad |= c[i] != 0u;
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(&g_dev_errors, USF_DEVERR_WORKSPACE_DIRTY);
}
}  // namespace

hipError_t zero_check_launch(const void* p, long long bytes, hipStream_t s) {
  const long long n = bytes / 4;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(zero_check_kernel, dim3((unsigned)std::min<long long>((n + 255) / 256, 2048)), dim3(256), 0,
                     s, static_cast<const unsigned*>(p), n);
  return hipGetLastError();
}

hipError_t warp_persist_check_launch(void* ws, int B, int C, int H, int W, hipStream_t s) {
  const BinLayout2 L = bin_layout2(B, C, H, W);
  const GatherGrid gg = gather_grid(B, C, H, W);
  char* w = static_cast<char*>(ws);
  const long long ncell = (long long)B * (H + 1) * (W + 1);
  hipLaunchKernelGGL(cnt_check_kernel, dim3((unsigned)std::min<long long>((ncell + 255) / 256, 2048)), dim3(256),
                     0, s, reinterpret_cast<const int*>(w + L.hdr_off),
                     reinterpret_cast<const unsigned*>(w + L.cnt_off), ncell, L.list);
  hipError_t e = hipGetLastError();
  if (L.list) return e;
  if (e == hipSuccess) e = zero_check_launch(w + L.dirty_off, 4LL * B * gg.ntiles, s);
  if (e == hipSuccess) e = zero_check_launch(w + L.ovfgx_off, 4LL * B * C * H * W, s);
  return e;
}

long long warp_bwd_workspace(int B, int H, int W) { return bin_layout(B, H, W).total; }
long long warp_bwd_persist_workspace(int B, int C, int H, int W) { return bin_layout2(B, C, H, W).total; }

hipError_t splat_launch(const float* flow, long long fbs, float* map, int B, int H, int W,
                        bool absolute, hipStream_t s) {
  hipError_t e = zero_fill(map, (size_t)B * H * W * sizeof(float), s);
  if (e != hipSuccess) return e;
  return splat_scatter(flow, fbs, map, B, H, W, absolute, s);
}

// the splat's scatter into a map that is already zero
hipError_t splat_scatter(const float* flow, long long fbs, float* map, int B, int H, int W, bool absolute,
                         hipStream_t s) {
  const long pairs = (long)W * ((H + 1) / 2);
  if (pairs >= 4096 && variant_override(2) != 0) {  // pixel pairs (as the warp backward)
    const dim3 grid((unsigned)((pairs + 255) / 256), (unsigned)B);
    if (absolute)
      hipLaunchKernelGGL((splat_pair_kernel<true>), grid, dim3(256), 0, s, flow, fbs, map, H, W);
    else
      hipLaunchKernelGGL((splat_pair_kernel<false>), grid, dim3(256), 0, s, flow, fbs, map, H, W);
    return hipGetLastError();
  }
  const dim3 grid((unsigned)((H * W + 255) / 256), (unsigned)B);
  if (absolute)
    hipLaunchKernelGGL((splat_kernel<true>), grid, dim3(256), 0, s, flow, fbs, map, H, W);
  else
    hipLaunchKernelGGL((splat_kernel<false>), grid, dim3(256), 0, s, flow, fbs, map, H, W);
  return hipGetLastError();
}

hipError_t occ_backward_persist_launch(const float* flow, long long fbs, float* occ, float* map, int B, int H,
                                       int W, float th, hipStream_t s) {
  // map: the caller's persistent splat buffer, zero on entry; the threshold pass
  // is its only reader and leaves it zero again (no fill launch)
  hipError_t e = splat_scatter(flow, fbs, map, B, H, W, false, s);
  if (e != hipSuccess) return e;
  const long long n = (long long)B * H * W;
  hipLaunchKernelGGL(occ_threshold_kernel<true>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, map, occ, n,
                     th);
  return hipGetLastError();
}

hipError_t occ_vis_pair_persist_launch(const float* flow4, float* vis, float* map, int B, int H, int W, float th,
                                      hipStream_t s) {
  // a dense [B,4,H,W] flow is a [2B,2,H,W] batch of (flow12, flow21) pairs: one
  // splat launch over 2B samples fills the interleaved map
  const long long HW = (long long)H * W;
  hipError_t e = splat_scatter(flow4, 2 * HW, map, 2 * B, H, W, false, s);
  if (e != hipSuccess) return e;
  const long long n = 2LL * B * HW;
  hipLaunchKernelGGL(occ_vis_pair_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, map, vis, (int)HW, B,
                     th);
  return hipGetLastError();
}

hipError_t occ_backward_launch(const float* flow, long long fbs, float* occ, int B, int H, int W,
                               float th, hipStream_t s) {
  hipError_t e = splat_launch(flow, fbs, occ, B, H, W, false, s);
  if (e != hipSuccess) return e;
  const long long n = (long long)B * H * W;
  hipLaunchKernelGGL(occ_threshold_kernel<false>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, occ, occ, n,
                     th);
  return hipGetLastError();
}

namespace {
// Forward-backward consistency occlusion (get_occu_mask_bidirection,
// warp_utils.py:109-117), one thread per pixel:
//   w21  = flow_warp(flow21, flow12, pad="zeros")            (:110)
//   diff = flow12 + w21                                        (:111)
//   mag  = (f12_u^2 + f12_v^2) + (w21_u^2 + w21_v^2)           (:112-114)
//   occ  = (diff_u^2 + diff_v^2) > 0.01 * mag + 0.5 ? 1 : 0    (:115-117)
// Each product and sum is rounded separately, as torch evaluates them (the
// channel sums over 2 elements are a + b), so the mask decision is the
// reference's bit for bit where the warp is.
__global__ __launch_bounds__(256) void occ_bidir_kernel(const float* __restrict__ f12, long long bs12,
                                                        const float* __restrict__ f21, long long bs21,
                                                        float* __restrict__ occ, int H, int W,
                                                        float scale, float bias) {
#pragma clang fp contract(off)
  const int HW = H * W;
  const int p = blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (p >= HW) return;
  const int y = p / W, x = p - y * W;
  const float* a = f12 + b * bs12;
  const float* c = f21 + b * bs21;
  const float u = a[p], v = a[HW + p];
  const Tap t = make_tap(u, v, x, y, H, W, false);
  const float wnw = t.s * t.e, wne = t.s * t.w, wsw = t.n * t.e, wse = t.n * t.w;
  float w[2];
#pragma unroll
  for (int ch = 0; ch < 2; ++ch) {
    const float* cc = c + ch * HW;
    const float vnw = t.m_nw ? cc[t.o_nw] : 0.f, vne = t.m_ne ? cc[t.o_ne] : 0.f;
    const float vsw = t.m_sw ? cc[t.o_sw] : 0.f, vse = t.m_se ? cc[t.o_se] : 0.f;
    w[ch] = vnw * wnw + vne * wne + vsw * wsw + vse * wse;
  }
  const float du = u + w[0], dv = v + w[1];
  const float mag = (u * u + v * v) + (w[0] * w[0] + w[1] * w[1]);
  const float th = scale * mag + bias;
  occ[(size_t)b * HW + p] = (du * du + dv * dv) > th ? 1.f : 0.f;
}
}  // namespace

hipError_t occ_bidirection_launch(const float* flow12, long long bs12, const float* flow21, long long bs21,
                                  float* occ, int B, int H, int W, float scale, float bias, hipStream_t s) {
  const int HW = H * W;
  hipLaunchKernelGGL(occ_bidir_kernel, dim3((unsigned)((HW + 255) / 256), (unsigned)B), dim3(256), 0, s,
                     flow12, bs12, flow21, bs21, occ, H, W, scale, bias);
  return hipGetLastError();
}

}  // namespace usf
