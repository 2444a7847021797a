// Shared helpers for the gfx950 kernels of libunsamflow_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

#include "unsamflow_hip.h"

namespace usf {

// Device-side error flags (warp.hip): read and optionally cleared after a
// stream sync; -1 if the sync or the copy failed.
int device_errors(hipStream_t s, bool clear);

// Thread-local error slot behind usf_last_error_string().
void set_error(const char* fmt, ...);
void clear_error();

// Round n up to a multiple of m (compile-time helper).
__host__ __device__ constexpr int round_up(int n, int m) { return ((n + m - 1) / m) * m; }

// Tuning override of usf_set_variant (op 0: corr fwd, 1: corr bwd, 2: warp grad_x; -1 = default).
int variant_override(int op);
int variant_count(int op);
void set_variant_override(int op, int index);

// Workgroups are dealt round-robin over the 8 XCDs, so blocks b and b + 8 share
// an L2 (MI355X_MICROARCH.md §Workgroup dispatch; a speed property, never a
// correctness one). Renumber the linear block id so that CONSECUTIVE work items
// -- which share staged data (a tile's displacement-row groups / channel
// groups, neighbouring tiles' halos) -- run on one XCD. Bijective on [0, n).
// Used by the correlation forward (L3 16.7 vs 18.6 us, FETCH traffic 3.9x -> 1.0x
// of algorithmic) and the photometric kernels. USF_XCD_REMAP=0
// (tools/ab_build.py A/B builds) turns it off.
#ifndef USF_XCD_REMAP
#define USF_XCD_REMAP 1
#endif
__device__ __forceinline__ int xcd_remap(int lin, int n) {
  if (!USF_XCD_REMAP) return lin;
  const int full = n & ~7;
  if (lin >= full) return lin;
  return (lin & 7) * (full >> 3) + (lin >> 3);
}

// Chunked variant: Q consecutive work items per XCD, chunks dealt round-robin
// (block lin runs on XCD lin % 8 and gets item Q (8 m + x) + j). Neighbouring
// items share one L2 a few at a time while every XCD still sees the whole
// range (a whole contiguous 1/8 per XCD -- xcd_remap -- measured slower for
// the correlation backward). Bijective on [0, n).
__device__ __forceinline__ int xcd_chunk(int lin, int n, int Q) {
  const int full = (n / (8 * Q)) * (8 * Q);
  if (Q <= 0 || lin >= full) return lin;
  const int x = lin & 7, r = lin >> 3;
  return Q * (8 * (r / Q) + x) + r % Q;
}

__device__ __forceinline__ int linear_block() {
  return blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
}

// Launchers implemented in corr.hip / warp.hip. They assume validated
// arguments (capi.cpp checks shapes, d and pointers) and return the
// hipError_t of the launch.
// Correlation epilogues: output / gradient batch strides (elements; a channel
// slice of a concat buffer) and an optional LeakyReLU (act = 1, slope).
struct FwdEpi {
  long long out_bstride;
  int act;
  float slope;
  // channel split (set by the dispatcher): groups > 1 -> every workgroup sums
  // a channel group and writes raw partials to part[g][b][k][p]; a reduce
  // kernel applies the mean and the epilogue. Not part of the C ABI.
  float* part = nullptr;
  int groups = 1;
  // LeakyReLU sign mask (act != 0, W % 4 == 0): word [b][dy][y][x / 4] holds
  // bit 4 dx + (x % 4) = (activated output at (dy, dx, y, x) > 0). The backward
  // applies the derivative from it instead of re-reading the activated output.
  unsigned long long* mask = nullptr;
};
struct BwdEpi {
  long long g_bstride;
  const unsigned long long* mask = nullptr;  // FwdEpi::mask of the forward: derivative in the prologue
  float slope = 0.f;
};
// words of the sign mask (0: layout unsupported, W % 4 != 0)
long long corr_act_mask_words(int B, int H, int W, int d);
hipError_t leaky_bwd_gather_launch(const float* g, const float* act, long long g_bstride,
                                   float slope, float* out, int B, int K2, int H, int W,
                                   hipStream_t s);
hipError_t corr_fwd_launch(const float* x1, const float* x2, float* out, int B, int C,
                           int H, int W, int d, hipStream_t s, FwdEpi ep, float* workspace = nullptr,
                           long long workspace_floats = 0);
// floats of workspace that lets the forward split its channel loop (0: no split)
long long corr_fwd_workspace(int B, int C, int H, int W, int d);
hipError_t corr_bwd_launch(const float* x1, const float* x2, const float* gout,
                           float* gx1, float* gx2, int B, int C, int H, int W, int d,
                           hipStream_t s, BwdEpi ep);
// the decoder's x2 flow upsampling fused into the warp forward: up = [B,2,H,W]
// = F.interpolate(coarse * 2, scale_factor=2, bilinear, align_corners=True)
// of coarse = [B,2,H/2,W/2] (H, W even), out = flow_warp(x, up)
hipError_t warp_fwd_up_launch(const float* x, const float* coarse, float* up, float* out, int B, int C, int H, int W,
                              int pad_mode, hipStream_t s);
hipError_t warp_fwd_launch(const float* x, const float* flow, long long flow_bstride,
                           float* out, int B, int C, int H, int W, int pad_mode,
                           hipStream_t s);
hipError_t warp_bwd_launch(const float* x, const float* flow, long long flow_bstride,
                           const float* gout, float* gx, float* gflow, int B, int C, int H,
                           int W, int pad_mode, hipStream_t s, void* workspace = nullptr,
                           long long workspace_bytes = 0, bool persist = false);
// bytes of workspace for the binned-gather grad_x (usf_warp_bwd_ex_f32)
long long warp_bwd_workspace(int B, int H, int W);
// bytes of the persistent workspace of usf_warp_bwd_persist_f32
long long warp_bwd_persist_workspace(int B, int C, int H, int W);
// USF_SYNC_CHECK only: raise USF_DEVERR_WORKSPACE_DIRTY unless a persistent
// workspace is back in the state the next call expects (warp: the next call's
// count buffer, the dirty words and the overflow buffer all zero; occlusion:
// the splat map zero)
hipError_t warp_persist_check_launch(void* ws, int B, int C, int H, int W, hipStream_t s);
hipError_t zero_check_launch(const void* p, long long bytes, hipStream_t s);

hipError_t splat_launch(const float* flow, long long flow_bstride, float* map, int B, int H, int W,
                        bool absolute, hipStream_t s);
hipError_t occ_backward_launch(const float* flow, long long flow_bstride, float* occ, int B, int H,
                               int W, float th, hipStream_t s);
hipError_t splat_scatter(const float* flow, long long flow_bstride, float* map, int B, int H, int W,
                         bool absolute, hipStream_t s);
hipError_t occ_vis_pair_persist_launch(const float* flow4, float* vis, float* map, int B, int H, int W, float th,
                                      hipStream_t s);
hipError_t occ_backward_persist_launch(const float* flow, long long flow_bstride, float* occ, float* map, int B,
                                       int H, int W, float th, hipStream_t s);
hipError_t occ_bidirection_launch(const float* flow12, long long bs12, const float* flow21, long long bs21,
                                  float* occ, int B, int H, int W, float scale, float bias, hipStream_t s);

int photo_partials(int B, int H, int W);
hipError_t photo_fwd_launch(const float* src, const float* tgt, const float* mask, const float* flow,
                            long long flow_bstride, float* partials, float* out, float* basis, int B,
                            int C, int H, int W, int pad_mode, float w_l1, float w_ssim, hipStream_t s);
hipError_t photo_pair_fwd_launch(const float* im1, const float* im2, const float* mask1,
                                 const float* mask2, const float* flow, long long flow_bstride,
                                 float* partials, float* out, float* basis, int B, int C, int H,
                                 int W, int pad_mode, float w_l1, float w_ssim, hipStream_t s);
hipError_t photo_pyr_fwd_launch(int nscale, const float* const* im1, const float* const* im2,
                                const float* const* mask1, const float* const* mask2, const float* const* flow,
                                const long long* fbs, const int* H, const int* W, float* partials, float* out,
                                float* const* basis, int B, int C, int pad_mode, float w_l1, float w_ssim,
                                hipStream_t s);
hipError_t photo_pyr_bwd_launch(int nscale, const float* const* basis, const float* coef, const float* gloss,
                                float* const* gflow, const int* H, const int* W, int B, hipStream_t s);
hipError_t photo_bwd_launch(const float* basis, const float* coef, const float* gloss, float* gflow,
                            int B, int H, int W, int ndir, hipStream_t s);

hipError_t upsample_fwd_launch(const float* x, float* out, int B, int C, int H, int W, int k,
                               hipStream_t s);
hipError_t upsample_bwd_launch(const float* gout, float* gx, int B, int C, int H, int W, int k,
                               hipStream_t s, const float* gout2 = nullptr);
int convex_pyramid_max_levels();
hipError_t convex_pyr_fwd_launch(int n, const float* const* flow, const float* const* mask, float* const* out,
                                 const int* H, const int* W, int B, int factor, float mask_scale, hipStream_t s);
hipError_t convex_pyr_bwd_launch(int n, const float* const* flow, const float* const* mask,
                                 const float* const* gout, float* const* gflow, float* const* gmask, float* scratch,
                                 const int* H, const int* W, int B, int factor, float mask_scale, hipStream_t s);
bool convex_factor_ok(int factor);
long long convex_bwd_scratch(int B, int H, int W);
hipError_t convex_fwd_launch(const float* flow, const float* mask, float* out, int B, int H, int W,
                             int factor, float mask_scale, hipStream_t s);
hipError_t convex_bwd_launch(const float* flow, const float* mask, const float* gout, float* gflow,
                             float* gmask, float* scratch, int B, int H, int W, int factor,
                             float mask_scale, hipStream_t s);
hipError_t stream_copy_launch(const float* src, float* dst, long long n, hipStream_t s);
hipError_t area_pyramid_launch(const float* x, float* o1, float* o2, float* o3, long long planes,
                               int H, int W, hipStream_t s);

}  // namespace usf
