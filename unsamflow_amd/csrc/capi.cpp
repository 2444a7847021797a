// C ABI of libunsamflow_hip.so (declared in include/unsamflow_hip.h).
// Argument validation + error reporting; the launches live in corr.hip / warp.hip.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>

#include "../../include/unsamflow_hip.h"
#include "usf_common.h"

namespace usf {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = '\0'; }

static bool check_dims(const char* fn, int B, int C, int H, int W) {
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0) {
    set_error("%s: non-positive shape B=%d C=%d H=%d W=%d", fn, B, C, H, W);
    return false;
  }
  // per-sample BYTE offsets are 32-bit inside the kernels (the correlation's
  // LDS-DMA descriptors span one sample and park masked lanes at 0x7FFFFFF0)
  const long long per_sample = (long long)C * H * W;
  const long long max_elems = 0x7FFFFFF0LL / 4 - 1;
  if (per_sample > max_elems || (long long)H * W * 81 > max_elems) {
    set_error("%s: per-sample tensor too large (C*H*W=%lld)", fn, per_sample);
    return false;
  }
  return true;
}

// USF_SYNC_CHECK=1: synchronise the stream after every launch and report any
// asynchronous fault against the launch that caused it (debug only).
static bool sync_check() {
  static const bool on = [] {
    const char* v = getenv("USF_SYNC_CHECK");
    return v && v[0] == '1';
  }();
  return on;
}

// A stream under graph capture cannot be synchronised: the debug checks skip it
// (the replays of the graph run the same kernels unchecked).
static bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

static bool sync_check_on(hipStream_t s) { return sync_check() && !capturing(s); }

// With USF_SYNC_CHECK=1 every entry point first drains the stream, so a fault
// raised by an EARLIER (non-usf) kernel is reported as such, not blamed on us.
static int pre_check(const char* fn, hipStream_t s) {
  if (!sync_check_on(s)) return 0;
  const hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    fprintf(stderr, "[usf] %s: stream already faulted BEFORE this launch: %s\n", fn, hipGetErrorString(e));
    set_error("%s: stream faulted before launch: %s (%d)", fn, hipGetErrorString(e), (int)e);
    return (int)e;
  }
  return 0;
}

static int finish(const char* fn, hipError_t e, hipStream_t s) {
  if (e == hipSuccess && sync_check_on(s)) {
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) fprintf(stderr, "[usf] %s: fault after launch: %s\n", fn, hipGetErrorString(e));
    const int flags = e == hipSuccess ? device_errors(s, true) : 0;
    if (flags > 0) {
      fprintf(stderr, "[usf] %s: device error flags 0x%x\n", fn, flags);
      set_error("%s: device error flags 0x%x", fn, flags);
      return USF_EDEVICE;
    }
  }
  if (e != hipSuccess) {
    set_error("%s: HIP launch failed: %s (%d)", fn, hipGetErrorString(e), (int)e);
    return (int)e;
  }
  return 0;
}

}  // namespace usf

using namespace usf;

extern "C" {

int usf_abi_version(void) { return USF_ABI_VERSION; }

#ifndef USF_BUILD_ID
#define USF_BUILD_ID "unstamped"
#endif
const char* usf_build_id(void) { return USF_BUILD_ID; }

const char* usf_last_error_string(void) { return g_err; }

int usf_corr_fwd_f32(const float* x1, const float* x2, float* out, int B, int C, int H, int W,
                     int d, void* stream) {
  clear_error();
  if (!check_dims("usf_corr_fwd_f32", B, C, H, W)) return USF_EINVAL;
  if (d < 1 || d > 4) {
    set_error("usf_corr_fwd_f32: max_displacement %d not in [1,4]", d);
    return USF_EINVAL;
  }
  if (!x1 || !x2 || !out) {
    set_error("usf_corr_fwd_f32: null pointer");
    return USF_EINVAL;
  }
  if (const int pe = pre_check("usf_corr_fwd_f32", (hipStream_t)stream)) return pe;
  const long long k2 = (long long)(2 * d + 1) * (2 * d + 1);
  return finish("usf_corr_fwd_f32",
                corr_fwd_launch(x1, x2, out, B, C, H, W, d, (hipStream_t)stream,
                                FwdEpi{k2 * H * W, 0, 0.f}),
                (hipStream_t)stream);
}

long long usf_corr_fwd_workspace(int B, int C, int H, int W, int d) {
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || d < 1 || d > 4) return 0;
  return corr_fwd_workspace(B, C, H, W, d);
}

long long usf_corr_act_mask_words(int B, int H, int W, int d) {
  if (B <= 0 || H <= 0 || W <= 0) return 0;
  return corr_act_mask_words(B, H, W, d);
}

int usf_corr_fwd_ex_f32(const float* x1, const float* x2, float* out, long long out_bstride,
                        int act, float slope, unsigned long long* act_mask, float* workspace,
                        long long workspace_floats, int B, int C, int H, int W, int d, void* stream) {
  clear_error();
  if (!check_dims("usf_corr_fwd_ex_f32", B, C, H, W)) return USF_EINVAL;
  if (d < 1 || d > 4) {
    set_error("usf_corr_fwd_ex_f32: max_displacement %d not in [1,4]", d);
    return USF_EINVAL;
  }
  if (!x1 || !x2 || !out) {
    set_error("usf_corr_fwd_ex_f32: null pointer");
    return USF_EINVAL;
  }
  const long long k2 = (long long)(2 * d + 1) * (2 * d + 1);
  if (out_bstride < k2 * H * W && B > 1) {
    set_error("usf_corr_fwd_ex_f32: out batch stride %lld < (2d+1)^2*H*W", out_bstride);
    return USF_EINVAL;
  }
  if (act != USF_ACT_NONE && act != USF_ACT_LEAKY_RELU) {
    set_error("usf_corr_fwd_ex_f32: unknown act %d", act);
    return USF_EINVAL;
  }
  if (act_mask && act != USF_ACT_LEAKY_RELU) {
    set_error("usf_corr_fwd_ex_f32: act_mask needs act = LeakyReLU (act=%d)", act);
    return USF_EINVAL;
  }
  if (const int pe = pre_check("usf_corr_fwd_ex_f32", (hipStream_t)stream)) return pe;
  FwdEpi ep{out_bstride, act, slope};
  ep.mask = act_mask;
  return finish("usf_corr_fwd_ex_f32",
                corr_fwd_launch(x1, x2, out, B, C, H, W, d, (hipStream_t)stream, ep, workspace,
                                workspace_floats),
                (hipStream_t)stream);
}

int usf_corr_bwd_f32(const float* x1, const float* x2, const float* gout, float* gx1,
                     float* gx2, int B, int C, int H, int W, int d, void* stream) {
  clear_error();
  if (!check_dims("usf_corr_bwd_f32", B, C, H, W)) return USF_EINVAL;
  if (d < 1 || d > 4) {
    set_error("usf_corr_bwd_f32: max_displacement %d not in [1,4]", d);
    return USF_EINVAL;
  }
  if (!gout || (gx1 && !x2) || (gx2 && !x1)) {
    set_error("usf_corr_bwd_f32: null input pointer");
    return USF_EINVAL;
  }
  if (const int pe = pre_check("usf_corr_bwd_f32", (hipStream_t)stream)) return pe;
  const long long k2 = (long long)(2 * d + 1) * (2 * d + 1);
  return finish("usf_corr_bwd_f32",
                corr_bwd_launch(x1, x2, gout, gx1, gx2, B, C, H, W, d, (hipStream_t)stream,
                                BwdEpi{k2 * H * W}),
                (hipStream_t)stream);
}

int usf_corr_bwd_ex_f32(const float* x1, const float* x2, const float* gout, long long g_bstride,
                        const float* act_out, const unsigned long long* act_mask, float slope,
                        float* scratch, float* gx1, float* gx2, int B, int C, int H, int W, int d,
                        void* stream) {
  clear_error();
  if (!check_dims("usf_corr_bwd_ex_f32", B, C, H, W)) return USF_EINVAL;
  if (d < 1 || d > 4) {
    set_error("usf_corr_bwd_ex_f32: max_displacement %d not in [1,4]", d);
    return USF_EINVAL;
  }
  if (!gout || (gx1 && !x2) || (gx2 && !x1)) {
    set_error("usf_corr_bwd_ex_f32: null input pointer");
    return USF_EINVAL;
  }
  const long long k2 = (long long)(2 * d + 1) * (2 * d + 1);
  if (g_bstride < k2 * H * W && B > 1) {
    set_error("usf_corr_bwd_ex_f32: gradient batch stride %lld < (2d+1)^2*H*W", g_bstride);
    return USF_EINVAL;
  }
  if (act_mask) {  // derivative from the forward's sign mask, inside the backward's g loads
    if (const int pe = pre_check("usf_corr_bwd_ex_f32", (hipStream_t)stream)) return pe;
    BwdEpi ep{g_bstride};
    ep.mask = act_mask;
    ep.slope = slope;
    return finish("usf_corr_bwd_ex_f32",
                  corr_bwd_launch(x1, x2, gout, gx1, gx2, B, C, H, W, d, (hipStream_t)stream, ep),
                  (hipStream_t)stream);
  }
  if (act_out && !scratch) {
    set_error("usf_corr_bwd_ex_f32: act_out needs a scratch of usf_corr_bwd_ex_scratch() floats here");
    return USF_EINVAL;
  }
  if (const int pe = pre_check("usf_corr_bwd_ex_f32", (hipStream_t)stream)) return pe;
  const BwdEpi ep{g_bstride};
  if (act_out) {  // derivative + de-concat in one dense pass, then the plain backward
    const hipError_t e = leaky_bwd_gather_launch(gout, act_out, g_bstride, slope, scratch, B,
                                                 (int)k2, H, W, (hipStream_t)stream);
    if (e != hipSuccess) return finish("usf_corr_bwd_ex_f32", e, (hipStream_t)stream);
    return finish("usf_corr_bwd_ex_f32",
                  corr_bwd_launch(x1, x2, scratch, gx1, gx2, B, C, H, W, d, (hipStream_t)stream,
                                  BwdEpi{k2 * H * W}),
                  (hipStream_t)stream);
  }
  return finish("usf_corr_bwd_ex_f32",
                corr_bwd_launch(x1, x2, gout, gx1, gx2, B, C, H, W, d, (hipStream_t)stream, ep),
                (hipStream_t)stream);
}

long long usf_corr_bwd_ex_scratch(int B, int C, int H, int W, int d) {
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || d < 1 || d > 4) return 0;
  return (long long)B * (2 * d + 1) * (2 * d + 1) * H * W;
}

int usf_warp_fwd_f32(const float* x, const float* flow, long long flow_bstride, float* out,
                     int B, int C, int H, int W, int pad_mode, void* stream) {
  clear_error();
  if (!check_dims("usf_warp_fwd_f32", B, C, H, W)) return USF_EINVAL;
  if (pad_mode != USF_PAD_ZEROS && pad_mode != USF_PAD_BORDER) {
    set_error("usf_warp_fwd_f32: unknown pad_mode %d", pad_mode);
    return USF_EINVAL;
  }
  if (!x || !flow || !out) {
    set_error("usf_warp_fwd_f32: null pointer");
    return USF_EINVAL;
  }
  if (flow_bstride < 2LL * H * W && B > 1) {
    set_error("usf_warp_fwd_f32: flow batch stride %lld < 2*H*W", flow_bstride);
    return USF_EINVAL;
  }
  if (const int pe = pre_check("usf_warp_fwd_f32", (hipStream_t)stream)) return pe;
  return finish("usf_warp_fwd_f32",
                warp_fwd_launch(x, flow, flow_bstride, out, B, C, H, W, pad_mode, (hipStream_t)stream),
                (hipStream_t)stream);
}

int usf_warp_fwd_up_f32(const float* x, const float* coarse_flow, float* up_flow, float* out, int B, int C, int H,
                        int W, int pad_mode, void* stream) {
  clear_error();
  const char* fn = "usf_warp_fwd_up_f32";
  if (!check_dims(fn, B, C, H, W)) return USF_EINVAL;
  if (pad_mode != USF_PAD_ZEROS && pad_mode != USF_PAD_BORDER) {
    set_error("%s: unknown pad_mode %d", fn, pad_mode);
    return USF_EINVAL;
  }
  if ((H & 1) || (W & 1) || H < 2 || W < 2) {
    set_error("%s: H=%d W=%d must be even (the coarse flow is [B,2,H/2,W/2])", fn, H, W);
    return USF_EINVAL;
  }
  if (!x || !coarse_flow || !up_flow || !out) {
    set_error("%s: null pointer", fn);
    return USF_EINVAL;
  }
  if (const int pe = pre_check(fn, (hipStream_t)stream)) return pe;
  return finish(fn, warp_fwd_up_launch(x, coarse_flow, up_flow, out, B, C, H, W, pad_mode, (hipStream_t)stream),
                (hipStream_t)stream);
}

static int warp_bwd_common(const char* fn, const float* x, const float* flow, long long flow_bstride,
                           const float* gout, float* gx, float* gflow, void* ws, long long ws_bytes, int B,
                           int C, int H, int W, int pad_mode, void* stream, bool persist = false) {
  clear_error();
  if (!check_dims(fn, B, C, H, W)) return USF_EINVAL;
  if (pad_mode != USF_PAD_ZEROS && pad_mode != USF_PAD_BORDER) {
    set_error("%s: unknown pad_mode %d", fn, pad_mode);
    return USF_EINVAL;
  }
  if (!flow || !gout || (gflow && !x)) {
    set_error("%s: null input pointer", fn);
    return USF_EINVAL;
  }
  if (flow_bstride < 2LL * H * W && B > 1) {
    set_error("%s: flow batch stride %lld < 2*H*W", fn, flow_bstride);
    return USF_EINVAL;
  }
  if (ws_bytes < 0) {
    set_error("%s: negative workspace size", fn);
    return USF_EINVAL;
  }
  if (ws && (reinterpret_cast<uintptr_t>(ws) & 15)) {  // the binned gather reads it with 16-byte loads
    set_error("%s: workspace must be 16-byte aligned", fn);
    return USF_EINVAL;
  }
  if (persist) {
    if (!ws || ws_bytes < warp_bwd_persist_workspace(B, C, H, W)) {
      set_error("%s: persistent workspace of %lld bytes < usf_warp_bwd_persist_workspace = %lld", fn, ws_bytes,
                warp_bwd_persist_workspace(B, C, H, W));
      return USF_EINVAL;
    }
    if (C > 256 || H >= 32768 || W >= 65536) {  // gather channel groups fit a 32-bit dirty mask; packed (y, x)
      set_error("%s: C=%d H=%d W=%d beyond the persistent form (C <= 256, H < 32768, W < 65536)", fn, C, H, W);
      return USF_EINVAL;
    }
    // the gather reads both count buffers through one buffer descriptor with
    // 32-bit byte offsets: 2 x 4 bytes per cell must stay below 2^31
    if (8LL * B * (H + 1) * (W + 1) >= (1LL << 31)) {
      set_error("%s: B=%d H=%d W=%d: 8*B*(H+1)*(W+1) >= 2^31 (count buffers past 32-bit offsets)", fn, B, H, W);
      return USF_EINVAL;
    }
  }
  if (const int pe = pre_check(fn, (hipStream_t)stream)) return pe;
  hipError_t e = warp_bwd_launch(x, flow, flow_bstride, gout, gx, gflow, B, C, H, W, pad_mode, (hipStream_t)stream,
                                 ws, ws_bytes, persist);
  if (e == hipSuccess && persist && gx && sync_check_on((hipStream_t)stream))
    e = warp_persist_check_launch(ws, B, C, H, W, (hipStream_t)stream);
  return finish(fn, e, (hipStream_t)stream);
}

int usf_warp_bwd_f32(const float* x, const float* flow, long long flow_bstride,
                     const float* gout, float* gx, float* gflow, int B, int C, int H, int W,
                     int pad_mode, void* stream) {
  return warp_bwd_common("usf_warp_bwd_f32", x, flow, flow_bstride, gout, gx, gflow, nullptr, 0, B, C, H, W,
                         pad_mode, stream);
}

int usf_warp_bwd_ex_f32(const float* x, const float* flow, long long flow_bstride, const float* gout,
                        float* gx, float* gflow, void* workspace, long long workspace_bytes, int B, int C,
                        int H, int W, int pad_mode, void* stream) {
  return warp_bwd_common("usf_warp_bwd_ex_f32", x, flow, flow_bstride, gout, gx, gflow, workspace,
                         workspace ? workspace_bytes : 0, B, C, H, W, pad_mode, stream);
}

long long usf_warp_bwd_workspace(int B, int H, int W) {
  if (B <= 0 || H <= 0 || W <= 0) return 0;
  return warp_bwd_workspace(B, H, W);
}

int usf_warp_bwd_persist_f32(const float* x, const float* flow, long long flow_bstride, const float* gout,
                             float* gx, float* gflow, void* workspace, long long workspace_bytes, int B, int C,
                             int H, int W, int pad_mode, void* stream) {
  return warp_bwd_common("usf_warp_bwd_persist_f32", x, flow, flow_bstride, gout, gx, gflow, workspace,
                         workspace_bytes, B, C, H, W, pad_mode, stream, true);
}

long long usf_warp_bwd_persist_workspace(int B, int C, int H, int W) {
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return 0;
  return warp_bwd_persist_workspace(B, C, H, W);
}

static bool check_splat(const char* fn, const float* flow, long long fbs, const float* out, int B,
                        int H, int W) {
  if (!check_dims(fn, B, 2, H, W)) return false;
  if (!flow || !out) {
    set_error("%s: null pointer", fn);
    return false;
  }
  if (fbs < 2LL * H * W && B > 1) {
    set_error("%s: flow batch stride %lld < 2*H*W", fn, fbs);
    return false;
  }
  return true;
}

int usf_splat_map_f32(const float* flow, long long flow_bstride, float* map, int B, int H, int W,
                      int absolute, void* stream) {
  clear_error();
  if (!check_splat("usf_splat_map_f32", flow, flow_bstride, map, B, H, W)) return USF_EINVAL;
  if (const int pe = pre_check("usf_splat_map_f32", (hipStream_t)stream)) return pe;
  return finish("usf_splat_map_f32",
                splat_launch(flow, flow_bstride, map, B, H, W, absolute != 0, (hipStream_t)stream),
                (hipStream_t)stream);
}

int usf_occ_backward_f32(const float* flow21, long long flow_bstride, float* occ, int B, int H,
                         int W, float th, void* stream) {
  clear_error();
  if (!check_splat("usf_occ_backward_f32", flow21, flow_bstride, occ, B, H, W)) return USF_EINVAL;
  if (const int pe = pre_check("usf_occ_backward_f32", (hipStream_t)stream)) return pe;
  return finish("usf_occ_backward_f32",
                occ_backward_launch(flow21, flow_bstride, occ, B, H, W, th, (hipStream_t)stream),
                (hipStream_t)stream);
}

int usf_occ_backward_persist_f32(const float* flow21, long long flow_bstride, float* occ, float* map,
                                 long long map_bytes, int B, int H, int W, float th, void* stream) {
  clear_error();
  const char* fn = "usf_occ_backward_persist_f32";
  if (!check_splat(fn, flow21, flow_bstride, occ, B, H, W)) return USF_EINVAL;
  if (!map || map_bytes < 4LL * B * H * W || map == occ) {
    set_error("%s: map must be a separate buffer of >= 4*B*H*W = %lld bytes (got %lld)", fn, 4LL * B * H * W,
              map_bytes);
    return USF_EINVAL;
  }
  if (const int pe = pre_check(fn, (hipStream_t)stream)) return pe;
  hipError_t e = occ_backward_persist_launch(flow21, flow_bstride, occ, map, B, H, W, th, (hipStream_t)stream);
  if (e == hipSuccess && sync_check_on((hipStream_t)stream))
    e = zero_check_launch(map, 4LL * B * H * W, (hipStream_t)stream);
  return finish(fn, e, (hipStream_t)stream);
}

int usf_occ_vis_pair_persist_f32(const float* flow4, long long flow_bstride, float* vis, float* map,
                                 long long map_bytes, int B, int H, int W, float th, void* stream) {
  clear_error();
  const char* fn = "usf_occ_vis_pair_persist_f32";
  if (!check_dims(fn, B, 4, H, W)) return USF_EINVAL;
  if (!flow4 || !vis) {
    set_error("%s: null pointer", fn);
    return USF_EINVAL;
  }
  if (B > 1 && flow_bstride != 4LL * H * W) {
    set_error("%s: flow4 must be a dense [B,4,H,W] tensor (batch stride %lld != 4*H*W)", fn, flow_bstride);
    return USF_EINVAL;
  }
  if (!map || map_bytes < 8LL * B * H * W || map == vis) {
    set_error("%s: map must be a separate buffer of >= 8*B*H*W = %lld bytes (got %lld)", fn, 8LL * B * H * W,
              map_bytes);
    return USF_EINVAL;
  }
  if (2LL * B * H * W >= (1LL << 31)) {
    set_error("%s: 2*B*H*W beyond 32-bit indexing", fn);
    return USF_EINVAL;
  }
  if (const int pe = pre_check(fn, (hipStream_t)stream)) return pe;
  hipError_t e = occ_vis_pair_persist_launch(flow4, vis, map, B, H, W, th, (hipStream_t)stream);
  if (e == hipSuccess && sync_check_on((hipStream_t)stream))
    e = zero_check_launch(map, 8LL * B * H * W, (hipStream_t)stream);
  return finish(fn, e, (hipStream_t)stream);
}

int usf_occ_bidirection_f32(const float* flow12, long long flow12_bstride, const float* flow21,
                            long long flow21_bstride, float* occ, int B, int H, int W, float scale,
                            float bias, void* stream) {
  clear_error();
  if (!check_splat("usf_occ_bidirection_f32", flow12, flow12_bstride, occ, B, H, W) ||
      !check_splat("usf_occ_bidirection_f32", flow21, flow21_bstride, occ, B, H, W))
    return USF_EINVAL;
  if (const int pe = pre_check("usf_occ_bidirection_f32", (hipStream_t)stream)) return pe;
  return finish("usf_occ_bidirection_f32",
                occ_bidirection_launch(flow12, flow12_bstride, flow21, flow21_bstride, occ, B, H, W, scale,
                                       bias, (hipStream_t)stream),
                (hipStream_t)stream);
}

int usf_photo_loss_partials(int B, int H, int W) {
  return (B > 0 && H > 0 && W > 0) ? photo_partials(B, H, W) : 0;
}

static bool check_photo(const char* fn, const float* src, const float* tgt, const float* mask,
                        const float* flow, long long fbs, int B, int C, int H, int W, int pad_mode) {
  if (!check_dims(fn, B, C, H, W)) return false;
  if (C > 3) {
    set_error("%s: C=%d image channels > 3", fn, C);
    return false;
  }
  if (pad_mode != USF_PAD_ZEROS && pad_mode != USF_PAD_BORDER) {
    set_error("%s: unknown pad_mode %d", fn, pad_mode);
    return false;
  }
  if (!src || !tgt || !mask || !flow) {
    set_error("%s: null input pointer", fn);
    return false;
  }
  if (fbs < 2LL * H * W && B > 1) {
    set_error("%s: flow batch stride %lld < 2*H*W", fn, fbs);
    return false;
  }
  return true;
}

int usf_photo_loss_fwd_f32(const float* src, const float* tgt, const float* mask, const float* flow,
                           long long flow_bstride, float* partials, float* out, float* grad_basis,
                           int B, int C, int H, int W, int pad_mode, float w_l1, float w_ssim,
                           void* stream) {
  clear_error();
  if (!check_photo("usf_photo_loss_fwd_f32", src, tgt, mask, flow, flow_bstride, B, C, H, W, pad_mode))
    return USF_EINVAL;
  if (!partials || !out) {
    set_error("usf_photo_loss_fwd_f32: null output pointer");
    return USF_EINVAL;
  }
  if (const int pe = pre_check("usf_photo_loss_fwd_f32", (hipStream_t)stream)) return pe;
  return finish("usf_photo_loss_fwd_f32",
                photo_fwd_launch(src, tgt, mask, flow, flow_bstride, partials, out, grad_basis, B, C,
                                 H, W, pad_mode, w_l1, w_ssim, (hipStream_t)stream),
                (hipStream_t)stream);
}

int usf_photo_loss_pair_fwd_f32(const float* im1, const float* im2, const float* mask1,
                                const float* mask2, const float* flow, long long flow_bstride,
                                float* partials, float* out, float* grad_basis, int B, int C, int H,
                                int W, int pad_mode, float w_l1, float w_ssim, void* stream) {
  clear_error();
  const char* fn = "usf_photo_loss_pair_fwd_f32";
  if (!check_photo(fn, im1, im2, mask1, flow, flow_bstride, B, C, H, W, pad_mode)) return USF_EINVAL;
  if (!mask2) {
    set_error("%s: null input pointer", fn);
    return USF_EINVAL;
  }
  if (flow_bstride < 4LL * H * W && B > 1) {
    set_error("%s: flow batch stride %lld < 4*H*W", fn, flow_bstride);
    return USF_EINVAL;
  }
  if (!partials || !out) {
    set_error("%s: null output pointer", fn);
    return USF_EINVAL;
  }
  if (const int pe = pre_check(fn, (hipStream_t)stream)) return pe;
  return finish(fn,
                photo_pair_fwd_launch(im1, im2, mask1, mask2, flow, flow_bstride, partials, out,
                                      grad_basis, B, C, H, W, pad_mode, w_l1, w_ssim,
                                      (hipStream_t)stream),
                (hipStream_t)stream);
}

long long usf_photo_loss_pyramid_partials(int nscale, const int* H, const int* W, int B) {
  if (nscale < 1 || nscale > 4 || !H || !W || B <= 0) return 0;
  long long n = 0;
  for (int k = 0; k < nscale; ++k) {
    if (H[k] <= 0 || W[k] <= 0) return 0;
    n += 2LL * photo_partials(B, H[k], W[k]);
  }
  return n;
}

int usf_photo_loss_pyramid_fwd_f32(int nscale, const float* const* im1, const float* const* im2,
                                   const float* const* mask1, const float* const* mask2, const float* const* flow,
                                   const long long* flow_bstride, const int* H, const int* W, float* partials,
                                   long long partials_floats, float* out, float* const* grad_basis, int B, int C,
                                   int pad_mode, float w_l1, float w_ssim, void* stream) {
  clear_error();
  const char* fn = "usf_photo_loss_pyramid_fwd_f32";
  if (nscale < 1 || nscale > 4 || !im1 || !im2 || !mask1 || !mask2 || !flow || !flow_bstride || !H || !W) {
    set_error("%s: nscale %d not in [1,4] or a null array", fn, nscale);
    return USF_EINVAL;
  }
  for (int k = 0; k < nscale; ++k) {
    if (!check_photo(fn, im1[k], im2[k], mask1[k], flow[k], flow_bstride[k], B, C, H[k], W[k], pad_mode))
      return USF_EINVAL;
    if (!mask2[k] || (B > 1 && flow_bstride[k] < 4LL * H[k] * W[k])) {
      set_error("%s: scale %d: null mask2 or flow batch stride %lld < 4*H*W", fn, k, flow_bstride[k]);
      return USF_EINVAL;
    }
    if (grad_basis && !grad_basis[k]) {
      set_error("%s: scale %d: grad_basis given for some scales only", fn, k);
      return USF_EINVAL;
    }
  }
  if (!partials || !out || partials_floats < usf_photo_loss_pyramid_partials(nscale, H, W, B)) {
    set_error("%s: partials of %lld floats < usf_photo_loss_pyramid_partials = %lld, or null out", fn,
              partials_floats, usf_photo_loss_pyramid_partials(nscale, H, W, B));
    return USF_EINVAL;
  }
  if (const int pe = pre_check(fn, (hipStream_t)stream)) return pe;
  return finish(fn,
                photo_pyr_fwd_launch(nscale, im1, im2, mask1, mask2, flow, flow_bstride, H, W, partials, out,
                                     grad_basis, B, C, pad_mode, w_l1, w_ssim, (hipStream_t)stream),
                (hipStream_t)stream);
}

int usf_photo_loss_pyramid_bwd_f32(int nscale, const float* const* grad_basis, const float* coef,
                                   const float* grad_loss, float* const* grad_flow, const int* H, const int* W, int B,
                                   void* stream) {
  clear_error();
  const char* fn = "usf_photo_loss_pyramid_bwd_f32";
  if (nscale < 1 || nscale > 4 || !grad_basis || !grad_flow || !H || !W || !coef || !grad_loss || B <= 0) {
    set_error("%s: nscale %d not in [1,4], B=%d, or a null pointer", fn, nscale, B);
    return USF_EINVAL;
  }
  for (int k = 0; k < nscale; ++k) {
    if (!check_dims(fn, B, 8, H[k], W[k])) return USF_EINVAL;
    if (!grad_basis[k] || !grad_flow[k]) {
      set_error("%s: scale %d: null pointer", fn, k);
      return USF_EINVAL;
    }
  }
  if (const int pe = pre_check(fn, (hipStream_t)stream)) return pe;
  return finish(fn, photo_pyr_bwd_launch(nscale, grad_basis, coef, grad_loss, grad_flow, H, W, B, (hipStream_t)stream),
                (hipStream_t)stream);
}

int usf_photo_loss_bwd_f32(const float* grad_basis, const float* coef, const float* grad_loss,
                           float* grad_flow, int B, int H, int W, int ndir, void* stream) {
  clear_error();
  if (!check_dims("usf_photo_loss_bwd_f32", B, 8, H, W)) return USF_EINVAL;
  if (ndir != 1 && ndir != 2) {
    set_error("usf_photo_loss_bwd_f32: ndir=%d (1 or 2)", ndir);
    return USF_EINVAL;
  }
  if (!grad_basis || !coef || !grad_loss || !grad_flow) {
    set_error("usf_photo_loss_bwd_f32: null pointer");
    return USF_EINVAL;
  }
  if (const int pe = pre_check("usf_photo_loss_bwd_f32", (hipStream_t)stream)) return pe;
  return finish("usf_photo_loss_bwd_f32",
                photo_bwd_launch(grad_basis, coef, grad_loss, grad_flow, B, H, W, ndir, (hipStream_t)stream),
                (hipStream_t)stream);
}

int usf_flow_upsample_f32(const float* flow, float* out, int B, int C, int H, int W, int factor,
                          void* stream) {
  clear_error();
  if (!check_dims("usf_flow_upsample_f32", B, C, H, W)) return USF_EINVAL;
  if (factor < 1 || factor > 16 || (long long)C * H * W * factor * factor > 0x1FFFFFFBLL) {
    set_error("usf_flow_upsample_f32: bad factor %d", factor);
    return USF_EINVAL;
  }
  if (!flow || !out) {
    set_error("usf_flow_upsample_f32: null pointer");
    return USF_EINVAL;
  }
  if (const int pe = pre_check("usf_flow_upsample_f32", (hipStream_t)stream)) return pe;
  return finish("usf_flow_upsample_f32",
                upsample_fwd_launch(flow, out, B, C, H, W, factor, (hipStream_t)stream),
                (hipStream_t)stream);
}

int usf_flow_upsample_bwd_f32(const float* grad_out, float* grad_flow, int B, int C, int H, int W,
                              int factor, void* stream) {
  clear_error();
  if (!check_dims("usf_flow_upsample_bwd_f32", B, C, H, W)) return USF_EINVAL;
  if (factor < 1 || factor > 16 || (long long)C * H * W * factor * factor > 0x1FFFFFFBLL) {
    set_error("usf_flow_upsample_bwd_f32: bad factor %d", factor);
    return USF_EINVAL;
  }
  if (!grad_out || !grad_flow) {
    set_error("usf_flow_upsample_bwd_f32: null pointer");
    return USF_EINVAL;
  }
  if (const int pe = pre_check("usf_flow_upsample_bwd_f32", (hipStream_t)stream)) return pe;
  return finish("usf_flow_upsample_bwd_f32",
                upsample_bwd_launch(grad_out, grad_flow, B, C, H, W, factor, (hipStream_t)stream),
                (hipStream_t)stream);
}

int usf_flow_upsample_bwd_sum_f32(const float* grad_a, const float* grad_b, float* grad_flow, int B, int C, int H,
                                  int W, int factor, void* stream) {
  clear_error();
  const char* fn = "usf_flow_upsample_bwd_sum_f32";
  if (!check_dims(fn, B, C, H, W)) return USF_EINVAL;
  if (factor < 1 || factor > 16 || (long long)C * H * W * factor * factor > 0x1FFFFFFBLL) {
    set_error("%s: bad factor %d", fn, factor);
    return USF_EINVAL;
  }
  if (!grad_a || !grad_b || !grad_flow) {
    set_error("%s: null pointer", fn);
    return USF_EINVAL;
  }
  if (const int pe = pre_check(fn, (hipStream_t)stream)) return pe;
  return finish(fn, upsample_bwd_launch(grad_a, grad_flow, B, C, H, W, factor, (hipStream_t)stream, grad_b),
                (hipStream_t)stream);
}

static bool check_convex(const char* fn, int B, int H, int W, int factor) {
  if (!check_dims(fn, B, 2, H, W)) return false;
  if (!convex_factor_ok(factor)) {
    set_error("%s: factor %d (2, 4 or 8)", fn, factor);
    return false;
  }
  if ((long long)9 * factor * factor * H * W > 0x1FFFFFFFLL) {
    set_error("%s: mask plane block too large", fn);
    return false;
  }
  return true;
}

int usf_convex_upsample_f32(const float* flow, const float* mask, float* out, int B, int H, int W,
                            int factor, float mask_scale, void* stream) {
  clear_error();
  const char* fn = "usf_convex_upsample_f32";
  if (!check_convex(fn, B, H, W, factor)) return USF_EINVAL;
  if (!flow || !mask || !out) {
    set_error("%s: null pointer", fn);
    return USF_EINVAL;
  }
  if (const int pe = pre_check(fn, (hipStream_t)stream)) return pe;
  return finish(fn, convex_fwd_launch(flow, mask, out, B, H, W, factor, mask_scale, (hipStream_t)stream),
                (hipStream_t)stream);
}

long long usf_convex_upsample_bwd_scratch(int B, int H, int W) {
  if (B < 0 || H < 0 || W < 0) return 0;
  return convex_bwd_scratch(B, H, W);
}

int usf_convex_upsample_bwd_f32(const float* flow, const float* mask, const float* grad_out,
                                float* grad_flow, float* grad_mask, float* scratch, int B, int H,
                                int W, int factor, float mask_scale, void* stream) {
  clear_error();
  const char* fn = "usf_convex_upsample_bwd_f32";
  if (!check_convex(fn, B, H, W, factor)) return USF_EINVAL;
  if (!flow || !mask || !grad_out) {
    set_error("%s: null input pointer", fn);
    return USF_EINVAL;
  }
  if (grad_flow && !scratch) {
    set_error("%s: grad_flow needs scratch (usf_convex_upsample_bwd_scratch floats)", fn);
    return USF_EINVAL;
  }
  if (!grad_flow && !grad_mask) return 0;
  if (const int pe = pre_check(fn, (hipStream_t)stream)) return pe;
  return finish(fn,
                convex_bwd_launch(flow, mask, grad_out, grad_flow, grad_mask, scratch, B, H, W, factor,
                                  mask_scale, (hipStream_t)stream),
                (hipStream_t)stream);
}

static bool check_convex_pyr(const char* fn, int n, const int* H, const int* W, int B, int factor) {
  if (n < 1 || n > convex_pyramid_max_levels() || !H || !W) {
    set_error("%s: nlevel %d not in [1,%d] or null size arrays", fn, n, convex_pyramid_max_levels());
    return false;
  }
  if (factor != 4) {
    set_error("%s: factor %d (the pyramid form takes 4, the decoder's)", fn, factor);
    return false;
  }
  for (int l = 0; l < n; ++l)
    if (!check_convex(fn, B, H[l], W[l], factor)) return false;
  return true;
}

long long usf_convex_upsample_pyramid_bwd_scratch(int nlevel, const int* H, const int* W, int B) {
  if (nlevel < 1 || nlevel > convex_pyramid_max_levels() || !H || !W || B <= 0) return 0;
  long long n = 0;
  for (int l = 0; l < nlevel; ++l) n += convex_bwd_scratch(B, H[l], W[l]);
  return n;
}

int usf_convex_upsample_pyramid_f32(int nlevel, const float* const* flow, const float* const* mask, float* const* out,
                                    const int* H, const int* W, int B, int factor, float mask_scale, void* stream) {
  clear_error();
  const char* fn = "usf_convex_upsample_pyramid_f32";
  if (!check_convex_pyr(fn, nlevel, H, W, B, factor)) return USF_EINVAL;
  if (!flow || !mask || !out) {
    set_error("%s: null pointer array", fn);
    return USF_EINVAL;
  }
  for (int l = 0; l < nlevel; ++l)
    if (!flow[l] || !mask[l] || !out[l]) {
      set_error("%s: level %d: null pointer", fn, l);
      return USF_EINVAL;
    }
  if (const int pe = pre_check(fn, (hipStream_t)stream)) return pe;
  return finish(fn, convex_pyr_fwd_launch(nlevel, flow, mask, out, H, W, B, factor, mask_scale, (hipStream_t)stream),
                (hipStream_t)stream);
}

int usf_convex_upsample_pyramid_bwd_f32(int nlevel, const float* const* flow, const float* const* mask,
                                        const float* const* grad_out, float* const* grad_flow,
                                        float* const* grad_mask, float* scratch, long long scratch_floats,
                                        const int* H, const int* W, int B, int factor, float mask_scale,
                                        void* stream) {
  clear_error();
  const char* fn = "usf_convex_upsample_pyramid_bwd_f32";
  if (!check_convex_pyr(fn, nlevel, H, W, B, factor)) return USF_EINVAL;
  if (!flow || !mask || !grad_out) {
    set_error("%s: null input pointer array", fn);
    return USF_EINVAL;
  }
  for (int l = 0; l < nlevel; ++l)
    if (!flow[l] || !mask[l] || !grad_out[l] || (grad_flow && !grad_flow[l]) || (grad_mask && !grad_mask[l])) {
      set_error("%s: level %d: null pointer", fn, l);
      return USF_EINVAL;
    }
  if (grad_flow && (!scratch || scratch_floats < usf_convex_upsample_pyramid_bwd_scratch(nlevel, H, W, B))) {
    set_error("%s: grad_flow needs scratch of usf_convex_upsample_pyramid_bwd_scratch floats", fn);
    return USF_EINVAL;
  }
  if (!grad_flow && !grad_mask) return 0;
  if (const int pe = pre_check(fn, (hipStream_t)stream)) return pe;
  return finish(fn,
                convex_pyr_bwd_launch(nlevel, flow, mask, grad_out, grad_flow, grad_mask, scratch, H, W, B, factor,
                                      mask_scale, (hipStream_t)stream),
                (hipStream_t)stream);
}

int usf_area_pyramid_f32(const float* x, float* out1, float* out2, float* out3, int B, int C, int H,
                         int W, void* stream) {
  clear_error();
  const char* fn = "usf_area_pyramid_f32";
  if (!check_dims(fn, B, C, H, W)) return USF_EINVAL;
  if (H % 8 != 0 || W % 8 != 0) {
    set_error("%s: H=%d and W=%d must be multiples of 8", fn, H, W);
    return USF_EINVAL;
  }
  if (!x || !out1 || !out2 || !out3) {
    set_error("%s: null pointer", fn);
    return USF_EINVAL;
  }
  if (const int pe = pre_check(fn, (hipStream_t)stream)) return pe;
  return finish(fn, area_pyramid_launch(x, out1, out2, out3, (long long)B * C, H, W, (hipStream_t)stream),
                (hipStream_t)stream);
}

int usf_stream_copy_f32(const float* src, float* dst, long long n, void* stream) {
  clear_error();
  if (!src || !dst || n <= 0 || n % 4 != 0 || (reinterpret_cast<uintptr_t>(src) & 15) ||
      (reinterpret_cast<uintptr_t>(dst) & 15)) {
    set_error("usf_stream_copy_f32: need 16-byte aligned pointers and n %% 4 == 0 (n=%lld)", n);
    return USF_EINVAL;
  }
  if (const int pe = pre_check("usf_stream_copy_f32", (hipStream_t)stream)) return pe;
  return finish("usf_stream_copy_f32", stream_copy_launch(src, dst, n, (hipStream_t)stream), (hipStream_t)stream);
}

int usf_device_errors(void* stream, int clear) {
  clear_error();
  const int v = device_errors((hipStream_t)stream, clear != 0);
  if (v < 0) set_error("usf_device_errors: stream sync or flag read failed");
  return v;
}

int usf_set_variant(int op, int index) {
  clear_error();
  if (op < 0 || op > 3 || index < -1 || index >= variant_count(op)) {
    set_error("usf_set_variant: bad op %d / index %d", op, index);
    return USF_EINVAL;
  }
  set_variant_override(op, index);
  return variant_count(op);
}

}  // extern "C"
