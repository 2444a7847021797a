/*
 * unsamflow_hip.h — C ABI of libunsamflow_hip.so, the MI355X (gfx950) native
 * plugin behind UnSAMFlow's cost-volume hot path.
 *
 * This library replaces, for the PWCLite call sites, the reference's native
 * plugin and the ATen sampler it leans on:
 *
 *   usf_corr_fwd_f32  <- correlation_cuda.forward
 *                        (models/correlation_package/correlation_cuda.cc:10-86,
 *                         pybind export :167-170; Python caller
 *                         models/correlation_package/correlation.py:9-38)
 *   usf_corr_bwd_f32  <- correlation_cuda.backward
 *                        (models/correlation_package/correlation_cuda.cc:88-165;
 *                         Python caller correlation.py:40-72)
 *   usf_corr_{fwd,bwd}_ex_f32 <- the same plus the decoder's LeakyReLU and the
 *                        concat into the flow-estimator input (pwclite.py:
 *                        307-308, 364-366)
 *   usf_warp_fwd_f32  <- grid_sample(bilinear, align_corners=True) inside
 *                        flow_warp (utils/warp_utils.py:97-106, incl.
 *                        mesh_grid :7-13 and norm_grid :16-23)
 *   usf_warp_fwd_up_f32 <- the decoder's F.interpolate(flow * 2) followed by
 *                        flow_warp (pwclite.py:299-302) in one launch
 *   usf_warp_bwd_f32 / usf_warp_bwd_ex_f32 / usf_warp_bwd_persist_f32
 *                     <- grid_sampler_2d_backward reached from flow_warp's
 *                        autograd graph (warp_utils.py:103-105)
 *   usf_splat_map_f32 <- get_corresponding_map (warp_utils.py:26-94,
 *                        scatter_add_ of bilinear weights)
 *   usf_occ_backward_f32 / usf_occ_backward_persist_f32
 *                     <- get_occu_mask_backward (warp_utils.py:120-126),
 *                        caller losses/flow_loss.py:101-103 (occ_from_back)
 *   usf_occ_vis_pair_persist_f32 <- both directions' 1 - get_occu_mask_backward
 *                        at once (losses/flow_loss.py:101-103)
 *   usf_occ_bidirection_f32 <- get_occu_mask_bidirection (warp_utils.py:109-117),
 *                        caller losses/flow_loss.py:104-107 (occ_from_back = false)
 *   usf_photo_loss_*  <- the per-scale warp + loss_photomatric composition of
 *                        losses/flow_loss.py:127-148
 *   usf_area_pyramid  <- the loss's per-scale F.interpolate(im, mode="area")
 *                        (losses/flow_loss.py:128-129)
 *   usf_flow_upsample_* <- F.interpolate(flow * k, scale_factor=k, bilinear,
 *                        align_corners=True) of the decoder (pwclite.py:299-301;
 *                        SURVEY §8f row 4)
 *   usf_convex_upsample_* <- UpFlowNetwork.upsample_flow + its 0.25 mask scale
 *                        (pwclite.py:148-166, the learned x4 output upsampler;
 *                        SURVEY §8f row 4)
 *
 * Contract (all entry points):
 *   - Pointers are DEVICE pointers to fp32 NCHW tensors. x/x1/x2/gout/out/gx*
 *     are dense (contiguous). The flow tensor may have any batch stride
 *     (flow_bstride, in elements) with a dense [2,H,W] per-sample block, so
 *     the loss's channel slices flow[:, :2] / flow[:, 2:]
 *     (losses/flow_loss.py:130-131) need no copy.
 *   - The caller allocates every output; the library never allocates,
 *     never keeps a pointer after return and has no global state except a
 *     thread-local error string and the usf_set_variant tuning override.
 *     Calls are reentrant (the backward runs on the autograd engine's device
 *     thread). The *_persist_* entries keep state in a CALLER-owned workspace
 *     from one call to the next (see each).
 *   - Calls are asynchronous on `stream` (a hipStream_t; NULL = legacy
 *     default stream).
 *   - Return value: 0 on success; a positive hipError_t from a failed
 *     launch; USF_EINVAL (-1) for bad arguments (nothing launched).
 *     usf_last_error_string() describes the last failure on this thread.
 *     The reference instead returned 1/0 and raised AT_ERROR("CUDA call
 *     failed") (correlation_cuda.cc:80-82, :160-162); the Python layer raises
 *     RuntimeError with this string.
 *   - Nullable gradient outputs mean "not needed" (ctx.needs_input_grad).
 */
#ifndef UNSAMFLOW_HIP_H
#define UNSAMFLOW_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define USF_ABI_VERSION 8
#define USF_EINVAL (-1)
#define USF_EDEVICE (-2) /* a kernel raised a device error flag (USF_SYNC_CHECK=1 only) */

/* device error flags (usf_device_errors) */
#define USF_DEVERR_WARP_OVERFLOW 1 /* binned warp backward: overflow list past its capacity */
#define USF_DEVERR_WORKSPACE_DIRTY 2 /* a *_persist_* workspace not left reusable (USF_SYNC_CHECK=1) */

/* padding modes for the warp (flow_warp `pad` argument) */
#define USF_PAD_ZEROS 0
#define USF_PAD_BORDER 1

/* ABI version of the loaded library (== USF_ABI_VERSION it was built with). */
int usf_abi_version(void);

/* Identity of this build: 16 hex digits of a sha256 over the library's
 * sources, headers and compiler flags (unsamflow_amd/build.py build_id).
 * Measurement summaries (PMC traffic) carry it, so a figure is only ever
 * attributed to the build it was measured on. */
const char* usf_build_id(void);

/* Human-readable description of the last error on the calling thread
 * ("" if none). The pointer stays valid until the next call on this thread. */
const char* usf_last_error_string(void);

/* Local correlation, forward.
 *   out[b, (dy+d)*(2d+1)+(dx+d), y, x] =
 *       (1/C) * sum_c x1[b,c,y,x] * X2(b,c,y+dy,x+dx),  X2 = 0 outside HxW
 * x1, x2: [B,C,H,W]; out: [B,(2d+1)^2,H,W]. 1 <= d <= 4.
 * Semantics of correlation_native.py:13-23 == correlation_cuda forward with
 * pad_size=d, kernel_size=1, stride1=stride2=1 (correlation_cuda.cc:19-34). */
int usf_corr_fwd_f32(const float* x1, const float* x2, float* out,
                     int B, int C, int H, int W, int d, void* stream);

/* Local correlation, backward. gout: [B,(2d+1)^2,H,W].
 *   gx1[b,c,y,x] = (1/C) sum_k gout[b,k,y,x]       * X2(b,c,y+dy_k,x+dx_k)
 *   gx2[b,c,y,x] = (1/C) sum_k G(b,k,y-dy_k,x-dx_k) * X1(b,c,y-dy_k,x-dx_k)
 * gx1 / gx2 may be NULL (not needed). Outputs are overwritten (not
 * accumulated) and the result is deterministic (no atomics). */
int usf_corr_bwd_f32(const float* x1, const float* x2, const float* gout,
                     float* gx1, float* gx2,
                     int B, int C, int H, int W, int d, void* stream);

/* Activations of the fused correlation epilogue (the decoder's in-place
 * nn.LeakyReLU(0.1) right after every correlation, pwclite.py:307-308). */
#define USF_ACT_NONE 0
#define USF_ACT_LEAKY_RELU 1

/* usf_corr_fwd_f32 writing into a channel slice of a larger buffer (the flow
 * estimator's concat input, pwclite.py:364-366): sample b's (2d+1)^2 output
 * planes start at out + b * out_bstride (elements; planes H*W apart), and
 * act = USF_ACT_LEAKY_RELU applies v > 0 ? v : v * slope to every output.
 * workspace (nullable, caller-provided device scratch of workspace_floats
 * floats): when it holds usf_corr_fwd_workspace(B,C,H,W,d) floats, small
 * levels split the channel loop over more workgroups and reduce the partials
 * in a fixed order (deterministic); otherwise the unsplit kernel runs.
 * act_mask (nullable; act = USF_ACT_LEAKY_RELU only): also write the sign
 * mask of the activated output, usf_corr_act_mask_words 64-bit words laid
 * out [B][2d+1][H][ceil(W/4)], bit 4*dx + (x % 4) of word
 * (b, dy, y, x/4) = (out at (b, dy*(2d+1)+dx, y, x) > 0). Pass it to
 * usf_corr_bwd_ex_f32 to apply the LeakyReLU derivative without re-reading
 * the activated output. */
int usf_corr_fwd_ex_f32(const float* x1, const float* x2, float* out, long long out_bstride,
                        int act, float slope, unsigned long long* act_mask, float* workspace,
                        long long workspace_floats, int B, int C, int H, int W, int d,
                        void* stream);

/* 64-bit words of the sign mask at this shape (0: bad arguments). */
long long usf_corr_act_mask_words(int B, int H, int W, int d);

/* Floats of workspace usf_corr_fwd_ex_f32 uses at this shape (0: no split). */
long long usf_corr_fwd_workspace(int B, int C, int H, int W, int d);

/* usf_corr_bwd_f32 reading its gradient from a channel slice (batch stride
 * g_bstride, elements). With act_out != NULL (the forward's activated output,
 * same layout as gout) the LeakyReLU derivative g * (act_out > 0 ? 1 : slope)
 * is applied first -- torch's leaky_relu_backward on the result, as for the
 * in-place module -- in one dense pass into `scratch` (caller-provided,
 * usf_corr_bwd_ex_scratch(B,C,H,W,d) floats; unused when act_out is NULL).
 * With act_mask != NULL (the forward's sign mask) the same
 * derivative is applied inside the backward kernel's gradient loads instead:
 * act_out and scratch are ignored and no extra pass runs. */
int usf_corr_bwd_ex_f32(const float* x1, const float* x2, const float* gout, long long g_bstride,
                        const float* act_out, const unsigned long long* act_mask, float slope,
                        float* scratch, float* gx1, float* gx2, int B, int C, int H, int W, int d,
                        void* stream);

/* Floats of `scratch` usf_corr_bwd_ex_f32 needs with act_out at this shape (0: none). */
long long usf_corr_bwd_ex_scratch(int B, int C, int H, int W, int d);

/* Bilinear backward warp (flow_warp), align_corners=True.
 * x: [B,C,H,W]; flow: [B,2,H,W] with batch stride flow_bstride (elements);
 * out: [B,C,H,W]. pad_mode: USF_PAD_BORDER or USF_PAD_ZEROS. */
int usf_warp_fwd_f32(const float* x, const float* flow, long long flow_bstride,
                     float* out, int B, int C, int H, int W, int pad_mode,
                     void* stream);

/* The decoder's flow upsampling and warp in ONE launch (ABI 8; pwclite.py:299-302:
 * flow = F.interpolate(coarse * 2, scale_factor=2, mode="bilinear",
 * align_corners=True); x2_warp = flow_warp(x2, flow)). coarse_flow: dense
 * [B,2,H/2,W/2] (H, W even); up_flow: dense [B,2,H,W], written (the same numbers
 * as usf_flow_upsample_f32 with factor 2); out: [B,C,H,W] = usf_warp_fwd_f32(x,
 * up_flow). */
int usf_warp_fwd_up_f32(const float* x, const float* coarse_flow, float* up_flow, float* out, int B, int C, int H,
                        int W, int pad_mode, void* stream);

/* Backward of usf_warp_fwd_f32. gout: [B,C,H,W] dense.
 * gx: [B,C,H,W] or NULL; overwritten (the library zeroes it, then scatters
 *     with fp32 atomics: summation order not fixed).
 * gflow: [B,2,H,W] dense or NULL; overwritten, deterministic. */
int usf_warp_bwd_f32(const float* x, const float* flow, long long flow_bstride,
                     const float* gout, float* gx, float* gflow,
                     int B, int C, int H, int W, int pad_mode, void* stream);

/* usf_warp_bwd_f32 with a caller workspace of usf_warp_bwd_workspace(B,H,W)
 * bytes (device memory, 16-byte aligned -- USF_EINVAL otherwise; contents need
 * not be initialised and are scratch after return). With it, gx is computed by
 * a binned gather: every source pixel is filed under the cell of its
 * north-west corner, then each target cell sums weight * gout over the
 * pixels filed under it and its three up-left neighbours in a fixed order,
 * and is written once -- no fp32 atomics and no zero fill, deterministic
 * except for pixels beyond 4 per cell (strongly compressive flow), which are
 * added with atomics afterwards. A smaller (or NULL) workspace falls back to
 * the scatter of usf_warp_bwd_f32. */
int usf_warp_bwd_ex_f32(const float* x, const float* flow, long long flow_bstride,
                        const float* gout, float* gx, float* gflow, void* workspace,
                        long long workspace_bytes, int B, int C, int H, int W, int pad_mode,
                        void* stream);

/* Workspace bytes usf_warp_bwd_ex_f32 uses for the binned gather. */
long long usf_warp_bwd_workspace(int B, int H, int W);

/* usf_warp_bwd_ex_f32's binned gather without the per-call zero fill (ABI 7):
 * workspace: usf_warp_bwd_persist_workspace(B,C,H,W) bytes, 16-byte aligned,
 * ZERO when first passed (one hipMemset at allocation). It is then reserved
 * for calls of this (B, C, H, W), ordered on one stream at a time; every call
 * leaves it in a state the next call uses as is (a parity word selects one of
 * two cell-count buffers; the gather zeroes the other), also under HIP graph
 * replay. Pixels beyond 4 per cell (fp32 atomics, summation order not fixed):
 * up to H*W = 8192, TWO launches, those pixels scattered into a dense overflow
 * buffer inside the workspace that the gather adds to its fixed-order sums and
 * re-zeroes; above, THREE launches, the pixels listed (the list length under
 * the same parity) and added by the overflow pass after the gather. gx may be
 * NULL (then no workspace is touched); C <= 256. Results equal
 * usf_warp_bwd_ex_f32's. */
int usf_warp_bwd_persist_f32(const float* x, const float* flow, long long flow_bstride,
                             const float* gout, float* gx, float* gflow, void* workspace,
                             long long workspace_bytes, int B, int C, int H, int W, int pad_mode,
                             void* stream);

/* Workspace bytes of usf_warp_bwd_persist_f32 (0 for invalid dimensions). */
long long usf_warp_bwd_persist_workspace(int B, int C, int H, int W);

/* Forward bilinear splat of unit mass (get_corresponding_map,
 * utils/warp_utils.py:26-94): every source pixel p lands at
 *   (x, y) = absolute ? (flow[b,0,p], flow[b,1,p]) : (px + flow[b,0,p], py + flow[b,1,p])
 * and adds (1-|x-cx|)*(1-|y-cy|) to each of its 4 integer neighbours inside
 * the image. map: [B,1,H,W] dense, overwritten (zeroed by the call on the
 * stream, then accumulated with fp32 atomics: summation order not fixed).
 * flow: [B,2,H,W] with batch stride flow_bstride. */
int usf_splat_map_f32(const float* flow, long long flow_bstride, float* map,
                      int B, int H, int W, int absolute, void* stream);

/* Occlusion mask from the backward flow (get_occu_mask_backward,
 * warp_utils.py:120-126): occ = clamp(splat_map(flow21), 0, 1) < th ? 1 : 0.
 * occ: [B,1,H,W] dense, overwritten. */
int usf_occ_backward_f32(const float* flow21, long long flow_bstride, float* occ,
                         int B, int H, int W, float th, void* stream);

/* usf_occ_backward_f32 in two launches (ABI 7): the splat accumulates into
 * map, the caller's persistent [B,1,H,W] fp32 buffer (map_bytes >= 4*B*H*W),
 * which must be ZERO when first passed; the threshold pass is its only reader
 * and zeroes it again, so no fill runs per call (graph-replay safe). One
 * stream at a time per map. occ: [B,1,H,W] dense, overwritten. */
int usf_occ_backward_persist_f32(const float* flow21, long long flow_bstride, float* occ, float* map,
                                 long long map_bytes, int B, int H, int W, float th, void* stream);

/* Both directions of the with_bk loss's visibility masks in two launches
 * (losses/flow_loss.py:101-103: vis_mask1 = 1 - get_occu_mask_backward(
 * top_flow[:, 2:], 0.2), vis_mask2 = 1 - get_occu_mask_backward(top_flow[:, :2],
 * 0.2)): one splat over both halves of the dense [B,4,H,W] flow4 (batch stride
 * 4*H*W) into the persistent map (a caller-owned buffer of >= 8*B*H*W bytes,
 * ZERO when first passed, re-zeroed by the call), then one threshold pass.
 * vis: [2,B,1,H,W] dense, overwritten: vis[0] = vis_mask1, vis[1] = vis_mask2
 * (1 or 0; masks equal get_occu_mask_backward's except where a splat sum lies
 * within fp32 rounding of th, whose summation order is not fixed). One stream
 * at a time per map. */
int usf_occ_vis_pair_persist_f32(const float* flow4, long long flow_bstride, float* vis, float* map,
                                 long long map_bytes, int B, int H, int W, float th, void* stream);

/* Forward-backward consistency occlusion mask (get_occu_mask_bidirection,
 * utils/warp_utils.py:109-117; stage-1 configs, occ_from_back = false), fused:
 *   w21 = flow_warp(flow21, flow12, pad="zeros"); d = flow12 + w21
 *   occ = |d|^2 > scale * (|flow12|^2 + |w21|^2) + bias ? 1 : 0
 * flow12, flow21: [B,2,H,W] with batch strides (channel slices allowed);
 * occ: [B,1,H,W] dense, overwritten. Each sum/product rounded as torch does. */
int usf_occ_bidirection_f32(const float* flow12, long long flow12_bstride, const float* flow21,
                            long long flow21_bstride, float* occ, int B, int H, int W,
                            float scale, float bias, void* stream);

/* Fused occlusion-aware photometric loss of one scale and direction
 * (losses/flow_loss.py:127-148, loss_photomatric :33-50, SSIM
 * losses/loss_blocks.py:53-72, w_ternary = 0):
 *   rec = flow_warp(src, flow, pad_mode)
 *   L = (w_l1 * mean |tgt - rec| * m + w_ssim * mean SSIM(rec*m, tgt*m))
 *       / (mean m + 1e-6)
 * src, tgt: [B,C,H,W] dense, 1 <= C <= 3 (images); mask: [B,1,H,W] dense; flow:
 * [B,2,H,W] with batch stride flow_bstride. partials: caller scratch of
 * usf_photo_loss_partials(B,H,W) floats. out: 3 floats = {L, c_l1, c_ssim}
 * (c_* are what the backward needs). grad_basis: NULL (no gradient wanted), or
 * [B,4,H,W] dense, overwritten with the per-pixel flow-gradient basis
 * {A_x, A_y, S_x, S_y}: dL/dflow = c_l1 * A + c_ssim * S (the L1 and the SSIM
 * parts; L is linear in both), computed in the same pass. Deterministic
 * (fixed-order sums). usf_photo_loss_partials(B,H,W) is per direction. */
int usf_photo_loss_partials(int B, int H, int W);
int usf_photo_loss_fwd_f32(const float* src, const float* tgt, const float* mask,
                           const float* flow, long long flow_bstride, float* partials,
                           float* out, float* grad_basis, int B, int C, int H, int W,
                           int pad_mode, float w_l1, float w_ssim, void* stream);

/* Both directions of a with_bk scale in one launch (flow_loss.py:130-131,
 * 143-148): direction 0 warps im2 by flow[:, 0:2] onto im1
 * under mask1, direction 1 warps im1 by flow[:, 2:4] onto im2 under mask2.
 * flow: [B,4,H,W] with batch stride flow_bstride (dense [4,H,W] per sample);
 * partials: 2 * usf_photo_loss_partials(B,H,W) floats; out: 6 floats
 * {L, c_l1, c_ssim} per direction; grad_basis: NULL or [B,2,4,H,W] dense. */
int usf_photo_loss_pair_fwd_f32(const float* im1, const float* im2, const float* mask1,
                                const float* mask2, const float* flow, long long flow_bstride,
                                float* partials, float* out, float* grad_basis, int B, int C,
                                int H, int W, int pad_mode, float w_l1, float w_ssim,
                                void* stream);

/* The with_bk pairs of up to 4 loss scales in ONE launch (+ one final
 * reduction): scale k (largest first) is usf_photo_loss_pair_fwd_f32's call
 * with im1[k], im2[k], mask1[k], mask2[k], flow[k] (batch stride
 * flow_bstride[k]), H[k] x W[k]; the small scales' strips fill the chip's tail
 * instead of each paying a launch and a drain (flow_loss.py:120-148, the scale
 * loop). Arrays are HOST arrays of nscale entries (1 <= nscale <= 4) holding
 * device pointers. partials: usf_photo_loss_pyramid_partials(nscale, H, W, B)
 * floats; out: 6 * nscale floats ({L, c_l1, c_ssim} per direction per scale);
 * grad_basis: NULL (no gradient) or nscale [B,8,H[k],W[k]] buffers. Results
 * equal nscale separate usf_photo_loss_pair_fwd_f32 calls bit for bit. */
long long usf_photo_loss_pyramid_partials(int nscale, const int* H, const int* W, int B);
int usf_photo_loss_pyramid_fwd_f32(int nscale, const float* const* im1, const float* const* im2,
                                   const float* const* mask1, const float* const* mask2, const float* const* flow,
                                   const long long* flow_bstride, const int* H, const int* W, float* partials,
                                   long long partials_floats, float* out, float* const* grad_basis, int B, int C,
                                   int pad_mode, float w_l1, float w_ssim, void* stream);

/* Its backward, every scale in one launch: grad_flow[k] ([B,4,H[k],W[k]],
 * overwritten) = per direction d (c_l1 A + c_ssim S) * grad_loss[2 k + d]
 * from grad_basis[k] and coef = the forward's out. Host arrays of device
 * pointers, as above. */
int usf_photo_loss_pyramid_bwd_f32(int nscale, const float* const* grad_basis, const float* coef,
                                   const float* grad_loss, float* const* grad_flow, const int* H, const int* W, int B,
                                   void* stream);

/* Backward of usf_photo_loss_fwd_f32 (ndir = 1) or _pair_fwd_f32 (ndir = 2)
 * w.r.t. the flow only (the mask and the images carry no gradient):
 * grad_flow[:, 2d:2d+2] = (c_l1 * A + c_ssim * S) * grad_loss[d] per direction d.
 * grad_basis: the forward's [B,ndir,4,H,W] basis; coef: the forward's `out`
 * (3 * ndir floats, device); grad_loss: ndir device floats; grad_flow:
 * [B,2*ndir,H,W] dense, overwritten, deterministic. */
int usf_photo_loss_bwd_f32(const float* grad_basis, const float* coef, const float* grad_loss,
                           float* grad_flow, int B, int H, int W, int ndir, void* stream);

/* Decoder flow upsampling (pwclite.py:299-301 and the x4 output flows):
 *   out = F.interpolate(flow * factor, scale_factor=factor, mode="bilinear",
 *                       align_corners=True)
 * flow: [B,C,H,W] dense; out: [B,C,H*factor,W*factor] dense, overwritten. */
int usf_flow_upsample_f32(const float* flow, float* out, int B, int C, int H, int W,
                          int factor, void* stream);

/* Its backward: grad_flow [B,C,H,W] (overwritten, deterministic gather form)
 * from grad_out [B,C,H*factor,W*factor]. */
int usf_flow_upsample_bwd_f32(const float* grad_out, float* grad_flow, int B, int C, int H,
                              int W, int factor, void* stream);

/* The same backward of grad_a + grad_b (summed per element in the kernel: the
 * same numbers as an add followed by usf_flow_upsample_bwd_f32; ABI 8) -- the
 * decoder's upsampled flow receives one gradient from the warp and one from
 * its other uses (usf_warp_fwd_up_f32's backward). */
int usf_flow_upsample_bwd_sum_f32(const float* grad_a, const float* grad_b, float* grad_flow, int B, int C, int H,
                                  int W, int factor, void* stream);

/* The learned (convex) x`factor` upsampler of the output flows
 * (UpFlowNetwork, pwclite.py:148-166; RAFT-style), factor in {2, 4, 8}
 * (the reference uses 4):
 *   w   = softmax(mask_scale * mask viewed [B,1,9,f,f,H,W], dim 2)
 *   out[b,c,f*y+i,f*x+j] = sum_k w[b,k,i,j,y,x] * f * flow[b,c,y+ky-1,x+kx-1]
 * (k = 3 ky + kx, zero outside the image; mask_scale = 0.25 at :165).
 * flow: [B,2,H,W] dense; mask: [B,9*f*f,H,W] dense (the convs' raw output);
 * out: [B,2,f*H,f*W] dense, overwritten. */
int usf_convex_upsample_f32(const float* flow, const float* mask, float* out, int B, int H, int W,
                            int factor, float mask_scale, void* stream);

/* Floats of scratch usf_convex_upsample_bwd_f32 needs when grad_flow is wanted
 * (18 * B * H * W). */
long long usf_convex_upsample_bwd_scratch(int B, int H, int W);

/* Its backward from grad_out [B,2,f*H,f*W]: grad_flow [B,2,H,W] and grad_mask
 * [B,9*f*f,H,W] w.r.t. the RAW mask (mask_scale applied), both dense,
 * overwritten, deterministic (no atomics); either may be NULL. scratch:
 * usf_convex_upsample_bwd_scratch floats when grad_flow is non-NULL. */
int usf_convex_upsample_bwd_f32(const float* flow, const float* mask, const float* grad_out,
                                float* grad_flow, float* grad_mask, float* scratch, int B, int H,
                                int W, int factor, float mask_scale, void* stream);

/* The decoder's output flows of every level (nlevel <= 6) through the convex
 * x4 upsampler in ONE launch (factor 4 only): level l is
 * usf_convex_upsample_f32(flow[l], mask[l], out[l], B, H[l], W[l], 4,
 * mask_scale); the levels' blocks share one grid, the largest level first.
 * Arrays are HOST arrays of device pointers. Results equal the per-level calls
 * bit for bit. PWCLite defers the upsampling to the end of its decoder (the
 * upsampled flows feed only the loss). */
int usf_convex_upsample_pyramid_f32(int nlevel, const float* const* flow, const float* const* mask, float* const* out,
                                    const int* H, const int* W, int B, int factor, float mask_scale, void* stream);

/* Floats of scratch usf_convex_upsample_pyramid_bwd_f32 needs with grad_flow
 * (the sum of usf_convex_upsample_bwd_scratch over the levels). */
long long usf_convex_upsample_pyramid_bwd_scratch(int nlevel, const int* H, const int* W, int B);

/* Its backward: usf_convex_upsample_bwd_f32 of every level in one launch (+
 * one 9-tap gather launch for all grad_flows). grad_flow / grad_mask: NULL
 * (not wanted) or host arrays of per-level device buffers. */
int usf_convex_upsample_pyramid_bwd_f32(int nlevel, const float* const* flow, const float* const* mask,
                                        const float* const* grad_out, float* const* grad_flow,
                                        float* const* grad_mask, float* scratch, long long scratch_floats,
                                        const int* H, const int* W, int B, int factor, float mask_scale,
                                        void* stream);

/* The loss's image pyramid (unFlowLoss per scale s: F.interpolate(im,
 * (H >> s, W >> s), mode="area"), flow_loss.py:128-129): out_s = mean of each
 * 2^s x 2^s block, summed in row-major order as torch's CPU kernel does
 * (bit-exact). x: [B,C,H,W] dense with H % 8 == 0 and W % 8 == 0; out1/2/3:
 * [B,C,H/2,W/2], [B,C,H/4,W/4], [B,C,H/8,W/8] dense, overwritten. */
int usf_area_pyramid_f32(const float* x, float* out1, float* out2, float* out3, int B, int C,
                         int H, int W, void* stream);

/* Device-side error flags raised by kernels since the last clear (a bitmask
 * of USF_DEVERR_*; 0 = none), after synchronising `stream`; clear != 0 resets
 * them. -1 if the synchronisation or the read failed. With USF_SYNC_CHECK=1
 * every entry point checks them after its launch and returns USF_EDEVICE. */
int usf_device_errors(void* stream, int clear);

/* STREAM copy of n floats (16-byte lanes; src and dst 16-byte aligned, n % 4
 * == 0): a measurement helper, bench.py's device-copy ceiling. */
int usf_stream_copy_f32(const float* src, float* dst, long long n, void* stream);

/* Tuning hook (benchmarking only; not needed for correct use).
 * Forces kernel variant `index` of `op` for d=4 launches in this process:
 * op 0 = correlation forward tile config, op 1 = correlation backward tile
 * config, op 2 = warp grad_x path (0 = the lane-merged per-pixel scatter, 1 =
 * the pixel-pair scatter, 2 = the binned gather, which needs a workspace), op 3 = photometric
 * loss kernel (one variant: 0 = row-streaming strips on producer / consumer wave
 * pairs; the tile and one-wave strip kernels were removed); index -1 restores the built-in choice. Returns the number of
 * variants of `op` (so index range is [0, n)), or USF_EINVAL for an unknown op
 * or out-of-range index. Process-wide; set it before launching, not
 * concurrently with launches. */
int usf_set_variant(int op, int index);

#ifdef __cplusplus
}
#endif
#endif /* UNSAMFLOW_HIP_H */
