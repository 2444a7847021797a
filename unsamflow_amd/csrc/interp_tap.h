// Bilinear align_corners=True tap of ATen's upsample_bilinear2d (third-party,
// torch 2.10; models/pwclite.py:299-301 calls it as F.interpolate(flow * k,
// scale_factor=k, mode="bilinear", align_corners=True)), shared by the flow
// upsampler (upsample.hip) and the warp forward that upsamples its flow on the
// fly (warp.hip), so both compute the same numbers: the source scale is
// (in - 1) / (out - 1) in fp32; src = scale * dst; i0 = floor(src),
// i1 = i0 + (i0 < in - 1), l1 = src - i0, l0 = 1 - l1;
// out = l0_y (l0_x v00 + l1_x v01) + l1_y (l0_x v10 + l1_x v11), v = k * x.
#pragma once
#include "usf_common.h"

namespace usf {

struct Lin {
  int i0, i1;
  float l0, l1;
};

__device__ __forceinline__ inline Lin lin_tap(int dst, float scale, int in) {
#pragma clang fp contract(off)
  const float src = scale * (float)dst;
  Lin t;
  t.i0 = (int)src;  // src >= 0: truncation == floor
  t.i1 = t.i0 + (t.i0 < in - 1 ? 1 : 0);
  t.l1 = src - (float)t.i0;
  t.l0 = 1.f - t.l1;
  return t;
}

// one output element of plane xp ([in_h][in_w]) at taps (ty, tx), times k
__device__ __forceinline__ inline float up_bilinear(const float* __restrict__ xp, int in_w, const Lin& ty,
                                                    const Lin& tx, float k) {
#pragma clang fp contract(off)
  const float v00 = xp[ty.i0 * in_w + tx.i0] * k, v01 = xp[ty.i0 * in_w + tx.i1] * k;
  const float v10 = xp[ty.i1 * in_w + tx.i0] * k, v11 = xp[ty.i1 * in_w + tx.i1] * k;
  return ty.l0 * (tx.l0 * v00 + tx.l1 * v01) + ty.l1 * (tx.l0 * v10 + tx.l1 * v11);
}

// align_corners=True source scale of one axis (host and device)
__host__ __device__ inline float ac_scale(int in, int out) {
  return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
}

}  // namespace usf
