// FP32 VALU rate probe: plain v_fmac_f32 vs packed v_pk_fma_f32 on gfx950.
// 16 independent accumulators per lane (8 register pairs), inline asm so the
// compiler can neither fold nor repack them. Reports FLOP/clk/SIMD-equivalent
// TFLOP/s for each form at several waves per SIMD.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/probes/fma_rate tools/probes/fma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 2048;

__global__ __launch_bounds__(256) void fma_plain(float* out, float a, float b) {
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = threadIdx.x * 0.001f + i;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_fmac_f32_dpp (src0 from the neighbouring lane of the 16-lane row): the
// correlation backward's DPP-window variant issues 20 of every 36 FMAs this way
__global__ __launch_bounds__(256) void fma_dpp(float* out, float a, float b) {
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = threadIdx.x * 0.001f + i;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      asm volatile("v_fmac_f32_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                   : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

using f2 = float __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void fma_packed(float* out, float a, float b) {
  f2 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f2{threadIdx.x * 0.001f + i, (float)i};
  const f2 av = {a, a}, bv = {b, b};
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(av), "v"(bv));
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i].x + acc[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 256 * 64 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int wps = 1; wps <= 8; wps *= 2) {
    const int blocks = 256 * wps;  // 256 CUs x wps workgroups of 4 waves = wps waves per SIMD
    for (int form = 0; form < 3; ++form) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (form == 0) hipLaunchKernelGGL(fma_plain, dim3(blocks), dim3(256), 0, 0, out, 1.0001f, 0.5f);
        else if (form == 1) hipLaunchKernelGGL(fma_packed, dim3(blocks), dim3(256), 0, 0, out, 1.0001f, 0.5f);
        else hipLaunchKernelGGL(fma_dpp, dim3(blocks), dim3(256), 0, 0, out, 1.0001f, 0.5f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        const double flops = 2.0 * 16 * kIters * (double)blocks * 256;  // 16 fp32 FMAs per iteration per lane
        if (rep == 1)
          printf("%s waves/SIMD=%d: %.3f ms  %.1f TFLOP/s\n",
                 form == 0 ? "v_fmac_f32    " : form == 1 ? "v_pk_fma_f32  " : "v_fmac_f32_dpp", wps, ms,
                 flops / (ms * 1e-3) / 1e12);
      }
    }
  }
  return 0;
}
