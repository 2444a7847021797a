// LDS bank-conflict calibration probe: each kernel issues ITERS ds_read_b128 (or
// ds_read_b64) per lane at a fixed per-lane address pattern, so
// SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS measures the extra cycles of the pattern.
// Build: hipcc --offload-arch=gfx950 -O3 lds_probe.hip -o lds_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__device__ int pattern(int l, int w) {
  if (MODE == 0) return l * 4;                               // b128 linear
  if (MODE == 1) return (l % 8 + w) * 48 + (l / 8) * 4;      // b128 col-major stride 48
  if (MODE == 2) return (l / 8 + w) * 40 + (l % 8) * 4;      // b128 row-major stride 40
  if (MODE == 3) return (l / 8 + w) * 74 + (l % 8) * 8;      // b64 row-major stride 74
  if (MODE == 4) return l * 2;                               // b64 linear
  if (MODE == 5) return (l / 8 + w) * 72 + (l % 8) * 8;      // b128 row-major stride 72 (PX=8 v3)
  if (MODE == 6) return (l / 8 + w) * 76 + (l % 8) * 8;      // b128 row-major stride 76
  return 0;
}

template <int MODE>
__global__ void probe(float* out, int iters) {
  __shared__ __attribute__((aligned(16))) float s[8192];
  for (int i = threadIdx.x; i < 8192; i += blockDim.x) s[i] = (float)i;
  __syncthreads();
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned addr = pattern<MODE>(l, w) * 4u;
  float acc = 0.f;
  constexpr bool B64 = MODE == 3 || MODE == 4;
  for (int it = 0; it < iters; ++it) {
    if (B64) {
      __attribute__((ext_vector_type(2))) float v;
      asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
      acc += v.x + v.y;
    } else {
      __attribute__((ext_vector_type(4))) float v;
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
      acc += v.x + v.y + v.z + v.w;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 256 * sizeof(float));
  probe<0><<<256, 256>>>(out, 1000);
  probe<1><<<256, 256>>>(out, 1000);
  probe<2><<<256, 256>>>(out, 1000);
  probe<3><<<256, 256>>>(out, 1000);
  probe<4><<<256, 256>>>(out, 1000);
  probe<5><<<256, 256>>>(out, 1000);
  probe<6><<<256, 256>>>(out, 1000);
  hipDeviceSynchronize();
  printf("probe done\n");
  hipFree(out);
  return 0;
}
