// STREAM copy with 16-byte lanes: the device-copy ceiling bench.py reports
// beside the roofline (MI355X_MICROARCH.md measures 6.29 TB/s with a float4
// copy; torch's copy_ measured 4.7-5.3 TB/s on the same box). A grid-stride
// loop over float4s, 4 loads in flight per lane, grid sized to 8 workgroups
// per CU.
#include "usf_common.h"

namespace usf {
namespace {

__global__ __launch_bounds__(256) void stream_copy_kernel(const float4* __restrict__ src, float4* __restrict__ dst,
                                                          long long n4) {
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + 3 * stride < n4; i += 4 * stride) {
    const float4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n4; i += stride) dst[i] = src[i];
}

}  // namespace

hipError_t stream_copy_launch(const float* src, float* dst, long long n, hipStream_t s) {
  const long long n4 = n / 4;
  hipLaunchKernelGGL(stream_copy_kernel, dim3(256 * 8), dim3(256), 0, s, reinterpret_cast<const float4*>(src),
                     reinterpret_cast<float4*>(dst), n4);
  return hipGetLastError();
}

}  // namespace usf
