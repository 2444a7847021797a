// STREAM copy with 16-byte lanes: the device-copy ceiling bench.py reports
// beside the roofline (MI355X_MICROARCH.md measures 6.29 TB/s with a float4
// copy; torch's copy_ measured 4.6-5.3 TB/s on the same box). One 16 KiB
// chunk per workgroup, 16-byte nontemporal loads and stores, 4 in flight per
// lane (a grid-stride form with 8 workgroups per CU measured 4.6 TB/s).
#include "usf_common.h"

namespace usf {
namespace {

using f4 = float __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_copy_kernel(const f4* __restrict__ src, f4* __restrict__ dst,
                                                          long long n4) {
  // one 16 KiB block-contiguous chunk per workgroup, 4 loads in flight per lane
  const long long base = (long long)blockIdx.x * 1024 + threadIdx.x;
  f4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (base + 256 * k < n4) v[k] = __builtin_nontemporal_load(src + base + 256 * k);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (base + 256 * k < n4) __builtin_nontemporal_store(v[k], dst + base + 256 * k);
}

}  // namespace

hipError_t stream_copy_launch(const float* src, float* dst, long long n, hipStream_t s) {
  const long long n4 = n / 4;
  hipLaunchKernelGGL(stream_copy_kernel, dim3((unsigned)((n4 + 1023) / 1024)), dim3(256), 0, s,
                     reinterpret_cast<const f4*>(src), reinterpret_cast<f4*>(dst), n4);
  return hipGetLastError();
}

}  // namespace usf
