// fp32 global-atomic throughput probe: the ceiling of the warp backward's
// grad_x scatter (global_atomic_add_f32, no return value).
// Each lane adds to one float; consecutive lanes hit consecutive floats (the
// scatter's run tails: one contiguous row piece per wave instruction). Cases:
//   contiguous: every atomic to a distinct address, N atomics over N floats;
//   reuse2: every address receives 2 atomics from different waves (the
//           north/south corner rows of neighbouring pixel rows);
//   store: plain stores of the same pattern, for comparison.
// Prints G atomic lane-ops per second per case (hipEvent timing, median of 5).
// Usage: atomic_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

__global__ void add_contig(float* __restrict__ p, long long n, int reps) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int r = 0; r < reps; ++r) atomicAdd(p + i, 1.0f);
}

__global__ void add_reuse2(float* __restrict__ p, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * n) return;
  atomicAdd(p + (i % n), 1.0f);  // the second half of the grid revisits the first half's cells
}

__global__ void store_contig(float* __restrict__ p, long long n) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  p[i] = 1.0f;
}

template <class F>
static float time_ms(F f) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  std::vector<float> v;
  for (int k = 0; k < 6; ++k) {
    (void)hipEventRecord(a);
    f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    if (k) v.push_back(ms);  // first launch is warm-up
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const long long n = 16LL * 32 * 64 * 208;  // the warp backward's L4 grad_x at batch 16 (6.8 M)
  float* p = nullptr;
  if (hipMalloc(&p, 2 * n * sizeof(float)) != hipSuccess) return 1;
  (void)hipMemset(p, 0, 2 * n * sizeof(float));
  const int bs = 256;
  const unsigned g1 = (unsigned)((n + bs - 1) / bs), g2 = (unsigned)((2 * n + bs - 1) / bs);
  const float t1 = time_ms([&] { hipLaunchKernelGGL(add_contig, dim3(g1), dim3(bs), 0, 0, p, n, 1); });
  const float t2 = time_ms([&] { hipLaunchKernelGGL(add_contig, dim3(g1), dim3(bs), 0, 0, p, n, 2); });
  const float t3 = time_ms([&] { hipLaunchKernelGGL(add_reuse2, dim3(g2), dim3(bs), 0, 0, p, n); });
  const float t4 = time_ms([&] { hipLaunchKernelGGL(store_contig, dim3(g1), dim3(bs), 0, 0, p, n); });
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("{\"n\": %lld, \"contig_1_us\": %.2f, \"contig_1_gops\": %.1f, \"contig_2_us\": %.2f, "
              "\"contig_2_gops\": %.1f, \"reuse2_us\": %.2f, \"reuse2_gops\": %.1f, \"store_us\": %.2f, "
              "\"store_gbps\": %.1f}\n",
              n, t1 * 1e3, n / (t1 * 1e-3) / 1e9, t2 * 1e3, 2 * n / (t2 * 1e-3) / 1e9, t3 * 1e3,
              2 * n / (t3 * 1e-3) / 1e9, t4 * 1e3, 4.0 * n / (t4 * 1e-3) / 1e9);
  (void)hipFree(p);
  return 0;
}
