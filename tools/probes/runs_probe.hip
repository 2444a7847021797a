// Unit probe for warp.hip's wave-level reduce-by-key helpers (row_runs,
// run_sum): one wave per test vector; dumps pos/maxlen/tail/take/give and the
// run sums per lane for comparison with a Python model (tools/gpu_runs_probe.sh).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../unsamflow_amd/csrc/warp.hip"

namespace usf {
void set_error(const char*, ...) {}
void clear_error() {}
int variant_override(int) { return -1; }
}  // namespace usf

__global__ void probe(const int* keys, const int* mw, const int* me, const int* hl, const int* hr,
                      const float* v, int* out_i, float* out_f) {
  const int l = threadIdx.x, base = blockIdx.x * 64;
  const usf::RowRuns r = usf::row_runs(keys[base + l], mw[base + l] != 0, me[base + l] != 0,
                                       hl[base + l] != 0, hr[base + l] != 0);
  const float s = usf::run_sum(v[base + l], r);
  int* o = out_i + (base + l) * 5;
  o[0] = r.pos; o[1] = r.maxlen; o[2] = r.tail; o[3] = r.take; o[4] = r.give;
  out_f[base + l] = s;
}

int main(int argc, char** argv) {
  const int n = atoi(argv[1]);  // number of vectors; input from stdin: per lane "key mw me hl hr v"
  std::vector<int> k(n * 64), mw(n * 64), me(n * 64), hl(n * 64), hr(n * 64);
  std::vector<float> v(n * 64);
  for (int i = 0; i < n * 64; ++i)
    if (scanf("%d %d %d %d %d %f", &k[i], &mw[i], &me[i], &hl[i], &hr[i], &v[i]) != 6) return 3;
  int *dk, *dmw, *dme, *dhl, *dhr, *oi;
  float *dv, *of;
  hipMalloc(&dk, n * 256); hipMalloc(&dmw, n * 256); hipMalloc(&dme, n * 256);
  hipMalloc(&dhl, n * 256); hipMalloc(&dhr, n * 256); hipMalloc(&dv, n * 256);
  hipMalloc(&oi, n * 64 * 5 * 4); hipMalloc(&of, n * 256);
  hipMemcpy(dk, k.data(), n * 256, hipMemcpyHostToDevice);
  hipMemcpy(dmw, mw.data(), n * 256, hipMemcpyHostToDevice);
  hipMemcpy(dme, me.data(), n * 256, hipMemcpyHostToDevice);
  hipMemcpy(dhl, hl.data(), n * 256, hipMemcpyHostToDevice);
  hipMemcpy(dhr, hr.data(), n * 256, hipMemcpyHostToDevice);
  hipMemcpy(dv, v.data(), n * 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(n), dim3(64), 0, 0, dk, dmw, dme, dhl, dhr, dv, oi, of);
  std::vector<int> hi(n * 64 * 5);
  std::vector<float> hf(n * 64);
  hipMemcpy(hi.data(), oi, hi.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hf.data(), of, hf.size() * 4, hipMemcpyDeviceToHost);
  for (int i = 0; i < n * 64; ++i)
    printf("%d %d %d %d %d %.9g\n", hi[i * 5], hi[i * 5 + 1], hi[i * 5 + 2], hi[i * 5 + 3], hi[i * 5 + 4], hf[i]);
  return 0;
}
