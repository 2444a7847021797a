// Phase-timing probe for the correlation kernels (not part of the library).
// Includes corr.hip with USF_TRACE so every wave records s_memrealtime
// (100 MHz) at its phase boundaries, runs one traced launch per shape and
// prints where the time goes:
//   span      first wave start -> last wave end
//   start     distribution of wave start times (dispatch / occupancy rounds)
//   phases    median per-wave duration of each phase
//   resident  max waves simultaneously resident per CU and per SIMD
// Caveat: the stamps cost registers (the fused backward goes from 163 to 189
// VGPRs, i.e. 2 instead of 3 waves/SIMD), so occupancy and absolute times of a
// traced run differ from the library's; use it for the phase breakdown.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -DUSF_TRACE -I unsamflow_amd/csrc -I include
//        -o tools/probes/bin/corr_trace tools/probes/corr_trace.hip; run: tools/gpu_trace.sh
// Usage: corr_trace fwd|bwd B C H W [variant]
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define USF_TRACE 1
#include "../../unsamflow_amd/csrc/corr.hip"

namespace usf {
void set_error(const char*, ...) {}
void clear_error() {}
}  // namespace usf

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

static double pct(std::vector<double> v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(p * (v.size() - 1) + 0.5))];
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s fwd|bwd B C H W [variant]\n", argv[0]);
    return 2;
  }
  const bool fwd = argv[1][0] == 'f';
  const int B = atoi(argv[2]), C = atoi(argv[3]), H = atoi(argv[4]), W = atoi(argv[5]);
  const int variant = argc > 6 ? atoi(argv[6]) : -1;
  usf::set_variant_override(fwd ? 0 : 1, variant);
  const size_t nx = (size_t)B * C * H * W, ng = (size_t)B * 81 * H * W;
  float *x1, *x2, *g, *o, *o2;
  CK(hipMalloc(&x1, nx * 4));
  CK(hipMalloc(&x2, nx * 4));
  CK(hipMalloc(&g, ng * 4));
  CK(hipMalloc(&o, std::max(nx, ng) * 4));
  CK(hipMalloc(&o2, nx * 4));
  CK(hipMemset(x1, 0, nx * 4));
  CK(hipMemset(x2, 0, nx * 4));
  CK(hipMemset(g, 0, ng * 4));
  const size_t max_waves = 1 << 18;
  unsigned long long* tr;
  CK(hipMalloc(&tr, max_waves * usf::kTraceSlots * 8));
  auto run = [&]() {
    if (fwd)
      CK(usf::corr_fwd_launch(x1, x2, o, B, C, H, W, 4, nullptr, usf::FwdEpi{81LL * H * W, 0, 0.f}));
    else
      CK(usf::corr_bwd_launch(x1, x2, g, o, o2, B, C, H, W, 4, nullptr, usf::BwdEpi{81LL * H * W}));  // both directions
  };
  for (int i = 0; i < 5; ++i) run();  // warm, untraced
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int i = 0; i < 20; ++i) run();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipMemset(tr, 0, max_waves * usf::kTraceSlots * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(usf::g_trace), &tr, sizeof(tr)));
  run();
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> h(max_waves * usf::kTraceSlots);
  CK(hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost));
  const int S = usf::kTraceSlots;
  size_t nw = 0;
  while (nw < max_waves && h[nw * S] != 0) ++nw;
  unsigned long long t0 = ~0ull, t1 = 0;
  std::vector<double> start, dur, ph[usf::kTraceSlots];
  struct Iv {
    unsigned long long a, b;
  };
  std::map<unsigned, std::vector<Iv>> per_cu, per_simd;
  for (size_t w = 0; w < nw; ++w) {
    const unsigned long long* r = &h[w * S];
    int last = 0;
    for (int k = 1; k < S - 1; ++k)
      if (r[k]) last = k;
    t0 = std::min(t0, r[0]);
    t1 = std::max(t1, r[last]);
    for (int k = 1; k <= last; ++k)
      if (r[k] && r[k - 1]) ph[k].push_back((r[k] - r[k - 1]) * 10.0 / 1000.0);
    const unsigned hw = (unsigned)r[S - 1], xcc = (unsigned)(r[S - 1] >> 32) & 0xF;
    const unsigned simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    const unsigned cu_key = (((xcc * 8 + se) * 2 + sh) * 16 + cu);
    per_cu[cu_key].push_back({r[0], r[last]});
    per_simd[cu_key * 4 + simd].push_back({r[0], r[last]});
    dur.push_back((r[last] - r[0]) * 10.0 / 1000.0);
  }
  for (size_t w = 0; w < nw; ++w) start.push_back((h[w * S] - t0) * 10.0 / 1000.0);
  auto max_res = [](std::map<unsigned, std::vector<Iv>>& m) {
    int best = 0;
    for (auto& kv : m) {
      std::vector<std::pair<unsigned long long, int>> ev;
      for (auto& iv : kv.second) {
        ev.push_back({iv.a, 1});
        ev.push_back({iv.b, -1});
      }
      std::sort(ev.begin(), ev.end());
      int cur = 0;
      for (auto& e : ev) best = std::max(best, cur += e.second);
    }
    return best;
  };
  printf("%s B=%d C=%d H=%d W=%d variant=%d: %.2f us/launch (20 launches), %zu waves, %zu CUs\n",
         fwd ? "fwd" : "bwd", B, C, H, W, variant, ms * 1000 / 20, nw, per_cu.size());
  printf("  traced span %.2f us; wave start p0/p50/p90/max %.2f/%.2f/%.2f/%.2f us\n",
         (t1 - t0) * 10.0 / 1000.0, pct(start, 0), pct(start, .5), pct(start, .9), pct(start, 1));
  printf("  wave duration p10/p50/p90/max %.2f/%.2f/%.2f/%.2f us\n", pct(dur, .1), pct(dur, .5),
         pct(dur, .9), pct(dur, 1));
  printf("  max resident waves per CU %d, per SIMD %d\n", max_res(per_cu), max_res(per_simd));
  // fwd: [1] prologue DMA issue, then per stage: loop, DMA wait, barrier + next DMA issue, compute
  // bwd: [1] prologue DMA + g slice (USF_TRACE waits for the g loads), [2] stage-0 wait, then
  //      per stage: barrier (after the previous combine), DMA issue, compute, wait for the
  //      next stage, barrier
  const int first = fwd ? 2 : 3, stride = fwd ? 4 : 5;
  printf("  prologue (median us):");
  for (int k = 1; k < first; ++k) printf(" [%d] %.2f", k, pct(ph[k], .5));
  printf("\n  per stage (median us) %s:\n",
         fwd ? "loop/wait/bar+issue/compute" : "combine+bar/issue/compute/wait/bar");
  for (int st = 0; first + stride * st + stride - 1 < S - 1 && !ph[first + stride * st].empty(); ++st) {
    printf("    stage %2d:", st);
    for (int k = 0; k < stride; ++k) printf(" %6.2f", pct(ph[first + stride * st + k], .5));
    printf("\n");
  }
  return 0;
}
