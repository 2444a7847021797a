// Occupancy probe: how many workgroups of a given size and LDS footprint are
// resident per CU at once. Every wave stamps s_memrealtime at start, spins for
// ~20 us, stamps again and records HW_ID/XCC_ID; the host computes the maximum
// number of simultaneously resident workgroups per CU.
// Usage: occ_probe  (sweeps workgroup sizes at 36 KB of LDS) | occ_probe T:LDS_BYTES ...
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

__global__ void spin(unsigned long long* tr, int lds_floats) {
  extern __shared__ float dyn[];
  if (threadIdx.x < (unsigned)lds_floats) dyn[threadIdx.x] = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) __builtin_amdgcn_s_sleep(2);
  if ((threadIdx.x & 63) == 0) {
    const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    tr[w * 4 + 0] = t0;
    tr[w * 4 + 1] = __builtin_amdgcn_s_memrealtime();
    tr[w * 4 + 2] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                    (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    tr[w * 4 + 3] = blockIdx.x;
  }
}

int main(int argc, char** argv) {
  const int nwg = 2048;
  unsigned long long* tr;
  hipMalloc(&tr, (size_t)nwg * 16 * 4 * 8);
  std::vector<std::pair<int, int>> cfgs;
  for (int a = 1; a < argc; ++a) {
    int t = 0, l = 0;
    if (sscanf(argv[a], "%d:%d", &t, &l) == 2) cfgs.push_back({t, l});
  }
  if (cfgs.empty())
    for (int nt : {192, 256, 384, 512, 576, 640, 1024})
      for (int lds : {0, 36 * 1024}) cfgs.push_back({nt, lds});
  hipFuncSetAttribute(reinterpret_cast<const void*>(&spin), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (auto [nt, lds] : cfgs) {
    {
      hipMemset(tr, 0, (size_t)nwg * 16 * 4 * 8);
      hipLaunchKernelGGL(spin, dim3(nwg), dim3(nt), lds, 0, tr, lds / 4);
      hipDeviceSynchronize();
      const int nw = nwg * (nt / 64);
      std::vector<unsigned long long> h((size_t)nw * 4);
      hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost);
      std::map<unsigned, std::map<unsigned long long, std::pair<unsigned long long, unsigned long long>>> cu;
      for (int w = 0; w < nw; ++w) {
        const unsigned hw = (unsigned)h[w * 4 + 2], xcc = (unsigned)(h[w * 4 + 2] >> 32) & 0xF;
        const unsigned key = ((xcc * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 16 + ((hw >> 8) & 15);
        auto& iv = cu[key][h[w * 4 + 3]];
        iv.first = iv.first ? std::min(iv.first, h[w * 4]) : h[w * 4];
        iv.second = std::max(iv.second, h[w * 4 + 1]);
      }
      int best = 0;
      double tot = 0;
      for (auto& kv : cu) {
        std::vector<std::pair<unsigned long long, int>> ev;
        for (auto& b : kv.second) {
          ev.push_back({b.second.first, 1});
          ev.push_back({b.second.second, -1});
        }
        std::sort(ev.begin(), ev.end());
        int c = 0, m = 0;
        for (auto& e : ev) m = std::max(m, c += e.second);
        best = std::max(best, m);
        tot += m;
      }
      printf("wg=%4d threads (%2d waves) lds=%5d B: %zu CUs, max resident wg/CU %d (mean of per-CU max %.2f)\n", nt,
             nt / 64, lds, cu.size(), best, tot / cu.size());
    }
  }
  return 0;
}
