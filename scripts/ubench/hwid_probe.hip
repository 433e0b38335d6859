// Where do the waves of a persistent launch land?  Every wave of a 4-wave workgroup records
// its HW_ID (SIMD, CU, SH, SE, workgroup slot) and XCC_ID; the host tallies, per SIMD, the
// physical wave indices (threadIdx.x / 64) of the workgroups resident on it.  Launch shape: the
// headline tile kernel's (4 waves, 40,800 B of dynamic LDS -> 4 workgroups per CU).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ void __launch_bounds__(256) probe(unsigned* out) {
  extern __shared__ unsigned lds[];
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
  if ((threadIdx.x & 63) == 0) {
    const unsigned w = blockIdx.x * 4 + (threadIdx.x >> 6);
    out[2 * w] = hw;
    out[2 * w + 1] = xcc;
  }
  lds[threadIdx.x] = hw;
  __syncthreads();
  // stay resident a while so all workgroups are co-resident
  for (int i = 0; i < 20000; ++i) __builtin_amdgcn_s_sleep(2);
  if (lds[threadIdx.x ^ 1] == 0xFFFFFFFFu) out[0] = 0;
}

int main() {
  const int G = 1024;
  unsigned* d;
  hipMalloc(&d, G * 4 * 2 * 4);
  hipFuncSetAttribute(reinterpret_cast<const void*>(probe),
                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipLaunchKernelGGL(probe, dim3(G), dim3(256), 40800, 0, d);
  if (hipDeviceSynchronize() != hipSuccess) { printf("fail\n"); return 1; }
  std::vector<unsigned> h(G * 8);
  hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  // per (xcc, se, sh, cu, simd): histogram of physical wave index; per CU: WG slots seen
  std::map<unsigned, std::vector<int>> simd;
  std::map<unsigned, int> cu_wgs;
  int same_slot = 0, diff_slot = 0, distinct_simd = 0;
  for (int g = 0; g < G; ++g) {
    unsigned slot0 = 0, mask = 0;
    for (int p = 0; p < 4; ++p) {
      const unsigned hw = h[2 * (g * 4 + p)], xcc = h[2 * (g * 4 + p) + 1] & 0xF;
      const unsigned s = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1,
                     se = (hw >> 13) & 7, tg = (hw >> 16) & 15;
      const unsigned key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + s;
      auto& v = simd[key];
      if (v.empty()) v.assign(4, 0);
      v[p]++;
      if (p == 0) { slot0 = tg; cu_wgs[key >> 2]++; }
      else if (tg == slot0) same_slot++; else diff_slot++;
      mask |= 1u << s;
    }
    if (mask == 0xF) distinct_simd++;
  }
  int balanced = 0, stacked = 0;
  for (auto& kv : simd) {
    int mx = 0;
    for (int c : kv.second) mx = std::max(mx, c);
    if (mx <= 1) balanced++; else stacked++;
  }
  printf("workgroups with 4 distinct SIMDs: %d / %d\n", distinct_simd, G);
  printf("tg_id equal across a workgroup's waves: %d, different: %d\n", same_slot, diff_slot);
  printf("CUs seen: %zu; SIMDs whose resident waves all have distinct wave indices: %d, "
         "with a repeated index: %d\n", cu_wgs.size(), balanced, stacked);
  int shown = 0;
  for (auto& kv : simd) {
    if (shown++ >= 8) break;
    printf("simd key %u: wave-index histogram %d %d %d %d\n", kv.first, kv.second[0],
           kv.second[1], kv.second[2], kv.second[3]);
  }
  return 0;
}
