// Two questions for the protein kernel's substitution add:
//  1. semantics: v_pk_fma_f16 D, A, B, H op_sel:[0,1,0] op_sel_hi:[1,0,1] clamp with profile
//     words A = {sA, 1.0}, B = {sB, 1.0} must give D = {clamp(H.lo + sA), clamp(H.hi + sB)}
//     (lo lane: A.lo * B.hi + H.lo, hi lane: A.hi * B.lo + H.hi), bit-exact on f16 multiples
//     of 2^-11 in [-2048, 2048] * 2^-11;
//  2. issue rate of v_pk_fma_f16 (with op_sel) + v_pk_maximum3_f16 against
//     v_pk_add_f16 + v_pk_maximum3_f16 (8 independent chains per thread).
// Prints one JSON line per measurement.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define ITERS 4096

__global__ void sem(const uint32_t* A, const uint32_t* B, const uint32_t* H, uint32_t* D,
                    uint32_t* Dn, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t d, dn;
  asm volatile("v_pk_fma_f16 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,0,1] clamp"
               : "=v"(d) : "v"(A[i]), "v"(B[i]), "v"(H[i]));
  asm volatile("v_pk_fma_f16 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,0,1]"
               : "=v"(dn) : "v"(A[i]), "v"(B[i]), "v"(H[i]));
  D[i] = d;
  Dn[i] = dn;
}

template <int KIND>
__global__ void __launch_bounds__(256) rate(uint32_t* out, uint32_t seed) {
  uint32_t a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + 1) + i * 77;
  const uint32_t b = seed ^ 0x3C003C00u, c = seed ^ 0x00053C00u;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (KIND == 0)
        asm volatile("v_pk_add_f16 %0, %0, %1 clamp\n\tv_pk_maximum3_f16 %0, %0, %1, %2"
                     : "+v"(a[i]) : "v"(b), "v"(c));
      else if (KIND == 1)
        asm volatile(
            "v_pk_fma_f16 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,0,1] clamp\n\t"
            "v_pk_maximum3_f16 %0, %0, %1, %2"
            : "+v"(a[i]) : "v"(b), "v"(c));
      else
        asm volatile("v_perm_b32 %0, %0, %1, %2\n\tv_pk_add_f16 %0, %0, %1 clamp"
                     : "+v"(a[i]) : "v"(b), "v"(c));
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static uint16_t f16bits(int v) {
  _Float16 h = (_Float16)((float)v / 2048.0f);
  uint16_t u;
  std::memcpy(&u, &h, 2);
  return u;
}

template <int KIND>
static void run_rate(const char* name, int blocks) {
  uint32_t* out;
  (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(rate<KIND>, dim3(blocks), dim3(256), 0, 0, out, 3u);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(rate<KIND>, dim3(blocks), dim3(256), 0, 0, out, 3u);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double instr = blocks * 4.0 * ITERS * 8 * 2;
  std::printf("{\"kind\": \"%s\", \"waves_per_simd\": %.1f, \"ms\": %.3f, "
              "\"wave_instr_per_simd_cycle_at_2.4GHz\": %.3f}\n",
              name, blocks * 4.0 / 1024, ms, instr / (1024.0 * ms * 1e-3 * 2.4e9));
  (void)hipFree(out);
}

int main() {
  // semantics over every (sA, sB, H) on a grid of the exact range
  std::vector<uint32_t> A, B, H;
  std::vector<int> vs, vh, va, vb;
  const int S[] = {-2048, -200, -11, -4, -1, 0, 1, 4, 11, 200, 2047};
  const int HV[] = {0, 1, 5, 100, 1000, 2037, 2048};
  for (int sa : S)
    for (int sb : S)
      for (int hl : HV)
        for (int hh : HV) {
          A.push_back(f16bits(sa) | (uint32_t)0x3C00u << 16);
          B.push_back(f16bits(sb) | (uint32_t)0x3C00u << 16);
          H.push_back(f16bits(hl) | (uint32_t)f16bits(hh) << 16);
          va.push_back(sa);
          vb.push_back(sb);
          vs.push_back(hl);
          vh.push_back(hh);
        }
  const int n = (int)A.size();
  uint32_t *dA, *dB, *dH, *dD, *dDn;
  (void)hipMalloc(&dA, n * 4);
  (void)hipMalloc(&dB, n * 4);
  (void)hipMalloc(&dH, n * 4);
  (void)hipMalloc(&dD, n * 4);
  (void)hipMalloc(&dDn, n * 4);
  (void)hipMemcpy(dA, A.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B.data(), n * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dH, H.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(sem, dim3((n + 255) / 256), dim3(256), 0, 0, dA, dB, dH, dD, dDn, n);
  std::vector<uint32_t> D(n), Dn(n);
  (void)hipMemcpy(D.data(), dD, n * 4, hipMemcpyDeviceToHost);
  (void)hipMemcpy(Dn.data(), dDn, n * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    const int lo = vs[i] + va[i], hi = vh[i] + vb[i];
    const uint32_t want = f16bits(std::max(0, std::min(2048, lo))) |
                          (uint32_t)f16bits(std::max(0, std::min(2048, hi))) << 16;
    // unclamped: exact while the sum stays in [-2048, 2048]
    const bool in = lo >= -2048 && lo <= 2048 && hi >= -2048 && hi <= 2048;
    const uint32_t wantn = f16bits(lo) | (uint32_t)f16bits(hi) << 16;
    if (D[i] != want || (in && Dn[i] != wantn)) {
      if (bad < 5)
        std::printf("{\"mismatch\": [%d, %d, %d, %d], \"got\": \"%08x/%08x\", \"want\": \"%08x/%08x\"}\n",
                    va[i], vb[i], vs[i], vh[i], D[i], Dn[i], want, wantn);
      ++bad;
    }
  }
  std::printf("{\"semantics_cases\": %d, \"mismatches\": %d}\n", n, bad);
  for (int blocks : {768, 1024, 2048}) {
    run_rate<0>("v_pk_add_f16 clamp+v_pk_maximum3_f16", blocks);
    run_rate<1>("v_pk_fma_f16 op_sel clamp+v_pk_maximum3_f16", blocks);
    run_rate<2>("v_perm_b32+v_pk_add_f16 clamp", blocks);
  }
  return bad != 0;
}
