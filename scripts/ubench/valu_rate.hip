// VALU issue-rate microbenchmark for the instructions of the score kernel's inner loop.
// Each thread runs 8 independent dependency chains (ILP 8) of one instruction kind, so the
// rate measured is the SIMD issue rate, not latency.  Prints wave-instructions per SIMD per
// cycle at the measured clock (GRBM-free: uses wall time x 2.4 GHz nominal, and s_memtime
// ticks per wave for the in-kernel clock).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
#define ITERS 4096

// NC: independent chains per thread (8: issue rate; 1-4: how much a wave's own dependency
// chains limit it at few waves per SIMD)
template <int KIND, int NC = 8>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed, unsigned long long* ticks) {
  uint32_t a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + 1) + i * 77;
  const uint32_t b = seed ^ 0x00050005u;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS * 8 / NC; ++it) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      if (KIND == 0) {  // v_pk_max_u16
        u16x2 x = __builtin_bit_cast(u16x2, a[i]), y = __builtin_bit_cast(u16x2, b);
        a[i] = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, y) + (u16x2){1, 1});
      } else if (KIND == 1) {  // v_max_u32 + v_add_u32
        a[i] = max(a[i], b) + 1u;
      } else if (KIND == 2) {  // v_perm_b32 + v_add
        a[i] = __builtin_amdgcn_perm(b, a[i], 0x0c010c00u) + 1u;
      } else if (KIND == 4) {  // v_add_f32 + v_max_f32
        float x = __builtin_bit_cast(float, a[i]);
        x = __builtin_fmaxf(x + 1.5f, __builtin_bit_cast(float, b));
        a[i] = __builtin_bit_cast(uint32_t, x);
      } else if (KIND == 5) {  // v_fma_f32 x 2
        float x = __builtin_bit_cast(float, a[i]);
        x = __builtin_fmaf(x, 0.999f, 0.5f);
        x = __builtin_fmaf(x, 1.001f, -0.25f);
        a[i] = __builtin_bit_cast(uint32_t, x);
      } else if (KIND == 6) {  // v_pk_add_f16 + v_pk_maximum3_f16
        typedef _Float16 h2 __attribute__((ext_vector_type(2)));
        h2 x = __builtin_bit_cast(h2, a[i]), y = __builtin_bit_cast(h2, b);
        x = x + (h2){(_Float16)1, (_Float16)1};
        x = __builtin_elementwise_maximum(__builtin_elementwise_maximum(x, y),
                                          (h2){(_Float16)-3, (_Float16)-3});
        a[i] = __builtin_bit_cast(uint32_t, x);
      } else if (KIND == 8) {  // chains 0-3: v_pk_add_f16 + v_pk_maximum3_f16, 4-7: f32 add + max
        if (i < 4) {
          typedef _Float16 h2 __attribute__((ext_vector_type(2)));
          h2 x = __builtin_bit_cast(h2, a[i]), y = __builtin_bit_cast(h2, b);
          x = x + (h2){(_Float16)1, (_Float16)1};
          x = __builtin_elementwise_maximum(__builtin_elementwise_maximum(x, y),
                                            (h2){(_Float16)-3, (_Float16)-3});
          a[i] = __builtin_bit_cast(uint32_t, x);
        } else {
          float x = __builtin_bit_cast(float, a[i]);
          x = __builtin_fmaxf(x + 1.5f, __builtin_bit_cast(float, b));
          a[i] = __builtin_bit_cast(uint32_t, x);
        }
      } else if (KIND == 9) {  // f32 add with clamp (VOP3) + v_max3_f32
        float x = __builtin_bit_cast(float, a[i]);
        asm volatile("v_add_f32_e64 %0, %0, 0.5 clamp\n\tv_max3_f32 %0, %0, %1, %2"
                     : "+v"(x) : "v"(b), "v"(a[(i + 1) & 7]));
        a[i] = __builtin_bit_cast(uint32_t, x);
      } else if (KIND == 10) {  // chains 0-3: v_max_u32 + v_add_u32, 4-7: f32 add + max
        if (i < 4) {
          a[i] = max(a[i], b) + 1u;
        } else {
          float x = __builtin_bit_cast(float, a[i]);
          x = __builtin_fmaxf(x + 1.5f, __builtin_bit_cast(float, b));
          a[i] = __builtin_bit_cast(uint32_t, x);
        }
      } else if (KIND == 7) {  // v_max3_u32 + v_add_u32
        a[i] = max(max(a[i], b), b ^ 5u) + 1u;
      } else {  // v_pk_sub_u16 clamp + v_pk_add_u16
        u16x2 x = __builtin_bit_cast(u16x2, a[i]), y = __builtin_bit_cast(u16x2, b);
        a[i] = __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(x, y) + (u16x2){7, 7});
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) atomicAdd(ticks, t1 - t0);
}

template <int KIND, int NC = 8>
void run(const char* name, int blocks) {
  uint32_t* out;
  unsigned long long* ticks;
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  hipMalloc(&ticks, 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k<KIND, NC>), dim3(blocks), dim3(256), 0, 0, out, 3u, ticks);
  hipMemset(ticks, 0, 8);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k<KIND, NC>), dim3(blocks), dim3(256), 0, 0, out, 3u, ticks);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long t;
  hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost);
  const double waves = blocks * 4.0;
  const double instr = waves * ITERS * 8 * 2;  // 2 VALU per chain step
  const double simd_cycles = 1024.0 * ms * 1e-3 * 2.4e9;
  printf("{\"kind\": \"%s\", \"chains\": %d, \"blocks\": %d, \"waves_per_simd\": %.2f, "
         "\"ms\": %.3f, \"wave_instr_per_simd_cycle_at_2.4GHz\": %.3f, \"avg_wave_ticks\": %.0f}\n",
         name, NC, blocks, waves / 1024.0, ms, instr / simd_cycles, (double)t / blocks);
  hipFree(out);
  hipFree(ticks);
}

int main() {
  // issue rates at 4 and 8 resident waves per SIMD (1,024 / 2,048 blocks of 4 waves), and a
  // longer run (8,192 blocks: 32 waves per SIMD over time)
  for (int blocks : {1024, 2048, 8192}) {
    run<0>("v_pk_max_u16+v_pk_add_u16", blocks);
    run<1>("v_max_u32+v_add_u32", blocks);
    run<2>("v_perm_b32+v_add_u32", blocks);
    run<3>("v_pk_sub_u16_clamp+v_pk_add_u16", blocks);
    run<4>("v_add_f32+v_max_f32", blocks);
    run<5>("v_fma_f32+v_fma_f32", blocks);
    run<6>("v_pk_add_f16+v_pk_maximum3_f16", blocks);
    run<7>("v_max3_u32+v_add_u32", blocks);
    run<8>("mix: pk_f16 add+max3 (4 chains) | f32 add+max (4 chains)", blocks);
    run<9>("v_add_f32_e64 clamp+v_max3_f32", blocks);
    run<10>("mix: u32 max+add (4 chains) | f32 add+max (4 chains)", blocks);
  }
  // dependency-limited issue: the packed f16 pair with 1, 2 or 4 chains per wave at 1-4 waves
  // per SIMD (the wave kernel runs 3 waves per SIMD on configs[4])
  for (int blocks : {256, 512, 768, 1024}) {
    run<6, 1>("v_pk_add_f16+v_pk_maximum3_f16", blocks);
    run<6, 2>("v_pk_add_f16+v_pk_maximum3_f16", blocks);
    run<6, 4>("v_pk_add_f16+v_pk_maximum3_f16", blocks);
    run<6, 8>("v_pk_add_f16+v_pk_maximum3_f16", blocks);
  }
  return 0;
}
