// swbank_kernels.hip — gfx950 kernels of the score bank.
//
// Mapping of the reference's systolic ScoreBank onto CDNA4:
//   PE (SW_ProcessingElement_v1.0.v)        -> one query row held in a lane's registers
//   ScoringModule (128-PE chain)            -> a workgroup of W waves, each owning R consecutive
//                                              query rows; the waves form a systolic chain and
//                                              hand the bottom row of every column to the next
//                                              wave through an LDS ring (one barrier per C cols)
//   toggle (2 targets time-shared per PE)   -> 2 targets per lane, one per u16 half of every
//                                              register, updated together by v_pk_* ops
//   MODULES (independent modules per bank)  -> 64 lanes x workgroups: 128 targets per tile
//   Feeder (SM_Feeder3.v target register)   -> each lane streams its two targets' codes from
//                                              HBM (unaligned 8-byte loads), one chunk ahead
//
// Cell update (merged gap matrix, SW_ProcessingElement_v1.0.v:119-141,287-291,411-420) in
// the shifted/clamped form used here (all u16, per half):
//   p   = S - s(q_i,t_j)                 one v_perm_b32 from the row's 4-byte LUT (SGPR)
//   M   = sat(Hd~ - p)                   = max(0, H(i-1,j-1) + s)        (Hd~ = H + S)
//   I   = sat(max(Gup, Gleft) - e)       = max(0, I(i,j))
//   H~  = max(M, I) + S
//   G   = max(sat(M - o), I)             G(x) = max(M(x) - o, I(x)); I(i,j) = max(Gup,Gleft)-e
//   best= max(best, M)
// with o = -gap_open, e = -gap_extend: 9 VALU per lane per 2 cells.  Negative I never reaches
// H (M >= 0), so clamping at zero is exact.  Column 0 of the HDL ignores the neighbours in I
// (:131-141); the COL0 variant reproduces that by passing G = 0 downwards in column 0 (only
// observable when max(s) > o + e).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "swbank_internal.h"

namespace swk {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ u16x2 vmax(u16x2 a, u16x2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ u16x2 vsubs(u16x2 a, u16x2 b) {
  return __builtin_elementwise_sub_sat(a, b);
}



// One column of R rows for one wave.  ZDOWN: HDL column-0 rule (G passed down = 0).
// RB: rows per scheduling group (a sched_barrier every RB rows bounds how far the scheduler
// may defer the H/best updates behind the G chain, i.e. register pressure).
template <int R, int RB, bool ZDOWN>
__device__ __forceinline__ void column(const uint32_t (&tab)[R], uint32_t nv, uint32_t selw,
                                       u16x2& diag, u16x2& upG, u16x2 (&Hl)[R], u16x2 (&Gl)[R],
                                       u16x2& best, u16x2 S2, u16x2 O2, u16x2 E2) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const u16x2 p = as_u16x2(__builtin_amdgcn_perm(nv, tab[r], selw));
    const u16x2 M = vsubs(diag, p);
    const u16x2 I = vsubs(vmax(upG, Gl[r]), E2);
    const u16x2 Hn = vmax(M, I) + S2;
    const u16x2 Gn = vmax(vsubs(M, O2), I);
    best = vmax(best, M);
    diag = Hl[r];
    Hl[r] = Hn;
    Gl[r] = Gn;
    upG = ZDOWN ? (u16x2){0, 0} : Gn;
    if ((r % RB) == RB - 1) __builtin_amdgcn_sched_barrier(0);
  }
}

// The lane's two targets of the current tile.
struct Lane2 {
  const uint8_t* plo;
  const uint8_t* phi;
  uint32_t llo, lhi;
};

// Raw codes of columns [8c, 8c+8) of both targets (x,y = bytes 0-3, 4-7).  Past a target's
// end the code is 4 (N): s(*, N) <= 0, so padding can only lower a score.  `full` (uniform):
// every lane has >= 8 codes left in both targets -> two unaligned 8-byte loads.
__device__ __forceinline__ void load_raw(const Lane2& t, int c, bool full, uint2& lo, uint2& hi) {
  const uint32_t j0 = (uint32_t)c * 8;
  if (full) {
    lo = *reinterpret_cast<const uint2*>(t.plo + j0);
    hi = *reinterpret_cast<const uint2*>(t.phi + j0);
  } else {
    uint32_t b[2][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // branch-free: clamped address, then select
      const uint32_t j = j0 + k;
      const uint32_t a = t.plo[j < t.llo ? j : 0];
      const uint32_t h = t.phi[j < t.lhi ? j : 0];
      b[0][k] = j < t.llo ? a : 4u;
      b[1][k] = j < t.lhi ? h : 4u;
    }
    lo.x = b[0][0] | b[0][1] << 8 | b[0][2] << 16 | b[0][3] << 24;
    lo.y = b[0][4] | b[0][5] << 8 | b[0][6] << 16 | b[0][7] << 24;
    hi.x = b[1][0] | b[1][1] << 8 | b[1][2] << 16 | b[1][3] << 24;
    hi.y = b[1][4] | b[1][5] << 8 | b[1][6] << 16 | b[1][7] << 24;
  }
}

// Per-tile metadata of one lane (uniform tile id).
__device__ __forceinline__ Lane2 lane_targets(const uint8_t* res, const uint64_t* offs,
                                              const uint32_t* lens, size_t n, int tile, int lane) {
  Lane2 t;
  const size_t a = (size_t)tile * SWB_TILE + lane, b = a + 64;
  t.llo = a < n ? lens[a] : 0u;
  t.lhi = b < n ? lens[b] : 0u;
  // an empty target still needs a readable address for the branch-free slow path
  t.plo = t.llo ? res + offs[a] : reinterpret_cast<const uint8_t*>(lens);
  t.phi = t.lhi ? res + offs[b] : reinterpret_cast<const uint8_t*>(lens);
  return t;
}

// Chunk counts of a tile (uniform): nch = ceil(max len / 8) (>= 1), nfull = min len / 8.
__device__ __forceinline__ void tile_chunks(const Lane2& t, size_t tlo, size_t thi, size_t n,
                                            int& nch, int& nfull) {
  uint32_t Lmax = max(t.llo, t.lhi);
  uint32_t Lmin = min(tlo < n ? t.llo : ~0u, thi < n ? t.lhi : ~0u);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    Lmax = max(Lmax, (uint32_t)__shfl_xor((int)Lmax, off));
    Lmin = min(Lmin, (uint32_t)__shfl_xor((int)Lmin, off));
  }
  nch = max(1, (int)((__builtin_amdgcn_readfirstlane(Lmax) + 7) / 8));
  nfull = (int)(__builtin_amdgcn_readfirstlane(Lmin) / 8);
}

// Score kernel: one workgroup = one tile of 128 targets x the whole query (W waves x R rows).
// Wave w processes chunk c (8 columns) at phase c + w; one __syncthreads per phase orders the
// LDS ring hand-off wave w -> w+1 (the RTL's PE-to-PE registers).
//   qtab   W*R row LUTs: byte b = S - s(q_i, b) for codes b = 0..3; pad rows 0xFFFFFFFF
//   nv     4 x (S - s(*, N)) for target codes 4..7
//   S,O,E  shift (>= max s), -gap_open, -gap_extend
// LDS: best[128] | edge[2][64] | ring[(W-1)][2][8][64] {H~, G}
template <int R, int RB, bool COL0>
__global__ void __launch_bounds__(R >= 64 ? 512 : 1024)
    score_dna(const uint8_t* __restrict__ res, const uint64_t* __restrict__ offs,
              const uint32_t* __restrict__ lens, size_t n, const uint32_t* __restrict__ qtab,
              uint32_t nv, uint32_t S, uint32_t O, uint32_t E, int32_t* __restrict__ scores) {
  constexpr int C = 8;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = __builtin_amdgcn_readfirstlane(blockDim.x >> 6);
  uint32_t* bestsh = smem;                                   // 128 words
  uint2* edge = reinterpret_cast<uint2*>(smem + SWB_TILE);   // 2 x 64: top boundary | sink
  uint2* ring = edge + 128;

  const int tile = blockIdx.x;
  const size_t tlo = (size_t)tile * SWB_TILE + lane, thi = tlo + 64;
  const Lane2 cur = lane_targets(res, offs, lens, n, tile, lane);
  int nch, nfull;
  tile_chunks(cur, tlo, thi, n, nch, nfull);

  if (wave == 0) {
    bestsh[lane] = 0;
    bestsh[lane + 64] = 0;
    edge[lane] = make_uint2(S | (S << 16), 0u);  // row -1: H~ = S, G = 0
  }
  // nv in a VGPR so each v_perm_b32 takes its row LUT straight from an SGPR (one scalar
  // operand per VOP3 on gfx950).
  asm volatile("" : "+v"(nv));
  uint32_t tab[R];
#pragma unroll
  for (int r = 0; r < R; ++r) tab[r] = __builtin_amdgcn_readfirstlane(qtab[wave * R + r]);
  const u16x2 S2 = {(unsigned short)S, (unsigned short)S};
  const u16x2 O2 = {(unsigned short)O, (unsigned short)O};
  const u16x2 E2 = {(unsigned short)E, (unsigned short)E};

  u16x2 Hl[R], Gl[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    Hl[r] = S2;
    Gl[r] = (u16x2){0, 0};
  }
  u16x2 best = {0, 0};
  u16x2 prevUpH = S2;  // H~(row above, column -1) = S
  uint2 rlo, rhi;      // raw codes of the next chunk (prefetched one phase ahead)
  load_raw(cur, 0, nfull > 0, rlo, rhi);
  __syncthreads();

  // branch-free hand-off: wave 0 reads the constant top boundary, the last wave writes into a
  // sink, both with column stride 0 (branches here split the column loop into blocks and LLVM
  // then sinks the H updates across columns, blowing up register pressure)
  const int istride = wave > 0 ? 64 : 0, ostride = wave < W - 1 ? 64 : 0;
  const int nph = nch + W - 1;
  for (int ph = 0; ph < nph; ++ph) {
    const int c = ph - wave;
    if (c >= 0 && c < nch) {
      const uint2 clo = rlo, chi = rhi;
      if (c + 1 < nch) load_raw(cur, c + 1, c + 1 < nfull, rlo, rhi);
      const int slot = c & 1;
      const uint2* rin = wave > 0 ? ring + ((size_t)((wave - 1) * 2 + slot) * C) * 64 + lane
                                  : edge + lane;
      uint2* rout = wave < W - 1 ? ring + ((size_t)(wave * 2 + slot) * C) * 64 + lane
                                 : edge + 64 + lane;
      uint2 rv = rin[0];
#pragma unroll
      for (int jj = 0; jj < C; ++jj) {
        const u16x2 upH = as_u16x2(rv.x);
        u16x2 upG = as_u16x2(rv.y);
        if (jj + 1 < C) rv = rin[(jj + 1) * istride];  // one column ahead
        u16x2 diag = prevUpH;
        prevUpH = upH;
        // selector: byte 0 = code of the low target, byte 2 = code of the high target
        const uint32_t sel = (uint32_t)(jj & 3) | ((uint32_t)(4 + (jj & 3)) << 16) | 0x0C000C00u;
        const uint32_t selw =
            __builtin_amdgcn_perm(jj < 4 ? chi.x : chi.y, jj < 4 ? clo.x : clo.y, sel) |
            0x0C000C00u;
        __builtin_amdgcn_sched_barrier(0);
        if (COL0 && jj == 0 && c == 0)
          column<R, RB, true>(tab, nv, selw, diag, upG, Hl, Gl, best, S2, O2, E2);
        else
          column<R, RB, false>(tab, nv, selw, diag, upG, Hl, Gl, best, S2, O2, E2);
        // pin the running max once per column: otherwise LLVM re-associates the max over the
        // whole phase into a tree and keeps every M live
        asm volatile("" : "+v"(best));
        rout[jj * ostride] = make_uint2(as_u32(Hl[R - 1]), as_u32(upG));
      }
    }
    __syncthreads();
  }

  atomicMax(&bestsh[lane], (uint32_t)best.x);
  atomicMax(&bestsh[lane + 64], (uint32_t)best.y);
  __syncthreads();
  if (wave == 0) {
    if (tlo < n) scores[tlo] = (int32_t)bestsh[lane];
    if (thi < n) scores[thi] = (int32_t)bestsh[lane + 64];
  }
}

template <int R, int RB, bool COL0>
static hipError_t launch_score(const uint8_t* res, const uint64_t* offs, const uint32_t* lens,
                               size_t n, const uint32_t* qtab, int W, uint32_t nv, uint32_t S,
                               uint32_t O, uint32_t E, int32_t* scores, hipStream_t st) {
  const size_t ntiles = (n + SWB_TILE - 1) / SWB_TILE;
  const size_t lds = SWB_TILE * 4 + (size_t)(128 + (W > 1 ? W - 1 : 0) * 2 * 8 * 64) * 8;
  auto fn = &score_dna<R, RB, COL0>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(fn, dim3((unsigned)ntiles), dim3(64 * W), (unsigned)lds, st, res, offs,
                     lens, n, qtab, nv, S, O, E, scores);
  return hipGetLastError();
}

}  // namespace swk

// Variants compiled in: (R, RB) — rows per wave, rows per scheduling group.  The host picks R
// from the query length (SWBANK_R / SWBANK_RB override it for tuning).
#define SWK_VARIANTS(X) \
  X(16, 4)              \
  X(32, 4)              \
  X(32, 8)              \
  X(64, 4)

extern "C" int swk_has_variant(int R, int RB) {
#define SWK_HAS(RR, BB) \
  if (R == RR && RB == BB) return 1;
  SWK_VARIANTS(SWK_HAS)
#undef SWK_HAS
  return 0;
}

extern "C" hipError_t swk_launch_score_dna(int R, int RB, int col0, const uint8_t* res,
                                           const uint64_t* offs, const uint32_t* lens, size_t n,
                                           unsigned* queue, const uint32_t* qtab, int W,
                                           uint32_t nv, uint32_t S, uint32_t O, uint32_t E,
                                           int32_t* scores, uint32_t max_len, int grid_cap,
                                           hipStream_t st) {
  if (n == 0) return hipSuccess;
  (void)queue;  // reserved for a persistent (tile-queue) variant
  (void)max_len;
  (void)grid_cap;
#define SWK_CASE(RR, BB)                                                                     \
  if (R == RR && RB == BB)                                                                   \
    return col0 ? swk::launch_score<RR, BB, true>(res, offs, lens, n, qtab, W, nv, S, O, E,   \
                                                  scores, st)                                \
                : swk::launch_score<RR, BB, false>(res, offs, lens, n, qtab, W, nv, S, O, E,  \
                                                   scores, st);
  SWK_VARIANTS(SWK_CASE)
#undef SWK_CASE
  return hipErrorInvalidValue;
}
