// swbank_kwave.hip — the wave kernels: lanes are query rows, one wave
// walks the anti-diagonals of one or two target pairs; configs[4]'s two-pairs kernel.
#include "swbank_kcommon.h"

namespace swk {

// ========================================================================================
// Wave kernel: the north-star wavefront form, for batches with few targets (few tiles) and
// queries up to 1024 rows.  One wave scores two targets (the u16 halves) against the whole
// query; lane l owns query rows [lK, lK+K).  Step t: lane l computes column t - l for its K
// rows (an anti-diagonal of K-row blocks across the wave); the bottom row {H~, G/F} and the
// two target codes move one lane down per step with DPP wave_shr:1 (the RTL's M_out/I_out/
// data_out from PE i to PE i+1); lane 0 takes row -1 = {S, 0} and the next codes of the
// target stream.  A lane that has not reached column 0 yet (or is past the end) sees padding
// codes and boundary inputs, which leave the boundary state unchanged — no masking needed.
template <int K>
struct ProfLookupK {
  uint32_t lo[(K + 3) / 4], hi[(K + 3) / 4];
  __device__ __forceinline__ u16x2 operator()(int r) const {
    const uint32_t sel = (uint32_t)(r & 3) | ((uint32_t)(4 + (r & 3)) << 16) | 0x0C000C00u;
    return as_u16x2(__builtin_amdgcn_perm(hi[r >> 2], lo[r >> 2], sel));
  }
};
template <int K>
struct ProfLookupK16 {  // f16 profile, 2-byte entries: word k = rows 2k, 2k+1 of a letter
  uint32_t lo[K / 2], hi[K / 2];
  __device__ __forceinline__ u16x2 operator()(int r) const {
    const uint32_t k = (uint32_t)(r & 1) * 2;
    const uint32_t sel = k | ((k + 1) << 8) | ((k + 4) << 16) | ((k + 5) << 24);
    return as_u16x2(__builtin_amdgcn_perm(hi[r >> 1], lo[r >> 1], sel));
  }
};
template <int K>
struct ProfLookupF {  // f16 profile words {s, 1.0}, one per row: a[r] target A's, b[r] B's
  uint32_t a[K], b[K];  // (the column asm adds them with one op_sel FMA, gen_f16_rows.py "F")
};
template <int K>
struct LaneLutLookup {  // per-lane row LUTs (the lane's own query rows) in VGPRs
  const uint32_t (&lut)[K];
  uint32_t nv, selw;
  __device__ __forceinline__ u16x2 operator()(int r) const {
    return as_u16x2(__builtin_amdgcn_perm(nv, lut[r], selw));
  }
};

// merged column with a per-lane column-0 mask (zmask = 0 in the lane's column 0)
template <int R, int RB, class LK>
__device__ __forceinline__ void column_merged_mask(const LK& lk, u16x2& diag, u16x2& upG,
                                                   u16x2 (&Hl)[R], u16x2 (&Gl)[R], u16x2& best,
                                                   u16x2 S2, u16x2 O2, u16x2 E2, uint32_t zmask) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const u16x2 p = lk(r);
    const u16x2 M = vsubs(diag, p);
    const u16x2 I = vsubs(vmax(upG, Gl[r]), E2);
    const u16x2 Hn = vmax(M, I) + S2;
    const u16x2 Gn = vmax(vsubs(M, O2), I);
    best = vmax(best, M);
    diag = Hl[r];
    Hl[r] = Hn;
    Gl[r] = Gn;
    upG = as_u16x2(as_u32(Gn) & zmask);
    if ((r % RB) == RB - 1) __builtin_amdgcn_sched_barrier(0);
  }
}

// f16 merged column with a per-lane column-0 mask (zdown: T passed down = -o-e)
template <int R, int RB, class LK>
__device__ __forceinline__ void column_merged_f16_mask(const LK& lk, u16x2& diag_, u16x2& upT_,
                                                       u16x2 (&Hl)[R], u16x2 (&Tl)[R],
                                                       u16x2& best_, f16x2 NOE2, f16x2 NE2,
                                                       bool zdown) {
  f16x2 diag = as_f16x2(diag_), upT = as_f16x2(upT_), best = as_f16x2(best_);
  const f16x2 Z = {(_Float16)0, (_Float16)0};
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const f16x2 D = diag + as_f16x2(lk(r));
    const f16x2 I = fmax2(upT, as_f16x2(Tl[r]));
    const f16x2 H = fmax2(fmax2(D, Z), I);
    const f16x2 T = fmax2(fmax2(D + NOE2, NOE2), I + NE2);
    best = fmax2(best, H);
    diag = as_f16x2(Hl[r]);
    Hl[r] = as_u16x2(H);
    Tl[r] = as_u16x2(T);
    upT = zdown ? NOE2 : T;
    if ((r % RB) == RB - 1) __builtin_amdgcn_sched_barrier(0);
  }
  upT_ = as_u16x2(upT);
  best_ = as_u16x2(best);
}

// Wave-kernel f16 column (K rows per lane, no column-0 rule), hand-ordered asm: the same
// generated row blocks as the tile kernel with the lane's own LUT words / profile words in
// VGPRs.  K = 4: one 4-row block; K = 8, 16: 8-row blocks.
#define SWK_CLAMP(x, n) ((x) < (n) ? (x) : (n) - 1)
#ifndef SWK_RING_PF
#define SWK_RING_PF 1  // wave kernel, f16 profile: read the code ring one step ahead
#endif
#ifndef SWK_HALF_UNROLL
#define SWK_HALF_UNROLL 4  // two-pairs wave kernel: steps per loop iteration (2 or 4)
#endif
#ifndef SWK_HALF_AHEAD
#define SWK_HALF_AHEAD 1  // two-pairs wave kernel: profile words one step ahead
#endif
#ifndef SWK_HALF_DPPSEL
// two-pairs wave kernel: the row above moves down and each half's lane 0 takes the row -1
// boundary in ONE v_cndmask_b32_dpp per value (the shift as the select's DPP operand, the
// boundary lanes in VCC) instead of a DPP move and a v_cndmask
#define SWK_HALF_DPPSEL 1
#endif
#ifndef SWK_HALF_FMA
// two-pairs wave kernel: LDS profile words {s, 1.0} (4 B per letter and row) added with one
// op_sel FMA per row (gen_f16_rows.py mode F) instead of 2-byte entries interleaved by a v_perm
#define SWK_HALF_FMA 1
#endif
#ifndef SWK_HALF_ABSRING
// two-pairs wave kernel (FMA profile, words a step ahead): the code ring holds each lane's
// profile ADDRESS (relative to the ring slot), so with the 32-step ring window unrolled no step
// computes an LDS address: no profile-address add, no ring-pointer op (wave_two_pairs)
#define SWK_HALF_ABSRING 1
#endif
// the two-pairs kernel's LDS: the profile (letter stride SWK_HALF_LS bytes, 512 rows) and
// each wave's code ring (profile offsets of both halves' targets, SWK_HALF_RING bytes a wave);
// SWK_HALF_ABSRING: wave 0's ring first, the profile at byte SWK_HALF_ABS_BASE, the other
// waves' rings after it (the same total)
#define SWK_HALF_LS (SWK_HALF_FMA ? 2048u : 1024u)
#define SWK_HALF_RING (SWK_HALF_FMA ? 512u : 1024u)
#define SWK_HALF_ABS (SWK_HALF_ABSRING && SWK_HALF_FMA && SWK_HALF_AHEAD)
#define SWK_HALF_ABS_BASE 512u
#define SWK_W_HT(B)                                                                           \
  [h0] "+v"(Hl[B]), [h1] "+v"(Hl[SWK_CLAMP(B + 1, K)]), [h2] "+v"(Hl[SWK_CLAMP(B + 2, K)]),    \
      [h3] "+v"(Hl[SWK_CLAMP(B + 3, K)]), [h4] "+v"(Hl[SWK_CLAMP(B + 4, K)]),                  \
      [h5] "+v"(Hl[SWK_CLAMP(B + 5, K)]), [h6] "+v"(Hl[SWK_CLAMP(B + 6, K)]),                  \
      [h7] "+v"(Hl[SWK_CLAMP(B + 7, K)]), [t0] "+v"(Xl[B]), [t1] "+v"(Xl[SWK_CLAMP(B + 1, K)]), \
      [t2] "+v"(Xl[SWK_CLAMP(B + 2, K)]), [t3] "+v"(Xl[SWK_CLAMP(B + 3, K)]),                  \
      [t4] "+v"(Xl[SWK_CLAMP(B + 4, K)]), [t5] "+v"(Xl[SWK_CLAMP(B + 5, K)]),                  \
      [t6] "+v"(Xl[SWK_CLAMP(B + 6, K)]), [t7] "+v"(Xl[SWK_CLAMP(B + 7, K)]), [Da] "+v"(Da),   \
      [Db] "=&v"(Db), [S1] "=&v"(S1), [best] "+v"(best)
#define SWK_W_OUT_M(B) SWK_W_HT(B), [X] "=&v"(X), [DN] "=&v"(DN), [IN] "=&v"(IN)
// K = 4: four distinct rows only (an output operand bound twice would copy back stale values)
#define SWK_W4_HT                                                                             \
  [h0] "+v"(Hl[0]), [h1] "+v"(Hl[1]), [h2] "+v"(Hl[2]), [h3] "+v"(Hl[3]), [t0] "+v"(Xl[0]),    \
      [t1] "+v"(Xl[1]), [t2] "+v"(Xl[2]), [t3] "+v"(Xl[3]), [Da] "+v"(Da), [Db] "=&v"(Db),     \
      [S1] "=&v"(S1), [best] "+v"(best)
#define SWK_W4_OUT_M SWK_W4_HT, [X] "=&v"(X), [DN] "=&v"(DN), [IN] "=&v"(IN)
// K = 2 (the split tail's quarter segments)
#define SWK_W2_HT                                                                             \
  [h0] "+v"(Hl[0]), [h1] "+v"(Hl[SWK_CLAMP(1, K)]), [t0] "+v"(Xl[0]),                          \
      [t1] "+v"(Xl[SWK_CLAMP(1, K)]), [Da] "+v"(Da), [Db] "=&v"(Db), [S1] "=&v"(S1),             \
      [best] "+v"(best)
#define SWK_W2_OUT_M SWK_W2_HT, [X] "=&v"(X), [DN] "=&v"(DN), [IN] "=&v"(IN)
#define SWK_W2_OUT_G SWK_W2_HT, [EN] "=&v"(X), [HN] "=&v"(DN), [FN] "=&v"(IN), [F] "+v"(up)
#define SWK_W2_IN_LM [nv] "v"(lk.nv), [sel] "v"(lk.selw), [noe] "s"(noe), [ne] "s"(ne), [no] "s"(no), [up] "v"(up), [tb0] "v"(lk.lut[SWK_CLAMP(1, K)])
#define SWK_W2_IN_LG [nv] "v"(lk.nv), [sel] "v"(lk.selw), [noe] "s"(noe), [ne] "s"(ne), [tb0] "v"(lk.lut[SWK_CLAMP(1, K)])
#define SWK_W2_IN_PM [noe] "s"(noe), [ne] "s"(ne), [no] "s"(no), [up] "v"(up), [selA] "s"(0x05040100u), [selB] "s"(0x07060302u), [lo0] "v"(lk.lo[0]), [hi0] "v"(lk.hi[0])
#define SWK_W2_IN_PG [noe] "s"(noe), [ne] "s"(ne), [selA] "s"(0x05040100u), [selB] "s"(0x07060302u), [lo0] "v"(lk.lo[0]), [hi0] "v"(lk.hi[0])
#define SWK_W4_OUT_G SWK_W4_HT, [EN] "=&v"(X), [HN] "=&v"(DN), [FN] "=&v"(IN), [F] "+v"(up)
#define SWK_W_OUT_G(B) SWK_W_HT(B), [EN] "=&v"(X), [HN] "=&v"(DN), [FN] "=&v"(IN), [F] "+v"(up)
#define SWK_W_TB(B)                                                                           \
  [tb0] "v"(lk.lut[SWK_CLAMP(B + 1, K)]), [tb1] "v"(lk.lut[SWK_CLAMP(B + 2, K)]),              \
      [tb2] "v"(lk.lut[SWK_CLAMP(B + 3, K)]), [tb3] "v"(lk.lut[SWK_CLAMP(B + 4, K)]),          \
      [tb4] "v"(lk.lut[SWK_CLAMP(B + 5, K)]), [tb5] "v"(lk.lut[SWK_CLAMP(B + 6, K)]),          \
      [tb6] "v"(lk.lut[SWK_CLAMP(B + 7, K)]), [tb7] "v"(lk.lut[SWK_CLAMP(B + 8, K)])
#define SWK_W_LH(B)                                                                           \
  [lo0] "v"(lk.lo[B / 2]), [lo1] "v"(lk.lo[SWK_CLAMP(B / 2 + 1, K / 2)]),                      \
      [lo2] "v"(lk.lo[SWK_CLAMP(B / 2 + 2, K / 2)]), [lo3] "v"(lk.lo[SWK_CLAMP(B / 2 + 3, K / 2)]), \
      [lo4] "v"(lk.lo[SWK_CLAMP(B / 2 + 4, K / 2)]), [hi0] "v"(lk.hi[B / 2]),                  \
      [hi1] "v"(lk.hi[SWK_CLAMP(B / 2 + 1, K / 2)]), [hi2] "v"(lk.hi[SWK_CLAMP(B / 2 + 2, K / 2)]), \
      [hi3] "v"(lk.hi[SWK_CLAMP(B / 2 + 3, K / 2)]), [hi4] "v"(lk.hi[SWK_CLAMP(B / 2 + 4, K / 2)])
#define SWK_W_IN_LM(B) [nv] "v"(lk.nv), [sel] "v"(lk.selw), [noe] "s"(noe), [ne] "s"(ne), [no] "s"(no), [up] "v"(up), SWK_W_TB(B)
#define SWK_W_IN_LG(B) [nv] "v"(lk.nv), [sel] "v"(lk.selw), [noe] "s"(noe), [ne] "s"(ne), SWK_W_TB(B)
#define SWK_W_IN_PM(B)                                                                        \
  [noe] "s"(noe), [ne] "s"(ne), [no] "s"(no), [up] "v"(up), [selA] "s"(0x05040100u), [selB] "s"(0x07060302u), \
      SWK_W_LH(B)
#define SWK_W_IN_PG(B) [noe] "s"(noe), [ne] "s"(ne), [selA] "s"(0x05040100u), [selB] "s"(0x07060302u), SWK_W_LH(B)
// mode F (ProfLookupF): block row i's next-row words a / b [B + i + 1]
#define SWK_W_FAB(B)                                                                          \
  [fa0] "v"(lk.a[SWK_CLAMP(B + 1, K)]), [fa1] "v"(lk.a[SWK_CLAMP(B + 2, K)]),                  \
      [fa2] "v"(lk.a[SWK_CLAMP(B + 3, K)]), [fa3] "v"(lk.a[SWK_CLAMP(B + 4, K)]),              \
      [fa4] "v"(lk.a[SWK_CLAMP(B + 5, K)]), [fa5] "v"(lk.a[SWK_CLAMP(B + 6, K)]),              \
      [fa6] "v"(lk.a[SWK_CLAMP(B + 7, K)]), [fa7] "v"(lk.a[SWK_CLAMP(B + 8, K)]),              \
      [fb0] "v"(lk.b[SWK_CLAMP(B + 1, K)]), [fb1] "v"(lk.b[SWK_CLAMP(B + 2, K)]),              \
      [fb2] "v"(lk.b[SWK_CLAMP(B + 3, K)]), [fb3] "v"(lk.b[SWK_CLAMP(B + 4, K)]),              \
      [fb4] "v"(lk.b[SWK_CLAMP(B + 5, K)]), [fb5] "v"(lk.b[SWK_CLAMP(B + 6, K)]),              \
      [fb6] "v"(lk.b[SWK_CLAMP(B + 7, K)]), [fb7] "v"(lk.b[SWK_CLAMP(B + 8, K)])
#define SWK_W_IN_FM(B) [noe] "s"(noe), [ne] "s"(ne), [no] "s"(no), [up] "v"(up), SWK_W_FAB(B)
#define SWK_W_IN_FG(B) [noe] "s"(noe), [ne] "s"(ne), SWK_W_FAB(B)

template <int K, bool GOTOH, class LK>
__device__ __forceinline__ void column_f16_lane_asm(const LK& lk, u16x2& diag_, u16x2& upX_,
                                                    u16x2 (&Hl)[K], u16x2 (&Xl)[K],
                                                    u16x2& best_, uint32_t noe, uint32_t ne,
                                                    uint32_t no) {
  constexpr bool FMA = std::is_same<LK, ProfLookupF<K>>::value;
  constexpr bool PROF = !std::is_same<LK, LaneLutLookup<K>>::value;
  uint32_t Da, Db, S1, X, DN, IN;
  u16x2 best = best_, up = upX_;
  if constexpr (FMA) {
    static_assert(K % 8 == 0, "mode F: 8-row blocks");
    asm volatile("v_pk_fma_f16 %[Da], %[a0], %[b0], %[dg] op_sel:[0,1,0] op_sel_hi:[1,0,1] clamp"
                 : [Da] "=&v"(Da)
                 : [a0] "v"(lk.a[0]), [b0] "v"(lk.b[0]), [dg] "v"(diag_));
#pragma unroll
    for (int b = 0; b < K; b += 8) {
      const bool last = b + 8 >= K;
      if constexpr (GOTOH) {
        if (last) asm volatile(SWK_F16G_F_L1 : SWK_W_OUT_G(b) : SWK_W_IN_FG(b));
        else      asm volatile(SWK_F16G_F_L0 : SWK_W_OUT_G(b) : SWK_W_IN_FG(b));
      } else {
        if (last) asm volatile(SWK_F16M_F_Z0_L1 : SWK_W_OUT_M(b) : SWK_W_IN_FM(b));
        else      asm volatile(SWK_F16M_F_Z0_L0 : SWK_W_OUT_M(b) : SWK_W_IN_FM(b));
        up = Xl[SWK_CLAMP(b + 7, K)];
      }
    }
  } else {
  if constexpr (PROF)
    asm volatile(
        "v_perm_b32 %[Da], %[h0], %[l0], %[sA]\n\t"
        "v_pk_add_f16 %[Da], %[dg], %[Da] clamp"
        : [Da] "=&v"(Da)
        : [h0] "v"(lk.hi[0]), [l0] "v"(lk.lo[0]), [sA] "s"(0x05040100u), [dg] "v"(diag_));
  else
    asm volatile(
        "v_perm_b32 %[Da], %[nv], %[t0], %[sel]\n\t"
        "v_pk_add_f16 %[Da], %[dg], %[Da] clamp"
        : [Da] "=&v"(Da)
        : [nv] "v"(lk.nv), [t0] "v"(lk.lut[0]), [sel] "v"(lk.selw), [dg] "v"(diag_));
  if constexpr (K == 2) {
    if constexpr (GOTOH && PROF) asm volatile(SWK_F16G_P_L1_R2 : SWK_W2_OUT_G : SWK_W2_IN_PG);
    else if constexpr (GOTOH)    asm volatile(SWK_F16G_L_L1_R2 : SWK_W2_OUT_G : SWK_W2_IN_LG);
    else if constexpr (PROF)     asm volatile(SWK_F16M_P_Z0_L1_R2 : SWK_W2_OUT_M : SWK_W2_IN_PM);
    else                         asm volatile(SWK_F16M_L_Z0_L1_R2 : SWK_W2_OUT_M : SWK_W2_IN_LM);
    if constexpr (!GOTOH) up = Xl[SWK_CLAMP(1, K)];
  } else if constexpr (K == 4) {
    if constexpr (GOTOH && PROF) asm volatile(SWK_F16G_P_L1_R4 : SWK_W4_OUT_G : SWK_W_IN_PG(0));
    else if constexpr (GOTOH)    asm volatile(SWK_F16G_L_L1_R4 : SWK_W4_OUT_G : SWK_W_IN_LG(0));
    else if constexpr (PROF)     asm volatile(SWK_F16M_P_Z0_L1_R4 : SWK_W4_OUT_M : SWK_W_IN_PM(0));
    else                         asm volatile(SWK_F16M_L_Z0_L1_R4 : SWK_W4_OUT_M : SWK_W_IN_LM(0));
    if constexpr (!GOTOH) up = Xl[3];
  } else {
#pragma unroll
    for (int b = 0; b < K; b += 8) {
      const bool last = b + 8 >= K;
      if constexpr (GOTOH && PROF) {
        if (last) asm volatile(SWK_F16G_P_L1 : SWK_W_OUT_G(b) : SWK_W_IN_PG(b));
        else      asm volatile(SWK_F16G_P_L0 : SWK_W_OUT_G(b) : SWK_W_IN_PG(b));
      } else if constexpr (GOTOH) {
        if (last) asm volatile(SWK_F16G_L_L1 : SWK_W_OUT_G(b) : SWK_W_IN_LG(b));
        else      asm volatile(SWK_F16G_L_L0 : SWK_W_OUT_G(b) : SWK_W_IN_LG(b));
      } else if constexpr (PROF) {
        if (last) asm volatile(SWK_F16M_P_Z0_L1 : SWK_W_OUT_M(b) : SWK_W_IN_PM(b));
        else      asm volatile(SWK_F16M_P_Z0_L0 : SWK_W_OUT_M(b) : SWK_W_IN_PM(b));
      } else {
        if (last) asm volatile(SWK_F16M_L_Z0_L1 : SWK_W_OUT_M(b) : SWK_W_IN_LM(b));
        else      asm volatile(SWK_F16M_L_Z0_L0 : SWK_W_OUT_M(b) : SWK_W_IN_LM(b));
      }
      if constexpr (!GOTOH) up = Xl[SWK_CLAMP(b + 7, K)];
    }
  }
  }  // (mode F)
  (void)Db; (void)S1; (void)X; (void)DN; (void)IN;
  upX_ = up;
  best_ = best;
}

// A target pointer typed global (address space 1): its code loads are global loads, which
// count on the vector-memory counter only (a flat load counts on the LDS counter too, so every
// LDS wait after one would wait for global memory).
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* global_ptr(T* p) {
  return (__attribute__((address_space(1))) T*)p;
}

// wave_pair's loop flavours: row -1 from a previous segment (in), bottom row written (out)
template <bool I, bool O>
struct SegT {
  static constexpr bool in = I, out = O;
};

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t lane0_value, uint32_t v) {
  return __builtin_amdgcn_update_dpp(lane0_value, v, 0x138 /* wave_shr:1 */, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dpp_shr1_zero(uint32_t v) {  // lane 0 reads 0
  return __builtin_amdgcn_mov_dpp(v, 0x138 /* wave_shr:1 */, 0xF, 0xF, true);
}

// One pair (targets 2*pair, 2*pair+1; tA < n) against the query (segment): returns the two
// best scores (every lane), and writes the segment's bottom row when a.edge_out is set.
// qtab (wave layout): LUT: 64*K row words | PROF: (pad+1) x PS bytes, PS = 64*K (u16) or
// 128*K (f16).  prof: the profile (PROF), in LDS for the main pass or in HBM for the u16
// re-score of an optimistic f16 pass (the compiler emits ds_ or flat loads per call site).
// SPLIT (the split tail): this wave is row segment `seg` of P of the pair; lin (the ring from
// the segment above, none for seg 0) / lout (the ring to the segment below, none for the last)
// hold 256 columns each, and the waves of the block run nph + 2(P - 1) phases of 64 steps
// with one barrier each, segment s two phases behind segment s - 1: its first step of a phase
// loads 64 ring columns that the segment above finished writing by the previous barrier.
// cring (f16 profile, main waves): the wave's 256-byte LDS code ring.  Instead of shifting a
// code word one lane down per step (readlane + move + DPP add + two extracts), every 64 steps
// each lane writes the letter codes of its column of the previous and of the next 64 columns
// into ring bytes l and 64 + l (target A; target B 128 bytes on); at step T + j lane l reads
// column T + j - l at ring position 64 + j - l and forms its two profile addresses with one
// mad each.
template <int K, bool COL0, bool PROF, bool GOTOH, bool F16, bool SPLIT = false>
__device__ __forceinline__ uint2 wave_pair(const ScoreArgs& a, const uint8_t* prof,
                                           const uint32_t* qtab, uint32_t nv, uint32_t PSb,
                                           size_t pair, int lane, const uint2* lin = nullptr,
                                           uint2* lout = nullptr, int nph = 0, int seg = 0,
                                           int P = 1, uint8_t* cring = nullptr) {
  constexpr bool RING = F16 && PROF && !SPLIT;
  constexpr bool PF = SWK_RING_PF != 0;  // ring letters read one step ahead
  const size_t tA = 2 * pair, tB = tA + 1;
  const size_t n = a.n;
  const bool packed = a.packed != SWK_PACK_BYTES, rec = a.packed == SWK_PACK_RECORDS;
  const bool nib = a.packed == SWK_PACK_NIBBLE;
  const bool uni = a.ustride != 0;
  const uint32_t LA = rec ? record_len(a.res + tA * SWB_RECORD) : uni ? a.ulen : a.lens[tA];
  const uint32_t LB = tB >= n ? 0u
                      : rec ? record_len(a.res + tB * SWB_RECORD)
                      : uni ? a.ulen
                            : a.lens[tB];
  const auto pA = global_ptr(rec ? a.res + tA * SWB_RECORD + 6
                                  : uni ? a.res + tA * a.ustride
                                        : a.res + (LA ? a.offs[tA] : 0));
  const auto pB = global_ptr(rec ? a.res + (tB < n ? tB : tA) * SWB_RECORD + 6
                                  : uni ? a.res + (tB < n ? tB : tA) * a.ustride
                                        : a.res + (LB ? a.offs[tB] : 0));
  const int Lmax = (int)__builtin_amdgcn_readfirstlane(max(LA, LB));
  const uint32_t S = a.S, pad = a.pad;
  const u16x2 S2 = {(unsigned short)S, (unsigned short)S};
  const u16x2 O2 = {(unsigned short)a.O, (unsigned short)a.O};
  const u16x2 E2 = {(unsigned short)a.E, (unsigned short)a.E};
  const uint32_t oes = a.O + a.E + S;
  const u16x2 OES2 = {(unsigned short)oes, (unsigned short)oes};
  // selector word: u16 {code_lo, 0x0C, code_hi, 0x0C}; f16 {0x0C, code_lo, 0x0C, code_hi}
  // (the f16 LUT byte is the high byte; 2-byte f16 profiles use the code byte only)
  // f16 profile: the code word carries the LDS byte offsets of both letters' profile rows
  // plus the lane's own row offset (2K bytes per lane, added per DPP hop), so the lane's two
  // addresses are one mask / shift each; the host keeps (pad + 1) x PS <= 64 KiB
  const uint32_t hop = (2u * K) | (2u * K) << 16;
  const auto code_word = [&](uint32_t x, uint32_t y) -> uint32_t {
    if constexpr (F16 && PROF) return x * PSb | (y * PSb) << 16;
    else if constexpr (F16) return (x << 8) | (y << 24) | 0x000C000Cu;
    else return x | (y << 16) | 0x0C000C00u;
  };
  const uint32_t padsel = code_word(pad, pad);
  // f16 encodings of -(o+e), -e, -o (host-computed, so they stay in SGPRs)
  const f16x2 NOE2 = as_f16x2(as_u16x2(a.f16_noe)), NE2 = as_f16x2(as_u16x2(a.f16_ne)),
              NO2 = as_f16x2(as_u16x2(a.f16_no));
  const u16x2 H0 = F16 ? (u16x2){0, 0} : S2;                          // H of row/col -1
  const u16x2 X0 = (F16 && !GOTOH) ? as_u16x2(NOE2) : (u16x2){0, 0};  // T/G/E/F of row/col -1
  const uint32_t noe = as_u32(as_u16x2(NOE2)), ne = as_u32(as_u16x2(NE2)),
                 no = as_u32(as_u16x2(NO2));

  uint32_t lut[PROF ? 1 : K];
  if constexpr (!PROF) {
#pragma unroll
    for (int k = 0; k < K; ++k) lut[k] = qtab[lane * K + k];
  }
  const uint8_t* prow = prof + lane * K;       // this lane's rows in every profile letter row

  u16x2 Hl[K], Xl[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    Hl[k] = H0;
    Xl[k] = X0;
  }
  u16x2 best = {0, 0};
  u16x2 prevUpH = H0;
  uint32_t botH = as_u32(H0), botX = as_u32(X0), buf = padsel;
  uint32_t let = F16 && PROF ? padsel + lane * hop : padsel;
  uint32_t ringprev = pad | pad << 8;  // RING: this lane's codes of the previous 64 columns
  // query segments (queries longer than 64K rows): lane 0 reads row -1 of this segment (the
  // previous segment's bottom row) from edge_in, lane 63 writes this segment's bottom row;
  // layout [pair][column] {H, G/T/F} of both targets
  const bool seg_in = SPLIT ? lin != nullptr : a.edge_in != nullptr;
  const bool seg_out = SPLIT ? lout != nullptr : a.edge_out != nullptr;
  const uint2* ein = SPLIT ? lin : seg_in ? a.edge_in + pair * a.ecols : nullptr;
  uint2* eout = SPLIT ? lout : seg_out ? a.edge_out + pair * a.ecols : nullptr;
  const uint32_t rmask = SPLIT ? 255u : ~0u;  // the split ring holds 256 columns
  uint2 ebuf = make_uint2(as_u32(H0), as_u32(X0));

  // two steps per iteration (the loop-carried values alternate registers instead of being
  // copied back); an odd count gets one extra all-padding step, which changes no score
  const int nsteps = Lmax + 63;
  // the codes of column c of both targets (pad past the end): RING as {A, B << 8}, else the
  // code word
  const auto load_codes = [&](const uint32_t c) __attribute__((always_inline)) -> uint32_t {
    uint32_t x = pad, y = pad;
    if (nib) {
      if (c < LA) x = (pA[c >> 1] >> (4 * (c & 1))) & 15u;
      if (c < LB) y = (pB[c >> 1] >> (4 * (c & 1))) & 15u;
    } else if (packed) {
      if (c < LA) x = (pA[c >> 2] >> (2 * (c & 3))) & 3u;
      if (c < LB) y = (pB[c >> 2] >> (2 * (c & 3))) & 3u;
    } else {
      if (c < LA) x = pA[c];
      if (c < LB) y = pB[c];
    }
    if constexpr (RING) return min(x, pad) | (min(y, pad) << 8);
    else return code_word(min(x, pad), min(y, pad));
  };
  const auto ring_write = [&](const uint32_t nc) __attribute__((always_inline)) {
    cring[lane] = (uint8_t)ringprev;  // letters of target A at [0, 128), B at [128, 256)
    cring[64 + lane] = (uint8_t)nc;
    cring[128 + lane] = (uint8_t)(ringprev >> 8);
    cring[192 + lane] = (uint8_t)(nc >> 8);
    ringprev = nc;
  };
  uint32_t nra = 0, nrb = 0;  // RING && PF: the letters of the next step's column
  // RING && PF: this lane's ring position of step 0 (step T + j reads ring byte 64 + j - lane)
  const uint8_t* const cring_l = RING && PF ? cring + 64 - lane : nullptr;
  if constexpr (RING && PF) {
    ring_write(load_codes((uint32_t)lane));
    nra = cring_l[0];
    nrb = cring_l[128];
  }
  // step t of the lane pipeline
  const auto step = [&](const int t, const bool even, auto segc) __attribute__((always_inline)) {
    constexpr bool SEG = decltype(segc)::in;  // query segment: row -1 from edge_in
    // false: this loop never writes a bottom row (no per-step branch around the store);
    // true: seg_out decides at run time
    constexpr bool SEGO = decltype(segc)::out;
    if (even && (t & 63) == 0) {  // next 64 columns, one code pair per lane
      const uint32_t c = (uint32_t)t + lane;
      if constexpr (RING && !PF) ring_write(load_codes(c));
      else if constexpr (!RING) buf = load_codes(c);
      if (SEG) ebuf = c < (uint32_t)Lmax ? ein[c & rmask] : make_uint2(as_u32(H0), as_u32(X0));
    }
    // prefetching ring: the next block's codes go in before step T + 64's codes are read
    if constexpr (RING && PF) {
      if (!even && (t & 63) == 63) ring_write(load_codes((uint32_t)t + 1u + lane));
    }
    const uint32_t inj = RING ? 0u : __builtin_amdgcn_readlane(buf, t & 63);
    u16x2 upH, upX;
    if constexpr (SEG) {
      upH = as_u16x2(dpp_shr1(__builtin_amdgcn_readlane(ebuf.x, t & 63), botH));
      upX = as_u16x2(dpp_shr1(__builtin_amdgcn_readlane(ebuf.y, t & 63), botX));
    } else {  // row -1 boundary; a zero boundary comes from DPP's bound_ctrl (no lane-0 move)
      upH = as_u16x2(as_u32(H0) == 0 ? dpp_shr1_zero(botH) : dpp_shr1(as_u32(H0), botH));
      upX = as_u16x2(as_u32(X0) == 0 ? dpp_shr1_zero(botX) : dpp_shr1(as_u32(X0), botX));
    }
    uint32_t rca = 0, rcb = 0;  // RING: the two letters of column t - lane
    if constexpr (RING && PF) {
      rca = nra;
      rcb = nrb;
    } else if constexpr (RING) {
      // (t & 62) is shared by the two steps of an iteration: one address add per two steps
      const uint8_t* rp = cring + (64 - lane) + (t & 62);
      rca = rp[even ? 0 : 1];
      rcb = rp[even ? 128 : 129];
    } else if constexpr (F16 && PROF) {  // shift down one lane and add the lane's row offset
      uint32_t nl = inj;
      asm volatile("s_nop 1\n\tv_add_u32_dpp %0, %1, %2 wave_shr:1 row_mask:0xf bank_mask:0xf"
                   : "+v"(nl) : "v"(let), "v"(hop));
      let = nl;
    } else {
      let = dpp_shr1(inj, let);
    }
    u16x2 diag = prevUpH;
    prevUpH = upH;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (F16) {
      const bool z = COL0 && t == lane;
      if constexpr (PROF) {
        ProfLookupK16<K> lk;
        const uint8_t* lds = RING ? prof + lane * 2 * K : prof;
        const uint32_t olo = RING ? __umul24(rca, PSb) : let & 0xFFFFu;
        const uint32_t ohi = RING ? __umul24(rcb, PSb) : let >> 16;
        if constexpr (K == 2) {
          lk.lo[0] = *reinterpret_cast<const uint32_t*>(lds + olo);
          lk.hi[0] = *reinterpret_cast<const uint32_t*>(lds + ohi);
        } else if constexpr (K == 4) {
          const uint2 x = *reinterpret_cast<const uint2*>(lds + olo);
          const uint2 y = *reinterpret_cast<const uint2*>(lds + ohi);
          lk.lo[0] = x.x; lk.lo[1] = x.y; lk.hi[0] = y.x; lk.hi[1] = y.y;
        } else {
#pragma unroll
          for (int q = 0; q < K / 8; ++q) {
            const uint4 x = reinterpret_cast<const uint4*>(lds + olo)[q];
            const uint4 y = reinterpret_cast<const uint4*>(lds + ohi)[q];
            lk.lo[4 * q] = x.x; lk.lo[4 * q + 1] = x.y; lk.lo[4 * q + 2] = x.z;
            lk.lo[4 * q + 3] = x.w;
            lk.hi[4 * q] = y.x; lk.hi[4 * q + 1] = y.y; lk.hi[4 * q + 2] = y.z;
            lk.hi[4 * q + 3] = y.w;
          }
        }
        if constexpr (RING && PF) {  // the next step's letters (block start: the new block)
          const uint8_t* np = cring_l + ((t + 1) & 63);
          nra = np[0];
          nrb = np[128];
        }
        if constexpr (COL0)
          column_merged_f16_mask<K, 4>(lk, diag, upX, Hl, Xl, best, NOE2, NE2, z);
        else
          column_f16_lane_asm<K, GOTOH>(lk, diag, upX, Hl, Xl, best, noe, ne, no);
      } else {
        const LaneLutLookup<K> lk{lut, nv, let};
        if constexpr (COL0)
          column_merged_f16_mask<K, 4>(lk, diag, upX, Hl, Xl, best, NOE2, NE2, z);
        else
          column_f16_lane_asm<K, GOTOH>(lk, diag, upX, Hl, Xl, best, noe, ne, no);
      }
    } else if constexpr (PROF) {
      ProfLookupK<K> lk;
      const uint32_t blo = let & 0xFFu, bhi = (let >> 16) & 0xFFu;
      if constexpr (K == 2) {  // 2 rows = 2 bytes
        lk.lo[0] = *reinterpret_cast<const uint16_t*>(prow + __umul24(blo, PSb));
        lk.hi[0] = *reinterpret_cast<const uint16_t*>(prow + __umul24(bhi, PSb));
      } else if constexpr (K == 4) {
        lk.lo[0] = *reinterpret_cast<const uint32_t*>(prow + __umul24(blo, PSb));
        lk.hi[0] = *reinterpret_cast<const uint32_t*>(prow + __umul24(bhi, PSb));
      } else if constexpr (K == 8) {
        const uint2 x = *reinterpret_cast<const uint2*>(prow + __umul24(blo, PSb));
        const uint2 y = *reinterpret_cast<const uint2*>(prow + __umul24(bhi, PSb));
        lk.lo[0] = x.x; lk.lo[1] = x.y; lk.hi[0] = y.x; lk.hi[1] = y.y;
      } else {
        const uint4 x = *reinterpret_cast<const uint4*>(prow + __umul24(blo, PSb));
        const uint4 y = *reinterpret_cast<const uint4*>(prow + __umul24(bhi, PSb));
        lk.lo[0] = x.x; lk.lo[1] = x.y; lk.lo[2] = x.z; lk.lo[3] = x.w;
        lk.hi[0] = y.x; lk.hi[1] = y.y; lk.hi[2] = y.z; lk.hi[3] = y.w;
      }
      if constexpr (GOTOH) {
        u16x2 uH = upH;
        column_gotoh<K, 4>(lk, diag, uH, upX, Hl, Xl, best, S2, OES2, E2);
      } else if constexpr (COL0) {
        column_merged_mask<K, 4>(lk, diag, upX, Hl, Xl, best, S2, O2, E2,
                                 t == lane ? 0u : 0xFFFFFFFFu);
      } else {
        column_merged<K, 4, false>(lk, diag, upX, Hl, Xl, best, S2, O2, E2);
      }
    } else {
      const LaneLutLookup<K> lk{lut, nv, let};
      if constexpr (GOTOH) {
        u16x2 uH = upH;
        column_gotoh<K, 4>(lk, diag, uH, upX, Hl, Xl, best, S2, OES2, E2);
      } else if constexpr (COL0) {
        column_merged_mask<K, 4>(lk, diag, upX, Hl, Xl, best, S2, O2, E2,
                                 t == lane ? 0u : 0xFFFFFFFFu);
      } else {
        column_merged<K, 4, false>(lk, diag, upX, Hl, Xl, best, S2, O2, E2);
      }
    }
    asm volatile("" : "+v"(best));
    botH = as_u32(Hl[K - 1]);
    botX = as_u32(upX);
    if (SEGO && seg_out && lane == 63 && t >= 63 && t - 63 < Lmax)
      eout[(uint32_t)(t - 63) & rmask] = make_uint2(botH, botX);
  };
  if constexpr (SPLIT) {
    // every wave of the block takes part in every phase's barrier (wave-uniform branches)
    const int lag = 2 * seg;
    for (int ph = 0; ph < nph + 2 * (P - 1); ++ph) {
      const int blk = ph - lag;
      if (blk >= 0 && blk < nph) {
        if (seg_in) {
          for (int t = 64 * blk; t < 64 * blk + 64; t += 2) {
            step(t, true, SegT<true, true>{});
            step(t + 1, false, SegT<true, true>{});
          }
        } else {
          for (int t = 64 * blk; t < 64 * blk + 64; t += 2) {
            step(t, true, SegT<false, true>{});
            step(t + 1, false, SegT<false, true>{});
          }
        }
      }
      __syncthreads();
    }
  } else if (seg_in) {
    for (int t = 0; t < nsteps; t += 2) {
      step(t, true, SegT<true, true>{});
      step(t + 1, false, SegT<true, true>{});
    }
  } else {
    for (int t = 0; t < nsteps; t += 2) {
      step(t, true, SegT<false, true>{});
      step(t + 1, false, SegT<false, true>{});
    }
  }
  // max over the wave's rows, per target (f16: non-negative integers -> int)
  uint32_t bx = best.x, by = best.y;
  if constexpr (F16) {
    bx = (uint32_t)f16_unscore(bx);
    by = (uint32_t)f16_unscore(by);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    bx = max(bx, (uint32_t)__shfl_xor((int)bx, off));
    by = max(by, (uint32_t)__shfl_xor((int)by, off));
  }
  return make_uint2(bx, by);
}

// Split-tail block (4 waves): 4 / P pairs from main_pairs + (4 / P) blockIdx.x on, wave w
// scoring row segment w % P of pair w / P at KS = K / P rows per lane (the main waves' K).  The
// segments' bests combine through LDS; an optimistic f16 pass whose block holds a pair above
// fb_thresh re-runs the whole block in u16 (a block-uniform choice: the barriers need every wave).
template <int KS, int P, bool COL0, bool PROF, bool GOTOH, bool F16>
__device__ __forceinline__ void wave_split_block(const ScoreArgs& a, uint32_t* smem, int lane) {
  constexpr int PPB = 4 / P;  // pairs per block
  uint8_t* prof = reinterpret_cast<uint8_t*>(smem);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int seg = wave % P;
  const size_t n = a.n, first = (size_t)a.main_pairs + (size_t)PPB * blockIdx.x;
  const size_t pair = first + wave / P;
  const size_t npairs = (n + 1) / 2;
  // the block's longest target -> phases (every wave runs the same number of barriers)
  uint32_t L = 0;
  if (lane < 2 * PPB) {
    const size_t t = 2 * first + lane;
    if (t < n)
      L = a.packed == SWK_PACK_RECORDS ? record_len(a.res + t * SWB_RECORD)
          : a.ustride                     ? a.ulen
                                          : a.lens[t];
  }
#pragma unroll
  for (int off = 2; off >= 1; off >>= 1) L = max(L, (uint32_t)__shfl_xor((int)L, off));
  const int nph = (int)((__builtin_amdgcn_readfirstlane(L) + 63 + 63) / 64);
  // a wave whose pair lies past the batch end (an odd tail) still runs every barrier: it
  // scores the block's first pair again and writes nothing
  const bool real = pair < npairs;
  const size_t p = real ? pair : first;
  uint2* ring = a.split_ring + ((size_t)PPB * blockIdx.x + wave / P) * (P - 1) * 256;
  const uint2* lin = seg > 0 ? ring + (seg - 1) * 256 : nullptr;
  uint2* lout = seg < P - 1 ? ring + seg * 256 : nullptr;
  if constexpr (PROF) {
    const uint32_t words = P * a.split_words / 4;  // every segment's profile, 16 B at a time
    const uint4* src = reinterpret_cast<const uint4*>(a.split_qtab);
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x)
      reinterpret_cast<uint4*>(prof)[i] = src[i];
    __syncthreads();
  }
  const uint8_t* sprof = PROF ? prof + (size_t)seg * a.split_words * 4 : nullptr;
  const uint32_t* sq = a.split_qtab + (size_t)seg * a.split_words;
  uint2 b = wave_pair<KS, COL0, PROF, GOTOH, F16, true>(a, sprof, sq, a.nv, a.split_PS, p, lane,
                                                         lin, lout, nph, seg, P);
  // LDS is free again (the last phase ended with a barrier): combine the pair's segments
  uint32_t blockmax = 0;
  const auto combine = [&](uint2 v) -> uint2 {
    if (lane == 0) {
      smem[2 * wave] = v.x;
      smem[2 * wave + 1] = v.y;
    }
    __syncthreads();
    const int w0 = wave - seg;
    uint2 r = make_uint2(0u, 0u);
#pragma unroll
    for (int k = 0; k < P; ++k) {
      r.x = max(r.x, smem[2 * (w0 + k)]);
      r.y = max(r.y, smem[2 * (w0 + k) + 1]);
    }
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) m = max(m, smem[k]);
    blockmax = m;
    __syncthreads();  // read before anyone rewrites the slots
    return r;
  };
  b = combine(b);
  if constexpr (F16) {
    if (a.fb_qtab && (int32_t)blockmax > a.fb_thresh) {
      const uint8_t* fprof = PROF ? reinterpret_cast<const uint8_t*>(a.split_fb_qtab) +
                                        (size_t)seg * a.split_fb_words * 4
                                  : nullptr;
      b = wave_pair<KS, COL0, PROF, GOTOH, false, true>(
          a, fprof, a.split_fb_qtab + (size_t)seg * a.split_fb_words, a.fb_nv, a.split_fb_PS, p,
          lane, lin, lout, nph, seg, P);
      b = combine(b);
    }
  }
  if (lane == 0 && seg == 0 && real) {
    const size_t tA = 2 * p, tB = tA + 1;
    int32_t sa = (int32_t)b.x, sb = (int32_t)b.y;
    if (a.accum) {
      sa = max(sa, a.scores[tA]);
      if (tB < n) sb = max(sb, a.scores[tB]);
    }
    a.scores[tA] = sa;
    if (tB < n) a.scores[tB] = sb;
  }
}

template <int K, bool COL0, bool PROF, bool GOTOH, bool F16>
__global__ void __launch_bounds__(512) score_wave(const ScoreArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint8_t* prof = reinterpret_cast<uint8_t*>(smem);
  const int lane = threadIdx.x & 63;
  if constexpr (K >= 8) {
    if (blockIdx.x < a.split_blocks) {  // block-uniform
      if (a.split_P == 4) wave_split_block<K / 4, 4, COL0, PROF, GOTOH, F16>(a, smem, lane);
      else wave_split_block<K / 2, 2, COL0, PROF, GOTOH, F16>(a, smem, lane);
      return;
    }
  }
  if constexpr (PROF) {
    const uint32_t words = (a.pad + 1) * a.PS / 16;
    const uint4* src = reinterpret_cast<const uint4*>(a.qtab);
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x)
      reinterpret_cast<uint4*>(prof)[i] = src[i];
    __syncthreads();
  }
  const size_t pair = (size_t)(blockIdx.x - a.split_blocks) * (blockDim.x >> 6) +
                      __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const size_t tA = 2 * pair, tB = tA + 1;
  const size_t n = a.n;
  if (tA >= n || pair >= a.main_pairs) return;  // whole wave
  // f16 profile: each wave's code ring follows the profile in LDS
  uint8_t* cring = F16 && PROF ? prof + (a.pad + 1) * a.PS + 256 * (threadIdx.x >> 6) : nullptr;
  uint2 b = wave_pair<K, COL0, PROF, GOTOH, F16>(a, prof, a.qtab, a.nv, a.PS, pair, lane,
                                                 nullptr, nullptr, 0, 0, 1, cring);
  if constexpr (F16) {
    // optimistic f16: a pair above 2048 - max(s) may have rounded; re-score it in u16 now
    // (the profile from HBM: rare, and no LDS for a second table)
    if (a.fb_qtab && (int32_t)max(b.x, b.y) > a.fb_thresh)
      b = wave_pair<K, COL0, PROF, GOTOH, false>(a, reinterpret_cast<const uint8_t*>(a.fb_qtab),
                                                 a.fb_qtab, a.fb_nv, a.fb_PS, pair, lane);
  }
  if (lane == 0) {
    int32_t sa = (int32_t)b.x, sb = (int32_t)b.y;
    if (a.accum) {  // best over the previous query segments
      sa = max(sa, a.scores[tA]);
      if (tB < n) sb = max(sb, a.scores[tB]);
    }
    a.scores[tA] = sa;
    if (tB < n) a.scores[tB] = sb;
  }
}

template <int K, bool COL0, bool PROF, bool GOTOH, bool F16>
static hipError_t launch_wave(const ScoreArgs& a, uint32_t prof_bytes, hipStream_t st) {
  // 4 waves (pairs) per block, sharing one LDS copy of the profile (measured on 12.5k protein
  // targets: 4 and 5 best, 8 -11 %, 2 -25 %); the split tail needs 4-wave blocks
  const unsigned wpb = 4u;
  const size_t blocks = a.split_blocks + ((size_t)a.main_pairs + wpb - 1) / wpb;
  size_t lds = PROF ? prof_bytes : 0;
  if (F16 && PROF) lds += 256 * wpb;  // the waves' code rings
  if (a.split_blocks)  // every segment's profile, or the 8 words of the segment combine
    lds = std::max<size_t>(lds, PROF ? (size_t)a.split_words * 4 * a.split_P : 64);
  auto fn = &score_wave<K, COL0, PROF, GOTOH, F16>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  if (lds > 160 * 1024) return hipErrorInvalidConfiguration;
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(64 * wpb), (unsigned)lds, st, a);
  return hipGetLastError();
}

// Two pairs per wave (f16 profile, one query segment of <= 512 rows: configs[4]'s protein
// shape).  Lanes 0-31 score pair p0, lanes 32-63 pair p0 + 1, lane l owning rows
// [16 (l % 32), 16 (l % 32) + 16) of the same 512-row profile as the one-pair kernel's K = 8
// layout (32 B per lane per letter).  Against one pair per wave at 8 rows per lane:
// * the per-step work besides the column (two DPP moves of the bottom row, two profile
//   addresses, the ring letters) is shared by 16 rows instead of 8;
// * the lane pipeline is 32 deep: a pair's fill and drain skew is 31 steps, not 63;
// * each half's lane 0 takes the row -1 boundary (lane 32 would otherwise read lane 31's
//   bottom row through wave_shr): one v_cndmask per moved value.
// Each half keeps its own 128-byte code ring (targets A, B: [previous 32 | next 32] columns).
// Returns the half's two bests (every lane of the half).
// Balanced ranges (score_wave_half, ScoreArgs.wbal_blocks): a visit may run steps [t0, t1) of
// the unit only (t0, t1 multiples of 32): it starts from the lane state a predecessor's head
// visit stored at sin and, when it stops before the unit's end, stores its own at sout (the
// return value is then meaningless).  The state is complete: the lanes' rows {H, E/T}, the
// running best, the diagonal above, the bottom row that moves down at the next step; the code
// ring and the profile words of the first steps are rebuilt from the codes.
constexpr int WBAL_WORDS = 2 * 16 + 4;  // state words per lane (K = 16)
template <bool GOTOH>
__device__ __forceinline__ uint2 wave_two_pairs(const ScoreArgs& a, const uint8_t* prof,
                                                uint8_t* cring, int lane, size_t p0,
                                                int t0 = 0, int t1 = 0x7FFFFFFF,
                                                const uint32_t* sin = nullptr,
                                                uint32_t* sout = nullptr) {
  constexpr int K = 16;
  t0 = __builtin_amdgcn_readfirstlane(t0);  // (wave-uniform step bounds)
  t1 = __builtin_amdgcn_readfirstlane(t1);
  const int h = lane >> 5, hl = lane & 31;
  const size_t pair = p0 + (size_t)h;
  const size_t n = a.n;
  const bool have = pair < a.main_pairs;
  const size_t tA = 2 * pair, tB = tA + 1;
  const bool packed = a.packed != SWK_PACK_BYTES, rec = a.packed == SWK_PACK_RECORDS;
  const bool nib = a.packed == SWK_PACK_NIBBLE;
  const bool uni = a.ustride != 0;
  uint32_t LA = 0, LB = 0;
  const uint8_t* pA = a.res;
  const uint8_t* pB = a.res;
  if (have) {
    LA = rec ? record_len(a.res + tA * SWB_RECORD) : uni ? a.ulen : a.lens[tA];
    LB = tB >= n ? 0u : rec ? record_len(a.res + tB * SWB_RECORD) : uni ? a.ulen : a.lens[tB];
    pA = rec ? a.res + tA * SWB_RECORD + 6 : uni ? a.res + tA * a.ustride
                                                 : a.res + (LA ? a.offs[tA] : 0);
    const size_t tb = tB < n ? tB : tA;
    pB = rec ? a.res + tb * SWB_RECORD + 6 : uni ? a.res + tb * a.ustride
                                                 : a.res + (LB ? a.offs[tB] : 0);
  }
  uint32_t Lh = max(LA, LB);
  Lh = max(Lh, (uint32_t)__shfl_xor((int)Lh, 32));
  const int Lmax = (int)__builtin_amdgcn_readfirstlane(Lh);
  const uint32_t pad = a.pad, PSb = a.PS;
  const f16x2 NOE2 = as_f16x2(as_u16x2(a.f16_noe)), NE2 = as_f16x2(as_u16x2(a.f16_ne)),
              NO2 = as_f16x2(as_u16x2(a.f16_no));
  const uint32_t noe = as_u32(as_u16x2(NOE2)), ne = as_u32(as_u16x2(NE2)),
                 no = as_u32(as_u16x2(NO2));
  (void)NO2;
  const u16x2 H0 = {0, 0};
  const u16x2 X0 = GOTOH ? (u16x2){0, 0} : as_u16x2(NOE2);  // F / T of row -1
  u16x2 Hl[K], Xl[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    Hl[k] = H0;
    Xl[k] = X0;
  }
  u16x2 best = {0, 0}, prevUpH = H0;
  uint32_t botH = as_u32(H0), botX = as_u32(X0);
  if (sin) {  // a tail visit: the predecessor's lane state (sc1 loads, word i at i x 64 + lane)
    const uint32_t* sp = sin + lane;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      Hl[k] = as_u16x2(__hip_atomic_load(sp + k * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      Xl[k] = as_u16x2(
          __hip_atomic_load(sp + (K + k) * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    best = as_u16x2(__hip_atomic_load(sp + 2 * K * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    prevUpH = as_u16x2(
        __hip_atomic_load(sp + (2 * K + 1) * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    botH = __hip_atomic_load(sp + (2 * K + 2) * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    botX = __hip_atomic_load(sp + (2 * K + 3) * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const bool top = hl == 0;  // row -1 of this half's pair
  // (SWK_HALF_DPPSEL) the boundary lanes 0 and 32, and row -1's H and F / T in VGPRs
  const uint64_t topmask = 0x0000000100000001ull;
  uint32_t h0v = as_u32(H0), x0v = as_u32(X0);
  asm volatile("" : "+v"(h0v), "+v"(x0v));
  (void)topmask;
  // the codes of column c of this half's targets (pad past the end) as {A, B << 8}
  const auto load_codes = [&](const uint32_t c) __attribute__((always_inline)) -> uint32_t {
    uint32_t x = pad, y = pad;
    if (nib) {
      if (c < LA) x = (pA[c >> 1] >> (4 * (c & 1))) & 15u;
      if (c < LB) y = (pB[c >> 1] >> (4 * (c & 1))) & 15u;
    } else if (packed) {
      if (c < LA) x = (pA[c >> 2] >> (2 * (c & 3))) & 3u;
      if (c < LB) y = (pB[c >> 2] >> (2 * (c & 3))) & 3u;
    } else {
      if (c < LA) x = pA[c];
      if (c < LB) y = pB[c];
    }
    return min(x, pad) | (min(y, pad) << 8);
  };
  // ring entries are profile offsets (letter x LS), 32-bit (or 16-bit loads that zero-extend):
  // a byte entry read in one step and used in the next would be masked again in every basic
  // block it crosses
  typedef typename std::conditional<SWK_HALF_FMA != 0, uint16_t, uint32_t>::type RingT;
  constexpr uint32_t LS = SWK_HALF_LS;
  (void)PSb;
  RingT* ring = reinterpret_cast<RingT*>(cring) + 128 * h;
  const RingT* ring_l = ring + 32 - hl;  // step T + j reads ring_l[j] (A), ring_l[64 + j] (B)
  uint32_t ringprev = pad | pad << 8;
  // SWK_HALF_ABS: slot j of a half's ring (j in [0, 64): the window before and the current 32
  // columns) holds the LDS byte address, from the block's LDS base, that lane hl needs at window
  // step u when it reads slot j = 32 - hl + u, minus 16 u: the lane's rows of the column's letter
  // sit at profile + letter x LS + 16 hl = (SWK_HALF_ABS_BASE + letter x LS + 16 (32 - j)) + 16 u,
  // so the step adds 16 u and the profile piece as load offsets (immediates once the window is
  // unrolled) and no address is computed.  Entries stay in [16, 65535] (24 letters x 2 KB).
  const auto ring_entry = [&](uint32_t letter, uint32_t j) __attribute__((always_inline)) {
    return SWK_HALF_ABS ? (RingT)(SWK_HALF_ABS_BASE + letter * LS + 512u - 16u * j)
                        : (RingT)(letter * LS);
  };
  const auto ring_write = [&](const uint32_t nc) __attribute__((always_inline)) {
    ring[hl] = ring_entry(ringprev & 0xFFu, hl);
    ring[32 + hl] = ring_entry(nc & 0xFFu, 32 + hl);
    ring[64 + hl] = ring_entry(ringprev >> 8, hl);
    ring[96 + hl] = ring_entry(nc >> 8, 32 + hl);
    ringprev = nc;
  };
  // the ring holds the 32-column blocks k - 1 and k while steps 32 k .. 32 k + 31 run (k = t0 /
  // 32 at the start of a visit); ncode the next block's codes, one block ahead
  const uint32_t c0 = (uint32_t)t0;
  if (c0) ringprev = load_codes(c0 - 32u + hl);
  ring_write(load_codes(c0 + hl));
  uint32_t ncode = load_codes(c0 + 32u + hl);
  // score_wave_half's LDS copy of the profile keeps each letter's rows of every lane in 16-byte
  // pieces 512 bytes apart (piece q of lane l at 512 q + 16 l): a ds_read_b128 of 16 lanes then
  // covers all 64 banks.  2-byte entries: 2 pieces (rows 0-7, 8-15); FMA words: 4 pieces.
  typedef typename std::conditional<SWK_HALF_FMA != 0, ProfLookupF<K>, ProfLookupK16<K>>::type LK;
  const uint8_t* plds = prof + hl * 16;
  // (SWK_HALF_ABS: u = the step's place in the ring window, 16 u a load offset; a ring entry IS
  // the LDS byte address: score_wave_half declares no static LDS, so its dynamic LDS -- the
  // profile at SWK_HALF_ABS_BASE -- starts at LDS address 0.  An integer turned into an LDS
  // pointer, because "dynamic LDS base + entry" keeps an add of the base symbol (0) per load
  // address that LLVM does not fold.)
  const auto load_prof = [&](auto& lk, uint32_t oa, uint32_t ob, uint32_t u = 0)
                             __attribute__((always_inline)) {
#if SWK_HALF_ABS
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) const v4u lds_v4u;
    (void)plds;
#pragma unroll
    for (int q = 0; q < K / 4; ++q) {
      const v4u x = *reinterpret_cast<lds_v4u*>((uintptr_t)(oa + 16u * u + 512u * q));
      const v4u y = *reinterpret_cast<lds_v4u*>((uintptr_t)(ob + 16u * u + 512u * q));
      lk.a[4 * q] = x.x; lk.a[4 * q + 1] = x.y; lk.a[4 * q + 2] = x.z; lk.a[4 * q + 3] = x.w;
      lk.b[4 * q] = y.x; lk.b[4 * q + 1] = y.y; lk.b[4 * q + 2] = y.z; lk.b[4 * q + 3] = y.w;
    }
#else
    (void)u;
    const uint8_t* la = plds + oa;
    const uint8_t* lb = plds + ob;
    if constexpr (SWK_HALF_FMA) {
#pragma unroll
      for (int q = 0; q < K / 4; ++q) {
        const uint4 x = *reinterpret_cast<const uint4*>(la + 512 * q);
        const uint4 y = *reinterpret_cast<const uint4*>(lb + 512 * q);
        lk.a[4 * q] = x.x; lk.a[4 * q + 1] = x.y; lk.a[4 * q + 2] = x.z; lk.a[4 * q + 3] = x.w;
        lk.b[4 * q] = y.x; lk.b[4 * q + 1] = y.y; lk.b[4 * q + 2] = y.z; lk.b[4 * q + 3] = y.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < K / 8; ++q) {
        const uint4 x = *reinterpret_cast<const uint4*>(la + 512 * q);
        const uint4 y = *reinterpret_cast<const uint4*>(lb + 512 * q);
        lk.lo[4 * q] = x.x; lk.lo[4 * q + 1] = x.y; lk.lo[4 * q + 2] = x.z; lk.lo[4 * q + 3] = x.w;
        lk.hi[4 * q] = y.x; lk.hi[4 * q + 1] = y.y; lk.hi[4 * q + 2] = y.z; lk.hi[4 * q + 3] = y.w;
      }
    }
#endif
  };
  // AHEAD: a step's profile words are loaded during the step before (its ring entries two
  // steps before), so no step waits on its own LDS reads: with 3-4 waves per SIMD the other
  // waves hide less of that latency than the one-pair kernel's 6
  constexpr bool AHEAD = SWK_HALF_AHEAD != 0;
  LK lkn;
  uint32_t nra, nrb;
  if constexpr (AHEAD) {
    load_prof(lkn, ring_l[0], ring_l[64]);
    nra = ring_l[1];
    nrb = ring_l[65];
  } else {
    nra = ring_l[0];
    nrb = ring_l[64];
  }
  // AHEAD: step t reads the ring entries of step t + 2 at rp = ring_l + ((t + 2) & 31); a pair
  // of steps from an even t never wraps, so one address per pair and immediate offsets.
  // SWK_HALF_UNROLL: steps per loop iteration (2 or 4)
  const RingT* rp = ring_l;
#if SWK_HALF_ABS
  // one step at window place u (t & 31 == u): the ring refill at u = 30, the words of step t + 1
  // (place u + 1) and the ring entries of step t + 2 (place u + 2) read with constant offsets
  // when u is a constant (the unrolled window below), else (the last partial window) computed
  const auto step_abs = [&](const int t, const int u) __attribute__((always_inline)) {
    if (u == 30) {
      ring_write(ncode);
      uint32_t tt = (uint32_t)t;
      asm volatile("" : "+s"(tt));
      ncode = load_codes(tt + 34u + hl);
    }
    LK lk = lkn;
    load_prof(lkn, nra, nrb, (uint32_t)((u + 1) & 31));
    nra = ring_l[(u + 2) & 31];
    nrb = ring_l[64 + ((u + 2) & 31)];
    __builtin_amdgcn_sched_barrier(0);
    u16x2 upH, upX;
    uint32_t uh, ux;
    asm volatile(
        "s_nop 1\n\t"
        "s_mov_b64 vcc, %[m]\n\t"
        "v_cndmask_b32_dpp %[uh], %[bh], %[h0], vcc wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "v_cndmask_b32_dpp %[ux], %[bx], %[x0], vcc wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : [uh] "=&v"(uh), [ux] "=&v"(ux)
        : [bh] "v"(botH), [bx] "v"(botX), [h0] "v"(h0v), [x0] "v"(x0v), [m] "s"(topmask)
        : "vcc");
    upH = as_u16x2(uh);
    upX = as_u16x2(ux);
    u16x2 diag = prevUpH;
    prevUpH = upH;
    __builtin_amdgcn_sched_barrier(0);
    column_f16_lane_asm<K, GOTOH>(lk, diag, upX, Hl, Xl, best, noe, ne, no);
    asm volatile("" : "+v"(best));
    botH = as_u32(Hl[K - 1]);
    botX = as_u32(upX);
  };
#endif
  const auto step = [&](const int t, const bool even) __attribute__((always_inline)) {
    // the next 32 columns go in before they are read (AHEAD: two steps before)
    if ((AHEAD ? even : !even) && (t & 31) == (AHEAD ? 30 : 31)) {
      ring_write(ncode);
      // (t through an opaque copy: no per-step pointer increments for these loads)
      uint32_t tt = (uint32_t)t;
      asm volatile("" : "+s"(tt));
      ncode = load_codes(tt + (AHEAD ? 34u : 33u) + hl);
    }
    LK lk;
    if constexpr (AHEAD) {
      lk = lkn;
      load_prof(lkn, nra, nrb);
      const RingT* np = rp + (even ? 0 : 1);  // (t is even in an even step: an immediate offset)
      nra = np[0];
      nrb = np[64];
      __builtin_amdgcn_sched_barrier(0);
    }
    u16x2 upH, upX;
    if constexpr (SWK_HALF_DPPSEL != 0) {
      // lanes 0 and 32 in VCC: v_cndmask_b32 D = VCC ? src1 : src0, src0 read through
      // wave_shr:1 (bound_ctrl: lane 0 reads 0 and is written); s_nop 1: the two wait states a
      // DPP read needs after the VALU write of its source (inside asm LLVM inserts none)
      uint32_t uh, ux;
      asm volatile(
          "s_nop 1\n\t"
          "s_mov_b64 vcc, %[m]\n\t"
          "v_cndmask_b32_dpp %[uh], %[bh], %[h0], vcc wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
          "v_cndmask_b32_dpp %[ux], %[bx], %[x0], vcc wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1"
          : [uh] "=&v"(uh), [ux] "=&v"(ux)
          : [bh] "v"(botH), [bx] "v"(botX), [h0] "v"(h0v), [x0] "v"(x0v), [m] "s"(topmask)
          : "vcc");
      upH = as_u16x2(uh);
      upX = as_u16x2(ux);
    } else {
      upH = as_u16x2(dpp_shr1_zero(botH));
      upX = as_u16x2(GOTOH ? dpp_shr1_zero(botX) : dpp_shr1(as_u32(X0), botX));
      upH = top ? H0 : upH;
      upX = top ? X0 : upX;
    }
    u16x2 diag = prevUpH;
    prevUpH = upH;
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!AHEAD) {
      load_prof(lk, nra, nrb);
      const RingT* np = ring_l + ((t + 1) & 31);  // the next step's profile offsets
      nra = np[0];
      nrb = np[64];
    }
    column_f16_lane_asm<K, GOTOH>(lk, diag, upX, Hl, Xl, best, noe, ne, no);
    asm volatile("" : "+v"(best));
    botH = as_u32(Hl[K - 1]);
    botX = as_u32(upX);
  };
  const int nsteps = min(Lmax + 31, t1);
#if SWK_HALF_ABS
  (void)step;
  (void)rp;
  // whole 32-step windows unrolled (t0 is a multiple of 32), then the last partial window
  int t = t0;
  for (; t + 32 <= nsteps; t += 32) {
#pragma unroll
    for (int u = 0; u < 32; ++u) step_abs(t + u, u);
  }
  for (; t < nsteps; ++t) step_abs(t, t & 31);
#else
  for (int t = t0; t < nsteps; t += SWK_HALF_UNROLL) {
#pragma unroll
    for (int u = 0; u < SWK_HALF_UNROLL; u += 2) {
      rp = ring_l + ((t + u + 2) & 31);
      step(t + u, true);
      step(t + u + 1, false);
    }
  }
#endif
  if (sout) {  // a head visit: the lane state for the successor's tail visit (sc1 stores)
    uint32_t* sp = sout + lane;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      __hip_atomic_store(sp + k * 64, as_u32(Hl[k]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sp + (K + k) * 64, as_u32(Xl[k]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    __hip_atomic_store(sp + 2 * K * 64, as_u32(best), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sp + (2 * K + 1) * 64, as_u32(prevUpH), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sp + (2 * K + 2) * 64, botH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sp + (2 * K + 3) * 64, botX, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint2(0u, 0u);
  }
  uint32_t bx = (uint32_t)f16_unscore(best.x), by = (uint32_t)f16_unscore(best.y);
#pragma unroll
  for (int off = 16; off >= 1; off >>= 1) {  // within the half
    bx = max(bx, (uint32_t)__shfl_xor((int)bx, off));
    by = max(by, (uint32_t)__shfl_xor((int)by, off));
  }
  return make_uint2(bx, by);
}

// A tail segment wave of the two-pairs kernel (ScoreArgs.tail_*): pair main_pairs + ti, rows
// [64 s, 64 s + 64) of the query, lane l = row 64 s + l (one row per lane), the one-pair wave
// walk (step t: lane l computes column t - l).  Row -1 of the segment (s > 0) is segment s - 1's
// bottom row from split_ring, read 64 columns at a time once segment s - 1 has finished the
// 64-column block after them (lane 63 of segment s - 1 writes column c at step c + 63); lane
// 63 writes this segment's bottom row.  Hand-offs: sc1 stores, vmcnt(0), an sc1 progress word;
// sc1 polls and sc1 loads (MI355X_MICROARCH.md, inter-workgroup visibility).  The ring holds
// every column, so no segment waits for the one below it: waits point only to lower block
// numbers (dispatched earlier).  The last segment combines the segments' bests, re-scores the
// pair in u16 when it crossed the optimistic f16 threshold, and writes the scores.
template <bool GOTOH>
__device__ __forceinline__ void wave_tail_seg(const ScoreArgs& a, uint8_t* wlds, int lane,
                                           unsigned u) {
  const unsigned T = a.tail_pairs, P = a.split_P;
  const unsigned s = u / T, ti = u % T;
  const size_t pair = (size_t)a.main_pairs + ti;
  const size_t n = a.n, tA = 2 * pair, tB = tA + 1;
  // this segment's f16 profile (letters x 64 rows x 2 B) into the wave's LDS slice
  {
    const uint32_t words = a.split_words;
    const uint32_t* src = a.split_qtab + (size_t)s * words;
    for (uint32_t i = lane; i < words; i += 64) reinterpret_cast<uint32_t*>(wlds)[i] = src[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  const bool packed = a.packed != SWK_PACK_BYTES, rec = a.packed == SWK_PACK_RECORDS;
  const bool nib = a.packed == SWK_PACK_NIBBLE, uni = a.ustride != 0;
  const uint32_t LA = rec ? record_len(a.res + tA * SWB_RECORD) : uni ? a.ulen : a.lens[tA];
  const uint32_t LB = tB >= n ? 0u : rec ? record_len(a.res + tB * SWB_RECORD) : uni ? a.ulen
                                                                                   : a.lens[tB];
  const uint8_t* pA = rec ? a.res + tA * SWB_RECORD + 6 : uni ? a.res + tA * a.ustride
                                                              : a.res + (LA ? a.offs[tA] : 0);
  const uint8_t* pB = rec ? a.res + (tB < n ? tB : tA) * SWB_RECORD + 6
                      : uni ? a.res + (tB < n ? tB : tA) * a.ustride
                            : a.res + (LB ? a.offs[tB] : 0);
  const int Lmax = (int)__builtin_amdgcn_readfirstlane(max(LA, LB));
  const int nblk = (Lmax + 63 + 63) / 64;
  const uint32_t pad = a.pad, PSb = a.split_PS;
  const f16x2 NOE2 = as_f16x2(as_u16x2(a.f16_noe)), NE2 = as_f16x2(as_u16x2(a.f16_ne));
  const u16x2 H0 = {0, 0};
  const u16x2 X0 = GOTOH ? (u16x2){0, 0} : as_u16x2(NOE2);  // F / T of row -1
  const auto code_word = [&](uint32_t c) -> uint32_t {  // letter offsets of column c
    uint32_t x = pad, y = pad;
    if (nib) {
      if (c < LA) x = (pA[c >> 1] >> (4 * (c & 1))) & 15u;
      if (c < LB) y = (pB[c >> 1] >> (4 * (c & 1))) & 15u;
    } else if (packed) {
      if (c < LA) x = (pA[c >> 2] >> (2 * (c & 3))) & 3u;
      if (c < LB) y = (pB[c >> 2] >> (2 * (c & 3))) & 3u;
    } else {
      if (c < LA) x = pA[c];
      if (c < LB) y = pB[c];
    }
    return min(x, pad) * PSb | (min(y, pad) * PSb) << 16;
  };
  uint32_t* prog = a.tail_prog + (size_t)ti * P;
  uint2* bests = reinterpret_cast<uint2*>(a.tail_prog + (size_t)T * P) + (size_t)ti * P;
  const auto wait_for = [&](const uint32_t* w, uint32_t v) {
    for (uint32_t it = 0; it < a.poll_limit; ++it) {
      if (__builtin_amdgcn_readfirstlane(
              __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >= v)
        return;
      __builtin_amdgcn_s_sleep(4);
    }
    if (lane == 0) report_fault(a.fault, SWK_FAULT_TAIL);
  };
  // (test hook) segment 0 of tail pair stall - 1 publishes nothing
  const bool mute = a.stall != 0 && s == 0 && ti + 1 == a.stall;
  const uint2* rin = s > 0 ? a.split_ring + ((size_t)ti * (P - 1) + (s - 1)) * a.tail_cols
                           : nullptr;
  uint2* rout = s + 1 < P ? a.split_ring + ((size_t)ti * (P - 1) + s) * a.tail_cols : nullptr;
  u16x2 Hl[1] = {H0}, Xl[1] = {X0};
  u16x2 best = {0, 0}, prevUpH = H0;
  uint32_t botH = as_u32(H0), botX = as_u32(X0);
  uint32_t let = code_word(~0u) + lane * (2u | 2u << 16);  // (padding, plus the row hop)
  const uint8_t* plds = wlds;
  for (int blk = 0; blk < nblk; ++blk) {
    const uint32_t c0 = 64u * (uint32_t)blk + (uint32_t)lane;
    const uint32_t buf = code_word(c0);
    uint2 ebuf = make_uint2(as_u32(H0), as_u32(X0));
    if (s > 0) {  // segment s - 1 finished block blk + 1 (or all of its blocks)
      wait_for(prog + s - 1, (uint32_t)min(blk + 2, nblk));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (c0 < (uint32_t)Lmax) {
        const uint64_t v =
            __hip_atomic_load(reinterpret_cast<const uint64_t*>(rin + c0), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
        ebuf = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
      }
    }
    for (int j = 0; j < 64; ++j) {
      const int t = 64 * blk + j;
      const uint32_t injH = s > 0 ? __builtin_amdgcn_readlane(ebuf.x, j) : as_u32(H0);
      const uint32_t injX = s > 0 ? __builtin_amdgcn_readlane(ebuf.y, j) : as_u32(X0);
      u16x2 upH = as_u16x2(__builtin_amdgcn_update_dpp(injH, botH, 0x138, 0xF, 0xF, false));
      u16x2 upX = as_u16x2(__builtin_amdgcn_update_dpp(injX, botX, 0x138, 0xF, 0xF, false));
      let = __builtin_amdgcn_update_dpp(__builtin_amdgcn_readlane(buf, j), let + (2u | 2u << 16),
                                        0x138, 0xF, 0xF, false);
      u16x2 diag = prevUpH;
      prevUpH = upH;
      // (let carries both letters' profile offsets plus this lane's row, 2 B per hop)
      const uint32_t eA = *reinterpret_cast<const uint16_t*>(plds + (let & 0xFFFFu));
      const uint32_t eB = *reinterpret_cast<const uint16_t*>(plds + (let >> 16));
      struct One {
        uint32_t w;
        __device__ __forceinline__ u16x2 operator()(int) const { return as_u16x2(w); }
      } lk{eA | eB << 16};
      if constexpr (GOTOH)
        column_gotoh_f16<1, 1>(lk, diag, upX, Hl, Xl, best, NOE2, NE2);
      else
        column_merged_f16<1, 1, false>(lk, diag, upX, Hl, Xl, best, NOE2, NE2);
      botH = as_u32(Hl[0]);
      botX = as_u32(GOTOH ? upX : Xl[0]);
      if (rout && lane == 63 && t >= 63 && t - 63 < Lmax) {
        const uint64_t v = (uint64_t)botX << 32 | botH;
        __hip_atomic_store(reinterpret_cast<uint64_t*>(rout + (t - 63)), v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (rout) {  // this block's ring columns are out
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0 && !mute)
        __hip_atomic_store(prog + s, (uint32_t)(blk + 1), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  uint32_t bx = (uint32_t)f16_unscore(best.x), by = (uint32_t)f16_unscore(best.y);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    bx = max(bx, (uint32_t)__shfl_xor((int)bx, off));
    by = max(by, (uint32_t)__shfl_xor((int)by, off));
  }
  if (s + 1 < P) {  // hand the segment's bests to the last segment
    if (lane == 0) {
      const uint64_t v = (uint64_t)by << 32 | bx;
      __hip_atomic_store(reinterpret_cast<uint64_t*>(bests + s), v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0 && !mute)
      __hip_atomic_store(prog + s, (uint32_t)nblk + 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  for (unsigned k = 0; k + 1 < P; ++k) {
    wait_for(prog + k, (uint32_t)nblk + 1u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t v = __hip_atomic_load(reinterpret_cast<const uint64_t*>(bests + k),
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bx = max(bx, (uint32_t)v);
    by = max(by, (uint32_t)(v >> 32));
  }
  uint2 b = make_uint2(bx, by);
  // optimistic f16: a pair above 2048 - max(s) is re-scored in u16 (one-pair K = 8 walk, the
  // u16 profile from HBM)
  if (a.fb_qtab && (int32_t)max(bx, by) > a.fb_thresh)
    b = wave_pair<8, false, true, GOTOH, false>(a, reinterpret_cast<const uint8_t*>(a.fb_qtab),
                                                a.fb_qtab, a.fb_nv, a.fb_PS, pair, lane);
  if (lane == 0) {
    a.scores[tA] = (int32_t)b.x;
    if (tB < n) a.scores[tB] = (int32_t)b.y;
  }
}

// configs[4]'s kernel: the wave kernel's split tail (blocks [0, split_blocks), as in
// score_wave<8>) and main blocks of 4 waves scoring two pairs each (wave_two_pairs).  A pair
// above the optimistic f16 threshold is re-scored in u16 by the whole wave with the one-pair
// K = 8 code and table (rare).
template <bool GOTOH>
__device__ __forceinline__ void wave_half_finish(const ScoreArgs& a, uint2 b, int lane,
                                                 size_t p0);

// W waves per block share one LDS copy of the profile: W = 4 (3 blocks per CU: 3 waves per
// SIMD) or W = 8 (2 blocks per CU: 4 waves per SIMD, <= 128 VGPRs; balanced launches only)
template <bool GOTOH, int W>
__global__ void __launch_bounds__(64 * W, W == 8 ? 4 : 1) score_wave_half(const ScoreArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint8_t* prof = reinterpret_cast<uint8_t*>(smem);
  const int lane = threadIdx.x & 63;
#if SWK_STAMPS
  // (measurement builds: launch_wave_half passes the record buffer in tctr) per wave: entry,
  // exit, the profile copy's end, ticks in hand-off waits, HW_ID, XCC, visits, block
  const uint64_t st_t0 = __builtin_amdgcn_s_memtime();
  uint64_t st_copy = 0, st_wait = 0;
  const auto stamp_out = [&](int wave_, int nvis_) {
    uint64_t* g = reinterpret_cast<uint64_t*>(a.tctr);
    if (!g || lane != 0) return;
    uint64_t* o = g + ((size_t)blockIdx.x * 4 + wave_) * 8;
    unsigned hw = 0, xcc = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    o[0] = st_t0;
    o[1] = __builtin_amdgcn_s_memtime();
    o[2] = st_copy;
    o[3] = st_wait;
    o[4] = hw;
    o[5] = xcc & 15;
    o[6] = (uint64_t)nvis_;
    o[7] = blockIdx.x;
  };
#endif
  if (blockIdx.x < a.split_blocks) {  // block-uniform
    if (a.split_P == 4) wave_split_block<2, 4, false, true, GOTOH, true>(a, smem, lane);
    else wave_split_block<4, 2, false, true, GOTOH, true>(a, smem, lane);
    return;
  }
  if (a.tail_pairs) {  // the segmented tail: blocks after the main ones, one unit per wave
    const unsigned mb = (a.main_pairs + 7) / 8;
    if (blockIdx.x >= a.split_blocks + mb) {
      const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      const unsigned u = (blockIdx.x - a.split_blocks - mb) * 4 + wave;
      // the tail waves are the youngest on their SIMDs: without the top priority the SIMD's
      // oldest-first issue starves their segment chain behind the main waves
      if (SWK_TAIL_TOP) __builtin_amdgcn_s_setprio(3);
      if (u < a.tail_pairs * a.split_P)
        wave_tail_seg<GOTOH>(a, prof + (size_t)wave * a.split_words * 4, lane, u);
      return;
    }
  }
  if constexpr (SWK_HALF_FMA) {
    // the K = 8 profile (2-byte entries, PS = 1024 bytes per letter) as words {s, 1.0}, 2048
    // bytes per letter: row r = 16 l + 4 q + j (lane l of a half, piece q, word j) at word
    // 128 q + 4 l + j, so lane l reads its 16 rows as 4 x 16 bytes, 512 apart
    // (16-byte loads of 8 entries, rows 8 m .. 8 m + 7 of a letter = pieces q, q + 1 of lane
    // l: two 16-byte LDS stores; the loads of a thread's iterations are independent)
    const uint32_t groups = (a.pad + 1) * 64;
    const uint4* src = reinterpret_cast<const uint4*>(a.qtab);
    uint4* dst = reinterpret_cast<uint4*>(prof + (SWK_HALF_ABS ? SWK_HALF_ABS_BASE : 0u));
    const auto widen = [](uint32_t x) {  // two entries -> two {s, 1.0} words
      return make_uint2((x & 0xFFFFu) | 0x3C000000u, (x >> 16) | 0x3C000000u);
    };
#pragma unroll 4
    for (uint32_t i = threadIdx.x; i < groups; i += blockDim.x) {
      const uint4 v = src[i];
      const uint32_t r = (i & 63u) * 8;  // first row of the group
      const uint32_t w = (i & ~63u) * 8 | ((r >> 2) & 3u) << 7 | (r >> 4) << 2;  // word index
      const uint2 a0 = widen(v.x), a1 = widen(v.y), a2 = widen(v.z), a3 = widen(v.w);
      dst[w / 4] = make_uint4(a0.x, a0.y, a1.x, a1.y);            // rows r .. r + 3
      dst[w / 4 + 32] = make_uint4(a2.x, a2.y, a3.x, a3.y);       // rows r + 4 .. r + 7
    }
    __syncthreads();
#if SWK_STAMPS
    st_copy = __builtin_amdgcn_s_memtime();
#endif
  } else {  // the K = 8 profile (64 16-byte row groups per letter, PS = 1024) with group 2l + q
            // at 32 q + l: lane l of a half reads its rows 16 l .. 16 l + 15 as 16 + 16 bytes,
            // 512 apart
    const uint32_t words = (a.pad + 1) * a.PS / 16;
    const uint4* src = reinterpret_cast<const uint4*>(a.qtab);
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x)
      reinterpret_cast<uint4*>(prof)[(i & ~63u) | (i & 1u) << 5 | (i & 63u) >> 1] = src[i];
    __syncthreads();
  }
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // (SWK_HALF_ABS: wave 0's ring at byte 0, the profile from SWK_HALF_ABS_BASE = one ring on)
  uint8_t* mprof = prof + (SWK_HALF_ABS ? SWK_HALF_ABS_BASE : 0u);
  uint8_t* cring = SWK_HALF_ABS && wave == 0
                       ? prof
                       : mprof + (a.pad + 1) * SWK_HALF_LS + SWK_HALF_RING * (wave - (SWK_HALF_ABS ? 1 : 0));
  // Balanced ranges (ScoreArgs.wbal_blocks): wave g of the G resident waves scores
  // blocks [A_g, A_g+1) of the unit-major sequence of 32-step blocks, A_g = g U B / G (U units
  // of two pairs, B blocks each), so every wave slot gets the same number of steps whatever
  // U / G is -- the ScoreBank's answer to an uneven batch end is the first free module
  // (ScoreBank_v2.v:142-148,164-165); here no slot idles while another runs one unit more.  The
  // cut unit at the range end is scored first (the head, lane state out), the cut unit at the
  // range start last (the tail, after the predecessor's flag).  U >= G (host): a range holds at
  // least one unit, so a unit is cut at most once and every wait points to an earlier wave.
  // Without: one unit per wave.  One call site of wave_two_pairs for every visit (an inlined
  // copy per visit kind spills).
  const uint32_t G = gridDim.x * W,
                 g = __builtin_amdgcn_readfirstlane(blockIdx.x * W + (uint32_t)wave);
  uint32_t u0 = 0, u1 = 0, whole0 = 0;
  int b0 = 0, b1 = 0, nvis = 1;
  if (a.wbal_blocks) {
    const uint64_t U = ((uint64_t)a.main_pairs + 1) / 2, B = a.wbal_blocks, UB = U * B;
    const uint64_t A0 = UB * g / G, A1 = UB * (g + 1) / G;
    u0 = (uint32_t)(A0 / B);
    u1 = (uint32_t)(A1 / B);
    b0 = __builtin_amdgcn_readfirstlane((int)(A0 % B));
    b1 = __builtin_amdgcn_readfirstlane((int)(A1 % B));
    whole0 = b0 ? u0 + 1 : u0;  // whole units [whole0, u1)
    nvis = (b1 ? 1 : 0) + (int)(u1 - whole0) + (b0 ? 1 : 0);
  } else {
    whole0 = (blockIdx.x - a.split_blocks) * W + (uint32_t)wave;
    if (2 * (size_t)whole0 >= a.main_pairs || 4 * (size_t)whole0 >= a.n) return;  // whole wave
  }
  const size_t sw = (size_t)WBAL_WORDS * 64;
  for (int v = 0; v < nvis; ++v) {
    const bool head = b1 && v == 0, tail = b0 && v == nvis - 1;
    const uint32_t unit = __builtin_amdgcn_readfirstlane(
        head ? u1 : tail ? u0 : whole0 + (uint32_t)(v - (b1 ? 1 : 0)));
    if (tail) {  // wave g - 1's head is done (a bounded poll, as DESIGN §3.8)
#if SWK_STAMPS
      const uint64_t sw0 = __builtin_amdgcn_s_memtime();
#endif
      uint32_t it = 0;
      for (; it < a.poll_limit; ++it) {
        if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(
                a.bal_flag + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == a.bal_gen)
          break;
        __builtin_amdgcn_s_sleep(8);
      }
      if (it == a.poll_limit && lane == 0) report_fault(a.fault, SWK_FAULT_WBAL);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if SWK_STAMPS
      st_wait += __builtin_amdgcn_s_memtime() - sw0;
#endif
    }
    const uint2 b = wave_two_pairs<GOTOH>(
        a, mprof, cring, lane, 2 * (size_t)unit, tail ? 32 * b0 : 0, head ? 32 * b1 : 0x7FFFFFFF,
        tail ? a.bal_state + (size_t)g * sw : nullptr,
        head ? a.bal_state + (size_t)(g + 1) * sw : nullptr);
    if (head) {  // the lane state is out: wave g + 1 may take the unit on
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0 && g + 1 != a.stall)  // (stall: a test hook)
        __hip_atomic_store(a.bal_flag + g + 1, a.bal_gen, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else {
      wave_half_finish<GOTOH>(a, b, lane, 2 * (size_t)unit);
    }
  }
#if SWK_STAMPS
  stamp_out(wave, nvis);
#endif
}

// The end of a two-pairs unit: a pair above the optimistic f16 threshold is re-scored in u16 by
// the whole wave (K = 8, rare), then each half's lane 0 writes its pair's two scores.
template <bool GOTOH>
__device__ __forceinline__ void wave_half_finish(const ScoreArgs& a, uint2 b, int lane,
                                                 size_t p0) {
  const size_t n = a.n;
  if (a.fb_qtab) {  // optimistic f16: re-score a flagged pair in u16 (whole wave, K = 8)
    const uint32_t m0 = __builtin_amdgcn_readlane(max(b.x, b.y), 0);
    const uint32_t m1 = __builtin_amdgcn_readlane(max(b.x, b.y), 32);
    const uint8_t* fp = reinterpret_cast<const uint8_t*>(a.fb_qtab);
    uint2 f0 = make_uint2(0u, 0u), f1 = make_uint2(0u, 0u);
    if ((int32_t)m0 > a.fb_thresh)
      f0 = wave_pair<8, false, true, GOTOH, false>(a, fp, a.fb_qtab, a.fb_nv, a.fb_PS, p0, lane);
    if ((int32_t)m1 > a.fb_thresh && p0 + 1 < a.main_pairs)
      f1 = wave_pair<8, false, true, GOTOH, false>(a, fp, a.fb_qtab, a.fb_nv, a.fb_PS, p0 + 1,
                                                   lane);
    if ((int32_t)m0 > a.fb_thresh && lane < 32) b = f0;
    if ((int32_t)m1 > a.fb_thresh && lane >= 32) b = f1;
  }
  if ((lane & 31) == 0) {
    const size_t pair = p0 + (size_t)(lane >> 5);
    const size_t tA = 2 * pair, tB = tA + 1;
    if (pair < a.main_pairs && tA < n) {
      a.scores[tA] = (int32_t)b.x;
      if (tB < n) a.scores[tB] = (int32_t)b.y;
    }
  }
}


// the main blocks' LDS: the profile (prof_bytes at PS = 1024: 2 bytes per letter and row;
// SWK_HALF_FMA: 4) + each wave's code rings
static size_t wave_half_lds(uint32_t prof_bytes, int W) {
  return (size_t)prof_bytes / 1024 * SWK_HALF_LS + SWK_HALF_RING * (size_t)W;
}

template <bool GOTOH, int W>
static hipError_t launch_wave_half(const ScoreArgs& a, uint32_t prof_bytes, hipStream_t st) {
  // 4 waves per block = 8 pairs, sharing one LDS copy of the profile; the split tail's blocks
  // hold every segment's profile
  // (W = 8: balanced launches only, which have no split or segmented tail)
  if (W != 4 && !a.wbal_blocks) return hipErrorInvalidValue;
  const size_t blocks = a.wbal_blocks ? (size_t)a.wbal_grid
                                      : a.split_blocks + ((size_t)a.main_pairs + 7) / 8 +
                                            ((size_t)a.tail_pairs * a.split_P + 3) / 4;
  size_t lds = wave_half_lds(prof_bytes, W);
  if (a.split_blocks) lds = std::max<size_t>(lds, (size_t)a.split_words * 4 * a.split_P);
  if (a.tail_pairs) lds = std::max<size_t>(lds, (size_t)a.split_words * 4 * 4);  // a slice a wave
  auto fn = &score_wave_half<GOTOH, W>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    // SWK_HALF_ABS: the ring entries are LDS addresses counted from 0, which holds only while
    // the kernel has no static LDS (its dynamic LDS then starts at 0)
    hipFuncAttributes fa;
    e = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(fn));
    if (e != hipSuccess) return e;
    if (SWK_HALF_ABS && fa.sharedSizeBytes != 0) return hipErrorInvalidConfiguration;
    attr_set = true;
  }
  if (lds > 160 * 1024) return hipErrorInvalidConfiguration;
#if SWK_STAMPS
  if (g_stamps_host) {  // (measurement builds) the record buffer in tctr, unused here
    ScoreArgs b = a;
    b.tctr = reinterpret_cast<uint32_t*>(g_stamps_host);
    hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(64 * W), (unsigned)lds, st, b);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(64 * W), (unsigned)lds, st, a);
  return hipGetLastError();
}

}  // namespace swk

// Resident W-wave blocks of the two-pairs kernel (the balanced grid) for a profile of
// prof_bytes at PS = 1024 (0 when the occupancy query fails); W = 4 or 8.
extern "C" unsigned swk_wave_half_grid(int gotoh, uint32_t prof_bytes, int W) {
  const void* fn =
      W == 8 ? (gotoh ? reinterpret_cast<const void*>(&swk::score_wave_half<true, 8>)
                      : reinterpret_cast<const void*>(&swk::score_wave_half<false, 8>))
             : (gotoh ? reinterpret_cast<const void*>(&swk::score_wave_half<true, 4>)
                      : reinterpret_cast<const void*>(&swk::score_wave_half<false, 4>));
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
      hipSuccess)
    return 0;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  const int occ = swk::cached_occupancy(fn, 64 * W, swk::wave_half_lds(prof_bytes, W), dev, &cus);
  return occ > 0 && cus > 0 ? (unsigned)(occ * cus) : 0u;
}

// (K, COL0, PROF, GOTOH) x {u16, f16}
#define SWK_WAVE_VARIANTS(X)                                                              \
  X(4, 0, 0, 0) X(4, 1, 0, 0) X(4, 0, 0, 1) X(4, 0, 1, 0) X(4, 1, 1, 0) X(4, 0, 1, 1)     \
  X(8, 0, 0, 0) X(8, 1, 0, 0) X(8, 0, 0, 1) X(8, 0, 1, 0) X(8, 1, 1, 0) X(8, 0, 1, 1)     \
  X(16, 0, 0, 0) X(16, 1, 0, 0) X(16, 0, 0, 1) X(16, 0, 1, 0) X(16, 1, 1, 0) X(16, 0, 1, 1)

extern "C" hipError_t swk_launch_wave(int K, int col0, int prof, int gotoh, int f16,
                                      const void* edge_in, void* edge_out, uint32_t ecols,
                                      int accum, const uint8_t* res,
                                      const uint64_t* offs, const uint32_t* lens, size_t n,
                                      const uint32_t* qtab, uint32_t nv, uint32_t S, uint32_t O,
                                      uint32_t E, uint32_t PS, uint32_t pad, int32_t* scores,
                                      int packed, const uint32_t* fb_qtab, uint32_t fb_nv,
                                      uint32_t fb_PS, int32_t fb_thresh,
                                      const SwkWaveSplit* split, uint32_t ulen,
                                      uint32_t ustride, int half, hipStream_t st) {
  if (n == 0) return hipSuccess;
  swk::ScoreArgs a{res, offs, lens, n, qtab, nv, S, O, E, PS, pad, scores,
                   static_cast<const uint2*>(edge_in), static_cast<uint2*>(edge_out), ecols,
                   (uint32_t)accum, (uint32_t)packed, nullptr, nullptr, 0u, nullptr, 0u, 0u,
                   swk::f16_pair(-(int)(O + E)), swk::f16_pair(-(int)E),
                   swk::f16_pair(-(int)O), fb_qtab, fb_nv, fb_PS, fb_thresh};
  a.ulen = ulen;
  a.ustride = ustride;
  const size_t pairs = (n + 1) / 2;
  a.main_pairs = (uint32_t)pairs;
  if (split && split->wbal_blocks > 0) {
    // balanced ranges of the two-pairs kernel (ScoreArgs.wbal_*): no split or tail
    if (!half || K != 8 || edge_in || edge_out || accum || split->pairs || !split->wbal_grid ||
        !split->wbal_flag || !split->wbal_state || !split->fault || split->poll_limit == 0 ||
        (split->wbal_waves != 4 && split->wbal_waves != 8) || pairs > 0xFFFFFFFFull ||
        // every range at least 4 blocks: U B >= 4 G (a unit may be cut more than once)
        (pairs + 1) / 2 * split->wbal_blocks < 4ull * split->wbal_waves * split->wbal_grid)
      return hipErrorInvalidValue;
    a.wbal_blocks = split->wbal_blocks;
    a.wbal_grid = split->wbal_grid;
    a.bal_flag = split->wbal_flag;
    a.bal_state = split->wbal_state;
    a.bal_gen = split->wbal_gen;
    a.fault = split->fault;
    a.poll_limit = split->poll_limit;
    a.stall = split->stall;
  } else if (split && split->pairs > 0 && split->P == 8) {
    // the segmented tail of the two-pairs kernel (ScoreArgs.tail_*)
    if (!half || K != 8 || edge_in || edge_out || accum || split->pairs > pairs ||
        pairs > 0xFFFFFFFFull || !split->prog || split->cols == 0 || !split->fault ||
        split->poll_limit == 0)
      return hipErrorInvalidValue;
    a.split_P = 8;
    a.fault = split->fault;
    a.poll_limit = split->poll_limit;
    a.stall = split->stall;
    a.tail_pairs = split->pairs;
    a.tail_cols = split->cols;
    a.tail_prog = split->prog;
    a.main_pairs = (uint32_t)(pairs - split->pairs);
    a.split_qtab = split->qtab;
    a.split_words = split->words;
    a.split_PS = split->PS;
    a.split_ring = static_cast<uint2*>(split->ring);
  } else if (split && split->pairs > 0) {
    // the split tail is the last split->pairs pairs (K >= 8, one segment); with an odd count
    // the last block's second pair lies past the batch end
    if (K < 8 || edge_in || edge_out || accum || split->pairs > pairs || pairs > 0xFFFFFFFFull ||
        (split->P != 2 && split->P != 4))
      return hipErrorInvalidValue;
    a.split_P = split->P;
    a.split_blocks = (split->pairs + 4 / split->P - 1) / (4 / split->P);
    a.main_pairs = (uint32_t)(pairs - split->pairs);
    a.split_qtab = split->qtab;
    a.split_fb_qtab = split->fb_qtab;
    a.split_words = split->words;
    a.split_fb_words = split->fb_words;
    a.split_PS = split->PS;
    a.split_fb_PS = split->fb_PS;
    a.split_ring = static_cast<uint2*>(split->ring);
  }
  const uint32_t prof_bytes = (pad + 1) * PS;
  // two pairs per wave: f16 profile, K = 8 tables (a <= 512-row query), one segment
  if (half) {
    if (K != 8 || PS != 1024 || col0 || !prof || !f16 || edge_in || edge_out || accum)
      return hipErrorInvalidValue;
    if (a.wbal_blocks && split->wbal_waves == 8)
      return gotoh ? swk::launch_wave_half<true, 8>(a, prof_bytes, st)
                   : swk::launch_wave_half<false, 8>(a, prof_bytes, st);
    return gotoh ? swk::launch_wave_half<true, 4>(a, prof_bytes, st)
                 : swk::launch_wave_half<false, 4>(a, prof_bytes, st);
  }
#define SWK_WCASE(KK, C0, PF, GT)                                                         \
  if (K == KK && col0 == C0 && prof == PF && gotoh == GT)                                 \
    return f16 ? swk::launch_wave<KK, (C0 != 0), (PF != 0), (GT != 0), true>(a, prof_bytes, st) \
               : swk::launch_wave<KK, (C0 != 0), (PF != 0), (GT != 0), false>(a, prof_bytes, st);
  SWK_WAVE_VARIANTS(SWK_WCASE)
#undef SWK_WCASE
  return hipErrorInvalidValue;
}

