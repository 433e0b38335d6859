// swbank_kcommon.h — the gfx950 kernels' shared part (internal): build settings, the
// kernel argument block, the column recurrences and lookups both kernel families use,
// the occupancy helpers.  Kernels: swbank_ktile.hip (tile kernel), swbank_kwave.hip
// (wave kernels), swbank_kaux.hip (int32 re-score, length sort, best hit, deal).
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
#ifndef SWBANK_KCOMMON_H
#define SWBANK_KCOMMON_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <type_traits>
#include <vector>

#include "swbank_internal.h"

#ifndef SWK_TAIL_TOP
#define SWK_TAIL_TOP 1
#endif
#ifndef SWK_PRIO_ROT
// Rotating wave priorities in the persistent tile kernel: the SIMD issues from the oldest ready
// wave first, so of the 4 resident workgroups of a CU the first dispatched ran ahead and
// finished at 37 % of the kernel, and the last one ran alone on its CU for the final 22 %
// (stamps).  Each workgroup takes priority (time / 2^SWK_PRIO_SHIFT + q) mod 4, q its
// quarter of the grid (the dispatcher puts block i, i + CUs, ... on one CU), so every resident
// workgroup holds each priority level for the same share of time.  Period: 2^18 s_memtime
// ticks (~0.11 ms, ~10 phases of the headline), 2^15 over the last 1/16 of a workgroup's
// phases (+0.1-1.2 %, so the four finish closer); measured 2^14..2^22.  (The
// two-pairs protein kernel: -2 % with it, and within +-0.5 % with its split-tail waves on top
// and the 3 main waves rotating over 3 levels: not used there.  Priorities from each
// workgroup's progress against its CU's others, published per phase: 0.2-2 % below.  16-wave
// workgroups with later pipeline stages on top: +0.2 %, not kept.)
#define SWK_PRIO_ROT 1
#endif
#ifndef SWK_PRIO_SHIFT
#define SWK_PRIO_SHIFT 18
#endif

#ifndef SWK_PRIO_END
#define SWK_PRIO_END 3  // the last 1/16 of a workgroup's phases rotate 8 times faster
#endif
#ifndef SWK_PRIO_END_FRAC
#define SWK_PRIO_END_FRAC 4
#endif

#ifndef SWK_STAMPS
#define SWK_STAMPS 0  // measurement builds: per-wave phase timing of the tile kernel (swk_set_stamps)
#endif

namespace swk {

#if SWK_PRIO_ROT
// (SWK_PRIO_ROT) the wave's issue priority for now: (time / 2^SWK_PRIO_SHIFT + q) mod 4, set when
// it changes (s_setprio takes an immediate)
__device__ __forceinline__ void prio_rotate(uint32_t q, uint32_t& prio, uint32_t shift) {
  const uint32_t pr = ((uint32_t)(__builtin_amdgcn_s_memtime() >> shift) + q) & 3u;
  if (pr != prio) {
    prio = pr;
    if (pr == 0) __builtin_amdgcn_s_setprio(0);
    else if (pr == 1) __builtin_amdgcn_s_setprio(1);
    else if (pr == 2) __builtin_amdgcn_s_setprio(2);
    else __builtin_amdgcn_s_setprio(3);
  }
}
#endif

#if SWK_STAMPS
inline uint64_t* g_stamps_host = nullptr;  // (one object across the kernel units)  // the buffer launch_score hands the tile kernel
#endif
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ u16x2 vmax(u16x2 a, u16x2 b) { return __builtin_elementwise_max(a, b); }
__device__ __forceinline__ u16x2 vsubs(u16x2 a, u16x2 b) {
  return __builtin_elementwise_sub_sat(a, b);
}



// ---- substitution lookup: p = S - s(q_row, t) for both targets of the lane --------------
// LUT mode (DNA): the row's query letter is wave-uniform, its 4-entry row of (S - s) is one
// SGPR; codes 4..7 (N and padding) read `nv`.  One v_perm_b32 per row.
template <int R>
struct LutLookup {
  const uint32_t (&tab)[R];
  uint32_t nv, selw;
  __device__ __forceinline__ u16x2 operator()(int r) const {
    return as_u16x2(__builtin_amdgcn_perm(nv, tab[r], selw));
  }
};
// Profile mode (any alphabet): per column each lane reads the wave's R profile bytes for its
// two target letters from LDS (query profile QP[letter][row]); one v_perm_b32 per row
// interleaves them into the two u16 halves.
template <int R>
struct ProfLookup {
  uint32_t lo[R / 4], hi[R / 4];
  __device__ __forceinline__ u16x2 operator()(int r) const {
    const uint32_t sel = (uint32_t)(r & 3) | ((uint32_t)(4 + (r & 3)) << 16) | 0x0C000C00u;
    return as_u16x2(__builtin_amdgcn_perm(hi[r >> 2], lo[r >> 2], sel));
  }
};

// f16 profile mode: 2-byte entries (the f16 bits of s); word k of lo/hi holds rows 2k, 2k+1 of
// the lane's low/high target letter; one v_perm_b32 per row picks the row's two halves.
template <int R>
struct ProfLookup16 {
  uint32_t lo[R / 2], hi[R / 2];
  __device__ __forceinline__ u16x2 operator()(int r) const {
    const uint32_t k = (uint32_t)(r & 1) * 2;
    const uint32_t sel = k | ((k + 1) << 8) | ((k + 4) << 16) | ((k + 5) << 24);
    return as_u16x2(__builtin_amdgcn_perm(hi[r >> 1], lo[r >> 1], sel));
  }
};

// ---- one column of R rows, merged gap matrix (the ScoreBank PE) --------------------------
// ZDOWN: HDL column-0 rule (G passed down = 0).  RB: rows per scheduling group (a
// sched_barrier every RB rows bounds how far the scheduler may defer the H/best updates
// behind the G chain, i.e. register pressure).
template <int R, int RB, bool ZDOWN, class LK>
__device__ __forceinline__ void column_merged(const LK& lk, u16x2& diag, u16x2& upG,
                                              u16x2 (&Hl)[R], u16x2 (&Gl)[R], u16x2& best,
                                              u16x2 S2, u16x2 O2, u16x2 E2) {
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
    upG = ZDOWN ? (u16x2){0, 0} : Gn;
    if ((r % RB) == RB - 1) __builtin_amdgcn_sched_barrier(0);
  }
}

// ---- one column of R rows, merged gap matrix, f16 arithmetic ------------------------------
// Exact for integer scores |x| <= 2048 (the host routes a batch here only when the score
// bound allows it, and when every substitution score is an f16 whose low byte is 0, so a
// one-byte LUT entry is its high byte).  Signed arithmetic needs no shift, and
// v_pk_maximum3_f16 takes three inputs.  Scores are stored as f16 multiples of 2^-11 (x as
// x/2048): every integer |x| <= 2048 is then an exact normal f16 (or 0), and the [0, 1] clamp
// modifier of v_pk_add_f16 is max(0, x) for free -- the asm columns (scripts/gen_f16_rows.py)
// use it to form M = max(0, H(i-1,j-1) + s) in the diagonal add.  The C++ form below:
//   D = H(i-1,j-1) + s      I = max(Tup, Tleft)      H = max(0, D, I)
//   T = max(-o-e, D-o-e, I-e)  (= G - e, the gap value the right and lower neighbours see)
// 8 VALU per lane per 2 cells (u16 form: 9).  Negative values never reach a positive one.
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f16x2 as_f16x2(u16x2 x) { return __builtin_bit_cast(f16x2, x); }
__device__ __forceinline__ u16x2 as_u16x2(f16x2 x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ f16x2 fmax2(f16x2 a, f16x2 b) {
  return __builtin_elementwise_maximum(a, b);
}
// integer score <-> its f16 encoding (x / 2048); f16_pair: both halves (host side, ScoreArgs)
__host__ __device__ inline uint32_t f16_pair(int x) {
  const uint16_t h = __builtin_bit_cast(uint16_t, (_Float16)((float)x * (1.0f / 2048.0f)));
  return (uint32_t)h * 0x10001u;
}
__device__ __forceinline__ int32_t f16_unscore(uint32_t bits) {
  return (int32_t)((float)__builtin_bit_cast(_Float16, (unsigned short)bits) * 2048.0f);
}
template <int R, int RB, bool ZDOWN, class LK>
__device__ __forceinline__ void column_merged_f16(const LK& lk, u16x2& diag_, u16x2& upT_,
                                                  u16x2 (&Hl)[R], u16x2 (&Tl)[R], u16x2& best_,
                                                  f16x2 NOE2, f16x2 NE2) {
  f16x2 diag = as_f16x2(diag_), upT = as_f16x2(upT_), best = as_f16x2(best_);
  const f16x2 Z = {(_Float16)0, (_Float16)0};
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const f16x2 sc = as_f16x2(lk(r));
    const f16x2 D = diag + sc;
    const f16x2 I = fmax2(upT, as_f16x2(Tl[r]));
    const f16x2 H = fmax2(fmax2(D, Z), I);
    const f16x2 T = fmax2(fmax2(D + NOE2, NOE2), I + NE2);
    best = fmax2(best, H);
    diag = as_f16x2(Hl[r]);
    Hl[r] = as_u16x2(H);
    Tl[r] = as_u16x2(T);
    upT = ZDOWN ? NOE2 : T;
    if ((r % RB) == RB - 1) __builtin_amdgcn_sched_barrier(0);
  }
  diag_ = as_u16x2(diag);
  upT_ = as_u16x2(upT);
  best_ = as_u16x2(best);
}

// Gotoh in f16.  E and F are kept one step ahead ("what the next cell reads") and floored at
// 0 (a non-positive gap value never reaches a positive H), so H needs one max3 and the
// H - o - e term is shared by both gap directions: 8.5 VALU per lane per 2 cells (u16: 11).
//   H = max(D, El, F)   HN = H - o - e   El = max(0, HN, El - e)   F = max(0, HN, F - e)
template <int R, int RB, class LK>
__device__ __forceinline__ void column_gotoh_f16(const LK& lk, u16x2& diag_, u16x2& upF_,
                                                 u16x2 (&Hl)[R], u16x2 (&El)[R], u16x2& best_,
                                                 f16x2 NOE2, f16x2 NE2) {
  f16x2 diag = as_f16x2(diag_), F = as_f16x2(upF_), best = as_f16x2(best_);
  const f16x2 Z = {(_Float16)0, (_Float16)0};
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const f16x2 D = diag + as_f16x2(lk(r));
    const f16x2 E = as_f16x2(El[r]);
    const f16x2 H = fmax2(fmax2(D, E), F);
    const f16x2 HN = H + NOE2;
    best = fmax2(best, H);
    diag = as_f16x2(Hl[r]);
    Hl[r] = as_u16x2(H);
    El[r] = as_u16x2(fmax2(fmax2(HN, Z), E + NE2));
    F = fmax2(fmax2(HN, Z), F + NE2);
    if ((r % RB) == RB - 1) __builtin_amdgcn_sched_barrier(0);
  }
  upF_ = as_u16x2(F);
  best_ = as_u16x2(best);
}

// The f16 columns are normally run as hand-ordered asm (column_f16_asm below): LLVM's order
// of these chains leaves ~2.5 s_nop per row (gfx950 needs a wait state between a VOP3P write
// and a dependent VOP3P read); the generated order needs none.  SWK_F16_ASM=0 builds the
// compiler-scheduled C++ forms above instead (A/B and debugging).
#ifndef SWK_F16_ASM
#define SWK_F16_ASM 1
#endif
#ifndef SWK_F16_COLBLOCK
#define SWK_F16_COLBLOCK 1
#endif
#include "swbank_f16_rows.inc"
#define SWK_F16_HT(B)                                                                         \
  [h0] "+v"(Hl[B]), [h1] "+v"(Hl[B + 1]), [h2] "+v"(Hl[B + 2]), [h3] "+v"(Hl[B + 3]),          \
      [h4] "+v"(Hl[B + 4]), [h5] "+v"(Hl[B + 5]), [h6] "+v"(Hl[B + 6]), [h7] "+v"(Hl[B + 7]),  \
      [t0] "+v"(Xl[B]), [t1] "+v"(Xl[B + 1]), [t2] "+v"(Xl[B + 2]), [t3] "+v"(Xl[B + 3]),      \
      [t4] "+v"(Xl[B + 4]), [t5] "+v"(Xl[B + 5]), [t6] "+v"(Xl[B + 6]), [t7] "+v"(Xl[B + 7]),  \
      [Da] "+v"(Da), [Db] "=&v"(Db), [S1] "=&v"(S1), [best] "+v"(best)
#define SWK_F16_OUT_M(B) SWK_F16_HT(B), [X] "=&v"(X), [DN] "=&v"(DN), [IN] "=&v"(IN)
#define SWK_F16_OUT_G(B) SWK_F16_HT(B), [EN] "=&v"(X), [HN] "=&v"(DN), [FN] "=&v"(IN), [F] "+v"(up)
#define SWK_F16_IN_L(B)                                                                       \
  [nv] "v"(lk.nv), [sel] "v"(lk.selw), [noe] "s"(noe), [ne] "s"(ne), [no] "s"(no), [up] "v"(up),            \
      [tb0] "s"(lk.tab[B + 1]), [tb1] "s"(lk.tab[B + 2]), [tb2] "s"(lk.tab[B + 3]),           \
      [tb3] "s"(lk.tab[B + 4]), [tb4] "s"(lk.tab[B + 5]), [tb5] "s"(lk.tab[B + 6]),           \
      [tb6] "s"(lk.tab[B + 7]), [tb7] "s"(lk.tab[(B + 8) < R ? B + 8 : R - 1])
#define SWK_F16_IN_P(B)                                                                       \
  [noe] "s"(noe), [ne] "s"(ne), [no] "s"(no), [up] "v"(up), [selA] "s"(0x05040100u), [selB] "s"(0x07060302u), \
      [lo0] "v"(lk.lo[B / 2]), [lo1] "v"(lk.lo[B / 2 + 1]), [lo2] "v"(lk.lo[B / 2 + 2]),       \
      [lo3] "v"(lk.lo[B / 2 + 3]), [lo4] "v"(lk.lo[(B + 8) < R ? B / 2 + 4 : B / 2 + 3]),      \
      [hi0] "v"(lk.hi[B / 2]), [hi1] "v"(lk.hi[B / 2 + 1]), [hi2] "v"(lk.hi[B / 2 + 2]),       \
      [hi3] "v"(lk.hi[B / 2 + 3]), [hi4] "v"(lk.hi[(B + 8) < R ? B / 2 + 4 : B / 2 + 3])
// The gotoh macros have no [up]/[X]/... in their text; unused operands are harmless.
#define SWK_F16_IN_LG(B)                                                                      \
  [nv] "v"(lk.nv), [sel] "v"(lk.selw), [noe] "s"(noe), [ne] "s"(ne),                          \
      [tb0] "s"(lk.tab[B + 1]), [tb1] "s"(lk.tab[B + 2]), [tb2] "s"(lk.tab[B + 3]),           \
      [tb3] "s"(lk.tab[B + 4]), [tb4] "s"(lk.tab[B + 5]), [tb5] "s"(lk.tab[B + 6]),           \
      [tb6] "s"(lk.tab[B + 7]), [tb7] "s"(lk.tab[(B + 8) < R ? B + 8 : R - 1])
#define SWK_F16_IN_PG(B)                                                                      \
  [noe] "s"(noe), [ne] "s"(ne), [selA] "s"(0x05040100u), [selB] "s"(0x07060302u),            \
      [lo0] "v"(lk.lo[B / 2]), [lo1] "v"(lk.lo[B / 2 + 1]), [lo2] "v"(lk.lo[B / 2 + 2]),       \
      [lo3] "v"(lk.lo[B / 2 + 3]), [lo4] "v"(lk.lo[(B + 8) < R ? B / 2 + 4 : B / 2 + 3]),      \
      [hi0] "v"(lk.hi[B / 2]), [hi1] "v"(lk.hi[B / 2 + 1]), [hi2] "v"(lk.hi[B / 2 + 2]),       \
      [hi3] "v"(lk.hi[B / 2 + 3]), [hi4] "v"(lk.hi[(B + 8) < R ? B / 2 + 4 : B / 2 + 3])

// One f16 column, hand-ordered asm in 8-row blocks (scripts/gen_f16_rows.py).  LK is
// LutLookup<R> (DNA, row LUT words in SGPRs) or ProfLookup16<R> (2-byte profile words).
// Merged: Xl = T (= G - e), upX = T passed down.  Gotoh: Xl = E, upX = F of the next row.
template <int R, bool GOTOH, bool ZDOWN, class LK>
__device__ __forceinline__ void column_f16_asm(const LK& lk, u16x2& diag_, u16x2& upX_,
                                               u16x2 (&Hl)[R], u16x2 (&Xl)[R], u16x2& best_,
                                               uint32_t noe, uint32_t ne, uint32_t no) {
  static_assert(R % 8 == 0, "rows come in blocks of 8");
  constexpr bool PROF = !std::is_same<LK, LutLookup<R>>::value;
  uint32_t Da, Db, S1, X, DN, IN;
  u16x2 best = best_, up = upX_;
#if SWK_F16_COLBLOCK
  if constexpr ((R == 32 || R == 16) && !GOTOH && !PROF && !ZDOWN) {
    // DNA LUT merged (the headline): the whole column (prologue + R rows) as one asm block
#define SWK_F16_COLASM(RR)                                                                    \
    asm volatile(                                                                             \
        "v_perm_b32 %[Da], %[nv], %[tz], %[sel]\n\t"                                          \
        "v_pk_add_f16 %[Da], %[dg], %[Da] clamp\n\t" SWK_F16M_L_Z0_COL##RR                          \
        : SWK_F16_COL##RR##_HT, [Da] "=&v"(Da), [Db] "=&v"(Db), [S1] "=&v"(S1), [X] "=&v"(X), \
          [DN] "=&v"(DN), [IN] "=&v"(IN), [best] "+v"(best)                                  \
        : [nv] "v"(lk.nv), [sel] "v"(lk.selw), [noe] "s"(noe), [ne] "s"(ne), [no] "s"(no), [up] "v"(up),     \
          [tz] "s"(lk.tab[0]), [dg] "v"(diag_), SWK_F16_COL##RR##_TB)
    if constexpr (R == 32) SWK_F16_COLASM(32);
    else SWK_F16_COLASM(16);
#undef SWK_F16_COLASM
    (void)Db; (void)S1; (void)X; (void)DN; (void)IN;
    upX_ = Xl[R - 1];
    best_ = best;
    return;
  }
#endif
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
        : [nv] "v"(lk.nv), [t0] "s"(lk.tab[0]), [sel] "v"(lk.selw), [dg] "v"(diag_));
#pragma unroll
  for (int b = 0; b < R; b += 8) {
    const bool last = b + 8 >= R;
    if constexpr (GOTOH) {
      if constexpr (PROF) {
        if (last) asm volatile(SWK_F16G_P_L1 : SWK_F16_OUT_G(b) : SWK_F16_IN_PG(b));
        else      asm volatile(SWK_F16G_P_L0 : SWK_F16_OUT_G(b) : SWK_F16_IN_PG(b));
      } else {
        if (last) asm volatile(SWK_F16G_L_L1 : SWK_F16_OUT_G(b) : SWK_F16_IN_LG(b));
        else      asm volatile(SWK_F16G_L_L0 : SWK_F16_OUT_G(b) : SWK_F16_IN_LG(b));
      }
    } else {
      if constexpr (PROF) {
        if constexpr (ZDOWN) {
          if (last) asm volatile(SWK_F16M_P_Z1_L1 : SWK_F16_OUT_M(b) : SWK_F16_IN_P(b));
          else      asm volatile(SWK_F16M_P_Z1_L0 : SWK_F16_OUT_M(b) : SWK_F16_IN_P(b));
        } else {
          if (last) asm volatile(SWK_F16M_P_Z0_L1 : SWK_F16_OUT_M(b) : SWK_F16_IN_P(b));
          else      asm volatile(SWK_F16M_P_Z0_L0 : SWK_F16_OUT_M(b) : SWK_F16_IN_P(b));
        }
      } else {
        if constexpr (ZDOWN) {
          if (last) asm volatile(SWK_F16M_L_Z1_L1 : SWK_F16_OUT_M(b) : SWK_F16_IN_L(b));
          else      asm volatile(SWK_F16M_L_Z1_L0 : SWK_F16_OUT_M(b) : SWK_F16_IN_L(b));
        } else {
          if (last) asm volatile(SWK_F16M_L_Z0_L1 : SWK_F16_OUT_M(b) : SWK_F16_IN_L(b));
          else      asm volatile(SWK_F16M_L_Z0_L0 : SWK_F16_OUT_M(b) : SWK_F16_IN_L(b));
        }
      }
      up = ZDOWN ? as_u16x2(noe) : Xl[b + 7];
    }
  }
  (void)Db; (void)S1; (void)X; (void)DN; (void)IN;
  upX_ = up;
  best_ = best;
}

// f16 column: hand-ordered asm (default) or the compiler-scheduled C++ form (SWK_F16_ASM=0).
template <int R, int RB, bool GOTOH, bool ZDOWN, class LK>
__device__ __forceinline__ void column_f16(const LK& lk, u16x2& diag, u16x2& upX,
                                           u16x2 (&Hl)[R], u16x2 (&Xl)[R], u16x2& best,
                                           f16x2 NOE2, f16x2 NE2, f16x2 NO2) {
#if SWK_F16_ASM
  column_f16_asm<R, GOTOH, ZDOWN>(lk, diag, upX, Hl, Xl, best, as_u32(as_u16x2(NOE2)),
                                  as_u32(as_u16x2(NE2)), as_u32(as_u16x2(NO2)));
#else
  (void)NO2;
  if constexpr (GOTOH)
    column_gotoh_f16<R, RB>(lk, diag, upX, Hl, Xl, best, NOE2, NE2);
  else
    column_merged_f16<R, RB, ZDOWN>(lk, diag, upX, Hl, Xl, best, NOE2, NE2);
#endif
}

// ---- one column of R rows, Gotoh (separate E/F; ssearch36 semantics) ---------------------
//   E(i,j) = max(H(i,j-1) - o - e, E(i,j-1) - e)     F(i,j) = max(H(i-1,j) - o - e, F(i-1,j) - e)
//   H(i,j) = max(0, H(i-1,j-1) + s, E, F)            (E, F clamped at 0: exact, H >= 0)
// OES = o + e + S because stored H~ = H + S.  12 VALU per lane per 2 cells.
template <int R, int RB, class LK>
__device__ __forceinline__ void column_gotoh(const LK& lk, u16x2& diag, u16x2& upH, u16x2& upF,
                                             u16x2 (&Hl)[R], u16x2 (&El)[R], u16x2& best,
                                             u16x2 S2, u16x2 OES2, u16x2 E2) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const u16x2 p = lk(r);
    const u16x2 M = vsubs(diag, p);
    const u16x2 Ei = vmax(vsubs(Hl[r], OES2), vsubs(El[r], E2));
    const u16x2 Fi = vmax(vsubs(upH, OES2), vsubs(upF, E2));
    const u16x2 Hn = vmax(vmax(M, Ei), Fi) + S2;
    best = vmax(best, M);
    diag = Hl[r];
    Hl[r] = Hn;
    El[r] = Ei;
    upH = Hn;
    upF = Fi;
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
// end the code is `pad` (LUT mode: 4 = N, s(*, N) <= 0; profile mode: a row of S - s = 255),
// so padding can only lower a score.  `full` (uniform): every lane has >= 8 codes left in
// both targets -> two unaligned 8-byte loads.
// 8 two-bit codes (LSB-first, charTo2bit order) -> 8 code bytes.
__device__ __forceinline__ uint2 unpack8(uint32_t b) {
  return make_uint2((b & 3u) | ((b << 6) & 0x300u) | ((b << 12) & 0x30000u) |
                        ((b << 18) & 0x3000000u),
                    ((b >> 8) & 3u) | ((b >> 2) & 0x300u) | ((b << 4) & 0x30000u) |
                        ((b << 10) & 0x3000000u));
}
// 8 four-bit codes (low nibble first) -> 8 code bytes: the nibbles of even and odd codes
// apart, then one v_perm per 4 codes interleaves them.
__device__ __forceinline__ uint2 unpack8n(uint32_t x) {
  const uint32_t lo = x & 0x0F0F0F0Fu, hi = (x >> 4) & 0x0F0F0F0Fu;
  return make_uint2(__builtin_amdgcn_perm(hi, lo, 0x05010400u),
                    __builtin_amdgcn_perm(hi, lo, 0x07030602u));
}
// Past-the-end codes of a chunk -> pad (bytes k with j0 + k >= len).
__device__ __forceinline__ uint2 pad_tail(uint2 w, uint32_t j0, uint32_t len, uint32_t pad) {
  const uint32_t n = len > j0 ? min(len - j0, 8u) : 0u;  // valid codes in this chunk
  const uint64_t keep = n >= 8 ? ~0ull : ((1ull << (8 * n)) - 1);
  const uint64_t v = ((uint64_t)w.y << 32 | w.x) & keep;
  const uint64_t p = (pad * 0x0101010101010101ull) & ~keep;
  return make_uint2((uint32_t)(v | p), (uint32_t)((v | p) >> 32));
}

// Loads at arbitrary byte offsets (target starts in the packed streams and records are not
// aligned): memcpy tells the compiler the alignment is 1; gfx950 global loads accept any
// alignment, so they stay single dword / dwordx2 loads.
template <class T>
__device__ __forceinline__ T load_u(const uint8_t* p) {
  T v;
  __builtin_memcpy(&v, p, sizeof(T));
  return v;
}
// CAPI record length, clamped to the record capacity (a corrupt length cannot send a lane past
// the 58-byte data field)
__device__ __forceinline__ uint32_t record_len(const uint8_t* rec) {
  return min((uint32_t)load_u<uint16_t>(rec + 4), SWB_RECORD_MAX);
}

// SWK_PACK_MIXED: the target's u32 offset word o is (byte << 1) | 1 for 4-bit codes and
// position << 1 for 2-bit codes, `position` counting 2-bit codes from res (targets packed back
// to back as one run start inside a byte).  Lane2 keeps the format in the pointer's top bits:
// bit 63 = 4-bit, bits 61-62 = the 2-bit start inside its byte (device addresses are < 2^57).
constexpr uint64_t SWK_MIX_NIB = 1ull << 63;
constexpr uint64_t SWK_MIX_ADDR = (1ull << 61) - 1;
__device__ __forceinline__ const uint8_t* mixed_ptr(const uint8_t* res, uint32_t o) {
  const uint64_t p = reinterpret_cast<uint64_t>(res);
  return reinterpret_cast<const uint8_t*>(
      (o & 1u) ? (p + (o >> 1)) | SWK_MIX_NIB : (p + (o >> 3)) | (uint64_t)((o >> 1) & 3u) << 61);
}
// Codes of C-column chunk cl of a mixed target (C = 8: a 32-bit load, C = 4: 16 bits), 2-bit
// codes shifted down to the chunk's first; nib: the target is in 4-bit codes
template <int C>
__device__ __forceinline__ uint32_t mixed_word(const uint8_t* tp, uint32_t cl, bool& nib) {
  const uint64_t v = reinterpret_cast<uint64_t>(tp);
  nib = (v & SWK_MIX_NIB) != 0;
  const uint8_t* p = reinterpret_cast<const uint8_t*>(v & SWK_MIX_ADDR);
  if (nib) return C == 4 ? (uint32_t)load_u<uint16_t>(p + 2 * cl) : load_u<uint32_t>(p + 4 * cl);
  const uint32_t w = C == 4 ? (uint32_t)load_u<uint16_t>(p + cl) : load_u<uint32_t>(p + 2 * cl);
  return w >> (2u * (uint32_t)(v >> 61 & 3u));
}

// C = 4 (the 16-wave query-set kernel's 4-column chunks): codes [4c, 4c+4) in lo.x / hi.x.
__device__ __forceinline__ uint32_t pad_tail4(uint32_t w, uint32_t j0, uint32_t len, uint32_t pad) {
  const uint32_t n = len > j0 ? min(len - j0, 4u) : 0u;
  const uint32_t keep = n >= 4 ? ~0u : ((1u << (8 * n)) - 1);
  return (w & keep) | ((pad * 0x01010101u) & ~keep);
}

// MIX = false: the caller never passes SWK_PACK_MIXED (the query-set variants)
template <int C = 8, bool MIX = true>
__device__ __forceinline__ void load_raw(const Lane2& t, int c, bool full, uint32_t pad,
                                         uint32_t packed, uint2& lo, uint2& hi) {
  static_assert(C == 8 || C == 4, "chunks of 8 or 4 columns");
  if constexpr (C == 4) {
    const uint32_t j0 = (uint32_t)c * 4;
    uint32_t x, y;
    if (packed == SWK_PACK_NIBBLE) {  // 2 bytes per 4 codes, chunk clamped to the target's last
      const uint32_t cl = min((uint32_t)c, max((t.llo + 3) / 4, 1u) - 1);
      const uint32_t ch = min((uint32_t)c, max((t.lhi + 3) / 4, 1u) - 1);
      x = unpack8n(load_u<uint16_t>(t.plo + 2 * cl)).x;
      y = unpack8n(load_u<uint16_t>(t.phi + 2 * ch)).x;
    } else if (MIX && packed == SWK_PACK_MIXED) {  // per target: 4-bit at an odd address
      const uint32_t cl = min((uint32_t)c, max((t.llo + 3) / 4, 1u) - 1);
      const uint32_t ch = min((uint32_t)c, max((t.lhi + 3) / 4, 1u) - 1);
      bool nl, nh;  // (2-bit: 4 codes from bit 0-6 of a 16-bit load)
      const uint32_t wl = mixed_word<4>(t.plo, cl, nl);
      const uint32_t wh = mixed_word<4>(t.phi, ch, nh);
      x = nl ? unpack8n(wl).x : unpack8(wl).x;
      y = nh ? unpack8n(wh).x : unpack8(wh).x;
    } else if (packed) {  // 1 byte per 4 codes (records: inside the data field)
      uint32_t cl = (uint32_t)c, ch = (uint32_t)c;
      if (packed == SWK_PACK_STREAM) {
        cl = min(cl, max((t.llo + 3) / 4, 1u) - 1);
        ch = min(ch, max((t.lhi + 3) / 4, 1u) - 1);
      }
      x = unpack8(t.plo[cl]).x;
      y = unpack8(t.phi[ch]).x;
    } else if (full) {
      x = load_u<uint32_t>(t.plo + j0);
      y = load_u<uint32_t>(t.phi + j0);
    } else {
      uint32_t b[2][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // branch-free: clamped address, then select
        const uint32_t j = j0 + k;
        const uint32_t av = t.plo[j < t.llo ? j : 0];
        const uint32_t hv = t.phi[j < t.lhi ? j : 0];
        b[0][k] = j < t.llo ? av : pad;
        b[1][k] = j < t.lhi ? hv : pad;
      }
      x = b[0][0] | b[0][1] << 8 | b[0][2] << 16 | b[0][3] << 24;
      y = b[1][0] | b[1][1] << 8 | b[1][2] << 16 | b[1][3] << 24;
    }
    if (packed && !full) {
      x = pad_tail4(x, j0, t.llo, pad);
      y = pad_tail4(y, j0, t.lhi, pad);
    }
    lo = make_uint2(x, 0u);
    hi = make_uint2(y, 0u);
    return;
  }
  const uint32_t j0 = (uint32_t)c * 8;
  if (MIX && packed == SWK_PACK_MIXED) {  // per target: 4-bit at an odd address, else 2-bit
    // (a 2-bit chunk reads 4 bytes for its 2-3: the rest is the next target's or the 16 zero
    // bytes the host writes after the last)
    const uint32_t cl = min((uint32_t)c, max((t.llo + 7) / 8, 1u) - 1);
    const uint32_t ch = min((uint32_t)c, max((t.lhi + 7) / 8, 1u) - 1);
    bool nl, nh;
    const uint32_t wl = mixed_word<8>(t.plo, cl, nl);
    const uint32_t wh = mixed_word<8>(t.phi, ch, nh);
    lo = nl ? unpack8n(wl) : unpack8(wl);
    hi = nh ? unpack8n(wh) : unpack8(wh);
    if (!full) {
      lo = pad_tail(lo, j0, t.llo, pad);
      hi = pad_tail(hi, j0, t.lhi, pad);
    }
  } else if (packed == SWK_PACK_NIBBLE) {  // 4-bit stream, 4 bytes per 8 codes, clamped like below
    const uint32_t cl = min((uint32_t)c, max((t.llo + 7) / 8, 1u) - 1);
    const uint32_t ch = min((uint32_t)c, max((t.lhi + 7) / 8, 1u) - 1);
    lo = unpack8n(load_u<uint32_t>(t.plo + 4 * cl));
    hi = unpack8n(load_u<uint32_t>(t.phi + 4 * ch));
    if (!full) {
      lo = pad_tail(lo, j0, t.llo, pad);
      hi = pad_tail(hi, j0, t.lhi, pad);
    }
  } else if (packed) {  // 2-bit codes, 2 bytes per 8 codes
    // CAPI records: always inside the 58-byte data field; 2-bit stream: the chunk index is
    // clamped to the target's last chunk (an empty target reads 2 bytes at its dummy address;
    // a last chunk may read 1 byte past the target, which the host pads)
    uint32_t cl = (uint32_t)c, ch = (uint32_t)c;
    if (packed == SWK_PACK_STREAM) {
      cl = min(cl, max((t.llo + 7) / 8, 1u) - 1);
      ch = min(ch, max((t.lhi + 7) / 8, 1u) - 1);
    }
    const uint32_t x = load_u<uint16_t>(t.plo + 2 * cl);
    const uint32_t y = load_u<uint16_t>(t.phi + 2 * ch);
    lo = unpack8(x);
    hi = unpack8(y);
    if (!full) {
      lo = pad_tail(lo, j0, t.llo, pad);
      hi = pad_tail(hi, j0, t.lhi, pad);
    }
  } else if (full) {
    lo = load_u<uint2>(t.plo + j0);
    hi = load_u<uint2>(t.phi + j0);
  } else {
    uint32_t b[2][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // branch-free: clamped address, then select
      const uint32_t j = j0 + k;
      const uint32_t a = t.plo[j < t.llo ? j : 0];
      const uint32_t h = t.phi[j < t.lhi ? j : 0];
      b[0][k] = j < t.llo ? a : pad;
      b[1][k] = j < t.lhi ? h : pad;
    }
    lo.x = b[0][0] | b[0][1] << 8 | b[0][2] << 16 | b[0][3] << 24;
    lo.y = b[0][4] | b[0][5] << 8 | b[0][6] << 16 | b[0][7] << 24;
    hi.x = b[1][0] | b[1][1] << 8 | b[1][2] << 16 | b[1][3] << 24;
    hi.y = b[1][4] | b[1][5] << 8 | b[1][6] << 16 | b[1][7] << 24;
  }
}

// Per-tile metadata of one lane (uniform tile id).  packed: `res` is an array of 64-byte CAPI
// records {u32 ID, u16 length, u8 data[58]} (aligner_Header.h:19-24).
// idx (optional): position k of the batch is target idx[k] (the u16 re-score of the pairs an
// optimistic f16 pass flagged).
template <bool MIX = true>
__device__ __forceinline__ Lane2 lane_targets(const uint8_t* res, const uint64_t* offs,
                                              const uint32_t* lens, size_t n, int tile, int lane,
                                              uint32_t packed, const uint32_t* idx,
                                              uint32_t ulen, uint32_t ustride) {
  Lane2 t;
  size_t a = (size_t)tile * SWB_TILE + lane, b = a + 64;
  const bool va = a < n, vb = b < n;  // positions in the batch
  // A lane past the batch end reads the tile's first target (position tile*128 always
  // exists): its codes are discarded, but the full-chunk loads (8 bytes while every valid
  // lane has >= 8 codes left) must stay inside a real target.
  // A workgroup whose first tile lies past the batch end (the device-side count of an index
  // list can be far below the launch size) dereferences nothing but lens[0] / record 0.
  const size_t p0 = (size_t)tile * SWB_TILE;
  if (p0 >= n) {
    t.llo = t.lhi = 0u;
    t.plo = t.phi = packed == SWK_PACK_RECORDS || ustride ? res + (packed ? 6 : 0)
                                                          : reinterpret_cast<const uint8_t*>(lens);
    return t;
  }
  if (!va) a = p0;
  if (!vb) b = p0;
  if (idx) {
    a = idx[a];
    b = idx[b];
  }
  if (packed == SWK_PACK_RECORDS) {
    t.llo = va ? record_len(res + a * SWB_RECORD) : 0u;
    t.lhi = vb ? record_len(res + b * SWB_RECORD) : 0u;
    t.plo = res + a * SWB_RECORD + 6;
    t.phi = res + b * SWB_RECORD + 6;
    return t;
  }
  if (ustride) {
    t.llo = va ? ulen : 0u;
    t.lhi = vb ? ulen : 0u;
    t.plo = res + a * ustride;
    t.phi = res + b * ustride;
    return t;
  }
  const uint32_t la = lens[a], lb = lens[b];
  t.llo = va ? la : 0u;
  t.lhi = vb ? lb : 0u;
  // an empty target still needs a readable address for the branch-free slow path
  // (SWK_PACK_MIXED: u32 offset words, see mixed_ptr; an empty target's untagged address
  // reads as 2-bit)
  if constexpr (MIX) {
    if (packed == SWK_PACK_MIXED) {
      const uint32_t* o32 = reinterpret_cast<const uint32_t*>(offs);
      t.plo = la ? mixed_ptr(res, o32[a]) : reinterpret_cast<const uint8_t*>(lens);
      t.phi = lb ? mixed_ptr(res, o32[b]) : reinterpret_cast<const uint8_t*>(lens);
      return t;
    }
  }
  t.plo = la ? res + offs[a] : reinterpret_cast<const uint8_t*>(lens);
  t.phi = lb ? res + offs[b] : reinterpret_cast<const uint8_t*>(lens);
  return t;
}

// Chunk counts of a tile (uniform): nch = ceil(max len / C) (>= 1), nfull = min len / C, ncl =
// the columns of chunk nch - 1 that hold a code of some lane (1..C).
template <int C = 8>
__device__ __forceinline__ void tile_chunks(const Lane2& t, size_t tlo, size_t thi, size_t n,
                                            int& nch, int& nfull, int& ncl) {
  uint32_t Lmax = max(t.llo, t.lhi);
  uint32_t Lmin = min(tlo < n ? t.llo : ~0u, thi < n ? t.lhi : ~0u);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    Lmax = max(Lmax, (uint32_t)__shfl_xor((int)Lmax, off));
    Lmin = min(Lmin, (uint32_t)__shfl_xor((int)Lmin, off));
  }
  const int lx = (int)__builtin_amdgcn_readfirstlane(Lmax);
  nch = max(1, (lx + C - 1) / C);
  ncl = lx == 0 ? C : lx - C * (nch - 1);
  const uint32_t lm = __builtin_amdgcn_readfirstlane(Lmin);
  nfull = lm == ~0u ? 0 : (int)(lm / C);  // no valid lane (a tile past the end): no full loads
}

// Kernel arguments (one struct, passed by value).
struct ScoreArgs {
  const uint8_t* res;     // target codes, any byte alignment
  const uint64_t* offs;   // target k = res[offs[k] .. offs[k] + lens[k])
  const uint32_t* lens;
  size_t n;
  const uint32_t* qtab;   // LUT: W*R row words | PROF: (alpha+1) x PS bytes of S - s
  uint32_t nv;            // LUT: 4 x (S - s(*, N)) for codes 4..7
  uint32_t S, O, E;       // shift (>= max s), -gap_open, -gap_extend
  uint32_t PS;            // PROF: profile row stride in bytes (multiple of 16, >= W*R)
  uint32_t pad;           // code used past a target's end (LUT: 4 = N; PROF: alpha = 0xFF row)
  int32_t* scores;        // out; with `accum` also in (best of the previous query segments)
  // Query segments (queries longer than one workgroup's rows): the bottom row {H~, G/F} of
  // the previous segment comes in through edge_in, this segment's goes out through edge_out;
  // layout [tile][ecols][64 lanes] uint2 (coalesced 512 B per column).
  const uint2* edge_in;
  uint2* edge_out;
  uint32_t ecols;
  uint32_t accum;
  uint32_t packed;        // SWK_PACK_*: code bytes | 64-byte CAPI records (2-bit codes;
                          // offs/lens unused) | 2-bit stream (offs in bytes, lens in codes)
  // optional position -> target map: positions [0, *nidx) score targets idx[k] (scores are
  // written to scores[idx[k]]); used to re-score the pairs an optimistic f16 pass flagged
  const uint32_t* idx;
  const uint32_t* nidx;   // with idx: positions [0, min(n, *nidx - idx_base)) are valid
  uint32_t idx_base;
  const uint32_t* ident;  // optional: *ident != 0 -> idx is the identity (ignore it)
  // PAIR (f16 DNA merged): letter-pair table strides; slot (a, b) at 16 + a*pS1 + b*pS2
  uint32_t pS1, pS2;
  // f16 kernels: f16_pair(-(o+e)), f16_pair(-e), f16_pair(-o)
  uint32_t f16_noe, f16_ne, f16_no;
  // wave kernel, optimistic f16 (single query segment): a pair scoring above fb_thresh is
  // re-scored at once in u16 by the same wave, from the u16 table fb_qtab in HBM (LUT words
  // or the profile, row stride fb_PS) with fb_nv; fb_qtab == nullptr: no fallback
  const uint32_t* fb_qtab;
  uint32_t fb_nv, fb_PS;
  int32_t fb_thresh;
  // wave kernel, split tail (K >= 8, one query segment): blocks [0, split_blocks) score pairs
  // [main_pairs, main_pairs + 2 split_blocks) as two row segments of K/2 rows per lane, one wave
  // per segment, the upper segment's bottom row handed to the lower one through split_ring (256
  // columns x uint2 per pair) one 64-step phase apart; blocks past split_blocks score pairs
  // [0, main_pairs) one wave per pair.  split_qtab / split_fb_qtab: the 2-segment tables (the
  // main pass's arithmetic / the u16 fallback), segment stride split_words / split_fb_words
  // 32-bit words, letter stride split_PS / split_fb_PS bytes.
  uint32_t split_blocks;
  uint32_t split_P;       // row segments per split pair: 2 or 4
  uint32_t main_pairs;
  const uint32_t* split_qtab;
  const uint32_t* split_fb_qtab;
  uint32_t split_words, split_fb_words, split_PS, split_fb_PS;
  uint2* split_ring;
  // uniform batch (ustride != 0): every target is ulen codes long and target k starts at byte
  // k * ustride of res; offs and lens are not read (the host feeder's equal-length chunks
  // cross PCIe without per-target headers)
  uint32_t ulen, ustride;
  // several queries, one batch (tile kernel, row-LUT variants): the grid's units are (query q,
  // tile) pairs, unit u = q * ntiles + tile; query q's row LUTs start qwords 32-bit words after
  // query q - 1's, its scores sstride entries after; edge rows are per unit.  nq <= 1: one query
  uint32_t nq, qwords;
  size_t sstride;
  // streamed batch (STREAM variants, the host feeder): equal-length targets (ulen codes; 0:
  // ragged, see stream_tile) in chunks of whole tiles that land in HBM while the kernel runs;
  // chunk c's record sc[c] (nsc records) gives its first tile and its codes (res + res_off);
  // its layout word is hflag[c] in host memory (set by the host once the copy landed) and
  // dflag[c] in uncached device memory (set by the first wave that saw hflag[c], polled by the
  // others); tiles past the first G go to workgroups dynamically (tctr: tiles taken, zeroed by
  // the host), so a workgroup that waited on a late chunk takes fewer tiles.
  // (Round 2 carried these in fields the streamed variants never read, after a build with
  // them appended had other launches score wrong targets now and then.  That was the host
  // feeder's sort scratch zeroed by a null-stream hipMemset racing the chunk's sort kernels on
  // a non-blocking stream -- a corrupt visiting order -- not the argument block)
  const SwkStreamChunk* sc;
  const uint32_t* hflag;
  uint32_t* dflag;
  uint32_t* tctr;
  uint32_t nsc;
  // balanced chunk ranges (BAL variants): workgroup g scores chunks [A_g, A_g+1) of the
  // tile-major chunk sequence, A_g = g x chunks / G, so every resident slot gets the same work
  // whatever tiles / slots is; its range starts at {tile, chunk, A_g} = bal_plan[g] and ends at
  // bal_plan[g + 1] (uniform batches: the host's, ragged ones: the device sort's, whose tiles
  // run longest first with different chunk counts).  A tile cut by a range boundary is scored
  // in two visits: workgroup g - 1 scores its first chunks first (its "head") and hands each
  // wave's column state over through bal_state (sc1 stores, then, a phase later, the flag
  // bal_flag[g][wave] = bal_gen); workgroup g scores the rest last (its "tail").
  uint32_t* bal_flag;
  uint32_t* bal_state;
  const uint4* bal_plan;
  uint32_t bal_gen;
  // two-pairs wave kernel, segmented tail (tail_pairs > 0; split_P = 8, the split_* tables and
  // split_ring): the last tail_pairs pairs run as split_P row segments of 64 rows, one wave
  // each, in 4-wave blocks after the main blocks; segment s hands its bottom row to s + 1
  // through split_ring (a whole row of columns per boundary) and tail_prog (64-column blocks
  // done, zeroed by the host before the launch) instead of a barrier, so a pair's segments sit
  // on different CUs.  tail_prog: [pair][segment] progress | [pair][segment] best (uint2).
  uint32_t* tail_prog;
  uint32_t tail_pairs, tail_cols;
  // cross-workgroup hand-off waits (balanced ranges, the segmented tail): a wait that runs out
  // after poll_limit polls stores its bit (SWK_FAULT_*) into *fault, a word in coherent host
  // memory the host reads at its next synchronisation and turns into SW_ERR_TIMEOUT or a re-run
  // (the scores of the launch are not trusted).  stall (a test hook, 0 = off): the producer the
  // g-th waiter depends on skips its hand-off (balanced ranges: workgroup g - 1's flag; the tail:
  // segment 0 of tail pair g - 1), so the time-out path runs.
  uint32_t* fault;
  uint32_t poll_limit, stall;
  // two-pairs wave kernel, balanced ranges (wbal_blocks > 0: the grid is the resident capacity,
  // G waves): the units (two pairs each, wbal_blocks 32-step blocks per unit) form one block
  // sequence, wave g takes blocks [g UB / G, (g + 1) UB / G); a unit cut by a range boundary is
  // scored in two visits, the head by wave g - 1 first, the tail by wave g last, the lane state
  // handed over through bal_state (WBAL_WORDS x 64 words a wave) and bal_flag[g] = bal_gen
  uint32_t wbal_blocks, wbal_grid;
  // (TRIM variants) sidx: position k's score goes to sidx[k] (the sort's permutation, ident
  // honoured) while its codes, offsets and lengths are read at k (a copy of the batch in its
  // visiting order, SWBANK_RAGGED_GATHER)
  const uint32_t* sidx;
};
static_assert(sizeof(ScoreArgs) == 376, "ScoreArgs layout (kernel argument block) changed");

// a hand-off wait ran out: mark the kind's word of the call's fault group (a vector store to
// host memory, one word per kind so two kinds in one call are both kept; only the host reads
// it, after the launch completed)
__device__ __forceinline__ void report_fault(uint32_t* fault, uint32_t bit) {
  if (fault) __hip_atomic_store(fault + __builtin_ctz(bit), bit, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_SYSTEM);
}

typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef __attribute__((address_space(1))) void* glob_void_ptr;

// C columns x 64 lanes x uint2 (4 KB for C = 8) global -> LDS by one wave: C / 2 LDS-DMA
// instructions of 16 B per lane, lane-linear (the source layout is already [col][lane]).
template <int C = 8>
__device__ __forceinline__ void dma_edge_chunk(const uint2* src, uint2* dst, int lane) {
#pragma unroll
  for (int q = 0; q < C / 2; ++q)
    __builtin_amdgcn_global_load_lds((glob_void_ptr)(src + q * 128 + lane * 2),
                                     (lds_void_ptr)(dst + q * 128), 16, 0, 0);
}

// Chunk count of a tile (uniform), from the lengths alone.
template <int C = 8>
__device__ __forceinline__ int tile_nch(const uint8_t* res, const uint32_t* lens, size_t n,
                                        int tile, int lane, uint32_t packed, const uint32_t* idx,
                                        uint32_t ulen, uint32_t ustride) {
  const size_t a = (size_t)tile * SWB_TILE + lane, b = a + 64;
  auto len = [&](size_t k) -> uint32_t {
    if (k >= n) return 0u;
    if (ustride) return ulen;
    if (idx) k = idx[k];
    return packed == SWK_PACK_RECORDS ? record_len(res + k * SWB_RECORD) : lens[k];
  };
  uint32_t L = max(len(a), len(b));
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) L = max(L, (uint32_t)__shfl_xor((int)L, off));
  return max(1, (int)((__builtin_amdgcn_readfirstlane(L) + C - 1) / C));
}

// Score kernel (persistent pipeline).  A workgroup of W waves x R rows holds the query (or
// one segment of it) and scores the tiles of 128 targets blockIdx.x, blockIdx.x + G, ...
// (G = gridDim.x) as ONE stream of 8-column chunks: wave w processes the workgroup's global
// chunk g at phase g + w, so the wave pipeline fills and drains once per workgroup instead of
// once per tile.  One __syncthreads per phase orders the LDS ring hand-off wave w -> w+1 (the
// RTL's PE-to-PE registers).  A wave that finishes its part of the k-th tile folds its running
// max into bestsh[k % W]; the last wave, which finishes that tile W-1 phases after wave 0,
// writes the scores and clears the slot (wave 0 reuses it for tile k + W, >= W phases later).
// LDS: PAIR: pair table (PS bytes) | bestsh[W][128] | bnd[64] | sink[8 or 1][64] |
//      ein[2][8][64] (segments) | ring[(W-1)][2][8][64] {H~, G or F} | PROF: profile
//
// PAIR (DNA, merged gaps, f16): the substitution words come from an LDS table of letter
// pairs instead of a v_perm per row.  Slot (a, b) (a = code of the low target, b = of the
// high target) holds word k = {s(q_{k+1}, a), s(q_{k+1}, b)} as f16 halves at
// 16 + a*pS1 + b*pS2 + 4k, and {s(q_0, a), s(q_0, b)} 4 bytes before it; the strides put the
// 16 A/C/G/T slots on 16 different 4-bank groups (conflict-free ds_read_b128).  A column of
// wave w reads its row words as 4 blocks of 8 (two ds_read_b128 each), one block ahead of
// the asm block that consumes them: 6.5 VALU per 2 cells instead of 7.5.
// Wave-uniform code layout of streamed chunk c, waiting until its copy landed.  Every wait
// polls the device word; a workgroup's first wave also reads the host word over PCIe (on
// arrival, then every SWK_STREAM_POLL-th wait) and copies it to the device word.  Bounded
// (2^20 polls, about a second): a wave that runs out marks the chunk SWK_STREAM_ABORT in the
// device word and in the host's abort word hflag[nsc + c].
#ifndef SWK_STREAM_POLL
#define SWK_STREAM_POLL 64  // streamed batches: waits between one workgroup's host-word reads
#endif
#ifndef SWK_STREAM_POLL_ALL
#define SWK_STREAM_POLL_ALL 0  // 1: every wave reads the host word (round-5 form)
#endif
__device__ __forceinline__ uint32_t stream_mode(const uint32_t* hflag, uint32_t* dflag, int c,
                                                int nsc, int lane) {
  for (int it = 0; it < (1 << 20); ++it) {
    uint32_t v = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(dflag + c, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT));
    if (v) {
      // the chunk's codes were written by a host-to-device copy, not by the wave that set the
      // device word: a system-scope acquire, so no cache line of the reused buffer (an earlier
      // call's codes) is read stale on this wave's XCD (once per chunk and wave)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      return v;
    }
    // The host word is read over PCIe: by each workgroup's first wave only (the others follow
    // the device word it sets), on arrival and then every SWK_STREAM_POLL-th wait, staggered over
    // the workgroups.  Every waiting wave reading it every 16th wait (the round-5 form,
    // SWK_STREAM_POLL_ALL=1 SWK_STREAM_POLL=16: ~600 PCIe reads a microsecond across the chip
    // while the first chunks cross) made host calls on the headline batch 2.3-2.6 ms instead of
    // 1.9-2.05 (same box, alternating).
    if ((SWK_STREAM_POLL_ALL || threadIdx.x < 64) &&
        (it == 0 || ((it + (int)blockIdx.x) % SWK_STREAM_POLL) == 0)) {
      v = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(hflag + c, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM));
      if (v) {
        if (lane == 0) __hip_atomic_store(dflag + c, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        return v;
      }
    }
    __builtin_amdgcn_s_sleep(16);
  }
  if (lane == 0) {
    __hip_atomic_store(dflag + c, SWK_STREAM_ABORT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(const_cast<uint32_t*>(hflag) + nsc + c, SWK_STREAM_ABORT,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  return SWK_STREAM_ABORT;
}

// Workgroups for a persistent launch: as many as fit on the device at once (occupancy x CUs),
// then evened out so every workgroup gets the same number of tiles (+-1).  (Every resident
// slot with the last round partial measured +0.1 %: a SIMD whose workgroup finished early does
// not speed its other waves up enough; the balanced chunk ranges of BAL launches do)

// Occupancy per (kernel, block size, LDS bytes, device), queried once: the runtime query costs
// microseconds, and the host feeder launches a kernel per chunk.
inline int cached_occupancy(const void* fn, int threads, size_t lds, int dev, int* cus) {
  struct Entry { const void* fn; int threads; size_t lds; int dev, occ, cus; };
  static std::mutex m;
  static std::vector<Entry> cache;
  std::lock_guard<std::mutex> g(m);
  for (const Entry& e : cache)
    if (e.fn == fn && e.threads == threads && e.lds == lds && e.dev == dev) {
      *cus = e.cus;
      return e.occ;
    }
  int occ = 0, c = 0;
  if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, threads, lds) != hipSuccess)
    return 0;
  cache.push_back({fn, threads, lds, dev, occ, c});
  *cus = c;
  return occ;
}

inline unsigned persistent_grid(const void* fn, size_t ntiles, int threads, size_t lds) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return (unsigned)ntiles;
  const int occ = cached_occupancy(fn, threads, lds, dev, &cus);
  if (cus <= 0 || occ <= 0) return (unsigned)ntiles;
  const size_t slots = (size_t)cus * occ;
  const size_t rounds = (ntiles + slots - 1) / slots;
  return (unsigned)((ntiles + rounds - 1) / rounds);
}

}  // namespace swk
#endif  // SWBANK_KCOMMON_H
