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
static uint64_t* g_stamps_host = nullptr;  // the buffer launch_score hands the tile kernel
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
};
static_assert(sizeof(ScoreArgs) == 368, "ScoreArgs layout (kernel argument block) changed");

// a hand-off wait ran out: mark the launch's fault word (a vector store to host memory; only the
// host reads it, after the launch completed)
__device__ __forceinline__ void report_fault(uint32_t* fault, uint32_t bit) {
  if (fault) __hip_atomic_store(fault, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
// polls the device word; one poll in 16 (staggered by workgroup) also reads the host word over
// PCIe, and the wave that sees it set copies it to the device word for the others.  Bounded
// (2^20 polls, about a second): a wave that runs out marks the chunk SWK_STREAM_ABORT in the
// device word and in the host's abort word hflag[nsc + c].
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
    if (((it + (int)blockIdx.x) & 15) == 0) {
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

// C: columns per chunk (one barrier per chunk); 4 for the 16-wave query-set pair kernel, whose
// hand-off ring would not fit LDS beside a 512-row pair table at 8.
// TRIM: a tile's last chunk stops after its last column holding a code of some lane (ragged
// batches: a tile's lengths are one sort bin, rarely a multiple of C; the per-column test costs
// a uniform batch ~25 VALU per chunk in register copies, so only the ragged launches take it).
template <int R, int RB, bool COL0, bool PROF, bool GOTOH, bool F16, bool PAIR = false,
          bool MQ = false, bool STREAM = false, int C = 8, bool BAL = false, bool TRIM = false>
__global__ void __launch_bounds__(R >= 64 ? 512 : 1024) score_kernel(const ScoreArgs a) {
  static_assert(!BAL || (!MQ && !STREAM && !COL0), "balanced ranges: one query, resident batch");
  static_assert(!TRIM || (BAL && PAIR), "trimmed last chunks: the balanced pair kernel");
  static_assert(!MQ || !PROF, "several queries: row-LUT or pair-table variants");
  static_assert(!STREAM || (!MQ && !PROF), "streamed batches: single-query LUT / pair variants");
  static_assert(C == 8 || (C == 4 && PAIR && !STREAM), "4-column chunks: pair tables only");
  static_assert(!PAIR || ((R == 32 || (R == 16 && GOTOH)) && F16 && !PROF && !COL0 &&
                          (!GOTOH || !MQ)),
                "PAIR: f16, merged R = 32 or Gotoh R = 16 / 32 (one query)");
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = __builtin_amdgcn_readfirstlane(blockDim.x >> 6);
  const bool seg_in = a.edge_in != nullptr, seg_out = a.edge_out != nullptr;
  uint32_t* bestsh = smem + (PAIR ? a.PS / 4 : 0);               // W x 128 words
  uint2* bnd = reinterpret_cast<uint2*>(bestsh + W * SWB_TILE);  // row -1 boundary
  uint2* sink = bnd + 64;                                        // last wave's bottom row
  uint2* ein = sink + (seg_out ? C * 64 : 64);                   // previous segment, 2 x 8 cols
  uint2* ring = ein + (seg_in ? 2 * C * 64 : 0);
  uint8_t* prof = reinterpret_cast<uint8_t*>(ring + (size_t)(W > 1 ? W - 1 : 0) * 2 * C * 64);

  size_t n = a.n;
  const uint32_t* idx = a.idx;
  if (idx && a.ident && __builtin_amdgcn_readfirstlane(*a.ident)) idx = nullptr;
  if (idx) {
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(*a.nidx);
    n = cnt > a.idx_base ? min(a.n, (size_t)(cnt - a.idx_base)) : 0;
  }
  const int ntiles = (int)((n + SWB_TILE - 1) / SWB_TILE);
  const int G = (int)gridDim.x;
  // units: (query, tile) pairs; one query: unit = tile.  A unit past the end keeps its number
  // as the tile (lane_targets then reads nothing)
  // (MQ only; otherwise unit = tile and q = 0)
  const int nunits = MQ ? ntiles * (int)a.nq : ntiles;
  int total = 0;  // chunks of all this workgroup's tiles: every wave runs total + W - 1 phases
  uint32_t packed = a.packed;
  // STREAM: tiles taken dynamically, so the total is open until wave 0 finds no tile left
  // (it then stores it in sq[W]; every wave reads sq[W] at each phase)
  int* sq = reinterpret_cast<int*>(prof);  // STREAM: next tile of ordinal k at [k % W] | total
  // BAL: this workgroup's chunk range [A0, A1) as visits: the head (tile be, chunks [0, bf)),
  // the whole tiles [bfirst, be), the tail (tile bs, chunks [bo, K)); a range holds >= 2 tiles
  // (the host checks), so the head and the tail are different tiles.  Visit v (= the tile
  // ordinal k) -> (tile, first chunk, end chunk), recomputed from blockIdx at each visit's end
  // (nothing of the plan stays live across the column loop)
  // (a visit's end chunk is the tile's own chunk count, c1 = -1 until the tile's lengths are
  // read; the plan is read once, into SGPRs: a global load at every visit's end stalls the wave)
  int bs = 0, bo = 0, be = 0, bf = 0;
  if constexpr (BAL) {
    const uint4 p0 = a.bal_plan[blockIdx.x], p1 = a.bal_plan[blockIdx.x + 1];
    bs = (int)__builtin_amdgcn_readfirstlane(p0.x), bo = (int)__builtin_amdgcn_readfirstlane(p0.y);
    be = (int)__builtin_amdgcn_readfirstlane(p1.x), bf = (int)__builtin_amdgcn_readfirstlane(p1.y);
    total = (int)__builtin_amdgcn_readfirstlane(p1.z - p0.z);
  }
  const auto bal_visit = [&](int v, int& t, int& c0, int& c1) {
    const int bK = -1;
    const int bfirst = bo ? bs + 1 : bs;
    const int hh = bf > 0 ? 1 : 0;
    if (v < hh) {
      t = be, c0 = 0, c1 = bf;
    } else if (v - hh < be - bfirst) {
      t = bfirst + v - hh, c0 = 0, c1 = bK;
    } else if (v - hh == be - bfirst && bo > 0) {
      t = bs, c0 = bo, c1 = bK;
    } else {
      t = nunits, c0 = 0, c1 = 1;  // no more visits
    }
    t = __builtin_amdgcn_readfirstlane(t);
    c0 = __builtin_amdgcn_readfirstlane(c0);
    c1 = __builtin_amdgcn_readfirstlane(c1);
  };
  if constexpr (BAL) {
  } else if constexpr (STREAM) {
    total = (int)blockIdx.x < ntiles ? (1 << 30) : 0;
  } else {
    for (int u = blockIdx.x; u < nunits; u += G)  // (the unit's tile: see the MQ order below)
      total += tile_nch<C>(a.res, a.lens, n, !MQ ? u : PAIR ? u / (int)a.nq : u % ntiles, lane,
                        packed, idx, a.ulen, a.ustride);
  }
  // STREAM: the chunk of this wave's current tile (tiles only grow), its first tile, target
  // count, code offset and layout
  // (wave-uniform, kept in SGPRs)
  const SwkStreamChunk* const ssc = a.sc;
  const int snc = (int)a.nsc;
  int scur = -1, st0 = 0;
  uint32_t scn = 0, sro_lo = 0, sro_hi = 0, smode = SWK_PACK_STREAM;
  // ragged streamed batches (ulen == 0): a chunk's region is mixed offset words u32 (see
  // mixed_ptr) | lengths u32 | visiting order u32 (scn each) | codes (SWK_PACK_MIXED: the 2-bit
  // region, then the 4-bit one) at the next 16-byte boundary; the order of the chunk of the tile
  // this wave is scoring (wperm, its first tile wst0) maps score positions to targets
  const uint32_t* cperm = nullptr;
  const uint32_t* wperm = nullptr;
  int wst0 = 0;
  const auto stream_tile = [&](int t, uint32_t& pk) -> Lane2 {
    if (t >= ntiles) {  // past the batch: reads nothing
      pk = SWK_PACK_STREAM;
      Lane2 e;
      e.llo = e.lhi = 0u;
      e.plo = e.phi = a.res;
      return e;
    }
    int c = scur < 0 ? 0 : scur;
    while (c + 1 < snc && t >= (int)ssc[c + 1].tile0) ++c;
    if (c != scur) {
      scur = __builtin_amdgcn_readfirstlane(c);
      st0 = __builtin_amdgcn_readfirstlane((int)ssc[c].tile0);
      scn = __builtin_amdgcn_readfirstlane(
          (uint32_t)((c + 1 < snc ? (size_t)ssc[c + 1].tile0 * SWB_TILE : n) -
                     (size_t)st0 * SWB_TILE));
      sro_lo = __builtin_amdgcn_readfirstlane(ssc[c].res_off_lo);
      sro_hi = __builtin_amdgcn_readfirstlane(ssc[c].res_off_hi);
      const uint32_t md = stream_mode(a.hflag, a.dflag, c, snc, lane);
      // (ragged chunks cross in the mixed layout; an aborted one reads as empty mixed targets)
      smode = a.ulen == 0 ? SWK_PACK_MIXED
                          : md == SWK_PACK_NIBBLE ? SWK_PACK_NIBBLE : SWK_PACK_STREAM;
      if (md == SWK_STREAM_ABORT && a.ulen == 0) {
        // a ragged chunk that never landed (the host re-runs the call): its region may hold
        // anything, so it is read from the zeroed region instead (empty targets, scores in
        // order; uniform chunks read their own region as codes, always in bounds)
        const uint64_t z = (uint64_t)__builtin_amdgcn_readfirstlane(ssc[c].zero_off256) * 256u;
        sro_lo = (uint32_t)z;
        sro_hi = (uint32_t)(z >> 32);
      }
    }
    pk = smode;
    const uint8_t* base = a.res + ((size_t)sro_hi << 32 | sro_lo);
    if (a.ulen == 0) {  // ragged: the chunk's own mixed offset words, lengths and order
      const uint32_t* co = reinterpret_cast<const uint32_t*>(base);
      const uint32_t* cl = co + scn;
      cperm = cl + scn;
      return lane_targets<true>(base + (((size_t)scn * 12 + 15) & ~(size_t)15),
                                reinterpret_cast<const uint64_t*>(co), cl, scn, t - st0, lane, pk,
                                cperm, 0u, 0u);
    }
    return lane_targets<true>(base, nullptr, nullptr, scn, t - st0, lane, pk, nullptr, a.ulen,
                               pk == SWK_PACK_NIBBLE ? (a.ulen + 1) / 2 : (a.ulen + 3) / 4);
  };

  // MQ order: row LUTs query-major (q = unit / ntiles; a wave reloads its LUT SGPRs when the
  // query changes); pair tables query-minor (q = unit % nq) with the grid a multiple of nq, so
  // a workgroup keeps one query and loads its LDS table once
  int unit = blockIdx.x, q = 0;
  int tile = unit;
  int vc0 = 0, vend = 0;  // BAL: the first visit's first and end chunk
  if constexpr (BAL) {
    bal_visit(0, tile, vc0, vend);
    unit = tile;
  }
  if constexpr (MQ) {
    if (unit < nunits) {
      q = PAIR ? unit % (int)a.nq : unit / ntiles;
      tile = PAIR ? unit / (int)a.nq : unit - q * ntiles;
    }
  }
  Lane2 cur;
  if constexpr (STREAM) {
    cur = stream_tile(tile, packed);
    wperm = cperm;
    wst0 = st0;
  } else {
    cur = lane_targets<!MQ>(a.res, a.offs, a.lens, n, tile, lane, packed, idx, a.ulen,
                            a.ustride);
  }
  int nch, nfull, ncl;
  tile_chunks<C>(cur, (size_t)tile * SWB_TILE + lane, (size_t)tile * SWB_TILE + lane + 64, n, nch,
              nfull, ncl);
  (void)ncl;
  if constexpr (BAL) {  // BAL: nch = the visit's end chunk (a head's last chunk is whole)
    if (vend >= 0 && vend < nch) ncl = C;
    nch = vend < 0 ? nch : vend;
  }
  const uint32_t S = a.S;

  for (int i = threadIdx.x; i < W * SWB_TILE; i += blockDim.x) bestsh[i] = 0;
  // row -1: u16 H~ = S, G/F = 0 | f16 H = 0, T = -(o+e)
  // f16 encodings of -(o+e), -e, -o (host-computed, so they stay in SGPRs)
  const f16x2 NOE2 = as_f16x2(as_u16x2(a.f16_noe)), NE2 = as_f16x2(as_u16x2(a.f16_ne)),
              NO2 = as_f16x2(as_u16x2(a.f16_no));
  if (wave == 0) {
    bnd[lane] = F16 ? make_uint2(0u, GOTOH ? 0u : as_u32(as_u16x2(NOE2)))
                    : make_uint2(S | (S << 16), 0u);
    if (seg_in)  // the previous segment's bottom row of chunk 0
      dma_edge_chunk<C>(a.edge_in + (size_t)(MQ ? unit : tile) * a.ecols * 64, ein, lane);
  }
  uint32_t nv = a.nv;
  uint32_t tab[PROF || PAIR ? 1 : R];
  if constexpr (PAIR) {
    const uint4* src = reinterpret_cast<const uint4*>(a.qtab + (MQ ? (size_t)q * a.qwords : 0));
    for (uint32_t i = threadIdx.x; i < a.PS / 16; i += blockDim.x)
      reinterpret_cast<uint4*>(smem)[i] = src[i];
  } else if constexpr (PROF) {
    // query profile -> LDS (the ScoringModule's query + penalty registers)
    const uint32_t words = (a.pad + 1) * a.PS / 16;
    const uint4* src = reinterpret_cast<const uint4*>(a.qtab);
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x)
      reinterpret_cast<uint4*>(prof)[i] = src[i];
  } else {
    // nv in a VGPR so each v_perm_b32 takes its row LUT straight from an SGPR (one scalar
    // operand per VOP3 on gfx950).
    asm volatile("" : "+v"(nv));
#pragma unroll
    for (int r = 0; r < R; ++r)
      tab[r] = __builtin_amdgcn_readfirstlane(a.qtab[(MQ ? (size_t)q * a.qwords : 0) + wave * R + r]);
  }
  const u16x2 S2 = {(unsigned short)S, (unsigned short)S};
  const u16x2 O2 = {(unsigned short)a.O, (unsigned short)a.O};
  const u16x2 E2 = {(unsigned short)a.E, (unsigned short)a.E};
  const uint32_t oes = a.O + a.E + S;
  const u16x2 OES2 = {(unsigned short)oes, (unsigned short)oes};
  const u16x2 H0 = F16 ? (u16x2){0, 0} : S2;          // H of row/column -1
  const u16x2 X0 = (F16 && !GOTOH) ? as_u16x2(NOE2) : (u16x2){0, 0};  // G/E/T of column -1

  // H~ and G (merged) / E (Gotoh) / T (f16) of the column to the left
  u16x2 Hl[R], Xl[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    Hl[r] = H0;
    Xl[r] = X0;
  }
  u16x2 best = {0, 0};
  u16x2 prevUpH = H0;  // H(row above, column -1)
  uint2 rlo, rhi;      // raw codes of the next chunk (prefetched one phase ahead)
  load_raw<C, !MQ>(cur, vc0, vc0 < nfull, a.pad, packed, rlo, rhi);
  if (STREAM && threadIdx.x == 0) sq[W] = total;
  __syncthreads();

  // PAIR: column state one column ahead: acur = this column's table address (slot + this
  // wave's rows - 16), pA = its first 8 row words, pw = its row-0 word
  // Table addresses are absolute LDS byte addresses (smem's link-time address folded into
  // wofs once), so a column's address needs no add for the base.
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) const u32x4 lds_u4;
  typedef __attribute__((address_space(3))) const uint32_t lds_u32;
  const auto ld4 = [](uint32_t addr) { return __builtin_bit_cast(uint4, *(lds_u4*)(size_t)addr); };
  // the row-0 word: a relaxed atomic load, so LLVM does not merge it with the neighbouring
  // 16-B reads (it splits them into ds_read2_b32 pairs otherwise)
  const auto ld1 = [](uint32_t addr) {
    return __atomic_load_n((lds_u32*)(size_t)addr, __ATOMIC_RELAXED);
  };
  const uint32_t wofs = (uint32_t)wave * R * 4 + (uint32_t)(size_t)(lds_void_ptr)smem;
  // codes clamped to N: lanes past the batch end (and codes >= 5 on the device API) would
  // otherwise pick a slot outside the table, and a slot feeds both halves (one v_min each,
  // SDWA byte-select)
  // (3 VALU: {a, b} as u16 halves by one v_perm, clamped by one v_pk_min_u16, then
  // a*pS1 + b*pS2 + wofs by one v_dot2_u32_u16; the host keeps pS1, pS2 < 65536)
  const u16x2 pS12 = {(unsigned short)a.pS1, (unsigned short)a.pS2};
  const auto pair_addr = [&](uint32_t wl, uint32_t wh, int sh) {
    const uint32_t sel = (uint32_t)(sh >> 3) | 0x0C00u | ((uint32_t)(4 + (sh >> 3)) << 16) |
                         0x0C000000u;
    const u16x2 ab = __builtin_elementwise_min(as_u16x2(__builtin_amdgcn_perm(wh, wl, sel)),
                                               (u16x2){4, 4});
    return __builtin_amdgcn_udot2(ab, pS12, wofs, false);
  };
  uint32_t acur = 0, pw = 0;
  uint4 pA0 = {0, 0, 0, 0}, pA1 = {0, 0, 0, 0};
  if constexpr (PAIR) {
    acur = pair_addr(rlo.x, rhi.x, 0);
    pA0 = ld4(acur + 16);
    pA1 = ld4(acur + 32);
    pw = ld1(acur + 12);
  }
  (void)pA0; (void)pA1; (void)pw; (void)acur; (void)wofs;

  // branch-free hand-off: wave 0 reads the top boundary (constant, stride 0, or the previous
  // segment's row), the last wave writes into an LDS sink (branches inside the column loop
  // split it into blocks and LLVM then sinks the H updates across columns, blowing up
  // register pressure)
  const int istride = (wave > 0 || seg_in) ? 64 : 0, ostride = (wave < W - 1 || seg_out) ? 64 : 0;
  const uint32_t pbase = (uint32_t)wave * R;
  const uint32_t padc = a.pad;
  // BAL hand-off of one wave's column state {H, T of its R rows, the diagonal H above, best}
  // at a head's end / a tail's start: word i of lane l at state[((g W + wave) (2R + 2) + i) 64
  // + l] (coalesced), written and read with sc1 (write-through / L2) accesses and a flag
  // (MI355X_MICROARCH.md, inter-workgroup visibility: sc1 stores, vmcnt(0), sc1 flag; sc1 poll,
  // sc1 loads).  The consumer's tail is its last visit and the producer's head its first, so
  // the flag is normally long set; the poll is bounded (poll_limit, about 4 s) and a time-out
  // marks the launch's fault word (the host fails the call) rather than hanging.
  // (the state addresses go through an opaque copy: loop-invariant, LLVM would otherwise hoist
  // all 2R + 2 of them out of the phase loop, 2 VGPRs each, and spill)
  int bal_pend = 0;  // BAL: phases until the head's flag goes out (0: none pending)
  const auto bal_store = [&](int g_to) {
    uint32_t* sp = a.bal_state + ((size_t)g_to * W + wave) * (2 * R + 2) * 64 + lane;
    asm volatile("" : "+v"(sp));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      __hip_atomic_store(sp + r * 64, as_u32(Hl[r]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sp + (R + r) * 64, as_u32(Xl[r]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    __hip_atomic_store(sp + 2 * R * 64, as_u32(prevUpH), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sp + (2 * R + 1) * 64, as_u32(best), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    bal_pend = 2;  // the flag goes out a phase later, when the stores have long completed
  };
  const auto bal_flag_out = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0 && blockIdx.x + 1 != a.stall)  // (stall: a test hook)
      __hip_atomic_store(a.bal_flag + ((size_t)blockIdx.x + 1) * W + wave, a.bal_gen,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
#if SWK_STAMPS
  uint64_t st_bload = 0;  // (measurement builds) cycles in tail state loads
#endif
  const auto bal_load = [&]() {
#if SWK_STAMPS
    const uint64_t sb0 = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t* fl = a.bal_flag + (size_t)blockIdx.x * W + wave;
    uint32_t it = 0;
    for (; it < a.poll_limit; ++it) {
      if (__builtin_amdgcn_readfirstlane(
              __hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == a.bal_gen)
        break;
      __builtin_amdgcn_s_sleep(8);
    }
    if (it == a.poll_limit && lane == 0) report_fault(a.fault, SWK_FAULT_BAL);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t* sp = a.bal_state + ((size_t)blockIdx.x * W + wave) * (2 * R + 2) * 64 + lane;
    asm volatile("" : "+v"(sp));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      Hl[r] = as_u16x2(__hip_atomic_load(sp + r * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      Xl[r] = as_u16x2(
          __hip_atomic_load(sp + (R + r) * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    prevUpH = as_u16x2(
        __hip_atomic_load(sp + 2 * R * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    best = as_u16x2(
        __hip_atomic_load(sp + (2 * R + 1) * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#if SWK_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_bload += __builtin_amdgcn_s_memtime() - sb0;
#endif
  };
  (void)bal_store; (void)bal_load; (void)bal_flag_out;
  // chunk within the current tile, tile ordinal in this workgroup (BAL: the visit ordinal; a
  // first visit is a head or a whole tile, never a tail)
  int c = vc0, k = 0;
  int nch_n = 1, nfull_n = 0, ncl_n = C;  // the next tile's chunk counts
  uint32_t packed_n = packed;  // STREAM: the next tile's code layout
#if SWK_PRIO_ROT
  const uint32_t prq = (uint32_t)((blockIdx.x * 4ull) / gridDim.x);
  uint32_t prio = 4;  // (none set yet)
#endif
#if SWK_STAMPS
  // (measurement builds only) per wave: kernel entry / exit, cycles in active phases (the
  // column work), in fill/drain phases (no chunk of its own) and in the per-phase barrier
  uint64_t st_t0 = __builtin_amdgcn_s_memtime(), st_act = 0, st_idle = 0, st_bar = 0;
  uint64_t st_p = st_t0;
#endif
  for (int ph = 0;; ++ph) {
    if constexpr (STREAM) total = __builtin_amdgcn_readfirstlane(sq[W]);
    if (ph >= total + W - 1) break;
#if SWK_PRIO_ROT
    // (a 16-wave workgroup has its CU alone; SWK_PRIO_END: the last 1/2^SWK_PRIO_END_FRAC of
    // the phases rotate 2^SWK_PRIO_END times faster, so the four finish closer together)
    if (W <= 8)
      prio_rotate(prq, prio,
                  SWK_PRIO_END && ph >= total - (total >> SWK_PRIO_END_FRAC)
                      ? SWK_PRIO_SHIFT - SWK_PRIO_END : SWK_PRIO_SHIFT);

#endif
    const int g = ph - wave;
    if (g >= 0 && g < total) {
      const uint2 clo = rlo, chi = rhi;
      const bool last = c + 1 == nch;
      int nunit = (MQ ? unit : tile) + G;
      int nc0 = 0, nvend = 0;  // BAL: the next visit's first and end chunk
      if constexpr (BAL) {
        if (last) bal_visit(k + 1, nunit, nc0, nvend);
      }
      if constexpr (STREAM) {  // wave 0 takes the next tile; the others read it W-1 phases on
        if (last) {
          if (wave == 0) {
            int nt = 0;
            if (lane == 0) nt = G + (int)atomicAdd(a.tctr, 1u);
            nt = min(__builtin_amdgcn_readfirstlane(nt), ntiles);
            if (lane == 0) {
              sq[(k + 1) % W] = nt;
              if (nt >= ntiles) sq[W] = g + 1;
            }
            nunit = nt;
          } else {
            nunit = __builtin_amdgcn_readfirstlane(sq[(k + 1) % W]);
          }
        }
      }
      int ntile = nunit, nqq = q;  // the next unit's tile and query
      if constexpr (MQ) {
        if (nunit < nunits) {
          if constexpr (PAIR) {
            ntile = nunit / (int)a.nq;  // same query (G is a multiple of nq)
          } else {
            ntile = tile + G;
            while (ntile >= ntiles) {
              ntile -= ntiles;
              ++nqq;
            }
          }
        }
      }
      if (!last) {
        load_raw<C, !MQ>(cur, c + 1, c + 1 < nfull, a.pad, packed, rlo, rhi);
      } else if (nunit < nunits) {  // first chunk of the next tile
        if constexpr (STREAM) cur = stream_tile(ntile, packed_n);
        else
          cur = lane_targets<!MQ>(a.res, a.offs, a.lens, n, ntile, lane, packed, idx, a.ulen,
                                  a.ustride);
        tile_chunks<C>(cur, (size_t)ntile * SWB_TILE + lane, (size_t)ntile * SWB_TILE + lane + 64,
                    n, nch_n, nfull_n, ncl_n);
        if (BAL && nvend >= 0 && nvend < nch_n) ncl_n = C;
        if (BAL && nvend < 0) nvend = nch_n;
        load_raw<C, !MQ>(cur, nc0, nc0 < nfull_n, a.pad, STREAM ? packed_n : packed, rlo, rhi);
      }
      const int slot = g & 1;
      // next chunk's boundary row (never past the last unit's edge rows)
      if (seg_in && wave == 0 && (last ? nunit < nunits : (MQ ? unit : tile) < nunits))
        dma_edge_chunk<C>(a.edge_in + ((size_t)(last ? nunit : MQ ? unit : tile) * a.ecols +
                                    (size_t)(last ? 0 : c + 1) * C) * 64,
                       ein + (size_t)((g + 1) & 1) * C * 64, lane);
      const uint2* rin = wave > 0 ? ring + ((size_t)((wave - 1) * 2 + slot) * C) * 64 + lane
                                  : (seg_in ? ein + (size_t)slot * C * 64 : bnd) + lane;
      uint2* rout = wave < W - 1 ? ring + ((size_t)(wave * 2 + slot) * C) * 64 + lane
                                 : sink + lane;
      uint2 rv = rin[0];
      ProfLookup16<PROF && F16 ? R : 2> lkq;  // f16 profile: the next column's words
      (void)lkq;
      // TRIM: the tile's last chunk stops after its last column holding a code (a tile runs to
      // its longest lane; every wave stops at the same column, so the ring stays consistent)
      const int ncols = TRIM && c + 1 == nch ? ncl : C;
      bool trimmed = false;
      (void)ncols;
#pragma unroll
      for (int jj = 0; jj < C; ++jj) {
        if (TRIM && jj > 0 && __builtin_expect(jj >= ncols, 0)) {
          trimmed = true;
          continue;
        }
        const u16x2 upH = as_u16x2(rv.x);
        u16x2 upX = as_u16x2(rv.y);
        if (jj + 1 < C) rv = rin[(jj + 1) * istride];  // one column ahead
        u16x2 diag = prevUpH;
        prevUpH = upH;
        const uint32_t wlo = jj < 4 ? clo.x : clo.y, whi = jj < 4 ? chi.x : chi.y;
        if constexpr (PROF && F16) {
          // profile words one column ahead (the LDS latency hides behind a column)
          const auto load16 = [&](int j, ProfLookup16<R>& out) {
            const uint32_t wl = j < 4 ? clo.x : clo.y, wh = j < 4 ? chi.x : chi.y;
            const uint32_t blo = min((wl >> (8 * (j & 3))) & 0xFFu, padc);
            const uint32_t bhi = min((wh >> (8 * (j & 3))) & 0xFFu, padc);
            // 24-bit multiplies (full rate; a 32-bit v_mul_lo is quarter rate)
            const uint4* plo = reinterpret_cast<const uint4*>(prof + __umul24(blo, a.PS) + 2 * pbase);
            const uint4* phi = reinterpret_cast<const uint4*>(prof + __umul24(bhi, a.PS) + 2 * pbase);
#pragma unroll
            for (int q = 0; q < R / 8; ++q) {
              const uint4 x = plo[q], y = phi[q];
              out.lo[4 * q] = x.x; out.lo[4 * q + 1] = x.y; out.lo[4 * q + 2] = x.z;
              out.lo[4 * q + 3] = x.w;
              out.hi[4 * q] = y.x; out.hi[4 * q + 1] = y.y; out.hi[4 * q + 2] = y.z;
              out.hi[4 * q + 3] = y.w;
            }
          };
          ProfLookup16<R> lk;
          if (jj == 0) load16(0, lk);
          else lk = lkq;
          if (jj + 1 < C) load16(jj + 1, lkq);
          __builtin_amdgcn_sched_barrier(0);
          if (COL0 && jj == 0 && c == 0)
            column_f16<R, RB, GOTOH, true>(lk, diag, upX, Hl, Xl, best, NOE2, NE2, NO2);
          else
            column_f16<R, RB, GOTOH, false>(lk, diag, upX, Hl, Xl, best, NOE2, NE2, NO2);
        } else if constexpr (PROF) {
          ProfLookup<R> lk;
          const uint32_t blo = min((wlo >> (8 * (jj & 3))) & 0xFFu, padc);
          const uint32_t bhi = min((whi >> (8 * (jj & 3))) & 0xFFu, padc);
          const uint4* plo = reinterpret_cast<const uint4*>(prof + __umul24(blo, a.PS) + pbase);
          const uint4* phi = reinterpret_cast<const uint4*>(prof + __umul24(bhi, a.PS) + pbase);
#pragma unroll
          for (int q = 0; q < R / 16; ++q) {
            const uint4 x = plo[q], y = phi[q];
            lk.lo[4 * q] = x.x; lk.lo[4 * q + 1] = x.y; lk.lo[4 * q + 2] = x.z;
            lk.lo[4 * q + 3] = x.w;
            lk.hi[4 * q] = y.x; lk.hi[4 * q + 1] = y.y; lk.hi[4 * q + 2] = y.z;
            lk.hi[4 * q + 3] = y.w;
          }
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (GOTOH) {
            u16x2 uH = upH;
            column_gotoh<R, RB>(lk, diag, uH, upX, Hl, Xl, best, S2, OES2, E2);
          } else if (COL0 && jj == 0 && c == 0) {
            column_merged<R, RB, true>(lk, diag, upX, Hl, Xl, best, S2, O2, E2);
          } else {
            column_merged<R, RB, false>(lk, diag, upX, Hl, Xl, best, S2, O2, E2);
          }
        } else if constexpr (PAIR) {
          // the next column's table address (its codes: this chunk, or byte 0 of the next)
          const uint32_t nwl = jj + 1 < C ? (jj + 1 < 4 ? clo.x : clo.y) : rlo.x;
          const uint32_t nwh = jj + 1 < C ? (jj + 1 < 4 ? chi.x : chi.y) : rhi.x;
          const int nsh = jj + 1 < C ? 8 * ((jj + 1) & 3) : 0;
          uint32_t Da, Db, X, DN, IN;
          const uint32_t noe = as_u32(as_u16x2(NOE2)), ne = as_u32(as_u16x2(NE2)),
                 no = as_u32(as_u16x2(NO2));
          u16x2 bst = best;
          u16x2 F = upX;  // Gotoh: F running down the column
#define SWK_PAIR_HT(B)                                                                        \
  [h0] "+v"(Hl[B]), [h1] "+v"(Hl[B + 1]), [h2] "+v"(Hl[B + 2]), [h3] "+v"(Hl[B + 3]),          \
      [h4] "+v"(Hl[B + 4]), [h5] "+v"(Hl[B + 5]), [h6] "+v"(Hl[B + 6]), [h7] "+v"(Hl[B + 7]),  \
      [t0] "+v"(Xl[B]), [t1] "+v"(Xl[B + 1]), [t2] "+v"(Xl[B + 2]), [t3] "+v"(Xl[B + 3]),      \
      [t4] "+v"(Xl[B + 4]), [t5] "+v"(Xl[B + 5]), [t6] "+v"(Xl[B + 6]), [t7] "+v"(Xl[B + 7]),  \
      [Db] "=&v"(Db), [best] "+v"(bst)
#define SWK_PAIR_OUT(B, DA) SWK_PAIR_HT(B), [Da] DA(Da), [X] "=&v"(X), [DN] "=&v"(DN), [IN] "=&v"(IN)
#define SWK_PAIR_OUTG(B, DA)                                                                  \
  SWK_PAIR_HT(B), [Da] DA(Da), [EN] "=&v"(X), [HN] "=&v"(DN), [FN] "=&v"(IN), [F] "+v"(F)
#define SWK_PAIR_IN(P0, P1)                                                                   \
  [p0] "v"(P0.x), [p1] "v"(P0.y), [p2] "v"(P0.z), [p3] "v"(P0.w), [p4] "v"(P1.x),             \
      [p5] "v"(P1.y), [p6] "v"(P1.z), [p7] "v"(P1.w), [noe] "s"(noe), [ne] "s"(ne), [no] "s"(no)
// block B of the column: first (row-0 prologue), middle or last (no successor row)
#define SWK_PAIR_BLOCK(KIND, B, P0, P1)                                                       \
  if constexpr (GOTOH) {                                                                      \
    if constexpr (KIND == 0)                                                                  \
      asm volatile(SWK_F16PAIRG_F : SWK_PAIR_OUTG(B, "=&v")                                   \
                   : SWK_PAIR_IN(P0, P1), [dg] "v"(diag), [pw] "v"(pw));                   \
    else if constexpr (KIND == 1)                                                             \
      asm volatile(SWK_F16PAIRG_M : SWK_PAIR_OUTG(B, "+v") : SWK_PAIR_IN(P0, P1));         \
    else                                                                                      \
      asm volatile(SWK_F16PAIRG_L : SWK_PAIR_OUTG(B, "+v") : SWK_PAIR_IN(P0, P1));         \
  } else {                                                                                    \
    if constexpr (KIND == 0)                                                                  \
      asm volatile(SWK_F16PAIR_F : SWK_PAIR_OUT(B, "=&v")                                     \
                   : SWK_PAIR_IN(P0, P1), [up] "v"(upX), [dg] "v"(diag), [pw] "v"(pw));                 \
    else if constexpr (KIND == 1)                                                             \
      asm volatile(SWK_F16PAIR_M : SWK_PAIR_OUT(B, "+v") : SWK_PAIR_IN(P0, P1), [up] "v"(Xl[B - 1]));   \
    else                                                                                      \
      asm volatile(SWK_F16PAIR_L : SWK_PAIR_OUT(B, "+v") : SWK_PAIR_IN(P0, P1), [up] "v"(Xl[B - 1]));   \
  }
          // each block's words are read one block ahead; the last block's wait for the next
          // column's block 0 and row-0 word
          uint4 pB0 = ld4(acur + 48), pB1 = ld4(acur + 64);  // block 1
          __builtin_amdgcn_sched_barrier(0);
          SWK_PAIR_BLOCK(0, 0, pA0, pA1)
          if constexpr (R == 32) {
            pA0 = ld4(acur + 80);  // block 2
            pA1 = ld4(acur + 96);
            __builtin_amdgcn_sched_barrier(0);
            SWK_PAIR_BLOCK(1, 8, pB0, pB1)
            pB0 = ld4(acur + 112);  // block 3
            pB1 = ld4(acur + 128);
            __builtin_amdgcn_sched_barrier(0);
            SWK_PAIR_BLOCK(1, 16, pA0, pA1)
          }
          acur = pair_addr(nwl, nwh, nsh);  // next column: block 0 and row-0 word
          pA0 = ld4(acur + 16);
          pA1 = ld4(acur + 32);
          pw = ld1(acur + 12);
          __builtin_amdgcn_sched_barrier(0);
          SWK_PAIR_BLOCK(2, R - 8, pB0, pB1)
#undef SWK_PAIR_BLOCK
#undef SWK_PAIR_HT
#undef SWK_PAIR_OUT
#undef SWK_PAIR_OUTG
#undef SWK_PAIR_IN
          (void)Db; (void)X; (void)DN; (void)IN;
          best = bst;
          upX = GOTOH ? F : Xl[R - 1];
        } else if constexpr (F16) {
          // selector bytes {0x0C, code_lo, 0x0C, code_hi}: the LUT byte is the f16 high byte
          const uint32_t sel16 = 0x0Cu | ((uint32_t)(jj & 3) << 8) | (0x0Cu << 16) |
                                 ((uint32_t)(4 + (jj & 3)) << 24);
          const LutLookup<R> lk{tab, nv, __builtin_amdgcn_perm(whi, wlo, sel16) | 0x000C000Cu};
          __builtin_amdgcn_sched_barrier(0);
          if (COL0 && jj == 0 && c == 0)
            column_f16<R, RB, GOTOH, true>(lk, diag, upX, Hl, Xl, best, NOE2, NE2, NO2);
          else
            column_f16<R, RB, GOTOH, false>(lk, diag, upX, Hl, Xl, best, NOE2, NE2, NO2);
        } else {
          // selector: byte 0 = code of the low target, byte 2 = code of the high target
          const uint32_t sel =
              (uint32_t)(jj & 3) | ((uint32_t)(4 + (jj & 3)) << 16) | 0x0C000C00u;
          const LutLookup<R> lk{tab, nv, __builtin_amdgcn_perm(whi, wlo, sel) | 0x0C000C00u};
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (GOTOH) {
            u16x2 uH = upH;
            column_gotoh<R, RB>(lk, diag, uH, upX, Hl, Xl, best, S2, OES2, E2);
          } else if (COL0 && jj == 0 && c == 0) {
            column_merged<R, RB, true>(lk, diag, upX, Hl, Xl, best, S2, O2, E2);
          } else {
            column_merged<R, RB, false>(lk, diag, upX, Hl, Xl, best, S2, O2, E2);
          }
        }
        // pin the running max once per column: otherwise LLVM re-associates the max over the
        // whole phase into a tree and keeps every M live
        asm volatile("" : "+v"(best));
        rout[jj * ostride] = make_uint2(as_u32(Hl[R - 1]), as_u32(upX));
      }
      if constexpr (PAIR && TRIM) {
        if (trimmed) {  // the next chunk's column 0, read ahead as at a chunk's end
          acur = pair_addr(rlo.x, rhi.x, 0);
          pA0 = ld4(acur + 16);
          pA1 = ld4(acur + 32);
          pw = ld1(acur + 12);
        }
      }
      (void)trimmed;
      if (seg_out && wave == W - 1) {  // this segment's bottom row -> the next segment
        uint2* dst = a.edge_out + ((size_t)(MQ ? unit : tile) * a.ecols + (size_t)c * C) * 64 + lane;
#pragma unroll
        for (int jj = 0; jj < C; ++jj) dst[jj * 64] = sink[jj * 64 + lane];
      }
      if (last) {
        // BAL: the first visit is a head when the range ends inside a tile
        if (BAL && k == 0 && bf > 0) {  // BAL: a head visit ends: hand its state over
          bal_store((int)blockIdx.x + 1);
        } else {  // this wave's part of tile k is done
        uint32_t* bs = bestsh + (k % W) * SWB_TILE;
        atomicMax(&bs[lane], (uint32_t)best.x);
        atomicMax(&bs[lane + 64], (uint32_t)best.y);
        if (wave == W - 1) {  // every other wave folded tile k in an earlier phase
          const size_t tlo = (size_t)tile * SWB_TILE + lane, thi = tlo + 64;
          int32_t blo = (int32_t)bs[lane], bhi = (int32_t)bs[lane + 64];
          bs[lane] = 0;
          bs[lane + 64] = 0;
          if constexpr (F16) {  // f16 bit patterns of non-negative integers -> int
            blo = f16_unscore((uint32_t)blo);
            bhi = f16_unscore((uint32_t)bhi);
          }
          size_t slo = idx && tlo < n ? idx[tlo] : tlo;
          size_t shi = idx && thi < n ? idx[thi] : thi;
          if constexpr (STREAM) {  // ragged: through the chunk's visiting order
            if (wperm) {
              const size_t b0 = (size_t)wst0 * SWB_TILE;
              if (tlo < n) slo = b0 + wperm[tlo - b0];
              if (thi < n) shi = b0 + wperm[thi - b0];
            }
          }
          int32_t* qsc = MQ ? a.scores + (size_t)q * a.sstride : a.scores;
          if (a.accum) {  // best over the previous query segments
            if (tlo < n) blo = max(blo, qsc[slo]);
            if (thi < n) bhi = max(bhi, qsc[shi]);
          }
          if (tlo < n) qsc[slo] = blo;
          if (thi < n) qsc[shi] = bhi;
        }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
          Hl[r] = H0;
          Xl[r] = X0;
        }
        best = (u16x2){0, 0};
        prevUpH = H0;
        tile = ntile;
        if constexpr (STREAM) {
          packed = packed_n;
          wperm = cperm;
          wst0 = st0;
        }
        if constexpr (MQ && PAIR) unit = nunit;
        if constexpr (MQ && !PAIR) {  // several queries: the next unit's row LUTs
          unit = nunit;
          if (nqq != q) {
            q = nqq;
#pragma unroll
            for (int r = 0; r < R; ++r)
              tab[r] = __builtin_amdgcn_readfirstlane(a.qtab[(size_t)q * a.qwords + wave * R + r]);
          }
        }
        nch = nch_n;
        nfull = nfull_n;
        ncl = ncl_n;
        c = 0;
        if constexpr (BAL) {
          c = nc0;
          nch = nvend;
          if (nc0 > 0) bal_load();  // a tail: the head's state
        }
        ++k;
      } else {
        ++c;
      }
    }
    if constexpr (BAL) {
      if (bal_pend > 0 && --bal_pend == 0) bal_flag_out();
    }
#if SWK_STAMPS
    const bool st_own = g >= 0 && g < total;  // (fill / drain phases: all of it to st_idle)
    const uint64_t st_b = __builtin_amdgcn_s_memtime();
    (st_own ? st_act : st_idle) += st_b - st_p;
#endif
    __syncthreads();
#if SWK_STAMPS
    st_p = __builtin_amdgcn_s_memtime();
    (st_own ? st_bar : st_idle) += st_p - st_b;
#endif
  }
  if constexpr (BAL) {
    if (bal_pend > 0) bal_flag_out();
  }
#if SWK_STAMPS
  // (the non-streamed variants never read tctr: measurement builds pass the buffer there)
  uint64_t* const g_stamps = STREAM ? nullptr : reinterpret_cast<uint64_t*>(a.tctr);
  if (lane == 0 && g_stamps) {
    uint64_t* o = g_stamps + ((size_t)blockIdx.x * 16 + wave) * 16;
    unsigned hw = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    o[0] = st_t0;
    o[1] = __builtin_amdgcn_s_memtime();
    o[2] = st_act;
    o[3] = st_idle;
    o[4] = st_bar;
    o[5] = hw;
    unsigned xcc = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    o[6] = (uint64_t)total;
    o[7] = (uint64_t)(xcc & 15);
    o[8] = st_bload;
  }
#endif
}

// Workgroups for a persistent launch: as many as fit on the device at once (occupancy x CUs),
// then evened out so every workgroup gets the same number of tiles (+-1).  (Every resident
// slot with the last round partial measured +0.1 %: a SIMD whose workgroup finished early does
// not speed its other waves up enough; the balanced chunk ranges of BAL launches do)

// Occupancy per (kernel, block size, LDS bytes, device), queried once: the runtime query costs
// microseconds, and the host feeder launches a kernel per chunk.
static int cached_occupancy(const void* fn, int threads, size_t lds, int dev, int* cus) {
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

static unsigned persistent_grid(const void* fn, size_t ntiles, int threads, size_t lds) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return (unsigned)ntiles;
  const int occ = cached_occupancy(fn, threads, lds, dev, &cus);
  if (cus <= 0 || occ <= 0) return (unsigned)ntiles;
  const size_t slots = (size_t)cus * occ;
  const size_t rounds = (ntiles + slots - 1) / slots;
  return (unsigned)((ntiles + rounds - 1) / rounds);
}

template <int R, int RB, bool COL0, bool PROF, bool GOTOH, bool F16, bool PAIR = false,
          bool MQ = false, bool STREAM = false, int C = 8, bool BAL = false, bool TRIM = false>
static hipError_t launch_score(const ScoreArgs& a, int W, uint32_t prof_bytes, hipStream_t st,
                               unsigned bal_grid = 0) {
  const size_t ntiles = (a.n + SWB_TILE - 1) / SWB_TILE * (MQ ? a.nq : 1);  // units
  const size_t lds = (size_t)W * SWB_TILE * 4 +
                     (size_t)(64 + (a.edge_out ? C * 64 : 64) + (a.edge_in ? 2 * C * 64 : 0) +
                              (W > 1 ? W - 1 : 0) * 2 * C * 64) * 8 +
                     (PROF ? prof_bytes : 0) + (PAIR ? a.PS : 0) + (STREAM ? 256 : 0);
  auto fn = &score_kernel<R, RB, COL0, PROF, GOTOH, F16, PAIR, MQ, STREAM, C, BAL, TRIM>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  if (lds > 160 * 1024) return hipErrorInvalidConfiguration;
  unsigned grid = BAL ? bal_grid
                      : persistent_grid(reinterpret_cast<const void*>(fn), ntiles, 64 * W, lds);
#if SWK_STAMPS
  if (!STREAM && g_stamps_host) {
    ScoreArgs b = a;
    b.tctr = reinterpret_cast<uint32_t*>(g_stamps_host);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(64 * W), (unsigned)lds, st, b);
    return hipGetLastError();
  }
#endif
  if (MQ && PAIR) grid = std::max(a.nq, grid / a.nq * a.nq);  // one query per workgroup
  if (BAL && (grid == 0 || ntiles < 2 * (size_t)grid)) return hipErrorInvalidConfiguration;
  hipLaunchKernelGGL(fn, dim3(grid), dim3(64 * W), (unsigned)lds, st, a);
  return hipGetLastError();
}

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
#ifndef SWK_HALF_FMA
// two-pairs wave kernel: LDS profile words {s, 1.0} (4 B per letter and row) added with one
// op_sel FMA per row (gen_f16_rows.py mode F) instead of 2-byte entries interleaved by a v_perm
#define SWK_HALF_FMA 1
#endif
// the two-pairs kernel's LDS: the profile (letter stride SWK_HALF_LS bytes, 512 rows) and
// each wave's code ring (profile offsets of both halves' targets, SWK_HALF_RING bytes a wave)
#define SWK_HALF_LS (SWK_HALF_FMA ? 2048u : 1024u)
#define SWK_HALF_RING (SWK_HALF_FMA ? 512u : 1024u)
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
  const auto ring_write = [&](const uint32_t nc) __attribute__((always_inline)) {
    ring[hl] = (RingT)((ringprev & 0xFFu) * LS);
    ring[32 + hl] = (RingT)((nc & 0xFFu) * LS);
    ring[64 + hl] = (RingT)((ringprev >> 8) * LS);
    ring[96 + hl] = (RingT)((nc >> 8) * LS);
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
  const auto load_prof = [&](auto& lk, uint32_t oa, uint32_t ob) __attribute__((always_inline)) {
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
      const RingT* np = rp + (t & 1);
      nra = np[0];
      nrb = np[64];
      __builtin_amdgcn_sched_barrier(0);
    }
    u16x2 upH = as_u16x2(dpp_shr1_zero(botH));
    u16x2 upX = as_u16x2(GOTOH ? dpp_shr1_zero(botX) : dpp_shr1(as_u32(X0), botX));
    upH = top ? H0 : upH;
    upX = top ? X0 : upX;
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
  for (int t = t0; t < nsteps; t += SWK_HALF_UNROLL) {
#pragma unroll
    for (int u = 0; u < SWK_HALF_UNROLL; u += 2) {
      rp = ring_l + ((t + u + 2) & 31);
      step(t + u, true);
      step(t + u + 1, false);
    }
  }
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

template <bool GOTOH>
__global__ void __launch_bounds__(256) score_wave_half(const ScoreArgs a) {
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
    uint4* dst = reinterpret_cast<uint4*>(prof);
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
  uint8_t* cring = prof + (a.pad + 1) * SWK_HALF_LS + SWK_HALF_RING * wave;
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
  const uint32_t G = gridDim.x * 4,
                 g = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (uint32_t)wave);
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
    whole0 = (blockIdx.x - a.split_blocks) * 4 + (uint32_t)wave;
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
        a, prof, cring, lane, 2 * (size_t)unit, tail ? 32 * b0 : 0, head ? 32 * b1 : 0x7FFFFFFF,
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
static size_t wave_half_lds(uint32_t prof_bytes) {
  return (size_t)prof_bytes / 1024 * SWK_HALF_LS + SWK_HALF_RING * 4;
}

template <bool GOTOH>
static hipError_t launch_wave_half(const ScoreArgs& a, uint32_t prof_bytes, hipStream_t st) {
  // 4 waves per block = 8 pairs, sharing one LDS copy of the profile; the split tail's blocks
  // hold every segment's profile
  const size_t blocks = a.wbal_blocks ? (size_t)a.wbal_grid
                                      : a.split_blocks + ((size_t)a.main_pairs + 7) / 8 +
                                            ((size_t)a.tail_pairs * a.split_P + 3) / 4;
  size_t lds = wave_half_lds(prof_bytes);
  if (a.split_blocks) lds = std::max<size_t>(lds, (size_t)a.split_words * 4 * a.split_P);
  if (a.tail_pairs) lds = std::max<size_t>(lds, (size_t)a.split_words * 4 * 4);  // a slice a wave
  auto fn = &score_wave_half<GOTOH>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  if (lds > 160 * 1024) return hipErrorInvalidConfiguration;
#if SWK_STAMPS
  if (g_stamps_host) {  // (measurement builds) the record buffer in tctr, unused here
    ScoreArgs b = a;
    b.tctr = reinterpret_cast<uint32_t*>(g_stamps_host);
    hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(256), (unsigned)lds, st, b);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL(fn, dim3((unsigned)blocks), dim3(256), (unsigned)lds, st, a);
  return hipGetLastError();
}

}  // namespace swk

// Variants compiled in: (R, RB, COL0, PROF, GOTOH, F16).  The host picks R from the query
// length (SWBANK_R / SWBANK_RB override it for tuning).
#define SWK_VARIANTS(X)                                                                       \
  X(16, 4, 0, 0, 0, 0) X(16, 4, 1, 0, 0, 0) X(32, 4, 0, 0, 0, 0) X(32, 4, 1, 0, 0, 0)         \
  X(32, 8, 0, 0, 0, 0) X(64, 4, 0, 0, 0, 0) X(64, 4, 1, 0, 0, 0)                              \
  X(16, 4, 0, 0, 1, 0) X(32, 4, 0, 0, 1, 0) X(64, 4, 0, 0, 1, 0)                              \
  X(16, 4, 0, 1, 0, 0) X(16, 4, 1, 1, 0, 0) X(32, 4, 0, 1, 0, 0) X(32, 4, 1, 1, 0, 0)         \
  X(64, 4, 0, 1, 0, 0) X(64, 4, 1, 1, 0, 0)                                                   \
  X(16, 4, 0, 1, 1, 0) X(32, 4, 0, 1, 1, 0) X(64, 4, 0, 1, 1, 0)                              \
  X(16, 4, 0, 0, 0, 1) X(16, 4, 1, 0, 0, 1) X(32, 4, 0, 0, 0, 1) X(64, 4, 0, 0, 0, 1)         \
  X(16, 4, 0, 0, 1, 1)                                                                        \
  X(16, 4, 0, 1, 0, 1) X(16, 4, 1, 1, 0, 1) X(16, 4, 0, 1, 1, 1) X(32, 4, 0, 0, 1, 1)


extern "C" int swk_has_variant(int R, int RB, int col0, int prof, int gotoh, int f16) {
#define SWK_HAS(RR, BB, C0, PF, GT, FH) \
  if (R == RR && RB == BB && col0 == C0 && prof == PF && gotoh == GT && f16 == FH) return 1;
  SWK_VARIANTS(SWK_HAS)
#undef SWK_HAS
  return 0;
}

extern "C" hipError_t swk_launch_score(int R, int RB, int col0, int prof, int gotoh, int f16,
                                       const uint8_t* res, const uint64_t* offs,
                                       const uint32_t* lens, size_t n, const uint32_t* qtab,
                                       uint32_t nv, uint32_t S, uint32_t O, uint32_t E,
                                       uint32_t PS, uint32_t pad, int W, int32_t* scores,
                                       const void* edge_in, void* edge_out, uint32_t ecols,
                                       int accum, int packed, const uint32_t* idx,
                                       const uint32_t* nidx, uint32_t idx_base,
                                       const uint32_t* ident, int pair, uint32_t pS1,
                                       uint32_t pS2, uint32_t ulen, uint32_t ustride,
                                       uint32_t nq, uint32_t qwords, size_t sstride,
                                       hipStream_t st) {
  if (n == 0) return hipSuccess;
  swk::ScoreArgs a{res,  offs, lens, n,  qtab, nv, S,
                   O,    E,    PS,   pad, scores, static_cast<const uint2*>(edge_in),
                   static_cast<uint2*>(edge_out), ecols, (uint32_t)accum, (uint32_t)packed,
                   idx, nidx, idx_base, ident, pS1, pS2,
                   swk::f16_pair(-(int)(O + E)), swk::f16_pair(-(int)E),
                   swk::f16_pair(-(int)O), nullptr, 0u, 0u, 0};
  a.ulen = ulen;
  a.ustride = ustride;
  a.nq = nq;
  a.qwords = qwords;
  a.sstride = sstride;
  const uint32_t prof_bytes = (pad + 1) * PS;
  if (nq > 1 && pair) {  // several queries, pair tables (PS = one table's bytes)
    // more than 4 waves (a 512-row table): 4-column chunks, so the ring fits beside the table;
    // every segment of a segmented set too (a short last segment reads exactly the edge
    // chunks the one before it wrote)
    if (R == 32 && f16 && !prof && !gotoh && !col0 && (W > 4 || a.edge_in || a.edge_out))
      return swk::launch_score<32, 4, false, false, false, true, true, true, false, 4>(a, W, 0, st);
    if (R == 32 && f16 && !prof && !gotoh && !col0)
      return swk::launch_score<32, 4, false, false, false, true, true, true>(a, W, 0, st);
    return hipErrorInvalidValue;
  }
  if (nq > 1) {  // several queries: row-LUT variants without the column-0 rule
#define SWK_MQ_CASE(RR, GT, FH)                                                                  \
  if (R == RR && RB == 4 && !col0 && !prof && !pair && gotoh == GT && f16 == FH)                 \
    return swk::launch_score<RR, 4, false, false, (GT != 0), (FH != 0), false, true>(a, W, 0, st);
    SWK_MQ_CASE(32, 0, 1) SWK_MQ_CASE(32, 0, 0) SWK_MQ_CASE(16, 0, 1) SWK_MQ_CASE(16, 0, 0)
    SWK_MQ_CASE(16, 1, 1) SWK_MQ_CASE(16, 1, 0) SWK_MQ_CASE(32, 1, 1) SWK_MQ_CASE(32, 1, 0)
#undef SWK_MQ_CASE
    return hipErrorInvalidValue;
  }
  if (pair) {  // PS = pair-table bytes
    if (R == 32 && f16 && !prof && !gotoh && !col0)
      return swk::launch_score<32, 4, false, false, false, true, true>(a, W, 0, st);
    // DNA Gotoh: 8-column chunks while the hand-off ring fits beside the table, else 4 (a
    // 512-row table beside 16 waves).  A segmented query runs every segment with 4: the edge
    // rows one segment writes are exactly the chunks the next one reads
#define SWK_GPAIR(RR)                                                                         \
    if (R == RR && f16 && !prof && gotoh && !col0) {                                          \
      const hipError_t e = a.edge_in || a.edge_out                                            \
          ? hipErrorInvalidConfiguration                                                      \
          : swk::launch_score<RR, 4, false, false, true, true, true>(a, W, 0, st);            \
      if (e != hipErrorInvalidConfiguration) return e;                                        \
      return swk::launch_score<RR, 4, false, false, true, true, true, false, false, 4>(a, W, 0, \
                                                                                         st); \
    }
    SWK_GPAIR(32) SWK_GPAIR(16)
#undef SWK_GPAIR
    return hipErrorInvalidValue;
  }
#define SWK_CASE(RR, BB, C0, PF, GT, FH)                                                      \
  if (R == RR && RB == BB && col0 == C0 && prof == PF && gotoh == GT && f16 == FH)            \
    return swk::launch_score<RR, BB, (C0 != 0), (PF != 0), (GT != 0), (FH != 0)>(a, W,        \
                                                                               prof_bytes, st);
  SWK_VARIANTS(SWK_CASE)
#undef SWK_CASE
  return hipErrorInvalidValue;
}

#if SWK_STAMPS
// (measurement builds) per-wave phase timing of the next tile-kernel launches into p:
// [block][16 waves][16] u64 = entry, exit, active, fill/drain, barrier cycles, HW_ID, chunks,
// XCC, tail state load cycles
extern "C" void swk_set_stamps(void* p) { swk::g_stamps_host = static_cast<uint64_t*>(p); }
#endif

// Balanced chunk ranges (ScoreArgs.bal_*) for the DNA merged f16 pair-table kernel (the
// headline shape): codes one byte each (or ustride / ulen), one query segment of W <= 4 waves.
// swk_bal_slots gives the grid (every resident slot); the host sizes bal_state ((grid + 1) x W
// x (2R + 2) x 64 words) and bal_flag ((grid + 1) x W words, zeroed once); a hand-off wait
// that runs out after poll_limit polls marks *fault (SWK_FAULT_BAL).  plan: grid + 1 entries {tile, chunk, chunk index} (swk_bal_plan_uniform for
// a uniform batch; a ragged batch visited longest first through the device sort's permutation
// idx / nidx / ident passes the sort's, swk_sort_lens with the same grid).
namespace swk {
__global__ void __launch_bounds__(256) bal_plan_uniform(uint4* plan, uint32_t ntiles, uint32_t K,
                                                        uint32_t G) {
  for (uint32_t g = threadIdx.x; g <= G; g += blockDim.x) {
    const uint64_t A = (uint64_t)ntiles * K * g / G;
    plan[g] = make_uint4((uint32_t)(A / K), (uint32_t)(A % K), (uint32_t)A, 0u);
  }
}
}  // namespace swk

// The plan of a uniform batch (ntiles tiles of K chunks, G workgroups): entry g = {tile, chunk,
// chunk index} of chunk floor(g ntiles K / G), g = 0..G (ntiles K < 2^31).
extern "C" hipError_t swk_bal_plan_uniform(void* plan, uint32_t ntiles, uint32_t K, uint32_t G,
                                           hipStream_t st) {
  if (!plan || K == 0 || G == 0 || (uint64_t)ntiles * K >= (1ull << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(swk::bal_plan_uniform, dim3(1), dim3(256), 0, st, static_cast<uint4*>(plan),
                     ntiles, K, G);
  return hipGetLastError();
}

// Resident 4-wave blocks of the two-pairs kernel (the balanced grid) for a profile of
// prof_bytes at PS = 1024 (0 when the occupancy query fails).
extern "C" unsigned swk_wave_half_grid(int gotoh, uint32_t prof_bytes) {
  const void* fn = gotoh ? reinterpret_cast<const void*>(&swk::score_wave_half<true>)
                         : reinterpret_cast<const void*>(&swk::score_wave_half<false>);
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
      hipSuccess)
    return 0;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  const int occ = swk::cached_occupancy(fn, 256, swk::wave_half_lds(prof_bytes), dev, &cus);
  return occ > 0 && cus > 0 ? (unsigned)(occ * cus) : 0u;
}

extern "C" unsigned swk_bal_slots(int W, uint32_t PS, int trim) {
  const void* fn =
      trim ? reinterpret_cast<const void*>(
                 &swk::score_kernel<32, 4, false, false, false, true, true, false, false, 8, true,
                                    true>)
           : reinterpret_cast<const void*>(
                 &swk::score_kernel<32, 4, false, false, false, true, true, false, false, 8, true>);
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
      hipSuccess)
    return 0;
  const size_t lds = (size_t)W * SWB_TILE * 4 + (size_t)(64 + 64 + (W - 1) * 2 * 8 * 64) * 8 + PS;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  const int occ = swk::cached_occupancy(fn, 64 * W, lds, dev, &cus);
  return occ > 0 && cus > 0 ? (unsigned)(occ * cus) : 0u;
}

extern "C" hipError_t swk_launch_pair_bal(const uint8_t* res, const uint64_t* offs,
                                          const uint32_t* lens, size_t n, const uint32_t* qtab,
                                          uint32_t nv, uint32_t S, uint32_t O, uint32_t E,
                                          uint32_t PS, uint32_t pad, int W, int32_t* scores,
                                          uint32_t pS1, uint32_t pS2, uint32_t ulen,
                                          uint32_t ustride, uint32_t* flag, uint32_t* state,
                                          uint32_t gen, unsigned grid, const uint32_t* idx,
                                          const uint32_t* nidx, const uint32_t* ident,
                                          const void* plan, uint32_t* fault, uint32_t poll_limit,
                                          uint32_t stall, int trim, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (W > 4 || !flag || !state || !plan || !fault || poll_limit == 0 || (idx && !nidx))
    return hipErrorInvalidValue;
  swk::ScoreArgs a{res,  offs, lens, n,  qtab, nv, S,
                   O,    E,    PS,   pad, scores, nullptr, nullptr, 0u, 0u, (uint32_t)SWK_PACK_BYTES,
                   idx, nidx, 0u, ident, pS1, pS2,
                   swk::f16_pair(-(int)(O + E)), swk::f16_pair(-(int)E),
                   swk::f16_pair(-(int)O), nullptr, 0u, 0u, 0};
  a.ulen = ulen;
  a.ustride = ustride;
  a.nq = 1;
  a.bal_flag = flag;
  a.bal_state = state;
  a.bal_gen = gen;
  a.bal_plan = static_cast<const uint4*>(plan);
  a.fault = fault;
  a.poll_limit = poll_limit;
  a.stall = stall;
  if (trim)  // (a ragged batch: its tiles' last chunks stop at their last column)
    return swk::launch_score<32, 4, false, false, false, true, true, false, false, 8, true, true>(
        a, W, 0, st, grid);
  return swk::launch_score<32, 4, false, false, false, true, true, false, false, 8, true>(
      a, W, 0, st, grid);
}

// Streamed host batch (the feeder's one-launch path): equal-length targets (ulen codes), or
// ragged ones (ulen = 0: each chunk's region starts with its offsets, lengths and order), the
// chunk records `sc` and layout words dflag (device) / hflag (host), the codes in the device
// buffer `res`; row-LUT or
// pair-table variants without the column-0 rule, one query segment.
extern "C" hipError_t swk_launch_stream(int R, int gotoh, int f16, int pair, const uint8_t* res,
                                        size_t n, uint32_t ulen, const SwkStreamChunk* sc,
                                        const uint32_t* hflag, uint32_t* dflag, uint32_t nsc,
                                        uint32_t* tctr, const uint32_t* qtab, uint32_t nv,
                                        uint32_t S, uint32_t O, uint32_t E, uint32_t PS,
                                        uint32_t pad, int W, int32_t* scores, uint32_t pS1,
                                        uint32_t pS2, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (!sc || !hflag || !dflag || !tctr || nsc == 0) return hipErrorInvalidValue;
  swk::ScoreArgs a{res,  nullptr, nullptr, n, qtab, nv, S, O, E, PS, pad, scores, nullptr, nullptr,
                   0u, 0u, (uint32_t)SWK_PACK_STREAM, nullptr, nullptr, 0u, nullptr, pS1, pS2,
                   swk::f16_pair(-(int)(O + E)), swk::f16_pair(-(int)E),
                   swk::f16_pair(-(int)O), nullptr, 0u, 0u, 0};
  a.ulen = ulen;
  a.sc = sc;
  a.hflag = hflag;
  a.dflag = dflag;
  a.tctr = tctr;
  a.nsc = nsc;
  if (pair) {
    if (R == 32 && f16 && !gotoh)
      return swk::launch_score<32, 4, false, false, false, true, true, false, true>(a, W, 0, st);
    if (R == 32 && f16 && gotoh)
      return swk::launch_score<32, 4, false, false, true, true, true, false, true>(a, W, 0, st);
    if (R == 16 && f16 && gotoh)
      return swk::launch_score<16, 4, false, false, true, true, true, false, true>(a, W, 0, st);
    return hipErrorInvalidValue;
  }
#define SWK_ST_CASE(RR, GT, FH)                                                                  \
  if (R == RR && gotoh == GT && f16 == FH)                                                       \
    return swk::launch_score<RR, 4, false, false, (GT != 0), (FH != 0), false, false, true>(     \
        a, W, 0, st);
  SWK_ST_CASE(32, 0, 1) SWK_ST_CASE(32, 0, 0) SWK_ST_CASE(16, 0, 1) SWK_ST_CASE(16, 0, 0)
  SWK_ST_CASE(16, 1, 1) SWK_ST_CASE(16, 1, 0) SWK_ST_CASE(32, 1, 1) SWK_ST_CASE(32, 1, 0)
#undef SWK_ST_CASE
  return hipErrorInvalidValue;
}

namespace swk {
// Pairs an optimistic f16 pass may have rounded: score > thresh (= 2048 - max s) -> idx list.
__global__ void __launch_bounds__(256) flag_kernel(const int32_t* scores, size_t n,
                                                   int32_t thresh, uint32_t* idx,
                                                   uint32_t* count) {
  const size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (k < n && scores[k] > thresh) idx[atomicAdd(count, 1u)] = (uint32_t)k;
}
}  // namespace swk

namespace swk {
// Bank best hit on the device (≙ ScoreBank_v2 max/vld_max): key = biased score << 32 |
// (2^32 - 1 - index), so one 64-bit max picks the highest score and, among equals, the
// lowest index.  Block-level max in LDS, one atomicMax per block.
__global__ void __launch_bounds__(256) best_kernel(const int32_t* scores, size_t n, size_t base,
                                                   unsigned long long* key) {
  __shared__ unsigned long long red[256];
  unsigned long long m = 0;
  for (size_t k = (size_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (size_t)gridDim.x * 256) {
    const unsigned long long v = ((unsigned long long)((uint32_t)scores[k] ^ 0x80000000u) << 32) |
                                 (0xFFFFFFFFull - (uint32_t)(base + k));
    m = v > m ? v : m;
  }
  red[threadIdx.x] = m;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w && red[threadIdx.x + w] > red[threadIdx.x])
      red[threadIdx.x] = red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicMax(key, red[0]);
}
__global__ void best_finalize(const unsigned long long* key, const uint64_t* ids, uint64_t* out,
                              uint64_t* out_index) {
  const unsigned long long v = *key;
  const uint64_t idx = 0xFFFFFFFFull - (v & 0xFFFFFFFFull);
  out[0] = ids ? ids[idx] : idx;
  out[1] = (uint64_t)(int64_t)(int32_t)((uint32_t)(v >> 32) ^ 0x80000000u);
  if (out_index) *out_index = idx;
}
}  // namespace swk

// Fold scores[0, n) (batch positions base + k) into the 64-bit best key (zeroed by the caller
// before the first part); few blocks, so the contended atomicMax stays cheap (2048 blocks cost
// ~25 us on 1 M scores, 256 about 3).
extern "C" hipError_t swk_best_part(const int32_t* scores, size_t n, size_t base,
                                    unsigned long long* key, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const size_t blocks = std::min<size_t>((n + 2047) / 2048, 256);
  hipLaunchKernelGGL(swk::best_kernel, dim3((unsigned)blocks), dim3(256), 0, st, scores, n, base,
                     key);
  return hipGetLastError();
}

// out[0] = best id (ids ? ids[index] : index), out[1] = best score (sign-extended), *out_index
// (optional) = its index, from the key.
extern "C" hipError_t swk_best_finalize(const unsigned long long* key, const uint64_t* ids,
                                        uint64_t* out, uint64_t* out_index, hipStream_t st) {
  hipLaunchKernelGGL(swk::best_finalize, dim3(1), dim3(1), 0, st, key, ids, out, out_index);
  return hipGetLastError();
}

// out[0] = best id, out[1] = best score (sign-extended), *out_index (optional) = its index;
// key: 8 bytes of device scratch.
extern "C" hipError_t swk_best_hit(const int32_t* scores, const uint64_t* ids, size_t n,
                                   unsigned long long* key, uint64_t* out, uint64_t* out_index,
                                   hipStream_t st) {
  hipError_t e = hipMemsetAsync(key, 0, sizeof(*key), st);
  if (e == hipSuccess) e = swk_best_part(scores, n, 0, key, st);
  if (e == hipSuccess) e = swk_best_finalize(key, ids, out, out_index, st);
  return e;
}

// ---- the deal of a multi-device bank's device batch (swbank_multi.hip) -------------------
namespace swk {
__device__ __forceinline__ size_t deal_target(const uint32_t* perm, bool id, size_t p) {
  return id ? p : (size_t)perm[p];
}
// one wave per position (grid-stride): the target's bytes, lane-strided, to its device's slot
__global__ void __launch_bounds__(256) deal_gather(const uint8_t* res, const uint64_t* offs,
                                                   const uint32_t* lens, const uint32_t* perm,
                                                   const uint32_t* ident, size_t n,
                                                   const SwkDeal dl) {
  const int lane = threadIdx.x & 63;
  const size_t w0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  const bool id = !perm || (ident && *ident != 0);
  for (size_t p = w0; p < n; p += nw) {
    const size_t t = deal_target(perm, id, p);
    const unsigned d = (unsigned)(p % dl.D);
    const size_t i = p / dl.D;
    const uint32_t L = lens[t];
    const uint8_t* src = res + offs[t];
    uint8_t* dst = dl.codes[d] + i * dl.stride;
    for (uint32_t j = lane; j < L; j += 64) dst[j] = src[j];
    if (lane == 0) {
      dl.offs[d][i] = (unsigned long long)i * dl.stride;
      dl.lens[d][i] = L;
    }
  }
}
__global__ void __launch_bounds__(256) deal_scatter(const uint32_t* perm, const uint32_t* ident,
                                                    size_t n, unsigned nq, size_t sstride,
                                                    const SwkDeal dl, int32_t* out) {
  const bool id = !perm || (ident && *ident != 0);
  const size_t total = n * nq;
  for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < total;
       x += (size_t)gridDim.x * blockDim.x) {
    const size_t q = x / n, p = x % n;
    const unsigned d = (unsigned)(p % dl.D);
    out[q * sstride + deal_target(perm, id, p)] = dl.scores[d][q * dl.cnt[d] + p / dl.D];
  }
}
}  // namespace swk

extern "C" hipError_t swk_deal_gather(const uint8_t* res, const uint64_t* offs,
                                      const uint32_t* lens, const uint32_t* perm,
                                      const uint32_t* ident, size_t n, const SwkDeal* deal,
                                      hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (!deal || deal->D == 0 || deal->D > SWK_DEAL_MAX || deal->stride == 0) return hipErrorInvalidValue;
  const size_t blocks = std::min<size_t>((n + 3) / 4, 8192);
  hipLaunchKernelGGL(swk::deal_gather, dim3((unsigned)blocks), dim3(256), 0, st, res, offs, lens,
                     perm, ident, n, *deal);
  return hipGetLastError();
}

extern "C" hipError_t swk_deal_scatter(const uint32_t* perm, const uint32_t* ident, size_t n,
                                       unsigned nq, size_t sstride, const SwkDeal* deal,
                                       int32_t* out, hipStream_t st) {
  if (n == 0 || nq == 0) return hipSuccess;
  if (!deal || deal->D == 0 || deal->D > SWK_DEAL_MAX) return hipErrorInvalidValue;
  const size_t blocks = std::min<size_t>((n * nq + 255) / 256, 8192);
  hipLaunchKernelGGL(swk::deal_scatter, dim3((unsigned)blocks), dim3(256), 0, st, perm, ident, n,
                     nq, sstride, *deal, out);
  return hipGetLastError();
}

extern "C" hipError_t swk_flag_high(const int32_t* scores, size_t n, int32_t thresh,
                                    uint32_t* idx, uint32_t* count, hipStream_t st) {
  hipError_t e = hipMemsetAsync(count, 0, sizeof(uint32_t), st);
  if (e != hipSuccess || n == 0) return e;
  hipLaunchKernelGGL(swk::flag_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     scores, n, thresh, idx, count);
  return hipGetLastError();
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
        (pairs + 1) / 2 < 4ull * split->wbal_grid || pairs > 0xFFFFFFFFull)
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
    return gotoh ? swk::launch_wave_half<true>(a, prof_bytes, st)
                 : swk::launch_wave_half<false>(a, prof_bytes, st);
  }
#define SWK_WCASE(KK, C0, PF, GT)                                                         \
  if (K == KK && col0 == C0 && prof == PF && gotoh == GT)                                 \
    return f16 ? swk::launch_wave<KK, (C0 != 0), (PF != 0), (GT != 0), true>(a, prof_bytes, st) \
               : swk::launch_wave<KK, (C0 != 0), (PF != 0), (GT != 0), false>(a, prof_bytes, st);
  SWK_WAVE_VARIANTS(SWK_WCASE)
#undef SWK_WCASE
  return hipErrorInvalidValue;
}

// ========================================================================================
// int32 kernel: exact scores past the 16-bit lanes (no bound on the score).  The u16 and f16
// passes are exact for every pair whose computed score stays <= 65535 - max(s) (resp. 2048 -
// max(s)): the first cell that would leave the lane range has an exact diagonal M above that
// threshold (a gap value is at most an earlier, exact H minus a penalty), and the running max
// keeps it.  So a batch past the 16-bit bound is scored by the 16-bit kernels as usual and the
// pairs above 65535 - max(s) are re-scored here (an index list, like the f16 -> u16 re-score).
//
// One wave per pair; strips of 256 query rows, lane l owns rows [4l, 4l+4) of a strip (the
// wave kernel's anti-diagonal walk: step t, lane l computes column t - l).  The strip's bottom
// row {H, T|F} goes to the next strip through a per-wave HBM scratch row (ping-pong, 64
// columns per coalesced load / store, readlane + a lane select per step).  Substitution scores come
// from a per-strip profile: for every letter, lane l's 4 rows as int16 (uint2), staged in the
// wave's own LDS slice (each lane reads only its own entries: no barrier).  Merged gaps apply
// the HDL's first-column rule always (it changes nothing unless max(s) > o + e), in the
// clamped form of the f16 kernels:
//   M = max(0, Hdiag + s)   I = j ? max(Tup, Tleft) : 0   H = max(M, I)   T = max(0, M-o-e, I-e)
// Gotoh (E, F one step ahead, floored at 0):
//   H = max(0, Hdiag + s, E, F)   HN = H - o - e   E' = max(0, HN, E - e)   F' = max(0, HN, F - e)
namespace swk {
constexpr int I32_K = 4, I32_LETTERS = 25;  // rows per lane; profile letters incl. padding

struct I32Args {
  const uint8_t* res;
  const uint64_t* offs;
  const uint32_t* lens;
  size_t n;
  uint32_t packed;
  const uint32_t* idx;   // optional: positions [0, min(n, *nidx - idx_base)) score idx[k]
  const uint32_t* nidx;
  uint32_t idx_base;
  const uint2* prof;     // [strip][letter 0..pad][lane] 4 x int16 (rows 4l..4l+3)
  uint32_t nstrips, qlen, pad, O, E;
  int32_t* scores;
  uint2* scratch;        // per wave: 2 x scols uint2
  uint32_t scols;
};

__device__ __forceinline__ uint32_t i32_code(const uint8_t* p, uint32_t c, uint32_t packed) {
  if (packed == SWK_PACK_BYTES) return p[c];
  if (packed == SWK_PACK_NIBBLE) return (p[c >> 1] >> (4 * (c & 1))) & 15u;
  return (p[c >> 2] >> (2 * (c & 3))) & 3u;  // records, 2-bit stream
}

__device__ __forceinline__ int32_t i32_lane0(int32_t inj, int32_t v) {  // wave_shr:1
  return __builtin_amdgcn_update_dpp(inj, v, 0x138, 0xF, 0xF, false);
}

template <bool GOTOH>
__global__ void __launch_bounds__(256) score_i32(const I32Args a) {
  __shared__ uint2 lp[4][I32_LETTERS][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const size_t gw = (size_t)blockIdx.x * 4 + wave, GW = (size_t)gridDim.x * 4;
  size_t n = a.n;
  if (a.idx) {
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(*a.nidx);
    n = cnt > a.idx_base ? min(a.n, (size_t)(cnt - a.idx_base)) : 0;
  }
  uint2* const scr[2] = {a.scratch + gw * 2 * a.scols, a.scratch + gw * 2 * a.scols + a.scols};
  const int32_t oe = (int32_t)(a.O + a.E), e = (int32_t)a.E;
  const uint32_t pad = a.pad;
  uint2 (&mine)[I32_LETTERS][64] = lp[wave];
  for (size_t p = gw; p < n; p += GW) {
    const size_t t = a.idx ? a.idx[p] : p;
    const uint8_t* tp;
    uint32_t L;
    if (a.packed == SWK_PACK_RECORDS) {
      tp = a.res + t * SWB_RECORD + 6;
      L = record_len(a.res + t * SWB_RECORD);
    } else {
      L = a.lens[t];
      tp = a.res + (L ? a.offs[t] : 0);
    }
    L = __builtin_amdgcn_readfirstlane(L);
    int32_t best = 0;
    for (uint32_t s = 0; s < a.nstrips && L; ++s) {
      for (uint32_t c = 0; c <= pad; ++c) mine[c][lane] = a.prof[((size_t)s * (pad + 1) + c) * 64 + lane];
      int32_t vmask[I32_K];
#pragma unroll
      for (int k = 0; k < I32_K; ++k)
        vmask[k] = s * 256u + (uint32_t)lane * I32_K + k < a.qlen ? -1 : 0;
      const bool seg_in = s > 0, seg_out = s + 1 < a.nstrips;
      const uint2* ein = scr[(s + 1) & 1];
      uint2* eout = scr[s & 1];
      int32_t H[I32_K], X[I32_K];
#pragma unroll
      for (int k = 0; k < I32_K; ++k) H[k] = X[k] = 0;
      int32_t botH = 0, botX = 0, prevUpH = 0;
      uint32_t code = pad, buf = pad;
      uint2 ebuf = make_uint2(0u, 0u), obuf = make_uint2(0u, 0u);
      const uint32_t nsteps = L + 63;
      for (uint32_t st = 0; st < nsteps; ++st) {
        if ((st & 63) == 0) {  // the next 64 columns: codes (and the previous strip's row)
          const uint32_t c = st + lane;
          buf = c < L ? min(i32_code(tp, c, a.packed), pad) : pad;
          if (seg_in) ebuf = c < L ? ein[c] : make_uint2(0u, 0u);
        }
        const uint32_t j = st - (uint32_t)lane;  // this lane's column (wraps when not started)
        code = (uint32_t)i32_lane0((int32_t)__builtin_amdgcn_readlane(buf, st & 63), (int32_t)code);
        const int32_t upH = i32_lane0(seg_in ? (int32_t)__builtin_amdgcn_readlane(ebuf.x, st & 63) : 0, botH);
        const int32_t upX = i32_lane0(seg_in ? (int32_t)__builtin_amdgcn_readlane(ebuf.y, st & 63) : 0, botX);
        const uint2 w = mine[code][lane];
        const int32_t sc[I32_K] = {(int32_t)(w.x << 16) >> 16, (int32_t)w.x >> 16,
                                   (int32_t)(w.y << 16) >> 16, (int32_t)w.y >> 16};
        if (j < L) {  // active: column j of the lane's 4 rows
          int32_t diag = prevUpH, up = upH, ux = upX;
#pragma unroll
          for (int k = 0; k < I32_K; ++k) {
            const int32_t D = diag + sc[k];
            diag = H[k];
            if constexpr (GOTOH) {
              const int32_t h = max(max(D, 0), max(X[k], ux));
              const int32_t hn = h - oe;
              X[k] = max(max(hn, 0), X[k] - e);  // E of (row, j+1)
              ux = max(max(hn, 0), ux - e);      // F of (row+1, j)
              H[k] = h;
              best = max(best, h & vmask[k]);
            } else {
              const int32_t M = max(D, 0);
              const int32_t I = j == 0 ? 0 : max(ux, X[k]);
              const int32_t h = max(M, I);
              ux = max(max(M - oe, I - e), 0);   // T: what the right and lower cells read
              X[k] = ux;
              H[k] = h;
              best = max(best, h & vmask[k]);
            }
            (void)up;
          }
          botH = H[I32_K - 1];
          botX = ux;
        }
        prevUpH = upH;
        if (seg_out) {  // lane 63's bottom row of column st - 63 -> eout
          const uint32_t c = st - 63;
          if (st >= 63) {
            const int32_t vh = __builtin_amdgcn_readlane(botH, 63);
            const int32_t vx = __builtin_amdgcn_readlane(botX, 63);
            const bool here = (uint32_t)lane == (c & 63);
            obuf.x = here ? (uint32_t)vh : obuf.x;
            obuf.y = here ? (uint32_t)vx : obuf.y;
            if ((c & 63) == 63 || c + 1 == L) {
              const uint32_t col = (c & ~63u) + lane;
              if (col < L) eout[col] = obuf;
            }
          }
        }
      }
      // the next strip's lane 0 reads these columns (same wave, same CU and L1): a
      // workgroup-scope fence orders the stores before those loads (no L2 write-back)
      if (seg_out) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) best = max(best, __shfl_xor(best, off));
    if (lane == 0) a.scores[t] = best;
  }
}
}  // namespace swk

// Waves to launch for n pairs of at most scols columns: one pair per wave at a time, up to
// 16 waves per CU, within the scratch budget (2 x scols x 8 B per wave).
extern "C" size_t swk_i32_waves(size_t n, uint32_t scols, size_t budget_bytes) {
  const size_t per = (size_t)std::max(scols, 1u) * 2 * sizeof(uint2);
  size_t w = std::min<size_t>(n, 256 * 16);
  w = std::min(w, std::max<size_t>(4, budget_bytes / per));
  return (w + 3) / 4 * 4;
}

extern "C" hipError_t swk_launch_i32(int gotoh, const uint8_t* res, const uint64_t* offs,
                                     const uint32_t* lens, size_t n, int packed,
                                     const uint32_t* idx, const uint32_t* nidx, uint32_t idx_base,
                                     const void* prof, uint32_t nstrips, uint32_t qlen,
                                     uint32_t pad, uint32_t O, uint32_t E, int32_t* scores,
                                     void* scratch, uint32_t scols, size_t waves, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (pad + 1 > (uint32_t)swk::I32_LETTERS || waves == 0 || waves % 4) return hipErrorInvalidValue;
  const swk::I32Args a{res, offs, lens, n, (uint32_t)packed, idx, nidx, idx_base,
                       static_cast<const uint2*>(prof), nstrips, qlen, pad, O, E, scores,
                       static_cast<uint2*>(scratch), scols};
  if (gotoh)
    hipLaunchKernelGGL(swk::score_i32<true>, dim3((unsigned)(waves / 4)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(swk::score_i32<false>, dim3((unsigned)(waves / 4)), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ========================================================================================
// Longest-first visiting order of a device batch (sw_score_batch_device with ragged lengths):
// the PrioEncoder's feed order (ScoreBank_v2.v:142-148) so that each 128-target tile holds
// similar lengths.  A counting sort over length bins (bin = (max_len - len) >> shift, at most
// 2048 bins; targets within a bin differ by < 2^shift codes, and the order inside a bin is
// free: scores are written at input positions).  hist: global bin counts; scan: exclusive
// offsets in place + perm_n = n; scatter: per block, LDS bin counts, one global atomic per
// non-empty bin reserves the block's range, LDS atomics place the elements.
namespace swk {
constexpr int SORT_BINS = 2048, SORT_BLOCK = 1024, SORT_ITEMS = 8;

__device__ __forceinline__ uint32_t sort_bin(uint32_t len, uint32_t max_len, uint32_t shift) {
  return (max_len - min(len, max_len)) >> shift;
}

// h[bin] += 1 for the active lanes; returns the lane's slot (the old value + its rank among
// the lanes of its bin).  A wave whose lanes share one bin (uniform or already sorted lengths)
// adds once from its first lane; otherwise every lane adds its own (distinct bins rarely
// collide, and 64 serialised atomics on one address were the cost this avoids).
__device__ __forceinline__ uint32_t wave_bin_add(uint32_t* h, uint32_t bin, bool active) {
  const int lane = threadIdx.x & 63;
  const uint64_t act = __ballot(active);
  if (!act) return 0;
  const int leader = __builtin_ctzll(act);
  const uint32_t lb = __builtin_amdgcn_readlane(bin, leader);
  const uint64_t m = __ballot(active && bin == lb);
  if (m == act) {
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&h[lb], (uint32_t)__builtin_popcountll(m));
    base = __builtin_amdgcn_readlane(base, leader);
    return base + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1));
  }
  return active ? atomicAdd(&h[bin], 1u) : 0u;
}

// scratch: hist[SORT_BINS] | done[2] (block counters), zero between calls: the last block of
// a call's last kernel zeroes them again, so no memset per call.
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Histogram of the bins, then (the last block to finish) exclusive offsets in place,
// *perm_n = n, and *ident = 1 when at most one bin is non-empty (the caller's order is kept:
// the scatter and the score kernel's indirection are skipped, and the hist is zeroed here).
// plan != nullptr (balanced chunk ranges of a ragged batch, shift == 0 so a bin is one length):
// the last block also writes, for g = 0..G, plan[g] = {tile, chunk, floor(g A / G), 0} of chunk
// floor(g A / G) of
// the longest-first tile sequence (A = its chunk count, tile t's chunk count ceil(len / 8) of the
// bin holding its first, longest target), i.e. where each of the score kernel's G workgroups
// starts.
__global__ void __launch_bounds__(SORT_BLOCK) sort_hist_scan(const uint32_t* lens, size_t n,
                                                             uint32_t max_len, uint32_t shift,
                                                             uint32_t nb, uint32_t* hist,
                                                             uint32_t* perm_n, uint32_t* ident,
                                                             uint4* plan, uint32_t G) {
  __shared__ uint32_t h[SORT_BINS];
  __shared__ uint32_t part[SORT_BLOCK];
  __shared__ int last;
  for (uint32_t i = threadIdx.x; i < nb; i += SORT_BLOCK) h[i] = 0;
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * SORT_BLOCK * SORT_ITEMS;
#pragma unroll
  for (int it = 0; it < SORT_ITEMS; ++it) {
    const size_t k = base + (size_t)it * SORT_BLOCK + threadIdx.x;
    (void)wave_bin_add(h, k < n ? sort_bin(lens[k], max_len, shift) : 0u, k < n);
  }
  __syncthreads();
  // hand-off (MI355X_MICROARCH.md, inter-workgroup visibility): the bins are written by
  // device-scope atomics, each wave waits for its own, the last block (told by the counter's
  // returned value) reads them with sc1 loads; no L2 write-back fence (__threadfence() here
  // cost ~35 us per call)
  for (uint32_t i = threadIdx.x; i < nb; i += SORT_BLOCK)
    if (h[i]) atomicAdd(&hist[i], h[i]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t* done = hist + SORT_BINS;
  if (threadIdx.x == 0) last = atomicAdd(&done[0], 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  // each thread owns 2 consecutive bins (nb <= 2048)
  const uint32_t i0 = threadIdx.x * 2;
  const uint32_t a = i0 < nb ? ld_agent(&hist[i0]) : 0u;
  const uint32_t c = i0 + 1 < nb ? ld_agent(&hist[i0 + 1]) : 0u;
  const int used = __syncthreads_count((a != 0) + (c != 0) > 0 ? 1 : 0) +
                   __syncthreads_count(a != 0 && c != 0 ? 1 : 0);
  part[threadIdx.x] = a + c;
  __syncthreads();
  for (uint32_t off = 1; off < SORT_BLOCK; off <<= 1) {  // inclusive Hillis-Steele scan
    const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  const uint32_t ex = part[threadIdx.x] - (a + c);
  const bool one = used <= 1;
  if (i0 < nb) hist[i0] = one ? 0u : ex;
  if (i0 + 1 < nb) hist[i0 + 1] = one ? 0u : ex + a;
  if (threadIdx.x == 0) {
    *perm_n = (uint32_t)n;
    *ident = one ? 1u : 0u;
    done[0] = 0;
  }
  if (!plan) return;
  // tiles whose first position falls in bin b: [ceil(off_b / 128), ceil((off_b + cnt_b) / 128)),
  // each of K_b = max(1, ceil(len_b / 8)) chunks (the bin's length is the tile's longest);
  // h[] <- first tile of the bin, part[] <- chunks before the bin's first tile (exclusive scan
  // of tiles x K over the bins, 2 bins per thread)
  const auto kb = [&](uint32_t b) { return max(1u, ((max_len - b) + 7u) / 8u); };
  const uint32_t t0 = (ex + 127) / 128, t1 = (ex + a + 127) / 128, t2 = (ex + a + c + 127) / 128;
  const uint32_t w0 = i0 < nb ? (t1 - t0) * kb(i0) : 0u, w1 = i0 + 1 < nb ? (t2 - t1) * kb(i0 + 1) : 0u;
  __syncthreads();
  part[threadIdx.x] = w0 + w1;
  if (i0 < nb) h[i0] = t0;
  if (i0 + 1 < nb) h[i0 + 1] = t1;
  __syncthreads();
  for (uint32_t off = 1; off < SORT_BLOCK; off <<= 1) {
    const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  const uint32_t total = part[SORT_BLOCK - 1];  // chunks of all tiles
  // chunks before bin b: part[b / 2 - 1] (inclusive prefix of the pairs before) plus, for an odd
  // b, the even bin's weight
  const auto before = [&](uint32_t b) -> uint32_t {
    const uint32_t pr = b >= 2 ? part[b / 2 - 1] : 0u;
    if ((b & 1) == 0) return pr;
    return pr + ((b < nb ? h[b] : (uint32_t)((n + 127) / 128)) - h[b - 1]) * kb(b - 1);
  };
  const uint32_t ntiles = (uint32_t)((n + 127) / 128);
  for (uint32_t g = threadIdx.x; g <= G; g += SORT_BLOCK) {
    const uint32_t A = (uint32_t)((uint64_t)total * g / G);
    uint4 r = make_uint4(ntiles, 0u, A, 0u);
    if (A < total) {
      uint32_t lo = 0, hi = nb;  // the last bin with before(bin) <= A (and a tile in it)
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (before(mid) <= A) lo = mid; else hi = mid;
      }
      while (lo + 1 < nb && before(lo + 1) <= A) ++lo;  // (bins without tiles have no width)
      const uint32_t d = A - before(lo), K = kb(lo);
      r = make_uint4(h[lo] + d / K, d % K, A, 0u);
    }
    plan[g] = r;
  }
}

__global__ void __launch_bounds__(SORT_BLOCK) sort_scatter(const uint32_t* lens, size_t n,
                                                           uint32_t max_len, uint32_t shift,
                                                           uint32_t nb, uint32_t* offs,
                                                           uint32_t* perm, const uint32_t* ident) {
  if (__builtin_amdgcn_readfirstlane(*ident)) return;  // one length bin: order unchanged
  __shared__ uint32_t h[SORT_BINS];
  __shared__ int last;
  for (uint32_t i = threadIdx.x; i < nb; i += SORT_BLOCK) h[i] = 0;
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * SORT_BLOCK * SORT_ITEMS;
  uint32_t bin[SORT_ITEMS], slot[SORT_ITEMS];
#pragma unroll
  for (int it = 0; it < SORT_ITEMS; ++it) {
    const size_t k = base + (size_t)it * SORT_BLOCK + threadIdx.x;
    bin[it] = k < n ? sort_bin(lens[k], max_len, shift) : 0u;
    slot[it] = wave_bin_add(h, bin[it], k < n);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nb; i += SORT_BLOCK)  // reserve this block's ranges
    if (h[i]) h[i] = atomicAdd(&offs[i], h[i]);
  __syncthreads();
#pragma unroll
  for (int it = 0; it < SORT_ITEMS; ++it) {
    const size_t k = base + (size_t)it * SORT_BLOCK + threadIdx.x;
    const uint32_t pos = h[bin[it]] + slot[it];
    if (k < n && pos < n) perm[pos] = (uint32_t)k;
  }
  // the last block zeroes the offsets and the counters for the next call (every block's
  // offset atomics returned before its counter add; the zeros reach the next call's kernels
  // through the kernel boundary)
  __syncthreads();
  uint32_t* done = offs + SORT_BINS;
  if (threadIdx.x == 0) last = atomicAdd(&done[1], 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  for (uint32_t i = threadIdx.x; i < nb; i += SORT_BLOCK) offs[i] = 0;
  if (threadIdx.x == 0) done[1] = 0;
}
}  // namespace swk

// perm[0, n) <- target numbers longest first, *perm_n <- n, *ident <- 1 when the lengths
// share one bin (perm then left unwritten: visit in input order); scratch:
// swk_sort_scratch_bytes(), zero on entry and on return.
extern "C" hipError_t swk_sort_lens(const uint32_t* lens, size_t n, uint32_t max_len,
                                    uint32_t* perm, uint32_t* perm_n, uint32_t* ident,
                                    uint32_t* scratch, hipStream_t st, void* plan, unsigned G) {
  if (n == 0 || n > 0xFFFFFFFFull) return hipErrorInvalidValue;
  uint32_t shift = 0;
  while ((max_len >> shift) >= (uint32_t)swk::SORT_BINS) ++shift;
  const uint32_t nb = (max_len >> shift) + 1;
  if (plan && (shift != 0 || G == 0)) return hipErrorInvalidValue;
  const unsigned blocks =
      (unsigned)((n + swk::SORT_BLOCK * swk::SORT_ITEMS - 1) / (swk::SORT_BLOCK * swk::SORT_ITEMS));
  hipLaunchKernelGGL(swk::sort_hist_scan, dim3(blocks), dim3(swk::SORT_BLOCK), 0, st, lens, n,
                     max_len, shift, nb, scratch, perm_n, ident, static_cast<uint4*>(plan), G);
  hipLaunchKernelGGL(swk::sort_scatter, dim3(blocks), dim3(swk::SORT_BLOCK), 0, st, lens, n,
                     max_len, shift, nb, scratch, perm, ident);
  return hipGetLastError();
}

// Bytes of sort scratch (zeroed once at allocation; the kernels leave it zeroed).
extern "C" size_t swk_sort_scratch_bytes(void) { return (swk::SORT_BINS + 2) * sizeof(uint32_t); }
