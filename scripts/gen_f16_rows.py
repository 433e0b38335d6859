#!/usr/bin/env python3
"""Generate csrc/swbank_f16_rows.inc: asm text for one 8-row block of the f16 tile-kernel
column, for both gap models and both substitution lookups.

Merged gap matrix (the ScoreBank PE), scores as f16 multiples of 2^-11 so that the packed
add's [0, 1] clamp is max(0, x); per row, with M = max(0, H(i-1,j-1) + s) already computed:

    s'  = v_perm(...)                 substitution word of the next row (VOP3; LUT/profile)
    MO  = M + (-o)
    T   = X(prev row) + (-e)   -> Tl  T of the previous row (= G - e: what the right and lower
                                      cells read), written one group late
    M'  = clamp(Hl(old) + s')         next row's M
    H   = max(M, Tup, Tl)      -> Hl  (= max(M, I), I = max(Tup, Tl))
    X   = max(MO, Tup, Tl)            G = max(M - o, I)
    best = max(best, H(prev row), H)  every second row

Gotoh (ssearch36), E and F one step ahead and floored at 0:

    s'  = v_perm(...)
    D'  = Hl(old) + s'
    H   = max(D, El, F)      -> Hl
    EN  = El + (-e)
    HN  = H + (-o-e)
    FN  = F + (-e)
    El  = max(0, HN, EN)
    F   = max(0, HN, FN)              (F of the next row)
    best = max(best, H(prev row), H)  every second row

Lookups: LUT (DNA) `v_perm_b32 s, nv, lut[row], sel` with the row's LUT word in an SGPR;
profile (any alphabet, 2-byte f16 entries) `v_perm_b32 s, hi[w], lo[w], selk` with the two
target letters' profile words in VGPRs and a per-parity selector in an SGPR.

Mode "F" (profile, 4-byte words {s, 1.0} per letter and row): no lookup instruction at all.
The next row's diagonal add is one packed FMA that takes target A's entry from the low half of
A's word and target B's from the low half of B's word, the 1.0 in the other word's high half
being the multiplier:
    v_pk_fma_f16 D, a, b, h op_sel:[0,1,0] op_sel_hi:[1,0,1]
    D.lo = a.lo * b.hi + h.lo = sA + h.lo      D.hi = a.hi * b.lo + h.hi = sB + h.hi
(exact: every operand is an f16 multiple of 2^-11 in [-1, 1], one rounding; the clamp modifier
is max(0, x) as for the add; scripts/ubench/fma_opsel.hip checks both and the issue rate, which
equals v_pk_add_f16's).  So a profile row costs 7.5 VALU (Gotoh) / 5.5 (merged) per 2 cells like
the DNA letter-pair table, without a table per letter pair.

No two dependent packed (VOP3P) ops are adjacent (gfx950 needs a wait state between them;
v_perm_b32 -> VOP3P needs none), so a block needs no s_nop inside; LLVM adds one wait state
per asm block.  D alternates between Da/Db by row parity.  The last block of a column ends
with a row that has no successor: `s_nop 0` stands in for its next-row add.
usage: python scripts/gen_f16_rows.py   (rewrites the .inc)
"""
import os

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "smith-waterman-fpga-module_amd", "csrc", "swbank_f16_rows.inc")


def perm(mode, i):
    """substitution word of block row i+1 into S1"""
    if mode == "L":
        return f"v_perm_b32 %[S1], %[nv], %[tb{i}], %[sel]"
    w = (i + 1) // 2
    k = "%[selB]" if (i + 1) % 2 else "%[selA]"
    return f"v_perm_b32 %[S1], %[hi{w}], %[lo{w}], {k}"


FMA_SEL = "op_sel:[0,1,0] op_sel_hi:[1,0,1]"


def next_d(mode, i, dnext, clamp):
    """the diagonal add of block row i + 1 (into dnext) for mode F / pair / L,P (S1)"""
    c = " clamp" if clamp else ""
    if mode == "F":
        return [f"v_pk_fma_f16 {dnext}, %[fa{i}], %[fb{i}], %[h{i}] {FMA_SEL}{c}"]
    if mode == "pair":
        return [f"v_pk_add_f16 {dnext}, %[h{i}], %[p{i}]{c}"]
    return [perm(mode, i), f"v_pk_add_f16 {dnext}, %[h{i}], %[S1]{c}"]


def merged_block(mode, zdown, last, nrows=8):
    """Merged gap matrix with the clamp modifier: values are f16 multiples of 2^-11, so the
    [0, 1] clamp of v_pk_add_f16 is max(0, x) on everything the exact path reaches, and the
    diagonal add yields M = max(0, H(i-1,j-1) + s) directly.  Then I = max(Tup, Tl) never has
    to be formed on its own: H = max(M, Tup, Tl) and G = max(M - o, Tup, Tl) are one max3 each
    and T = G - e.  5.5 VALU per 2 cells (+ the substitution lookup).  T of row i is written
    one group late (after the next row's M - o), so no two dependent packed ops are adjacent.
    mode "L"/"P": perm lookups into S1; "pair": ready-made words p{i} (no lookup)."""
    out = []
    for i in range(nrows):
        dcur, dnext = ("%[Da]", "%[Db]") if i % 2 == 0 else ("%[Db]", "%[Da]")
        up = "%[up]" if i == 0 else ("%[noe]" if zdown else f"%[t{i - 1}]")
        final = last and i == nrows - 1
        if final:
            nxt = ["s_nop 0"]
        else:
            nd = next_d(mode, i, dnext, True)
            out += nd[:-1]  # (the perm of the L / P lookups)
            nxt = nd[-1:]
        if i == 0:
            out += nxt
            out.append(f"v_pk_add_f16 %[DN], {dcur}, %[no]")
        else:
            out.append(f"v_pk_add_f16 %[DN], {dcur}, %[no]")
            out.append(f"v_pk_add_f16 %[t{i - 1}], %[X], %[ne]")
            out += nxt
        out.append(f"v_pk_maximum3_f16 %[h{i}], {dcur}, {up}, %[t{i}]")
        out.append(f"v_pk_maximum3_f16 %[X], %[DN], {up}, %[t{i}]")
        if i % 2 == 1:
            out.append(f"v_pk_maximum3_f16 %[best], %[best], %[h{i - 1}], %[h{i}]")
    if nrows % 2 == 1:
        out.append("s_nop 0")
    out.append(f"v_pk_add_f16 %[t{nrows - 1}], %[X], %[ne]")
    return out


def gotoh_block(mode, last, nrows=8):
    """mode "L"/"P": perm lookups into S1; "pair": ready-made words p{i} (no lookup)."""
    out = []
    for i in range(nrows):
        dcur, dnext = ("%[Da]", "%[Db]") if i % 2 == 0 else ("%[Db]", "%[Da]")
        final = last and i == nrows - 1
        if final:
            out.append("s_nop 0")
        else:
            out += next_d(mode, i, dnext, False)
        out.append(f"v_pk_maximum3_f16 %[h{i}], {dcur}, %[t{i}], %[F]")
        out.append(f"v_pk_add_f16 %[EN], %[t{i}], %[ne]")
        out.append(f"v_pk_add_f16 %[HN], %[h{i}], %[noe]")
        out.append("v_pk_add_f16 %[FN], %[F], %[ne]")
        out.append(f"v_pk_maximum3_f16 %[t{i}], 0, %[HN], %[EN]")
        out.append("v_pk_maximum3_f16 %[F], 0, %[HN], %[FN]")
        if i % 2 == 1:
            out.append(f"v_pk_maximum3_f16 %[best], %[best], %[h{i - 1}], %[h{i}]")
    return out


def pair_block(first, last, nrows=8):
    """Pair-profile block (DNA, merged gaps): the substitution words of both targets come
    ready-made from an LDS table of letter pairs, word p{i} = s(row i+1) for (lo, hi), so
    there is no v_perm per row: 5.5 VALU per 2 cells.  Da carries M of the block's first row
    in and of the next block's first row out; the first block computes it from dg + pw."""
    out = ["v_pk_add_f16 %[Da], %[dg], %[pw] clamp"] if first else []
    return out + merged_block("pair", False, last, nrows)

def pair_gotoh_block(first, last, nrows=8):
    """Pair-profile block, Gotoh (DNA): as gotoh_block with the substitution words p{i} from
    the letter-pair table, 7.5 VALU per 2 cells instead of 8.5.  F runs down the column in
    %[F]; the first block computes row 0's D from dg + pw (the clamp is harmless: H is the max
    of D and the floored E, F)."""
    out = ["v_pk_add_f16 %[Da], %[dg], %[pw] clamp"] if first else []
    return out + gotoh_block("pair", last, nrows)


def fmt(lines):
    return "".join(f'  "{ln}\\n\\t" \\\n' for ln in lines) + '  ""\n'


def main():
    parts = ["// Generated by scripts/gen_f16_rows.py -- do not edit.\n"
             "// 8-row blocks of the f16 tile-kernel column (see the generator's docstring).\n"]
    for mode in ("L", "P"):
        for zd in (0, 1):
            for last in (0, 1):
                parts.append(f"#define SWK_F16M_{mode}_Z{zd}_L{last} \\\n" +
                             fmt(merged_block(mode, zd, last)))
        for last in (0, 1):
            parts.append(f"#define SWK_F16G_{mode}_L{last} \\\n" + fmt(gotoh_block(mode, last)))
    # whole-column blocks for the DNA LUT merged variants (R = 16, 32): one asm block
    # per column, so LLVM adds one wait state per column instead of one per 8 rows; the
    # operand lists are generated too (h/t/tb numbered 0..R-1)
    for R in (16, 32):
        parts.append(f"#define SWK_F16M_L_Z0_COL{R} \\\n" + fmt(merged_block("L", 0, 1, R)))
        hts = ", ".join([f'[h{i}] "+v"(Hl[{i}])' for i in range(R)] +
                        [f'[t{i}] "+v"(Xl[{i}])' for i in range(R)])
        parts.append(f"#define SWK_F16_COL{R}_HT {hts}\n")
        tbs = ", ".join(f'[tb{i}] "s"(lk.tab[{min(i + 1, R - 1)}])' for i in range(R))
        parts.append(f"#define SWK_F16_COL{R}_TB {tbs}\n")
    # pair-profile blocks: first (with the column prologue), middle, last (final row)
    parts.append("#define SWK_F16PAIR_F \\\n" + fmt(pair_block(True, False)))
    parts.append("#define SWK_F16PAIR_M \\\n" + fmt(pair_block(False, False)))
    parts.append("#define SWK_F16PAIR_L \\\n" + fmt(pair_block(False, True)))
    parts.append("#define SWK_F16PAIRG_F \\\n" + fmt(pair_gotoh_block(True, False)))
    parts.append("#define SWK_F16PAIRG_M \\\n" + fmt(pair_gotoh_block(False, False)))
    parts.append("#define SWK_F16PAIRG_L \\\n" + fmt(pair_gotoh_block(False, True)))
    # mode F (profile words {s, 1.0}: one packed FMA per row, no lookup), 8-row blocks
    for last in (0, 1):
        parts.append(f"#define SWK_F16M_F_Z0_L{last} \\\n" + fmt(merged_block("F", 0, last)))
        parts.append(f"#define SWK_F16G_F_L{last} \\\n" + fmt(gotoh_block("F", last)))
    # 4- and 2-row single blocks (the wave kernel's K = 4, and K = 2 of its split tail: a
    # whole column in one block)
    for nr in (4, 2):
        for mode in ("L", "P"):
            parts.append(f"#define SWK_F16M_{mode}_Z0_L1_R{nr} \\\n" +
                         fmt(merged_block(mode, 0, 1, nr)))
            parts.append(f"#define SWK_F16G_{mode}_L1_R{nr} \\\n" + fmt(gotoh_block(mode, 1, nr)))
    open(OUT, "w").write("".join(parts))
    print("wrote", OUT)


if __name__ == "__main__":
    main()
