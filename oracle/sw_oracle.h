/*
 * sw_oracle.h — CPU restatement of the reference's Smith-Waterman scoring path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker, never the product: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  The product
 * library (libswbank.so) does not link it and has no CPU fallback.
 *
 * Pinned against every golden score the reference holds (tests/golden/ref_scores.tsv:
 * 730 ScoreBank HDL transcript scores, 598 ssearch36 scores, the CAPI host's result) —
 * see tests/test_oracle_golden.py.
 */
#ifndef SW_ORACLE_H
#define SW_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  SWO_GAP_MERGED = 0, /* ScoreBank PE semantics (one merged gap matrix I) */
  SWO_GAP_GOTOH = 1   /* separate E/F gap matrices (ssearch36 / Gotoh)   */
};

/* Exact-integer score of one pair (int32 arithmetic, no width limit). */
int32_t swo_score_pair(const uint8_t *q, int32_t qlen, const uint8_t *t, int32_t tlen,
                       const int8_t *sub, int32_t alpha, int32_t gap_open, int32_t gap_extend,
                       int32_t gap_model);

/* Bit-level functional model of SW_ProcessingElement_v1 + ScoringModule_v1_1 with
 * SCORE_WIDTH-bit biased arithmetic (wraps exactly like the RTL). Returns biased-ZERO. */
int32_t swo_score_pair_rtl(const uint8_t *q, int32_t qlen, const uint8_t *t, int32_t tlen,
                           const int8_t *sub, int32_t alpha, int32_t gap_open, int32_t gap_extend,
                           int32_t score_width);

/* One query against n targets (targets at res + offs[k], length lens[k]); OpenMP over
 * targets with nthreads threads (<=0: all).  Scores into out[k]. */
void swo_score_batch(const uint8_t *q, int32_t qlen, const uint8_t *res, const uint64_t *offs,
                     const uint32_t *lens, size_t n, const int8_t *sub, int32_t alpha,
                     int32_t gap_open, int32_t gap_extend, int32_t gap_model, int32_t *out,
                     int32_t nthreads);

/* General pair list: pair k = (query qidx[k], target tidx[k]) from two residue pools. */
void swo_score_pairs(const uint8_t *qres, const uint64_t *qoffs, const uint32_t *qlens,
                     const uint8_t *tres, const uint64_t *toffs, const uint32_t *tlens,
                     const uint32_t *qidx, const uint32_t *tidx, size_t npairs,
                     const int8_t *sub, int32_t alpha, int32_t gap_open, int32_t gap_extend,
                     int32_t gap_model, int32_t *out, int32_t nthreads);

#ifdef __cplusplus
}
#endif
#endif
