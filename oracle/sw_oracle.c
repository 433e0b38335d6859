/*
 * sw_oracle.c — CPU restatement of the reference's scoring recurrence.
 *
 * TEST INFRASTRUCTURE ONLY (the checker).  Never linked into libswbank.so; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it (as liboracle_sw.so).
 *
 * Reference semantics followed (paths relative to the reference repo root):
 *   s(i,j)  = (q_i == t_j) ? match : mismatch         ScoreBank/SW_ProcessingElement_v1.0.v:119
 *   M(i,j)  = max(0, max(M,I)(i-1,j-1) + s(i,j))       :123, :287-288
 *   I(i,j)  = max(max(M(i-1,j), M(i,j-1)) + go + ge,   :126-128
 *                 max(I(i-1,j), I(i,j-1)) + ge)        :126, :129, :291
 *   first target column: I(i,0) = max(go+ge, ge)       :131-141 (idle-state branch uses ZERO
 *                                                        instead of the neighbours)
 *   score   = max over the matrix of max(M,I), >= 0    :402-420; taken at PE[len(q)-1],
 *                                                        ScoringModule_v1.1.v:103-107,125
 *   row -1 (PE0 inputs) M = I = 0                      ScoringModule_v1.1.v:176-179
 *   column -1 diagonal registers = 0                   SW_ProcessingElement_v1.0.v:156-164
 * Constants of the reference (match 5, mismatch -4, open -12, extend -4):
 *   data/smith-waterman.py:6-10, ScoreBank/ScoreBank_v1_tb.sv:16-19.
 */
#include "sw_oracle.h"

#include <limits.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAX2(a, b) ((a) > (b) ? (a) : (b))
#define NEG_INF (INT32_MIN / 4)

static int32_t score_merged(const uint8_t *q, int32_t qlen, const uint8_t *t, int32_t tlen,
                            const int8_t *sub, int32_t alpha, int32_t go, int32_t ge,
                            int32_t *buf) {
  /* buf: 2*(tlen) ints: M and I of the previous query row (row i-1). */
  int32_t *Mp = buf, *Ip = buf + tlen;
  for (int32_t j = 0; j < tlen; ++j) Mp[j] = Ip[j] = 0; /* row -1: PE0 inputs are ZERO */
  int32_t best = 0;
  for (int32_t i = 0; i < qlen; ++i) {
    const int8_t *srow = sub + (size_t)q[i] * alpha;
    int32_t diagM = 0, diagI = 0; /* (i-1, -1): diagonal registers reset to ZERO */
    int32_t leftM = 0, leftI = 0; /* (i, -1) */
    for (int32_t j = 0; j < tlen; ++j) {
      const int32_t upM = Mp[j], upI = Ip[j];
      const int32_t s = srow[t[j]];
      int32_t m = MAX2(diagM, diagI) + s;
      m = MAX2(m, 0);
      int32_t in;
      if (j == 0) {
        in = MAX2(go + ge, ge); /* first column: neighbours replaced by ZERO (:131-141) */
      } else {
        in = MAX2(MAX2(upM, leftM) + go + ge, MAX2(upI, leftI) + ge);
      }
      best = MAX2(best, MAX2(m, in));
      diagM = upM;
      diagI = upI;
      leftM = m;
      leftI = in;
      Mp[j] = m;
      Ip[j] = in;
    }
  }
  return best;
}

static int32_t score_gotoh(const uint8_t *q, int32_t qlen, const uint8_t *t, int32_t tlen,
                           const int8_t *sub, int32_t alpha, int32_t go, int32_t ge,
                           int32_t *buf) {
  int32_t *Hp = buf, *Fp = buf + tlen;
  for (int32_t j = 0; j < tlen; ++j) {
    Hp[j] = 0;
    Fp[j] = NEG_INF;
  }
  int32_t best = 0;
  for (int32_t i = 0; i < qlen; ++i) {
    const int8_t *srow = sub + (size_t)q[i] * alpha;
    int32_t diagH = 0, leftH = 0, E = NEG_INF;
    for (int32_t j = 0; j < tlen; ++j) {
      const int32_t upH = Hp[j];
      E = MAX2(leftH + go + ge, E + ge);
      const int32_t F = MAX2(upH + go + ge, Fp[j] + ge);
      int32_t h = diagH + srow[t[j]];
      h = MAX2(h, 0);
      h = MAX2(h, E);
      h = MAX2(h, F);
      best = MAX2(best, h);
      diagH = upH;
      leftH = h;
      Hp[j] = h;
      Fp[j] = F;
    }
  }
  return best;
}

int32_t swo_score_pair(const uint8_t *q, int32_t qlen, const uint8_t *t, int32_t tlen,
                       const int8_t *sub, int32_t alpha, int32_t gap_open, int32_t gap_extend,
                       int32_t gap_model) {
  if (qlen <= 0 || tlen <= 0) return 0;
  int32_t stackbuf[4096];
  int32_t *buf = (2 * tlen <= 4096) ? stackbuf : (int32_t *)malloc(sizeof(int32_t) * 2 * tlen);
  if (!buf) return INT32_MIN;
  int32_t r = (gap_model == SWO_GAP_GOTOH)
                  ? score_gotoh(q, qlen, t, tlen, sub, alpha, gap_open, gap_extend, buf)
                  : score_merged(q, qlen, t, tlen, sub, alpha, gap_open, gap_extend, buf);
  if (buf != stackbuf) free(buf);
  return r;
}

/* ---- bit-level RTL model ------------------------------------------------------------
 * SW_ProcessingElement_v1 with SCORE_WIDTH-bit unsigned biased registers (ZERO = 2^(W-1)).
 * Stage 1 (:106-141): diag_max, M_open = max(M_in,M_out)+go+ge, I_extend = max(I_in,I_out)+ge
 *   (first column: ZERO+go+ge / ZERO+ge).  Stage 2 (:280-291): M = bit W-1 of (LUT+diag_max)
 *   ? that : ZERO; I = max(M_open, I_extend).  Stage 3 (:404-420): High = max(High_in,
 *   High_out (not on the first column), max(M,I)).  All adds wrap mod 2^W. */
int32_t swo_score_pair_rtl(const uint8_t *q, int32_t qlen, const uint8_t *t, int32_t tlen,
                           const int8_t *sub, int32_t alpha, int32_t gap_open, int32_t gap_extend,
                           int32_t W) {
  if (qlen <= 0 || tlen <= 0) return 0;
  const uint32_t mask = (W >= 32) ? 0xFFFFFFFFu : ((1u << W) - 1u);
  const uint32_t ZERO = 1u << (W - 1);
  const uint32_t go = (uint32_t)gap_open & mask, ge = (uint32_t)gap_extend & mask;
  uint32_t *Mp = (uint32_t *)malloc(sizeof(uint32_t) * 3 * tlen);
  if (!Mp) return INT32_MIN;
  uint32_t *Ip = Mp + tlen, *Hp = Mp + 2 * tlen;
  for (int32_t j = 0; j < tlen; ++j) Mp[j] = Ip[j] = Hp[j] = ZERO; /* PE0 inputs ZERO */
  for (int32_t i = 0; i < qlen; ++i) {
    const int8_t *srow = sub + (size_t)q[i] * alpha;
    uint32_t dM = ZERO, dI = ZERO, lM = ZERO, lI = ZERO, lH = ZERO;
    for (int32_t j = 0; j < tlen; ++j) {
      const uint32_t uM = Mp[j], uI = Ip[j], uH = Hp[j];
      const uint32_t lut = (uint32_t)(int32_t)srow[t[j]] & mask;
      const uint32_t diag = MAX2(dM, dI);
      uint32_t mopen, iext;
      if (j == 0) {
        mopen = (ZERO + go + ge) & mask;
        iext = (ZERO + ge) & mask;
      } else {
        mopen = (MAX2(uM, lM) + go + ge) & mask;
        iext = (MAX2(uI, lI) + ge) & mask;
      }
      const uint32_t mscore = (lut + diag) & mask;
      const uint32_t m = (mscore & ZERO) ? mscore : ZERO;
      const uint32_t in = MAX2(mopen, iext);
      const uint32_t imm = MAX2(m, in);
      const uint32_t hmax = (j == 0) ? uH : MAX2(uH, lH);
      const uint32_t h = MAX2(hmax, imm);
      dM = uM;
      dI = uI;
      lM = m;
      lI = in;
      lH = h;
      Mp[j] = m;
      Ip[j] = in;
      Hp[j] = h;
    }
  }
  const int32_t r = (int32_t)Hp[tlen - 1] - (int32_t)ZERO;
  free(Mp);
  return r;
}

void swo_score_batch(const uint8_t *q, int32_t qlen, const uint8_t *res, const uint64_t *offs,
                     const uint32_t *lens, size_t n, const int8_t *sub, int32_t alpha,
                     int32_t gap_open, int32_t gap_extend, int32_t gap_model, int32_t *out,
                     int32_t nthreads) {
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
#endif
  for (long k = 0; k < (long)n; ++k)
    out[k] = swo_score_pair(q, qlen, res + offs[k], (int32_t)lens[k], sub, alpha, gap_open,
                            gap_extend, gap_model);
  (void)nthreads;
}

void swo_score_pairs(const uint8_t *qres, const uint64_t *qoffs, const uint32_t *qlens,
                     const uint8_t *tres, const uint64_t *toffs, const uint32_t *tlens,
                     const uint32_t *qidx, const uint32_t *tidx, size_t npairs,
                     const int8_t *sub, int32_t alpha, int32_t gap_open, int32_t gap_extend,
                     int32_t gap_model, int32_t *out, int32_t nthreads) {
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
#endif
  for (long k = 0; k < (long)npairs; ++k) {
    const uint32_t a = qidx[k], b = tidx[k];
    out[k] = swo_score_pair(qres + qoffs[a], (int32_t)qlens[a], tres + toffs[b],
                            (int32_t)tlens[b], sub, alpha, gap_open, gap_extend, gap_model);
  }
  (void)nthreads;
}
