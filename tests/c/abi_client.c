/* abi_client.c — a plain C99 client of libswbank.so, written the way the reference's C host
 * (capi_sample_aligner/software-C,C++/src/main_test.c) would call the bank: it checks the ABI
 * from C (no C++ or Python in between) and prints one line per result for tests/test_c_abi.py.
 *
 *   abi_client host                 host-only checks (no device needed), prints "host ok"
 *   abi_client score q.fa lib.fa    scores every record of lib.fa against q.fa with the
 *                                   reference penalties, through sw_score_batch AND
 *                                   sw_score_records, prints "name score" lines, then the
 *                                   best hit, the kernel name and the error-path checks.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "swbank.h"

#define CHECK(cond, msg)                                     \
  do {                                                       \
    if (!(cond)) {                                           \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, msg); \
      return 1;                                              \
    }                                                        \
  } while (0)

/* one-record-per-two-lines FASTA (the layout of the reference's data files) */
static int read_fa(const char *path, char names[][32], char seqs[][512], int cap) {
  FILE *f = fopen(path, "r");
  if (!f) return -1;
  char line[1024];
  int n = -1;
  while (fgets(line, sizeof line, f)) {
    line[strcspn(line, "\r\n")] = 0;
    if (!line[0]) continue;
    if (line[0] == '>') {
      if (++n >= cap) break;
      size_t k = strlen(line + 1);
      if (k > 31) k = 31;
      memcpy(names[n], line + 1, k);
      names[n][k] = 0;
      seqs[n][0] = 0;
    } else if (n >= 0) {
      const size_t have = strlen(seqs[n]), add = strlen(line);
      const size_t take = add < 511 - have ? add : 511 - have;
      memcpy(seqs[n] + have, line, take);
      seqs[n][have + take] = 0;
    }
  }
  fclose(f);
  return n + 1;
}

static int host_checks(void) {
  CHECK(sw_abi_version() == SWBANK_ABI_VERSION, "abi version");
  CHECK(strcmp(sw_status_string(SW_OK), "") != 0, "status string");
  sw_config cfg;
  CHECK(sw_config_default(&cfg) == SW_OK, "config default");
  CHECK(cfg.alphabet == SW_ALPHABET_DNA && cfg.gap_model == SW_GAP_MERGED, "defaults");
  uint8_t codes[8];
  CHECK(sw_encode_ascii(SW_ALPHABET_DNA, "ACGTNacg", 8, codes) == 8, "encode");
  CHECK(codes[0] == SW_DNA_A && codes[1] == SW_DNA_C && codes[2] == SW_DNA_G &&
            codes[3] == SW_DNA_T && codes[4] == SW_DNA_N && codes[5] == SW_DNA_A,
        "ConvertToBase codes");
  uint8_t packed[2] = {0, 0};
  CHECK(sw_pack_2bit("ACGTACGT", 8, packed) == 2, "pack");
  uint8_t back[8];
  CHECK(sw_unpack_2bit(packed, 8, back) == 8 && memcmp(back, codes, 4) == 0, "unpack");
  int8_t m[SW_DNA_ALPHA * SW_DNA_ALPHA];
  CHECK(sw_fill_matrix(SW_ALPHABET_DNA, 5, -4, m) == SW_OK && m[0] == 5 && m[1] == -4,
        "fill matrix");
  sw_bank *bank = NULL;
  CHECK(sw_bank_create(NULL, &cfg) == SW_ERR_ARG, "create(NULL)");
  if (sw_device_count() == 0) {
    CHECK(sw_bank_create(&bank, &cfg) == SW_ERR_NO_DEVICE && bank == NULL, "no CPU fallback");
  }
  printf("host ok\n");
  return 0;
}

static int score(const char *qpath, const char *lpath) {
  static char qn[1][32], qs[1][512], ln[600][32], ls[600][512];
  CHECK(read_fa(qpath, qn, qs, 1) == 1, "query file");
  const int n = read_fa(lpath, ln, ls, 600);
  CHECK(n > 0, "library file");

  sw_config cfg;
  sw_config_default(&cfg);
  sw_bank *bank = NULL;
  CHECK(sw_bank_create(&bank, &cfg) == SW_OK, "bank create");

  /* state errors before ld_penalties / ld_sequence */
  int32_t dummy = 0;
  uint64_t off0 = 0;
  uint32_t len0 = 1;
  uint8_t c0 = 0;
  CHECK(sw_score_batch(bank, &c0, 1, &off0, &len0, NULL, 1, &dummy) == SW_ERR_STATE, "state error");
  CHECK(strlen(sw_last_error(bank)) > 0, "error text");

  CHECK(sw_set_penalties(bank, 5, -4, -12, -4) == SW_OK, "penalties");
  const size_t qlen = strlen(qs[0]);
  uint8_t *q = malloc(qlen + 1);
  sw_encode_ascii(SW_ALPHABET_DNA, qs[0], qlen, q);
  CHECK(sw_load_query(bank, 0, q, (uint32_t)qlen) == SW_OK, "load query");

  size_t total = 0;
  for (int k = 0; k < n; ++k) total += strlen(ls[k]);
  uint8_t *res = malloc(total + 1);
  uint64_t *offs = malloc(n * sizeof *offs);
  uint32_t *lens = malloc(n * sizeof *lens);
  int32_t *s1 = malloc(n * sizeof *s1), *s2 = malloc(n * sizeof *s2);
  uint64_t *ids = malloc(n * sizeof *ids);
  for (int k = 0; k < n; ++k) ids[k] = 1000000007ull * (uint64_t)(k + 1);  /* 48-bit-style tags */
  size_t pos = 0;
  for (int k = 0; k < n; ++k) {
    const size_t l = strlen(ls[k]);
    sw_encode_ascii(SW_ALPHABET_DNA, ls[k], l, res + pos);
    offs[k] = pos;
    lens[k] = (uint32_t)l;
    pos += l;
  }
  CHECK(sw_score_batch(bank, res, total, offs, lens, ids, (size_t)n, s1) == SW_OK, sw_last_error(bank));
  printf("kernel %s\n", sw_last_kernel(bank));
  /* the batch best hit (≙ max / vld_max) carries the caller's id */
  uint64_t bb_id = 0, bb_ix = 0;
  int32_t bb_sc = 0;
  CHECK(sw_batch_best(bank, &bb_id, &bb_sc, &bb_ix) == SW_OK, sw_last_error(bank));
  CHECK(bb_ix < (uint64_t)n && bb_id == ids[bb_ix] && bb_sc == s1[bb_ix], "batch best");
  for (uint64_t k = 0; k < (uint64_t)n; ++k)
    CHECK(s1[k] < bb_sc || (s1[k] == bb_sc && k >= bb_ix), "batch best = lowest max index");

  /* the same library as CAPI sequence_t records (64 B each), query from a record */
  unsigned char (*recs)[SW_RECORD_BYTES] = calloc((size_t)n + 1, SW_RECORD_BYTES);
  int nrec = 0;
  for (int k = 0; k < n; ++k) {
    const size_t l = strlen(ls[k]);
    if (l > SW_RECORD_MAX_BASES) continue;
    const uint32_t id = (uint32_t)k;
    const uint16_t l16 = (uint16_t)l;
    memcpy(recs[nrec], &id, 4);
    memcpy(recs[nrec] + 4, &l16, 2);
    sw_pack_2bit(ls[k], l, recs[nrec] + 6);
    ++nrec;
  }
  unsigned char qrec[SW_RECORD_BYTES] = {0};
  const uint16_t ql16 = (uint16_t)qlen;
  memcpy(qrec + 4, &ql16, 2);
  sw_pack_2bit(qs[0], qlen, qrec + 6);
  CHECK(sw_load_query_record(bank, qrec) == SW_OK, "query record");
  CHECK(sw_score_records(bank, recs, (size_t)nrec, s2) == SW_OK, sw_last_error(bank));
  CHECK(sw_batch_best(bank, &bb_id, &bb_sc, &bb_ix) == SW_OK, "records best");
  CHECK(bb_sc == s2[bb_ix], "records best score");
  {
    uint32_t rid;
    memcpy(&rid, recs[bb_ix], 4);
    CHECK(bb_id == rid, "records best carries the record ID");
  }
  for (int k = 0, r = 0; k < n; ++k) {
    if (strlen(ls[k]) > SW_RECORD_MAX_BASES) continue;
    CHECK(s2[r] == s1[k], "records path == byte path");
    ++r;
  }
  for (int k = 0; k < n; ++k) printf("%s %d\n", ln[k], s1[k]);

  uint64_t best_id = 0;
  int32_t best = 0;
  CHECK(sw_best_hit(bank, s1, NULL, (size_t)n, &best_id, &best) == SW_OK, "best hit");
  printf("best %s %d\n", ln[best_id], best);

  /* the AFU error-bit check (main_test.c:64-100): nothing latched after good calls */
  CHECK(sw_bank_sync(bank) == SW_OK, sw_last_error(bank));
  /* an ABI-3 caller's 8-counter struct through the two-argument call: 64 bytes written, the
   * word after them untouched */
  {
    uint64_t v3[9];
    memset(v3, 0xA5, sizeof v3);
    CHECK(sw_bank_counters(bank, (sw_counters *)v3) == SW_OK, "counters (ABI 3 form)");
    CHECK(v3[8] == 0xA5A5A5A5A5A5A5A5ull, "counters wrote past the ABI-3 struct");
    CHECK(v3[0] + v3[3] >= 1, "stream_calls + chunked_calls count the host-buffer calls");
    sw_counters c;
    memset(&c, 0xFF, sizeof c);
    CHECK(sw_bank_counters_ex(bank, &c, sizeof c) == SW_OK, "counters_ex");
    CHECK(c.stream_calls == v3[0] && c.chunked_calls == v3[3] && c.balanced_timeouts == 0 && c.tail_timeouts == 0 &&
              c.wave_balanced_timeouts == 0 && c.handoff_reruns == 0,
          "counters_ex = the ABI-3 prefix, no time-outs");
    CHECK(sw_bank_counters_ex(bank, &c, sizeof c - 4) == SW_ERR_ARG, "odd counter size");
    printf("counters host_calls=%llu\n", (unsigned long long)(c.stream_calls + c.chunked_calls));
  }

  /* argument errors */
  CHECK(sw_score_batch(bank, res, total, NULL, lens, NULL, (size_t)n, s1) == SW_ERR_ARG, "null offsets");
  /* a target past the residues is refused before anything is read */
  CHECK(sw_score_batch(bank, res, total - 1, offs, lens, NULL, (size_t)n, s1) == SW_ERR_ARG,
        "target outside residues");
  CHECK(strstr(sw_last_error(bank), "outside") != NULL, "range error text");
  uint8_t bad = 9;
  CHECK(sw_load_query(bank, 0, &bad, 1) == SW_ERR_ARG, "code outside alphabet");
  sw_bank_destroy(bank);
  free(q); free(res); free(offs); free(lens); free(s1); free(s2); free(recs); free(ids);
  printf("score ok\n");
  return 0;
}

int main(int argc, char **argv) {
  if (argc >= 2 && strcmp(argv[1], "host") == 0) return host_checks();
  if (argc >= 4 && strcmp(argv[1], "score") == 0) return score(argv[2], argv[3]);
  fprintf(stderr, "usage: %s host | score query.fa library.fa\n", argv[0]);
  return 2;
}
