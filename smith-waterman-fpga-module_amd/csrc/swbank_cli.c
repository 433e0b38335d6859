/*
 * swbank — command-line host for libswbank.so.
 *
 * Mirrors the reference's two hosts:
 *   - the CAPI sample host's flags  -q query -l library  (capi_sample_aligner/software-C,C++/
 *     src/main_test.c:231-279), without the libcxl/AFU plumbing;
 *   - the ScoreBank testbench's transcript lines ">name score: S" (ScoreBank/ScoreBank_v1_tb.sv:
 *     271-285), one per library record, in library order (the RTL printed completion order).
 *
 * Usage: swbank -q query.fa -l library.fa [-p match,mismatch,open,extend] [-P] [-g]
 *               [-d device[,device...]] [-o out.txt] [-T] [-R scores.txt] [-b]
 *   -p  penalties (default 5,-4,-12,-4: ScoreBank_v1_tb.sv:16-19, data/smith-waterman.py:6-10)
 *   -P  protein mode (BLOSUM62; -p gives only open,extend)      -g  Gotoh gap model
 *   -T  testbench transcript format "@     0ns: %10s score: \t%d"
 *   -R  also write an ssearch36 "-R" score file (data/score500.txt layout: one line per
 *       library record with name, length, score, record index and byte offset)
 *   -d  HIP device, or a comma list for a multi-device bank (the library is dealt over the
 *       devices, length-balanced, and the scores gathered back with RCCL; ScoreBank_v2.v:76-148
 *       spreads targets over MODULES the same way)
 *   -b  also print the bank's best hit ("best: >name score: S", ≙ max / vld_max) to stderr
 * FASTA: '>' starts a record (name = first token); sequence lines are concatenated; CR/LF,
 * blank lines and lower case are accepted; bytes outside the alphabet encode to N (DNA) or X
 * (protein), which score as mismatches (the testbench left them undefined, the CAPI host
 * mapped them to T: unpinned by any fixture).
 * Exit status: 0 ok, 1 usage, 2 I/O, 3 library/device error.
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "swbank.h"

typedef struct {
  char **names;
  char **seqs;
  long *offs; /* byte offset of each record's '>' line */
  size_t n, cap;
} fasta_t;

static int fasta_push(fasta_t *f, char *name, long off) {
  if (f->n == f->cap) {
    size_t nc = f->cap ? 2 * f->cap : 64;
    char **nn = realloc(f->names, nc * sizeof(char *));
    if (nn) f->names = nn;
    char **ns = realloc(f->seqs, nc * sizeof(char *));
    if (ns) f->seqs = ns;
    long *no = realloc(f->offs, nc * sizeof(long));
    if (no) f->offs = no;
    if (!nn || !ns || !no) return -1;
    f->cap = nc;
  }
  f->offs[f->n] = off;
  f->names[f->n] = name;
  f->seqs[f->n] = calloc(1, 1);
  if (!f->seqs[f->n]) return -1;
  f->n++;
  return 0;
}

/* '>' starts a record (name = first token); sequence lines are concatenated (the testbench
 * read exactly one token per record, ScoreBank_v1_tb.sv:185-212; multi-line is a superset). */
static int read_fasta(const char *path, fasta_t *f) {
  FILE *fp = fopen(path, "r");
  if (!fp) return -1;
  char *line = NULL;
  size_t cap = 0;
  ssize_t len;
  long pos = 0, here;
  while ((here = pos, len = getline(&line, &cap, fp)) >= 0) {
    pos += (long)len;
    while (len > 0 && (line[len - 1] == '\n' || line[len - 1] == '\r' || line[len - 1] == ' '))
      line[--len] = 0;
    if (len == 0) continue;
    if (line[0] == '>') {
      char *p = line + 1;
      size_t k = strcspn(p, " \t");
      char *name = strndup(p, k);
      if (!name || fasta_push(f, name, here)) goto fail;
    } else {
      if (f->n == 0) { /* bare sequence file (the CAPI host's build/query) */
        char *name = strdup("seq");
        if (!name || fasta_push(f, name, here)) goto fail;
      }
      char **s = &f->seqs[f->n - 1];
      size_t old = strlen(*s);
      char *ns = realloc(*s, old + (size_t)len + 1);
      if (!ns) goto fail;
      memcpy(ns + old, line, (size_t)len + 1);
      *s = ns;
    }
  }
  free(line);
  fclose(fp);
  return 0;
fail:
  free(line);
  fclose(fp);
  return -1;
}

static void usage(const char *argv0) {
  fprintf(stderr,
          "usage: %s -q query.fa -l library.fa [-p match,mismatch,open,extend] [-P] [-g]\n"
          "          [-d device[,device...]] [-o out.txt] [-T] [-R scores.txt] [-b]\n",
          argv0);
}

int main(int argc, char **argv) {
  const char *qpath = NULL, *lpath = NULL, *opath = NULL, *pen = NULL, *rpath = NULL;
  int protein = 0, gotoh = 0, device = -1, transcript = 0, best = 0, opt;
  int ndev = 0, devs[SW_MAX_DEVICES];
  while ((opt = getopt(argc, argv, "q:l:p:Pgd:o:TR:bh")) != -1) {
    switch (opt) {
      case 'q': qpath = optarg; break;
      case 'l': lpath = optarg; break;
      case 'p': pen = optarg; break;
      case 'P': protein = 1; break;
      case 'g': gotoh = 1; break;
      case 'd': {
        char *p = optarg, *end;
        ndev = 0;
        while (*p && ndev < SW_MAX_DEVICES) {
          devs[ndev++] = (int)strtol(p, &end, 10);
          if (end == p || (*end && *end != ',')) return usage(argv[0]), 1;
          p = *end ? end + 1 : end;
        }
        /* an empty list, or more devices than a bank holds */
        if (ndev == 0 || *p) return usage(argv[0]), 1;
        device = devs[0];
        break;
      }
      case 'b': best = 1; break;
      case 'o': opath = optarg; break;
      case 'T': transcript = 1; break;
      case 'R': rpath = optarg; break;
      default: usage(argv[0]); return opt == 'h' ? 0 : 1;
    }
  }
  if (!qpath || !lpath) {
    fprintf(stderr, "Input files missing\n");
    usage(argv[0]);
    return 1;
  }
  int ma = 5, mm = -4, go = -12, ge = -4;
  if (protein) {
    go = -11;
    ge = -1;
    if (pen && sscanf(pen, "%d,%d", &go, &ge) != 2) return usage(argv[0]), 1;
  } else if (pen && sscanf(pen, "%d,%d,%d,%d", &ma, &mm, &go, &ge) != 4) {
    return usage(argv[0]), 1;
  }

  fasta_t q = {0}, lib = {0};
  if (read_fasta(qpath, &q) || q.n == 0) {
    fprintf(stderr, "Query file error!\n");
    return 2;
  }
  if (read_fasta(lpath, &lib)) {
    fprintf(stderr, "Database file error!\n");
    return 2;
  }
  const int alphabet = protein ? SW_ALPHABET_PROTEIN : SW_ALPHABET_DNA;

  sw_config cfg;
  sw_config_default(&cfg);
  cfg.device = device;
  if (ndev > 1) { /* multi-device bank */
    cfg.n_devices = ndev;
    memcpy(cfg.devices, devs, sizeof(int) * (size_t)ndev);
  }
  cfg.alphabet = alphabet;
  cfg.gap_model = gotoh ? SW_GAP_GOTOH : SW_GAP_MERGED;
  sw_bank *bank = NULL;
  sw_status st = sw_bank_create(&bank, &cfg);
  if (st != SW_OK) {
    fprintf(stderr, "swbank: bank create failed: %s\n", sw_status_string(st));
    return 3;
  }
  if (protein) {
    int8_t m[SW_PROTEIN_ALPHA * SW_PROTEIN_ALPHA];
    sw_fill_matrix(SW_ALPHABET_PROTEIN, 0, 0, m);
    st = sw_set_matrix(bank, m, SW_PROTEIN_ALPHA, go, ge);
  } else {
    st = sw_set_penalties(bank, ma, mm, go, ge);
  }
  size_t qlen = strlen(q.seqs[0]);
  uint8_t *qc = malloc(qlen + 1);
  if (st == SW_OK && qc) {
    sw_encode_ascii(alphabet, q.seqs[0], qlen, qc);
    st = sw_load_query(bank, 0, qc, (uint32_t)qlen);
  }
  size_t total = 0;
  for (size_t k = 0; k < lib.n; ++k) total += strlen(lib.seqs[k]);
  uint8_t *res = malloc(total + 1);
  uint64_t *offs = malloc((lib.n + 1) * sizeof(uint64_t));
  uint32_t *lens = malloc((lib.n + 1) * sizeof(uint32_t));
  int32_t *scores = malloc((lib.n + 1) * sizeof(int32_t));
  if (!res || !offs || !lens || !scores) st = SW_ERR_NOMEM;
  size_t pos = 0;
  for (size_t k = 0; st == SW_OK && k < lib.n; ++k) {
    size_t l = strlen(lib.seqs[k]);
    sw_encode_ascii(alphabet, lib.seqs[k], l, res + pos);
    offs[k] = pos;
    lens[k] = (uint32_t)l;
    pos += l;
  }
  if (st == SW_OK) st = sw_score_batch(bank, res, total, offs, lens, NULL, lib.n, scores);
  if (st != SW_OK) {
    fprintf(stderr, "swbank: %s: %s\n", sw_status_string(st), sw_last_error(bank));
    sw_bank_destroy(bank);
    return 3;
  }
  FILE *out = opath ? fopen(opath, "w") : stdout;
  if (!out) {
    sw_bank_destroy(bank);
    return 2;
  }
  for (size_t k = 0; k < lib.n; ++k) {
    char nm[256];
    snprintf(nm, sizeof(nm), ">%s", lib.names[k]);
    if (transcript)
      fprintf(out, "@%6dns: %10s score: \t%10d\n", 0, nm, scores[k]);
    else
      fprintf(out, "%s score: %d\n", nm, scores[k]);
  }
  if (opath) fclose(out);
  uint64_t bid = 0;
  int32_t bsc = 0;
  if (best && lib.n && sw_batch_best(bank, &bid, &bsc, NULL) == SW_OK)
    fprintf(stderr, "best: >%s score: %d\n", lib.names[bid], bsc);
  if (rpath) { /* ssearch36 -R layout (data/score500.txt:1-3,502-503) */
    FILE *rf = fopen(rpath, "w");
    if (!rf) {
      sw_bank_destroy(bank);
      return 2;
    }
    fprintf(rf, "# swbank -R %s -q %s -l %s\n", rpath, qpath, lpath);
    fprintf(rf, ">>>0 %zu\t%s - %zu %s\n", qlen, q.names[0], qlen, protein ? "aa" : "nt");
    for (size_t k = 0; k < lib.n; ++k)
      fprintf(rf,
              "%-15s %3zu 0 -1.00000 -1.00000 %4d    0    0  1  0    0    0    0  1  0 %5zu "
              "%8ld\n",
              lib.names[k], strlen(lib.seqs[k]), scores[k], k, lib.offs[k]);
    fprintf(rf, "#Algorithm : Smith-Waterman (libswbank, %s gaps, MI355X)\n",
            gotoh ? "Gotoh" : "merged");
    if (protein)
      fprintf(rf, "#Parameters : BLOSUM62 matrix, open/ext: %d/%d\n", go, ge);
    else
      fprintf(rf, "#Parameters : +%d/%d matrix (%d:%d), open/ext: %d/%d\n", ma, mm, ma, mm, go, ge);
    fprintf(rf, "#Query: %3d>>>%s - %zu %s\n", 0, q.names[0], qlen, protein ? "aa" : "nt");
    fclose(rf);
  }
  sw_bank_destroy(bank);
  free(qc);
  free(res);
  free(offs);
  free(lens);
  free(scores);
  return 0;
}
