/*
 * swbank_host.c — host-side helpers of libswbank.so (no device needed).
 *
 * Encoding follows the reference's two encoders:
 *   ConvertToBase  ScoreBank/ScoreBank_v1_tb.sv:44-52        (A=10b G=11b T=00b C=01b)
 *   charTo2bit     capi_sample_aligner/software-C,C++/include/aligner_Header.c:14-47
 *                  (2 bits per base, LSB first, 4 bases per byte; 'N' and other bytes -> 00b)
 */
#include <string.h>

#include "swbank.h"
#include "swbank_internal.h"

int32_t sw_abi_version(void) { return SWBANK_ABI_VERSION; }

const char *sw_status_string(sw_status s) {
  switch (s) {
    case SW_OK: return "ok";
    case SW_ERR_ARG: return "invalid argument";
    case SW_ERR_NO_DEVICE: return "no usable gfx950 HIP device";
    case SW_ERR_HIP: return "HIP runtime error";
    case SW_ERR_RANGE: return "substitution or gap range outside the kernels";
    case SW_ERR_STATE: return "penalties or query not loaded";
    case SW_ERR_NOMEM: return "out of memory";
    case SW_ERR_IO: return "I/O or parse error";
    case SW_ERR_UNSUPPORTED: return "unsupported configuration";
    case SW_ERR_TIMEOUT: return "device-side hand-off wait timed out (scores invalid)";
    default: return "unknown status";
  }
}

uint32_t sw_max_query_len(void) { return SWB_MAX_QUERY; }

sw_status sw_config_default(sw_config *cfg) {
  if (!cfg) return SW_ERR_ARG;
  memset(cfg, 0, sizeof(*cfg));
  cfg->device = -1;
  cfg->alphabet = SW_ALPHABET_DNA;
  cfg->gap_model = SW_GAP_MERGED;
  cfg->max_query_len = 0;
  return SW_OK;
}

static const char kProtLetters[SW_PROTEIN_ALPHA + 1] = "ARNDCQEGHILKMFPSTWYVBZX*";

static uint8_t dna_code(unsigned char c) {
  switch (c) {
    case 'T': case 't': return SW_DNA_T;
    case 'C': case 'c': return SW_DNA_C;
    case 'A': case 'a': return SW_DNA_A;
    case 'G': case 'g': return SW_DNA_G;
    default: return SW_DNA_N;
  }
}

static uint8_t prot_code(unsigned char c) {
  if (c >= 'a' && c <= 'z') c = (unsigned char)(c - 'a' + 'A');
  for (int i = 0; i < SW_PROTEIN_ALPHA; ++i)
    if ((unsigned char)kProtLetters[i] == c) return (uint8_t)i;
  return 22; /* X */
}

size_t sw_encode_ascii(int32_t alphabet, const char *ascii, size_t n, uint8_t *codes) {
  if (!ascii || !codes) return 0;
  if (alphabet == SW_ALPHABET_PROTEIN) {
    for (size_t i = 0; i < n; ++i) codes[i] = prot_code((unsigned char)ascii[i]);
  } else {
    for (size_t i = 0; i < n; ++i) codes[i] = dna_code((unsigned char)ascii[i]);
  }
  return n;
}

size_t sw_pack_2bit(const char *ascii, size_t n, uint8_t *out) {
  if (!ascii || !out) return 0;
  for (size_t i = 0; i < n; ++i) {
    uint8_t c = dna_code((unsigned char)ascii[i]);
    if (c > 3) c = 0; /* charTo2bit: unknown bases -> 00b */
    out[i >> 2] |= (uint8_t)(c << ((i & 3) * 2));
  }
  return (n + 3) / 4;
}

size_t sw_unpack_2bit(const uint8_t *packed, size_t n, uint8_t *codes) {
  if (!packed || !codes) return 0;
  for (size_t i = 0; i < n; ++i) codes[i] = (uint8_t)((packed[i >> 2] >> ((i & 3) * 2)) & 3u);
  return n;
}

/* BLOSUM62 in NCBI order ARNDCQEGHILKMFPSTWYVBZX*. */
static const int8_t kBlosum62[SW_PROTEIN_ALPHA][SW_PROTEIN_ALPHA] = {
    {4, -1, -2, -2, 0, -1, -1, 0, -2, -1, -1, -1, -1, -2, -1, 1, 0, -3, -2, 0, -2, -1, 0, -4},
    {-1, 5, 0, -2, -3, 1, 0, -2, 0, -3, -2, 2, -1, -3, -2, -1, -1, -3, -2, -3, -1, 0, -1, -4},
    {-2, 0, 6, 1, -3, 0, 0, 0, 1, -3, -3, 0, -2, -3, -2, 1, 0, -4, -2, -3, 3, 0, -1, -4},
    {-2, -2, 1, 6, -3, 0, 2, -1, -1, -3, -4, -1, -3, -3, -1, 0, -1, -4, -3, -3, 4, 1, -1, -4},
    {0, -3, -3, -3, 9, -3, -4, -3, -3, -1, -1, -3, -1, -2, -3, -1, -1, -2, -2, -1, -3, -3, -2, -4},
    {-1, 1, 0, 0, -3, 5, 2, -2, 0, -3, -2, 1, 0, -3, -1, 0, -1, -2, -1, -2, 0, 3, -1, -4},
    {-1, 0, 0, 2, -4, 2, 5, -2, 0, -3, -3, 1, -2, -3, -1, 0, -1, -3, -2, -2, 1, 4, -1, -4},
    {0, -2, 0, -1, -3, -2, -2, 6, -2, -4, -4, -2, -3, -3, -2, 0, -2, -2, -3, -3, -1, -2, -1, -4},
    {-2, 0, 1, -1, -3, 0, 0, -2, 8, -3, -3, -1, -2, -1, -2, -1, -2, -2, 2, -3, 0, 0, -1, -4},
    {-1, -3, -3, -3, -1, -3, -3, -4, -3, 4, 2, -3, 1, 0, -3, -2, -1, -3, -1, 3, -3, -3, -1, -4},
    {-1, -2, -3, -4, -1, -2, -3, -4, -3, 2, 4, -2, 2, 0, -3, -2, -1, -2, -1, 1, -4, -3, -1, -4},
    {-1, 2, 0, -1, -3, 1, 1, -2, -1, -3, -2, 5, -1, -3, -1, 0, -1, -3, -2, -2, 0, 1, -1, -4},
    {-1, -1, -2, -3, -1, 0, -2, -3, -2, 1, 2, -1, 5, 0, -2, -1, -1, -1, -1, 1, -3, -1, -1, -4},
    {-2, -3, -3, -3, -2, -3, -3, -3, -1, 0, 0, -3, 0, 6, -4, -2, -2, 1, 3, -1, -3, -3, -1, -4},
    {-1, -2, -2, -1, -3, -1, -1, -2, -2, -3, -3, -1, -2, -4, 7, -1, -1, -4, -3, -2, -2, -1, -2, -4},
    {1, -1, 1, 0, -1, 0, 0, 0, -1, -2, -2, 0, -1, -2, -1, 4, 1, -3, -2, -2, 0, 0, 0, -4},
    {0, -1, 0, -1, -1, -1, -1, -2, -2, -1, -1, -1, -1, -2, -1, 1, 5, -2, -2, 0, -1, -1, 0, -4},
    {-3, -3, -4, -4, -2, -2, -3, -2, -2, -3, -2, -3, -1, 1, -4, -3, -2, 11, 2, -3, -4, -3, -2, -4},
    {-2, -2, -2, -3, -2, -1, -2, -3, 2, -1, -1, -2, -1, 3, -3, -2, -2, 2, 7, -1, -3, -2, -1, -4},
    {0, -3, -3, -3, -1, -2, -2, -3, -3, 3, 1, -2, 1, -1, -2, -2, 0, -3, -1, 4, -3, -2, -1, -4},
    {-2, -1, 3, 4, -3, 0, 1, -1, 0, -3, -4, 0, -3, -3, -2, 0, -1, -4, -3, -3, 4, 1, -1, -4},
    {-1, 0, 0, 1, -3, 3, 4, -2, 0, -3, -3, 1, -1, -3, -1, 0, -1, -3, -2, -2, 1, 4, -1, -4},
    {0, -1, -1, -1, -2, -1, -1, -1, -1, -1, -1, -1, -1, -1, -2, 0, 0, -2, -1, -1, -1, -1, -1, -4},
    {-4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, 1},
};

sw_status sw_fill_matrix(int32_t alphabet, int32_t match, int32_t mismatch, int8_t *m) {
  if (!m) return SW_ERR_ARG;
  if (alphabet == SW_ALPHABET_PROTEIN) {
    memcpy(m, kBlosum62, sizeof(kBlosum62));
    return SW_OK;
  }
  if (alphabet != SW_ALPHABET_DNA) return SW_ERR_ARG;
  if (match < -128 || match > 127 || mismatch < -128 || mismatch > 127) return SW_ERR_ARG;
  for (int a = 0; a < SW_DNA_ALPHA; ++a)
    for (int b = 0; b < SW_DNA_ALPHA; ++b)
      m[a * SW_DNA_ALPHA + b] = (int8_t)((a == b && a < 4) ? match : mismatch);
  return SW_OK;
}
