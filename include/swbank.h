/*
 * swbank.h — C ABI of the MI355X Smith-Waterman score bank (libswbank.so).
 *
 * This is the drop-in boundary for the reference's scoring path.  Each entry point
 * replaces one port group of the ScoreBank hardware (paths relative to the reference repo,
 * ilirlikalla/Smith-Waterman-FPGA-module) or one call of its C host over libcxl:
 *
 *   sw_bank_create / sw_bank_destroy
 *       ≙ instantiating ScoreBank_v2 (ScoreBank/ScoreBank_v2.v:11-44) + reset; on the CAPI
 *         host, cxl_afu_open_dev / cxl_afu_attach / cxl_afu_free
 *         (capi_sample_aligner/software-C,C++/src/main_test.c:342,370,530)
 *   sw_set_penalties
 *       ≙ ld_penalties with penalties = {match, mismatch, gap_open, gap_extend}
 *         (ScoreBank_v2.v:33-34,161; propagated to every PE, ScoringModule_v1.1.v:128-148)
 *   sw_set_matrix
 *       ≙ the PE's substitution LUT (SW_ProcessingElement_v1.0.v:119) widened to a full
 *         alphabet x alphabet matrix (protein mode; not in the reference)
 *   sw_load_query
 *       ≙ ld_sequence with the query flag, data_in = {01, ID, LEN, SEQ}
 *         (ScoreBank_v2.v:101-102,162; ScoreBank_v1_tb.sv:193-197)
 *   sw_score_batch / sw_score_batch_device
 *       ≙ streaming target records {10, ID, LEN, SEQ} (ScoreBank_v2.v:164-165,
 *         ScoreBank_v1_tb.sv:236-266) and collecting results/IDs/vld (ScoreBank_v2.v:39-41).
 *         Scores come back UNBIASED (the RTL's biased - 2048, ScoreBank_v1_tb.sv:280) and in
 *         INPUT order (the RTL reports completion order; callers re-keyed by ID).
 *   sw_best_hit
 *       ≙ the bank's max / vld_max outputs (ScoreBank_v2.v:42-43, declared but never driven).
 *   sw_encode_ascii
 *       ≙ ConvertToBase (ScoreBank_v1_tb.sv:44-52): A=2 G=3 T=0 C=1 (lower case too);
 *         any other byte -> SW_DNA_N (4), which mismatches every code.
 *   sw_pack_2bit
 *       ≙ charTo2bit (capi_sample_aligner/software-C,C++/include/aligner_Header.c:14-47):
 *         2 bits per base, base i at bits 2*(i%4) of byte i/4 (LSB first), N -> 00.
 *
 * Conventions (mirroring the reference host, main_test.c):
 *   - every call returns sw_status: 0 = SW_OK, negative = error; sw_last_error() gives text.
 *     The library never prints and never exits.
 *   - the caller owns every host buffer; the bank owns its device buffers and stream.
 *   - a bank is not thread-safe; use one bank per host thread (like one AFU context).
 *   - there is NO CPU fallback: without a usable gfx950 device sw_bank_create fails with
 *     SW_ERR_NO_DEVICE.
 */
#ifndef SWBANK_H
#define SWBANK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 2: ids on the batch calls and the batch best hit (ScoreBank_v2.v:39-43), multi-device
 * banks (sw_config.n_devices / devices[]), scores past the 16-bit lanes (int32 re-score).
 * ABI 3: sw_score_batch_device_range (caller length range) and sw_bank_counters.
 * ABI 4: sw_bank_counters took the caller's struct size; multi-device banks take device
 *        batches and query sets.
 * ABI 5: SW_ERR_TIMEOUT and sw_bank_sync (device-side hand-off waits that run out fail the call,
 *        ≙ the CAPI host failing on the AFU's error bits, main_test.c:64-100); sw_bank_counters
 *        is the two-argument ABI-3 form again, sw_bank_counters_ex takes the struct size;
 *        multi-device device calls copy each device's share into its own HBM.
 * ABI 6: sw_counters.wave_balanced_timeouts; sw_score_batch_device_multi (each device scores
 *        a batch already resident in its own HBM, only the int32 scores cross xGMI); every entry
 *        point leaves the caller's current HIP device as it found it. */
#define SWBANK_ABI_VERSION 6

typedef int32_t sw_status;
enum {
  SW_OK = 0,
  SW_ERR_ARG = -1,         /* bad argument (NULL pointer, code out of alphabet, ...)      */
  SW_ERR_NO_DEVICE = -2,   /* no HIP device / not gfx950                                 */
  SW_ERR_HIP = -3,         /* HIP runtime error (text in sw_last_error)                  */
  SW_ERR_RANGE = -4,       /* substitution span > 254 or gap penalties past the kernels  */
  SW_ERR_STATE = -5,       /* penalties or query not loaded yet                          */
  SW_ERR_NOMEM = -6,       /* host or device allocation failed                           */
  SW_ERR_IO = -7,          /* file I/O or parse error (FASTA helpers)                    */
  SW_ERR_UNSUPPORTED = -8, /* configuration not implemented (e.g. query too long)       */
  SW_ERR_TIMEOUT = -9      /* a device-side hand-off wait ran out: the scores of the call
                              (device calls: of the device calls since the last
                              synchronising call) are invalid; see sw_bank_sync            */
};

enum { SW_ALPHABET_DNA = 0, SW_ALPHABET_PROTEIN = 1 };
enum {
  SW_GAP_MERGED = 0, /* ScoreBank PE: one gap matrix I shared by both directions (default) */
  SW_GAP_GOTOH = 1   /* separate E/F matrices (ssearch36); equal to MERGED when
                        2*gap_extend <= min substitution score                           */
};
/* DNA codes (ConvertToBase). */
enum { SW_DNA_T = 0, SW_DNA_C = 1, SW_DNA_A = 2, SW_DNA_G = 3, SW_DNA_N = 4 };
#define SW_DNA_ALPHA 5
#define SW_PROTEIN_ALPHA 24 /* ARNDCQEGHILKMFPSTWYVBZX* */

#define SW_MAX_DEVICES 16

typedef struct sw_config {
  int32_t device;        /* HIP device ordinal; -1 = current device                       */
  int32_t alphabet;      /* SW_ALPHABET_*                                                 */
  int32_t gap_model;     /* SW_GAP_*                                                      */
  uint32_t max_query_len;/* 0 = library maximum (sw_max_query_len())                      */
  uint32_t flags;        /* reserved, 0                                                   */
  /* Multi-device bank (≙ MODULES scoring modules behind one PrioEncoder,
   * ScoreBank_v2.v:76-148): n_devices > 1 spreads every host batch over devices[0..n)
   * (length-balanced deal, one host thread per device) and gathers the scores on devices[0]
   * with one RCCL gather (rccl.h ncclCommInitAll + ncclGather) when the devices are distinct,
   * else with device copies.  0 or 1 = the single device `device`. */
  int32_t n_devices;
  int32_t devices[SW_MAX_DEVICES];
} sw_config;

typedef struct sw_bank sw_bank;

/* ---- library / device ---------------------------------------------------------------- */
int32_t sw_abi_version(void);
const char *sw_status_string(sw_status s);
int32_t sw_device_count(void);           /* HIP devices visible; 0 when none               */
uint32_t sw_max_query_len(void);
sw_status sw_config_default(sw_config *cfg);

/* ---- bank lifecycle (≙ ScoreBank_v2 instance) ------------------------------------------ */
sw_status sw_bank_create(sw_bank **out, const sw_config *cfg);
void sw_bank_destroy(sw_bank *bank);
const char *sw_last_error(const sw_bank *bank);

/* ---- ld_penalties / LUT ---------------------------------------------------------------- */
sw_status sw_set_penalties(sw_bank *bank, int32_t match, int32_t mismatch, int32_t gap_open,
                           int32_t gap_extend);
sw_status sw_set_matrix(sw_bank *bank, const int8_t *matrix, int32_t alpha, int32_t gap_open,
                        int32_t gap_extend);

/* ---- ld_sequence (query) --------------------------------------------------------------- */
sw_status sw_load_query(sw_bank *bank, uint64_t id, const uint8_t *codes, uint32_t len);

/* A query set (ld_sequence for several queries; not in the reference, whose bank holds one):
 * query i = codes[offsets[i] .. + lens[i]) with id ids[i] (ids may be NULL).  Until the next
 * sw_load_query / sw_load_queries, sw_score_batch_device scores its batch against every query
 * of the set into d_scores[i * n + k] (query-major), in one launch per query segment (the
 * tile kernel streams (query, tile) units, so a workgroup scores many tiles per launch); the
 * other scoring calls return SW_ERR_STATE while a set of more than one query is loaded.
 * nq == 1 is sw_load_query.  A multi-device bank loads the set on every device (the
 * reference broadcasts its query to every module, ScoreBank_v2.v:101-102). */
sw_status sw_load_queries(sw_bank *bank, size_t nq, const uint64_t *ids, const uint8_t *codes,
                          const uint64_t *offsets, const uint32_t *lens);

/* Queries loaded (0 before any, 1 after sw_load_query). */
size_t sw_query_count(const sw_bank *bank);

/* ---- target stream -> scores ----------------------------------------------------------- */
/* Host buffers, blocking.  Target k = residues[offsets[k] .. offsets[k]+lens[k]) (codes) of
 * the residues_len-byte buffer (a target outside it is SW_ERR_ARG, nothing past it is read),
 * tagged ids[k] (the RTL's 48-bit record ID, ScoreBank_v2.v:26-28,39-41; NULL = the index k).
 * scores_out[k] = max local-alignment score of (query, target k).  The bank feeds the batch in
 * chunks through pinned staging on its own worker threads and a copy stream (gather, PCIe and
 * scoring overlap), so host buffers need no pinning or layout; n < 2^32.  The call also records
 * the batch's best hit for sw_batch_best.  A multi-device bank deals the batch over its
 * devices and gathers the scores back in input order. */
sw_status sw_score_batch(sw_bank *bank, const uint8_t *residues, size_t residues_len,
                         const uint64_t *offsets, const uint32_t *lens, const uint64_t *ids,
                         size_t n, int32_t *scores_out);

/* Device buffers, asynchronous on `stream` (a hipStream_t; NULL = the bank's stream).
 * max_len must be >= every lens[k]; targets are visited in the caller's order unless their
 * lengths differ, then longest first (an on-device length sort).  d_scores receives int32
 * scores in input order.  With d_ids (device, may be NULL) the call also records the batch's
 * best hit on the device (sw_batch_best); without, it records nothing.  Nothing is copied to
 * or from the host.  On a multi-device bank (ABI 5) the buffers and the stream belong to the
 * root device (devices[0]): the batch is ordered longest first on the root (when its lengths
 * differ) and dealt round robin over the devices (length-balanced); each device copies its
 * share into its own HBM (DNA as 4-bit codes, ceil(max_len / 8) * 4 + 12 bytes per target over
 * xGMI, a share of more than one round of the kernel's slots in chunks that copy while the
 * previous chunk is scored; other alphabets max_len + 12 bytes), scores it there and copies
 * its int32 scores back, and the root writes them to d_scores in input order; the devices'
 * work is ordered after the caller's stream and the caller's stream after it (n < 2^32).
 * Device memory is not validated: the caller keeps every target inside d_residues
 * (d_offsets[k] + d_lens[k] <= its size) and every d_lens[k] <= max_len. */
sw_status sw_score_batch_device(sw_bank *bank, const uint8_t *d_residues,
                                const uint64_t *d_offsets, const uint32_t *d_lens,
                                const uint64_t *d_ids, size_t n, uint32_t max_len,
                                int32_t *d_scores, void *stream);

/* The same with the caller's length range: every d_lens[k] lies in [min_len, max_len].  The
 * RTL's feeder takes each target's LEN as given (SM_Feeder3.v:135-140) and feeds in arrival
 * order (ScoreBank_v2.v:142-148); when the range holds one length (a fixed-length read batch,
 * min_len == max_len) no visiting order is built on the device at all, as there.
 * sw_score_batch_device is this call with min_len = 0. */
sw_status sw_score_batch_device_range(sw_bank *bank, const uint8_t *d_residues,
                                      const uint64_t *d_offsets, const uint32_t *d_lens,
                                      const uint64_t *d_ids, size_t n, uint32_t min_len,
                                      uint32_t max_len, int32_t *d_scores, void *stream);

/* ABI 6: one batch per device, each ALREADY RESIDENT in that device's HBM (≙ every
 * ScoringModule's feeder latching its own targets before scoring them, ScoreBank_v2.v:117-137,
 * SM_Feeder3.v:104-182; BASELINE north_star: "RCCL over xGMI only to gather the final score
 * vector").  batches[d] belongs to the bank's d-th device (sw_bank_devices order; a single-device
 * bank takes one): its buffers and stream (NULL = that device's bank stream) are on that device,
 * and it is scored there against the loaded query (or query set) like
 * sw_score_batch_device_range -- no target byte crosses xGMI.  Its int32 scores go to
 * batches[d].d_scores (on device d, may be NULL; nq x n query-major for a query set) and/or are
 * gathered to the root device (devices[0]) into d_gathered (may be NULL if every d_scores is
 * given): query-major over the concatenated batch, N = sum of the n, query i, device d, target k at
 * d_gathered[i * N + (n_0 + ... + n_{d-1}) + k], written on `stream` (a root-device stream,
 * NULL = the bank's).  Distinct devices gather with one ncclGather (RCCL over xGMI: nq x max n
 * int32 per device), a device listed twice with peer copies.  Asynchronous: each device's work
 * follows its stream, `stream` follows every device's work.  No best hit is tracked (d_ids are
 * not taken); sw_bank_sync waits for it and returns a latched hand-off fault. */
typedef struct sw_device_batch {
  const uint8_t *d_residues;  /* codes on this device                                      */
  const uint64_t *d_offsets;
  const uint32_t *d_lens;
  size_t n;                   /* targets (0: the device scores nothing, still joins the gather) */
  uint32_t min_len, max_len;  /* every d_lens[k] in [min_len, max_len]                     */
  int32_t *d_scores;          /* this device's scores, or NULL                             */
  void *stream;               /* a hipStream_t of this device, or NULL                     */
} sw_device_batch;
sw_status sw_score_batch_device_multi(sw_bank *bank, const sw_device_batch *batches,
                                      size_t n_batches, int32_t *d_gathered, void *stream);

/* Best hit of the last batch call (≙ the bank's max / vld_max outputs, ScoreBank_v2.v:42-43):
 * the lowest input index with the maximum score, its id (ids[index], the record's ID for
 * sw_score_records, else the index) and score.  Waits for a device call's stream.
 * SW_ERR_STATE when the last call tracked no best hit (a device call without d_ids). */
sw_status sw_batch_best(sw_bank *bank, uint64_t *best_id, int32_t *best_score,
                        uint64_t *best_index);

/* Devices of the bank (1 for a single-device bank); writes min(count, cap) ordinals. */
int32_t sw_bank_devices(const sw_bank *bank, int32_t *devices, int32_t cap);

/* ---- CAPI record path: the reference host's packed wire format ---------
 * A record is the 64-byte `sequence_t` of capi_sample_aligner/.../aligner_Header.h:19-24:
 * { u32 ID; u16 length; u8 data[58]; } with 2-bit codes LSB-first (charTo2bit,
 * aligner_Header.c:14-47: T=0 C=1 A=2 G=3), at most 232 bases.  main_test.c:297-314 builds
 * such an array (query in record 0, targets after it) and hands it to the AFU through the
 * WED; here the query comes from sw_load_query_record and every record passed to
 * sw_score_records is a target.  DNA banks only (2 bits cannot carry N). */
#define SW_RECORD_BYTES 64
#define SW_RECORD_MAX_BASES 232
sw_status sw_load_query_record(sw_bank *bank, const void *record);
/* Host records in, unbiased scores out in input order (the kernel reads the 2-bit codes); the
 * best hit (sw_batch_best) carries the record's ID.  Multi-device banks deal the records. */
sw_status sw_score_records(sw_bank *bank, const void *records, size_t n, int32_t *scores_out);
/* Device-resident records (n x 64 B) -> device scores, asynchronous on `stream` (a
 * multi-device bank: device d copies the contiguous range [n*d/D, n*(d+1)/D) of records into
 * its own HBM and writes its scores into d_scores). */
sw_status sw_score_records_device(sw_bank *bank, const void *d_records, size_t n,
                                  int32_t *d_scores, void *stream);

/* Best hit of a host score vector (≙ max / vld_max): the lowest index with the maximum
 * score; *best_id = ids ? ids[index] : index. */
sw_status sw_best_hit(sw_bank *bank, const int32_t *scores, const uint64_t *ids, size_t n,
                      uint64_t *best_id, int32_t *best_score);
/* The same on device buffers, asynchronous on `stream`: d_out[0] = best id
 * (d_ids ? d_ids[index] : index), d_out[1] = best score (int32 sign-extended to 64 bits).
 * n <= 2^32. */
sw_status sw_best_hit_device(sw_bank *bank, const int32_t *d_scores, const uint64_t *d_ids,
                             size_t n, uint64_t *d_out, void *stream);

/* ---- profiling (≙ the CAPI AFU's cycle counters, capi_sample_aligner/hdl-verliog/afu.v
 *      _DEBUGGING_ "calculation #N completed, runtime: C cycles") ------------------------- */
/* When enabled, every launch is bracketed by hipEvents on the stream it runs on. */
sw_status sw_bank_set_timing(sw_bank *bank, int32_t enable);
/* Synchronises on the recorded events and returns the launches and the summed milliseconds of
 * the feeder (pack: host gather / packing time of the host-buffer calls) and of the score
 * kernels (device time) since the previous call. */
sw_status sw_bank_timing(sw_bank *bank, uint64_t *launches, double *pack_ms, double *score_ms);
/* Feeder / fallback counters since the bank was created (a multi-device bank sums its
 * devices'), so silent slow paths show: host calls that ran as one streamed kernel, streamed
 * calls re-run through the chunked feeder because a chunk's wait ran out, streamed calls
 * declined for the memory cap (SWBANK_STREAM_MB) or a failed allocation, chunked host calls,
 * device-side length sorts, multi-device gathers abandoned after their time limit, chunks
 * of chunked calls sent as mixed 2-bit / 4-bit codes (ragged DNA), and the pool parts of those
 * chunks packed as one run (targets back to back in the caller's residues), device calls
 * with balanced chunk ranges. */
typedef struct sw_counters {
  uint64_t stream_calls;
  uint64_t stream_reruns;
  uint64_t stream_declined;
  uint64_t chunked_calls;
  uint64_t device_sorts;
  uint64_t gather_timeouts;
  uint64_t mixed_chunks;
  uint64_t mixed_runs;
  /* ABI 4: device calls run with balanced chunk ranges (tiles handed between workgroups),
   * and hand-off waits that ran out (0 unless a workgroup never started) */
  uint64_t balanced_calls;
  uint64_t balanced_timeouts;
  /* ABI 5: protein-tail hand-off waits that ran out, and host-buffer calls re-run without
   * hand-offs because one did (counted when a synchronising call observed them) */
  uint64_t tail_timeouts;
  uint64_t handoff_reruns;
  /* ABI 6: hand-off waits of the protein wave kernel's balanced ranges that ran out (the
   * tile kernel's are balanced_timeouts); each kind of time-out in a call is counted once */
  uint64_t wave_balanced_timeouts;
  /* ABI 6: bytes the host-buffer calls copied host -> device (packed codes and metadata): the
   * PCIe traffic of the drop-in path */
  uint64_t h2d_bytes;
} sw_counters;
/* The first 8 counters (the ABI-3 struct, 64 bytes): safe for a caller of any ABI. */
sw_status sw_bank_counters(const sw_bank *bank, sw_counters *out);
/* out_size = sizeof(sw_counters) as the caller compiled it: 64 (ABI 3), 80 (ABI 4), 96 (ABI 5)
 * or 112 (ABI 6); any other size is SW_ERR_ARG.  No HIP call: the counts are host-side. */
sw_status sw_bank_counters_ex(const sw_bank *bank, sw_counters *out, size_t out_size);

/* Device-side failure reporting (≙ the CAPI host decoding the AFU's error bits and failing the
 * call, capi_sample_aligner/software-C,C++/src/main_test.c:64-100).  Two launch shapes hand
 * work between workgroups of one launch (balanced chunk ranges of device batches, the segmented
 * protein tail); each wait is bounded, and one that runs out marks the launch as failed instead
 * of hanging.  A host-buffer call that sees the mark re-runs itself without hand-offs
 * (handoff_reruns) and returns SW_ERR_TIMEOUT only if that fails too.  A device call is
 * asynchronous, so its mark is latched on the bank and returned (once, as SW_ERR_TIMEOUT) by
 * the next call that synchronises with it -- sw_bank_sync, sw_batch_best, sw_bank_timing -- or
 * by the next device scoring call on the bank, which then scores nothing.
 * sw_bank_sync waits for the bank's last scoring call (any stream) and returns that status. */
sw_status sw_bank_sync(sw_bank *bank);

/* Which kernel the last score call ran, e.g. "tile f16 R=32 W=4 segs=1 grid=998" or
 * "wave u16 K=4" (empty before the first call).  No reference counterpart: the RTL has one
 * datapath; this lets tests and profiles confirm the path taken. */
const char *sw_last_kernel(const sw_bank *bank);

/* ---- host-side helpers (no device needed) ---------------------------------------------- */
/* ASCII -> codes for the alphabet; returns n. */
size_t sw_encode_ascii(int32_t alphabet, const char *ascii, size_t n, uint8_t *codes);
/* ASCII DNA -> 2-bit LSB-first packing (charTo2bit); out must hold (n+3)/4 bytes, which are
 * OR-ed into (caller zeroes them, as the reference host's posix_memalign'd buffer).  */
size_t sw_pack_2bit(const char *ascii, size_t n, uint8_t *out);
/* 2-bit packed -> DNA codes (inverse of sw_pack_2bit for A/C/G/T). */
size_t sw_unpack_2bit(const uint8_t *packed, size_t n, uint8_t *codes);
/* Fill a substitution matrix: DNA (alpha 5) from match/mismatch, or BLOSUM62 (alpha 24). */
sw_status sw_fill_matrix(int32_t alphabet, int32_t match, int32_t mismatch, int8_t *matrix);

#ifdef __cplusplus
}
#endif
#endif /* SWBANK_H */
