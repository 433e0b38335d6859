/* swbank_internal.h — constants shared by the host helpers and the device code. */
#ifndef SWBANK_INTERNAL_H
#define SWBANK_INTERNAL_H

/* Longest query a bank accepts; past 512 rows it runs as segments of SWBANK_SEG rows whose
 * bottom rows are handed on through HBM. */
#define SWB_MAX_QUERY 65536u
/* Targets per workgroup tile: 64 lanes x 2 packed u16 halves (the PE "toggle" pair). */
#define SWB_TILE 128
/* Selector byte that reads 0xFF from v_perm_b32 (padding: substitution = S - 255 < 0). */
#define SWB_SEL_PAD 0x0Du
/* Selector byte that reads 0x00 from v_perm_b32. */
#define SWB_SEL_ZERO 0x0Cu

/* CAPI sequence record (aligner_Header.h:19-24): u32 ID, u16 length, u8 data[58]. */
#define SWB_RECORD 64
#define SWB_RECORD_MAX 232u

/* Target layouts the kernels read (ScoreArgs.packed): one code byte per residue; 64-byte CAPI
 * records; a 2-bit stream (4 codes per byte, LSB first, each target starting on a byte, offsets
 * in bytes; the host feeder packs DNA chunks without N into it). */
#define SWK_PACK_BYTES 0u
#define SWK_PACK_RECORDS 1u
#define SWK_PACK_STREAM 2u
/* 4-bit stream: 2 codes per byte, low nibble first (DNA chunks that hold an N). */
#define SWK_PACK_NIBBLE 3u
/* Mixed stream (the host feeder's ragged DNA chunks, tile kernel only): each target in 2-bit
 * codes, or, when it holds an N, in 4-bit codes; u32 offset words from the codes' start:
 * (byte << 1) | 1 for a 4-bit target, position << 1 for a 2-bit one, the position counting
 * 2-bit codes (a target of a run packed back to back starts inside a byte). */
#define SWK_PACK_MIXED 4u

/* Wave kernel split tail (swk_launch_wave): the last `pairs` pairs run as P (2 or 4) row
 * segments of K/P rows per lane, one wave each, each segment's bottom row handed down through
 * `ring` (256 columns x 8 B per segment boundary and pair).  qtab / fb_qtab: the P segments'
 * tables for the main pass and the u16 fallback, `words` / `fb_words` 32-bit words apart,
 * letter strides PS / fb_PS bytes (profiles). */
typedef struct SwkWaveSplit {
  unsigned pairs, P;
  const unsigned* qtab;
  const unsigned* fb_qtab;
  unsigned words, fb_words, PS, fb_PS;
  void* ring;
  /* P = 8 (two-pairs kernel only): the segmented tail, one 64-row segment per wave in blocks
   * after the main ones; ring = pairs x 7 x cols columns of 8 B, prog = pairs x 8 x 3 words
   * zeroed before the launch (progress, bests); a hand-off wait that runs out after poll_limit
   * polls marks *fault (SWK_FAULT_TAIL, coherent host memory); stall: a test hook (ScoreArgs) */
  unsigned cols;
  unsigned* prog;
  unsigned* fault;
  unsigned poll_limit, stall;
  /* balanced ranges of the two-pairs kernel (pairs = 0, P = 0; wbal_blocks > 0): a grid of
   * wbal_grid blocks of 4 waves (the resident capacity), wbal_blocks 32-step blocks per unit,
   * the hand-off flags ((4 wbal_grid + 1) words, zeroed once, compared with wbal_gen) and lane
   * states ((4 wbal_grid + 1) x 36 x 64 words); fault / poll_limit / stall as above */
  unsigned wbal_blocks, wbal_grid, wbal_gen;
  /* waves per block of the balanced launch (swk_wave_half_grid): 4 = one LDS profile copy per
   * 4 waves (3 blocks, 3 waves per SIMD), 8 = one copy per 8 waves (2 blocks per CU, 4 waves
   * per SIMD at <= 128 VGPRs); other launches of the two-pairs kernel use 4 */
  unsigned wbal_waves;
  unsigned* wbal_flag;
  unsigned* wbal_state;
} SwkWaveSplit;

/* Kinds of a launch's fault marks (cross-workgroup hand-off waits that ran out).  Each kind has
 * its own word in the call's group of SWK_FAULT_WORDS words (word ctz(bit) holds bit), so a call
 * whose launches run out in two kinds keeps both (a plain store per kind, no read-modify-write
 * on host memory); a bank has one group for device calls and one for host-buffer calls. */
#define SWK_FAULT_BAL 1u
#define SWK_FAULT_TAIL 2u
#define SWK_FAULT_WBAL 4u
#define SWK_FAULT_WORDS 4


/* One chunk of a streamed host batch (uploaded before the launch): its first tile and the
 * offset of its codes in the device batch buffer.  Its code layout travels in a flag word per
 * chunk, 0 until the chunk's copy landed, then SWK_PACK_STREAM or SWK_PACK_NIBBLE;
 * SWK_STREAM_ABORT from a wave whose wait ran out, or from the host for a chunk it never sent
 * (the host re-runs or fails the call; a ragged chunk is then read from the zeroed region at
 * byte zero_off256 * 256 of the buffer: empty targets). */
typedef struct SwkStreamChunk {
  unsigned tile0, res_off_lo, res_off_hi, zero_off256;
} SwkStreamChunk;
#define SWK_STREAM_ABORT 0xFFFFFFFFu

/* The deal of a device batch over the devices of a multi-device bank (swk_deal_gather /
 * swk_deal_scatter): position p of the visiting order (a permutation, or the identity) goes to
 * device p % D as its target p / D, copied into that device's region of a staging buffer at a
 * fixed stride of `stride` bytes (offsets rebased, lengths kept); its scores come back from
 * scores[d] (nq rows, cnt[d] apart). */
#define SWK_DEAL_MAX 16
typedef struct SwkDeal {
  unsigned D, stride;
  unsigned char* codes[SWK_DEAL_MAX];
  unsigned long long* offs[SWK_DEAL_MAX];
  unsigned* lens[SWK_DEAL_MAX];
  const int* scores[SWK_DEAL_MAX];
  unsigned long long cnt[SWK_DEAL_MAX];
  unsigned nib; /* codes written 4-bit (SWK_PACK_NIBBLE: low nibble first), stride in bytes */
} SwkDeal;

#ifdef __cplusplus
/* (declared here so the definition in swbank_ktile.hip and the call in swbank_stream.hip are
 * checked against one signature) */
extern "C" hipError_t swk_launch_stream(int R, int gotoh, int f16, int pair, const uint8_t* res,
                                        size_t n, uint32_t ulen, const SwkStreamChunk* sc,
                                        const uint32_t* hflag, uint32_t* dflag, uint32_t nsc,
                                        uint32_t* tctr, const uint32_t* qtab, uint32_t nv,
                                        uint32_t S, uint32_t O, uint32_t E, uint32_t PS,
                                        uint32_t pad, int W, int32_t* scores, uint32_t pS1,
                                        uint32_t pS2, hipStream_t st);
/* perm / ident: the device sort's order (ident[0] != 0: the identity), or perm = nullptr */
extern "C" hipError_t swk_deal_gather(const uint8_t* res, const uint64_t* offs,
                                      const uint32_t* lens, const uint32_t* perm,
                                      const uint32_t* ident, size_t n, const SwkDeal* deal,
                                      hipStream_t st);
/* out[q * sstride + t] = scores[d][q * cnt[d] + i] for every position p = i D + d of target t */
extern "C" hipError_t swk_deal_scatter(const uint32_t* perm, const uint32_t* ident, size_t n,
                                       unsigned nq, size_t sstride, const SwkDeal* deal,
                                       int32_t* out, hipStream_t st);
#endif

#endif
