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
} SwkWaveSplit;

#endif
