// swbank_pack.h — the host feeder's code packers (host-only, header-inline so the CPU test
// harness tests/c/pack_check.cc exercises the same code the library runs).
//
// pack_2bit: l code bytes -> ceil(l/4) bytes of 2-bit codes, 4 per byte LSB first (the CAPI
// host's charTo2bit order, aligner_Header.c:25-40).  Returns the OR of all l codes: the packing
// is valid only when it is <= 3 (a DNA chunk without N).
// pack_4bit: l code bytes -> ceil(l/2) bytes of 4-bit codes, low nibble first.  Returns the
// largest code (valid when below the alphabet size, at most 15).
// In both, the bits past the last code of the last byte are 0.
//
// The AVX2 forms take 32 codes per step (2-bit: u8 pairs c0 + 4 c1 by one multiply-add, u16
// pairs into the byte c0 + 4 c1 + 16 c2 + 64 c3 by a second, byte 0 of every dword gathered by
// a shuffle and a dword permute; 4-bit: c0 + 16 c1 per u16 by one multiply-add, a pack and a
// permute).  With `wide` set the caller guarantees 32 readable bytes at every 32-code step of
// src (even past l) and 16 writable bytes at every step of dst that a later write will
// overwrite: the last < 32 codes then go through the same step with the codes past l masked to
// 0 — no data-dependent scalar loop per target (ragged lengths made that loop's branches the
// feeder's largest cost).  Codes past 3 (resp. 15) give garbage bytes, but the returned OR (max)
// rejects the chunk.
#ifndef SWBANK_PACK_H
#define SWBANK_PACK_H

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>
#if defined(__SSE2__)
#include <emmintrin.h>
#endif
#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace swpack {

inline uint32_t pack_2bit(const uint8_t* src, uint32_t l, uint8_t* dst) {
  uint32_t j = 0, orc = 0;
#if defined(__SSE2__)
  __m128i orv = _mm_setzero_si128();
  const __m128i m16 = _mm_set1_epi16(0x000F), m32 = _mm_set1_epi32(0xFF);
  for (; j + 16 <= l; j += 16) {  // 16 codes -> 4 bytes
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + j));
    orv = _mm_or_si128(orv, v);
    __m128i x = _mm_and_si128(_mm_or_si128(v, _mm_srli_epi16(v, 6)), m16);  // 2 codes / u16
    x = _mm_and_si128(_mm_or_si128(x, _mm_srli_epi32(x, 12)), m32);        // 4 codes / u32
    x = _mm_packus_epi16(_mm_packs_epi32(x, x), x);
    const uint32_t w = (uint32_t)_mm_cvtsi128_si32(x);
    memcpy(dst + j / 4, &w, 4);
  }
  orv = _mm_or_si128(orv, _mm_srli_si128(orv, 8));
  orv = _mm_or_si128(orv, _mm_srli_si128(orv, 4));
  orv = _mm_or_si128(orv, _mm_srli_si128(orv, 2));
  orv = _mm_or_si128(orv, _mm_srli_si128(orv, 1));
  orc = (uint32_t)_mm_cvtsi128_si32(orv) & 0xFFu;
#endif
  for (; j < l; j += 4) {
    uint32_t byte = 0;
    for (uint32_t t = 0; t < 4 && j + t < l; ++t) {
      orc |= src[j + t];
      byte |= (uint32_t)(src[j + t] & 3u) << (2 * t);
    }
    dst[j / 4] = (uint8_t)byte;
  }
  return orc;
}

inline uint32_t pack_4bit(const uint8_t* src, uint32_t l, uint8_t* dst) {
  uint32_t j = 0, mx = 0;
#if defined(__SSE2__)
  __m128i mv = _mm_setzero_si128();
  const __m128i m16 = _mm_set1_epi16(0x00FF);
  for (; j + 16 <= l; j += 16) {  // 16 codes -> 8 bytes
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + j));
    mv = _mm_max_epu8(mv, v);
    __m128i x = _mm_and_si128(_mm_or_si128(v, _mm_srli_epi16(v, 4)), m16);
    x = _mm_packus_epi16(x, x);
    _mm_storel_epi64(reinterpret_cast<__m128i*>(dst + j / 2), x);
  }
  mv = _mm_max_epu8(mv, _mm_srli_si128(mv, 8));
  mv = _mm_max_epu8(mv, _mm_srli_si128(mv, 4));
  mv = _mm_max_epu8(mv, _mm_srli_si128(mv, 2));
  mv = _mm_max_epu8(mv, _mm_srli_si128(mv, 1));
  mx = (uint32_t)_mm_cvtsi128_si32(mv) & 0xFFu;
#endif
  for (; j < l; j += 2) {
    const uint32_t a = src[j], c = j + 1 < l ? src[j + 1] : 0u;
    mx = std::max(mx, std::max(a, c));
    dst[j / 2] = (uint8_t)((a & 15u) | (c & 15u) << 4);
  }
  return mx;
}

#if defined(__x86_64__)
// codes >= n of a 32-code step masked to 0 (n < 32)
__attribute__((target("avx2"))) inline __m256i keep_first(__m256i v, uint32_t n) {
  const __m256i iota = _mm256_setr_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16,
                                        17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31);
  return _mm256_and_si256(v, _mm256_cmpgt_epi8(_mm256_set1_epi8((char)n), iota));
}

__attribute__((target("avx2"))) inline uint32_t pack_2bit_avx2(const uint8_t* src, uint32_t l,
                                                               uint8_t* dst, bool wide) {
  uint32_t j = 0;
  __m256i orv = _mm256_setzero_si256();
  const __m256i w1 = _mm256_set1_epi16(0x0401), w2 = _mm256_set1_epi32(0x00100001);
  const __m256i sh = _mm256_setr_epi8(0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
                                      0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1);
  const __m256i pd = _mm256_setr_epi32(0, 4, 1, 1, 1, 1, 1, 1);
  const uint32_t end = wide ? l : l & ~31u;
  for (; j < end; j += 32) {
    __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + j));
    if (j + 32 > l) v = keep_first(v, l - j);
    orv = _mm256_or_si256(orv, v);
    const __m256i u = _mm256_madd_epi16(_mm256_maddubs_epi16(v, w1), w2);
    const __m256i x = _mm256_permutevar8x32_epi32(_mm256_shuffle_epi8(u, sh), pd);
    _mm_storel_epi64(reinterpret_cast<__m128i*>(dst + j / 4), _mm256_castsi256_si128(x));
  }
  __m128i o = _mm_or_si128(_mm256_castsi256_si128(orv), _mm256_extracti128_si256(orv, 1));
  o = _mm_or_si128(o, _mm_srli_si128(o, 8));
  o = _mm_or_si128(o, _mm_srli_si128(o, 4));
  o = _mm_or_si128(o, _mm_srli_si128(o, 2));
  o = _mm_or_si128(o, _mm_srli_si128(o, 1));
  const uint32_t orc = (uint32_t)_mm_cvtsi128_si32(o) & 0xFFu;
  return j >= l ? orc : orc | pack_2bit(src + j, l - j, dst + j / 4);
}

__attribute__((target("avx2"))) inline uint32_t pack_4bit_avx2(const uint8_t* src, uint32_t l,
                                                               uint8_t* dst, bool wide) {
  uint32_t j = 0;
  __m256i mv = _mm256_setzero_si256();
  const __m256i w = _mm256_set1_epi16(0x1001);
  const uint32_t end = wide ? l : l & ~31u;
  for (; j < end; j += 32) {
    __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + j));
    if (j + 32 > l) v = keep_first(v, l - j);
    mv = _mm256_max_epu8(mv, v);
    const __m256i p = _mm256_maddubs_epi16(v, w);
    const __m256i x = _mm256_permute4x64_epi64(_mm256_packus_epi16(p, p), 0x08);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + j / 2), _mm256_castsi256_si128(x));
  }
  __m128i m = _mm_max_epu8(_mm256_castsi256_si128(mv), _mm256_extracti128_si256(mv, 1));
  m = _mm_max_epu8(m, _mm_srli_si128(m, 8));
  m = _mm_max_epu8(m, _mm_srli_si128(m, 4));
  m = _mm_max_epu8(m, _mm_srli_si128(m, 2));
  m = _mm_max_epu8(m, _mm_srli_si128(m, 1));
  const uint32_t mx = (uint32_t)_mm_cvtsi128_si32(m) & 0xFFu;
  return j >= l ? mx : std::max(mx, pack_4bit(src + j, l - j, dst + j / 2));
}
#endif

// pack_2bit_flag: a RUN of l codes (several targets back to back in the caller's residues) ->
// ceil(l/4) bytes of 2-bit codes, as pack_2bit, and the position (+ base) of every code past 3
// appended to `bad` in ascending order: the caller finds the targets that hold an N from them
// and packs those again in 4-bit codes.  One call per run instead of one per target (the call
// overhead was most of a ragged gather).  No `wide` form: only the run's last < 32 codes take
// the short loop.
inline void pack_2bit_flag(const uint8_t* src, size_t l, uint8_t* dst, uint32_t base,
                           std::vector<uint32_t>& bad) {
  for (size_t j = 0; j < l; j += 32) {
    const uint32_t m = (uint32_t)std::min<size_t>(32, l - j);
    if (pack_2bit(src + j, m, dst + j / 4) > 3u) {
      // a code past 3 spills into its byte's other codes (the packers assume codes <= 3), and
      // in a run those may belong to the neighbouring target: the step again from codes & 3
      uint8_t tmp[32];
      for (uint32_t t = 0; t < m; ++t) {
        if (src[j + t] > 3u) bad.push_back(base + (uint32_t)(j + t));
        tmp[t] = src[j + t] & 3u;
      }
      pack_2bit(tmp, m, dst + j / 4);
    }
  }
}

#if defined(__x86_64__)
__attribute__((target("avx2"))) inline void pack_2bit_flag_avx2(const uint8_t* src, size_t l,
                                                                uint8_t* dst, uint32_t base,
                                                                std::vector<uint32_t>& bad) {
  size_t j = 0;
  const __m256i w1 = _mm256_set1_epi16(0x0401), w2 = _mm256_set1_epi32(0x00100001);
  const __m256i sh = _mm256_setr_epi8(0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
                                      0, 4, 8, 12, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1);
  const __m256i pd = _mm256_setr_epi32(0, 4, 1, 1, 1, 1, 1, 1);
  const __m256i three = _mm256_set1_epi8(3);
  for (; j + 32 <= l; j += 32) {
    const __m256i r = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + j));
    // bit t set: code t <= 3 (unsigned: min(r, 3) == r)
    const uint32_t ok =
        (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(_mm256_min_epu8(r, three), r));
    if (__builtin_expect(ok != 0xFFFFFFFFu, 0))
      for (uint32_t m = ~ok; m; m &= m - 1) bad.push_back(base + (uint32_t)j + __builtin_ctz(m));
    // codes & 3: a code past 3 would spill into its byte's other codes, which in a run may be
    // the neighbouring target's
    const __m256i v = _mm256_and_si256(r, three);
    const __m256i u = _mm256_madd_epi16(_mm256_maddubs_epi16(v, w1), w2);
    const __m256i x = _mm256_permutevar8x32_epi32(_mm256_shuffle_epi8(u, sh), pd);
    _mm_storel_epi64(reinterpret_cast<__m128i*>(dst + j / 4), _mm256_castsi256_si128(x));
  }
  if (j < l) pack_2bit_flag(src + j, l - j, dst + j / 4, base + (uint32_t)j, bad);
}
#endif

typedef void (*PackRunFn)(const uint8_t*, size_t, uint8_t*, uint32_t, std::vector<uint32_t>&);
inline PackRunFn run_packer(bool avx2) {
#if defined(__x86_64__)
  if (avx2 && __builtin_cpu_supports("avx2")) return pack_2bit_flag_avx2;
#else
  (void)avx2;
#endif
  return pack_2bit_flag;
}

// The packers for this host: AVX2 forms when the CPU has AVX2 and `avx2` is allowed, else the
// SSE2 ones (which ignore `wide`).
typedef uint32_t (*PackFn)(const uint8_t*, uint32_t, uint8_t*, bool);
inline uint32_t pack_2bit_any(const uint8_t* s, uint32_t l, uint8_t* d, bool) {
  return pack_2bit(s, l, d);
}
inline uint32_t pack_4bit_any(const uint8_t* s, uint32_t l, uint8_t* d, bool) {
  return pack_4bit(s, l, d);
}
inline PackFn packer(int bits, bool avx2) {
#if defined(__x86_64__)
  if (avx2 && __builtin_cpu_supports("avx2")) return bits == 2 ? pack_2bit_avx2 : pack_4bit_avx2;
#else
  (void)avx2;
#endif
  return bits == 2 ? pack_2bit_any : pack_4bit_any;
}

}  // namespace swpack

#endif
