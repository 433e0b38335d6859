// Host packer check (swbank_pack.h, the code the feeder runs): random targets of every length
// 0..300 with and without N, packed back to back the way a pool part packs them (the last one
// without `wide`), against a byte-at-a-time restatement of the 2-bit (charTo2bit order,
// aligner_Header.c:25-40) and 4-bit layouts, the returned OR / max, and the zero bits past the
// last code.  usage: pack_check [avx2|sse2]
#include <stdio.h>
#include <string.h>

#include <random>
#include <vector>

#include "swbank_pack.h"

static int check(bool avx2, int bits, bool with_n, unsigned seed) {
  std::mt19937 rng(seed);
  const int n = 600;
  std::vector<uint32_t> len(n);
  size_t total = 0;
  for (int i = 0; i < n; ++i) total += len[i] = rng() % 301;
  std::vector<uint8_t> res(total + 64);  // 32 readable bytes past every step: the caller's slack
  for (size_t i = 0; i < total; ++i) {
    res[i] = rng() & 3;
    if (with_n && rng() % 97 == 0) res[i] = 4;
  }
  const uint32_t per = bits == 2 ? 4 : 2;
  std::vector<uint8_t> out(total + 64, 0xEE), want(total + 64, 0xEE);
  const swpack::PackFn fn = swpack::packer(bits, avx2);
  // the feeder's pool parts: 7 parts of consecutive targets, each writing its own output range;
  // a target packs its tail in the vector step only when its full-step stores end inside its
  // part (the feeder's rule).  Parts run last to first here, so a store past a part's end
  // would clobber bytes already written.
  const int parts = 7, pstep = (n + parts - 1) / parts;
  std::vector<size_t> poff(parts + 1, 0), pat(parts + 1, 0);
  for (int i = 0; i < n; ++i) {
    poff[i / pstep + 1] += len[i];
    pat[i / pstep + 1] += (len[i] + per - 1) / per;
  }
  for (int p = 0; p < parts; ++p) {
    poff[p + 1] += poff[p];
    pat[p + 1] += pat[p];
  }
  for (int p = parts - 1; p >= 0; --p) {
    size_t o = poff[p], a = pat[p];
    for (int i = p * pstep; i < std::min(n, (p + 1) * pstep); ++i) {
      const uint32_t l = len[i], steps = (l + 31) / 32;
      const bool wide = a + steps * (bits == 2 ? 8 : 16) <= pat[p + 1];
      fn(res.data() + o, l, out.data() + a, wide);
      o += l;
      a += (l + per - 1) / per;
    }
  }
  size_t off = 0, at = 0;
  for (int i = 0; i < n; ++i) {
    const uint32_t l = len[i];
    std::vector<uint8_t> tmp((l + per - 1) / per + 32);
    const uint32_t got = fn(res.data() + off, l, tmp.data(), false);
    uint32_t ref = 0;
    for (uint32_t j = 0; j < l; ++j) ref = bits == 2 ? (ref | res[off + j]) : std::max<uint32_t>(ref, res[off + j]);
    const uint32_t nb = (l + per - 1) / per;
    for (uint32_t q = 0; q < nb; ++q) {
      uint32_t byte = 0;
      for (uint32_t t = 0; t < per && q * per + t < l; ++t)
        byte |= (uint32_t)(res[off + q * per + t] & (bits == 2 ? 3u : 15u)) << (bits * t);
      want[at + q] = (uint8_t)byte;
    }
    if (got != ref) {
      fprintf(stderr, "bits %d target %d len %u: returned %u, want %u\n", bits, i, l, got, ref);
      return 1;
    }
    off += l;
    at += nb;
  }
  // a 2-bit chunk holding an N is rejected by the returned OR: its bytes are not defined
  if (!(bits == 2 && with_n) && memcmp(out.data(), want.data(), at) != 0) {
    for (size_t q = 0; q < at; ++q)
      if (out[q] != want[q]) {
        fprintf(stderr, "bits %d avx2 %d: byte %zu is %02x, want %02x\n", bits, (int)avx2, q,
                out[q], want[q]);
        break;
      }
    return 1;
  }
  return 0;
}

// The run packer (one call per run of back-to-back targets): 2-bit bytes of every code (& 3)
// and the ascending positions (+ base) of the codes past 3, including codes >= 128 (an
// unsigned compare), runs of every length 0..700 (the short tail) with and without N.
static int check_run(bool avx2, unsigned seed) {
  std::mt19937 rng(seed);
  const swpack::PackRunFn fn = swpack::run_packer(avx2);
  for (int rep = 0; rep < 40; ++rep) {
    const size_t l = rng() % 701;
    std::vector<uint8_t> src(l + 32);
    std::vector<uint32_t> want_bad, got_bad{7u};  // (appended to, not cleared)
    const unsigned dens = 1 + rng() % 60;
    for (size_t i = 0; i < l; ++i) {
      src[i] = rng() & 3;
      if (rng() % dens == 0) src[i] = (uint8_t)(rng() % 3 == 0 ? 4 + rng() % 252 : 4);
      if (src[i] > 3) want_bad.push_back(1000u + (uint32_t)i);
    }
    std::vector<uint8_t> out((l + 3) / 4 + 16, 0xEE), want((l + 3) / 4, 0);
    for (size_t i = 0; i < l; ++i) want[i / 4] |= (uint8_t)((src[i] & 3u) << (2 * (i % 4)));
    fn(src.data(), l, out.data(), 1000u, got_bad);
    if (memcmp(out.data(), want.data(), want.size()) != 0 || got_bad.size() != want_bad.size() + 1 ||
        !std::equal(want_bad.begin(), want_bad.end(), got_bad.begin() + 1)) {
      fprintf(stderr, "run packer avx2 %d seed %u len %zu: bytes or N positions differ\n",
              (int)avx2, seed, l);
      return 1;
    }
  }
  return 0;
}

int main(int argc, char** argv) {
  const bool avx2 = argc > 1 && strcmp(argv[1], "avx2") == 0;
  int bad = 0;
  for (unsigned seed = 1; seed <= 20; ++seed) bad |= check_run(avx2, seed);
  for (int bits : {2, 4})
    for (int nn = 0; nn < 2; ++nn)
      for (unsigned seed = 1; seed <= 20; ++seed) bad |= check(avx2, bits, nn != 0, seed);
  if (bad) return 1;
  printf("pack ok (%s)\n", avx2 ? "avx2" : "sse2");
  return 0;
}
