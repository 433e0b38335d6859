// swbank_device.hip — C-ABI of libswbank.so: the bank object and its device plumbing.
//
// Call surface mirrors ScoreBank_v2 (reference ScoreBank/ScoreBank_v2.v:30-44): penalties once,
// a query once, then any number of target batches; one max score per target.  See
// include/swbank.h for the per-function reference citations.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "swbank.h"
#include "swbank_internal.h"

extern "C" int swk_has_variant(int R, int RB, int col0, int prof, int gotoh, int f16);
extern "C" hipError_t swk_launch_wave(int K, int col0, int prof, int gotoh, int f16,
                                      const void* edge_in, void* edge_out, uint32_t ecols,
                                      int accum, const uint8_t* res,
                                      const uint64_t* offs, const uint32_t* lens, size_t n,
                                      const uint32_t* qtab, uint32_t nv, uint32_t S, uint32_t O,
                                      uint32_t E, uint32_t PS, uint32_t pad, int32_t* scores,
                                      int packed, hipStream_t st);
extern "C" hipError_t swk_launch_score(int R, int RB, int col0, int prof, int gotoh, int f16,
                                       const uint8_t* res, const uint64_t* offs,
                                       const uint32_t* lens, size_t n, const uint32_t* qtab,
                                       uint32_t nv, uint32_t S, uint32_t O, uint32_t E,
                                       uint32_t PS, uint32_t pad, int W, int32_t* scores,
                                       const void* edge_in, void* edge_out, uint32_t ecols,
                                       int accum, int packed, const uint32_t* idx,
                                       const uint32_t* nidx, uint32_t idx_base, hipStream_t st);
extern "C" hipError_t swk_best_hit(const int32_t* scores, const uint64_t* ids, size_t n,
                                   unsigned long long* key, uint64_t* out, hipStream_t st);
extern "C" hipError_t swk_flag_high(const int32_t* scores, size_t n, int32_t thresh,
                                    uint32_t* idx, uint32_t* count, hipStream_t st);

namespace {
int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;  // elements
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 64);
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), want * sizeof(T));
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Pinned host staging for the query tables (so their uploads are truly asynchronous).
struct PinBuf {
  uint8_t* p = nullptr;
  size_t cap = 0;  // bytes
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(n, 4096);
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};
}  // namespace

struct sw_bank {
  sw_config cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  char err[512] = {0};

  // ld_penalties
  bool have_pen = false;
  int alpha = SW_DNA_ALPHA;
  std::vector<int8_t> matrix;  // alpha x alpha
  int32_t gap_open = 0, gap_extend = 0;

  // ld_sequence (query)
  bool have_query = false;
  uint64_t qid = 0;
  std::vector<uint8_t> query;

  // derived per (penalties, query)
  bool dirty = true;
  int R = 32, RB = 4, W = 1, col0 = 0, prof = 0;
  uint32_t S = 0, O = 0, E = 0, nv = 0, PS = 0, pad = 4;
  int32_t smax = 0;
  DevBuf<uint32_t> qtab;  // LUT words or query-profile bytes, per query segment
  // f16 tile kernel (DNA LUT, merged gaps): LUT bytes are f16 high bytes; used for a batch
  // whose score bound fits f16's exact integers (|x| <= 2048)
  bool f16 = false;
  uint32_t nv16 = 0, PS16 = 0;  // PS16: f16 profile row stride (bytes)
  int32_t f16_neg = 0;     // most negative intermediate: -(o + 2e + |min s|)
  DevBuf<uint32_t> qtab16;
  DevBuf<uint32_t> fb_idx, fb_cnt;  // pairs an optimistic f16 pass re-scores in u16
  DevBuf<unsigned long long> best_key;  // sw_best_hit_device scratch
  struct Seg { int W; size_t off, off16; };  // rows = W*R (last may be shorter); word offsets
                                              // in qtab and qtab16
  std::vector<Seg> segs;
  DevBuf<uint2> edge[2];  // bottom rows handed from segment to segment
  // wave kernel (few targets, query <= 1024 rows): lane l owns rows [lK, lK+K)
  int wK = 0;              // rows per lane: 4, 8 or 16 (16 with several segments)
  int wsegs = 1;           // 1024-row segments of the wave kernel
  size_t wseg_words = 0, wseg_words16 = 0;  // table words per segment (u16, f16)
  uint32_t wPS = 0;
  DevBuf<uint32_t> wtab;   // LUT: 64K row words | PROF: (A+1) x 64K profile bytes
  DevBuf<uint32_t> wtab16; // the same in f16 (LUT: high bytes | PROF: 2-byte entries)
  uint32_t wPS16 = 0;

  // workspaces
  DevBuf<uint8_t> res;
  DevBuf<uint64_t> offs;
  DevBuf<uint32_t> lens;
  DevBuf<int32_t> scores;

  char last_kernel[96] = {0};

  // Query tables are rewritten in place by prepare() while earlier launches may still read
  // them on the caller's stream: the upload (on the bank stream) waits for ev_used (recorded
  // after every launch), and every launch waits for ev_ready (recorded after the upload).
  // Nothing blocks the host except reusing the pinned staging of a copy still in flight.
  hipEvent_t ev_ready = nullptr, ev_used = nullptr;
  PinBuf stage;

  // profiling
  bool timing = false;
  struct Ev { hipEvent_t a, b, c; };
  std::vector<Ev> events;
};

static sw_status fail(sw_bank* b, sw_status st, const char* fmt, ...) {
  if (b) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(b->err, sizeof(b->err), fmt, ap);
    va_end(ap);
  }
  return st;
}

#define HIPOK(bank, expr)                                                                 \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail((bank), SW_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),    \
                  __FILE__, __LINE__);                                                    \
  } while (0)

extern "C" int32_t sw_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" sw_status sw_bank_create(sw_bank** out, const sw_config* cfg_in) {
  if (!out) return SW_ERR_ARG;
  *out = nullptr;
  sw_config cfg;
  if (cfg_in)
    cfg = *cfg_in;
  else
    sw_config_default(&cfg);
  if (cfg.alphabet != SW_ALPHABET_DNA && cfg.alphabet != SW_ALPHABET_PROTEIN) return SW_ERR_ARG;
  if (cfg.gap_model != SW_GAP_MERGED && cfg.gap_model != SW_GAP_GOTOH) return SW_ERR_ARG;
  if (cfg.max_query_len > SWB_MAX_QUERY) return SW_ERR_UNSUPPORTED;

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SW_ERR_NO_DEVICE;
  int dev = cfg.device;
  if (dev < 0) {
    if (hipGetDevice(&dev) != hipSuccess) return SW_ERR_NO_DEVICE;
  }
  if (dev >= ndev) return SW_ERR_NO_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return SW_ERR_NO_DEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return SW_ERR_NO_DEVICE;

  sw_bank* b = new (std::nothrow) sw_bank();
  if (!b) return SW_ERR_NOMEM;
  b->cfg = cfg;
  b->device = dev;
  if (hipSetDevice(dev) != hipSuccess ||
      hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess) {
    delete b;
    return SW_ERR_HIP;
  }
  b->alpha = cfg.alphabet == SW_ALPHABET_DNA ? SW_DNA_ALPHA : SW_PROTEIN_ALPHA;
  if (cfg.alphabet == SW_ALPHABET_PROTEIN) {  // BLOSUM62 -11/-1 until sw_set_matrix is called
    int8_t m[SW_PROTEIN_ALPHA * SW_PROTEIN_ALPHA];
    sw_fill_matrix(SW_ALPHABET_PROTEIN, 0, 0, m);
    b->matrix.assign(m, m + sizeof(m));
    b->gap_open = -11;
    b->gap_extend = -1;
    b->have_pen = true;
  }
  *out = b;
  return SW_OK;
}

extern "C" void sw_bank_destroy(sw_bank* b) {
  if (!b) return;
  (void)hipSetDevice(b->device);
  if (b->stream) (void)hipStreamSynchronize(b->stream);
  uint64_t nl;
  double pm, sm;
  (void)sw_bank_timing(b, &nl, &pm, &sm);
  b->qtab.release();
  b->qtab16.release();
  b->stage.release();
  if (b->ev_ready) (void)hipEventDestroy(b->ev_ready);
  if (b->ev_used) (void)hipEventDestroy(b->ev_used);
  b->fb_idx.release();
  b->fb_cnt.release();
  b->best_key.release();
  b->wtab.release();
  b->wtab16.release();
  b->edge[0].release();
  b->edge[1].release();
  b->res.release();
  b->offs.release();
  b->lens.release();
  b->scores.release();
  if (b->stream) (void)hipStreamDestroy(b->stream);
  delete b;
}

extern "C" const char* sw_last_error(const sw_bank* b) { return b ? b->err : "null bank"; }

extern "C" const char* sw_last_kernel(const sw_bank* b) { return b ? b->last_kernel : ""; }

static sw_status set_matrix_impl(sw_bank* b, const int8_t* m, int alpha, int32_t go,
                                 int32_t ge) {
  if (go > 0 || ge > 0 || go < -32767 || ge < -32767)
    return fail(b, SW_ERR_ARG, "gap penalties must be <= 0 (got open %d, extend %d)", go, ge);
  b->matrix.assign(m, m + (size_t)alpha * alpha);
  b->alpha = alpha;
  b->gap_open = go;
  b->gap_extend = ge;
  b->have_pen = true;
  b->dirty = true;
  return SW_OK;
}

extern "C" sw_status sw_set_penalties(sw_bank* b, int32_t match, int32_t mismatch,
                                      int32_t gap_open, int32_t gap_extend) {
  if (!b) return SW_ERR_ARG;
  if (b->cfg.alphabet != SW_ALPHABET_DNA)
    return fail(b, SW_ERR_ARG, "sw_set_penalties needs a DNA bank; use sw_set_matrix");
  int8_t m[SW_DNA_ALPHA * SW_DNA_ALPHA];
  if (sw_fill_matrix(SW_ALPHABET_DNA, match, mismatch, m) != SW_OK)
    return fail(b, SW_ERR_ARG, "match/mismatch outside int8 (%d, %d)", match, mismatch);
  return set_matrix_impl(b, m, SW_DNA_ALPHA, gap_open, gap_extend);
}

extern "C" sw_status sw_set_matrix(sw_bank* b, const int8_t* m, int32_t alpha, int32_t gap_open,
                                   int32_t gap_extend) {
  if (!b || !m) return SW_ERR_ARG;
  const int want = b->cfg.alphabet == SW_ALPHABET_DNA ? SW_DNA_ALPHA : SW_PROTEIN_ALPHA;
  if (alpha != want) return fail(b, SW_ERR_ARG, "matrix alphabet %d, bank expects %d", alpha, want);
  return set_matrix_impl(b, m, alpha, gap_open, gap_extend);
}

extern "C" sw_status sw_load_query(sw_bank* b, uint64_t id, const uint8_t* codes, uint32_t len) {
  if (!b || (!codes && len)) return SW_ERR_ARG;
  const uint32_t cap = b->cfg.max_query_len ? b->cfg.max_query_len : SWB_MAX_QUERY;
  if (len > cap)
    return fail(b, SW_ERR_UNSUPPORTED, "query length %u exceeds the bank maximum %u", len, cap);
  for (uint32_t i = 0; i < len; ++i)
    if (codes[i] >= (uint32_t)b->alpha)
      return fail(b, SW_ERR_ARG, "query code %u at %u outside alphabet %d", codes[i], i, b->alpha);
  b->query.assign(codes, codes + len);
  b->qid = id;
  b->have_query = true;
  b->dirty = true;
  return SW_OK;
}

// Build the resident query state (the ScoringModule's query + penalty registers,
// ScoringModule_v1.1.v:110-150): either per-row 4-byte LUTs (DNA fast path) or a query
// profile QP[letter][row] = S - s(q_row, letter) (any alphabet).
static sw_status prepare(sw_bank* b) {
  if (!b->have_pen || !b->have_query)
    return fail(b, SW_ERR_STATE, "load penalties (ld_penalties) and a query (ld_sequence) first");
  if (!b->dirty) return SW_OK;
  const int A = b->alpha;
  const int8_t* m = b->matrix.data();
  int smax = -128, smin = 127;
  for (int i = 0; i < A * A; ++i) {
    smax = std::max<int>(smax, m[i]);
    smin = std::min<int>(smin, m[i]);
  }
  const int S = std::max(0, smax);
  if (S - smin > 254)
    return fail(b, SW_ERR_RANGE, "substitution range [%d, %d] exceeds 254", smin, smax);
  const int o = -b->gap_open, e = -b->gap_extend;
  const bool gotoh = b->cfg.gap_model == SW_GAP_GOTOH;
  if (gotoh && o + e + S > 65535) return fail(b, SW_ERR_RANGE, "gap penalties too large");

  // LUT mode needs a DNA matrix whose N column (codes 4..7 share one word) is uniform and <= 0
  bool lut = A == SW_DNA_ALPHA;
  const int sN = m[4];
  for (int i = 0; lut && i < A; ++i) lut = m[i * A + 4] == sN;
  lut = lut && sN <= 0;
  // The f16 LUT holds one byte per entry (the f16 high byte): only scores whose f16 low byte
  // is 0 (|s| <= 8, or coarser even values) qualify.  Other DNA matrices run in profile mode
  // (2-byte f16 entries) when f16 applies at all: faster than the u16 LUT kernel.
  bool lut_f16 = true;
  for (int i = 0; i < A * A; ++i) {
    const uint16_t bits = __builtin_bit_cast(uint16_t, (_Float16)(float)m[i]);
    lut_f16 = lut_f16 && (bits & 0xFFu) == 0;
  }
  const bool f16_range = -(o + 2 * e + (std::max(0, smax) - smin)) >= -2048;
  const int prof =
      (env_int("SWBANK_PROFILE", 0) || !lut || (!lut_f16 && f16_range)) ? 1 : 0;

  const int qlen = (int)b->query.size();
  // the HDL column-0 rule differs from the plain recurrence only if a match pays for a gap
  const int col0 = (!gotoh && smax > o + e) ? 1 : 0;
  // Rows per wave: 32 for the merged DNA LUT kernels; 16 for tiny queries and for the
  // Gotoh / profile / column-0 variants, whose 32-row columns do not fit 128 VGPRs (the
  // occupancy-4 budget) without spilling.  Queries longer than one workgroup (16 waves) run
  // as segments of SWBANK_SEG rows (default: a full 16-wave workgroup, 16·R rows), each
  // segment's bottom row handed to the next through HBM.  SWBANK_R / SWBANK_RB / SWBANK_SEG
  // override (tuning only).
  int R = (qlen <= 16 || gotoh || prof || col0) ? 16 : 32, RB = 4;
  R = env_int("SWBANK_R", R);
  RB = env_int("SWBANK_RB", RB);
  const int max_rows = (R >= 64 ? 8 : 16) * R;
  int seg_rows = qlen > max_rows ? env_int("SWBANK_SEG", max_rows)
                                 : std::max(qlen, 1);
  if (seg_rows % R != 0 && seg_rows < qlen)
    return fail(b, SW_ERR_ARG, "segment rows %d not a multiple of R=%d", seg_rows, R);
  if (!swk_has_variant(R, RB, col0, prof, gotoh ? 1 : 0, 0))
    return fail(b, SW_ERR_UNSUPPORTED, "no kernel variant R=%d RB=%d col0=%d prof=%d gotoh=%d", R,
                RB, col0, prof, (int)gotoh);
  const int Wseg = std::max(1, (seg_rows + R - 1) / R);
  if (Wseg * 64 > (R >= 64 ? 512 : 1024))
    return fail(b, SW_ERR_UNSUPPORTED, "segment of %d rows too tall for one workgroup", seg_rows);

  // per segment: LUT words (W*R) or a query profile ((A+1) x PS bytes), concatenated
  std::vector<uint32_t> tab;
  std::vector<sw_bank::Seg> segs;
  // profile row stride: a multiple of 16 B that is 16 mod 256, so the 16-B reads of lanes
  // holding different letters fall in different LDS banks (a stride of 0 mod 256 puts every
  // letter row on the same 4 banks)
  uint32_t PS = prof ? (uint32_t)((Wseg * R + 15) / 16 * 16) : 0;
  if (prof) PS += (16u + 256u - PS % 256u) % 256u;
  const uint32_t pad = prof ? (uint32_t)A : 4u;  // profile letter A = padding row (all 0xFF)
  const uint32_t nv = prof ? 0u : (uint32_t)(uint8_t)(S - sN) * 0x01010101u;
  for (int r0 = 0; r0 < std::max(qlen, 1); r0 += seg_rows) {
    const int rows = std::min(seg_rows, std::max(qlen, 1) - r0);
    const int W = std::max(1, (rows + R - 1) / R);
    segs.push_back({W, tab.size(), 0});
    if (!prof) {
      const size_t base = tab.size();
      tab.resize(base + (size_t)W * R, 0xFFFFFFFFu);
      for (int i = 0; i < rows && r0 + i < qlen; ++i) {
        uint32_t w = 0;
        for (int c = 0; c < 4; ++c)
          w |= (uint32_t)(uint8_t)(S - m[b->query[r0 + i] * A + c]) << (8 * c);
        tab[base + i] = w;
      }
    } else {
      std::vector<uint8_t> qp((size_t)(A + 1) * PS, 0xFF);
      for (int c = 0; c < A; ++c)
        for (int i = 0; i < rows && r0 + i < qlen; ++i)
          qp[(size_t)c * PS + i] = (uint8_t)(S - m[b->query[r0 + i] * A + c]);
      const size_t base = tab.size();
      tab.resize(base + qp.size() / 4);
      std::memcpy(tab.data() + base, qp.data(), qp.size());
    }
  }
  // f16 variant of the LUT: each substitution score must be an f16 whose low byte is 0
  // (|s| <= 8 or a coarser even value), so the byte perm yields the exact f16 bits
  auto f16_hi = [](int v, uint8_t* out) {
    const _Float16 h = (_Float16)(float)v;
    const uint16_t bits = __builtin_bit_cast(uint16_t, h);
    *out = (uint8_t)(bits >> 8);
    return (bits & 0xFFu) == 0 && (int)(float)h == v;
  };
  // LUT mode: one byte per entry (the f16 high byte); profile mode: two bytes (any |s| <= 127
  // is an exact f16), row stride PS16 = 2 x rows, 16 mod 256 like PS
  bool f16 = swk_has_variant(R, RB, col0, prof, gotoh ? 1 : 0, 1) != 0;
  std::vector<uint32_t> tab16;
  uint8_t hN = 0;
  uint32_t PS16 = 0;
  if (!prof) {
    f16 = f16 && f16_hi(sN, &hN);
    for (int i = 0; f16 && i < A * A; ++i) {
      uint8_t h;
      f16 = f16_hi(m[i], &h);
    }
  }
  if (f16 && !prof) {
    tab16.assign(tab.size(), 0xE8E8E8E8u);  // padding rows: -2048
    for (sw_bank::Seg& sg : segs) {
      const int r0 = (int)(&sg - segs.data()) * seg_rows;
      sg.off16 = sg.off;
      for (int i = 0; i < sg.W * R && r0 + i < qlen && i < seg_rows; ++i) {
        uint32_t w = 0;
        for (int c = 0; c < 4; ++c) {
          uint8_t h;
          f16_hi(m[b->query[r0 + i] * A + c], &h);
          w |= (uint32_t)h << (8 * c);
        }
        tab16[sg.off + i] = w;
      }
    }
  } else if (f16) {
    PS16 = (uint32_t)((2 * Wseg * R + 15) / 16 * 16);
    PS16 += (16u + 256u - PS16 % 256u) % 256u;
    const uint16_t padv = 0xE800u;  // -2048: padding letter and rows past the query
    for (sw_bank::Seg& sg : segs) {
      const int r0 = (int)(&sg - segs.data()) * seg_rows;
      std::vector<uint16_t> qp((size_t)(A + 1) * PS16 / 2, padv);
      for (int c = 0; c < A; ++c)
        for (int i = 0; i < sg.W * R && r0 + i < qlen && i < seg_rows; ++i)
          qp[(size_t)c * PS16 / 2 + i] =
              __builtin_bit_cast(uint16_t, (_Float16)(float)m[b->query[r0 + i] * A + c]);
      sg.off16 = tab16.size();
      tab16.resize(sg.off16 + qp.size() / 2);
      std::memcpy(tab16.data() + sg.off16, qp.data(), qp.size() * 2);
    }
  }
  // wave-kernel layout of the same query: rows padded to 64K; queries past 1024 rows run as
  // 1024-row segments (K = 16), one table per segment, concatenated
  std::vector<uint32_t> wt, wt16;
  const int wK = qlen <= 256 ? 4 : qlen <= 512 ? 8 : 16;
  const int wrows = 64 * wK;
  const int wsegs = std::max(1, (qlen + wrows - 1) / wrows);
  const uint32_t wPS = prof ? (uint32_t)wrows : 0, wPS16 = prof ? (uint32_t)wrows * 2 : 0;
  for (int sg = 0; sg < wsegs; ++sg) {
    const int r0 = sg * wrows, nr = std::min(wrows, std::max(0, qlen - r0));
    if (!prof) {
      const size_t base = wt.size();
      wt.resize(base + wrows, 0xFFFFFFFFu);
      for (int i = 0; i < nr; ++i) {
        uint32_t w = 0;
        for (int c = 0; c < 4; ++c)
          w |= (uint32_t)(uint8_t)(S - m[b->query[r0 + i] * A + c]) << (8 * c);
        wt[base + i] = w;
      }
      if (f16) {
        const size_t b16 = wt16.size();
        wt16.resize(b16 + wrows, 0xE8E8E8E8u);  // rows past the query: -2048
        for (int i = 0; i < nr; ++i) {
          uint32_t w = 0;
          for (int c = 0; c < 4; ++c) {
            uint8_t h;
            f16_hi(m[b->query[r0 + i] * A + c], &h);
            w |= (uint32_t)h << (8 * c);
          }
          wt16[b16 + i] = w;
        }
      }
    } else {
      std::vector<uint8_t> qp((size_t)(A + 1) * wPS, 0xFF);
      for (int c = 0; c < A; ++c)
        for (int i = 0; i < nr; ++i)
          qp[(size_t)c * wPS + i] = (uint8_t)(S - m[b->query[r0 + i] * A + c]);
      const size_t base = wt.size();
      wt.resize(base + qp.size() / 4);
      std::memcpy(wt.data() + base, qp.data(), qp.size());
      if (f16) {
        std::vector<uint16_t> q16((size_t)(A + 1) * wrows, 0xE800u);
        for (int c = 0; c < A; ++c)
          for (int i = 0; i < nr; ++i)
            q16[(size_t)c * wrows + i] =
                __builtin_bit_cast(uint16_t, (_Float16)(float)m[b->query[r0 + i] * A + c]);
        const size_t b16 = wt16.size();
        wt16.resize(b16 + q16.size() / 2);
        std::memcpy(wt16.data() + b16, q16.data(), q16.size() * 2);
      }
    }
  }
  HIPOK(b, hipSetDevice(b->device));
  if (!b->ev_ready) {
    HIPOK(b, hipEventCreateWithFlags(&b->ev_ready, hipEventDisableTiming));
    HIPOK(b, hipEventCreateWithFlags(&b->ev_used, hipEventDisableTiming));
    HIPOK(b, hipEventRecord(b->ev_ready, b->stream));
    HIPOK(b, hipEventRecord(b->ev_used, b->stream));
  }
  // the previous upload must have left the staging buffer before it is refilled
  HIPOK(b, hipEventSynchronize(b->ev_ready));
  const size_t nbytes = (wt16.size() + wt.size() + tab.size() + tab16.size()) * 4;
  HIPOK(b, b->stage.reserve(nbytes));
  // earlier launches (any stream) must be done reading the tables this upload overwrites
  HIPOK(b, hipStreamWaitEvent(b->stream, b->ev_used, 0));
  size_t at = 0;
  auto upload = [&](DevBuf<uint32_t>& dst, const std::vector<uint32_t>& src) -> hipError_t {
    hipError_t e = dst.reserve(src.size());
    if (e != hipSuccess || src.empty()) return e;
    std::memcpy(b->stage.p + at, src.data(), src.size() * 4);
    e = hipMemcpyAsync(dst.p, b->stage.p + at, src.size() * 4, hipMemcpyHostToDevice, b->stream);
    at += src.size() * 4;
    return e;
  };
  if (!wt16.empty()) HIPOK(b, upload(b->wtab16, wt16));
  HIPOK(b, upload(b->wtab, wt));
  b->wPS16 = wPS16;
  b->wK = wK;
  b->wPS = wPS;
  b->wsegs = wsegs;
  b->wseg_words = wt.size() / wsegs;
  b->wseg_words16 = wt16.empty() ? 0 : wt16.size() / wsegs;
  HIPOK(b, upload(b->qtab, tab));
  if (f16) HIPOK(b, upload(b->qtab16, tab16));
  HIPOK(b, hipEventRecord(b->ev_ready, b->stream));
  b->f16 = f16;
  b->nv16 = (uint32_t)hN * 0x01010101u;
  b->PS16 = PS16;
  b->f16_neg = -(o + 2 * e + (S - smin));
  b->R = R;
  b->RB = RB;
  b->W = segs[0].W;
  b->segs = segs;
  b->S = (uint32_t)S;
  b->O = (uint32_t)o;
  b->E = (uint32_t)e;
  b->nv = nv;
  b->PS = PS;
  b->pad = pad;
  b->prof = prof;
  b->smax = smax;
  b->col0 = col0;
  b->dirty = false;
  return SW_OK;
}

static sw_status range_check(sw_bank* b, uint32_t max_len) {
  const uint64_t qlen = b->query.size();
  const uint64_t cells = std::min<uint64_t>(qlen, max_len);
  const uint64_t top = cells * (uint64_t)std::max(0, b->smax) + b->S;
  if (top > 65535u)
    return fail(b, SW_ERR_RANGE, "max score bound %llu exceeds the 16-bit lanes",
                (unsigned long long)top);
  return SW_OK;
}

// packed: d_res holds n 64-byte CAPI records (2-bit codes); d_offs/d_lens are unused.
static sw_status launch(sw_bank* b, const uint8_t* d_res, const uint64_t* d_offs,
                        const uint32_t* d_lens, size_t n, uint32_t max_len, int32_t* d_scores,
                        hipStream_t st, bool packed = false) {
  sw_bank::Ev ev{};
  if (b->timing) {
    HIPOK(b, hipEventCreate(&ev.a));
    HIPOK(b, hipEventCreate(&ev.b));
    HIPOK(b, hipEventCreate(&ev.c));
    HIPOK(b, hipEventRecord(ev.a, st));
  }
  // no separate feeder kernel: the score kernel streams the codes itself, so the "pack"
  // interval (a..b) is empty and kept only for ABI stability
  if (b->timing) HIPOK(b, hipEventRecord(ev.b, st));
  HIPOK(b, hipStreamWaitEvent(st, b->ev_ready, 0));  // the query tables are uploaded
  const size_t nseg = b->segs.size();
  const uint32_t ecols = (max_len + 7) / 8 * 8;
  const size_t ntiles = (n + SWB_TILE - 1) / SWB_TILE;
  const bool gotoh = b->cfg.gap_model == SW_GAP_GOTOH;
  // f16 arithmetic (8 VALU per 2 cells instead of 9) when every value the recurrence can
  // reach is an exact f16 integer: the positive bound min(|q|, max|t|) * max(s) + max(s)
  // and the most negative intermediate both within 2048
  const uint64_t top = std::min<uint64_t>(b->query.size(), max_len) * (uint64_t)std::max(0, b->smax) +
                       (uint64_t)std::max(0, b->smax);
  // Past that bound the f16 pass is still exact for every pair whose computed score stays
  // <= 2048 - max(s): a first rounded value needs an exact H > 2048 - max(s) on its
  // diagonal, and the running max keeps it.  Optimistic mode scores all pairs in f16, then
  // re-scores the pairs above that threshold in u16 (SWBANK_F16_OPT=0 disables).
  const bool f16_ok = b->f16 && b->f16_neg >= -2048 && env_int("SWBANK_F16", 1) != 0;
  const bool exact16 = f16_ok && top <= 2048u;
  const bool opt16 = f16_ok && !exact16 && env_int("SWBANK_F16_OPT", 1) != 0 &&
                     n <= 0xFFFFFFFFull;  // the re-score list holds 32-bit target numbers
  const bool use_f16 = exact16 || opt16;
  // Kernel choice by a throughput model calibrated on MI355X (scripts/kernel_choice.py):
  //  tile kernel: base rate x fraction of the 256 CUs holding a tile x f(waves per SIMD),
  //    f = min(1, 0.45 + 0.15 w), x 0.85 when the query runs as several segments;
  //  wave kernel (queries <= 1024 rows): base rate x row fill (query / 64K lanes' rows) x
  //    column fill (L / (L + 63): the 63-step skew of the lane pipeline).
  // Base GCUPS: tile f16 merged 9000 (profile 8000), f16 Gotoh 7500 (profile 7100), u16
  // merged 7400 (profile 6500), u16 Gotoh 5800 (profile 5600); wave f16 merged 8600
  // (profile 7700), f16 Gotoh 7800 (profile 6800), u16 merged 7600 (profile 6600), u16 Gotoh
  // 6100 (profile 5200).  SWBANK_KERNEL=tile|wave forces one.
  const double tiles = (double)ntiles, W = b->segs[0].W;
  const double cu_frac = std::min(1.0, tiles / 256.0);
  const double wps = std::min(4.0, std::max(1.0, std::ceil(tiles / 256.0)) * W / 4.0);
  const double tile_base = use_f16 ? (gotoh ? (b->prof ? 7100 : 7500) : (b->prof ? 8000 : 9000))
                                   : (gotoh ? (b->prof ? 5600 : 5800) : (b->prof ? 6500 : 7400));
  const double tile_est = tile_base * cu_frac * std::min(1.0, 0.45 + 0.15 * wps) *
                          (nseg > 1 ? 0.85 : 1.0);
  double wave_est = 0;
  if (b->wK > 0) {
    const double rowfill = (double)b->query.size() / (64.0 * b->wK * b->wsegs);
    const double colfill = max_len / (max_len + 63.0);
    const double wave_base = use_f16 ? (gotoh ? (b->prof ? 6800 : 7800) : (b->prof ? 7700 : 8600))
                                     : (gotoh ? (b->prof ? 5200 : 6100) : (b->prof ? 6600 : 7600));
    wave_est = wave_base * rowfill * colfill *
               (b->wsegs > 1 ? 0.9 : 1.0);
  }
  const char* kforce = std::getenv("SWBANK_KERNEL");
  bool use_wave = b->wK > 0 && wave_est > tile_est;
  if (kforce && std::strcmp(kforce, "tile") == 0) use_wave = false;
  if (kforce && std::strcmp(kforce, "wave") == 0 && b->wK > 0) use_wave = true;
  // the f16 wave kernel carries profile offsets in 16-bit halves (24 letters + pad fit)
  if (use_f16 && b->prof && (size_t)(b->alpha + 1) * b->wPS16 > 65536) use_wave = false;
  const char* arith = opt16 ? "f16+u16-rescore" : use_f16 ? "f16" : "u16";
  if (use_wave) {
    snprintf(b->last_kernel, sizeof(b->last_kernel), "wave %s%s K=%d segs=%d", arith,
             b->prof ? "-profile" : "", b->wK, b->wsegs);
    // segments hand the bottom row on through HBM: pairs x ecols x 8 B per edge buffer,
    // in position ranges under SWBANK_EDGE_MB like the tile kernel
    size_t wspan = n;
    if (b->wsegs > 1) {
      const size_t budget = (size_t)std::max(1, env_int("SWBANK_EDGE_MB", 2048)) << 20;
      wspan = std::min(n, std::max<size_t>(1, budget / ((size_t)ecols * sizeof(uint2))) * 2);
      const size_t words = std::max<size_t>(1, (wspan + 1) / 2 * ecols);
      HIPOK(b, b->edge[0].reserve(words));
      HIPOK(b, b->edge[1].reserve(words));
    }
    for (size_t p0 = 0; p0 < n; p0 += wspan) {
      const size_t np = std::min(wspan, n - p0);
      for (int sg = 0; sg < b->wsegs; ++sg) {
        const void* ein = sg > 0 ? b->edge[(sg - 1) & 1].p : nullptr;
        void* eout = sg + 1 < b->wsegs ? b->edge[sg & 1].p : nullptr;
        HIPOK(b, swk_launch_wave(
                     b->wK, b->col0, b->prof, gotoh ? 1 : 0, use_f16 ? 1 : 0, ein, eout, ecols,
                     sg > 0 ? 1 : 0, packed ? d_res + p0 * SWB_RECORD : d_res,
                     packed ? d_offs : d_offs + p0, packed ? d_lens : d_lens + p0, np,
                     use_f16 ? b->wtab16.p + sg * b->wseg_words16 : b->wtab.p + sg * b->wseg_words,
                     use_f16 ? b->nv16 : b->nv, b->S, b->O, b->E,
                     use_f16 && b->prof ? b->wPS16 : b->wPS, b->pad, d_scores + p0,
                     packed ? 1 : 0, st));
      }
    }
  } else {
    snprintf(b->last_kernel, sizeof(b->last_kernel), "tile %s%s R=%d W=%d segs=%zu", arith,
             b->prof ? "-profile" : "", b->R, b->segs[0].W, nseg);
  }
  // Segmented queries hand each segment's bottom row to the next through HBM: ntiles x ecols
  // x 512 B per edge buffer.  Past SWBANK_EDGE_MB (default 2048) the batch runs as
  // consecutive position ranges, each with its own edge rows.
  size_t span = n;
  if (nseg > 1) {
    const size_t budget = (size_t)std::max(1, env_int("SWBANK_EDGE_MB", 2048)) << 20;
    const size_t per_tile = (size_t)ecols * 64 * sizeof(uint2);
    span = std::max<size_t>(1, budget / std::max<size_t>(per_tile, 1)) * SWB_TILE;
    span = std::min(span, n);
    if (!use_wave || opt16) {
      const size_t words = std::max<size_t>(1, (span + SWB_TILE - 1) / SWB_TILE * ecols * 64);
      HIPOK(b, b->edge[0].reserve(words));
      HIPOK(b, b->edge[1].reserve(words));
    }
  }
  // pass 0: every pair with the tile kernel (unless the wave kernel ran); pass 1 (optimistic
  // f16 only): the pairs scoring above 2048 - max(s), re-scored in u16 by the tile kernel
  for (int pass = use_wave ? 1 : 0; pass < (opt16 ? 2 : 1); ++pass) {
    const bool f16 = use_f16 && pass == 0;
    if (pass == 1) {
      HIPOK(b, b->fb_idx.reserve(n));
      HIPOK(b, b->fb_cnt.reserve(1));
      HIPOK(b, swk_flag_high(d_scores, n, 2048 - std::max(0, b->smax), b->fb_idx.p, b->fb_cnt.p,
                             st));
    }
    for (size_t p0 = 0; p0 < n; p0 += span) {
      const size_t np = std::min(span, n - p0);
      // pass 0 offsets the batch arrays; pass 1 keeps them whole (idx holds target numbers)
      const uint8_t* res = d_res;
      const uint64_t* offs = d_offs;
      const uint32_t* lens = d_lens;
      int32_t* scores = d_scores;
      const uint32_t* idx = nullptr;
      if (pass == 0 && packed) {
        res = d_res + p0 * SWB_RECORD;
        scores = d_scores + p0;
      } else if (pass == 0) {
        offs = d_offs + p0;
        lens = d_lens + p0;
        scores = d_scores + p0;
      } else {
        idx = b->fb_idx.p + p0;
      }
      for (size_t s = 0; s < nseg; ++s) {
        const void* ein = s > 0 ? b->edge[(s - 1) & 1].p : nullptr;
        void* eout = s + 1 < nseg ? b->edge[s & 1].p : nullptr;
        HIPOK(b, swk_launch_score(b->R, b->RB, b->col0, b->prof, gotoh ? 1 : 0, f16 ? 1 : 0, res,
                                  offs, lens, np,
                                  f16 ? b->qtab16.p + b->segs[s].off16
                                      : b->qtab.p + b->segs[s].off,
                                  f16 ? b->nv16 : b->nv, b->S, b->O, b->E,
                                  f16 && b->prof ? b->PS16 : b->PS, b->pad, b->segs[s].W,
                                  scores, ein, eout, ecols, s > 0 ? 1 : 0, packed ? 1 : 0, idx,
                                  idx ? b->fb_cnt.p : nullptr, (uint32_t)p0, st));
      }
    }
  }
  HIPOK(b, hipEventRecord(b->ev_used, st));  // the next table upload waits for this
  if (b->timing) {
    HIPOK(b, hipEventRecord(ev.c, st));
    b->events.push_back(ev);
  }
  return SW_OK;
}

extern "C" sw_status sw_score_batch_device(sw_bank* b, const uint8_t* d_res,
                                           const uint64_t* d_offs, const uint32_t* d_lens,
                                           size_t n, uint32_t max_len, int32_t* d_scores,
                                           void* stream) {
  if (!b) return SW_ERR_ARG;
  if (n == 0) return SW_OK;
  if (!d_res || !d_offs || !d_lens || !d_scores) return fail(b, SW_ERR_ARG, "null device buffer");
  sw_status st = prepare(b);
  if (st != SW_OK) return st;
  if ((st = range_check(b, max_len)) != SW_OK) return st;
  HIPOK(b, hipSetDevice(b->device));
  return launch(b, d_res, d_offs, d_lens, n, max_len, d_scores,
                stream ? reinterpret_cast<hipStream_t>(stream) : b->stream);
}

extern "C" sw_status sw_score_batch(sw_bank* b, const uint8_t* residues, const uint64_t* offsets,
                                    const uint32_t* lens, size_t n, int32_t* scores_out) {
  if (!b) return SW_ERR_ARG;
  if (n == 0) return SW_OK;
  if (!offsets || !lens || !scores_out) return fail(b, SW_ERR_ARG, "null host buffer");
  sw_status st = prepare(b);
  if (st != SW_OK) return st;

  // Feeder order: longest targets first so each 128-target tile has similar lengths
  // (the RTL's PrioEncoder routes to the first free module, ScoreBank_v2.v:142-148).
  std::vector<uint32_t> order(n);
  std::iota(order.begin(), order.end(), 0u);
  std::stable_sort(order.begin(), order.end(),
                   [&](uint32_t a, uint32_t c) { return lens[a] > lens[c]; });
  uint32_t max_len = n ? lens[order[0]] : 0;
  if (max_len && !residues) return fail(b, SW_ERR_ARG, "null residues");
  if ((st = range_check(b, max_len)) != SW_OK) return st;

  size_t total = 0;
  for (size_t k = 0; k < n; ++k) total += lens[k];
  std::vector<uint8_t> hres(std::max<size_t>(total, 1));
  std::vector<uint64_t> hoffs(n);
  std::vector<uint32_t> hlens(n);
  size_t pos = 0;
  for (size_t k = 0; k < n; ++k) {
    const uint32_t src = order[k];
    const uint8_t* p = residues + offsets[src];
    for (uint32_t j = 0; j < lens[src]; ++j)
      if (p[j] >= (uint32_t)b->alpha)
        return fail(b, SW_ERR_ARG, "target %u code %u outside alphabet", src, p[j]);
    std::memcpy(hres.data() + pos, p, lens[src]);
    hoffs[k] = pos;
    hlens[k] = lens[src];
    pos += lens[src];
  }

  HIPOK(b, hipSetDevice(b->device));
  HIPOK(b, b->res.reserve(hres.size()));
  HIPOK(b, b->offs.reserve(n));
  HIPOK(b, b->lens.reserve(n));
  HIPOK(b, b->scores.reserve(n));
  HIPOK(b, hipMemcpyAsync(b->res.p, hres.data(), hres.size(), hipMemcpyHostToDevice, b->stream));
  HIPOK(b, hipMemcpyAsync(b->offs.p, hoffs.data(), n * 8, hipMemcpyHostToDevice, b->stream));
  HIPOK(b, hipMemcpyAsync(b->lens.p, hlens.data(), n * 4, hipMemcpyHostToDevice, b->stream));
  st = launch(b, b->res.p, b->offs.p, b->lens.p, n, max_len, b->scores.p, b->stream);
  if (st != SW_OK) return st;
  std::vector<int32_t> sorted(n);
  HIPOK(b, hipMemcpyAsync(sorted.data(), b->scores.p, n * 4, hipMemcpyDeviceToHost, b->stream));
  HIPOK(b, hipStreamSynchronize(b->stream));
  for (size_t k = 0; k < n; ++k) scores_out[order[k]] = sorted[k];
  return SW_OK;
}

// ---- CAPI record path (row f2): sequence_t arrays as the reference host builds them ------
static inline uint32_t record_len(const uint8_t* rec) {
  uint16_t l;
  std::memcpy(&l, rec + 4, 2);
  return l;
}

extern "C" sw_status sw_load_query_record(sw_bank* b, const void* record) {
  if (!b || !record) return SW_ERR_ARG;
  if (b->alpha != SW_DNA_ALPHA) return fail(b, SW_ERR_UNSUPPORTED, "records carry DNA only");
  const uint8_t* rec = static_cast<const uint8_t*>(record);
  const uint32_t len = record_len(rec);
  if (len > SWB_RECORD_MAX) return fail(b, SW_ERR_ARG, "record length %u > %u", len, SWB_RECORD_MAX);
  uint32_t id;
  std::memcpy(&id, rec, 4);
  uint8_t codes[SWB_RECORD_MAX];
  for (uint32_t j = 0; j < len; ++j) codes[j] = (rec[6 + j / 4] >> (2 * (j % 4))) & 3u;
  return sw_load_query(b, id, codes, len);
}

extern "C" sw_status sw_score_records_device(sw_bank* b, const void* d_records, size_t n,
                                             int32_t* d_scores, void* stream) {
  if (!b) return SW_ERR_ARG;
  if (n == 0) return SW_OK;
  if (!d_records || !d_scores) return fail(b, SW_ERR_ARG, "null device buffer");
  if (b->alpha != SW_DNA_ALPHA) return fail(b, SW_ERR_UNSUPPORTED, "records carry DNA only");
  sw_status st = prepare(b);
  if (st != SW_OK) return st;
  // lengths live on the device: bound them by the record capacity
  if ((st = range_check(b, SWB_RECORD_MAX)) != SW_OK) return st;
  HIPOK(b, hipSetDevice(b->device));
  return launch(b, static_cast<const uint8_t*>(d_records), nullptr, nullptr, n, SWB_RECORD_MAX,
                d_scores, stream ? reinterpret_cast<hipStream_t>(stream) : b->stream, true);
}

extern "C" sw_status sw_score_records(sw_bank* b, const void* records, size_t n,
                                      int32_t* scores_out) {
  if (!b) return SW_ERR_ARG;
  if (n == 0) return SW_OK;
  if (!records || !scores_out) return fail(b, SW_ERR_ARG, "null host buffer");
  if (b->alpha != SW_DNA_ALPHA) return fail(b, SW_ERR_UNSUPPORTED, "records carry DNA only");
  sw_status st = prepare(b);
  if (st != SW_OK) return st;
  const uint8_t* recs = static_cast<const uint8_t*>(records);
  std::vector<uint32_t> order(n);
  std::iota(order.begin(), order.end(), 0u);
  for (size_t k = 0; k < n; ++k)
    if (record_len(recs + k * SWB_RECORD) > SWB_RECORD_MAX)
      return fail(b, SW_ERR_ARG, "record %zu length %u > %u", k, record_len(recs + k * SWB_RECORD),
                  SWB_RECORD_MAX);
  // longest first, as sw_score_batch (PrioEncoder order)
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t c) {
    return record_len(recs + (size_t)a * SWB_RECORD) > record_len(recs + (size_t)c * SWB_RECORD);
  });
  const uint32_t max_len = record_len(recs + (size_t)order[0] * SWB_RECORD);
  if ((st = range_check(b, max_len)) != SW_OK) return st;
  std::vector<uint8_t> sorted(n * SWB_RECORD);
  for (size_t k = 0; k < n; ++k)
    std::memcpy(sorted.data() + k * SWB_RECORD, recs + (size_t)order[k] * SWB_RECORD, SWB_RECORD);
  HIPOK(b, hipSetDevice(b->device));
  HIPOK(b, b->res.reserve(sorted.size()));
  HIPOK(b, b->scores.reserve(n));
  HIPOK(b, hipMemcpyAsync(b->res.p, sorted.data(), sorted.size(), hipMemcpyHostToDevice,
                          b->stream));
  st = launch(b, b->res.p, nullptr, nullptr, n, max_len, b->scores.p, b->stream, true);
  if (st != SW_OK) return st;
  std::vector<int32_t> out(n);
  HIPOK(b, hipMemcpyAsync(out.data(), b->scores.p, n * 4, hipMemcpyDeviceToHost, b->stream));
  HIPOK(b, hipStreamSynchronize(b->stream));
  for (size_t k = 0; k < n; ++k) scores_out[order[k]] = out[k];
  return SW_OK;
}

extern "C" sw_status sw_bank_set_timing(sw_bank* b, int32_t enable) {
  if (!b) return SW_ERR_ARG;
  b->timing = enable != 0;
  return SW_OK;
}

extern "C" sw_status sw_bank_timing(sw_bank* b, uint64_t* launches, double* pack_ms,
                                    double* score_ms) {
  if (!b) return SW_ERR_ARG;
  double p = 0, s = 0;
  uint64_t n = 0;
  sw_status st = SW_OK;
  for (auto& ev : b->events) {
    float t1 = 0, t2 = 0;
    if (st == SW_OK && hipEventSynchronize(ev.c) == hipSuccess &&
        hipEventElapsedTime(&t1, ev.a, ev.b) == hipSuccess &&
        hipEventElapsedTime(&t2, ev.b, ev.c) == hipSuccess) {
      p += t1;
      s += t2;
      ++n;
    } else {
      st = fail(b, SW_ERR_HIP, "event timing failed");
    }
    (void)hipEventDestroy(ev.a);
    (void)hipEventDestroy(ev.b);
    (void)hipEventDestroy(ev.c);
  }
  b->events.clear();
  if (launches) *launches = n;
  if (pack_ms) *pack_ms = p;
  if (score_ms) *score_ms = s;
  return st;
}

extern "C" sw_status sw_best_hit_device(sw_bank* b, const int32_t* d_scores, const uint64_t* d_ids,
                                        size_t n, uint64_t* d_out, void* stream) {
  if (!b) return SW_ERR_ARG;
  if (!d_scores || !d_out || n == 0 || n > 0xFFFFFFFFull)
    return fail(b, SW_ERR_ARG, "sw_best_hit_device: empty, null or > 2^32 scores");
  HIPOK(b, hipSetDevice(b->device));
  HIPOK(b, b->best_key.reserve(1));
  HIPOK(b, swk_best_hit(d_scores, d_ids, n, b->best_key.p, d_out,
                        stream ? reinterpret_cast<hipStream_t>(stream) : b->stream));
  return SW_OK;
}

extern "C" sw_status sw_best_hit(sw_bank* b, const int32_t* scores, const uint64_t* ids, size_t n,
                                 uint64_t* best_id, int32_t* best_score) {
  if (!scores || !best_id || !best_score || n == 0)
    return b ? fail(b, SW_ERR_ARG, "sw_best_hit: empty or null input") : SW_ERR_ARG;
  size_t bi = 0;
  for (size_t k = 1; k < n; ++k)
    if (scores[k] > scores[bi]) bi = k;
  *best_id = ids ? ids[bi] : (uint64_t)bi;
  *best_score = scores[bi];
  return SW_OK;
}
