// swbank_kaux.hip — the small kernels around the score kernels: the int32 re-score past
// the 16-bit lanes, the on-device length sort (§3.6), the best hit
// (§2), the multi-device deal (§7).
#include "swbank_kcommon.h"

namespace swk {
// Pairs an optimistic f16 pass may have rounded: score > thresh (= 2048 - max s) -> idx list.
__global__ void __launch_bounds__(256) flag_kernel(const int32_t* scores, size_t n,
                                                   int32_t thresh, uint32_t* idx,
                                                   uint32_t* count) {
  const size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (k < n && scores[k] > thresh) idx[atomicAdd(count, 1u)] = (uint32_t)k;
}
}  // namespace swk

namespace swk {
// Bank best hit on the device (≙ ScoreBank_v2 max/vld_max): key = biased score << 32 |
// (2^32 - 1 - index), so one 64-bit max picks the highest score and, among equals, the
// lowest index.  Block-level max in LDS, one atomicMax per block.
__global__ void __launch_bounds__(256) best_kernel(const int32_t* scores, size_t n, size_t base,
                                                   unsigned long long* key) {
  __shared__ unsigned long long red[256];
  unsigned long long m = 0;
  for (size_t k = (size_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (size_t)gridDim.x * 256) {
    const unsigned long long v = ((unsigned long long)((uint32_t)scores[k] ^ 0x80000000u) << 32) |
                                 (0xFFFFFFFFull - (uint32_t)(base + k));
    m = v > m ? v : m;
  }
  red[threadIdx.x] = m;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w && red[threadIdx.x + w] > red[threadIdx.x])
      red[threadIdx.x] = red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicMax(key, red[0]);
}
__global__ void best_finalize(const unsigned long long* key, const uint64_t* ids, uint64_t* out,
                              uint64_t* out_index) {
  const unsigned long long v = *key;
  const uint64_t idx = 0xFFFFFFFFull - (v & 0xFFFFFFFFull);
  out[0] = ids ? ids[idx] : idx;
  out[1] = (uint64_t)(int64_t)(int32_t)((uint32_t)(v >> 32) ^ 0x80000000u);
  if (out_index) *out_index = idx;
}
}  // namespace swk

// Fold scores[0, n) (batch positions base + k) into the 64-bit best key (zeroed by the caller
// before the first part); few blocks, so the contended atomicMax stays cheap (2048 blocks cost
// ~25 us on 1 M scores, 256 about 3).
extern "C" hipError_t swk_best_part(const int32_t* scores, size_t n, size_t base,
                                    unsigned long long* key, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const size_t blocks = std::min<size_t>((n + 2047) / 2048, 256);
  hipLaunchKernelGGL(swk::best_kernel, dim3((unsigned)blocks), dim3(256), 0, st, scores, n, base,
                     key);
  return hipGetLastError();
}

// out[0] = best id (ids ? ids[index] : index), out[1] = best score (sign-extended), *out_index
// (optional) = its index, from the key.
extern "C" hipError_t swk_best_finalize(const unsigned long long* key, const uint64_t* ids,
                                        uint64_t* out, uint64_t* out_index, hipStream_t st) {
  hipLaunchKernelGGL(swk::best_finalize, dim3(1), dim3(1), 0, st, key, ids, out, out_index);
  return hipGetLastError();
}

// out[0] = best id, out[1] = best score (sign-extended), *out_index (optional) = its index;
// key: 8 bytes of device scratch.
extern "C" hipError_t swk_best_hit(const int32_t* scores, const uint64_t* ids, size_t n,
                                   unsigned long long* key, uint64_t* out, uint64_t* out_index,
                                   hipStream_t st) {
  hipError_t e = hipMemsetAsync(key, 0, sizeof(*key), st);
  if (e == hipSuccess) e = swk_best_part(scores, n, 0, key, st);
  if (e == hipSuccess) e = swk_best_finalize(key, ids, out, out_index, st);
  return e;
}

// ---- the deal of a multi-device bank's device batch (swbank_multi.hip) -------------------
namespace swk {
__device__ __forceinline__ size_t deal_target(const uint32_t* perm, bool id, size_t p) {
  return id ? p : (size_t)perm[p];
}
// A wave takes 64 positions at a time: lane l reads position l's metadata (one coalesced load
// per array), then each 16-lane quarter copies one position per step, 4 per step, lane k of a
// quarter chunk k (8 codes), the chunks past the 16th (targets over 128 codes) after.  A chunk
// is read as the 2-3 aligned dwords that hold it, each loaded only when it holds a byte of the
// target (an aligned dword never crosses a page, so no read can fault past the buffer), and
// funnel-shifted (v_alignbyte): no branch around a load, so all 16 steps' loads are in flight
// before the first store.  Each chunk goes out as one u64 of bytes or one u32 of 4-bit codes.
// (Byte loads for a target's last chunk serialised the steps on their waits: 134 us for the
// ragged bench batch; one wave per position, or one lane per position looping over its chunks:
// 3-4x slower still.  DESIGN 3.6)
__device__ __forceinline__ uint32_t nib_pack4(uint32_t w) {  // 4 code bytes -> 16 bits
  uint32_t t = w & 0x0F0F0F0Fu;
  t = (t | (t >> 4)) & 0x00FF00FFu;
  return (t | (t >> 8)) & 0x0000FFFFu;
}
struct DealWords {  // the aligned dwords holding one 8-code chunk
  uint32_t w0, w1, w2;
};
__device__ __forceinline__ DealWords deal_load(const uint8_t* src, uint32_t L, uint32_t j) {
  DealWords r{0u, 0u, 0u};
  const uint32_t m = (uint32_t)(reinterpret_cast<uintptr_t>(src + j) & 3);
  // (pointer arithmetic from src, not from an integer: the loads stay global, not flat)
  const uint32_t* ap = reinterpret_cast<const uint32_t*>(src + j - m);
  const uint32_t e = L - j + m;  // bytes from the first dword's start to the target's end
  if (j < L) r.w0 = ap[0];
  if (j < L && e > 4) r.w1 = ap[1];
  if (j < L && m && e > 8) r.w2 = ap[2];
  return r;
}
// the chunk's 8 codes (zero past the target's end)
__device__ __forceinline__ uint2 deal_codes(const DealWords& w, const uint8_t* src, uint32_t L,
                                            uint32_t j) {
  const uint32_t m = (uint32_t)((reinterpret_cast<uintptr_t>(src) + j) & 3);
  uint2 v = make_uint2(__builtin_amdgcn_alignbyte(w.w1, w.w0, m),
                       __builtin_amdgcn_alignbyte(w.w2, w.w1, m));
  const uint32_t nv = L > j ? min(L - j, 8u) : 0u;
  if (nv < 8) {
    const uint64_t keep = (1ull << (8 * nv)) - 1;
    const uint64_t x = ((uint64_t)v.y << 32 | v.x) & keep;
    v = make_uint2((uint32_t)x, (uint32_t)(x >> 32));
  }
  return v;
}
__global__ void __launch_bounds__(256) deal_gather(const uint8_t* res, const uint64_t* offs,
                                                   const uint32_t* lens, const uint32_t* perm,
                                                   const uint32_t* ident, size_t n,
                                                   const SwkDeal dl) {
  const uint32_t lane = threadIdx.x & 63, qd = lane >> 4, ql = lane & 15;
  const size_t w0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  const bool id = !perm || (ident && *ident != 0);
  const bool wide = (dl.stride & 7u) == 0;  // whole u64 stores stay inside the slot
  const auto store = [&](uint8_t* dst, uint32_t L, uint32_t c, uint2 v) {
    const uint32_t j = c * 8;
    if (dl.nib) {  // code k of the chunk in nibble k (SWK_PACK_NIBBLE)
      *reinterpret_cast<uint32_t*>(dst + (size_t)c * 4) = nib_pack4(v.x) | nib_pack4(v.y) << 16;
    } else if (wide) {
      *reinterpret_cast<uint2*>(dst + j) = v;
    } else {
      const uint64_t x = (uint64_t)v.y << 32 | v.x;
#pragma unroll
      for (uint32_t k = 0; k < 8; ++k)
        if (j + k < L) dst[j + k] = (uint8_t)(x >> (8 * k));
    }
  };
  for (size_t base = w0 * 64; base < n; base += nw * 64) {
    const size_t p = base + lane;
    const bool live = p < n;
    const size_t t = live ? deal_target(perm, id, p) : 0;
    const uint32_t Lm = live ? lens[t] : 0u;
    const uint64_t om = live ? offs[t] : 0u;
    const uint32_t dm = (uint32_t)(p % dl.D);
    const uint64_t im = p / dl.D;
    if (live) {
      dl.offs[dm][im] = im * dl.stride;
      dl.lens[dm][im] = Lm;
    }
    // position 4 s + qd's source and slot (the metadata from its lane; every lane active)
    const auto src_of = [&](int sl) {
      const uint64_t o = (uint64_t)(uint32_t)__shfl((int)(uint32_t)om, sl) |
                         (uint64_t)(uint32_t)__shfl((int)(uint32_t)(om >> 32), sl) << 32;
      return res + o;
    };
    const auto dst_of = [&](int sl) {
      const uint32_t d = (uint32_t)__shfl((int)dm, sl);
      const uint64_t i = (uint64_t)(uint32_t)__shfl((int)(uint32_t)im, sl) |
                         (uint64_t)(uint32_t)__shfl((int)(uint32_t)(im >> 32), sl) << 32;
      return dl.codes[d] + i * dl.stride;
    };
    DealWords w[16];
    uint32_t Ls[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {  // loads: position 4 s + qd, chunk ql
      const int sl = 4 * s + (int)qd;
      Ls[s] = (uint32_t)__shfl((int)Lm, sl);  // (0 past the batch end)
      w[s] = deal_load(src_of(sl), Ls[s], ql * 8);
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int sl = 4 * s + (int)qd;
      const uint8_t* src = src_of(sl);
      uint8_t* dst = dst_of(sl);
      if (ql * 8 < Ls[s]) store(dst, Ls[s], ql, deal_codes(w[s], src, Ls[s], ql * 8));
    }
    for (int s = 0; s < 16; ++s) {  // chunks 16 on (targets of more than 128 codes)
      const int sl = 4 * s + (int)qd;
      if (__builtin_amdgcn_readfirstlane(__ballot(Ls[s] > 128u) != 0)) {
        const uint8_t* src = src_of(sl);
        uint8_t* dst = dst_of(sl);
        for (uint32_t c = ql + 16; c * 8 < Ls[s]; c += 16)
          store(dst, Ls[s], c, deal_codes(deal_load(src, Ls[s], c * 8), src, Ls[s], c * 8));
      }
    }
  }
}
__global__ void __launch_bounds__(256) deal_scatter(const uint32_t* perm, const uint32_t* ident,
                                                    size_t n, unsigned nq, size_t sstride,
                                                    const SwkDeal dl, int32_t* out) {
  const bool id = !perm || (ident && *ident != 0);
  const size_t total = n * nq;
  for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < total;
       x += (size_t)gridDim.x * blockDim.x) {
    const size_t q = x / n, p = x % n;
    const unsigned d = (unsigned)(p % dl.D);
    out[q * sstride + deal_target(perm, id, p)] = dl.scores[d][q * dl.cnt[d] + p / dl.D];
  }
}
}  // namespace swk

extern "C" hipError_t swk_deal_gather(const uint8_t* res, const uint64_t* offs,
                                      const uint32_t* lens, const uint32_t* perm,
                                      const uint32_t* ident, size_t n, const SwkDeal* deal,
                                      hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (!deal || deal->D == 0 || deal->D > SWK_DEAL_MAX || deal->stride == 0) return hipErrorInvalidValue;
  const size_t blocks = std::min<size_t>((n + 255) / 256, (size_t)1 << 20);  // 64 per wave
  hipLaunchKernelGGL(swk::deal_gather, dim3((unsigned)blocks), dim3(256), 0, st, res, offs, lens,
                     perm, ident, n, *deal);
  return hipGetLastError();
}

extern "C" hipError_t swk_deal_scatter(const uint32_t* perm, const uint32_t* ident, size_t n,
                                       unsigned nq, size_t sstride, const SwkDeal* deal,
                                       int32_t* out, hipStream_t st) {
  if (n == 0 || nq == 0) return hipSuccess;
  if (!deal || deal->D == 0 || deal->D > SWK_DEAL_MAX) return hipErrorInvalidValue;
  const size_t blocks = std::min<size_t>((n * nq + 255) / 256, 8192);
  hipLaunchKernelGGL(swk::deal_scatter, dim3((unsigned)blocks), dim3(256), 0, st, perm, ident, n,
                     nq, sstride, *deal, out);
  return hipGetLastError();
}

extern "C" hipError_t swk_flag_high(const int32_t* scores, size_t n, int32_t thresh,
                                    uint32_t* idx, uint32_t* count, hipStream_t st) {
  hipError_t e = hipMemsetAsync(count, 0, sizeof(uint32_t), st);
  if (e != hipSuccess || n == 0) return e;
  hipLaunchKernelGGL(swk::flag_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     scores, n, thresh, idx, count);
  return hipGetLastError();
}

// ========================================================================================
// int32 kernel: exact scores past the 16-bit lanes (no bound on the score).  The u16 and f16
// passes are exact for every pair whose computed score stays <= 65535 - max(s) (resp. 2048 -
// max(s)): the first cell that would leave the lane range has an exact diagonal M above that
// threshold (a gap value is at most an earlier, exact H minus a penalty), and the running max
// keeps it.  So a batch past the 16-bit bound is scored by the 16-bit kernels as usual and the
// pairs above 65535 - max(s) are re-scored here (an index list, like the f16 -> u16 re-score).
//
// One wave per pair; strips of 256 query rows, lane l owns rows [4l, 4l+4) of a strip (the
// wave kernel's anti-diagonal walk: step t, lane l computes column t - l).  The strip's bottom
// row {H, T|F} goes to the next strip through a per-wave HBM scratch row (ping-pong, 64
// columns per coalesced load / store, readlane + a lane select per step).  Substitution scores come
// from a per-strip profile: for every letter, lane l's 4 rows as int16 (uint2), staged in the
// wave's own LDS slice (each lane reads only its own entries: no barrier).  Merged gaps apply
// the HDL's first-column rule always (it changes nothing unless max(s) > o + e), in the
// clamped form of the f16 kernels:
//   M = max(0, Hdiag + s)   I = j ? max(Tup, Tleft) : 0   H = max(M, I)   T = max(0, M-o-e, I-e)
// Gotoh (E, F one step ahead, floored at 0):
//   H = max(0, Hdiag + s, E, F)   HN = H - o - e   E' = max(0, HN, E - e)   F' = max(0, HN, F - e)
namespace swk {
constexpr int I32_K = 4, I32_LETTERS = 25;  // rows per lane; profile letters incl. padding

struct I32Args {
  const uint8_t* res;
  const uint64_t* offs;
  const uint32_t* lens;
  size_t n;
  uint32_t packed;
  const uint32_t* idx;   // optional: positions [0, min(n, *nidx - idx_base)) score idx[k]
  const uint32_t* nidx;
  uint32_t idx_base;
  const uint2* prof;     // [strip][letter 0..pad][lane] 4 x int16 (rows 4l..4l+3)
  uint32_t nstrips, qlen, pad, O, E;
  int32_t* scores;
  uint2* scratch;        // per wave: 2 x scols uint2
  uint32_t scols;
};

__device__ __forceinline__ uint32_t i32_code(const uint8_t* p, uint32_t c, uint32_t packed) {
  if (packed == SWK_PACK_BYTES) return p[c];
  if (packed == SWK_PACK_NIBBLE) return (p[c >> 1] >> (4 * (c & 1))) & 15u;
  return (p[c >> 2] >> (2 * (c & 3))) & 3u;  // records, 2-bit stream
}

__device__ __forceinline__ int32_t i32_lane0(int32_t inj, int32_t v) {  // wave_shr:1
  return __builtin_amdgcn_update_dpp(inj, v, 0x138, 0xF, 0xF, false);
}

template <bool GOTOH>
__global__ void __launch_bounds__(256) score_i32(const I32Args a) {
  __shared__ uint2 lp[4][I32_LETTERS][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const size_t gw = (size_t)blockIdx.x * 4 + wave, GW = (size_t)gridDim.x * 4;
  size_t n = a.n;
  if (a.idx) {
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(*a.nidx);
    n = cnt > a.idx_base ? min(a.n, (size_t)(cnt - a.idx_base)) : 0;
  }
  uint2* const scr[2] = {a.scratch + gw * 2 * a.scols, a.scratch + gw * 2 * a.scols + a.scols};
  const int32_t oe = (int32_t)(a.O + a.E), e = (int32_t)a.E;
  const uint32_t pad = a.pad;
  uint2 (&mine)[I32_LETTERS][64] = lp[wave];
  for (size_t p = gw; p < n; p += GW) {
    const size_t t = a.idx ? a.idx[p] : p;
    const uint8_t* tp;
    uint32_t L;
    if (a.packed == SWK_PACK_RECORDS) {
      tp = a.res + t * SWB_RECORD + 6;
      L = record_len(a.res + t * SWB_RECORD);
    } else {
      L = a.lens[t];
      tp = a.res + (L ? a.offs[t] : 0);
    }
    L = __builtin_amdgcn_readfirstlane(L);
    int32_t best = 0;
    for (uint32_t s = 0; s < a.nstrips && L; ++s) {
      for (uint32_t c = 0; c <= pad; ++c) mine[c][lane] = a.prof[((size_t)s * (pad + 1) + c) * 64 + lane];
      int32_t vmask[I32_K];
#pragma unroll
      for (int k = 0; k < I32_K; ++k)
        vmask[k] = s * 256u + (uint32_t)lane * I32_K + k < a.qlen ? -1 : 0;
      const bool seg_in = s > 0, seg_out = s + 1 < a.nstrips;
      const uint2* ein = scr[(s + 1) & 1];
      uint2* eout = scr[s & 1];
      int32_t H[I32_K], X[I32_K];
#pragma unroll
      for (int k = 0; k < I32_K; ++k) H[k] = X[k] = 0;
      int32_t botH = 0, botX = 0, prevUpH = 0;
      uint32_t code = pad, buf = pad;
      uint2 ebuf = make_uint2(0u, 0u), obuf = make_uint2(0u, 0u);
      const uint32_t nsteps = L + 63;
      for (uint32_t st = 0; st < nsteps; ++st) {
        if ((st & 63) == 0) {  // the next 64 columns: codes (and the previous strip's row)
          const uint32_t c = st + lane;
          buf = c < L ? min(i32_code(tp, c, a.packed), pad) : pad;
          if (seg_in) ebuf = c < L ? ein[c] : make_uint2(0u, 0u);
        }
        const uint32_t j = st - (uint32_t)lane;  // this lane's column (wraps when not started)
        code = (uint32_t)i32_lane0((int32_t)__builtin_amdgcn_readlane(buf, st & 63), (int32_t)code);
        const int32_t upH = i32_lane0(seg_in ? (int32_t)__builtin_amdgcn_readlane(ebuf.x, st & 63) : 0, botH);
        const int32_t upX = i32_lane0(seg_in ? (int32_t)__builtin_amdgcn_readlane(ebuf.y, st & 63) : 0, botX);
        const uint2 w = mine[code][lane];
        const int32_t sc[I32_K] = {(int32_t)(w.x << 16) >> 16, (int32_t)w.x >> 16,
                                   (int32_t)(w.y << 16) >> 16, (int32_t)w.y >> 16};
        if (j < L) {  // active: column j of the lane's 4 rows
          int32_t diag = prevUpH, up = upH, ux = upX;
#pragma unroll
          for (int k = 0; k < I32_K; ++k) {
            const int32_t D = diag + sc[k];
            diag = H[k];
            if constexpr (GOTOH) {
              const int32_t h = max(max(D, 0), max(X[k], ux));
              const int32_t hn = h - oe;
              X[k] = max(max(hn, 0), X[k] - e);  // E of (row, j+1)
              ux = max(max(hn, 0), ux - e);      // F of (row+1, j)
              H[k] = h;
              best = max(best, h & vmask[k]);
            } else {
              const int32_t M = max(D, 0);
              const int32_t I = j == 0 ? 0 : max(ux, X[k]);
              const int32_t h = max(M, I);
              ux = max(max(M - oe, I - e), 0);   // T: what the right and lower cells read
              X[k] = ux;
              H[k] = h;
              best = max(best, h & vmask[k]);
            }
            (void)up;
          }
          botH = H[I32_K - 1];
          botX = ux;
        }
        prevUpH = upH;
        if (seg_out) {  // lane 63's bottom row of column st - 63 -> eout
          const uint32_t c = st - 63;
          if (st >= 63) {
            const int32_t vh = __builtin_amdgcn_readlane(botH, 63);
            const int32_t vx = __builtin_amdgcn_readlane(botX, 63);
            const bool here = (uint32_t)lane == (c & 63);
            obuf.x = here ? (uint32_t)vh : obuf.x;
            obuf.y = here ? (uint32_t)vx : obuf.y;
            if ((c & 63) == 63 || c + 1 == L) {
              const uint32_t col = (c & ~63u) + lane;
              if (col < L) eout[col] = obuf;
            }
          }
        }
      }
      // the next strip's lane 0 reads these columns (same wave, same CU and L1): a
      // workgroup-scope fence orders the stores before those loads (no L2 write-back)
      if (seg_out) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) best = max(best, __shfl_xor(best, off));
    if (lane == 0) a.scores[t] = best;
  }
}
}  // namespace swk

// Waves to launch for n pairs of at most scols columns: one pair per wave at a time, up to
// 16 waves per CU, within the scratch budget (2 x scols x 8 B per wave).
extern "C" size_t swk_i32_waves(size_t n, uint32_t scols, size_t budget_bytes) {
  const size_t per = (size_t)std::max(scols, 1u) * 2 * sizeof(uint2);
  size_t w = std::min<size_t>(n, 256 * 16);
  w = std::min(w, std::max<size_t>(4, budget_bytes / per));
  return (w + 3) / 4 * 4;
}

extern "C" hipError_t swk_launch_i32(int gotoh, const uint8_t* res, const uint64_t* offs,
                                     const uint32_t* lens, size_t n, int packed,
                                     const uint32_t* idx, const uint32_t* nidx, uint32_t idx_base,
                                     const void* prof, uint32_t nstrips, uint32_t qlen,
                                     uint32_t pad, uint32_t O, uint32_t E, int32_t* scores,
                                     void* scratch, uint32_t scols, size_t waves, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (pad + 1 > (uint32_t)swk::I32_LETTERS || waves == 0 || waves % 4) return hipErrorInvalidValue;
  const swk::I32Args a{res, offs, lens, n, (uint32_t)packed, idx, nidx, idx_base,
                       static_cast<const uint2*>(prof), nstrips, qlen, pad, O, E, scores,
                       static_cast<uint2*>(scratch), scols};
  if (gotoh)
    hipLaunchKernelGGL(swk::score_i32<true>, dim3((unsigned)(waves / 4)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(swk::score_i32<false>, dim3((unsigned)(waves / 4)), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ========================================================================================
// Longest-first visiting order of a device batch (sw_score_batch_device with ragged lengths):
// the PrioEncoder's feed order (ScoreBank_v2.v:142-148) so that each 128-target tile holds
// similar lengths.  A counting sort over length bins (bin = (max_len - len) >> shift, at most
// 2048 bins; targets within a bin differ by < 2^shift codes, and the order inside a bin is
// free: scores are written at input positions).  hist: global bin counts; scan: exclusive
// offsets in place + perm_n = n; scatter: per block, LDS bin counts, one global atomic per
// non-empty bin reserves the block's range, LDS atomics place the elements.
namespace swk {
#ifndef SWK_SORT_ITEMS
#define SWK_SORT_ITEMS 8  // lengths per thread of the device sort's kernels
#endif
constexpr int SORT_BINS = 2048, SORT_BLOCK = 1024, SORT_ITEMS = SWK_SORT_ITEMS;

__device__ __forceinline__ uint32_t sort_bin(uint32_t len, uint32_t max_len, uint32_t shift) {
  return (max_len - min(len, max_len)) >> shift;
}

// h[bin] += 1 for the active lanes; returns the lane's slot (the old value + its rank among
// the lanes of its bin).  A wave whose lanes share one bin (uniform or already sorted lengths)
// adds once from its first lane; otherwise every lane adds its own (distinct bins rarely
// collide, and 64 serialised atomics on one address were the cost this avoids).
__device__ __forceinline__ uint32_t wave_bin_add(uint32_t* h, uint32_t bin, bool active) {
  const int lane = threadIdx.x & 63;
  const uint64_t act = __ballot(active);
  if (!act) return 0;
  const int leader = __builtin_ctzll(act);
  const uint32_t lb = __builtin_amdgcn_readlane(bin, leader);
  const uint64_t m = __ballot(active && bin == lb);
  if (m == act) {
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&h[lb], (uint32_t)__builtin_popcountll(m));
    base = __builtin_amdgcn_readlane(base, leader);
    return base + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1));
  }
  return active ? atomicAdd(&h[bin], 1u) : 0u;
}

// scratch: hist[SORT_BINS] | done[2] (block counters), zero between calls: the last block of
// a call's last kernel zeroes them again, so no memset per call.
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Histogram of the bins, then (the last block to finish) exclusive offsets in place,
// *perm_n = n, and *ident = 1 when at most one bin is non-empty (the caller's order is kept:
// the scatter and the score kernel's indirection are skipped, and the hist is zeroed here).
// plan != nullptr (balanced chunk ranges of a ragged batch, shift == 0 so a bin is one length):
// the last block also writes, for g = 0..G, plan[g] = {tile, chunk, floor(g A / G), 0} of chunk
// floor(g A / G) of
// the longest-first tile sequence (A = its chunk count, tile t's chunk count ceil(len / 8) of the
// bin holding its first, longest target), i.e. where each of the score kernel's G workgroups
// starts.
__global__ void __launch_bounds__(SORT_BLOCK) sort_hist_scan(const uint32_t* lens, size_t n,
                                                             uint32_t max_len, uint32_t shift,
                                                             uint32_t nb, uint32_t* hist,
                                                             uint32_t* perm_n, uint32_t* ident,
                                                             uint4* plan, uint32_t G) {
  __shared__ uint32_t h[SORT_BINS];
  __shared__ uint32_t part[SORT_BLOCK];
  __shared__ int last;
  for (uint32_t i = threadIdx.x; i < nb; i += SORT_BLOCK) h[i] = 0;
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * SORT_BLOCK * SORT_ITEMS;
#pragma unroll
  for (int it = 0; it < SORT_ITEMS; ++it) {
    const size_t k = base + (size_t)it * SORT_BLOCK + threadIdx.x;
    (void)wave_bin_add(h, k < n ? sort_bin(lens[k], max_len, shift) : 0u, k < n);
  }
  __syncthreads();
  // hand-off (MI355X_MICROARCH.md, inter-workgroup visibility): the bins are written by
  // device-scope atomics, each wave waits for its own, the last block (told by the counter's
  // returned value) reads them with sc1 loads; no L2 write-back fence (__threadfence() here
  // cost ~35 us per call)
  for (uint32_t i = threadIdx.x; i < nb; i += SORT_BLOCK)
    if (h[i]) atomicAdd(&hist[i], h[i]);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t* done = hist + SORT_BINS;
  if (threadIdx.x == 0) last = atomicAdd(&done[0], 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  // each thread owns 2 consecutive bins (nb <= 2048)
  const uint32_t i0 = threadIdx.x * 2;
  const uint32_t a = i0 < nb ? ld_agent(&hist[i0]) : 0u;
  const uint32_t c = i0 + 1 < nb ? ld_agent(&hist[i0 + 1]) : 0u;
  const int used = __syncthreads_count((a != 0) + (c != 0) > 0 ? 1 : 0) +
                   __syncthreads_count(a != 0 && c != 0 ? 1 : 0);
  part[threadIdx.x] = a + c;
  __syncthreads();
  for (uint32_t off = 1; off < SORT_BLOCK; off <<= 1) {  // inclusive Hillis-Steele scan
    const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  const uint32_t ex = part[threadIdx.x] - (a + c);
  const bool one = used <= 1;
  if (i0 < nb) hist[i0] = one ? 0u : ex;
  if (i0 + 1 < nb) hist[i0 + 1] = one ? 0u : ex + a;
  if (threadIdx.x == 0) {
    *perm_n = (uint32_t)n;
    *ident = one ? 1u : 0u;
    done[0] = 0;
  }
  if (!plan) return;
  // tiles whose first position falls in bin b: [ceil(off_b / 128), ceil((off_b + cnt_b) / 128)),
  // each of K_b = max(1, ceil(len_b / 8)) chunks (the bin's length is the tile's longest);
  // h[] <- first tile of the bin, part[] <- chunks before the bin's first tile (exclusive scan
  // of tiles x K over the bins, 2 bins per thread)
  const auto kb = [&](uint32_t b) { return max(1u, ((max_len - b) + 7u) / 8u); };
  const uint32_t t0 = (ex + 127) / 128, t1 = (ex + a + 127) / 128, t2 = (ex + a + c + 127) / 128;
  const uint32_t w0 = i0 < nb ? (t1 - t0) * kb(i0) : 0u, w1 = i0 + 1 < nb ? (t2 - t1) * kb(i0 + 1) : 0u;
  __syncthreads();
  part[threadIdx.x] = w0 + w1;
  if (i0 < nb) h[i0] = t0;
  if (i0 + 1 < nb) h[i0 + 1] = t1;
  __syncthreads();
  for (uint32_t off = 1; off < SORT_BLOCK; off <<= 1) {
    const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  const uint32_t total = part[SORT_BLOCK - 1];  // chunks of all tiles
  // chunks before bin b: part[b / 2 - 1] (inclusive prefix of the pairs before) plus, for an odd
  // b, the even bin's weight
  const auto before = [&](uint32_t b) -> uint32_t {
    const uint32_t pr = b >= 2 ? part[b / 2 - 1] : 0u;
    if ((b & 1) == 0) return pr;
    return pr + ((b < nb ? h[b] : (uint32_t)((n + 127) / 128)) - h[b - 1]) * kb(b - 1);
  };
  const uint32_t ntiles = (uint32_t)((n + 127) / 128);
  for (uint32_t g = threadIdx.x; g <= G; g += SORT_BLOCK) {
    const uint32_t A = (uint32_t)((uint64_t)total * g / G);
    uint4 r = make_uint4(ntiles, 0u, A, 0u);
    if (A < total) {
      uint32_t lo = 0, hi = nb;  // the last bin with before(bin) <= A (and a tile in it)
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (before(mid) <= A) lo = mid; else hi = mid;
      }
      while (lo + 1 < nb && before(lo + 1) <= A) ++lo;  // (bins without tiles have no width)
      const uint32_t d = A - before(lo), K = kb(lo);
      r = make_uint4(h[lo] + d / K, d % K, A, 0u);
    }
    plan[g] = r;
  }
}

__global__ void __launch_bounds__(SORT_BLOCK) sort_scatter(const uint32_t* lens, size_t n,
                                                           uint32_t max_len, uint32_t shift,
                                                           uint32_t nb, uint32_t* offs,
                                                           uint32_t* perm, const uint32_t* ident) {
  if (__builtin_amdgcn_readfirstlane(*ident)) return;  // one length bin: order unchanged
  __shared__ uint32_t h[SORT_BINS];
  __shared__ int last;
  for (uint32_t i = threadIdx.x; i < nb; i += SORT_BLOCK) h[i] = 0;
  __syncthreads();
  const size_t base = (size_t)blockIdx.x * SORT_BLOCK * SORT_ITEMS;
  uint32_t bin[SORT_ITEMS], slot[SORT_ITEMS];
#pragma unroll
  for (int it = 0; it < SORT_ITEMS; ++it) {
    const size_t k = base + (size_t)it * SORT_BLOCK + threadIdx.x;
    bin[it] = k < n ? sort_bin(lens[k], max_len, shift) : 0u;
    slot[it] = wave_bin_add(h, bin[it], k < n);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < nb; i += SORT_BLOCK)  // reserve this block's ranges
    if (h[i]) h[i] = atomicAdd(&offs[i], h[i]);
  __syncthreads();
#pragma unroll
  for (int it = 0; it < SORT_ITEMS; ++it) {
    const size_t k = base + (size_t)it * SORT_BLOCK + threadIdx.x;
    const uint32_t pos = h[bin[it]] + slot[it];
    if (k < n && pos < n) perm[pos] = (uint32_t)k;
  }
  // the last block zeroes the offsets and the counters for the next call (every block's
  // offset atomics returned before its counter add; the zeros reach the next call's kernels
  // through the kernel boundary)
  __syncthreads();
  uint32_t* done = offs + SORT_BINS;
  if (threadIdx.x == 0) last = atomicAdd(&done[1], 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  for (uint32_t i = threadIdx.x; i < nb; i += SORT_BLOCK) offs[i] = 0;
  if (threadIdx.x == 0) done[1] = 0;
}
}  // namespace swk

// perm[0, n) <- target numbers longest first, *perm_n <- n, *ident <- 1 when the lengths
// share one bin (perm then left unwritten: visit in input order); scratch:
// swk_sort_scratch_bytes(), zero on entry and on return.
extern "C" hipError_t swk_sort_lens(const uint32_t* lens, size_t n, uint32_t max_len,
                                    uint32_t* perm, uint32_t* perm_n, uint32_t* ident,
                                    uint32_t* scratch, hipStream_t st, void* plan, unsigned G) {
  if (n == 0 || n > 0xFFFFFFFFull) return hipErrorInvalidValue;
  uint32_t shift = 0;
  while ((max_len >> shift) >= (uint32_t)swk::SORT_BINS) ++shift;
  const uint32_t nb = (max_len >> shift) + 1;
  if (plan && (shift != 0 || G == 0)) return hipErrorInvalidValue;
  const unsigned blocks =
      (unsigned)((n + swk::SORT_BLOCK * swk::SORT_ITEMS - 1) / (swk::SORT_BLOCK * swk::SORT_ITEMS));
  hipLaunchKernelGGL(swk::sort_hist_scan, dim3(blocks), dim3(swk::SORT_BLOCK), 0, st, lens, n,
                     max_len, shift, nb, scratch, perm_n, ident, static_cast<uint4*>(plan), G);
  hipLaunchKernelGGL(swk::sort_scatter, dim3(blocks), dim3(swk::SORT_BLOCK), 0, st, lens, n,
                     max_len, shift, nb, scratch, perm, ident);
  return hipGetLastError();
}

// Bytes of sort scratch (zeroed once at allocation; the kernels leave it zeroed).
extern "C" size_t swk_sort_scratch_bytes(void) { return (swk::SORT_BINS + 2) * sizeof(uint32_t); }
