// swbank_ktile.hip — the tile kernel (the bulk path) and its
// launchers: a workgroup of W waves x R query rows scores 128 targets per tile.
#include "swbank_kcommon.h"

namespace swk {

// C: columns per chunk (one barrier per chunk); 4 for the 16-wave query-set pair kernel, whose
// hand-off ring would not fit LDS beside a 512-row pair table at 8.
// TRIM: a tile's last chunk stops after its last column holding a code of some lane (ragged
// batches: a tile's lengths are one sort bin, rarely a multiple of C; the per-column test costs
// a uniform batch ~25 VALU per chunk in register copies, so only the ragged launches take it).
#ifndef SWK_TRIM_BREAK
// TRIM: leave the chunk's column loop at the first column past the tile's last code (break)
// rather than skipping each later column (continue): the continue form's per-column joins cost
// 25 register copies per chunk on every chunk (1,475 VALU against 1,450), the break form's
// exits are out of line (1,458)
#define SWK_TRIM_BREAK 1
#endif
template <int R, int RB, bool COL0, bool PROF, bool GOTOH, bool F16, bool PAIR = false,
          bool MQ = false, bool STREAM = false, int C = 8, bool BAL = false, bool TRIM = false>
__global__ void __launch_bounds__(R >= 64 ? 512 : 1024) score_kernel(const ScoreArgs a) {
  static_assert(!BAL || (!MQ && !STREAM && !COL0), "balanced ranges: one query, resident batch");
  static_assert(!TRIM || (BAL && PAIR), "trimmed last chunks: the balanced pair kernel");
  static_assert(!MQ || !PROF, "several queries: row-LUT or pair-table variants");
  static_assert(!STREAM || (!MQ && !PROF), "streamed batches: single-query LUT / pair variants");
  static_assert(C == 8 || (C == 4 && PAIR && !STREAM), "4-column chunks: pair tables only");
  static_assert(!PAIR || ((R == 32 || (R == 16 && GOTOH)) && F16 && !PROF && !COL0 &&
                          (!GOTOH || !MQ)),
                "PAIR: f16, merged R = 32 or Gotoh R = 16 / 32 (one query)");
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int W = __builtin_amdgcn_readfirstlane(blockDim.x >> 6);
  const bool seg_in = a.edge_in != nullptr, seg_out = a.edge_out != nullptr;
  uint32_t* bestsh = smem + (PAIR ? a.PS / 4 : 0);               // W x 128 words
  uint2* bnd = reinterpret_cast<uint2*>(bestsh + W * SWB_TILE);  // row -1 boundary
  uint2* sink = bnd + 64;                                        // last wave's bottom row
  uint2* ein = sink + (seg_out ? C * 64 : 64);                   // previous segment, 2 x 8 cols
  uint2* ring = ein + (seg_in ? 2 * C * 64 : 0);
  uint8_t* prof = reinterpret_cast<uint8_t*>(ring + (size_t)(W > 1 ? W - 1 : 0) * 2 * C * 64);

  size_t n = a.n;
  const uint32_t* idx = a.idx;
  if (idx && a.ident && __builtin_amdgcn_readfirstlane(*a.ident)) idx = nullptr;
  const uint32_t* sidx = TRIM ? a.sidx : nullptr;  // (scores only, see ScoreArgs.sidx)
  if (TRIM && sidx && a.ident && __builtin_amdgcn_readfirstlane(*a.ident)) sidx = nullptr;
  if (idx) {
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(*a.nidx);
    n = cnt > a.idx_base ? min(a.n, (size_t)(cnt - a.idx_base)) : 0;
  }
  const int ntiles = (int)((n + SWB_TILE - 1) / SWB_TILE);
  const int G = (int)gridDim.x;
  // units: (query, tile) pairs; one query: unit = tile.  A unit past the end keeps its number
  // as the tile (lane_targets then reads nothing)
  // (MQ only; otherwise unit = tile and q = 0)
  const int nunits = MQ ? ntiles * (int)a.nq : ntiles;
  int total = 0;  // chunks of all this workgroup's tiles: every wave runs total + W - 1 phases
  uint32_t packed = a.packed;
  // STREAM: tiles taken dynamically, so the total is open until wave 0 finds no tile left
  // (it then stores it in sq[W]; every wave reads sq[W] at each phase)
  int* sq = reinterpret_cast<int*>(prof);  // STREAM: next tile of ordinal k at [k % W] | total
  // BAL: this workgroup's chunk range [A0, A1) as visits: the head (tile be, chunks [0, bf)),
  // the whole tiles [bfirst, be), the tail (tile bs, chunks [bo, K)); a range holds >= 2 tiles
  // (the host checks), so the head and the tail are different tiles.  Visit v (= the tile
  // ordinal k) -> (tile, first chunk, end chunk), recomputed from blockIdx at each visit's end
  // (nothing of the plan stays live across the column loop)
  // (a visit's end chunk is the tile's own chunk count, c1 = -1 until the tile's lengths are
  // read; the plan is read once, into SGPRs: a global load at every visit's end stalls the wave)
  int bs = 0, bo = 0, be = 0, bf = 0;
  if constexpr (BAL) {
    const uint4 p0 = a.bal_plan[blockIdx.x], p1 = a.bal_plan[blockIdx.x + 1];
    bs = (int)__builtin_amdgcn_readfirstlane(p0.x), bo = (int)__builtin_amdgcn_readfirstlane(p0.y);
    be = (int)__builtin_amdgcn_readfirstlane(p1.x), bf = (int)__builtin_amdgcn_readfirstlane(p1.y);
    total = (int)__builtin_amdgcn_readfirstlane(p1.z - p0.z);
  }
  const auto bal_visit = [&](int v, int& t, int& c0, int& c1) {
    const int bK = -1;
    const int bfirst = bo ? bs + 1 : bs;
    const int hh = bf > 0 ? 1 : 0;
    if (v < hh) {
      t = be, c0 = 0, c1 = bf;
    } else if (v - hh < be - bfirst) {
      t = bfirst + v - hh, c0 = 0, c1 = bK;
    } else if (v - hh == be - bfirst && bo > 0) {
      t = bs, c0 = bo, c1 = bK;
    } else {
      t = nunits, c0 = 0, c1 = 1;  // no more visits
    }
    t = __builtin_amdgcn_readfirstlane(t);
    c0 = __builtin_amdgcn_readfirstlane(c0);
    c1 = __builtin_amdgcn_readfirstlane(c1);
  };
  if constexpr (BAL) {
  } else if constexpr (STREAM) {
    total = (int)blockIdx.x < ntiles ? (1 << 30) : 0;
  } else {
    for (int u = blockIdx.x; u < nunits; u += G)  // (the unit's tile: see the MQ order below)
      total += tile_nch<C>(a.res, a.lens, n, !MQ ? u : PAIR ? u / (int)a.nq : u % ntiles, lane,
                        packed, idx, a.ulen, a.ustride);
  }
  // STREAM: the chunk of this wave's current tile (tiles only grow), its first tile, target
  // count, code offset and layout
  // (wave-uniform, kept in SGPRs)
  const SwkStreamChunk* const ssc = a.sc;
  const int snc = (int)a.nsc;
  int scur = -1, st0 = 0;
  uint32_t scn = 0, sro_lo = 0, sro_hi = 0, smode = SWK_PACK_STREAM;
  // ragged streamed batches (ulen == 0): a chunk's region is mixed offset words u32 (see
  // mixed_ptr) | lengths u32 | visiting order u32 (scn each) | codes (SWK_PACK_MIXED: the 2-bit
  // region, then the 4-bit one) at the next 16-byte boundary; the order of the chunk of the tile
  // this wave is scoring (wperm, its first tile wst0) maps score positions to targets
  const uint32_t* cperm = nullptr;
  const uint32_t* wperm = nullptr;
  int wst0 = 0;
  const auto stream_tile = [&](int t, uint32_t& pk) -> Lane2 {
    if (t >= ntiles) {  // past the batch: reads nothing
      pk = SWK_PACK_STREAM;
      Lane2 e;
      e.llo = e.lhi = 0u;
      e.plo = e.phi = a.res;
      return e;
    }
    int c = scur < 0 ? 0 : scur;
    while (c + 1 < snc && t >= (int)ssc[c + 1].tile0) ++c;
    if (c != scur) {
      scur = __builtin_amdgcn_readfirstlane(c);
      st0 = __builtin_amdgcn_readfirstlane((int)ssc[c].tile0);
      scn = __builtin_amdgcn_readfirstlane(
          (uint32_t)((c + 1 < snc ? (size_t)ssc[c + 1].tile0 * SWB_TILE : n) -
                     (size_t)st0 * SWB_TILE));
      sro_lo = __builtin_amdgcn_readfirstlane(ssc[c].res_off_lo);
      sro_hi = __builtin_amdgcn_readfirstlane(ssc[c].res_off_hi);
      const uint32_t md = stream_mode(a.hflag, a.dflag, c, snc, lane);
      // (ragged chunks cross in the mixed layout; an aborted one reads as empty mixed targets)
      smode = a.ulen == 0 ? SWK_PACK_MIXED
                          : md == SWK_PACK_NIBBLE ? SWK_PACK_NIBBLE : SWK_PACK_STREAM;
      if (md == SWK_STREAM_ABORT && a.ulen == 0) {
        // a ragged chunk that never landed (the host re-runs the call): its region may hold
        // anything, so it is read from the zeroed region instead (empty targets, scores in
        // order; uniform chunks read their own region as codes, always in bounds)
        const uint64_t z = (uint64_t)__builtin_amdgcn_readfirstlane(ssc[c].zero_off256) * 256u;
        sro_lo = (uint32_t)z;
        sro_hi = (uint32_t)(z >> 32);
      }
    }
    pk = smode;
    const uint8_t* base = a.res + ((size_t)sro_hi << 32 | sro_lo);
    if (a.ulen == 0) {  // ragged: the chunk's own mixed offset words, lengths and order
      const uint32_t* co = reinterpret_cast<const uint32_t*>(base);
      const uint32_t* cl = co + scn;
      cperm = cl + scn;
      return lane_targets<true>(base + (((size_t)scn * 12 + 15) & ~(size_t)15),
                                reinterpret_cast<const uint64_t*>(co), cl, scn, t - st0, lane, pk,
                                cperm, 0u, 0u);
    }
    return lane_targets<true>(base, nullptr, nullptr, scn, t - st0, lane, pk, nullptr, a.ulen,
                               pk == SWK_PACK_NIBBLE ? (a.ulen + 1) / 2 : (a.ulen + 3) / 4);
  };

  // MQ order: row LUTs query-major (q = unit / ntiles; a wave reloads its LUT SGPRs when the
  // query changes); pair tables query-minor (q = unit % nq) with the grid a multiple of nq, so
  // a workgroup keeps one query and loads its LDS table once
  int unit = blockIdx.x, q = 0;
  int tile = unit;
  int vc0 = 0, vend = 0;  // BAL: the first visit's first and end chunk
  if constexpr (BAL) {
    bal_visit(0, tile, vc0, vend);
    unit = tile;
  }
  if constexpr (MQ) {
    if (unit < nunits) {
      q = PAIR ? unit % (int)a.nq : unit / ntiles;
      tile = PAIR ? unit / (int)a.nq : unit - q * ntiles;
    }
  }
  Lane2 cur;
  if constexpr (STREAM) {
    cur = stream_tile(tile, packed);
    wperm = cperm;
    wst0 = st0;
  } else {
    cur = lane_targets<!MQ>(a.res, a.offs, a.lens, n, tile, lane, packed, idx, a.ulen,
                            a.ustride);
  }
  int nch, nfull, ncl;
  tile_chunks<C>(cur, (size_t)tile * SWB_TILE + lane, (size_t)tile * SWB_TILE + lane + 64, n, nch,
              nfull, ncl);
  (void)ncl;
  if constexpr (BAL) {  // BAL: nch = the visit's end chunk (a head's last chunk is whole)
    if (vend >= 0 && vend < nch) ncl = C;
    nch = vend < 0 ? nch : vend;
  }
  const uint32_t S = a.S;

  for (int i = threadIdx.x; i < W * SWB_TILE; i += blockDim.x) bestsh[i] = 0;
  // row -1: u16 H~ = S, G/F = 0 | f16 H = 0, T = -(o+e)
  // f16 encodings of -(o+e), -e, -o (host-computed, so they stay in SGPRs)
  const f16x2 NOE2 = as_f16x2(as_u16x2(a.f16_noe)), NE2 = as_f16x2(as_u16x2(a.f16_ne)),
              NO2 = as_f16x2(as_u16x2(a.f16_no));
  if (wave == 0) {
    bnd[lane] = F16 ? make_uint2(0u, GOTOH ? 0u : as_u32(as_u16x2(NOE2)))
                    : make_uint2(S | (S << 16), 0u);
    if (seg_in)  // the previous segment's bottom row of chunk 0
      dma_edge_chunk<C>(a.edge_in + (size_t)(MQ ? unit : tile) * a.ecols * 64, ein, lane);
  }
  uint32_t nv = a.nv;
  uint32_t tab[PROF || PAIR ? 1 : R];
  if constexpr (PAIR) {
    const uint4* src = reinterpret_cast<const uint4*>(a.qtab + (MQ ? (size_t)q * a.qwords : 0));
    for (uint32_t i = threadIdx.x; i < a.PS / 16; i += blockDim.x)
      reinterpret_cast<uint4*>(smem)[i] = src[i];
  } else if constexpr (PROF) {
    // query profile -> LDS (the ScoringModule's query + penalty registers)
    const uint32_t words = (a.pad + 1) * a.PS / 16;
    const uint4* src = reinterpret_cast<const uint4*>(a.qtab);
    for (uint32_t i = threadIdx.x; i < words; i += blockDim.x)
      reinterpret_cast<uint4*>(prof)[i] = src[i];
  } else {
    // nv in a VGPR so each v_perm_b32 takes its row LUT straight from an SGPR (one scalar
    // operand per VOP3 on gfx950).
    asm volatile("" : "+v"(nv));
#pragma unroll
    for (int r = 0; r < R; ++r)
      tab[r] = __builtin_amdgcn_readfirstlane(a.qtab[(MQ ? (size_t)q * a.qwords : 0) + wave * R + r]);
  }
  const u16x2 S2 = {(unsigned short)S, (unsigned short)S};
  const u16x2 O2 = {(unsigned short)a.O, (unsigned short)a.O};
  const u16x2 E2 = {(unsigned short)a.E, (unsigned short)a.E};
  const uint32_t oes = a.O + a.E + S;
  const u16x2 OES2 = {(unsigned short)oes, (unsigned short)oes};
  const u16x2 H0 = F16 ? (u16x2){0, 0} : S2;          // H of row/column -1
  const u16x2 X0 = (F16 && !GOTOH) ? as_u16x2(NOE2) : (u16x2){0, 0};  // G/E/T of column -1

  // H~ and G (merged) / E (Gotoh) / T (f16) of the column to the left
  u16x2 Hl[R], Xl[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    Hl[r] = H0;
    Xl[r] = X0;
  }
  u16x2 best = {0, 0};
  u16x2 prevUpH = H0;  // H(row above, column -1)
  uint2 rlo, rhi;      // raw codes of the next chunk (prefetched one phase ahead)
  load_raw<C, !MQ>(cur, vc0, vc0 < nfull, a.pad, packed, rlo, rhi);
  if (STREAM && threadIdx.x == 0) sq[W] = total;
  __syncthreads();

  // PAIR: column state one column ahead: acur = this column's table address (slot + this
  // wave's rows - 16), pA = its first 8 row words, pw = its row-0 word
  // Table addresses are absolute LDS byte addresses (smem's link-time address folded into
  // wofs once), so a column's address needs no add for the base.
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) const u32x4 lds_u4;
  typedef __attribute__((address_space(3))) const uint32_t lds_u32;
  const auto ld4 = [](uint32_t addr) { return __builtin_bit_cast(uint4, *(lds_u4*)(size_t)addr); };
  // the row-0 word: a relaxed atomic load, so LLVM does not merge it with the neighbouring
  // 16-B reads (it splits them into ds_read2_b32 pairs otherwise)
  const auto ld1 = [](uint32_t addr) {
    return __atomic_load_n((lds_u32*)(size_t)addr, __ATOMIC_RELAXED);
  };
  const uint32_t wofs = (uint32_t)wave * R * 4 + (uint32_t)(size_t)(lds_void_ptr)smem;
  // codes clamped to N: lanes past the batch end (and codes >= 5 on the device API) would
  // otherwise pick a slot outside the table, and a slot feeds both halves (one v_min each,
  // SDWA byte-select)
  // (3 VALU: {a, b} as u16 halves by one v_perm, clamped by one v_pk_min_u16, then
  // a*pS1 + b*pS2 + wofs by one v_dot2_u32_u16; the host keeps pS1, pS2 < 65536)
  const u16x2 pS12 = {(unsigned short)a.pS1, (unsigned short)a.pS2};
  const auto pair_addr = [&](uint32_t wl, uint32_t wh, int sh) {
    const uint32_t sel = (uint32_t)(sh >> 3) | 0x0C00u | ((uint32_t)(4 + (sh >> 3)) << 16) |
                         0x0C000000u;
    const u16x2 ab = __builtin_elementwise_min(as_u16x2(__builtin_amdgcn_perm(wh, wl, sel)),
                                               (u16x2){4, 4});
    return __builtin_amdgcn_udot2(ab, pS12, wofs, false);
  };
  uint32_t acur = 0, pw = 0;
  uint4 pA0 = {0, 0, 0, 0}, pA1 = {0, 0, 0, 0};
  if constexpr (PAIR) {
    acur = pair_addr(rlo.x, rhi.x, 0);
    pA0 = ld4(acur + 16);
    pA1 = ld4(acur + 32);
    pw = ld1(acur + 12);
  }
  (void)pA0; (void)pA1; (void)pw; (void)acur; (void)wofs;

  // branch-free hand-off: wave 0 reads the top boundary (constant, stride 0, or the previous
  // segment's row), the last wave writes into an LDS sink (branches inside the column loop
  // split it into blocks and LLVM then sinks the H updates across columns, blowing up
  // register pressure)
  const int istride = (wave > 0 || seg_in) ? 64 : 0, ostride = (wave < W - 1 || seg_out) ? 64 : 0;
  const uint32_t pbase = (uint32_t)wave * R;
  const uint32_t padc = a.pad;
  // BAL hand-off of one wave's column state {H, T of its R rows, the diagonal H above, best}
  // at a head's end / a tail's start: word i of lane l at state[((g W + wave) (2R + 2) + i) 64
  // + l] (coalesced), written and read with sc1 (write-through / L2) accesses and a flag
  // (MI355X_MICROARCH.md, inter-workgroup visibility: sc1 stores, vmcnt(0), sc1 flag; sc1 poll,
  // sc1 loads).  The consumer's tail is its last visit and the producer's head its first, so
  // the flag is normally long set; the poll is bounded (poll_limit, about 4 s) and a time-out
  // marks the launch's fault word (the host fails the call) rather than hanging.
  // (the state addresses go through an opaque copy: loop-invariant, LLVM would otherwise hoist
  // all 2R + 2 of them out of the phase loop, 2 VGPRs each, and spill)
  int bal_pend = 0;  // BAL: phases until the head's flag goes out (0: none pending)
  const auto bal_store = [&](int g_to) {
    uint32_t* sp = a.bal_state + ((size_t)g_to * W + wave) * (2 * R + 2) * 64 + lane;
    asm volatile("" : "+v"(sp));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      __hip_atomic_store(sp + r * 64, as_u32(Hl[r]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sp + (R + r) * 64, as_u32(Xl[r]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    __hip_atomic_store(sp + 2 * R * 64, as_u32(prevUpH), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(sp + (2 * R + 1) * 64, as_u32(best), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    bal_pend = 2;  // the flag goes out a phase later, when the stores have long completed
  };
  const auto bal_flag_out = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0 && blockIdx.x + 1 != a.stall)  // (stall: a test hook)
      __hip_atomic_store(a.bal_flag + ((size_t)blockIdx.x + 1) * W + wave, a.bal_gen,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
#if SWK_STAMPS
  uint64_t st_bload = 0;  // (measurement builds) cycles in tail state loads
#endif
  const auto bal_load = [&]() {
#if SWK_STAMPS
    const uint64_t sb0 = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t* fl = a.bal_flag + (size_t)blockIdx.x * W + wave;
    uint32_t it = 0;
    for (; it < a.poll_limit; ++it) {
      if (__builtin_amdgcn_readfirstlane(
              __hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == a.bal_gen)
        break;
      __builtin_amdgcn_s_sleep(8);
    }
    if (it == a.poll_limit && lane == 0) report_fault(a.fault, SWK_FAULT_BAL);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t* sp = a.bal_state + ((size_t)blockIdx.x * W + wave) * (2 * R + 2) * 64 + lane;
    asm volatile("" : "+v"(sp));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      Hl[r] = as_u16x2(__hip_atomic_load(sp + r * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      Xl[r] = as_u16x2(
          __hip_atomic_load(sp + (R + r) * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    prevUpH = as_u16x2(
        __hip_atomic_load(sp + 2 * R * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    best = as_u16x2(
        __hip_atomic_load(sp + (2 * R + 1) * 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#if SWK_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st_bload += __builtin_amdgcn_s_memtime() - sb0;
#endif
  };
  (void)bal_store; (void)bal_load; (void)bal_flag_out;
  // chunk within the current tile, tile ordinal in this workgroup (BAL: the visit ordinal; a
  // first visit is a head or a whole tile, never a tail)
  int c = vc0, k = 0;
  int nch_n = 1, nfull_n = 0, ncl_n = C;  // the next tile's chunk counts
  uint32_t packed_n = packed;  // STREAM: the next tile's code layout
#if SWK_PRIO_ROT
  const uint32_t prq = (uint32_t)((blockIdx.x * 4ull) / gridDim.x);
  uint32_t prio = 4;  // (none set yet)
#endif
#if SWK_STAMPS
  // (measurement builds only) per wave: kernel entry / exit, cycles in active phases (the
  // column work), in fill/drain phases (no chunk of its own) and in the per-phase barrier
  uint64_t st_t0 = __builtin_amdgcn_s_memtime(), st_act = 0, st_idle = 0, st_bar = 0;
  uint64_t st_p = st_t0;
#endif
  for (int ph = 0;; ++ph) {
    if constexpr (STREAM) total = __builtin_amdgcn_readfirstlane(sq[W]);
    if (ph >= total + W - 1) break;
#if SWK_PRIO_ROT
    // (a 16-wave workgroup has its CU alone; SWK_PRIO_END: the last 1/2^SWK_PRIO_END_FRAC of
    // the phases rotate 2^SWK_PRIO_END times faster, so the four finish closer together)
    if (W <= 8)
      prio_rotate(prq, prio,
                  SWK_PRIO_END && ph >= total - (total >> SWK_PRIO_END_FRAC)
                      ? SWK_PRIO_SHIFT - SWK_PRIO_END : SWK_PRIO_SHIFT);

#endif
    const int g = ph - wave;
    if (g >= 0 && g < total) {
      const uint2 clo = rlo, chi = rhi;
      const bool last = c + 1 == nch;
      int nunit = (MQ ? unit : tile) + G;
      int nc0 = 0, nvend = 0;  // BAL: the next visit's first and end chunk
      if constexpr (BAL) {
        if (last) bal_visit(k + 1, nunit, nc0, nvend);
      }
      if constexpr (STREAM) {  // wave 0 takes the next tile; the others read it W-1 phases on
        if (last) {
          if (wave == 0) {
            int nt = 0;
            if (lane == 0) nt = G + (int)atomicAdd(a.tctr, 1u);
            nt = min(__builtin_amdgcn_readfirstlane(nt), ntiles);
            if (lane == 0) {
              sq[(k + 1) % W] = nt;
              if (nt >= ntiles) sq[W] = g + 1;
            }
            nunit = nt;
          } else {
            nunit = __builtin_amdgcn_readfirstlane(sq[(k + 1) % W]);
          }
        }
      }
      int ntile = nunit, nqq = q;  // the next unit's tile and query
      if constexpr (MQ) {
        if (nunit < nunits) {
          if constexpr (PAIR) {
            ntile = nunit / (int)a.nq;  // same query (G is a multiple of nq)
          } else {
            ntile = tile + G;
            while (ntile >= ntiles) {
              ntile -= ntiles;
              ++nqq;
            }
          }
        }
      }
      if (!last) {
        load_raw<C, !MQ>(cur, c + 1, c + 1 < nfull, a.pad, packed, rlo, rhi);
      } else if (nunit < nunits) {  // first chunk of the next tile
        if constexpr (STREAM) cur = stream_tile(ntile, packed_n);
        else
          cur = lane_targets<!MQ>(a.res, a.offs, a.lens, n, ntile, lane, packed, idx, a.ulen,
                                  a.ustride);
        tile_chunks<C>(cur, (size_t)ntile * SWB_TILE + lane, (size_t)ntile * SWB_TILE + lane + 64,
                    n, nch_n, nfull_n, ncl_n);
        if (BAL && nvend >= 0 && nvend < nch_n) ncl_n = C;
        if (BAL && nvend < 0) nvend = nch_n;
        load_raw<C, !MQ>(cur, nc0, nc0 < nfull_n, a.pad, STREAM ? packed_n : packed, rlo, rhi);
      }
      const int slot = g & 1;
      // next chunk's boundary row (never past the last unit's edge rows)
      if (seg_in && wave == 0 && (last ? nunit < nunits : (MQ ? unit : tile) < nunits))
        dma_edge_chunk<C>(a.edge_in + ((size_t)(last ? nunit : MQ ? unit : tile) * a.ecols +
                                    (size_t)(last ? 0 : c + 1) * C) * 64,
                       ein + (size_t)((g + 1) & 1) * C * 64, lane);
      const uint2* rin = wave > 0 ? ring + ((size_t)((wave - 1) * 2 + slot) * C) * 64 + lane
                                  : (seg_in ? ein + (size_t)slot * C * 64 : bnd) + lane;
      uint2* rout = wave < W - 1 ? ring + ((size_t)(wave * 2 + slot) * C) * 64 + lane
                                 : sink + lane;
      uint2 rv = rin[0];
      ProfLookup16<PROF && F16 ? R : 2> lkq;  // f16 profile: the next column's words
      (void)lkq;
      // TRIM: the tile's last chunk stops after its last column holding a code (a tile runs to
      // its longest lane; every wave stops at the same column, so the ring stays consistent)
      const int ncols = TRIM && c + 1 == nch ? ncl : C;
      bool trimmed = false;
      (void)ncols;
#pragma unroll
      for (int jj = 0; jj < C; ++jj) {
        if (TRIM && jj > 0 && __builtin_expect(jj >= ncols, 0)) {
          trimmed = true;
#if SWK_TRIM_BREAK
          break;  // (every later column is past ncols too: one exit edge per column, out of line)
#else
          continue;
#endif
        }
        const u16x2 upH = as_u16x2(rv.x);
        u16x2 upX = as_u16x2(rv.y);
        if (jj + 1 < C) rv = rin[(jj + 1) * istride];  // one column ahead
        u16x2 diag = prevUpH;
        prevUpH = upH;
        const uint32_t wlo = jj < 4 ? clo.x : clo.y, whi = jj < 4 ? chi.x : chi.y;
        if constexpr (PROF && F16) {
          // profile words one column ahead (the LDS latency hides behind a column)
          const auto load16 = [&](int j, ProfLookup16<R>& out) {
            const uint32_t wl = j < 4 ? clo.x : clo.y, wh = j < 4 ? chi.x : chi.y;
            const uint32_t blo = min((wl >> (8 * (j & 3))) & 0xFFu, padc);
            const uint32_t bhi = min((wh >> (8 * (j & 3))) & 0xFFu, padc);
            // 24-bit multiplies (full rate; a 32-bit v_mul_lo is quarter rate)
            const uint4* plo = reinterpret_cast<const uint4*>(prof + __umul24(blo, a.PS) + 2 * pbase);
            const uint4* phi = reinterpret_cast<const uint4*>(prof + __umul24(bhi, a.PS) + 2 * pbase);
#pragma unroll
            for (int q = 0; q < R / 8; ++q) {
              const uint4 x = plo[q], y = phi[q];
              out.lo[4 * q] = x.x; out.lo[4 * q + 1] = x.y; out.lo[4 * q + 2] = x.z;
              out.lo[4 * q + 3] = x.w;
              out.hi[4 * q] = y.x; out.hi[4 * q + 1] = y.y; out.hi[4 * q + 2] = y.z;
              out.hi[4 * q + 3] = y.w;
            }
          };
          ProfLookup16<R> lk;
          if (jj == 0) load16(0, lk);
          else lk = lkq;
          if (jj + 1 < C) load16(jj + 1, lkq);
          __builtin_amdgcn_sched_barrier(0);
          if (COL0 && jj == 0 && c == 0)
            column_f16<R, RB, GOTOH, true>(lk, diag, upX, Hl, Xl, best, NOE2, NE2, NO2);
          else
            column_f16<R, RB, GOTOH, false>(lk, diag, upX, Hl, Xl, best, NOE2, NE2, NO2);
        } else if constexpr (PROF) {
          ProfLookup<R> lk;
          const uint32_t blo = min((wlo >> (8 * (jj & 3))) & 0xFFu, padc);
          const uint32_t bhi = min((whi >> (8 * (jj & 3))) & 0xFFu, padc);
          const uint4* plo = reinterpret_cast<const uint4*>(prof + __umul24(blo, a.PS) + pbase);
          const uint4* phi = reinterpret_cast<const uint4*>(prof + __umul24(bhi, a.PS) + pbase);
#pragma unroll
          for (int q = 0; q < R / 16; ++q) {
            const uint4 x = plo[q], y = phi[q];
            lk.lo[4 * q] = x.x; lk.lo[4 * q + 1] = x.y; lk.lo[4 * q + 2] = x.z;
            lk.lo[4 * q + 3] = x.w;
            lk.hi[4 * q] = y.x; lk.hi[4 * q + 1] = y.y; lk.hi[4 * q + 2] = y.z;
            lk.hi[4 * q + 3] = y.w;
          }
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (GOTOH) {
            u16x2 uH = upH;
            column_gotoh<R, RB>(lk, diag, uH, upX, Hl, Xl, best, S2, OES2, E2);
          } else if (COL0 && jj == 0 && c == 0) {
            column_merged<R, RB, true>(lk, diag, upX, Hl, Xl, best, S2, O2, E2);
          } else {
            column_merged<R, RB, false>(lk, diag, upX, Hl, Xl, best, S2, O2, E2);
          }
        } else if constexpr (PAIR) {
          // the next column's table address (its codes: this chunk, or byte 0 of the next)
          const uint32_t nwl = jj + 1 < C ? (jj + 1 < 4 ? clo.x : clo.y) : rlo.x;
          const uint32_t nwh = jj + 1 < C ? (jj + 1 < 4 ? chi.x : chi.y) : rhi.x;
          const int nsh = jj + 1 < C ? 8 * ((jj + 1) & 3) : 0;
          uint32_t Da, Db, X, DN, IN;
          const uint32_t noe = as_u32(as_u16x2(NOE2)), ne = as_u32(as_u16x2(NE2)),
                 no = as_u32(as_u16x2(NO2));
          u16x2 bst = best;
          u16x2 F = upX;  // Gotoh: F running down the column
#define SWK_PAIR_HT(B)                                                                        \
  [h0] "+v"(Hl[B]), [h1] "+v"(Hl[B + 1]), [h2] "+v"(Hl[B + 2]), [h3] "+v"(Hl[B + 3]),          \
      [h4] "+v"(Hl[B + 4]), [h5] "+v"(Hl[B + 5]), [h6] "+v"(Hl[B + 6]), [h7] "+v"(Hl[B + 7]),  \
      [t0] "+v"(Xl[B]), [t1] "+v"(Xl[B + 1]), [t2] "+v"(Xl[B + 2]), [t3] "+v"(Xl[B + 3]),      \
      [t4] "+v"(Xl[B + 4]), [t5] "+v"(Xl[B + 5]), [t6] "+v"(Xl[B + 6]), [t7] "+v"(Xl[B + 7]),  \
      [Db] "=&v"(Db), [best] "+v"(bst)
#define SWK_PAIR_OUT(B, DA) SWK_PAIR_HT(B), [Da] DA(Da), [X] "=&v"(X), [DN] "=&v"(DN), [IN] "=&v"(IN)
#define SWK_PAIR_OUTG(B, DA)                                                                  \
  SWK_PAIR_HT(B), [Da] DA(Da), [EN] "=&v"(X), [HN] "=&v"(DN), [FN] "=&v"(IN), [F] "+v"(F)
#define SWK_PAIR_IN(P0, P1)                                                                   \
  [p0] "v"(P0.x), [p1] "v"(P0.y), [p2] "v"(P0.z), [p3] "v"(P0.w), [p4] "v"(P1.x),             \
      [p5] "v"(P1.y), [p6] "v"(P1.z), [p7] "v"(P1.w), [noe] "s"(noe), [ne] "s"(ne), [no] "s"(no)
// block B of the column: first (row-0 prologue), middle or last (no successor row)
#define SWK_PAIR_BLOCK(KIND, B, P0, P1)                                                       \
  if constexpr (GOTOH) {                                                                      \
    if constexpr (KIND == 0)                                                                  \
      asm volatile(SWK_F16PAIRG_F : SWK_PAIR_OUTG(B, "=&v")                                   \
                   : SWK_PAIR_IN(P0, P1), [dg] "v"(diag), [pw] "v"(pw));                   \
    else if constexpr (KIND == 1)                                                             \
      asm volatile(SWK_F16PAIRG_M : SWK_PAIR_OUTG(B, "+v") : SWK_PAIR_IN(P0, P1));         \
    else                                                                                      \
      asm volatile(SWK_F16PAIRG_L : SWK_PAIR_OUTG(B, "+v") : SWK_PAIR_IN(P0, P1));         \
  } else {                                                                                    \
    if constexpr (KIND == 0)                                                                  \
      asm volatile(SWK_F16PAIR_F : SWK_PAIR_OUT(B, "=&v")                                     \
                   : SWK_PAIR_IN(P0, P1), [up] "v"(upX), [dg] "v"(diag), [pw] "v"(pw));                 \
    else if constexpr (KIND == 1)                                                             \
      asm volatile(SWK_F16PAIR_M : SWK_PAIR_OUT(B, "+v") : SWK_PAIR_IN(P0, P1), [up] "v"(Xl[B - 1]));   \
    else                                                                                      \
      asm volatile(SWK_F16PAIR_L : SWK_PAIR_OUT(B, "+v") : SWK_PAIR_IN(P0, P1), [up] "v"(Xl[B - 1]));   \
  }
          // each block's words are read one block ahead; the last block's wait for the next
          // column's block 0 and row-0 word
          uint4 pB0 = ld4(acur + 48), pB1 = ld4(acur + 64);  // block 1
          __builtin_amdgcn_sched_barrier(0);
          SWK_PAIR_BLOCK(0, 0, pA0, pA1)
          if constexpr (R == 32) {
            pA0 = ld4(acur + 80);  // block 2
            pA1 = ld4(acur + 96);
            __builtin_amdgcn_sched_barrier(0);
            SWK_PAIR_BLOCK(1, 8, pB0, pB1)
            pB0 = ld4(acur + 112);  // block 3
            pB1 = ld4(acur + 128);
            __builtin_amdgcn_sched_barrier(0);
            SWK_PAIR_BLOCK(1, 16, pA0, pA1)
          }
          acur = pair_addr(nwl, nwh, nsh);  // next column: block 0 and row-0 word
          pA0 = ld4(acur + 16);
          pA1 = ld4(acur + 32);
          pw = ld1(acur + 12);
          __builtin_amdgcn_sched_barrier(0);
          SWK_PAIR_BLOCK(2, R - 8, pB0, pB1)
#undef SWK_PAIR_BLOCK
#undef SWK_PAIR_HT
#undef SWK_PAIR_OUT
#undef SWK_PAIR_OUTG
#undef SWK_PAIR_IN
          (void)Db; (void)X; (void)DN; (void)IN;
          best = bst;
          upX = GOTOH ? F : Xl[R - 1];
        } else if constexpr (F16) {
          // selector bytes {0x0C, code_lo, 0x0C, code_hi}: the LUT byte is the f16 high byte
          const uint32_t sel16 = 0x0Cu | ((uint32_t)(jj & 3) << 8) | (0x0Cu << 16) |
                                 ((uint32_t)(4 + (jj & 3)) << 24);
          const LutLookup<R> lk{tab, nv, __builtin_amdgcn_perm(whi, wlo, sel16) | 0x000C000Cu};
          __builtin_amdgcn_sched_barrier(0);
          if (COL0 && jj == 0 && c == 0)
            column_f16<R, RB, GOTOH, true>(lk, diag, upX, Hl, Xl, best, NOE2, NE2, NO2);
          else
            column_f16<R, RB, GOTOH, false>(lk, diag, upX, Hl, Xl, best, NOE2, NE2, NO2);
        } else {
          // selector: byte 0 = code of the low target, byte 2 = code of the high target
          const uint32_t sel =
              (uint32_t)(jj & 3) | ((uint32_t)(4 + (jj & 3)) << 16) | 0x0C000C00u;
          const LutLookup<R> lk{tab, nv, __builtin_amdgcn_perm(whi, wlo, sel) | 0x0C000C00u};
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (GOTOH) {
            u16x2 uH = upH;
            column_gotoh<R, RB>(lk, diag, uH, upX, Hl, Xl, best, S2, OES2, E2);
          } else if (COL0 && jj == 0 && c == 0) {
            column_merged<R, RB, true>(lk, diag, upX, Hl, Xl, best, S2, O2, E2);
          } else {
            column_merged<R, RB, false>(lk, diag, upX, Hl, Xl, best, S2, O2, E2);
          }
        }
        // pin the running max once per column: otherwise LLVM re-associates the max over the
        // whole phase into a tree and keeps every M live
        asm volatile("" : "+v"(best));
        rout[jj * ostride] = make_uint2(as_u32(Hl[R - 1]), as_u32(upX));
      }
      if constexpr (PAIR && TRIM) {
        if (trimmed) {  // the next chunk's column 0, read ahead as at a chunk's end
          acur = pair_addr(rlo.x, rhi.x, 0);
          pA0 = ld4(acur + 16);
          pA1 = ld4(acur + 32);
          pw = ld1(acur + 12);
        }
      }
      (void)trimmed;
      if (seg_out && wave == W - 1) {  // this segment's bottom row -> the next segment
        uint2* dst = a.edge_out + ((size_t)(MQ ? unit : tile) * a.ecols + (size_t)c * C) * 64 + lane;
#pragma unroll
        for (int jj = 0; jj < C; ++jj) dst[jj * 64] = sink[jj * 64 + lane];
      }
      if (last) {
        // BAL: the first visit is a head when the range ends inside a tile
        if (BAL && k == 0 && bf > 0) {  // BAL: a head visit ends: hand its state over
          bal_store((int)blockIdx.x + 1);
        } else {  // this wave's part of tile k is done
        uint32_t* bs = bestsh + (k % W) * SWB_TILE;
        atomicMax(&bs[lane], (uint32_t)best.x);
        atomicMax(&bs[lane + 64], (uint32_t)best.y);
        if (wave == W - 1) {  // every other wave folded tile k in an earlier phase
          const size_t tlo = (size_t)tile * SWB_TILE + lane, thi = tlo + 64;
          int32_t blo = (int32_t)bs[lane], bhi = (int32_t)bs[lane + 64];
          bs[lane] = 0;
          bs[lane + 64] = 0;
          if constexpr (F16) {  // f16 bit patterns of non-negative integers -> int
            blo = f16_unscore((uint32_t)blo);
            bhi = f16_unscore((uint32_t)bhi);
          }
          const uint32_t* sx = TRIM && sidx ? sidx : idx;
          size_t slo = sx && tlo < n ? sx[tlo] : tlo;
          size_t shi = sx && thi < n ? sx[thi] : thi;
          if constexpr (STREAM) {  // ragged: through the chunk's visiting order
            if (wperm) {
              const size_t b0 = (size_t)wst0 * SWB_TILE;
              if (tlo < n) slo = b0 + wperm[tlo - b0];
              if (thi < n) shi = b0 + wperm[thi - b0];
            }
          }
          int32_t* qsc = MQ ? a.scores + (size_t)q * a.sstride : a.scores;
          if (a.accum) {  // best over the previous query segments
            if (tlo < n) blo = max(blo, qsc[slo]);
            if (thi < n) bhi = max(bhi, qsc[shi]);
          }
          if (tlo < n) qsc[slo] = blo;
          if (thi < n) qsc[shi] = bhi;
        }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
          Hl[r] = H0;
          Xl[r] = X0;
        }
        best = (u16x2){0, 0};
        prevUpH = H0;
        tile = ntile;
        if constexpr (STREAM) {
          packed = packed_n;
          wperm = cperm;
          wst0 = st0;
        }
        if constexpr (MQ && PAIR) unit = nunit;
        if constexpr (MQ && !PAIR) {  // several queries: the next unit's row LUTs
          unit = nunit;
          if (nqq != q) {
            q = nqq;
#pragma unroll
            for (int r = 0; r < R; ++r)
              tab[r] = __builtin_amdgcn_readfirstlane(a.qtab[(size_t)q * a.qwords + wave * R + r]);
          }
        }
        nch = nch_n;
        nfull = nfull_n;
        ncl = ncl_n;
        c = 0;
        if constexpr (BAL) {
          c = nc0;
          nch = nvend;
          if (nc0 > 0) bal_load();  // a tail: the head's state
        }
        ++k;
      } else {
        ++c;
      }
    }
    if constexpr (BAL) {
      if (bal_pend > 0 && --bal_pend == 0) bal_flag_out();
    }
#if SWK_STAMPS
    const bool st_own = g >= 0 && g < total;  // (fill / drain phases: all of it to st_idle)
    const uint64_t st_b = __builtin_amdgcn_s_memtime();
    (st_own ? st_act : st_idle) += st_b - st_p;
#endif
    __syncthreads();
#if SWK_STAMPS
    st_p = __builtin_amdgcn_s_memtime();
    (st_own ? st_bar : st_idle) += st_p - st_b;
#endif
  }
  if constexpr (BAL) {
    if (bal_pend > 0) bal_flag_out();
  }
#if SWK_STAMPS
  // (the non-streamed variants never read tctr: measurement builds pass the buffer there)
  uint64_t* const g_stamps = STREAM ? nullptr : reinterpret_cast<uint64_t*>(a.tctr);
  if (lane == 0 && g_stamps) {
    uint64_t* o = g_stamps + ((size_t)blockIdx.x * 16 + wave) * 16;
    unsigned hw = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    o[0] = st_t0;
    o[1] = __builtin_amdgcn_s_memtime();
    o[2] = st_act;
    o[3] = st_idle;
    o[4] = st_bar;
    o[5] = hw;
    unsigned xcc = 0;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    o[6] = (uint64_t)total;
    o[7] = (uint64_t)(xcc & 15);
    o[8] = st_bload;
  }
#endif
}

template <int R, int RB, bool COL0, bool PROF, bool GOTOH, bool F16, bool PAIR = false,
          bool MQ = false, bool STREAM = false, int C = 8, bool BAL = false, bool TRIM = false>
static hipError_t launch_score(const ScoreArgs& a, int W, uint32_t prof_bytes, hipStream_t st,
                               unsigned bal_grid = 0) {
  const size_t ntiles = (a.n + SWB_TILE - 1) / SWB_TILE * (MQ ? a.nq : 1);  // units
  const size_t lds = (size_t)W * SWB_TILE * 4 +
                     (size_t)(64 + (a.edge_out ? C * 64 : 64) + (a.edge_in ? 2 * C * 64 : 0) +
                              (W > 1 ? W - 1 : 0) * 2 * C * 64) * 8 +
                     (PROF ? prof_bytes : 0) + (PAIR ? a.PS : 0) + (STREAM ? 256 : 0);
  auto fn = &score_kernel<R, RB, COL0, PROF, GOTOH, F16, PAIR, MQ, STREAM, C, BAL, TRIM>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  if (lds > 160 * 1024) return hipErrorInvalidConfiguration;
  unsigned grid = BAL ? bal_grid
                      : persistent_grid(reinterpret_cast<const void*>(fn), ntiles, 64 * W, lds);
#if SWK_STAMPS
  if (!STREAM && g_stamps_host) {
    ScoreArgs b = a;
    b.tctr = reinterpret_cast<uint32_t*>(g_stamps_host);
    hipLaunchKernelGGL(fn, dim3(grid), dim3(64 * W), (unsigned)lds, st, b);
    return hipGetLastError();
  }
#endif
  if (MQ && PAIR) grid = std::max(a.nq, grid / a.nq * a.nq);  // one query per workgroup
  if (BAL && (grid == 0 || ntiles < 2 * (size_t)grid)) return hipErrorInvalidConfiguration;
  hipLaunchKernelGGL(fn, dim3(grid), dim3(64 * W), (unsigned)lds, st, a);
  return hipGetLastError();
}

}  // namespace swk

// Variants compiled in: (R, RB, COL0, PROF, GOTOH, F16).  The host picks R from the query
// length (SWBANK_R / SWBANK_RB override it for tuning).
#define SWK_VARIANTS(X)                                                                       \
  X(16, 4, 0, 0, 0, 0) X(16, 4, 1, 0, 0, 0) X(32, 4, 0, 0, 0, 0) X(32, 4, 1, 0, 0, 0)         \
  X(32, 8, 0, 0, 0, 0) X(64, 4, 0, 0, 0, 0) X(64, 4, 1, 0, 0, 0)                              \
  X(16, 4, 0, 0, 1, 0) X(32, 4, 0, 0, 1, 0) X(64, 4, 0, 0, 1, 0)                              \
  X(16, 4, 0, 1, 0, 0) X(16, 4, 1, 1, 0, 0) X(32, 4, 0, 1, 0, 0) X(32, 4, 1, 1, 0, 0)         \
  X(64, 4, 0, 1, 0, 0) X(64, 4, 1, 1, 0, 0)                                                   \
  X(16, 4, 0, 1, 1, 0) X(32, 4, 0, 1, 1, 0) X(64, 4, 0, 1, 1, 0)                              \
  X(16, 4, 0, 0, 0, 1) X(16, 4, 1, 0, 0, 1) X(32, 4, 0, 0, 0, 1) X(64, 4, 0, 0, 0, 1)         \
  X(16, 4, 0, 0, 1, 1)                                                                        \
  X(16, 4, 0, 1, 0, 1) X(16, 4, 1, 1, 0, 1) X(16, 4, 0, 1, 1, 1) X(32, 4, 0, 0, 1, 1)


extern "C" int swk_has_variant(int R, int RB, int col0, int prof, int gotoh, int f16) {
#define SWK_HAS(RR, BB, C0, PF, GT, FH) \
  if (R == RR && RB == BB && col0 == C0 && prof == PF && gotoh == GT && f16 == FH) return 1;
  SWK_VARIANTS(SWK_HAS)
#undef SWK_HAS
  return 0;
}

extern "C" hipError_t swk_launch_score(int R, int RB, int col0, int prof, int gotoh, int f16,
                                       const uint8_t* res, const uint64_t* offs,
                                       const uint32_t* lens, size_t n, const uint32_t* qtab,
                                       uint32_t nv, uint32_t S, uint32_t O, uint32_t E,
                                       uint32_t PS, uint32_t pad, int W, int32_t* scores,
                                       const void* edge_in, void* edge_out, uint32_t ecols,
                                       int accum, int packed, const uint32_t* idx,
                                       const uint32_t* nidx, uint32_t idx_base,
                                       const uint32_t* ident, int pair, uint32_t pS1,
                                       uint32_t pS2, uint32_t ulen, uint32_t ustride,
                                       uint32_t nq, uint32_t qwords, size_t sstride,
                                       hipStream_t st) {
  if (n == 0) return hipSuccess;
  swk::ScoreArgs a{res,  offs, lens, n,  qtab, nv, S,
                   O,    E,    PS,   pad, scores, static_cast<const uint2*>(edge_in),
                   static_cast<uint2*>(edge_out), ecols, (uint32_t)accum, (uint32_t)packed,
                   idx, nidx, idx_base, ident, pS1, pS2,
                   swk::f16_pair(-(int)(O + E)), swk::f16_pair(-(int)E),
                   swk::f16_pair(-(int)O), nullptr, 0u, 0u, 0};
  a.ulen = ulen;
  a.ustride = ustride;
  a.nq = nq;
  a.qwords = qwords;
  a.sstride = sstride;
  const uint32_t prof_bytes = (pad + 1) * PS;
  if (nq > 1 && pair) {  // several queries, pair tables (PS = one table's bytes)
    // more than 4 waves (a 512-row table): 4-column chunks, so the ring fits beside the table;
    // every segment of a segmented set too (a short last segment reads exactly the edge
    // chunks the one before it wrote)
    if (R == 32 && f16 && !prof && !gotoh && !col0 && (W > 4 || a.edge_in || a.edge_out))
      return swk::launch_score<32, 4, false, false, false, true, true, true, false, 4>(a, W, 0, st);
    if (R == 32 && f16 && !prof && !gotoh && !col0)
      return swk::launch_score<32, 4, false, false, false, true, true, true>(a, W, 0, st);
    return hipErrorInvalidValue;
  }
  if (nq > 1) {  // several queries: row-LUT variants without the column-0 rule
#define SWK_MQ_CASE(RR, GT, FH)                                                                  \
  if (R == RR && RB == 4 && !col0 && !prof && !pair && gotoh == GT && f16 == FH)                 \
    return swk::launch_score<RR, 4, false, false, (GT != 0), (FH != 0), false, true>(a, W, 0, st);
    SWK_MQ_CASE(32, 0, 1) SWK_MQ_CASE(32, 0, 0) SWK_MQ_CASE(16, 0, 1) SWK_MQ_CASE(16, 0, 0)
    SWK_MQ_CASE(16, 1, 1) SWK_MQ_CASE(16, 1, 0) SWK_MQ_CASE(32, 1, 1) SWK_MQ_CASE(32, 1, 0)
#undef SWK_MQ_CASE
    return hipErrorInvalidValue;
  }
  if (pair) {  // PS = pair-table bytes
    if (R == 32 && f16 && !prof && !gotoh && !col0)
      return swk::launch_score<32, 4, false, false, false, true, true>(a, W, 0, st);
    // DNA Gotoh: 8-column chunks while the hand-off ring fits beside the table, else 4 (a
    // 512-row table beside 16 waves).  A segmented query runs every segment with 4: the edge
    // rows one segment writes are exactly the chunks the next one reads
#define SWK_GPAIR(RR)                                                                         \
    if (R == RR && f16 && !prof && gotoh && !col0) {                                          \
      const hipError_t e = a.edge_in || a.edge_out                                            \
          ? hipErrorInvalidConfiguration                                                      \
          : swk::launch_score<RR, 4, false, false, true, true, true>(a, W, 0, st);            \
      if (e != hipErrorInvalidConfiguration) return e;                                        \
      return swk::launch_score<RR, 4, false, false, true, true, true, false, false, 4>(a, W, 0, \
                                                                                         st); \
    }
    SWK_GPAIR(32) SWK_GPAIR(16)
#undef SWK_GPAIR
    return hipErrorInvalidValue;
  }
#define SWK_CASE(RR, BB, C0, PF, GT, FH)                                                      \
  if (R == RR && RB == BB && col0 == C0 && prof == PF && gotoh == GT && f16 == FH)            \
    return swk::launch_score<RR, BB, (C0 != 0), (PF != 0), (GT != 0), (FH != 0)>(a, W,        \
                                                                               prof_bytes, st);
  SWK_VARIANTS(SWK_CASE)
#undef SWK_CASE
  return hipErrorInvalidValue;
}

#if SWK_STAMPS
// (measurement builds) per-wave phase timing of the next tile-kernel launches into p:
// [block][16 waves][16] u64 = entry, exit, active, fill/drain, barrier cycles, HW_ID, chunks,
// XCC, tail state load cycles
extern "C" void swk_set_stamps(void* p) { swk::g_stamps_host = static_cast<uint64_t*>(p); }
#endif

// Balanced chunk ranges (ScoreArgs.bal_*) for the DNA merged f16 pair-table kernel (the
// headline shape): codes one byte each (or ustride / ulen), one query segment of W <= 4 waves.
// swk_bal_slots gives the grid (every resident slot); the host sizes bal_state ((grid + 1) x W
// x (2R + 2) x 64 words) and bal_flag ((grid + 1) x W words, zeroed once); a hand-off wait
// that runs out after poll_limit polls marks *fault (SWK_FAULT_BAL).  plan: grid + 1 entries {tile, chunk, chunk index} (swk_bal_plan_uniform for
// a uniform batch; a ragged batch visited longest first through the device sort's permutation
// idx / nidx / ident passes the sort's, swk_sort_lens with the same grid).
namespace swk {
__global__ void __launch_bounds__(256) bal_plan_uniform(uint4* plan, uint32_t ntiles, uint32_t K,
                                                        uint32_t G) {
  for (uint32_t g = threadIdx.x; g <= G; g += blockDim.x) {
    const uint64_t A = (uint64_t)ntiles * K * g / G;
    plan[g] = make_uint4((uint32_t)(A / K), (uint32_t)(A % K), (uint32_t)A, 0u);
  }
}
}  // namespace swk

// The plan of a uniform batch (ntiles tiles of K chunks, G workgroups): entry g = {tile, chunk,
// chunk index} of chunk floor(g ntiles K / G), g = 0..G (ntiles K < 2^31).
extern "C" hipError_t swk_bal_plan_uniform(void* plan, uint32_t ntiles, uint32_t K, uint32_t G,
                                           hipStream_t st) {
  if (!plan || K == 0 || G == 0 || (uint64_t)ntiles * K >= (1ull << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(swk::bal_plan_uniform, dim3(1), dim3(256), 0, st, static_cast<uint4*>(plan),
                     ntiles, K, G);
  return hipGetLastError();
}

extern "C" unsigned swk_bal_slots(int W, uint32_t PS, int trim) {
  const void* fn =
      trim ? reinterpret_cast<const void*>(
                 &swk::score_kernel<32, 4, false, false, false, true, true, false, false, 8, true,
                                    true>)
           : reinterpret_cast<const void*>(
                 &swk::score_kernel<32, 4, false, false, false, true, true, false, false, 8, true>);
  if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
      hipSuccess)
    return 0;
  const size_t lds = (size_t)W * SWB_TILE * 4 + (size_t)(64 + 64 + (W - 1) * 2 * 8 * 64) * 8 + PS;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  const int occ = swk::cached_occupancy(fn, 64 * W, lds, dev, &cus);
  return occ > 0 && cus > 0 ? (unsigned)(occ * cus) : 0u;
}

extern "C" hipError_t swk_launch_pair_bal(const uint8_t* res, const uint64_t* offs,
                                          const uint32_t* lens, size_t n, const uint32_t* qtab,
                                          uint32_t nv, uint32_t S, uint32_t O, uint32_t E,
                                          uint32_t PS, uint32_t pad, int W, int32_t* scores,
                                          uint32_t pS1, uint32_t pS2, uint32_t ulen,
                                          uint32_t ustride, uint32_t* flag, uint32_t* state,
                                          uint32_t gen, unsigned grid, const uint32_t* idx,
                                          const uint32_t* nidx, const uint32_t* ident,
                                          const void* plan, uint32_t* fault, uint32_t poll_limit,
                                          uint32_t stall, int trim, uint32_t packed,
                                          const uint32_t* sidx, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (W > 4 || !flag || !state || !plan || !fault || poll_limit == 0 || (idx && !nidx) ||
      (packed != SWK_PACK_BYTES && packed != SWK_PACK_NIBBLE) || (sidx && (!trim || idx)))
    return hipErrorInvalidValue;
  swk::ScoreArgs a{res,  offs, lens, n,  qtab, nv, S,
                   O,    E,    PS,   pad, scores, nullptr, nullptr, 0u, 0u, packed,
                   idx, nidx, 0u, ident, pS1, pS2,
                   swk::f16_pair(-(int)(O + E)), swk::f16_pair(-(int)E),
                   swk::f16_pair(-(int)O), nullptr, 0u, 0u, 0};
  a.ulen = ulen;
  a.ustride = ustride;
  a.nq = 1;
  a.bal_flag = flag;
  a.bal_state = state;
  a.bal_gen = gen;
  a.bal_plan = static_cast<const uint4*>(plan);
  a.fault = fault;
  a.poll_limit = poll_limit;
  a.stall = stall;
  a.sidx = sidx;
  if (trim)  // (a ragged batch: its tiles' last chunks stop at their last column)
    return swk::launch_score<32, 4, false, false, false, true, true, false, false, 8, true, true>(
        a, W, 0, st, grid);
  return swk::launch_score<32, 4, false, false, false, true, true, false, false, 8, true>(
      a, W, 0, st, grid);
}

// Streamed host batch (the feeder's one-launch path): equal-length targets (ulen codes), or
// ragged ones (ulen = 0: each chunk's region starts with its offsets, lengths and order), the
// chunk records `sc` and layout words dflag (device) / hflag (host), the codes in the device
// buffer `res`; row-LUT or
// pair-table variants without the column-0 rule, one query segment.
extern "C" hipError_t swk_launch_stream(int R, int gotoh, int f16, int pair, const uint8_t* res,
                                        size_t n, uint32_t ulen, const SwkStreamChunk* sc,
                                        const uint32_t* hflag, uint32_t* dflag, uint32_t nsc,
                                        uint32_t* tctr, const uint32_t* qtab, uint32_t nv,
                                        uint32_t S, uint32_t O, uint32_t E, uint32_t PS,
                                        uint32_t pad, int W, int32_t* scores, uint32_t pS1,
                                        uint32_t pS2, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (!sc || !hflag || !dflag || !tctr || nsc == 0) return hipErrorInvalidValue;
  swk::ScoreArgs a{res,  nullptr, nullptr, n, qtab, nv, S, O, E, PS, pad, scores, nullptr, nullptr,
                   0u, 0u, (uint32_t)SWK_PACK_STREAM, nullptr, nullptr, 0u, nullptr, pS1, pS2,
                   swk::f16_pair(-(int)(O + E)), swk::f16_pair(-(int)E),
                   swk::f16_pair(-(int)O), nullptr, 0u, 0u, 0};
  a.ulen = ulen;
  a.sc = sc;
  a.hflag = hflag;
  a.dflag = dflag;
  a.tctr = tctr;
  a.nsc = nsc;
  if (pair) {
    if (R == 32 && f16 && !gotoh)
      return swk::launch_score<32, 4, false, false, false, true, true, false, true>(a, W, 0, st);
    if (R == 32 && f16 && gotoh)
      return swk::launch_score<32, 4, false, false, true, true, true, false, true>(a, W, 0, st);
    if (R == 16 && f16 && gotoh)
      return swk::launch_score<16, 4, false, false, true, true, true, false, true>(a, W, 0, st);
    return hipErrorInvalidValue;
  }
#define SWK_ST_CASE(RR, GT, FH)                                                                  \
  if (R == RR && gotoh == GT && f16 == FH)                                                       \
    return swk::launch_score<RR, 4, false, false, (GT != 0), (FH != 0), false, false, true>(     \
        a, W, 0, st);
  SWK_ST_CASE(32, 0, 1) SWK_ST_CASE(32, 0, 0) SWK_ST_CASE(16, 0, 1) SWK_ST_CASE(16, 0, 0)
  SWK_ST_CASE(16, 1, 1) SWK_ST_CASE(16, 1, 0) SWK_ST_CASE(32, 1, 1) SWK_ST_CASE(32, 1, 0)
#undef SWK_ST_CASE
  return hipErrorInvalidValue;
}

