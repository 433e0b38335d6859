// swbank_launch.hip — kernel choice and launches; the device-buffer API.
// 
// sw_score_batch_device[_range] ≙ the ScoreBank port group data_in{tflag, ID, LEN, SEQ} ->
// results / IDs / vld (ScoreBank/ScoreBank_v2.v:39-41,164-165) on device-resident batches.
#include "swbank_bank.h"

// True when every length in [min_len, max_len] falls in the device sort's first length bin
// (swk_sort_lens: bins of 2^shift lengths below max_len, at most 2048 of them): the caller's
// order is then already longest first, and the sort kernels are not launched at all.
static bool one_len_bin(uint32_t min_len, uint32_t max_len) {
  if (min_len > max_len) return false;
  uint32_t shift = 0;
  while ((max_len >> shift) >= 2048u) ++shift;
  return ((max_len - min_len) >> shift) == 0;
}

// The u16 Gotoh column at R = 32 does not fit 128 VGPRs (it spills); a one-segment query of
// at most 256 rows runs it at R = 16 over the same row LUT (rows are laid out linearly, W x R
// words padded past the query), in ceil(|q| / 16) waves.
void u16_gotoh_rows(const sw_bank* b, bool f16, int& R, int& W) {
  if (f16 || !b->gotoh() || b->prof || R != 32 || b->segs.size() != 1 || b->query.size() > 256)
    return;
  R = 16;
  W = std::max(1, (int)((b->query.size() + 15) / 16));
}

// The tile / wave choice for n targets of at most max_len codes in the given arithmetic
// (before the layout constraints launch() adds).
bool wave_preferred(const sw_bank* b, size_t n, uint32_t max_len, bool use_f16) {
  const size_t nseg = b->segs.size();
  const size_t ntiles = (n + SWB_TILE - 1) / SWB_TILE;
  const bool gotoh = b->cfg.gap_model == SW_GAP_GOTOH;
  // Kernel choice by a throughput model calibrated on MI355X (scripts/kernel_choice.py):
  //  tile kernel: base rate x fraction of the 256 CUs holding a tile x f(waves per SIMD),
  //    f = min(1, 0.45 + 0.15 w), x 0.85 when the query runs as several segments;
  //  wave kernel (queries <= 1024 rows): base rate x row fill (query / 64K lanes' rows) x
  //    column fill (L / (L + 63): the 63-step skew of the lane pipeline).
  // Base GCUPS: tile f16 merged 9000 (profile 8000), f16 Gotoh 8500 with the letter-pair
  // table (7500 row LUT, profile 7100), u16
  // merged 7400 (profile 6500), u16 Gotoh 5800 (profile 5600); wave f16 merged 8600
  // (profile 7700), f16 Gotoh 7800 (profile 6800), u16 merged 7600 (profile 6600), u16 Gotoh
  // 6100 (profile 5200).  SWBANK_KERNEL=tile|wave forces one.
  const double tiles = (double)ntiles, W = b->segs[0].W;
  const double cu_frac = std::min(1.0, tiles / 256.0);
  const double wps = std::min(4.0, std::max(1.0, std::ceil(tiles / 256.0)) * W / 4.0);
  const bool pair_tab = use_f16 && b->pair_bytes != 0 && env_int("SWBANK_PAIR", 1) != 0;
  const double tile_base = use_f16 ? (gotoh ? (b->prof ? 7100 : pair_tab ? 8500 : 7500)
                                            : (b->prof ? 8000 : 9000))
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
  return use_wave;
}

// Polls of a cross-workgroup hand-off wait before it gives up (ScoreArgs.poll_limit): the
// kernel's default (about 4 s), or SWBANK_POLL_LIMIT (a test hook: short waits with SWBANK_STALL).
static uint32_t poll_limit(uint32_t dflt) {
  const int v = env_int("SWBANK_POLL_LIMIT", 0);
  return v > 0 ? (uint32_t)v : dflt;
}

// Ragged balanced launches stop each tile's last chunk at its last column (the TRIM variant of
// the pair kernel); SWBANK_TRIM=0 keeps whole chunks (A/B).
static int ragged_trim() { return env_int("SWBANK_TRIM", 1) != 0 ? 1 : 0; }

// packed (SWK_PACK_*): RECORDS: d_res holds n 64-byte CAPI records (2-bit codes), d_offs and
// d_lens are unused; STREAM: 2-bit codes, d_offs in bytes (the host feeder's DNA chunks).
// perm/perm_n (optional, tile kernel): pass 0 visits the targets in the order perm[0..n)
// (target numbers; *perm_n = n on the device), e.g. longest first; the wave kernel ignores it.
sw_status launch(sw_bank* b, const uint8_t* d_res, const uint64_t* d_offs,
                 const uint32_t* d_lens, size_t n, uint32_t max_len, int32_t* d_scores,
                 hipStream_t st, uint32_t packed, const uint32_t* perm, const uint32_t* perm_n,
                 bool dsort, bool wait_prev, uint32_t* sort_out, uint32_t* sort_scr, uint32_t ulen,
                 uint32_t ustride, uint32_t min_len) {
  // Past the 16-bit lanes (min(|q|, max|t|) * max(s) + max(s) > 65535) the 16-bit passes are
  // still exact for every pair scoring <= 65535 - max(s); the pairs above are re-scored by the
  // int32 kernel through an index list (swk_launch_i32).
  const uint64_t bound = std::min<uint64_t>(b->query.size(), max_len) *
                             (uint64_t)std::max(0, b->smax) + (uint64_t)std::max(0, b->smax);
  const bool need32 = bound > 65535u || env_int("SWBANK_I32", 0) != 0;
  // a uniform batch (ustride != 0: no offset / length arrays) cannot feed the int32 kernel
  if (need32 && ustride) return fail(b, SW_ERR_ARG, "uniform batch past the 16-bit bound");
  if (need32) {
    if (n > 0xFFFFFFFFull)
      return fail(b, SW_ERR_RANGE, "batches past the 16-bit score bound hold < 2^32 targets");
    const sw_status ps = prepare_i32(b);
    if (ps != SW_OK) return ps;
  }
  sw_bank::Ev ev{};
  // no separate feeder kernel: the score kernel streams the codes itself, so the "pack"
  // interval is empty (b = a: one event fewer between two steps' kernels, ~4 us)
  if (b->timing) {
    HIPOK(b, hipEventCreate(&ev.a));
    HIPOK(b, hipEventCreate(&ev.c));
    HIPOK(b, hipEventRecord(ev.a, st));
    ev.b = ev.a;
  }
  HIPOK(b, hipStreamWaitEvent(st, b->ev_ready, 0));  // the query tables are uploaded
  // bank-owned scratch (edge rows, re-score lists, the device sort order, int32 scratch) is
  // reused by every call: a call on another stream waits for the previous call to finish
  // (the host feeder's scratch-free chunk launches on two streams skip it, wait_prev = false)
  if (wait_prev) HIPOK(b, hipStreamWaitEvent(st, b->ev_used, 0));
  const size_t nseg = b->segs.size();
  const bool rec = packed == SWK_PACK_RECORDS;
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
  // re-scores the pairs above that threshold in u16.
  const bool f16_ok = b->f16 && b->f16_neg >= -2048 && env_int("SWBANK_F16", 1) != 0;
  const bool exact16 = f16_ok && top <= 2048u;
  const bool opt16 = f16_ok && !exact16 && n <= 0xFFFFFFFFull;  // the re-score list holds 32-bit target numbers
  const bool use_f16 = exact16 || opt16;
  bool use_wave = wave_preferred(b, n, max_len, use_f16);
  if (packed == SWK_PACK_MIXED) use_wave = false;  // (the feeder's mixed chunks: tile kernel)
  // the f16 wave kernel carries profile offsets in 16-bit halves (24 letters + pad fit)
  if (use_f16 && b->prof && (size_t)(b->alpha + 1) * b->wPS16 > 65536) use_wave = false;
  const char* arith = opt16 ? "f16+u16-rescore" : use_f16 ? "f16" : "u16";
  // the f16 pass of the tile kernel reads the letter-pair table when the query has one
  const bool use_pair = use_f16 && b->pair_bytes != 0 && env_int("SWBANK_PAIR", 1) != 0;
  bool wave_fb = false;  // the wave kernel re-scores its own flagged pairs
  if (use_wave) {
    // f16 profile, one segment of <= 512 rows (configs[4]): two pairs per wave, 16 rows per
    // lane (swk wave_two_pairs); SWBANK_WAVE_HALF=0 keeps one pair per wave
    const bool half = use_f16 && b->prof && !b->col0 && b->wK == 8 && b->wsegs == 1 &&
                      env_int("SWBANK_WAVE_HALF", 1) != 0;
    snprintf(b->last_kernel, sizeof(b->last_kernel), "wave %s%s K=%d segs=%d%s", arith,
             b->prof ? "-profile" : "", b->wK, b->wsegs, half ? " pairs/wave=2" : "");
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
    // optimistic f16 with one query segment: the wave re-scores a flagged pair in u16 itself
    // (no flag kernel, no re-score launches)
    wave_fb = opt16 && b->wsegs == 1;
    // Split tail: pairs beyond a whole number of waves per SIMD (one wave per pair, all
    // resident) would put one more wave on some SIMDs and set the kernel's length; the last
    // pairs % SIMDs pairs (when at most half the SIMDs) run instead as P row segments of K/P
    // rows per lane each (P = 4 with 4 x that many waves, else 2), in the same launch.
    // SWBANK_WAVE_SPLIT=0 disables, =N splits the last N pairs (tests); SWBANK_WAVE_SPLIT_P
    // forces P.
    SwkWaveSplit sp{};
    const size_t pairs = (n + 1) / 2;
    const int sforce = env_int("SWBANK_WAVE_SPLIT", -1);
    // Balanced ranges (two pairs per wave, equal target lengths): every resident
    // wave slot scores the same number of 32-step blocks of the unit sequence, a unit cut by a
    // range boundary handed between waves, instead of a tail of pairs % slots pairs.
    // * 8-wave blocks (one LDS profile per 8 waves: 4 waves per SIMD, 4,096 slots) when there is
    //   a unit per slot: +4-5 % over 4-wave blocks from 16,384 targets up.  Below, a unit is
    //   longer than a range and its pieces form a chain (a middle visit waits for its
    //   predecessor): the unit's serial length at a quarter of a SIMD outlasts the whole launch
    //   at 3 waves per SIMD (12,500 targets: -11 %), so 4-wave blocks stay.
    // * 4-wave blocks (3 waves per SIMD, 3,072 slots) with at least one unit per slot and a
    //   remainder.
    // SWBANK_WAVE_BAL=0 disables; SWBANK_WAVE_W=4 / =8 forces the block size (=8 down to ranges
    // of 4 blocks: tests of the chained visits).
    bool wbal = false;
    if (half && b->wsegs == 1 && n == wspan && !b->no_handoff && (ustride || min_len == max_len) &&
        sforce < 0 && pairs <= 0xFFFFFFFFull && env_int("SWBANK_WAVE_BAL", 1) != 0) {
      const size_t U = (pairs + 1) / 2, B = (max_len + 31 + 31) / 32;
      const int wforce = env_int("SWBANK_WAVE_W", 0);
      int W = wforce == 4 ? 4 : 8;
      unsigned grid = swk_wave_half_grid(gotoh ? 1 : 0, (b->pad + 1) * b->wPS16, W);
      if (W == 8 && !(grid && (wforce == 8 ? U * B >= 4 * (size_t)W * grid
                                            : U >= (size_t)W * grid))) {
        W = 4;
        grid = swk_wave_half_grid(gotoh ? 1 : 0, (b->pad + 1) * b->wPS16, W);
      }
      const size_t G = (size_t)W * grid;
      uint32_t* fw = grid ? fault_word(b) : nullptr;
      if (grid && fw && (W == 8 || (U >= G && U % G))) {
        const size_t sw = (G + 1) * 36 * 64;  // (WBAL_WORDS per lane)
        HIPOK(b, b->wbal_state.reserve(sw));
        if (b->wbal_flag.cap < G + 1) {  // zeroed once: flags carry wbal_gen
          HIPOK(b, b->wbal_flag.reserve(G + 1));
          HIPOK(b, hipMemsetAsync(b->wbal_flag.p, 0, b->wbal_flag.cap * 4, st));
        }
        sp.wbal_blocks = (uint32_t)B;
        sp.wbal_grid = grid;
        sp.wbal_waves = (unsigned)W;
        sp.wbal_gen = ++b->wbal_gen;
        sp.wbal_flag = b->wbal_flag.p;
        sp.wbal_state = b->wbal_state.p;
        sp.fault = fw + (b->host_call ? SWK_FAULT_WORDS : 0);
        sp.poll_limit = poll_limit(1u << 23);
        sp.stall = (unsigned)std::max(0, env_int("SWBANK_STALL", 0));
        wbal = true;
        const size_t L = strlen(b->last_kernel);
        snprintf(b->last_kernel + L, sizeof(b->last_kernel) - L, " balanced grid=%ux%d", grid, W);
      }
    }
    if (!wbal && b->sK[0] && b->wsegs == 1 && n == wspan && pairs <= 0xFFFFFFFFull) {
      const size_t simds = 4 * (size_t)std::max(b->cus, 1);
      const size_t units = half ? 2 * simds : simds;  // pairs per layer of one wave per SIMD
      size_t T = 0;
      if (sforce >= 0) T = std::min(pairs, (size_t)sforce);
      else if (pairs >= units && pairs % units <= units / 2) T = pairs % units;
      const int pforce = env_int("SWBANK_WAVE_SPLIT_P", 0);
      // two pairs per wave (f16): a tail of at most SIMDs / 8 pairs runs as 8 segments of 64
      // rows, one wave each on its own SIMD at the top issue priority, handed on through global
      // memory; SWBANK_WAVE_SPLIT_P=4 forces the in-block split
      // (no_handoff: a host call's re-run after a hand-off wait ran out, take_fault)
      const bool seg8 = half && b->sK[2] == 1 && T && !b->no_handoff &&
                        (pforce == 8 || (!pforce && 8 * T <= simds));
      const int i = pforce == 2 ? 0 : pforce == 4 ? 1 : (4 * T <= simds ? 1 : 0);
      uint32_t* fw = seg8 ? fault_word(b) : nullptr;
      if (seg8 && !fw) return fail(b, SW_ERR_NOMEM, "fault word allocation failed");
      if (seg8) {
        HIPOK(b, b->sring.reserve(std::max<size_t>(1, T * 7 * (size_t)ecols)));
        const size_t pw = T * 8 * 3;  // progress, bests (uint2)
        HIPOK(b, b->tprog.reserve(pw));
        HIPOK(b, hipMemsetAsync(b->tprog.p, 0, pw * 4, st));
        sp.pairs = (unsigned)T;
        sp.P = 8;
        sp.qtab = b->stab16[2].p;
        sp.words = (unsigned)b->sseg_words16[2];
        sp.PS = b->sPS16[2];
        sp.ring = b->sring.p;
        sp.cols = ecols;
        sp.prog = b->tprog.p;
        sp.fault = fw + (b->host_call ? SWK_FAULT_WORDS : 0);
        sp.poll_limit = poll_limit(1u << 24);
        sp.stall = (unsigned)std::max(0, env_int("SWBANK_STALL", 0));
        const size_t L = strlen(b->last_kernel);
        snprintf(b->last_kernel + L, sizeof(b->last_kernel) - L, " tail=%zu/8", T);
      } else if (T && b->sK[i]) {
        const unsigned P = 2u << i;
        HIPOK(b, b->sring.reserve((T + 4 / P - 1) / (4 / P) * (4 / P) * (P - 1) * 256));
        sp.pairs = (unsigned)T;
        sp.P = P;
        sp.qtab = use_f16 ? b->stab16[i].p : b->stab[i].p;
        sp.words = (unsigned)(use_f16 ? b->sseg_words16[i] : b->sseg_words[i]);
        sp.PS = use_f16 && b->prof ? b->sPS16[i] : b->sPS[i];
        sp.fb_qtab = b->stab[i].p;
        sp.fb_words = (unsigned)b->sseg_words[i];
        sp.fb_PS = b->sPS[i];
        sp.ring = b->sring.p;
        const size_t L = strlen(b->last_kernel);
        snprintf(b->last_kernel + L, sizeof(b->last_kernel) - L, " split=%zu/%u", T, P);
      }
    }
    for (size_t p0 = 0; p0 < n; p0 += wspan) {
      const size_t np = std::min(wspan, n - p0);
      for (int sg = 0; sg < b->wsegs; ++sg) {
        const void* ein = sg > 0 ? b->edge[(sg - 1) & 1].p : nullptr;
        void* eout = sg + 1 < b->wsegs ? b->edge[sg & 1].p : nullptr;
        HIPOK(b, swk_launch_wave(
                     b->wK, b->col0, b->prof, gotoh ? 1 : 0, use_f16 ? 1 : 0, ein, eout, ecols,
                     sg > 0 ? 1 : 0, rec ? d_res + p0 * SWB_RECORD : d_res,
                     rec ? d_offs : d_offs + p0, rec ? d_lens : d_lens + p0, np,
                     use_f16 ? b->wtab16.p + sg * b->wseg_words16 : b->wtab.p + sg * b->wseg_words,
                     use_f16 ? b->nv16 : b->nv, b->S, b->O, b->E,
                     use_f16 && b->prof ? b->wPS16 : b->wPS, b->pad, d_scores + p0,
                     (int)packed, wave_fb ? b->wtab.p : nullptr, b->nv, b->wPS,
                     2048 - std::max(0, b->smax), &sp, ulen, ustride, half ? 1 : 0, st));
      }
    }
  } else {
    int R0 = b->R, W0 = b->segs[0].W;  // (the first pass's rows per wave)
    u16_gotoh_rows(b, use_f16, R0, W0);
    snprintf(b->last_kernel, sizeof(b->last_kernel), "tile %s%s R=%d W=%d segs=%zu", arith,
             b->prof ? "-profile" : use_pair ? " pair" : "", R0, W0, nseg);
  }
  // A device batch (dsort) visits its targets longest first, sorted on the device, so every
  // tile holds similar lengths (a tile runs to its longest lane); SWBANK_DSORT=0 disables.
  const uint32_t* ident = nullptr;  // device sort: 1 when the lengths share one bin
  // Balanced chunk ranges over a ragged device batch: the sort's last block also
  // writes where each workgroup's range starts in the longest-first tile sequence, so the choice
  // is made before the sort.  Every range must hold two of the longest tiles' chunks (the head
  // and the tail of a range are different tiles): checked with the caller's length bounds.
  unsigned rbal_grid = 0;
  if (dsort && !sort_out && !b->no_handoff && !use_wave && !perm && use_f16 && use_pair && !gotoh && nseg == 1 &&
      wait_prev && (packed == SWK_PACK_BYTES || packed == SWK_PACK_NIBBLE) && min_len < max_len &&
      max_len < 2048 && !opt16 &&
      b->R == 32 && b->segs[0].W <= 4 && n <= 0xFFFFFFFFull && env_int("SWBANK_DSORT", 1) != 0 &&
      env_int("SWBANK_BAL", 1) != 0 && env_int("SWBANK_BAL_RAGGED", 1) != 0 &&
      !one_len_bin(min_len, max_len)) {
    const unsigned grid = swk_bal_slots(b->segs[0].W, b->pair_bytes, ragged_trim());
    const size_t kmin = std::max<uint32_t>(1u, (min_len + 7) / 8), kmax = (max_len + 7) / 8;
    if (grid && ntiles * kmin >= 2 * (size_t)grid * kmax && ntiles * kmax < (1ull << 31))
      rbal_grid = grid;
  }
  // (the host feeder passes a chunk's own order (n + 2 words in its slot) and sort scratch, so
  // chunks on two streams do not share them)
  if (dsort && !use_wave && !perm && packed != SWK_PACK_RECORDS && ntiles > 1 &&
      n <= 0xFFFFFFFFull && !one_len_bin(min_len, max_len) && env_int("SWBANK_DSORT", 1) != 0) {
    uint32_t* order = sort_out;
    if (!order) {
      HIPOK(b, b->dperm.reserve(n + 2));
      order = b->dperm.p;
    }
    uint32_t* scr = sort_scr;
    if (!scr) {
      const size_t sw = swk_sort_scratch_bytes() / 4;
      if (b->dsort.cap < sw) {  // zeroed once; the sort kernels leave it zeroed
        HIPOK(b, b->dsort.reserve(sw));
        HIPOK(b, hipMemsetAsync(b->dsort.p, 0, sw * 4, st));
      }
      scr = b->dsort.p;
    }
    if (rbal_grid) {
      HIPOK(b, b->bal_plan.reserve((size_t)(rbal_grid + 1) * 4));
      b->bal_key[0] = 0;  // the uniform plan is overwritten
    }
    HIPOK(b, swk_sort_lens(d_lens, n, max_len, order, order + n, order + n + 1, scr, st,
                           rbal_grid ? b->bal_plan.p : nullptr, rbal_grid));
    ++b->ctr.device_sorts;
    if (!sort_out) {  // (the host feeder's chunks sort too: not named per chunk)
      const size_t L = strlen(b->last_kernel);
      snprintf(b->last_kernel + L, sizeof(b->last_kernel) - L, " dsort");
    }
    perm = order;
    perm_n = order + n;
    ident = order + n + 1;
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
  for (int pass = use_wave ? 1 : 0; pass < (opt16 && !wave_fb ? 2 : 1); ++pass) {
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
      const uint32_t* nidx = nullptr;
      if (pass == 0 && perm) {  // whole arrays, visited through the permutation
        idx = perm + p0;
        nidx = perm_n;
      } else if (pass == 0 && rec) {
        res = d_res + p0 * SWB_RECORD;
        scores = d_scores + p0;
      } else if (pass == 0) {
        offs = d_offs + p0;
        lens = d_lens + p0;
        scores = d_scores + p0;
      } else {
        idx = b->fb_idx.p + p0;
        nidx = b->fb_cnt.p;
      }
      // Balanced chunk ranges (the headline shape: a uniform batch through the pair-table
      // kernel): every resident workgroup slot scores the same number of 8-column chunks, tiles
      // cut by a range boundary handed between workgroups (ScoreArgs.bal_*).  Persistent
      // workgroups with whole tiles leave the slots past tiles mod slots idle in the last round
      // (998 of 1,024 on the headline batch, -2.4 %).  A ragged device batch (rbal_grid) runs
      // through the sort's permutation with the sort's plan.  SWBANK_BAL=0 disables.
      const bool rbal = pass == 0 && rbal_grid && perm && idx == perm && span == n;
      if (rbal || (pass == 0 && !b->no_handoff && f16 && use_pair && !gotoh && nseg == 1 && !idx && wait_prev &&
                   (packed == SWK_PACK_BYTES || packed == SWK_PACK_NIBBLE) && min_len == max_len &&
                   max_len > 0 && span == n &&
                   ntiles * ((max_len + 7) / 8) < (1ull << 31) && !opt16 && b->R == 32 &&
                   b->segs[0].W <= 4 && env_int("SWBANK_BAL", 1) != 0)) {
        const int Wl = b->segs[0].W;
        const unsigned grid = rbal ? rbal_grid : swk_bal_slots(Wl, b->pair_bytes, 0);
        uint32_t* fw = fault_word(b);
        if (!fw) return fail(b, SW_ERR_NOMEM, "fault word allocation failed");
        if (grid && (rbal || ntiles >= 2 * (size_t)grid)) {
          const size_t sw = (size_t)(grid + 1) * Wl * (2 * 32 + 2) * 64;
          HIPOK(b, b->bal_state.reserve(sw));
          if (b->bal_flag.cap < (size_t)(grid + 1) * Wl) {  // zeroed once: flags carry bal_gen
            HIPOK(b, b->bal_flag.reserve((size_t)(grid + 1) * Wl));
            HIPOK(b, hipMemsetAsync(b->bal_flag.p, 0, b->bal_flag.cap * 4, st));
          }
          if (!rbal) {  // uniform: workgroup g starts at chunk floor(g x tiles x K / grid)
            const size_t K = (max_len + 7) / 8;
            if (b->bal_key[0] != ntiles || b->bal_key[1] != K || b->bal_key[2] != grid) {
              HIPOK(b, b->bal_plan.reserve((size_t)(grid + 1) * 4));
              HIPOK(b, swk_bal_plan_uniform(b->bal_plan.p, (uint32_t)ntiles, (uint32_t)K, grid,
                                            st));
              b->bal_key[0] = ntiles;
              b->bal_key[1] = K;
              b->bal_key[2] = grid;
            }
          }
          // (A/B, SWBANK_RAGGED_GATHER=1) a ragged batch copied in its sorted order first, at a
          // 16-byte aligned stride (swk_deal_gather, one device), scored without the
          // permutation, each score written through it (ScoreArgs.sidx): a tile's targets are
          // then neighbours in memory (the codes' scatter).  =2: the copy in 4-bit
          // codes (SWK_PACK_NIBBLE), for alphabets of <= 16 codes
          const int gmode = rbal && ragged_trim() && packed == SWK_PACK_BYTES
                                ? env_int("SWBANK_RAGGED_GATHER", 0) : 0;
          const bool gat = gmode != 0;
          const bool gnib = gat && gmode == 2 && b->alpha <= 16;
          SwkDeal dl{};
          if (gat) {
            const size_t stride = ((gnib ? ((size_t)max_len + 7) / 8 * 4 : (size_t)max_len) + 15) &
                                  ~(size_t)15;
            HIPOK(b, b->gres.reserve(n * stride + 16));
            HIPOK(b, b->goffs.reserve(n));
            HIPOK(b, b->glens.reserve(n));
            dl.D = 1;
            dl.stride = (unsigned)stride;
            dl.codes[0] = b->gres.p;
            dl.offs[0] = reinterpret_cast<unsigned long long*>(b->goffs.p);
            dl.lens[0] = b->glens.p;
            dl.cnt[0] = n;
            dl.nib = gnib ? 1u : 0u;
            HIPOK(b, swk_deal_gather(res, offs, lens, idx, ident, n, &dl, st));
          }
          HIPOK(b, swk_launch_pair_bal(gat ? b->gres.p : res, gat ? b->goffs.p : offs,
                                       gat ? b->glens.p : lens, np, b->qpair.p, b->nv16, b->S, b->O,
                                       b->E, b->pair_bytes, b->pad, Wl,
                                       scores, b->pS1, b->pS2, ulen,
                                       ustride, b->bal_flag.p, b->bal_state.p, ++b->bal_gen, grid,
                                       gat ? nullptr : idx, gat ? nullptr : nidx,
                                       ident, b->bal_plan.p,
                                       fw + (b->host_call ? SWK_FAULT_WORDS : 0), poll_limit(1u << 23),
                                       (uint32_t)std::max(0, env_int("SWBANK_STALL", 0)),
                                       rbal && ragged_trim(),
                                       gnib ? (uint32_t)SWK_PACK_NIBBLE
                                            : gat ? (uint32_t)SWK_PACK_BYTES : packed,
                                       gat ? idx : nullptr, st));
          ++b->ctr.balanced_calls;
          const size_t L = strlen(b->last_kernel);
          snprintf(b->last_kernel + L, sizeof(b->last_kernel) - L, " balanced grid=%u%s", grid,
                   gnib ? " gather4" : gat ? " gather" : "");
          continue;
        }
      }
      for (size_t s = 0; s < nseg; ++s) {
        const void* ein = s > 0 ? b->edge[(s - 1) & 1].p : nullptr;
        void* eout = s + 1 < nseg ? b->edge[s & 1].p : nullptr;
        const bool pair = f16 && use_pair;
        int R = b->R, Wl = b->segs[s].W;
        u16_gotoh_rows(b, f16, R, Wl);
        HIPOK(b, swk_launch_score(R, b->RB, b->col0, b->prof, gotoh ? 1 : 0, f16 ? 1 : 0, res,
                                  offs, lens, np,
                                  pair ? b->qpair.p + s * (b->pair_bytes / 4)
                                  : f16 ? b->qtab16.p + b->segs[s].off16
                                        : b->qtab.p + b->segs[s].off,
                                  f16 ? b->nv16 : b->nv, b->S, b->O, b->E,
                                  pair ? b->pair_bytes : f16 && b->prof ? b->PS16 : b->PS,
                                  b->pad, Wl, scores, ein, eout, ecols, s > 0 ? 1 : 0,
                                  (int)packed, idx, nidx, (uint32_t)p0,
                                  pass == 0 ? ident : nullptr, pair ? 1 : 0, b->pS1, b->pS2,
                                  ulen, ustride, 1u, 0u, 0, st));
      }
    }
  }
  if (need32) {  // pairs above the 16-bit lanes' exact range -> int32 re-score
    const uint32_t scols = std::max(max_len, 1u);
    const size_t budget = (size_t)std::max(1, env_int("SWBANK_EDGE_MB", 2048)) << 20;
    const size_t waves = swk_i32_waves(n, scols, budget);
    HIPOK(b, b->fb_idx.reserve(n));
    HIPOK(b, b->fb_cnt.reserve(1));
    HIPOK(b, b->i32scr.reserve(waves * 2 * scols));
    // SWBANK_I32=1 (tests): every pair through the int32 kernel
    const int32_t thresh = bound > 65535u ? 65535 - std::max(0, b->smax) : -1;
    HIPOK(b, swk_flag_high(d_scores, n, thresh, b->fb_idx.p, b->fb_cnt.p, st));
    HIPOK(b, swk_launch_i32(gotoh ? 1 : 0, d_res, d_offs, d_lens, n, (int)packed, b->fb_idx.p,
                            b->fb_cnt.p, 0, b->i32prof.p, b->i32_strips,
                            (uint32_t)b->query.size(), b->pad, b->O, b->E, d_scores, b->i32scr.p,
                            scols, waves, st));
    const size_t L = strlen(b->last_kernel);
    snprintf(b->last_kernel + L, sizeof(b->last_kernel) - L, " +i32-rescore");
  }
  HIPOK(b, hipEventRecord(b->ev_used, st));  // the next table upload waits for this
  if (b->timing) {
    HIPOK(b, hipEventRecord(ev.c, st));
    b->events.push_back(ev);
  }
  return SW_OK;
}

// Record the batch best hit on the device (sw_batch_best reads it after best_ev).
sw_status track_best_device(sw_bank* b, const int32_t* d_scores, const uint64_t* d_ids, size_t n,
                            hipStream_t st) {
  if (n > 0xFFFFFFFFull) return SW_OK;  // the key holds a 32-bit index: not tracked
  HIPOK(b, b->best_key.reserve(1));
  HIPOK(b, b->best_dev.reserve(3));
  HIPOK(b, swk_best_hit(d_scores, d_ids, n, b->best_key.p, b->best_dev.p, b->best_dev.p + 2, st));
  if (!b->best_ev) HIPOK(b, hipEventCreateWithFlags(&b->best_ev, hipEventDisableTiming));
  HIPOK(b, hipEventRecord(b->best_ev, st));
  b->best_kind = 2;
  return SW_OK;
}

// A device batch against every query of a set (sw_load_queries): d_scores[q * n + k].  The
// tile kernel's several-queries variant takes the whole set in one launch per query segment
// (units = (query, tile) pairs, so every workgroup streams many tiles and the pipeline fills
// once); row-LUT tables only, exact 16-bit arithmetic.  Otherwise (profiles, the column-0 rule,
// optimistic f16, int32 re-scores, a wave-kernel shape; SWBANK_MQ=0) the queries run one after
// the other through launch().
sw_status launch_set(sw_bank* b, const uint8_t* d_res, const uint64_t* d_offs,
                     const uint32_t* d_lens, size_t n, uint32_t min_len, uint32_t max_len,
                     int32_t* d_scores, hipStream_t st, size_t sstride) {
  const size_t nq = b->qset.size();
  const uint64_t smax = (uint64_t)std::max(0, b->smax);
  const uint64_t top = std::min<uint64_t>(b->query.size(), max_len) * smax + smax;
  const bool f16_ok = b->f16 && b->f16_neg >= -2048 && env_int("SWBANK_F16", 1) != 0;
  const bool use_f16 = f16_ok && top <= 2048u;
  const bool exact = use_f16 || top <= 65535u;
  const size_t ntiles = (n + SWB_TILE - 1) / SWB_TILE;
  const char* kforce = std::getenv("SWBANK_KERNEL");
  const bool mq = env_int("SWBANK_MQ", 1) != 0 && !b->prof && !b->col0 && exact &&
                  env_int("SWBANK_I32", 0) == 0 && (b->R == 16 || b->R == 32) && b->RB == 4 &&
                  n <= 0xFFFFFFFFull &&
                  !(kforce && std::strcmp(kforce, "wave") == 0) && ntiles * nq <= 0x7FFFFFFFull;
  if (!mq) {  // one query at a time (each prepare()d in turn), then the set's layout again
    const std::vector<uint8_t> longest = b->query;
    sw_status rs = SW_OK;
    for (size_t i = 0; i < nq && rs == SW_OK; ++i) {
      b->query = b->qset[i];
      b->dirty = true;
      rs = prepare(b);
      if (rs == SW_OK)
        rs = launch(b, d_res, d_offs, d_lens, n, max_len, d_scores + i * sstride, st, SWK_PACK_BYTES,
                    nullptr, nullptr, true, true, nullptr, nullptr, 0, 0, min_len);
    }
    b->query = longest;
    b->dirty = true;
    const size_t L = strlen(b->last_kernel);
    snprintf(b->last_kernel + L, sizeof(b->last_kernel) - L, " x%zu queries", nq);
    return rs;
  }
  sw_status rs = prepare_multi(b);
  if (rs != SW_OK) return rs;
  const bool gotoh = b->gotoh();
  // pair tables (5.5 instead of 6.5 VALU per row) when the set has them, the batch is f16-exact
  // and a grid that is a multiple of nq (one query per workgroup) loses at most 1/8 of the
  // resident slots
  // (resident workgroups: 4 per CU for 128-row tables, 2 for 256-row, 1 for the 16-wave
  // 512-row ones)
  const int prow = std::max(b->mq_pair_rows, 32);
  const size_t slots = (prow > 256 ? 1 : prow > 128 ? 2 : 4) * (size_t)std::max(b->cus, 1);
  const bool mpair = b->mq_pair_segs > 0 && use_f16 && nq <= slots &&
                     8 * (slots - slots / nq * nq) <= slots;
  const size_t nseg = mpair ? (size_t)b->mq_pair_segs : b->segs.size();
  snprintf(b->last_kernel, sizeof(b->last_kernel), "tile %s%s R=%d W=%d segs=%zu queries=%zu",
           use_f16 ? "f16" : "u16", mpair ? " pair" : "", b->R,
           mpair ? std::min(prow / 32, (int)(b->query.size() + 31) / 32) : b->segs[0].W, nseg,
           nq);
  HIPOK(b, hipStreamWaitEvent(st, b->ev_ready, 0));  // the query tables are uploaded
  HIPOK(b, hipStreamWaitEvent(st, b->ev_used, 0));   // bank scratch is free
  sw_bank::Ev ev{};
  if (b->timing) {  // (an empty "pack" interval: b = a)
    HIPOK(b, hipEventCreate(&ev.a));
    HIPOK(b, hipEventCreate(&ev.c));
    HIPOK(b, hipEventRecord(ev.a, st));
    ev.b = ev.a;
  }
  const uint32_t ecols = (max_len + 7) / 8 * 8;
  // longest-first order of a ragged batch (shared by every query)
  const uint32_t *perm = nullptr, *perm_n = nullptr, *ident = nullptr;
  if (ntiles > 1 && !one_len_bin(min_len, max_len) && env_int("SWBANK_DSORT", 1) != 0) {
    HIPOK(b, b->dperm.reserve(n + 2));
    const size_t sw = swk_sort_scratch_bytes() / 4;
    if (b->dsort.cap < sw) {
      HIPOK(b, b->dsort.reserve(sw));
      HIPOK(b, hipMemsetAsync(b->dsort.p, 0, sw * 4, st));
    }
    HIPOK(b, swk_sort_lens(d_lens, n, max_len, b->dperm.p, b->dperm.p + n, b->dperm.p + n + 1,
                           b->dsort.p, st));
    ++b->ctr.device_sorts;
    perm = b->dperm.p;
    perm_n = b->dperm.p + n;
    ident = b->dperm.p + n + 1;
  }
  // edge rows per (query, tile) unit; past SWBANK_EDGE_MB the batch runs as position ranges
  size_t span = n;
  if (nseg > 1) {
    const size_t budget = (size_t)std::max(1, env_int("SWBANK_EDGE_MB", 2048)) << 20;
    const size_t per_tile = (size_t)ecols * 64 * sizeof(uint2) * nq;
    span = std::min(n, std::max<size_t>(1, budget / per_tile) * SWB_TILE);
    const size_t words = (span + SWB_TILE - 1) / SWB_TILE * ecols * 64 * nq;
    HIPOK(b, b->edge[0].reserve(words));
    HIPOK(b, b->edge[1].reserve(words));
  }
  const uint32_t* tabs = use_f16 ? b->mqtab16.p : b->mqtab.p;
  for (size_t p0 = 0; p0 < n; p0 += span) {
    const size_t np = std::min(span, n - p0);
    // with the order: whole arrays through it; else this range's slice
    const uint64_t* offs = perm ? d_offs : d_offs + p0;
    const uint32_t* lens = perm ? d_lens : d_lens + p0;
    int32_t* scores = perm ? d_scores : d_scores + p0;
    for (size_t sg = 0; sg < nseg; ++sg) {
      const void* ein = sg > 0 ? b->edge[(sg - 1) & 1].p : nullptr;
      void* eout = sg + 1 < nseg ? b->edge[sg & 1].p : nullptr;
      if (mpair) {  // prow-row segments, waves of 32 rows (fewer for a short last one)
        const int rows = std::min(prow, (int)b->query.size() - (int)sg * prow);
        const int Wp = std::max(1, (rows + 31) / 32);
        HIPOK(b, swk_launch_score(32, 4, 0, 0, 0, 1, d_res, offs, lens, np,
                                  b->mqpair.p + sg * nq * b->mq_pair_words, b->nv16, b->S, b->O,
                                  b->E, (uint32_t)b->mq_pair_words * 4, b->pad, Wp, scores, ein,
                                  eout, ecols, sg > 0 ? 1 : 0, (int)SWK_PACK_BYTES,
                                  perm ? perm + p0 : nullptr, perm_n, (uint32_t)p0, ident, 1,
                                  b->mq_pS1, b->mq_pS2, 0, 0, (uint32_t)nq,
                                  (uint32_t)b->mq_pair_words, sstride, st));
        continue;
      }
      HIPOK(b, swk_launch_score(b->R, b->RB, 0, 0, gotoh ? 1 : 0, use_f16 ? 1 : 0, d_res, offs,
                                lens, np, tabs + b->segs[sg].off, use_f16 ? b->nv16 : b->nv,
                                b->S, b->O, b->E, 0, b->pad, b->segs[sg].W, scores, ein, eout,
                                ecols, sg > 0 ? 1 : 0, (int)SWK_PACK_BYTES,
                                perm ? perm + p0 : nullptr, perm_n, (uint32_t)p0, ident, 0, 0, 0,
                                0, 0, (uint32_t)nq, (uint32_t)b->mq_words, sstride, st));
    }
  }
  HIPOK(b, hipEventRecord(b->ev_used, st));
  if (b->timing) {
    HIPOK(b, hipEventRecord(ev.c, st));
    b->events.push_back(ev);
  }
  return SW_OK;
}

extern "C" sw_status sw_score_batch_device(sw_bank* b, const uint8_t* d_res,
                                           const uint64_t* d_offs, const uint32_t* d_lens,
                                           const uint64_t* d_ids, size_t n, uint32_t max_len,
                                           int32_t* d_scores, void* stream) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  return sw_score_batch_device_range(b, d_res, d_offs, d_lens, d_ids, n, 0, max_len, d_scores,
                                     stream);
}

extern "C" sw_status sw_score_batch_device_range(sw_bank* b, const uint8_t* d_res,
                                                 const uint64_t* d_offs, const uint32_t* d_lens,
                                                 const uint64_t* d_ids, size_t n,
                                                 uint32_t min_len, uint32_t max_len,
                                                 int32_t* d_scores, void* stream) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (!b) return SW_ERR_ARG;
  if (min_len > max_len) return fail(b, SW_ERR_ARG, "min_len %u > max_len %u", min_len, max_len);
  b->best_kind = 0;
  b->best_root = false;
  // a hand-off fault latched by an earlier device call is returned before anything is scored
  if (const sw_status fs = take_fault(b, 0); fs != SW_OK) return fs;
  if (n == 0) return SW_OK;
  if (!d_res || !d_offs || !d_lens || !d_scores) return fail(b, SW_ERR_ARG, "null device buffer");
  if (b->is_multi()) {
    if (b->qset.size() > 1 && d_ids) return fail(b, SW_ERR_UNSUPPORTED, "best hit over a query set");
    return multi_device(b, d_res, d_offs, d_lens, d_ids, n, min_len, max_len, d_scores,
                        reinterpret_cast<hipStream_t>(stream), false);
  }
  sw_status st = prepare(b);
  if (st != SW_OK) return st;
  HIPOK(b, hipSetDevice(b->device));
  hipStream_t hs = stream ? reinterpret_cast<hipStream_t>(stream) : b->stream;
  if (b->qset.size() > 1) {  // a query set: nq x n scores; the best hit is not tracked
    if (d_ids) return fail(b, SW_ERR_UNSUPPORTED, "best hit over a query set");
    return launch_set(b, d_res, d_offs, d_lens, n, min_len, max_len, d_scores, hs, n);
  }
  if ((st = launch(b, d_res, d_offs, d_lens, n, max_len, d_scores, hs, SWK_PACK_BYTES, nullptr,
                   nullptr, true, true, nullptr, nullptr, 0, 0, min_len)) != SW_OK)
    return st;
  return d_ids ? track_best_device(b, d_scores, d_ids, n, hs) : SW_OK;
}

extern "C" sw_status sw_batch_best(sw_bank* b, uint64_t* best_id, int32_t* best_score,
                                   uint64_t* best_index) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (!b) return SW_ERR_ARG;
  if (b->is_multi() && b->best_root) {
    // the root tracked it after the scatter, which waited for every device's work: once it is
    // in, every device's hand-off faults of the call are visible too
    const sw_status st = sw_batch_best(b->kids[0], best_id, best_score, best_index);
    if (st != SW_OK) return fail(b, st, "device %d: %s", b->kids[0]->device, b->kids[0]->err);
    if (const sw_status fs = take_fault(b, 0); fs != SW_OK) {
      b->kids[0]->best_kind = 0;
      return fs;
    }
    return SW_OK;
  }
  if (b->best_kind == 2) {
    uint64_t h[3];
    HIPOK(b, hipSetDevice(b->device));
    HIPOK(b, hipEventSynchronize(b->best_ev));
    if (const sw_status fs = take_fault(b, 0); fs != SW_OK) {  // the call's scores are invalid
      b->best_kind = 0;
      return fs;
    }
    HIPOK(b, hipMemcpy(h, b->best_dev.p, sizeof(h), hipMemcpyDeviceToHost));
    b->best_id = h[0];
    b->best_score = (int32_t)(int64_t)h[1];
    b->best_index = h[2];
    b->best_kind = 1;
  }
  if (b->best_kind != 1)
    return fail(b, SW_ERR_STATE, "no best hit recorded (empty batch, or a device call without ids)");
  if (best_id) *best_id = b->best_id;
  if (best_score) *best_score = b->best_score;
  if (best_index) *best_index = b->best_index;
  return SW_OK;
}

