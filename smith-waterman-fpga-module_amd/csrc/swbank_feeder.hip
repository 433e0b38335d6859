// swbank_feeder.hip — the host-buffer API (sw_score_batch, sw_score_records): a pipelined feeder.
// 
// The reference host hands the accelerator host buffers (main_test.c:297-370 builds the WED and
// sequence_t arrays in host memory); the RTL feeder streams each target LEN codes long
// (ScoreBank/SM_Feeder3.v:135-140,184-196).
#include "swbank_bank.h"

// ---- host-buffer batches: a pipelined feeder ----------------------------------------------
// The reference host hands the accelerator host buffers (main_test.c:297-370 builds the WED
// and sequence_t arrays in host memory).  A host batch is put in longest-first feed order,
// cut into chunks and fed through NSLOT pinned staging slots: host threads gather chunk i
// (code validation fused into the copy) while chunk i-1 crosses PCIe on the copy stream and
// chunk i-2 is scored on the bank stream.
unsigned host_threads() {
  const int t = env_int("SWBANK_HOST_THREADS", 0);
  if (t > 0) return (unsigned)std::min(t, 64);
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const int omp = env_int("OMP_NUM_THREADS", 0);
  return std::min(hw, omp > 0 ? (unsigned)std::min(omp, 16) : 8u);
}

// Longest-first visiting order of a chunk (the PrioEncoder feed order, ScoreBank_v2.v:142-148:
// each 128-target tile then holds similar lengths): false when the lengths are already
// non-increasing (no permutation needed), else perm[] = a stable counting sort over the
// length range (parallel over the pool's parts when the range is small), or a stable
// comparison sort when the range is wide.
bool chunk_perm(HostPool& pool, const uint32_t* len, size_t n, uint32_t* perm) {
  const unsigned T = n >= 8192 ? pool.size() : 1;
  const size_t step = (n + T - 1) / T;
  std::vector<uint32_t> plo(T, UINT32_MAX), phi(T, 0);
  std::vector<char> pinc(T, 1);
  const auto scan = [&](unsigned p) {
    const size_t a = std::min(n, p * step), e = std::min(n, a + step);
    uint32_t lo = UINT32_MAX, hi = 0, prev = a > 0 ? len[a - 1] : UINT32_MAX;
    bool inc = true;
    for (size_t k = a; k < e; ++k) {
      const uint32_t l = len[k];
      lo = std::min(lo, l);
      hi = std::max(hi, l);
      inc &= l <= prev;
      prev = l;
    }
    plo[p] = lo;
    phi[p] = hi;
    pinc[p] = inc;
  };
  if (T > 1) pool.run(scan); else scan(0);
  const uint32_t lo = *std::min_element(plo.begin(), plo.end());
  const uint32_t hi = *std::max_element(phi.begin(), phi.end());
  if (std::all_of(pinc.begin(), pinc.end(), [](char c) { return c != 0; })) return false;
  const size_t range = (size_t)hi - lo + 1;
  if (range <= 65536 && range <= 4 * n + 4096) {
    // per-part histograms of bucket hi - l (longest first), then each part scatters at the
    // prefix over (bucket, part): stable
    std::vector<uint32_t> h((size_t)T * range, 0);
    const auto count = [&](unsigned p) {
      uint32_t* hp = h.data() + (size_t)p * range;
      const size_t a = std::min(n, p * step), e = std::min(n, a + step);
      for (size_t k = a; k < e; ++k) ++hp[hi - len[k]];
    };
    if (T > 1) pool.run(count); else count(0);
    uint32_t acc = 0;
    for (size_t bkt = 0; bkt < range; ++bkt)
      for (unsigned p = 0; p < T; ++p) {
        const uint32_t c = h[(size_t)p * range + bkt];
        h[(size_t)p * range + bkt] = acc;
        acc += c;
      }
    const auto place = [&](unsigned p) {
      uint32_t* hp = h.data() + (size_t)p * range;
      const size_t a = std::min(n, p * step), e = std::min(n, a + step);
      for (size_t k = a; k < e; ++k) perm[hp[hi - len[k]]++] = (uint32_t)k;
    };
    if (T > 1) pool.run(place); else place(0);
  } else {
    std::iota(perm, perm + n, 0u);
    std::stable_sort(perm, perm + n, [&](uint32_t a, uint32_t c) { return len[a] > len[c]; });
  }
  return true;
}

// chunk target: an eighth of the batch (so gather, copy and score overlap), 8-256 MiB
// (measured on the headline batch: 16-18 MiB chunks 4.5-5.0 ms, 35 MiB 5.1-5.2 ms)
static size_t chunk_target(size_t total) {
  const int mb = env_int("SWBANK_CHUNK_MB", 0);
  if (mb > 0) return (size_t)mb << 20;
  return std::min<size_t>((size_t)256 << 20, std::max<size_t>((size_t)8 << 20, total / 8));
}

// Cumulative chunk boundaries (in input bytes) of a host batch: the first chunk a quarter of
// chunk_target() (at least 1 MiB) so the GPU starts early, then doubling up to chunk_target()
// (SWBANK_CHUNK_MB: fixed size).  Boundaries strictly inside (0, total).  min_bytes: no chunk
// smaller (the last one included), unless SWBANK_CHUNK_MB is set.
static std::vector<size_t> chunk_bounds(size_t total, size_t min_bytes = 0) {
  std::vector<size_t> bounds;
  const bool fixed = env_int("SWBANK_CHUNK_MB", 0) > 0;
  if (fixed) min_bytes = 0;
  const size_t cap = std::max(chunk_target(total), min_bytes);
  size_t sz = fixed ? cap : std::max<size_t>({(size_t)1 << 20, cap / 4, min_bytes});
  for (size_t at = sz; at < total && total - at >= min_bytes; at += sz, sz = std::min(cap, sz * 2))
    bounds.push_back(at);
  // A remainder below min_bytes stays with the last chunk, which can then pass the cap (up to
  // cap + min_bytes); such a last chunk is halved when both halves keep min_bytes, so
  // every chunk stays within max(cap, 2 min_bytes) -- and so do the slots sized to it.
  if (!bounds.empty()) {
    const size_t last = total - bounds.back();
    if (last > cap && last / 2 >= min_bytes) bounds.push_back(bounds.back() + last / 2);
  }
  return bounds;
}

static sw_status feeder_init(sw_bank* b) {
  HIPOK(b, hipSetDevice(b->device));
  if (!b->pool) b->pool.reset(new (std::nothrow) HostPool(b->pool_threads ? b->pool_threads
                                                                          : host_threads()));
  if (!b->pool) return fail(b, SW_ERR_NOMEM, "host worker pool");
  if (!b->launcher) b->launcher.reset(new (std::nothrow) Launcher(b->device));
  if (!b->launcher) return fail(b, SW_ERR_NOMEM, "feeder launch thread");
  if (b->ev_s2) return SW_OK;  // (the streams are the bank's, created with it)
  HIPOK(b, hipEventCreateWithFlags(&b->ev_s2, hipEventDisableTiming));
  for (int i = 0; i < sw_bank::NSLOT; ++i)
    HIPOK(b, hipEventCreateWithFlags(&b->h2d_done[i], hipEventDisableTiming));
  for (int i = 0; i < sw_bank::NDSLOT; ++i)
    HIPOK(b, hipEventCreateWithFlags(&b->kern_done[i], hipEventDisableTiming));
  return SW_OK;
}

// One chunk = input positions [c0, c1), staged as `bytes` bytes in slot c % NSLOT.
struct Chunk {
  size_t c0, c1, bytes;
};

// Runs the feeder: gather(slot, chunk, from) fills the host slot and returns how many leading
// bytes of it to copy, from byte `from` on (0: bad input, message set); they go to the device on the copy stream, score(dslot, chunk, d_scores) launches the
// kernel on the bank stream; the scores come back to the pinned hscores in input order.
// out != nullptr: every chunk's scores go back to the pinned hscores on out_stream right after
// its kernel (beside the next chunk's kernel on the bank stream) and are copied into out in
// input order as they land, the batch best hit (lowest index of the maximum) tracked in the same
// pass; out == nullptr: they stay in b->scores on the device, enqueued on b->stream (a
// multi-device bank gathers them).
// overlap: the chunks' launches use no bank scratch (scratch_free), so odd chunks run on
// stream2 and one launch's drain overlaps the next one's start.
template <class GatherF, class ScoreF>
static sw_status feed(sw_bank* b, size_t n, const std::vector<Chunk>& chunks, GatherF gather,
                      ScoreF score, int32_t* out, bool overlap) {
  sw_status st = feeder_init(b);
  if (st != SW_OK) return st;
  ++b->ctr.chunked_calls;
  size_t slot_bytes = 0;
  for (const Chunk& c : chunks) slot_bytes = std::max(slot_bytes, c.bytes);
  // device slots: NDSLOT while they take at most 1 GiB, else NSLOT
  const int nds = slot_bytes * sw_bank::NDSLOT <= ((size_t)1 << 30) ? sw_bank::NDSLOT
                                                                    : sw_bank::NSLOT;
  b->feed_dslots = nds;
  for (int i = 0; i < std::min<int>(sw_bank::NSLOT, (int)chunks.size()); ++i)
    HIPOK(b, b->hslot[i].reserve(slot_bytes));
  for (int i = 0; i < std::min<int>(nds, (int)chunks.size()); ++i)
    HIPOK(b, b->dslot[i].reserve(slot_bytes));
  HIPOK(b, b->scores.reserve(n));
  if (out) {
    HIPOK(b, b->hscores.reserve(n * 4));
    while (b->out_ev.size() < chunks.size()) {
      hipEvent_t e;
      HIPOK(b, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      b->out_ev.push_back(e);
    }
  }
  // (overlapped chunk launches run at full occupancy: with the launch thread and 6 device slots
  // they are paced by the gather and mostly run one at a time, and a half-chip kernel running
  // alone took ~220 us per 1/8 chunk against ~175 at full occupancy, measured in round 4)
  Launcher* lz = b->launcher.get();
  if (lz) lz->reset();
  const auto fail_sync = [&](sw_status s) {
    if (lz) lz->wait_all();
    (void)hipStreamSynchronize(b->stream);
    (void)hipStreamSynchronize(b->stream2);
    (void)hipStreamSynchronize(b->copy_stream);
    (void)hipStreamSynchronize(b->out_stream);
    return s;
  };
  // a HIP failure once jobs are posted: the launch thread may still hold jobs that reference
  // this frame (launch_chunk, chunks, the caller's gather state), so drain it before returning.
  // SWBANK_FEED_FAULT=k (a test hook) reports a failure at sync point k: chunk k's slot wait
  // (NSLOT <= k < chunks, jobs in flight), then the stream join, each chunk's result wait and
  // the final sync
  const int fault_at = env_int("SWBANK_FEED_FAULT", -1);
  const auto hip_sync = [&](hipError_t e, size_t i, const char* what) -> sw_status {
    if (e == hipSuccess && fault_at >= 0 && (size_t)fault_at == i) e = hipErrorLaunchFailure;
    if (e == hipSuccess) return SW_OK;
    return fail_sync(fail(b, SW_ERR_HIP, "%s (chunk %zu): %s", what, i, hipGetErrorString(e)));
  };
  PhaseTrace* tr = g_trace;
  // chunk i's HIP work: its copy once slot s is free, the score launches, the scores' return
  const auto launch_chunk = [&, tr](size_t i, size_t from, size_t bytes) -> sw_status {
    const int s = (int)(i % sw_bank::NSLOT), d = (int)(i % nds);
    const Chunk& c = chunks[i];
    if (i >= (size_t)nds) HIPOK(b, hipStreamWaitEvent(b->copy_stream, b->kern_done[d], 0));
    HIPOK(b, hipMemcpyAsync(b->dslot[d].p + from, b->hslot[s].p + from, bytes - from,
                            hipMemcpyHostToDevice, b->copy_stream));
    __atomic_fetch_add(&b->ctr.h2d_bytes, (uint64_t)(bytes - from), __ATOMIC_RELAXED);
    HIPOK(b, hipEventRecord(b->h2d_done[s], b->copy_stream));
    hipStream_t ks = overlap && (i & 1) ? b->stream2 : b->stream;
    HIPOK(b, hipStreamWaitEvent(ks, b->h2d_done[s], 0));
    const sw_status sst = score(b->dslot[d].p, c, b->scores.p + c.c0, ks);
    if (sst != SW_OK) return sst;
    if (tr) tr->mark("launched");
    HIPOK(b, hipEventRecord(b->kern_done[d], ks));
    if (out) {
      HIPOK(b, hipStreamWaitEvent(b->out_stream, b->kern_done[d], 0));
      HIPOK(b, hipMemcpyAsync(b->hscores.p + c.c0 * 4, b->scores.p + c.c0, (c.c1 - c.c0) * 4,
                              hipMemcpyDeviceToHost, b->out_stream));
      HIPOK(b, hipEventRecord(b->out_ev[i], b->out_stream));
    }
    return SW_OK;
  };
  for (size_t i = 0; i < chunks.size(); ++i) {
    const int s = (int)(i % sw_bank::NSLOT);
    const Chunk& c = chunks[i];
    if (i >= (size_t)sw_bank::NSLOT) {
      // slot s is free once chunk i - NSLOT's copy (enqueued by the launch thread) landed
      if (lz && (st = lz->wait(i - sw_bank::NSLOT + 1)) != SW_OK) return fail_sync(st);
      if ((st = hip_sync(hipEventSynchronize(b->h2d_done[s]), i, "slot wait")) != SW_OK)
        return st;
    }
    trace_mark("gather<");
    const auto t0 = std::chrono::steady_clock::now();
    size_t from = 0;  // leading slot bytes the device does not need (a uniform chunk's headers)
    const size_t bytes = gather(b->hslot[s].p, c, from);
    trace_mark("gather>");
    if (b->timing)
      b->host_pack_ms +=
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (bytes == 0) return fail_sync(SW_ERR_ARG);
    if (lz)
      lz->post([&launch_chunk, i, from, bytes] { return launch_chunk(i, from, bytes); });
    else if ((st = launch_chunk(i, from, bytes)) != SW_OK)
      return fail_sync(st);
  }
  if (lz && (st = lz->wait_all()) != SW_OK) return fail_sync(st);
  if (overlap) {  // the bank stream (the multi-device gather, the next call) after stream2
    if ((st = hip_sync(hipEventRecord(b->ev_s2, b->stream2), chunks.size(), "stream join")) !=
            SW_OK ||
        (st = hip_sync(hipStreamWaitEvent(b->stream, b->ev_s2, 0), chunks.size(),
                       "stream join")) != SW_OK)
      return st;
  }
  if (!out) return SW_OK;
  // scores into the caller's buffer as they land, with the best hit: per pool part the lowest
  // index of its maximum, then the lowest index among the parts' maxima
  const int32_t* hs = reinterpret_cast<const int32_t*>(b->hscores.p);
  const unsigned T = b->pool->size();
  std::vector<size_t> pbest(T);
  size_t best = 0;
  for (size_t i = 0; i < chunks.size(); ++i) {
    const Chunk& c = chunks[i];
    if ((st = hip_sync(hipEventSynchronize(b->out_ev[i]), chunks.size() + i, "scores wait")) !=
        SW_OK)
      return st;
    trace_mark("landed");
    const size_t cnt = c.c1 - c.c0;
    const unsigned parts = cnt >= 4096 ? T : 1;
    const size_t step = (cnt + parts - 1) / parts;
    std::fill(pbest.begin(), pbest.end(), SIZE_MAX);
    const auto part = [&](unsigned p) {
      const size_t lo = c.c0 + std::min(cnt, p * step), hi = c.c0 + std::min(cnt, (p + 1) * step);
      size_t bi = lo;
      for (size_t k = lo; k < hi; ++k) {
        const int32_t v = hs[k];
        out[k] = v;
        if (v > hs[bi]) bi = k;
      }
      if (lo < hi) pbest[p] = bi;
    };
    if (parts > 1) b->pool->run(part);
    else part(0);
    for (size_t x : pbest)  // parts and chunks in index order: strictly greater keeps the lowest
      if (x != SIZE_MAX && hs[x] > hs[best]) best = x;
  }
  b->best_index = best;
  b->best_id = best;
  b->best_score = hs[best];
  b->best_kind = 1;
  if ((st = hip_sync(hipStreamSynchronize(b->stream), 2 * chunks.size(), "final sync")) != SW_OK)
    return st;
  trace_mark("done");
  return SW_OK;
}


// Chunk slot tail shared by both host paths: lens u32 x cnt | perm u32 x cnt | count u32.
struct SlotTail {
  size_t lens_at, perm_at, cnt_at;
};
static SlotTail slot_tail(size_t tail_at, size_t cnt) {
  return {tail_at, tail_at + cnt * 4, tail_at + cnt * 8};
}

// True when launches for targets of at most max_len use no bank scratch (one query segment,
// no optimistic f16 re-score list, no int32 re-score), so host-feeder chunks may run on two
// streams.  Mirrors launch()'s choices.
bool scratch_free(const sw_bank* b, uint32_t max_len) {
  const uint64_t s = (uint64_t)std::max(0, b->smax);
  const uint64_t top = std::min<uint64_t>(b->query.size(), max_len) * s + s;
  const bool need32 = top > 65535u || env_int("SWBANK_I32", 0) != 0;
  const bool f16_ok = b->f16 && b->f16_neg >= -2048 && env_int("SWBANK_F16", 1) != 0;
  const bool opt16 = f16_ok && top > 2048u;
  return b->segs.size() == 1 && b->wsegs == 1 && !need32 && !opt16;
}

// Pass 1: every target in 2-bit codes (offset word: its 2-bit position << 1, see
// SWK_PACK_MIXED) -- a part whose targets lie back to back in the residues as ONE run (one
// packer call per 16 Ki codes, the positions of codes past 3 reported), else one call per
// target.  A target with a code past 3 is packed again at once in 4-bit codes into the part's
// staging buffer (its residues still in cache: scattered re-reads later were latency bound).
// Pass 2: each part's staged 4-bit targets land as one block after the 2-bit region (their
// 2-bit bytes stay unused), offset words (byte << 1) | 1.  (Declared in swbank_bank.h.)
bool mixed_pack(sw_bank* b, const uint8_t* residues, size_t nres, const uint64_t* offsets,
                const uint32_t* lens, size_t c0, size_t cnt, size_t step,
                const std::vector<uint64_t>& rbase, const std::vector<uint64_t>& rspan,
                const std::vector<size_t>& psz, const std::vector<size_t>& part4, uint32_t* so32,
                uint32_t* sl32, uint8_t* mcodes, uint32_t* order, MixedOrder* mo, size_t& end) {
  HostPool& pool = *b->pool;
  const unsigned T = pool.size();
  const bool avx2 = env_int("SWBANK_AVX2", 1) != 0;
  const swpack::PackFn pack2fn = swpack::packer(2, avx2), pack4fn = swpack::packer(4, avx2);
  const swpack::PackRunFn runfn = swpack::run_packer(avx2);
  const uint32_t alpha = (uint32_t)b->alpha;
  // a target's last 32-code step may store past its end while it stays inside the part's output
  // (later targets of the part rewrite those bytes) and reads inside the residues
  const auto wide_ok = [&](size_t k, uint32_t l, size_t at, size_t step_bytes, size_t part_end) {
    const size_t steps = (l + 31u) / 32u;
    return offsets[k] + steps * 32 <= nres && at + steps * step_bytes <= part_end;
  };
  if (b->mlist.size() < T) b->mlist.resize(T);
  if (b->mstage.size() < T) b->mstage.resize(T);
  if (b->mbad.size() < T) b->mbad.resize(T);
  std::vector<size_t> r4(T + 1, 0);  // staged 4-bit bytes per part
  std::atomic<uint32_t> nruns{0}, wide{0};
  pool.run([&](unsigned p) {
    const size_t lo = std::min(cnt, p * step), hi = std::min(cnt, (p + 1) * step);
    // (list and stage live in this thread while they grow: the parts' vector headers share
    // cache lines)
    std::vector<uint32_t> nl, bad;
    std::vector<uint8_t> sg;
    nl.swap(b->mlist[p]);
    sg.swap(b->mstage[p]);
    bad.swap(b->mbad[p]);
    nl.clear();
    const size_t scap = part4[p + 1] - part4[p] + 64;
    if (sg.size() < scap) sg.resize(scap);
    size_t sat = 0;
    uint32_t mx = 0;
    uint32_t* opos = mo ? mo->pos.data() + (size_t)p * mo->nbin : nullptr;
    const auto place = [&](size_t i, uint32_t l) {  // (the fused counting sort's scatter)
      if (opos) order[opos[(mo->hi - std::min(l, mo->hi)) >> mo->shift]++] = (uint32_t)i;
    };
    const auto stage4 = [&](size_t i) {
      const size_t k = c0 + i;
      const uint32_t l = lens[k];
      mx = std::max(mx, pack4fn(residues + offsets[k], l, sg.data() + sat,
                                wide_ok(k, l, sat, 16, scap)));
      nl.push_back((uint32_t)i);
      sat += (l + 1) / 2;
    };
    if (rbase[p] != UINT64_MAX) {
      const uint64_t o0 = rbase[p], span = rspan[p];
      const uint64_t pos0 = 4 * (uint64_t)psz[p];  // the run's first 2-bit position
      for (size_t i = lo; i < hi; ++i) {
        const size_t k = c0 + i;
        const uint32_t l = lens[k];
        so32[i] = l ? (uint32_t)((pos0 + offsets[k] - o0) << 1) : 0u;
        sl32[i] = l;
        place(i, l);
      }
      // 16 Ki codes per packer call: the N targets of a block are re-packed while its
      // residues are in cache; `cur` walks the targets (ascending, non-overlapping)
      size_t cur = lo, marked = SIZE_MAX;
      for (uint64_t x0 = 0; x0 < span; x0 += 16384) {
        const uint64_t x1 = std::min<uint64_t>(span, x0 + 16384);
        bad.clear();
        runfn(residues + o0 + x0, (size_t)(x1 - x0), mcodes + psz[p] + x0 / 4, (uint32_t)x0, bad);
        for (const uint32_t x : bad) {
          const uint64_t r = o0 + x;
          while (cur < hi &&
                 (lens[c0 + cur] == 0 || offsets[c0 + cur] + lens[c0 + cur] <= r))
            ++cur;
          if (cur >= hi) break;
          if (offsets[c0 + cur] > r || cur == marked) continue;  // a gap; done already
          stage4(cur);
          marked = cur;
        }
      }
      ++nruns;
    } else {
      size_t at = psz[p];
      for (size_t i = lo; i < hi; ++i) {
        const size_t k = c0 + i;
        const uint32_t l = lens[k];
        if (pack2fn(residues + offsets[k], l, mcodes + at, wide_ok(k, l, at, 8, psz[p + 1])) > 3u)
          stage4(i);
        so32[i] = (uint32_t)(at << 3);
        sl32[i] = l;
        place(i, l);
        at += (l + 3) / 4;
      }
    }
    b->mlist[p].swap(nl);
    b->mstage[p].swap(sg);
    b->mbad[p].swap(bad);
    r4[p + 1] = sat;
    if (mx >= alpha) wide = 1;  // a code outside the alphabet
  });
  if (wide.load() != 0) return false;
  for (unsigned p = 0; p < T; ++p) r4[p + 1] += r4[p];
  const size_t b4 = psz[T];  // the 4-bit region, right after the 2-bit one
  trace_mark("g-mixed2");
  if (r4[T]) {
    pool.run([&](unsigned p) {
      const size_t base = b4 + r4[p];
      std::memcpy(mcodes + base, b->mstage[p].data(), r4[p + 1] - r4[p]);
      size_t sat = 0;
      for (const uint32_t i : b->mlist[p]) {
        so32[i] = (uint32_t)((base + sat) << 1) | 1u;
        sat += (lens[c0 + i] + 1) / 2;
      }
    });
  }
  trace_mark("g-mixed4");
  b->ctr.mixed_runs += nruns.load();
  end = b4 + r4[T];
  std::memset(mcodes + end, 0, 16);  // a last target's chunk reads up to 3 bytes past
  return true;
}

// A host-buffer call `run` (its launches complete when it returns) with the hand-off fault
// check: a wait that ran out in one of its launches (fault word [1]) re-runs the call once
// without hand-offs (neither balanced ranges nor the segmented protein tail: every dependency
// inside a workgroup), which returns SW_ERR_TIMEOUT only if it faults too.
template <class F>
static sw_status with_fault_check(sw_bank* b, F&& run) {
  struct Scope {
    sw_bank* b;
    ~Scope() { b->host_call = b->no_handoff = false; }
  } scope{b};
  b->host_call = true;
  sw_status st = run();
  const sw_status fs = take_fault(b, 1);
  if (st != SW_OK || fs == SW_OK) return st;
  ++b->ctr.handoff_reruns;
  b->no_handoff = true;
  st = run();
  const sw_status fs2 = take_fault(b, 1);
  return st != SW_OK ? st : fs2;
}

static sw_status batch_feed_once(sw_bank* b, const uint8_t* residues, size_t nres,
                                 const uint64_t* offsets, const uint32_t* lens, size_t n,
                                 int32_t* out);

// The host-buffer batch through the feeder (n >= 1, buffers checked by the caller).
sw_status batch_feed(sw_bank* b, const uint8_t* residues, size_t nres, const uint64_t* offsets,
                     const uint32_t* lens, size_t n, int32_t* out) {
  return with_fault_check(b, [&] { return batch_feed_once(b, residues, nres, offsets, lens, n, out); });
}

static sw_status batch_feed_once(sw_bank* b, const uint8_t* residues, size_t nres,
                                 const uint64_t* offsets, const uint32_t* lens, size_t n,
                                 int32_t* out) {
  sw_status st = prepare(b);
  if (st != SW_OK) return st;
  if ((st = feeder_init(b)) != SW_OK) return st;

  // Two passes over the lengths on the pool (inline for small batches): total and longest,
  // then the chunk cuts in input order, after target k when the running code count crosses a
  // multiple of chunk_target().
  HostPool& pool = *b->pool;
  const unsigned T = pool.size();
  const unsigned P = n >= 65536 ? T : 1;
  // parts of whole 1024-target blocks: the pass also keeps each block's code count, from which
  // the chunk cuts below are found without a second pass over the lengths
  constexpr size_t CB = 1024;
  const size_t pstep = ((n + P - 1) / P + CB - 1) / CB * CB;
  const size_t nblk = (n + CB - 1) / CB;
  std::vector<size_t> cpre(nblk + 1, 0);  // block code counts, then their exclusive prefix
  const auto run_parts = [&](const std::function<void(unsigned)>& f) {
    if (P > 1) pool.run(f);
    else f(0u);
  };
  std::vector<size_t> psum(P + 1, 0);
  std::vector<uint32_t> pmax(P, 0), pmin(P, UINT32_MAX);
  run_parts([&](unsigned p) {
    size_t acc = 0;
    uint32_t m = 0, mn = UINT32_MAX;
    const size_t e = std::min(n, (p + 1) * pstep);
    for (size_t b0 = std::min(n, p * pstep); b0 < e; b0 += CB) {
      size_t bs = 0;
      for (size_t k = b0; k < std::min(e, b0 + CB); ++k) {
        bs += lens[k];
        m = std::max(m, lens[k]);
        mn = std::min(mn, lens[k]);
      }
      cpre[b0 / CB + 1] = bs;
      acc += bs;
    }
    psum[p + 1] = acc;
    pmax[p] = m;
    pmin[p] = mn;
  });
  for (unsigned p = 0; p < P; ++p) psum[p + 1] += psum[p];
  trace_mark("lens-pass");
  const size_t total = psum[P];
  const uint32_t max_len = *std::max_element(pmax.begin(), pmax.end());
  if (max_len && !residues) return fail(b, SW_ERR_ARG, "null residues");
  // equal-length DNA batches: one streamed kernel for the whole call (stream_feed)
  if (max_len && *std::min_element(pmin.begin(), pmin.end()) == max_len) {
    bool used = false;
    st = stream_feed(b, residues, nres, offsets, n, max_len, out, used);
    if (used) return st;
  } else if (max_len && env_int("SWBANK_STREAM_RAGGED", 0) != 0) {
    // ragged streamed (opt-in): exact, but slower than the chunked feeder on the ragged
    // bench shape (host-side order per chunk on the gather's critical path; LEDGER §3.3)
    bool used = false;
    st = stream_feed(b, residues, nres, offsets, n, max_len, out, used, nullptr, lens);
    if (used) return st;
  }
  // slot: offsets u64 | lens | perm | count | ident (SlotTail) | codes at codes_at(cnt): one byte per
  // residue, or, for a DNA chunk without N, the 2-bit stream (a quarter of the PCIe bytes;
  // SWBANK_PACK2=0 disables), each target from a byte boundary, 16 zero bytes after the last
  const auto codes_at = [](size_t cnt) { return align16(cnt * 16 + 8); };
  // A batch for the wave kernel: every launch holds at least one unit per resident wave slot (a
  // launch of fewer units leaves SIMDs idle for a whole unit's time: configs[4]'s 12,500
  // targets in 2 + 4 + 6.5 MB chunks took 1.63 ms through this path, in one chunk 1.22 ms,
  // the kernel alone 0.81)
  size_t min_chunk = 0;
  if (max_len && wave_preferred(b, n, max_len, b->f16 && b->f16_neg >= -2048 &&
                                                   env_int("SWBANK_F16", 1) != 0)) {
    const unsigned grid = swk_wave_half_grid(b->gotoh() ? 1 : 0, (b->pad + 1) * b->wPS16, 4);
    min_chunk = (size_t)(grid ? grid : 1024) * 16 * max_len;  // 4 waves x 2 pairs x 2 targets
    min_chunk = std::min(min_chunk, (size_t)256 << 20);          // (chunk_target's cap)
  }
  std::vector<size_t> bounds = chunk_bounds(total, min_chunk);
  bounds.push_back(SIZE_MAX);  // sentinel
  for (size_t i = 0; i < nblk; ++i) cpre[i + 1] += cpre[i];
  std::vector<Chunk> chunks;
  size_t c0 = 0, a0 = 0;
  const auto add_chunk = [&](size_t c1, size_t a1) {
    chunks.push_back({c0, c1, codes_at(c1 - c0) + align16(a1 - a0 + 16)});
    c0 = c1;
    a0 = a1;
  };
  // a cut after target k when the running code count reaches the next boundary (several
  // boundaries inside one target make one cut): the block where the count crosses it (the block
  // prefix), then a scan of that block only
  for (size_t j = 0, blk = 0; bounds[j] <= total;) {
    const size_t B = bounds[j];
    while (blk + 1 < nblk && cpre[blk + 1] < B) ++blk;
    size_t acc = cpre[blk], k = blk * CB;
    for (; k < n; ++k)
      if ((acc += lens[k]) >= B) break;
    if (k >= n) break;  // (not reached: B <= total)
    while (bounds[j] <= acc) ++j;
    if (k + 1 < n) add_chunk(k + 1, acc);
  }
  trace_mark("cuts");
  add_chunk(n, total);
  std::vector<uint32_t> chunk_max(chunks.size(), 0);  // set by the chunk's gather
  const uint32_t alpha = (uint32_t)b->alpha;
  // DNA: the 2-bit stream while the chunks hold no N; from the first chunk with N on, the
  // 4-bit stream (2-bit attempts would be discarded packing passes where N is common)
  const bool dna_pack = b->alpha == SW_DNA_ALPHA && env_int("SWBANK_PACK2", 1) != 0;
  // AVX2 packers when the host has them (SWBANK_AVX2=0: the SSE2 forms); a target whose last
  // 32-code step has 32 readable bytes and whose full-step stores (8 or 16 bytes per step) end
  // inside its pool part's output packs its tail in the same vector step (swbank_pack.h): the
  // bytes it stores past its own end belong to later targets of the same part, which rewrite
  // them afterwards on the same thread
  const bool avx2 = env_int("SWBANK_AVX2", 1) != 0;
  const swpack::PackFn pack2fn = swpack::packer(2, avx2), pack4fn = swpack::packer(4, avx2);
  const auto wide_ok = [&](size_t k, uint32_t l, size_t at, size_t step_bytes, size_t part_end) {
    const size_t steps = (l + 31u) / 32u;
    return offsets[k] + steps * 32 <= nres && at + steps * step_bytes <= part_end;
  };
  bool pack2 = dna_pack;
  HIPOK(b, hipSetDevice(b->device));
  std::vector<char> has_perm(chunks.size(), 0);
  // ragged chunks: longest-first order sorted on the device (the sort kernels of
  // sw_score_batch_device, into the chunk's slot) instead of on the host; SWBANK_HOST_DSORT=0
  // sorts on the host
  std::vector<char> dev_sort(chunks.size(), 0);
  const bool host_dsort = env_int("SWBANK_HOST_DSORT", 1) != 0 && env_int("SWBANK_DSORT", 1) != 0;
  std::vector<uint32_t> chunk_mode(chunks.size(), SWK_PACK_BYTES);
  // equal-length chunks cross PCIe without the per-target offsets and lengths (the kernels
  // compute them: ScoreArgs.ulen / ustride) unless the int32 re-score would need them;
  // SWBANK_UNIFORM=0 always sends them
  std::vector<uint32_t> chunk_stride(chunks.size(), 0);
  const uint64_t smax0 = (uint64_t)std::max(0, b->smax);
  const bool uni_ok = env_int("SWBANK_UNIFORM", 1) != 0 && env_int("SWBANK_I32", 0) == 0 &&
                      std::min<uint64_t>(b->query.size(), max_len) * smax0 + smax0 <= 65535u;
  // Ragged DNA chunks cross as SWK_PACK_MIXED: every target in 2-bit codes from an even byte,
  // or in 4-bit codes from an odd byte when it holds an N, with u32 offsets (8 header bytes per
  // target instead of 16, and N costs 4 bits only in the targets that hold one); the tile
  // kernel reads it (launches that would take the wave kernel or the int32 re-score, and host
  // sorted chunks, keep the whole-chunk layouts).  SWBANK_MIXED=0 disables.
  const bool mixed_ok = dna_pack && env_int("SWBANK_MIXED", 1) != 0 &&
                        env_int("SWBANK_I32", 0) == 0 &&
                        std::min<uint64_t>(b->query.size(), max_len) * smax0 + smax0 <= 65535u;
  const bool f16_ok = b->f16 && b->f16_neg >= -2048 && env_int("SWBANK_F16", 1) != 0;
  std::vector<size_t> mperm(chunks.size(), 0);  // a mixed chunk's sort order (device only)
  std::vector<size_t> part(T + 1), part2(T + 1), part4(T + 1), psz(T + 1);
  std::vector<uint32_t> partmax(T), partmin(T);
  // mixed chunks: a part whose non-empty targets lie in ascending, non-overlapping order in the
  // residues with gaps of at most 1/8 of its codes packs as ONE run from rbase[p] (rspan codes,
  // gaps included); UINT64_MAX: one packer call per target.  SWBANK_MIXED_RUNS=0 disables.
  std::vector<uint64_t> rbase(T), rspan(T);
  const bool runs_ok = env_int("SWBANK_MIXED_RUNS", 1) != 0;
  std::atomic<size_t> bad{SIZE_MAX}, oob{SIZE_MAX};
  std::atomic<uint32_t> wide{0};
  size_t gi = 0, si = 0;
  const auto gather = [&](uint8_t* slot, const Chunk& c, size_t& from) -> size_t {
    const size_t cnt = c.c1 - c.c0, ca = codes_at(cnt);
    const SlotTail tl = slot_tail(cnt * 8, cnt);
    uint64_t* so = reinterpret_cast<uint64_t*>(slot);
    uint32_t* sl = reinterpret_cast<uint32_t*>(slot + tl.lens_at);
    uint8_t* codes = slot + ca;
    // two passes over the pool's parts: code bytes (and 2-bit bytes) per part, then each part
    // writes at its prefix
    const size_t step = (cnt + T - 1) / T;
    std::fill(part.begin(), part.end(), 0);
    std::fill(part2.begin(), part2.end(), 0);
    std::fill(part4.begin(), part4.end(), 0);
    std::fill(psz.begin(), psz.end(), 0);
    oob = SIZE_MAX;
    pool.run([&](unsigned p) {
      size_t acc = 0, acc2 = 0, acc4 = 0;
      uint32_t m = 0, mn = UINT32_MAX;
      bool out = false, mono = runs_ok;
      uint64_t first = UINT64_MAX, end = 0;  // the run: first start, last end
      for (size_t k = c.c0 + std::min(cnt, p * step); k < c.c0 + std::min(cnt, (p + 1) * step);
           ++k) {
        const uint32_t l = lens[k];
        acc += l;
        acc2 += (l + 3) / 4;
        acc4 += (l + 1) / 2;
        m = std::max(m, l);
        mn = std::min(mn, l);
        // the target must lie inside the caller's residues (checked before any byte is read;
        // the pack passes below re-read this part's offsets from cache)
        out |= offsets[k] > nres || l > nres - offsets[k];
        if (l) {
          mono &= first == UINT64_MAX || offsets[k] >= end;
          if (first == UINT64_MAX) first = offsets[k];
          end = offsets[k] + l;
        }
      }
      const uint64_t span = first == UINT64_MAX ? 0 : end - first;
      const bool run = mono && first != UINT64_MAX && !out && span <= acc + acc / 8 + 64 &&
                       span < (1ull << 30);
      rbase[p] = run ? first : UINT64_MAX;
      rspan[p] = run ? span : 0;
      const size_t acc2e = run ? (span + 3) / 4 : acc2;  // (mixed: this part's 2-bit bytes)
      if (out)
        for (size_t k = c.c0 + std::min(cnt, p * step); k < c.c0 + std::min(cnt, (p + 1) * step);
             ++k)
          if (offsets[k] > nres || lens[k] > nres - offsets[k]) {
            size_t cur = oob.load();
            while (k < cur && !oob.compare_exchange_weak(cur, k)) {
            }
            break;
          }
      part[p + 1] = acc;
      part2[p + 1] = acc2;
      part4[p + 1] = acc4;
      psz[p + 1] = acc2e;
      partmax[p] = m;
      partmin[p] = mn;
    });
    if (oob.load() != SIZE_MAX) {
      const size_t k = oob.load();
      fail(b, SW_ERR_ARG, "target %zu [%llu, +%u) outside the %zu residues", k,
           (unsigned long long)offsets[k], lens[k], nres);
      return 0;
    }
    trace_mark("g-lens");
    chunk_max[gi] = *std::max_element(partmax.begin(), partmax.end());
    const uint32_t chunk_min = *std::min_element(partmin.begin(), partmin.end());
    const bool uni = uni_ok && chunk_min == chunk_max[gi] && chunk_min > 0;
    for (unsigned p = 0; p < T; ++p) {
      part[p + 1] += part[p];
      part2[p + 1] += part2[p];
      part4[p + 1] += part4[p];
      psz[p + 1] += psz[p];
    }
    uint32_t mode = SWK_PACK_BYTES;
    const uint64_t ctop = std::min<uint64_t>(b->query.size(), chunk_max[gi]) * smax0 + smax0;
    const bool cf16 = f16_ok;  // (exact, or optimistic past 2048)
    (void)ctop;
    const size_t ca32 = align16(cnt * 8);
    if (mixed_ok && !uni && (host_dsort || cnt <= SWB_TILE) &&
        ca32 + align16(psz[T] + part4[T] + 3 * cnt + 32) + align16(cnt * 4 + 8) <= c.bytes &&
        psz[T] + part4[T] + 16 < (1ull << 29) && !wave_preferred(b, cnt, chunk_max[gi], cf16)) {
      // the mixed layout (mixed_pack): u32 offset words | lengths | codes; a code outside the
      // alphabet sends the chunk on to the whole-chunk layouts, where the byte path reports it
      uint32_t* so32 = reinterpret_cast<uint32_t*>(slot);
      size_t end = 0;
      if (mixed_pack(b, residues, nres, offsets, lens, c.c0, cnt, step, rbase, rspan, psz, part4,
                     so32, so32 + cnt, slot + ca32, nullptr, nullptr, end)) {
        chunk_mode[gi] = SWK_PACK_MIXED;
        ++b->ctr.mixed_chunks;
        const bool uniform = chunk_min == chunk_max[gi];
        dev_sort[gi] = !uniform && cnt > SWB_TILE;  // (one tile needs no order)
        const size_t copied = ca32 + align16(end + 16);
        mperm[gi++] = copied;  // the device sort's order (n + 2 words) goes after the codes
        return copied;
      }
    }
    bool two = pack2;
    if (two) {  // optimistic: any code > 3 (N, or outside the alphabet) -> 4 bits or bytes
      wide = 0;
      pool.run([&](unsigned p) {
        size_t at = part2[p];
        uint32_t orc = 0;
        const size_t ie = std::min(cnt, (p + 1) * step);
        for (size_t i = std::min(cnt, p * step); i < ie; ++i) {
          const size_t k = c.c0 + i;
          const uint32_t l = lens[k];
          orc |= pack2fn(residues + offsets[k], l, codes + at, wide_ok(k, l, at, 8, part2[p + 1]));
          if (!uni) {
            so[i] = at;
            sl[i] = l;
          }
          at += (l + 3) / 4;
        }
        if (orc > 3u) wide = 1;
      });
      two = wide.load() == 0;
      trace_mark("g-pack2");
      if (two) {
        std::memset(codes + part2[T], 0, 16);  // a last chunk reads 1 byte past
        mode = SWK_PACK_STREAM;
      } else {
        pack2 = false;
      }
    }
    if (mode == SWK_PACK_BYTES && dna_pack) {  // 4-bit: every code below the alphabet size
      wide = 0;
      pool.run([&](unsigned p) {
        size_t at = part4[p];
        uint32_t mx = 0;
        const size_t ie = std::min(cnt, (p + 1) * step);
        for (size_t i = std::min(cnt, p * step); i < ie; ++i) {
          const size_t k = c.c0 + i;
          const uint32_t l = lens[k];
          mx = std::max(mx, pack4fn(residues + offsets[k], l, codes + at,
                                    wide_ok(k, l, at, 16, part4[p + 1])));
          if (!uni) {
            so[i] = at;
            sl[i] = l;
          }
          at += (l + 1) / 2;
        }
        if (mx >= alpha) wide = 1;
      });
      trace_mark("g-pack4");
      if (wide.load() == 0) {
        std::memset(codes + part4[T], 0, 16);  // a last chunk reads up to 3 bytes past
        mode = SWK_PACK_NIBBLE;
      }
    }
    if (mode == SWK_PACK_BYTES) {
      pool.run([&](unsigned p) {
        size_t at = part[p];
        for (size_t i = std::min(cnt, p * step); i < std::min(cnt, (p + 1) * step); ++i) {
          const size_t k = c.c0 + i;
          const uint32_t l = lens[k];
          const uint8_t* src = residues + offsets[k];
          uint8_t* d = codes + at;
          uint8_t m = 0;
          for (uint32_t j = 0; j < l; ++j) {  // copy + alphabet check, vectorised
            const uint8_t v = src[j];
            d[j] = v;
            m = v > m ? v : m;
          }
          if (l && m >= alpha) {
            size_t cur = bad.load();
            while (k < cur && !bad.compare_exchange_weak(cur, k)) {
            }
          }
          so[i] = at;
          sl[i] = l;
          at += l;
        }
      });
      if (bad.load() != SIZE_MAX) {
        const size_t k = bad.load();
        uint8_t m = 0;
        for (uint32_t j = 0; j < lens[k]; ++j) m = std::max(m, residues[offsets[k] + j]);
        fail(b, SW_ERR_ARG, "target %zu code %u outside alphabet", k, (unsigned)m);
        return 0;
      }
    }
    chunk_mode[gi] = mode;
    if (uni) {  // the device needs the codes only
      from = ca;
      chunk_stride[gi] = mode == SWK_PACK_STREAM   ? (chunk_max[gi] + 3) / 4
                         : mode == SWK_PACK_NIBBLE ? (chunk_max[gi] + 1) / 2
                                                   : chunk_max[gi];
    }
    const bool uniform = chunk_min == chunk_max[gi];
    if (!uniform && host_dsort && cnt > SWB_TILE)
      dev_sort[gi++] = 1;
    else
      has_perm[gi++] =
          !uniform && chunk_perm(pool, sl, cnt, reinterpret_cast<uint32_t*>(slot + tl.perm_at));
    trace_mark("g-perm");
    *reinterpret_cast<uint32_t*>(slot + tl.cnt_at) = (uint32_t)cnt;
    return ca + (mode == SWK_PACK_STREAM   ? align16(part2[T] + 16)
                 : mode == SWK_PACK_NIBBLE ? align16(part4[T] + 16)
                                           : align16(part[T]));
  };
  const bool overlap = scratch_free(b, max_len);
  const auto score = [&](uint8_t* dslot, const Chunk& c, int32_t* d_scores,
                         hipStream_t ks) -> sw_status {
    const size_t cnt = c.c1 - c.c0;
    const SlotTail tl = slot_tail(cnt * 8, cnt);
    const bool pm = has_perm[si], ds = dev_sort[si];
    const uint32_t mode = chunk_mode[si], ustride = chunk_stride[si];
    const int slot = (int)(si % b->feed_dslots);  // (the chunk's device slot)
    const size_t mp = mperm[si];
    const uint32_t ml = chunk_max[si++];
    uint32_t* scr = nullptr;
    if (ds) {  // the slot's own sort scratch, zeroed once (the sort kernels leave it zeroed)
      const size_t sw = swk_sort_scratch_bytes() / 4;
      if (b->sortscr[slot].cap < sw) {
        HIPOK(b, b->sortscr[slot].reserve(sw));
        // on the chunk's own stream: a hipMemset is ordered on the null stream only, which
        // does not order the bank's non-blocking streams, so the zeroing could land while the
        // chunk's sort kernels were already counting (a corrupt visiting order: some targets
        // scored twice, others never written)
        HIPOK(b, hipMemsetAsync(b->sortscr[slot].p, 0, sw * 4, ks));
      }
      scr = b->sortscr[slot].p;
    }
    if (ustride)
      return launch(b, dslot + codes_at(cnt), nullptr, nullptr, cnt, ml, d_scores, ks, mode,
                    nullptr, nullptr, false, !overlap, nullptr, nullptr, ml, ustride);
    if (mode == SWK_PACK_MIXED)  // u32 offsets | lengths | codes; the order after the codes
      return launch(b, dslot + align16(cnt * 8), reinterpret_cast<const uint64_t*>(dslot),
                    reinterpret_cast<const uint32_t*>(dslot + cnt * 4), cnt, ml, d_scores, ks,
                    mode, nullptr, nullptr, ds, !overlap,
                    ds ? reinterpret_cast<uint32_t*>(dslot + mp) : nullptr, scr);
    return launch(b, dslot + codes_at(cnt), reinterpret_cast<const uint64_t*>(dslot),
                  reinterpret_cast<const uint32_t*>(dslot + tl.lens_at), cnt, ml, d_scores,
                  ks, mode,
                  pm ? reinterpret_cast<const uint32_t*>(dslot + tl.perm_at) : nullptr,
                  pm ? reinterpret_cast<const uint32_t*>(dslot + tl.cnt_at) : nullptr, ds,
                  !overlap, ds ? reinterpret_cast<uint32_t*>(dslot + tl.perm_at) : nullptr, scr);
  };
  return feed(b, n, chunks, gather, score, out, overlap);
}

// ---- CAPI record path (row f2): sequence_t arrays as the reference host builds them ------

extern "C" sw_status sw_load_query_record(sw_bank* b, const void* record) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
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
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (b && b->qset.size() > 1)
    return fail(b, SW_ERR_STATE, "a query set is loaded: score it with sw_score_batch_device");
  if (!b) return SW_ERR_ARG;
  b->best_kind = 0;
  b->best_root = false;
  if (const sw_status fs = take_fault(b, 0); fs != SW_OK) return fs;  // latched, see swbank.h
  if (n == 0) return SW_OK;
  if (!d_records || !d_scores) return fail(b, SW_ERR_ARG, "null device buffer");
  if (b->alpha != SW_DNA_ALPHA) return fail(b, SW_ERR_UNSUPPORTED, "records carry DNA only");
  if (b->is_multi())
    return multi_device(b, static_cast<const uint8_t*>(d_records), nullptr, nullptr, nullptr, n,
                        0, SWB_RECORD_MAX, d_scores, reinterpret_cast<hipStream_t>(stream), true);
  sw_status st = prepare(b);
  if (st != SW_OK) return st;
  // lengths live on the device: the kernels clamp them to the record capacity
  HIPOK(b, hipSetDevice(b->device));
  return launch(b, static_cast<const uint8_t*>(d_records), nullptr, nullptr, n, SWB_RECORD_MAX,
                d_scores, stream ? reinterpret_cast<hipStream_t>(stream) : b->stream,
                SWK_PACK_RECORDS);
}

static sw_status records_feed_once(sw_bank* b, const uint8_t* recs, size_t n, int32_t* out);

// Host records through the feeder (n >= 1, buffers checked by the caller); lengths are
// checked while gathering.
sw_status records_feed(sw_bank* b, const uint8_t* recs, size_t n, int32_t* out) {
  return with_fault_check(b, [&] { return records_feed_once(b, recs, n, out); });
}

static sw_status records_feed_once(sw_bank* b, const uint8_t* recs, size_t n, int32_t* out) {
  sw_status st = prepare(b);
  if (st != SW_OK) return st;
  if ((st = feeder_init(b)) != SW_OK) return st;
  if (n) {  // equal-length records: one streamed kernel (stream_feed), else the chunks below
    uint16_t l0;
    std::memcpy(&l0, recs + 4, 2);
    bool used = false;
    st = stream_feed(b, nullptr, 0, nullptr, n, l0, out, used, recs);
    if (used) return st;
  }
  const auto rlen = [&](size_t k) { return record_len(recs + k * SWB_RECORD); };
  // chunks in input order: records | lens | perm | count (longest-first order per chunk)
  std::vector<Chunk> chunks;
  size_t c0 = 0;
  for (size_t at : chunk_bounds(n * SWB_RECORD)) {
    const size_t c1 = std::min(n, std::max(c0 + 1, at / SWB_RECORD));
    if (c1 >= n) break;
    chunks.push_back({c0, c1, align16((c1 - c0) * (SWB_RECORD + 8) + 4)});
    c0 = c1;
  }
  chunks.push_back({c0, n, align16((n - c0) * (SWB_RECORD + 8) + 4)});
  HostPool& pool = *b->pool;
  HIPOK(b, hipSetDevice(b->device));
  std::vector<char> has_perm(chunks.size(), 0);
  std::vector<uint32_t> chunk_max(chunks.size(), 0);
  std::atomic<size_t> bad{SIZE_MAX};
  std::atomic<uint32_t> cmax{0};
  size_t gi = 0, si = 0;
  const auto gather = [&](uint8_t* slot, const Chunk& c, size_t&) -> size_t {
    const size_t cnt = c.c1 - c.c0;
    const SlotTail tl = slot_tail(cnt * SWB_RECORD, cnt);
    uint32_t* sl = reinterpret_cast<uint32_t*>(slot + tl.lens_at);
    cmax = 0;
    parallel_for(pool, cnt, [&](size_t lo, size_t hi) {
      std::memcpy(slot + lo * SWB_RECORD, recs + (c.c0 + lo) * SWB_RECORD, (hi - lo) * SWB_RECORD);
      uint32_t m = 0;
      for (size_t i = lo; i < hi; ++i) {
        const uint32_t l = record_len(slot + i * SWB_RECORD);
        sl[i] = l;
        m = std::max(m, l);
      }
      uint32_t cur = cmax.load();
      while (m > cur && !cmax.compare_exchange_weak(cur, m)) {
      }
      if (m > SWB_RECORD_MAX) {
        for (size_t i = lo; i < hi; ++i) {
          size_t cb = bad.load();
          while (sl[i] > SWB_RECORD_MAX && c.c0 + i < cb &&
                 !bad.compare_exchange_weak(cb, c.c0 + i)) {
          }
        }
      }
    });
    if (bad.load() != SIZE_MAX) {
      const size_t k = bad.load();
      fail(b, SW_ERR_ARG, "record %zu length %u > %u", k, rlen(k), SWB_RECORD_MAX);
      return 0;
    }
    has_perm[gi] = chunk_perm(pool, sl, cnt, reinterpret_cast<uint32_t*>(slot + tl.perm_at));
    chunk_max[gi++] = cmax.load();
    *reinterpret_cast<uint32_t*>(slot + tl.cnt_at) = (uint32_t)cnt;
    return c.bytes;
  };
  const bool overlap = scratch_free(b, SWB_RECORD_MAX);
  const auto score = [&](uint8_t* dslot, const Chunk& c, int32_t* d_scores,
                         hipStream_t ks) -> sw_status {
    const size_t cnt = c.c1 - c.c0;
    const SlotTail tl = slot_tail(cnt * SWB_RECORD, cnt);
    const bool pm = has_perm[si];
    const uint32_t ml = chunk_max[si++];
    return launch(b, dslot, nullptr, nullptr, cnt, ml, d_scores, ks, SWK_PACK_RECORDS,
                  pm ? reinterpret_cast<const uint32_t*>(dslot + tl.perm_at) : nullptr,
                  pm ? reinterpret_cast<const uint32_t*>(dslot + tl.cnt_at) : nullptr, false,
                  !overlap);
  };
  return feed(b, n, chunks, gather, score, out, overlap);
}

extern "C" sw_status sw_score_batch(sw_bank* b, const uint8_t* residues, size_t residues_len,
                                    const uint64_t* offsets, const uint32_t* lens,
                                    const uint64_t* ids, size_t n, int32_t* scores_out) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (b && b->qset.size() > 1)
    return fail(b, SW_ERR_STATE, "a query set is loaded: score it with sw_score_batch_device");
  if (!b) return SW_ERR_ARG;
  b->best_kind = 0;
  if (n == 0) return SW_OK;
  if (!offsets || !lens || !scores_out) return fail(b, SW_ERR_ARG, "null host buffer");
  if (n > 0xFFFFFFFFull)
    return fail(b, SW_ERR_ARG, "host batches hold < 2^32 targets (sw_score_batch_device does not)");
  PhaseTrace trace;
  g_trace = trace.path ? &trace : nullptr;
  struct Reset { ~Reset() { g_trace = nullptr; } } reset_trace;
  trace_mark("entry");
  if (b->is_multi()) {
    const sw_status st = multi_batch(b, residues, residues_len, offsets, lens, n, scores_out);
    if (st == SW_OK && ids) b->best_id = ids[b->best_index];
    return st;
  }
  const sw_status st = batch_feed(b, residues, residues_len, offsets, lens, n, scores_out);
  if (st != SW_OK) return st;
  if (ids) b->best_id = ids[b->best_index];
  return SW_OK;
}

extern "C" sw_status sw_score_records(sw_bank* b, const void* records, size_t n,
                                      int32_t* scores_out) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (b && b->qset.size() > 1)
    return fail(b, SW_ERR_STATE, "a query set is loaded: score it with sw_score_batch_device");
  if (!b) return SW_ERR_ARG;
  b->best_kind = 0;
  if (n == 0) return SW_OK;
  if (!records || !scores_out) return fail(b, SW_ERR_ARG, "null host buffer");
  if (b->alpha != SW_DNA_ALPHA) return fail(b, SW_ERR_UNSUPPORTED, "records carry DNA only");
  if (n > 0xFFFFFFFFull)
    return fail(b, SW_ERR_ARG, "host batches hold < 2^32 records (sw_score_records_device does not)");
  const uint8_t* recs = static_cast<const uint8_t*>(records);
  sw_status st;
  if (b->is_multi()) {
    st = multi_records(b, recs, n, scores_out);
  } else {
    st = records_feed(b, recs, n, scores_out);
  }
  if (st == SW_OK) {  // the record's own ID (sequence_t.ID, aligner_Header.h:20)
    uint32_t id;
    std::memcpy(&id, recs + b->best_index * SWB_RECORD, 4);
    b->best_id = id;
  }
  return st;
}

