// swbank_stream.hip — streamed host batches: one kernel per call, chunks published as their
// copies land (the host side of swk_launch_stream).
#include "swbank_bank.h"

// Streamed host batch: every target L codes long (DNA, one query segment, exact 16-bit
// arithmetic, the tile kernel, enough tiles for two rounds of the resident workgroups).  ONE
// kernel launch scores the whole call: chunks of whole tiles are gathered (2-bit, or 4-bit from
// the first chunk holding an N on) into the pinned slots and copied to their own ranges of an
// device buffer; a publisher thread sets a chunk's host layout word once its copy
// landed, and the kernel's waves wait on it before they read the chunk (swk_launch_stream).
// One pipeline fill and drain per call instead of one per chunk, and no chunk kernel on half
// the chip.  `used` = false when the batch does not qualify (the chunked feeder runs instead;
// always for a multi-device bank's per-device parts, out == nullptr); SWBANK_STREAM=0 disables.
// recs != nullptr: the batch is n CAPI records (sw_score_records) of length L (record 0's); each
// chunk takes the first ceil(L/4) bytes of every record's 2-bit data field, so equal-length
// records cross PCIe at half the record bytes.  A record of another length ends streaming:
// found in chunk 0 (before the launch) it costs nothing; later, the kernel drains and the call
// runs through the chunked feeder (`used` = false), which reports bad lengths.
// rlens != nullptr: a ragged batch (L = its longest target); each chunk's region carries the
// chunk's code offsets, lengths and longest-first visiting order ahead of its codes.
sw_status stream_feed(sw_bank* b, const uint8_t* residues, size_t nres,
                      const uint64_t* offsets, size_t n, uint32_t L, int32_t* out, bool& used,
                      const uint8_t* recs, const uint32_t* rlens) {
  used = false;
  if (recs && (L == 0 || L > SWB_RECORD_MAX)) return SW_OK;
  const int mode_env = env_int("SWBANK_STREAM", 1);  // 2: also below the size threshold (tests)
  if (mode_env == 0 || !out || b->alpha != SW_DNA_ALPHA || b->prof || b->col0 || b->RB != 4 ||
      env_int("SWBANK_PACK2", 1) == 0 || env_int("SWBANK_UNIFORM", 1) == 0 ||
      !scratch_free(b, L) || n > 0x7FFFFFFFull)
    return SW_OK;
  if (rlens && env_int("SWBANK_MIXED", 1) == 0) return SW_OK;  // (ragged: the mixed layout)
  const char* kforce = std::getenv("SWBANK_KERNEL");
  if (kforce && std::strcmp(kforce, "wave") == 0) return SW_OK;
  const size_t T = (n + SWB_TILE - 1) / SWB_TILE;
  // two rounds of 4 workgroups per CU: the throughput model picks the tile kernel there
  if (mode_env != 2 && T < 8 * (size_t)std::max(b->cus, 1)) return SW_OK;
  const uint64_t smax = (uint64_t)std::max(0, b->smax);
  const bool use_f16 = b->f16 && b->f16_neg >= -2048 && env_int("SWBANK_F16", 1) != 0 &&
                       std::min<uint64_t>(b->query.size(), L) * smax + smax <= 2048u;
  const bool pair = use_f16 && b->pair_bytes != 0 && env_int("SWBANK_PAIR", 1) != 0;
  if (!(b->R == 16 || b->R == 32)) return SW_OK;  // streamed variants
  int sR = b->R, sW = b->segs[0].W;
  u16_gotoh_rows(b, use_f16, sR, sW);

  // chunks of whole tiles: 1/64 of the batch first, doubling up to 1/8
  std::vector<size_t> tile0;
  const size_t cap = std::max<size_t>(1, T / 8);
  for (size_t t = 0, sz = std::max<size_t>(1, T / 64); t < T; t += sz, sz = std::min(cap, 2 * sz))
    tile0.push_back(t);
  const size_t nsc = tile0.size();
  tile0.push_back(T);
  const size_t nib = (L + 1) / 2;  // 4-bit bytes per target (the 2-bit stream needs fewer)
  const size_t PT0 = b->pool ? b->pool->size() : 1;
  std::vector<size_t> roff(nsc + 1, 0);
  size_t slot_bytes = 0, zbytes = 0;
  for (size_t i = 0; i < nsc; ++i) {
    const size_t cnt = std::min(n, tile0[i + 1] * SWB_TILE) - tile0[i] * SWB_TILE;
    // ragged: offset words | lengths | order, then the mixed codes: the 2-bit region (a run's
    // gaps included: at most 1/8 more codes, + a byte per part) and the 4-bit one (bounded by
    // every target in 4-bit codes)
    const size_t head = rlens ? align16(cnt * 12) : 0;
    const size_t body = rlens ? cnt * ((L + 3) / 4) + cnt * (size_t)L / 32 + cnt * nib + 32 * PT0
                              : cnt * nib;
    if (rlens && head + body + 64 >= ((size_t)1 << 29)) return SW_OK;  // (u32 offset words)
    roff[i + 1] = roff[i] + (head + body + 64 + 255) / 256 * 256;
    slot_bytes = std::max(slot_bytes, roff[i + 1] - roff[i]);
    zbytes = std::max(zbytes, head + 64);
  }
  // ragged: a zeroed region after the chunks, which the kernel reads instead of a chunk the
  // host never sent (released as aborted: its own region may hold anything)
  if (!rlens) zbytes = 0;
  // Memory the streamed call keeps for the bank's lifetime: the batch's 4-bit codes on the
  // device (sbuf), NSLOT pinned host slots of the largest chunk (<= 1/8 of it each) and the
  // batch's scores in coherent host memory.  Past SWBANK_STREAM_MB (default 4096 MiB of device
  // codes + host scores), or when any of it cannot be allocated, the call runs through the
  // chunked feeder, whose slots are bounded by chunk_target() (counted: stream_declined).
  const size_t cap_bytes = (size_t)std::max(1, env_int("SWBANK_STREAM_MB", 4096)) << 20;
  if (roff[nsc] + zbytes + n * 4 > cap_bytes) {
    ++b->ctr.stream_declined;
    return SW_OK;
  }
  HIPOK(b, hipSetDevice(b->device));
  if (!b->kstream) {  // (no queue of its own: the chunked feeder)
    if (b->cus <= 0) return SW_OK;
    std::vector<uint32_t> mask(((size_t)b->cus + 31) / 32, 0xFFFFFFFFu);
    if (hipExtStreamCreateWithCUMask(&b->kstream, (uint32_t)mask.size(), mask.data()) !=
        hipSuccess) {
      b->kstream = nullptr;
      (void)hipGetLastError();
      return SW_OK;
    }
  }
  hipStream_t ks = b->kstream;
  {
    bool ok = b->sbuf.reserve(roff[nsc] + zbytes) == hipSuccess &&
              b->sflag.reserve(nsc * 4) == hipSuccess &&
              b->sdrec.reserve(nsc) == hipSuccess && b->sctr.reserve(1) == hipSuccess &&
              b->srec.reserve(nsc * sizeof(SwkStreamChunk)) == hipSuccess &&
              b->shflag.reserve(nsc * 8) == hipSuccess &&  // layout words | abort words
              b->shscores.reserve(n * 4) == hipSuccess;
    for (int i = 0; ok && i < std::min<int>(sw_bank::NSLOT, (int)nsc); ++i)
      ok = b->hslot[i].reserve(slot_bytes) == hipSuccess;
    while (ok && b->sev.size() < nsc) {  // blocking sync: the publisher sleeps in them
      hipEvent_t e;
      ok = hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventBlockingSync) == hipSuccess;
      if (ok) b->sev.push_back(e);
    }
    if (!ok) {  // out of device or pinned memory: the chunked feeder (bounded slots) instead
      (void)hipGetLastError();
      b->sbuf.release();
      b->shscores.release();
      ++b->ctr.stream_declined;
      return SW_OK;
    }
  }
  used = true;
  SwkStreamChunk* rec = reinterpret_cast<SwkStreamChunk*>(b->srec.p);
  uint32_t* hflag = reinterpret_cast<uint32_t*>(b->shflag.p);
  for (size_t i = 0; i < nsc; ++i) {
    rec[i] = SwkStreamChunk{(unsigned)tile0[i], (unsigned)roff[i], (unsigned)(roff[i] >> 32),
                            (unsigned)(roff[nsc] / 256)};
    __atomic_store_n(&hflag[i], 0u, __ATOMIC_RELAXED);
    __atomic_store_n(&hflag[nsc + i], 0u, __ATOMIC_RELAXED);
  }
  std::atomic_thread_fence(std::memory_order_seq_cst);

  // records and cleared device words, then the kernel (its waves wait on the layout words);
  // enqueued once chunk 0's copy is, so the gather of chunk 0 starts at once
  sw_bank::Ev ev{};
  const auto start_kernel = [&]() -> sw_status {
    HIPOK(b, hipStreamWaitEvent(ks, b->ev_ready, 0));  // query tables uploaded
    HIPOK(b, hipStreamWaitEvent(ks, b->ev_used, 0));   // bank scratch free
    HIPOK(b, hipMemcpyAsync(b->sdrec.p, rec, nsc * sizeof(SwkStreamChunk), hipMemcpyHostToDevice,
                            ks));
    HIPOK(b, hipMemsetAsync(b->sflag.p, 0, nsc * 4, ks));
    HIPOK(b, hipMemsetAsync(b->sctr.p, 0, 4, ks));
    if (zbytes) HIPOK(b, hipMemsetAsync(b->sbuf.p + roff[nsc], 0, zbytes, ks));
    if (b->timing) {  // (an empty "pack" interval: b = a)
      HIPOK(b, hipEventCreate(&ev.a));
      HIPOK(b, hipEventCreate(&ev.c));
      HIPOK(b, hipEventRecord(ev.a, ks));
      ev.b = ev.a;
    }
    HIPOK(b, swk_launch_stream(sR, b->gotoh() ? 1 : 0, use_f16 ? 1 : 0, pair ? 1 : 0, b->sbuf.p,
                               n, rlens ? 0u : L, b->sdrec.p, hflag,
                               reinterpret_cast<uint32_t*>(b->sflag.p),
                               (uint32_t)nsc, b->sctr.p,
                               pair ? b->qpair.p : use_f16 ? b->qtab16.p : b->qtab.p,
                               use_f16 ? b->nv16 : b->nv, b->S, b->O, b->E,
                               pair ? b->pair_bytes : 0, b->pad, sW,
                               reinterpret_cast<int32_t*>(b->shscores.p),
                               b->pS1, b->pS2, ks));
    HIPOK(b, hipEventRecord(b->ev_used, ks));
    if (b->timing) {
      HIPOK(b, hipEventRecord(ev.c, ks));
      b->events.push_back(ev);
    }
    snprintf(b->last_kernel, sizeof(b->last_kernel), "tile %s%s R=%d W=%d segs=1 streamed=%zu",
             use_f16 ? "f16" : "u16", pair ? " pair" : "", sR, sW, nsc);
    trace_mark("kernel");
    return SW_OK;
  };

  // the publisher: chunk i's layout word once its copy landed.  It sleeps in the copy event
  // (blocking-sync events) and on a condition variable for the next issued chunk: spinning
  // threads beside the 16 gather threads burnt the process's CPU quota (multi-ms stalls), and
  // polling from this thread between gather pieces made the gather 3-4x slower
  std::vector<uint32_t> mode(nsc, 0);
  size_t issued = 0;  // (under pm)
  bool stop = false;
  std::mutex pm;
  std::condition_variable pcv;
  // (tests) SWBANK_STREAM_HOLD_MS=t: chunk 1 is published t ms late, past the kernel's wait
  // bound, to exercise the abort and the chunked re-run
  const int hold_ms = env_int("SWBANK_STREAM_HOLD_MS", 0);
  std::vector<std::chrono::steady_clock::time_point> pub_t(nsc);  // (SWBANK_TRACE_FILE)
  size_t published = 0;
  // a copy that failed is never published as landed: the chunk and every later one are released
  // to the kernel as aborted (it drains), and the call fails with SW_ERR_HIP
  hipError_t pub_err = hipSuccess;
  std::thread publisher([&] {
    for (size_t i = 0; i < nsc; ++i) {
      {
        std::unique_lock<std::mutex> lk(pm);
        pcv.wait(lk, [&] { return issued > i || stop; });
        if (issued <= i) return;
      }
      const hipError_t e = hipEventSynchronize(b->sev[i]);
      if (e != hipSuccess) {
        pub_err = e;
        for (size_t j = i; j < nsc; ++j) __atomic_store_n(&hflag[j], SWK_STREAM_ABORT, __ATOMIC_RELEASE);
        return;
      }
      if (i == 1 && hold_ms > 0) std::this_thread::sleep_for(std::chrono::milliseconds(hold_ms));
      __atomic_store_n(&hflag[i], mode[i], __ATOMIC_RELEASE);
      pub_t[i] = std::chrono::steady_clock::now();
      published = i + 1;
    }
  });

  HostPool& pool = *b->pool;
  const unsigned PT = pool.size();
  const bool avx2 = env_int("SWBANK_AVX2", 1) != 0;
  const swpack::PackFn pack2fn = swpack::packer(2, avx2), pack4fn = swpack::packer(4, avx2);
  const size_t steps32 = (L + 31u) / 32u;
  bool nib_mode = false;  // from the first chunk holding an N on: 4-bit chunks
  std::atomic<size_t> oob{SIZE_MAX};
  // ragged: per part its run, 2-bit and 4-bit byte prefixes; the order's length bins (batch
  // longest first, at most 1024 bins of 2^shift lengths) and each part's next slot per bin
  std::vector<uint64_t> rbase(PT), rspan(PT);
  std::vector<size_t> psz(PT + 1, 0), p4(PT + 1, 0);
  const bool runs_ok = env_int("SWBANK_MIXED_RUNS", 1) != 0;
  MixedOrder mo;
  if (rlens) {
    mo.hi = L;
    while ((L >> mo.shift) >= 1024u) ++mo.shift;
    mo.nbin = (L >> mo.shift) + 1;
    mo.pos.assign((size_t)PT * mo.nbin, 0u);
  }
  std::atomic<uint32_t> wide{0};
  sw_status err = SW_OK;
  bool started = false;     // the kernel is enqueued
  bool nonuniform = false;  // (records) a record of another length: the chunked feeder
  for (size_t i = 0; i < nsc && err == SW_OK; ++i) {
    const int s = (int)(i % sw_bank::NSLOT);
    if (i >= (size_t)sw_bank::NSLOT) {
      const hipError_t e = hipEventSynchronize(b->h2d_done[s]);
      if (e != hipSuccess) {
        fail(b, SW_ERR_HIP, "hipEventSynchronize: %s", hipGetErrorString(e));
        err = SW_ERR_HIP;
        break;
      }
    }
    const size_t c0 = tile0[i] * SWB_TILE, c1 = std::min(n, tile0[i + 1] * SWB_TILE);
    const size_t cnt = c1 - c0, step = (cnt + PT - 1) / PT;
    uint8_t* codes = b->hslot[s].p;
    trace_mark("gather<");
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t md = 0;
    size_t sb = 0, bytes = 0;
    if (rlens) {  // ragged: mixed offset words | lengths | order, then the codes (mixed layout)
      const size_t ca = align16(cnt * 12);
      uint32_t* so32 = reinterpret_cast<uint32_t*>(codes);
      uint32_t* sl32 = so32 + cnt;
      uint32_t* sp = sl32 + cnt;
      // lengths pass: bounds, each part's run (targets back to back in the residues, as the
      // chunked feeder's mixed chunks), its 2-bit and 4-bit bytes, and its histogram over the
      // order's length bins (the longest-first order is then placed while packing: no sort pass)
      std::fill(mo.pos.begin(), mo.pos.end(), 0u);
      pool.run([&](unsigned p) {
        const size_t lo = std::min(cnt, p * step), hi = std::min(cnt, (p + 1) * step);
        size_t a1 = 0, a2 = 0, a4 = 0;
        bool mono = runs_ok;
        uint64_t first = UINT64_MAX, last = 0;
        uint32_t* h = mo.pos.data() + (size_t)p * mo.nbin;
        for (size_t j = lo; j < hi; ++j) {
          const size_t k = c0 + j;
          const uint32_t l = rlens[k];
          if (offsets[k] > nres || l > nres - offsets[k]) {
            size_t cur = oob.load();
            while (k < cur && !oob.compare_exchange_weak(cur, k)) {
            }
            return;
          }
          a1 += l;
          a2 += (l + 3) / 4;
          a4 += (l + 1) / 2;
          ++h[(mo.hi - std::min(l, mo.hi)) >> mo.shift];
          if (l) {
            mono &= first == UINT64_MAX || offsets[k] >= last;
            if (first == UINT64_MAX) first = offsets[k];
            last = offsets[k] + l;
          }
        }
        const uint64_t span = first == UINT64_MAX ? 0 : last - first;
        const bool run = mono && first != UINT64_MAX && span <= a1 + a1 / 8 + 64 &&
                         span < (1ull << 30);
        rbase[p] = run ? first : UINT64_MAX;
        rspan[p] = run ? span : 0;
        psz[p + 1] = run ? (span + 3) / 4 : a2;
        p4[p + 1] = a4;
      });
      if (oob.load() == SIZE_MAX) {
        for (unsigned p = 0; p < PT; ++p) {
          psz[p + 1] += psz[p];
          p4[p + 1] += p4[p];
        }
        uint32_t at = 0;  // bins longest first, parts in input order: a stable order
        for (uint32_t bin = 0; bin < mo.nbin; ++bin)
          for (unsigned p = 0; p < PT; ++p) {
            uint32_t& x = mo.pos[(size_t)p * mo.nbin + bin];
            const uint32_t c = x;
            x = at;
            at += c;
          }
        size_t end = 0;
        if (mixed_pack(b, residues, nres, offsets, rlens, c0, cnt, step, rbase, rspan, psz, p4,
                       so32, sl32, codes + ca, sp, &mo, end)) {
          md = SWK_PACK_MIXED;
          bytes = ca + end;
          ++b->ctr.mixed_chunks;
        }
      }
      if (oob.load() == SIZE_MAX && md == 0) {  // a code outside the alphabet
        for (size_t j = 0; j < cnt && err == SW_OK; ++j)
          for (uint32_t x = 0; x < rlens[c0 + j]; ++x)
            if (residues[offsets[c0 + j] + x] >= (uint8_t)SW_DNA_ALPHA) {
              fail(b, SW_ERR_ARG, "target %zu code %u outside alphabet", c0 + j,
                   (unsigned)residues[offsets[c0 + j] + x]);
              err = SW_ERR_ARG;
              break;
            }
        if (err == SW_OK) err = fail(b, SW_ERR_ARG, "code outside alphabet");
        break;
      }
    } else if (recs) {  // 2-bit data bytes of every record; lengths must all be L
      sb = (L + 3) / 4;
      std::atomic<bool> other{false};
      const size_t step = (cnt + PT - 1) / PT;
      pool.run([&](unsigned p) {
        const size_t lo = std::min(cnt, p * step), hi = std::min(cnt, (p + 1) * step);
        for (size_t j = lo; j < hi; ++j) {
          const uint8_t* r = recs + (c0 + j) * SWB_RECORD;
          uint16_t l;
          std::memcpy(&l, r + 4, 2);
          if (l != L) {
            other = true;
            return;
          }
          std::memcpy(codes + j * sb, r + 6, sb);
        }
      });
      if (other.load()) {
        nonuniform = true;
        break;
      }
      md = SWK_PACK_STREAM;
    }
    for (int pass = nib_mode ? 1 : 0; !recs && !rlens && pass < 2 && md == 0; ++pass) {
      sb = pass == 0 ? (L + 3) / 4 : nib;
      const size_t stepb = pass == 0 ? 8 : 16;  // bytes one 32-code vector step stores
      const swpack::PackFn fn = pass == 0 ? pack2fn : pack4fn;
      wide = 0;
      // a part whose targets lie back to back in the residues (offsets k * L apart) and end on
      // a byte boundary of the packed stream packs as ONE run: the per-target call overhead
      // was most of the gather (SWBANK_STREAM_RUNS=0: per target)
      const bool runs = (pass == 0 ? L % 4 == 0 : L % 2 == 0) &&
                        env_int("SWBANK_STREAM_RUNS", 1) != 0;
      pool.run([&](unsigned p) {
        const size_t lo = std::min(cnt, p * step), hi = std::min(cnt, (p + 1) * step);
        uint32_t acc = 0;
        if (runs && hi > lo && (hi - lo) * (size_t)L < 0x80000000ull) {
          const uint64_t o0 = offsets[c0 + lo];
          const size_t total = (hi - lo) * (size_t)L;
          bool back = o0 <= nres && total <= nres - o0;
          for (size_t j = lo + 1; back && j < hi; ++j)
            back = offsets[c0 + j] == o0 + (j - lo) * (uint64_t)L;
          if (back) {
            acc = fn(residues + o0, (uint32_t)total, codes + lo * sb, total % 32 == 0);
            if (pass == 0 ? acc > 3u : acc >= (uint32_t)SW_DNA_ALPHA) wide = 1;
            return;
          }
        }
        for (size_t j = lo; j < hi; ++j) {
          const size_t k = c0 + j;
          if (offsets[k] > nres || L > nres - offsets[k]) {
            size_t cur = oob.load();
            while (k < cur && !oob.compare_exchange_weak(cur, k)) {
            }
            return;
          }
          // full vector steps past the target's end stay inside this part's output (later
          // targets of the part rewrite those bytes) and read inside the residues
          const bool w = offsets[k] + steps32 * 32 <= nres && j * sb + steps32 * stepb <= hi * sb;
          const uint32_t v = fn(residues + offsets[k], L, codes + j * sb, w);
          acc = pass == 0 ? (acc | v) : std::max(acc, v);
        }
        if (pass == 0 ? acc > 3u : acc >= (uint32_t)SW_DNA_ALPHA) wide = 1;
      });
      if (oob.load() != SIZE_MAX) break;
      if (wide.load() == 0) md = pass == 0 ? SWK_PACK_STREAM : SWK_PACK_NIBBLE;
      else if (pass == 0) nib_mode = true;
    }
    if (b->timing)
      b->host_pack_ms +=
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    trace_mark("gather>");
    if (oob.load() != SIZE_MAX) {
      const size_t k = oob.load();
      fail(b, SW_ERR_ARG, "target %zu [%llu, +%u) outside the %zu residues", k,
           (unsigned long long)offsets[k], L, nres);
      err = SW_ERR_ARG;
      break;
    }
    if (md == 0) {  // a code outside the alphabet: the first such target
      for (size_t j = 0; j < cnt && err == SW_OK; ++j)
        for (uint32_t x = 0; x < L; ++x)
          if (residues[offsets[c0 + j] + x] >= (uint8_t)SW_DNA_ALPHA) {
            fail(b, SW_ERR_ARG, "target %zu code %u outside alphabet", c0 + j,
                 (unsigned)residues[offsets[c0 + j] + x]);
            err = SW_ERR_ARG;
            break;
          }
      if (err == SW_OK) err = fail(b, SW_ERR_ARG, "code outside alphabet");
      break;
    }
    if (!rlens) bytes = cnt * sb;
    std::memset(codes + bytes, 0, 16);  // the last targets' final step reads a few bytes past
    const hipError_t e1 = hipMemcpyAsync(b->sbuf.p + roff[i], codes, bytes + 16,
                                         hipMemcpyHostToDevice, b->copy_stream);
    __atomic_fetch_add(&b->ctr.h2d_bytes, (uint64_t)(bytes + 16), __ATOMIC_RELAXED);
    const hipError_t e2 = e1 != hipSuccess ? e1 : hipEventRecord(b->h2d_done[s], b->copy_stream);
    const hipError_t e3 = e2 != hipSuccess ? e2 : hipEventRecord(b->sev[i], b->copy_stream);
    if (e3 != hipSuccess) {
      fail(b, SW_ERR_HIP, "streamed chunk copy: %s", hipGetErrorString(e3));
      err = SW_ERR_HIP;
      break;
    }
    mode[i] = md;
    {
      std::lock_guard<std::mutex> lk(pm);
      issued = i + 1;
    }
    pcv.notify_one();
    trace_mark("launched");
    if (i == 0 && (err = start_kernel()) != SW_OK) break;
    started = i == 0 || started;
  }
  // the issued chunks' words once their copies landed; on failure the chunks never sent are
  // released to the kernel as aborted (their targets read as empty) so it drains, and
  // the call reports the error
  {
    std::lock_guard<std::mutex> lk(pm);
    stop = true;
  }
  pcv.notify_one();
  publisher.join();
  if (g_trace)
    for (size_t i = 0; i < published; ++i) g_trace->mark_at("published", pub_t[i]);
  for (size_t i = issued; i < nsc; ++i)
    __atomic_store_n(&hflag[i], SWK_STREAM_ABORT, __ATOMIC_RELEASE);
  if (!started) {  // nothing enqueued on the bank stream; chunk 0's copy may be in flight
    (void)hipStreamSynchronize(b->copy_stream);
    if (nonuniform) used = false;
    return err;
  }
  // no copy follows the kernel: it writes the scores (and any abort word) straight to coherent
  // host memory.  (A copy enqueued behind the running kernel may hold the copy engine the
  // chunks' copies need until the kernel ends: chunks that never reach the kernel.)
  const hipError_t se = hipStreamSynchronize(ks);
  if (err != SW_OK) return err;
  if (pub_err != hipSuccess)
    return fail(b, SW_ERR_HIP, "streamed chunk copy: %s", hipGetErrorString(pub_err));
  if (nonuniform) {  // the kernel drained on aborted chunks: the chunked feeder runs the call
    used = false;
    return SW_OK;
  }
  if (se != hipSuccess) return fail(b, SW_ERR_HIP, "streamed batch: %s", hipGetErrorString(se));
  trace_mark("landed");
  // a chunk whose wait ran out (its copy held up past the kernel's bound, e.g. by other work on
  // the device's copy engines): the call runs again through the chunked feeder
  for (size_t i = 0; i < nsc; ++i)
    if (__atomic_load_n(&hflag[nsc + i], __ATOMIC_ACQUIRE) == SWK_STREAM_ABORT) {
      used = false;
      ++b->ctr.stream_reruns;
      return SW_OK;
    }
  ++b->ctr.stream_calls;
  // scores into the caller's buffer with the best hit (lowest index of the maximum)
  const int32_t* hs = reinterpret_cast<const int32_t*>(b->shscores.p);
  std::vector<size_t> pbest(PT, SIZE_MAX);
  const size_t ostep = (n + PT - 1) / PT;
  pool.run([&](unsigned p) {
    const size_t lo = std::min(n, p * ostep), hi = std::min(n, (p + 1) * ostep);
    size_t bi = lo;
    for (size_t k = lo; k < hi; ++k) {
      const int32_t v = hs[k];
      out[k] = v;
      if (v > hs[bi]) bi = k;
    }
    if (lo < hi) pbest[p] = bi;
  });
  size_t best = 0;
  for (size_t x : pbest)  // parts in index order: strictly greater keeps the lowest
    if (x != SIZE_MAX && hs[x] > hs[best]) best = x;
  b->best_index = best;
  b->best_id = best;
  b->best_score = hs[best];
  b->best_kind = 1;
  trace_mark("done");
  return SW_OK;
}

