// swbank_bank.hip — the bank object: lifecycle, penalties, queries and the query tables.
// 
// Call surface mirrors ScoreBank_v2 (reference ScoreBank/ScoreBank_v2.v:30-44): penalties once,
// a query once, then any number of target batches; one max score per target.  See
// include/swbank.h for the per-function reference citations.
#include "swbank_bank.h"

sw_status fail(sw_bank* b, sw_status st, const char* fmt, ...) {
  if (b) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(b->err, sizeof(b->err), fmt, ap);
    va_end(ap);
  }
  return st;
}

extern "C" int32_t sw_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// RCCL for the multi-device score gather (SURVEY §8 e: ncclCommInitAll, rccl.h:236, and
// ncclGather, rccl.h:745).  Loaded on first use so single-device users never map it; in a
// process where PyTorch already mapped its librccl.so.1 that copy is reused (same SONAME).
static sw_status check_device(int dev) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SW_ERR_NO_DEVICE;
  if (dev < 0 || dev >= ndev) return SW_ERR_NO_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return SW_ERR_NO_DEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return SW_ERR_NO_DEVICE;
  return SW_OK;
}


extern "C" sw_status sw_bank_create(sw_bank** out, const sw_config* cfg_in) {
  DevGuard dev_guard;  // the caller's current device is restored on return (ABI 6)
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
  if (cfg.n_devices < 0 || cfg.n_devices > SW_MAX_DEVICES) return SW_ERR_ARG;

  if (cfg.n_devices >= 1) {
    // Multi-device bank (≙ MODULES ScoringModules behind one PrioEncoder, ScoreBank_v2.v:76-148):
    // a child bank per device; every host batch is dealt over them.
    for (int d = 0; d < cfg.n_devices; ++d) {
      const sw_status st = check_device(cfg.devices[d]);
      if (st != SW_OK) return st;
    }
    sw_bank* b = new (std::nothrow) sw_bank();
    if (!b) return SW_ERR_NOMEM;
    b->cfg = cfg;
    b->device = cfg.devices[0];
    b->alpha = cfg.alphabet == SW_ALPHABET_DNA ? SW_DNA_ALPHA : SW_PROTEIN_ALPHA;
    for (int d = 0; d < cfg.n_devices; ++d) {
      sw_config kc = cfg;
      kc.n_devices = 0;
      kc.device = cfg.devices[d];
      sw_bank* k = nullptr;
      const sw_status st = sw_bank_create(&k, &kc);
      if (st != SW_OK) {
        sw_bank_destroy(b);
        return st;
      }
      k->pool_threads = std::max(2u, host_threads() / (unsigned)cfg.n_devices);
      b->kids.push_back(k);
    }
    b->dpool.reset(new (std::nothrow) HostPool((unsigned)cfg.n_devices));
    b->pool.reset(new (std::nothrow) HostPool(host_threads()));
    if (!b->dpool || !b->pool) {
      sw_bank_destroy(b);
      return SW_ERR_NOMEM;
    }
    // RCCL gather when every device is distinct (RCCL refuses two ranks on one device) unless
    // SWBANK_GATHER=copy; SWBANK_GATHER=rccl makes an RCCL failure an error instead of a
    // fallback to device copies.
    const char* gm = std::getenv("SWBANK_GATHER");
    const bool force_copy = gm && std::strcmp(gm, "copy") == 0;
    const bool force_rccl = gm && std::strcmp(gm, "rccl") == 0;
    bool distinct = true;
    for (int i = 0; i < cfg.n_devices; ++i)
      for (int j = 0; j < i; ++j) distinct = distinct && cfg.devices[i] != cfg.devices[j];
    if (!force_copy && (distinct || force_rccl)) {
      const Rccl& r = rccl();
      ncclResult_t nr = ncclSuccess;
      if (r.ok) {
        std::vector<ncclComm_t> comms((size_t)cfg.n_devices);
        nr = r.commInitAll(comms.data(), cfg.n_devices, cfg.devices);
        if (nr == ncclSuccess) b->comms.assign(comms.begin(), comms.end());
      }
      b->rccl_gather = !b->comms.empty();
      if (b->comms.empty() && force_rccl) {
        sw_bank_destroy(b);
        return SW_ERR_UNSUPPORTED;
      }
      if (b->comms.empty())
        snprintf(b->err, sizeof(b->err), "RCCL unavailable (%s), gathering with device copies",
                 r.ok ? r.errorString(nr) : r.err);
    }
    (void)hipSetDevice(b->device);
    *out = b;
    return SW_OK;
  }

  int dev = cfg.device;
  if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return SW_ERR_NO_DEVICE;
  const sw_status dst = check_device(dev);
  if (dst != SW_OK) return dst;

  sw_bank* b = new (std::nothrow) sw_bank();
  if (!b) return SW_ERR_NOMEM;
  b->cfg = cfg;
  b->device = dev;
  // The bank's four streams are created together, here: HIP maps streams onto its hardware
  // queues (GPU_MAX_HW_QUEUES, 4 by default) in creation order, so streams the caller creates
  // between the bank's creation and its first host-buffer call (torch's, in bench.py) used to
  // push the feeder's second kernel stream onto the bank stream's queue -- the two chunk
  // streams then serialised: ragged host calls 2.8-3.2 ms instead of 2.2-2.5 (LEDGER §3.2)
  if (hipSetDevice(dev) != hipSuccess ||
      hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&b->copy_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&b->out_stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&b->stream2, hipStreamNonBlocking) != hipSuccess) {
    for (hipStream_t* x : {&b->stream, &b->copy_stream, &b->out_stream, &b->stream2})
      if (*x) (void)hipStreamDestroy(*x);
    delete b;
    return SW_ERR_HIP;
  }
  b->alpha = cfg.alphabet == SW_ALPHABET_DNA ? SW_DNA_ALPHA : SW_PROTEIN_ALPHA;
  if (hipDeviceGetAttribute(&b->cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    b->cus = 0;
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
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (!b) return;
  if (b->is_multi() || !b->comms.empty()) {
    const Rccl& r = rccl();
    for (void* c : b->comms) (void)r.commDestroy(static_cast<ncclComm_t>(c));
    (void)hipSetDevice(b->device);
    if (b->ev_used) (void)hipEventSynchronize(b->ev_used);  // the last device call's scatter
    if (b->ev_join) (void)hipEventDestroy(b->ev_join);
    if (b->ev_used) (void)hipEventDestroy(b->ev_used);
    for (sw_bank* k : b->kids) sw_bank_destroy(k);
    b->dpool.reset();
    b->pool.reset();
    (void)hipSetDevice(b->device);
    b->grecv.release();
    b->hrecv.release();
    b->res.release();  // the device-call deal's staging (multi_device)
    b->offs.release();
    b->lens.release();
    b->dperm.release();
    b->dsort.release();
    delete b;
    return;
  }
  (void)hipSetDevice(b->device);
  if (b->stream) (void)hipStreamSynchronize(b->stream);
  uint64_t nl;
  double pm, sm;
  (void)sw_bank_timing(b, &nl, &pm, &sm);
  b->faultw.release();
  b->qtab.release();
  b->qtab16.release();
  b->mqtab.release();
  b->mqtab16.release();
  b->mqpair.release();
  b->qpair.release();
  b->stage.release();
  if (b->ev_ready) (void)hipEventDestroy(b->ev_ready);
  if (b->ev_used) (void)hipEventDestroy(b->ev_used);
  if (b->best_ev) (void)hipEventDestroy(b->best_ev);
  if (b->ev_join) (void)hipEventDestroy(b->ev_join);
  for (hipEvent_t e : b->deal_ev) (void)hipEventDestroy(e);
  b->fb_idx.release();
  b->fb_cnt.release();
  b->best_key.release();
  b->best_dev.release();
  b->i32prof.release();
  b->i32scr.release();
  b->dperm.release();
  b->dsort.release();
  b->bal_state.release();
  b->bal_flag.release();
  b->wbal_state.release();
  b->wbal_flag.release();
  b->bal_plan.release();
  b->wtab.release();
  b->wtab16.release();
  b->tprog.release();
  for (int i = 0; i < 3; ++i) {
    b->stab[i].release();
    b->stab16[i].release();
  }
  b->sring.release();
  b->edge[0].release();
  b->edge[1].release();
  if (b->copy_stream) (void)hipStreamSynchronize(b->copy_stream);
  if (b->out_stream) (void)hipStreamSynchronize(b->out_stream);
  if (b->stream2) (void)hipStreamSynchronize(b->stream2);
  for (hipEvent_t e : b->out_ev) (void)hipEventDestroy(e);
  for (int i = 0; i < sw_bank::NSLOT; ++i) b->hslot[i].release();
  for (int i = 0; i < sw_bank::NDSLOT; ++i) {
    b->dslot[i].release();
    b->sortscr[i].release();
  }
  b->sbuf.release();
  b->sflag.release();
  b->sdrec.release();
  b->sctr.release();
  b->srec.release();
  b->shflag.release();
  b->shscores.release();
  for (hipEvent_t e : b->sev) (void)hipEventDestroy(e);
  for (int i = 0; i < sw_bank::NSLOT; ++i)
    if (b->h2d_done[i]) (void)hipEventDestroy(b->h2d_done[i]);
  for (int i = 0; i < sw_bank::NDSLOT; ++i)
    if (b->kern_done[i]) (void)hipEventDestroy(b->kern_done[i]);
  b->hscores.release();
  b->launcher.reset();
  b->pool.reset();
  if (b->copy_stream) (void)hipStreamDestroy(b->copy_stream);
  if (b->out_stream) (void)hipStreamDestroy(b->out_stream);
  if (b->stream2) (void)hipStreamDestroy(b->stream2);
  if (b->kstream) (void)hipStreamDestroy(b->kstream);
  if (b->ev_s2) (void)hipEventDestroy(b->ev_s2);
  b->res.release();
  b->offs.release();
  b->lens.release();
  b->scores.release();
  b->gres.release();
  b->goffs.release();
  b->glens.release();
  if (b->stream) (void)hipStreamDestroy(b->stream);
  delete b;
}

extern "C" int32_t sw_bank_devices(const sw_bank* b, int32_t* devices, int32_t cap) {
  if (!b) return 0;
  const int32_t n = b->is_multi() ? (int32_t)b->kids.size() : 1;
  for (int32_t i = 0; devices && i < std::min(n, cap); ++i)
    devices[i] = b->is_multi() ? b->kids[(size_t)i]->device : b->device;
  return n;
}

extern "C" const char* sw_last_error(const sw_bank* b) { return b ? b->err : "null bank"; }

extern "C" const char* sw_last_kernel(const sw_bank* b) { return b ? b->last_kernel : ""; }

uint32_t* fault_word(sw_bank* b) {
  if (!b->faultw.p) {
    if (b->faultw.reserve(64) != hipSuccess) return nullptr;
    std::memset(b->faultw.p, 0, b->faultw.cap);
  }
  return reinterpret_cast<uint32_t*>(b->faultw.p);
}

sw_status take_fault(sw_bank* b, int which) {
  if (b->is_multi()) {
    sw_status st = SW_OK;
    for (sw_bank* k : b->kids) {  // every child's word is cleared, the first fault reported
      const sw_status ks = take_fault(k, which);
      if (ks != SW_OK && st == SW_OK) st = fail(b, ks, "device %d: %s", k->device, k->err);
    }
    return st;
  }
  if (!b->faultw.p) return SW_OK;
  // the call kind's group: one word per fault kind (SWK_FAULT_WORDS, swbank_internal.h)
  volatile uint32_t* w = reinterpret_cast<volatile uint32_t*>(b->faultw.p) + which * SWK_FAULT_WORDS;
  uint32_t f = 0;
  for (int i = 0; i < SWK_FAULT_WORDS; ++i) {
    f |= w[i];
    w[i] = 0;
  }
  if (f == 0) return SW_OK;
  if (f & SWK_FAULT_BAL) ++b->ctr.balanced_timeouts;
  if (f & SWK_FAULT_TAIL) ++b->ctr.tail_timeouts;
  if (f & SWK_FAULT_WBAL) ++b->ctr.wave_balanced_timeouts;
  char kinds[96] = "";
  const char* names[3] = {"balanced ranges", "protein tail", "wave balanced ranges"};
  for (int i = 0; i < 3; ++i)
    if (f & (1u << i)) {
      if (kinds[0]) strncat(kinds, ", ", sizeof(kinds) - strlen(kinds) - 1);
      strncat(kinds, names[i], sizeof(kinds) - strlen(kinds) - 1);
    }
  return fail(b, SW_ERR_TIMEOUT,
              "a cross-workgroup hand-off wait ran out (%s) in a %s call: its scores are invalid",
              kinds, which ? "host-buffer" : "device");
}

extern "C" sw_status sw_bank_sync(sw_bank* b) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (!b) return SW_ERR_ARG;
  if (b->is_multi()) {
    for (sw_bank* k : b->kids) {
      const sw_status st = sw_bank_sync(k);
      if (st != SW_OK) {
        (void)take_fault(b, 0);  // (clear the other devices' words too)
        return fail(b, st, "device %d: %s", k->device, k->err);
      }
    }
    if (b->ev_used) {  // the device-call deal's scatter on the root (multi_device)
      int cur = -1;
      HIPOK(b, hipGetDevice(&cur));
      hipError_t e = hipSetDevice(b->device);
      if (e == hipSuccess) e = hipEventSynchronize(b->ev_used);
      (void)hipSetDevice(cur);
      HIPOK(b, e);
    }
    return SW_OK;
  }
  int cur = -1;
  HIPOK(b, hipGetDevice(&cur));
  hipError_t e = hipSetDevice(b->device);
  // ev_used follows every launch of a scoring call on the stream it ran on
  if (e == hipSuccess && b->ev_used) e = hipEventSynchronize(b->ev_used);
  if (e == hipSuccess) e = hipStreamSynchronize(b->stream);
  (void)hipSetDevice(cur);
  HIPOK(b, e);
  return take_fault(b, 0);
}

static void sum_counters(sw_counters& c, const sw_bank* b) {
  c.stream_calls += b->ctr.stream_calls;
  c.stream_reruns += b->ctr.stream_reruns;
  c.stream_declined += b->ctr.stream_declined;
  c.chunked_calls += b->ctr.chunked_calls;
  c.device_sorts += b->ctr.device_sorts;
  c.gather_timeouts += b->ctr.gather_timeouts;
  c.mixed_chunks += b->ctr.mixed_chunks;
  c.mixed_runs += b->ctr.mixed_runs;
  c.balanced_calls += b->ctr.balanced_calls;
  c.balanced_timeouts += b->ctr.balanced_timeouts;
  c.tail_timeouts += b->ctr.tail_timeouts;
  c.handoff_reruns += b->ctr.handoff_reruns;
  c.wave_balanced_timeouts += b->ctr.wave_balanced_timeouts;
  c.h2d_bytes += __atomic_load_n(&b->ctr.h2d_bytes, __ATOMIC_RELAXED);
}

// Host-side counts only (no HIP call): a hand-off time-out is counted when a synchronising call
// takes it from the fault word.
extern "C" sw_status sw_bank_counters_ex(const sw_bank* b, sw_counters* out, size_t out_size) {
  if (!b || !out) return SW_ERR_ARG;
  // the struct sizes of ABI 3 (8 counters), ABI 4 (10), ABI 5 (12) and ABI 6 (14)
  if (out_size != 64 && out_size != 80 && out_size != 96 && out_size != sizeof(sw_counters))
    return SW_ERR_ARG;
  sw_counters c{};
  sum_counters(c, b);
  for (const sw_bank* k : b->kids) sum_counters(c, k);
  std::memcpy(out, &c, out_size);
  return SW_OK;
}

// ABI 5: the two-argument form of ABI 3 again, writing the ABI-3 prefix (8 counters), so a
// caller of either earlier ABI never gets more bytes than its struct holds.
extern "C" sw_status sw_bank_counters(const sw_bank* b, sw_counters* out) {
  return sw_bank_counters_ex(b, out, 64);
}

void copy_kernel_name(sw_bank* b, const char* gather) {
  snprintf(b->last_kernel, sizeof(b->last_kernel), "multi[%zu] gather=%s: %s", b->kids.size(),
           gather, b->kids[0]->last_kernel);
}

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
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (!b) return SW_ERR_ARG;
  if (b->is_multi())
    return each_kid(b, [&](sw_bank* k) {
      return sw_set_penalties(k, match, mismatch, gap_open, gap_extend);
    });
  if (b->cfg.alphabet != SW_ALPHABET_DNA)
    return fail(b, SW_ERR_ARG, "sw_set_penalties needs a DNA bank; use sw_set_matrix");
  int8_t m[SW_DNA_ALPHA * SW_DNA_ALPHA];
  if (sw_fill_matrix(SW_ALPHABET_DNA, match, mismatch, m) != SW_OK)
    return fail(b, SW_ERR_ARG, "match/mismatch outside int8 (%d, %d)", match, mismatch);
  return set_matrix_impl(b, m, SW_DNA_ALPHA, gap_open, gap_extend);
}

extern "C" sw_status sw_set_matrix(sw_bank* b, const int8_t* m, int32_t alpha, int32_t gap_open,
                                   int32_t gap_extend) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (!b || !m) return SW_ERR_ARG;
  if (b->is_multi())
    return each_kid(b, [&](sw_bank* k) { return sw_set_matrix(k, m, alpha, gap_open, gap_extend); });
  const int want = b->cfg.alphabet == SW_ALPHABET_DNA ? SW_DNA_ALPHA : SW_PROTEIN_ALPHA;
  if (alpha != want) return fail(b, SW_ERR_ARG, "matrix alphabet %d, bank expects %d", alpha, want);
  return set_matrix_impl(b, m, alpha, gap_open, gap_extend);
}

extern "C" sw_status sw_load_query(sw_bank* b, uint64_t id, const uint8_t* codes, uint32_t len) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (!b || (!codes && len)) return SW_ERR_ARG;
  if (b->is_multi()) {  // the query goes to every device (ScoreBank_v2.v:101-102)
    const sw_status st = each_kid(b, [&](sw_bank* k) { return sw_load_query(k, id, codes, len); });
    b->qset.clear();
    b->have_query = st == SW_OK;
    return st;
  }
  const uint32_t cap = b->cfg.max_query_len ? b->cfg.max_query_len : SWB_MAX_QUERY;
  if (len > cap)
    return fail(b, SW_ERR_UNSUPPORTED, "query length %u exceeds the bank maximum %u", len, cap);
  for (uint32_t i = 0; i < len; ++i)
    if (codes[i] >= (uint32_t)b->alpha)
      return fail(b, SW_ERR_ARG, "query code %u at %u outside alphabet %d", codes[i], i, b->alpha);
  b->query.assign(codes, codes + len);
  b->qid = id;
  b->qset.clear();
  b->have_query = true;
  b->dirty = true;
  return SW_OK;
}

// A query set: ld_sequence for several queries that every following device batch is scored
// against (scores query-major, nq x n).  One query = sw_load_query.
extern "C" sw_status sw_load_queries(sw_bank* b, size_t nq, const uint64_t* ids,
                                     const uint8_t* codes, const uint64_t* offsets,
                                     const uint32_t* lens) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (!b || nq == 0 || !offsets || !lens) return SW_ERR_ARG;
  if (b->is_multi()) {  // the set goes to every device (ScoreBank_v2.v:101-102)
    const sw_status st = each_kid(
        b, [&](sw_bank* k) { return sw_load_queries(k, nq, ids, codes, offsets, lens); });
    b->qset = b->kids[0]->qset;  // (sizes only: the guards and sw_query_count read it)
    b->have_query = st == SW_OK;
    return st;
  }
  if (nq > 65536) return fail(b, SW_ERR_UNSUPPORTED, "more than 65536 queries in one set");
  if (nq == 1) return sw_load_query(b, ids ? ids[0] : 0, codes + offsets[0], lens[0]);
  const uint32_t cap = b->cfg.max_query_len ? b->cfg.max_query_len : SWB_MAX_QUERY;
  size_t longest = 0;
  for (size_t i = 0; i < nq; ++i) {
    if (lens[i] > cap)
      return fail(b, SW_ERR_UNSUPPORTED, "query %zu length %u exceeds the bank maximum %u", i,
                  lens[i], cap);
    if (lens[i] && !codes) return fail(b, SW_ERR_ARG, "null query codes");
    for (uint32_t j = 0; j < lens[i]; ++j)
      if (codes[offsets[i] + j] >= (uint32_t)b->alpha)
        return fail(b, SW_ERR_ARG, "query %zu code %u at %u outside alphabet %d", i,
                    codes[offsets[i] + j], j, b->alpha);
    if (lens[i] > lens[longest]) longest = i;
  }
  b->qset.assign(nq, {});
  for (size_t i = 0; i < nq; ++i)
    b->qset[i].assign(codes + offsets[i], codes + offsets[i] + lens[i]);
  b->query = b->qset[longest];
  b->qid = ids ? ids[longest] : 0;
  b->have_query = true;
  b->dirty = true;
  b->mq_ready = false;
  return SW_OK;
}

extern "C" size_t sw_query_count(const sw_bank* b) {
  return !b || !b->have_query ? 0 : b->qset.size() > 1 ? b->qset.size() : 1;
}

// Letter-pair table layout for NR rows: slot (a, b) at 16 + a*pS1 + b*pS2 (bytes), pS2/16 = 1 and
// pS1/16 = 4 (mod 16) so the 16 A/C/G/T slots sit on 16 different 4-bank LDS groups.
static void pair_strides(uint32_t NR, uint32_t& pS1, uint32_t& pS2) {
  const uint32_t B = 4 * NR;
  pS2 = (B + 15) / 16 * 16;
  while ((pS2 / 16) % 16 != 1) pS2 += 16;
  pS1 = (4 * pS2 + B + 15) / 16 * 16;
  while ((pS1 / 16) % 16 != 4) pS1 += 16;
}

// The letter-pair table of query rows [r0, r0 + NR) (the PAIR tile kernel, DNA merged f16):
// slot (a, b) holds word k = {s(q_{r0+k+1}, a), s(q_{r0+k+1}, b)} (f16 halves; rows past the
// query -2048) and the row-r0 word 4 bytes before it.
static std::vector<uint32_t> pair_table(const uint8_t* q, int qlen, int r0, uint32_t NR,
                                        const int8_t* m, int A, uint32_t pS1, uint32_t pS2) {
  const uint32_t bytes = 16 + 4 * pS1 + 4 * pS2 + 4 * NR;
  std::vector<uint32_t> t(bytes / 4, 0xBC00BC00u);
  auto word = [&](int r, int x, int y) -> uint32_t {  // row r of the segment, letters x, y
    if (r0 + r >= qlen) return 0xBC00BC00u;
    const int c = q[r0 + r];
    return (uint32_t)f16_score_bits(m[c * A + x]) | (uint32_t)f16_score_bits(m[c * A + y]) << 16;
  };
  for (int x = 0; x < A; ++x)
    for (int y = 0; y < A; ++y) {
      const uint32_t base = (16 + x * pS1 + y * pS2) / 4;
      for (uint32_t k = 0; k + 1 < NR; ++k) t[base + k] = word((int)k + 1, x, y);
    }
  for (int x = 0; x < A; ++x)  // row-0 words last: they may reuse word NR-1 of a slot
    for (int y = 0; y < A; ++y) t[(16 + x * pS1 + y * pS2) / 4 - 1] = word(0, x, y);
  return t;
}

// Build the resident query state (the ScoringModule's query + penalty registers,
// ScoringModule_v1.1.v:110-150): either per-row 4-byte LUTs (DNA fast path) or a query
// profile QP[letter][row] = S - s(q_row, letter) (any alphabet).
sw_status prepare(sw_bank* b) {
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
    const uint16_t bits = f16_score_bits(m[i]);
    lut_f16 = lut_f16 && (bits & 0xFFu) == 0;
  }
  const bool f16_range = -(o + 2 * e + (std::max(0, smax) - smin)) >= -2048;
  const int prof =
      (env_int("SWBANK_PROFILE", 0) || !lut || (!lut_f16 && f16_range)) ? 1 : 0;

  const int qlen = (int)b->query.size();
  // the HDL column-0 rule differs from the plain recurrence only if a match pays for a gap
  const int col0 = (!gotoh && smax > o + e) ? 1 : 0;
  // Rows per wave: 32 for the DNA LUT kernels (merged and Gotoh: the Gotoh f16 column with
  // the letter-pair table runs 8.3-8.6 TCUPS at R = 32 against 7.8-8.2 at R = 16, and a
  // 512-row query fits one workgroup); 16 for tiny queries and for the profile / column-0
  // variants, whose 32-row columns do not fit 128 VGPRs (the occupancy-4 budget) without
  // spilling.  Queries longer than one workgroup (16 waves) run
  // as segments of SWBANK_SEG rows (default: a full 16-wave workgroup, 16·R rows), each
  // segment's bottom row handed to the next through HBM.  SWBANK_R / SWBANK_RB / SWBANK_SEG
  // override (tuning only).
  // u16 Gotoh keeps R = 16 when no f16 pass can run (its 32-row column spills past 128 VGPRs);
  // u16 passes that follow an f16 pass (optimistic re-scores) are rare and use the f16 layout
  const bool u16_only = gotoh && (!f16_range || env_int("SWBANK_F16", 1) == 0);
  int R = (qlen <= 16 || prof || col0 || u16_only) ? 16 : 32, RB = 4;
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
    const uint16_t bits = f16_score_bits(v);
    *out = (uint8_t)(bits >> 8);
    return (bits & 0xFFu) == 0 &&
           (int)((float)__builtin_bit_cast(_Float16, bits) * 2048.0f) == v;
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
    tab16.assign(tab.size(), 0xBCBCBCBCu);  // padding rows: -2048
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
    const uint16_t padv = 0xBC00u;  // -2048: padding letter and rows past the query
    for (sw_bank::Seg& sg : segs) {
      const int r0 = (int)(&sg - segs.data()) * seg_rows;
      std::vector<uint16_t> qp((size_t)(A + 1) * PS16 / 2, padv);
      for (int c = 0; c < A; ++c)
        for (int i = 0; i < sg.W * R && r0 + i < qlen && i < seg_rows; ++i)
          qp[(size_t)c * PS16 / 2 + i] =
              f16_score_bits(m[b->query[r0 + i] * A + c]);
      sg.off16 = tab16.size();
      tab16.resize(sg.off16 + qp.size() / 2);
      std::memcpy(tab16.data() + sg.off16, qp.data(), qp.size() * 2);
    }
  }
  // Letter-pair table for the PAIR tile kernel (SWBANK_PAIR=0 at launch time disables it):
  // DNA merged gaps,
  // the f16 LUT kernel's R = 32, one segment of at most 4 waves (the table's 25 slots then fit
  // beside the ring at 4 workgroups per CU).  Slot (a, b) at 16 + a*S1 + b*S2 holds word k =
  // {s(q_{k+1}, a), s(q_{k+1}, b)} (f16 halves; rows past the query -2048) and the row-0 word
  // 4 bytes before it.  S2/16 = 1 and S1/16 = 4 (mod 16) put the 16 A/C/G/T slots on 16
  // different 4-bank LDS groups.
  // DNA Gotoh (R = 16): one table per query segment, each of the tallest segment's rows (the
  // Gotoh column is 7.5 VALU per 2 cells from the table against 8.5 with the row LUT).
  std::vector<uint32_t> tpair;
  uint32_t pS1 = 0, pS2 = 0, pair_words = 0;
  if (f16 && !prof && !col0 && A == SW_DNA_ALPHA &&
      (gotoh ? R == 16 || R == 32 : R == 32 && segs.size() == 1 && segs[0].W <= 4)) {
    const uint32_t NR = (uint32_t)segs[0].W * R;
    pair_strides(NR, pS1, pS2);
    for (size_t sg = 0; sg < segs.size(); ++sg) {
      const std::vector<uint32_t> t =
          pair_table(b->query.data(), qlen, (int)sg * seg_rows, NR, m, A, pS1, pS2);
      pair_words = (uint32_t)t.size();
      tpair.insert(tpair.end(), t.begin(), t.end());
    }
  }
  // wave-kernel layout of the same query: rows padded to 64K; queries past 1024 rows run as
  // 1024-row segments (K = 16), one table per segment, concatenated
  const auto wave_tables = [&](int wrows, int nsegs, std::vector<uint32_t>& wt,
                               std::vector<uint32_t>& wt16) {
    for (int sg = 0; sg < nsegs; ++sg) {
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
          wt16.resize(b16 + wrows, 0xBCBCBCBCu);  // rows past the query: -2048
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
        std::vector<uint8_t> qp((size_t)(A + 1) * wrows, 0xFF);
        for (int c = 0; c < A; ++c)
          for (int i = 0; i < nr; ++i)
            qp[(size_t)c * wrows + i] = (uint8_t)(S - m[b->query[r0 + i] * A + c]);
        const size_t base = wt.size();
        wt.resize(base + qp.size() / 4);
        std::memcpy(wt.data() + base, qp.data(), qp.size());
        if (f16) {
          std::vector<uint16_t> q16((size_t)(A + 1) * wrows, 0xBC00u);
          for (int c = 0; c < A; ++c)
            for (int i = 0; i < nr; ++i)
              q16[(size_t)c * wrows + i] = f16_score_bits(m[b->query[r0 + i] * A + c]);
          const size_t b16 = wt16.size();
          wt16.resize(b16 + q16.size() / 2);
          std::memcpy(wt16.data() + b16, q16.data(), q16.size() * 2);
        }
      }
    }
  };
  std::vector<uint32_t> wt, wt16;
  const int wK = qlen <= 256 ? 4 : qlen <= 512 ? 8 : 16;
  const int wrows = 64 * wK;
  const int wsegs = std::max(1, (qlen + wrows - 1) / wrows);
  const uint32_t wPS = prof ? (uint32_t)wrows : 0, wPS16 = prof ? (uint32_t)wrows * 2 : 0;
  wave_tables(wrows, wsegs, wt, wt16);
  // split tail of the wave kernel (one segment, K >= 8): the query as P = 2, 4 and 8 segments
  // of K/P rows per lane, tables concatenated like the segments above
  std::vector<uint32_t> st[3], st16[3];
  int sK[3] = {0, 0, 0};
  for (int i = 0; i < 3; ++i) {
    sK[i] = (wsegs == 1 && wK >= 8) ? wK / (2 << i) : 0;
    if (sK[i]) wave_tables(64 * sK[i], 2 << i, st[i], st16[i]);
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
  const size_t nbytes =
      (wt16.size() + wt.size() + st16[0].size() + st[0].size() + st16[1].size() +
       st[1].size() + st16[2].size() + st[2].size() + tab.size() + tab16.size() + tpair.size()) *
      4;
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
  for (int i = 0; i < 3; ++i) {
    if (!st16[i].empty()) HIPOK(b, upload(b->stab16[i], st16[i]));
    HIPOK(b, upload(b->stab[i], st[i]));
    b->sK[i] = sK[i];
    b->sseg_words[i] = st[i].size() / (2 << i);
    b->sseg_words16[i] = st16[i].size() / (2 << i);
    b->sPS[i] = prof ? (uint32_t)(64 * sK[i]) : 0;
    b->sPS16[i] = prof ? (uint32_t)(128 * sK[i]) : 0;
  }
  HIPOK(b, upload(b->qtab, tab));
  if (f16) HIPOK(b, upload(b->qtab16, tab16));
  if (!tpair.empty()) HIPOK(b, upload(b->qpair, tpair));
  b->pair_bytes = pair_words * 4;  // one segment's table
  b->pS1 = pS1;
  b->pS2 = pS2;
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
  b->i32_ready = false;
  b->mq_ready = false;
  b->dirty = false;
  return SW_OK;
}

// Row-LUT tables of every query of a set in the segment layout of the longest one (prepare()
// ran on it): query i's words at i * mq_words, rows past its end padding (u16 0xFF: S - 255,
// f16 0xBC: -2048, as in prepare()).  LUT mode only (DNA matrices without the column-0 rule).
sw_status prepare_multi(sw_bank* b) {
  if (b->mq_ready) return SW_OK;
  const int A = b->alpha;
  const int8_t* m = b->matrix.data();
  const int R = b->R, S = (int)b->S;
  const size_t words = b->segs.back().off + (size_t)b->segs.back().W * R;
  const int seg_rows = b->segs[0].W * R;
  const size_t nq = b->qset.size();
  std::vector<uint32_t> t16, t8(nq * words, 0xFFFFFFFFu);
  if (b->f16) t16.assign(nq * words, 0xBCBCBCBCu);
  for (size_t i = 0; i < nq; ++i) {
    const std::vector<uint8_t>& qi = b->qset[i];
    for (size_t sg = 0; sg < b->segs.size(); ++sg) {
      const size_t base = i * words + b->segs[sg].off;
      const int r0 = (int)sg * seg_rows;
      for (int j = 0; j < b->segs[sg].W * R && r0 + j < (int)qi.size(); ++j) {
        uint32_t w = 0, h = 0;
        for (int c = 0; c < 4; ++c) {
          const int v = m[qi[r0 + j] * A + c];
          w |= (uint32_t)(uint8_t)(S - v) << (8 * c);
          h |= (uint32_t)(f16_score_bits(v) >> 8) << (8 * c);
        }
        t8[base + j] = w;
        if (b->f16) t16[base + j] = h;
      }
    }
  }
  // letter-pair tables (DNA merged f16 without the column-0 rule), one per (segment, query):
  // 128-row segments (4 waves of 32 rows, 4-column chunks, 4 workgroups per CU whose wave
  // priorities rotate: a 1-kbp query is 8 segments, 7 bottom-row hand-offs through HBM; +11 %
  // against 512-row segments, one workgroup per CU) unless SWBANK_MQ_PAIR_ROWS=256
  // (8 waves, 2 workgroups per CU) or 512 (16 waves)
  std::vector<uint32_t> tp;
  b->mq_pair_segs = 0;
  if (b->f16 && !b->prof && !b->gotoh() && !b->col0 && A == SW_DNA_ALPHA &&
      env_int("SWBANK_MQ_PAIR", 1) != 0) {
    const int want = env_int("SWBANK_MQ_PAIR_ROWS", 128);
    const uint32_t NR = want == 128 ? 128 : want == 256 ? 256 : 512;
    b->mq_pair_rows = (int)NR;
    pair_strides(NR, b->mq_pS1, b->mq_pS2);
    const int qmax = (int)b->query.size();
    b->mq_pair_segs = std::max(1, (qmax + (int)NR - 1) / (int)NR);
    for (int sg = 0; sg < b->mq_pair_segs; ++sg)
      for (size_t i = 0; i < nq; ++i) {
        const std::vector<uint32_t> t = pair_table(b->qset[i].data(), (int)b->qset[i].size(),
                                                   sg * (int)NR, NR, m, A, b->mq_pS1, b->mq_pS2);
        b->mq_pair_words = t.size();
        tp.insert(tp.end(), t.begin(), t.end());
      }
  }
  HIPOK(b, hipSetDevice(b->device));
  HIPOK(b, hipEventSynchronize(b->ev_ready));  // the staging buffer is free again
  HIPOK(b, b->stage.reserve((t8.size() + t16.size() + tp.size()) * 4));
  HIPOK(b, b->mqtab.reserve(t8.size()));
  if (!t16.empty()) HIPOK(b, b->mqtab16.reserve(t16.size()));
  HIPOK(b, hipStreamWaitEvent(b->stream, b->ev_used, 0));
  std::memcpy(b->stage.p, t8.data(), t8.size() * 4);
  HIPOK(b, hipMemcpyAsync(b->mqtab.p, b->stage.p, t8.size() * 4, hipMemcpyHostToDevice,
                          b->stream));
  if (!t16.empty()) {
    std::memcpy(b->stage.p + t8.size() * 4, t16.data(), t16.size() * 4);
    HIPOK(b, hipMemcpyAsync(b->mqtab16.p, b->stage.p + t8.size() * 4, t16.size() * 4,
                            hipMemcpyHostToDevice, b->stream));
  }
  if (!tp.empty()) {
    const size_t at = (t8.size() + t16.size()) * 4;
    HIPOK(b, b->mqpair.reserve(tp.size()));
    std::memcpy(b->stage.p + at, tp.data(), tp.size() * 4);
    HIPOK(b, hipMemcpyAsync(b->mqpair.p, b->stage.p + at, tp.size() * 4, hipMemcpyHostToDevice,
                            b->stream));
  }
  HIPOK(b, hipEventRecord(b->ev_ready, b->stream));
  b->mq_words = words;
  b->mq_ready = true;
  return SW_OK;
}

// int32 re-score state, built on first use per (penalties, query): the per-strip profile of
// swk_launch_i32 ([strip][letter 0..pad][lane] 4 x int16: rows 4l..4l+3 of a 256-row strip;
// letter = min(code, pad) as in the 16-bit kernels, the padding letter scoring S - 255 like
// their padding row), uploaded on the bank stream like the other query tables.
sw_status prepare_i32(sw_bank* b) {
  if (b->i32_ready) return SW_OK;
  const int A = b->alpha;
  const int8_t* m = b->matrix.data();
  const uint32_t qlen = (uint32_t)b->query.size();
  const uint32_t strips = std::max(1u, (qlen + 255) / 256), pad = b->pad;
  if (pad + 1 > 25) return fail(b, SW_ERR_UNSUPPORTED, "int32 kernel: alphabet %d too large", A);
  std::vector<int16_t> h((size_t)strips * (pad + 1) * 64 * 4, 0);
  for (uint32_t s = 0; s < strips; ++s)
    for (uint32_t c = 0; c <= pad; ++c)
      for (uint32_t l = 0; l < 64; ++l)
        for (uint32_t k = 0; k < 4; ++k) {
          const uint32_t r = s * 256 + 4 * l + k;
          int v = 0;
          if (r < qlen) v = c < (uint32_t)A ? m[b->query[r] * A + c] : (int)b->S - 255;
          h[(((size_t)s * (pad + 1) + c) * 64 + l) * 4 + k] = (int16_t)v;
        }
  HIPOK(b, hipSetDevice(b->device));
  HIPOK(b, hipEventSynchronize(b->ev_ready));  // the staging buffer is free again
  HIPOK(b, b->stage.reserve(h.size() * 2));
  HIPOK(b, b->i32prof.reserve(h.size() / 4));
  HIPOK(b, hipStreamWaitEvent(b->stream, b->ev_used, 0));
  std::memcpy(b->stage.p, h.data(), h.size() * 2);
  HIPOK(b, hipMemcpyAsync(b->i32prof.p, b->stage.p, h.size() * 2, hipMemcpyHostToDevice,
                          b->stream));
  HIPOK(b, hipEventRecord(b->ev_ready, b->stream));
  b->i32_strips = strips;
  b->i32_ready = true;
  return SW_OK;
}

extern "C" sw_status sw_bank_set_timing(sw_bank* b, int32_t enable) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (!b) return SW_ERR_ARG;
  if (b->is_multi()) return each_kid(b, [&](sw_bank* k) { return sw_bank_set_timing(k, enable); });
  b->timing = enable != 0;
  return SW_OK;
}

extern "C" sw_status sw_bank_timing(sw_bank* b, uint64_t* launches, double* pack_ms,
                                    double* score_ms) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (!b) return SW_ERR_ARG;
  double p = 0, s = 0;
  uint64_t n = 0;
  sw_status st = SW_OK;
  if (b->is_multi()) {  // summed over the devices
    for (sw_bank* k : b->kids) {
      uint64_t kn = 0;
      double kp = 0, ks = 0;
      if ((st = sw_bank_timing(k, &kn, &kp, &ks)) != SW_OK)
        return fail(b, st, "device %d: %s", k->device, k->err);
      n += kn;
      p += kp;
      s += ks;
    }
    if (launches) *launches = n;
    if (pack_ms) *pack_ms = p;
    if (score_ms) *score_ms = s;
    return SW_OK;
  }
  for (auto& ev : b->events) {  // (b == a: the launch had no separate pack interval)
    float t1 = 0, t2 = 0;
    if (st == SW_OK && hipEventSynchronize(ev.c) == hipSuccess &&
        (ev.b == ev.a || hipEventElapsedTime(&t1, ev.a, ev.b) == hipSuccess) &&
        hipEventElapsedTime(&t2, ev.b, ev.c) == hipSuccess) {
      p += t1;
      s += t2;
      ++n;
    } else {
      st = fail(b, SW_ERR_HIP, "event timing failed");
    }
    (void)hipEventDestroy(ev.a);
    if (ev.b != ev.a) (void)hipEventDestroy(ev.b);
    (void)hipEventDestroy(ev.c);
  }
  b->events.clear();
  p += b->host_pack_ms;  // host calls: the feeder's gather / pack time on the host
  b->host_pack_ms = 0;
  if (launches) *launches = n;
  if (pack_ms) *pack_ms = p;
  if (score_ms) *score_ms = s;
  // the launches timed are complete: a device call's latched hand-off fault surfaces here
  if (st == SW_OK && n > 0) st = take_fault(b, 0);
  return st;
}

extern "C" sw_status sw_best_hit_device(sw_bank* b, const int32_t* d_scores, const uint64_t* d_ids,
                                        size_t n, uint64_t* d_out, void* stream) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (!b) return SW_ERR_ARG;
  if (b->is_multi())  // on the root device, where the multi-device calls leave the scores
    return sw_best_hit_device(b->kids[0], d_scores, d_ids, n, d_out,
                              stream ? stream : b->kids[0]->stream);
  if (!d_scores || !d_out || n == 0 || n > 0xFFFFFFFFull)
    return fail(b, SW_ERR_ARG, "sw_best_hit_device: empty, null or > 2^32 scores");
  HIPOK(b, hipSetDevice(b->device));
  HIPOK(b, b->best_key.reserve(1));
  HIPOK(b, swk_best_hit(d_scores, d_ids, n, b->best_key.p, d_out, nullptr,
                        stream ? reinterpret_cast<hipStream_t>(stream) : b->stream));
  return SW_OK;
}

extern "C" sw_status sw_best_hit(sw_bank* b, const int32_t* scores, const uint64_t* ids, size_t n,
                                 uint64_t* best_id, int32_t* best_score) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (!scores || !best_id || !best_score || n == 0)
    return b ? fail(b, SW_ERR_ARG, "sw_best_hit: empty or null input") : SW_ERR_ARG;
  size_t bi = 0;
  for (size_t k = 1; k < n; ++k)
    if (scores[k] > scores[bi]) bi = k;
  *best_id = ids ? ids[bi] : (uint64_t)bi;
  *best_score = scores[bi];
  return SW_OK;
}

