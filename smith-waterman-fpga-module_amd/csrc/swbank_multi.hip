// swbank_multi.hip — multi-device banks: one child bank per device, the RCCL score gather.
// 
// SURVEY §8 e: pairs shard with no data-path collective; one ncclGather (rccl.h:745) over
// communicators from ncclCommInitAll (rccl.h:236); librccl is dlopen-ed on first use.
#include "swbank_bank.h"

// RCCL for the multi-device score gather (SURVEY §8 e: ncclCommInitAll, rccl.h:236, and
// ncclGather, rccl.h:745).  Loaded on first use so single-device users never map it; in a
// process where PyTorch already mapped its librccl.so.1 that copy is reused (same SONAME).
const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      snprintf(r.err, sizeof(r.err), "dlopen librccl.so.1: %s", dlerror());
      return;
    }
    r.commInitAll = reinterpret_cast<decltype(&ncclCommInitAll)>(dlsym(h, "ncclCommInitAll"));
    r.commDestroy = reinterpret_cast<decltype(&ncclCommDestroy)>(dlsym(h, "ncclCommDestroy"));
    r.gather = reinterpret_cast<decltype(&ncclGather)>(dlsym(h, "ncclGather"));
    r.errorString = reinterpret_cast<decltype(&ncclGetErrorString)>(dlsym(h, "ncclGetErrorString"));
    r.commAbort = reinterpret_cast<decltype(&ncclCommAbort)>(dlsym(h, "ncclCommAbort"));
    r.asyncError =
        reinterpret_cast<decltype(&ncclCommGetAsyncError)>(dlsym(h, "ncclCommGetAsyncError"));
    r.groupStart = reinterpret_cast<decltype(&ncclGroupStart)>(dlsym(h, "ncclGroupStart"));
    r.groupEnd = reinterpret_cast<decltype(&ncclGroupEnd)>(dlsym(h, "ncclGroupEnd"));
    r.ok = r.commInitAll && r.commDestroy && r.gather && r.errorString && r.commAbort &&
           r.asyncError && r.groupStart && r.groupEnd;
    if (!r.ok)
      snprintf(r.err, sizeof(r.err),
               "librccl.so.1 lacks ncclCommInitAll/ncclGather/ncclCommAbort/ncclCommGetAsyncError");
  });
  return r;
}

// ---- multi-device banks (≙ MODULES ScoringModules behind the PrioEncoder,
//      ScoreBank_v2.v:76-148; SURVEY §8 e) ---------------------------------------------------
// A batch is dealt over the child banks (phase 1: every device scores its share, scores stay on
// the device), then gathered on the first device (phase 2: one ncclGather of equal, padded
// counts over RCCL/xGMI, or device copies), copied back once and scattered to input order on
// the host.  The collective is issued only after every share was accepted, so a bad input on
// one device cannot leave the others blocked inside the gather.
template <class FeedF>
static sw_status multi_gather(sw_bank* b, const std::vector<size_t>& cnt, FeedF feed_kid) {
  const size_t D = b->kids.size();
  const size_t cmax = *std::max_element(cnt.begin(), cnt.end());
  // A device call before this one (multi_device, asynchronous) may still read grecv (its
  // scatter) or a child's scores (its copy-out): its ev_used follows both.
  if (b->ev_used) {
    HIPOK(b, hipSetDevice(b->device));
    HIPOK(b, hipEventSynchronize(b->ev_used));
  }
  for (size_t d = 0; d < D; ++d) {  // padded send buffers, sized before any score lands
    sw_bank* k = b->kids[d];
    HIPOK(b, hipSetDevice(k->device));
    HIPOK(b, k->scores.reserve(std::max<size_t>(cmax, 1)));
  }
  std::vector<sw_status> st(D, SW_OK);
  b->dpool->run([&](unsigned d) {
    sw_bank* k = b->kids[d];
    if (hipSetDevice(k->device) != hipSuccess) st[d] = SW_ERR_HIP;
    else if (cnt[d]) st[d] = feed_kid(d);
  });
  for (size_t d = 0; d < D; ++d)
    if (st[d] != SW_OK) {
      for (sw_bank* k : b->kids) {
        (void)hipSetDevice(k->device);
        (void)hipStreamSynchronize(k->stream);
      }
      (void)hipSetDevice(b->device);
      return fail(b, st[d], "device %d: %s", b->kids[d]->device, b->kids[d]->err);
    }
  sw_bank* root = b->kids[0];
  HIPOK(b, hipSetDevice(root->device));
  HIPOK(b, b->grecv.reserve(D * cmax));
  HIPOK(b, b->hrecv.reserve(D * cmax * 4));
  const Rccl& r = rccl();
  if (b->rccl_gather && b->comms.empty()) {  // re-created after an aborted gather
    std::vector<ncclComm_t> comms(D);
    std::vector<int> devs(D);
    for (size_t d = 0; d < D; ++d) devs[d] = b->kids[d]->device;
    const ncclResult_t nr = r.commInitAll(comms.data(), (int)D, devs.data());
    if (nr != ncclSuccess)
      return fail(b, SW_ERR_HIP, "ncclCommInitAll after an aborted gather: %s", r.errorString(nr));
    b->comms.assign(comms.begin(), comms.end());
    HIPOK(b, hipSetDevice(root->device));
  }
  if (!b->comms.empty()) {
    // One host thread per device issues its ncclGather and then watches it: done, an async
    // RCCL error, a failure on another device, or SWBANK_GATHER_TIMEOUT_MS (default 60 s)
    // without completion.  Any of the latter aborts every communicator (ncclCommAbort ends the
    // collective kernels still waiting for a peer), the call fails with SW_ERR_HIP, and the next
    // call creates the communicators again, so a device that dropped out of one gather does not
    // leave the others blocked or the bank unusable.  (SWBANK_GATHER_FAULT=d, tests: device d
    // reports a failure instead of joining the gather.)
    const int timeout_ms = std::max(1, env_int("SWBANK_GATHER_TIMEOUT_MS", 60000));
    const int fault_dev = env_int("SWBANK_GATHER_FAULT", -1);
    std::vector<int> nst(D, 0);  // 0 ok, > 0 ncclResult_t, -1 HIP, -2 timeout, -3 peer failed
    std::atomic<bool> failed{false};
    b->dpool->run([&](unsigned d) {
      sw_bank* k = b->kids[d];
      const ncclComm_t comm = static_cast<ncclComm_t>(b->comms[d]);
      if (hipSetDevice(k->device) != hipSuccess || (int)d == fault_dev) {
        nst[d] = -1;
        failed = true;
        return;
      }
      const ncclResult_t e = r.gather(k->scores.p, d == 0 ? b->grecv.p : nullptr, cmax, ncclInt32, 0,
                                      comm, k->stream);
      if (e != ncclSuccess) {
        nst[d] = (int)e;
        failed = true;
        return;
      }
      const auto t0 = std::chrono::steady_clock::now();
      for (unsigned it = 0;; ++it) {
        const hipError_t q = hipStreamQuery(k->stream);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) {
          nst[d] = -1;
          break;
        }
        ncclResult_t ae = ncclSuccess;
        if (r.asyncError(comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
          nst[d] = (int)ae;
          break;
        }
        if (failed.load()) {
          nst[d] = -3;
          break;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) {
          nst[d] = -2;
          break;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(it < 1000 ? 20 : 500));
      }
      failed = true;
    });
    if (failed.load()) {
      bool timed_out = false;
      for (size_t d = 0; d < D; ++d) timed_out |= nst[d] == -2;
      for (size_t d = 0; d < D; ++d) {
        (void)hipSetDevice(b->kids[d]->device);
        (void)r.commAbort(static_cast<ncclComm_t>(b->comms[d]));
      }
      b->comms.clear();
      for (sw_bank* k : b->kids) {  // the aborted collectives have left the streams
        (void)hipSetDevice(k->device);
        (void)hipStreamSynchronize(k->stream);
        (void)hipGetLastError();
      }
      (void)hipSetDevice(b->device);
      if (timed_out) ++b->ctr.gather_timeouts;
      size_t d0 = 0;
      while (d0 + 1 < D && nst[d0] == 0) ++d0;
      for (size_t d = 0; d < D; ++d)  // the first device that failed on its own, not by a peer
        if (nst[d] != 0 && nst[d] != -3) {
          d0 = d;
          break;
        }
      return fail(b, SW_ERR_HIP, "ncclGather on device %d failed (%s); communicators aborted",
                  b->kids[d0]->device,
                  nst[d0] > 0    ? r.errorString((ncclResult_t)nst[d0])
                  : nst[d0] == -2 ? "timed out (SWBANK_GATHER_TIMEOUT_MS)"
                                  : "HIP or device fault");
    }
    HIPOK(b, hipSetDevice(root->device));
  } else {
    for (size_t d = 0; d < D; ++d) {
      sw_bank* k = b->kids[d];
      if (!cnt[d]) continue;
      HIPOK(b, hipSetDevice(k->device));
      HIPOK(b, hipMemcpyPeerAsync(b->grecv.p + d * cmax, root->device, k->scores.p, k->device,
                                  cnt[d] * 4, k->stream));
      HIPOK(b, hipStreamSynchronize(k->stream));
    }
    HIPOK(b, hipSetDevice(root->device));
  }
  HIPOK(b, hipMemcpyAsync(b->hrecv.p, b->grecv.p, D * cmax * 4, hipMemcpyDeviceToHost,
                          root->stream));
  HIPOK(b, hipStreamSynchronize(root->stream));
  copy_kernel_name(b, b->comms.empty() ? "copy" : "rccl");
  return SW_OK;
}

// The lowest index with the maximum score over scores[0, n), in parallel on the pool.
static void host_best(sw_bank* b, const int32_t* scores, size_t n) {
  const unsigned T = b->pool->size();
  std::vector<size_t> pi(T, SIZE_MAX);
  const size_t step = (n + T - 1) / T;
  b->pool->run([&](unsigned p) {
    const size_t lo = std::min(n, p * step), hi = std::min(n, lo + step);
    size_t bi = lo;
    for (size_t k = lo + 1; k < hi; ++k)
      if (scores[k] > scores[bi]) bi = k;
    if (lo < hi) pi[p] = bi;
  });
  size_t bi = SIZE_MAX;
  for (size_t x : pi)
    if (x != SIZE_MAX && (bi == SIZE_MAX || scores[x] > scores[bi])) bi = x;
  b->best_index = bi;
  b->best_id = bi;
  b->best_score = scores[bi];
  b->best_kind = 1;
  b->best_root = false;
}

sw_status multi_batch(sw_bank* b, const uint8_t* residues, size_t nres,
                             const uint64_t* offsets, const uint32_t* lens, size_t n,
                             int32_t* scores_out) {
  const size_t D = b->kids.size();
  // length-balanced deal (SURVEY §8 e): longest first, round robin -> each device gets every
  // D-th target of the sorted order, itself already longest first (its feeder skips the sort)
  std::vector<uint32_t> order(n);
  if (!chunk_perm(*b->pool, lens, n, order.data())) std::iota(order.begin(), order.end(), 0u);
  std::vector<size_t> cnt(D);
  for (size_t d = 0; d < D; ++d) cnt[d] = n > d ? (n - d + D - 1) / D : 0;
  std::vector<std::vector<uint64_t>> offs(D);
  std::vector<std::vector<uint32_t>> lns(D), idx(D);
  for (size_t d = 0; d < D; ++d) {
    offs[d].resize(cnt[d]);
    lns[d].resize(cnt[d]);
    idx[d].resize(cnt[d]);
  }
  parallel_for(*b->pool, n, [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; ++k) {
      const uint32_t t = order[k];
      const size_t d = k % D, i = k / D;
      idx[d][i] = t;
      offs[d][i] = offsets[t];
      lns[d][i] = lens[t];
    }
  });
  sw_status st = multi_gather(b, cnt, [&](unsigned d) {
    return batch_feed(b->kids[d], residues, nres, offs[d].data(), lns[d].data(), cnt[d], nullptr);
  });
  if (st != SW_OK) return st;
  const size_t cmax = cnt[0];
  const int32_t* hr = reinterpret_cast<const int32_t*>(b->hrecv.p);
  parallel_for(*b->pool, n, [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; ++k) {
      const size_t d = k % D, i = k / D;
      scores_out[idx[d][i]] = hr[d * cmax + i];
    }
  });
  host_best(b, scores_out, n);
  return SW_OK;
}

sw_status multi_records(sw_bank* b, const uint8_t* recs, size_t n, int32_t* scores_out) {
  // records are at most 232 bases: contiguous ranges (no copy of the 64-byte records)
  const size_t D = b->kids.size();
  std::vector<size_t> cnt(D), first(D);
  for (size_t d = 0; d < D; ++d) {
    first[d] = n * d / D;
    cnt[d] = n * (d + 1) / D - first[d];
  }
  sw_status st = multi_gather(b, cnt, [&](unsigned d) {
    return records_feed(b->kids[d], recs + first[d] * SWB_RECORD, cnt[d], nullptr);
  });
  if (st != SW_OK) return st;
  const size_t cmax = *std::max_element(cnt.begin(), cnt.end());
  const int32_t* hr = reinterpret_cast<const int32_t*>(b->hrecv.p);
  for (size_t d = 0; d < D; ++d)
    std::memcpy(scores_out + first[d], hr + d * cmax, cnt[d] * 4);
  host_best(b, scores_out, n);
  return SW_OK;
}

// Targets per chunk of a pipelined deal (multi_device): a share bigger than one round of the tile
// kernel's resident workgroup slots (G x 128 targets, G = swk_bal_slots) is copied and scored in
// chunks of whole rounds, at most SWK_DEAL_PIPE_MAX of them, so chunk p + 1 crosses xGMI while
// chunk p is scored.  A share within one round is latency-bound at one tile's duration, which a
// cut cannot shorten, and a device that is the root itself copies within its own HBM:
// both stay whole.  SWBANK_DEAL_PIPE=0 disables; SWBANK_DEAL_CHUNK=n forces chunks of n targets
// (tests: it also applies to the root's own share; at most 64 chunks).
constexpr size_t SWK_DEAL_PIPE_MAX = 8;
static size_t deal_chunk(sw_bank* k, const sw_bank* root, size_t c) {
  if (env_int("SWBANK_DEAL_PIPE", 1) == 0) return c;
  const int forced = env_int("SWBANK_DEAL_CHUNK", 0);
  if (forced > 0) return std::min(c, std::max((size_t)forced, (c + 63) / 64));  // <= 64 chunks
  if (k->device == root->device) return c;
  const unsigned G = swk_bal_slots(k->segs[0].W, k->pair_bytes, 0);  // (on k's device)
  const size_t round = (size_t)G * SWB_TILE;
  if (!G || c <= round) return c;
  const size_t rounds = (c + round - 1) / round;
  return (rounds + SWK_DEAL_PIPE_MAX - 1) / SWK_DEAL_PIPE_MAX * round;
}

// Device buffers on a multi-device bank (the caller's buffers live on the root device,
// devices[0]; ≙ the ScoreBank's MODULES, each latching its own copy of its target before
// scoring it, ScoreBank_v2.v:117-137, SM_Feeder3.v:104-182).  Every device scores its share
// from its OWN HBM: xGMI carries one bulk copy in and the scores out, never the kernel's reads.
//  1. the visiting order: a ragged batch is sorted longest first on the root (swk_sort_lens),
//     and position p goes to device p % D -- the length-balanced deal of the host path
//     (multi_batch); a batch of one length keeps its order;
//  2. one gather kernel on the root copies each device's targets into its region of a staging
//     buffer at a fixed stride of max_len bytes rounded up to 16 (offsets rebased, lengths kept);
//  3. device d copies its region into its own buffers (hipMemcpyPeerAsync on its stream: codes
//     cnt_d x stride bytes + 12 bytes per target; a 4-bit share of more than one round in
//     chunks on its copy stream, each scored as it lands, deal_chunk), scores them there
//     (launch / launch_set) and copies its nq x cnt_d int32 scores back into the root's
//     receive buffer;
//  4. one scatter kernel on the root writes them to d_scores in input order.
// CAPI records (fixed 64 bytes, contiguous ranges) skip 1, 2 and 4: each device copies its
// range of records and writes its scores straight into the caller's d_scores.
// Asynchronous: the devices' work waits for the caller's stream (an event after the gather),
// the caller's stream waits for every device (an event each) before the scatter; the next call
// reuses the staging buffers only after this call's scatter (ev_done).  A device listed twice,
// or the root itself, copies within its own memory.  With d_ids the batch best hit is tracked on
// the root after the scatter (sw_batch_best).
sw_status multi_device(sw_bank* b, const uint8_t* d_res, const uint64_t* d_offs,
                       const uint32_t* d_lens, const uint64_t* d_ids, size_t n, uint32_t min_len,
                       uint32_t max_len, int32_t* d_scores, hipStream_t hs, bool records) {
  const size_t D = b->kids.size();
  sw_bank* root = b->kids[0];
  const bool set = b->qset.size() > 1;
  const size_t nq = set ? b->qset.size() : 1;
  if (D > SWK_DEAL_MAX) return fail(b, SW_ERR_UNSUPPORTED, "more than %d devices", SWK_DEAL_MAX);
  if (n > 0xFFFFFFFFull) return fail(b, SW_ERR_RANGE, "multi-device device batches hold < 2^32 targets");
  if (!b->peer_ready) {  // direct xGMI copies (without: staged through the host by the runtime)
    for (sw_bank* k : b->kids) {
      if (k->device == root->device) continue;
      int can = 0;
      HIPOK(b, hipDeviceCanAccessPeer(&can, k->device, root->device));
      if (!can) continue;
      HIPOK(b, hipSetDevice(k->device));
      const hipError_t e = hipDeviceEnablePeerAccess(root->device, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
        return fail(b, SW_ERR_HIP, "hipDeviceEnablePeerAccess(%d -> %d): %s", k->device,
                    root->device, hipGetErrorString(e));
      (void)hipGetLastError();
    }
    b->peer_ready = true;
  }
  HIPOK(b, hipSetDevice(root->device));
  if (!hs) hs = root->stream;
  if (!b->ev_join) HIPOK(b, hipEventCreateWithFlags(&b->ev_join, hipEventDisableTiming));
  if (!b->ev_used) HIPOK(b, hipEventCreateWithFlags(&b->ev_used, hipEventDisableTiming));
  else HIPOK(b, hipStreamWaitEvent(hs, b->ev_used, 0));  // the previous call's scatter is done
  // shares: round robin over the visiting order (records: contiguous ranges)
  std::vector<size_t> cnt(D), lo(D, 0);
  for (size_t d = 0; d < D; ++d) {
    if (records) {
      lo[d] = n * d / D;
      cnt[d] = n * (d + 1) / D - lo[d];
    } else {
      cnt[d] = n > d ? (n - d + D - 1) / D : 0;
    }
  }
  // DNA shares cross xGMI as 4-bit codes (SWK_PACK_NIBBLE: half the bytes of the copy that
  // bounds this path, §7 of DESIGN); query sets and other alphabets as bytes.
  // SWBANK_DEAL_NIB=0 keeps bytes.
  const bool nib = !records && !set && b->alpha <= 16 && env_int("SWBANK_DEAL_NIB", 1) != 0;
  // (a 16-byte multiple: the deal gather stores whole 8-code chunks, not bytes)
  const size_t stride = records ? SWB_RECORD
                        : nib   ? align16(((size_t)std::max<uint32_t>(max_len, 1u) + 7) / 8 * 4)
                                : align16(std::max<uint32_t>(max_len, 1u));
  SwkDeal dl{};
  dl.D = (unsigned)D;
  dl.stride = (unsigned)stride;
  dl.nib = nib ? 1u : 0u;
  const uint32_t *perm = nullptr, *ident = nullptr;
  if (!records) {
    // 1. longest first (the sort's scratch zeroes itself; zeroed once here)
    if (n > 1 && min_len < max_len && env_int("SWBANK_DSORT", 1) != 0) {
      HIPOK(b, b->dperm.reserve(n + 2));
      const size_t sw = swk_sort_scratch_bytes() / 4;
      if (b->dsort.cap < sw) {
        HIPOK(b, b->dsort.reserve(sw));
        HIPOK(b, hipMemsetAsync(b->dsort.p, 0, sw * 4, hs));
      }
      HIPOK(b, swk_sort_lens(d_lens, n, max_len, b->dperm.p, b->dperm.p + n, b->dperm.p + n + 1,
                             b->dsort.p, hs));
      ++b->ctr.device_sorts;
      perm = b->dperm.p;
      ident = b->dperm.p + n + 1;
    }
    // 2. the staging regions on the root, then the gather
    HIPOK(b, b->res.reserve(n * stride + 16));
    HIPOK(b, b->offs.reserve(n));
    HIPOK(b, b->lens.reserve(n));
    HIPOK(b, b->grecv.reserve(n * nq));
    size_t at = 0;
    for (size_t d = 0; d < D; ++d) {
      dl.codes[d] = b->res.p + at * stride;
      dl.offs[d] = reinterpret_cast<unsigned long long*>(b->offs.p + at);
      dl.lens[d] = b->lens.p + at;
      dl.scores[d] = b->grecv.p + at * nq;
      dl.cnt[d] = cnt[d];
      at += cnt[d];
    }
    HIPOK(b, swk_deal_gather(d_res, d_offs, d_lens, perm, ident, n, &dl, hs));
  }
  HIPOK(b, hipEventRecord(b->ev_join, hs));  // the inputs (and the staging) are ready
  // 3. every device: its share in, scored in its own HBM, scores out
  sw_status st = SW_OK;
  std::vector<bool> launched(D, false);
  size_t pipe = 1;  // the most chunks a share was cut into
  for (size_t d = 0; d < D && st == SW_OK; ++d) {
    sw_bank* k = b->kids[d];
    const size_t c = cnt[d];
    if (!c) continue;
    if ((st = prepare(k)) != SW_OK) break;
    const auto hip = [&](hipError_t e, const char* what) {
      if (e != hipSuccess && st == SW_OK)
        st = fail(k, SW_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
      return st == SW_OK;
    };
    if (!hip(hipSetDevice(k->device), "hipSetDevice")) break;
    if (!k->ev_join && !hip(hipEventCreateWithFlags(&k->ev_join, hipEventDisableTiming), "event"))
      break;
    const hipStream_t ks = k->stream;
    if (!hip(hipStreamWaitEvent(ks, b->ev_join, 0), "stream wait")) break;
    // the bank's own buffers: its previous launch is done with them (launch waits for ev_used,
    // the copies below must too)
    if (!hip(hipStreamWaitEvent(ks, k->ev_used, 0), "stream wait")) break;
    if (!hip(k->res.reserve(c * stride + 16), "device buffer") ||
        !hip(k->offs.reserve(c), "device buffer") || !hip(k->lens.reserve(c), "device buffer") ||
        !hip(k->scores.reserve(c * nq), "device buffer"))
      break;
    launched[d] = true;
    if (records) {
      if (!hip(hipMemcpyPeerAsync(k->res.p, k->device, d_res + lo[d] * SWB_RECORD, root->device,
                                  c * SWB_RECORD, ks), "records in"))
        break;
      st = launch(k, k->res.p, nullptr, nullptr, c, SWB_RECORD_MAX, k->scores.p, ks,
                  SWK_PACK_RECORDS);
      if (st == SW_OK &&
          hip(hipMemcpyPeerAsync(d_scores + lo[d], root->device, k->scores.p, k->device, c * 4,
                                 ks), "scores out"))
        (void)hip(hipEventRecord(k->ev_used, ks), "event");  // the copy-out read k->scores
    } else if (const size_t chunk = nib ? deal_chunk(k, root, c) : c; chunk < c) {
      // pipelined: chunk p + 1 crosses xGMI on the copy stream while chunk p is scored on ks.
      // The share is longest first already (positions d, d + D, ... of the sorted order), so
      // the chunks launch without a sort of their own.
      const hipStream_t cs = k->copy_stream;
      const size_t P = (c + chunk - 1) / chunk;
      if (!hip(hipStreamWaitEvent(cs, b->ev_join, 0), "stream wait") ||
          !hip(hipStreamWaitEvent(cs, k->ev_used, 0), "stream wait"))
        break;
      while (k->deal_ev.size() < P && st == SW_OK) {
        hipEvent_t e = nullptr;
        if (hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event")) k->deal_ev.push_back(e);
      }
      size_t copied = 0;  // chunks whose copies are enqueued (and their event recorded)
      for (; copied < P && st == SW_OK; ++copied) {
        const size_t c0 = copied * chunk, cc = std::min(chunk, c - c0);
        if (!hip(hipMemcpyPeerAsync(k->res.p + c0 * stride, k->device, dl.codes[d] + c0 * stride,
                                    root->device, cc * stride, cs), "codes in") ||
            !hip(hipMemcpyPeerAsync(k->offs.p + c0, k->device, dl.offs[d] + c0, root->device,
                                    cc * 8, cs), "offsets in") ||
            !hip(hipMemcpyPeerAsync(k->lens.p + c0, k->device, dl.lens[d] + c0, root->device,
                                    cc * 4, cs), "lengths in") ||
            !hip(hipEventRecord(k->deal_ev[copied], cs), "event"))
          break;
      }
      for (size_t p = 0; p < copied && st == SW_OK; ++p) {
        const size_t c0 = p * chunk, cc = std::min(chunk, c - c0);
        if (!hip(hipStreamWaitEvent(ks, k->deal_ev[p], 0), "stream wait")) break;
        st = launch(k, k->res.p, k->offs.p + c0, k->lens.p + c0, cc, max_len, k->scores.p + c0,
                    ks, SWK_PACK_NIBBLE, nullptr, nullptr, false, true, nullptr, nullptr, 0, 0,
                    min_len);
      }
      // (after a failure too: nothing on ks may run ahead of copies still reading the staging)
      if (copied) (void)hipStreamWaitEvent(ks, k->deal_ev[copied - 1], 0);
      pipe = std::max(pipe, P);
      if (st == SW_OK &&
          hip(hipMemcpyPeerAsync(const_cast<int*>(dl.scores[d]), root->device, k->scores.p,
                                 k->device, c * 4, ks), "scores out"))
        (void)hip(hipEventRecord(k->ev_used, ks), "event");  // the copy-out read k->scores
    } else {
      if (!hip(hipMemcpyPeerAsync(k->res.p, k->device, dl.codes[d], root->device, c * stride, ks),
               "codes in") ||
          !hip(hipMemcpyPeerAsync(k->offs.p, k->device, dl.offs[d], root->device, c * 8, ks),
               "offsets in") ||
          !hip(hipMemcpyPeerAsync(k->lens.p, k->device, dl.lens[d], root->device, c * 4, ks),
               "lengths in"))
        break;
      st = set ? launch_set(k, k->res.p, k->offs.p, k->lens.p, c, min_len, max_len, k->scores.p,
                            ks, c)
               : launch(k, k->res.p, k->offs.p, k->lens.p, c, max_len, k->scores.p, ks,
                        nib ? SWK_PACK_NIBBLE : SWK_PACK_BYTES, nullptr, nullptr, true, true,
                        nullptr, nullptr, 0, 0, min_len);
      if (st == SW_OK &&
          hip(hipMemcpyPeerAsync(const_cast<int*>(dl.scores[d]), root->device, k->scores.p,
                                 k->device, c * nq * 4, ks), "scores out"))
        (void)hip(hipEventRecord(k->ev_used, ks), "event");  // the copy-out read k->scores
    }
  }
  // (recorded even after a failure: the caller's stream must not run ahead of what was enqueued)
  for (size_t d = 0; d < D; ++d) {
    if (!launched[d]) continue;
    sw_bank* k = b->kids[d];
    (void)hipSetDevice(k->device);
    if (hipEventRecord(k->ev_join, k->stream) == hipSuccess) {
      (void)hipSetDevice(root->device);
      HIPOK(b, hipStreamWaitEvent(hs, k->ev_join, 0));
    }
  }
  HIPOK(b, hipSetDevice(root->device));
  if (st != SW_OK) {
    (void)hipEventRecord(b->ev_used, hs);
    for (sw_bank* k : b->kids)
      if (k->err[0]) return fail(b, st, "device %d: %s", k->device, k->err);
    return st;
  }
  // 4. scores to input order (query-major rows n apart for a set)
  if (!records) HIPOK(b, swk_deal_scatter(perm, ident, n, (unsigned)nq, n, &dl, d_scores, hs));
  HIPOK(b, hipEventRecord(b->ev_used, hs));
  char pl[32] = "";
  if (pipe > 1) snprintf(pl, sizeof(pl), " pipelined x%zu", pipe);
  snprintf(b->last_kernel, sizeof(b->last_kernel), "multi[%zu] device deal%s%s%s: %s", D,
           perm ? " longest-first" : "", nib ? " 4-bit" : "", pl, root->last_kernel);
  if (d_ids && !records) {
    if ((st = track_best_device(root, d_scores, d_ids, n, hs)) != SW_OK)
      return fail(b, st, "device %d: %s", root->device, root->err);
    b->best_root = true;
  }
  return SW_OK;
}

// ABI 6: every device scores a batch that already lives in its own HBM (≙ each ScoringModule's
// feeder latching its own targets, ScoreBank_v2.v:117-137, SM_Feeder3.v:104-182): no target byte
// crosses xGMI, only the int32 scores -- north_star's "RCCL over xGMI only to gather the final
// score vector".  Device d scores batches[d] on its stream into its padded send buffer (nq rows of
// cmax = max_d n_d words), copies them to batches[d].d_scores when given, and the send buffers are
// gathered to the root: one ncclGather (grouped, issued from this thread) into grecv when the
// devices are distinct, then one 2-D copy per device into d_gathered on the caller's stream
// (query-major over the concatenated batch, N = sum n_d: query i, device d, target k at
// d_gathered[i * N + off_d + k]); a device listed twice copies its rows with hipMemcpyPeerAsync.
// Asynchronous: each device's work is ordered after the previous call's readers of the shared
// buffers (ev_used) and the caller's stream after every device's work.
sw_status multi_resident(sw_bank* b, const sw_device_batch* per, int32_t* d_gathered,
                         hipStream_t hs) {
  const size_t D = b->kids.size();
  sw_bank* root = b->kids[0];
  const bool set = b->qset.size() > 1;
  const size_t nq = set ? b->qset.size() : 1;
  size_t N = 0, cmax = 1;
  std::vector<size_t> off(D);
  for (size_t d = 0; d < D; ++d) {
    off[d] = N;
    N += per[d].n;
    cmax = std::max(cmax, per[d].n);
  }
  HIPOK(b, hipSetDevice(root->device));
  if (!hs) hs = root->stream;
  if (!b->ev_join) HIPOK(b, hipEventCreateWithFlags(&b->ev_join, hipEventDisableTiming));
  const bool first = !b->ev_used;
  if (first) HIPOK(b, hipEventCreateWithFlags(&b->ev_used, hipEventDisableTiming));
  const bool use_rccl = d_gathered && !b->comms.empty();
  if (use_rccl) HIPOK(b, b->grecv.reserve(D * nq * cmax));
  // 1. every device scores its own batch (its own length sort and balanced ranges included)
  std::vector<hipStream_t> ks(D, nullptr);
  sw_status st = SW_OK;
  for (sw_bank* k : b->kids) k->err[0] = 0;
  for (size_t d = 0; d < D && st == SW_OK; ++d) {
    sw_bank* k = b->kids[d];
    const sw_device_batch& bt = per[d];
    if ((st = prepare(k)) != SW_OK) break;
    const auto hip = [&](hipError_t e, const char* what) {
      if (e != hipSuccess && st == SW_OK)
        st = fail(k, SW_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
      return st == SW_OK;
    };
    if (!hip(hipSetDevice(k->device), "hipSetDevice")) break;
    ks[d] = bt.stream ? reinterpret_cast<hipStream_t>(bt.stream) : k->stream;
    if (!k->ev_join && !hip(hipEventCreateWithFlags(&k->ev_join, hipEventDisableTiming), "event"))
      break;
    // the previous device call's gather / scatter read this device's send buffer and grecv
    if (!first && !hip(hipStreamWaitEvent(ks[d], b->ev_used, 0), "stream wait")) break;
    if (!hip(k->scores.reserve(nq * cmax), "device buffer")) break;
    if (bt.n) {
      st = set ? launch_set(k, bt.d_residues, bt.d_offsets, bt.d_lens, bt.n, bt.min_len,
                            bt.max_len, k->scores.p, ks[d], cmax)
               : launch(k, bt.d_residues, bt.d_offsets, bt.d_lens, bt.n, bt.max_len, k->scores.p,
                        ks[d], SWK_PACK_BYTES, nullptr, nullptr, true, true, nullptr, nullptr, 0,
                        0, bt.min_len);
      if (st == SW_OK && bt.d_scores)
        (void)hip(hipMemcpy2DAsync(bt.d_scores, bt.n * 4, k->scores.p, cmax * 4, bt.n * 4, nq,
                                   hipMemcpyDeviceToDevice, ks[d]),
                  "scores to the device's own buffer");
    }
  }
  // 2. the gather of the int32 scores to the root
  const Rccl& r = rccl();
  if (st == SW_OK && use_rccl) {
    ncclResult_t e = r.groupStart();
    for (size_t d = 0; d < D && e == ncclSuccess; ++d)
      e = r.gather(b->kids[d]->scores.p, d == 0 ? b->grecv.p : nullptr, nq * cmax, ncclInt32, 0,
                   static_cast<ncclComm_t>(b->comms[d]), ks[d]);
    const ncclResult_t e2 = r.groupEnd();
    if (e == ncclSuccess) e = e2;
    if (e != ncclSuccess) {  // the communicators are re-created by the next host call
      for (size_t d = 0; d < D; ++d) {
        (void)hipSetDevice(b->kids[d]->device);
        (void)r.commAbort(static_cast<ncclComm_t>(b->comms[d]));
      }
      b->comms.clear();
      st = fail(b, SW_ERR_HIP, "ncclGather of the resident scores: %s", r.errorString(e));
    }
  } else if (st == SW_OK && d_gathered) {
    for (size_t d = 0; d < D && st == SW_OK; ++d) {
      sw_bank* k = b->kids[d];
      if (!per[d].n) continue;
      HIPOK(b, hipSetDevice(k->device));
      for (size_t i = 0; i < nq; ++i)
        HIPOK(b, hipMemcpyPeerAsync(d_gathered + i * N + off[d], root->device,
                                    k->scores.p + i * cmax, k->device, per[d].n * 4, ks[d]));
    }
  }
  // 3. the caller's stream after every device's work (recorded even after a failure: the
  //    caller's stream must not run ahead of what was enqueued)
  for (size_t d = 0; d < D; ++d) {
    sw_bank* k = b->kids[d];
    if (!ks[d]) continue;  // (set once the device's work could be enqueued)
    (void)hipSetDevice(k->device);
    (void)hipEventRecord(k->ev_used, ks[d]);  // the send buffer's readers are done after it
    if (hipEventRecord(k->ev_join, ks[d]) == hipSuccess) {
      (void)hipSetDevice(root->device);
      HIPOK(b, hipStreamWaitEvent(hs, k->ev_join, 0));
    }
  }
  HIPOK(b, hipSetDevice(root->device));
  if (st == SW_OK && use_rccl)
    for (size_t d = 0; d < D; ++d)
      if (per[d].n)
        HIPOK(b, hipMemcpy2DAsync(d_gathered + off[d], N * 4, b->grecv.p + d * nq * cmax,
                                  cmax * 4, per[d].n * 4, nq, hipMemcpyDeviceToDevice, hs));
  HIPOK(b, hipEventRecord(b->ev_used, hs));
  if (st != SW_OK) {
    if (!b->err[0])
      for (sw_bank* k : b->kids)
        if (k->err[0]) return fail(b, st, "device %d: %s", k->device, k->err);
    return st;
  }
  snprintf(b->last_kernel, sizeof(b->last_kernel), "multi[%zu] resident gather=%s: %s", D,
           !d_gathered ? "none" : use_rccl ? "rccl" : "copy", root->last_kernel);
  return SW_OK;
}

extern "C" sw_status sw_score_batch_device_multi(sw_bank* b, const sw_device_batch* batches,
                                                 size_t n_batches, int32_t* d_gathered,
                                                 void* stream) {
  DevGuard dev_guard(b);  // on the bank's device; the caller's is restored on return (ABI 6)
  if (!b || !batches) return SW_ERR_ARG;
  const size_t D = b->is_multi() ? b->kids.size() : 1;
  if (n_batches != D)
    return fail(b, SW_ERR_ARG, "%zu device batches for a bank of %zu devices", n_batches, D);
  b->err[0] = 0;
  b->best_kind = 0;
  b->best_root = false;
  if (const sw_status fs = take_fault(b, 0); fs != SW_OK) return fs;
  size_t N = 0;
  for (size_t d = 0; d < D; ++d) {
    const sw_device_batch& bt = batches[d];
    if (bt.min_len > bt.max_len)
      return fail(b, SW_ERR_ARG, "device batch %zu: min_len %u > max_len %u", d, bt.min_len,
                  bt.max_len);
    if (bt.n > 0xFFFFFFFFull) return fail(b, SW_ERR_RANGE, "device batch %zu: n >= 2^32", d);
    if (bt.n && (!bt.d_residues || !bt.d_offsets || !bt.d_lens))
      return fail(b, SW_ERR_ARG, "device batch %zu: null device buffer", d);
    if (bt.n && !bt.d_scores && !d_gathered)
      return fail(b, SW_ERR_ARG, "device batch %zu: no d_scores and no d_gathered", d);
    N += bt.n;
  }
  if (N > 0xFFFFFFFFull) return fail(b, SW_ERR_RANGE, "more than 2^32 targets");
  if (N == 0) return SW_OK;
  if (b->is_multi()) return multi_resident(b, batches, d_gathered, reinterpret_cast<hipStream_t>(stream));
  // one device: sw_score_batch_device_range on the one batch, its scores in both places asked for
  const sw_device_batch& bt = batches[0];
  hipStream_t hs = stream ? reinterpret_cast<hipStream_t>(stream) : b->stream;
  hipStream_t bs = bt.stream ? reinterpret_cast<hipStream_t>(bt.stream) : b->stream;
  int32_t* out = bt.d_scores ? bt.d_scores : d_gathered;
  sw_status st = sw_score_batch_device_range(b, bt.d_residues, bt.d_offsets, bt.d_lens, nullptr,
                                             bt.n, bt.min_len, bt.max_len, out, bs);
  if (st != SW_OK) return st;
  const size_t nq = b->qset.size() > 1 ? b->qset.size() : 1;
  if (bt.d_scores && d_gathered) {
    if (!b->ev_join) HIPOK(b, hipEventCreateWithFlags(&b->ev_join, hipEventDisableTiming));
    HIPOK(b, hipEventRecord(b->ev_join, bs));
    HIPOK(b, hipStreamWaitEvent(hs, b->ev_join, 0));
    HIPOK(b, hipMemcpyAsync(d_gathered, bt.d_scores, nq * bt.n * 4, hipMemcpyDeviceToDevice, hs));
  } else if (hs != bs) {
    if (!b->ev_join) HIPOK(b, hipEventCreateWithFlags(&b->ev_join, hipEventDisableTiming));
    HIPOK(b, hipEventRecord(b->ev_join, bs));
    HIPOK(b, hipStreamWaitEvent(hs, b->ev_join, 0));
  }
  return SW_OK;
}
