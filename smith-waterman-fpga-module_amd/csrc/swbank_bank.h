// swbank_bank.h — the bank object shared by the C-ABI units of libswbank.so (internal).
//
// Units: swbank_bank.hip (lifecycle, penalties, queries, the query tables), swbank_launch.hip
// (kernel choice and launches, the device-buffer API), swbank_feeder.hip (the chunked
// host-buffer feeder and the host API), swbank_stream.hip (streamed host batches, one kernel
// per call), swbank_multi.hip (multi-device banks and the RCCL gather).
#ifndef SWBANK_BANK_H
#define SWBANK_BANK_H

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: librccl is dlopen-ed by the first multi-device bank

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <numeric>
#include <thread>
#include <chrono>
#include <vector>
#if defined(__SSE2__)
#include <emmintrin.h>
#endif
#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "swbank.h"
#include "swbank_internal.h"
#include "swbank_pack.h"

extern "C" int swk_has_variant(int R, int RB, int col0, int prof, int gotoh, int f16);
extern "C" hipError_t swk_launch_wave(int K, int col0, int prof, int gotoh, int f16,
                                      const void* edge_in, void* edge_out, uint32_t ecols,
                                      int accum, const uint8_t* res,
                                      const uint64_t* offs, const uint32_t* lens, size_t n,
                                      const uint32_t* qtab, uint32_t nv, uint32_t S, uint32_t O,
                                      uint32_t E, uint32_t PS, uint32_t pad, int32_t* scores,
                                      int packed, const uint32_t* fb_qtab, uint32_t fb_nv,
                                      uint32_t fb_PS, int32_t fb_thresh,
                                      const SwkWaveSplit* split, uint32_t ulen,
                                      uint32_t ustride, int half, hipStream_t st);
extern "C" hipError_t swk_launch_score(int R, int RB, int col0, int prof, int gotoh, int f16,
                                       const uint8_t* res, const uint64_t* offs,
                                       const uint32_t* lens, size_t n, const uint32_t* qtab,
                                       uint32_t nv, uint32_t S, uint32_t O, uint32_t E,
                                       uint32_t PS, uint32_t pad, int W, int32_t* scores,
                                       const void* edge_in, void* edge_out, uint32_t ecols,
                                       int accum, int packed, const uint32_t* idx,
                                       const uint32_t* nidx, uint32_t idx_base,
                                       const uint32_t* ident, int pair, uint32_t pS1,
                                       uint32_t pS2, uint32_t ulen, uint32_t ustride, uint32_t nq,
                                       uint32_t qwords, size_t sstride, hipStream_t st);
extern "C" unsigned swk_bal_slots(int W, uint32_t PS, int trim);
extern "C" unsigned swk_wave_half_grid(int gotoh, uint32_t prof_bytes, int W);
extern "C" hipError_t swk_bal_plan_uniform(void* plan, uint32_t ntiles, uint32_t K, uint32_t G,
                                           hipStream_t st);
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
                                          const uint32_t* sidx, hipStream_t st);
extern "C" hipError_t swk_best_hit(const int32_t* scores, const uint64_t* ids, size_t n,
                                   unsigned long long* key, uint64_t* out, uint64_t* out_index,
                                   hipStream_t st);
extern "C" hipError_t swk_best_part(const int32_t* scores, size_t n, size_t base,
                                    unsigned long long* key, hipStream_t st);
extern "C" hipError_t swk_best_finalize(const unsigned long long* key, const uint64_t* ids,
                                        uint64_t* out, uint64_t* out_index, hipStream_t st);
extern "C" hipError_t swk_sort_lens(const uint32_t* lens, size_t n, uint32_t max_len,
                                    uint32_t* perm, uint32_t* perm_n, uint32_t* ident,
                                    uint32_t* scratch, hipStream_t st, void* plan = nullptr,
                                    unsigned G = 0);
extern "C" size_t swk_sort_scratch_bytes(void);
extern "C" hipError_t swk_flag_high(const int32_t* scores, size_t n, int32_t thresh,
                                    uint32_t* idx, uint32_t* count, hipStream_t st);
extern "C" size_t swk_i32_waves(size_t n, uint32_t scols, size_t budget_bytes);
extern "C" hipError_t swk_launch_i32(int gotoh, const uint8_t* res, const uint64_t* offs,
                                     const uint32_t* lens, size_t n, int packed,
                                     const uint32_t* idx, const uint32_t* nidx, uint32_t idx_base,
                                     const void* prof, uint32_t nstrips, uint32_t qlen,
                                     uint32_t pad, uint32_t O, uint32_t E, int32_t* scores,
                                     void* scratch, uint32_t scols, size_t waves, hipStream_t st);

// ---- helpers shared by the units ----------------------------------------------------
inline int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

// Debug-only host phase trace (tuning aid): with SWBANK_TRACE_FILE set, host-buffer calls append
// "phase microseconds-since-call-entry" lines to that file.  Off by default; the library never
// prints otherwise.
struct PhaseTrace {
  const char* path = std::getenv("SWBANK_TRACE_FILE");
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  std::vector<std::pair<const char*, double>> marks;
  std::mutex mu;  // (the feeder's launch thread marks too)
  void mark(const char* what) { mark_at(what, std::chrono::steady_clock::now()); }
  void mark_at(const char* what, std::chrono::steady_clock::time_point t) {
    if (!path) return;
    std::lock_guard<std::mutex> g(mu);
    marks.push_back({what, std::chrono::duration<double, std::micro>(t - t0).count()});
  }
  ~PhaseTrace() {
    if (!path || marks.empty()) return;
    if (FILE* f = std::fopen(path, "a")) {
      for (auto& m : marks) std::fprintf(f, "%s %.1f\n", m.first, m.second);
      std::fprintf(f, "--\n");
      std::fclose(f);
    }
  }
};
inline thread_local PhaseTrace* g_trace = nullptr;
inline void trace_mark(const char* what) {
  if (g_trace) g_trace->mark(what);
}

inline bool poison_buffers() {  // (read at every allocation: tests switch it per case)
  const char* v = std::getenv("SWBANK_POISON");
  return v && v[0] == '1';
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
    // (tests) SWBANK_POISON=1: new device buffers start as 0x3C bytes (f16 1.0 in every half)
    // instead of whatever the allocator hands back, so a read of a word nobody wrote shows;
    // complete before any bank stream uses the buffer
    if (e == hipSuccess && poison_buffers()) {
      e = hipMemset(p, 0x3C, want * sizeof(T));
      if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    }
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Device memory the caches do not keep (hipDeviceMallocUncached): a streamed batch's codes land
// there by DMA while the kernel that reads them runs, so no cache line can be stale.
struct UcBuf {
  uint8_t* p = nullptr;
  size_t cap = 0;  // bytes
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&p), n, hipDeviceMallocUncached);
    if (e == hipSuccess) cap = n;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// Pinned host staging for the query tables (so their uploads are truly asynchronous).
// `flags`: hipHostMallocCoherent for words a running kernel reads (streamed chunk records).
struct PinBuf {
  unsigned flags = hipHostMallocDefault;
  uint8_t* p = nullptr;
  size_t cap = 0;  // bytes
  hipError_t reserve(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(n, 4096);
    hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), want, flags);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};


// Host worker threads for the host-buffer feeder (gather / scatter of a chunk): run(f) calls
// f(part) for part = 0..size()-1, part 0 on the calling thread, and returns when all are done.
// A host-API call runs several short jobs per chunk back to back, so idle workers spin on the
// job counter for up to 200 us before they sleep (a futex wake-up per job cost more than the
// jobs), and the caller spins for the last part to finish.
class HostPool {
 public:
  explicit HostPool(unsigned n) : n_(std::max(1u, n)) {
    for (unsigned i = 1; i < n_; ++i) th_.emplace_back([this, i] { loop(i); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_.store(true);
      gen_.fetch_add(1);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  unsigned size() const { return n_; }
  void run(const std::function<void(unsigned)>& f) {
    if (n_ == 1) {
      f(0);
      return;
    }
    job_ = &f;
    pending_.store(n_ - 1, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> g(m_);  // a worker about to sleep re-checks gen_ under m_
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    f(0);
    for (unsigned it = 1; pending_.load(std::memory_order_acquire) != 0; ++it) relax(it);
    job_ = nullptr;
  }

 private:
  static void relax(unsigned) {
#if defined(__SSE2__)
    _mm_pause();
#endif
  }
  void loop(unsigned i) {
    uint64_t seen = 0;
    for (;;) {
      const auto t0 = std::chrono::steady_clock::now();
      for (unsigned it = 1; gen_.load(std::memory_order_acquire) == seen; ++it) {
        relax(it);
        if ((it & 255) == 0 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) {
          std::unique_lock<std::mutex> l(m_);
          cv_.wait(l, [&] { return gen_.load() != seen; });
        }
      }
      seen = gen_.load(std::memory_order_acquire);
      if (stop_.load()) return;
      (*job_)(i);
      pending_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  unsigned n_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_;
  const std::function<void(unsigned)>* job_ = nullptr;  // published by gen_ (release/acquire)
  std::atomic<unsigned> pending_{0};
  std::atomic<uint64_t> gen_{0};
  std::atomic<bool> stop_{false};
};

// The host feeder's launch thread: runs the HIP work of each chunk (its copy, the score
// launches, the scores' return) in posting order while the caller's thread and the pool gather
// the next chunk -- the chunk's ~11 HIP calls (30-60 us) were on the gather's critical path.
// It sleeps on a condition variable between jobs (a spinning thread next to the pool's workers
// would take a core from the gather); the caller spins in wait(k) for the first k jobs to be
// done.  The first failing job's status sticks (later jobs are skipped) until reset().
class Launcher {
 public:
  explicit Launcher(int device) : th_([this, device] { loop(device); }) {}
  ~Launcher() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_one();
    th_.join();
  }
  void post(std::function<sw_status()> f) {
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(std::move(f));
      ++posted_;
    }
    cv_.notify_one();
  }
  // spins until the first k posted jobs ran; their status
  sw_status wait(size_t k) {
    while (done_.load(std::memory_order_acquire) < k) {
#if defined(__SSE2__)
      _mm_pause();
#endif
    }
    return st_.load(std::memory_order_acquire);
  }
  sw_status wait_all() { return wait(posted_); }  // (posted_ is the caller's own count)
  void reset() {  // between calls, all jobs done
    wait_all();
    posted_ = 0;
    done_.store(0);
    st_.store(SW_OK);
  }

 private:
  void loop(int device) {
    (void)hipSetDevice(device);
    for (;;) {
      std::function<sw_status()> f;
      {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;  // stop_
        f = std::move(q_.front());
        q_.erase(q_.begin());
      }
      if (st_.load(std::memory_order_relaxed) == SW_OK) {
        const sw_status s = f();
        if (s != SW_OK) st_.store(s, std::memory_order_release);
      }
      done_.fetch_add(1, std::memory_order_acq_rel);
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::vector<std::function<sw_status()>> q_;
  bool stop_ = false;
  size_t posted_ = 0;  // (the posting thread's count)
  std::atomic<size_t> done_{0};
  std::atomic<sw_status> st_{SW_OK};
  std::thread th_;  // last: started after the fields it reads
};

struct sw_bank {
  sw_config cfg{};
  int device = 0;
  int cus = 0;  // compute units (4 SIMDs each): the wave kernel's split-tail policy
  hipStream_t stream = nullptr;
  char err[512] = {0};

  // ld_penalties
  bool have_pen = false;
  int alpha = SW_DNA_ALPHA;
  std::vector<int8_t> matrix;  // alpha x alpha
  int32_t gap_open = 0, gap_extend = 0;

  // ld_sequence (query); a query set (sw_load_queries, > 1 query) keeps every query in qset
  // and its longest one in `query` (which sets the segment layout of all of them)
  bool have_query = false;
  uint64_t qid = 0;
  std::vector<uint8_t> query;
  std::vector<std::vector<uint8_t>> qset;
  bool mq_ready = false;               // mqtab / mqtab16 match qset and the penalties
  DevBuf<uint32_t> mqtab, mqtab16;     // [query][the single-query LUT layout] (u16, f16)
  size_t mq_words = 0;                 // words per query
  // letter-pair tables of a DNA merged f16 set: [segment][query][mq_pair_words], segments of
  // mq_pair_rows rows (512: 16 waves of 32 rows, 4-column chunks; 128: 4 waves, 8 columns)
  DevBuf<uint32_t> mqpair;
  size_t mq_pair_words = 0;
  int mq_pair_segs = 0, mq_pair_rows = 0;
  uint32_t mq_pS1 = 0, mq_pS2 = 0;

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
  // f16 letter-pair table (DNA merged gaps, one segment of <= 4 waves): the tile kernel's
  // PAIR variant; pair_bytes = 0 when the query does not qualify
  DevBuf<uint32_t> qpair;
  uint32_t pair_bytes = 0, pS1 = 0, pS2 = 0;
  DevBuf<uint32_t> fb_idx, fb_cnt;  // pairs an optimistic f16 pass re-scores in u16
  // int32 re-score of the pairs past the 16-bit lanes (built on first use per query):
  // [strip][letter 0..pad][lane] 4 x int16, strips of 256 rows; per-wave scratch rows
  bool i32_ready = false;
  uint32_t i32_strips = 0;
  DevBuf<uint2> i32prof, i32scr;
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
  // wave kernel split tail (one segment, K >= 8): [i] = the query as P = 2 << i segments of
  // sK = K/P rows per lane (stab: u16, stab16: f16, sseg_words* apart); sring: 256 columns x
  // uint2 per segment boundary of every tail pair (P = 8, the two-pairs kernel's segmented
  // tail: a whole row of columns per boundary, tprog its progress / best words)
  int sK[3] = {0, 0, 0};
  size_t sseg_words[3] = {0, 0, 0}, sseg_words16[3] = {0, 0, 0};
  uint32_t sPS[3] = {0, 0, 0}, sPS16[3] = {0, 0, 0};
  DevBuf<uint32_t> stab[3], stab16[3];
  DevBuf<uint2> sring;
  DevBuf<uint32_t> tprog;

  // host-buffer feeder (sw_score_batch / sw_score_records): NSLOT pinned staging slots, chunk
  // i gathered on the host while chunk i-1 crosses PCIe on copy_stream and earlier chunks are
  // scored on `stream` / stream2; NDSLOT device slots (chunk i's copy waits for the kernel of
  // chunk i - NDSLOT only: with NSLOT device slots too, the copies trailed the kernels)
  static constexpr int NSLOT = 3, NDSLOT = 6;
  hipStream_t copy_stream = nullptr;
  hipEvent_t h2d_done[NSLOT] = {}, kern_done[NDSLOT] = {};
  PinBuf hslot[NSLOT], hscores;
  std::vector<std::vector<uint32_t>> mlist;  // per pool part: a mixed chunk's 4-bit targets
  std::vector<std::vector<uint8_t>> mstage;  // ... and their codes, packed while gathering
  std::vector<std::vector<uint32_t>> mbad;   // ... a run block's positions of codes past 3
  std::vector<hipEvent_t> out_ev;  // per chunk: its scores are back in hscores
  hipStream_t out_stream = nullptr;  // scores back to the host, beside the next chunk's kernel
  hipStream_t stream2 = nullptr;     // odd chunks' kernels (scratch-free launches overlap)
  hipEvent_t ev_s2 = nullptr;
  double host_pack_ms = 0;         // feeder gather time of host calls (with timing on)
  int feed_dslots = NSLOT;         // device slots of the current feeder call
  DevBuf<uint8_t> dslot[NDSLOT];
  DevBuf<uint32_t> sortscr[NDSLOT];  // device sort scratch of each device slot's chunk
  // streamed host batches (one kernel for the whole call, equal-length DNA): the batch's codes
  // (chunks 256-byte aligned: no cache line holds two chunks, and nothing of a chunk is read
  // before its layout word is set, so no line is cached before its copy landed), the chunks'
  // device layout words (uncached device memory), the chunk records (device, staged in srec),
  // the host layout and abort words (coherent host memory), a copy event per chunk
  DevBuf<uint8_t> sbuf;
  UcBuf sflag;
  DevBuf<SwkStreamChunk> sdrec;
  DevBuf<uint32_t> sctr;  // tiles the streamed kernel's workgroups took
  // the streamed kernel's stream: a queue of its own (a CU-masked stream, every CU set), so no
  // copy-stream marker the publisher waits on can sit behind the running kernel in a queue
  // shared with another stream
  hipStream_t kstream = nullptr;
  PinBuf srec, shflag{hipHostMallocCoherent};
  PinBuf shscores{hipHostMallocCoherent};  // the streamed kernel writes the scores here
  std::vector<hipEvent_t> sev;
  std::unique_ptr<HostPool> pool;
  std::unique_ptr<Launcher> launcher;  // the feeder's launch thread

  // workspaces
  DevBuf<uint8_t> res;
  DevBuf<uint64_t> offs;
  DevBuf<uint32_t> lens;
  DevBuf<int32_t> scores;
  // the sorted copy of SWBANK_RAGGED_GATHER (launch): its own buffers, never the batch it
  // copies from (a multi-device child's batch IS res / offs / lens: ADVICE r5)
  DevBuf<uint8_t> gres;
  DevBuf<uint64_t> goffs;
  DevBuf<uint32_t> glens;

  char last_kernel[160] = {0};

  // best hit of the last batch call (sw_batch_best, ≙ max / vld_max): 0 none, 1 on the host,
  // 2 pending on the device (best_dev = {id, score, index} after best_ev)
  int best_kind = 0;
  uint64_t best_id = 0, best_index = 0;
  int32_t best_score = 0;
  DevBuf<uint64_t> best_dev;
  hipEvent_t best_ev = nullptr;

  // multi-device bank (cfg.n_devices > 1): one child bank per device, a host thread per device
  // (dpool part d drives kids[d]), scores gathered on kids[0]'s device (grecv) by RCCL or copies
  std::vector<sw_bank*> kids;
  std::unique_ptr<HostPool> dpool;
  std::vector<void*> comms;  // ncclComm_t per device (RCCL gather), empty -> copy gather
  bool rccl_gather = false;  // comms wanted (re-created after an aborted gather)
  unsigned pool_threads = 0; // feeder threads (0: host_threads(); children share the host)
  DevBuf<int32_t> grecv;
  PinBuf hrecv;
  // device batches on a multi-device bank (multi_device): the caller's batch on the root is
  // dealt into a staging buffer (res / offs / lens of the parent, on the root), each child
  // copies its region into its own buffers (peer access enabled once, peer_ready) and its
  // scores back (grecv); ev_join: the staging is ready (parent) / a child's work on its stream
  // is done (child; the caller's stream waits on it); ev_used (parent): the call's scatter;
  // best_root: the last device call's best hit is tracked by kids[0]
  // balanced chunk ranges (swk_launch_pair_bal): the hand-off states and flags, the launch
  // generation the flags are compared with
  DevBuf<uint32_t> bal_state, bal_flag;
  // balanced ranges of the two-pairs wave kernel: lane states, flags, their generation
  DevBuf<uint32_t> wbal_state, wbal_flag;
  uint32_t wbal_gen = 0;
  // range starts, 4 words each: a ragged batch's (the device sort writes them per call) or a
  // uniform batch's (swk_bal_plan_uniform for bal_key = {tiles, chunks per tile, grid}, kept
  // while the key holds; bal_key[0] = 0 when the sort overwrote them)
  DevBuf<uint32_t> bal_plan;
  size_t bal_key[3] = {0, 0, 0};
  uint32_t bal_gen = 0;
  bool peer_ready = false;
  hipEvent_t ev_join = nullptr;
  // a multi-device child's pipelined deal: chunk p of its share is in its HBM (copy_stream)
  std::vector<hipEvent_t> deal_ev;
  bool best_root = false;
  // on-device longest-first order of a ragged device batch (sw_score_batch_device):
  // dperm = visiting order + count, dsort = histogram / scan scratch
  DevBuf<uint32_t> dperm, dsort;
  bool is_multi() const { return !kids.empty(); }
  bool gotoh() const { return cfg.gap_model == SW_GAP_GOTOH; }

  // Query tables are rewritten in place by prepare() while earlier launches may still read
  // them on the caller's stream: the upload (on the bank stream) waits for ev_used (recorded
  // after every launch), and every launch waits for ev_ready (recorded after the upload).
  // Nothing blocks the host except reusing the pinned staging of a copy still in flight.
  hipEvent_t ev_ready = nullptr, ev_used = nullptr;
  PinBuf stage;

  // feeder / fallback counters (sw_bank_counters)
  sw_counters ctr{};

  // Fault words of the cross-workgroup hand-off waits (balanced ranges, the segmented protein
  // tail; ScoreArgs.fault): coherent host memory, [0] for device calls, [1] for host-buffer
  // calls, written only by a wait that ran out (SWK_FAULT_* bits) and read after the launch
  // completed: a host-buffer call re-runs itself without hand-offs (no_handoff), a device call's
  // fault is latched until the next synchronising call returns it (SW_ERR_TIMEOUT).
  PinBuf faultw{hipHostMallocCoherent};
  bool host_call = false;   // launches belong to a host-buffer call (fault word [1])
  bool no_handoff = false;  // launch() runs neither balanced ranges nor the segmented tail

  // profiling
  bool timing = false;
  struct Ev { hipEvent_t a, b, c; };
  std::vector<Ev> events;
};

// Every C-ABI entry point works on its bank's device and hands the calling thread back on the
// device it was on (a one-thread caller holding several banks, or torch beside a
// bank, got its next allocation on the wrong GPU after a library call).
struct DevGuard {
  int prev = -1;
  DevGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  explicit DevGuard(const sw_bank* b) : DevGuard() {
    if (b && b->device >= 0) (void)hipSetDevice(b->device);
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DevGuard(const DevGuard&) = delete;
  DevGuard& operator=(const DevGuard&) = delete;
};

// Scores in the f16 kernels are f16 multiples of 2^-11 (x as x/2048, swbank_kcommon.h), so
// the packed add's [0, 1] clamp is max(0, x); -2048 (padding rows / letters) is 0xBC00.
inline uint16_t f16_score_bits(int v) {
  return __builtin_bit_cast(uint16_t, (_Float16)((float)v * (1.0f / 2048.0f)));
}


// Sets the bank's error text (sw_last_error) and returns st.
sw_status fail(sw_bank* b, sw_status st, const char* fmt, ...);

#define HIPOK(bank, expr)                                                                 \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail((bank), SW_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),    \
                  __FILE__, __LINE__);                                                    \
  } while (0)

// RCCL for the multi-device score gather (SURVEY §8 e), loaded on first use (swbank_multi.hip).
struct Rccl {
  bool ok = false;
  char err[160] = {0};
  decltype(&ncclCommInitAll) commInitAll = nullptr;
  decltype(&ncclCommDestroy) commDestroy = nullptr;
  decltype(&ncclGather) gather = nullptr;
  decltype(&ncclGetErrorString) errorString = nullptr;
  decltype(&ncclCommAbort) commAbort = nullptr;
  decltype(&ncclCommGetAsyncError) asyncError = nullptr;
  decltype(&ncclGroupStart) groupStart = nullptr;  // one thread issuing every device's gather
  decltype(&ncclGroupEnd) groupEnd = nullptr;
};
const Rccl& rccl();

// Multi-device bank: apply a call to every child bank (the first failure's text is the bank's).
template <class F>
sw_status each_kid(sw_bank* b, F&& f) {
  for (sw_bank* k : b->kids) {
    const sw_status st = f(k);
    if (st != SW_OK) return fail(b, st, "device %d: %s", k->device, k->err);
  }
  return SW_OK;
}

// Feeder threads: SWBANK_HOST_THREADS, else the process's CPU share when OMP_NUM_THREADS
// states it (capped at 16), else 8 (and never more than the machine has).
unsigned host_threads();

// f(lo, hi) over [0, n) split into the pool's parts (inline below 2048 items)
template <class F>
void parallel_for(HostPool& pool, size_t n, F&& f) {
  const unsigned T = pool.size();
  if (T <= 1 || n < 2048) {
    f((size_t)0, n);
    return;
  }
  const size_t step = (n + T - 1) / T;
  pool.run([&](unsigned p) {
    const size_t lo = std::min(n, p * step), hi = std::min(n, lo + step);
    if (lo < hi) f(lo, hi);
  });
}

inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }
inline uint32_t record_len(const uint8_t* rec) {
  uint16_t l;
  std::memcpy(&l, rec + 4, 2);
  return l;
}

// ---- swbank_bank.hip
void copy_kernel_name(sw_bank* b, const char* gather);
// The fault word launch() hands the kernels (allocated and zeroed on first use; nullptr when the
// allocation failed), and the check of it: SW_ERR_TIMEOUT (counted, the word cleared) when a
// hand-off wait of the given kind of call (0 device, 1 host) ran out since the last check.  The
// caller has synchronised with the launches it means to cover.  A multi-device bank checks every
// child.
uint32_t* fault_word(sw_bank* b);
sw_status take_fault(sw_bank* b, int which);
sw_status prepare(sw_bank* b);
sw_status prepare_multi(sw_bank* b);
sw_status prepare_i32(sw_bank* b);
// ---- swbank_launch.hip
void u16_gotoh_rows(const sw_bank* b, bool f16, int& R, int& W);
bool wave_preferred(const sw_bank* b, size_t n, uint32_t max_len, bool use_f16);
sw_status launch(sw_bank* b, const uint8_t* d_res, const uint64_t* d_offs,
                 const uint32_t* d_lens, size_t n, uint32_t max_len, int32_t* d_scores,
                 hipStream_t st, uint32_t packed = SWK_PACK_BYTES,
                 const uint32_t* perm = nullptr, const uint32_t* perm_n = nullptr,
                 bool dsort = false, bool wait_prev = true, uint32_t* sort_out = nullptr,
                 uint32_t* sort_scr = nullptr, uint32_t ulen = 0, uint32_t ustride = 0,
                 uint32_t min_len = 0);
// ---- swbank_feeder.hip
bool chunk_perm(HostPool& pool, const uint32_t* len, size_t n, uint32_t* perm);
bool scratch_free(const sw_bank* b, uint32_t max_len);
// A ragged DNA chunk [c0, c0 + cnt) in the mixed layout (SWK_PACK_MIXED), the pool's parts of
// `step` targets each, planned by the caller's lengths pass: part p packs as one run from
// residue rbase[p] (rspan[p] codes, gaps included) or, rbase[p] == UINT64_MAX, per target; its
// 2-bit bytes start at psz[p] of mcodes, psz[T] and part4[T] bound the 2-bit and 4-bit regions.
// Writes the offset words so32[], lengths sl32[] and the codes; `end` = the codes' end (16 zero
// bytes follow).  order != nullptr: the chunk's longest-first visiting order (a stable counting
// sort) is written to order[] in the same pass, part p's next position in bin (hi - len) >> shift
// at order_pos[p * nbin + bin].  False when a code is outside the alphabet (nothing usable).
struct MixedOrder {
  std::vector<uint32_t> pos;
  uint32_t hi = 0, shift = 0, nbin = 0;
};
bool mixed_pack(sw_bank* b, const uint8_t* residues, size_t nres, const uint64_t* offsets,
                const uint32_t* lens, size_t c0, size_t cnt, size_t step,
                const std::vector<uint64_t>& rbase, const std::vector<uint64_t>& rspan,
                const std::vector<size_t>& psz, const std::vector<size_t>& part4, uint32_t* so32,
                uint32_t* sl32, uint8_t* mcodes, uint32_t* order, MixedOrder* mo, size_t& end);
sw_status batch_feed(sw_bank* b, const uint8_t* residues, size_t nres, const uint64_t* offsets,
                     const uint32_t* lens, size_t n, int32_t* out);
sw_status records_feed(sw_bank* b, const uint8_t* recs, size_t n, int32_t* out);
// ---- swbank_stream.hip
sw_status stream_feed(sw_bank* b, const uint8_t* residues, size_t nres, const uint64_t* offsets,
                      size_t n, uint32_t L, int32_t* out, bool& used,
                      const uint8_t* recs = nullptr, const uint32_t* rlens = nullptr);
// ---- swbank_multi.hip
sw_status multi_batch(sw_bank* b, const uint8_t* residues, size_t nres, const uint64_t* offsets,
                      const uint32_t* lens, size_t n, int32_t* scores_out);
sw_status multi_records(sw_bank* b, const uint8_t* recs, size_t n, int32_t* scores_out);
// Device buffers (on the root device, devices[0]) over a multi-device bank: contiguous ranges
// of the batch, one per device, asynchronous on the caller's stream (records: n x 64-B
// records at d_res, d_offs / d_lens unused).
sw_status multi_device(sw_bank* b, const uint8_t* d_res, const uint64_t* d_offs,
                       const uint32_t* d_lens, const uint64_t* d_ids, size_t n, uint32_t min_len,
                       uint32_t max_len, int32_t* d_scores, hipStream_t hs, bool records);
// One batch per device, resident in that device's HBM (ABI 6, sw_score_batch_device_multi):
// scored in place, only the int32 scores gathered to the root into d_gathered (may be null).
sw_status multi_resident(sw_bank* b, const sw_device_batch* per, int32_t* d_gathered,
                         hipStream_t hs);
// ---- swbank_launch.hip (device batches against a query set; sstride: between query rows)
sw_status launch_set(sw_bank* b, const uint8_t* d_res, const uint64_t* d_offs,
                     const uint32_t* d_lens, size_t n, uint32_t min_len, uint32_t max_len,
                     int32_t* d_scores, hipStream_t st, size_t sstride);
sw_status track_best_device(sw_bank* b, const int32_t* d_scores, const uint64_t* d_ids, size_t n,
                            hipStream_t st);

#endif  // SWBANK_BANK_H
