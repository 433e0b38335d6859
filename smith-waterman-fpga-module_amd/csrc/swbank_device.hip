// swbank_device.hip — C-ABI of libswbank.so: the bank object and its device plumbing.
//
// Call surface mirrors ScoreBank_v2 (reference ScoreBank/ScoreBank_v2.v:30-44): penalties once,
// a query once, then any number of target batches; one max score per target.  See
// include/swbank.h for the per-function reference citations.
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
                                      uint32_t ustride, hipStream_t st);
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
extern "C" hipError_t swk_best_hit(const int32_t* scores, const uint64_t* ids, size_t n,
                                   unsigned long long* key, uint64_t* out, uint64_t* out_index,
                                   hipStream_t st);
extern "C" hipError_t swk_best_part(const int32_t* scores, size_t n, size_t base,
                                    unsigned long long* key, hipStream_t st);
extern "C" hipError_t swk_best_finalize(const unsigned long long* key, const uint64_t* ids,
                                        uint64_t* out, uint64_t* out_index, hipStream_t st);
extern "C" hipError_t swk_sort_lens(const uint32_t* lens, size_t n, uint32_t max_len,
                                    uint32_t* perm, uint32_t* perm_n, uint32_t* ident,
                                    uint32_t* scratch, hipStream_t st);
extern "C" size_t swk_sort_scratch_bytes(void);
extern "C" hipError_t swk_flag_high(const int32_t* scores, size_t n, int32_t thresh,
                                    uint32_t* idx, uint32_t* count, hipStream_t st);
extern "C" void swk_set_occ_cap(int per_cu);
extern "C" size_t swk_i32_waves(size_t n, uint32_t scols, size_t budget_bytes);
extern "C" hipError_t swk_launch_i32(int gotoh, const uint8_t* res, const uint64_t* offs,
                                     const uint32_t* lens, size_t n, int packed,
                                     const uint32_t* idx, const uint32_t* nidx, uint32_t idx_base,
                                     const void* prof, uint32_t nstrips, uint32_t qlen,
                                     uint32_t pad, uint32_t O, uint32_t E, int32_t* scores,
                                     void* scratch, uint32_t scols, size_t waves, hipStream_t st);

namespace {
int env_int(const char* name, int dflt) {
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
  void mark(const char* what) {
    if (path)
      marks.push_back({what, std::chrono::duration<double, std::micro>(
                                 std::chrono::steady_clock::now() - t0).count()});
  }
  void mark_at(const char* what, std::chrono::steady_clock::time_point t) {
    if (path) marks.push_back({what, std::chrono::duration<double, std::micro>(t - t0).count()});
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
thread_local PhaseTrace* g_trace = nullptr;
inline void trace_mark(const char* what) {
  if (g_trace) g_trace->mark(what);
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
    while (pending_.load(std::memory_order_acquire) != 0) relax();
    job_ = nullptr;
  }

 private:
  static void relax() {
#if defined(__SSE2__)
    _mm_pause();
#endif
  }
  void loop(unsigned i) {
    uint64_t seen = 0;
    for (;;) {
      const auto t0 = std::chrono::steady_clock::now();
      for (unsigned it = 1; gen_.load(std::memory_order_acquire) == seen; ++it) {
        relax();
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
}  // namespace

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
  // letter-pair tables of a DNA merged f16 set: [128-row segment][query][mq_pair_words]
  DevBuf<uint32_t> mqpair;
  size_t mq_pair_words = 0;
  int mq_pair_segs = 0;
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
  // uint2 per segment boundary of every tail pair
  int sK[2] = {0, 0};
  size_t sseg_words[2] = {0, 0}, sseg_words16[2] = {0, 0};
  uint32_t sPS[2] = {0, 0}, sPS16[2] = {0, 0};
  DevBuf<uint32_t> stab[2], stab16[2];
  DevBuf<uint2> sring;

  // host-buffer feeder (sw_score_batch / sw_score_records): NSLOT pinned staging slots and
  // device slots, chunk i gathered on the host while chunk i-1 crosses PCIe on copy_stream
  // and chunk i-2 is scored on `stream`
  static constexpr int NSLOT = 3;
  hipStream_t copy_stream = nullptr;
  hipEvent_t h2d_done[NSLOT] = {}, kern_done[NSLOT] = {};
  PinBuf hslot[NSLOT], hscores;
  std::vector<hipEvent_t> out_ev;  // per chunk: its scores are back in hscores
  hipStream_t out_stream = nullptr;  // scores back to the host, beside the next chunk's kernel
  hipStream_t stream2 = nullptr;     // odd chunks' kernels (scratch-free launches overlap)
  hipEvent_t ev_s2 = nullptr;
  double host_pack_ms = 0;         // feeder gather time of host calls (with timing on)
  DevBuf<uint8_t> dslot[NSLOT];
  DevBuf<uint32_t> sortscr[NSLOT];  // device sort scratch of each slot's chunk
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

  // workspaces
  DevBuf<uint8_t> res;
  DevBuf<uint64_t> offs;
  DevBuf<uint32_t> lens;
  DevBuf<int32_t> scores;

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

  // profiling
  bool timing = false;
  struct Ev { hipEvent_t a, b, c; };
  std::vector<Ev> events;
};

// Scores in the f16 kernels are f16 multiples of 2^-11 (x as x/2048, swbank_kernels.hip), so
// the packed add's [0, 1] clamp is max(0, x); -2048 (padding rows / letters) is 0xBC00.
static inline uint16_t f16_score_bits(int v) {
  return __builtin_bit_cast(uint16_t, (_Float16)((float)v * (1.0f / 2048.0f)));
}

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

// RCCL for the multi-device score gather (SURVEY §8 e: ncclCommInitAll, rccl.h:236, and
// ncclGather, rccl.h:745).  Loaded on first use so single-device users never map it; in a
// process where PyTorch already mapped its librccl.so.1 that copy is reused (same SONAME).
namespace {
struct Rccl {
  bool ok = false;
  char err[160] = {0};
  decltype(&ncclCommInitAll) commInitAll = nullptr;
  decltype(&ncclCommDestroy) commDestroy = nullptr;
  decltype(&ncclGather) gather = nullptr;
  decltype(&ncclGetErrorString) errorString = nullptr;
  decltype(&ncclCommAbort) commAbort = nullptr;
  decltype(&ncclCommGetAsyncError) asyncError = nullptr;
};
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
    r.ok = r.commInitAll && r.commDestroy && r.gather && r.errorString && r.commAbort &&
           r.asyncError;
    if (!r.ok)
      snprintf(r.err, sizeof(r.err),
               "librccl.so.1 lacks ncclCommInitAll/ncclGather/ncclCommAbort/ncclCommGetAsyncError");
  });
  return r;
}
}  // namespace

static sw_status check_device(int dev) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SW_ERR_NO_DEVICE;
  if (dev < 0 || dev >= ndev) return SW_ERR_NO_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return SW_ERR_NO_DEVICE;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return SW_ERR_NO_DEVICE;
  return SW_OK;
}

static unsigned host_threads_total();

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
      k->pool_threads = std::max(2u, host_threads_total() / (unsigned)cfg.n_devices);
      b->kids.push_back(k);
    }
    b->dpool.reset(new (std::nothrow) HostPool((unsigned)cfg.n_devices));
    b->pool.reset(new (std::nothrow) HostPool(host_threads_total()));
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
  if (hipSetDevice(dev) != hipSuccess ||
      hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess) {
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
  if (!b) return;
  if (b->is_multi() || !b->comms.empty()) {
    const Rccl& r = rccl();
    for (void* c : b->comms) (void)r.commDestroy(static_cast<ncclComm_t>(c));
    for (sw_bank* k : b->kids) sw_bank_destroy(k);
    b->dpool.reset();
    b->pool.reset();
    (void)hipSetDevice(b->device);
    b->grecv.release();
    b->hrecv.release();
    delete b;
    return;
  }
  (void)hipSetDevice(b->device);
  if (b->stream) (void)hipStreamSynchronize(b->stream);
  uint64_t nl;
  double pm, sm;
  (void)sw_bank_timing(b, &nl, &pm, &sm);
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
  b->fb_idx.release();
  b->fb_cnt.release();
  b->best_key.release();
  b->best_dev.release();
  b->i32prof.release();
  b->i32scr.release();
  b->dperm.release();
  b->dsort.release();
  b->wtab.release();
  b->wtab16.release();
  for (int i = 0; i < 2; ++i) {
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
  for (int i = 0; i < sw_bank::NSLOT; ++i) {
    b->hslot[i].release();
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
  for (int i = 0; i < sw_bank::NSLOT; ++i) {
    if (b->h2d_done[i]) (void)hipEventDestroy(b->h2d_done[i]);
    if (b->kern_done[i]) (void)hipEventDestroy(b->kern_done[i]);
  }
  b->hscores.release();
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

extern "C" sw_status sw_bank_counters(const sw_bank* b, sw_counters* out) {
  if (!b || !out) return SW_ERR_ARG;
  *out = b->ctr;
  for (const sw_bank* k : b->kids) {
    out->stream_calls += k->ctr.stream_calls;
    out->stream_reruns += k->ctr.stream_reruns;
    out->stream_declined += k->ctr.stream_declined;
    out->chunked_calls += k->ctr.chunked_calls;
    out->device_sorts += k->ctr.device_sorts;
    out->gather_timeouts += k->ctr.gather_timeouts;
  }
  return SW_OK;
}

static void copy_kernel_name(sw_bank* b, const char* gather) {
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

// Multi-device bank: apply a call to every child bank (the first failure's text is the bank's).
template <class F>
static sw_status each_kid(sw_bank* b, F&& f) {
  for (sw_bank* k : b->kids) {
    const sw_status st = f(k);
    if (st != SW_OK) return fail(b, st, "device %d: %s", k->device, k->err);
  }
  return SW_OK;
}

extern "C" sw_status sw_set_penalties(sw_bank* b, int32_t match, int32_t mismatch,
                                      int32_t gap_open, int32_t gap_extend) {
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
  if (!b || !m) return SW_ERR_ARG;
  if (b->is_multi())
    return each_kid(b, [&](sw_bank* k) { return sw_set_matrix(k, m, alpha, gap_open, gap_extend); });
  const int want = b->cfg.alphabet == SW_ALPHABET_DNA ? SW_DNA_ALPHA : SW_PROTEIN_ALPHA;
  if (alpha != want) return fail(b, SW_ERR_ARG, "matrix alphabet %d, bank expects %d", alpha, want);
  return set_matrix_impl(b, m, alpha, gap_open, gap_extend);
}

extern "C" sw_status sw_load_query(sw_bank* b, uint64_t id, const uint8_t* codes, uint32_t len) {
  if (!b || (!codes && len)) return SW_ERR_ARG;
  if (b->is_multi())
    return each_kid(b, [&](sw_bank* k) { return sw_load_query(k, id, codes, len); });
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
  if (!b || nq == 0 || !offsets || !lens) return SW_ERR_ARG;
  if (b->is_multi())
    return fail(b, SW_ERR_UNSUPPORTED, "query sets need a single-device bank");
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
    const uint16_t bits = f16_score_bits(m[i]);
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
  std::vector<uint32_t> tpair;
  uint32_t pS1 = 0, pS2 = 0;
  if (f16 && !prof && !gotoh && !col0 && R == 32 && segs.size() == 1 && segs[0].W <= 4 &&
      A == SW_DNA_ALPHA) {
    const uint32_t NR = (uint32_t)segs[0].W * R;
    pair_strides(NR, pS1, pS2);
    tpair = pair_table(b->query.data(), qlen, 0, NR, m, A, pS1, pS2);
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
  // split tail of the wave kernel (one segment, K >= 8): the query as P = 2 and 4 segments of
  // K/P rows per lane, tables concatenated like the segments above
  std::vector<uint32_t> st[2], st16[2];
  int sK[2] = {0, 0};
  for (int i = 0; i < 2; ++i) {
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
       st[1].size() + tab.size() + tab16.size() + tpair.size()) * 4;
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
  for (int i = 0; i < 2; ++i) {
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
  b->pair_bytes = (uint32_t)tpair.size() * 4;
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
static sw_status prepare_multi(sw_bank* b) {
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
  // letter-pair tables (DNA merged f16 without the column-0 rule): 128-row segments (4 waves of
  // 32 rows: the pair kernel's layout), one table per (segment, query)
  std::vector<uint32_t> tp;
  b->mq_pair_segs = 0;
  if (b->f16 && !b->prof && !b->gotoh() && !b->col0 && A == SW_DNA_ALPHA &&
      env_int("SWBANK_MQ_PAIR", 1) != 0) {
    const uint32_t NR = 128;
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
static sw_status prepare_i32(sw_bank* b) {
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

// True when every length in [min_len, max_len] falls in the device sort's first length bin
// (swk_sort_lens: bins of 2^shift lengths below max_len, at most 2048 of them): the caller's
// order is then already longest first, and the sort kernels are not launched at all.
static bool one_len_bin(uint32_t min_len, uint32_t max_len) {
  if (min_len > max_len) return false;
  uint32_t shift = 0;
  while ((max_len >> shift) >= 2048u) ++shift;
  return ((max_len - min_len) >> shift) == 0;
}

// packed (SWK_PACK_*): RECORDS: d_res holds n 64-byte CAPI records (2-bit codes), d_offs and
// d_lens are unused; STREAM: 2-bit codes, d_offs in bytes (the host feeder's DNA chunks).
// perm/perm_n (optional, tile kernel): pass 0 visits the targets in the order perm[0..n)
// (target numbers; *perm_n = n on the device), e.g. longest first; the wave kernel ignores it.
static sw_status launch(sw_bank* b, const uint8_t* d_res, const uint64_t* d_offs,
                        const uint32_t* d_lens, size_t n, uint32_t max_len, int32_t* d_scores,
                        hipStream_t st, uint32_t packed = SWK_PACK_BYTES,
                        const uint32_t* perm = nullptr,
                        const uint32_t* perm_n = nullptr, bool dsort = false,
                        bool wait_prev = true, uint32_t* sort_out = nullptr,
                        uint32_t* sort_scr = nullptr, uint32_t ulen = 0, uint32_t ustride = 0,
                        uint32_t min_len = 0) {
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
  // the f16 pass of the tile kernel reads the letter-pair table when the query has one
  const bool use_pair = use_f16 && b->pair_bytes != 0 && env_int("SWBANK_PAIR", 1) != 0;
  bool wave_fb = false;  // the wave kernel re-scores its own flagged pairs
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
    // optimistic f16 with one query segment: the wave re-scores a flagged pair in u16 itself
    // (no flag kernel, no re-score launches)
    wave_fb = opt16 && b->wsegs == 1 && env_int("SWBANK_WAVE_FB", 1) != 0;
    // Split tail: pairs beyond a whole number of waves per SIMD (one wave per pair, all
    // resident) would put one more wave on some SIMDs and set the kernel's length; the last
    // pairs % SIMDs pairs (when at most half the SIMDs) run instead as P row segments of K/P
    // rows per lane each (P = 4 with 4 x that many waves, else 2), in the same launch.
    // SWBANK_WAVE_SPLIT=0 disables, =N splits the last N pairs (tests); SWBANK_WAVE_SPLIT_P
    // forces P.
    SwkWaveSplit sp{};
    const size_t pairs = (n + 1) / 2;
    const int sforce = env_int("SWBANK_WAVE_SPLIT", -1);
    if (b->sK[0] && b->wsegs == 1 && n == wspan && env_int("SWBANK_WAVE_BLOCK", 4) == 4 &&
        pairs <= 0xFFFFFFFFull) {
      const size_t simds = 4 * (size_t)std::max(b->cus, 1);
      size_t T = 0;
      if (sforce >= 0) T = std::min(pairs, (size_t)sforce);
      else if (pairs >= simds && pairs % simds <= simds / 2) T = pairs % simds;
      const int pforce = env_int("SWBANK_WAVE_SPLIT_P", 0);
      const int i = pforce == 2 ? 0 : pforce == 4 ? 1 : (4 * T <= simds ? 1 : 0);
      if (T && b->sK[i]) {
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
                     2048 - std::max(0, b->smax), &sp, ulen, ustride, st));
      }
    }
  } else {
    snprintf(b->last_kernel, sizeof(b->last_kernel), "tile %s%s R=%d W=%d segs=%zu", arith,
             b->prof ? "-profile" : use_pair ? " pair" : "", b->R, b->segs[0].W, nseg);
  }
  // A device batch (dsort) visits its targets longest first, sorted on the device, so every
  // tile holds similar lengths (a tile runs to its longest lane); SWBANK_DSORT=0 disables.
  const uint32_t* ident = nullptr;  // device sort: 1 when the lengths share one bin
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
    HIPOK(b, swk_sort_lens(d_lens, n, max_len, order, order + n, order + n + 1, scr, st));
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
      for (size_t s = 0; s < nseg; ++s) {
        const void* ein = s > 0 ? b->edge[(s - 1) & 1].p : nullptr;
        void* eout = s + 1 < nseg ? b->edge[s & 1].p : nullptr;
        const bool pair = f16 && use_pair;
        HIPOK(b, swk_launch_score(b->R, b->RB, b->col0, b->prof, gotoh ? 1 : 0, f16 ? 1 : 0, res,
                                  offs, lens, np,
                                  pair ? b->qpair.p
                                  : f16 ? b->qtab16.p + b->segs[s].off16
                                        : b->qtab.p + b->segs[s].off,
                                  f16 ? b->nv16 : b->nv, b->S, b->O, b->E,
                                  pair ? b->pair_bytes : f16 && b->prof ? b->PS16 : b->PS,
                                  b->pad, b->segs[s].W, scores, ein, eout, ecols, s > 0 ? 1 : 0,
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
static sw_status track_best_device(sw_bank* b, const int32_t* d_scores, const uint64_t* d_ids,
                                   size_t n, hipStream_t st) {
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
static sw_status launch_set(sw_bank* b, const uint8_t* d_res, const uint64_t* d_offs,
                            const uint32_t* d_lens, size_t n, uint32_t min_len, uint32_t max_len,
                            int32_t* d_scores, hipStream_t st) {
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
                  !(b->gotoh() && !use_f16 && b->R != 16) && n <= 0xFFFFFFFFull &&
                  !(kforce && std::strcmp(kforce, "wave") == 0) && ntiles * nq <= 0x7FFFFFFFull;
  if (!mq) {  // one query at a time (each prepare()d in turn), then the set's layout again
    const std::vector<uint8_t> longest = b->query;
    sw_status rs = SW_OK;
    for (size_t i = 0; i < nq && rs == SW_OK; ++i) {
      b->query = b->qset[i];
      b->dirty = true;
      rs = prepare(b);
      if (rs == SW_OK)
        rs = launch(b, d_res, d_offs, d_lens, n, max_len, d_scores + i * n, st, SWK_PACK_BYTES,
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
  const size_t slots = 4 * (size_t)std::max(b->cus, 1);
  const bool mpair = b->mq_pair_segs > 0 && use_f16 && nq <= slots &&
                     8 * (slots - slots / nq * nq) <= slots;
  const size_t nseg = mpair ? (size_t)b->mq_pair_segs : b->segs.size();
  snprintf(b->last_kernel, sizeof(b->last_kernel), "tile %s%s R=%d W=%d segs=%zu queries=%zu",
           use_f16 ? "f16" : "u16", mpair ? " pair" : "", b->R,
           mpair ? std::min(4, (int)(b->query.size() + 31) / 32) : b->segs[0].W, nseg, nq);
  HIPOK(b, hipStreamWaitEvent(st, b->ev_ready, 0));  // the query tables are uploaded
  HIPOK(b, hipStreamWaitEvent(st, b->ev_used, 0));   // bank scratch is free
  sw_bank::Ev ev{};
  if (b->timing) {
    HIPOK(b, hipEventCreate(&ev.a));
    HIPOK(b, hipEventCreate(&ev.b));
    HIPOK(b, hipEventCreate(&ev.c));
    HIPOK(b, hipEventRecord(ev.a, st));
    HIPOK(b, hipEventRecord(ev.b, st));
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
      if (mpair) {  // 128-row segments, 4 waves of 32 rows (fewer for a short last one)
        const int rows = std::min(128, (int)b->query.size() - (int)sg * 128);
        const int Wp = std::max(1, (rows + 31) / 32);
        HIPOK(b, swk_launch_score(32, 4, 0, 0, 0, 1, d_res, offs, lens, np,
                                  b->mqpair.p + sg * nq * b->mq_pair_words, b->nv16, b->S, b->O,
                                  b->E, (uint32_t)b->mq_pair_words * 4, b->pad, Wp, scores, ein,
                                  eout, ecols, sg > 0 ? 1 : 0, (int)SWK_PACK_BYTES,
                                  perm ? perm + p0 : nullptr, perm_n, (uint32_t)p0, ident, 1,
                                  b->mq_pS1, b->mq_pS2, 0, 0, (uint32_t)nq,
                                  (uint32_t)b->mq_pair_words, n, st));
        continue;
      }
      HIPOK(b, swk_launch_score(b->R, b->RB, 0, 0, gotoh ? 1 : 0, use_f16 ? 1 : 0, d_res, offs,
                                lens, np, tabs + b->segs[sg].off, use_f16 ? b->nv16 : b->nv,
                                b->S, b->O, b->E, 0, b->pad, b->segs[sg].W, scores, ein, eout,
                                ecols, sg > 0 ? 1 : 0, (int)SWK_PACK_BYTES,
                                perm ? perm + p0 : nullptr, perm_n, (uint32_t)p0, ident, 0, 0, 0,
                                0, 0, (uint32_t)nq, (uint32_t)b->mq_words, n, st));
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
  return sw_score_batch_device_range(b, d_res, d_offs, d_lens, d_ids, n, 0, max_len, d_scores,
                                     stream);
}

extern "C" sw_status sw_score_batch_device_range(sw_bank* b, const uint8_t* d_res,
                                                 const uint64_t* d_offs, const uint32_t* d_lens,
                                                 const uint64_t* d_ids, size_t n,
                                                 uint32_t min_len, uint32_t max_len,
                                                 int32_t* d_scores, void* stream) {
  if (!b) return SW_ERR_ARG;
  if (min_len > max_len) return fail(b, SW_ERR_ARG, "min_len %u > max_len %u", min_len, max_len);
  if (b->is_multi())
    return fail(b, SW_ERR_UNSUPPORTED, "device buffers need a single-device bank");
  b->best_kind = 0;
  if (n == 0) return SW_OK;
  if (!d_res || !d_offs || !d_lens || !d_scores) return fail(b, SW_ERR_ARG, "null device buffer");
  sw_status st = prepare(b);
  if (st != SW_OK) return st;
  HIPOK(b, hipSetDevice(b->device));
  hipStream_t hs = stream ? reinterpret_cast<hipStream_t>(stream) : b->stream;
  if (b->qset.size() > 1) {  // a query set: nq x n scores; the best hit is not tracked
    if (d_ids) return fail(b, SW_ERR_UNSUPPORTED, "best hit over a query set");
    return launch_set(b, d_res, d_offs, d_lens, n, min_len, max_len, d_scores, hs);
  }
  if ((st = launch(b, d_res, d_offs, d_lens, n, max_len, d_scores, hs, SWK_PACK_BYTES, nullptr,
                   nullptr, true, true, nullptr, nullptr, 0, 0, min_len)) != SW_OK)
    return st;
  return d_ids ? track_best_device(b, d_scores, d_ids, n, hs) : SW_OK;
}

extern "C" sw_status sw_batch_best(sw_bank* b, uint64_t* best_id, int32_t* best_score,
                                   uint64_t* best_index) {
  if (!b) return SW_ERR_ARG;
  if (b->best_kind == 2) {
    uint64_t h[3];
    HIPOK(b, hipSetDevice(b->device));
    HIPOK(b, hipEventSynchronize(b->best_ev));
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

// ---- host-buffer batches: a pipelined feeder ----------------------------------------------
// The reference host hands the accelerator host buffers (main_test.c:297-370 builds the WED
// and sequence_t arrays in host memory).  A host batch is put in longest-first feed order,
// cut into chunks and fed through NSLOT pinned staging slots: host threads gather chunk i
// (code validation fused into the copy) while chunk i-1 crosses PCIe on the copy stream and
// chunk i-2 is scored on the bank stream.
namespace {
// Feeder threads: SWBANK_HOST_THREADS, else the process's CPU share when OMP_NUM_THREADS
// states it (capped at 16), else 8 (and never more than the machine has).
unsigned host_threads() {
  const int t = env_int("SWBANK_HOST_THREADS", 0);
  if (t > 0) return (unsigned)std::min(t, 64);
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const int omp = env_int("OMP_NUM_THREADS", 0);
  return std::min(hw, omp > 0 ? (unsigned)std::min(omp, 16) : 8u);
}

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
size_t chunk_target(size_t total) {
  const int mb = env_int("SWBANK_CHUNK_MB", 0);
  if (mb > 0) return (size_t)mb << 20;
  return std::min<size_t>((size_t)256 << 20, std::max<size_t>((size_t)8 << 20, total / 8));
}

// Cumulative chunk boundaries (in input bytes) of a host batch: the first chunk a quarter of
// chunk_target() (at least 1 MiB) so the GPU starts early, then doubling up to chunk_target()
// (SWBANK_CHUNK_MB: fixed size).  Boundaries strictly inside (0, total).
std::vector<size_t> chunk_bounds(size_t total) {
  std::vector<size_t> bounds;
  const size_t cap = chunk_target(total);
  const int first_kb = env_int("SWBANK_CHUNK_FIRST_KB", 0);
  size_t sz = first_kb > 0 ? (size_t)first_kb << 10
              : env_int("SWBANK_CHUNK_MB", 0) > 0 ? cap : std::max<size_t>(1 << 20, cap / 4);
  for (size_t at = sz; at < total; at += sz, sz = std::min(cap, sz * 2)) bounds.push_back(at);
  // SWBANK_CHUNK_TAIL=1: the last chunk as a half and two quarters, so the call's final
  // launches (which nothing overlaps) are short
  const size_t last = bounds.empty() ? 0 : bounds.back(), rem = total - last;
  if (env_int("SWBANK_CHUNK_TAIL", 0) != 0 && rem >= ((size_t)4 << 20)) {
    bounds.push_back(last + rem / 2);
    bounds.push_back(last + rem / 2 + rem / 4);
  }
  return bounds;
}
}  // namespace

static unsigned host_threads_total() { return host_threads(); }

static sw_status feeder_init(sw_bank* b) {
  HIPOK(b, hipSetDevice(b->device));
  if (!b->pool) b->pool.reset(new (std::nothrow) HostPool(b->pool_threads ? b->pool_threads
                                                                          : host_threads()));
  if (!b->pool) return fail(b, SW_ERR_NOMEM, "host worker pool");
  if (b->copy_stream) return SW_OK;
  HIPOK(b, hipStreamCreateWithFlags(&b->copy_stream, hipStreamNonBlocking));
  HIPOK(b, hipStreamCreateWithFlags(&b->out_stream, hipStreamNonBlocking));
  HIPOK(b, hipStreamCreateWithFlags(&b->stream2, hipStreamNonBlocking));
  HIPOK(b, hipEventCreateWithFlags(&b->ev_s2, hipEventDisableTiming));
  for (int i = 0; i < sw_bank::NSLOT; ++i) {
    HIPOK(b, hipEventCreateWithFlags(&b->h2d_done[i], hipEventDisableTiming));
    HIPOK(b, hipEventCreateWithFlags(&b->kern_done[i], hipEventDisableTiming));
  }
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
  for (int i = 0; i < std::min<int>(sw_bank::NSLOT, (int)chunks.size()); ++i) {
    HIPOK(b, b->hslot[i].reserve(slot_bytes));
    HIPOK(b, b->dslot[i].reserve(slot_bytes));
  }
  HIPOK(b, b->scores.reserve(n));
  if (out) {
    HIPOK(b, b->hscores.reserve(n * 4));
    while (b->out_ev.size() < chunks.size()) {
      hipEvent_t e;
      HIPOK(b, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      b->out_ev.push_back(e);
    }
  }
  // overlapped chunk launches run two at a time: each takes at most SWBANK_CHUNK_OCC (2)
  // workgroups per CU, so a chunk's tiles are several per workgroup (less pipeline fill and
  // drain per tile) and the two streams share the chip
  struct OccCap {
    explicit OccCap(int c) { swk_set_occ_cap(c); }
    ~OccCap() { swk_set_occ_cap(0); }
  } occ_cap(overlap ? std::max(0, env_int("SWBANK_CHUNK_OCC", 2)) : 0);
  const auto fail_sync = [&](sw_status s) {
    (void)hipStreamSynchronize(b->stream);
    (void)hipStreamSynchronize(b->stream2);
    (void)hipStreamSynchronize(b->copy_stream);
    (void)hipStreamSynchronize(b->out_stream);
    return s;
  };
  for (size_t i = 0; i < chunks.size(); ++i) {
    const int s = (int)(i % sw_bank::NSLOT);
    const Chunk& c = chunks[i];
    if (i >= (size_t)sw_bank::NSLOT) HIPOK(b, hipEventSynchronize(b->h2d_done[s]));
    trace_mark("gather<");
    const auto t0 = std::chrono::steady_clock::now();
    size_t from = 0;  // leading slot bytes the device does not need (a uniform chunk's headers)
    const size_t bytes = gather(b->hslot[s].p, c, from);
    trace_mark("gather>");
    if (b->timing)
      b->host_pack_ms +=
          std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (bytes == 0) return fail_sync(SW_ERR_ARG);
    if (i >= (size_t)sw_bank::NSLOT)
      HIPOK(b, hipStreamWaitEvent(b->copy_stream, b->kern_done[s], 0));
    HIPOK(b, hipMemcpyAsync(b->dslot[s].p + from, b->hslot[s].p + from, bytes - from,
                            hipMemcpyHostToDevice, b->copy_stream));
    HIPOK(b, hipEventRecord(b->h2d_done[s], b->copy_stream));
    hipStream_t ks = overlap && (i & 1) ? b->stream2 : b->stream;
    HIPOK(b, hipStreamWaitEvent(ks, b->h2d_done[s], 0));
    // the last chunk has no later launch to share the chip with: the whole GPU
    if (overlap && i + 1 == chunks.size()) swk_set_occ_cap(0);
    if ((st = score(b->dslot[s].p, c, b->scores.p + c.c0, ks)) != SW_OK) return fail_sync(st);
    trace_mark("launched");
    HIPOK(b, hipEventRecord(b->kern_done[s], ks));
    if (out) {
      HIPOK(b, hipStreamWaitEvent(b->out_stream, b->kern_done[s], 0));
      HIPOK(b, hipMemcpyAsync(b->hscores.p + c.c0 * 4, b->scores.p + c.c0, (c.c1 - c.c0) * 4,
                              hipMemcpyDeviceToHost, b->out_stream));
      HIPOK(b, hipEventRecord(b->out_ev[i], b->out_stream));
    }
  }
  if (overlap) {  // the bank stream (the multi-device gather, the next call) after stream2
    HIPOK(b, hipEventRecord(b->ev_s2, b->stream2));
    HIPOK(b, hipStreamWaitEvent(b->stream, b->ev_s2, 0));
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
    HIPOK(b, hipEventSynchronize(b->out_ev[i]));
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
  HIPOK(b, hipStreamSynchronize(b->stream));
  trace_mark("done");
  return SW_OK;
}

static inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// Chunk slot tail shared by both host paths: lens u32 x cnt | perm u32 x cnt | count u32.
struct SlotTail {
  size_t lens_at, perm_at, cnt_at;
};
static SlotTail slot_tail(size_t tail_at, size_t cnt) {
  return {tail_at, tail_at + cnt * 4, tail_at + cnt * 8};
}

// True when launches for targets of at most max_len use no bank scratch (one query segment,
// no optimistic f16 re-score list, no int32 re-score), so host-feeder chunks may run on two
// streams (SWBANK_OVERLAP=0 disables).  Mirrors launch()'s choices.
static bool scratch_free(const sw_bank* b, uint32_t max_len) {
  if (env_int("SWBANK_OVERLAP", 1) == 0) return false;
  const uint64_t s = (uint64_t)std::max(0, b->smax);
  const uint64_t top = std::min<uint64_t>(b->query.size(), max_len) * s + s;
  const bool need32 = top > 65535u || env_int("SWBANK_I32", 0) != 0;
  const bool f16_ok = b->f16 && b->f16_neg >= -2048 && env_int("SWBANK_F16", 1) != 0;
  const bool opt16 = f16_ok && top > 2048u && env_int("SWBANK_F16_OPT", 1) != 0;
  return b->segs.size() == 1 && b->wsegs == 1 && !need32 && !opt16;
}

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
static sw_status stream_feed(sw_bank* b, const uint8_t* residues, size_t nres,
                             const uint64_t* offsets, size_t n, uint32_t L, int32_t* out,
                             bool& used, const uint8_t* recs = nullptr,
                             const uint32_t* rlens = nullptr) {
  used = false;
  if (recs && (L == 0 || L > SWB_RECORD_MAX)) return SW_OK;
  const int mode_env = env_int("SWBANK_STREAM", 1);  // 2: also below the size threshold (tests)
  if (mode_env == 0 || !out || b->alpha != SW_DNA_ALPHA || b->prof || b->col0 || b->RB != 4 ||
      env_int("SWBANK_PACK2", 1) == 0 || env_int("SWBANK_UNIFORM", 1) == 0 ||
      !scratch_free(b, L) || n > 0x7FFFFFFFull)
    return SW_OK;
  const char* kforce = std::getenv("SWBANK_KERNEL");
  if (kforce && std::strcmp(kforce, "wave") == 0) return SW_OK;
  const size_t T = (n + SWB_TILE - 1) / SWB_TILE;
  // two rounds of 4 workgroups per CU: the throughput model picks the tile kernel there
  if (mode_env != 2 && T < 8 * (size_t)std::max(b->cus, 1)) return SW_OK;
  const uint64_t smax = (uint64_t)std::max(0, b->smax);
  const bool use_f16 = b->f16 && b->f16_neg >= -2048 && env_int("SWBANK_F16", 1) != 0 &&
                       std::min<uint64_t>(b->query.size(), L) * smax + smax <= 2048u;
  const bool pair = use_f16 && b->pair_bytes != 0 && env_int("SWBANK_PAIR", 1) != 0;
  if (!(b->R == 16 || (b->R == 32 && !b->gotoh()))) return SW_OK;  // streamed variants

  // chunks of whole tiles: 1/64 of the batch first, doubling up to 1/8
  std::vector<size_t> tile0;
  const size_t cap = std::max<size_t>(1, T / 8);
  for (size_t t = 0, sz = std::max<size_t>(1, T / 64); t < T; t += sz, sz = std::min(cap, 2 * sz))
    tile0.push_back(t);
  const size_t nsc = tile0.size();
  tile0.push_back(T);
  const size_t nib = (L + 1) / 2;  // 4-bit bytes per target (the 2-bit stream needs fewer)
  std::vector<size_t> roff(nsc + 1, 0);
  size_t slot_bytes = 0;
  for (size_t i = 0; i < nsc; ++i) {
    const size_t cnt = std::min(n, tile0[i + 1] * SWB_TILE) - tile0[i] * SWB_TILE;
    const size_t head = rlens ? align16(cnt * 16) : 0;  // ragged: offsets | lengths | order
    roff[i + 1] = roff[i] + (head + cnt * nib + 64 + 255) / 256 * 256;
    slot_bytes = std::max(slot_bytes, roff[i + 1] - roff[i]);
  }
  // Memory the streamed call keeps for the bank's lifetime: the batch's 4-bit codes on the
  // device (sbuf), NSLOT pinned host slots of the largest chunk (<= 1/8 of it each) and the
  // batch's scores in coherent host memory.  Past SWBANK_STREAM_MB (default 4096 MiB of device
  // codes + host scores), or when any of it cannot be allocated, the call runs through the
  // chunked feeder, whose slots are bounded by chunk_target() (counted: stream_declined).
  const size_t cap_bytes = (size_t)std::max(1, env_int("SWBANK_STREAM_MB", 4096)) << 20;
  if (roff[nsc] + n * 4 > cap_bytes) {
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
    bool ok = b->sbuf.reserve(roff[nsc]) == hipSuccess && b->sflag.reserve(nsc * 4) == hipSuccess &&
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
    rec[i] = SwkStreamChunk{(unsigned)tile0[i], (unsigned)roff[i], (unsigned)(roff[i] >> 32), 0u};
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
    if (b->timing) {
      HIPOK(b, hipEventCreate(&ev.a));
      HIPOK(b, hipEventCreate(&ev.b));
      HIPOK(b, hipEventCreate(&ev.c));
      HIPOK(b, hipEventRecord(ev.a, ks));
      HIPOK(b, hipEventRecord(ev.b, ks));
    }
    HIPOK(b, swk_launch_stream(b->R, b->gotoh() ? 1 : 0, use_f16 ? 1 : 0, pair ? 1 : 0, b->sbuf.p,
                               n, rlens ? 0u : L, b->sdrec.p, hflag,
                               reinterpret_cast<uint32_t*>(b->sflag.p),
                               (uint32_t)nsc, b->sctr.p,
                               pair ? b->qpair.p : use_f16 ? b->qtab16.p : b->qtab.p,
                               use_f16 ? b->nv16 : b->nv, b->S, b->O, b->E,
                               pair ? b->pair_bytes : 0, b->pad, b->segs[0].W,
                               reinterpret_cast<int32_t*>(b->shscores.p),
                               b->pS1, b->pS2, ks));
    HIPOK(b, hipEventRecord(b->ev_used, ks));
    if (b->timing) {
      HIPOK(b, hipEventRecord(ev.c, ks));
      b->events.push_back(ev);
    }
    snprintf(b->last_kernel, sizeof(b->last_kernel), "tile %s%s R=%d W=%d segs=1 streamed=%zu",
             use_f16 ? "f16" : "u16", pair ? " pair" : "", b->R, b->segs[0].W, nsc);
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
    if (rlens) {  // ragged: offsets | lengths | order, then the codes at the next 16 bytes
      const size_t ca = align16(cnt * 16), step = (cnt + PT - 1) / PT;
      uint64_t* so = reinterpret_cast<uint64_t*>(codes);
      uint32_t* sl = reinterpret_cast<uint32_t*>(codes + cnt * 8);
      uint32_t* sp = sl + cnt;
      uint8_t* cb = codes + ca;
      std::vector<size_t> p2(PT + 1, 0), p4(PT + 1, 0);
      pool.run([&](unsigned p) {  // lengths, bounds, packed bytes per part
        const size_t lo = std::min(cnt, p * step), hi = std::min(cnt, (p + 1) * step);
        size_t a2 = 0, a4 = 0;
        for (size_t j = lo; j < hi; ++j) {
          const size_t k = c0 + j;
          const uint32_t l = rlens[k];
          if (offsets[k] > nres || l > nres - offsets[k]) {
            size_t cur = oob.load();
            while (k < cur && !oob.compare_exchange_weak(cur, k)) {
            }
            return;
          }
          sl[j] = l;
          a2 += (l + 3) / 4;
          a4 += (l + 1) / 2;
        }
        p2[p + 1] = a2;
        p4[p + 1] = a4;
      });
      for (unsigned p = 0; p < PT; ++p) {
        p2[p + 1] += p2[p];
        p4[p + 1] += p4[p];
      }
      for (int pass = nib_mode ? 1 : 0; oob.load() == SIZE_MAX && pass < 2 && md == 0; ++pass) {
        const bool two = pass == 0;
        const std::vector<size_t>& pre = two ? p2 : p4;
        const size_t stepb = two ? 8 : 16;
        const swpack::PackFn fn = two ? pack2fn : pack4fn;
        wide = 0;
        pool.run([&](unsigned p) {
          const size_t lo = std::min(cnt, p * step), hi = std::min(cnt, (p + 1) * step);
          size_t at = pre[p];
          uint32_t acc = 0;
          for (size_t j = lo; j < hi; ++j) {
            const size_t k = c0 + j;
            const uint32_t l = sl[j];
            const size_t st = (l + 31u) / 32u;
            // full vector steps past the target's end stay inside this part's output and read
            // inside the residues (later targets of the part rewrite those bytes)
            const bool w = offsets[k] + st * 32 <= nres && at + st * stepb <= pre[p + 1];
            const uint32_t v = fn(residues + offsets[k], l, cb + at, w);
            acc = two ? (acc | v) : std::max(acc, v);
            so[j] = at;
            at += two ? (l + 3) / 4 : (l + 1) / 2;
          }
          if (two ? acc > 3u : acc >= (uint32_t)SW_DNA_ALPHA) wide = 1;
        });
        if (wide.load() == 0) md = two ? SWK_PACK_STREAM : SWK_PACK_NIBBLE;
        else if (two) nib_mode = true;
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
      if (md != 0) {
        if (!chunk_perm(pool, sl, cnt, sp))  // already longest first: the identity
          for (size_t j = 0; j < cnt; ++j) sp[j] = (uint32_t)j;
        bytes = ca + (md == SWK_PACK_STREAM ? p2[PT] : p4[PT]);
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
  // released to the kernel as aborted (it reads whatever their range holds) so it drains, and
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

// The host-buffer batch through the feeder (n >= 1, buffers checked by the caller).
static sw_status batch_feed(sw_bank* b, const uint8_t* residues, size_t nres,
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
  const size_t pstep = (n + P - 1) / P;
  const auto run_parts = [&](const std::function<void(unsigned)>& f) {
    if (P > 1) pool.run(f);
    else f(0u);
  };
  std::vector<size_t> psum(P + 1, 0);
  std::vector<uint32_t> pmax(P, 0), pmin(P, UINT32_MAX);
  run_parts([&](unsigned p) {
    size_t acc = 0;
    uint32_t m = 0, mn = UINT32_MAX;
    for (size_t k = std::min(n, p * pstep); k < std::min(n, (p + 1) * pstep); ++k) {
      acc += lens[k];
      m = std::max(m, lens[k]);
      mn = std::min(mn, lens[k]);
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
    // bench shape (host-side order per chunk on the gather's critical path)
    bool used = false;
    st = stream_feed(b, residues, nres, offsets, n, max_len, out, used, nullptr, lens);
    if (used) return st;
  }
  // slot: offsets u64 | lens | perm | count | ident (SlotTail) | codes at codes_at(cnt): one byte per
  // residue, or, for a DNA chunk without N, the 2-bit stream (a quarter of the PCIe bytes;
  // SWBANK_PACK2=0 disables), each target from a byte boundary, 16 zero bytes after the last
  const auto codes_at = [](size_t cnt) { return align16(cnt * 16 + 8); };
  std::vector<size_t> bounds = chunk_bounds(total);
  bounds.push_back(SIZE_MAX);  // sentinel
  std::vector<std::vector<std::pair<size_t, size_t>>> pcut(P);  // (end position, code prefix)
  run_parts([&](unsigned p) {
    size_t acc = psum[p];
    // the next boundary above this part's start; a cut after target k when the running code
    // count reaches it (several boundaries inside one target make one cut)
    size_t j = std::upper_bound(bounds.begin(), bounds.end(), acc) - bounds.begin();
    for (size_t k = std::min(n, p * pstep); k < std::min(n, (p + 1) * pstep); ++k) {
      acc += lens[k];
      if (acc >= bounds[j]) {
        while (acc >= bounds[j]) ++j;
        if (k + 1 < n) pcut[p].push_back({k + 1, acc});
      }
    }
  });
  std::vector<Chunk> chunks;
  size_t c0 = 0, a0 = 0;
  const auto add_chunk = [&](size_t c1, size_t a1) {
    chunks.push_back({c0, c1, codes_at(c1 - c0) + align16(a1 - a0 + 16)});
    c0 = c1;
    a0 = a1;
  };
  for (const auto& cuts : pcut)
    for (const auto& ca : cuts) add_chunk(ca.first, ca.second);
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
  std::vector<size_t> part(T + 1), part2(T + 1), part4(T + 1);
  std::vector<uint32_t> partmax(T), partmin(T);
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
    oob = SIZE_MAX;
    pool.run([&](unsigned p) {
      size_t acc = 0, acc2 = 0, acc4 = 0;
      uint32_t m = 0, mn = UINT32_MAX;
      bool out = false;
      for (size_t k = c.c0 + std::min(cnt, p * step); k < c.c0 + std::min(cnt, (p + 1) * step);
           ++k) {
        acc += lens[k];
        acc2 += (lens[k] + 3) / 4;
        acc4 += (lens[k] + 1) / 2;
        m = std::max(m, lens[k]);
        mn = std::min(mn, lens[k]);
        // the target must lie inside the caller's residues (checked before any byte is read;
        // the pack passes below re-read this part's offsets from cache)
        out |= offsets[k] > nres || lens[k] > nres - offsets[k];
      }
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
    }
    uint32_t mode = SWK_PACK_BYTES;
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
    const int slot = (int)(si % sw_bank::NSLOT);
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
  if (b && b->qset.size() > 1)
    return fail(b, SW_ERR_STATE, "a query set is loaded: score it with sw_score_batch_device");
  if (!b) return SW_ERR_ARG;
  if (b->is_multi())
    return fail(b, SW_ERR_UNSUPPORTED, "device buffers need a single-device bank");
  b->best_kind = 0;
  if (n == 0) return SW_OK;
  if (!d_records || !d_scores) return fail(b, SW_ERR_ARG, "null device buffer");
  if (b->alpha != SW_DNA_ALPHA) return fail(b, SW_ERR_UNSUPPORTED, "records carry DNA only");
  sw_status st = prepare(b);
  if (st != SW_OK) return st;
  // lengths live on the device: the kernels clamp them to the record capacity
  HIPOK(b, hipSetDevice(b->device));
  return launch(b, static_cast<const uint8_t*>(d_records), nullptr, nullptr, n, SWB_RECORD_MAX,
                d_scores, stream ? reinterpret_cast<hipStream_t>(stream) : b->stream,
                SWK_PACK_RECORDS);
}

// Host records through the feeder (n >= 1, buffers checked by the caller); lengths are
// checked while gathering.
static sw_status records_feed(sw_bank* b, const uint8_t* recs, size_t n, int32_t* out) {
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
}

static sw_status multi_batch(sw_bank* b, const uint8_t* residues, size_t nres,
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

static sw_status multi_records(sw_bank* b, const uint8_t* recs, size_t n, int32_t* scores_out) {
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

extern "C" sw_status sw_score_batch(sw_bank* b, const uint8_t* residues, size_t residues_len,
                                    const uint64_t* offsets, const uint32_t* lens,
                                    const uint64_t* ids, size_t n, int32_t* scores_out) {
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

extern "C" sw_status sw_bank_set_timing(sw_bank* b, int32_t enable) {
  if (!b) return SW_ERR_ARG;
  if (b->is_multi()) return each_kid(b, [&](sw_bank* k) { return sw_bank_set_timing(k, enable); });
  b->timing = enable != 0;
  return SW_OK;
}

extern "C" sw_status sw_bank_timing(sw_bank* b, uint64_t* launches, double* pack_ms,
                                    double* score_ms) {
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
  p += b->host_pack_ms;  // host calls: the feeder's gather / pack time on the host
  b->host_pack_ms = 0;
  if (launches) *launches = n;
  if (pack_ms) *pack_ms = p;
  if (score_ms) *score_ms = s;
  return st;
}

extern "C" sw_status sw_best_hit_device(sw_bank* b, const int32_t* d_scores, const uint64_t* d_ids,
                                        size_t n, uint64_t* d_out, void* stream) {
  if (!b) return SW_ERR_ARG;
  if (b->is_multi())
    return fail(b, SW_ERR_UNSUPPORTED, "device buffers need a single-device bank");
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
  if (!scores || !best_id || !best_score || n == 0)
    return b ? fail(b, SW_ERR_ARG, "sw_best_hit: empty or null input") : SW_ERR_ARG;
  size_t bi = 0;
  for (size_t k = 1; k < n; ++k)
    if (scores[k] > scores[bi]) bi = k;
  *best_id = ids ? ids[bi] : (uint64_t)bi;
  *best_score = scores[bi];
  return SW_OK;
}
