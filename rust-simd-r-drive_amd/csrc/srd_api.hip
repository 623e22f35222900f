// srd_api.hip -- host orchestration + C ABI (include/srd_amd.h).
//
// One translation unit with the kernels (device globals live here).
// Glue scans/compactions use hipCUB (library primitives, like calling
// rocBLAS for a plain GEMM); every byte-touching hot kernel is hand-written
// in srd_kernels.hip.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <functional>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "srd_amd.h"
#include "srd_host.cpp"
#include "srd_kernels.hip"
#include "srd_glue.hip"
#include "srd_writer.hip"
#include "srd_index.hip"
#include "srd_probe.hip"

using namespace srd;

static thread_local std::string g_err;
static void set_err(const std::string& s) { g_err = s; }
extern "C" const char* srd_last_error(void) { return g_err.c_str(); }
#ifndef SRD_SOURCE_HASH
#define SRD_SOURCE_HASH "unknown"  // (built without the Makefile)
#endif
extern "C" const char* srd_build_info(void) { return SRD_SOURCE_HASH; }

#define HIPCHK(x)                                                                         \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      set_err(std::string(#x) + ": " + hipGetErrorString(e_));                            \
      return SRD_ERR_HIP;                                                                 \
    }                                                                                     \
  } while (0)

namespace {

// SRD_SYNC_DEBUG=1: synchronise after every kernel and name the first one
// that fails (debugging aid; off by default)
static int sync_debug() {
  static int v = -1;
  if (v < 0) { const char* e = getenv("SRD_SYNC_DEBUG"); v = (e && *e && *e != '0') ? 1 : 0; }
  return v;
}
#define KCHK(c, name)                                                                           \
  do {                                                                                          \
    if (sync_debug()) {                                                                         \
      hipError_t e_ = hipStreamSynchronize((c)->stream);                                        \
      if (e_ == hipSuccess) e_ = hipGetLastError();                                             \
      if (e_ != hipSuccess) {                                                                   \
        set_err(std::string("kernel ") + name + ": " + hipGetErrorString(e_));                  \
        fprintf(stderr, "srd: kernel %s failed: %s\n", name, hipGetErrorString(e_));            \
        return SRD_ERR_HIP;                                                                     \
      }                                                                                         \
    }                                                                                           \
  } while (0)

struct Buf {
  void* p = nullptr;
  size_t n = 0;
};

// Candidate record slots per span; grow x4 on overflow and are remembered by
// the context for stores of a similar size.  The optimistic pass starts at 8
// (a C2 span holds ~4 records): its 4096 scan waves write their records into
// regions of spans x cap slots, and with 64 slots the regions were 135 KiB
// apart (a 604 MB record buffer for C2) -- on the first-allocated workspace of
// a process that cost 6-8 % of the scan (same-box A/B, profiles/r03/
// scan_record_regions_ab.txt); at 8 the regions are 17 KiB apart and every
// placement runs at the fast rate.
struct CandCap {
  uint32_t cap;          // slots per span
  uint32_t grown_cap;    // the cap the last overflow needed ...
  uint64_t grown_bytes;  // ... for a store (span) of this many bytes
  uint32_t floor;        // the default (a store of another size starts here again)
};

// A context's persistent host thread (the multi-GPU open runs each shard's
// work on its context's worker: no thread spawn / join per phase).  One job
// at a time; post() then wait().
struct Worker {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::function<void()> job;
  bool has = false, stop = false;
  Worker() {
    th = std::thread([this] {
      std::unique_lock<std::mutex> lk(mu);
      for (;;) {
        cv.wait(lk, [this] { return has || stop; });
        if (!has) return;  // stop
        lk.unlock();
        job();
        lk.lock();
        has = false;
        job = nullptr;
        cv.notify_all();
      }
    });
  }
  ~Worker() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    th.join();
  }
  void post(std::function<void()> f) {
    std::lock_guard<std::mutex> lk(mu);
    job = std::move(f);
    has = true;
    cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [this] { return !has; });
  }
};

struct Ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::vector<Buf> bufs;  // indexed by the enum below
  // candidate slots per span (4 tiles) of the optimistic pass's scan and of
  // the full pass's (CandCap): each scan wave's records are dense in a region
  // of (its spans x cap) slots, so the cap sets how far apart the waves'
  // record stores land -- see CandCap
  CandCap copt{8, 8, 0, 8};
  CandCap cfull{32, 32, 0, 32};
  unsigned scan_blocks = 256;  // persistent scan grid (one 16-wave block per CU)
  unsigned scan_cus = 256;
  uint32_t scan_wq[16] = {};  // ScanPart::wq (scan_weights())
  uint32_t scan_variant = 0;  // ScanArgs::variant (srd_debug_set_scan_variant)
  // the optimistic pass's slot-space bound (the glue's parent words are 31-bit):
  // 2^31; SRD_SLOT_LIMIT_LOG2 (10..31, read at srd_ctx_create) lowers it so the
  // SRD_FULL_SLOT_SPACE fallback can be tested on a small store
  uint64_t slot_limit = 1ull << 31;
  // the scan's tile loads: SRD_SCAN_LOADS pins one pattern (0 coalesced +
  // transpose, SCAN_LINES line per lane); -1 = chosen per store by measuring
  // both (LoadTune, scan_variant_tune)
  int loads_pin = -1;
  int last_loads = -1;  // srd_ctx_scan_loads: the last optimistic scan's pattern
  struct LoadTune {
    uint64_t ns = ~0ull;       // the store (resident spans, grid) the state is for
    uint32_t g = 0;
    uint32_t calls = 0;        // optimistic scans of this store so far
    uint64_t best[2] = {0, 0};  // the fastest scan of each pattern, ticks (0 coalesced, 1 line per lane)
    uint32_t n[2] = {0, 0};
    int choice = -1;           // -1: still measuring
  } tune;
  // round 0 of the optimistic pass runs the shape check inside
  // chain_finalize_kernel<true> (look-back ranks) instead of check_kernel +
  // chain_finalize_kernel<false>; srd_debug_set_glue_fused A/Bs the two
  bool glue_fused = true;
  // test knobs read at srd_ctx_create: SRD_GLUE_FUSED=0 (round 0 through
  // check_kernel + chain_finalize_kernel<false>, the retry rounds' shape) and
  // SRD_LB_FAIL_BLOCK=b (chain block b's look-back treated as timed out)
  uint32_t lb_fail = ~0u;
  // XCD-aware block shares of the optimistic scan (XPart, B_XPART; SRD_XPART=0
  // at srd_ctx_create turns them off): the parity of the table the next scan
  // reads, and the span count / grid the table was made for
  bool xpart_on = true, xp_valid = false;
  uint32_t xp_par = 0, xp_g = 0;
  uint64_t xp_ns = 0;
  srd_device_result res{};
  // host-input staging
  Buf file;
  // timing (HIP events on `stream`)
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  // srd_ctx_set_timing: 0 none (default), 1 scan kernel (a ring of start /
  // stop pairs stamped by the scan dispatches), 2 + whole call (ev[2],
  // ev[3]).  The scan pairs are read out when srd_ctx_timings asks (or when
  // the ring wraps), not inside the calls: hipEventElapsedTime per call was
  // host time on every call's critical path
  int timing = SRD_TIMING_NONE;
  static constexpr uint32_t kScanRing = 64;
  hipEvent_t sev[2 * kScanRing] = {};
  uint32_t sev_next = 0, sev_pending = 0;  // next pair, pairs not yet read out
  double scan_ms = 0, total_ms = 0;  // scan_ms / scan_launches: since the last srd_ctx_timings
  int scan_launches = 0;
  uint32_t timing_every = 1, timing_seq = 0;  // srd_ctx_set_timing_every
  // the individual scan durations behind scan_ms (scan_list), and those of
  // the last srd_ctx_timings read (scan_last: srd_ctx_scan_list)
  std::vector<float> scan_list, scan_last;
  // sync-free optimistic pass
  uint32_t gen = 0;     // generation tag of has_child / childof
  uint64_t last_n = 0;  // chain length of the previous call (index bucket sizing)
  Plan* h_plan = nullptr;  // pinned host copy
  uint64_t* h_pub = nullptr;  // pinned: idx_emit's published outcome (IdxArgs::pub)
  uint64_t* h_small = nullptr;  // pinned: small device reads (counters, K, ...): async copies, one wait
  uint32_t pub_seq = 0;
  // batch writer (srd_batch_write): side copy stream, double-buffer events,
  // pinned entry tables and pinned bounce buffers (non-contiguous inputs)
  hipStream_t cstream = nullptr;
  hipEvent_t wev_copied[2] = {nullptr, nullptr}, wev_done[2] = {nullptr, nullptr};
  void* pin_ent[2] = {nullptr, nullptr};
  // host-input staging (stage_host): bounce buffers, one stream per worker
  int stage_workers = 8;
  int stage_mode = -1;  // last call: 0 pinned input, 1 registered, 2 bounce buffers, 3 pageable
  double stage_ms = 0;  // host wall time of the last staging
  bool ev3_recorded = false;  // the optimistic pass recorded ev[3] before its final sync
  std::vector<void*> stage_pin;
  std::vector<hipStream_t> stage_streams;
  std::vector<hipEvent_t> stage_ev;
  srd_multi_summary last_multi{};  // the last multi-GPU open with this context as ctxs[0]
  std::vector<double> last_shard_ms;  // its per-shard validate times (srd_ctx_multi_shard_ms)
  void* h_out = nullptr;  // pinned host result arrays (srd_validate_index / _multi)
  uint64_t h_out_n = 0;
  uint8_t lgen = 0;  // generation of the index build's non-latest marks (B_LATEST8)
  // multi-GPU open: the context's persistent host worker (created on first
  // use) and the event every cross-context copy out of this context's memory
  // waits on (recorded on `stream` once the data it reads is enqueued)
  Worker* worker = nullptr;
  hipEvent_t ev_ready = nullptr;
  bool ready_recorded = false;
};

enum BufId {
  B_TILE, B_SPAN_COUNT, B_SPAN_BASE,
  B_CM, B_CREC,
  B_COUNTERS,  // [0]=max_root [1]=start tail (find_top) [2]=overflow [3]=best_g1 [4]=changed [5]=n_slow [6]=n_bad [7]=special
  B_DM, B_DPAR, B_DSLOT, B_DHEAD, B_RUNHEAD, B_INTS, B_WALK,
  B_ST, B_JMP, B_VFLAG, B_VLIST, B_NV, B_VPOS, B_VPAR, B_VHEAD, B_VSLOT,
  B_ONPATH, B_CPOS, B_CHAIN_G, B_CORE,
  B_O_MO, B_O_KH, B_O_PREV, B_O_START, B_O_LEN, B_O_CRCST, B_O_CRC, B_O_OK,
  B_O_PIECES, B_O_SUF, B_O_SXM, B_O_TAIL, B_SLOW,
  B_HKEYS, B_HVALS, B_LATEST, B_IPOS, B_IKEY, B_IPACKED,
  B_CUB_TMP,
  B_PLAN, B_HASCHILD, B_CHILDOF, B_FLAG, B_PART, B_PARTEX, B_HOFF, B_SKEY, B_SIDX, B_LATEST8, B_XPART,
  B_MPLAN, B_MKEY, B_MVAL, B_PCNT, B_POFF, B_HASCHILD2,
  B_WPAY0, B_WPAY1, B_WKEY0, B_WKEY1, B_WENT0, B_WENT1, B_WKH, B_WMO,
  B_IT_FLAG, B_IT_POS, B_IT_ST, B_IT_EN, B_IT_KEPT, B_IT_OST, B_IT_OEN, B_IT_OKH, B_IT_ENT, B_IT_RLEN, B_IT_PST,
  B_GKEY, B_GVAL, B_GOKEY, B_GOPACKED,
  B_WTOT, B_WROOT, B_KTOT, B_DONE, B_SPAN_FIRST,
  B_XKEY, B_XVAL, B_GATHER, B_RFLAG, B_O_PACKED, B_VSCAN, B_LOOKB, B_PROBE, B_XTOT,
  B_COUNT_
};

int ensure(Ctx* c, BufId id, size_t bytes) {
  Buf& b = c->bufs[id];
  if (b.n >= bytes && b.p) return 0;
  if (b.p) HIPCHK(hipFree(b.p));
  b.p = nullptr;
  b.n = 0;
  size_t want = std::max<size_t>(bytes, 256);
  if (hipMalloc(&b.p, want) != hipSuccess) {
    set_err("hipMalloc failed for " + std::to_string(want) + " bytes");
    b.p = nullptr;
    return SRD_ERR_ALLOC;
  }
  b.n = want;
  return 0;
}
template <class T>
T* P(Ctx* c, BufId id) { return (T*)c->bufs[id].p; }

// ensure + zero-fill whenever the buffer is (re)allocated
int ensure_z(Ctx* c, BufId id, size_t bytes) {
  void* before = c->bufs[id].p;
  size_t nb = c->bufs[id].n;
  int r = ensure(c, id, bytes);
  if (r) return r;
  if (c->bufs[id].p != before || c->bufs[id].n != nb) HIPCHK(hipMemsetAsync(c->bufs[id].p, 0, c->bufs[id].n, c->stream));
  return 0;
}

std::once_flag g_tab_once;
CrcTables g_host_tabs;

int upload_tables() {
  static int rc = 1;
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  std::call_once(g_tab_once, [] { build_crc_tables(g_host_tabs); });
  // per device upload
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  static uint64_t uploaded = 0;
  if (uploaded & (1ull << dev)) return 0;
  DevTables t;
  memcpy(t.tab, g_host_tabs.tab, sizeof t.tab);
  memcpy(t.lw, g_host_tabs.lw, sizeof t.lw);
  memcpy(t.winit, g_host_tabs.winit, sizeof t.winit);
  memcpy(t.zero_crc, g_host_tabs.zero_crc, sizeof t.zero_crc);
  t.x32768 = g_host_tabs.x32768;
  t.xtile[0] = kX0;
  for (int e = 1; e <= 64; e++) t.xtile[e] = mulp(g_host_tabs.x32768, t.xtile[e - 1]);
  t.xt64[0] = kX0;
  for (int q = 1; q <= 64; q++) t.xt64[q] = mulp(t.xtile[64], t.xt64[q - 1]);
  for (int tb = 0; tb < 4; tb++)
    for (int b = 0; b < 256; b++) t.mx64[tb][b] = mulp(t.xtile[64], (uint32_t)b << (8 * tb));
  memcpy(t.pow8, g_host_tabs.pow8, sizeof t.pow8);
  memcpy(t.invpow, g_host_tabs.invpow, sizeof t.invpow);
  for (int pos = 0; pos < 8; pos++)
    for (int nb = 0; nb < 16; nb++)
      for (int l = 0; l < 32; l++)  // x^(512*(31-l)) = lw[l + 32]
        t.nib[((pos * 16 + nb) << 5) + l] = mulp(g_host_tabs.lw[l + 32], (uint32_t)nb << (4 * pos));
  {
    const uint32_t x16k = host_xpow8(g_host_tabs, 2048);
    for (int tb = 0; tb < 4; tb++)
      for (int b = 0; b < 256; b++) {
        t.m16k[tb][b] = mulp(x16k, (uint32_t)b << (8 * tb));
        for (int q = 0; q < 3; q++) {
          t.last[q][tb][b] = mulp(host_xpow8(g_host_tabs, 4 + 16 * (3 - q)), (uint32_t)b << (8 * tb));
          t.last_c[q][tb][b] = mulp(host_xpow8(g_host_tabs, 4 + 1024 * (3 - q)), (uint32_t)b << (8 * tb));
        }
        t.m4096[tb][b] = mulp(host_xpow8(g_host_tabs, 512), (uint32_t)b << (8 * tb));
        t.m32k[tb][b] = mulp(g_host_tabs.x32768, (uint32_t)b << (8 * tb));
        for (int j = 0; j < 3; j++) t.mtk[j][tb][b] = mulp(host_xpow8(g_host_tabs, 4096 * (j + 2)), (uint32_t)b << (8 * tb));
      }
    for (int pos = 0; pos < 8; pos++)
      for (int nb = 0; nb < 16; nb++)
        for (int l = 0; l < 32; l++)
          t.nib_c[((pos * 16 + nb) << 5) + l] = mulp(host_xpow8(g_host_tabs, 16 * (31 - l)), (uint32_t)nb << (4 * pos));
  }
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_tabs), &t, sizeof t));
  uploaded |= 1ull << dev;
  (void)rc;
  return 0;
}

inline unsigned blocks(uint64_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

#define TRY(x)                 \
  do {                         \
    int r_ = (x);              \
    if (r_) return r_;         \
  } while (0)

// hipCUB temp size for all glue ops up to n elements
int ensure_cub(Ctx* c, uint64_t n) {
  size_t t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;
  int nn = (int)std::min<uint64_t>(n + 1, 0x7fffffff);
  hipcub::DeviceScan::ExclusiveSum(nullptr, t1, (uint32_t*)nullptr, (uint64_t*)nullptr, nn);
  hipcub::DeviceScan::InclusiveScan(nullptr, t2, (uint32_t*)nullptr, (uint32_t*)nullptr, hipcub::Max(), nn);
  hipcub::DeviceScan::ExclusiveSum(nullptr, t3, (uint32_t*)nullptr, (uint32_t*)nullptr, nn);
  hipcub::DeviceSelect::Flagged(nullptr, t4, hipcub::CountingInputIterator<uint64_t>(0), (uint32_t*)nullptr,
                                (uint64_t*)nullptr, (uint64_t*)nullptr, nn);
  t5 = std::max(std::max(t1, t2), std::max(t3, t4));
  return ensure(c, B_CUB_TMP, t5 + 256);
}

// stores above 2^40 bytes take the WIDE scan (48-bit prev offsets)
constexpr uint64_t kWide = 1ull << 40;
constexpr uint64_t kMaxFile = 1ull << 48;  // packed offsets are 48-bit (key_indexer.rs:12-15, 79-85)
#ifdef SRD_DEBUG_API
constexpr uint32_t kDbgScanOnly = 1u << 30;  // SRD_DEBUG_API timing builds: the optimistic scan alone
#endif
// With timing events, the scan is launched by hipExtLaunchKernel, which
// stamps the events with the kernel's own start and stop (the dispatch
// packet's, as rocprofv3 sees them) instead of marker packets around it: a
// marker recorded on an idle stream before the launch runs while the host is
// still submitting the kernel (+30 us on the bracket), and one after it
// delays the next kernel (~6 us per call).
template <bool FULL>
static void launch_scan(unsigned g, const ScanArgs& a, hipStream_t s, hipEvent_t e0 = nullptr,
                        hipEvent_t e1 = nullptr) {
  const dim3 grid(g), block(scan_nw((int)a.variant) * 64);
#ifdef SRD_SCAN_MARKER_EVENTS  // timing A/B builds: marker events around a plain launch
  constexpr bool marker = true;
#else
  constexpr bool marker = false;
#endif
  if (e0 && marker) {  // timing A/B only: marker events around a plain launch
    (void)hipEventRecord(e0, s);
    launch_scan<FULL>(g, a, s);
    (void)hipEventRecord(e1, s);
  } else if (a.variant == SCAN_LINES) {  // line-per-lane tile loads (large stores: scan_variant_for)
    if (a.flen > kWide) hipExtLaunchKernelGGL(scan_kernel<FULL, true, SCAN_LINES>, grid, block, 0, s, e0, e1, 0, a);
    else hipExtLaunchKernelGGL(scan_kernel<FULL, false, SCAN_LINES>, grid, block, 0, s, e0, e1, 0, a);
#ifdef SRD_DEBUG_API
  } else if (a.variant == 7) {  // timing-only ablations (scan_kernel's V) inside one context
    hipExtLaunchKernelGGL(scan_kernel<FULL, false, 7>, grid, block, 0, s, e0, e1, 0, a);
  } else if (a.variant == 8) {
    hipExtLaunchKernelGGL(scan_kernel<FULL, false, 8>, grid, block, 0, s, e0, e1, 0, a);
#endif
  } else if (e0) {
    if (a.flen > kWide)
      hipExtLaunchKernelGGL(scan_kernel<FULL, true>, grid, block, 0, s, e0, e1, 0, a);
    else
      hipExtLaunchKernelGGL(scan_kernel<FULL, false>, grid, block, 0, s, e0, e1, 0, a);
  } else if (a.flen > kWide) {
    scan_kernel<FULL, true><<<grid, block, 0, s>>>(a);
  } else {
    scan_kernel<FULL, false><<<grid, block, 0, s>>>(a);
  }
}

static bool debug_env() {
  static const bool v = [] { const char* e = getenv("SRD_DEBUG"); return e && *e && *e != '0'; }();
  return v;
}

// Wait for the stream by polling (the call's result is on the host's
// critical path: a blocking wait's wake-up adds tens of us per call)
static hipError_t spin_sync(hipStream_t s) {
#ifdef SRD_NO_SPIN
  return hipStreamSynchronize(s);
#else
  hipError_t e;
  while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
  }
  return e;
#endif
}

// Spin until idx_emit's published words (IdxArgs::pub) all carry this
// call's seq; if the stream completes without them (an error), fail.
static int wait_publish(Ctx* c, uint64_t* w) {
  const uint32_t seq = c->pub_seq;
  volatile const uint64_t* pub = c->h_pub;
  for (uint64_t it = 0;; it++) {
    bool ok = true;
    for (int i = 0; i < PUB_WORDS; i++) {
      w[i] = pub[i];
      ok = ok && (uint32_t)(w[i] >> 32) == seq;
    }
    if (ok) return 0;
    if ((it & 1023) == 1023) {
      const hipError_t e = hipStreamQuery(c->stream);
      if (e == hipSuccess) {  // finished: re-read once, the words may have landed meanwhile
        bool ok2 = true;
        for (int i = 0; i < PUB_WORDS; i++) {
          w[i] = pub[i];
          ok2 = ok2 && (uint32_t)(w[i] >> 32) == seq;
        }
        if (ok2) return 0;
        set_err("internal: the glue finished without publishing its outcome");
        return SRD_ERR_INTERNAL;
      }
      if (e != hipErrorNotReady) HIPCHK(e);
    }
  }
}

// the 8 counters into pinned h_small[0..8) (no wait) / with the wait: the
// counters and, if extra != nullptr, the n_extra words enqueued into
// h_small[8..) before (one host wait for all of them; a copy into pageable
// memory would wait by itself)
static int enqueue_counters(Ctx* c) {
  HIPCHK(hipMemcpyAsync(c->h_small, P<uint64_t>(c, B_COUNTERS), 8 * 8, hipMemcpyDeviceToHost, c->stream));
  return 0;
}
static int enqueue_small(Ctx* c, const void* src, uint32_t word) {  // one u64 into h_small[8 + word]
  HIPCHK(hipMemcpyAsync(c->h_small + 8 + word, src, 8, hipMemcpyDeviceToHost, c->stream));
  return 0;
}
int read_counters(Ctx* c, uint64_t* h) {
  TRY(enqueue_counters(c));
  HIPCHK(spin_sync(c->stream));
  memcpy(h, c->h_small, 64);
  return 0;
}

// walk state (start) must already be on the device
int walk_and_mark(Ctx* c, const int64_t* par, const uint64_t* slot, uint64_t n, const uint64_t* map,
                  WalkState* hws) {
  WalkState* ws = P<WalkState>(c, B_WALK);
  uint8_t* core = P<uint8_t>(c, B_CORE);
  uint32_t* key = P<uint32_t>(c, B_DHEAD);
  HIPCHK(hipMemsetAsync(core, 0, n, c->stream));
  child_kernel<<<blocks(n, 256), 256, 0, c->stream>>>(par, n, core);
  KCHK(c, "child_kernel");
  core_key_kernel<<<blocks(n, 256), 256, 0, c->stream>>>(core, ws, n, key);
  KCHK(c, "core_key_kernel");
  size_t tb = c->bufs[B_CUB_TMP].n;
  HIPCHK(hipcub::DeviceScan::InclusiveScan(P<void>(c, B_CUB_TMP), tb, key, P<uint32_t>(c, B_RUNHEAD),
                                           hipcub::Max(), (int)n, c->stream));
  KCHK(c, "hipcub");
  head_key_kernel<<<blocks(n, 256), 256, 0, c->stream>>>(core, par, P<uint32_t>(c, B_RUNHEAD), n, key);
  KCHK(c, "head_key_kernel");
  tb = c->bufs[B_CUB_TMP].n;
  HIPCHK(hipcub::DeviceScan::InclusiveScan(P<void>(c, B_CUB_TMP), tb, key, P<uint32_t>(c, B_RUNHEAD),
                                           hipcub::Max(), (int)n, c->stream));
  KCHK(c, "hipcub");
  walk_kernel<<<1, 64, 0, c->stream>>>(par, P<uint32_t>(c, B_RUNHEAD), slot, P<u32x4>(c, B_CREC),
                                       P<uint64_t>(c, B_INTS), ws, n);
  KCHK(c, "walk_kernel");
  HIPCHK(hipGetLastError());
  static_assert(sizeof(WalkState) <= 64, "h_small[8..16)");
  HIPCHK(hipMemcpyAsync(c->h_small + 8, ws, sizeof(WalkState), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(spin_sync(c->stream));
  memcpy(hws, c->h_small + 8, sizeof(WalkState));
  if (hws->status != 1) return 0;
  mark_kernel<<<blocks(n, 256), 256, 0, c->stream>>>(P<uint64_t>(c, B_INTS), ws, n, core,
                                                     P<uint32_t>(c, B_ONPATH));
  KCHK(c, "mark_kernel");
  HIPCHK(hipMemsetAsync(P<uint32_t>(c, B_ONPATH) + n, 0, 4, c->stream));
  tb = c->bufs[B_CUB_TMP].n;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(P<void>(c, B_CUB_TMP), tb, P<uint32_t>(c, B_ONPATH),
                                          P<uint32_t>(c, B_CPOS), (int)(n + 1), c->stream));
  KCHK(c, "hipcub");
  scatter_chain_kernel<<<blocks(n, 256), 256, 0, c->stream>>>(P<uint32_t>(c, B_ONPATH), P<uint32_t>(c, B_CPOS), n,
                                                              map, P<uint64_t>(c, B_CHAIN_G));
  KCHK(c, "scatter_chain_kernel");
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(c->h_small + 8, P<uint32_t>(c, B_CPOS) + n, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(spin_sync(c->stream));
  hws->chain_len = 1 + (uint64_t)(uint32_t)c->h_small[8];
  return 0;
}

}  // namespace

struct srd_ctx : Ctx {};

// ScanPart::wq, the share of each wave slot of a block.  The SIMD's issue
// arbitration favours its older waves (slots 0-3 are the oldest on each
// SIMD, 12-15 the youngest), so an even split ended the slots at 1 : 1.069 :
// 1.125 : 1.179 by age group (tools/wave_stamps.py).  Default: per-slot
// shares from the wave stamps of per-age-group shares (1 : 1/1.069 : 1/1.125
// : 1/1.179), each slot's share scaled by (mean end / its end)^1.5: -1.3 to
// -1.6 % scan against the age-group shares, -0.8 % at power 1, -0.6 % at 2
// (tools/weights_ab.py: every set inside the same contexts).
// SRD_SCAN_WEIGHTS sets relative shares: 4 values (one per age group;
// "1,1,1,1" is the even split) or 16 (one per slot).
static void scan_weights(uint32_t (&wq)[16]) {
  double f[16] = {1.0000, 0.9787, 0.9796, 0.9788, 0.9081, 0.9072, 0.9074, 0.8915,
                  0.8432, 0.8324, 0.8337, 0.8314, 0.7726, 0.7701, 0.7712, 0.7590};
  if (const char* e = getenv("SRD_SCAN_WEIGHTS")) {
    // 4 or 16 finite positive values whose sum is finite; anything else
    // (unparsable, 'inf', 'nan', an overflowing sum) keeps the defaults
    double g[16], gs = 0;
    int n = 0;
    for (const char* q = e; n < 16 && *q;) {
      char* end = nullptr;
      const double x = strtod(q, &end);
      if (end == q || !(x > 0) || !std::isfinite(x)) { n = 0; break; }
      g[n++] = x;
      gs += x;
      q = *end == ',' ? end + 1 : end;
      if (*end && *end != ',') { n = 0; break; }
    }
    if (!std::isfinite(gs)) n = 0;
    if (n == 4)
      for (int v = 0; v < 16; v++) f[v] = g[v / 4];
    else if (n == 16)
      for (int v = 0; v < 16; v++) f[v] = g[v];
  }
  double sum = 0;
  for (double x : f) sum += x;
  uint32_t used = 0;
  for (int v = 0; v < 15; v++) used += wq[v] = (uint32_t)(65536.0 * f[v] / sum);
  wq[15] = 65536 - used;
}
#ifdef SRD_DEBUG_API  // timing builds: A/B of scan variants inside one context (one workspace)
extern "C" int srd_debug_set_scan_variant(srd_ctx* c, int v) {
  if (!c || !(v == 0 || v == 7 || v == 8 || v == SCAN_LINES)) return SRD_ERR_ARG;
  c->scan_variant = (uint32_t)v;
  return 0;
}
extern "C" int srd_debug_set_scan_bpc(srd_ctx* c, int bpc) {  // scan blocks per CU (1 or 2; one resident at a time)
  if (!c || bpc < 1 || bpc > 2) return SRD_ERR_ARG;
  c->scan_blocks = c->scan_cus * (unsigned)bpc;
  return 0;
}
extern "C" int srd_debug_set_xpart(srd_ctx* c, int on) {  // XCD-aware scan block shares on / off
  if (!c) return SRD_ERR_ARG;
  c->xpart_on = on != 0;
  return 0;
}
extern "C" int srd_debug_set_glue_fused(srd_ctx* c, int fused) {
  if (!c) return SRD_ERR_ARG;
  c->glue_fused = fused != 0;
  return 0;
}
extern "C" int srd_debug_set_scan_weights(srd_ctx* c, const double* w, int n) {
  if (!c || !w || (n != 4 && n != 16)) return SRD_ERR_ARG;
  double f[16], sum = 0;
  for (int v = 0; v < 16; v++) {
    sum += f[v] = n == 4 ? w[v / 4] : w[v];
    if (!(f[v] > 0) || !std::isfinite(f[v])) return SRD_ERR_ARG;
  }
  if (!std::isfinite(sum)) return SRD_ERR_ARG;
  uint32_t used = 0;
  for (int v = 0; v < 15; v++) used += c->scan_wq[v] = (uint32_t)(65536.0 * f[v] / sum);
  c->scan_wq[15] = 65536 - used;
  return 0;
}
#endif
extern "C" int srd_ctx_create(int device, srd_ctx** out) {
  if (!out) { set_err("null out"); return SRD_ERR_ARG; }
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) { set_err("bad device index"); return SRD_ERR_ARG; }
  HIPCHK(hipSetDevice(device));
  auto* c = new srd_ctx();
  c->device = device;
  c->bufs.resize(B_COUNT_);
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    set_err("hipStreamCreate failed");
    return SRD_ERR_HIP;
  }
  int r = upload_tables();
  if (r) { delete c; return r; }
  // timing events (srd_ctx_timings) with a device-scope release: a default
  // event's system-scope release (an L2 write-back) put ~5 us into the
  // timeline at each record (four per call)
  for (auto& e : c->ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventReleaseToDevice));
  HIPCHK(hipEventCreateWithFlags(&c->ev_ready, hipEventDisableTiming));
  HIPCHK(hipHostMalloc((void**)&c->h_plan, sizeof(Plan), hipHostMallocDefault));
  HIPCHK(hipHostMalloc((void**)&c->h_pub, 64, hipHostMallocCoherent));  // fine-grained: the device's system-scope stores land here
  memset(c->h_pub, 0, 64);
  HIPCHK(hipHostMalloc((void**)&c->h_small, 256, hipHostMallocDefault));
  c->stage_workers = (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
    c->scan_cus = c->scan_blocks = (unsigned)ncu;
  scan_weights(c->scan_wq);
  if (const char* e = getenv("SRD_SLOT_LIMIT_LOG2")) {
    const long v = strtol(e, nullptr, 10);
    if (v >= 10 && v <= 31) c->slot_limit = 1ull << v;
  }
  // the scan's tile loads for every store size: "lines" (line-per-lane) or
  // "coal" (coalesced + transpose); unset = by size (scan_variant_for).  The
  // results are identical either way (tests/test_gpu_parity.py runs both)
  if (const char* e = getenv("SRD_SCAN_LOADS")) {
    if (!strcmp(e, "lines")) c->loads_pin = SCAN_LINES;
    else if (!strcmp(e, "coal")) c->loads_pin = 0;
  }
  if (const char* e = getenv("SRD_GLUE_FUSED")) c->glue_fused = strcmp(e, "0") != 0;
  if (const char* e = getenv("SRD_XPART")) c->xpart_on = strcmp(e, "0") != 0;
  if (const char* e = getenv("SRD_LB_FAIL_BLOCK")) {
    char* end = nullptr;
    const unsigned long v = strtoul(e, &end, 10);
    if (end != e && v < CHAIN_BLOCKS) c->lb_fail = (uint32_t)v;
  }
  *out = c;
  return 0;
}

extern "C" void srd_ctx_destroy(srd_ctx* c) {
  if (!c) return;
  delete c->worker;  // idle between calls: joins at once
  hipSetDevice(c->device);
  if (c->ev_ready) hipEventDestroy(c->ev_ready);
  for (auto& b : c->bufs)
    if (b.p) hipFree(b.p);
  if (c->file.p) hipFree(c->file.p);
  for (auto& e : c->ev)
    if (e) hipEventDestroy(e);
  for (auto& e : c->sev)
    if (e) hipEventDestroy(e);
  if (c->h_plan) hipHostFree(c->h_plan);
  if (c->h_pub) hipHostFree(c->h_pub);
  if (c->h_small) hipHostFree(c->h_small);
  if (c->h_out) hipHostFree(c->h_out);
  for (int i = 0; i < 2; i++) {
    if (c->pin_ent[i]) hipHostFree(c->pin_ent[i]);
    if (c->wev_copied[i]) hipEventDestroy(c->wev_copied[i]);
    if (c->wev_done[i]) hipEventDestroy(c->wev_done[i]);
  }
  if (c->cstream) hipStreamDestroy(c->cstream);
  for (auto p : c->stage_pin)
    if (p) hipHostFree(p);
  for (auto e : c->stage_ev)
    if (e) hipEventDestroy(e);
  for (auto st : c->stage_streams)
    if (st) hipStreamDestroy(st);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

extern "C" void* srd_ctx_stream(srd_ctx* c) { return c ? (void*)c->stream : nullptr; }
extern "C" int srd_ctx_scan_loads(srd_ctx* c) { return c ? c->last_loads : -1; }
extern "C" int srd_ctx_scan_trial(srd_ctx* c, double* ms) {
  if (!c) return -1;
  if (ms)
    for (int k = 0; k < 2; k++) ms[k] = c->tune.n[k] ? (double)c->tune.best[k] * 1e-5 : 0.0;  // 10 ns ticks
  return c->tune.choice;
}
extern "C" uint64_t srd_ctx_device_bytes(srd_ctx* c) {
  if (!c) return 0;
  uint64_t n = c->file.n;
  for (const Buf& b : c->bufs) n += b.n;
  return n;
}

// A store of another size starts at the default again; a store within 2x of
// the size whose overflow grew the cap keeps that cap (a dense store would
// otherwise overflow -- and rescan -- on every call).
static void fit_cap(CandCap& k, uint64_t bytes) {
  const bool similar = k.grown_bytes && bytes <= 2 * k.grown_bytes && 2 * bytes >= k.grown_bytes;
  k.cap = similar ? std::max(k.grown_cap, k.floor) : k.floor;
}
static void grow_cap(CandCap& k, uint64_t bytes) {
  k.cap = (uint32_t)std::min<uint64_t>((uint64_t)k.cap * 4, SPAN_BYTES);
  k.grown_cap = k.cap;
  k.grown_bytes = bytes;
}

// the scan grid of `variant` over ns resident spans: blocks (<= blocks per
// CU x CUs) and waves per block (scan_nw / scan_bpc)
static unsigned scan_grid(const Ctx* c, uint32_t variant, uint64_t ns, uint32_t* nw) {
  *nw = (uint32_t)scan_nw((int)variant);
  return (unsigned)std::min<uint64_t>((ns + *nw - 1) / *nw, (uint64_t)c->scan_blocks);
}
static ScanPart scan_part(const Ctx* c, uint64_t s_lo, uint64_t ns, unsigned g, uint32_t nw) {
  ScanPart p{};
  p.s_lo = s_lo;
  p.ns = ns;
  p.g = g;
  p.nw = nw;
  if (nw == 16) {
    for (int q = 0; q < 16; q++) p.wq[q] = c->scan_wq[q];
  } else {  // (the fitted shares are the 16-wave block's) an even split
    for (uint32_t q = 0; q < nw; q++) p.wq[q] = 65536u / nw;
    p.wq[nw - 1] += 65536u - nw * (65536u / nw);
  }
  part_fill_cw(p);
  return p;
}
// an upper bound on the spans of one wave; xpart: with XCD-aware block
// shares, a block holds at most (1 + XP_CLAMP) / (1 - XP_CLAMP) < 1.25 of
// the even share + 1 span (xpart_update)
static uint64_t part_max_wave_spans(const ScanPart& p, bool xpart = false) {
  if (!p.g) return 1;
  const uint32_t wmax = *std::max_element(p.wq, p.wq + p.nw);
  const uint64_t nb = xpart ? (p.ns * 5 + 4 * p.g - 1) / (4 * p.g) + 1 : (p.ns + p.g - 1) / p.g;
  return (nb * wmax + 65535) / 65536 + 1;
}

// the scan kernel's per-wave results and last-block reduction (ScanArgs)
static int scan_wave_args(Ctx* c, ScanArgs* a) {
  const uint64_t W = (uint64_t)c->scan_blocks * 32;  // up to 32 waves per CU (scan_grid)
  TRY(ensure(c, B_WTOT, W * 8));
  TRY(ensure(c, B_WROOT, W * 8));
  TRY(ensure(c, B_KTOT, 64));
  TRY(ensure_z(c, B_DONE, 64));  // zero once; the scan's last block resets it
  a->wave_total = P<uint64_t>(c, B_WTOT);
  a->wave_root = P<uint64_t>(c, B_WROOT);
  a->k_total = P<uint64_t>(c, B_KTOT);
  a->done = P<uint32_t>(c, B_DONE);
  return 0;
}

static int alloc_scan(Ctx* c, uint64_t n_tiles, uint64_t n_spans, uint32_t cap) {
  const uint64_t slots = n_spans * cap;
  TRY(ensure(c, B_TILE, n_tiles * 16));
  TRY(ensure(c, B_SPAN_COUNT, (n_spans + 1) * 4));
  TRY(ensure(c, B_SPAN_BASE, (n_spans + 1) * 8));
  TRY(ensure(c, B_CM, slots * 8));
  TRY(ensure(c, B_CREC, slots * 32));
  TRY(ensure(c, B_COUNTERS, 8 * 8));
  TRY(ensure(c, B_WALK, sizeof(WalkState)));
  return 0;
}

// the second half of every candidate record (ScanArgs::c_rec1): B_CREC's
// upper half (its lower half is c_rec), fixed while the buffer is
static u32x4* crec1(Ctx* c) { return P<u32x4>(c, B_CREC) + c->bufs[B_CREC].n / 32; }

static int alloc_dense(Ctx* c, uint64_t K) {
  TRY(ensure(c, B_DM, K * 8));
  TRY(ensure(c, B_DPAR, K * 8));
  TRY(ensure(c, B_DSLOT, K * 8));
  TRY(ensure(c, B_DHEAD, K * 4));    // run keys / heads: g + 1 in 32 bits (K < 2^32 - 1: run_scan)
  TRY(ensure(c, B_RUNHEAD, K * 4));
  TRY(ensure(c, B_INTS, K * 16 + 16));
  TRY(ensure(c, B_ONPATH, (K + 1) * 4));
  TRY(ensure(c, B_CPOS, (K + 1) * 4));
  TRY(ensure(c, B_CHAIN_G, (K + 1) * 8));
  TRY(ensure(c, B_CORE, K + 1));
  TRY(ensure_cub(c, K + 1));
  return 0;
}

static int alloc_out(Ctx* c, uint64_t n) {
  TRY(ensure(c, B_O_MO, n * 8));
  TRY(ensure(c, B_O_KH, n * 8));
  TRY(ensure(c, B_O_PREV, n * 8));
  TRY(ensure(c, B_O_START, n * 8));
  TRY(ensure(c, B_O_LEN, n * 8));
  TRY(ensure(c, B_O_CRCST, n * 4));
  TRY(ensure(c, B_O_CRC, n * 4));
  TRY(ensure(c, B_O_OK, n));
  TRY(ensure(c, B_O_PIECES, n * 4));
  TRY(ensure(c, B_O_SUF, n * 4));
  TRY(ensure(c, B_O_SXM, n * 4));
  TRY(ensure(c, B_O_TAIL, n * 4));
  TRY(ensure(c, B_SLOW, n * 8));
  TRY(ensure(c, B_IKEY, n * 8));
  TRY(ensure(c, B_IPACKED, n * 8));
  TRY(ensure(c, B_O_PACKED, n * 8));
  return 0;
}

// global-table KeyIndexer::build workspace (full pass / skewed-bucket fallback)
static int alloc_hash(Ctx* c, uint64_t n) {
  uint64_t hc = 64;
  while (hc < 2 * n) hc <<= 1;
  TRY(ensure(c, B_HKEYS, hc * 8));
  TRY(ensure(c, B_HVALS, hc * 8));
  TRY(ensure(c, B_LATEST, (n + 1) * 4));
  TRY(ensure(c, B_IPOS, (n + 1) * 4));
  TRY(ensure_cub(c, n + 1));
  return 0;
}

// timing-only builds (make variant DEFS=-DSRD_INDEX_GLOBAL): every index by
// the global table; the product build takes it only on a bucket overflow
static constexpr bool index_global_env() {
#ifdef SRD_INDEX_GLOBAL
  return true;
#else
  return false;
#endif
}

// KeyIndexer::build over n (key_hash, meta_off) pairs in file order with one
// global open-addressing table (device-wide atomics); syncs for the count.
// Default pairs: the chain in B_O_KH / B_O_MO -> B_IKEY / B_IPACKED.
static int index_global(Ctx* c, uint64_t n, uint64_t* n_index, const uint64_t* kh = nullptr,
                        const uint64_t* mo = nullptr, uint64_t* okey = nullptr, uint64_t* opacked = nullptr) {
  if (!kh) { kh = P<uint64_t>(c, B_O_KH); mo = P<uint64_t>(c, B_O_MO); }
  TRY(alloc_hash(c, n));
  if (!okey) { okey = P<uint64_t>(c, B_IKEY); opacked = P<uint64_t>(c, B_IPACKED); }
  uint64_t* cnt = P<uint64_t>(c, B_COUNTERS);
  uint64_t hc = 64;
  while (hc < 2 * n) hc <<= 1;
  HIPCHK(hipMemsetAsync(P<void>(c, B_HKEYS), 0xff, hc * 8, c->stream));
  HIPCHK(hipMemsetAsync(P<void>(c, B_HVALS), 0, hc * 8, c->stream));
  HIPCHK(hipMemsetAsync(cnt + 7, 0, 8, c->stream));
  HIPCHK(hipMemsetAsync(P<uint32_t>(c, B_LATEST) + n, 0, 4, c->stream));
  if (n) {
    index_insert_kernel<<<blocks(n, 256), 256, 0, c->stream>>>(
        kh, mo, n, P<uint64_t>(c, B_HKEYS), P<unsigned long long>(c, B_HVALS), hc - 1, (unsigned long long*)(cnt + 7));
    KCHK(c, "index_insert_kernel");
    index_latest_kernel<<<blocks(n, 256), 256, 0, c->stream>>>(
        kh, mo, n, P<uint64_t>(c, B_HKEYS), P<unsigned long long>(c, B_HVALS), hc - 1, (unsigned long long*)(cnt + 7),
        P<uint32_t>(c, B_LATEST));
    KCHK(c, "index_latest_kernel");
    HIPCHK(hipGetLastError());
  }
  size_t tb = c->bufs[B_CUB_TMP].n;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(P<void>(c, B_CUB_TMP), tb, P<uint32_t>(c, B_LATEST),
                                          P<uint32_t>(c, B_IPOS), (int)(n + 1), c->stream));
  KCHK(c, "hipcub");
  if (n) {
    index_emit_kernel<<<blocks(n, 256), 256, 0, c->stream>>>(kh, mo, P<uint32_t>(c, B_LATEST), P<uint32_t>(c, B_IPOS),
                                                             n, okey, opacked);
    KCHK(c, "index_emit_kernel");
    HIPCHK(hipGetLastError());
  }
  uint32_t nidx = 0;
  HIPCHK(hipMemcpyAsync(&nidx, P<uint32_t>(c, B_IPOS) + n, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(spin_sync(c->stream));
  *n_index = nidx;
  return 0;
}

static void set_out_ptrs(Ctx* c, srd_device_result* out) {
  out->meta_off = P<uint64_t>(c, B_O_MO);
  out->key_hash = P<uint64_t>(c, B_O_KH);
  out->prev_offset = P<uint64_t>(c, B_O_PREV);
  out->payload_start = P<uint64_t>(c, B_O_START);
  out->payload_len = P<uint64_t>(c, B_O_LEN);
  out->crc_stored = P<uint32_t>(c, B_O_CRCST);
  out->crc_computed = P<uint32_t>(c, B_O_CRC);
  out->crc_ok = P<uint8_t>(c, B_O_OK);
  out->index_key_hash = P<uint64_t>(c, B_IKEY);
  out->index_packed = P<uint64_t>(c, B_IPACKED);
}

static int index_build_sep(Ctx* c, const uint64_t* keys, const uint64_t* vals, uint64_t n, uint64_t* okeys,
                           uint64_t* opacked, uint64_t* n_index);
// finalize + index for a chain of n entries whose chain_g / walk state are set
static int finish(Ctx* c, const uint8_t* d_file, uint64_t flen, uint64_t n, uint32_t flags,
                  srd_device_result* out) {
  TRY(alloc_out(c, n));
  uint64_t* cnt = P<uint64_t>(c, B_COUNTERS);
  HIPCHK(hipMemsetAsync(cnt + 5, 0, 16, c->stream));  // n_slow, n_bad
  FinArgs f{};
  f.file = d_file;
  f.flen = flen;
  f.n_chain = n;
  f.chain_g = P<uint64_t>(c, B_CHAIN_G);
  f.slot = P<uint64_t>(c, B_DSLOT);
  f.par = P<int64_t>(c, B_DPAR);
  f.ws = P<WalkState>(c, B_WALK);
  f.c_m = P<uint64_t>(c, B_CM);
  f.c_rec = P<u32x4>(c, B_CREC);
  f.c_rec1 = crec1(c);
  f.tile = P<uint32_t>(c, B_TILE);
  f.no_crc = (flags & SRD_FLAG_NO_CRC) ? 1 : 0;
  f.coff = 1;
  f.o_mo = P<uint64_t>(c, B_O_MO);
  f.o_kh = P<uint64_t>(c, B_O_KH);
  f.o_prev = P<uint64_t>(c, B_O_PREV);
  f.o_start = P<uint64_t>(c, B_O_START);
  f.o_len = P<uint64_t>(c, B_O_LEN);
  f.o_crc_st = P<uint32_t>(c, B_O_CRCST);
  f.o_crc = P<uint32_t>(c, B_O_CRC);
  f.o_pieces = P<uint32_t>(c, B_O_PIECES);
  f.o_suf = P<uint32_t>(c, B_O_SUF);
  f.o_sxm = P<uint32_t>(c, B_O_SXM);
  f.o_tail = P<uint32_t>(c, B_O_TAIL);
  f.o_ok = P<uint8_t>(c, B_O_OK);
  f.slow_list = P<uint64_t>(c, B_SLOW);
  f.n_slow = (unsigned long long*)(cnt + 5);
  f.n_bad = (unsigned long long*)(cnt + 6);
  if (n) {
    finalize_kernel<<<blocks(n, 256), 256, 0, c->stream>>>(f);
    KCHK(c, "finalize_kernel");
    HIPCHK(hipGetLastError());
    if (!f.no_crc) {
      slow_kernel<<<2048 / SLOW_WAVES, SLOW_WAVES * 64, 0, c->stream>>>(f);
      KCHK(c, "slow_kernel");
      HIPCHK(hipGetLastError());
    }
  }
  // ---- KeyIndexer::build (bucketed; the global table if a bucket overflows) ----
  // the counters (n_bad: final after finalize / slow) ride on the build's wait
  TRY(enqueue_counters(c));
  uint64_t nidx = 0;
  TRY(index_build_sep(c, P<uint64_t>(c, B_O_KH), P<uint64_t>(c, B_O_MO), n, P<uint64_t>(c, B_IKEY),
                      P<uint64_t>(c, B_IPACKED), &nidx));
  if (!n) HIPCHK(spin_sync(c->stream));  // index_build_sep waited only for n > 0
  uint64_t h[8];
  memcpy(h, c->h_small, 64);
  out->n_index = nidx;
  out->n_crc_bad = h[6];
  out->n_chain = n;
  set_out_ptrs(c, out);
  return 0;
}

// read out the oldest n pending scan event pairs (their launches completed
// before the call that made them returned)
static int drain_scan_events(Ctx* c, uint32_t n) {
  for (; n && c->sev_pending; n--) {
    const uint32_t i = (c->sev_next - c->sev_pending) % Ctx::kScanRing;
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, c->sev[2 * i], c->sev[2 * i + 1]));
    c->scan_ms += ms;
    c->scan_launches++;
    if (c->scan_list.size() < (1u << 16)) c->scan_list.push_back(ms);
    c->sev_pending--;
  }
  return 0;
}
// the event pair for the next scan launch (none below SRD_TIMING_SCAN)
static int next_scan_events(Ctx* c, hipEvent_t* e0, hipEvent_t* e1) {
  *e0 = *e1 = nullptr;
  if (c->timing < SRD_TIMING_SCAN) return 0;
  if (c->timing_seq++ % c->timing_every) return 0;  // srd_ctx_set_timing_every: a sampled launch only
  if (c->sev_pending == Ctx::kScanRing) TRY(drain_scan_events(c, 1));
  const uint32_t i = c->sev_next++ % Ctx::kScanRing;
  c->sev_pending++;
  *e0 = c->sev[2 * i];
  *e1 = c->sev[2 * i + 1];
  return 0;
}

// The scan's tile loads (scan_kernel): coalesced nontemporal loads + an
// in-register transpose (V 0) or round 4's line-per-lane loads (SCAN_LINES).
// Which one streams faster depends on the store and on the box: in round 5's
// same-context A/Bs (profiles/r05/variant_ab_coal_*.txt) the coalesced loads
// were 7.5 % faster on C2, 4.8 % slower on C3 (72.5 GB), and on round 6's
// boxes the line-per-lane loads were also faster on C2 in 2 of 3 contexts
// (profiles/r06/variant_ab_body_stream_c2.txt).  So the optimistic pass
// measures: for each store (span count, grid) its first scan runs coalesced
// and is not counted, the next ones alternate the patterns, each timed on the
// device (the scan's first block start to its last block end, XPart::
// scan_ticks, published with the outcome: no host wait, no event), and the
// pattern with the faster best time is kept for the store: from the fourth
// measured call on as soon as the bests differ by more than TUNE_MARGIN, at
// the eighth in any case (a close call costs little either way); measured
// again every 4096 calls.  srd_ctx_scan_trial reports the two best times.
// SRD_SCAN_LOADS pins a pattern; the debug build's srd_debug_set_scan_variant
// overrides both; the full pass takes the current choice (coalesced before one).
constexpr uint32_t TUNE_WARM = 1, TUNE_TRIAL = 4, TUNE_TRIAL_MAX = 8, TUNE_EVERY = 4096;
constexpr double TUNE_MARGIN = 0.02;
static uint32_t scan_variant_for(const Ctx* c, uint64_t) {
  if (c->scan_variant) return c->scan_variant;
  if (c->loads_pin >= 0) return (uint32_t)c->loads_pin;
  return c->tune.choice == 1 ? (uint32_t)SCAN_LINES : 0u;
}
static uint32_t scan_variant_tune(Ctx* c, uint64_t ns, uint32_t g) {
  if (c->scan_variant) return c->scan_variant;
  if (c->loads_pin >= 0) return (uint32_t)c->loads_pin;
  Ctx::LoadTune& t = c->tune;
  if (t.ns != ns || t.g != g || (t.choice >= 0 && t.calls >= TUNE_WARM + TUNE_TRIAL_MAX + TUNE_EVERY)) {
    t = Ctx::LoadTune{};
    t.ns = ns;
    t.g = g;
  }
  if (t.choice >= 0) return t.choice ? (uint32_t)SCAN_LINES : 0u;
  const uint32_t i = t.calls;  // the trial's order: coalesced (warm-up), then coalesced, lines, coalesced, ...
  return i >= TUNE_WARM && ((i - TUNE_WARM) & 1) ? (uint32_t)SCAN_LINES : 0u;
}
// one optimistic scan of the tuned store done: its pattern and device ticks
// (0: not measured -- XCD-aware shares off)
static void scan_tune_feedback(Ctx* c, uint32_t var, uint64_t ticks) {
  Ctx::LoadTune& t = c->tune;
  const uint32_t i = t.calls++;
  if (t.choice >= 0 || i < TUNE_WARM || !ticks || c->scan_variant || c->loads_pin >= 0) return;
  const int k = var == SCAN_LINES ? 1 : 0;
  if (!t.n[k] || ticks < t.best[k]) t.best[k] = ticks;
  t.n[k]++;
  const uint32_t m = t.n[0] + t.n[1];
  if (m < TUNE_TRIAL || !t.n[0] || !t.n[1]) return;
  const double b0 = (double)t.best[0], b1 = (double)t.best[1];
  if (m >= TUNE_TRIAL_MAX || fabs(b0 - b1) > TUNE_MARGIN * fmin(b0, b1)) t.choice = b1 < b0 ? 1 : 0;
}

static int run_scan(Ctx* c, const uint8_t* d_file, uint64_t flen, bool full, uint64_t* K, uint64_t* h) {
  const uint64_t n_tiles = (flen + TILE - 1) / TILE;
  const uint64_t n_spans = (n_tiles + SPAN_TILES - 1) / SPAN_TILES;
  fit_cap(c->cfull, flen);
  while (true) {
    TRY(alloc_scan(c, n_tiles, n_spans, c->cfull.cap));
    TRY(ensure_cub(c, n_spans + 1));
    uint64_t* cnt = P<uint64_t>(c, B_COUNTERS);
    HIPCHK(hipMemsetAsync(cnt, 0, 64, c->stream));
    // the scan writes every span's count; only the scan sentinel needs a zero
    HIPCHK(hipMemsetAsync(P<uint32_t>(c, B_SPAN_COUNT) + n_spans, 0, 4, c->stream));
    ScanArgs a{};
    a.variant = scan_variant_for(c, flen);
    a.file = d_file;
    a.flen = flen;
    a.n_tiles = n_tiles;
    a.n_spans = n_spans;
    a.cap = c->cfull.cap;
    a.tile = P<uint32_t>(c, B_TILE);
    a.span_count = P<uint32_t>(c, B_SPAN_COUNT);
    a.c_m = P<uint64_t>(c, B_CM);
    a.c_rec = P<u32x4>(c, B_CREC);
    a.c_rec1 = crec1(c);
    a.counters = (unsigned long long*)cnt;
    a.filt_hb = (uint32_t)((flen ? flen - 1 : 0) >> 32);
    TRY(ensure(c, B_SPAN_FIRST, (n_spans + 1) * 4));
    a.span_first = P<uint32_t>(c, B_SPAN_FIRST);
    a.wcap = 0;  // the full pass stores records at span * cap + slot
    TRY(scan_wave_args(c, &a));
    if (n_spans) {
      uint32_t nw;
      const unsigned g = scan_grid(c, a.variant, n_spans, &nw);
      a.part = scan_part(c, 0, n_spans, g, nw);
      hipEvent_t e0, e1;
      TRY(next_scan_events(c, &e0, &e1));
      if (full)
        launch_scan<true>(g, a, c->stream, e0, e1);
      else
        launch_scan<false>(g, a, c->stream, e0, e1);
      KCHK(c, "scan_kernel");
      HIPCHK(hipGetLastError());
    }
    size_t tb = c->bufs[B_CUB_TMP].n;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(P<void>(c, B_CUB_TMP), tb, P<uint32_t>(c, B_SPAN_COUNT),
                                            P<uint64_t>(c, B_SPAN_BASE), (int)(n_spans + 1), c->stream));
    KCHK(c, "hipcub");
    TRY(enqueue_small(c, P<uint64_t>(c, B_SPAN_BASE) + n_spans, 0));
    TRY(read_counters(c, h));
    *K = c->h_small[8];
    if (*K >= 0xFFFFFFFFull) { set_err("more than 2^32 - 2 chain-node candidates (full pass)"); return SRD_ERR_ALLOC; }
    if ((uint32_t)h[2] == 0) break;
    if (c->cfull.cap >= SPAN_BYTES) { set_err("candidate overflow"); return SRD_ERR_INTERNAL; }
    grow_cap(c->cfull, flen);
  }
  if (*K) {
    TRY(alloc_dense(c, *K));
    LinkArgs l{};
    l.file = d_file;
    l.flen = flen;
    l.n_spans = n_spans;
    l.cap = c->cfull.cap;
    l.span_count = P<uint32_t>(c, B_SPAN_COUNT);
    l.span_base = P<uint64_t>(c, B_SPAN_BASE);
    l.c_m = P<uint64_t>(c, B_CM);
    l.c_rec = P<u32x4>(c, B_CREC);
    l.d_m = P<uint64_t>(c, B_DM);
    l.d_par = P<int64_t>(c, B_DPAR);
    l.d_slot = P<uint64_t>(c, B_DSLOT);
    link_kernel<<<blocks(n_spans, 256 / LINK_LANES), 256, 0, c->stream>>>(l);
    KCHK(c, "link_kernel");
    HIPCHK(hipGetLastError());
  } else {
    TRY(alloc_dense(c, 1));
  }
  return 0;
}

__global__ void walk_start_kernel(WalkState* ws, const uint64_t* vpos, uint64_t g) {
  if (threadIdx.x == 0) {
    WalkState w{};
    w.start = vpos[g];
    *ws = w;
  }
}
__global__ void compact_valid_kernel(const uint32_t* vflag, const uint32_t* vscan, uint64_t K, uint64_t* vlist,
                                     uint64_t* vpos, uint64_t* nv) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= K) return;
  const uint32_t pos = vscan[g], f = vflag[g];
  if (f) {
    vlist[pos] = g;
    vpos[g] = pos;
  }
  if (g == K - 1) *nv = (uint64_t)pos + (f ? 1 : 0);
}

static int set_single_root(Ctx* c, uint64_t t) {
  WalkState w{};
  w.status = 1;
  w.chain_len = 1;
  w.root_t = t;
  w.final_len = t;
  HIPCHK(hipMemcpyAsync(P<WalkState>(c, B_WALK), &w, sizeof w, hipMemcpyHostToDevice, c->stream));
  return 0;
}


// KeyIndexer::build (key_indexer.rs:98-124) as a bucketed build over the
// pairs (kh[i], mo[i]), i < *n_dev, in file order (latest = last position);
// *status != 0 disables it.  Scratch (alloc_index): B_HOFF = the bucket fills [nbk] (zero
// before the claims) followed by the chunk counts [GLUE_BLOCKS], B_SKEY = nbk
// buckets of IDX_TCAP records, B_LATEST8.  pl->n_index / pl->idx_overflow are
// written.
static int alloc_index(Ctx* c, uint64_t n_cap, uint32_t log2_nbk) {
  const uint64_t nbk = (uint64_t)1 << log2_nbk;
  TRY(ensure(c, B_HOFF, (nbk + GLUE_BLOCKS) * 4));
  TRY(ensure(c, B_SKEY, nbk * IDX_TCAP * 8));
  TRY(ensure_z(c, B_LATEST8, n_cap + 1));  // zero on (re)allocation: no entry carries a live generation
  return 0;
}
// a fresh generation of the non-latest marks for each index build (the
// array is cleared once every 255 builds)
static int next_lgen(Ctx* c) {
  if (++c->lgen == 0) {
    HIPCHK(hipMemsetAsync(P<void>(c, B_LATEST8), 0, c->bufs[B_LATEST8].n, c->stream));
    c->lgen = 1;
  }
  return 0;
}
// the words every index build needs zeroed: the bucket fills and, after them,
// the per-chunk non-latest counts (IdxArgs::ccount)
static uint32_t* index_zero_words(Ctx* c, uint32_t log2_nbk, uint32_t* n) {
  *n = (1u << log2_nbk) + GLUE_BLOCKS;
  return P<uint32_t>(c, B_HOFF);
}
static uint32_t index_log2_buckets(uint64_t n_est) {
  uint32_t log2_nbk = 1;  // >= 1: the bucket is the hash's top log2_nbk bits
  while (log2_nbk < 14 && ((uint64_t)IDX_BUCKET_AVG << log2_nbk) < n_est) log2_nbk++;
  return log2_nbk;
}
static IdxArgs index_args(Ctx* c, uint32_t log2_nbk) {
  IdxArgs ia{};
  ia.log2_nbk = log2_nbk;
  ia.bfill = P<uint32_t>(c, B_HOFF);
  ia.ccount = ia.bfill + ((size_t)1 << log2_nbk);
  ia.srec = P<uint64_t>(c, B_SKEY);
  ia.latest = P<uint8_t>(c, B_LATEST8);
  ia.lgen = c->lgen;
  return ia;
}
// fused: chain_finalize_kernel already claimed the bucket ranges and wrote
// the records (child2_kernel zeroed the fills); otherwise the fills are
// zeroed here, and idx_hist_scatter_kernel claims the ranges and fills them
static int launch_index_bucketed(Ctx* c, const uint64_t* kh, const uint64_t* mo, const uint64_t* n_dev,
                                 const uint32_t* status, uint32_t log2_nbk, uint64_t* okey, uint64_t* opacked,
                                 Plan* pl, bool fused = false, const FinArgs* slow = nullptr, bool zeroed = false,
                                 const uint64_t* scan_ticks = nullptr) {
  TRY(next_lgen(c));
  IdxArgs ia = index_args(c, log2_nbk);
  ia.alias = fused ? 1u : 0u;
  if (fused) {
    ia.pub = c->h_pub;
    ia.pub_seq = ++c->pub_seq;
    ia.scan_ticks = scan_ticks;  // (the optimistic scan's device time, XPart)
  }
  ia.kh = kh;
  ia.mo = mo;
  ia.n_dev = n_dev;
  ia.status = status;
  ia.okey = okey;
  ia.opacked = opacked;
  ia.plan = pl;
  const uint32_t nbk = 1u << log2_nbk;
  if (!fused) {
    uint32_t nz = 0;
    uint32_t* zw = index_zero_words(c, log2_nbk, &nz);
    if (!zeroed) HIPCHK(hipMemsetAsync(zw, 0, (size_t)nz * 4, c->stream));
    idx_hist_scatter_kernel<<<IDX_HBLOCKS, 256, nbk * 4, c->stream>>>(ia);
    KCHK(c, "idx_hist_scatter_kernel");
  }
  FinArgs fs{};  // n_slow == nullptr: no slow list
  if (slow) fs = *slow;
  idx_dedup_kernel<<<nbk, 512, 0, c->stream>>>(ia, fs);
  KCHK(c, "idx_dedup_kernel");
  idx_emit_kernel<<<GLUE_BLOCKS, GLUE_THREADS, 0, c->stream>>>(ia);
  KCHK(c, "idx_emit_kernel");
  HIPCHK(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------
// Optimistic pass, sync-free: scan (strong candidates only) -> link -> shape
// check -> chain scatter -> finalize -> bucketed index, all counts on the
// device; one host sync at the end.  *done=false sends the call to the full
// pass (the check could not prove the chain from file_len).
static int alloc_fast(Ctx* c, uint64_t capK, uint32_t log2_nbk) {
  TRY(ensure(c, B_DPAR, capK * 4));
  TRY(ensure_z(c, B_HASCHILD, capK * 4));
  TRY(ensure_z(c, B_HASCHILD2, capK * 4));
  TRY(ensure_z(c, B_CHILDOF, capK * 8));
  TRY(ensure(c, B_FLAG, capK));
  TRY(ensure(c, B_PART, GLUE_BLOCKS * 4));
  TRY(ensure(c, B_PARTEX, CHAIN_BLOCKS * CHAIN_WAVES * 4));
  TRY(ensure_z(c, B_LOOKB, CHAIN_BLOCKS * 8));  // look-back granules: zero = no call's tag
  TRY(ensure(c, B_PLAN, sizeof(Plan)));
  TRY(alloc_out(c, capK + 1));
  TRY(alloc_index(c, capK, log2_nbk));
  return 0;
}

// Span mode (lo > 0): d_span holds file bytes [span_off, flen) (span_off a
// multiple of SPAN_BYTES, <= lo); the chain must run from flen down to an
// entry whose prev == lo.  Whole file: span_off = lo = 0.
static int optimistic_pass(Ctx* c, const uint8_t* d_span, uint64_t span_off, uint64_t lo, uint64_t flen,
                           uint32_t flags, srd_device_result* out, bool* done) {
  *done = false;
  const uint8_t* d_file = d_span - span_off;  // absolute file offsets index d_file (only [span_off, ..) is read)
  const uint64_t n_tiles = (flen + TILE - 1) / TILE;
  const uint64_t n_spans = (n_tiles + SPAN_TILES - 1) / SPAN_TILES;
  const uint64_t k_lo = span_off / TILE, s_lo = k_lo / SPAN_TILES;
  const uint64_t nt_rel = n_tiles - k_lo, ns_rel = n_spans - s_lo;
  const uint32_t coff = lo ? 0u : 1u;
  fit_cap(c->copt, flen - span_off);
  for (int attempt = 0; attempt < 6; attempt++) {
    // index buckets: ~IDX_BUCKET_AVG chain entries per bucket
    const uint64_t n_est = std::max<uint64_t>(std::max<uint64_t>(c->last_n, (flen - span_off) / 4096), 1);
    const uint32_t log2_nbk = index_log2_buckets(n_est);
    // the scan's partition (ScanPart): total_waves waves of at most spw
    // spans; each wave's records are dense in its region of wcap = spw * cap slots
    // (the variant once: its geometry sizes the partition and the launch;
    // every variant has the same grid)
    uint32_t nw;
    const unsigned g = scan_grid(c, 0, ns_rel, &nw);
    const uint32_t var = scan_variant_tune(c, ns_rel, g);
    c->last_loads = var == SCAN_LINES ? 1 : var == 0 ? 0 : -1;
    ScanPart part = scan_part(c, s_lo, ns_rel, g, nw);
    const bool xpart = c->xpart_on && g <= XP_MAX_BLOCKS;
    XPart* xp = nullptr;
    if (xpart) {
      TRY(ensure_z(c, B_XPART, sizeof(XPart)));
      xp = P<XPart>(c, B_XPART);
      // the table the previous scan's link2 wrote, if it was made for this span count and grid
      if (c->xp_valid && c->xp_ns == ns_rel && c->xp_g == g) part.bs = &xp->bs[c->xp_par][0];
    }
    const uint64_t total_waves = (uint64_t)g * nw;
    const uint64_t spw = part_max_wave_spans(part, xpart);
    const uint64_t wcap = spw * c->copt.cap;
    // the glue works in slot space (slot = wave * wcap + record): its parent
    // words are 31-bit; stores above ~1 TiB (or a denser cap) take the full pass
    const uint64_t capK = total_waves * wcap;
    if (capK >= c->slot_limit) { out->full_reason = SRD_FULL_SLOT_SPACE; return 0; }
    const uint32_t wpb = (uint32_t)((total_waves + CHAIN_BLOCKS - 1) / CHAIN_BLOCKS);  // scan waves per chain block
    if (wpb > BW_MAX) { out->full_reason = SRD_FULL_WAVES; return 0; }
    TRY(alloc_scan(c, nt_rel, std::max<uint64_t>(ns_rel, total_waves * spw), c->copt.cap));
    TRY(ensure(c, B_SPAN_FIRST, (ns_rel + 1) * 4));
    TRY(alloc_fast(c, capK, log2_nbk));
    if (c->gen >= 0xFFFFFFF0u || c->gen == 0) {  // tag wrap: clear the marks once
      c->gen = 0;
      HIPCHK(hipMemsetAsync(P<void>(c, B_HASCHILD), 0, c->bufs[B_HASCHILD].n, c->stream));
      HIPCHK(hipMemsetAsync(P<void>(c, B_HASCHILD2), 0, c->bufs[B_HASCHILD2].n, c->stream));
      HIPCHK(hipMemsetAsync(P<void>(c, B_CHILDOF), 0, c->bufs[B_CHILDOF].n, c->stream));
    }
    ++c->gen;
    Plan* pl = P<Plan>(c, B_PLAN);
    uint64_t* cnt = P<uint64_t>(c, B_COUNTERS);
    // the scan writes every span's count and (its last block) the counters,
    // the wave bases and K; block 0 zeroes the plan
    // per-tile / per-span arrays hold the resident range only: their base
    // pointers are shifted so kernels index them by absolute tile / span
    ScanArgs a{};
    a.variant = var;
    a.part = part;
    a.xp = xp;
    a.xp_next = c->xp_par ^ 1u;
    a.file = d_file;
    a.flen = flen;
    a.n_tiles = n_tiles;
    a.n_spans = n_spans;
    a.cap = c->copt.cap;
    a.tile = P<uint32_t>(c, B_TILE) - 4 * k_lo;
    a.span_count = P<uint32_t>(c, B_SPAN_COUNT) - s_lo;
    a.c_m = P<uint64_t>(c, B_CM);  // wave regions, indexed by the wave of this launch
    a.c_rec = P<u32x4>(c, B_CREC);
    a.c_rec1 = crec1(c);
    a.span_first = P<uint32_t>(c, B_SPAN_FIRST) - s_lo;
    a.wcap = wcap;
    a.counters = (unsigned long long*)cnt;
    a.filt_hb = (uint32_t)((flen ? flen - 1 : 0) >> 32);
    a.k_lo = k_lo;
    a.m_lo = lo;
    a.zero_words = (uint32_t*)pl;
    a.n_zero_words = (uint32_t)(sizeof(Plan) / 4);
    a.sentinel = nullptr;
    // the link phase (every node claims its parent) and the index bucket fills
    // chain_finalize claims (zeroed by block 0)
    a.d_par = P<int32_t>(c, B_DPAR);
    a.childof = P<unsigned long long>(c, B_CHILDOF);
    a.gen = c->gen;
    a.span_lo = lo;
    a.zero2 = index_zero_words(c, log2_nbk, &a.n_zero2);
    TRY(scan_wave_args(c, &a));
    hipEvent_t e0, e1;
    TRY(next_scan_events(c, &e0, &e1));
    launch_scan<false>(g, a, c->stream, e0, e1);
    KCHK(c, "scan_kernel");
    HIPCHK(hipGetLastError());
#ifdef SRD_DEBUG_API
    if (flags & kDbgScanOnly) {  // timing-only ablations: the scan alone, no result
      HIPCHK(hipStreamSynchronize(c->stream));
      *done = true;
      return 0;
    }
#endif
    // every record's node test, parent and claim (slot space), one block per scan wave
    link2_kernel<<<(unsigned)((total_waves + LINK_WPB - 1) / LINK_WPB), 256 * LINK_WPB, 0, c->stream>>>(
        a, (uint32_t)total_waves);
    KCHK(c, "link2_kernel");
    if (xp) {  // link2 wrote the next call's block starts into the other half
      c->xp_par ^= 1u;
      c->xp_valid = true;
      c->xp_ns = ns_rel;
      c->xp_g = g;
    }
    // ---- shape check, chain, finalize, index; retried on device with more
    //      prune rounds when false candidates chained onto each other ----
    Plan hp{};
    uint32_t* marks = P<uint32_t>(c, B_HASCHILD);
    uint32_t* marks2 = P<uint32_t>(c, B_HASCHILD2);
    uint32_t mgen = c->gen;
    for (int rounds = 0;; rounds += 2) {
      if (rounds) HIPCHK(hipMemsetAsync(pl, 0, sizeof(Plan), c->stream));  // round 0: zeroed by the scan
      ShapeArgs sa{};
      sa.file = d_file;
      sa.flen = flen;
      sa.Kp = a.k_total;
      sa.wave_total = a.wave_total;
      sa.wcap = wcap;
      sa.n_waves = (uint32_t)total_waves;
      sa.wpb = wpb;
      sa.n_slots = capK;
      sa.coff = coff;
      sa.c_m = a.c_m;
      sa.d_par = a.d_par;
      sa.c_rec = a.c_rec;
      sa.childof = P<uint64_t>(c, B_CHILDOF);
      sa.flag = P<uint8_t>(c, B_FLAG);
      sa.part = P<uint32_t>(c, B_PART);
      sa.wpart = P<uint32_t>(c, B_PARTEX);
      sa.counters = (const unsigned long long*)cnt;
      sa.plan = pl;
      sa.zero = index_zero_words(c, log2_nbk, &sa.n_zero);  // child2 zeroes the index's bucket fills
      sa.lb_fail = c->lb_fail;
      if (rounds == 0) {
        // round 0: the link phase's claims (every node claims its parent) are the
        // core flags and the branch test; no marks
        sa.has_child = nullptr;
        sa.gen = mgen;
      } else {
        if (rounds == 2) {  // the retry's first marks: the nodes the link claims were made on
          sa.gen = mgen;
          marks_from_claims_kernel<<<GLUE_BLOCKS, GLUE_THREADS, 0, c->stream>>>(sa, marks);
          KCHK(c, "marks_from_claims_kernel");
        }
        for (int r = 0; r < 2; r++) {  // two more prune rounds per retry
          sa.has_child = marks;
          sa.gen = mgen;
          const uint32_t g2 = ++c->gen;
          prune_kernel<<<GLUE_BLOCKS, GLUE_THREADS, 0, c->stream>>>(sa, marks2, g2);
          KCHK(c, "prune_kernel");
          std::swap(marks, marks2);
          mgen = g2;
        }
        sa.has_child = marks;
        sa.gen = mgen;
        child2_kernel<<<GLUE_BLOCKS, GLUE_THREADS, 0, c->stream>>>(sa);  // core-only claims
        KCHK(c, "child2_kernel");
      }
      const bool fused = rounds == 0 && c->glue_fused;
      if (!fused) {
        check_kernel<<<CHAIN_BLOCKS, CHAIN_THREADS, 0, c->stream>>>(sa);
        KCHK(c, "check_kernel");
        HIPCHK(hipGetLastError());
      }
      // ---- plan + chain ranks + per-entry outputs / CRC + index histogram ----
      FinArgs f{};
      f.file = d_file;
      f.flen = flen;
      f.c_m = a.c_m;
      f.c_rec = a.c_rec;
      f.c_rec1 = a.c_rec1;
      f.tile = a.tile;
      f.no_crc = (flags & SRD_FLAG_NO_CRC) ? 1 : 0;
      f.coff = coff;
      f.o_mo = P<uint64_t>(c, B_O_MO);
      f.o_kh = P<uint64_t>(c, B_O_KH);
      f.o_prev = P<uint64_t>(c, B_O_PREV);
      f.o_start = P<uint64_t>(c, B_O_START);
      f.o_len = P<uint64_t>(c, B_O_LEN);
      f.o_crc_st = P<uint32_t>(c, B_O_CRCST);
      f.o_crc = P<uint32_t>(c, B_O_CRC);
      f.o_pieces = P<uint32_t>(c, B_O_PIECES);
      f.o_suf = P<uint32_t>(c, B_O_SUF);
      f.o_sxm = P<uint32_t>(c, B_O_SXM);
      f.o_tail = P<uint32_t>(c, B_O_TAIL);
      f.o_ok = P<uint8_t>(c, B_O_OK);
      f.n_bad = (unsigned long long*)&pl->n_bad;
      f.slow_list = P<uint64_t>(c, B_SLOW);       // entries that need a wave (idx_dedup runs them)
      f.n_slow = (unsigned long long*)&pl->n_slow;  // zeroed with the plan
      f.o_packed = P<uint64_t>(c, B_O_PACKED);
      unsigned long long* lb = P<unsigned long long>(c, B_LOOKB);
      if (fused)
        chain_finalize_kernel<true><<<CHAIN_BLOCKS, CHAIN_THREADS, (1u << log2_nbk) * 4, c->stream>>>(
            sa, f, index_args(c, log2_nbk), log2_nbk, lb);
      else
        chain_finalize_kernel<false><<<CHAIN_BLOCKS, CHAIN_THREADS, (1u << log2_nbk) * 4, c->stream>>>(
            sa, f, index_args(c, log2_nbk), log2_nbk, lb);
      KCHK(c, "chain_finalize_kernel");
      HIPCHK(hipGetLastError());
      // ---- KeyIndexer::build (bucketed; the global table in SRD_INDEX_GLOBAL timing builds) ----
      if (!index_global_env()) {
        TRY(launch_index_bucketed(c, f.o_kh, f.o_mo, &pl->n_chain, &pl->status, log2_nbk, P<uint64_t>(c, B_IKEY),
                                  P<uint64_t>(c, B_IPACKED), pl, true, &f, false, xp ? &xp->scan_ticks : nullptr));
      } else {  // timing builds without the bucketed index: the slow list by its own kernel
        slow_kernel<<<2048 / SLOW_WAVES, SLOW_WAVES * 64, 0, c->stream>>>(f);
        KCHK(c, "slow_kernel");
      }
      if (c->timing >= SRD_TIMING_CALL) {
        HIPCHK(hipEventRecord(c->ev[3], c->stream));  // end of the device work (srd_ctx_timings)
        c->ev3_recorded = true;
      }
      // the outcome idx_emit publishes to pinned memory when it starts; a
      // proven chain whose index aliases the chain arrays needs nothing else
      // (no plan copy is enqueued: the next call's scan would queue behind
      // it); anything else copies the whole plan and waits for the stream
      bool fast = false;
      if (!index_global_env() && !(c->timing >= SRD_TIMING_CALL)) {
        uint64_t w[PUB_WORDS];
        TRY(wait_publish(c, w));
        const uint32_t fl = (uint32_t)w[0];
        if ((fl & 0x3ffu) == 0x100u) {  // status 0, aliased index, no bucket overflow
          fast = true;
          scan_tune_feedback(c, var, (uint32_t)w[6]);
          hp = Plan{};
          hp.n_chain = (uint32_t)w[1];
          hp.n_index = (uint32_t)w[2];
          hp.n_bad = (uint32_t)w[3];
          hp.K = (uint32_t)w[4];
          hp.top_gap = (uint32_t)w[5];
          hp.idx_alias = 1;
        }
      }
      if (!fast) {
        HIPCHK(hipMemcpyAsync(c->h_plan, pl, sizeof(Plan), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(spin_sync(c->stream));
        hp = *c->h_plan;
      }
      if (debug_env()) {
        fprintf(stderr, "plan K=%lu n_chain=%lu root_t=%lu start=%lu n_index=%lu bad=%lu slow=%lu st=%u nroot=%u "
                "troot=%u idxov=%u log2nbk=%u capK=%lu rounds=%d\n",
                (unsigned long)hp.K, (unsigned long)hp.n_chain, (unsigned long)hp.root_t, (unsigned long)hp.start,
                (unsigned long)hp.n_index, (unsigned long)hp.n_bad, (unsigned long)hp.n_slow, hp.status, hp.nroot,
                hp.troot, hp.idx_overflow, log2_nbk, (unsigned long)capK, rounds);
      }
      // only a shape / root-count failure can be a false chain; at most 6 extra rounds
      const uint32_t retry_bits = ST_SHAPE | ST_ROOTS;
      if (!(hp.status & retry_bits) || (hp.status & ~retry_bits) || rounds >= 6) break;
    }
    out->n_candidates = hp.K;
    if (hp.status & ST_OVERFLOW) {
      // (cannot happen: <= one candidate per byte) not provable here
      if (c->copt.cap >= SPAN_BYTES) { out->full_reason = SRD_FULL_CAP; return 0; }
      grow_cap(c->copt, flen - span_off);
      out->full_reason = SRD_FULL_CAP;  // (if the attempts run out)
      continue;
    }
    if (hp.status) {  // not provable here -> full pass (whole file) / unproven (span)
      out->full_reason = (hp.status & ST_LOOKBACK) ? SRD_FULL_LOOKBACK
                         : (hp.status & ST_NOSTART) ? SRD_FULL_NO_START
                                                    : SRD_FULL_UNPROVEN;
      return 0;
    }
    out->full_reason = SRD_FULL_NONE;
    out->final_len = flen - hp.top_gap;  // find_top's start tail (a torn tail within TOP_WINDOW bytes: below flen)
    out->n_chain = hp.n_chain;
    out->n_crc_bad = hp.n_bad;
    out->n_index = hp.n_index;
    c->last_n = hp.n_chain;
    if (hp.idx_overflow || index_global_env()) {
      c->ev3_recorded = false;
      TRY(index_global(c, hp.n_chain, &out->n_index));
      hp.idx_alias = 0;
    }
    set_out_ptrs(c, out);
    if (hp.idx_alias) {  // every entry its key's latest: the index is the chain's own arrays
      out->index_key_hash = P<uint64_t>(c, B_O_KH);
      out->index_packed = P<uint64_t>(c, B_O_PACKED);
    }
    *done = true;
    return 0;
  }
  return 0;
}

static int validate_device_impl(srd_ctx* c, const uint8_t* d_file, uint64_t flen, uint32_t flags,
                                srd_device_result* out);

extern "C" int srd_validate_index_device(srd_ctx* c, const uint8_t* d_file, uint64_t flen, uint32_t flags,
                                         srd_device_result* out) {
  if (!c) { set_err("bad argument"); return SRD_ERR_ARG; }
  HIPCHK(hipSetDevice(c->device));
  c->total_ms = 0;
  c->ev3_recorded = false;
  const bool tcall = c->timing >= SRD_TIMING_CALL;
  if (tcall) HIPCHK(hipEventRecord(c->ev[2], c->stream));
  int r = validate_device_impl(c, d_file, flen, flags, out);
  if (!(r == 0 && out->mode == SRD_MODE_OPTIMISTIC && (c->ev3_recorded || !tcall))) {
    if (tcall) {
      HIPCHK(hipEventRecord(c->ev[3], c->stream));
      HIPCHK(hipEventSynchronize(c->ev[3]));
    } else {
      HIPCHK(spin_sync(c->stream));
    }
  }
  if (tcall) {
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, c->ev[2], c->ev[3]));
    c->total_ms = ms;
  }
  return r;
}

extern "C" int srd_validate_span_device(srd_ctx* c, const uint8_t* d_span, uint64_t span_off, uint64_t lo,
                                        uint64_t hi, uint32_t flags, srd_device_result* out) {
  if (!c || !out || !d_span) { set_err("bad argument"); return SRD_ERR_ARG; }
  if (lo == 0) {
    if (span_off) { set_err("bad argument: a span starting at tail 0 is the whole file (span_off must be 0)"); return SRD_ERR_ARG; }
    return srd_validate_index_device(c, d_span, hi, flags, out);
  }
  if (span_off % SPAN_BYTES || span_off > lo || hi < lo + 21 || hi > kMaxFile) {
    set_err("bad span: need span_off % 16384 == 0, span_off <= lo, lo + 21 <= hi <= 2^48");
    return SRD_ERR_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  memset(out, 0, sizeof *out);
  out->file_len = hi;
  c->total_ms = 0;
  const bool tcall = c->timing >= SRD_TIMING_CALL;
  if (tcall) HIPCHK(hipEventRecord(c->ev[2], c->stream));
  bool done = false;
  int r = optimistic_pass(c, d_span, span_off, lo, hi, flags, out, &done);
  if (!r && !done) {
    out->mode = SRD_MODE_SPAN_UNPROVEN;
    out->final_len = 0;
    out->n_chain = 0;
    out->n_index = 0;
    out->n_crc_bad = 0;
  }
  if (tcall) {
    HIPCHK(hipEventRecord(c->ev[3], c->stream));
    HIPCHK(hipEventSynchronize(c->ev[3]));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, c->ev[2], c->ev[3]));
    c->total_ms = ms;
  } else {
    HIPCHK(spin_sync(c->stream));
  }
  return r;
}

// stable partition of n (key, value) device pairs by owner rank; interleaved
// output at out (out_v == nullptr) or keys at out / values at out_v.  counts
// (host, [world]) receives the group sizes.  Synchronises.
// counts (host, nullable): the per-owner pair counts, read back with one
// host round trip; d_counts (nullable): their device address instead, no
// sync (the multi-GPU exchange's owners read them over xGMI)
static int partition_impl(Ctx* c, const uint64_t* keys, const uint64_t* vals, uint64_t n, uint32_t world,
                          uint64_t* out, uint64_t* out_v, uint64_t* counts, const uint64_t** d_counts = nullptr) {
  const uint64_t nc = (uint64_t)world * GLUE_BLOCKS + 1;
  TRY(ensure(c, B_PCNT, nc * 4));
  TRY(ensure(c, B_POFF, nc * 4 + 8 * PART_MAX_WORLD));
  TRY(ensure_cub(c, nc));
  PartArgs a{};
  a.keys = keys;
  a.vals = vals;
  a.n = n;
  a.world = world;
  a.cnt = P<uint32_t>(c, B_PCNT);
  a.off = P<uint32_t>(c, B_POFF);
  a.out = out;
  a.out_v = out_v;
  a.counts = (uint64_t*)(P<uint32_t>(c, B_POFF) + ((nc + 1) & ~1ull));
  part_count_kernel<<<GLUE_BLOCKS, 256, 0, c->stream>>>(a);
  KCHK(c, "part_count_kernel");
  size_t tb = c->bufs[B_CUB_TMP].n;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(P<void>(c, B_CUB_TMP), tb, a.cnt, a.off, (int)nc, c->stream));
  KCHK(c, "hipcub");
  part_scatter_kernel<<<GLUE_BLOCKS, 256, 0, c->stream>>>(a);
  KCHK(c, "part_scatter_kernel");
  part_counts_kernel<<<1, 64, 0, c->stream>>>(a);
  KCHK(c, "part_counts_kernel");
  HIPCHK(hipGetLastError());
  if (d_counts) *d_counts = a.counts;
  if (counts) {
    HIPCHK(hipMemcpyAsync(counts, a.counts, world * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(spin_sync(c->stream));
  }
  return 0;
}

extern "C" int srd_index_partition_device(srd_ctx* c, const uint64_t* d_keys, const uint64_t* d_vals, uint64_t n,
                                          uint32_t world, uint64_t* d_out_pairs, uint64_t* counts) {
  if (!c || !counts || world == 0 || world > PART_MAX_WORLD || (n && (!d_keys || !d_vals || !d_out_pairs))) {
    set_err("bad argument");
    return SRD_ERR_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  return partition_impl(c, d_keys, d_vals, n, world, d_out_pairs, nullptr, counts);
}

__global__ void index_prep_kernel(Plan* pl, uint64_t n, uint32_t* zero, uint32_t nz) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nz) zero[i] = 0;
  if (i < sizeof(Plan) / 4) ((uint32_t*)pl)[i] = 0;
  __syncthreads();
  if (i == 0) pl->n_chain = n;
}

// KeyIndexer::build over n (key_hash, meta_off or packed) device pairs given
// as two arrays, in file order (latest position wins); output in chain order
// of each key's latest entry.  Synchronises.
static int index_build_sep(Ctx* c, const uint64_t* keys, const uint64_t* vals, uint64_t n, uint64_t* okeys,
                           uint64_t* opacked, uint64_t* n_index) {
  *n_index = 0;
  if (!n) return 0;
  TRY(ensure(c, B_MPLAN, sizeof(Plan)));
  const uint32_t log2_nbk = index_log2_buckets(n);
  TRY(alloc_index(c, n, log2_nbk));
  Plan* pl = P<Plan>(c, B_MPLAN);
  // one launch zeroes the plan (n_chain = n) and the bucket fills (was a
  // memset, a one-thread kernel and a second memset)
  uint32_t nz = 0;
  uint32_t* zw = index_zero_words(c, log2_nbk, &nz);
  index_prep_kernel<<<(nz + 255) / 256, 256, 0, c->stream>>>(pl, n, zw, nz);
  KCHK(c, "index_prep_kernel");
  TRY(launch_index_bucketed(c, keys, vals, &pl->n_chain, &pl->status, log2_nbk, okeys, opacked, pl, false, nullptr,
                            true));
  HIPCHK(hipMemcpyAsync(c->h_plan, pl, sizeof(Plan), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(spin_sync(c->stream));
  if (c->h_plan->idx_overflow) return index_global(c, n, n_index, keys, vals, okeys, opacked);
  *n_index = c->h_plan->n_index;
  return 0;
}

__global__ void index_prep_dev_kernel(Plan* pl, const uint64_t* d_n, uint32_t* zero, uint32_t nz) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nz) zero[i] = 0;
  if (i < sizeof(Plan) / 4) ((uint32_t*)pl)[i] = 0;
  __syncthreads();
  if (i == 0) pl->n_chain = *d_n;
}
// index_build_sep with the pair count on the device (*d_n <= n_max): the
// multi-GPU owners' build right behind their gather, no host round trip for
// the count; buckets sized for n_est expected pairs.  Synchronises once.
static int index_build_dev(Ctx* c, const uint64_t* keys, const uint64_t* vals, uint64_t n_max, const uint64_t* d_n,
                           uint64_t n_est, uint64_t* okeys, uint64_t* opacked, uint64_t* n_index) {
  *n_index = 0;
  if (!n_max) return 0;
  TRY(ensure(c, B_MPLAN, sizeof(Plan)));
  const uint32_t log2_nbk = index_log2_buckets(std::max<uint64_t>(n_est, 1));
  TRY(alloc_index(c, n_max, log2_nbk));
  Plan* pl = P<Plan>(c, B_MPLAN);
  uint32_t nz = 0;
  uint32_t* zw = index_zero_words(c, log2_nbk, &nz);
  index_prep_dev_kernel<<<(std::max<uint32_t>(nz, 64) + 255) / 256, 256, 0, c->stream>>>(pl, d_n, zw, nz);
  KCHK(c, "index_prep_dev_kernel");
  TRY(launch_index_bucketed(c, keys, vals, &pl->n_chain, &pl->status, log2_nbk, okeys, opacked, pl, false, nullptr,
                            true));
  HIPCHK(hipMemcpyAsync(c->h_plan, pl, sizeof(Plan), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(spin_sync(c->stream));
  if (c->h_plan->idx_overflow) return index_global(c, c->h_plan->n_chain, n_index, keys, vals, okeys, opacked);
  *n_index = c->h_plan->n_index;
  return 0;
}

extern "C" int srd_index_build_device(srd_ctx* c, const uint64_t* d_pairs, uint64_t n, uint64_t* d_out_keys,
                                      uint64_t* d_out_packed, uint64_t* n_index) {
  if (!c || !n_index || (n && (!d_pairs || !d_out_keys || !d_out_packed))) { set_err("bad argument"); return SRD_ERR_ARG; }
  if (n >= (1ull << 31)) { set_err("too many pairs"); return SRD_ERR_ARG; }
  HIPCHK(hipSetDevice(c->device));
  *n_index = 0;
  if (!n) return 0;
  TRY(ensure(c, B_MKEY, n * 8));
  TRY(ensure(c, B_MVAL, n * 8));
  deinterleave_kernel<<<blocks(std::min<uint64_t>(n, 1 << 20), 256), 256, 0, c->stream>>>(
      d_pairs, n, P<uint64_t>(c, B_MKEY), P<uint64_t>(c, B_MVAL));
  KCHK(c, "deinterleave_kernel");
  HIPCHK(hipGetLastError());
  return index_build_sep(c, P<uint64_t>(c, B_MKEY), P<uint64_t>(c, B_MVAL), n, d_out_keys, d_out_packed, n_index);
}

extern "C" int srd_ctx_set_timing(srd_ctx* c, int level) {
  if (!c || level < SRD_TIMING_NONE || level > SRD_TIMING_CALL) { set_err("bad argument"); return SRD_ERR_ARG; }
  if (level >= SRD_TIMING_SCAN && !c->sev[0]) {
    HIPCHK(hipSetDevice(c->device));
    for (auto& e : c->sev) HIPCHK(hipEventCreateWithFlags(&e, hipEventReleaseToDevice));
  }
  c->timing = level;
  return 0;
}

extern "C" int srd_ctx_set_timing_every(srd_ctx* c, int n) {
  if (!c || n < 1) { set_err("bad argument"); return SRD_ERR_ARG; }
  c->timing_every = (uint32_t)n;
  c->timing_seq = 0;
  return 0;
}

extern "C" int srd_ctx_timings(srd_ctx* c, double* scan_ms, int* scan_launches, double* total_ms) {
  if (!c) { set_err("bad argument"); return SRD_ERR_ARG; }
  HIPCHK(hipSetDevice(c->device));
  TRY(drain_scan_events(c, c->sev_pending));
  if (scan_ms) *scan_ms = c->scan_ms;
  if (scan_launches) *scan_launches = c->scan_launches;
  if (total_ms) *total_ms = c->total_ms;
  c->scan_ms = 0;
  c->scan_launches = 0;
  c->scan_last.swap(c->scan_list);
  c->scan_list.clear();
  return 0;
}

extern "C" int srd_ctx_scan_list(srd_ctx* c, float* out, int cap) {
  if (!c || (cap > 0 && !out)) { set_err("bad argument"); return SRD_ERR_ARG; }
  const int n = (int)std::min<size_t>(c->scan_last.size(), (size_t)std::max(cap, 0));
  for (int i = 0; i < n; i++) out[i] = c->scan_last[i];
  return (int)c->scan_last.size();
}

static int validate_device_impl(srd_ctx* c, const uint8_t* d_file, uint64_t flen, uint32_t flags,
                                srd_device_result* out) {
  if (!c || !out || (!d_file && flen)) { set_err("bad argument"); return SRD_ERR_ARG; }
  if (flen > kMaxFile) { set_err("stores above 2^48 bytes cannot be indexed (48-bit packed offsets)"); return SRD_ERR_ARG; }
  HIPCHK(hipSetDevice(c->device));
  memset(out, 0, sizeof *out);
  out->file_len = flen;
  if (flen < 21) {  // no tail can be valid (recover_valid_chain :384-386, t>=21)
    TRY(alloc_dense(c, 1));
    TRY(alloc_scan(c, 1, 1, c->copt.cap));
    return finish(c, d_file, flen, 0, flags, out);
  }
  bool full = flags & SRD_FLAG_FORCE_FULL;
  if (full) out->full_reason = SRD_FULL_FORCED;
  uint64_t K = 0, h[8];
  // ---- optimistic pass: strong candidates only; valid iff the chain from
  //      file_len is proven through recorded nodes ----
  if (!full) {
    bool done = false;
    TRY(optimistic_pass(c, d_file, 0, 0, flen, flags, out, &done));
    if (done) return 0;
  }
  // ---- full pass ----
  out->mode = 1;
  TRY(run_scan(c, d_file, flen, true, &K, h));
  out->n_candidates = K;
  if (debug_env()) fprintf(stderr, "full pass: K=%lu candidates (reason %lu)\n", (unsigned long)K,
                           (unsigned long)out->full_reason);
  const uint64_t max_root = h[0];
  uint64_t best_g1 = 0, tlin = 0;
  if (K) {
    TRY(ensure(c, B_ST, K));
    TRY(ensure(c, B_JMP, K * 8));
    TRY(ensure(c, B_VFLAG, K * 4));
    // core runs (alloc_dense sized B_CORE, B_DHEAD / B_RUNHEAD and the hipCUB
    // scratch for K): core[g] = something links to g; prevcore = 1 + the last
    // core node <= g; chead = 1 + the head of a core node's run
    const unsigned kb = blocks(K, 256);
    const int64_t* par = P<int64_t>(c, B_DPAR);
    uint8_t* core = P<uint8_t>(c, B_CORE);
    uint32_t* key = P<uint32_t>(c, B_DHEAD);
    uint32_t* chead = P<uint32_t>(c, B_RUNHEAD);
    uint8_t* st = P<uint8_t>(c, B_ST);
    int64_t* jmp = P<int64_t>(c, B_JMP);
    HIPCHK(hipMemsetAsync(core, 0, K, c->stream));
    child_kernel<<<kb, 256, 0, c->stream>>>(par, K, core);
    KCHK(c, "child_kernel");
    core_flag_key_kernel<<<kb, 256, 0, c->stream>>>(core, K, key);
    KCHK(c, "core_flag_key_kernel");
    size_t tbs = c->bufs[B_CUB_TMP].n;
    HIPCHK(hipcub::DeviceScan::InclusiveScan(P<void>(c, B_CUB_TMP), tbs, key, chead, hipcub::Max(), (int)K, c->stream));
    KCHK(c, "hipcub");
    head_key_kernel<<<kb, 256, 0, c->stream>>>(core, par, chead, K, key);
    KCHK(c, "head_key_kernel");
    tbs = c->bufs[B_CUB_TMP].n;
    HIPCHK(hipcub::DeviceScan::InclusiveScan(P<void>(c, B_CUB_TMP), tbs, key, chead, hipcub::Max(), (int)K, c->stream));
    KCHK(c, "hipcub");
    status_init_kernel<<<kb, 256, 0, c->stream>>>(par, core, chead, K, st, jmp);
    KCHK(c, "status_init_kernel");
    uint64_t* cnt = P<uint64_t>(c, B_COUNTERS);
    // pointer jumping over the core run heads: every round doubles how far
    // each unresolved head looks along its chain of runs, so ceil(log2 K) + 1
    // rounds resolve every head.  Rounds run back to back (a round after
    // convergence exits at once) and one more round, with the change flag
    // cleared before it, proves convergence with one host wait: first 12
    // rounds (C2's chain of runs converges in ~10), then 8, 16, ... more
    int rounds = 1;
    while ((1ull << rounds) < K) rounds++;
    TRY(ensure(c, B_RFLAG, 4 * 72));
    unsigned int* rflag = P<unsigned int>(c, B_RFLAG);
    int done_rounds = 0;
    for (int pass = 0; pass < 8; pass++) {
      const int nr = std::max(1, std::min(pass ? 4 << pass : 12, rounds + 1 - done_rounds));
      done_rounds += nr;
      HIPCHK(hipMemsetAsync(rflag, 0, 4 * 72, c->stream));
      for (int r = 0; r < std::min(nr, 70); r++) {
        // a fixed grid (grid-stride): a round after convergence exits at once
        status_round_kernel<<<std::min(kb, 1024u), 256, 0, c->stream>>>(K, core, chead, st, jmp, rflag + r,
                                                                       r ? rflag + r - 1 : nullptr);
        KCHK(c, "status_round_kernel");
      }
      HIPCHK(hipMemsetAsync(cnt + 4, 0, 8, c->stream));
      status_round_kernel<<<std::min(kb, 1024u), 256, 0, c->stream>>>(K, core, chead, st, jmp, (unsigned int*)(cnt + 4),
                                                                     nullptr);
      KCHK(c, "status_round_kernel");
      HIPCHK(hipGetLastError());
      TRY(read_counters(c, h));
      if (!h[4]) break;
      if (pass == 7) { set_err("internal: pointer jumping did not converge"); return SRD_ERR_INTERNAL; }
    }
    status_spread_core_kernel<<<kb, 256, 0, c->stream>>>(K, core, chead, st);
    KCHK(c, "status_spread_core_kernel");
    status_spread_leaf_kernel<<<kb, 256, 0, c->stream>>>(K, par, core, st);
    KCHK(c, "status_spread_leaf_kernel");
    const unsigned vb = blocks(K, 256);
    TRY(ensure(c, B_JMP, std::max<uint64_t>(K, vb) * 8));  // per-block maxima (the jump pointers are dead now)
    valid_max_kernel<<<vb, 256, 0, c->stream>>>(P<uint8_t>(c, B_ST), K, P<uint64_t>(c, B_JMP), P<uint32_t>(c, B_VFLAG));
    KCHK(c, "valid_max_kernel");
    max_reduce_kernel<<<1, 1024, 0, c->stream>>>(P<uint64_t>(c, B_JMP), vb, (unsigned long long*)(cnt + 3),
                                                 P<uint64_t>(c, B_DM), (unsigned long long*)(cnt + 7));
    KCHK(c, "max_reduce_kernel");
    HIPCHK(hipGetLastError());
    TRY(read_counters(c, h));
    best_g1 = h[3];
    if (best_g1) tlin = h[7] + 20;  // d_m[best_g1 - 1] + 20
  }
  const uint64_t final_len = std::max(tlin, max_root);
  out->final_len = final_len;
  if (final_len == 0) return finish(c, d_file, flen, 0, flags, out);
  if (final_len == max_root && max_root > tlin) {
    TRY(set_single_root(c, final_len));
    return finish(c, d_file, flen, 1, flags, out);
  }
  // compact the valid nodes, walk from the best one
  TRY(ensure(c, B_VLIST, K * 8));
  TRY(ensure(c, B_NV, 8));
  TRY(ensure(c, B_VPOS, K * 8));
  TRY(ensure(c, B_VPAR, K * 8));
  TRY(ensure(c, B_VSLOT, K * 8));
  // valid nodes in dense order: an exclusive scan of the flags, then one
  // scatter writes vlist[pos] = g, vpos[g] = pos and nv (no host wait before
  // the remap: its grid covers K and stops at nv on the device)
  TRY(ensure(c, B_VSCAN, K * 4));
  size_t tb = c->bufs[B_CUB_TMP].n;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(P<void>(c, B_CUB_TMP), tb, P<uint32_t>(c, B_VFLAG), P<uint32_t>(c, B_VSCAN),
                                          (int)K, c->stream));
  KCHK(c, "hipcub");
  compact_valid_kernel<<<blocks(K, 256), 256, 0, c->stream>>>(P<uint32_t>(c, B_VFLAG), P<uint32_t>(c, B_VSCAN), K,
                                                              P<uint64_t>(c, B_VLIST), P<uint64_t>(c, B_VPOS),
                                                              P<uint64_t>(c, B_NV));
  KCHK(c, "compact_valid_kernel");
  remap_kernel<<<blocks(K, 256), 256, 0, c->stream>>>(P<uint64_t>(c, B_VLIST), P<uint64_t>(c, B_NV),
                                                      P<int64_t>(c, B_DPAR), P<uint64_t>(c, B_VPOS),
                                                      P<int64_t>(c, B_VPAR), P<uint64_t>(c, B_VSLOT),
                                                      P<uint64_t>(c, B_DSLOT));
  KCHK(c, "remap_kernel");
  // the walk starts at the best node's compacted position
  walk_start_kernel<<<1, 64, 0, c->stream>>>(P<WalkState>(c, B_WALK), P<uint64_t>(c, B_VPOS), best_g1 - 1);
  KCHK(c, "walk_start_kernel");
  HIPCHK(hipGetLastError());
  TRY(enqueue_small(c, P<uint64_t>(c, B_NV), 0));
  HIPCHK(spin_sync(c->stream));
  const uint64_t nv = c->h_small[8];
  WalkState hw{};
  TRY(walk_and_mark(c, P<int64_t>(c, B_VPAR), P<uint64_t>(c, B_VSLOT), nv, P<uint64_t>(c, B_VLIST), &hw));
  if (hw.status != 1) { set_err("internal: valid walk did not reach a root"); return SRD_ERR_INTERNAL; }
  return finish(c, d_file, flen, hw.chain_len, flags, out);
}

extern "C" uint64_t srd_padded_size(uint64_t flen) { return ((flen + TILE - 1) / TILE) * TILE + 2 * TILE; }

// ---------------------------------------------------------- shard boundaries
// Host pre-pass for the entry-range shards of an arbitrary store (SURVEY.md
// 8(e)); the parser lives in srd_host.cpp (no HIP, sanitizer-tested).
extern "C" int srd_shard_cuts(const uint8_t* file, uint64_t flen, uint32_t world, uint64_t* cuts) {
  const char* why = "";
  const int r = srd_host::shard_cuts(file, flen, world, cuts, &why);
  if (r) set_err(why);
  return r;
}

// ---------------------------------------------------------------- host input
// The path starts in host memory: the mmap'd single-file store
// (data_store.rs:172-174 init_mmap, called from open :84-117).  Staging modes:
//  - already pinned host memory: one DMA copy;
//  - default: host threads copy 16 MiB chunks into double-buffered pinned
//    bounce buffers, each worker DMA-ing its previous chunk on its own stream
//    meanwhile (the memcpy also takes the mapping's page faults on several
//    cores): the pinned-buffer rate from a page-cache-warm mmap (C2: 87 ms,
//    vs 114 ms registered and 133 ms pageable);
//  - SRD_FLAG_STAGE_REGISTER: hipHostRegister (read-only) of the mapped
//    range, one DMA copy, unregister (bounce buffers if refused);
//  - SRD_FLAG_STAGE_PAGEABLE: one pageable hipMemcpy (the runtime's own
//    staging; measurement baseline).
constexpr uint32_t kStageFlags = SRD_FLAG_STAGE_PAGEABLE | SRD_FLAG_STAGE_REGISTER;
constexpr uint64_t kBounceBytes = 16ull << 20;

static int ensure_file_buf(Ctx* c, uint64_t flen, uint8_t** d) {
  const uint64_t need = srd_padded_size(flen);
  if (c->file.n < need) {
    if (c->file.p) HIPCHK(hipFree(c->file.p));
    c->file.p = nullptr;
    c->file.n = 0;
    if (hipMalloc(&c->file.p, need) != hipSuccess) { set_err("hipMalloc(file)"); return SRD_ERR_ALLOC; }
    c->file.n = need;
  }
  *d = (uint8_t*)c->file.p;
  return 0;
}

static int stage_bounce(Ctx* c, const uint8_t* src, uint64_t len, uint8_t* dst, int workers) {
  const uint64_t nch = (len + kBounceBytes - 1) / kBounceBytes;
  // T workers, each with two pinned bounce buffers and a stream: allocated
  // when a call first needs them (the multi-GPU open gives each shard fewer)
  const int T = (int)std::min<uint64_t>((uint64_t)std::max(1, std::min(workers, c->stage_workers)), nch);
  for (int w = (int)c->stage_streams.size(); w < T; w++) {
    void* pin[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    hipStream_t st = nullptr;
    for (int k = 0; k < 2; k++) {
      HIPCHK(hipHostMalloc(&pin[k], kBounceBytes, hipHostMallocDefault));
      HIPCHK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
    }
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    c->stage_pin.insert(c->stage_pin.end(), pin, pin + 2);
    c->stage_ev.insert(c->stage_ev.end(), ev, ev + 2);
    c->stage_streams.push_back(st);
  }
  std::vector<int> rc(T, 0);
  auto work = [&](int w) {
    if (hipSetDevice(c->device) != hipSuccess) { rc[w] = SRD_ERR_HIP; return; }
    uint64_t j = 0;
    for (uint64_t ch = w; ch < nch; ch += T, j++) {
      const int b = 2 * w + (int)(j & 1);
      if (j >= 2 && hipEventSynchronize(c->stage_ev[b]) != hipSuccess) { rc[w] = SRD_ERR_HIP; return; }
      const uint64_t off = ch * kBounceBytes, n = std::min(kBounceBytes, len - off);
      memcpy(c->stage_pin[b], src + off, n);
      if (hipMemcpyAsync(dst + off, c->stage_pin[b], n, hipMemcpyHostToDevice, c->stage_streams[w]) != hipSuccess ||
          hipEventRecord(c->stage_ev[b], c->stage_streams[w]) != hipSuccess) {
        rc[w] = SRD_ERR_HIP;
        return;
      }
    }
    if (hipStreamSynchronize(c->stage_streams[w]) != hipSuccess) rc[w] = SRD_ERR_HIP;
  };
  std::vector<std::thread> th;
  for (int w = 1; w < T; w++) th.emplace_back(work, w);
  if (T) work(0);
  for (auto& t : th) t.join();
  for (int w = 0; w < T; w++)
    if (rc[w]) { set_err("bounce-buffer staging failed"); return rc[w]; }
  c->stage_mode = 2;
  return 0;
}

// pinned or registered host memory? (a pointer the runtime does not know is
// not an error here)
static bool host_is_pinned(const void* p) {
  hipPointerAttribute_t at{};
  const bool r = hipPointerGetAttributes(&at, p) == hipSuccess && at.type == hipMemoryTypeHost;
  (void)hipGetLastError();
  return r;
}

// stage host bytes [src, src + len) into the context's device file buffer;
// pinned = the caller knows the range is pinned / registered
static int stage_host_impl(Ctx* c, const uint8_t* src, uint64_t len, uint32_t flags, const uint8_t** d_out,
                           bool pinned, int workers);
// workers: bounce-buffer threads (the multi-GPU open splits them over its shards)
static int stage_host(Ctx* c, const uint8_t* src, uint64_t len, uint32_t flags, const uint8_t** d_out,
                      bool pinned = false, int workers = 1 << 20) {
  const auto t0 = std::chrono::steady_clock::now();
  const int r = stage_host_impl(c, src, len, flags, d_out, pinned, workers);
  c->stage_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return r;
}
static int stage_host_impl(Ctx* c, const uint8_t* src, uint64_t len, uint32_t flags, const uint8_t** d_out,
                           bool pinned, int workers) {
  uint8_t* d = nullptr;
  TRY(ensure_file_buf(c, len, &d));
  *d_out = d;
  if (!len) return 0;
  if (pinned) {
    HIPCHK(hipMemcpyAsync(d, src, len, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->stage_mode = 1;
    return 0;
  }
  if (flags & SRD_FLAG_STAGE_PAGEABLE) {
    HIPCHK(hipMemcpyAsync(d, src, len, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->stage_mode = 3;
    return 0;
  }
  if (host_is_pinned(src)) {
    HIPCHK(hipMemcpyAsync(d, src, len, hipMemcpyHostToDevice, c->stream));  // already pinned
    HIPCHK(hipStreamSynchronize(c->stream));
    c->stage_mode = 0;
    return 0;
  }
  if (flags & SRD_FLAG_STAGE_REGISTER) {
    const uintptr_t a = (uintptr_t)src & ~(uintptr_t)4095, e = ((uintptr_t)src + len + 4095) & ~(uintptr_t)4095;
    if (hipHostRegister((void*)a, e - a, hipHostRegisterReadOnly) == hipSuccess) {
      const hipError_t e1 = hipMemcpyAsync(d, src, len, hipMemcpyHostToDevice, c->stream);
      const hipError_t e2 = hipStreamSynchronize(c->stream);
      hipHostUnregister((void*)a);
      HIPCHK(e1);
      HIPCHK(e2);
      c->stage_mode = 1;
      return 0;
    }
    (void)hipGetLastError();
  }
  return stage_bounce(c, src, len, d, workers);
}

// Host results live in one pinned buffer the context owns (valid until the
// next host-input call on it): the device arrays are DMA'd straight into it
// -- no malloc'd pageable destinations (the runtime's own staging and their
// first-touch page faults cost ~10 ms of a C2 open) -- and srd_result_free
// only clears the struct (SRD_RESULT_CTX_OWNED in `reserved`).
constexpr uint32_t SRD_RESULT_CTX_OWNED = 1u;
static int host_result_arrays(Ctx* c, uint64_t n, uint64_t ni, srd_result* out) {
  const uint64_t n1 = std::max<uint64_t>(n, 1), k1 = std::max<uint64_t>(ni, 1);
  const uint64_t need = n1 * (5 * 8 + 2 * 4 + 1) + k1 * 16 + 64;
  if (c->h_out_n < need) {
    if (c->h_out) HIPCHK(hipHostFree(c->h_out));
    c->h_out = nullptr;
    c->h_out_n = 0;
    if (hipHostMalloc(&c->h_out, need, hipHostMallocDefault) != hipSuccess) {
      set_err("hipHostMalloc(results) failed");
      return SRD_ERR_ALLOC;
    }
    c->h_out_n = need;
  }
  uint8_t* b = (uint8_t*)c->h_out;
  auto take = [&](uint64_t bytes) { uint8_t* p = b; b += (bytes + 7) & ~7ull; return p; };
  out->meta_off = (uint64_t*)take(n1 * 8);
  out->key_hash = (uint64_t*)take(n1 * 8);
  out->prev_offset = (uint64_t*)take(n1 * 8);
  out->payload_start = (uint64_t*)take(n1 * 8);
  out->payload_len = (uint64_t*)take(n1 * 8);
  out->index_key_hash = (uint64_t*)take(k1 * 8);
  out->index_packed = (uint64_t*)take(k1 * 8);
  out->crc_stored = (uint32_t*)take(n1 * 4);
  out->crc_computed = (uint32_t*)take(n1 * 4);
  out->crc_ok = (uint8_t*)take(n1);
  out->reserved = SRD_RESULT_CTX_OWNED;
  return 0;
}

// chain entries [0, n) of a device result into host result entries [b, b + n)
static hipError_t copy_chain_d2h(hipStream_t st, const srd_device_result& r, uint64_t n, srd_result* out,
                                 uint64_t b) {
  hipError_t e = hipSuccess;
  auto cp = [&](void* dst, const void* src, uint64_t bytes) {
    if (e == hipSuccess && bytes) e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
  };
  cp(out->meta_off + b, r.meta_off, n * 8);
  cp(out->key_hash + b, r.key_hash, n * 8);
  cp(out->prev_offset + b, r.prev_offset, n * 8);
  cp(out->payload_start + b, r.payload_start, n * 8);
  cp(out->payload_len + b, r.payload_len, n * 8);
  cp(out->crc_stored + b, r.crc_stored, n * 4);
  cp(out->crc_computed + b, r.crc_computed, n * 4);
  cp(out->crc_ok + b, r.crc_ok, n);
  return e;
}

extern "C" int srd_validate_index(srd_ctx* c, const uint8_t* file, uint64_t flen, uint32_t flags, srd_result* out) {
  if (!c || !out || (!file && flen)) { set_err("bad argument"); return SRD_ERR_ARG; }
  HIPCHK(hipSetDevice(c->device));
  const uint8_t* d = nullptr;
  TRY(stage_host(c, file, flen, flags, &d));
  srd_device_result r;
  TRY(srd_validate_index_device(c, d, flen, flags & ~kStageFlags, &r));
  *out = r;
  TRY(host_result_arrays(c, r.n_chain, r.n_index, out));
  HIPCHK(copy_chain_d2h(c->stream, r, r.n_chain, out, 0));
  if (r.n_index) {
    HIPCHK(hipMemcpyAsync(out->index_key_hash, r.index_key_hash, r.n_index * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(out->index_packed, r.index_packed, r.n_index * 8, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(spin_sync(c->stream));
  return 0;
}

extern "C" void srd_result_free(srd_result* r) {
  if (!r) return;
  if (!(r->reserved & SRD_RESULT_CTX_OWNED)) {
    free(r->meta_off); free(r->key_hash); free(r->prev_offset); free(r->payload_start); free(r->payload_len);
    free(r->crc_stored); free(r->crc_computed); free(r->crc_ok); free(r->index_key_hash); free(r->index_packed);
  }
  memset(r, 0, sizeof *r);
}

extern "C" int srd_ctx_stage_info(srd_ctx* c, int* mode, double* stage_ms) {
  if (!c) { set_err("bad argument"); return SRD_ERR_ARG; }
  if (mode) *mode = c->stage_mode;
  if (stage_ms) *stage_ms = c->stage_ms;
  return 0;
}

// ---------------------------------------------------------------------------
// DataStore::open on n GPUs in one process, no RCCL.
//
// srd_validate_index_multi_device: every context holds its entry-range shard
// in its own HBM.  One host thread per context validates its span
// (srd_validate_span_device) and, for the by-owner index, partitions its
// shard-local index by owner; the host composes the shards; each owner then
// pulls its runs from every shard in shard (= file) order over xGMI
// (hipMemcpyPeerAsync; no collective library) and builds its part of the
// latest-wins index.  With SRD_FLAG_MERGE_INDEX ctxs[0] pulls the whole
// shard indexes instead and builds the one merged index.
// srd_validate_index_multi (host input) stages the spans and calls the same
// implementation with the merged index, then copies the result to the host.
//
// Peer access of device dev0 to dev's memory, enabled once per pair and
// process.  Returns false when it cannot be enabled (no xGMI path, or the
// runtime refused): hipMemcpyPeerAsync still works then, staged through host
// memory, and the call counts the pair in srd_multi_summary::peer_errors.
static bool enable_peer(int dev0, int dev) {
  static std::mutex mu;
  static uint8_t state[64][64] = {};  // 0 not tried, 1 enabled, 2 failed
  if (dev0 == dev) return true;
  if (dev0 < 0 || dev < 0 || dev0 >= 64 || dev >= 64) return false;
  std::lock_guard<std::mutex> lk(mu);
  if (!state[dev0][dev]) {
    int can = 0, cur = 0;
    bool ok = hipDeviceCanAccessPeer(&can, dev0, dev) == hipSuccess && can;
    if (ok && hipGetDevice(&cur) == hipSuccess && hipSetDevice(dev0) == hipSuccess) {
      const hipError_t e = hipDeviceEnablePeerAccess(dev, 0);
      ok = e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled;
      (void)hipSetDevice(cur);
    } else {
      ok = false;
    }
    (void)hipGetLastError();
    state[dev0][dev] = ok ? 1 : 2;
  }
  return state[dev0][dev] == 1;
}

// the same context twice would be driven by two host threads at once (its
// stream, workspace and staging buffers are not shareable)
static int check_ctxs(srd_ctx* const* ctxs, uint32_t nc) {
  if (nc > PART_MAX_WORLD) { set_err("bad argument: at most 64 contexts"); return SRD_ERR_ARG; }
  for (uint32_t i = 0; i < nc; i++) {
    if (!ctxs[i]) { set_err("bad argument: null context"); return SRD_ERR_ARG; }
    for (uint32_t j = 0; j < i; j++)
      if (ctxs[j] == ctxs[i]) { set_err("bad argument: each entry of ctxs must be a distinct context"); return SRD_ERR_ARG; }
  }
  return 0;
}

// Task i of n runs on the persistent worker of context on(i) (task 0 on the
// calling thread); the contexts of one call are distinct (check_ctxs), so no
// worker gets two tasks.  Replaces a std::thread per task per phase.
template <class On, class F>
static void parallel_for(uint32_t n, On&& on, F&& f) {
  for (uint32_t i = 1; i < n; i++) {
    Ctx* c = on(i);
    if (!c->worker) c->worker = new Worker();
    c->worker->post([&f, i] { f(i); });
  }
  if (n) f(0);
  for (uint32_t i = 1; i < n; i++) on(i)->worker->wait();
}

// Record, on the context's stream, that the device data a later cross-
// context copy will read is enqueued (the copy's stream waits on it)
static hipError_t mark_ready(Ctx* c) {
  const hipError_t e = hipEventRecord(c->ev_ready, c->stream);
  c->ready_recorded = e == hipSuccess;
  return e;
}

// device copy into dst's memory on dst's stream (peer copy over xGMI when the
// source lives on another GPU), ordered after the source context's last
// mark_ready by an explicit event wait on dst's stream; *peer_fail counts the
// copies between devices without peer access (staged by the runtime)
static hipError_t copy_to(Ctx* dst, void* d, const Ctx* src, const void* s, uint64_t bytes,
                          std::atomic<uint32_t>* peer_fail) {
  if (!bytes) return hipSuccess;
  if (src != dst && src->ready_recorded) {
    const hipError_t e = hipStreamWaitEvent(dst->stream, src->ev_ready, 0);
    if (e != hipSuccess) return e;
  }
  if (src->device == dst->device) return hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, dst->stream);
  if (!enable_peer(dst->device, src->device) && peer_fail) peer_fail->fetch_add(1);
  return hipMemcpyPeerAsync(d, dst->device, s, src->device, bytes, dst->stream);
}

using Clock = std::chrono::steady_clock;
static double ms_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

struct MultiIn {
  srd_ctx* const* ctxs;
  uint32_t nc;
  const uint8_t* const* span;  // span[i] = file byte soff[i] on ctxs[i]'s device
  const uint64_t* soff;
  const uint64_t* cuts;        // [nc + 1]: shard i holds [soff[i], cuts[i + 1]) when cuts[i] < cuts[i + 1]
  uint64_t flen;
  std::atomic<uint32_t>* peer_fail;  // copies between devices without peer access
};

// file bytes [x, y) assembled in dst's B_GATHER buffer from the shards whose
// resident range covers them (the re-validation of a run of unproven shards
// with its lower neighbour, and the whole-file path)
static int gather_range(Ctx* dst, const MultiIn& in, uint64_t x, uint64_t y, const uint8_t** out) {
  TRY(ensure(dst, B_GATHER, srd_padded_size(y - x)));
  uint8_t* d = P<uint8_t>(dst, B_GATHER);
  for (uint64_t pos = x; pos < y;) {
    int best = -1;
    uint64_t reach = pos;
    for (uint32_t j = 0; j < in.nc; j++)
      if (in.cuts[j] < in.cuts[j + 1] && in.soff[j] <= pos && in.cuts[j + 1] > reach) {
        reach = in.cuts[j + 1];
        best = (int)j;
      }
    if (best < 0) { set_err("internal: no shard holds file byte " + std::to_string(pos)); return SRD_ERR_INTERNAL; }
    const uint64_t e = std::min(y, reach);
    HIPCHK(copy_to(dst, d + (pos - x), in.ctxs[best], in.span[best] + (pos - in.soff[best]), e - pos, in.peer_fail));
    pos = e;
  }
  *out = d;
  return 0;
}

static void release_gather(Ctx* c) {
  Buf& b = c->bufs[B_GATHER];
  if (b.p) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(b.p);
  }
  b.p = nullptr;
  b.n = 0;
}

struct MShard {
  int rc = 0;
  std::string err;
  srd_device_result r{};
  bool proven = false;
  bool parted = false;
  uint64_t cnt[PART_MAX_WORLD] = {};  // owner run lengths of the partitioned shard index (host counts)
  const uint64_t* d_cnt = nullptr;     // or their device address (dev_counts: no host round trip)
};

static int multi_device_impl(const MultiIn& in, uint32_t flags, srd_device_result* shards, srd_multi_summary* sum) {
  const auto t_call = Clock::now();
  const uint32_t nc = in.nc;
  const bool merged = flags & SRD_FLAG_MERGE_INDEX;
  const uint32_t vflags = flags & ~(kStageFlags | SRD_FLAG_MERGE_INDEX);
  std::vector<uint64_t> cuts(in.cuts, in.cuts + nc + 1);
  std::vector<MShard> sh(nc);
  std::vector<double> vms(nc, 0.0);
  uint32_t path = SRD_MULTI_COMPOSED, n_err = 0;
  std::string first_err;
  // every owner can read every source's HBM (peer access, or one device):
  // the partition counts stay on the devices and the owners' gather reads
  // them (no host round trip per shard); otherwise host counts and copies
  bool dev_counts = !merged && nc > 1;
  for (uint32_t p = 0; p < nc && dev_counts; p++)
    for (uint32_t q = 0; q < nc && dev_counts; q++)
      if (in.ctxs[p]->device != in.ctxs[q]->device && !enable_peer(in.ctxs[p]->device, in.ctxs[q]->device))
        dev_counts = false;

  // owner partition of shard i's index (by-owner layout, nc > 1)
  auto part = [&](uint32_t i) -> int {
    MShard& s = sh[i];
    if (merged || nc == 1 || s.parted) return 0;
    Ctx* c = in.ctxs[i];
    const uint64_t n = s.r.n_index;
    TRY(ensure(c, B_XKEY, std::max<uint64_t>(n, 1) * 8));
    TRY(ensure(c, B_XVAL, std::max<uint64_t>(n, 1) * 8));
    if (dev_counts)  // (n == 0 too: the owners read its zero counts)
      TRY(partition_impl(c, s.r.index_key_hash, s.r.index_packed, n, nc, P<uint64_t>(c, B_XKEY), P<uint64_t>(c, B_XVAL),
                         nullptr, &s.d_cnt));
    else if (n)
      TRY(partition_impl(c, s.r.index_key_hash, s.r.index_packed, n, nc, P<uint64_t>(c, B_XKEY), P<uint64_t>(c, B_XVAL), s.cnt));
    s.parted = true;
    HIPCHK(mark_ready(c));  // the owners' pulls wait on it
    return 0;
  };
  auto validate = [&](uint32_t i, const uint8_t* d, uint64_t soff, uint64_t lo, uint64_t hi) {
    const auto t0 = Clock::now();
    MShard& s = sh[i];
    s = MShard{};
    if (lo == hi) { s.proven = true; return; }  // an empty shard composes trivially
    srd_ctx* c = in.ctxs[i];
    s.rc = srd_validate_span_device(c, d, soff, lo, hi, vflags, &s.r);
    if (!s.rc) {
      s.proven = s.r.final_len == hi && s.r.mode != SRD_MODE_SPAN_UNPROVEN;
      if (s.proven) s.rc = part(i);
      // the merged gather reads the shard's result arrays from another stream
      if (!s.rc && mark_ready(c) != hipSuccess) { set_err("hipEventRecord"); s.rc = SRD_ERR_HIP; }
    }
    if (s.rc) s.err = g_err;
    vms[i] += ms_since(t0);
  };
  auto composes = [&] {
    bool ok = true;
    for (auto& x : sh) ok = ok && !x.rc && x.proven;
    return ok;
  };
  auto note_errors = [&] {
    for (auto& x : sh)
      if (x.rc) {
        n_err++;
        if (first_err.empty()) first_err = x.err;
      }
  };

  const auto on = [&](uint32_t i) -> Ctx* { return in.ctxs[i]; };
  parallel_for(nc, on, [&](uint32_t i) {
    if (hipSetDevice(in.ctxs[i]->device) != hipSuccess) { sh[i] = MShard{}; sh[i].rc = SRD_ERR_HIP; sh[i].err = "hipSetDevice"; return; }
    validate(i, in.span[i], in.soff[i], cuts[i], cuts[i + 1]);
  });
  bool composed = composes();
  note_errors();
  // shard 0 over the whole store IS the whole-file path (lo = 0)
  const bool whole_already = cuts[1] == in.flen;
  if (!composed && !n_err && !whole_already) {
    // A cut that is no chain tail (a forged metadata record in a payload)
    // leaves the shard above it unproven (no node has prev == the cut).
    // Each run [a, b] of unproven shards is re-validated once together with
    // its lower neighbour, as the span [cuts[a], cuts[b+1]) whose ends are
    // tails the neighbours proved -- its bytes gathered onto ctxs[a]'s GPU:
    // 2/nc of the store instead of all of it.  Still unproven (a torn tail,
    // corruption): the whole-file path decides.
    path = SRD_MULTI_NEIGHBOUR;
    std::vector<std::pair<uint32_t, uint32_t>> runs;
    uint32_t floor = 0;  // the first shard the next run may take
    for (uint32_t i = 0; i < nc; i++) {
      if (sh[i].proven) continue;
      uint32_t b = i;
      while (b + 1 < nc && !sh[b + 1].proven) b++;
      // the lower neighbour: the first non-empty shard below (an empty shard
      // "proves" nothing; its cut may be the forged one)
      uint32_t a = i ? i - 1 : 0;
      while (a > floor && cuts[a] == cuts[a + 1]) a--;
      if (!runs.empty() && a <= floor && cuts[a] == cuts[a + 1]) {
        // the walk reached the previous run through empty shards only: no
        // shard between proves a tail, so this run joins the previous one
        // (two runs would both start or end at the suspect cut)
        runs.back().second = b;
      } else {
        runs.emplace_back(std::max(a, floor), b);
      }
      floor = b + 1;
      i = b;
    }
    for (auto [a, b] : runs)
      for (uint32_t i = a + 1; i <= b; i++) {
        cuts[i] = cuts[b + 1];  // shards a+1..b become empty; shard a spans the run
        sh[i] = MShard{};
        sh[i].proven = true;
      }
    parallel_for((uint32_t)runs.size(), [&](uint32_t k) -> Ctx* { return in.ctxs[runs[k].first]; }, [&](uint32_t k) {
      const uint32_t a = runs[k].first;
      const uint64_t lo = cuts[a], hi = cuts[a + 1], x = lo - lo % SPAN_BYTES;
      const uint8_t* d = nullptr;
      Ctx* c = in.ctxs[a];
      int r = hipSetDevice(c->device) == hipSuccess ? 0 : SRD_ERR_HIP;
      if (!r && lo < hi) r = gather_range(c, in, x, hi, &d);
      if (r) {
        sh[a] = MShard{};
        sh[a].rc = r;
        sh[a].err = g_err;
        return;
      }
      validate(a, d, x, lo, hi);
    });
    composed = composes();
    note_errors();
  }
  if (!composed && !whole_already) {
    // a torn tail, corruption, or a shard that failed (capacity, allocation):
    // recover_valid_chain's byte-wise search is global, so the whole-file
    // path decides, on ctxs[0] with the store gathered there
    path = SRD_MULTI_WHOLE_FILE;
    for (uint32_t i = 1; i < nc; i++) {
      sh[i] = MShard{};
      cuts[i] = in.flen;
    }
    srd_ctx* c0 = in.ctxs[0];
    const auto t0 = Clock::now();
    sh[0] = MShard{};
    const uint8_t* d = nullptr;
    int r = hipSetDevice(c0->device) == hipSuccess ? 0 : SRD_ERR_HIP;
    if (!r) r = gather_range(c0, in, 0, in.flen, &d);
    if (!r) r = srd_validate_index_device(c0, d, in.flen, vflags, &sh[0].r);
    if (!r) r = part(0);
    vms[0] += ms_since(t0);
    if (r) {
      if (!first_err.empty()) set_err(g_err + " (after a shard error: " + first_err + ")");
      release_gather(c0);
      return r;
    }
  } else if (!composed) {
    path = SRD_MULTI_WHOLE_FILE;  // shard 0 was the whole store: its answer is final
    if (sh[0].rc) {
      set_err(sh[0].err);
      return sh[0].rc;
    }
  }
  for (uint32_t i = 0; i < nc; i++) release_gather(in.ctxs[i]);

  // ---- index exchange ----
  const auto t_ex = Clock::now();
  std::vector<uint64_t> ni(nc, 0);
  std::vector<int> erc(nc, 0);
  std::vector<std::string> eerr(nc);
  uint64_t merged_n = 0;
  uint64_t *mkey = nullptr, *mpacked = nullptr;
  if (nc == 1) {
    ni[0] = sh[0].r.n_index;
    mkey = sh[0].r.index_key_hash;
    mpacked = sh[0].r.index_packed;
    merged_n = ni[0];
  } else if (merged) {
    Ctx* c0 = in.ctxs[0];
    int r = hipSetDevice(c0->device) == hipSuccess ? 0 : SRD_ERR_HIP;
    uint64_t NI = 0;
    for (auto& x : sh) NI += x.r.n_index;
    const uint64_t m1 = std::max<uint64_t>(NI, 1);
    if (!r) r = ensure(c0, B_GKEY, m1 * 8);
    if (!r) r = ensure(c0, B_GVAL, m1 * 8);
    if (!r) r = ensure(c0, B_GOKEY, m1 * 8);
    if (!r) r = ensure(c0, B_GOPACKED, m1 * 8);
    uint64_t acc = 0;
    for (uint32_t s = 0; s < nc && !r; s++) {
      const uint64_t n = sh[s].r.n_index;
      if (copy_to(c0, P<uint64_t>(c0, B_GKEY) + acc, in.ctxs[s], sh[s].r.index_key_hash, n * 8, in.peer_fail) != hipSuccess ||
          copy_to(c0, P<uint64_t>(c0, B_GVAL) + acc, in.ctxs[s], sh[s].r.index_packed, n * 8, in.peer_fail) != hipSuccess) {
        set_err("index gather: peer copy failed");
        r = SRD_ERR_HIP;
      }
      acc += n;
    }
    if (!r) r = index_build_sep(c0, P<uint64_t>(c0, B_GKEY), P<uint64_t>(c0, B_GVAL), NI, P<uint64_t>(c0, B_GOKEY),
                                P<uint64_t>(c0, B_GOPACKED), &merged_n);
    if (r) return r;
    mkey = P<uint64_t>(c0, B_GOKEY);
    mpacked = P<uint64_t>(c0, B_GOPACKED);
  } else {
    // by owner: the shards re-validated above partition now
    parallel_for(nc, on, [&](uint32_t i) {
      if (hipSetDevice(in.ctxs[i]->device) != hipSuccess) { erc[i] = SRD_ERR_HIP; return; }
      if ((erc[i] = part(i))) eerr[i] = g_err;
    });
    for (uint32_t i = 0; i < nc; i++)
      if (erc[i]) { set_err(eerr[i]); return erc[i]; }
    uint64_t ni_all = 0, ni_max1 = 0;  // pairs of every shard; the largest shard's
    for (auto& x : sh) {
      ni_all += x.r.n_index;
      ni_max1 = std::max<uint64_t>(ni_max1, x.r.n_index);
    }
    parallel_for(nc, on, [&](uint32_t p) {
      Ctx* c = in.ctxs[p];
      int& r = erc[p];
      if (hipSetDevice(c->device) != hipSuccess) { r = SRD_ERR_HIP; eerr[p] = "hipSetDevice"; return; }
      if (dev_counts) {
        // the owner's runs: lengths and offsets from the sources' partition
        // counts in their HBM (gather_runs_kernel), the build's n on the
        // device; sized by the bound ni_all, buckets for ni_all / nc pairs
        // (owner = the key hash's top bits: an even split)
        const uint64_t m1 = std::max<uint64_t>(ni_all, 1);
        if (!r) r = ensure(c, B_GKEY, m1 * 8);
        if (!r) r = ensure(c, B_GVAL, m1 * 8);
        if (!r) r = ensure(c, B_GOKEY, m1 * 8);
        if (!r) r = ensure(c, B_GOPACKED, m1 * 8);
        if (!r) r = ensure(c, B_XTOT, 64);
        GatherArgs ga{};
        for (uint32_t s = 0; s < nc; s++) {
          Ctx* cs = in.ctxs[s];
          ga.src_k[s] = P<uint64_t>(cs, B_XKEY);
          ga.src_v[s] = P<uint64_t>(cs, B_XVAL);
          ga.src_cnt[s] = sh[s].d_cnt;
          if (!r && cs != c && cs->ready_recorded && hipStreamWaitEvent(c->stream, cs->ev_ready, 0) != hipSuccess) {
            set_err("index exchange: event wait failed");
            r = SRD_ERR_HIP;
          }
        }
        ga.dst_k = P<uint64_t>(c, B_GKEY);
        ga.dst_v = P<uint64_t>(c, B_GVAL);
        ga.d_total = P<uint64_t>(c, B_XTOT);
        ga.owner = p;
        ga.nsrc = nc;
        if (!r) {
          const uint64_t per = ni_max1 / nc + 1;  // ~ a source's run for one owner
          const dim3 grid((unsigned)std::min<uint64_t>(std::max<uint64_t>((2 * per + 255) / 256, 1), 128), nc);
          gather_runs_kernel<<<grid, 256, 0, c->stream>>>(ga);
          if (hipGetLastError() != hipSuccess) { set_err("index exchange: gather launch failed"); r = SRD_ERR_HIP; }
        }
        if (!r) r = index_build_dev(c, ga.dst_k, ga.dst_v, ni_all, ga.d_total, ni_all / nc + 1, P<uint64_t>(c, B_GOKEY),
                                    P<uint64_t>(c, B_GOPACKED), &ni[p]);
        if (r) eerr[p] = g_err;
        return;
      }
      uint64_t NI = 0;
      for (auto& x : sh) NI += x.cnt[p];
      const uint64_t m1 = std::max<uint64_t>(NI, 1);
      if (!r) r = ensure(c, B_GKEY, m1 * 8);
      if (!r) r = ensure(c, B_GVAL, m1 * 8);
      if (!r) r = ensure(c, B_GOKEY, m1 * 8);
      if (!r) r = ensure(c, B_GOPACKED, m1 * 8);
      // every source's run: one gather launch reading the peers' HBM when
      // every source GPU is peer-accessible, else one copy per run
      GatherArgs ga{};
      bool direct = true;
      uint64_t acc = 0, nmax = 0;
      for (uint32_t s = 0; s < nc; s++) {
        uint64_t off = 0;
        for (uint32_t q = 0; q < p; q++) off += sh[s].cnt[q];
        Ctx* cs = in.ctxs[s];
        ga.src_k[s] = P<uint64_t>(cs, B_XKEY) + off;
        ga.src_v[s] = P<uint64_t>(cs, B_XVAL) + off;
        ga.dst_off[s] = acc;
        acc += sh[s].cnt[p];
        nmax = std::max<uint64_t>(nmax, sh[s].cnt[p]);
        if (cs->device != c->device && !enable_peer(c->device, cs->device)) direct = false;
      }
      ga.dst_off[nc] = acc;
      ga.dst_k = P<uint64_t>(c, B_GKEY);
      ga.dst_v = P<uint64_t>(c, B_GVAL);
      if (!r && direct && nmax) {
        for (uint32_t s = 0; s < nc && !r; s++) {
          Ctx* cs = in.ctxs[s];
          if (cs != c && cs->ready_recorded && hipStreamWaitEvent(c->stream, cs->ev_ready, 0) != hipSuccess) {
            set_err("index exchange: event wait failed");
            r = SRD_ERR_HIP;
          }
        }
        if (!r) {
          const dim3 grid((unsigned)std::min<uint64_t>((nmax + 255) / 256, 128), nc);
          gather_runs_kernel<<<grid, 256, 0, c->stream>>>(ga);
          if (hipGetLastError() != hipSuccess) { set_err("index exchange: gather launch failed"); r = SRD_ERR_HIP; }
        }
      } else if (!r) {
        for (uint32_t s = 0; s < nc && !r; s++) {
          const uint64_t n = sh[s].cnt[p];
          Ctx* cs = in.ctxs[s];
          if (copy_to(c, ga.dst_k + ga.dst_off[s], cs, ga.src_k[s], n * 8, in.peer_fail) != hipSuccess ||
              copy_to(c, ga.dst_v + ga.dst_off[s], cs, ga.src_v[s], n * 8, in.peer_fail) != hipSuccess) {
            set_err("index exchange: peer copy failed");
            r = SRD_ERR_HIP;
          }
        }
      }
      if (!r) r = index_build_sep(c, P<uint64_t>(c, B_GKEY), P<uint64_t>(c, B_GVAL), NI, P<uint64_t>(c, B_GOKEY),
                                  P<uint64_t>(c, B_GOPACKED), &ni[p]);
      if (r) eerr[p] = g_err;
    });
    for (uint32_t i = 0; i < nc; i++)
      if (erc[i]) { set_err(eerr[i]); return erc[i]; }
  }
  const double ex_ms = ms_since(t_ex);

  srd_multi_summary S{};
  S.file_len = in.flen;
  S.final_len = path == SRD_MULTI_WHOLE_FILE ? sh[0].r.final_len : in.flen;
  S.mode = SRD_MODE_OPTIMISTIC;
  for (uint32_t i = 0; i < nc; i++) {
    srd_device_result o = sh[i].r;
    if (cuts[i] == cuts[i + 1] && path != SRD_MULTI_WHOLE_FILE) memset(&o, 0, sizeof o);
    if (path == SRD_MULTI_WHOLE_FILE && i) memset(&o, 0, sizeof o);
    S.n_chain += o.n_chain;
    S.n_crc_bad += o.n_crc_bad;
    S.n_candidates += o.n_candidates;
    if ((o.n_chain || i == 0) && o.mode != SRD_MODE_OPTIMISTIC) S.mode = SRD_MODE_FULL;
    if (merged || nc == 1) {
      if (nc > 1) {
        o.n_index = 0;
        o.index_key_hash = o.index_packed = nullptr;
      }
    } else {
      Ctx* c = in.ctxs[i];
      o.n_index = ni[i];
      o.index_key_hash = P<uint64_t>(c, B_GOKEY);
      o.index_packed = P<uint64_t>(c, B_GOPACKED);
      S.n_index += ni[i];
    }
    shards[i] = o;
  }
  if (merged || nc == 1) {
    S.n_index = merged_n;
    S.index_key_hash = mkey;
    S.index_packed = mpacked;
  }
  S.path = path;
  S.n_shards = nc;
  S.merged = (merged || nc == 1) ? 1u : 0u;
  S.shard_errors = n_err;
  S.peer_errors = in.peer_fail ? in.peer_fail->load() : 0u;
  for (double v : vms) S.validate_ms = std::max(S.validate_ms, v);
  S.exchange_ms = ex_ms;
  S.total_ms = ms_since(t_call);
  if (sum) *sum = S;
  in.ctxs[0]->last_multi = S;
  in.ctxs[0]->last_shard_ms = vms;
  return 0;
}

extern "C" int srd_validate_index_multi_device(srd_ctx* const* ctxs, uint32_t nc, const uint8_t* const* d_spans,
                                               const uint64_t* span_offs, const uint64_t* cuts, uint32_t flags,
                                               srd_device_result* shards, srd_multi_summary* summary) {
  if (!ctxs || !nc || !d_spans || !span_offs || !cuts || !shards) { set_err("bad argument"); return SRD_ERR_ARG; }
  TRY(check_ctxs(ctxs, nc));
  const uint64_t flen = cuts[nc];
  if (cuts[0] != 0 || flen > kMaxFile) { set_err("bad argument: cuts[0] must be 0 and file_len <= 2^48"); return SRD_ERR_ARG; }
  for (uint32_t i = 0; i < nc; i++) {
    if (cuts[i] > cuts[i + 1]) { set_err("bad argument: cuts must be non-decreasing"); return SRD_ERR_ARG; }
    if (cuts[i] == cuts[i + 1]) continue;
    if (!d_spans[i] || span_offs[i] % SPAN_BYTES || span_offs[i] > cuts[i] || (cuts[i] == 0 && span_offs[i])) {
      set_err("bad argument: shard " + std::to_string(i) +
              " needs a span starting at a multiple of 16 KiB at or below its lower tail");
      return SRD_ERR_ARG;
    }
  }
  std::atomic<uint32_t> peer_fail{0};
  MultiIn in{ctxs, nc, d_spans, span_offs, cuts, flen, &peer_fail};
  return multi_device_impl(in, flags, shards, summary);
}

extern "C" int srd_ctx_multi_shard_ms(srd_ctx* c, double* out, int cap) {
  if (!c || cap < 0 || (cap && !out)) { set_err("bad argument"); return SRD_ERR_ARG; }
  const int n = (int)c->last_shard_ms.size();
  for (int i = 0; i < std::min(n, cap); i++) out[i] = c->last_shard_ms[i];
  return n;
}

extern "C" int srd_ctx_multi_summary(srd_ctx* c, srd_multi_summary* out) {
  if (!c || !out) { set_err("bad argument"); return SRD_ERR_ARG; }
  *out = c->last_multi;
  return 0;
}

extern "C" int srd_validate_index_multi(srd_ctx* const* ctxs, uint32_t nc, const uint8_t* file, uint64_t flen,
                                        uint32_t flags, srd_result* out) {
  if (!ctxs || !nc || !out || (!file && flen)) { set_err("bad argument"); return SRD_ERR_ARG; }
  TRY(check_ctxs(ctxs, nc));
  if (nc == 1) return srd_validate_index(ctxs[0], file, flen, flags, out);
  std::vector<uint64_t> cuts(nc + 1), soff(nc, 0);
  {
    const char* why = "";
    const int r = srd_host::shard_cuts(file, flen, nc, cuts.data(), &why);
    if (r) { set_err(why); return r; }
  }
  // pinned input: each shard copies its span directly.  SRD_FLAG_STAGE_REGISTER:
  // the mapping is registered once for all shards (their spans overlap by
  // up to 16 KiB).  Otherwise each shard's bounce workers (the host threads
  // split over the shards) stage its span.
  uintptr_t reg_a = 0, reg_e = 0;
  bool pinned = false;
  if (flen && !(flags & SRD_FLAG_STAGE_PAGEABLE)) {
    if (host_is_pinned(file)) {
      pinned = true;
    } else if (flags & SRD_FLAG_STAGE_REGISTER) {
      HIPCHK(hipSetDevice(ctxs[0]->device));
      reg_a = (uintptr_t)file & ~(uintptr_t)4095;
      reg_e = ((uintptr_t)file + flen + 4095) & ~(uintptr_t)4095;
      pinned = hipHostRegister((void*)reg_a, reg_e - reg_a, hipHostRegisterReadOnly | hipHostRegisterPortable) ==
               hipSuccess;
      (void)hipGetLastError();
      if (!pinned) reg_a = reg_e = 0;
    }
  }
  std::vector<const uint8_t*> span(nc, nullptr);
  std::vector<int> rc(nc, 0);
  std::vector<std::string> err(nc);
  const auto on = [&](uint32_t i) -> Ctx* { return ctxs[i]; };
  parallel_for(nc, on, [&](uint32_t i) {
    srd_ctx* c = ctxs[i];
    const uint64_t lo = cuts[i], hi = cuts[i + 1];
    if (lo == hi) return;
    soff[i] = lo - lo % SPAN_BYTES;
    if (hipSetDevice(c->device) != hipSuccess) { rc[i] = SRD_ERR_HIP; err[i] = "hipSetDevice"; return; }
    rc[i] = stage_host(c, file + soff[i], hi - soff[i], flags, &span[i], pinned,
                       std::max(1, ctxs[0]->stage_workers / (int)nc));
    if (rc[i]) err[i] = g_err;
  });
  if (reg_a) {
    (void)hipSetDevice(ctxs[0]->device);
    (void)hipHostUnregister((void*)reg_a);
  }
  for (uint32_t i = 0; i < nc; i++)
    if (rc[i]) { set_err(err[i]); return rc[i]; }
  std::vector<srd_device_result> sr(nc);
  srd_multi_summary sum{};
  std::atomic<uint32_t> peer_fail{0};
  MultiIn in{ctxs, nc, span.data(), soff.data(), cuts.data(), flen, &peer_fail};
  TRY(multi_device_impl(in, (flags & ~kStageFlags) | SRD_FLAG_MERGE_INDEX, sr.data(), &sum));

  memset(out, 0, sizeof *out);
  const uint64_t N = sum.n_chain;
  TRY(host_result_arrays(ctxs[0], N, sum.n_index, out));
  // chain segments D2H on each shard's stream (file order); the merged
  // index from ctxs[0]
  std::vector<uint64_t> cb(nc, 0);
  for (uint32_t i = 1; i < nc; i++) cb[i] = cb[i - 1] + sr[i - 1].n_chain;
  parallel_for(nc, on, [&](uint32_t i) {
    srd_ctx* c = ctxs[i];
    const uint64_t nk = i == 0 ? sum.n_index : 0;
    if (!sr[i].n_chain && !nk) return;
    if (hipSetDevice(c->device) != hipSuccess) { rc[i] = SRD_ERR_HIP; return; }
    hipError_t e = copy_chain_d2h(c->stream, sr[i], sr[i].n_chain, out, cb[i]);
    if (e == hipSuccess && nk)
      e = hipMemcpyAsync(out->index_key_hash, sum.index_key_hash, nk * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && nk)
      e = hipMemcpyAsync(out->index_packed, sum.index_packed, nk * 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) rc[i] = SRD_ERR_HIP;
  });
  for (uint32_t i = 0; i < nc; i++)
    if (rc[i]) { srd_result_free(out); set_err("result copy failed"); return rc[i]; }
  out->file_len = flen;
  out->final_len = sum.final_len;
  out->n_chain = N;
  out->n_index = sum.n_index;
  out->n_crc_bad = sum.n_crc_bad;
  out->n_candidates = sum.n_candidates;
  out->mode = sum.mode;
  return 0;
}

extern "C" int srd_stream_probe_device(srd_ctx* c, const uint8_t* d_buf, uint64_t bytes, int reps, double* best_ms,
                                       double* median_ms) {
  if (!c || !d_buf || bytes < TILE || reps < 1 || !best_ms) { set_err("bad argument"); return SRD_ERR_ARG; }
  HIPCHK(hipSetDevice(c->device));
  const uint64_t ntiles = bytes / TILE;
  TRY(ensure(c, B_PROBE, (uint64_t)c->scan_blocks * 16 * 4));
  hipEvent_t e[2];
  for (auto& x : e) HIPCHK(hipEventCreateWithFlags(&x, hipEventReleaseToDevice));
  std::vector<float> ms;
  int rc = 0;
  for (int r = 0; r < reps + 1 && !rc; r++) {  // (the first run warms the code and the TLB)
    hipExtLaunchKernelGGL(stream_probe_kernel, dim3(c->scan_blocks), dim3(1024), 0, c->stream, e[0], e[1], 0, d_buf,
                          ntiles, P<uint32_t>(c, B_PROBE));
    float t = 0;
    if (hipGetLastError() != hipSuccess || hipEventSynchronize(e[1]) != hipSuccess ||
        hipEventElapsedTime(&t, e[0], e[1]) != hipSuccess) {
      set_err("stream probe launch failed");
      rc = SRD_ERR_HIP;
    }
    if (r) ms.push_back(t);
  }
  for (auto& x : e) hipEventDestroy(x);
  if (rc) return rc;
  std::sort(ms.begin(), ms.end());
  *best_ms = ms[0];
  if (median_ms) *median_ms = ms[ms.size() / 2];
  return 0;
}

extern "C" int srd_index_hash_device(srd_ctx* c, const uint64_t* d_keys, uint64_t n, uint64_t* d_out, void* stream) {
  if (!c || (n && (!d_keys || !d_out))) { set_err("bad argument"); return SRD_ERR_ARG; }
  if (!n) return 0;
  HIPCHK(hipSetDevice(c->device));
  index_hash_kernel<<<(unsigned)std::min<uint64_t>((n + 255) / 256, 8192), 256, 0,
                      stream ? (hipStream_t)stream : c->stream>>>(d_keys, n, d_out);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int srd_recover_valid_chain(srd_ctx* c, const uint8_t* file, uint64_t flen, uint64_t* final_len) {
  if (!final_len) { set_err("bad argument"); return SRD_ERR_ARG; }
  if (!c) { set_err("bad argument"); return SRD_ERR_ARG; }
  HIPCHK(hipSetDevice(c->device));
  const uint8_t* d = nullptr;
  TRY(stage_host(c, file, flen, 0, &d));
  srd_device_result r;
  TRY(srd_validate_index_device(c, d, flen, SRD_FLAG_NO_CRC, &r));
  *final_len = r.final_len;
  return 0;
}

extern "C" int srd_key_indexer_build(srd_ctx* c, const uint8_t* file, uint64_t tail, uint64_t* keys,
                                     uint64_t* packed, uint64_t cap, uint64_t* n_out) {
  if (!n_out) { set_err("bad argument"); return SRD_ERR_ARG; }
  if (!c) { set_err("bad argument"); return SRD_ERR_ARG; }
  HIPCHK(hipSetDevice(c->device));
  const uint8_t* d = nullptr;
  TRY(stage_host(c, file, tail, 0, &d));
  srd_device_result r;
  TRY(srd_validate_index_device(c, d, tail, SRD_FLAG_NO_CRC, &r));
  if (r.final_len != tail) {
    set_err("tail is not a valid chain tail (KeyIndexer::build expects the recovered tail)");
    return SRD_ERR_ARG;
  }
  *n_out = r.n_index;
  uint64_t k = std::min(cap, r.n_index);
  if (k) {
    HIPCHK(hipMemcpyAsync(keys, r.index_key_hash, k * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(packed, r.index_packed, k * 8, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(spin_sync(c->stream));
  return 0;
}

extern "C" int srd_crc32_batch_device(srd_ctx* c, const uint8_t* d_buf, const uint64_t* d_offs,
                                      const uint64_t* d_lens, uint64_t n, uint32_t* d_out, void* stream) {
  if (!c) { set_err("bad argument"); return SRD_ERR_ARG; }
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  if (!n) return 0;
  crc_batch_kernel<<<(unsigned)std::min<uint64_t>(n, 8192), 64, 0, s>>>(d_buf, d_offs, d_lens, n, d_out);
  KCHK(c, "crc_batch_kernel");
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int srd_xxh3_64_batch_device(srd_ctx* c, const uint8_t* d_keys, const uint64_t* d_offs,
                                        const uint64_t* d_lens, uint64_t n, uint64_t* d_out, void* stream) {
  if (!c) { set_err("bad argument"); return SRD_ERR_ARG; }
  hipStream_t s = stream ? (hipStream_t)stream : c->stream;
  if (!n) return 0;
  xxh3_batch_kernel<<<blocks(n, 256), 256, 0, s>>>(d_keys, d_offs, d_lens, n, d_out);
  KCHK(c, "xxh3_batch_kernel");
  HIPCHK(hipGetLastError());
  return 0;
}

template <class OUT, class F>
static int batch_host(srd_ctx* c, const uint8_t* buf, uint64_t blen, const uint64_t* offs, const uint64_t* lens,
                      uint64_t n, OUT* out, F launch) {
  HIPCHK(hipSetDevice(c->device));
  for (uint64_t i = 0; i < n; i++)
    if (offs[i] > blen || lens[i] > blen - offs[i]) { set_err("range out of bounds"); return SRD_ERR_ARG; }
  void *db = nullptr, *dof = nullptr, *dl = nullptr, *dout = nullptr;
  HIPCHK(hipMalloc(&db, blen + 1));
  HIPCHK(hipMalloc(&dof, n * 8 + 8));
  HIPCHK(hipMalloc(&dl, n * 8 + 8));
  HIPCHK(hipMalloc(&dout, n * sizeof(OUT) + 8));
  if (blen) HIPCHK(hipMemcpyAsync(db, buf, blen, hipMemcpyHostToDevice, c->stream));
  if (n) {
    HIPCHK(hipMemcpyAsync(dof, offs, n * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(dl, lens, n * 8, hipMemcpyHostToDevice, c->stream));
  }
  int r = launch((const uint8_t*)db, (const uint64_t*)dof, (const uint64_t*)dl, (OUT*)dout);
  if (!r && n) HIPCHK(hipMemcpyAsync(out, dout, n * sizeof(OUT), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(spin_sync(c->stream));
  hipFree(db); hipFree(dof); hipFree(dl); hipFree(dout);
  return r;
}

extern "C" int srd_crc32_batch(srd_ctx* c, const uint8_t* buf, uint64_t blen, const uint64_t* offs,
                               const uint64_t* lens, uint64_t n, uint32_t* out) {
  if (!c || (n && (!offs || !lens || !out))) { set_err("bad argument"); return SRD_ERR_ARG; }
  return batch_host<uint32_t>(c, buf, blen, offs, lens, n, out, [&](auto db, auto dof, auto dl, auto dout) {
    return srd_crc32_batch_device(c, db, dof, dl, n, dout, nullptr);
  });
}

extern "C" int srd_xxh3_64_batch(srd_ctx* c, const uint8_t* keys, uint64_t klen, const uint64_t* offs,
                                 const uint64_t* lens, uint64_t n, uint64_t* out) {
  if (!c || (n && (!offs || !lens || !out))) { set_err("bad argument"); return SRD_ERR_ARG; }
  return batch_host<uint64_t>(c, keys, klen, offs, lens, n, out, [&](auto db, auto dof, auto dl, auto dout) {
    return srd_xxh3_64_batch_device(c, db, dof, dl, n, dout, nullptr);
  });
}

// entry tails: lens (if given) holds the lengths of entries 0 .. first+n-1
static int synth_offsets(uint64_t first, uint64_t n, uint64_t fixed_len, const uint64_t* lens, uint64_t span_off,
                         std::vector<uint64_t>* off, uint64_t* e0, uint64_t* lo, uint64_t* hi) {
  uint64_t tail = 0;
  *lo = 0;
  *e0 = first;
  bool have_e0 = false;
  if (off) off->clear();
  for (uint64_t i = 0; i < first + n; i++) {
    const uint64_t L = lens ? lens[i] : fixed_len;
    if (L == 0) { set_err("empty payload"); return SRD_ERR_ARG; }
    if (i == first) *lo = tail;
    const uint64_t end = tail + ((64 - tail % 64) & 63) + L + 20;
    if (!have_e0 && (end > span_off || i == first)) { *e0 = i; have_e0 = true; }
    if (have_e0 && off) off->push_back(tail);
    tail = end;
  }
  *hi = tail;
  return 0;
}

static int synth_launch(Ctx* c, uint8_t* d_abs, const std::vector<uint64_t>& off, uint64_t e0, uint64_t fixed_len,
                        const uint64_t* lens, uint64_t seed, uint64_t clip_lo) {
  const uint64_t n = off.size();
  if (!n) return 0;
  HIPCHK(hipSetDevice(c->device));
  void *doff = nullptr, *dl = nullptr;
  HIPCHK(hipMalloc(&doff, n * 8));
  HIPCHK(hipMemcpyAsync(doff, off.data(), n * 8, hipMemcpyHostToDevice, c->stream));
  if (lens) {
    HIPCHK(hipMalloc(&dl, n * 8));
    HIPCHK(hipMemcpyAsync(dl, lens + e0, n * 8, hipMemcpyHostToDevice, c->stream));
  }
  synth_kernel<<<(unsigned)std::min<uint64_t>(n, 65536), 64, 0, c->stream>>>(
      d_abs, (const uint64_t*)doff, (const uint64_t*)dl, fixed_len, n, seed, e0, clip_lo);
  KCHK(c, "synth_kernel");
  HIPCHK(hipGetLastError());
  HIPCHK(spin_sync(c->stream));
  hipFree(doff);
  if (dl) hipFree(dl);
  return 0;
}

extern "C" int srd_synth_store_device(srd_ctx* c, uint8_t* d_out, uint64_t n, uint64_t fixed_len,
                                      const uint64_t* lens, uint64_t seed, uint64_t* len_out) {
  if (!len_out) { set_err("bad argument"); return SRD_ERR_ARG; }
  std::vector<uint64_t> off;
  uint64_t e0, lo, hi;
  TRY(synth_offsets(0, n, fixed_len, lens, 0, d_out ? &off : nullptr, &e0, &lo, &hi));
  *len_out = hi;
  if (!d_out || !n) return 0;
  if (!c) { set_err("bad argument"); return SRD_ERR_ARG; }
  return synth_launch(c, d_out, off, 0, fixed_len, lens, seed, 0);
}

extern "C" int srd_synth_span_device(srd_ctx* c, uint8_t* d_span, uint64_t span_off, uint64_t first,
                                     uint64_t n, uint64_t fixed_len, const uint64_t* lens, uint64_t seed,
                                     uint64_t* lo_out, uint64_t* hi_out) {
  if (!lo_out || !hi_out || (span_off % SPAN_BYTES)) { set_err("bad argument"); return SRD_ERR_ARG; }
  std::vector<uint64_t> off;
  uint64_t e0, lo, hi;
  TRY(synth_offsets(first, n, fixed_len, lens, span_off, d_span ? &off : nullptr, &e0, &lo, &hi));
  *lo_out = lo;
  *hi_out = hi;
  if (!d_span || !n) return 0;
  if (!c || span_off > lo) { set_err("bad argument: span_off must be <= the shard's lower tail"); return SRD_ERR_ARG; }
  return synth_launch(c, d_span - span_off, off, e0, fixed_len, lens, seed, span_off);
}

// ---------------------------------------------------------------------------
// Checksum-on-append batch writer (C5): layout on the host (prepad_len chains
// every start to all earlier lengths), serialization + CRC + key hash on the
// device (write_kernel), chunked H2D of the inputs on a side stream.
extern "C" int srd_batch_layout(uint64_t tail, const uint8_t* payloads, const uint64_t* key_offs,
                                const uint64_t* key_lens, const uint64_t* pay_offs, const uint64_t* pay_lens,
                                uint64_t n, uint32_t flags, srd_write_entry* out, uint64_t* new_tail) {
  const char* why = "";
  const int r = srd_host::batch_layout(tail, payloads, key_offs, key_lens, pay_offs, pay_lens, n, flags, out, new_tail,
                                       &why);
  if (r) set_err(why);
  return r;
}

static int launch_write(Ctx* c, hipStream_t s, const uint8_t* pay, const uint8_t* keys, const srd_write_entry* ent,
                        uint64_t n, uint8_t* out, uint64_t base, uint64_t* kh, uint64_t* mo,
                        unsigned int* null_only = nullptr) {
  if (!n) return 0;
  WriteArgs w{pay, keys, ent, n, out, base, kh, mo, null_only};
  const unsigned g = (unsigned)std::min<uint64_t>((n + SCAN_WAVES_V2 - 1) / SCAN_WAVES_V2, c->scan_blocks);
#ifdef SRD_DEBUG_API
  if (c->scan_variant == 21)
    write_kernel<1><<<g, SCAN_WAVES_V2 * 64, 0, s>>>(w);
  else if (c->scan_variant == 22)
    write_kernel<2><<<g, SCAN_WAVES_V2 * 64, 0, s>>>(w);
  else if (c->scan_variant == 29)
    write_kernel<9><<<g, SCAN_WAVES_V2 * 64, 0, s>>>(w);
  else
#endif
    write_kernel<<<g, SCAN_WAVES_V2 * 64, 0, s>>>(w);
  HIPCHK(hipGetLastError());
  if (sync_debug()) {
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipGetLastError());
  }
  return 0;
}

extern "C" int srd_batch_write_device(srd_ctx* c, const uint8_t* d_keys, const uint8_t* d_payloads,
                                      const srd_write_entry* d_entries, uint64_t n, uint8_t* d_out,
                                      uint64_t out_base, uint64_t* d_kh_out, uint64_t* d_mo_out, void* stream) {
  if (!c || (out_base & 63) ||
      (n && (!d_keys || !d_payloads || !d_entries || !d_out || !d_kh_out || !d_mo_out))) {
    set_err("bad argument");
    return SRD_ERR_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  return launch_write(c, stream ? (hipStream_t)stream : c->stream, d_payloads, d_keys, d_entries, n, d_out, out_base,
                      d_kh_out, d_mo_out);
}

extern "C" int srd_batch_write(srd_ctx* c, uint64_t tail, const uint8_t* keys, const uint64_t* key_offs,
                               const uint64_t* key_lens, const uint8_t* payloads, const uint64_t* pay_offs,
                               const uint64_t* pay_lens, uint64_t n, uint32_t flags, uint8_t* d_out, uint64_t out_cap,
                               uint64_t* new_tail, uint64_t* kh_out, uint64_t* mo_out) {
  if (!c || !new_tail || (n && (!payloads || !keys))) { set_err("bad argument"); return SRD_ERR_ARG; }
  std::vector<srd_write_entry> E(n);
  uint64_t nt = 0;
  TRY(srd_batch_layout(tail, payloads, key_offs, key_lens, pay_offs, pay_lens, n, flags, E.data(), &nt));
  *new_tail = nt;
  if (!d_out || !n) return 0;
  const uint64_t base = tail & ~63ull;
  if (nt - base > out_cap) { set_err("out_cap too small for the batch"); return SRD_ERR_ARG; }
  HIPCHK(hipSetDevice(c->device));
  constexpr uint64_t CH = 64ull << 20;  // payload bytes per chunk (double-buffered in HBM)
  constexpr uint64_t KCH = 8ull << 20;  // key bytes per chunk
  constexpr uint64_t ENT_MAX = 1u << 16;
  if (!c->cstream) {
    HIPCHK(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
    for (int i = 0; i < 2; i++) {
      HIPCHK(hipEventCreateWithFlags(&c->wev_copied[i], hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&c->wev_done[i], hipEventDisableTiming));
      HIPCHK(hipHostMalloc(&c->pin_ent[i], ENT_MAX * sizeof(srd_write_entry), hipHostMallocDefault));
    }
  }
  TRY(ensure(c, B_WKH, n * 8));
  TRY(ensure(c, B_WMO, n * 8));
  uint64_t* kh_dev = P<uint64_t>(c, B_WKH);
  uint64_t* mo_dev = P<uint64_t>(c, B_WMO);
  uint64_t e0 = 0;
  for (int ci = 0; e0 < n; ci++) {
    // a chunk: consecutive entries whose payload and key source ranges stay
    // within CH / KCH (one entry at least); the ranges are copied as they lie
    uint64_t plo = E[e0].src, phi = E[e0].src + E[e0].len;
    uint64_t klo = E[e0].key_src, khi = klo + E[e0].key_len;
    uint64_t e1 = e0 + 1;
    while (e1 < n && e1 - e0 < ENT_MAX) {
      const uint64_t pl2 = std::min(plo, E[e1].src), ph2 = std::max(phi, E[e1].src + E[e1].len);
      const uint64_t kl2 = std::min(klo, E[e1].key_src), kh2 = std::max(khi, E[e1].key_src + E[e1].key_len);
      if (ph2 - (pl2 & ~15ull) > CH || kh2 - kl2 > KCH) break;
      plo = pl2; phi = ph2; klo = kl2; khi = kh2;
      e1++;
    }
    const uint64_t pa = plo & ~15ull;  // keeps every source's 16-byte alignment in the staging buffer
    const int slot = ci & 1;
    if (ci >= 2) HIPCHK(hipEventSynchronize(c->wev_done[slot]));  // chunk ci-2's kernel has released the slot
    TRY(ensure(c, (BufId)(B_WPAY0 + slot), phi - pa));
    TRY(ensure(c, (BufId)(B_WKEY0 + slot), std::max<uint64_t>(khi - klo, 1)));
    TRY(ensure(c, (BufId)(B_WENT0 + slot), ENT_MAX * sizeof(srd_write_entry)));
    srd_write_entry* pe = (srd_write_entry*)c->pin_ent[slot];
    for (uint64_t i = e0; i < e1; i++) {
      pe[i - e0] = E[i];
      pe[i - e0].src -= pa;
      pe[i - e0].key_src -= klo;
    }
    HIPCHK(hipMemcpyAsync(P<void>(c, (BufId)(B_WPAY0 + slot)), payloads + pa, phi - pa, hipMemcpyHostToDevice,
                          c->cstream));
    if (khi > klo)
      HIPCHK(hipMemcpyAsync(P<void>(c, (BufId)(B_WKEY0 + slot)), keys + klo, khi - klo, hipMemcpyHostToDevice,
                            c->cstream));
    HIPCHK(hipMemcpyAsync(P<void>(c, (BufId)(B_WENT0 + slot)), pe, (e1 - e0) * sizeof(srd_write_entry),
                          hipMemcpyHostToDevice, c->cstream));
    HIPCHK(hipEventRecord(c->wev_copied[slot], c->cstream));
    HIPCHK(hipStreamWaitEvent(c->stream, c->wev_copied[slot], 0));
    TRY(launch_write(c, c->stream, P<uint8_t>(c, (BufId)(B_WPAY0 + slot)), P<uint8_t>(c, (BufId)(B_WKEY0 + slot)),
                     P<srd_write_entry>(c, (BufId)(B_WENT0 + slot)), e1 - e0, d_out, base, kh_dev + e0, mo_dev + e0));
    HIPCHK(hipEventRecord(c->wev_done[slot], c->stream));
    e0 = e1;
  }
  if (kh_out) HIPCHK(hipMemcpyAsync(kh_out, kh_dev, n * 8, hipMemcpyDeviceToHost, c->stream));
  if (mo_out) HIPCHK(hipMemcpyAsync(mo_out, mo_dev, n * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(spin_sync(c->stream));
  return 0;
}

// ---------------------------------------------------------------------------
// Device KeyIndexer table + batched keyed reads (srd_index.hip)
static uint32_t table_log2cap(uint64_t table_bytes) {
  uint32_t l = 0;
  while (l < 62 && (16ull << (l + 1)) <= table_bytes) l++;
  return l;
}
extern "C" uint64_t srd_index_table_bytes(uint64_t n) {
  uint64_t cap = 64;
  while (cap < 2 * n) cap <<= 1;
  return 16 * cap;
}
static unsigned grid_for(uint64_t n) { return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, 8192)); }

extern "C" int srd_index_table_build_device(srd_ctx* c, const uint64_t* d_keys, const uint64_t* d_packed, uint64_t n,
                                            void* d_table, uint64_t table_bytes) {
  if (!c || !d_table || (n && (!d_keys || !d_packed)) || table_bytes < srd_index_table_bytes(n)) {
    set_err("bad argument (table_bytes < srd_index_table_bytes(n)?)");
    return SRD_ERR_ARG;
  }
  HIPCHK(hipSetDevice(c->device));
  const uint32_t l = table_log2cap(table_bytes);
  uint64_t* tk = (uint64_t*)d_table;
  uint64_t* tp = tk + (1ull << l);
  HIPCHK(hipMemsetAsync(tp, 0xFF, (1ull << l) * 8, c->stream));
  if (n) {
    idx_table_insert_kernel<<<grid_for(n), 256, 0, c->stream>>>(d_keys, d_packed, n, tk, (unsigned long long*)tp, l);
    KCHK(c, "idx_table_insert_kernel");
    HIPCHK(hipGetLastError());
  }
  HIPCHK(spin_sync(c->stream));
  return 0;
}

extern "C" int srd_index_get_packed_device(srd_ctx* c, const void* d_table, uint64_t table_bytes,
                                           const uint64_t* d_hashes, uint64_t n, uint64_t* d_packed_out,
                                           void* stream) {
  if (!c || !d_table || table_bytes < 16 * 64 || (n && (!d_hashes || !d_packed_out))) {
    set_err("bad argument");
    return SRD_ERR_ARG;
  }
  if (!n) return 0;
  HIPCHK(hipSetDevice(c->device));
  const uint32_t l = table_log2cap(table_bytes);
  const uint64_t* tk = (const uint64_t*)d_table;
  idx_get_packed_kernel<<<grid_for(n), 256, 0, stream ? (hipStream_t)stream : c->stream>>>(tk, tk + (1ull << l), l,
                                                                                             d_hashes, n, d_packed_out);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int srd_batch_read_hashed_device(srd_ctx* c, const void* d_table, uint64_t table_bytes,
                                            const uint8_t* d_file, uint64_t flen, const uint64_t* d_hashes,
                                            const uint64_t* d_verify, uint64_t n, uint64_t* d_start, uint64_t* d_end,
                                            void* stream) {
  if (!c || !d_table || table_bytes < 16 * 64 || (n && (!d_hashes || !d_start || !d_end || (flen && !d_file)))) {
    set_err("bad argument");
    return SRD_ERR_ARG;
  }
  if (!n) return 0;
  HIPCHK(hipSetDevice(c->device));
  const uint32_t l = table_log2cap(table_bytes);
  const uint64_t* tk = (const uint64_t*)d_table;
  batch_read_kernel<<<grid_for(n), 256, 0, stream ? (hipStream_t)stream : c->stream>>>(
      tk, tk + (1ull << l), l, d_file, flen, d_hashes, d_verify, n, d_start, d_end);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int srd_batch_read(srd_ctx* c, const void* d_table, uint64_t table_bytes, const uint8_t* d_file,
                              uint64_t flen, const uint8_t* keys, const uint64_t* key_offs, const uint64_t* key_lens,
                              uint64_t n, uint64_t* start_out, uint64_t* end_out) {
  if (!c || (n && (!keys || !key_offs || !key_lens || !start_out || !end_out))) {
    set_err("bad argument");
    return SRD_ERR_ARG;
  }
  if (!n) return 0;
  HIPCHK(hipSetDevice(c->device));
  uint64_t klen = 0;
  for (uint64_t i = 0; i < n; i++) klen = std::max(klen, key_offs[i] + key_lens[i]);
  void *dk = nullptr, *dof = nullptr, *dl = nullptr, *dh = nullptr, *ds = nullptr, *de = nullptr;
  int r = 0;
  auto cleanup = [&] { hipFree(dk); hipFree(dof); hipFree(dl); hipFree(dh); hipFree(ds); hipFree(de); };
  if (hipMalloc(&dk, klen + 1) || hipMalloc(&dof, n * 8) || hipMalloc(&dl, n * 8) || hipMalloc(&dh, n * 8) ||
      hipMalloc(&ds, n * 8) || hipMalloc(&de, n * 8)) {
    cleanup();
    set_err("hipMalloc failed");
    return SRD_ERR_ALLOC;
  }
  if (klen) HIPCHK(hipMemcpyAsync(dk, keys, klen, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(dof, key_offs, n * 8, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(dl, key_lens, n * 8, hipMemcpyHostToDevice, c->stream));
  r = srd_xxh3_64_batch_device(c, (const uint8_t*)dk, (const uint64_t*)dof, (const uint64_t*)dl, n, (uint64_t*)dh,
                               nullptr);  // compute_hash_batch (data_store.rs:1112)
  // batch_read verifies every key by its own tag (Some(keys), :1113)
  if (!r) r = srd_batch_read_hashed_device(c, d_table, table_bytes, d_file, flen, (const uint64_t*)dh,
                                           (const uint64_t*)dh, n, (uint64_t*)ds, (uint64_t*)de, nullptr);
  if (!r) {
    HIPCHK(hipMemcpyAsync(start_out, ds, n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(end_out, de, n * 8, hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(spin_sync(c->stream));
  cleanup();
  return r;
}

// ---------------------------------------------------------------------------
// par_iter_entries / EntryIterator, estimate_compaction_savings and compact
// over the device index (srd_index.hip iter_* kernels + the writer)
static int iter_run(Ctx* c, const uint8_t* d_file, uint64_t flen, const uint64_t* d_packed, uint64_t n,
                    uint64_t* d_start, uint64_t* d_end, uint64_t* d_meta, uint64_t* d_kh, uint64_t* n_out,
                    uint64_t* kept_bytes) {
  *n_out = 0;
  if (kept_bytes) *kept_bytes = 0;
  if (!n) return 0;
  HIPCHK(hipSetDevice(c->device));
  TRY(ensure(c, B_IT_FLAG, n * 4));
  TRY(ensure(c, B_IT_POS, n * 4));
  TRY(ensure(c, B_IT_ST, n * 8));
  TRY(ensure(c, B_IT_EN, n * 8));
  TRY(ensure(c, B_IT_KEPT, 64));
  TRY(ensure_cub(c, n));
  uint32_t* flag = P<uint32_t>(c, B_IT_FLAG);
  uint32_t* pos = P<uint32_t>(c, B_IT_POS);
  unsigned long long* kept = P<unsigned long long>(c, B_IT_KEPT);
  HIPCHK(hipMemsetAsync(kept, 0, 8, c->stream));
  iter_flag_kernel<<<grid_for(n), 256, 0, c->stream>>>(d_file, flen, d_packed, n, flag, P<uint64_t>(c, B_IT_ST),
                                                       P<uint64_t>(c, B_IT_EN), kept);
  KCHK(c, "iter_flag_kernel");
  size_t tb = c->bufs[B_CUB_TMP].n;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(P<void>(c, B_CUB_TMP), tb, flag, pos, (int)n, c->stream));
  KCHK(c, "hipcub");
  uint32_t last[2] = {0, 0};
  unsigned long long hk = 0;
  HIPCHK(hipMemcpyAsync(&last[0], pos + n - 1, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(&last[1], flag + n - 1, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(&hk, kept, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(spin_sync(c->stream));
  const uint64_t nv = (uint64_t)last[0] + last[1];
  if (d_start && nv) {
    iter_emit_kernel<<<grid_for(n), 256, 0, c->stream>>>(d_file, d_packed, flag, pos, n, nv, P<uint64_t>(c, B_IT_ST),
                                                         P<uint64_t>(c, B_IT_EN), d_start, d_end, d_meta, d_kh);
    KCHK(c, "iter_emit_kernel");
    HIPCHK(hipGetLastError());
    HIPCHK(spin_sync(c->stream));
  }
  *n_out = nv;
  if (kept_bytes) *kept_bytes = hk;
  return 0;
}

extern "C" int srd_iter_entries_device(srd_ctx* c, const uint8_t* d_file, uint64_t flen, const uint64_t* d_packed,
                                       uint64_t n_index, uint64_t* d_start, uint64_t* d_end, uint64_t* d_meta_off,
                                       uint64_t* d_key_hash, uint64_t* n_out) {
  if (!c || !n_out || (n_index && (!d_file || !d_packed || !d_start || !d_end))) {
    set_err("bad argument");
    return SRD_ERR_ARG;
  }
  return iter_run(c, d_file, flen, d_packed, n_index, d_start, d_end, d_meta_off, d_key_hash, n_out, nullptr);
}

extern "C" int srd_estimate_compaction_savings_device(srd_ctx* c, const uint8_t* d_file, uint64_t flen,
                                                      const uint64_t* d_packed, uint64_t n_index, uint64_t* savings) {
  if (!c || !savings || (n_index && (!d_file || !d_packed))) { set_err("bad argument"); return SRD_ERR_ARG; }
  uint64_t nv = 0, kept = 0;
  TRY(iter_run(c, d_file, flen, d_packed, n_index, nullptr, nullptr, nullptr, nullptr, &nv, &kept));
  *savings = flen > kept ? flen - kept : 0;  // total_size.saturating_sub(unique_entry_size)
  return 0;
}

extern "C" int srd_compact_device(srd_ctx* c, const uint8_t* d_file, uint64_t flen, const uint64_t* d_packed,
                                  uint64_t n_index, uint8_t* d_out, uint64_t out_cap, uint64_t* new_len,
                                  uint64_t* d_key_hash_out, uint64_t* d_meta_off_out) {
  if (!c || !new_len || (n_index && (!d_file || !d_packed))) { set_err("bad argument"); return SRD_ERR_ARG; }
  *new_len = 0;
  if (!n_index) return 0;
  TRY(ensure(c, B_IT_OST, n_index * 8));
  TRY(ensure(c, B_IT_OEN, n_index * 8));
  TRY(ensure(c, B_IT_OKH, n_index * 8));
  uint64_t nv = 0;
  TRY(iter_run(c, d_file, flen, d_packed, n_index, P<uint64_t>(c, B_IT_OST), P<uint64_t>(c, B_IT_OEN), nullptr,
               P<uint64_t>(c, B_IT_OKH), &nv, nullptr));
  // layout of the compacted file on the device: write_stream_with_key_hash
  // per entry in iter_entries order (data_store.rs:706-719, 758-825), tail
  // from 0 -- a prefix sum (compact_sizes_kernel), then the write entries
  if (!nv) return 0;
  const uint64_t* st = P<uint64_t>(c, B_IT_OST);
  const uint64_t* en = P<uint64_t>(c, B_IT_OEN);
  TRY(ensure(c, B_IT_RLEN, nv * 8));
  TRY(ensure(c, B_IT_PST, nv * 8));
  TRY(ensure(c, B_IT_ENT, nv * sizeof(srd_write_entry)));
  TRY(ensure(c, B_IT_KEPT, 64));
  size_t tb = 0;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (uint64_t*)nullptr, (uint64_t*)nullptr, (int)nv));
  KCHK(c, "hipcub");
  TRY(ensure(c, B_CUB_TMP, tb + 256));
  tb = c->bufs[B_CUB_TMP].n;
  compact_sizes_kernel<<<grid_for(nv), 256, 0, c->stream>>>(st, en, nv, P<uint64_t>(c, B_IT_RLEN));
  KCHK(c, "compact_sizes_kernel");
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(P<void>(c, B_CUB_TMP), tb, P<uint64_t>(c, B_IT_RLEN),
                                          P<uint64_t>(c, B_IT_PST), (int)nv, c->stream));
  KCHK(c, "hipcub");
  uint64_t* d_new_len = P<uint64_t>(c, B_IT_KEPT) + 2;
  compact_entries_kernel<<<grid_for(nv), 256, 0, c->stream>>>(st, en, P<uint64_t>(c, B_IT_OKH), P<uint64_t>(c, B_IT_PST),
                                                             nv, P<srd_write_entry>(c, B_IT_ENT), d_new_len);
  KCHK(c, "compact_entries_kernel");
  HIPCHK(hipGetLastError());
  uint64_t tail = 0;
  HIPCHK(hipMemcpyAsync(&tail, d_new_len, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(spin_sync(c->stream));
  *new_len = tail;
  if (!d_out) return 0;
  if (tail > out_cap) { set_err("out_cap too small for the compacted store"); return SRD_ERR_ARG; }
  TRY(ensure(c, B_WKH, nv * 8));
  TRY(ensure(c, B_WMO, nv * 8));
  unsigned int* nullf = (unsigned int*)(P<uint8_t>(c, B_IT_KEPT) + 8);
  HIPCHK(hipMemsetAsync(nullf, 0, 4, c->stream));
  TRY(launch_write(c, c->stream, d_file, nullptr, P<srd_write_entry>(c, B_IT_ENT), nv, d_out, 0,
                   d_key_hash_out ? d_key_hash_out : P<uint64_t>(c, B_WKH),
                   d_meta_off_out ? d_meta_off_out : P<uint64_t>(c, B_WMO), nullf));
  unsigned int hn = 0;
  HIPCHK(hipMemcpyAsync(&hn, nullf, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(spin_sync(c->stream));
  if (hn) {  // write_stream rejects NULL-only payloads (data_store.rs:792-797); compact() fails with it
    set_err("NULL-byte-only streams cannot be written directly.");
    return SRD_ERR_ARG;
  }
  return 0;
}

#ifdef SRD_GLUE_STAMPS
// timing-only build: the last fused chain_finalize's per-block phase stamps
extern "C" int srd_debug_glue_stamps(uint64_t* out) {
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_glue_stamp), sizeof(uint64_t) * CHAIN_BLOCKS * 8));
  return 0;
}
#endif
#ifdef SRD_WAVE_STAMPS
// timing-only build: the last scan's per-wave end stamps and per-block start
// stamps (s_memrealtime, 100 MHz)
extern "C" int srd_debug_wave_stamps(uint64_t* out) {
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_stamp), sizeof(uint64_t) * (8192 + 1024)));
  return 0;
}
// and the shader-clock counter (s_memtime) at the same wave ends / block starts
extern "C" int srd_debug_wave_clk(uint64_t* out) {
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_clk), sizeof(uint64_t) * (4096 + 256)));
  return 0;
}
#endif

// host self-test of the CRC algebra (no GPU): checks the tables against a
// byte-wise CRC on pseudo-random data with the same combine the kernels use.
extern "C" int srd_selftest_host(void) {
  std::call_once(g_tab_once, [] { build_crc_tables(g_host_tabs); });
  const CrcTables& t = g_host_tabs;
  static uint8_t buf[5 * 4096];
  memset(buf, 0, sizeof buf);
  uint64_t z = 12345;
  for (int i = 0; i < 3 * 4096 + 200; i++) { auto& b = buf[i]; z = z * 6364136223846793005ull + 1442695040888963407ull; b = (uint8_t)(z >> 56); }
  // x^-8 * x^8 == 1
  if (mulp(t.invpow[1], t.pow8[0]) != kX0) return 1;
  // check crc_from_pieces-style assembly for several (s, m)
  auto raw = [&](uint64_t a, uint64_t b) { return host_crc_raw_bytes(t, 0, buf + a, b - a); };
  auto crc32 = [&](uint64_t a, uint64_t b) { return ~host_crc_raw_bytes(t, ~0u, buf + a, b - a); };
  auto sx = [&](uint64_t k, uint32_t j) {  // crc_raw(lines j..63 of tile k)
    return raw(k * 4096 + 64 * j, k * 4096 + 4096);
  };
  const uint64_t cases[][2] = {{0, 100}, {64, 4096}, {128, 5000}, {4096, 8192 + 77}, {192, 12288 + 3}, {0, 63}};
  for (auto& cs : cases) {
    uint64_t s = cs[0], m = cs[1];
    uint64_t len = m - s;
    uint32_t want = crc32(s, m);
    uint32_t tail = raw(m & ~63ull, m);
    uint32_t got;
    if (len < 64) {
      got = tail ^ t.zero_crc[len];
    } else {
      uint64_t k0 = s / 4096, k1 = m / 4096;
      uint32_t acc = sx(k0, (uint32_t)((s % 4096) / 64)) ^ t.winit[(s % 4096) / 64];
      uint32_t sxm = sx(k1, (uint32_t)((m % 4096) / 64));
      uint32_t y;
      if (k0 == k1) y = acc ^ sxm;
      else {
        for (uint64_t k = k0 + 1; k < k1; k++) acc = mulp(t.x32768, acc) ^ sx(k, 0);
        y = mulp(t.x32768, acc) ^ sx(k1, 0) ^ sxm;
      }
      got = ~(mulp(t.invpow[(k1 + 1) * 4096 - m], y) ^ tail);
    }
    if (got != want) return 2;
  }
  return 0;
}
