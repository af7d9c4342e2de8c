// C-ABI host layer of the MI355X batch key-hashing stage (include/shf_hash_batch.h).
//
// Replaces, for batches, the per-key seam shf_make_hash() (/root/reference/src/shf.c:450-462):
// same 16 output bytes per key (SHF_HASH layout, shf.private.h:180-185), computed by the
// kernels in kernels.hip. This file owns: argument checking, per-thread/per-device HIP
// contexts (streams + staging buffers), the host-memory pipeline (pinned chunks, H2D /
// kernel / D2H overlapped on one stream per chunk in flight) and the multi-GPU split.
// There is deliberately no CPU path: without a gfx950 device every call fails loudly.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>


#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/shf_hash_batch.h"
#include "kernels.h"
#include "host_plan.h"

// Row index: device copies of a store's tab map and rows (shf_hash_batch.h).
struct shf_row_index {
  int dev = -1;
  uint32_t* d_tab_slot = nullptr;
  uint8_t* d_rows = nullptr;
  uint64_t n_slots = 0;
  // the probes' compact copy of tab_slot (kernels.h launch_compact_map), made by set_tabs;
  // not used once the device pointers were handed out (tab_slot may then change under it)
  uint8_t* d_map8 = nullptr;
  uint32_t* d_win_tab = nullptr;
  bool compact = false;
  mutable bool external = false;
};

namespace {

thread_local int tls_last_hip = 0;

int map_hip(hipError_t e) {
  if (e == hipSuccess) return SHF_HB_OK;
  tls_last_hip = (int)e;
  switch (e) {
    case hipErrorOutOfMemory:
      return SHF_HB_ERR_NOMEM;
    case hipErrorNoDevice:
    case hipErrorInsufficientDriver:
    case hipErrorInvalidDevice:
      return SHF_HB_ERR_NODEV;
    case hipErrorNoBinaryForGpu:
      return SHF_HB_ERR_ARCH;
    default:
      return SHF_HB_ERR_HIP;
  }
}

// SHF_HB_DEBUG=1 (read once): every failing HIP call is named on stderr.
bool debug_errors() {
  static const bool on = [] {
    const char* e = getenv("SHF_HB_DEBUG");
    return e && e[0] == '1';
  }();
  return on;
}

#define HB_TRY(expr)                                                                                  \
  do {                                                                                                \
    hipError_t e_ = (expr);                                                                           \
    if (e_ != hipSuccess) {                                                                           \
      if (debug_errors())                                                                             \
        fprintf(stderr, "shf_hash_batch: %s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #expr, (int)e_, \
                hipGetErrorString(e_));                                                               \
      return map_hip(e_);                                                                             \
    }                                                                                                 \
  } while (0)

constexpr uint32_t kMaxKeyLen = 0x7fffffffu;      // murmurhash3.c:75 takes `const int len`
// Shape of the host-memory pipelines. Every process stages through one pool of
// slots per device (host_plan.h SlotPool), shared by all calling threads: a
// slot is a pinned host arena and a device arena of SHF_HB_STAGE_MB MiB each
// (default 16) with its own stream, and the pool holds at most SHF_HB_POOL_MB
// MiB of them (default 64, i.e. 64 MiB of device and 64 MiB of pinned memory
// per device, whatever the number of threads). A call borrows up to
// SHF_HB_SLOTS (1..4, default 4) slots, no more than its batch has chunks, and
// beyond the first only while no other call waits; one chunk in flight on
// each. All three are read on every call. A 16-MiB slot carries 512 Ki 16-B keys with their
// records (the 8 MiB x 4 chunks of round 4: 10M x 16 B pageable 2.04, page-
// locked staged 2.19 G keys/s; profiles/r4/stage_sweep/), or ~15 MiB of
// variable-length keys with their offsets and records.
constexpr int kMaxSlots = 4;
constexpr long kDefaultStageMb = 16, kDefaultPoolMb = 64;

size_t stage_bytes() {
  const char* e = getenv("SHF_HB_STAGE_MB");
  const long mb = e ? strtol(e, nullptr, 10) : 0;
  return (size_t)(mb >= 1 && mb <= 4096 ? mb : kDefaultStageMb) << 20;
}

size_t pool_bytes() {
  const char* e = getenv("SHF_HB_POOL_MB");
  const long mb = e ? strtol(e, nullptr, 10) : 0;
  return (size_t)(mb >= 1 && mb <= (1L << 20) ? mb : kDefaultPoolMb) << 20;
}

int pipeline_slots() {
  const char* e = getenv("SHF_HB_SLOTS");
  const long v = e ? strtol(e, nullptr, 10) : 0;
  return v >= 1 && v <= kMaxSlots ? (int)v : kMaxSlots;
}

shfhb::Sink out_sink(void* out) {
  shfhb::Sink k;
  k.out = out;
  return k;
}

// One staging slot of a device's pool: chunks are carved out of the arenas by
// host_plan.h slot_layout (keys, hash records, probe records, offsets).
struct Slot {
  int dev = -1;
  size_t bytes = 0;
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr;
  uint8_t* h = nullptr;      // pinned host arena
  uint8_t* h_dev = nullptr;  // its device address (kernels store records there over PCIe), or null
  uint8_t* d = nullptr;      // device arena
};

void unmake_slot(Slot* s) {
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(s->dev);
  if (s->st) (void)hipStreamSynchronize(s->st);
  if (s->h) (void)hipHostFree(s->h);
  if (s->d) (void)hipFree(s->d);
  if (s->done) (void)hipEventDestroy(s->done);
  if (s->st) (void)hipStreamDestroy(s->st);
  (void)hipGetLastError();
  (void)hipSetDevice(prev);
  delete s;
}

int make_slot(int dev, size_t bytes, Slot** out) {
  Slot* s = new Slot();
  s->dev = dev;
  s->bytes = bytes;
  int prev = 0;
  (void)hipGetDevice(&prev);
  hipError_t e = hipSetDevice(dev);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&s->done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipHostMalloc((void**)&s->h, bytes, hipHostMallocDefault);
  if (e == hipSuccess) e = hipMalloc((void**)&s->d, bytes);
  if (e == hipSuccess && hipHostGetDevicePointer((void**)&s->h_dev, s->h, 0) != hipSuccess) {
    (void)hipGetLastError();
    s->h_dev = nullptr;
  }
  (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    const int rc = map_hip(e);
    unmake_slot(s);
    return rc;
  }
  *out = s;
  return SHF_HB_OK;
}

using Pool = shfhb::plan::SlotPool<Slot>;

// The process's pools, one per device, made on first use and kept for the
// process's life (shf_hash_batch_release() frees their idle slots).
std::mutex g_pools_mu;
std::map<int, Pool*> g_pools;

Pool* device_pool(int dev) {
  std::lock_guard<std::mutex> g(g_pools_mu);
  Pool*& p = g_pools[dev];
  if (!p)
    p = new Pool([dev](size_t bytes, Slot** out) { return make_slot(dev, bytes, out); },
                 [](Slot* s) { unmake_slot(s); });
  return p;
}

// The slots one call borrows; given back (after their streams are idle) when it ends.
struct Lease {
  Pool* pool = nullptr;
  Slot* s[kMaxSlots] = {};
  int n = 0;
  Lease() = default;
  Lease(const Lease&) = delete;
  Lease& operator=(const Lease&) = delete;
  ~Lease() {
    if (!n) return;
    for (int i = 0; i < n; ++i) (void)hipStreamSynchronize(s[i]->st);  // on every path, errors included
    (void)hipGetLastError();
    pool->release(s, n);
  }
};

int lease_slots(int dev, int want, Lease* L) {
  const size_t bytes = std::max(stage_bytes(), shfhb::plan::kMinSlotBytes);
  const int max_slots = (int)std::max<size_t>(1, std::min<size_t>(64, pool_bytes() / bytes));
  L->pool = device_pool(dev);
  return L->pool->acquire(bytes, std::min(std::max(want, 1), kMaxSlots), max_slots, L->s, &L->n);
}

// Per (thread, device) state, made lazily and kept across calls: one stream for
// launches that stage nothing, the variable-length status words and the
// window-order buffers. No staging: that is the process pool's.
struct DevCtx {
  int dev = -1;
  int status = SHF_HB_OK;
  hipStream_t st = nullptr;
  // Variable-length key checks done by the kernels (kernels.h Sink::status):
  // word 0 collects this thread's async calls until shf_hash_batch_status()
  // takes it (word 2 receives the taken value), word 1 is cleared and read by
  // each synchronous call.
  uint32_t* d_status = nullptr;
  uint32_t* h_status = nullptr;  // pinned, 1 word
  void* d_win_ws = nullptr;      // shf_win_order's workspace, kept across calls (grows only)
  size_t win_ws_cap = 0;
  uint32_t* d_perm = nullptr;    // host-memory window orders: the order on the device (+ 257 starts)
  size_t perm_cap = 0;
};

void release_ctx(DevCtx* c);

// Contexts of threads that have exited, per device, kept for the next thread
// that needs one: a thread's exit makes no HIP call (the runtime's own
// per-thread state may already be gone by then, and freeing pinned memory from
// a thread-exit handler is the one pattern this library does not trust), and
// short-lived threads reuse a few contexts instead of making and freeing their
// own. shf_hash_batch_release() frees the idle ones.
std::mutex g_ctx_mu;
std::map<int, std::vector<DevCtx*>> g_ctx_idle;

void park_ctx(DevCtx* c) {
  std::lock_guard<std::mutex> g(g_ctx_mu);
  g_ctx_idle[c->dev].push_back(c);
}

// The calling thread's contexts, one per device; parked for reuse when it exits.
struct ThreadCtxs {
  std::map<int, DevCtx*> m;
  ~ThreadCtxs();
};
thread_local ThreadCtxs tls_ctx;

int check_arch(int dev) {
  hipDeviceProp_t p;
  HB_TRY(hipGetDeviceProperties(&p, dev));
  if (strncmp(p.gcnArchName, "gfx950", 6) != 0) return SHF_HB_ERR_ARCH;
  return SHF_HB_OK;
}

int current_ctx(DevCtx** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return map_hip(e) == SHF_HB_ERR_HIP ? SHF_HB_ERR_NODEV : map_hip(e);
  }
  auto it = tls_ctx.m.find(dev);
  if (it != tls_ctx.m.end()) {
    *out = it->second;
    return it->second->status;
  }
  DevCtx* c = nullptr;
  {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    auto& idle = g_ctx_idle[dev];
    if (!idle.empty()) {
      c = idle.back();
      idle.pop_back();
    }
  }
  if (c) {  // an exited thread's context: its work is done once its stream is idle; fresh status words
    if (c->status == SHF_HB_OK) {  // (a context that failed to start keeps its error)
      (void)hipStreamSynchronize(c->st);
      c->status = map_hip(hipMemset(c->d_status, 0, 3 * sizeof(uint32_t)));
    }
  } else {
    c = new DevCtx();
    c->dev = dev;
    c->status = check_arch(dev);
    if (c->status == SHF_HB_OK) c->status = map_hip(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    if (c->status == SHF_HB_OK) c->status = map_hip(hipMalloc((void**)&c->d_status, 3 * sizeof(uint32_t)));
    if (c->status == SHF_HB_OK) c->status = map_hip(hipMemset(c->d_status, 0, 3 * sizeof(uint32_t)));
    if (c->status == SHF_HB_OK)
      c->status = map_hip(hipHostMalloc((void**)&c->h_status, sizeof(uint32_t), hipHostMallocDefault));
  }
  tls_ctx.m[dev] = c;
  *out = c;
  return c->status;
}

void release_ctx(DevCtx* c) {
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(c->dev);
  if (c->st) (void)hipStreamSynchronize(c->st);
  if (c->st) (void)hipStreamDestroy(c->st);
  if (c->d_status) (void)hipFree(c->d_status);
  if (c->h_status) (void)hipHostFree(c->h_status);
  if (c->d_win_ws) (void)hipFree(c->d_win_ws);
  if (c->d_perm) (void)hipFree(c->d_perm);
  (void)hipGetLastError();
  (void)hipSetDevice(prev);
  delete c;
}

// Hand this thread's contexts back now (the *_multi workers before they report
// back); they are parked for the next thread, as at thread exit.
void release_thread_ctx() {
  for (auto& kv : tls_ctx.m) park_ctx(kv.second);
  tls_ctx.m.clear();
}

// Frees this thread's contexts and every parked one (shf_hash_batch_release()).
void free_contexts() {
  release_thread_ctx();
  std::vector<DevCtx*> all;
  {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    for (auto& kv : g_ctx_idle) {
      all.insert(all.end(), kv.second.begin(), kv.second.end());
      kv.second.clear();
    }
  }
  for (DevCtx* c : all) release_ctx(c);
}

// shf_win_order's workspace: grown when a batch needs more, else reused (a hipFree per call
// would synchronise the device every batch). The context's stream and the null stream are idle first.
int ensure_win_ws(DevCtx* c, size_t bytes, void** out) {
  if (bytes > c->win_ws_cap) {
    HB_TRY(hipStreamSynchronize(c->st));
    HB_TRY(hipStreamSynchronize(nullptr));
    if (c->d_win_ws) (void)hipFree(c->d_win_ws);
    c->d_win_ws = nullptr;
    c->win_ws_cap = 0;
    HB_TRY(hipMalloc(&c->d_win_ws, bytes));
    c->win_ws_cap = bytes;
  }
  *out = c->d_win_ws;
  return SHF_HB_OK;
}

// Device room for a host-memory window order: n indices then 257 window starts (grows only;
// this is the only function that frees or replaces d_perm).
int ensure_perm(DevCtx* c, uint64_t n, uint32_t** out) {
  const size_t need = ((size_t)n + 257u) * sizeof(uint32_t);
  if (need > c->perm_cap) {
    HB_TRY(hipStreamSynchronize(c->st));
    if (c->d_perm) (void)hipFree(c->d_perm);
    c->d_perm = nullptr;
    c->perm_cap = 0;
    HB_TRY(hipMalloc((void**)&c->d_perm, need));
    c->perm_cap = need;
  }
  *out = c->d_perm;
  return SHF_HB_OK;
}

// Caller host memory that is already page-locked (hipHostMalloc /
// hipHostRegister by the caller): DMA straight from / into it, no staging copy.
bool is_host_pinned(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: clear the sticky error
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// memcpy split over a few threads (SHF_HB_COPY_THREADS, default 12, read per
// call): one core cannot keep up with PCIe. 10M x 16-B pageable keys with
// streaming stores, G keys/s per repeat (profiles/r5/pool_sweep/): 12 threads
// 2.1-2.27 on both passes, 8 threads 1.5-1.9 on one and 2.35-2.4 on the other,
// 16 threads 1.7-2.1; memcpy instead of streaming stores 1.5-1.96.
size_t copy_threads() {
  const char* e = getenv("SHF_HB_COPY_THREADS");
  const long v = e ? strtol(e, nullptr, 10) : 0;
  return v >= 1 && v <= 64 ? (size_t)v : 12;
}

// Staging-copy workers shared by every calling thread (host_plan.h CopyPool):
// started on first use (up to SHF_HB_COPY_THREADS - 1), never per chunk; a
// worker that finds no piece for 10 s ends, and the next batch starts workers
// again. The pool object itself is deliberately never destroyed (a worker may
// still be returning from it at process exit).
using shfhb::plan::CopyPool;
using shfhb::plan::Ticket;

std::atomic<CopyPool*> g_copy_pool{nullptr};

CopyPool& copy_pool() {
  static CopyPool* p = [] {
    CopyPool* q = new CopyPool();
    g_copy_pool.store(q);
    return q;
  }();
  return *p;
}

// fork() (include/shf_hash_batch.h, "fork"): the HIP runtime's device state,
// streams, pinned memory and this library's staging pools and copy workers do
// not survive into a child. A child forked after this process used the library
// gets SHF_HB_ERR_FORKED from every entry point, before any HIP call (instead
// of undefined behaviour in the runtime or a wait on copy workers the child does
// not have); the copy pool's own handlers (host_plan.h CopyPool) keep its queue
// consistent across the fork. A child forked before any use is a fresh process
// for the library. The reference's own load test forks its workers
// (/root/reference/src/test.f.shf.c:274-336): fork them first, then hash.
std::atomic<bool> g_used{false}, g_forked{false};
CopyPool* g_fork_locked = nullptr;  // the pool fork_prepare locked (only the forking thread touches it)

void atfork_prepare() {
  g_fork_locked = g_copy_pool.load();
  if (g_fork_locked) g_fork_locked->fork_prepare();
}
void atfork_parent() {
  if (g_fork_locked) g_fork_locked->fork_parent();
  g_fork_locked = nullptr;
}
void atfork_child() {
  if (g_used.load(std::memory_order_relaxed)) g_forked.store(true, std::memory_order_relaxed);
  if (g_fork_locked) g_fork_locked->fork_child();
  g_fork_locked = nullptr;
}
[[maybe_unused]] const int g_atfork_registered = pthread_atfork(atfork_prepare, atfork_parent, atfork_child);

// First statement of every entry point that may reach HIP.
inline int enter() {
  if (g_forked.load(std::memory_order_relaxed)) return SHF_HB_ERR_FORKED;
  if (!g_used.load(std::memory_order_relaxed)) g_used.store(true, std::memory_order_relaxed);
  return SHF_HB_OK;
}
#define HB_ENTER()                       \
  do {                                   \
    const int entered_ = enter();        \
    if (entered_ != SHF_HB_OK) return entered_; \
  } while (0)

// A thread's exit parks its contexts for reuse -- except in a forked child,
// where they are the parent's (and the lock that guards the parked ones may
// have been held by a thread the child does not have).
ThreadCtxs::~ThreadCtxs() {
  if (g_forked.load(std::memory_order_relaxed)) return;
  for (auto& kv : m) park_ctx(kv.second);
  m.clear();
}

// Staging copies with non-temporal stores: the destination of every staging
// copy is written once and not read back by this core soon (pinned staging the
// device reads by DMA, or the caller's records), so streaming stores skip the
// read-for-ownership a cached store pays and leave the caches to the caller.
// SHF_HB_COPY_NT=0 (read per call) uses memcpy throughout.
bool copy_nt() {
  const char* e = getenv("SHF_HB_COPY_NT");
  static const bool avx2 = __builtin_cpu_supports("avx2");  // (the runtime's constructor filled the CPU model in)
  return avx2 && !(e && e[0] == '0');
}

void copy_piece(void* dst, const void* src, size_t n, bool nt) {
  if (nt && n >= 4096)
    shfhb::plan::stream_copy_avx2(dst, src, n);
  else
    memcpy(dst, src, n);
}

void par_memcpy(void* dst, const void* src, size_t n) {
  constexpr size_t kMinPerThread = (size_t)2 << 20;
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const size_t t = std::min<size_t>({copy_threads(), (size_t)hw, std::max<size_t>(1, n / kMinPerThread)});
  const bool nt = copy_nt();
  if (t <= 1) {
    copy_piece(dst, src, n, nt);
    return;
  }
  const size_t per = (n + t - 1) / t;
  std::vector<std::function<void()>> pieces;
  for (size_t i = 0; i < t; ++i) {
    const size_t a = i * per, b = std::min(n, a + per);
    if (a < b) pieces.emplace_back([=] { copy_piece((char*)dst + a, (const char*)src + a, b - a, nt); });
  }
  copy_pool().run(pieces);
}

// What a host pipeline writes: hash records (16-B SHF_HASH, or 8-B UID parts)
// and/or row pre-probe records.
struct HostJob {
  void* hash = nullptr;      // the caller's records, rec() bytes per key
  void* hash_dev = nullptr;  // device address of `hash` (page-locked): the kernel stores there
  bool uid = false;          // 8-B UID parts (kOutUid: the bits shf.c:800-803 reads) instead of 16-B records
  bool stage_direct = false;  // else (pageable `hash`): the kernel stores into the slot's pinned staging
  shf_probe* probe = nullptr;
  const shf_row_index* index = nullptr;  // with probe
  uint8_t* wins = nullptr;  // device: the batch's window bytes (kOutHashWin / kOutUidWin), key i's at wins[i]
  size_t rec() const { return uid ? sizeof(uint64_t) : sizeof(shf_hash128); }
  uint8_t* at(void* p, uint64_t i) const { return static_cast<uint8_t*>(p) + i * rec(); }
  int hash_mode() const { return uid ? shfhb::kOutUid : shfhb::kOutHash; }
};

// One chunk in flight per slot; where its results go once the slot's event fires.
struct Pending {
  bool busy = false;
  void* hash = nullptr;            // nullptr: not requested, or DMA'd / stored straight to the caller
  const void* hash_src = nullptr;  // the slot's pinned records to copy from
  size_t rec = sizeof(shf_hash128);  // bytes per record
  shf_probe* probe = nullptr;
  const shf_probe* probe_src = nullptr;
  uint64_t count = 0;
  std::shared_ptr<Ticket> copy_out;  // the copy-out running on the copy workers (drain_async)
  Pending() = default;
  Pending(const Pending&) = delete;
  Pending& operator=(const Pending&) = delete;
  ~Pending() {
    if (copy_out) (void)copy_out->wait();  // on every path: the slot goes back to the pool only after it
  }
  // For the slot's next chunk (drain_slot has run: a copy-out still going is waited for, never dropped).
  void reset() {
    if (copy_out) (void)copy_out->wait();
    busy = false;
    hash = nullptr;
    hash_src = nullptr;
    probe = nullptr;
    probe_src = nullptr;
    count = 0;
    copy_out.reset();
  }
};

// SHF_HB_TRACE=1 (read once): each host-pipeline call prints one line on
// stderr with where its time went -- staging copies in, waits for the device,
// copies out -- so a slow call can be told apart (tools/diag_pageable_staged.py).
bool trace_on() {
  static const bool on = [] {
    const char* e = getenv("SHF_HB_TRACE");
    return e && e[0] == '1';
  }();
  return on;
}

struct PipeTrace {
  double copy_in = 0, wait = 0, copy_out = 0, enqueue = 0;
  uint64_t chunks = 0;
  int slots = 0;
};
thread_local PipeTrace tls_trace;

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int drain_slot(Slot* s, Pending& p) {
  if (!p.busy) return SHF_HB_OK;
  if (p.copy_out) {  // handed to the workers by drain_async: wait for them
    const double t0 = trace_on() ? now_ms() : 0;
    const int rc = p.copy_out->wait();
    if (trace_on()) tls_trace.wait += now_ms() - t0;
    p.copy_out.reset();
    p.busy = false;
    return rc;
  }
  const bool tr = trace_on();
  const double t0 = tr ? now_ms() : 0;
  HB_TRY(hipEventSynchronize(s->done));
  const double t1 = tr ? now_ms() : 0;
  if (p.hash) par_memcpy(p.hash, p.hash_src, p.count * p.rec);
  if (p.probe) par_memcpy(p.probe, p.probe_src, p.count * sizeof(shf_probe));
  if (tr) {
    tls_trace.wait += t1 - t0;
    tls_trace.copy_out += now_ms() - t1;
  }
  p.busy = false;
  return SHF_HB_OK;
}

// drain_slot's work handed to the copy workers, the caller going on at once: each
// piece waits for the slot's event, then copies its part of the records out.
// Used where the caller spends the chunk's time inside a blocking copy of its
// own (the runtime's pageable H2D), so the copy-out runs beside it.
// At most four pieces per copy-out: beside the runtime's pageable H2D, 4-6 copy threads
// gave 2.39-2.40 G keys/s on 10M x 16-B keys in both rounds of an alternating sweep, 8-16
// threads 2.24-2.40 and 2 threads 2.18-2.38 (more threads take host memory bandwidth from
// the runtime's own copy; profiles/r5/runtime_copy/threads_sweep.txt).
void drain_async(Slot* s, Pending& p) {
  if (!p.busy || p.copy_out || (!p.hash && !p.probe)) return;
  constexpr size_t kMinPiece = (size_t)2 << 20, kMaxPieces = 4;
  std::vector<std::function<int()>> pieces;
  const bool nt = copy_nt();
  auto split = [&](void* dst, const void* src, size_t n) {
    const size_t k = std::min<size_t>({copy_threads(), kMaxPieces, std::max<size_t>(1, n / kMinPiece)}),
                 per = (n + k - 1) / k;
    for (size_t a = 0; a < n; a += per) {
      const size_t b = std::min(n, a + per);
      hipEvent_t ev = s->done;
      pieces.emplace_back([=] {
        const hipError_t e = hipEventSynchronize(ev);
        if (e != hipSuccess) return map_hip(e);
        copy_piece((char*)dst + a, (const char*)src + a, b - a, nt);
        return (int)SHF_HB_OK;
      });
    }
  };
  if (p.hash) split(p.hash, p.hash_src, p.count * p.rec);
  if (p.probe) split(p.probe, p.probe_src, p.count * sizeof(shf_probe));
  p.copy_out = copy_pool().submit(std::move(pieces));
}

int drain_all(Lease& L, Pending* pend) {
  for (int q = 0; q < L.n; ++q) {
    const int rc = drain_slot(L.s[q], pend[q]);
    if (rc) return rc;
  }
  return SHF_HB_OK;
}

// One chunk's buffers inside a slot (host_plan.h slot_layout).
struct ChunkBufs {
  uint8_t *h_in, *d_in;
  uint8_t *h_out, *d_out, *hd_out;  // the chunk's records; hd_out: device address of h_out, or null
  shf_probe *h_probe, *d_probe;
  uint64_t *h_off, *d_off;
};

ChunkBufs carve(const Slot* s, const shfhb::plan::SlotLayout& l) {
  ChunkBufs b;
  b.h_in = s->h;
  b.d_in = s->d;
  b.h_out = s->h + l.out;
  b.d_out = s->d + l.out;
  b.hd_out = s->h_dev ? s->h_dev + l.out : nullptr;
  b.h_probe = reinterpret_cast<shf_probe*>(s->h + l.probe);
  b.d_probe = reinterpret_cast<shf_probe*>(s->d + l.probe);
  b.h_off = reinterpret_cast<uint64_t*>(s->h + l.off);
  b.d_off = reinterpret_cast<uint64_t*>(s->d + l.off);
  return b;
}

// Kernel output of one chunk [i0, ...) for `job`.
void job_sink(const ChunkBufs& b, const HostJob& job, uint64_t i0, shfhb::Sink* k, int* mode) {
  *k = shfhb::Sink();
  if (job.probe) {
    k->out = b.d_probe;
    k->hash_out = job.hash ? b.d_out : nullptr;
    k->tab_slot = job.index->d_tab_slot;
    if (job.index->compact && !job.index->external) {
      k->map8 = job.index->d_map8;
      k->win_tab = job.index->d_win_tab;
    }
    k->rows = job.index->d_rows;
    k->n_slots = job.index->n_slots;
    *mode = shfhb::kOutProbe;
  } else {
    k->out = job.hash_dev ? job.at(job.hash_dev, i0) : (job.stage_direct && b.hd_out) ? b.hd_out : b.d_out;
    *mode = job.hash_mode();
    if (job.wins) {
      k->wins = job.wins + i0;
      *mode = job.uid ? shfhb::kOutUidWin : shfhb::kOutHashWin;
    }
  }
}

// The sink of a whole-batch launch straight into the caller's records (zero copy).
int direct_sink(const HostJob& job, void* d_out, shfhb::Sink* k) {
  *k = out_sink(d_out);
  if (!job.wins) return job.hash_mode();
  k->wins = job.wins;
  return job.uid ? shfhb::kOutUidWin : shfhb::kOutHashWin;
}

// Results of chunk [i0, i0 + cnt) back to the caller (straight into page-locked
// caller memory, else into the slot's pinned arena for drain_slot to copy).
int job_d2h(Slot* s, const ChunkBufs& b, const HostJob& job, uint64_t i0, uint64_t cnt, bool hash_pinned,
            bool probe_pinned, Pending* p) {
  p->reset();
  p->busy = true;
  p->count = cnt;
  p->rec = job.rec();
  if (job.hash && !job.hash_dev && job.stage_direct && !job.probe && b.hd_out) {
    p->hash = job.at(job.hash, i0);  // the kernel stored into the slot's pinned records (job_sink): copied out by drain_slot
    p->hash_src = b.h_out;
  } else if (job.hash && !job.hash_dev) {
    HB_TRY(hipMemcpyAsync(hash_pinned ? job.at(job.hash, i0) : b.h_out, b.d_out, cnt * job.rec(),
                          hipMemcpyDeviceToHost, s->st));
    if (!hash_pinned) {
      p->hash = job.at(job.hash, i0);
      p->hash_src = b.h_out;
    }
  }
  if (job.probe) {
    HB_TRY(hipMemcpyAsync(probe_pinned ? job.probe + i0 : b.h_probe, b.d_probe, cnt * sizeof(shf_probe),
                          hipMemcpyDeviceToHost, s->st));
    if (!probe_pinned) {
      p->probe = job.probe + i0;
      p->probe_src = b.h_probe;
    }
  }
  HB_TRY(hipEventRecord(s->done, s->st));
  return SHF_HB_OK;
}

// A device buffer for one key larger than a slot: allocated for the chunk that
// needs it and freed with it (after the stream that reads it is idle), so the
// slots never grow past the stage size.
struct TmpDevBuf {
  void* p = nullptr;
  hipStream_t st = nullptr;
  ~TmpDevBuf() {
    if (!p) return;
    if (st) (void)hipStreamSynchronize(st);
    (void)hipFree(p);
  }
};

// Fixed-length keys larger than a slot: one key at a time on one slot, through
// a temporary device buffer (pageable sources are staged by HIP).
int host_fixed_big(int dev, const uint8_t* keys, uint32_t key_len, uint64_t n, uint32_t seed, const HostJob& job) {
  Lease L;
  int rc = lease_slots(dev, 1, &L);
  if (rc) return rc;
  Slot* s = L.s[0];
  const ChunkBufs b = carve(s, shfhb::plan::slot_layout(0, 1, job.probe != nullptr, false, job.rec()));
  TmpDevBuf tmp;
  tmp.st = s->st;
  HB_TRY(hipMalloc(&tmp.p, key_len));
  const bool hash_pinned = is_host_pinned(job.hash), probe_pinned = is_host_pinned(job.probe);
  for (uint64_t i = 0; i < n; ++i) {
    Pending p;
    HB_TRY(hipMemcpyAsync(tmp.p, keys + i * (uint64_t)key_len, key_len, hipMemcpyHostToDevice, s->st));
    shfhb::Sink k;
    int mode = 0;
    job_sink(b, job, i, &k, &mode);
    HB_TRY(shfhb::launch_fixed(tmp.p, key_len, 1, seed, k, mode, s->st, shfhb::kKernelAuto));
    if ((rc = job_d2h(s, b, job, i, 1, hash_pinned, probe_pinned, &p))) return rc;
    if ((rc = drain_slot(s, p))) return rc;
  }
  return SHF_HB_OK;
}

// Zero copy: page-locked caller buffers that the device can address are read
// and written by the hashing kernel itself over PCIe. The copy engines run one
// direction at a time (bench.py pcie_ceilings, same run as the host lines:
// H2D 57, D2H 57, both at once on two streams 57 GB/s together), while a
// kernel's loads and stores use both directions together (a 16-B copy kernel
// over PCIe: 81 GB/s together). 160 MB of keys, G keys/s zero copy vs staged
// (profiles/r2/host_zero_copy/): 16 B 2.54 vs 1.74, 32 B 1.55 vs 1.11,
// 48 B 1.01 vs 0.81, 64 B 0.79 vs 0.68, 128 B 0.38 vs 0.33. Used for keys up
// to SHF_HB_ZERO_COPY_MAX_KEY bytes (default 128; 0 turns it off): past that
// the keys dominate the traffic and a kernel's PCIe reads (~49 GB/s at
// 128 B) approach the copy engine's 57 GB/s.
uint32_t zero_copy_max_key() {
  const char* e = getenv("SHF_HB_ZERO_COPY_MAX_KEY");
  if (!e) return 128u;
  const long v = strtol(e, nullptr, 10);
  return v < 0 ? 0u : (uint32_t)std::min<long>(v, 1L << 20);
}

// Device address of host bytes [p, p + bytes), when they lie in one
// page-locked allocation that the current device maps; else nullptr.
void* host_range_device_ptr(const void* p, size_t bytes) {
  if (!p || !bytes) return nullptr;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  void* d = nullptr;
  if (hipMemGetAddressRange(&base, &size, const_cast<void*>(p)) != hipSuccess ||
      reinterpret_cast<uintptr_t>(p) + bytes > reinterpret_cast<uintptr_t>(base) + size ||
      hipHostGetDevicePointer(&d, const_cast<void*>(p), 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return d;
}

// Staged pipelines: the kernel stores each chunk's hashes over PCIe (posted
// writes beside the copy engine's H2D of the next chunk) instead of a D2H
// copy on that same engine -- straight into a page-locked caller output, or
// into the slot's page-locked staging that drain_slot copies to a pageable
// one. SHF_HB_DIRECT_OUT=0 turns it off.
HostJob with_direct_out(const HostJob& job, uint64_t n) {
  HostJob j = job;
  const char* e = getenv("SHF_HB_DIRECT_OUT");
  if (job.hash && !job.probe && !(e && e[0] == '0')) {
    j.hash_dev = host_range_device_ptr(job.hash, (size_t)n * job.rec());
    j.stage_direct = !j.hash_dev;
  }
  return j;
}

// Pageable caller buffers are never page-locked by this library: they go
// through the staged pipeline. Rounds 3-5 locked their whole interior pages
// for a call (hipHostRegister) and let the kernel read and write them over
// PCIe (2.38 against 2.03 G keys/s staged for 10M x 16-B keys); in 3 of the
// last 5 full GPU test runs with that path on, a later pageable copy of the
// same process (torch's .to(device) / .cpu() of a >= 1 MB buffer) failed with
// hipErrorIllegalAddress, and in none of 6 with it off. A registration that
// outlives its memory produces exactly that failure
// (tools/pageable_register_repro.hip, scenario D); the lock / unlock / free /
// reuse sequences the library used, replayed alone, do not (scenarios A-C, E),
// even with every lock checked against the runtime both ways. The interaction lies inside the runtime's own
// pageable-copy path; a library must not put its caller's unrelated copies at
// risk for 15 %, so the path is gone.

// Pageable fixed-length keys go to the device through the HIP runtime's own
// pageable copy (hipMemcpyAsync from the caller's memory, which holds the
// calling thread until its bytes are on their way), while the copy workers
// move each earlier chunk's records out (drain_async); SHF_HB_RUNTIME_H2D=0
// copies them into the slot's pinned arena on the CPU first instead. The
// runtime moves pageable bytes at 49-56 GB/s, as fast as page-locked ones,
// and two threads' pageable copies in opposite directions overlap (81 GB/s
// together at 8-MiB chunks; tools/pageable_*_probe.py, profiles/r5/runtime_copy/).
// 10M x 16-B pageable keys: 2.34-2.39 against 1.96-2.17 G keys/s staged on
// the CPU, 16 threads at once 2.18-2.27 against 1.89-1.95 (same box, alternating).
// (The records back by the runtime's pageable D2H too, issued from a copy worker beside
// the next chunk's H2D, instead of kernel stores into the slot plus a host copy: 1.68-2.00
// against 2.14-2.29 G keys/s, profiles/r5/runtime_copy/ab_runtime_d2h/; not kept.)
bool runtime_h2d() {
  const char* e = getenv("SHF_HB_RUNTIME_H2D");
  return !(e && e[0] == '0');
}

// Host-memory fixed-length pipeline on the current device.
int host_fixed_run(const uint8_t* keys, uint32_t key_len, uint64_t n, uint32_t seed, const HostJob& job_in) {
  const HostJob job = with_direct_out(job_in, n);
  DevCtx* c = nullptr;
  int rc = current_ctx(&c);
  if (rc) return rc;
  if (job.hash && !job.probe && key_len && key_len <= zero_copy_max_key()) {
    void* dk = host_range_device_ptr(keys, (size_t)n * key_len);
    void* dh = dk ? host_range_device_ptr(job.hash, (size_t)n * job.rec()) : nullptr;
    if (dh) {
      shfhb::Sink dsk;
      const int dmode = direct_sink(job, dh, &dsk);
      HB_TRY(shfhb::launch_fixed(dk, key_len, n, seed, dsk, dmode, c->st, shfhb::kKernelAuto));
      HB_TRY(hipStreamSynchronize(c->st));
      return SHF_HB_OK;
    }
  }
  const bool probe = job.probe != nullptr;
  const uint64_t per = shfhb::plan::fixed_chunk_keys(std::max(stage_bytes(), shfhb::plan::kMinSlotBytes), key_len,
                                                     probe, job.rec());
  if (!per) return host_fixed_big(c->dev, keys, key_len, n, seed, job);
  Lease L;  // no more slots than the batch has chunks: the rest stay free for other threads' calls
  if ((rc = lease_slots(c->dev, (int)std::min<uint64_t>((n + per - 1) / per, pipeline_slots()), &L))) return rc;
  const uint64_t chunk =
      shfhb::plan::even_chunk(n, shfhb::plan::fixed_chunk_keys(L.s[0]->bytes, key_len, probe, job.rec()));
  const shfhb::plan::SlotLayout lay = shfhb::plan::slot_layout((size_t)chunk * key_len, chunk, probe, false, job.rec());
  const bool in_pinned = is_host_pinned(keys), hash_pinned = is_host_pinned(job.hash),
             probe_pinned = is_host_pinned(job.probe);
  const bool via_runtime = !in_pinned && runtime_h2d();
  if (trace_on()) tls_trace.slots = L.n;
  Pending pend[kMaxSlots];
  uint64_t idx = 0;
  for (uint64_t i0 = 0; i0 < n; i0 += chunk, ++idx) {
    const int q = (int)(idx % L.n);
    Slot* s = L.s[q];
    if ((rc = drain_slot(s, pend[q]))) return rc;
    const ChunkBufs b = carve(s, lay);
    const uint64_t cnt = std::min(chunk, n - i0);
    const size_t nb = (size_t)cnt * key_len;
    const uint8_t* src = (in_pinned || via_runtime) ? keys + i0 * key_len : b.h_in;
    const double t0 = trace_on() ? now_ms() : 0;
    if (nb && !in_pinned && !via_runtime) par_memcpy(b.h_in, keys + i0 * key_len, nb);
    if (nb) HB_TRY(hipMemcpyAsync(b.d_in, src, nb, hipMemcpyHostToDevice, s->st));
    const double t1 = trace_on() ? now_ms() : 0;
    shfhb::Sink k;
    int mode = 0;
    job_sink(b, job, i0, &k, &mode);
    HB_TRY(shfhb::launch_fixed(b.d_in, key_len, cnt, seed, k, mode, s->st, shfhb::kKernelAuto));
    if ((rc = job_d2h(s, b, job, i0, cnt, hash_pinned, probe_pinned, &pend[q]))) return rc;
    if (via_runtime) drain_async(s, pend[q]);
    if (trace_on()) {
      tls_trace.copy_in += t1 - t0;
      tls_trace.enqueue += now_ms() - t1;
      ++tls_trace.chunks;
    }
  }
  return drain_all(L, pend);
}

// Host-memory variable-length pipeline: chunks of whole keys that fit one slot
// with their offsets and records (host_plan.h var_chunk_end); a single key too
// long for a slot gets a chunk of its own, its bytes in a temporary buffer.
int host_var_run(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint32_t seed, const HostJob& job_in) {
  const HostJob job = with_direct_out(job_in, n);
  DevCtx* c = nullptr;
  int rc = current_ctx(&c);
  if (rc) return rc;
  const bool probe = job.probe != nullptr;
  Lease L;  // about as many slots as the batch has chunks (host_plan.h var_chunks_estimate)
  const uint64_t est = shfhb::plan::var_chunks_estimate(offsets[n] - offsets[0], n,
                                                        std::max(stage_bytes(), shfhb::plan::kMinSlotBytes), probe,
                                                        job.rec());
  if ((rc = lease_slots(c->dev, (int)std::min<uint64_t>(est, pipeline_slots()), &L))) return rc;
  const size_t slot_bytes = L.s[0]->bytes;
  const bool in_pinned = is_host_pinned(bytes), off_pinned = is_host_pinned(offsets),
             hash_pinned = is_host_pinned(job.hash), probe_pinned = is_host_pinned(job.probe);
  // (staged on the CPU, not through the runtime's pageable copy: a slot's ~15 MiB of variable-
  // length key bytes per chunk came out 7 % slower that way, 0.178-0.179 against 0.191-0.193 G
  // keys/s on U[8,512] B; the runtime's opposite-direction copies stop overlapping at 16-32 MiB)
  Pending pend[kMaxSlots];
  uint64_t idx = 0;
  for (uint64_t i0 = 0; i0 < n; ++idx) {
    bool alone = false;
    const uint64_t i1 = shfhb::plan::var_chunk_end(offsets, i0, n, slot_bytes, probe, &alone, job.rec());
    const uint64_t cnt = i1 - i0, base = offsets[i0];
    const size_t nb = (size_t)(offsets[i1] - base);
    const int q = (int)(idx % L.n);
    Slot* s = L.s[q];
    TmpDevBuf tmp;
    if (alone) {
      if ((rc = drain_all(L, pend))) return rc;
      tmp.st = s->st;
      HB_TRY(hipMalloc(&tmp.p, nb));
    } else if ((rc = drain_slot(s, pend[q]))) {
      return rc;
    }
    const ChunkBufs b = carve(s, shfhb::plan::slot_layout(alone ? 0 : nb, cnt, probe, true, job.rec()));
    uint8_t* d_in = alone ? (uint8_t*)tmp.p : b.d_in;
    if (nb && !in_pinned && !alone) par_memcpy(b.h_in, bytes + base, nb);
    const uint64_t* off_src = offsets + i0;
    if (!off_pinned) {
      par_memcpy(b.h_off, offsets + i0, (cnt + 1) * sizeof(uint64_t));
      off_src = b.h_off;
    }
    if (nb)
      HB_TRY(hipMemcpyAsync(d_in, (in_pinned || alone) ? bytes + base : b.h_in, nb, hipMemcpyHostToDevice, s->st));
    HB_TRY(hipMemcpyAsync(b.d_off, off_src, (cnt + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s->st));
    shfhb::Sink k;
    int mode = 0;
    job_sink(b, job, i0, &k, &mode);
    // the chunk's byte count sizes the span kernel's window (kernels.hip span_window)
    HB_TRY(shfhb::launch_var(d_in, b.d_off, base, cnt, seed, k, mode, s->st, shfhb::kKernelAuto, nb));
    if ((rc = job_d2h(s, b, job, i0, cnt, hash_pinned, probe_pinned, &pend[q]))) return rc;
    if (alone && (rc = drain_slot(s, pend[q]))) return rc;  // before tmp is freed
    i0 = i1;
  }
  return drain_all(L, pend);
}

// On an error mid-pipeline, work may still be in flight, some DMA-ing into the
// caller's (page-locked) output: wait for it before handing the buffers back to
// the caller (the slots' streams are waited for by their Lease).
int drain_on_error(int rc) {
  if (rc == SHF_HB_OK) return rc;
  const int hip = tls_last_hip;
  DevCtx* c = nullptr;
  if (current_ctx(&c) == SHF_HB_OK) (void)hipStreamSynchronize(c->st);
  (void)hipGetLastError();
  tls_last_hip = hip;
  return rc;
}

int host_fixed(const uint8_t* keys, uint32_t key_len, uint64_t n, uint32_t seed, const HostJob& job) {
  if (!trace_on()) return drain_on_error(host_fixed_run(keys, key_len, n, seed, job));
  tls_trace = PipeTrace();
  const double t0 = now_ms();
  const int rc = drain_on_error(host_fixed_run(keys, key_len, n, seed, job));
  fprintf(stderr,
          "shf_hash_batch trace: fixed n=%llu chunks=%llu total_ms=%.3f copy_in_ms=%.3f enqueue_ms=%.3f "
          "wait_ms=%.3f copy_out_ms=%.3f rc=%d\n",
          (unsigned long long)n, (unsigned long long)tls_trace.chunks, now_ms() - t0, tls_trace.copy_in,
          tls_trace.enqueue, tls_trace.wait, tls_trace.copy_out, rc);
  return rc;
}

int host_var(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint32_t seed, const HostJob& job) {
  return drain_on_error(host_var_run(bytes, offsets, n, seed, job));
}

HostJob hash_job(shf_hash128* out) {
  HostJob j;
  j.hash = out;
  return j;
}

HostJob uid_job(uint64_t* parts) {
  HostJob j;
  j.hash = parts;
  j.uid = true;
  return j;
}

int check_var_lengths_host(const uint64_t* offsets, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) {
    if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > kMaxKeyLen) return SHF_HB_ERR_ARG;
  }
  return SHF_HB_OK;
}

int device_fixed(const void* keys, uint32_t key_len, uint64_t n, uint32_t seed, const shfhb::Sink& sink,
                 int out_mode, hipStream_t st, int kernel, bool sync) {
  DevCtx* c = nullptr;
  int rc = current_ctx(&c);
  if (rc) return rc;
  if (sync) st = nullptr;  // after the caller's null-stream work (e.g. the keys' producer)
  HB_TRY(shfhb::launch_fixed(keys, key_len, n, seed, sink, out_mode, st, kernel));
  if (sync) HB_TRY(hipStreamSynchronize(st));
  return SHF_HB_OK;
}

// Device-resident variable-length keys. The offsets are only on the device, so
// the kernels check them (o1 < o0 or o1 - o0 >= 2^31: kernels.hip var_key_bad),
// skip such keys without reading their bytes and set a status word:
// synchronous calls clear and read their own word and return SHF_HB_ERR_ARG;
// asynchronous ones set the thread's sticky word, read by shf_hash_batch_status().
int device_var(const void* bytes, const uint64_t* offsets, uint64_t n, uint32_t seed, const shfhb::Sink& sink,
               int out_mode, hipStream_t st, bool sync, int kernel = shfhb::kKernelAuto, uint64_t key_bytes = 0) {
  DevCtx* c = nullptr;
  int rc = current_ctx(&c);
  if (rc) return rc;
  shfhb::Sink k = sink;
  if (sync) {
    st = nullptr;  // after the caller's null-stream work
    k.status = c->d_status + 1;
    HB_TRY(hipMemsetAsync(k.status, 0, sizeof(uint32_t), st));
  } else {
    k.status = c->d_status;
  }
  HB_TRY(shfhb::launch_var(bytes, offsets, 0, n, seed, k, out_mode, st, kernel, key_bytes));
  if (sync) {
    HB_TRY(hipMemcpyAsync(c->h_status, k.status, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HB_TRY(hipStreamSynchronize(st));
    if (*c->h_status) return SHF_HB_ERR_ARG;
  }
  return SHF_HB_OK;
}

bool var_kernel_valid(int kernel) {
  return kernel == SHF_HB_KERNEL_AUTO || kernel == SHF_HB_KERNEL_SPAN || kernel == SHF_HB_KERNEL_SPAN_PP ||
         kernel == SHF_HB_KERNEL_GENERIC || kernel == SHF_HB_KERNEL_ROUND;
}

// Can the forced fixed-length kernel take this shape? (AUTO always can.)
bool fixed_kernel_fits(const void* d_keys, uint32_t key_len, int kernel) {
  const bool al16 = ((uintptr_t)d_keys & 15u) == 0;
  switch (kernel) {
    case SHF_HB_KERNEL_AUTO:
    case SHF_HB_KERNEL_GENERIC:
      return true;
    case SHF_HB_KERNEL_FIXED16:
      return key_len == 16 && al16;
    case SHF_HB_KERNEL_TILED:
      return key_len >= 32 && (key_len & 15u) == 0 && al16;
    case SHF_HB_KERNEL_SPAN:
      return (uint64_t)key_len * 64u + 16u <= 20416u;  // one 64-key tile in the LDS window
    default:
      return false;
  }
}


// A caller's window-order workspace: big enough for n keys and 16-B aligned
// (the window bytes move 16 B at a time).
bool win_workspace_ok(const void* ws, size_t bytes, uint64_t n) {
  return ws && bytes >= shfhb::win_order_workspace_bytes(n) && ((uintptr_t)ws & 15u) == 0;
}

// Probe sink for `index` on the calling thread's current device.
int probe_sink(const shf_row_index* index, void* d_probe, void* d_hashes, shfhb::Sink* sink) {
  if (!index || !d_probe) return SHF_HB_ERR_ARG;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != index->dev) return SHF_HB_ERR_ARG;
  sink->out = d_probe;
  sink->hash_out = d_hashes;
  sink->tab_slot = index->d_tab_slot;
  sink->rows = index->d_rows;
  sink->n_slots = index->n_slots;
  if (index->compact && !index->external) {
    sink->map8 = index->d_map8;
    sink->win_tab = index->d_win_tab;
  }
  return SHF_HB_OK;
}

int visible_devices() {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return SHF_HB_ERR_NODEV;
  }
  return n;
}

// Test-only knob SHF_HB_MULTI_SHARE_DEVICES=1: shard d runs on device
// d % visible, so n_devices may exceed the visible devices (exercises the
// multi-GPU split with several host threads on a one-GPU box).
bool multi_share_devices() {
  const char* e = getenv("SHF_HB_MULTI_SHARE_DEVICES");
  return e && e[0] == '1';
}

template <class F>
int run_multi(uint64_t n, int n_devices, F&& shard_fn) {
  const int vis = visible_devices();
  if (vis < 0) return vis;
  if (vis == 0) return SHF_HB_ERR_NODEV;
  const bool share = multi_share_devices();
  int g = n_devices <= 0 ? vis : (share ? std::min(n_devices, 64) : std::min(n_devices, vis));
  if ((uint64_t)g > n) g = (int)std::max<uint64_t>(1, n);
  std::vector<int> rcs(g, SHF_HB_OK);
  std::vector<int> errs(g, 0);
  std::vector<std::thread> th;
  for (int d = 0; d < g; ++d) {
    const uint64_t lo = n * (uint64_t)d / (uint64_t)g, hi = n * (uint64_t)(d + 1) / (uint64_t)g;
    th.emplace_back([&, d, lo, hi]() {
      hipError_t e = hipSetDevice(d % vis);
      if (e != hipSuccess) {
        rcs[d] = map_hip(e);
      } else if (hi > lo) {
        rcs[d] = shard_fn(lo, hi);
      }
      errs[d] = tls_last_hip;
      release_thread_ctx();
    });
  }
  for (auto& t : th) t.join();
  for (int d = 0; d < g; ++d) {
    if (rcs[d] != SHF_HB_OK) {
      tls_last_hip = errs[d];
      return rcs[d];
    }
  }
  return SHF_HB_OK;
}

}  // namespace

extern "C" {

int shf_hash_batch_fixed(const void* keys, uint32_t key_len, uint64_t n, uint32_t seed, shf_hash128* out,
                         int mem) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!out || (!keys && key_len) || key_len > kMaxKeyLen) return SHF_HB_ERR_ARG;
  if (mem == SHF_HASH_MEM_DEVICE)
    return device_fixed(keys, key_len, n, seed, out_sink(out), shfhb::kOutHash, nullptr, shfhb::kKernelAuto, true);
  if (mem == SHF_HASH_MEM_HOST) return host_fixed((const uint8_t*)keys, key_len, n, seed, hash_job(out));
  return SHF_HB_ERR_ARG;
}

int shf_hash_batch_fixed_async(const void* d_keys, uint32_t key_len, uint64_t n, uint32_t seed, shf_hash128* d_out,
                               void* hip_stream) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!d_out || (!d_keys && key_len) || key_len > kMaxKeyLen) return SHF_HB_ERR_ARG;
  return device_fixed(d_keys, key_len, n, seed, out_sink(d_out), shfhb::kOutHash, (hipStream_t)hip_stream,
                      shfhb::kKernelAuto, false);
}

int shf_hash_batch_fixed_kernel_async(const void* d_keys, uint32_t key_len, uint64_t n, uint32_t seed,
                                      shf_hash128* d_out, int kernel, void* hip_stream) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!d_out || (!d_keys && key_len) || key_len > kMaxKeyLen) return SHF_HB_ERR_ARG;
  if (!fixed_kernel_fits(d_keys, key_len, kernel)) return SHF_HB_ERR_ARG;
  return device_fixed(d_keys, key_len, n, seed, out_sink(d_out), shfhb::kOutHash, (hipStream_t)hip_stream, kernel, false);
}

int shf_hash_batch_var(const void* bytes, const uint64_t* offsets, uint64_t n, uint32_t seed, shf_hash128* out,
                       int mem) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!out || !offsets || !bytes) return SHF_HB_ERR_ARG;
  if (mem == SHF_HASH_MEM_DEVICE) return device_var(bytes, offsets, n, seed, out_sink(out), shfhb::kOutHash, nullptr, true);
  if (mem == SHF_HASH_MEM_HOST) {
    int rc = check_var_lengths_host(offsets, n);
    if (rc) return rc;
    return host_var((const uint8_t*)bytes, offsets, n, seed, hash_job(out));
  }
  return SHF_HB_ERR_ARG;
}

int shf_hash_batch_var_async(const void* d_bytes, const uint64_t* d_offsets, uint64_t n, uint32_t seed,
                             shf_hash128* d_out, void* hip_stream) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!d_out || !d_offsets || !d_bytes) return SHF_HB_ERR_ARG;
  return device_var(d_bytes, d_offsets, n, seed, out_sink(d_out), shfhb::kOutHash, (hipStream_t)hip_stream, false);
}

int shf_hash_batch_var_kernel_async(const void* d_bytes, const uint64_t* d_offsets, uint64_t n, uint32_t seed,
                                    shf_hash128* d_out, int kernel, void* hip_stream) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!d_out || !d_offsets || !d_bytes) return SHF_HB_ERR_ARG;
  if (!var_kernel_valid(kernel)) return SHF_HB_ERR_ARG;
  return device_var(d_bytes, d_offsets, n, seed, out_sink(d_out), shfhb::kOutHash, (hipStream_t)hip_stream, false, kernel);
}

int shf_hash_batch_var_sized_async(const void* d_bytes, const uint64_t* d_offsets, uint64_t n, uint64_t key_bytes,
                                   uint32_t seed, shf_hash128* d_out, void* hip_stream) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!d_out || !d_offsets || !d_bytes) return SHF_HB_ERR_ARG;
  return device_var(d_bytes, d_offsets, n, seed, out_sink(d_out), shfhb::kOutHash, (hipStream_t)hip_stream, false,
                    shfhb::kKernelAuto, key_bytes);
}

int shf_hash_batch_var_sized_kernel_async(const void* d_bytes, const uint64_t* d_offsets, uint64_t n,
                                          uint64_t key_bytes, uint32_t seed, shf_hash128* d_out, int kernel,
                                          void* hip_stream) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!d_out || !d_offsets || !d_bytes) return SHF_HB_ERR_ARG;
  if (!var_kernel_valid(kernel)) return SHF_HB_ERR_ARG;
  return device_var(d_bytes, d_offsets, n, seed, out_sink(d_out), shfhb::kOutHash, (hipStream_t)hip_stream, false,
                    kernel, key_bytes);
}

int shf_uid_parts_batch_fixed_async(const void* d_keys, uint32_t key_len, uint64_t n, uint32_t seed,
                                    uint64_t* d_parts, void* hip_stream) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!d_parts || (!d_keys && key_len) || key_len > kMaxKeyLen) return SHF_HB_ERR_ARG;
  return device_fixed(d_keys, key_len, n, seed, out_sink(d_parts), shfhb::kOutUid, (hipStream_t)hip_stream,
                      shfhb::kKernelAuto, false);
}

int shf_uid_parts_batch_var_async(const void* d_bytes, const uint64_t* d_offsets, uint64_t n, uint32_t seed,
                                  uint64_t* d_parts, void* hip_stream) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!d_parts || !d_offsets || !d_bytes) return SHF_HB_ERR_ARG;
  return device_var(d_bytes, d_offsets, n, seed, out_sink(d_parts), shfhb::kOutUid, (hipStream_t)hip_stream, false);
}

int shf_uid_parts_batch_fixed(const void* keys, uint32_t key_len, uint64_t n, uint32_t seed, uint64_t* parts,
                              int mem) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!parts || (!keys && key_len) || key_len > kMaxKeyLen) return SHF_HB_ERR_ARG;
  if (mem == SHF_HASH_MEM_DEVICE)
    return device_fixed(keys, key_len, n, seed, out_sink(parts), shfhb::kOutUid, nullptr, shfhb::kKernelAuto, true);
  if (mem == SHF_HASH_MEM_HOST) return host_fixed((const uint8_t*)keys, key_len, n, seed, uid_job(parts));
  return SHF_HB_ERR_ARG;
}

int shf_uid_parts_batch_var(const void* bytes, const uint64_t* offsets, uint64_t n, uint32_t seed, uint64_t* parts,
                            int mem) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!parts || !offsets || !bytes) return SHF_HB_ERR_ARG;
  if (mem == SHF_HASH_MEM_DEVICE)
    return device_var(bytes, offsets, n, seed, out_sink(parts), shfhb::kOutUid, nullptr, true);
  if (mem == SHF_HASH_MEM_HOST) {
    const int rc = check_var_lengths_host(offsets, n);
    if (rc) return rc;
    return host_var((const uint8_t*)bytes, offsets, n, seed, uid_job(parts));
  }
  return SHF_HB_ERR_ARG;
}

int shf_hash_batch_fixed_win_kernel_async(const void* d_keys, uint32_t key_len, uint64_t n, uint32_t seed,
                                          shf_hash128* d_out, uint32_t* d_perm, uint32_t* d_win_start,
                                          void* d_workspace, size_t workspace_bytes, int kernel, void* hip_stream) {
  HB_ENTER();
  if (n == 0 && !d_win_start) return SHF_HB_OK;
  if (n && (!d_out || !d_perm || (!d_keys && key_len))) return SHF_HB_ERR_ARG;
  if (key_len > kMaxKeyLen || n > 0xffffffffull || !fixed_kernel_fits(d_keys, key_len, kernel)) return SHF_HB_ERR_ARG;
  if (n && !win_workspace_ok(d_workspace, workspace_bytes, n)) return SHF_HB_ERR_ARG;
  DevCtx* c = nullptr;
  int rc = current_ctx(&c);
  if (rc) return rc;
  const hipStream_t st = (hipStream_t)hip_stream;
  bool ranked = false;
  if (n) {
    shfhb::Sink k = out_sink(d_out);
    k.wins = shfhb::win_order_wins(d_workspace, n);
    k.win_counts = shfhb::win_order_counts(d_workspace);
    k.win_sorted = shfhb::win_order_sorted(d_workspace, n);
    HB_TRY(shfhb::launch_fixed_win(d_keys, key_len, n, seed, k, st, kernel, &ranked));
  }
  HB_TRY(shfhb::launch_win_order_bytes(n, ranked, d_perm, d_win_start, d_workspace, st));
  return SHF_HB_OK;
}

int shf_hash_batch_fixed_win_async(const void* d_keys, uint32_t key_len, uint64_t n, uint32_t seed,
                                   shf_hash128* d_out, uint32_t* d_perm, uint32_t* d_win_start, void* d_workspace,
                                   size_t workspace_bytes, void* hip_stream) {
  HB_ENTER();
  return shf_hash_batch_fixed_win_kernel_async(d_keys, key_len, n, seed, d_out, d_perm, d_win_start, d_workspace,
                                                workspace_bytes, SHF_HB_KERNEL_AUTO, hip_stream);
}

int shf_hash_batch_var_win_kernel_async(const void* d_bytes, const uint64_t* d_offsets, uint64_t n, uint32_t seed,
                                        shf_hash128* d_out, uint32_t* d_perm, uint32_t* d_win_start,
                                        void* d_workspace, size_t workspace_bytes, int kernel, void* hip_stream) {
  HB_ENTER();
  if (n == 0 && !d_win_start) return SHF_HB_OK;
  if (n && (!d_out || !d_perm || !d_offsets || !d_bytes)) return SHF_HB_ERR_ARG;
  if (n > 0xffffffffull || !var_kernel_valid(kernel)) return SHF_HB_ERR_ARG;
  if (n && !win_workspace_ok(d_workspace, workspace_bytes, n)) return SHF_HB_ERR_ARG;
  shfhb::Sink k = out_sink(d_out);
  if (n) {
    k.wins = shfhb::win_order_wins(d_workspace, n);
    int rc = device_var(d_bytes, d_offsets, n, seed, k, shfhb::kOutHashWin, (hipStream_t)hip_stream, false, kernel);
    if (rc) return rc;
  } else {
    DevCtx* c = nullptr;
    int rc = current_ctx(&c);
    if (rc) return rc;
  }
  HB_TRY(shfhb::launch_win_order_bytes(n, false, d_perm, d_win_start, d_workspace, (hipStream_t)hip_stream));
  return SHF_HB_OK;
}

int shf_hash_batch_var_win_async(const void* d_bytes, const uint64_t* d_offsets, uint64_t n, uint32_t seed,
                                 shf_hash128* d_out, uint32_t* d_perm, uint32_t* d_win_start, void* d_workspace,
                                 size_t workspace_bytes, void* hip_stream) {
  HB_ENTER();
  return shf_hash_batch_var_win_kernel_async(d_bytes, d_offsets, n, seed, d_out, d_perm, d_win_start, d_workspace,
                                             workspace_bytes, SHF_HB_KERNEL_AUTO, hip_stream);
}

}  // extern "C"

namespace {

// Synchronous hash + window order (shf_hash_batch_{fixed,var}_win, and with
// 8-B UID parts instead of the records: shf_uid_parts_batch_{fixed,var}_win).
// Device memory: the records (or parts) and each key's window byte, then the
// order from the bytes (16-B records: the fused k_fixed16_win ranks the
// chunks itself), then a wait. Host memory: the host pipelines write the
// records (parts) to `out` and leave each key's window byte in the device
// workspace (the records are never copied back in to be ordered), the order is
// made on the device, and only perm / win_start come back.
int hash_win_sync(bool var, bool uid, const void* keys, const uint64_t* offsets, uint32_t key_len, uint64_t n,
                  uint32_t seed, void* out, uint32_t* perm, uint32_t* win_start, int mem) {
  if (mem != SHF_HASH_MEM_DEVICE && mem != SHF_HASH_MEM_HOST) return SHF_HB_ERR_ARG;
  if (n == 0 && !win_start) return SHF_HB_OK;
  if (n > 0xffffffffull || (!var && key_len > kMaxKeyLen)) return SHF_HB_ERR_ARG;
  if (n && (!out || !perm || (var ? (!keys || !offsets) : (!keys && key_len)))) return SHF_HB_ERR_ARG;
  DevCtx* c = nullptr;
  int rc = current_ctx(&c);
  if (rc) return rc;
  if (var && mem == SHF_HASH_MEM_HOST && (rc = check_var_lengths_host(offsets, n))) return rc;
  void* ws = nullptr;
  if ((rc = ensure_win_ws(c, (size_t)shfhb::win_order_workspace_bytes(n), &ws))) return rc;
  // device memory: on the null stream, as every synchronous device entry point, so the
  // hash and order run after whatever the caller enqueued there (e.g. the keys' producer)
  const hipStream_t st = mem == SHF_HASH_MEM_DEVICE ? nullptr : c->st;
  const int mode = uid ? shfhb::kOutUidWin : shfhb::kOutHashWin;
  if (mem == SHF_HASH_MEM_DEVICE) {
    shfhb::Sink k = out_sink(out);
    bool ranked = false;
    if (n) {
      k.wins = shfhb::win_order_wins(ws, n);
      if (var) {
        k.status = c->d_status + 1;
        HB_TRY(hipMemsetAsync(k.status, 0, sizeof(uint32_t), st));
        HB_TRY(shfhb::launch_var(keys, offsets, 0, n, seed, k, mode, st));
      } else if (uid) {
        HB_TRY(shfhb::launch_fixed(keys, key_len, n, seed, k, mode, st, shfhb::kKernelAuto));
      } else {
        k.win_counts = shfhb::win_order_counts(ws);
        k.win_sorted = shfhb::win_order_sorted(ws, n);
        HB_TRY(shfhb::launch_fixed_win(keys, key_len, n, seed, k, st, shfhb::kKernelAuto, &ranked));
      }
    }
    HB_TRY(shfhb::launch_win_order_bytes(n, ranked, perm, win_start, ws, st));
    if (var && n) HB_TRY(hipMemcpyAsync(c->h_status, k.status, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HB_TRY(hipStreamSynchronize(st));
    return var && n && *c->h_status ? SHF_HB_ERR_ARG : SHF_HB_OK;
  }
  uint32_t* d_perm = nullptr;
  if ((rc = ensure_perm(c, n, &d_perm))) return rc;
  if (n) {
    HostJob job = uid ? uid_job(static_cast<uint64_t*>(out)) : hash_job(static_cast<shf_hash128*>(out));
    job.wins = shfhb::win_order_wins(ws, n);
    rc = var ? host_var((const uint8_t*)keys, offsets, n, seed, job)
             : host_fixed((const uint8_t*)keys, key_len, n, seed, job);
    if (rc) return rc;
  }
  HB_TRY(shfhb::launch_win_order_bytes(n, false, d_perm, d_perm + n, ws, st));
  if (n) HB_TRY(hipMemcpyAsync(perm, d_perm, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  if (win_start) HB_TRY(hipMemcpyAsync(win_start, d_perm + n, 257u * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HB_TRY(hipStreamSynchronize(st));
  return SHF_HB_OK;
}

}  // namespace

extern "C" {

int shf_hash_batch_fixed_win(const void* keys, uint32_t key_len, uint64_t n, uint32_t seed, shf_hash128* out,
                             uint32_t* perm, uint32_t* win_start, int mem) {
  HB_ENTER();
  return hash_win_sync(false, false, keys, nullptr, key_len, n, seed, out, perm, win_start, mem);
}

int shf_hash_batch_var_win(const void* bytes, const uint64_t* offsets, uint64_t n, uint32_t seed, shf_hash128* out,
                           uint32_t* perm, uint32_t* win_start, int mem) {
  HB_ENTER();
  return hash_win_sync(true, false, bytes, offsets, 0, n, seed, out, perm, win_start, mem);
}

int shf_uid_parts_batch_fixed_win(const void* keys, uint32_t key_len, uint64_t n, uint32_t seed, uint64_t* parts,
                                  uint32_t* perm, uint32_t* win_start, int mem) {
  HB_ENTER();
  return hash_win_sync(false, true, keys, nullptr, key_len, n, seed, parts, perm, win_start, mem);
}

int shf_uid_parts_batch_var_win(const void* bytes, const uint64_t* offsets, uint64_t n, uint32_t seed,
                                uint64_t* parts, uint32_t* perm, uint32_t* win_start, int mem) {
  HB_ENTER();
  return hash_win_sync(true, true, bytes, offsets, 0, n, seed, parts, perm, win_start, mem);
}

int shf_hash_batch_fixed_multi(const void* keys, uint32_t key_len, uint64_t n, uint32_t seed, shf_hash128* out,
                               int n_devices) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!out || (!keys && key_len) || key_len > kMaxKeyLen) return SHF_HB_ERR_ARG;
  const uint8_t* k = (const uint8_t*)keys;
  return run_multi(n, n_devices, [&](uint64_t lo, uint64_t hi) {
    return host_fixed(k ? k + lo * key_len : nullptr, key_len, hi - lo, seed, hash_job(out + lo));
  });
}

int shf_hash_batch_var_multi(const void* bytes, const uint64_t* offsets, uint64_t n, uint32_t seed,
                             shf_hash128* out, int n_devices) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!out || !offsets || !bytes) return SHF_HB_ERR_ARG;
  int rc = check_var_lengths_host(offsets, n);
  if (rc) return rc;
  const uint8_t* b = (const uint8_t*)bytes;
  return run_multi(n, n_devices, [&](uint64_t lo, uint64_t hi) {
    return host_var(b, offsets + lo, hi - lo, seed, hash_job(out + lo));
  });
}

int shf_uid_parts_batch_fixed_multi(const void* keys, uint32_t key_len, uint64_t n, uint32_t seed, uint64_t* parts,
                                    int n_devices) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!parts || (!keys && key_len) || key_len > kMaxKeyLen) return SHF_HB_ERR_ARG;
  const uint8_t* k = (const uint8_t*)keys;
  return run_multi(n, n_devices, [&](uint64_t lo, uint64_t hi) {
    return host_fixed(k ? k + lo * key_len : nullptr, key_len, hi - lo, seed, uid_job(parts + lo));
  });
}

int shf_uid_parts_batch_var_multi(const void* bytes, const uint64_t* offsets, uint64_t n, uint32_t seed,
                                  uint64_t* parts, int n_devices) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!parts || !offsets || !bytes) return SHF_HB_ERR_ARG;
  int rc = check_var_lengths_host(offsets, n);
  if (rc) return rc;
  const uint8_t* b = (const uint8_t*)bytes;
  return run_multi(n, n_devices, [&](uint64_t lo, uint64_t hi) {
    return host_var(b, offsets + lo, hi - lo, seed, uid_job(parts + lo));
  });
}

int shf_row_index_create(uint64_t n_slots, shf_row_index** out) {
  HB_ENTER();
  if (!out) return SHF_HB_ERR_ARG;
  *out = nullptr;
  if (n_slots > ((uint64_t)1 << 21)) return SHF_HB_ERR_ARG;  // slot must fit the 21 high bits of tab_slot
  DevCtx* c = nullptr;
  int rc = current_ctx(&c);
  if (rc) return rc;
  shf_row_index* x = new shf_row_index();
  x->dev = c->dev;
  x->n_slots = n_slots;
  hipError_t e = hipMalloc((void**)&x->d_tab_slot, SHF_ROW_INDEX_TABS * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemset(x->d_tab_slot, 0xff, SHF_ROW_INDEX_TABS * sizeof(uint32_t));
  if (e == hipSuccess && n_slots) e = hipMalloc((void**)&x->d_rows, n_slots * SHF_ROW_INDEX_SLOT_BYTES);
  if (e == hipSuccess && n_slots) e = hipMemset(x->d_rows, 0, n_slots * SHF_ROW_INDEX_SLOT_BYTES);
  if (e == hipSuccess) e = hipMalloc((void**)&x->d_map8, SHF_ROW_INDEX_TABS);
  if (e == hipSuccess) e = hipMalloc((void**)&x->d_win_tab, 256u * 256u * sizeof(uint32_t));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    (void)shf_row_index_destroy(x);
    return map_hip(e);
  }
  *out = x;
  return SHF_HB_OK;
}

int shf_row_index_destroy(shf_row_index* index) {
  HB_ENTER();
  if (!index) return SHF_HB_OK;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(index->dev);
  if (index->d_tab_slot) (void)hipFree(index->d_tab_slot);
  if (index->d_rows) (void)hipFree(index->d_rows);
  if (index->d_map8) (void)hipFree(index->d_map8);
  if (index->d_win_tab) (void)hipFree(index->d_win_tab);
  (void)hipSetDevice(prev);
  delete index;
  return SHF_HB_OK;
}

int shf_row_index_set_tabs(shf_row_index* index, const uint32_t* tab_slot) {
  HB_ENTER();
  if (!index || !tab_slot) return SHF_HB_ERR_ARG;
  index->compact = false;
  HB_TRY(hipMemcpy(index->d_tab_slot, tab_slot, SHF_ROW_INDEX_TABS * sizeof(uint32_t), hipMemcpyDefault));
  int prev = 0;
  HB_TRY(hipGetDevice(&prev));
  HB_TRY(hipSetDevice(index->dev));  // the compact copy is made on the index's device
  hipError_t e = shfhb::launch_compact_map(index->d_tab_slot, index->n_slots, index->d_map8, index->d_win_tab, nullptr);
  if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
  (void)hipSetDevice(prev);
  HB_TRY(e);
  index->compact = true;
  return SHF_HB_OK;
}

int shf_row_index_set_rows(shf_row_index* index, uint64_t first, uint64_t count, const void* rows) {
  HB_ENTER();
  if (!index || (!rows && count) || first > index->n_slots || count > index->n_slots - first) return SHF_HB_ERR_ARG;
  if (!count) return SHF_HB_OK;
  HB_TRY(hipMemcpy(index->d_rows + first * SHF_ROW_INDEX_SLOT_BYTES, rows, count * SHF_ROW_INDEX_SLOT_BYTES,
                   hipMemcpyDefault));
  return SHF_HB_OK;
}

int shf_row_index_device_ptrs(const shf_row_index* index, uint32_t** d_tab_slot, void** d_rows, uint64_t* n_slots) {
  HB_ENTER();
  if (!index) return SHF_HB_ERR_ARG;
  index->external = true;  // the caller may now write tab_slot: the probes read it directly
  if (d_tab_slot) *d_tab_slot = index->d_tab_slot;
  if (d_rows) *d_rows = index->d_rows;
  if (n_slots) *n_slots = index->n_slots;
  return SHF_HB_OK;
}

int shf_probe_batch_fixed_kernel_async(const shf_row_index* index, const void* d_keys, uint32_t key_len, uint64_t n,
                                       uint32_t seed, shf_hash128* d_hashes, shf_probe* d_probe, int kernel,
                                       void* hip_stream) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if ((!d_keys && key_len) || key_len > kMaxKeyLen || !fixed_kernel_fits(d_keys, key_len, kernel))
    return SHF_HB_ERR_ARG;
  shfhb::Sink sink;
  int rc = probe_sink(index, d_probe, d_hashes, &sink);
  if (rc) return rc;
  return device_fixed(d_keys, key_len, n, seed, sink, shfhb::kOutProbe, (hipStream_t)hip_stream, kernel, false);
}

int shf_probe_batch_fixed_async(const shf_row_index* index, const void* d_keys, uint32_t key_len, uint64_t n,
                                uint32_t seed, shf_hash128* d_hashes, shf_probe* d_probe, void* hip_stream) {
  HB_ENTER();
  return shf_probe_batch_fixed_kernel_async(index, d_keys, key_len, n, seed, d_hashes, d_probe, SHF_HB_KERNEL_AUTO,
                                            hip_stream);
}

int shf_probe_batch_var_async(const shf_row_index* index, const void* d_bytes, const uint64_t* d_offsets, uint64_t n,
                              uint32_t seed, shf_hash128* d_hashes, shf_probe* d_probe, void* hip_stream) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!d_offsets || !d_bytes) return SHF_HB_ERR_ARG;
  shfhb::Sink sink;
  int rc = probe_sink(index, d_probe, d_hashes, &sink);
  if (rc) return rc;
  return device_var(d_bytes, d_offsets, n, seed, sink, shfhb::kOutProbe, (hipStream_t)hip_stream, false);
}

int shf_probe_batch_fixed(const shf_row_index* index, const void* keys, uint32_t key_len, uint64_t n, uint32_t seed,
                          shf_hash128* hashes, shf_probe* probes, int mem) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!probes || (!keys && key_len) || key_len > kMaxKeyLen) return SHF_HB_ERR_ARG;
  shfhb::Sink sink;
  int rc = probe_sink(index, probes, hashes, &sink);
  if (rc) return rc;
  if (mem == SHF_HASH_MEM_DEVICE)
    return device_fixed(keys, key_len, n, seed, sink, shfhb::kOutProbe, nullptr, shfhb::kKernelAuto, true);
  if (mem != SHF_HASH_MEM_HOST) return SHF_HB_ERR_ARG;
  HostJob job;
  job.hash = hashes;
  job.probe = probes;
  job.index = index;
  return host_fixed((const uint8_t*)keys, key_len, n, seed, job);
}

int shf_probe_batch_var(const shf_row_index* index, const void* bytes, const uint64_t* offsets, uint64_t n,
                        uint32_t seed, shf_hash128* hashes, shf_probe* probes, int mem) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!probes || !offsets || !bytes) return SHF_HB_ERR_ARG;
  shfhb::Sink sink;
  int rc = probe_sink(index, probes, hashes, &sink);
  if (rc) return rc;
  if (mem == SHF_HASH_MEM_DEVICE) return device_var(bytes, offsets, n, seed, sink, shfhb::kOutProbe, nullptr, true);
  if (mem != SHF_HASH_MEM_HOST) return SHF_HB_ERR_ARG;
  if ((rc = check_var_lengths_host(offsets, n))) return rc;
  HostJob job;
  job.hash = hashes;
  job.probe = probes;
  job.index = index;
  return host_var((const uint8_t*)bytes, offsets, n, seed, job);
}

int shf_probe_batch_hashes_async(const shf_row_index* index, const shf_hash128* d_hashes, uint64_t n,
                                 shf_probe* d_probe, void* hip_stream) {
  HB_ENTER();
  if (n == 0) return SHF_HB_OK;
  if (!d_hashes) return SHF_HB_ERR_ARG;
  shfhb::Sink sink;
  int rc = probe_sink(index, d_probe, nullptr, &sink);
  if (rc) return rc;
  DevCtx* c = nullptr;
  if ((rc = current_ctx(&c))) return rc;
  HB_TRY(shfhb::launch_probe_hashes(d_hashes, n, sink, (hipStream_t)hip_stream));
  return SHF_HB_OK;
}

int shf_tab_copy_batch_async(const void* d_src, uint64_t src_bytes, void* d_dst, uint64_t dst_bytes,
                             shf_tab_job* d_jobs, uint32_t n_jobs, const uint16_t* d_maps, uint32_t n_maps,
                             const shf_tab_params* params, void* hip_stream) {
  HB_ENTER();
  if (n_jobs == 0) return SHF_HB_OK;
  if (!d_src || !d_dst || !d_jobs || !params) return SHF_HB_ERR_ARG;
  DevCtx* c = nullptr;
  int rc = current_ctx(&c);
  if (rc) return rc;
  HB_TRY(shfhb::launch_tab_split(d_src, src_bytes, d_dst, dst_bytes, d_jobs, n_jobs, d_maps, d_maps ? n_maps : 0,
                                 *params, (hipStream_t)hip_stream));
  return SHF_HB_OK;
}

int shf_tab_copy_batch(const void* src, uint64_t src_bytes, void* dst, uint64_t dst_bytes, shf_tab_job* jobs,
                       uint32_t n_jobs, const uint16_t* maps, uint32_t n_maps, const shf_tab_params* params, int mem) {
  HB_ENTER();
  if (n_jobs == 0) return SHF_HB_OK;
  if (!src || !dst || !jobs || !params || (mem != SHF_HASH_MEM_DEVICE && mem != SHF_HASH_MEM_HOST))
    return SHF_HB_ERR_ARG;
  DevCtx* c = nullptr;
  int rc = current_ctx(&c);
  if (rc) return rc;
  hipStream_t st = mem == SHF_HASH_MEM_DEVICE ? nullptr : c->st;  // device memory: after the caller's null-stream work
  const size_t job_bytes = (size_t)n_jobs * sizeof(shf_tab_job), map_bytes = (size_t)n_maps * 2048u * 2u;
  if (mem == SHF_HASH_MEM_DEVICE) {
    HB_TRY(shfhb::launch_tab_split(src, src_bytes, dst, dst_bytes, jobs, n_jobs, maps, maps ? n_maps : 0, *params, st));
    HB_TRY(hipStreamSynchronize(st));
    std::vector<shf_tab_job> h(n_jobs);
    HB_TRY(hipMemcpy(h.data(), jobs, job_bytes, hipMemcpyDeviceToHost));
    for (const auto& j : h)
      if (j.status != SHF_HB_OK) return SHF_HB_ERR_ARG;
    return SHF_HB_OK;
  }
  // host buffers: through temporary device copies (dst too, so bytes the copy does not write keep their values)
  TmpDevBuf d_src, d_dst, d_jobs, d_maps;
  HB_TRY(hipMalloc(&d_src.p, src_bytes ? src_bytes : 1));
  HB_TRY(hipMalloc(&d_dst.p, dst_bytes ? dst_bytes : 1));
  HB_TRY(hipMalloc(&d_jobs.p, job_bytes));
  if (maps && n_maps) HB_TRY(hipMalloc(&d_maps.p, map_bytes));
  HB_TRY(hipMemcpyAsync(d_src.p, src, src_bytes, hipMemcpyHostToDevice, st));
  HB_TRY(hipMemcpyAsync(d_dst.p, dst, dst_bytes, hipMemcpyHostToDevice, st));
  HB_TRY(hipMemcpyAsync(d_jobs.p, jobs, job_bytes, hipMemcpyHostToDevice, st));
  if (d_maps.p) HB_TRY(hipMemcpyAsync(d_maps.p, maps, map_bytes, hipMemcpyHostToDevice, st));
  HB_TRY(shfhb::launch_tab_split(d_src.p, src_bytes, d_dst.p, dst_bytes, (shf_tab_job*)d_jobs.p, n_jobs,
                                 (const uint16_t*)d_maps.p, d_maps.p ? n_maps : 0, *params, st));
  HB_TRY(hipMemcpyAsync(dst, d_dst.p, dst_bytes, hipMemcpyDeviceToHost, st));
  HB_TRY(hipMemcpyAsync(jobs, d_jobs.p, job_bytes, hipMemcpyDeviceToHost, st));
  HB_TRY(hipStreamSynchronize(st));
  for (uint32_t i = 0; i < n_jobs; ++i)
    if (jobs[i].status != SHF_HB_OK) return SHF_HB_ERR_ARG;
  return SHF_HB_OK;
}

size_t shf_win_order_workspace_bytes(uint64_t n) { return (size_t)shfhb::win_order_workspace_bytes(n); }

int shf_win_order_async(const shf_hash128* d_hashes, uint64_t n, uint32_t* d_perm, uint32_t* d_win_start,
                        void* d_workspace, size_t workspace_bytes, void* hip_stream) {
  HB_ENTER();
  if (n == 0 && !d_win_start) return SHF_HB_OK;
  if (n > 0xffffffffull) return SHF_HB_ERR_ARG;
  if (n && (!d_hashes || !d_perm || !win_workspace_ok(d_workspace, workspace_bytes, n))) return SHF_HB_ERR_ARG;
  DevCtx* c = nullptr;
  int rc = current_ctx(&c);
  if (rc) return rc;
  HB_TRY(shfhb::launch_win_order(d_hashes, n, d_perm, d_win_start, d_workspace, (hipStream_t)hip_stream));
  return SHF_HB_OK;
}

int shf_win_order(const shf_hash128* hashes, uint64_t n, uint32_t* perm, uint32_t* win_start, int mem) {
  HB_ENTER();
  if (mem != SHF_HASH_MEM_DEVICE && mem != SHF_HASH_MEM_HOST) return SHF_HB_ERR_ARG;
  if (n == 0 && !win_start) return SHF_HB_OK;
  if (n > 0xffffffffull || (n && (!hashes || !perm))) return SHF_HB_ERR_ARG;
  DevCtx* c = nullptr;
  int rc = current_ctx(&c);
  if (rc) return rc;
  // device memory: on the null stream, as the synchronous hashing calls do, so the order
  // runs after whatever the caller enqueued there (e.g. the hashes it orders)
  hipStream_t st = mem == SHF_HASH_MEM_DEVICE ? nullptr : c->st;
  const size_t ws = (size_t)shfhb::win_order_workspace_bytes(n), ws_start = 257u * sizeof(uint32_t);
  void* d_ws = nullptr;
  if ((rc = ensure_win_ws(c, ws, &d_ws))) return rc;
  TmpDevBuf d_h, d_p, d_s;
  if (mem == SHF_HASH_MEM_DEVICE) {
    HB_TRY(shfhb::launch_win_order(hashes, n, perm, win_start, d_ws, st));
    HB_TRY(hipStreamSynchronize(st));
    return SHF_HB_OK;
  }
  if (n) {
    HB_TRY(hipMalloc(&d_h.p, n * sizeof(shf_hash128)));
    HB_TRY(hipMalloc(&d_p.p, n * sizeof(uint32_t)));
    HB_TRY(hipMemcpyAsync(d_h.p, hashes, n * sizeof(shf_hash128), hipMemcpyHostToDevice, st));
  }
  if (win_start) HB_TRY(hipMalloc(&d_s.p, ws_start));
  HB_TRY(shfhb::launch_win_order(d_h.p, n, (uint32_t*)d_p.p, (uint32_t*)d_s.p, d_ws, st));
  if (n) HB_TRY(hipMemcpyAsync(perm, d_p.p, n * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  if (win_start) HB_TRY(hipMemcpyAsync(win_start, d_s.p, ws_start, hipMemcpyDeviceToHost, st));
  HB_TRY(hipStreamSynchronize(st));
  return SHF_HB_OK;
}

int shf_tab_part_redirect(uint16_t* map, uint32_t tab_old, uint32_t tab_new) {
  if (!map || tab_old >= 2048u || tab_new >= 2048u || tab_old == tab_new) return SHF_HB_ERR_ARG;
  bool second = false;  // shf.c:683-692: the 1st, 3rd, ... stay, the 2nd, 4th, ... move
  for (uint32_t tab2 = 0; tab2 < 2048u; ++tab2) {
    if (map[tab2] != tab_old) continue;
    if (second) map[tab2] = (uint16_t)tab_new;
    second = !second;
  }
  return SHF_HB_OK;
}

int shf_hash_batch_status(void* hip_stream) {
  HB_ENTER();
  DevCtx* c = nullptr;
  int rc = current_ctx(&c);
  if (rc) return rc;
  HB_TRY(hipStreamSynchronize((hipStream_t)hip_stream));
  // read and clear in one atomic exchange on the device: a kernel on another
  // stream that flags a key meanwhile leaves the word set for the next query
  HB_TRY(shfhb::launch_status_take(c->d_status, c->d_status + 2, c->st));
  HB_TRY(hipMemcpyAsync(c->h_status, c->d_status + 2, sizeof(uint32_t), hipMemcpyDeviceToHost, c->st));
  HB_TRY(hipStreamSynchronize(c->st));
  return *c->h_status ? SHF_HB_ERR_ARG : SHF_HB_OK;
}

int shf_hash_batch_device_count(void) {
  HB_ENTER();
  return visible_devices();
}

int shf_hash_batch_check_device(void) {
  HB_ENTER();
  DevCtx* c = nullptr;
  return current_ctx(&c);
}

int shf_hash_batch_last_hip_error(void) { return tls_last_hip; }

int shf_hash_batch_release(void) {
  HB_ENTER();
  free_contexts();
  std::vector<Pool*> pools;
  {
    std::lock_guard<std::mutex> g(g_pools_mu);
    for (auto& kv : g_pools) pools.push_back(kv.second);
  }
  for (Pool* p : pools) p->trim();
  return SHF_HB_OK;
}

const char* shf_hash_batch_strerror(int status) {
  switch (status) {
    case SHF_HB_OK:
      return "ok";
    case SHF_HB_ERR_ARG:
      return "invalid argument";
    case SHF_HB_ERR_NODEV:
      return "no HIP device available";
    case SHF_HB_ERR_HIP:
      return "HIP runtime error";
    case SHF_HB_ERR_NOMEM:
      return "out of device or pinned host memory";
    case SHF_HB_ERR_ARCH:
      return "device is not gfx950 (MI355X)";
    case SHF_HB_ERR_FORKED:
      return "forked after this process used the library: HIP state does not survive fork()";
    default:
      return "unknown status";
  }
}

const char* shf_hash_batch_version(void) { return "shf_hash_batch 0.1 gfx950"; }

}  // extern "C"
