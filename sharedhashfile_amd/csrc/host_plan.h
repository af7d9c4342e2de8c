// Host-only arithmetic of the host-memory pipelines (shf_hash_batch.hip), kept
// free of HIP so that it compiles with g++ -fsanitize=address,undefined and is
// unit-tested on the CPU (tests/c/test_host_plan.cpp, tests/test_host_plan.py):
//
//   * slot_layout / fixed_chunk_keys / var_chunk_end / var_chunks_estimate: how one chunk of keys, its
//     hash records, probe records and offsets are carved out of one staging slot
//     (a pinned host arena and a device arena of the same size);
//   * stream_copy_avx2: the staging copies' non-temporal memcpy;
//   * SlotPool: the per-device pool of staging slots that every calling thread
//     borrows from (a bounded footprint per process, not per thread);
//   * CopyPool / Ticket: the staging copies' worker threads, with batches run
//     in place (run) or handed off and joined later (submit, Ticket::wait).
//
// Key lengths follow the reference's contract: MurmurHash3_x64_128 takes
// `const int len` (/root/reference/src/murmurhash3.c:75), so a key is < 2^31 B;
// variable-length batches are validated (offsets non-decreasing, lengths < 2^31)
// before any of this runs (check_var_lengths_host).
#pragma once
#include <immintrin.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

namespace shfhb {
namespace plan {

constexpr size_t kAlign = 256;  // every region of a slot starts 256-B aligned (16-B kernel loads, whole lines)
constexpr size_t kMinSlotBytes = (size_t)64 << 10;
constexpr size_t kHashBytes = 16, kProbeBytes = 16, kOffBytes = 8;

inline size_t align_up(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

// Byte offsets of one chunk's buffers inside a slot arena: keys at 0, then the
// output records (rec bytes each: 16-B hashes, or 8-B UID parts), the probe
// records (when asked) and the cnt + 1 offsets (when asked).
struct SlotLayout {
  size_t out = 0, probe = 0, off = 0, end = 0;
};

inline SlotLayout slot_layout(size_t in_bytes, uint64_t cnt, bool probe, bool offsets, size_t rec = kHashBytes) {
  SlotLayout l;
  size_t o = align_up(in_bytes);
  l.out = o;
  o += align_up((size_t)cnt * rec);
  l.probe = o;
  if (probe) o += align_up((size_t)cnt * kProbeBytes);
  l.off = o;
  if (offsets) o += align_up(((size_t)cnt + 1) * kOffBytes);
  l.end = o;
  return l;
}

// Most fixed-length keys of key_len bytes one slot of slot_bytes holds with
// their records; 0 when not even one does (the key then goes through a
// temporary device buffer of its own).
inline uint64_t fixed_chunk_keys(size_t slot_bytes, uint32_t key_len, bool probe, size_t rec = kHashBytes) {
  const size_t per = (size_t)key_len + rec + (probe ? kProbeBytes : 0);
  auto fits = [&](uint64_t c) { return slot_layout((size_t)c * key_len, c, probe, false, rec).end <= slot_bytes; };
  if (!fits(1)) return 0;
  // within a few keys of the answer (the regions' alignment costs at most 3 x kAlign bytes)
  uint64_t c = slot_bytes > 3 * kAlign ? std::max<uint64_t>(1, (slot_bytes - 3 * kAlign) / per) : 1;
  while (c > 1 && !fits(c)) --c;
  while (fits(c + 1)) ++c;
  return c;
}

// Keys per chunk when n keys go in chunks of at most `most`: as few chunks as
// that allows, of equal size (the last one never a sliver that drains the
// pipeline alone). 0 when most is 0.
inline uint64_t even_chunk(uint64_t n, uint64_t most) {
  if (!most || !n) return most ? 1 : 0;
  const uint64_t chunks = (n + most - 1) / most;
  return (n + chunks - 1) / chunks;
}

// Variable-length keys from key i0 (offsets[i0..n] non-decreasing): the end i1 of
// the longest chunk [i0, i1) whose key bytes, records and offsets fit one slot.
// A single key too long for the slot gives i1 = i0 + 1 with *alone = true: its
// bytes go through a temporary device buffer, its record and offsets through the slot.
inline uint64_t var_chunk_end(const uint64_t* offsets, uint64_t i0, uint64_t n, size_t slot_bytes, bool probe,
                              bool* alone, size_t rec = kHashBytes) {
  const uint64_t base = offsets[i0];
  // each key costs at least its record and offset: no chunk holds more keys than this
  const uint64_t cap = std::max<uint64_t>(1, slot_bytes / (rec + kOffBytes));
  uint64_t lo = i0 + 1, hi = std::min(n, i0 + std::min(cap, n - i0));
  auto fits = [&](uint64_t i1) {
    return slot_layout(offsets[i1] - base, i1 - i0, probe, true, rec).end <= slot_bytes;
  };
  *alone = !fits(lo);
  if (*alone) return lo;
  // largest i1 in [lo, hi] that fits (fits() is monotone: offsets never decrease)
  while (lo < hi) {
    const uint64_t mid = lo + (hi - lo + 1) / 2;
    if (fits(mid))
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

// About how many chunks var_chunk_end cuts a batch of n keys and key_bytes bytes
// into (at least 1): what a call asks the pool for, no more slots than it can use.
inline uint64_t var_chunks_estimate(uint64_t key_bytes, uint64_t n, size_t slot_bytes, bool probe,
                                    size_t rec = kHashBytes) {
  const uint64_t per_key = rec + kOffBytes + (probe ? kProbeBytes : 0);
  const uint64_t room = slot_bytes > 4 * kAlign ? slot_bytes - 4 * kAlign : 1;
  uint64_t need = 0;
  if (__builtin_mul_overflow(n, per_key, &need) || __builtin_add_overflow(need, key_bytes, &need)) return UINT64_MAX;
  return std::max<uint64_t>(1, (need + room - 1) / room);
}

// memcpy with non-temporal 32-B stores (the CPU must have AVX2): head bytes up
// to the destination's next 32-B boundary and the last n % 128 bytes by
// memcpy, 128 B per step between them; an sfence at the end makes the streamed
// lines visible before the caller hands the buffer on (a DMA, the caller).
__attribute__((target("avx2"))) inline void stream_copy_avx2(void* dst, const void* src, size_t n) {
  char* d = static_cast<char*>(dst);
  const char* s = static_cast<const char*>(src);
  const size_t head = std::min(n, (size_t)((32u - (reinterpret_cast<uintptr_t>(d) & 31u)) & 31u));
  memcpy(d, s, head);
  d += head, s += head, n -= head;
  for (size_t k = n / 128; k; --k, d += 128, s += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + 64));
    const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d), a);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + 96), e);
  }
  memcpy(d, s, n & 127u);
  _mm_sfence();
}

// A bounded pool of staging slots, shared by every thread of the process that
// stages host memory for one device. A call borrows between one and `want`
// slots: the first blocks until a slot is free (or may be made), the others are
// taken only if free right now and no other call is waiting, so no caller ever
// waits while holding slots, slots spread over the callers under contention, and
// the pool cannot deadlock (as long as no caller borrows again while it holds
// slots: the library never nests its leases). Slots are made lazily, at most max_slots of them at
// once, and one of another size (SHF_HB_STAGE_MB changed) is remade on reuse.
// Slot must have a `size_t bytes` member; make/unmake allocate and free one.
template <class Slot>
class SlotPool {
 public:
  using Make = std::function<int(size_t bytes, Slot** out)>;
  using Unmake = std::function<void(Slot*)>;

  SlotPool(Make make, Unmake unmake) : make_(std::move(make)), unmake_(std::move(unmake)) {}

  // Borrows 1..want slots of `bytes` each into out[]; returns 0 and their number in *got,
  // or the first error of `make` (then nothing is held). A slot counts against max_slots
  // from the moment it is to be made until it has been freed, so the memory the pool
  // holds never exceeds max_slots slots, even while sizes change.
  int acquire(size_t bytes, int want, int max_slots, Slot** out, int* got) {
    *got = 0;
    max_slots = std::max(1, max_slots);
    for (;;) {
      std::vector<Slot*> stale;
      int to_make = 0;
      {
        std::unique_lock<std::mutex> lk(mu_);
        max_slots_ = max_slots;
        bytes_ = bytes;
        auto can = [&] { return !idle_.empty() || live_ < max_slots_; };
        ++waiting_;
        cv_.wait(lk, can);
        --waiting_;
        // beyond its first slot a call takes more only while no other call waits for one: under
        // contention the slots spread over the callers (one chunk in flight each) instead of
        // deepening one caller's pipeline while the others queue
        while (*got + to_make < want && can() && (*got + to_make == 0 || waiting_ == 0)) {
          if (!idle_.empty()) {
            Slot* s = idle_.back();
            idle_.pop_back();
            if (s->bytes != bytes)
              stale.push_back(s);  // freed below, still counted until then
            else
              out[(*got)++] = s;
          } else {
            ++live_;
            ++to_make;
          }
        }
      }
      forget(stale);
      int rc = 0;
      for (; to_make > 0; --to_make) {
        Slot* s = nullptr;
        const int r = rc ? rc : make_(bytes, &s);
        if (r) {
          rc = r;
          std::lock_guard<std::mutex> lk(mu_);
          --live_;
          cv_.notify_all();
          continue;
        }
        out[(*got)++] = s;
      }
      if (*got) return 0;  // with fewer slots than wanted if some could not be made
      if (rc) return rc;
      // only stale slots were found: they are freed now, try again
    }
  }

  // Returns slots to the pool (their work must be finished); a slot of a stale
  // size, or above the current cap, is freed instead.
  void release(Slot** s, int n) {
    std::vector<Slot*> drop;
    {
      std::lock_guard<std::mutex> lk(mu_);
      int live_after = live_;  // live_ itself drops once forget() has freed them
      for (int i = 0; i < n; ++i) {
        if (s[i]->bytes != bytes_ || live_after > max_slots_) {
          drop.push_back(s[i]);
          --live_after;
        } else {
          idle_.push_back(s[i]);
        }
      }
    }
    cv_.notify_all();
    forget(drop);
  }

  // Frees every idle slot (slots on loan come back later and are kept).
  void trim() {
    std::vector<Slot*> drop;
    {
      std::lock_guard<std::mutex> lk(mu_);
      drop.swap(idle_);
    }
    forget(drop);
  }

  int live() {
    std::lock_guard<std::mutex> lk(mu_);
    return live_;
  }
  int idle() {
    std::lock_guard<std::mutex> lk(mu_);
    return (int)idle_.size();
  }
  int waiting() {
    std::lock_guard<std::mutex> lk(mu_);
    return waiting_;
  }

 private:
  Make make_;
  Unmake unmake_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Slot*> idle_;
  int live_ = 0;  // slots being made, idle, on loan or being freed
  int waiting_ = 0;  // calls waiting for their first slot
  int max_slots_ = 1;
  size_t bytes_ = 0;

  // Frees slots taken out of the pool, then stops counting them.
  void forget(std::vector<Slot*>& v) {
    if (v.empty()) return;
    for (Slot* x : v) unmake_(x);
    {
      std::lock_guard<std::mutex> lk(mu_);
      live_ -= (int)v.size();
    }
    cv_.notify_all();
    v.clear();
  }
};

// A batch of pieces handed to a CopyPool's workers: wait() returns once every
// piece has run, with the first non-zero status a piece returned.
struct Ticket {
  std::mutex m;
  std::condition_variable cv;
  size_t left = 0;
  int rc = 0;
  void done(int r) {
    std::lock_guard<std::mutex> lk(m);
    if (r && !rc) rc = r;
    if (--left == 0) cv.notify_all();
  }
  int wait() {
    std::unique_lock<std::mutex> lk(m);
    cv.wait(lk, [&] { return left == 0; });
    return rc;
  }
};

// Worker threads for the staging copies, shared by every calling thread: a
// worker is started when a batch has more pieces than there are workers, parks
// on the queue between batches and ends after `idle` without a piece (the
// library keeps one pool for the process's life; its workers live only while
// the process hashes). submit() returns at once with a Ticket; run() runs
// pieces[0] on the caller and returns when every piece has run.
//
// fork(): a child has only the forking thread, so the parent's workers do not
// exist there. The pool's pthread_atfork handlers (fork_prepare / fork_parent /
// fork_child, registered by whoever owns the pool) hold the queue's lock across
// the fork, so the child inherits a consistent queue; the child then drops the
// queued pieces (their callers are not in the child), forgets the workers, makes
// a fresh condition variable (the old one may count waiters that are gone) and
// never starts a worker again: every later piece runs on its caller. Without
// this a child's run() queued its pieces to workers that do not exist and
// waited on its latch forever (the reference forks its load-test
// workers, /root/reference/src/test.f.shf.c:274-336).
class CopyPool {
 public:
  // idle: a worker that finds no piece for this long ends (a later batch starts
  // workers again), so a process that stops hashing keeps no copy threads.
  explicit CopyPool(size_t max_workers = (size_t)-1, std::chrono::milliseconds idle = std::chrono::seconds(10))
      : max_workers_(max_workers), idle_(idle) {}

  std::shared_ptr<Ticket> submit(std::vector<std::function<int()>> pieces) {
    auto t = std::make_shared<Ticket>();
    t->left = pieces.size();
    if (pieces.empty()) return t;
    bool queued = false;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (grow(pieces.size())) {
        for (auto& f : pieces) q_.push_back([t, f] { t->done(f()); });
        pieces.clear();
        queued = true;
      }
    }
    for (auto& f : pieces) t->done(f());  // no worker could be started: on the caller, now
    if (queued) cv_.notify_all();
    return t;
  }

  void run(const std::vector<std::function<void()>>& pieces) {
    if (pieces.empty()) return;
    struct Latch {
      std::mutex m;
      std::condition_variable cv;
      size_t left;
    } latch;
    latch.left = pieces.size() - 1;
    bool alone = false;
    {
      std::lock_guard<std::mutex> lk(mu_);
      alone = pieces.size() > 1 && !grow(pieces.size() - 1);  // no worker could be started
      for (size_t i = 1; i < pieces.size() && !alone; ++i) {
        const std::function<void()>* f = &pieces[i];
        q_.push_back([f, &latch] {
          (*f)();
          std::lock_guard<std::mutex> l2(latch.m);
          if (--latch.left == 0) latch.cv.notify_one();
        });
      }
    }
    if (alone) {  // every piece on the caller
      for (auto& f : pieces) f();
      return;
    }
    cv_.notify_all();
    pieces[0]();
    std::unique_lock<std::mutex> lk(latch.m);
    latch.cv.wait(lk, [&] { return latch.left == 0; });
  }

  size_t workers() {
    std::lock_guard<std::mutex> lk(mu_);
    return workers_;
  }

  // pthread_atfork handlers (see the class comment). fork_prepare runs in the
  // forking thread before fork(), fork_parent after it in the parent,
  // fork_child in the child (where only the forking thread exists).
  void fork_prepare() { mu_.lock(); }
  void fork_parent() { mu_.unlock(); }
  void fork_child() {
    // the queued pieces belong to callers that are not in this process: dropped
    // without running (nobody here waits for their Tickets or latches)
    q_.clear();
    workers_ = 0;
    forked_ = true;
    new (&cv_) std::condition_variable();  // the inherited one may count waiters that do not exist here
    mu_.unlock();
  }
  bool forked() {
    std::lock_guard<std::mutex> lk(mu_);
    return forked_;
  }

 private:
  // Under mu_: starts workers up to `want`; returns how many there are (a thread the
  // system refuses is left out, and what is queued runs on those that exist). A
  // forked child starts none: its pieces run on their callers.
  size_t grow(size_t want) {
    if (forked_) return 0;
    while (workers_ < want && workers_ < max_workers_) {
      try {
        std::thread([this] { work(); }).detach();
      } catch (...) {
        break;
      }
      ++workers_;
    }
    return workers_;
  }
  void work() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        // (a system_clock deadline: libstdc++ waits on it with pthread_cond_timedwait, which
        // ThreadSanitizer follows; a steady_clock wait_for uses pthread_cond_clockwait, which
        // gcc 11's TSan does not intercept -- it then reports false double locks)
        if (!cv_.wait_until(lk, std::chrono::system_clock::now() + idle_, [&] { return !q_.empty(); })) {
          // idle: end this worker (the count drops under the lock, so a batch queued
          // from now on starts a worker of its own; one queued before was seen above)
          --workers_;
          return;
        }
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  size_t workers_ = 0;
  const size_t max_workers_;
  const std::chrono::milliseconds idle_;
  bool forked_ = false;
};

}  // namespace plan
}  // namespace shfhb
