// TEST INFRASTRUCTURE: unit tests of the host-only arithmetic of the host-memory
// pipelines (sharedhashfile_amd/csrc/host_plan.h), built with
// g++ -fsanitize=address,undefined by tests/c/Makefile (target `sanitize`) and
// run by tests/test_host_plan.py on the CPU. Exit status 0 = every check held;
// any sanitizer report aborts the program (-fno-sanitize-recover=all).
//
// Edge cases follow VERDICT r4 item 5: slots shorter than one key, key lengths
// and batches at the 2^31-byte limit of the reference's `const int len`
// (/root/reference/src/murmurhash3.c:75), byte totals past 2^32. (The page
// arithmetic of the pageable zero copy it also named went with that path.)
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <pthread.h>
#include <signal.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <random>
#include <thread>
#include <vector>

#include "../../sharedhashfile_amd/csrc/host_plan.h"

using namespace shfhb::plan;

static int failures = 0;
#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                    \
    }                                                                \
  } while (0)

// Regions of a layout are aligned, disjoint, in order and inside the slot.
static void check_layout(size_t slot, size_t in_bytes, uint64_t cnt, bool probe, bool offsets) {
  const SlotLayout l = slot_layout(in_bytes, cnt, probe, offsets);
  CHECK(l.out % kAlign == 0 && l.probe % kAlign == 0 && l.off % kAlign == 0 && l.end % kAlign == 0);
  CHECK(l.out >= in_bytes);
  CHECK(l.probe >= l.out + cnt * kHashBytes);
  if (probe) CHECK(l.off >= l.probe + cnt * kProbeBytes);
  if (offsets) CHECK(l.end >= l.off + (cnt + 1) * kOffBytes);
  CHECK(l.end <= slot);
}

static void test_fixed_chunks() {
  const size_t slots[] = {kMinSlotBytes, (size_t)1 << 20, (size_t)16 << 20, ((size_t)16 << 20) + 4096 + 17};
  const uint32_t lens[] = {0, 1, 7, 15, 16, 17, 255, 256, 511, 4096, 65535, 1u << 20, (1u << 24) - 1};
  for (size_t slot : slots)
    for (uint32_t L : lens)
      for (int probe = 0; probe < 2; ++probe) {
        const uint64_t c = fixed_chunk_keys(slot, L, probe);
        if (c) {
          check_layout(slot, (size_t)c * L, c, probe, false);
          // maximal: one more key does not fit
          CHECK(slot_layout((size_t)(c + 1) * L, c + 1, probe, false).end > slot);
        } else {
          CHECK(slot_layout(L, 1, probe, false).end > slot);  // not even one key: the big-key path
        }
      }
  // the default slot holds the round-4 chunk of 16-B keys (8 MiB of keys)
  CHECK(fixed_chunk_keys((size_t)16 << 20, 16, false) == ((size_t)16 << 20) / 32);
  // 8-B UID parts instead of 16-B records: a third more 16-B keys per slot, every layout inside it
  {
    const uint64_t c8 = fixed_chunk_keys((size_t)16 << 20, 16, false, 8);
    CHECK(c8 <= ((size_t)16 << 20) / 24 && c8 + 64 >= ((size_t)16 << 20) / 24);
  }
  for (size_t slot : slots)
    for (uint32_t L : lens) {
      const uint64_t c = fixed_chunk_keys(slot, L, false, 8);
      if (!c) continue;
      const SlotLayout l = slot_layout((size_t)c * L, c, false, false, 8);
      CHECK(l.out % kAlign == 0 && l.end % kAlign == 0 && l.end <= slot && l.probe >= l.out + c * 8);
      CHECK(slot_layout((size_t)(c + 1) * L, c + 1, false, false, 8).end > slot);
    }
  // even chunks: never more chunks than the slot size forces, none above it, sizes within one chunk's rounding
  for (uint64_t most : {1ull, 7ull, 512ull << 10, 1000003ull})
    for (uint64_t n : {1ull, 6ull, 7ull, 8ull, 625000ull, 10000000ull, 1000000007ull}) {
      const uint64_t c = even_chunk(n, most);
      const uint64_t chunks = (n + c - 1) / c;
      CHECK(c >= 1 && c <= most && chunks == (n + most - 1) / most);
      CHECK(n - (chunks - 1) * c <= c && n - (chunks - 1) * c + chunks > c);  // the last chunk is about as big
    }
  CHECK(even_chunk(100, 0) == 0 && even_chunk(0, 5) == 1);
  // a key at the reference's limit never fits a slot
  CHECK(fixed_chunk_keys((size_t)16 << 20, 0x7fffffffu, false) == 0);
  CHECK(fixed_chunk_keys(2 * kAlign - 1, 1, false) == 0);  // not even the key's own 256-B region and its record
}

// Walks a batch the way host_var_run does and checks every chunk.
static void walk_var(const std::vector<uint64_t>& off, size_t slot, bool probe) {
  const uint64_t n = off.size() - 1;
  uint64_t i0 = 0, chunks = 0;
  while (i0 < n) {
    bool alone = false;
    const uint64_t i1 = var_chunk_end(off.data(), i0, n, slot, probe, &alone);
    CHECK(i1 > i0 && i1 <= n);
    if (i1 <= i0 || i1 > n) return;
    const uint64_t nb = off[i1] - off[i0];
    if (alone) {
      CHECK(i1 == i0 + 1);
      CHECK(slot_layout(nb, 1, probe, true).end > slot);  // really too long for the slot
      check_layout(slot, 0, 1, probe, true);             // its record and offsets still fit
    } else {
      check_layout(slot, nb, i1 - i0, probe, true);
      if (i1 < n) CHECK(slot_layout(off[i1 + 1] - off[i0], i1 + 1 - i0, probe, true).end > slot);  // maximal
    }
    i0 = i1;
    ++chunks;
  }
  CHECK(i0 == n);
  // the estimate a call leases slots by: never more than one below the chunks actually cut, and above
  // them only by what keys too long for a slot add (each is cut alone, its bytes staged elsewhere)
  const uint64_t est = var_chunks_estimate(off[n] - off[0], n, slot, probe);
  uint64_t alone_bytes = 0;
  for (uint64_t i = 0; i < n; ++i)
    if (slot_layout(off[i + 1] - off[i], 1, probe, true).end > slot) alone_bytes += off[i + 1] - off[i];
  CHECK(est >= 1 && est + 1 >= chunks);
  CHECK(est <= chunks + 1 + alone_bytes / (slot / 2));
}

static void test_var_chunks() {
  std::mt19937_64 rng(5);
  const size_t slot = (size_t)1 << 20;
  for (int probe = 0; probe < 2; ++probe) {
    // U[8,512] keys, zero-length keys, one key of every size around the slot
    std::vector<uint64_t> off{0};
    for (int i = 0; i < 20000; ++i) off.push_back(off.back() + 8 + rng() % 505);
    walk_var(off, slot, probe);
    std::vector<uint64_t> zeros(100001, 123);  // 100000 empty keys starting at byte 123
    walk_var(zeros, slot, probe);
    for (uint64_t big : {slot - 1024, slot - 256, slot, slot + 1, (uint64_t)0x7fffffff}) {
      std::vector<uint64_t> o{0, 10, 10 + big, 20 + big, 20 + big, 21 + big};
      walk_var(o, slot, probe);
    }
    // lengths at the reference's limit, batches whose byte total passes 2^32 (only offsets are read)
    std::vector<uint64_t> huge{0};
    for (int i = 0; i < 5; ++i) huge.push_back(huge.back() + 0x7fffffffu);
    walk_var(huge, slot, probe);
    std::vector<uint64_t> one{(uint64_t)1 << 40, ((uint64_t)1 << 40) + 7};
    walk_var(one, kMinSlotBytes, probe);
  }
}

// The staging copies' streaming memcpy: every length 0..600 and some long ones,
// at every source and destination offset within 64 B, into exact-size heap
// buffers (ASan reports any byte written or read outside them).
static void test_stream_copy() {
  if (!__builtin_cpu_supports("avx2")) {
    printf("stream_copy: no AVX2 on this CPU, skipped\n");
    return;
  }
  std::mt19937 rng(9);
  std::vector<size_t> lens;
  for (size_t n = 0; n <= 600; ++n) lens.push_back(n);
  for (size_t n : {4095, 4096, 4097, 65536 + 31, 1000003}) lens.push_back(n);
  for (size_t n : lens)
    for (size_t so = 0; so < 64; so += (n > 600 ? 13 : 5))
      for (size_t dof = 0; dof < 64; dof += (n > 600 ? 11 : 7)) {
        char* src = (char*)malloc(n + so + 1);
        char* dst = (char*)malloc(n + dof + 1);
        for (size_t i = 0; i < n + so + 1; ++i) src[i] = (char)rng();
        memset(dst, 0x5a, n + dof + 1);
        stream_copy_avx2(dst + dof, src + so, n);
        CHECK(memcmp(dst + dof, src + so, n) == 0);
        bool guard = dst[n + dof] == 0x5a;
        for (size_t i = 0; i < dof; ++i) guard = guard && dst[i] == 0x5a;
        CHECK(guard);  // nothing outside [dof, dof + n) written
        free(src);
        free(dst);
      }
}

// The pool under 16 threads: never more than max_slots slots alive, never one
// slot lent twice, sizes changed while slots are on loan, failing allocations.
struct FakeSlot {
  size_t bytes = 0;
  std::atomic<int> owners{0};
  char* mem = nullptr;
};

static void test_pool() {
  std::atomic<int> alive{0}, peak{0}, made{0}, fail_next{0};
  SlotPool<FakeSlot> pool(
      [&](size_t bytes, FakeSlot** out) {
        if (fail_next.exchange(0)) return -4;
        FakeSlot* s = new FakeSlot();
        s->bytes = bytes;
        s->mem = (char*)malloc(bytes);
        memset(s->mem, 0, bytes);
        const int a = ++alive;
        int p = peak.load();
        while (a > p && !peak.compare_exchange_weak(p, a)) {
        }
        ++made;
        *out = s;
        return 0;
      },
      [&](FakeSlot* s) {
        CHECK(s->owners.load() == 0);
        free(s->mem);
        delete s;
        --alive;
      });
  const int kMax = 4;
  std::vector<std::thread> ts;
  std::atomic<int> errors{0};
  for (int t = 0; t < 16; ++t)
    ts.emplace_back([&, t] {
      std::mt19937 rng(t);
      for (int it = 0; it < 400; ++it) {
        FakeSlot* got[4] = {};
        int n = 0;
        const size_t bytes = (it / 100 % 2) ? 8192 : 4096;  // sizes change while others hold slots
        if (t == 3 && it % 50 == 0) fail_next = 1;
        const int rc = pool.acquire(bytes, 1 + rng() % 4, kMax, got, &n);
        if (rc) {
          ++errors;
          CHECK(n == 0);
          continue;
        }
        CHECK(n >= 1 && n <= 4);
        for (int i = 0; i < n; ++i) {
          CHECK(got[i]->bytes == bytes);
          CHECK(got[i]->owners.fetch_add(1) == 0);  // lent to nobody else
          got[i]->mem[rng() % bytes] = (char)t;      // ASan: inside the slot's arena
        }
        std::this_thread::yield();
        for (int i = 0; i < n; ++i) got[i]->owners.fetch_sub(1);
        pool.release(got, n);
      }
    });
  for (auto& t : ts) t.join();
  CHECK(peak.load() <= kMax);
  CHECK(pool.live() == alive.load());
  CHECK(pool.live() <= kMax);
  pool.trim();
  CHECK(alive.load() == 0 && pool.live() == 0);
  // a smaller cap after use: extra slots are freed as they come back
  FakeSlot* got[4] = {};
  int n = 0;
  CHECK(pool.acquire(4096, 4, 4, got, &n) == 0 && n == 4);
  pool.release(got, 2);
  FakeSlot* one[4] = {};
  int m = 0;
  CHECK(pool.acquire(4096, 4, 1, one, &m) == 0 && m >= 1);  // idle slots are lent even above the new cap
  pool.release(got + 2, 2);
  pool.release(one, m);
  CHECK(pool.live() <= 1);
  pool.trim();
  CHECK(alive.load() == 0);
  // while a call waits for its first slot, a returning borrower's slots go one per caller:
  // A holds all four; B waits; A gives two back; C then gets only one (B is served first or
  // B takes one of them and C the other), never both.
  {
    FakeSlot* a[4] = {};
    int na = 0;
    CHECK(pool.acquire(4096, 4, 4, a, &na) == 0 && na == 4);
    std::atomic<int> nb{-1};
    FakeSlot* b[4] = {};
    std::thread tb([&] {
      int k = 0;
      CHECK(pool.acquire(4096, 4, 4, b, &k) == 0);
      nb = k;
    });
    while (true) {  // until B is waiting
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
      if (pool.waiting() == 1) break;
    }
    pool.release(a, 2);
    tb.join();
    CHECK(nb.load() >= 1 && nb.load() <= 2);
    pool.release(a + 2, 2);
    pool.release(b, nb.load());
    pool.trim();
    CHECK(alive.load() == 0);
  }
  printf("pool: %d slots made, peak %d alive, %d injected failures\n", made.load(), peak.load(), errors.load());
}

// The copy workers under 16 calling threads at once, as the library uses them:
// run() (a staging copy split over the workers, the caller doing piece 0) mixed
// with submit() (a copy-out handed off, joined later through its Ticket, the
// first failing piece's status kept); every piece runs exactly once, and a
// Ticket outlives the caller's own wait (the library's Pending waits in its
// destructor). ThreadSanitizer checks the queue and the latches.
static void test_copy_pool() {
  static CopyPool* pool = new CopyPool();  // never destroyed, as in the library
  std::vector<std::thread> ts;
  std::atomic<int> bad{0};
  for (int t = 0; t < 16; ++t)
    ts.emplace_back([&, t] {
      std::mt19937 rng(100 + t);
      std::vector<std::shared_ptr<Ticket>> held;
      for (int it = 0; it < 300; ++it) {
        const size_t k = 1 + rng() % 12;
        std::vector<int> hits(k, 0);
        if (it % 3 == 0) {
          std::vector<std::function<void()>> pieces;
          for (size_t i = 0; i < k; ++i) pieces.emplace_back([&hits, i] { ++hits[i]; });
          pool->run(pieces);
          for (size_t i = 0; i < k; ++i)
            if (hits[i] != 1) ++bad;
        } else {
          auto out = std::make_shared<std::vector<int>>(k, 0);
          const int fail_at = (it % 7 == 0) ? (int)(rng() % k) : -1;
          std::vector<std::function<int()>> pieces;
          for (size_t i = 0; i < k; ++i)
            pieces.emplace_back([out, i, fail_at] {
              ++(*out)[i];
              return (int)i == fail_at ? -3 : 0;
            });
          auto tk = pool->submit(std::move(pieces));
          if (it % 2) {  // joined now
            const int rc = tk->wait();
            if (rc != (fail_at >= 0 ? -3 : 0)) ++bad;
            for (size_t i = 0; i < k; ++i)
              if ((*out)[i] != 1) ++bad;
          } else {
            held.push_back(tk);  // joined later, after more batches went through
          }
        }
      }
      for (auto& tk : held) {
        const int rc = tk->wait();
        if (rc != 0 && rc != -3) ++bad;
      }
    });
  for (auto& t : ts) t.join();
  CHECK(bad.load() == 0);
  CHECK(pool->workers() <= 12);  // never more workers than the largest batch asked for
  auto empty = pool->submit({});
  CHECK(empty->wait() == 0);
  pool->run({});
  // no worker can be started (a system that refuses threads, here a pool capped at 0):
  // both forms run every piece on the caller and return with it done
  CopyPool none(0);
  std::vector<int> hit(5, 0);
  std::vector<std::function<void()>> rp;
  for (int i = 0; i < 5; ++i) rp.emplace_back([&hit, i] { ++hit[i]; });
  none.run(rp);
  std::vector<std::function<int()>> sp;
  for (int i = 0; i < 5; ++i) sp.emplace_back([&hit, i] { ++hit[i]; return i == 3 ? -7 : 0; });
  auto tk = none.submit(std::move(sp));
  CHECK(tk->wait() == -7);
  for (int i = 0; i < 5; ++i) CHECK(hit[i] == 2);
  CHECK(none.workers() == 0);
  printf("copy pool: %zu workers, 16 threads x 300 batches\n", pool->workers());
}

// fork() after the copy workers have run (the reference
// forks up to 36 load-test workers, /root/reference/src/test.f.shf.c:274-336):
// with the pool's pthread_atfork handlers registered, a child forked while
// another thread keeps the workers busy finishes run() and submit() on its own
// thread and exits 0 within a time limit, instead of waiting forever on
// workers it does not have; the parent's pool keeps working.
static CopyPool* g_fork_pool = nullptr;
static void fork_prepare() { g_fork_pool->fork_prepare(); }
static void fork_parent() { g_fork_pool->fork_parent(); }
static void fork_child() { g_fork_pool->fork_child(); }

static bool pool_round(CopyPool* pool, size_t k) {
  std::vector<int> hits(k, 0);
  std::vector<std::function<void()>> pieces;
  for (size_t i = 0; i < k; ++i) pieces.emplace_back([&hits, i] { ++hits[i]; });
  pool->run(pieces);
  auto out = std::make_shared<std::vector<int>>(k, 0);
  std::vector<std::function<int()>> sp;
  for (size_t i = 0; i < k; ++i) sp.emplace_back([out, i] { ++(*out)[i]; return i == 1 ? -5 : 0; });
  const int rc = pool->submit(std::move(sp))->wait();
  bool ok = rc == (k > 1 ? -5 : 0);
  for (size_t i = 0; i < k; ++i) ok = ok && hits[i] == 1 && (*out)[i] == 1;
  return ok;
}

static void test_fork() {
  g_fork_pool = new CopyPool();  // never destroyed, as in the library
  CHECK(pthread_atfork(fork_prepare, fork_parent, fork_child) == 0);
  CHECK(pool_round(g_fork_pool, 8));
  CHECK(g_fork_pool->workers() >= 7);  // the parent has workers the child will not have
  std::atomic<bool> stop{false};
  std::atomic<long> busy_rounds{0};
  std::thread busy([&] {  // the workers stay busy (queue and latches in use) across every fork
    while (!stop.load()) {
      if (!pool_round(g_fork_pool, 6)) ++failures;
      ++busy_rounds;
    }
  });
  for (int round = 0; round < 8; ++round) {
    const pid_t pid = fork();
    if (pid == 0) {
      // the child: no workers, every piece on this thread; then the same again
      const bool ok = g_fork_pool->forked() && pool_round(g_fork_pool, 8) && pool_round(g_fork_pool, 1) &&
                      g_fork_pool->workers() == 0 && pool_round(g_fork_pool, 12);
      _exit(ok ? 0 : 3);
    }
    CHECK(pid > 0);
    if (pid <= 0) break;
    int status = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const pid_t r = waitpid(pid, &status, WNOHANG);
      if (r == pid) break;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
        kill(pid, SIGKILL);
        waitpid(pid, &status, 0);
        fprintf(stderr, "fork: child %d hung\n", (int)pid);
        ++failures;
        break;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
    }
    CHECK(WIFEXITED(status) && WEXITSTATUS(status) == 0);
  }
  stop = true;
  busy.join();
  CHECK(!g_fork_pool->forked() && pool_round(g_fork_pool, 12));  // the parent's pool is unchanged
  printf("fork: 8 children finished on their own thread, %ld parent rounds alongside\n", busy_rounds.load());
}

// Idle workers end (the copy workers never stopped): a pool
// whose workers find no piece for `idle` has none left, and the next batch
// starts them again; under TSan, batches racing the workers' exits.
static void test_idle_workers_end() {
  static CopyPool* pool = new CopyPool((size_t)-1, std::chrono::milliseconds(20));  // reachable: not a leak
  for (int round = 0; round < 3; ++round) {
    CHECK(pool_round(pool, 8));
    CHECK(pool->workers() >= 7);
    const auto t0 = std::chrono::steady_clock::now();
    while (pool->workers() != 0 && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10))
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    CHECK(pool->workers() == 0);
  }
  // batches that arrive just as workers give up: every piece still runs exactly once
  std::vector<std::thread> ts;
  std::atomic<int> bad{0};
  for (int t = 0; t < 4; ++t)
    ts.emplace_back([&, t] {
      std::mt19937 rng(300 + t);
      for (int it = 0; it < 40; ++it) {
        if (!pool_round(pool, 1 + rng() % 10)) ++bad;
        std::this_thread::sleep_for(std::chrono::milliseconds(rng() % 30));
      }
    });
  for (auto& t : ts) t.join();
  CHECK(bad.load() == 0);
  const auto t0 = std::chrono::steady_clock::now();
  while (pool->workers() != 0 && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10))
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  CHECK(pool->workers() == 0);
  // every worker has left work() once the count is 0 ... but may still be returning from it:
  // the pool is deliberately not destroyed (as in the library)
  printf("idle workers: ended after each batch, 4 threads x 40 batches racing their exits\n");
}

int main() {
  test_fixed_chunks();
  test_var_chunks();
  test_stream_copy();
  test_pool();
  test_copy_pool();
  test_fork();
  test_idle_workers_end();
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("host_plan: all checks passed\n");
  return 0;
}
