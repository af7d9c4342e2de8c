// Round 6 probe: where the host pipeline's pageable H2D loses against one big
// copy (48 vs 56 GB/s, profiles/r6/host_uid/). Times hipMemcpyAsync from a
// pageable buffer into HBM, 160 MB in total:
//   one   : one call;
//   seqN  : N chunks, one thread, each call on the next of 4 streams (the pipeline's shape);
//   altN  : N chunks alternating between two threads (each its own pair of streams), so one
//           thread's per-call setup can overlap the other's transfer.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/pageable_chunk_probe tools/pageable_chunk_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t total = 160u * 1000u * 1000u;
  uint8_t* h = (uint8_t*)malloc(total);
  memset(h, 1, total);
  uint8_t* d = nullptr;
  CHECK(hipMalloc((void**)&d, total));
  hipStream_t st[4];
  for (auto& s : st) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto sync_all = [&] {
    for (auto& s : st) CHECK(hipStreamSynchronize(s));
  };
  auto run = [&](int chunks, bool alt) {
    const size_t per = (total + chunks - 1) / chunks;
    sync_all();
    const double t0 = now();
    if (!alt) {
      for (int i = 0; i < chunks; ++i) {
        const size_t a = i * per, b = std::min(total, a + per);
        CHECK(hipMemcpyAsync(d + a, h + a, b - a, hipMemcpyHostToDevice, st[i % 4]));
      }
    } else {
      std::thread t1([&] {
        for (int i = 1; i < chunks; i += 2) {
          const size_t a = i * per, b = std::min(total, a + per);
          CHECK(hipMemcpyAsync(d + a, h + a, b - a, hipMemcpyHostToDevice, st[2 + (i / 2) % 2]));
        }
      });
      for (int i = 0; i < chunks; i += 2) {
        const size_t a = i * per, b = std::min(total, a + per);
        CHECK(hipMemcpyAsync(d + a, h + a, b - a, hipMemcpyHostToDevice, st[(i / 2) % 2]));
      }
      t1.join();
    }
    sync_all();
    return total / (now() - t0) / 1e9;
  };
  for (int rep = 0; rep < 2; ++rep) run(1, false), run(15, false), run(15, true);  // warm
  printf("{");
  const char* sep = "";
  for (int chunks : {1, 4, 8, 15, 30}) {
    for (int alt = 0; alt < (chunks > 1 ? 2 : 1); ++alt) {
      std::vector<double> v;
      for (int rep = 0; rep < 7; ++rep) v.push_back(run(chunks, alt));
      std::sort(v.begin(), v.end());
      printf("%s\"%s%d\": {\"median_gbs\": %.2f, \"min\": %.2f, \"max\": %.2f}", sep, alt ? "alt" : "seq", chunks,
             v[3], v[0], v[6]);
      sep = ", ";
    }
  }
  printf("}\n");
  return 0;
}
