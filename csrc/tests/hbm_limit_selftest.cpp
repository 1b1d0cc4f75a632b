// Self-test of the HBM-limit shim's budget accounting under concurrent allocation (host only; the
// HIP runtime is csrc/tests/fake_hip.cpp). Built and run with -fsanitize=address,undefined and
// -fsanitize=thread by tests/test_native_sanitizers.py. Exit code 0 = every check passed.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

extern "C" {
int hipMalloc(void** p, size_t n);
int hipFree(void* p);
int hipMemGetInfo(size_t* free_b, size_t* total_b);
int hipMallocPitch(void** p, size_t* pitch, size_t w, size_t h);
int hipMemCreate(void** handle, size_t n, const void* prop, unsigned long long flags);
int hipMemRelease(void* handle);
size_t nos_hbm_limit_bytes();
size_t nos_hbm_live_bytes();
size_t nos_hbm_peak_bytes();
}

#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::fprintf(stderr, "CHECK failed: %s (line %d)\n", #c, __LINE__); \
      std::exit(1);                                               \
    }                                                             \
  } while (0)

int main() {
  const size_t limit = size_t(64) << 20;  // 64 MiB budget
  CHECK(nos_hbm_limit_bytes() == limit);
  // over-budget single allocation fails with out-of-memory and leaves nothing live
  void* p = nullptr;
  CHECK(hipMalloc(&p, limit + 1) == 2 && p == nullptr);
  CHECK(nos_hbm_live_bytes() == 0);
  // hipMemGetInfo is clamped to the budget
  size_t fr = 0, tot = 0;
  CHECK(hipMalloc(&p, size_t(16) << 20) == 0 && p);
  CHECK(hipMemGetInfo(&fr, &tot) == 0);
  CHECK(tot == limit && fr == limit - (size_t(16) << 20));
  CHECK(hipFree(p) == 0 && nos_hbm_live_bytes() == 0);
  // pitched allocations are charged at pitch x height (the padded size the runtime chose)
  size_t pitch = 0;
  CHECK(hipMallocPitch(&p, &pitch, 1000, 1024) == 0 && p && pitch == 1024);
  CHECK(nos_hbm_live_bytes() == size_t(1024) * 1024);
  CHECK(hipFree(p) == 0 && nos_hbm_live_bytes() == 0);
  CHECK(hipMallocPitch(&p, &pitch, 67100, 1000) == 2 && p == nullptr);  // fits unpadded, not padded
  CHECK(nos_hbm_live_bytes() == 0);
  // virtual-memory handles (expandable segments) carry their physical size until released
  void* h1 = nullptr;
  void* h2 = nullptr;
  CHECK(hipMemCreate(&h1, size_t(48) << 20, nullptr, 0) == 0 && h1);
  CHECK(hipMemCreate(&h2, size_t(32) << 20, nullptr, 0) == 2);
  CHECK(hipMemRelease(h1) == 0 && nos_hbm_live_bytes() == 0);
  CHECK(hipMemCreate(&h2, size_t(32) << 20, nullptr, 0) == 0 && hipMemRelease(h2) == 0);
  // concurrent random alloc/free: the live total never exceeds the budget
  std::atomic<int> oom{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t) {
    ts.emplace_back([t, &oom] {
      std::mt19937 rng(1234 + t);
      std::vector<void*> mine;
      for (int i = 0; i < 4000; ++i) {
        if (mine.empty() || rng() % 3) {
          void* q = nullptr;
          const size_t n = 1 + rng() % (size_t(4) << 20);
          const int rc = hipMalloc(&q, n);
          if (rc == 0)
            mine.push_back(q);
          else
            oom++;
        } else {
          const size_t k = rng() % mine.size();
          hipFree(mine[k]);
          mine[k] = mine.back();
          mine.pop_back();
        }
      }
      for (void* q : mine) hipFree(q);
    });
  }
  for (auto& th : ts) th.join();
  CHECK(oom.load() > 0);                      // the budget was actually hit
  CHECK(nos_hbm_peak_bytes() <= limit);       // and never exceeded
  CHECK(nos_hbm_live_bytes() == 0);           // every byte accounted back
  std::printf("hbm_limit selftest ok: %d OOMs, peak %zu / %zu bytes\n", oom.load(), nos_hbm_peak_bytes(), limit);
  return 0;
}
