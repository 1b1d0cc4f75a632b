// Host-only stand-in for the HIP allocation entry points (libamdhip64), backed by malloc with a
// 1 GiB "device": lets the HBM-limit shim (csrc/hbm_limit.cpp) run under AddressSanitizer /
// UndefinedBehaviorSanitizer / ThreadSanitizer on a machine without a GPU
// (tests/test_native_sanitizers.py).
#include <atomic>
#include <cstddef>
#include <cstdlib>

namespace {
std::atomic<size_t> g_used{0};
constexpr size_t kTotal = size_t(1) << 30;
}  // namespace

extern "C" {

int hipMalloc(void** p, size_t n) {
  *p = std::malloc(n ? n : 1);
  if (!*p) return 2;
  g_used += n;
  return 0;
}
int hipExtMallocWithFlags(void** p, size_t n, unsigned int) { return hipMalloc(p, n); }
int hipMallocAsync(void** p, size_t n, void*) { return hipMalloc(p, n); }
int hipMallocManaged(void** p, size_t n, unsigned int) { return hipMalloc(p, n); }
int hipFree(void* p) {
  std::free(p);
  return 0;
}
int hipFreeAsync(void* p, void*) { return hipFree(p); }
// pitched: rows padded to 256 B, like the real runtime's texture-aligned pitch
int hipMallocPitch(void** p, size_t* pitch, size_t w, size_t h) {
  *pitch = (w + 255) / 256 * 256;
  *p = std::malloc(*pitch * h);  // not through hipMalloc: the real runtime allocates internally
  return *p ? 0 : 2;
}
struct FakeHandle { size_t n; };
int hipMemCreate(void** handle, size_t n, const void*, unsigned long long) {
  *handle = new FakeHandle{n};
  return 0;
}
int hipMemRelease(void* handle) {
  delete static_cast<FakeHandle*>(handle);
  return 0;
}
int hipMemGetInfo(size_t* free_b, size_t* total_b) {
  *total_b = kTotal;
  *free_b = kTotal / 2;
  return 0;
}

}  // extern "C"
