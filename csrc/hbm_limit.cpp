// nos HBM budget shim (LD_PRELOAD) for CU-mask slices.
//
// The reference enforces MPS memory slices with CUDA_MPS_PINNED_DEVICE_MEM_LIMIT
// (docs getting-started-mps.md). HIP has no MPS daemon, so a slice's HBM budget is enforced in the
// workload process itself: this library interposes the HIP device-allocation entry points, tracks
// live bytes per pointer and fails an allocation that would exceed NOS_HBM_LIMIT_BYTES with
// hipErrorOutOfMemory. hipMemGetInfo is clamped to the budget so caching allocators (PyTorch's)
// size themselves to the slice. Compute isolation comes from HSA_CU_MASK (ROCr applies it to every
// queue the process creates, hsa_ext_amd.h:1330-1345); both variables are injected by the nos device
// plugin at Allocate time.
//
// Interposed: hipMalloc, hipExtMallocWithFlags, hipMallocAsync, hipMallocFromPoolAsync,
// hipMallocManaged, hipMallocPitch and hipMalloc3D (charged pitch x height [x depth] after the
// runtime picked the pitch; over budget -> freed again, hipErrorOutOfMemory), and the virtual-
// memory path PyTorch's expandable segments use: hipMemCreate charges the physical allocation,
// hipMemRelease returns it (mapping it with hipMemMap allocates nothing more).
//
// Isolation is cooperative: nothing stops a process from unsetting LD_PRELOAD, or from allocating
// through entry points not listed above (texture arrays: hipMallocArray / hipArray3DCreate), as
// docs/partitioning.md ("Caveats") says — the reference documents MPS's limits the same way.
#include <dlfcn.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

namespace {

using hipErr = int;  // hipError_t is an int-sized enum
constexpr hipErr kSuccess = 0;
constexpr hipErr kOutOfMemory = 2;  // hipErrorOutOfMemory

std::mutex g_mu;
std::unordered_map<void*, size_t>* g_sizes = nullptr;
std::unordered_map<void*, size_t>* g_handles = nullptr;  // hipMemCreate handles (VMM)
std::atomic<size_t> g_live{0};
std::atomic<size_t> g_peak{0};
size_t g_limit = 0;
bool g_loaded = false;

void init_once() {
  static std::once_flag once;
  std::call_once(once, [] {
    g_sizes = new std::unordered_map<void*, size_t>();
    g_handles = new std::unordered_map<void*, size_t>();
    if (const char* v = std::getenv("NOS_HBM_LIMIT_BYTES")) g_limit = std::strtoull(v, nullptr, 10);
    g_loaded = true;
  });
}

// Resolve the real HIP entry point. RTLD_NEXT only searches the global scope; a runtime that was
// dlopen'ed RTLD_LOCAL (PyTorch loads its bundled libamdhip64 that way) is invisible to it, so fall
// back to the already-loaded runtime by soname. Never return null: abort with a message instead of
// jumping to address 0.
template <typename F>
F next(const char* name) {
  void* p = dlsym(RTLD_NEXT, name);
  if (!p) {
    void* h = dlopen("libamdhip64.so.7", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("libamdhip64.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("libamdhip64.so.7", RTLD_NOW | RTLD_GLOBAL);
    if (h) p = dlsym(h, name);
  }
  if (!p) {
    std::fprintf(stderr, "nos hbm-limit shim: cannot resolve %s\n", name);
    std::abort();
  }
  return reinterpret_cast<F>(p);
}

bool reserve(size_t bytes) {
  if (g_limit == 0) {
    g_live += bytes;
    return true;
  }
  size_t cur = g_live.load();
  while (true) {
    if (cur + bytes > g_limit) return false;
    if (g_live.compare_exchange_weak(cur, cur + bytes)) return true;
  }
}

void track(void* p, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_mu);
  (*g_sizes)[p] = bytes;
  size_t live = g_live.load();
  if (live > g_peak.load()) g_peak = live;
}

// Removes p's entry BEFORE the real free and returns its size (0 if untracked): once the runtime
// has freed p, another thread's allocation may get the same address and track it, so an entry
// removed after the free could be that thread's. The bytes stay charged until the free succeeded.
size_t take(void* p) {
  if (!p) return 0;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_sizes->find(p);
  if (it == g_sizes->end()) return 0;
  const size_t n = it->second;
  g_sizes->erase(it);
  return n;
}

template <typename Free>
hipErr guarded_free(void* ptr, Free&& free_fn) {
  init_once();
  const size_t n = take(ptr);
  const hipErr rc = free_fn();
  if (rc == kSuccess) {
    g_live -= n;
  } else if (n) {
    std::lock_guard<std::mutex> lk(g_mu);
    (*g_sizes)[ptr] = n;  // still allocated: keep it on the books
  }
  return rc;
}

template <typename Alloc>
hipErr guarded(void** ptr, size_t size, Alloc&& alloc) {
  init_once();
  if (!reserve(size)) {
    if (ptr) *ptr = nullptr;
    return kOutOfMemory;
  }
  hipErr rc = alloc();
  if (rc != kSuccess || !ptr || !*ptr) {
    g_live -= size;
    return rc;
  }
  track(*ptr, size);
  return rc;
}

// Allocations whose size the runtime decides (pitched): allocate, then charge the real size; over
// budget -> give the memory back and fail like a real out-of-memory.
template <typename Alloc, typename Free>
hipErr charged_after(void* p, size_t bytes, hipErr rc, Free&& free_fn) {
  if (rc != kSuccess || p == nullptr) return rc;
  if (!reserve(bytes)) {
    free_fn();
    return kOutOfMemory;
  }
  track(p, bytes);
  return rc;
}

}  // namespace

struct nos_pitched_ptr {  // hipPitchedPtr (driver_types.h:385)
  void* ptr;
  size_t pitch;
  size_t xsize;
  size_t ysize;
};
struct nos_extent {  // hipExtent (driver_types.h:394)
  size_t width;
  size_t height;
  size_t depth;
};

extern "C" {

hipErr hipMalloc(void** ptr, size_t size) {
  static auto real = next<hipErr (*)(void**, size_t)>("hipMalloc");
  return guarded(ptr, size, [&] { return real(ptr, size); });
}

hipErr hipExtMallocWithFlags(void** ptr, size_t size, unsigned int flags) {
  static auto real = next<hipErr (*)(void**, size_t, unsigned int)>("hipExtMallocWithFlags");
  return guarded(ptr, size, [&] { return real(ptr, size, flags); });
}

hipErr hipMallocAsync(void** ptr, size_t size, void* stream) {
  static auto real = next<hipErr (*)(void**, size_t, void*)>("hipMallocAsync");
  return guarded(ptr, size, [&] { return real(ptr, size, stream); });
}

hipErr hipMallocManaged(void** ptr, size_t size, unsigned int flags) {
  static auto real = next<hipErr (*)(void**, size_t, unsigned int)>("hipMallocManaged");
  return guarded(ptr, size, [&] { return real(ptr, size, flags); });
}

hipErr hipMallocFromPoolAsync(void** ptr, size_t size, void* pool, void* stream) {
  static auto real = next<hipErr (*)(void**, size_t, void*, void*)>("hipMallocFromPoolAsync");
  return guarded(ptr, size, [&] { return real(ptr, size, pool, stream); });
}

hipErr hipMallocPitch(void** ptr, size_t* pitch, size_t width, size_t height) {
  static auto real = next<hipErr (*)(void**, size_t*, size_t, size_t)>("hipMallocPitch");
  static auto real_free = next<hipErr (*)(void*)>("hipFree");
  init_once();
  if (!reserve(width * height)) {  // cannot fit even unpadded: fail before touching the device
    if (ptr) *ptr = nullptr;
    return kOutOfMemory;
  }
  g_live -= width * height;
  hipErr rc = real(ptr, pitch, width, height);
  if (rc != kSuccess || !ptr || !pitch) return rc;
  void* p = *ptr;
  rc = charged_after<int>(p, *pitch * height, rc, [&] { real_free(p); });
  if (rc != kSuccess) *ptr = nullptr;
  return rc;
}

hipErr hipMalloc3D(nos_pitched_ptr* pp, nos_extent extent) {
  static auto real = next<hipErr (*)(nos_pitched_ptr*, nos_extent)>("hipMalloc3D");
  static auto real_free = next<hipErr (*)(void*)>("hipFree");
  init_once();
  const size_t minimum = extent.width * extent.height * (extent.depth ? extent.depth : 1);
  if (!reserve(minimum)) {
    if (pp) pp->ptr = nullptr;
    return kOutOfMemory;
  }
  g_live -= minimum;
  hipErr rc = real(pp, extent);
  if (rc != kSuccess || !pp) return rc;
  void* p = pp->ptr;
  rc = charged_after<int>(p, pp->pitch * extent.height * (extent.depth ? extent.depth : 1), rc,
                          [&] { real_free(p); });
  if (rc != kSuccess) pp->ptr = nullptr;
  return rc;
}

// Virtual memory management (PyTorch PYTORCH_HIP_ALLOC_CONF=expandable_segments:True): the
// physical backing is created by hipMemCreate and returned by hipMemRelease; hipMemMap only maps
// an existing handle, so the handle is what carries the bytes.
hipErr hipMemCreate(void** handle, size_t size, const void* prop, unsigned long long flags) {
  static auto real = next<hipErr (*)(void**, size_t, const void*, unsigned long long)>("hipMemCreate");
  init_once();
  if (!reserve(size)) return kOutOfMemory;
  hipErr rc = real(handle, size, prop, flags);
  if (rc != kSuccess || !handle || !*handle) {
    g_live -= size;
    return rc;
  }
  std::lock_guard<std::mutex> lk(g_mu);
  (*g_handles)[*handle] = size;
  size_t live = g_live.load();
  if (live > g_peak.load()) g_peak = live;
  return rc;
}

hipErr hipMemRelease(void* handle) {
  static auto real = next<hipErr (*)(void*)>("hipMemRelease");
  init_once();
  size_t n = 0;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_handles->find(handle);
    if (it != g_handles->end()) {
      n = it->second;
      g_handles->erase(it);
    }
  }
  const hipErr rc = real(handle);
  if (rc == kSuccess) {
    g_live -= n;
  } else if (n) {
    std::lock_guard<std::mutex> lk(g_mu);
    (*g_handles)[handle] = n;
  }
  return rc;
}

hipErr hipFree(void* ptr) {
  static auto real = next<hipErr (*)(void*)>("hipFree");
  return guarded_free(ptr, [&] { return real(ptr); });
}

hipErr hipFreeAsync(void* ptr, void* stream) {
  static auto real = next<hipErr (*)(void*, void*)>("hipFreeAsync");
  return guarded_free(ptr, [&] { return real(ptr, stream); });
}

hipErr hipMemGetInfo(size_t* free_b, size_t* total_b) {
  static auto real = next<hipErr (*)(size_t*, size_t*)>("hipMemGetInfo");
  init_once();
  hipErr rc = real(free_b, total_b);
  if (rc == kSuccess && g_limit > 0) {
    size_t live = g_live.load();
    size_t budget_free = live >= g_limit ? 0 : g_limit - live;
    if (*total_b > g_limit) *total_b = g_limit;
    if (*free_b > budget_free) *free_b = budget_free;
  }
  return rc;
}

// introspection for tests / the workload runner
size_t nos_hbm_limit_bytes() { init_once(); return g_limit; }
size_t nos_hbm_live_bytes() { return g_live.load(); }
size_t nos_hbm_peak_bytes() { return g_peak.load(); }
int nos_hbm_shim_loaded() { init_once(); return g_loaded ? 1 : 0; }

}  // extern "C"
