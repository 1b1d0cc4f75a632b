// Multi-device host fake of the HIP runtime subset of csrc/p2p_barrier_host.h (see the header).
#include "fake_hip_multi.h"

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

struct FakeHipEvent {
  int device = -1;
  uint64_t ticket = 0;   // launches of `device` that must have run
};

namespace {

struct Device {
  int id = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> queue;
  uint64_t submitted = 0;                 // under mu
  std::atomic<uint64_t> completed{0};     // release by the worker, acquire by queries
  std::atomic<int> fault{0};
  bool stop = false;                      // under mu
  bool hung = false;
  bool corrupt = false;
  std::vector<uint8_t> enabled;           // peer access enabled towards device j
  std::thread worker;

  void run() {
    for (;;) {
      std::function<void()> task;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || (!hung && !queue.empty()); });
        if (stop) return;
        task = std::move(queue.front());
        queue.pop_front();
      }
      task();
      completed.fetch_add(1, std::memory_order_release);
    }
  }
};

struct Alloc {
  int device;
  size_t size;
};

std::mutex g_mu;                                   // devices, matrix, allocations
std::vector<std::unique_ptr<Device>> g_dev;
std::vector<uint8_t> g_no_peer, g_fail_enable;     // n x n
std::map<uintptr_t, Alloc> g_alloc;
std::map<FakeHipEvent*, int> g_events;             // live events (a context teardown reclaims them)
std::atomic<int> g_links{0};
thread_local int t_dev = 0;
thread_local hipError_t t_last = hipSuccess;

hipError_t ret(hipError_t e) {
  if (e != hipSuccess) t_last = e;
  return e;
}

Device* dev(int d) { return d >= 0 && d < static_cast<int>(g_dev.size()) ? g_dev[d].get() : nullptr; }

int owner_of(const void* p, size_t n) {
  std::lock_guard<std::mutex> lk(g_mu);
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  auto it = g_alloc.upper_bound(a);
  if (it == g_alloc.begin()) return -1;
  --it;
  return a + n <= it->first + it->second.size ? it->second.device : -1;
}

}  // namespace

hipError_t hipSetDevice(int d) {
  if (!dev(d)) return ret(hipErrorInvalidDevice);
  t_dev = d;
  return hipSuccess;
}

hipError_t hipGetLastError() {
  hipError_t e = t_last;
  t_last = hipSuccess;
  return e;
}

const char* hipGetErrorString(hipError_t e) {
  switch (e) {
    case hipSuccess: return "hipSuccess";
    case hipErrorInvalidValue: return "hipErrorInvalidValue";
    case hipErrorOutOfMemory: return "hipErrorOutOfMemory";
    case hipErrorInvalidDevice: return "hipErrorInvalidDevice";
    case hipErrorInvalidResourceHandle: return "hipErrorInvalidResourceHandle";
    case hipErrorNotReady: return "hipErrorNotReady";
    case hipErrorIllegalAddress: return "hipErrorIllegalAddress";
    case hipErrorPeerAccessUnsupported: return "hipErrorPeerAccessUnsupported";
    case hipErrorPeerAccessAlreadyEnabled: return "hipErrorPeerAccessAlreadyEnabled";
    default: return "hipErrorUnknown";
  }
}

hipError_t hipMalloc(void** p, size_t n) {
  *p = std::calloc(1, n ? n : 1);
  if (!*p) return ret(hipErrorOutOfMemory);
  std::lock_guard<std::mutex> lk(g_mu);
  g_alloc[reinterpret_cast<uintptr_t>(*p)] = Alloc{t_dev, n ? n : 1};
  return hipSuccess;
}

hipError_t hipFree(void* p) {
  if (!p) return hipSuccess;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_alloc.erase(reinterpret_cast<uintptr_t>(p))) return ret(hipErrorInvalidValue);
  }
  std::free(p);
  return hipSuccess;
}

hipError_t hipMemset(void* p, int v, size_t n) {
  if (owner_of(p, n) < 0) return ret(hipErrorInvalidValue);
  std::memset(p, v, n);
  return hipSuccess;
}

hipError_t hipMemcpy(void* dst, const void* src, size_t n, hipMemcpyKind kind) {
  if (kind != hipMemcpyDeviceToHost || owner_of(src, n) < 0) return ret(hipErrorInvalidValue);
  // the null stream of the current device: its launches finish first
  Device* d = dev(t_dev);
  uint64_t want;
  {
    std::lock_guard<std::mutex> lk(d->mu);
    want = d->submitted;
  }
  while (d->completed.load(std::memory_order_acquire) < want) std::this_thread::yield();
  std::memcpy(dst, src, n);
  return hipSuccess;
}

hipError_t hipEventCreateWithFlags(hipEvent_t* ev, unsigned) {
  *ev = new FakeHipEvent();
  std::lock_guard<std::mutex> lk(g_mu);
  g_events[*ev] = 1;
  return hipSuccess;
}

hipError_t hipEventRecord(hipEvent_t ev, hipStream_t) {
  if (!ev) return ret(hipErrorInvalidResourceHandle);
  Device* d = dev(t_dev);
  std::lock_guard<std::mutex> lk(d->mu);
  ev->device = t_dev;
  ev->ticket = d->submitted;
  return hipSuccess;
}

hipError_t hipEventQuery(hipEvent_t ev) {
  if (!ev || ev->device < 0) return ret(hipErrorInvalidResourceHandle);
  Device* d = dev(ev->device);
  if (int f = d->fault.load(std::memory_order_acquire)) return ret(f);
  return d->completed.load(std::memory_order_acquire) >= ev->ticket ? hipSuccess : hipErrorNotReady;
}

hipError_t hipEventDestroy(hipEvent_t ev) {
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_events.erase(ev)) return ret(hipErrorInvalidResourceHandle);
  }
  delete ev;
  return hipSuccess;
}

hipError_t hipDeviceCanAccessPeer(int* can, int d, int peer) {
  const int n = static_cast<int>(g_dev.size());
  if (!dev(d) || !dev(peer)) return ret(hipErrorInvalidDevice);
  *can = d != peer && !g_no_peer[static_cast<size_t>(d) * n + peer];
  return hipSuccess;
}

hipError_t hipDeviceEnablePeerAccess(int peer, unsigned) {
  const int n = static_cast<int>(g_dev.size());
  Device* d = dev(t_dev);
  if (!dev(peer) || peer == t_dev) return ret(hipErrorInvalidDevice);
  const size_t k = static_cast<size_t>(t_dev) * n + peer;
  if (g_no_peer[k] || g_fail_enable[k]) return ret(hipErrorPeerAccessUnsupported);
  std::lock_guard<std::mutex> lk(d->mu);
  if (d->enabled[peer]) return ret(hipErrorPeerAccessAlreadyEnabled);
  d->enabled[peer] = 1;
  g_links.fetch_add(1);
  return hipSuccess;
}

namespace fake_hip {

void reset() {
  for (auto& d : g_dev) {
    {
      std::lock_guard<std::mutex> lk(d->mu);
      d->stop = true;
    }
    d->cv.notify_all();
    if (d->worker.joinable()) d->worker.join();
  }
  g_dev.clear();
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& a : g_alloc) std::free(reinterpret_cast<void*>(a.first));
  g_alloc.clear();
  for (auto& e : g_events) delete e.first;
  g_events.clear();
  g_links = 0;
}

void configure(int n) {
  reset();
  g_no_peer.assign(static_cast<size_t>(n) * n, 0);
  g_fail_enable.assign(static_cast<size_t>(n) * n, 0);
  for (int i = 0; i < n; ++i) {
    auto d = std::make_unique<Device>();
    d->id = i;
    d->enabled.assign(n, 0);
    g_dev.push_back(std::move(d));
  }
  for (auto& d : g_dev) d->worker = std::thread(&Device::run, d.get());
  t_dev = 0;
}

void set_no_peer(int i, int j) {
  const int n = static_cast<int>(g_dev.size());
  g_no_peer[static_cast<size_t>(i) * n + j] = g_no_peer[static_cast<size_t>(j) * n + i] = 1;
}

void fail_enable(int i, int j) { g_fail_enable[static_cast<size_t>(i) * g_dev.size() + j] = 1; }

void hang(int d) {
  std::lock_guard<std::mutex> lk(g_dev[d]->mu);
  g_dev[d]->hung = true;
}

void corrupt(int d) { g_dev[d]->corrupt = true; }

hipError_t launch_write(uint32_t* dst, uint32_t token, int lanes) {
  Device* d = dev(t_dev);
  const int owner = owner_of(dst, sizeof(uint32_t) * lanes);
  if (owner < 0) return ret(hipErrorInvalidValue);
  bool allowed;
  {
    std::lock_guard<std::mutex> lk(d->mu);
    allowed = owner == t_dev || d->enabled[owner];
  }
  const bool flip = d->corrupt;
  auto task = [d, dst, token, lanes, allowed, flip] {
    if (!allowed) {  // a write into another device's memory without peer access: a GPU fault
      d->fault.store(hipErrorIllegalAddress, std::memory_order_release);
      return;
    }
    for (int l = 0; l < lanes; ++l) dst[l] = token ^ static_cast<uint32_t>(l) ^ (flip && l == 5 ? 1u : 0u);
  };
  {
    std::lock_guard<std::mutex> lk(d->mu);
    d->queue.push_back(task);
    ++d->submitted;
  }
  d->cv.notify_one();
  return hipSuccess;
}

int enabled_links() { return g_links.load(); }

int faults() {
  int n = 0;
  for (auto& d : g_dev) n += d->fault.load() != 0;
  return n;
}

size_t live_allocations() {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_alloc.size();
}

}  // namespace fake_hip
