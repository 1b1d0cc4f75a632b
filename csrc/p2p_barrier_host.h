// Host side of the xGMI commit barrier (csrc/p2p_barrier.hip): allocation, the peer matrix, the
// token-ring plan (csrc/ring_plan.h), peer enabling with re-planning, the token writes, the
// deadline-bounded completion wait and the read-back check.
//
// Written against the HIP runtime API names only, so the same code runs on the GPU (included by
// csrc/p2p_barrier.hip after <hip/hip_runtime.h>) and on a CPU against a multi-device fake of that
// API (csrc/tests/fake_hip_multi.h: n devices, a peer matrix, peer-enable failures, devices that
// never complete, corrupted writes), where tests/test_p2p_barrier_host.py drives the n > 1 paths at
// 8 and 64 devices under ASan/UBSan and TSan. The includer defines ring_put_launch(): the token
// write on the current device (a kernel launch on the GPU, a queued host write in the fake).
#pragma once

#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "ring_plan.h"

namespace nos_p2p {

constexpr int kLanes = 64;
constexpr uint32_t kYes = 0x6e6f7331u;  // "nos1"
constexpr uint32_t kNo = 0x6e6f7330u;   // "nos0"

// the token write of the current device: lane l of dst[0..kLanes) = token ^ l (defined by the includer)
hipError_t ring_put_launch(uint32_t* dst, uint32_t token);

struct Result {
  std::string err;
  std::string plan;   // "0>1>2>0", "0>1*;2*": * = a local write
  int peer = 0;       // writes over a peer link
  int local = 0;      // writes into the writer's own memory
};

inline uint32_t token_of(int d, int vote) { return (vote ? kYes : kNo) ^ (static_cast<uint32_t>(d) << 8); }

inline int fail(Result& r, const std::string& what, hipError_t e) {
  r.err = what + ": " + hipGetErrorString(e);
  return int(e) ? int(e) : -1;
}

// NOS_BARRIER_NO_PEER="i-j,...": pairs masked out of the peer matrix (the fallback on a fully
// connected node)
inline void mask_pairs(int n, std::vector<uint8_t>& can) {
  const char* v = std::getenv("NOS_BARRIER_NO_PEER");
  if (!v) return;
  std::string s(v);
  size_t pos = 0;
  while (pos < s.size()) {
    size_t c = s.find(',', pos);
    std::string tok = s.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
    size_t dash = tok.find('-');
    if (dash != std::string::npos) {
      const int i = std::atoi(tok.substr(0, dash).c_str()), j = std::atoi(tok.substr(dash + 1).c_str());
      if (i >= 0 && j >= 0 && i < n && j < n) can[static_cast<size_t>(i) * n + j] = can[static_cast<size_t>(j) * n + i] = 0;
    }
    if (c == std::string::npos) break;
    pos = c + 1;
  }
}

inline std::string describe(const nos::RingPlan& p) {
  std::string out;
  for (const auto& c : p.chains) {
    if (!out.empty()) out += ";";
    for (size_t k = 0; k < c.size(); ++k) out += (k ? ">" : "") + std::to_string(c[k]);
    const int last = c.back();
    for (const auto& s : p.steps)
      if (s.src == last) out += s.region ? "*" : ">" + std::to_string(s.dst);
  }
  return out;
}

// votes[d] != 0: device d's own checks passed. *sum = devices whose yes-vote arrived intact;
// *intact = tokens (yes or no) that arrived intact. Returns 0, a HIP error code, -1 (no devices) or
// -3 (a device did not complete its write before NOS_BARRIER_DEADLINE_MS, default 10000).
inline int run(int n, const int32_t* votes, int32_t* sum, int32_t* intact, Result& res) {
  *sum = 0;
  *intact = 0;
  res = Result();
  if (n <= 0) {
    res.err = "no devices";
    return -1;
  }
  const char* dl = std::getenv("NOS_BARRIER_DEADLINE_MS");
  const double deadline_ms = dl ? std::atof(dl) : 10000.0;
  std::vector<uint32_t*> slot(n, nullptr);
  std::vector<hipEvent_t> done(n, nullptr);
  int rc = 0;
  for (int d = 0; d < n && !rc; ++d) {
    hipError_t e = hipSetDevice(d);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&slot[d]), 2 * kLanes * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(slot[d], 0, 2 * kLanes * sizeof(uint32_t));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&done[d], hipEventDisableTiming);
    if (e != hipSuccess) rc = fail(res, "device " + std::to_string(d) + " alloc", e);
  }
  // peer matrix; a failing query counts as "no path"
  std::vector<uint8_t> can(static_cast<size_t>(n) * n, 0);
  for (int i = 0; i < n && !rc; ++i)
    for (int j = 0; j < n; ++j) {
      int ok = 0;
      if (i != j && hipDeviceCanAccessPeer(&ok, i, j) != hipSuccess) {
        (void)hipGetLastError();
        ok = 0;
      }
      can[static_cast<size_t>(i) * n + j] = ok ? 1 : 0;
    }
  mask_pairs(n, can);
  nos::RingPlan plan;
  // plan, enable the planned peer links; a link that cannot be enabled leaves the matrix and the
  // ring is planned again (each round removes one link, so this ends)
  for (int round = 0; !rc && round <= n * n; ++round) {
    plan = nos::plan_ring(n, can);
    bool replan = false;
    for (const auto& s : plan.steps) {
      if (s.region) continue;
      hipError_t e = hipSetDevice(s.src);
      if (e == hipSuccess) e = hipDeviceEnablePeerAccess(s.dst, 0);
      if (e == hipErrorPeerAccessAlreadyEnabled) e = hipSuccess;
      if (e != hipSuccess) {
        (void)hipGetLastError();
        can[static_cast<size_t>(s.src) * n + s.dst] = 0;
        replan = true;
        break;
      }
    }
    if (!replan) break;
  }
  if (!rc) {
    res.plan = describe(plan);
    res.peer = plan.peer_links;
    res.local = plan.local;
  }
  for (const auto& s : plan.steps) {
    if (rc) break;
    hipError_t e = hipSetDevice(s.src);
    if (e == hipSuccess) e = ring_put_launch(slot[s.dst] + s.region * kLanes, token_of(s.src, votes[s.src]));
    if (e == hipSuccess) e = hipEventRecord(done[s.src], nullptr);
    if (e != hipSuccess) rc = fail(res, "device " + std::to_string(s.src) + " token write launch", e);
  }
  // wait for every write under one deadline (a device that never completes is a veto, not a hang)
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<char> finished(n, 0);
  for (int left = n; !rc && left > 0;) {
    for (int d = 0; d < n && !rc; ++d) {
      if (finished[d]) continue;
      (void)hipSetDevice(d);
      hipError_t e = hipEventQuery(done[d]);
      if (e == hipSuccess) {
        finished[d] = 1;
        --left;
      } else if (e != hipErrorNotReady) {
        rc = fail(res, "device " + std::to_string(d) + " token write", e);
      }
    }
    if (!rc && left > 0) {
      const double el = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (el > deadline_ms) {
        int d = 0;
        while (finished[d]) ++d;
        res.err = "device " + std::to_string(d) + " did not complete its token write within " +
                  std::to_string(static_cast<int>(deadline_ms)) + " ms";
        return -3;  // nothing is freed: a device may still be running the write
      }
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  if (!rc) {
    std::vector<uint32_t> got(kLanes);
    for (const auto& s : plan.steps) {
      hipError_t e = hipSetDevice(s.dst);
      if (e == hipSuccess)
        e = hipMemcpy(got.data(), slot[s.dst] + s.region * kLanes, kLanes * sizeof(uint32_t), hipMemcpyDeviceToHost);
      if (e != hipSuccess) {
        rc = fail(res, "device " + std::to_string(s.dst) + " read back", e);
        break;
      }
      const uint32_t yes = token_of(s.src, 1), no = token_of(s.src, 0);
      bool all_yes = true, all_no = true;
      for (int l = 0; l < kLanes; ++l) {
        all_yes = all_yes && got[l] == (yes ^ static_cast<uint32_t>(l));
        all_no = all_no && got[l] == (no ^ static_cast<uint32_t>(l));
      }
      if (all_yes || all_no) ++*intact;
      if (all_yes) ++*sum;
    }
  }
  for (int d = 0; d < n; ++d) {
    (void)hipSetDevice(d);
    if (done[d]) (void)hipEventDestroy(done[d]);
    if (slot[d]) (void)hipFree(slot[d]);
  }
  return rc;
}

}  // namespace nos_p2p
