// nos node-atomic commit barrier over xGMI peer-to-peer writes (no communicator).
//
// The commit barrier must show that every logical device of the re-enumerated node executes and
// that the xGMI fabric between them carries traffic. An RCCL communicator shows that too, but its
// set-up dominates the cost of a commit: 1.7-1.9 s of ncclCommInitAll + 0.49 s of ncclCommDestroy
// for ONE device on the box, against 3-5 ms for the all-reduce itself
// (profiles/operator_gpu_report_r3_rccl.json) — paid on every flip, while the flipped GPU's pods
// wait. This barrier does the same check directly:
//
//   the peer matrix (hipDeviceCanAccessPeer for every pair) is turned into a token ring by the host
//   logic of csrc/ring_plan.h: every device writes one 64-lane token (its vote, tagged with its
//   index) into the next device it can reach over xGMI, or into its own memory when it reaches
//   nobody; a peer link that cannot be enabled is dropped from the plan the same way. Every token
//   is then read back and checked.
//
// The commit holds iff every device voted yes AND every token arrived intact. Vetoes: a device
// that cannot allocate or launch, a write that does not complete before the deadline
// (NOS_BARRIER_DEADLINE_MS, default 10000: a hung device must not hang the flip), a token that is
// missing or corrupt. A missing peer path is NOT a veto (it costs the fabric check of that link
// only). NOS_BARRIER_NO_PEER="i-j,..." masks pairs out of the peer matrix (tests of the fallback on
// a fully connected node).
//
// Each lane stores its own element (lane-indexed addresses: plain vector stores).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ring_plan.h"

namespace {
constexpr int kLanes = 64;
constexpr uint32_t kYes = 0x6e6f7331u;  // "nos1"
constexpr uint32_t kNo = 0x6e6f7330u;   // "nos0"

thread_local std::string g_p2p_err;
thread_local std::string g_p2p_plan;
thread_local int g_p2p_peer = 0, g_p2p_local = 0;

__global__ void ring_put(uint32_t* __restrict__ dst, uint32_t token) {
  const int lane = threadIdx.x;
  if (lane < kLanes) dst[lane] = token ^ static_cast<uint32_t>(lane);
}

int fail(const std::string& what, hipError_t e) {
  g_p2p_err = what + ": " + hipGetErrorString(e);
  return int(e) ? int(e) : -1;
}

uint32_t token_of(int d, int vote) { return (vote ? kYes : kNo) ^ (static_cast<uint32_t>(d) << 8); }

void mask_pairs(int n, std::vector<uint8_t>& can) {
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

std::string describe(const nos::RingPlan& p) {
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
}  // namespace

extern "C" {

const char* nos_p2p_last_error() { return g_p2p_err.c_str(); }
// the ring of the last barrier ("0>1>2>0", "0>1*;2*": * = a local write) and its link counts
const char* nos_p2p_last_plan() { return g_p2p_plan.c_str(); }
int nos_p2p_last_peer_links() { return g_p2p_peer; }
int nos_p2p_last_local() { return g_p2p_local; }

// votes[d] != 0: device d's own checks passed. *sum = devices whose yes-vote arrived intact;
// *intact = tokens (yes or no) that arrived intact. Returns 0, or a HIP error code / negative value.
int nos_p2p_barrier(int n, const int32_t* votes, int32_t* sum, int32_t* intact) {
  *sum = 0;
  *intact = 0;
  g_p2p_plan.clear();
  g_p2p_peer = g_p2p_local = 0;
  if (n <= 0) {
    g_p2p_err = "no devices";
    return -1;
  }
  const char* dl = std::getenv("NOS_BARRIER_DEADLINE_MS");
  const double deadline_ms = dl ? std::atof(dl) : 10000.0;
  std::vector<uint32_t*> slot(n, nullptr);
  std::vector<hipEvent_t> done(n, nullptr);
  int rc = 0;
  for (int d = 0; d < n && !rc; ++d) {
    hipError_t e = hipSetDevice(d);
    if (e == hipSuccess) e = hipMalloc(&slot[d], 2 * kLanes * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(slot[d], 0, 2 * kLanes * sizeof(uint32_t));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&done[d], hipEventDisableTiming);
    if (e != hipSuccess) rc = fail("device " + std::to_string(d) + " alloc", e);
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
    g_p2p_plan = describe(plan);
    g_p2p_peer = plan.peer_links;
    g_p2p_local = plan.local;
  }
  for (const auto& s : plan.steps) {
    if (rc) break;
    hipError_t e = hipSetDevice(s.src);
    if (e == hipSuccess) {
      ring_put<<<1, kLanes>>>(slot[s.dst] + s.region * kLanes, token_of(s.src, votes[s.src]));
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipEventRecord(done[s.src], nullptr);
    if (e != hipSuccess) rc = fail("device " + std::to_string(s.src) + " token write launch", e);
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
        rc = fail("device " + std::to_string(d) + " token write", e);
      }
    }
    if (!rc && left > 0) {
      const double el = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (el > deadline_ms) {
        int d = 0;
        while (finished[d]) ++d;
        g_p2p_err = "device " + std::to_string(d) + " did not complete its token write within " +
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
        rc = fail("device " + std::to_string(s.dst) + " read back", e);
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

}  // extern "C"
