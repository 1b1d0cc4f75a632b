// Token-ring plan of the node commit barrier (csrc/p2p_barrier.hip): pure host logic, no HIP, so
// the ordering and its fallbacks are unit-tested on a CPU (csrc/ring_plan_capi.cpp ->
// libnos_ringplan.so, tests/test_ring_plan.py).
//
// Input: n logical devices and the peer matrix can[i*n + j] != 0 <=> device i can write device j's
// memory (hipDeviceCanAccessPeer(i, j)). Output: one token write per device —
//
//   * devices are chained greedily, each one writing into the next device it can reach (the lowest
//     index after it, cyclically, so a fully connected node gives the plain ring 0 > 1 > ... > n-1 > 0);
//   * a chain closes into a ring when its last device can reach its first; otherwise, and for a
//     device that reaches nobody, the last device writes its token into its OWN memory (a "local"
//     write). A local write still proves that the device executes; it only leaves out a fabric link
//     that does not exist, so a missing peer path is not a veto (before, one pair without P2P vetoed
//     every commit of the node: a livelock for a 64-device CPX node if any pair lacks a path);
//   * every write has its own destination region (region 0 of the successor for peer writes, region 1
//     of the device itself for local ones), so no two writes ever target the same memory.
//
// The barrier then vetoes only what a commit must not survive: a device that fails to execute its
// write (launch error, or no completion before the deadline) and a token that does not read back
// intact.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace nos {

struct RingStep {
  int src;     // device that writes its token
  int dst;     // device whose memory receives it (== src for a local write)
  int region;  // 0: the peer region of dst; 1: src's own local region
};

struct RingPlan {
  std::vector<std::vector<int>> chains;  // device order of each chain
  std::vector<RingStep> steps;           // exactly one per device
  int peer_links = 0;                    // writes that cross a peer link
  int local = 0;                         // writes into the device's own memory
  int closed = 0;                        // chains that close into a ring
};

inline RingPlan plan_ring(int n, const std::vector<uint8_t>& can) {
  RingPlan p;
  if (n <= 0 || static_cast<int>(can.size()) < n * n) return p;
  auto reach = [&](int i, int j) { return i != j && can[static_cast<size_t>(i) * n + j] != 0; };
  std::vector<char> seen(n, 0);
  for (int start = 0; start < n; ++start) {
    if (seen[start]) continue;
    std::vector<int> chain{start};
    seen[start] = 1;
    int cur = start;
    for (;;) {
      int next = -1;
      for (int k = 1; k < n && next < 0; ++k) {
        const int j = (cur + k) % n;
        if (!seen[j] && reach(cur, j)) next = j;
      }
      if (next < 0) break;
      chain.push_back(next);
      seen[next] = 1;
      cur = next;
    }
    const int len = static_cast<int>(chain.size());
    for (int k = 0; k + 1 < len; ++k) p.steps.push_back({chain[k], chain[k + 1], 0});
    const int last = chain[len - 1];
    if (len >= 2 && reach(last, chain[0])) {
      p.steps.push_back({last, chain[0], 0});
      ++p.closed;
    } else {
      p.steps.push_back({last, last, 1});
    }
    p.chains.push_back(chain);
  }
  for (const auto& s : p.steps) (s.region ? p.local : p.peer_links) += 1;
  return p;
}

}  // namespace nos
