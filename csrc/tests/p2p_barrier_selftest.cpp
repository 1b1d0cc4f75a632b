// The commit barrier's host code (csrc/p2p_barrier_host.h) on the multi-device fake HIP
// (csrc/tests/fake_hip_multi.*): every n > 1 path — a full ring, peer links that fail to enable
// (re-plan), missing peer paths (local writes), a hung device (deadline), a corrupted token and a
// no-vote (vetoes). Prints one JSON line per scenario; exits non-zero if any expectation fails.
//
//   p2p_barrier_selftest <n>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "fake_hip_multi.h"
#include "../p2p_barrier_host.h"

hipError_t nos_p2p::ring_put_launch(uint32_t* dst, uint32_t token) {
  return fake_hip::launch_write(dst, token, nos_p2p::kLanes);
}

namespace {

int g_failures = 0;

struct Outcome {
  int rc;
  int sum;
  int intact;
  double ms;
  nos_p2p::Result res;
};

Outcome barrier(int n, const std::vector<int32_t>& votes) {
  Outcome o{};
  int32_t sum = 0, intact = 0;
  const auto t0 = std::chrono::steady_clock::now();
  o.rc = nos_p2p::run(n, votes.data(), &sum, &intact, o.res);
  o.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  o.sum = sum;
  o.intact = intact;
  return o;
}

void report(const char* name, int n, const Outcome& o, bool ok) {
  std::printf("{\"scenario\": \"%s\", \"n\": %d, \"rc\": %d, \"sum\": %d, \"intact\": %d, \"peer\": %d, "
              "\"local\": %d, \"ms\": %.1f, \"enabled_links\": %d, \"faults\": %d, \"ok\": %s, \"err\": \"%s\", "
              "\"plan_len\": %zu}\n",
              name, n, o.rc, o.sum, o.intact, o.res.peer, o.res.local, o.ms, fake_hip::enabled_links(),
              fake_hip::faults(), ok ? "true" : "false", o.res.err.c_str(), o.res.plan.size());
  std::fflush(stdout);
  if (!ok) ++g_failures;
}

}  // namespace

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 8;
  std::vector<int32_t> yes(n, 1);

  // 1. fully connected: the plain ring 0 > 1 > ... > n-1 > 0, every token a peer write
  fake_hip::configure(n);
  Outcome o = barrier(n, yes);
  report("full_ring", n, o, o.rc == 0 && o.sum == n && o.intact == n && o.res.peer == n && o.res.local == 0 &&
                                fake_hip::faults() == 0 && fake_hip::live_allocations() == 0);

  // 2. two planned links refuse to enable: dropped, the ring re-planned around them, committed
  fake_hip::configure(n);
  fake_hip::fail_enable(0, 1);
  fake_hip::fail_enable(n / 2, n / 2 + 1);
  o = barrier(n, yes);
  report("enable_fails_replan", n, o, o.rc == 0 && o.sum == n && o.intact == n && o.res.plan.find("0>1>") != 0 &&
                                          fake_hip::faults() == 0);

  // 3. device 1 reaches nobody (no P2P path at all): its write stays local, the rest still ring
  fake_hip::configure(n);
  for (int j = 0; j < n; ++j)
    if (j != 1) fake_hip::set_no_peer(1, j);
  o = barrier(n, yes);
  report("no_peer_path_local_write", n, o, o.rc == 0 && o.sum == n && o.intact == n && o.res.local >= 1 &&
                                               fake_hip::faults() == 0);

  // 4. a corrupted token: intact n-1, the commit (sum == n) fails
  fake_hip::configure(n);
  fake_hip::corrupt(n - 1);
  o = barrier(n, yes);
  report("corrupt_token_vetoes", n, o, o.rc == 0 && o.intact == n - 1 && o.sum == n - 1);

  // 5. one device votes no: its token arrives intact, the sum is short
  fake_hip::configure(n);
  std::vector<int32_t> one_no(yes);
  one_no[n / 3] = 0;
  o = barrier(n, one_no);
  report("no_vote_vetoes", n, o, o.rc == 0 && o.intact == n && o.sum == n - 1);

  // 6. a device that never completes its write: -3 within the deadline, never a hang
  fake_hip::configure(n);
  fake_hip::hang(n > 3 ? 3 : n - 1);
  setenv("NOS_BARRIER_DEADLINE_MS", "200", 1);
  o = barrier(n, yes);
  unsetenv("NOS_BARRIER_DEADLINE_MS");
  // (well under the 10 s default: the 200 ms deadline applied; loose enough for a loaded sanitizer run)
  report("hung_device_deadline", n, o, o.rc == -3 && o.ms < 5000.0 &&
                                           o.res.err.find("did not complete") != std::string::npos);

  // 7. a second barrier on the same devices: links already enabled are reused, not an error
  fake_hip::configure(n);
  Outcome first = barrier(n, yes);
  o = barrier(n, yes);
  report("repeat_reuses_links", n, o, first.rc == 0 && o.rc == 0 && o.sum == n && fake_hip::enabled_links() == n);

  // 8. the fake itself: a write into another device's memory without peer access enabled faults
  //    that device (so a barrier that skipped the enable would be caught by the scenarios above)
  fake_hip::configure(2);
  uint32_t* far = nullptr;
  hipEvent_t ev = nullptr;
  hipSetDevice(1);
  hipMalloc(reinterpret_cast<void**>(&far), nos_p2p::kLanes * sizeof(uint32_t));
  hipSetDevice(0);
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  fake_hip::launch_write(far, 1u, nos_p2p::kLanes);
  hipEventRecord(ev, nullptr);
  hipError_t q = hipErrorNotReady;
  for (auto t = std::chrono::steady_clock::now(); q == hipErrorNotReady &&
       std::chrono::steady_clock::now() - t < std::chrono::seconds(20);) {
    q = hipEventQuery(ev);
    std::this_thread::yield();
  }
  hipEventDestroy(ev);
  const bool caught = q == hipErrorIllegalAddress && fake_hip::faults() == 1;
  std::printf("{\"scenario\": \"fake_catches_write_without_peer_access\", \"ok\": %s}\n", caught ? "true" : "false");
  if (!caught) ++g_failures;

  fake_hip::reset();
  std::printf("{\"selftest\": \"%s\", \"failures\": %d}\n", g_failures ? "failed" : "ok", g_failures);
  return g_failures ? 1 : 0;
}
