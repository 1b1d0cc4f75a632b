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
// The host logic lives in csrc/p2p_barrier_host.h (run on a CPU against a multi-device fake of the
// HIP API by tests/test_p2p_barrier_host.py); this file adds the token-write kernel and the C ABI.
// Each lane stores its own element (lane-indexed addresses: plain vector stores).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "p2p_barrier_host.h"

namespace {
__global__ void ring_put(uint32_t* __restrict__ dst, uint32_t token) {
  const int lane = threadIdx.x;
  if (lane < nos_p2p::kLanes) dst[lane] = token ^ static_cast<uint32_t>(lane);
}

thread_local nos_p2p::Result g_last;
}  // namespace

hipError_t nos_p2p::ring_put_launch(uint32_t* dst, uint32_t token) {
  ring_put<<<1, nos_p2p::kLanes>>>(dst, token);
  return hipGetLastError();
}

extern "C" {

const char* nos_p2p_last_error() { return g_last.err.c_str(); }
// the ring of the last barrier ("0>1>2>0", "0>1*;2*": * = a local write) and its link counts
const char* nos_p2p_last_plan() { return g_last.plan.c_str(); }
int nos_p2p_last_peer_links() { return g_last.peer; }
int nos_p2p_last_local() { return g_last.local; }

// votes[d] != 0: device d's own checks passed. *sum = devices whose yes-vote arrived intact;
// *intact = tokens (yes or no) that arrived intact. Returns 0, or a HIP error code / negative value.
int nos_p2p_barrier(int n, const int32_t* votes, int32_t* sum, int32_t* intact) {
  return nos_p2p::run(n, votes, sum, intact, g_last);
}

}  // extern "C"
