// nos node-atomic commit barrier over xGMI peer-to-peer writes (no communicator).
//
// The commit barrier must show that every logical device of the re-enumerated node executes and
// that the xGMI fabric between them carries traffic. An RCCL communicator shows that too, but its
// set-up dominates the cost of a commit: 1.7-1.9 s of ncclCommInitAll + 0.49 s of ncclCommDestroy
// for ONE device on the box, against 3-5 ms for the all-reduce itself
// (profiles/operator_gpu_report_r3_rccl.json) — paid on every flip, while the flipped GPU's pods
// wait. This barrier does the same check directly:
//
//   device d writes a 64-lane token (its vote, tagged with d) into a buffer on device (d+1) mod n
//   through peer access — a ring of P2P writes over xGMI, one per link of the ring — then every
//   token is read back and checked. The commit holds iff every device voted yes AND every token
//   arrived intact; a device that cannot execute, a peer link that cannot be enabled or a token that
//   did not arrive is a veto.
//
// Each lane stores its own element (lane-indexed addresses: plain vector stores).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {
constexpr int kLanes = 64;
constexpr uint32_t kYes = 0x6e6f7331u;  // "nos1"
constexpr uint32_t kNo = 0x6e6f7330u;   // "nos0"

thread_local std::string g_p2p_err;

__global__ void ring_put(uint32_t* __restrict__ peer, uint32_t token) {
  const int lane = threadIdx.x;
  if (lane < kLanes) peer[lane] = token ^ static_cast<uint32_t>(lane);
}

int fail(const char* what, hipError_t e) {
  g_p2p_err = std::string(what) + ": " + hipGetErrorString(e);
  return int(e) ? int(e) : -1;
}
}  // namespace

extern "C" {

const char* nos_p2p_last_error() { return g_p2p_err.c_str(); }

// votes[d] != 0: device d's own checks passed. *sum = devices whose yes-vote arrived intact over
// the ring; *intact = tokens (yes or no) that arrived intact. Returns 0, or a HIP error code.
int nos_p2p_barrier(int n, const int32_t* votes, int32_t* sum, int32_t* intact) {
  *sum = 0;
  *intact = 0;
  if (n <= 0) {
    g_p2p_err = "no devices";
    return -1;
  }
  std::vector<uint32_t*> slot(n, nullptr);
  int rc = 0;
  for (int d = 0; d < n && !rc; ++d) {
    hipError_t e = hipSetDevice(d);
    if (e == hipSuccess) e = hipMalloc(&slot[d], kLanes * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(slot[d], 0, kLanes * sizeof(uint32_t));
    if (e != hipSuccess) rc = fail("device alloc", e);
  }
  for (int d = 0; d < n && !rc && n > 1; ++d) {
    const int peer = (d + 1) % n;
    int can = 0;
    hipError_t e = hipDeviceCanAccessPeer(&can, d, peer);
    if (e != hipSuccess) {
      rc = fail("hipDeviceCanAccessPeer", e);
      break;
    }
    if (!can) {
      g_p2p_err = "device " + std::to_string(d) + " cannot reach device " + std::to_string(peer) + " (no P2P path)";
      rc = -2;
      break;
    }
    e = hipSetDevice(d);
    if (e == hipSuccess) e = hipDeviceEnablePeerAccess(peer, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) {
      (void)hipGetLastError();
      e = hipSuccess;
    }
    if (e != hipSuccess) rc = fail("hipDeviceEnablePeerAccess", e);
  }
  for (int d = 0; d < n && !rc; ++d) {
    const uint32_t token = (votes[d] ? kYes : kNo) ^ (static_cast<uint32_t>(d) << 8);
    hipError_t e = hipSetDevice(d);
    if (e == hipSuccess) {
      ring_put<<<1, kLanes>>>(slot[(d + 1) % n], token);
      e = hipGetLastError();
    }
    if (e != hipSuccess) rc = fail("ring_put launch", e);
  }
  for (int d = 0; d < n && !rc; ++d) {
    hipError_t e = hipSetDevice(d);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) rc = fail("ring_put", e);
  }
  if (!rc) {
    std::vector<uint32_t> got(kLanes);
    for (int d = 0; d < n && !rc; ++d) {
      const int src = (d - 1 + n) % n;
      hipError_t e = hipSetDevice(d);
      if (e == hipSuccess) e = hipMemcpy(got.data(), slot[d], kLanes * sizeof(uint32_t), hipMemcpyDeviceToHost);
      if (e != hipSuccess) {
        rc = fail("read back", e);
        break;
      }
      const uint32_t yes = kYes ^ (static_cast<uint32_t>(src) << 8), no = kNo ^ (static_cast<uint32_t>(src) << 8);
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
    if (slot[d]) {
      (void)hipSetDevice(d);
      (void)hipFree(slot[d]);
    }
  }
  return rc;
}

}  // extern "C"
