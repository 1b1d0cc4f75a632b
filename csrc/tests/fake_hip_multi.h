// Multi-device host fake of the HIP runtime subset the commit barrier's host code uses
// (csrc/p2p_barrier_host.h), for CPU tests of its n > 1 paths (tests/test_p2p_barrier_host.py):
//
//   * n devices, each with its own worker thread executing its launches in order; events complete
//     when the device's worker has run every launch recorded before them;
//   * a peer matrix (hipDeviceCanAccessPeer), peer links whose hipDeviceEnablePeerAccess fails;
//   * a write into another device's memory without peer access enabled faults that device (the
//     error surfaces at its next event query, as an asynchronous GPU fault would);
//   * devices that never complete (hung), and devices whose writes arrive corrupted.
//
// Device memory is host memory, so the workers' writes and the host's read-back are real
// cross-thread accesses that ThreadSanitizer checks.
#pragma once

#include <cstddef>
#include <cstdint>

typedef int hipError_t;
enum : int {
  hipSuccess = 0,
  hipErrorInvalidValue = 1,
  hipErrorOutOfMemory = 2,
  hipErrorInvalidDevice = 101,
  hipErrorInvalidResourceHandle = 400,
  hipErrorNotReady = 600,
  hipErrorIllegalAddress = 700,
  hipErrorPeerAccessUnsupported = 217,
  hipErrorPeerAccessAlreadyEnabled = 704,
};
enum hipMemcpyKind { hipMemcpyHostToHost = 0, hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice,
                     hipMemcpyDefault };
constexpr unsigned hipEventDisableTiming = 2;

struct FakeHipEvent;
typedef FakeHipEvent* hipEvent_t;
typedef void* hipStream_t;

hipError_t hipSetDevice(int d);
hipError_t hipGetLastError();
const char* hipGetErrorString(hipError_t e);
hipError_t hipMalloc(void** p, size_t n);
hipError_t hipFree(void* p);
hipError_t hipMemset(void* p, int v, size_t n);
hipError_t hipMemcpy(void* dst, const void* src, size_t n, hipMemcpyKind kind);
hipError_t hipEventCreateWithFlags(hipEvent_t* ev, unsigned flags);
hipError_t hipEventRecord(hipEvent_t ev, hipStream_t stream);
hipError_t hipEventQuery(hipEvent_t ev);
hipError_t hipEventDestroy(hipEvent_t ev);
hipError_t hipDeviceCanAccessPeer(int* can, int dev, int peer);
hipError_t hipDeviceEnablePeerAccess(int peer, unsigned flags);

namespace fake_hip {
void configure(int n);                 // n fresh devices, fully connected, nothing enabled
void reset();                          // stop the workers (pending launches are dropped), free everything
void set_no_peer(int i, int j);        // no P2P path between i and j (both directions)
void fail_enable(int i, int j);        // hipDeviceEnablePeerAccess(j) on device i fails
void hang(int d);                      // device d never runs its launches
void corrupt(int d);                   // device d's writes arrive with one lane flipped
// a lanes-wide token write on the current device: lane l of dst = token ^ l
hipError_t launch_write(uint32_t* dst, uint32_t token, int lanes);
int enabled_links();                   // peer links enabled so far
int faults();                          // devices that faulted (e.g. a write without peer access)
size_t live_allocations();
}  // namespace fake_hip
