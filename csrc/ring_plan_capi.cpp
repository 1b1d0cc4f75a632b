// C entry point of the commit-barrier ring plan (csrc/ring_plan.h) for host-side tests: the same
// header the native helper links, exposed through a host-only shared library (no HIP).
#include <cstddef>
#include <cstdint>
#include <vector>

#include "ring_plan.h"

extern "C" {

// Steps (one per device) into src/dst/region (each of capacity n); returns the step count, or -1.
int nos_ring_plan(int n, const uint8_t* can, int* src, int* dst, int* region, int* peer_links, int* local,
                  int* closed) {
  if (n <= 0 || can == nullptr) return -1;
  std::vector<uint8_t> m(can, can + static_cast<size_t>(n) * n);
  const nos::RingPlan p = nos::plan_ring(n, m);
  for (std::size_t k = 0; k < p.steps.size(); ++k) {
    src[k] = p.steps[k].src;
    dst[k] = p.steps[k].dst;
    region[k] = p.steps[k].region;
  }
  *peer_links = p.peer_links;
  *local = p.local;
  *closed = p.closed;
  return static_cast<int>(p.steps.size());
}

}  // extern "C"
