// Partition pinning: a compute partition emulated on an SPX device runs on ITS OWN XCDs.
//
// A real CPX partition is one XCD — 32 CUs and a private 4 MB L2; QPX two XCDs, DPX four. A CU
// mask cannot emulate that on SPX: an XCD whose mask bits are all zero is not disabled but fully
// enabled (profiles/xcd_mask_probe_r2.json), so the previous emulation spread every slice over all
// eight XCDs, and eight concurrent slices then replicated each other's operands into all eight L2s.
// A pinned launch instead dispatches 8 * ceil(n / nx) workgroups for n logical ones (nx = XCDs in
// the partition's mask): the dispatcher deals consecutive workgroups to the 8 XCDs in turn (blocks
// b .. b+7 of one dispatch land on 8 distinct XCDs; which XCD block 0 gets is not fixed), so a block
// reads its XCD from HW_REG_XCC_ID, exits at once if that XCD is outside the mask, and otherwise is
// logical block (b / 8) * nx + (rank of its XCD in the mask). tests/test_gpu_pin.py checks on the
// GPU, under 8 concurrent streams, that every logical block runs exactly once and only on its XCDs.
//
// The mask rides into each kernel as an argument (0 = unpinned: block b is logical block b of
// gridDim.x, and the XCD-major remaps assume all 8 XCDs).
#pragma once
#include <hip/hip_runtime.h>

struct PinnedBlock {
  int id;  // logical block, -1 = not this partition's XCD (exit)
  int n;   // logical blocks of the launch (>= the n the host asked for)
  int nx;  // XCDs the logical blocks are dealt over (8 unpinned)
};

__device__ __forceinline__ int xcc_id() { return int(__builtin_amdgcn_s_getreg(20 | (31 << 11)) & 15); }

__device__ __forceinline__ PinnedBlock pinned_block(unsigned pin) {
  if (!pin) return {int(blockIdx.x), int(gridDim.x), 8};
  const unsigned x = unsigned(xcc_id());
  const int nx = __builtin_popcount(pin);
  if (!((pin >> x) & 1u)) return {-1, 0, nx};
  return {int(blockIdx.x / 8) * nx + __builtin_popcount(pin & ((1u << x) - 1u)), int(gridDim.x / 8) * nx, nx};
}

// Logical block `phys` of n dealt round-robin over nx XCDs (phys % nx = XCD): XCD x gets the
// contiguous logical range starting at x*(n/nx) + min(x, n%nx). A bijection on [0, n) for every n.
__device__ __forceinline__ int xcd_major_n(int phys, int n, int nx) {
  const int x = phys % nx, q = n / nx, r = n % nx;
  return x * q + min(x, r) + phys / nx;
}

// physical grid of a launch of n logical blocks
inline unsigned pinned_grid(unsigned n, unsigned pin) {
  if (!pin) return n;
  const unsigned nx = unsigned(__builtin_popcount(pin));
  return 8u * ((n + nx - 1u) / nx);
}

// Logical grid of a grid-stride kernel under a pin: every physical workgroup outside the mask is a
// wave launch that only exits, so pinned grid-stride launches keep 64 workgroups per XCD (2 per CU).
inline unsigned pinned_cap(unsigned n, unsigned pin) {
  if (!pin) return n;
  const unsigned cap = 64u * unsigned(__builtin_popcount(pin));
  return n < cap ? n : cap;
}

// the enqueuing thread's pin (set per slice, like its CU count)
extern "C" unsigned nos_pin_mask();
