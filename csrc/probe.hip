// nos slice probe: MFMA-saturating, LDS-resident CDNA4 kernels that measure what a GPU slice
// (a compute partition, or a CU-masked stream) can actually deliver, plus an HBM stream probe and
// a workgroup-placement census.  Exposed through a plain C ABI (ctypes) so the node agent can run
// it without PyTorch; inside a PyTorch process the same HIP runtime instance is shared (one soname).
//
// Design (gfx950, MI355X_MICROARCH.md "Matrix cores" + "Per-instruction cycle constants"):
//  * 256-thread workgroups = 4 waves = one wave per SIMD; default 2 workgroups per CU.
//  * operands are random data staged once through LDS into eight register-resident (A, B) pairs
//    that the loop cycles through: the loop body is MFMAs only, matrix-pipe bound, and every MFMA
//    still sees different random operands (DVFS-realistic).
//  * four independent accumulators per wave; a 32x32x16 bf16 MFMA issues every 32 cycles per SIMD
//    = 1024 FLOP/clk/SIMD -> 2.5 PF dense at 2.4 GHz on 256 CUs.
//  * dtype variants: bf16 32x32x16, bf16 16x16x32, f32-input 32x32x2 (exact fp32, 1/16 rate),
//    fp8 e4m3 32x32x16 (bf16 rate, non-scaled form).
//  * census: each workgroup records HW_REG_HW_ID (CU/SE ids) and HW_REG_XCC_ID so CU-mask bit ->
//    XCD placement can be verified on the box.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;

namespace {
thread_local std::string g_err;

int check(hipError_t e, const char* what) {
  if (e == hipSuccess) return 0;
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return int(e);
}

constexpr int kThreads = 256;
constexpr int kLdsVec = 1024;  // uint4 entries = 16 KiB of operand tiles per workgroup

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

template <int DTYPE>
__global__ __launch_bounds__(kThreads) void mfma_probe(const uint4* __restrict__ src, uint32_t src_len,
                                                      float* __restrict__ out, int iters,
                                                      unsigned long long* __restrict__ clk) {
  // Operands: random data staged through LDS once, then held in registers as kOps distinct
  // (A, B) pairs that every iteration cycles through — each MFMA still sees different random
  // operands (DVFS-realistic toggling), but the loop body is nothing but MFMAs: no LDS reads, no
  // address arithmetic, one scalar loop branch per kOps MFMAs (the r1 loop re-read both operands
  // from LDS every 4 MFMAs and reached 78-83% of the clock peak).
  constexpr int kOps = 8;
  __shared__ uint4 lds[kLdsVec];
  const int t = threadIdx.x;
  for (int i = t; i < kLdsVec; i += kThreads) lds[i] = src[(blockIdx.x * 131u + i) % src_len];
  __syncthreads();
  uint4 ra[kOps], rb[kOps];
#pragma unroll
  for (int k = 0; k < kOps; ++k) {
    ra[k] = lds[(t * 3 + k * 97) & (kLdsVec - 1)];
    rb[k] = lds[(t * 5 + k * 61 + 512) & (kLdsVec - 1)];
  }
  // shader-clock cycles (s_memtime) vs the constant-rate wall clock (s_memrealtime) over the loop:
  // their ratio is the core clock the matrix pipes actually ran at under this load (DVFS).
  const unsigned long long c0 = clock64(), w0 = wall_clock64();

  float result = 0.f;
  if constexpr (DTYPE == 0) {  // bf16 32x32x16
    f32x16 acc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = f32x16{0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < kOps; ++k)
        acc[k & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf16x8(ra[k]), as_bf16x8(rb[k]), acc[k & 3], 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) result += acc[k][r];
  } else if constexpr (DTYPE == 1) {  // bf16 16x16x32
    // one accumulator per MFMA of the unrolled body: with fewer, the compiler rotates accumulator
    // registers across iterations and consecutive MFMAs end up with overlapping source/destination
    // ranges (measured: 78% of the clock peak instead of 99%)
    f32x4 acc[2 * kOps];
#pragma unroll
    for (int k = 0; k < 2 * kOps; ++k) acc[k] = f32x4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < 2 * kOps; ++k)
        acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(ra[k & (kOps - 1)]), as_bf16x8(rb[(k + 3) & (kOps - 1)]),
                                                         acc[k], 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < 2 * kOps; ++k) result += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  } else if constexpr (DTYPE == 2) {  // f32-input 32x32x2 (exact fp32)
    f32x16 acc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = f32x16{0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < kOps; ++k)
        acc[k & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(__builtin_bit_cast(float, ra[k].x),
                                                          __builtin_bit_cast(float, rb[k].y), acc[k & 3], 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) result += acc[k][r];
  } else if constexpr (DTYPE == 4) {  // fp8 e4m3, block-scaled 32x32x64 (2x the bf16 rate)
    f32x16 acc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = f32x16{0};
    i32x8 fa[kOps], fb[kOps];
#pragma unroll
    for (int k = 0; k < kOps; ++k) {
      const uint4 a0 = ra[k], a1 = ra[(k + 1) & (kOps - 1)], b0 = rb[k], b1 = rb[(k + 2) & (kOps - 1)];
      fa[k] = i32x8{int(a0.x), int(a0.y), int(a0.z), int(a0.w), int(a1.x), int(a1.y), int(a1.z), int(a1.w)};
      fb[k] = i32x8{int(b0.x), int(b0.y), int(b0.z), int(b0.w), int(b1.x), int(b1.y), int(b1.z), int(b1.w)};
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < kOps; ++k)  // format 0 = e4m3 for A and B, unit E8M0 scales (127 = 2^0)
        acc[k & 3] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[k], fb[k], acc[k & 3], 0, 0, 0, 127, 0, 127);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) result += acc[k][r];
  } else {  // fp8 e4m3 32x32x16
    f32x16 acc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = f32x16{0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int k = 0; k < kOps; ++k) {
        const long a = (long(ra[k].y) << 32) | ra[k].x, b = (long(rb[k].w) << 32) | rb[k].z;
        acc[k & 3] = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a, b, acc[k & 3], 0, 0, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int r = 0; r < 16; ++r) result += acc[k][r];
  }
  out[blockIdx.x * kThreads + t] = result;
  if (clk != nullptr && t == 0) {
    clk[2 * blockIdx.x] = clock64() - c0;
    clk[2 * blockIdx.x + 1] = wall_clock64() - w0;
  }
}

// FLOP per loop iteration per wave for each dtype variant
constexpr double kFlopPerIterWave[5] = {8.0 * 2 * 32 * 32 * 16, 16.0 * 2 * 16 * 16 * 32, 8.0 * 2 * 32 * 32 * 2,
                                        8.0 * 2 * 32 * 32 * 16, 8.0 * 2 * 32 * 32 * 64};

__global__ __launch_bounds__(kThreads) void hbm_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
  // Streaming copy: each lane keeps 8 x 16 B loads in flight (the guide's measured float4 copy
  // needs ~32 KiB in flight per CU to cover an HBM miss), and the non-temporal hint keeps the
  // once-touched lines from evicting the L2/Infinity-Cache working set of co-running partitions.
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
  constexpr int U = 8;
  const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
  u32x4* d4 = reinterpret_cast<u32x4*>(dst);
  const size_t stride = size_t(gridDim.x) * kThreads;
  size_t i = size_t(blockIdx.x) * kThreads + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = __builtin_nontemporal_load(s4 + i + k * stride);
#pragma unroll
    for (int k = 0; k < U; ++k) __builtin_nontemporal_store(v[k], d4 + i + k * stride);
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

// Slab copy: each workgroup streams one contiguous slab (DRAM page locality; the grid-stride form
// above makes every wave-instruction of a workgroup touch a different region of the buffer).
template <bool NT, int U>
__global__ __launch_bounds__(kThreads) void hbm_copy_slab(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                          size_t n) {
  typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
  const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
  u32x4* d4 = reinterpret_cast<u32x4*>(dst);
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t lo = size_t(blockIdx.x) * per, hi = min(n, lo + per);
  size_t i = lo + threadIdx.x;
  for (; i + (U - 1) * kThreads < hi; i += U * kThreads) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = NT ? __builtin_nontemporal_load(s4 + i + k * kThreads) : s4[i + k * kThreads];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (NT)
        __builtin_nontemporal_store(v[k], d4 + i + k * kThreads);
      else
        d4[i + k * kThreads] = v[k];
    }
  }
  for (; i < hi; i += kThreads) d4[i] = s4[i];
}

__global__ void fill_random(uint32_t* p, size_t n, uint32_t seed) {
  size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const size_t stride = size_t(gridDim.x) * blockDim.x;
  for (; i < n; i += stride) {
    uint32_t x = uint32_t(i) * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    // keep bf16/fp8 lanes finite and in [-1, 1): clear the top exponent bits of each 16-bit half
    p[i] = x & 0xBF7FBF7Fu;
  }
}

__global__ void census(uint32_t* out, int spin) {
  if (threadIdx.x == 0) {
    uint32_t hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));    // HW_REG_HW_ID
    uint32_t xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));  // HW_REG_XCC_ID
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
  // hold the CU briefly so that the dispatcher spreads the grid over every enabled CU
  for (volatile int i = 0; i < spin; ++i) {
  }
}

struct Scratch {
  int device = -1;
  uint4* src = nullptr;
  uint32_t src_len = 0;
  float* out = nullptr;
  size_t out_len = 0;
  unsigned long long* clk = nullptr;
  size_t clk_len = 0;
};
thread_local Scratch g_s;

int ensure_scratch(int device, int n_wg) {
  if (g_s.device != device) {
    g_s = Scratch{};
    g_s.device = device;
  }
  if (!g_s.src) {
    g_s.src_len = 1u << 16;  // 1 MiB of random operands
    if (int rc = check(hipMalloc(&g_s.src, size_t(g_s.src_len) * sizeof(uint4)), "hipMalloc src")) return rc;
    hipLaunchKernelGGL(fill_random, dim3(256), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(g_s.src),
                       size_t(g_s.src_len) * 4, 0x9E3779B9u);
    if (int rc = check(hipGetLastError(), "fill_random")) return rc;
  }
  size_t need = size_t(n_wg) * kThreads;
  if (g_s.out_len < need) {
    if (g_s.out) hipFree(g_s.out);
    if (int rc = check(hipMalloc(&g_s.out, need * sizeof(float)), "hipMalloc out")) return rc;
    g_s.out_len = need;
  }
  if (g_s.clk_len < size_t(n_wg) * 2) {
    if (g_s.clk) hipFree(g_s.clk);
    if (int rc = check(hipMalloc(&g_s.clk, size_t(n_wg) * 2 * sizeof(unsigned long long)), "hipMalloc clk")) return rc;
    g_s.clk_len = size_t(n_wg) * 2;
  }
  return 0;
}

}  // namespace

extern "C" {

struct nos_probe_result {
  double ms;       // best-of-reps kernel time
  double flops;    // FLOP (or bytes moved for the HBM probe) per launch
  double rate;     // TFLOP/s (or GB/s)
  int32_t n_wg;
  double mhz;      // mean shader clock over the MFMA loop (0 for the HBM probe)
};

const char* nos_probe_last_error() { return g_err.c_str(); }

int nos_probe_device_count(int* n) { return check(hipGetDeviceCount(n), "hipGetDeviceCount"); }

int nos_probe_cu_count(int device, int* n) {
  hipDeviceProp_t p;
  if (int rc = check(hipGetDeviceProperties(&p, device), "hipGetDeviceProperties")) return rc;
  *n = p.multiProcessorCount;
  return 0;
}

// CU-masked stream (hipExtStreamCreateWithCUMask, hip_runtime_api.h:2999). n_words == 0 -> plain
// non-blocking stream.
int nos_stream_create(int device, const uint32_t* mask, uint32_t n_words, void** stream_out) {
  if (int rc = check(hipSetDevice(device), "hipSetDevice")) return rc;
  hipStream_t s = nullptr;
  if (n_words > 0) {
    if (int rc = check(hipExtStreamCreateWithCUMask(&s, n_words, mask), "hipExtStreamCreateWithCUMask")) return rc;
  } else {
    if (int rc = check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate")) return rc;
  }
  *stream_out = s;
  return 0;
}

int nos_stream_get_cumask(void* stream, uint32_t n_words, uint32_t* mask) {
  return check(hipExtStreamGetCUMask(reinterpret_cast<hipStream_t>(stream), n_words, mask), "hipExtStreamGetCUMask");
}

int nos_stream_destroy(void* stream) {
  return check(hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)), "hipStreamDestroy");
}

int nos_probe_mfma(int device, void* stream, int dtype, int n_wg, int iters, int reps, nos_probe_result* res) {
  if (dtype < 0 || dtype > 4 || n_wg <= 0 || iters <= 0 || reps <= 0) {
    g_err = "invalid probe arguments";
    return -1;
  }
  if (int rc = check(hipSetDevice(device), "hipSetDevice")) return rc;
  if (int rc = ensure_scratch(device, n_wg)) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto launch = [&]() {
    switch (dtype) {
      case 0: hipLaunchKernelGGL(mfma_probe<0>, dim3(n_wg), dim3(kThreads), 0, s, g_s.src, g_s.src_len, g_s.out, iters, g_s.clk); break;
      case 1: hipLaunchKernelGGL(mfma_probe<1>, dim3(n_wg), dim3(kThreads), 0, s, g_s.src, g_s.src_len, g_s.out, iters, g_s.clk); break;
      case 2: hipLaunchKernelGGL(mfma_probe<2>, dim3(n_wg), dim3(kThreads), 0, s, g_s.src, g_s.src_len, g_s.out, iters, g_s.clk); break;
      case 4: hipLaunchKernelGGL(mfma_probe<4>, dim3(n_wg), dim3(kThreads), 0, s, g_s.src, g_s.src_len, g_s.out, iters, g_s.clk); break;
      default: hipLaunchKernelGGL(mfma_probe<3>, dim3(n_wg), dim3(kThreads), 0, s, g_s.src, g_s.src_len, g_s.out, iters, g_s.clk); break;
    }
  };
  launch();  // warm-up (code object load, clocks)
  if (int rc = check(hipStreamSynchronize(s), "warm-up")) return rc;
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(e0, s);
    launch();
    hipEventRecord(e1, s);
    if (int rc = check(hipEventSynchronize(e1), "probe")) return rc;
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  res->ms = best;
  res->flops = kFlopPerIterWave[dtype] * double(iters) * double(n_wg) * (kThreads / 64);
  res->rate = res->flops / (best * 1e-3) / 1e12;
  res->n_wg = n_wg;
  // clock of the last rep: sum of shader cycles / sum of wall ticks x wall-clock rate
  res->mhz = 0;
  int wall_khz = 0;
  if (hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && wall_khz > 0) {
    std::vector<unsigned long long> h(size_t(n_wg) * 2);
    if (hipMemcpy(h.data(), g_s.clk, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost) == hipSuccess) {
      double cyc = 0, wall = 0;
      for (int i = 0; i < n_wg; ++i) {
        cyc += double(h[2 * i]);
        wall += double(h[2 * i + 1]);
      }
      if (wall > 0) res->mhz = cyc / wall * (wall_khz / 1000.0);
    }
  }
  return 0;
}

// mode 0: grid-stride non-temporal copy; 1: slab, non-temporal, 8 loads in flight per lane;
// 2: slab, default cache policy; 3: slab, non-temporal, 16 in flight; 4: slab, non-temporal, 4
int nos_probe_hbm_mode(int device, void* stream, size_t bytes, int n_wg, int reps, int mode, nos_probe_result* res);

int nos_probe_hbm(int device, void* stream, size_t bytes, int n_wg, int reps, nos_probe_result* res) {
  return nos_probe_hbm_mode(device, stream, bytes, n_wg, reps, 1, res);
}

int nos_probe_hbm_mode(int device, void* stream, size_t bytes, int n_wg, int reps, int mode, nos_probe_result* res) {
  if (int rc = check(hipSetDevice(device), "hipSetDevice")) return rc;
  size_t n = bytes / sizeof(uint4);
  uint4 *a = nullptr, *b = nullptr;
  if (int rc = check(hipMalloc(&a, n * sizeof(uint4)), "hipMalloc a")) return rc;
  if (int rc = check(hipMalloc(&b, n * sizeof(uint4)), "hipMalloc b")) { hipFree(a); return rc; }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(fill_random, dim3(1024), dim3(256), 0, s, reinterpret_cast<uint32_t*>(a), n * 4, 1234u);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto launch = [&]() {
    if (mode == 0)
      hipLaunchKernelGGL(hbm_copy, dim3(n_wg), dim3(kThreads), 0, s, a, b, n);
    else if (mode == 1)
      hipLaunchKernelGGL((hbm_copy_slab<true, 8>), dim3(n_wg), dim3(kThreads), 0, s, a, b, n);
    else if (mode == 2)
      hipLaunchKernelGGL((hbm_copy_slab<false, 8>), dim3(n_wg), dim3(kThreads), 0, s, a, b, n);
    else if (mode == 3)
      hipLaunchKernelGGL((hbm_copy_slab<true, 16>), dim3(n_wg), dim3(kThreads), 0, s, a, b, n);
    else
      hipLaunchKernelGGL((hbm_copy_slab<true, 4>), dim3(n_wg), dim3(kThreads), 0, s, a, b, n);
  };
  launch();
  int rc = check(hipStreamSynchronize(s), "hbm warm-up");
  float best = 1e30f;
  for (int r = 0; r < reps && rc == 0; ++r) {
    hipEventRecord(e0, s);
    launch();
    hipEventRecord(e1, s);
    rc = check(hipEventSynchronize(e1), "hbm probe");
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(a);
  hipFree(b);
  if (rc) return rc;
  res->ms = best;
  res->flops = 2.0 * double(n) * sizeof(uint4);
  res->rate = res->flops / (best * 1e-3) / 1e9;
  res->n_wg = n_wg;
  res->mhz = 0;
  return 0;
}

int nos_probe_census(int device, void* stream, int n_wg, int spin, uint32_t* host_out) {
  if (int rc = check(hipSetDevice(device), "hipSetDevice")) return rc;
  uint32_t* d = nullptr;
  if (int rc = check(hipMalloc(&d, size_t(n_wg) * 2 * sizeof(uint32_t)), "hipMalloc census")) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(census, dim3(n_wg), dim3(64), 0, s, d, spin);
  int rc = check(hipStreamSynchronize(s), "census");
  if (rc == 0) rc = check(hipMemcpy(host_out, d, size_t(n_wg) * 2 * sizeof(uint32_t), hipMemcpyDeviceToHost), "census copy");
  hipFree(d);
  return rc;
}

}  // extern "C"
