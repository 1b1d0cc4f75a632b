// Device helpers shared by the x3 attention kernels of kernels.hip and attn_wide.hip: the vector
// types, the exact three-bf16-plane split of fp32 ("x3", see kernels.hip "fp32 as three bf16
// planes"), the 32x32 MFMA accumulator layout, the stream-K bookkeeping and the LDS tile strides.
// attn_wide.hip is its own translation unit because it is compiled with its own code-generation
// options (walkai_nos_amd/ops/build.py); every helper here is inline and TU-local.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace {

template <typename F, typename H>
__device__ __forceinline__ void split3(const F& x, H& a, H& b, H& c) {
  a = __builtin_convertvector(x, H);  // v_cvt_pk_bf16_f32: round to nearest even
  const F r = x - __builtin_convertvector(a, F);
  b = __builtin_convertvector(r, H);
  c = __builtin_convertvector(r - __builtin_convertvector(b, F), H);
}

// store v as three exact bf16 terms at y[i], y[plane + i], y[2*plane + i] (x3 format).
// The empty asm pins v as a rounded f32: a caller's product (o * inv) would otherwise be contracted
// into the first residual (fma(o, inv, -h0)), splitting a value the fp32 output never holds — and
// whether the compiler contracts differs kernel to kernel.
__device__ __forceinline__ void store_x3(__bf16* __restrict__ y, size_t plane, size_t i, float v) {
  asm volatile("" : "+v"(v));
  const __bf16 h0 = (__bf16)v;
  const float r1 = v - (float)h0;
  const __bf16 h1 = (__bf16)r1;
  y[i] = h0;
  y[plane + i] = h1;
  y[2 * plane + i] = (__bf16)(r1 - (float)h1);
}

// head dimension of every attention kernel
constexpr int HD = 64;

// the key (or head dim) that accumulator register `reg` of lane half `half` holds (32x32 MFMA)
__device__ __forceinline__ int key_of(int reg, int half) { return (reg & 3) + 8 * (reg >> 2) + 4 * half; }

// lane l and lane l^32 combined without the LDS crossbar: v_permlane32_swap with the value as both
// operands leaves {x[l%32]} in one result and {x[32 + l%32]} in the other, on every lane (a VALU op,
// where __shfl_xor's ds_bpermute is an LDS round trip on the softmax critical path)
__device__ __forceinline__ float half_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// stream-K: wave w of P owns the units [w*U/P, (w+1)*U/P)
__device__ __forceinline__ long long sk_begin(long long w, long long U, long long P) { return w * U / P; }

// floor(n / d) for 0 <= n < 2^23 through the f32 reciprocal rd = 1/d (within one of the quotient
// there; one integer correction makes it exact): the stream-K bookkeeping of a segment as a few
// vector instructions instead of 64-bit scalar divisions (~150 instructions each, before the
// segment's first load can be addressed)
__device__ __forceinline__ long long udiv23(long long n, long long d, float rd) {
  int q = int(float(int(n)) * rd);
  const int r = int(n) - q * int(d);
  q += (r < 0) ? -1 : (r >= int(d) ? 1 : 0);
  return q;
}

// D += A·B with A, B given as three bf16 planes each (6 MFMAs, small terms first)
__device__ __forceinline__ f32x16 mfma_x3(const bf16x8& a0, const bf16x8& a1, const bf16x8& a2, const bf16x8& b0,
                                          const bf16x8& b1, const bf16x8& b2, f32x16 d) {
  d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, d, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, d, 0, 0, 0);
}

// LDS tiles of the x3 kernels (bf16 elements): K rows of 64 dims padded to 72, V^T read groups at
// a 96-element row stride (kernels.hip "x3 attention": conflict-free ds_read_b128 / read_tr16)
constexpr int XK_STR = 72, XV_STR = 96;
constexpr int XK_PLANE = 32 * XK_STR, XV_PLANE = 32 * XV_STR;

}  // namespace

// attn_wide.hip: the one-wave-per-SIMD fp32-input x3 attention (attn_fwd_x3w) — launch (returns the
// launch's hipError_t; cnt: B*H*QG zeroed row counters for the in-kernel stream-K merge, or nullptr
// to leave split tiles' partials for attn_sk_lds_fixup) and resident workgroups per CU
int nos_attn_x3w_launch(bool fdiv, dim3 grid, hipStream_t s, const float* qkv, float* out, __bf16* outp,
                        float* part_o, float* part_ml, int B, int T, int H, int h0, int Ht, float scale_log2e, int Pk,
                        int* cnt);
int nos_attn_x3w_occupancy();
