// Packed fp32 epilogue math for gfx950: exact-erf GELU and the x3 plane split on pairs of values.
//
// A lane's accumulator registers r, r+1 (r even) hold two adjacent rows of one output column, so
// the epilogue works on float pairs: v_pk_fma/mul/add_f32 do both in one issue, and
// v_cvt_pk_bf16_f32 rounds both to bf16 in one. Per value this is ~14 VALU issues for GELU + split
// where erff() + scalar converts took ~45 (ocml's erff evaluates both of its branches for a wave
// whose values straddle |z| = 1, as the fc1 pre-activations always do).
//
// erf(z), |z| < 1: z + z*P(z^2), P of degree 5; |z| >= 1: 1 - exp(-z^2) * R(min(|z|, 4) - 2.5), R
// of degree 7 (erf = 1 in fp32 past 3.92). Coefficients: weighted least squares on the absolute
// error of erf (tools/erf_fit.py); in fp32 the max |error| of erf is 7.0e-8 and of GELU 3.3e-7
// over [-12, 12], against 4.5e-7 for the textbook fp32 formula with a correctly rounded erf.
#pragma once
#include <hip/hip_runtime.h>

typedef float nos_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 nos_bf2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ nos_f2 nos_f2s(float a) { return nos_f2{a, a}; }

__device__ __forceinline__ nos_f2 nos_fma2(nos_f2 a, nos_f2 b, nos_f2 c) { return __builtin_elementwise_fma(a, b, c); }

__device__ __forceinline__ nos_f2 nos_erf2(nos_f2 z) {
  const nos_f2 az = __builtin_elementwise_abs(z);
  const nos_f2 u = az * az;
  // |z| < 1
  nos_f2 p = nos_f2s(-5.463449634e-04f);
  p = nos_fma2(u, p, nos_f2s(4.870838486e-03f));
  p = nos_fma2(u, p, nos_f2s(-2.666393667e-02f));
  p = nos_fma2(u, p, nos_f2s(1.127806902e-01f));
  p = nos_fma2(u, p, nos_f2s(-3.761194050e-01f));
  p = nos_fma2(u, p, nos_f2s(1.283789277e-01f));
  const nos_f2 small = nos_fma2(az, p, az);
  // |z| >= 1
  const nos_f2 zc = __builtin_elementwise_min(az, nos_f2s(4.f));
  const nos_f2 t = zc - nos_f2s(2.5f);
  nos_f2 r = nos_f2s(-3.887849161e-04f);
  r = nos_fma2(t, r, nos_f2s(-7.998283836e-04f));
  r = nos_fma2(t, r, nos_f2s(-1.961313887e-03f));
  r = nos_fma2(t, r, nos_f2s(1.966925571e-03f));
  r = nos_fma2(t, r, nos_f2s(-7.804186549e-03f));
  r = nos_fma2(t, r, nos_f2s(2.515763976e-02f));
  r = nos_fma2(t, r, nos_f2s(-7.429978251e-02f));
  r = nos_fma2(t, r, nos_f2s(2.108065486e-01f));
  const nos_f2 ex = (zc * zc) * nos_f2s(-1.4426950408889634f);
  const nos_f2 e = nos_f2{__builtin_amdgcn_exp2f(ex.x), __builtin_amdgcn_exp2f(ex.y)};
  const nos_f2 big = nos_fma2(-e, r, nos_f2s(1.f));
  const nos_f2 m = nos_f2{az.x < 1.f ? small.x : big.x, az.y < 1.f ? small.y : big.y};
  return nos_f2{__builtin_copysignf(m.x, z.x), __builtin_copysignf(m.y, z.y)};
}

// GELU(x) = x/2 * (1 + erf(x / sqrt 2))
__device__ __forceinline__ nos_f2 nos_gelu2(nos_f2 x) {
  const nos_f2 hx = x * nos_f2s(0.5f);
  return nos_fma2(hx, nos_erf2(x * nos_f2s(0.70710678118654752f)), hx);
}

// x = x0 + x1 + x2 exactly, each plane the round-to-nearest bf16 of the remaining residual; for two
// values at once (pl[q] holds plane q of both)
__device__ __forceinline__ void nos_split3_pair(nos_f2 v, nos_bf2 (&pl)[3]) {
  pl[0] = __builtin_convertvector(v, nos_bf2);
  const nos_f2 r1 = v - __builtin_convertvector(pl[0], nos_f2);
  pl[1] = __builtin_convertvector(r1, nos_bf2);
  pl[2] = __builtin_convertvector(r1 - __builtin_convertvector(pl[1], nos_f2), nos_bf2);
}
