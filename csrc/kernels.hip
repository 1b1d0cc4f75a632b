// nos workload kernels for gfx950 (MI355X): the hot ops of the fp32 YOLOS-small fractional-GPU
// workload (the GEMMs are in gemm.hip / gemm_x3.hip).
//
//  * attn_fwd_x3p: fp32-accurate flash attention on the bf16 matrix cores over the exact
//    three-bf16-plane ("x3") form of Q/K/V, software-pipelined — see "fp32 as three bf16 planes"
//    below; attn_fwd_x3 is its block-at-a-time A/B reference. For fp32 QKV input (the model's path)
//    the production kernel is attn_fwd_x3w in attn_wide.hip (same units, partials and arithmetic,
//    one wave per SIMD carrying two query tiles), dispatched by attention_x3_launch below;
//  * attn_fwd_f32 / attn_fwd_sk / attn_fwd_sk_lds (the f32-MFMA path, set_fp32_matmul("f32")): flash attention over a packed [B, T, 3*H*64] fp32 QKV tensor on the exact-fp32
//    matrix cores (v_mfma_f32_32x32x2_f32, 64 FLOP/clk/SIMD). One wave owns 32 queries of one head.
//    It computes S^T = K Q^T so that every lane owns ONE query column: the softmax row reductions
//    are 16 in-register ops plus a single cross-half exchange (lane l <-> l^32), no LDS. The
//    accumulator of S^T is fed straight back as the B operand of O^T += V^T P^T (accumulator-as-
//    operand, cdna_hip_programming.md §3), so P never leaves registers. Head-dim -> MFMA K-slot
//    assignment is dim = 32*half + step, which makes every lane's Q and K fragment one contiguous
//    128-byte run (8 x dwordx4). K/V of one head (3401 x 64 x 4 B x 2 = 1.7 MB) stays L2-resident
//    across the query tiles of that head. The production launch is stream-K (attn_fwd_sk): a
//    persistent grid sized to the slice's resident-wave capacity splits the (query tile x key
//    block) work evenly, so a 32-CU CPX slice and the whole 256-CU GPU are both tail-free.
//  * layernorm_f32: two rows per wave in flight, values kept in registers (two-pass mean/variance), wave64
//    shuffles; writes fp32 or the x3 planes the next GEMM consumes.
//  * bias_gelu_f32: in-place exact (erf) GELU(y + b) epilogue, dwordx4 vectorised.
#include <hip/hip_runtime.h>

#include "pin.h"
#include "streamk.h"
#include "x3_common.h"

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <string>

namespace {
thread_local std::string g_err;

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) return 0;
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return int(e);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ------------------------------------------------------------------------------------------
// LayerNorm (output fp32 y, or x3 planes yp with plane stride rows*D when yp != nullptr). Lane l
// owns the column pairs (2l + 128i, 2l + 128i + 1): 8-B loads, and packed 4-B bf16-pair stores per
// plane on the x3 path. R rows per wave per iteration, all R loaded before any is reduced: a slice
// sharing the GPU runs a few waves per CU over many rows each, and each iteration is one memory
// round trip, so R rows in flight cut the round trips per wave by R.
template <int NPL, int R>
__global__ __launch_bounds__(256) void layernorm_f32(const float* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, float* __restrict__ y,
                                                     __bf16* __restrict__ yp, int rows, float eps, unsigned pin) {
  static_assert(NPL % 2 == 0, "hidden size must be a multiple of 128");
  const PinnedBlock pb = pinned_block(pin);
  if (pb.id < 0) return;
  constexpr int D = NPL * 64, NP = NPL / 2;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float2* w2 = reinterpret_cast<const float2*>(w);
  const float2* b2 = reinterpret_cast<const float2*>(b);
  const size_t plane2 = size_t(rows) * D / 2;  // plane stride in bf16 pairs
  // grid-stride over rows: a slice sharing the GPU launches a few workgroups per CU instead of one
  // per 4R rows (workgroup dispatch is what concurrent partitions contend for)
  const int stride = pb.n * 4;
  for (int row0 = pb.id * 4 + wave; row0 < rows; row0 += R * stride) {
    float2 v[R][NP];
    float mean[R], rstd[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      // rows past the end re-read the last row (in bounds) and are never stored
      const float2* xr = reinterpret_cast<const float2*>(x + size_t(min(row0 + k * stride, rows - 1)) * D);
#pragma unroll
      for (int i = 0; i < NP; ++i) v[k][i] = xr[i * 64 + lane];
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < NP; ++i) s += v[k][i].x + v[k][i].y;
      mean[k] = wave_sum(s) * (1.0f / D);
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        v[k][i].x -= mean[k];
        v[k][i].y -= mean[k];
        q += v[k][i].x * v[k][i].x + v[k][i].y * v[k][i].y;
      }
      rstd[k] = rsqrtf(wave_sum(q) * (1.0f / D) + eps);
    }
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int row = row0 + k * stride;
      if (row >= rows) break;
      if (yp) {
        uint32_t* dst = reinterpret_cast<uint32_t*>(yp) + size_t(row) * (D / 2);
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const int c2 = i * 64 + lane;
          const float2 ww = w2[c2], bb = b2[c2];
          const f32x2 val = {v[k][i].x * rstd[k] * ww.x + bb.x, v[k][i].y * rstd[k] * ww.y + bb.y};
          bf16x2 h0, h1, h2;
          split3(val, h0, h1, h2);
          dst[c2] = __builtin_bit_cast(uint32_t, h0);
          dst[plane2 + c2] = __builtin_bit_cast(uint32_t, h1);
          dst[2 * plane2 + c2] = __builtin_bit_cast(uint32_t, h2);
        }
      } else {
        float2* yr = reinterpret_cast<float2*>(y + size_t(row) * D);
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          const int c2 = i * 64 + lane;
          const float2 ww = w2[c2], bb = b2[c2];
          yr[c2] = make_float2(v[k][i].x * rstd[k] * ww.x + bb.x, v[k][i].y * rstd[k] * ww.y + bb.y);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Split-K combine + residuals + LayerNorm: x = (part_0 + ... + part_{S-1}) + bias + res (+ r2[row %
// r2_rows]) — the split-K GEMM's epilogue, in the same order as the fused one — stored as the fp32
// residual stream xout, and, when w is given, LayerNorm(x) stored as x3 planes yp (the next GEMM's
// operand). One wave per row, grid-stride, lanes on column pairs as layernorm_f32.
template <int NPL>
__global__ __launch_bounds__(256) void splitk_layernorm_f32(const float* __restrict__ part, int splits, SkMap sk,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ res,
                                                            const float* __restrict__ r2, int r2_rows,
                                                            float* __restrict__ xout, const float* __restrict__ w,
                                                            const float* __restrict__ b, __bf16* __restrict__ yp,
                                                            int rows, float eps, unsigned pin) {
  constexpr int D = NPL * 64, NP = NPL / 2;
  const PinnedBlock pb = pinned_block(pin);
  if (pb.id < 0) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t pstride = size_t(rows) * (D / 2);  // partial plane stride in float2
  const float2* p2 = reinterpret_cast<const float2*>(part);
  const float2* bias2 = reinterpret_cast<const float2*>(bias);
  for (int row = pb.id * 4 + wave; row < rows; row += pb.n * 4) {
    const size_t r2i = size_t(row) * (D / 2);
    float2 v[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) v[i] = p2[r2i + i * 64 + lane];
    if (sk.P > 0) {
      // stream-K partials: tile t of this row and column pair holds sk_segments(t) planes
      int ns[NP], most = 1;
      const int tr = (row / sk.bm) * sk.tiles_n;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        ns[i] = sk_segments(tr + (2 * (i * 64 + lane)) / sk.bn, sk);
        most = max(most, ns[i]);
      }
      for (int sp = 1; sp < most; ++sp) {
#pragma unroll
        for (int i = 0; i < NP; ++i) {
          if (sp < ns[i]) {
            const float2 q = p2[sp * pstride + r2i + i * 64 + lane];
            v[i].x += q.x;
            v[i].y += q.y;
          }
        }
      }
    }
    for (int sp = 1; sp < splits; ++sp) {
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const float2 q = p2[sp * pstride + r2i + i * 64 + lane];
        v[i].x += q.x;
        v[i].y += q.y;
      }
    }
    const float2* rr = reinterpret_cast<const float2*>(res) + r2i;
    const float2* rr2 = r2 ? reinterpret_cast<const float2*>(r2) + size_t(row % r2_rows) * (D / 2) : nullptr;
    float2* xo = reinterpret_cast<float2*>(xout) + r2i;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int c2 = i * 64 + lane;
      const float2 bb = bias2[c2], r = rr[c2];
      v[i].x = v[i].x + bb.x + r.x;
      v[i].y = v[i].y + bb.y + r.y;
      if (rr2) {
        const float2 q = rr2[c2];
        v[i].x += q.x;
        v[i].y += q.y;
      }
      xo[c2] = v[i];
      s += v[i].x + v[i].y;
    }
    if (!w) continue;
    const float mean = wave_sum(s) * (1.0f / D);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      v[i].x -= mean;
      v[i].y -= mean;
      q += v[i].x * v[i].x + v[i].y * v[i].y;
    }
    const float rstd = rsqrtf(wave_sum(q) * (1.0f / D) + eps);
    const float2* w2 = reinterpret_cast<const float2*>(w);
    const float2* b2 = reinterpret_cast<const float2*>(b);
    const size_t plane2 = size_t(rows) * D / 2;
    uint32_t* dst = reinterpret_cast<uint32_t*>(yp) + r2i;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int c2 = i * 64 + lane;
      const float2 ww = w2[c2], bb = b2[c2];
      const f32x2 val = {v[i].x * rstd * ww.x + bb.x, v[i].y * rstd * ww.y + bb.y};
      bf16x2 h0, h1, h2;
      split3(val, h0, h1, h2);
      dst[c2] = __builtin_bit_cast(uint32_t, h0);
      dst[plane2 + c2] = __builtin_bit_cast(uint32_t, h1);
      dst[2 * plane2 + c2] = __builtin_bit_cast(uint32_t, h2);
    }
  }
}

// ------------------------------------------------------------------------------------------
// bias + exact GELU, in place
__global__ __launch_bounds__(256) void bias_gelu_f32(float* __restrict__ y, const float* __restrict__ b, size_t n4,
                                                     int N4) {
  size_t i = size_t(blockIdx.x) * 256 + threadIdx.x;
  const size_t stride = size_t(gridDim.x) * 256;
  float4* y4 = reinterpret_cast<float4*>(y);
  const float4* b4 = reinterpret_cast<const float4*>(b);
  for (; i < n4; i += stride) {
    float4 v = y4[i];
    const float4 bb = b4[i % N4];
    v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
    v.x = 0.5f * v.x * (1.f + erff(v.x * 0.70710678118654752f));
    v.y = 0.5f * v.y * (1.f + erff(v.y * 0.70710678118654752f));
    v.z = 0.5f * v.z * (1.f + erff(v.z * 0.70710678118654752f));
    v.w = 0.5f * v.w * (1.f + erff(v.w * 0.70710678118654752f));
    y4[i] = v;
  }
}

// ------------------------------------------------------------------------------------------
// Flash attention, fp32, head_dim 64.
// (HD, key_of, half_max, half_sum: x3_common.h)

// Online-softmax flash attention over key blocks [kb0, kb1) (32 keys each) for the 32 queries
// q0..q0+31 of one head. Returns the unnormalised O^T accumulators and the running (m, l).
struct AttnAcc {
  f32x16 o0, o1;
  float m, l;
};

__device__ __forceinline__ AttnAcc attn_segment(const float* __restrict__ base, int q0, int head, int kb0, int kb1,
                                                int T, int D, float scale_log2e) {
  const int lane = threadIdx.x & 63;
  const int j = lane & 31, hf = lane >> 5;
  const int ld = 3 * D;
  // Q^T fragment: Q[q0 + j][32*hf + s], s = 0..31, pre-scaled into the log2 domain
  float qreg[32];
  {
    const int qrow = min(q0 + j, T - 1);
    const float4* qp = reinterpret_cast<const float4*>(base + size_t(qrow) * ld + head * HD + 32 * hf);
#pragma unroll
    for (int s4 = 0; s4 < 8; ++s4) {
      const float4 v = qp[s4];
      qreg[4 * s4 + 0] = v.x * scale_log2e;
      qreg[4 * s4 + 1] = v.y * scale_log2e;
      qreg[4 * s4 + 2] = v.z * scale_log2e;
      qreg[4 * s4 + 3] = v.w * scale_log2e;
    }
  }
  AttnAcc a;
  a.o0 = f32x16{0};
  a.o1 = f32x16{0};
  a.m = -INFINITY;
  a.l = 0.f;
  const float* kbase = base + D + head * HD + 32 * hf;
  const float* vbase = base + 2 * D + head * HD + j;

  for (int blk = kb0; blk < kb1; ++blk) {
    const int kb = blk * 32;
    // K fragment: K[kb + j][32*hf + s]
    float kreg[32];
    {
      const int krow = min(kb + j, T - 1);
      const float4* kp = reinterpret_cast<const float4*>(kbase + size_t(krow) * ld);
#pragma unroll
      for (int s4 = 0; s4 < 8; ++s4) {
        const float4 v = kp[s4];
        kreg[4 * s4 + 0] = v.x;
        kreg[4 * s4 + 1] = v.y;
        kreg[4 * s4 + 2] = v.z;
        kreg[4 * s4 + 3] = v.w;
      }
    }
    // V operands for this block, issued early to overlap the S^T MFMAs: V[kb + key(t, hf)][j], [32 + j]
    float v0[16], v1[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int vrow = min(kb + key_of(t, hf), T - 1);
      v0[t] = vbase[size_t(vrow) * ld];
      v1[t] = vbase[size_t(vrow) * ld + 32];
    }
    // S^T[key][query] = sum_d K[key][d] Q[query][d]
    f32x16 s = {0};
#pragma unroll
    for (int st = 0; st < 32; ++st) s = __builtin_amdgcn_mfma_f32_32x32x2f32(kreg[st], qreg[st], s, 0, 0, 0);

    if (kb + 32 > T) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (kb + key_of(r, hf) >= T) s[r] = -INFINITY;
    }
    float mx = s[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s[r]);
    mx = half_max(mx);
    const float m_new = fmaxf(a.m, mx);
    const float alpha = __builtin_amdgcn_exp2f(a.m - m_new);
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] = __builtin_amdgcn_exp2f(s[r] - m_new);
      psum += s[r];
    }
    psum = half_sum(psum);
    a.l = a.l * alpha + psum;
    a.m = m_new;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      a.o0[r] *= alpha;
      a.o1[r] *= alpha;
    }
    // O^T[d][query] += sum_key V^T[d][key] P^T[key][query]; P^T register t is key key_of(t, hf)
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      a.o0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v0[t], s[t], a.o0, 0, 0, 0);
      a.o1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v1[t], s[t], a.o1, 0, 0, 0);
    }
  }
  return a;
}

__device__ __forceinline__ void attn_store_out(const AttnAcc& a, float* __restrict__ out, int b, int q0, int head,
                                               int T, int D) {
  const int lane = threadIdx.x & 63;
  const int j = lane & 31, hf = lane >> 5;
  const int q = q0 + j;
  if (q >= T) return;
  const float inv = 1.f / a.l;
  float* orow = out + (size_t(b) * T + q) * D + head * HD;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int d = key_of(r, hf);
    orow[d] = a.o0[r] * inv;
    orow[32 + d] = a.o1[r] * inv;
  }
}

// One wave per (query tile, head, batch): the whole key range, normalised output. Used when no
// workspace is available (nos_attention_f32).
__global__ __launch_bounds__(64, 2) void attn_fwd_f32(const float* __restrict__ qkv, float* __restrict__ out, int T,
                                                      int H, float scale_log2e) {
  const int qt = blockIdx.x, head = blockIdx.y, b = blockIdx.z;
  const int D = H * HD;
  const AttnAcc a = attn_segment(qkv + size_t(b) * T * 3 * D, qt * 32, head, 0, (T + 31) / 32, T, D, scale_log2e);
  attn_store_out(a, out, b, qt * 32, head, T, D);
}

// ---- stream-K attention ----------------------------------------------------------------------
// The work is U = B*H*QT*NK units (one 32-query x 32-key block each, QT = NK = ceil(T/32)), laid out
// tile-major so consecutive units share a head's K/V. A persistent grid of exactly P waves (slice
// CUs x resident waves per CU) gives wave w the contiguous range [w*U/P, (w+1)*U/P): every SIMD of
// the slice gets the same number of MFMAs, so there is no wave-quantisation tail whatever the slice
// size (a fixed split count leaves 1.25 or 2.5 "rounds" for 256 or 32 CUs). Segments covering a
// whole tile are normalised and stored directly; a wave's first and last segments may be partial
// and go to its two workspace slots, merged by attn_sk_fixup (a second launch on the same stream,
// so no inter-wave spin-waits exist). Logical wave ids are XCD-major: hardware round-robins
// workgroups over the 8 XCDs, so remapping keeps each XCD on a contiguous run of units and its
// 4 MB L2 holds at most two heads' K/V (1.7 MB each at T=3401) instead of all of them.
// (sk_begin, udiv23: x3_common.h)

// any P: XCD x (= phys % 8) owns the contiguous logical run of its P/8 (+1 for the first P % 8
// XCDs) workgroups — a bijection, so a grid trimmed to query-group boundaries (252 on 256 CUs)
// keeps each XCD on about one head's K/V
__device__ __forceinline__ int sk_logical(int phys, int P) {
  const int x = phys % 8, q = P / 8, r = P % 8;
  return x * q + min(x, r) + phys / 8;
}

template <int WPE>
__global__ __launch_bounds__(64, WPE) void attn_fwd_sk(const float* __restrict__ qkv, float* __restrict__ out,
                                                     float* __restrict__ part_o, float* __restrict__ part_ml, int B,
                                                     int T, int H, float scale_log2e, int P) {
  const int w = sk_logical(blockIdx.x, P);
  const int NK = (T + 31) / 32, QT = NK;
  const long long U = (long long)B * H * QT * NK;
  long long u = sk_begin(w, U, P);
  const long long u1 = sk_begin(w + 1, U, P);
  const int D = H * HD;
  const int lane = threadIdx.x & 63;
  const int j = lane & 31, hf = lane >> 5;
  bool first = true;
  while (u < u1) {
    const long long tile = u / NK;
    const int kb0 = int(u - tile * NK);
    const int kb1 = int(min<long long>(NK, kb0 + (u1 - u)));
    const int qt = int(tile % QT);
    const int head = int((tile / QT) % H);
    const int b = int(tile / ((long long)QT * H));
    const AttnAcc a = attn_segment(qkv + size_t(b) * T * 3 * D, qt * 32, head, kb0, kb1, T, D, scale_log2e);
    if (kb0 == 0 && kb1 == NK) {
      attn_store_out(a, out, b, qt * 32, head, T, D);
    } else {
      // slot layout: part_o[slot][d][32 queries] (lane-contiguous stores), part_ml[slot][2][32]
      const size_t slot = size_t(w) * 2 + (first ? 0 : 1);
      float* po = part_o + slot * (HD * 32);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int d = key_of(r, hf);
        po[d * 32 + j] = a.o0[r];
        po[(32 + d) * 32 + j] = a.o1[r];
      }
      if (hf == 0) {
        part_ml[slot * 64 + j] = a.m;
        part_ml[slot * 64 + 32 + j] = a.l;
      }
    }
    u += kb1 - kb0;
    first = false;
  }
}

// Merge the partial segments of every tile that more than one wave touched. One 256-thread block
// per tile: thread = (query quad, d); contributors are the waves whose ranges intersect the tile.
__global__ __launch_bounds__(256) void attn_sk_fixup(const float* __restrict__ part_o,
                                                     const float* __restrict__ part_ml, float* __restrict__ out,
                                                     int B, int T, int H, int P) {
  const int NK = (T + 31) / 32, QT = NK;
  const long long U = (long long)B * H * QT * NK;
  const long long tile = blockIdx.x;
  const long long t0 = tile * NK, t1 = t0 + NK;  // unit range of this tile
  // wave containing unit u: largest w with w*U/P <= u
  const long long w_lo = ((t0 + 1) * P + U - 1) / U - 1;
  const long long w_hi = (t1 * P + U - 1) / U - 1;
  if (w_lo == w_hi) return;  // one wave did the whole tile and stored it normalised
  const int qt = int(tile % QT);
  const int head = int((tile / QT) % H);
  const int b = int(tile / ((long long)QT * H));
  const int D = H * HD;
  const int d = threadIdx.x & 63;
  for (int jq = threadIdx.x >> 6; jq < 32; jq += 4) {
    const int q = qt * 32 + jq;
    if (q >= T) break;
    float mmax = -INFINITY;
    for (long long w = w_lo; w <= w_hi; ++w) {
      const long long s = w * U / P;
      if (s == (w + 1) * U / P) continue;
      const size_t slot = size_t(w) * 2 + (s >= t0 ? 0 : 1);
      mmax = fmaxf(mmax, part_ml[slot * 64 + jq]);
    }
    float num = 0.f, den = 0.f;
    for (long long w = w_lo; w <= w_hi; ++w) {
      const long long s = w * U / P;
      if (s == (w + 1) * U / P) continue;
      const size_t slot = size_t(w) * 2 + (s >= t0 ? 0 : 1);
      const float sc = __builtin_amdgcn_exp2f(part_ml[slot * 64 + jq] - mmax);
      num += part_o[slot * (HD * 32) + d * 32 + jq] * sc;
      den += part_ml[slot * 64 + 32 + jq] * sc;
    }
    out[(size_t(b) * T + q) * D + head * HD + d] = num / den;
  }
}


// ---- stream-K attention, LDS-shared K/V (production path) --------------------------------------
// A 256-thread workgroup = 4 waves = 4 consecutive 32-query tiles (a 128-query "group") of one
// head. The workgroup streams 32-key blocks of K and V through LDS once for all four waves
// (coalesced dwordx4 global loads, register-prefetched one block ahead, double-buffered, one
// barrier per block), so L2->CU traffic and texture-address work drop 4x versus every wave
// fetching its own fragments (the v1 kernel above is TA-bound at ~640 cache-line lookups per wave
// per block). LDS images: K row-major with a 68-float stride — the per-lane ds_read_b128 of
// K[key=j][32*hf + 4*s4] then hits 16 distinct 16-B slots per lane group (17*j mod 16); V
// row-major (stride 64), read as ds_read_b32 V[key][j] with 32 consecutive banks per half-wave.
// Stream-K runs over (group x key block) units with a persistent grid of P workgroups, the same
// first/last-segment workspace scheme and XCD-major order as attn_fwd_sk.
constexpr int KSTR = 68, VSTR = 64;
constexpr int KBUF = 32 * KSTR, VBUF = 32 * VSTR;

__global__ __launch_bounds__(256, 2) void attn_fwd_sk_lds(const float* __restrict__ qkv, float* __restrict__ out,
                                                          float* __restrict__ part_o, float* __restrict__ part_ml,
                                                          int B, int T, int H, float scale_log2e, int P) {
  __shared__ __attribute__((aligned(16))) float lds_k[2 * KBUF];
  __shared__ __attribute__((aligned(16))) float lds_v[2 * VBUF];
  const int w = sk_logical(blockIdx.x, P);
  const int NK = (T + 31) / 32, QT = NK, QG = (QT + 3) / 4;
  const long long U = (long long)B * H * QG * NK;
  long long u = sk_begin(w, U, P);
  const long long u1 = sk_begin(w + 1, U, P);
  const int D = H * HD, ld = 3 * D;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int j = lane & 31, hf = lane >> 5;
  // cooperative-load mapping: float4 f = tid + 256*i, i = 0..1 -> key row f/16, dims 4*(f%16)
  const int lrow = tid >> 4, lc4 = tid & 15;
  bool first = true;
  while (u < u1) {
    const long long grp = u / NK;
    const int kb0 = int(u - grp * NK);
    const int kb1 = int(min<long long>(NK, kb0 + (u1 - u)));
    const int qg = int(grp % QG);
    const int head = int((grp / QG) % H);
    const int b = int(grp / ((long long)QG * H));
    const float* base = qkv + size_t(b) * T * ld;
    const int qt = qg * 4 + wv;
    const bool active = qt < QT;
    const int q0 = qt * 32;

    float qreg[32];
    {
      const int qrow = min(q0 + j, T - 1);
      const float4* qp = reinterpret_cast<const float4*>(base + size_t(qrow) * ld + head * HD + 32 * hf);
#pragma unroll
      for (int s4 = 0; s4 < 8; ++s4) {
        const float4 v = qp[s4];
        qreg[4 * s4 + 0] = v.x * scale_log2e;
        qreg[4 * s4 + 1] = v.y * scale_log2e;
        qreg[4 * s4 + 2] = v.z * scale_log2e;
        qreg[4 * s4 + 3] = v.w * scale_log2e;
      }
    }
    const float* kg = base + D + head * HD + 4 * lc4;
    const float* vg = base + 2 * D + head * HD + 4 * lc4;
    float4 pk0, pk1, pv0, pv1;
    auto fetch = [&](int blk) {
      const int r0 = min(blk * 32 + lrow, T - 1), r1 = min(blk * 32 + 16 + lrow, T - 1);
      pk0 = *reinterpret_cast<const float4*>(kg + size_t(r0) * ld);
      pk1 = *reinterpret_cast<const float4*>(kg + size_t(r1) * ld);
      pv0 = *reinterpret_cast<const float4*>(vg + size_t(r0) * ld);
      pv1 = *reinterpret_cast<const float4*>(vg + size_t(r1) * ld);
    };
    auto stash = [&](int buf) {
      *reinterpret_cast<float4*>(&lds_k[buf * KBUF + lrow * KSTR + 4 * lc4]) = pk0;
      *reinterpret_cast<float4*>(&lds_k[buf * KBUF + (16 + lrow) * KSTR + 4 * lc4]) = pk1;
      *reinterpret_cast<float4*>(&lds_v[buf * VBUF + lrow * VSTR + 4 * lc4]) = pv0;
      *reinterpret_cast<float4*>(&lds_v[buf * VBUF + (16 + lrow) * VSTR + 4 * lc4]) = pv1;
    };
    __syncthreads();  // the previous segment's last block is no longer being read
    fetch(kb0);
    stash(0);
    __syncthreads();

    f32x16 o0 = {0}, o1 = {0};
    float m = -INFINITY, l = 0.f;
    for (int blk = kb0; blk < kb1; ++blk) {
      const int buf = (blk - kb0) & 1;
      const bool more = blk + 1 < kb1;
      if (more) fetch(blk + 1);
      if (active) {
        const float* ks = &lds_k[buf * KBUF + j * KSTR + 32 * hf];
        float kreg[32];
#pragma unroll
        for (int s4 = 0; s4 < 8; ++s4) {
          const float4 v = *reinterpret_cast<const float4*>(ks + 4 * s4);
          kreg[4 * s4 + 0] = v.x;
          kreg[4 * s4 + 1] = v.y;
          kreg[4 * s4 + 2] = v.z;
          kreg[4 * s4 + 3] = v.w;
        }
        const float* vs = &lds_v[buf * VBUF + j];
        float v0[16], v1[16];
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          v0[t] = vs[key_of(t, hf) * VSTR];
          v1[t] = vs[key_of(t, hf) * VSTR + 32];
        }
        f32x16 sacc = {0};
#pragma unroll
        for (int st = 0; st < 32; ++st) sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(kreg[st], qreg[st], sacc, 0, 0, 0);
        const int kb = blk * 32;
        if (kb + 32 > T) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (kb + key_of(r, hf) >= T) sacc[r] = -INFINITY;
        }
        float mx = sacc[0];
#pragma unroll
        for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sacc[r]);
        mx = half_max(mx);
        const float m_new = fmaxf(m, mx);
        const float alpha = __builtin_amdgcn_exp2f(m - m_new);
        float psum = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          sacc[r] = __builtin_amdgcn_exp2f(sacc[r] - m_new);
          psum += sacc[r];
        }
        psum = half_sum(psum);
        l = l * alpha + psum;
        m = m_new;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          o0[r] *= alpha;
          o1[r] *= alpha;
        }
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          o0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v0[t], sacc[t], o0, 0, 0, 0);
          o1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v1[t], sacc[t], o1, 0, 0, 0);
        }
      }
      if (more) stash(buf ^ 1);
      __syncthreads();
    }

    if (active) {
      if (kb0 == 0 && kb1 == NK) {
        const int q = q0 + j;
        if (q < T) {
          const float inv = 1.f / l;
          float* orow = out + (size_t(b) * T + q) * D + head * HD;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int d = key_of(r, hf);
            orow[d] = o0[r] * inv;
            orow[32 + d] = o1[r] * inv;
          }
        }
      } else {
        // slot layout: part_o[wg][first?0:1][wave][d][32 queries], part_ml[wg][slot][wave][2][32]
        const size_t slot = (size_t(w) * 2 + (first ? 0 : 1)) * 4 + wv;
        float* po = part_o + slot * (HD * 32);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int d = key_of(r, hf);
          po[d * 32 + j] = o0[r];
          po[(32 + d) * 32 + j] = o1[r];
        }
        if (hf == 0) {
          part_ml[slot * 64 + j] = m;
          part_ml[slot * 64 + 32 + j] = l;
        }
      }
    }
    u += kb1 - kb0;
    first = false;
  }
}

// Merge for attn_fwd_sk_lds: one 256-thread block per 32-query tile. Partials are [d][32 q]
// images, so thread t reads elements e = t + 256*i (q = t % 32, d = e / 32): every contributor's
// 8 KB image is read with fully coalesced 1 KB wave loads, scaled by exp2(m_w[q] - m_max[q]) and
// accumulated in registers; the normalised tile is transposed through LDS so the [q][d] output rows
// are written as 256-B runs.
template <int G>
__global__ __launch_bounds__(256) void attn_sk_lds_fixup(const float* __restrict__ part_o,
                                                         const float* __restrict__ part_ml, float* __restrict__ out,
                                                         int B, int T, int H, int P, __bf16* __restrict__ outp,
                                                         int h0, int Ht, unsigned pin) {
  __shared__ float s_tile[64][33];
  const int NK = (T + 31) / 32, QT = NK, QG = (QT + G - 1) / G;
  const long long U = (long long)B * H * QG * NK;
  const bool narrow_stores = (pin >> 8) & 1u;  // A/B: the earlier 2-byte plane stores
  const bool xcd_local = (pin >> 9) & 1u;
  pin &= 0xffu;
  const PinnedBlock pb = pinned_block(pin);
  if (pb.id < 0) return;
  // XCD-local order (unpinned launches, bit 9): a block merges tiles whose contributors ran on the
  // block's own XCD (block b runs on XCD b % 8, as the attention's xcd_major_n order assumes), so
  // their partials are read from that XCD's L2 rather than across the fabric. XCD x's workgroups
  // are the logical range [ws(x), ws(x+1)), ws(x) = x*(P/8) + min(x, P%8); a row is XCD x's when its
  // first contributor is, i.e. rows [rlo(x), rlo(x+1)) with rlo(x) = ceil((ws(x)*U + 1 - P) / (NK*P)).
  // Only the order changes: every tile is still merged exactly once, with the same arithmetic.
  // Opt-in (flag bit 6): measured no faster than the plain order (profiles/attn_fixup_order_ab_r6.json)
  // — the partials are read from beyond the XCD's L2 either way after the kernel boundary.
  const int R = B * H * QG;
  int id0 = pb.id, idn = R * G, step = pb.n, base = 0;
  if (xcd_local && !pin) {
    const int x = int(blockIdx.x) % 8, qq = P / 8, rr = P % 8;
    auto rlo = [&](int xx) -> int {
      if (xx >= 8) return R;
      const long long ws = (long long)xx * qq + min(xx, rr);
      const long long num = ws * U + 1 - P, den = (long long)NK * P;
      const long long r0 = num <= 0 ? 0 : (num + den - 1) / den;
      return int(min<long long>(r0, R));
    };
    const int r0 = rlo(x), r1 = rlo(x + 1);
    base = r0 * G;
    idn = max(0, r1 - r0) * G;
    id0 = int(blockIdx.x) / 8;
    step = int(gridDim.x) / 8;
  }
  // grid-stride over the (group, query tile) units: a pinned launch runs a few workgroups per CU
  for (int id_ = id0; id_ < idn; id_ += step) {
  const int id = base + id_;
  const int wv = id % G;
  const long long grp = id / G;
  const int qg = int(grp % QG);
  const int qt = qg * G + wv;
  if (qt >= QT) continue;
  const long long t0 = grp * NK, t1 = t0 + NK;
  const long long w_lo = ((t0 + 1) * P + U - 1) / U - 1;
  const long long w_hi = (t1 * P + U - 1) / U - 1;
  if (w_lo == w_hi) continue;
  const int head = h0 + int((grp / QG) % H);
  const int b = int(grp / ((long long)QG * H));
  const int D = Ht * HD;
  const int tid = threadIdx.x;
  auto slot_of = [&](long long w) -> long long {
    const long long s = w * U / P;
    if (s == (w + 1) * U / P) return -1;  // empty range
    return (w * 2 + (s >= t0 ? 0 : 1)) * G + wv;
  };
  // one online-softmax merge pass over the contributors, their loads issued up to four at a time
  // (every thread merges its own query's m/l redundantly: no serial phase, no extra barrier)
  const int q = tid & 31;
  float M = -INFINITY, L = 0.f;
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  for (long long w0 = w_lo; w0 <= w_hi; w0 += 4) {
    float mw[4], lw[4], ow[4][8];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const long long w = w0 + c;
      const long long sl = w <= w_hi ? slot_of(w) : -1;
      mw[c] = -INFINITY;
      lw[c] = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) ow[c][i] = 0.f;
      if (sl >= 0) {
        mw[c] = part_ml[sl * 64 + q];
        lw[c] = part_ml[sl * 64 + 32 + q];
        const float* po = part_o + sl * (HD * 32);
#pragma unroll
        for (int i = 0; i < 8; ++i) ow[c][i] = po[tid + 256 * i];
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (mw[c] == -INFINITY) continue;
      const float Mn = fmaxf(M, mw[c]);
      const float so = __builtin_amdgcn_exp2f(M - Mn), sn = __builtin_amdgcn_exp2f(mw[c] - Mn);
      // explicit fmas (no contraction left to the compiler): attn_fwd_x3w's in-kernel merge does
      // the same operations and matches this kernel bit for bit
      L = fmaf(lw[c], sn, L * so);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = fmaf(ow[c][i], sn, acc[i] * so);
      M = Mn;
    }
  }
  const float inv = 1.f / L;
#pragma unroll
  for (int i = 0; i < 8; ++i) s_tile[(tid + 256 * i) >> 5][q] = acc[i] * inv;
  __syncthreads();
  const size_t plane = size_t(B) * T * D;
  if (!narrow_stores) {
    // transposed store: thread -> (query row, 8 consecutive dims), one pass: each plane row of the
    // tile leaves as 16-B stores (the fp32 output as two)
    const int jq = tid >> 3, c8 = 8 * (tid & 7);
    const int qq = qt * 32 + jq;
    if (qq < T) {
      const size_t i = (size_t(b) * T + qq) * D + head * HD + c8;
      f32x8 v;
#pragma unroll
      for (int dd = 0; dd < 8; ++dd) v[dd] = s_tile[c8 + dd][jq];
      if (outp) {
        bf16x8 p0, p1, p2;
        split3(v, p0, p1, p2);
        *reinterpret_cast<bf16x8*>(outp + i) = p0;
        *reinterpret_cast<bf16x8*>(outp + plane + i) = p1;
        *reinterpret_cast<bf16x8*>(outp + 2 * plane + i) = p2;
      } else {
        *reinterpret_cast<f32x4*>(out + i) = f32x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4*>(out + i + 4) = f32x4{v[4], v[5], v[6], v[7]};
      }
    }
  } else {
  // transposed store: thread -> (query row, 64 dims), 4 rows per pass
  const int d = tid & 63;
  for (int jq = tid >> 6; jq < 32; jq += 4) {
    const int qq = qt * 32 + jq;
    if (qq >= T) break;
    const size_t i = (size_t(b) * T + qq) * D + head * HD + d;
    if (outp)
      store_x3(outp, plane, i, s_tile[d][jq]);
    else
      out[i] = s_tile[d][jq];
  }
  }
  __syncthreads();  // s_tile is rewritten by the next unit
  }
}

// ---- fp32 as three bf16 planes ("x3") ----------------------------------------------------------
// gfx950 has no xf32 and runs f32-input MFMA at 1/16 of the bf16 rate. An fp32 value splits
// exactly into three bf16 terms, x = x0 + x1 + x2 (each residual of a round-to-nearest bf16
// conversion is exact in f32 and carries the next 8 mantissa bits), so a product a·b of two fp32
// operands is a0b0 + a0b1 + a1b0 + a0b2 + a1b1 + a2b0 up to terms of relative size 2^-24 — the
// fp32 rounding level. Six bf16 MFMAs (32x32x16, 32 cycles each) replace eight f32 MFMAs
// (32x32x2, 64 cycles each) per 32x32x16 block: 2.67x fewer matrix-pipe cycles at fp32 accuracy.
// The small products are accumulated first so the running sum absorbs them at fp32 rounding.

// Exact three-term split of acc[e0 .. e0+7] by truncation: x0 = the high 16 bits of x (its f32
// value is x & 0xffff0000, so no conversion back is needed), x1 = the high half of x - x0, x2 =
// the rest (<= 8 significant bits, exact in bf16); pairs are packed with one v_perm_b32 each.
__device__ __forceinline__ void split3_trunc8(const f32x16& acc, int e0, bf16x8& p0, bf16x8& p1, bf16x8& p2) {
  uint32_t w0[4], w1[4], w2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = acc[e0 + 2 * i], b = acc[e0 + 2 * i + 1];
    const uint32_t ua = __float_as_uint(a), ub = __float_as_uint(b);
    w0[i] = __builtin_amdgcn_perm(ub, ua, 0x07060302u);
    const float ra = a - __uint_as_float(ua & 0xffff0000u), rb = b - __uint_as_float(ub & 0xffff0000u);
    const uint32_t ura = __float_as_uint(ra), urb = __float_as_uint(rb);
    w1[i] = __builtin_amdgcn_perm(urb, ura, 0x07060302u);
    const float sa = ra - __uint_as_float(ura & 0xffff0000u), sb = rb - __uint_as_float(urb & 0xffff0000u);
    w2[i] = __builtin_amdgcn_perm(__float_as_uint(sb), __float_as_uint(sa), 0x07060302u);
  }
  p0 = __builtin_bit_cast(bf16x8, (uint4){w0[0], w0[1], w0[2], w0[3]});
  p1 = __builtin_bit_cast(bf16x8, (uint4){w1[0], w1[1], w1[2], w1[3]});
  p2 = __builtin_bit_cast(bf16x8, (uint4){w2[0], w2[1], w2[2], w2[3]});
}

// (mfma_x3: x3_common.h)

// fp32 [n] -> bf16 planes [3][n] (plane stride n); 4 elements per thread
__global__ __launch_bounds__(256) void split3_f32(const float* __restrict__ x, __bf16* __restrict__ y, size_t n4,
                                                  unsigned pin) {
  const PinnedBlock pb = pinned_block(pin);
  if (pb.id < 0) return;
  const size_t stride = size_t(pb.n) * 256;
  for (size_t i = size_t(pb.id) * 256 + threadIdx.x; i < n4; i += stride) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    bf16x4 p0, p1, p2;
    split3(v, p0, p1, p2);
    reinterpret_cast<bf16x4*>(y)[i] = p0;
    reinterpret_cast<bf16x4*>(y)[n4 + i] = p1;
    reinterpret_cast<bf16x4*>(y)[2 * n4 + i] = p2;
  }
}

// Stream-K flash attention on x3 planes of the packed QKV tensor: the same (128-query group x
// 32-key block) units, persistent grid, XCD-major order and partial-segment workspace as
// attn_fwd_sk_lds (so attn_sk_lds_fixup merges its partials), with every product on
// v_mfma_f32_32x32x16_bf16:
//  * S^T = K·Q^T: lane (j, h) holds Q[q0+j][16s+8h .. +7] per plane (12 x 16-B loads per segment,
//    kept in registers); K fragments are ds_read_b128 row reads of a [plane][key][72] bf16 image
//    (144-B rows: 9r mod 16 is a bijection on every ds_read_b128 lane group — conflict-free);
//  * softmax on the S^T accumulator (one query per lane, keys in registers) as in the f32 kernel,
//    the log2e/sqrt(d) scale applied inside the exp2's fma;
//  * P^T is split into planes in registers and used as the B operand of O^T += V^T·P^T straight
//    from the accumulator (registers 8s..8s+7 = k-step s, key 16s + 8(e>>2) + 4h + (e&3) in
//    element e); the matching V^T fragments come from a row-major [plane][key][96] V image through
//    ds_read_b64_tr_b16 (two 4-key transposed reads per fragment; 192-B rows put the four rows of a
//    read group at bank offsets 0/48/32/16 — conflict-free);
//  * K and V blocks arrive as coalesced 16-B loads of pre-split planes (the producer splits once;
//    every query group re-reads them), register-prefetched one block ahead, double-buffered.
// (XK_STR, XV_STR, XK_PLANE, XV_PLANE: x3_common.h)

__global__ __launch_bounds__(256, 2) void attn_fwd_x3(const __bf16* __restrict__ qkv3, size_t plane,
                                                      float* __restrict__ out, __bf16* __restrict__ outp,
                                                      float* __restrict__ part_o, float* __restrict__ part_ml, int B,
                                                      int T, int H, float scale_log2e, int P) {
  __shared__ __attribute__((aligned(16))) __bf16 lds_k[2 * 3 * XK_PLANE];
  __shared__ __attribute__((aligned(16))) __bf16 lds_v[2 * 3 * XV_PLANE];
  const int w = sk_logical(blockIdx.x, P);
  const int NK = (T + 31) / 32, QT = NK, QG = (QT + 3) / 4;
  const long long U = (long long)B * H * QG * NK;
  long long u = sk_begin(w, U, P);
  const long long u1 = sk_begin(w + 1, U, P);
  const int D = H * HD, ld = 3 * D;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int j = lane & 31, hf = lane >> 5;
  // loader: 16-B chunk (8 bf16) per plane: key row tid/8, dims 8*(tid%8)
  const int lrow = tid >> 3, lch = tid & 7;
  // transposed-read lane address inside a plane image: group g = lane/16 (h = g/2, column block
  // 16*(g&1)), lane i = lane%16 supplies row 4h + i/4, columns 4*(i%4)
  const int gi = lane & 15, gg = lane >> 4;
  const int vtr = (4 * hf + (gi >> 2)) * XV_STR + 16 * (gg & 1) + 4 * (gi & 3);
  bool first = true;
  while (u < u1) {
    const long long grp = u / NK;
    const int kb0 = int(u - grp * NK);
    const int kb1 = int(min<long long>(NK, kb0 + (u1 - u)));
    const int qg = int(grp % QG);
    const int head = int((grp / QG) % H);
    const int b = int(grp / ((long long)QG * H));
    const __bf16* base = qkv3 + size_t(b) * T * ld;
    const int qt = qg * 4 + wv;
    const bool active = qt < QT;
    const int q0 = qt * 32;

    bf16x8 qf[3][4];
    {
      const int qrow = min(q0 + j, T - 1);
      const __bf16* qp = base + size_t(qrow) * ld + head * HD + 8 * hf;
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int s = 0; s < 4; ++s) qf[p][s] = *reinterpret_cast<const bf16x8*>(qp + p * plane + 16 * s);
    }
    const __bf16* kg = base + D + head * HD + 8 * lch;
    const __bf16* vg = base + 2 * D + head * HD + 8 * lch;
    // one block = 32 key rows x 128 B per plane of K and of V: one 16-B chunk per thread each
    uint4 pk0, pk1, pk2, pv0, pv1, pv2;
    auto fetch = [&](int blk) {
      const size_t r = size_t(min(blk * 32 + lrow, T - 1)) * ld;
      pk0 = *reinterpret_cast<const uint4*>(kg + r);
      pk1 = *reinterpret_cast<const uint4*>(kg + plane + r);
      pk2 = *reinterpret_cast<const uint4*>(kg + 2 * plane + r);
      pv0 = *reinterpret_cast<const uint4*>(vg + r);
      pv1 = *reinterpret_cast<const uint4*>(vg + plane + r);
      pv2 = *reinterpret_cast<const uint4*>(vg + 2 * plane + r);
    };
    auto stash = [&](int buf) {
      __bf16* kd = &lds_k[buf * 3 * XK_PLANE + lrow * XK_STR + 8 * lch];
      __bf16* vd = &lds_v[buf * 3 * XV_PLANE + lrow * XV_STR + 8 * lch];
      *reinterpret_cast<uint4*>(kd) = pk0;
      *reinterpret_cast<uint4*>(kd + XK_PLANE) = pk1;
      *reinterpret_cast<uint4*>(kd + 2 * XK_PLANE) = pk2;
      *reinterpret_cast<uint4*>(vd) = pv0;
      *reinterpret_cast<uint4*>(vd + XV_PLANE) = pv1;
      *reinterpret_cast<uint4*>(vd + 2 * XV_PLANE) = pv2;
    };
    __syncthreads();  // the previous segment's last block is no longer being read
    fetch(kb0);
    stash(0);
    __syncthreads();

    f32x16 o0 = {0}, o1 = {0};
    float m = -INFINITY, l = 0.f;
    for (int blk = kb0; blk < kb1; ++blk) {
      const int buf = (blk - kb0) & 1;
      const bool more = blk + 1 < kb1;
      if (more) fetch(blk + 1);
// One 32-key block of the x3 flash-attention loop. The key mask of the tail block sits behind a
// real (wave-uniform) branch, so full blocks carry no per-key compares. Lazy rescale: the running max m only moves
// when some lane's block max exceeds it by more than 2^8 in exp2 units (wave-uniform decision), so
// the O/l rescale and its exp2 run on a few blocks per segment instead of every block; between
// moves P may reach 2^8, which fp32 P/l/O absorb without loss.
#define X3_ATTN_BLOCK(MASKED)                                                                        \
  {                                                                                                  \
    const __bf16* ks = &lds_k[buf * 3 * XK_PLANE + j * XK_STR + 8 * hf];                             \
    f32x16 sacc = {0};                                                                               \
    _Pragma("unroll") for (int s = 0; s < 4; ++s) {                                                  \
      const bf16x8 k0 = *reinterpret_cast<const bf16x8*>(ks + 16 * s);                               \
      const bf16x8 k1 = *reinterpret_cast<const bf16x8*>(ks + XK_PLANE + 16 * s);                     \
      const bf16x8 k2 = *reinterpret_cast<const bf16x8*>(ks + 2 * XK_PLANE + 16 * s);                 \
      sacc = mfma_x3(k0, k1, k2, qf[0][s], qf[1][s], qf[2][s], sacc);                                \
    }                                                                                                \
    if (MASKED) {                                                                                    \
      asm volatile("; tail block: mask keys >= T" ::: "memory"); /* keep a real branch */          \
      _Pragma("unroll") for (int r = 0; r < 16; ++r) if (blk * 32 + key_of(r, hf) >= T) sacc[r] = -INFINITY; \
    }                                                                                                \
    float mx = fmaxf(sacc[0], sacc[1]);                                                              \
    _Pragma("unroll") for (int r = 2; r < 16; ++r) mx = fmaxf(mx, sacc[r]);                          \
    mx = half_max(mx);                                                          \
    if (__builtin_amdgcn_ballot_w64((mx - m) * scale_log2e > 8.f)) {                                 \
      const float m_new = fmaxf(m, mx);                                                              \
      const float alpha = __builtin_amdgcn_exp2f((m - m_new) * scale_log2e);                         \
      l *= alpha;                                                                                    \
      o0 *= alpha;                                                                                   \
      o1 *= alpha;                                                                                   \
      m = m_new;                                                                                     \
    }                                                                                                \
    const float mc = m * scale_log2e;                                                                \
    float psum = 0.f;                                                                                \
    _Pragma("unroll") for (int r = 0; r < 16; ++r) {                                                 \
      sacc[r] = __builtin_amdgcn_exp2f(fmaf(sacc[r], scale_log2e, -mc));                             \
      psum += sacc[r];                                                                               \
    }                                                                                                \
    psum = half_sum(psum);                                                                \
    l += psum;                                                                                       \
    const __bf16* vs = &lds_v[buf * 3 * XV_PLANE + vtr];                                             \
    _Pragma("unroll") for (int s2 = 0; s2 < 2; ++s2) {                                               \
      bf16x8 p0, p1, p2;                                                                             \
      split3_trunc8(sacc, 8 * s2, p0, p1, p2);                                                       \
      _Pragma("unroll") for (int dh = 0; dh < 2; ++dh) {                                             \
        bf16x8 vf[3];                                                                                \
        _Pragma("unroll") for (int p = 0; p < 3; ++p) {                                              \
          const __bf16* a = vs + p * XV_PLANE + 16 * s2 * XV_STR + 32 * dh;                          \
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a));              \
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a + 8 * XV_STR)); \
          vf[p] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};                    \
        }                                                                                            \
        if (dh == 0)                                                                                 \
          o0 = mfma_x3(vf[0], vf[1], vf[2], p0, p1, p2, o0);                                         \
        else                                                                                         \
          o1 = mfma_x3(vf[0], vf[1], vf[2], p0, p1, p2, o1);                                         \
      }                                                                                              \
    }                                                                                                \
  }
      if (active) X3_ATTN_BLOCK(blk * 32 + 32 > T)
#undef X3_ATTN_BLOCK
      if (more) stash(buf ^ 1);
      __syncthreads();
    }

    if (active) {
      if (kb0 == 0 && kb1 == NK) {
        const int q = q0 + j;
        if (q < T) {
          const float inv = 1.f / l;
          const size_t orow = (size_t(b) * T + q) * D + head * HD;
          if (outp) {
            const size_t op = size_t(B) * T * D;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int d = key_of(r, hf);
              store_x3(outp, op, orow + d, o0[r] * inv);
              store_x3(outp, op, orow + 32 + d, o1[r] * inv);
            }
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int d = key_of(r, hf);
              out[orow + d] = o0[r] * inv;
              out[orow + 32 + d] = o1[r] * inv;
            }
          }
        }
      } else {
        const size_t slot = (size_t(w) * 2 + (first ? 0 : 1)) * 4 + wv;
        float* po = part_o + slot * (HD * 32);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int d = key_of(r, hf);
          po[d * 32 + j] = o0[r];
          po[(32 + d) * 32 + j] = o1[r];
        }
        if (hf == 0) {
          part_ml[slot * 64 + j] = m * scale_log2e;
          part_ml[slot * 64 + 32 + j] = l;
        }
      }
    }
    u += kb1 - kb0;
    first = false;
  }
}

// Software-pipelined x3 attention: iteration i runs the softmax, P split and P·V of key block i
// while the S^T = K·Q^T MFMAs of block i+1 are already in flight in the same wave's instruction
// stream, so the ~190 vector instructions per block issue in the matrix pipe's shadow instead of
// between its bursts. K and V have their own double-buffered rings (iteration i reads K of block
// i+1 and V of block i), one barrier per iteration. Same units, partials and fixup as attn_fwd_x3.
// G = query tiles (waves) per workgroup sharing each K/V block: 4 (two workgroups per CU) or 8 (one
// 512-thread workgroup per CU: half the K/V bytes per query, the L2/Infinity-Cache traffic that
// concurrent partitions share; the K and V loads are split between the two halves of the group).
template <int G, bool QW = false, bool F32IN = false, bool PRIO = false, bool FDIV = false>
__global__ __launch_bounds__(64 * G, 8 / G) void attn_fwd_x3p(const __bf16* __restrict__ qkv3, size_t plane,
                                                             float* __restrict__ out, __bf16* __restrict__ outp,
                                                             float* __restrict__ part_o, float* __restrict__ part_ml,
                                                             int B, int T, int H, int h0, int Ht, float scale_log2e,
                                                             int Pk) {
  static_assert(G == 4 || G == 8, "4 or 8 query tiles per workgroup");
  __shared__ __attribute__((aligned(16))) __bf16 lds_k[2 * 3 * XK_PLANE];
  __shared__ __attribute__((aligned(16))) __bf16 lds_v[2 * 3 * XV_PLANE];
  // grid word: bits 0-21 = P (logical workgroups), 22-29 = partition pin (pin.h), bit 30 = logical
  // workgroup order = dispatch order (no XCD-major remap; A/B switch)
  const int P = Pk & 0x3fffff;
  const PinnedBlock pb = pinned_block(unsigned(Pk >> 22) & 0xffu);
  if (pb.id < 0 || pb.id >= P) return;
  const int w = (Pk >> 30) ? pb.id : xcd_major_n(pb.id, P, pb.nx);
  const int NK = (T + 31) / 32, QT = NK, QG = (QT + G - 1) / G;
  const long long U = (long long)B * H * QG * NK;
  // FDIV (host-checked: every numerator < 2^23): reciprocal divisions for the bookkeeping
  const float rP = FDIV ? 1.f / float(P) : 0.f, rNK = FDIV ? 1.f / float(NK) : 0.f;
  const float rQG = FDIV ? 1.f / float(QG) : 0.f, rH = FDIV ? 1.f / float(H) : 0.f;
  long long u = FDIV ? udiv23(w * U, P, rP) : sk_begin(w, U, P);
  const long long u1 = FDIV ? udiv23((w + 1) * U, P, rP) : sk_begin(w + 1, U, P);
  const int D = Ht * HD, ld = 3 * D;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const int j = lane & 31, hf = lane >> 5;
  const int lrow = (tid & 255) >> 3, lch = tid & 7;
  const bool kload = G == 4 || tid < 256;  // G = 8: waves 0-3 stage K, waves 4-7 stage V
  const bool vload = G == 4 || tid >= 256;
  const int gi = lane & 15, gg = lane >> 4;
  const int vtr = (4 * hf + (gi >> 2)) * XV_STR + 16 * (gg & 1) + 4 * (gi & 3);
  bool first = true;
  while (u < u1) {
    const long long grp = FDIV ? udiv23(u, NK, rNK) : u / NK;
    const int kb0 = int(u - grp * NK);
    const int kb1 = int(min<long long>(NK, kb0 + (u1 - u)));
    const int nb = kb1 - kb0;
    const long long gq = FDIV ? udiv23(grp, QG, rQG) : grp / QG;  // (b, head) of the group
    const int qg = int(grp - gq * QG);
    const long long bq = FDIV ? udiv23(gq, H, rH) : gq / H;
    const int head = h0 + int(gq - bq * H);
    const int b = int(bq);
    const __bf16* base = qkv3 + size_t(b) * T * ld;
    // F32IN: qkv arrives as fp32 [B][T][3D] (4 B per element instead of three 2-B planes) and is
    // split here — Q once per segment, each K/V chunk as it is stashed (the same RNE split the
    // producers use, so the planes are bit-identical to a planes-in run)
    const float* basef = reinterpret_cast<const float*>(qkv3) + size_t(b) * T * ld;
    const int qt = qg * G + wv;
    const bool active = qt < QT;
    const int q0 = qt * 32;

    bf16x8 qf[3][4];
    {
      const int qrow = min(q0 + j, T - 1);
      if constexpr (F32IN) {
        const float* qp = basef + size_t(qrow) * ld + head * HD + 8 * hf;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const f32x4 lo = *reinterpret_cast<const f32x4*>(qp + 16 * s);
          const f32x4 hi = *reinterpret_cast<const f32x4*>(qp + 16 * s + 4);
          const f32x8 x = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          split3(x, qf[0][s], qf[1][s], qf[2][s]);
        }
      } else {
        const __bf16* qp = base + size_t(qrow) * ld + head * HD + 8 * hf;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int s = 0; s < 4; ++s) qf[p][s] = *reinterpret_cast<const bf16x8*>(qp + p * plane + 16 * s);
      }
    }
    const __bf16* kg = base + D + head * HD + 8 * lch;
    const __bf16* vg = base + 2 * D + head * HD + 8 * lch;
    const float* kgf = basef + D + head * HD + 8 * lch;
    const float* vgf = basef + 2 * D + head * HD + 8 * lch;
    uint4 pk0, pk1, pk2, pv0, pv1, pv2;
    f32x4 fk0, fk1, fv0, fv1;  // F32IN staging: the chunk's 8 fp32 values
    auto fetch_k = [&](int blk) {
      const size_t r = size_t(min(blk * 32 + lrow, T - 1)) * ld;
      if constexpr (F32IN) {
        fk0 = *reinterpret_cast<const f32x4*>(kgf + r);
        fk1 = *reinterpret_cast<const f32x4*>(kgf + r + 4);
      } else {
        pk0 = *reinterpret_cast<const uint4*>(kg + r);
        pk1 = *reinterpret_cast<const uint4*>(kg + plane + r);
        pk2 = *reinterpret_cast<const uint4*>(kg + 2 * plane + r);
      }
    };
    auto fetch_v = [&](int blk) {
      const size_t r = size_t(min(blk * 32 + lrow, T - 1)) * ld;
      if constexpr (F32IN) {
        fv0 = *reinterpret_cast<const f32x4*>(vgf + r);
        fv1 = *reinterpret_cast<const f32x4*>(vgf + r + 4);
      } else {
        pv0 = *reinterpret_cast<const uint4*>(vg + r);
        pv1 = *reinterpret_cast<const uint4*>(vg + plane + r);
        pv2 = *reinterpret_cast<const uint4*>(vg + 2 * plane + r);
      }
    };
    auto split_chunk = [](const f32x4& lo, const f32x4& hi, uint4& c0, uint4& c1, uint4& c2) {
      const f32x8 x = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      bf16x8 a0, a1, a2;
      split3(x, a0, a1, a2);
      c0 = __builtin_bit_cast(uint4, a0), c1 = __builtin_bit_cast(uint4, a1), c2 = __builtin_bit_cast(uint4, a2);
    };
    auto stash_k = [&](int buf) {
      if constexpr (F32IN) split_chunk(fk0, fk1, pk0, pk1, pk2);
      __bf16* kd = &lds_k[buf * 3 * XK_PLANE + lrow * XK_STR + 8 * lch];
      *reinterpret_cast<uint4*>(kd) = pk0;
      *reinterpret_cast<uint4*>(kd + XK_PLANE) = pk1;
      *reinterpret_cast<uint4*>(kd + 2 * XK_PLANE) = pk2;
    };
    auto stash_v = [&](int buf) {
      if constexpr (F32IN) split_chunk(fv0, fv1, pv0, pv1, pv2);
      __bf16* vd = &lds_v[buf * 3 * XV_PLANE + lrow * XV_STR + 8 * lch];
      *reinterpret_cast<uint4*>(vd) = pv0;
      *reinterpret_cast<uint4*>(vd + XV_PLANE) = pv1;
      *reinterpret_cast<uint4*>(vd + 2 * XV_PLANE) = pv2;
    };
#define X3P_QK(SACC, BUF)                                                                        \
  {                                                                                              \
    const __bf16* ks_ = &lds_k[(BUF) * 3 * XK_PLANE + j * XK_STR + 8 * hf];                      \
    SACC = f32x16{0};                                                                            \
    _Pragma("unroll") for (int s = 0; s < 4; ++s) {                                              \
      const bf16x8 k0 = *reinterpret_cast<const bf16x8*>(ks_ + 16 * s);                           \
      const bf16x8 k1 = *reinterpret_cast<const bf16x8*>(ks_ + XK_PLANE + 16 * s);                 \
      const bf16x8 k2 = *reinterpret_cast<const bf16x8*>(ks_ + 2 * XK_PLANE + 16 * s);             \
      SACC = mfma_x3(k0, k1, k2, qf[0][s], qf[1][s], qf[2][s], SACC);                            \
    }                                                                                            \
  }
    __syncthreads();  // the previous segment's last blocks are no longer being read
    if (kload) {
      fetch_k(kb0);
      stash_k(0);
      if (nb > 1) {
        fetch_k(kb0 + 1);
        stash_k(1);
      }
    }
    if (vload) {
      fetch_v(kb0);
      stash_v(0);
    }
    __syncthreads();

    // the Q fragments (and the first K/V blocks) have landed: say so explicitly, or the waitcnt
    // pass, merging the loop's back edge with this entry, keeps a vmcnt wait on the Q loads in
    // front of every block's score MFMAs — which in steady state waits for the K/V prefetch
    // issued at the top of that same iteration (its global-load latency on the critical path)
    if constexpr (QW) __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0)
    f32x16 o0 = {0}, o1 = {0}, scur = {0};
    float m = -INFINITY, l = 0.f;
    if (active) X3P_QK(scur, 0)
    __syncthreads();  // iteration 0 refills K buffer 0, which the line above reads
// One key block: softmax + P.V of block i from SC while block i+1's scores go to SN; the loop
// alternates the two registers sets (no copy of the 16 scores per block).
// P.V of one key block from the P planes pa*/pb* (keys 0-15 / 16-31) and V buffer VB
#define X3P_PV(VB)                                                                                        \
  {                                                                                                       \
    const __bf16* vs_ = &lds_v[(VB) * 3 * XV_PLANE + vtr];                                                \
    _Pragma("unroll") for (int s2 = 0; s2 < 2; ++s2) {                                                    \
      _Pragma("unroll") for (int dh = 0; dh < 2; ++dh) {                                                  \
        bf16x8 vf[3];                                                                                     \
        _Pragma("unroll") for (int p = 0; p < 3; ++p) {                                                   \
          const __bf16* a = vs_ + p * XV_PLANE + 16 * s2 * XV_STR + 32 * dh;                              \
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a));                   \
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a + 8 * XV_STR));      \
          vf[p] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};                         \
        }                                                                                                 \
        const bf16x8 q0_ = s2 ? pb0 : pa0;                                                                \
        const bf16x8 q1_ = s2 ? pb1 : pa1;                                                                \
        const bf16x8 q2_ = s2 ? pb2 : pa2;                                                                \
        if (dh == 0)                                                                                      \
          o0 = mfma_x3(vf[0], vf[1], vf[2], q0_, q1_, q2_, o0);                                           \
        else                                                                                              \
          o1 = mfma_x3(vf[0], vf[1], vf[2], q0_, q1_, q2_, o1);                                           \
      }                                                                                                   \
    }                                                                                                     \
  }
#define X3P_ITER(SC, SN)                                                                                  \
  {                                                                                                       \
      const int blk = kb0 + i;                                                                            \
      const bool more_k = i + 2 < nb, more_v = i + 1 < nb;                                                \
      if (kload && more_k) fetch_k(blk + 2);                                                                      \
      if (vload && more_v) fetch_v(blk + 1);                                                                      \
      if (active) {                                                                                       \
        if (blk * 32 + 32 > T) {                                                                          \
          asm volatile("; tail block: mask keys >= T" ::: "memory");                                      \
          _Pragma("unroll") for (int r = 0; r < 16; ++r)                                                  \
            if (blk * 32 + key_of(r, hf) >= T) SC[r] = -INFINITY;                                         \
        }                                                                                                 \
        float mx = fmaxf(SC[0], SC[1]);                                                                   \
        _Pragma("unroll") for (int r = 2; r < 16; ++r) mx = fmaxf(mx, SC[r]);                             \
        mx = half_max(mx);                                                                                \
        if (__builtin_amdgcn_ballot_w64((mx - m) * scale_log2e > 8.f)) {                                  \
          const float m_new = fmaxf(m, mx);                                                               \
          const float alpha = __builtin_amdgcn_exp2f((m - m_new) * scale_log2e);                          \
          l *= alpha;                                                                                     \
          o0 *= alpha;                                                                                    \
          o1 *= alpha;                                                                                    \
          m = m_new;                                                                                      \
        }                                                                                                 \
                /* block i+1's scores (the last block: a throwaway product keeps one basic block) */ X3P_QK(SN, (i + 1) & 1)                                                                   \
        const float mc = m * scale_log2e;                                                                 \
        float psum = 0.f;                                                                                 \
        _Pragma("unroll") for (int r = 0; r < 16; ++r) {                                                  \
          SC[r] = __builtin_amdgcn_exp2f(fmaf(SC[r], scale_log2e, -mc));                                  \
          psum += SC[r];                                                                                  \
        }                                                                                                 \
        psum = half_sum(psum);                                                                            \
        l += psum;                                                                                        \
        const __bf16* vs = &lds_v[(i & 1) * 3 * XV_PLANE + vtr];                                          \
        _Pragma("unroll") for (int s2 = 0; s2 < 2; ++s2) {                                                \
          bf16x8 p0, p1, p2;                                                                              \
          split3_trunc8(SC, 8 * s2, p0, p1, p2);                                                          \
          _Pragma("unroll") for (int dh = 0; dh < 2; ++dh) {                                              \
            bf16x8 vf[3];                                                                                 \
            _Pragma("unroll") for (int p = 0; p < 3; ++p) {                                               \
              const __bf16* a = vs + p * XV_PLANE + 16 * s2 * XV_STR + 32 * dh;                           \
              const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a));               \
              const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a + 8 * XV_STR));  \
              vf[p] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};                     \
            }                                                                                             \
            if (dh == 0)                                                                                  \
              o0 = mfma_x3(vf[0], vf[1], vf[2], p0, p1, p2, o0);                                          \
            else                                                                                          \
              o1 = mfma_x3(vf[0], vf[1], vf[2], p0, p1, p2, o1);                                          \
          }                                                                                               \
        }                                                                                                 \
      }                                                                                                   \
      if (kload && more_k) stash_k(i & 1);                                                                 \
      if (vload && more_v) stash_v((i + 1) & 1);                                                           \
      __syncthreads();                                                                                    \
  }
#define X3P_ITER_LATE(SC, SN)                                                                                  \
  {                                                                                                       \
      const int blk = kb0 + i;                                                                            \
      const bool more_k = i + 2 < nb, more_v = i + 1 < nb;                                                \
      if (kload && more_k) fetch_k(blk + 2);                                                                      \
      if (vload && more_v) fetch_v(blk + 1);                                                                      \
      if (active) {                                                                                       \
        if (i > 0) X3P_PV((i - 1) & 1) /* the previous block's P.V, half a block behind waves 0-3 */   \
        if (blk * 32 + 32 > T) {                                                                          \
          asm volatile("; tail block: mask keys >= T" ::: "memory");                                      \
          _Pragma("unroll") for (int r = 0; r < 16; ++r)                                                  \
            if (blk * 32 + key_of(r, hf) >= T) SC[r] = -INFINITY;                                         \
        }                                                                                                 \
        float mx = fmaxf(SC[0], SC[1]);                                                                   \
        _Pragma("unroll") for (int r = 2; r < 16; ++r) mx = fmaxf(mx, SC[r]);                             \
        mx = half_max(mx);                                                                                \
        if (__builtin_amdgcn_ballot_w64((mx - m) * scale_log2e > 8.f)) {                                  \
          const float m_new = fmaxf(m, mx);                                                               \
          const float alpha = __builtin_amdgcn_exp2f((m - m_new) * scale_log2e);                          \
          l *= alpha;                                                                                     \
          o0 *= alpha;                                                                                    \
          o1 *= alpha;                                                                                    \
          m = m_new;                                                                                      \
        }                                                                                                 \
                /* block i+1's scores (the last block: a throwaway product keeps one basic block) */ X3P_QK(SN, (i + 1) & 1)                                                                   \
        const float mc = m * scale_log2e;                                                                 \
        float psum = 0.f;                                                                                 \
        _Pragma("unroll") for (int r = 0; r < 16; ++r) {                                                  \
          SC[r] = __builtin_amdgcn_exp2f(fmaf(SC[r], scale_log2e, -mc));                                  \
          psum += SC[r];                                                                                  \
        }                                                                                                 \
        psum = half_sum(psum);                                                                            \
        l += psum;                                                                                        \
        split3_trunc8(SC, 0, pa0, pa1, pa2);                                                              \
        split3_trunc8(SC, 8, pb0, pb1, pb2);                                                              \
      }                                                                                                   \
      if (kload && more_k) stash_k(i & 1);                                                                 \
      if (vload && more_v) stash_v((i + 1) & 1);                                                           \
      __syncthreads();                                                                                    \
  }
    f32x16 snext;
    // G = 8: waves 4-7 run each block's P.V half a block late (after the barrier, beside waves
    // 0-3's score MFMAs and softmax), so the two waves sharing a SIMD stop reaching their MFMA and
    // VALU phases together; their P planes wait in registers and the V block stays in its buffer
    // (its next refill is staged by these same waves, after the deferred P.V)
    bf16x8 pa0, pa1, pa2, pb0, pb1, pb2;
    // PRIO: the second-dispatched half (waves 4-7) loses every VALU arbitration against its SIMD
    // partner at equal priority; one static s_setprio 1 for that half (A/B switch)
    if constexpr (PRIO) {
      if (G == 8 && wv >= 4) __builtin_amdgcn_s_setprio(1);
    }
    if (G == 8 && wv >= 4) {
      for (int i = 0; i < nb;) {
        X3P_ITER_LATE(scur, snext)
        if (++i >= nb) break;
        X3P_ITER_LATE(snext, scur)
        ++i;
      }
      if (active && nb > 0) X3P_PV((nb - 1) & 1)
    } else {
      for (int i = 0; i < nb;) {
        X3P_ITER(scur, snext)
        if (++i >= nb) break;
        X3P_ITER(snext, scur)
        ++i;
      }
    }
#undef X3P_ITER
#undef X3P_ITER_LATE
#undef X3P_PV
#undef X3P_QK

    if (active) {
      if (kb0 == 0 && kb1 == NK) {
        const int q = q0 + j;
        if (q < T) {
          const float inv = 1.f / l;
          const size_t orow = (size_t(b) * T + q) * D + head * HD;
          if (outp) {
            const size_t op = size_t(B) * T * D;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int d = key_of(r, hf);
              store_x3(outp, op, orow + d, o0[r] * inv);
              store_x3(outp, op, orow + 32 + d, o1[r] * inv);
            }
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int d = key_of(r, hf);
              out[orow + d] = o0[r] * inv;
              out[orow + 32 + d] = o1[r] * inv;
            }
          }
        }
      } else {
        const size_t slot = (size_t(w) * 2 + (first ? 0 : 1)) * G + wv;
        float* po = part_o + slot * (HD * 32);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int d = key_of(r, hf);
          po[d * 32 + j] = o0[r];
          po[(32 + d) * 32 + j] = o1[r];
        }
        if (hf == 0) {
          part_ml[slot * 64 + j] = m * scale_log2e;
          part_ml[slot * 64 + 32 + j] = l;
        }
      }
    }
    u += kb1 - kb0;
    first = false;
  }
}

// attn_fwd_x3w (one wave per SIMD, two query tiles per wave): attn_wide.hip

}  // namespace

// ------------------------------------------------------------------------------------------
// Pinning census (tests/test_gpu_pin.py): every logical block of a pinned launch counts itself and
// records the XCD it ran on.
__global__ __launch_bounds__(64) void pin_census(int* __restrict__ counts, int* __restrict__ xcc, int n,
                                                 unsigned pin) {
  const PinnedBlock pb = pinned_block(pin);
  if (pb.id < 0 || pb.id >= n || threadIdx.x) return;
  atomicAdd(&counts[pb.id], 1);
  xcc[pb.id] = xcc_id();
}

extern "C" {

static thread_local unsigned g_pin = 0;  // per enqueuing thread, like the Python slice state

// XCD mask of the partition whose launches are being enqueued (0 = unpinned; pin.h). Set per slice
// before its work is enqueued or captured, like its CU count: a captured graph keeps the pin.
int nos_set_pin(unsigned mask) {
  if (mask > 0xffu) {
    g_err = "pin: XCD mask must fit 8 bits";
    return -1;
  }
  g_pin = mask;
  return 0;
}

unsigned nos_pin_mask() { return g_pin; }

int nos_pin_census(int* counts, int* xcc, int n, unsigned pin, void* stream) {
  hipLaunchKernelGGL(pin_census, dim3(pinned_grid(n, pin)), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), counts,
                     xcc, n, pin);
  return check_launch("pin_census");
}

const char* nos_kernels_last_error() { return g_err.c_str(); }

// fp32 [n] -> three bf16 planes [3][n]; n % 4 == 0
int nos_split3_f32(const float* x, void* planes, size_t n, void* stream) {
  if (n % 4) {
    g_err = "split3: n must be a multiple of 4";
    return -1;
  }
  const size_t n4 = n / 4;
  const int grid = int(std::min<size_t>((n4 + 255) / 256, 4096));
  hipLaunchKernelGGL(split3_f32, dim3(pinned_grid(pinned_cap(grid, g_pin), g_pin)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     x, reinterpret_cast<__bf16*>(planes), n4, g_pin);
  return check_launch("split3_f32");
}

static int g_x3_pipelined = 1;
static int g_x3_flags = 0;  // A/B switches: bit 0 explicit vmcnt(0) after a segment's prologue (planes input),
                            // bit 1 static s_setprio 1 for waves 4-7 (fp32 input), bit 3 64-bit
                            // stream-K bookkeeping (no reciprocal divisions), bit 5 the fixup's
                            // 2-byte plane stores, bit 6 the fixup's XCD-local tile order (measured
                            // no faster: profiles/attn_fixup_order_ab_r6.json)

int nos_attention_x3_set_flags(int f) {
  g_x3_flags = f;
  return 0;
}
static int g_x3_group = 8;  // query tiles per workgroup of the pipelined x3 kernel (4 or 8; 8 measured faster)
// fp32-input 8-tile launches: 1 = attn_fwd_x3w (attn_wide.hip: one wave per SIMD, two tiles per wave;
// 4-8% faster on the box, profiles/attn_wide_ab_r6.json), 0 = attn_fwd_x3p<8> (two waves per SIMD);
// NOS_ATTN_WIDE=0 at load time, nos_attention_x3_set_wide for A/B runs
static int g_x3_wide = [] {
  const char* e = std::getenv("NOS_ATTN_WIDE");
  return (e && std::string(e) == "0") ? 0 : 1;
}();

int nos_attention_x3_set_wide(int on) {
  g_x3_wide = on ? 1 : 0;
  return 0;
}

int nos_attention_x3_wide() { return g_x3_wide; }

// 4 = two 256-thread workgroups per CU, 8 = one 512-thread workgroup sharing K/V (default)
int nos_attention_x3_set_group(int g) {
  if (g != 4 && g != 8) {
    g_err = "attention x3: group must be 4 or 8";
    return -1;
  }
  g_x3_group = g;
  return 0;
}

int nos_attention_x3_group() { return g_x3_pipelined ? g_x3_group : 4; }

// 1 = software-pipelined x3 kernel (default), 0 = the block-at-a-time x3 kernel (A/B reference)
int nos_attention_x3_set_pipelined(int on) {
  g_x3_pipelined = on ? 1 : 0;
  return 0;
}

// workgroups per CU of the x3 attention kernel (persistent grid = this x slice CUs)
int nos_attention_x3_wg_per_cu() {
  if (g_x3_pipelined && g_x3_group == 8 && g_x3_wide) return nos_attn_x3w_occupancy();
  int n = 0;
  const hipError_t e =
      !g_x3_pipelined  ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, attn_fwd_x3, 256, 0)
      : g_x3_group == 8 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, attn_fwd_x3p<8>, 512, 0)
                        : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, attn_fwd_x3p<4>, 256, 0);
  if (e != hipSuccess || n <= 0) n = 1;
  return n;
}

// Stream-K attention over x3 planes of a packed [B, T, 3*H*64] QKV tensor (plane stride
// `plane_stride` elements); output fp32 [B, T, H*64] (out) or its x3 planes [3][B*T*H*64] (outp),
// exactly one non-null. Heads h0 .. h0+hn-1 only: a slice of few CUs runs the heads in blocks so its
// workgroups share one block's K/V in L2 (with every head in flight at once, the K/V planes of all
// heads are the L2 working set — the traffic concurrent partitions contend for). Workspace:
// nos_attention_ws_bytes of the LDS variant (variant 0 layout), merged by the same fixup kernel.
static int attention_x3_launch(const void* qkv3, size_t plane_stride, float* out, void* outp, float* ws, int B,
                               int T, int H, int h0, int hn, int head_dim, float scale, int waves, void* stream,
                               bool f32in, bool fixup = true, int* cnt = nullptr) {
  if ((out == nullptr) == (outp == nullptr)) {
    g_err = "attention x3: exactly one of out / outp";
    return -1;
  }
  if (head_dim != HD) {
    g_err = "attention x3: head_dim must be 64";
    return -1;
  }
  if (ws == nullptr || waves <= 0) {
    g_err = "attention x3: needs waves > 0 and a workspace";
    return -1;
  }
  if (plane_stride % 8) {
    g_err = "attention x3: plane stride must be a multiple of 8 elements (16-B aligned planes)";
    return -1;
  }
  if (h0 < 0 || hn <= 0 || h0 + hn > H) {
    g_err = "attention x3: head block out of range";
    return -1;
  }
  if (!g_x3_pipelined && (h0 != 0 || hn != H)) {
    g_err = "attention x3: head blocks need the pipelined kernel";
    return -1;
  }
  if (f32in && (!g_x3_pipelined || nos_attention_x3_group() != 8)) {
    g_err = "attention x3: fp32 input needs the pipelined 8-tile kernel";
    return -1;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int G = nos_attention_x3_group();
  const int NK = (T + 31) / 32, QG = (NK + G - 1) / G;
  float* part_o = ws;
  float* part_ml = ws + size_t(waves) * 2 * G * HD * 32;
  __bf16* op = reinterpret_cast<__bf16*>(outp);
  const float sl2 = scale * 1.4426950408889634f;
  const __bf16* q3 = reinterpret_cast<const __bf16*>(qkv3);
  if (waves >= (1 << 22)) {
    g_err = "attention x3: at most 2^22 workgroups";
    return -1;
  }
  if (g_pin && !g_x3_pipelined) {
    g_err = "attention x3: pinned launches need the pipelined kernel";
    return -1;
  }
  const unsigned pin = g_pin;
  const int pk = waves | int(pin << 22) | ((g_x3_flags & 4) ? (1 << 30) : 0);
  // reciprocal-division bookkeeping while every numerator (w * U <= (P + 1) * U) is < 2^23;
  // flag bit 3 keeps the 64-bit form (A/B runs)
  const long long Uk = (long long)B * hn * QG * NK;
  const bool fdiv = !(g_x3_flags & 8) && (Uk + 1) * (waves + 1) < (1ll << 23);
  const dim3 grid(pinned_grid(waves, pin));
  if (!g_x3_pipelined)
    hipLaunchKernelGGL(attn_fwd_x3, dim3(waves), dim3(256), 0, s, q3, plane_stride, out, op, part_o, part_ml, B, T, H,
                       sl2, waves);
  else if (G == 8 && f32in && g_x3_wide)
    nos_attn_x3w_launch(fdiv, grid, s, reinterpret_cast<const float*>(qkv3), out, op, part_o, part_ml, B, T, hn, h0,
                        H, sl2, pk, fixup ? cnt : nullptr);
  else if (G == 8 && f32in && (g_x3_flags & 2))
    hipLaunchKernelGGL((attn_fwd_x3p<8, false, true, true>), grid, dim3(512), 0, s, q3, plane_stride, out, op,
                       part_o, part_ml, B, T, hn, h0, H, sl2, pk);
  else if (G == 8 && f32in && fdiv)
    hipLaunchKernelGGL((attn_fwd_x3p<8, false, true, false, true>), grid, dim3(512), 0, s, q3, plane_stride, out,
                       op, part_o, part_ml, B, T, hn, h0, H, sl2, pk);
  else if (G == 8 && f32in)
    hipLaunchKernelGGL((attn_fwd_x3p<8, false, true>), grid, dim3(512), 0, s, q3, plane_stride, out, op, part_o,
                       part_ml, B, T, hn, h0, H, sl2, pk);
  else if (G == 8 && (g_x3_flags & 1))
    hipLaunchKernelGGL((attn_fwd_x3p<8, true>), grid, dim3(512), 0, s, q3, plane_stride, out, op, part_o,
                       part_ml, B, T, hn, h0, H, sl2, pk);
  else if (G == 8)
    hipLaunchKernelGGL(attn_fwd_x3p<8>, grid, dim3(512), 0, s, q3, plane_stride, out, op, part_o, part_ml, B,
                       T, hn, h0, H, sl2, pk);
  else
    hipLaunchKernelGGL(attn_fwd_x3p<4>, grid, dim3(256), 0, s, q3, plane_stride, out, op, part_o, part_ml, B,
                       T, hn, h0, H, sl2, pk);
  if (int rc = check_launch("attn_fwd_x3")) return rc;
  if (!fixup) return 0;  // the partials are merged by the consumer (attn_proj.hip)
  if (cnt && G == 8 && f32in && g_x3_wide && g_x3_pipelined) return 0;  // merged in the kernel
  // bit 8: the earlier 2-byte stores (A/B); bit 9: XCD-local tile order (unpinned launches, flag bit 6)
  const unsigned fpin = pin | ((g_x3_flags & 32) ? 0x100u : 0u) | ((!pin && (g_x3_flags & 64)) ? 0x200u : 0u);
  if (G == 8)
    hipLaunchKernelGGL(attn_sk_lds_fixup<8>, dim3(pinned_grid(8 * ((B * hn * QG * 8 + 7) / 8), pin)), dim3(256), 0, s,
                       part_o, part_ml,
                       out, B, T, hn, waves, op, h0, H, fpin);
  else
    hipLaunchKernelGGL(attn_sk_lds_fixup<4>, dim3(pinned_grid(B * hn * QG * 4, pin)), dim3(256), 0, s,
                       part_o, part_ml,
                       out, B, T, hn, waves, op, h0, H, fpin);
  return check_launch("attn_sk_lds_fixup");
}

int nos_attention_x3_sk_heads(const void* qkv3, size_t plane_stride, float* out, void* outp, float* ws, int B,
                              int T, int H, int h0, int hn, int head_dim, float scale, int waves, void* stream) {
  return attention_x3_launch(qkv3, plane_stride, out, outp, ws, B, T, H, h0, hn, head_dim, scale, waves, stream, false);
}

// the same from an fp32 packed QKV tensor [B, T, 3*H*64] (split to planes inside the kernel)
int nos_attention_x3f_sk_heads(const float* qkv, float* out, void* outp, float* ws, int B, int T, int H, int h0,
                               int hn, int head_dim, float scale, int waves, void* stream) {
  return attention_x3_launch(qkv, 8, out, outp, ws, B, T, H, h0, hn, head_dim, scale, waves, stream, true);
}

// the same with the stream-K merge inside the wide kernel (attn_fwd_x3w) when it runs: cnt holds
// ncnt >= B*hn*ceil(ceil(T/32)/8) row counters, zero before the first launch (every launch leaves
// them zero); launches that share cnt must not run concurrently (one counter array per stream)
int nos_attention_x3f_sk_heads_merged(const float* qkv, float* out, void* outp, float* ws, int* cnt, int ncnt, int B,
                                      int T, int H, int h0, int hn, int head_dim, float scale, int waves,
                                      void* stream) {
  const int QG = ((T + 31) / 32 + 7) / 8;
  if (cnt == nullptr || (long long)ncnt < (long long)B * hn * QG) {
    g_err = "attention x3 merged: needs B*hn*QG row counters";
    return -1;
  }
  return attention_x3_launch(qkv, 8, out, outp, ws, B, T, H, h0, hn, head_dim, scale, waves, stream, true, true, cnt);
}

// The x3 attention from fp32 QKV over all heads WITHOUT the stream-K fixup: split query tiles
// leave their partials in ws, tiles one workgroup finished go to `out` (fp32); the fused
// merge + projection + LayerNorm kernel (nos_attn_merge_proj_ln) consumes both.
int nos_attention_x3f_partials(const float* qkv, float* out, float* ws, int B, int T, int H, int head_dim,
                               float scale, int waves, void* stream) {
  if (out == nullptr) {
    g_err = "attention x3 partials: needs the fp32 direct-output buffer";
    return -1;
  }
  return attention_x3_launch(qkv, 8, out, nullptr, ws, B, T, H, 0, H, head_dim, scale, waves, stream, true, false);
}

int nos_attention_x3_sk(const void* qkv3, size_t plane_stride, float* out, void* outp, float* ws, int B, int T,
                        int H, int head_dim, float scale, int waves, void* stream) {
  return nos_attention_x3_sk_heads(qkv3, plane_stride, out, outp, ws, B, T, H, 0, H, head_dim, scale, waves, stream);
}

// y (fp32) or yp (x3 planes [3][rows][D]) — exactly one of them non-null; `wgs` workgroups of 4
// rows each (grid-stride), 0 = one per 4 rows
int nos_layernorm_f32_grid(const float* x, const float* w, const float* b, float* y, void* yp, int rows, int D,
                           float eps, int wgs, void* stream) {
  if ((y == nullptr) == (yp == nullptr)) {
    g_err = "layernorm: exactly one of y / yp";
    return -1;
  }
  if (rows <= 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // rows in flight per wave (NOS_LN_ROWS, 1 or 2; read once)
  static const int R = [] {
    const char* e = std::getenv("NOS_LN_ROWS");
    return (e && std::atoi(e) == 1) ? 1 : 2;
  }();
  const int full = (rows + 4 * R - 1) / (4 * R);
  const dim3 grid(pinned_grid(pinned_cap(wgs > 0 ? std::min(wgs, full) : full, g_pin), g_pin)), block(256);
  __bf16* p = reinterpret_cast<__bf16*>(yp);
  const unsigned pin = g_pin;
#define NOS_LN_CASE(DD, NPL)                                                                      \
  case DD:                                                                                        \
    if (R == 2)                                                                                   \
      hipLaunchKernelGGL((layernorm_f32<NPL, 2>), grid, block, 0, s, x, w, b, y, p, rows, eps, pin); \
    else                                                                                          \
      hipLaunchKernelGGL((layernorm_f32<NPL, 1>), grid, block, 0, s, x, w, b, y, p, rows, eps, pin); \
    break;
  switch (D) {
    NOS_LN_CASE(384, 6)
    NOS_LN_CASE(768, 12)
    NOS_LN_CASE(1024, 16)
    NOS_LN_CASE(1536, 24)
    NOS_LN_CASE(2048, 32)
    default:
      g_err = "layernorm: unsupported hidden size " + std::to_string(D);
      return -1;
  }
#undef NOS_LN_CASE
  return check_launch("layernorm_f32");
}

// Split-K combine (+ bias, residual, broadcast residual r2 or null) into xout, and LayerNorm(xout) as
// x3 planes into yp when w/b/yp are given; part = [splits][rows][D] fp32; D in {384, 768}; `wgs`
// workgroups of 4 rows (grid-stride), 0 = one per 4 rows.
static int splitk_layernorm(const float* part, int splits, SkMap sk, const float* bias, const float* res,
                            const float* r2, int r2_rows, float* xout, const float* w, const float* b, void* yp,
                            int rows, int D, float eps, int wgs, void* stream) {
  if (!part || splits < 1 || !bias || !res || !xout || (r2 && r2_rows <= 0) || ((w == nullptr) != (yp == nullptr)) ||
      ((w == nullptr) != (b == nullptr))) {
    g_err = "splitk_layernorm: partials, bias, residual and output required; LayerNorm needs w, b and yp";
    return -1;
  }
  if (rows <= 0) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int full = (rows + 3) / 4;
  const unsigned pin = g_pin;
  const dim3 grid(pinned_grid(pinned_cap(wgs > 0 ? std::min(wgs, full) : full, pin), pin)), block(256);
  __bf16* p = reinterpret_cast<__bf16*>(yp);
  switch (D) {
    case 384:
      hipLaunchKernelGGL(splitk_layernorm_f32<6>, grid, block, 0, s, part, splits, sk, bias, res, r2, r2_rows, xout, w,
                         b, p, rows, eps, pin);
      break;
    case 768:
      hipLaunchKernelGGL(splitk_layernorm_f32<12>, grid, block, 0, s, part, splits, sk, bias, res, r2, r2_rows, xout, w,
                         b, p, rows, eps, pin);
      break;
    default:
      g_err = "splitk_layernorm: unsupported hidden size " + std::to_string(D);
      return -1;
  }
  return check_launch("splitk_layernorm_f32");
}

int nos_splitk_layernorm_f32(const float* part, int splits, const float* bias, const float* res, const float* r2,
                             int r2_rows, float* xout, const float* w, const float* b, void* yp, int rows, int D,
                             float eps, int wgs, void* stream) {
  return splitk_layernorm(part, splits, SkMap{0, 0, 0, 1, 1, 1}, bias, res, r2, r2_rows, xout, w, b, yp, rows, D, eps,
                          wgs, stream);
}

// The same over stream-K partials (gemm_x3k): map = {P, U, nk, bm, bn, tiles_n} from
// nos_gemm_x3_streamk_map; tile t's planes 0 .. sk_segments(t)-1 are added in order.
int nos_streamk_layernorm_f32(const float* part, const int* map, const float* bias, const float* res, const float* r2,
                              int r2_rows, float* xout, const float* w, const float* b, void* yp, int rows, int D,
                              float eps, int wgs, void* stream) {
  if (!map || map[0] <= 0 || map[1] < map[0] || map[2] <= 0 || map[3] <= 0 || map[4] <= 0 || map[4] % 2 ||
      map[5] * map[4] != D) {
    g_err = "streamk_layernorm: map must be {P <= U, U, nk, bm, bn (even), tiles_n} with tiles_n * bn = D";
    return -1;
  }
  return splitk_layernorm(part, 1, SkMap{map[0], map[1], map[2], map[3], map[4], map[5]}, bias, res, r2, r2_rows,
                          xout, w, b, yp, rows, D, eps, wgs, stream);
}

int nos_layernorm_f32(const float* x, const float* w, const float* b, float* y, void* yp, int rows, int D,
                      float eps, void* stream) {
  return nos_layernorm_f32_grid(x, w, b, y, yp, rows, D, eps, 0, stream);
}

int nos_bias_gelu_f32(float* y, const float* b, int rows, int N, void* stream) {
  if (N % 4) {
    g_err = "bias_gelu: N must be a multiple of 4";
    return -1;
  }
  const size_t n4 = size_t(rows) * N / 4;
  const int grid = int(std::min<size_t>((n4 + 255) / 256, 2048));
  hipLaunchKernelGGL(bias_gelu_f32, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), y, b, n4, N / 4);
  return check_launch("bias_gelu_f32");
}

// Resident attention waves per CU (occupancy of attn_fwd_sk); the persistent grid is this times
// the slice's CU count.
// Variant: 0 = LDS-shared K/V workgroup kernel (default); 2 / 3 = one-wave kernel with 2 or 3
// resident waves per SIMD (register budget 256 or 168 VGPRs), kept for A/B measurement.
static int g_variant = 0;

int nos_attention_set_variant(int v) {
  if (v != 0 && v != 2 && v != 3) return -1;
  g_variant = v;
  return 0;
}

// Persistent grid slots per CU for the selected variant (workgroups, not waves).
int nos_attention_waves_per_cu() {
  int n = 0;
  hipError_t e;
  if (g_variant == 0)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, attn_fwd_sk_lds, 256, 0);
  else if (g_variant == 3)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, attn_fwd_sk<3>, 64, 0);
  else
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, attn_fwd_sk<2>, 64, 0);
  if (e != hipSuccess || n <= 0) n = g_variant == 0 ? 2 : 4 * g_variant;
  return n;
}

// bytes of caller-provided workspace for a stream-K launch of `waves` waves. The workspace comes
// from the caller's stream-ordered allocator, so concurrent slices never share scratch and a launch
// inside graph capture never allocates.
size_t nos_attention_ws_bytes(int waves) {
  return size_t(waves) * 2 * (HD * 32 + 64) * sizeof(float) * (g_variant == 0 ? 4 : 1);
}

int nos_attention_f32_sk(const float* qkv, float* out, float* ws, int B, int T, int H, int head_dim, float scale,
                         int waves, void* stream) {
  if (head_dim != HD) {
    g_err = "attention: head_dim must be 64";
    return -1;
  }
  if (ws == nullptr || waves <= 0) {
    g_err = "attention: stream-K launch needs waves > 0 and a workspace (nos_attention_ws_bytes)";
    return -1;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float scale_log2e = scale * 1.4426950408889634f;
  const int NK = (T + 31) / 32;
  if (g_variant == 0) {
    const int QG = (NK + 3) / 4;
    float* part_o = ws;
    float* part_ml = ws + size_t(waves) * 8 * HD * 32;
    hipLaunchKernelGGL(attn_fwd_sk_lds, dim3(waves), dim3(256), 0, s, qkv, out, part_o, part_ml, B, T, H,
                       scale_log2e, waves);
    if (int rc = check_launch("attn_fwd_sk_lds")) return rc;
    hipLaunchKernelGGL(attn_sk_lds_fixup<4>, dim3(B * H * QG * 4), dim3(256), 0, s, part_o, part_ml, out, B, T, H, waves,
                       static_cast<__bf16*>(nullptr), 0, H, 0u);
    return check_launch("attn_sk_lds_fixup");
  }
  float* part_o = ws;
  float* part_ml = ws + size_t(waves) * 2 * HD * 32;
  if (g_variant == 3)
    hipLaunchKernelGGL(attn_fwd_sk<3>, dim3(waves), dim3(64), 0, s, qkv, out, part_o, part_ml, B, T, H, scale_log2e,
                       waves);
  else
    hipLaunchKernelGGL(attn_fwd_sk<2>, dim3(waves), dim3(64), 0, s, qkv, out, part_o, part_ml, B, T, H, scale_log2e,
                       waves);
  if (int rc = check_launch("attn_fwd_sk")) return rc;
  hipLaunchKernelGGL(attn_sk_fixup, dim3(B * H * NK), dim3(256), 0, s, part_o, part_ml, out, B, T, H, waves);
  return check_launch("attn_sk_fixup");
}

int nos_attention_f32(const float* qkv, float* out, int B, int T, int H, int head_dim, float scale, void* stream) {
  if (head_dim != HD) {
    g_err = "attention: head_dim must be 64";
    return -1;
  }
  const int qtiles = (T + 31) / 32;
  hipLaunchKernelGGL(attn_fwd_f32, dim3(qtiles, H, B), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), qkv, out,
                     T, H, scale * 1.4426950408889634f);
  return check_launch("attn_fwd_f32");
}

}  // extern "C"
