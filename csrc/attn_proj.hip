// nos fused attention epilogue for gfx950: stream-K merge + output projection + bias + residual +
// LayerNorm, fp32-accurate on the bf16 matrix cores (x3 planes).
//
// The transformer step after attention was three launches on the round-3 tree: the stream-K fixup
// (merge the key-range partials of every split query tile, write O as x3 planes), the projection
// GEMM with the residual in its epilogue, and a LayerNorm kernel emitting LN2's planes
// (profiles/rocprof_r3_spx_replay_packed_epilogue.txt: 8.7 + 15.3 + 5.8 us per layer on the whole
// GPU). Here one 512-thread workgroup owns 32 whole rows:
//
//  1. merge: for each (row, head) the partial images of the attention workgroups whose key ranges
//     cover that query tile (the same slot map attn_sk_lds_fixup reads) are combined with their
//     (m, l) in one online-softmax pass, or O is taken from the direct output of a tile one
//     workgroup finished; O goes to LDS as three exact bf16 planes [plane][32 rows][D] (no global
//     round trip for O);
//  2. projection: every wave owns D/8 columns (3 blocks of 16 for D = 384) and both 16-row blocks;
//     its weight fragments are private to it, so they stream from L2 straight into registers
//     (two k-steps in flight) while the A fragments come from the LDS image: six
//     v_mfma_f32_16x16x32_bf16 per block and k-step (the x3 product);
//  3. epilogue: + bias + residual (the fp32 residual stream, stored), then LayerNorm over the whole
//     row (the workgroup owns it: cross-lane then cross-wave sums through LDS, two passes) and its
//     planes for fc1.
//
// Workspace contract (attention_x3_launch with the fixup skipped): part_o [slot][64 d][32 q],
// part_ml [slot][m (log2 domain) 32 | l 32], slot = (w * 2 + (not the workgroup's first segment)) * 8
// + query tile in group — only a workgroup's first and last segments can be partial, every group it
// covers whole goes to o_direct [B*T][D] fp32, as does a group one workgroup covers alone.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <string>

#include "pin.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {
thread_local std::string g_err;

constexpr int HD = 64;   // head dim
constexpr int QPG = 8;   // query tiles per attention workgroup (attn_fwd_x3p<8>)
constexpr int BM = 32;   // rows per workgroup
constexpr int NW = 8;    // waves

__device__ __forceinline__ f32x4 mfma_x3_16(const bf16x8& a0, const bf16x8& a1, const bf16x8& a2, const bf16x8& b0,
                                            const bf16x8& b1, const bf16x8& b2, f32x4 d) {
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b0, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b2, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b0, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b1, d, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, d, 0, 0, 0);
}

__device__ __forceinline__ void split3v(const f32x8& x, bf16x8& a, bf16x8& b, bf16x8& c) {
  a = __builtin_convertvector(x, bf16x8);  // round to nearest even, then the exact residuals
  const f32x8 r = x - __builtin_convertvector(a, f32x8);
  b = __builtin_convertvector(r, bf16x8);
  c = __builtin_convertvector(r - __builtin_convertvector(b, f32x8), bf16x8);
}

// floor(n / d) for n < 2^23 through the f32 reciprocal (rd = 1/d): the product is within one of the
// quotient there, and one integer correction makes it exact. The merge's stream-K bookkeeping
// (unit ranges of the attention grid) would otherwise be 64-bit divisions: hundreds of VALU
// instructions each, several per task.
__device__ __forceinline__ long long udiv23(long long n, long long d, float rd) {
  int q = int(float(int(n)) * rd);
  const int r = int(n) - q * int(d);
  q += (r < 0) ? -1 : (r >= int(d) ? 1 : 0);
  return q;
}

template <bool WIDE>
__device__ __forceinline__ long long sk_div(long long n, long long d, float rd) {
  if constexpr (WIDE)
    return n / d;
  else
    return udiv23(n, d, rd);
}

// sum over the 16 lanes that share lane >> 4 (the 16 columns of a 16x16 accumulator block)
__device__ __forceinline__ float sum16(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int D, bool WIDE>
__global__ __launch_bounds__(512, 1) void attn_merge_proj_ln(
    const float* __restrict__ part_o, const float* __restrict__ part_ml, const float* __restrict__ o_direct,
    int B, int T, int H, int P, const __bf16* __restrict__ W, size_t w_plane, const float* __restrict__ bias,
    const float* __restrict__ res, const float* __restrict__ ln_w, const float* __restrict__ ln_b, float eps,
    float* __restrict__ xout, __bf16* __restrict__ yp, unsigned pin, int ablate) {
  static_assert(D % (NW * 16) == 0 && D % 32 == 0, "D must split into 16-column blocks over 8 waves");
  constexpr int LSTR = D + 8;        // LDS row (bf16): +16 B per row spreads a fragment read's rows over banks
  constexpr int NB = D / NW / 16;    // 16-column blocks per wave
  constexpr int KS = D / 32;         // k-steps of the projection
  constexpr int CH = HD / 8;         // 8-dim chunks per head
  constexpr int NBUF = 3;            // weight k-steps in registers (two in flight behind the MFMAs)
  __shared__ __attribute__((aligned(16))) __bf16 As[3 * BM * LSTR];
  __shared__ float red[2][NW][BM];

  const PinnedBlock pb = pinned_block(pin);
  if (pb.id < 0) return;
  const int M = B * T;
  const int tiles = (M + BM - 1) / BM;
  const int NK = (T + 31) / 32, QG = (NK + QPG - 1) / QPG;
  const long long U = (long long)B * H * QG * NK;
  const float rU = 1.f / float(U), rP = 1.f / float(P), rT = 1.f / float(T);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int n0 = wave * (NB * 16);
  const size_t plane_out = size_t(M) * D;
  // this lane's weight fragment rows: W[p][n0 + 16 cb + r16][32 s + 8 kq .. +7]
  const __bf16* wb = W + size_t(n0 + r16) * D + 8 * kq;

  // one tile per logical workgroup (the launch covers every tile, pinned or not); no grid-stride
  // loop: its weight loads would be loop-invariant and the compiler would hoist (and spill) them all
  const int tile = pb.id;
  if (tile >= tiles) return;
  {
    const int r0 = tile * BM;
    bf16x8 bq[NBUF][NB][3];
    auto load_b = [&](int s, bf16x8 (&dst)[NB][3]) {
#pragma unroll
      for (int cb = 0; cb < NB; ++cb)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          dst[cb][p] = *reinterpret_cast<const bf16x8*>(wb + ((ablate & 2) ? 0 : p * w_plane + size_t(16 * cb) * D + 32 * s));
    };
    // the first weight k-steps do not depend on the merge: their L2 latency hides behind it
#pragma unroll
    for (int s = 0; s < NBUF - 1; ++s) load_b(s, bq[s]);

    // ---- 1. merge the attention partials of the 32 rows, O -> LDS planes ----
    // Every load of the thread's TPT tasks (up to MC contributors each) is issued before any is
    // used: the merge is a few hundred bytes per task, so its time is the L2/MALL round trips,
    // which overlap only when they are in flight together. A tile one workgroup finished is
    // contributor 0 with (m, l) = (0, 1) and stride 1 into o_direct.
    constexpr int TPT = (D / HD) * CH * BM / (NW * 64);
    static_assert((D / HD) * CH * BM % (NW * 64) == 0, "tasks must divide over the workgroup");
    constexpr int MC = 4;
    if (ablate & 1) {  // timing only: no merge, O = 0
#pragma unroll
      for (int t = 0; t < TPT; ++t) {
        const int task = tid + t * NW * 64;
        const int i = task % BM, c = (task / BM) % CH, h = task / (BM * CH);
        __bf16* dst = &As[i * LSTR + h * HD + 8 * c];
        *reinterpret_cast<bf16x8*>(dst) = bf16x8{};
        *reinterpret_cast<bf16x8*>(dst + BM * LSTR) = bf16x8{};
        *reinterpret_cast<bf16x8*>(dst + 2 * BM * LSTR) = bf16x8{};
      }
    } else {
    f32x8 ow[TPT][MC];
    float mw[TPT][MC], lw[TPT][MC];
    long long more_lo[TPT], more_hi[TPT], t0s[TPT];
#pragma unroll
    for (int t = 0; t < TPT; ++t) {
      const int task = tid + t * NW * 64;
      const int i = task % BM, c = (task / BM) % CH, h = task / (BM * CH);
      const int row = min(r0 + i, M - 1);
      const int b = int(sk_div<WIDE>(row, T, rT)), q = row - b * T;
      const int qt = q >> 5, wv = qt % QPG, qg = qt / QPG, j = q & 31;
      const long long grp = ((long long)b * H + h) * QG + qg;
      const long long t0 = grp * NK, t1 = t0 + NK;
      const long long w_lo = sk_div<WIDE>((t0 + 1) * P + U - 1, U, rU) - 1;
      const long long w_hi = sk_div<WIDE>(t1 * P + U - 1, U, rU) - 1;
      const bool direct = w_lo == w_hi;
      t0s[t] = t0;
      more_lo[t] = direct ? 1 : w_lo + MC;
      more_hi[t] = direct ? 0 : w_hi;
#pragma unroll
      for (int k = 0; k < MC; ++k) {
        const long long w = w_lo + k;
        const long long s0 = sk_div<WIDE>(w * U, P, rP);
        const bool part = !direct && w <= w_hi && s0 != sk_div<WIDE>((w + 1) * U, P, rP);
        const long long slot = part ? (w * 2 + (s0 >= t0 ? 0 : 1)) * QPG + wv : 0;
        const bool dir0 = direct && k == 0;
        const float* po = dir0 ? o_direct + size_t(row) * D + h * HD + 8 * c : part_o + slot * (HD * 32) + (8 * c) * 32 + j;
        const int st = dir0 ? 1 : 32;
        // an unused contributor reads slot 0 (always mapped, possibly never written): its values
        // are zeroed, not just weighted by 0, since uninitialised words may be NaN
#pragma unroll
        for (int dd = 0; dd < 8; ++dd) {
          const float v = po[dd * st];
          ow[t][k][dd] = (part || dir0) ? v : 0.f;
        }
        const float m_ = part_ml[slot * 64 + j], l_ = part_ml[slot * 64 + 32 + j];
        mw[t][k] = part ? m_ : (dir0 ? 0.f : -INFINITY);
        lw[t][k] = part ? l_ : (dir0 ? 1.f : 0.f);
      }
    }
#pragma unroll
    for (int t = 0; t < TPT; ++t) {
      const int task = tid + t * NW * 64;
      const int i = task % BM, c = (task / BM) % CH, h = task / (BM * CH);
      float mx = mw[t][0];
#pragma unroll
      for (int k = 1; k < MC; ++k) mx = fmaxf(mx, mw[t][k]);
      float l = 0.f;
      f32x8 o = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < MC; ++k) {
        const float sn = __builtin_amdgcn_exp2f(mw[t][k] - mx);
        l += lw[t][k] * sn;
        o += ow[t][k] * sn;
      }
      // more than MC contributors (grids far above the CU count): the rest, one at a time
      for (long long w = more_lo[t]; w <= more_hi[t]; ++w) {
        const long long s0 = sk_div<WIDE>(w * U, P, rP);
        if (s0 == sk_div<WIDE>((w + 1) * U, P, rP)) continue;  // empty range
        const int row = min(r0 + i, M - 1);
        const int q = row % T, qt = q >> 5, wv = qt % QPG, j = q & 31;
        const long long slot = (w * 2 + (s0 >= t0s[t] ? 0 : 1)) * QPG + wv;
        const float m_ = part_ml[slot * 64 + j], l_ = part_ml[slot * 64 + 32 + j];
        const float* po = part_o + slot * (HD * 32) + (8 * c) * 32 + j;
        f32x8 v;
#pragma unroll
        for (int dd = 0; dd < 8; ++dd) v[dd] = po[dd * 32];
        const float mn = fmaxf(mx, m_);
        const float so = __builtin_amdgcn_exp2f(mx - mn), sn = __builtin_amdgcn_exp2f(m_ - mn);
        l = l * so + l_ * sn;
        o = o * so + v * sn;
        mx = mn;
      }
      o = o * (1.f / l);
      if (r0 + i >= M) o = f32x8{0, 0, 0, 0, 0, 0, 0, 0};
      bf16x8 p0, p1, p2;
      split3v(o, p0, p1, p2);
      __bf16* dst = &As[i * LSTR + h * HD + 8 * c];
      *reinterpret_cast<bf16x8*>(dst) = p0;
      *reinterpret_cast<bf16x8*>(dst + BM * LSTR) = p1;
      *reinterpret_cast<bf16x8*>(dst + 2 * BM * LSTR) = p2;
    }
    }
    __syncthreads();

    // ---- 2. projection: C[32][D] = O . W^T on x3 planes, three weight k-steps in flight ----
    f32x4 acc[2][NB];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int cb = 0; cb < NB; ++cb) acc[rb][cb] = f32x4{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s + NBUF - 1 < KS) load_b(s + NBUF - 1, bq[(s + NBUF - 1) % NBUF]);
      // keep the prefetch at the top of its step: loads retire in order, so the waits before this
      // step's MFMAs are then vmcnt(loads of the NBUF-1 younger steps), never vmcnt(0)
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 af[2][3];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          af[rb][p] = *reinterpret_cast<const bf16x8*>(&As[p * BM * LSTR + (16 * rb + r16) * LSTR + 32 * s + 8 * kq]);
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int cb = 0; cb < NB; ++cb)
          acc[rb][cb] = mfma_x3_16(af[rb][0], af[rb][1], af[rb][2], bq[s % NBUF][cb][0], bq[s % NBUF][cb][1],
                                   bq[s % NBUF][cb][2], acc[rb][cb]);
    }

    // ---- 3. + bias + residual -> x (stored); LayerNorm over the row -> planes ----
    // acc[rb][cb][r] = C[16 rb + 4 kq + r][n0 + 16 cb + r16]
    float rs[2][4];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) rs[rb][r] = 0.f;
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) {
      const int col = n0 + 16 * cb + r16;
      const float bv = bias[col];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = min(r0 + 16 * rb + 4 * kq + r, M - 1);
          const float v = acc[rb][cb][r] + bv + res[size_t(row) * D + col];
          acc[rb][cb][r] = v;
          rs[rb][r] += v;
        }
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float t = sum16(rs[rb][r]);
        if (r16 == 0) red[0][wave][16 * rb + 4 * kq + r] = t;
      }
    __syncthreads();
    float mean[2][4], rstd[2][4];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += red[0][w][16 * rb + 4 * kq + r];
        mean[rb][r] = t * (1.0f / D);
        rs[rb][r] = 0.f;
      }
#pragma unroll
    for (int cb = 0; cb < NB; ++cb)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float dv = acc[rb][cb][r] - mean[rb][r];
          rs[rb][r] += dv * dv;
        }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float t = sum16(rs[rb][r]);
        if (r16 == 0) red[1][wave][16 * rb + 4 * kq + r] = t;
      }
    __syncthreads();
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += red[1][w][16 * rb + 4 * kq + r];
        rstd[rb][r] = rsqrtf(t * (1.0f / D) + eps);
      }
    // LN(x) as planes through LDS (the A image is free: the two reductions above were barriers
    // behind the last fragment read), then whole 16-B row chunks to global
#pragma unroll
    for (int cb = 0; cb < NB; ++cb) {
      const int col = n0 + 16 * cb + r16;
      const float gw = ln_w[col], gb = ln_b[col];
#pragma unroll
      for (int rb = 0; rb < 2; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int li = 16 * rb + 4 * kq + r;
          const int row = r0 + li;
          const float v = acc[rb][cb][r];
          if (row < M && !(ablate & 4)) xout[size_t(row) * D + col] = v;
          const float y = (v - mean[rb][r]) * rstd[rb][r] * gw + gb;
          const __bf16 h0 = (__bf16)y;
          const float r1 = y - (float)h0;
          const __bf16 h1 = (__bf16)r1;
          __bf16* d = &As[li * LSTR + col];
          d[0] = h0;
          d[BM * LSTR] = h1;
          d[2 * BM * LSTR] = (__bf16)(r1 - (float)h1);
        }
    }
    __syncthreads();
    constexpr int CPR = D / 8;  // 16-B chunks per row and plane
#pragma unroll
    for (int k = 0; k < 3 * BM * CPR / (NW * 64); ++k) {
      const int f = tid + k * NW * 64;
      const int p = f / (BM * CPR), li = (f / CPR) % BM, ch = f % CPR;
      const int row = r0 + li;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(&As[p * BM * LSTR + li * LSTR + 8 * ch]);
      if (row < M && !(ablate & 4))
        *reinterpret_cast<bf16x8*>(yp + p * plane_out + size_t(row) * D + 8 * ch) = v;
    }
  }
}

}  // namespace

extern "C" {

// timing-only ablation switch (bit 0: no merge, bit 1: one weight fragment for every k-step, bit 2:
// no stores); 0 in production
static int g_ablate = 0;
int nos_attn_proj_set_ablate(int a) {
  g_ablate = a;
  return 0;
}

const char* nos_attn_proj_last_error() { return g_err.c_str(); }

// Rows per workgroup of the fused kernel (the host sizes nothing else from it).
int nos_attn_proj_rows() { return BM; }

// ws: the attention workspace of a launch of `waves` workgroups with the fixup skipped
// (part_o = ws, part_ml = ws + waves * 2 * 8 * 64 * 32); o_direct, res, xout: fp32 [B*T][D];
// w3: bf16 weight planes [3][D][D] (plane stride w_plane elements); yp: bf16 [3][B*T][D].
int nos_attn_merge_proj_ln(const float* ws, int waves, const float* o_direct, int B, int T, int H,
                           const void* w3, size_t w_plane, const float* bias, const float* res, const float* ln_w,
                           const float* ln_b, float eps, float* xout, void* yp, void* stream) {
  const int D = H * HD;
  if (D != 384) {
    g_err = "attn_merge_proj_ln: hidden size must be 384 (6 heads of 64)";
    return -1;
  }
  if (waves <= 0 || B <= 0 || T <= 0) {
    g_err = "attn_merge_proj_ln: needs B, T, waves > 0";
    return -1;
  }
  if (w_plane % 8) {
    g_err = "attn_merge_proj_ln: weight plane stride must be a multiple of 8 elements";
    return -1;
  }
  const float* part_o = ws;
  const float* part_ml = ws + size_t(waves) * 2 * QPG * HD * 32;
  const unsigned pin = nos_pin_mask();
  const int tiles = (B * T + BM - 1) / BM;
  // the f32-reciprocal divisions hold while every numerator of the unit bookkeeping is < 2^23
  const long long NK = (T + 31) / 32, QG = (NK + QPG - 1) / QPG, U = (long long)B * H * QG * NK;
  const bool wide = (U + 1) * (waves + 8) >= (1ll << 23) || (long long)B * T >= (1ll << 23);
  auto kern = wide ? attn_merge_proj_ln<384, true> : attn_merge_proj_ln<384, false>;
  hipLaunchKernelGGL(kern, dim3(pinned_grid(tiles, pin)), dim3(512), 0,
                     reinterpret_cast<hipStream_t>(stream), part_o, part_ml, o_direct, B, T, H, waves,
                     reinterpret_cast<const __bf16*>(w3), w_plane, bias, res, ln_w, ln_b, eps, xout,
                     reinterpret_cast<__bf16*>(yp), pin, g_ablate);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string("attn_merge_proj_ln: ") + hipGetErrorString(e);
    return int(e);
  }
  return 0;
}

}  // extern "C"
