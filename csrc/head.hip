// Small-M fp32 kernels around the transformer blocks of the workload model (YOLOS-small, batch 1):
//
//  * small_linear_f32 — y = act(LN?(x) · W^T + b) for M <= a few hundred rows (the 100 detection
//    tokens), exact fp32 FMAs on the vector ALUs: the detection heads are six 100-row GEMMs whose
//    library launches cost ~7-23 us each at this size. Up to two independent GEMMs (the class and
//    box heads) run as the two z-slices of one launch, so the heads take three launches in all;
//    the first also applies the final LayerNorm to its staged rows (two-pass mean/variance of each
//    full row).
//  * patch_planes_f32 — the patch embedding's im2col and x3 split in one pass: pixels [B][C][H][W]
//    straight to the three bf16 planes of the [B*P, C*p*p] patch matrix (the MFMA GEMM's operand),
//    instead of a permute copy plus a split kernel and their round trip.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace {
thread_local std::string g_err;

// tile rows x columns; K <= KMAX. Row stride KS = KMAX + 4 floats: 16-byte aligned rows for
// ds_read_b128, and KS mod 64 = 4 puts the 16 column rows a ds_read_b128 lane group reads on 16
// distinct 4-bank slots (conflict-free)
constexpr int TM = 16, TN = 32, KMAX = 384, KS = KMAX + 4;

struct LinGroup {
  const float* x;  // [M][ldx]
  const float* w;  // [n][K]
  const float* b;  // [n] (may be null)
  float* y;        // [M][ldy]
  int ldx, ldy, n, act;  // act: 0 none, 1 ReLU, 2 sigmoid
};

struct LinArgs {
  LinGroup g[2];
  const float* ln_w;  // LayerNorm of x's rows (K = the full row) when non-null
  const float* ln_b;
  float eps;
  int M, K;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Tile (TM rows x TN columns) of group blockIdx.z; 256 threads: column tid % 32, rows 2*(tid / 32)
// and +1. The whole x tile (LayerNorm-ed) and W tile (K <= 384) are loaded into LDS in one round of
// 16-byte loads — one memory latency per launch instead of one per K chunk — then every FMA reads
// LDS (odd row stride: the 32 column reads of a wave hit 32 banks; the row reads broadcast).
__global__ __launch_bounds__(256) void small_linear_f32(LinArgs a) {
  const LinGroup& g = a.g[blockIdx.z];
  const int n0 = blockIdx.x * TN, m0 = blockIdx.y * TM;
  if (n0 >= g.n) return;
  __shared__ __attribute__((aligned(16))) float xs[TM * KS];
  __shared__ __attribute__((aligned(16))) float ws[TN * KS];
  __shared__ float s_mean[TM], s_rstd[TM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K = a.K, K4 = K / 4;
  // W tile rows n0.., x tile rows m0.. (clamped: out-of-range rows/columns are computed, never
  // stored): every 16-byte load is issued before the first LDS write, so the tile costs one latency
  constexpr int WV = TN * KMAX / 4 / 256, XV = TM * KMAX / 4 / 256;
  float4 wv[WV], xv[XV];
#pragma unroll
  for (int j = 0; j < WV; ++j) {
    const int i = tid + 256 * j;
    if (i < TN * K4) {
      const int c = i / K4, k = 4 * (i % K4), col = min(n0 + c, g.n - 1);
      wv[j] = *reinterpret_cast<const float4*>(g.w + size_t(col) * K + k);
    }
  }
#pragma unroll
  for (int j = 0; j < XV; ++j) {
    const int i = tid + 256 * j;
    if (i < TM * K4) {
      const int r = i / K4, k = 4 * (i % K4), row = min(m0 + r, a.M - 1);
      xv[j] = *reinterpret_cast<const float4*>(g.x + size_t(row) * g.ldx + k);
    }
  }
#pragma unroll
  for (int j = 0; j < WV; ++j) {
    const int i = tid + 256 * j;
    if (i < TN * K4) {
      float* d = ws + (i / K4) * KS + 4 * (i % K4);
      d[0] = wv[j].x, d[1] = wv[j].y, d[2] = wv[j].z, d[3] = wv[j].w;
    }
  }
#pragma unroll
  for (int j = 0; j < XV; ++j) {
    const int i = tid + 256 * j;
    if (i < TM * K4) {
      float* d = xs + (i / K4) * KS + 4 * (i % K4);
      d[0] = xv[j].x, d[1] = xv[j].y, d[2] = xv[j].z, d[3] = xv[j].w;
    }
  }
  __syncthreads();
  if (a.ln_w != nullptr) {  // two-pass statistics of the tile's rows (one wave per 4 rows), then normalise in place
    for (int r = wave; r < TM; r += 4) {
      const float* xr = xs + r * KS;
      float s = 0.f;
      for (int k = lane; k < K; k += 64) s += xr[k];
      const float mean = wave_sum(s) / K;
      float q = 0.f;
      for (int k = lane; k < K; k += 64) {
        const float d = xr[k] - mean;
        q += d * d;
      }
      const float var = wave_sum(q) / K;
      if (lane == 0) {
        s_mean[r] = mean;
        s_rstd[r] = rsqrtf(var + a.eps);
      }
    }
    __syncthreads();
    for (int i = tid; i < TM * K; i += 256) {
      const int r = i / K, k = i % K;
      xs[r * KS + k] = (xs[r * KS + k] - s_mean[r]) * s_rstd[r] * a.ln_w[k] + a.ln_b[k];
    }
    __syncthreads();
  }
  const int c = tid & 31, r2 = 2 * (tid >> 5);
  const float* wr = ws + c * KS;
  const float* x0 = xs + r2 * KS;
  const float* x1 = x0 + KS;
  float acc0 = 0.f, acc1 = 0.f;
  // 4 k per step: three ds_read_b128 for 8 FMAs (K % 4 == 0 is checked at launch); the FMA order
  // per output is k ascending, as before
#pragma unroll 4
  for (int k = 0; k < K; k += 4) {
    const float4 w4 = *reinterpret_cast<const float4*>(wr + k);
    const float4 a4 = *reinterpret_cast<const float4*>(x0 + k);
    const float4 b4 = *reinterpret_cast<const float4*>(x1 + k);
    acc0 = fmaf(a4.x, w4.x, acc0);
    acc1 = fmaf(b4.x, w4.x, acc1);
    acc0 = fmaf(a4.y, w4.y, acc0);
    acc1 = fmaf(b4.y, w4.y, acc1);
    acc0 = fmaf(a4.z, w4.z, acc0);
    acc1 = fmaf(b4.z, w4.z, acc1);
    acc0 = fmaf(a4.w, w4.w, acc0);
    acc1 = fmaf(b4.w, w4.w, acc1);
  }
  const int col = n0 + c;
  if (col >= g.n) return;
  const float bv = g.b ? g.b[col] : 0.f;
  const float accs[2] = {acc0, acc1};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = m0 + r2 + i;
    if (row >= a.M) break;
    float v = accs[i] + bv;
    if (g.act == 1) v = fmaxf(v, 0.f);
    else if (g.act == 2) v = 1.f / (1.f + expf(-v));
    g.y[size_t(row) * g.ldy + col] = v;
  }
}

// pixels [B][C][H][W] -> planes [3][B*gh*gw][C*p*p]: row (b, i, j), column (c, u, v) =
// pixels[b][c][i*p + u][j*p + v]; each thread one 2-wide run of v (an image row of odd-multiple-of-2
// width, e.g. 1066, keeps only 8-byte alignment)
__global__ __launch_bounds__(256) void patch_planes_f32(const float* __restrict__ px, __bf16* __restrict__ out,
                                                        int B, int C, int H, int W, int p, int gh, int gw) {
  const int ck = C * p * p, q = p / 2;
  const size_t rows = size_t(B) * gh * gw, n2 = rows * ck / 2, plane = rows * ck;
  for (size_t t = size_t(blockIdx.x) * 256 + threadIdx.x; t < n2; t += size_t(gridDim.x) * 256) {
    const size_t row = t / (ck / 2);
    const int c2 = int(t % (ck / 2));
    const int c = c2 / (p * q), u = (c2 / q) % p, v = 2 * (c2 % q);
    const int b = int(row / (size_t(gh) * gw)), ij = int(row % (size_t(gh) * gw)), i = ij / gw, j = ij % gw;
    const float2 x = *reinterpret_cast<const float2*>(px + ((size_t(b) * C + c) * H + i * p + u) * W + j * p + v);
    const float in[2] = {x.x, x.y};
    __bf16 h[3][2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const __bf16 h0 = (__bf16)in[e];
      const float r1 = in[e] - (float)h0;
      const __bf16 h1 = (__bf16)r1;
      h[0][e] = h0;
      h[1][e] = h1;
      h[2][e] = (__bf16)(r1 - (float)h1);
    }
    const size_t o = row * ck + size_t(c2) * 2;
#pragma unroll
    for (int s = 0; s < 3; ++s)
      *reinterpret_cast<uint32_t*>(out + s * plane + o) = *reinterpret_cast<const uint32_t*>(h[s]);
  }
}

int check(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return int(e);
  }
  return 0;
}
}  // namespace

extern "C" {

const char* nos_head_last_error() { return g_err.c_str(); }

// One launch of up to two row-aligned fp32 GEMMs (M rows, K deep) with bias and activation;
// group g: x_g [M][ldx_g], w_g [n_g][K], b_g [n_g] or null, y_g [M][ldy_g], act_g (0/1 ReLU/2
// sigmoid). ln_w/ln_b non-null: x rows are LayerNorm-ed (over K) while staged.
int nos_small_linear_f32(int groups, const float* const* xs, const int* ldx, const float* const* ws,
                         const float* const* bs, float* const* ys, const int* ldy, const int* ns, const int* acts,
                         int M, int K, const float* ln_w, const float* ln_b, float eps, void* stream) {
  if (groups < 1 || groups > 2 || M <= 0 || K <= 0 || K > KMAX || K % 4) {
    g_err = "small_linear: 1-2 groups, M > 0, 0 < K <= 384, K % 4 == 0";
    return -1;
  }
  if ((ln_w == nullptr) != (ln_b == nullptr)) {
    g_err = "small_linear: LayerNorm needs weight and bias";
    return -1;
  }
  LinArgs a{};
  int maxn = 0;
  for (int i = 0; i < groups; ++i) {
    if (!xs[i] || !ws[i] || !ys[i] || ns[i] <= 0 || ldx[i] < K || ldx[i] % 4 || ldy[i] < ns[i] || acts[i] < 0 ||
        acts[i] > 2 || reinterpret_cast<uintptr_t>(xs[i]) % 16 || reinterpret_cast<uintptr_t>(ws[i]) % 16) {
      g_err = "small_linear: bad group operands";
      return -1;
    }
    a.g[i] = LinGroup{xs[i], ws[i], bs[i], ys[i], ldx[i], ldy[i], ns[i], acts[i]};
    maxn = ns[i] > maxn ? ns[i] : maxn;
  }
  a.ln_w = ln_w;
  a.ln_b = ln_b;
  a.eps = eps;
  a.M = M;
  a.K = K;
  hipLaunchKernelGGL(small_linear_f32, dim3((maxn + TN - 1) / TN, (M + TM - 1) / TM, groups), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  return check("small_linear_f32");
}

// pixels [B][C][H][W] fp32 (contiguous; H, W cropped to whole patches by the caller's gh, gw) ->
// x3 planes [3][B*gh*gw][C*p*p] bf16; p and W even
int nos_patch_planes_f32(const float* px, void* out, int B, int C, int H, int W, int p, int gh, int gw,
                         void* stream) {
  if (p % 2 || W % 2 || gh * p > H || gw * p > W || B <= 0 || C <= 0) {
    g_err = "patch_planes: even patch and image width, whole patches inside the image";
    return -1;
  }
  const size_t n2 = size_t(B) * gh * gw * C * p * p / 2;
  const int grid = int(n2 / 256 + 1 < 4096 ? n2 / 256 + 1 : 4096);
  hipLaunchKernelGGL(patch_planes_f32, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), px,
                     reinterpret_cast<__bf16*>(out), B, C, H, W, p, gh, gw);
  return check("patch_planes_f32");
}

}  // extern "C"
