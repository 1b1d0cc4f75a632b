// nos fp32 GEMM for gfx950 with fused epilogues: C = A · W^T (+ bias) (+ GELU | + residual).
//
// The YOLOS-small layer's four GEMMs (M = 3401 tokens; N x K = 1152x384, 384x384, 1536x384,
// 384x1536) are small enough that on a whole MI355X the library's tile choice leaves most of the
// 1024 SIMDs idle (81-324 tiles of 128x128 for 512 workgroup slots), and the fc1/fc2 epilogues
// (bias + exact GELU, bias + residual) cost a second pass over a 21 MB activation. This kernel:
//
//  * runs on the exact-fp32 matrix cores (v_mfma_f32_32x32x2_f32); four waves in a 2x2 grid, each
//    owning a WM x WN sub-tile (1-4 32x32 accumulators), BK = 32 or 64 per stage;
//  * permutes the K index inside a stage (k = BK/2*half + step) so every lane's operand fragment is
//    BK/2 contiguous floats: ds_read_b128 runs instead of scalar reads;
//  * stages A and W tiles through LDS with a BK+4-float row stride: a 16-lane ds_read_b128 group
//    reads rows i..i+15 at slot ((BK+4)/4*i + c) mod 16, a bijection, so reads are conflict-free;
//    stores are 8-lane 128-B runs (conflict-free for ds_write_b128);
//  * double-buffers LDS with the next stage's global loads held in registers across the MFMAs, one
//    barrier per stage;
//  * maps workgroups to tiles XCD-major (hardware round-robins workgroups over the 8 XCDs), so each
//    XCD's 4 MB L2 sees a contiguous band of row panels;
//  * fuses bias, exact-erf GELU and the residual add into the store (each lane stores 32 consecutive
//    columns of a row pair per accumulator register: 128-B coalesced);
//  * is instantiated for four tile shapes; the host picks the one that fills the calling slice
//    (ops/gemm.py autotunes per (M, N, K, slice CUs) outside graph capture).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <string>

typedef __attribute__((ext_vector_type(16))) float f32x16;

namespace {
thread_local std::string g_err;

constexpr int KALIGN = 32;  // K must be a multiple of this (the smallest stage depth)

enum : int { EPI_NONE = 0, EPI_BIAS = 1, EPI_GELU = 2, EPI_RES = 4, EPI_RES2 = 8 };

__device__ __forceinline__ int acc_row(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }

__device__ __forceinline__ int xcd_major(int phys, int n) {
  return (n % 8 == 0) ? (phys % 8) * (n / 8) + phys / 8 : phys;
}

// stage of BK k-values: a row segment is BK/4 float4; LDS row stride BK+4 floats keeps the
// (row * stride / 4) mod 16 slot map a bijection over 16 consecutive rows (stride/4 odd)
template <int BK>
struct Stage {
  static constexpr int C4 = BK / 4;        // float4 per row segment
  static constexpr int LSTR = BK + 4;      // LDS row stride (floats)
};

template <int BK, int AV, int BV>
__device__ __forceinline__ void stage_fetch(float4 (&pa)[AV], float4 (&pb)[BV], const float* __restrict__ A,
                                            const float* __restrict__ W, int m0, int n0, int M, int K, int k0,
                                            int tid) {
  constexpr int C4 = Stage<BK>::C4;
#pragma unroll
  for (int v = 0; v < AV; ++v) {
    const int f = tid + 256 * v, row = f / C4, c4 = f % C4;
    const int gr = min(m0 + row, M - 1);
    pa[v] = *reinterpret_cast<const float4*>(A + size_t(gr) * K + k0 + 4 * c4);
  }
#pragma unroll
  for (int v = 0; v < BV; ++v) {
    const int f = tid + 256 * v, row = f / C4, c4 = f % C4;
    pb[v] = *reinterpret_cast<const float4*>(W + size_t(n0 + row) * K + k0 + 4 * c4);
  }
}

template <int BK, int AV, int BV>
__device__ __forceinline__ void stage_stash(const float4 (&pa)[AV], const float4 (&pb)[BV], float* as, float* bs,
                                            int tid) {
  constexpr int C4 = Stage<BK>::C4, LSTR = Stage<BK>::LSTR;
#pragma unroll
  for (int v = 0; v < AV; ++v) {
    const int f = tid + 256 * v, row = f / C4, c4 = f % C4;
    *reinterpret_cast<float4*>(&as[row * LSTR + 4 * c4]) = pa[v];
  }
#pragma unroll
  for (int v = 0; v < BV; ++v) {
    const int f = tid + 256 * v, row = f / C4, c4 = f % C4;
    *reinterpret_cast<float4*>(&bs[row * LSTR + 4 * c4]) = pb[v];
  }
}

template <int WM, int WN, int BK, int NBUF>
__global__ __launch_bounds__(256, 2) void gemm_f32(const float* __restrict__ A, const float* __restrict__ W,
                                                  const float* __restrict__ bias, const float* __restrict__ R,
                                                  const float* __restrict__ R2, int r2_rows, float* __restrict__ C,
                                                  int M, int N, int K, int epi) {
  constexpr int BM = 2 * WM, BN = 2 * WN;
  constexpr int TM = WM / 32, TN = WN / 32;          // 32x32 accumulators per wave
  constexpr int AV = BM * BK / 4 / 256;               // float4 per thread per stage (A)
  constexpr int BV = BN * BK / 4 / 256;               // (W)
  constexpr int LSTR = Stage<BK>::LSTR;
  constexpr int KS = BK / 2;                          // MFMA k-steps per stage
  // NBUF = 2: double-buffered stages, one barrier per stage; NBUF = 1: half the LDS (twice the
  // resident workgroups per CU) for a second barrier per stage
  __shared__ __attribute__((aligned(16))) float As[NBUF][BM * LSTR];
  __shared__ __attribute__((aligned(16))) float Bs[NBUF][BN * LSTR];

  const int tiles_n = N / BN;
  const int tiles = ((M + BM - 1) / BM) * tiles_n;
  const int t = xcd_major(blockIdx.x, gridDim.x);
  if (t >= tiles) return;
  const int tm = t / tiles_n, tn = t % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int j = lane & 31, hf = lane >> 5;

  // cooperative stage loads: float4 f = tid + 256*v -> row f/8, k offset 4*(f%8)
  float4 pa[AV], pb[BV];
  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x16{0};

  const int nk = K / BK;
  stage_fetch<BK, AV, BV>(pa, pb, A, W, m0, n0, M, K, 0, tid);
  stage_stash<BK, AV, BV>(pa, pb, As[0], Bs[0], tid);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = NBUF == 2 ? (ks & 1) : 0;
    // unconditional prefetch (the last stage re-reads itself) keeps pa/pb in registers: a
    // conditional update makes the compiler demote them to scratch
    stage_fetch<BK, AV, BV>(pa, pb, A, W, m0, n0, M, K, min(ks + 1, nk - 1) * BK, tid);
    float af[TM][KS], bf[TN][KS];
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const float* p = &As[buf][(wm * WM + 32 * a + j) * LSTR + KS * hf];
#pragma unroll
      for (int q = 0; q < KS / 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(p + 4 * q);
        af[a][4 * q + 0] = v.x;
        af[a][4 * q + 1] = v.y;
        af[a][4 * q + 2] = v.z;
        af[a][4 * q + 3] = v.w;
      }
    }
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const float* p = &Bs[buf][(wn * WN + 32 * b + j) * LSTR + KS * hf];
#pragma unroll
      for (int q = 0; q < KS / 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(p + 4 * q);
        bf[b][4 * q + 0] = v.x;
        bf[b][4 * q + 1] = v.y;
        bf[b][4 * q + 2] = v.z;
        bf[b][4 * q + 3] = v.w;
      }
    }
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][s], bf[b][s], acc[a][b], 0, 0, 0);
    if constexpr (NBUF == 1) {
      // every wave has its fragments (own LDS reads drained) before anyone overwrites the buffer;
      // a raw barrier: __syncthreads()'s fences here make the compiler demote pa/pb to scratch
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
    }
    stage_stash<BK, AV, BV>(pa, pb, As[NBUF == 2 ? (buf ^ 1) : 0], Bs[NBUF == 2 ? (buf ^ 1) : 0], tid);
    __syncthreads();
  }

  // epilogue: acc[a][b] register r is C[m0 + wm*WM + 32a + acc_row(r, hf)][n0 + wn*WN + 32b + j]
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int col = n0 + wn * WN + 32 * b + j;
    const float bv = (epi & EPI_BIAS) ? bias[col] : 0.f;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * WM + 32 * a + acc_row(r, hf);
        if (row >= M) continue;
        float v = acc[a][b][r] + bv;
        if (epi & EPI_GELU) v = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
        const size_t idx = size_t(row) * N + col;
        if (epi & EPI_RES) v += R[idx];
        if (epi & EPI_RES2) v += R2[size_t(row % r2_rows) * N + col];  // broadcast over batch
        C[idx] = v;
      }
    }
  }
}

template <int WM, int WN, int BK, int NBUF = 2>
int launch(const float* A, const float* W, const float* bias, const float* R, const float* R2, int r2_rows, float* C,
           int M, int N, int K, int epi, hipStream_t s) {
  constexpr int BM = 2 * WM, BN = 2 * WN;
  if (N % BN) {
    g_err = "gemm: N must be a multiple of the tile width " + std::to_string(BN);
    return -1;
  }
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  if (K % BK) {
    g_err = "gemm: K must be a multiple of the stage depth " + std::to_string(BK);
    return -1;
  }
  hipLaunchKernelGGL((gemm_f32<WM, WN, BK, NBUF>), dim3(tiles), dim3(256), 0, s, A, W, bias, R, R2, r2_rows, C, M, N, K, epi);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string("gemm_f32: ") + hipGetErrorString(e);
    return int(e);
  }
  return 0;
}
}  // namespace

extern "C" {

const char* nos_gemm_last_error() { return g_err.c_str(); }

// Tile configurations (BM x BN, stage depth BK): 0 = 64x64/32, 1 = 128x64/32, 2 = 64x128/32,
// 3 = 128x128/32, 4 = 64x64/64, 5 = 128x64/64, 6 = 64x128/64; single-buffered LDS:
// 7 = 64x64/32, 8 = 128x64/32, 9 = 64x128/32.
static const int kCfg[10][3] = {{64, 64, 32}, {128, 64, 32}, {64, 128, 32}, {128, 128, 32}, {64, 64, 64},
                                {128, 64, 64}, {64, 128, 64}, {64, 64, 32}, {128, 64, 32}, {64, 128, 32}};

int nos_gemm_num_configs() { return 10; }

int nos_gemm_tile(int cfg, int* bm, int* bn, int* bk) {
  if (cfg < 0 || cfg > 9) return -1;
  *bm = kCfg[cfg][0];
  *bn = kCfg[cfg][1];
  *bk = kCfg[cfg][2];
  return 0;
}

// C[M,N] = A[M,K] · W[N,K]^T, epilogue flags: 1 = + bias[N], 2 = exact GELU (after bias),
// 4 = + R[M,N] (after GELU), 8 = + R2[row % r2_rows, N] (a second residual broadcast over the
// batch, e.g. YOLOS's per-layer mid position embeddings). K % 32 == 0, N % BN == 0; row-major
// contiguous operands.
int nos_gemm_f32(const float* A, const float* W, const float* bias, const float* R, const float* R2, int r2_rows,
                 float* C, int M, int N, int K, int epi, int cfg, void* stream) {
  if (K % KALIGN) {
    g_err = "gemm: K must be a multiple of 32";
    return -1;
  }
  if (((epi & EPI_BIAS) && !bias) || ((epi & EPI_RES) && !R) || ((epi & EPI_RES2) && (!R2 || r2_rows <= 0))) {
    g_err = "gemm: epilogue operand missing";
    return -1;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (cfg) {
    case 0: return launch<32, 32, 32>(A, W, bias, R, R2, r2_rows, C, M, N, K, epi, s);
    case 1: return launch<64, 32, 32>(A, W, bias, R, R2, r2_rows, C, M, N, K, epi, s);
    case 2: return launch<32, 64, 32>(A, W, bias, R, R2, r2_rows, C, M, N, K, epi, s);
    case 3: return launch<64, 64, 32>(A, W, bias, R, R2, r2_rows, C, M, N, K, epi, s);
    case 4: return launch<32, 32, 64>(A, W, bias, R, R2, r2_rows, C, M, N, K, epi, s);
    case 5: return launch<64, 32, 64>(A, W, bias, R, R2, r2_rows, C, M, N, K, epi, s);
    case 6: return launch<32, 64, 64>(A, W, bias, R, R2, r2_rows, C, M, N, K, epi, s);
    case 7: return launch<32, 32, 32, 1>(A, W, bias, R, R2, r2_rows, C, M, N, K, epi, s);
    case 8: return launch<64, 32, 32, 1>(A, W, bias, R, R2, r2_rows, C, M, N, K, epi, s);
    case 9: return launch<32, 64, 32, 1>(A, W, bias, R, R2, r2_rows, C, M, N, K, epi, s);
    default:
      g_err = "gemm: unknown tile config";
      return -1;
  }
}

}  // extern "C"
