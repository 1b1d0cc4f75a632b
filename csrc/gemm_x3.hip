// nos x3 GEMM for gfx950: fp32-accurate C = A · W^T on the bf16 matrix cores.
//
// Every fp32 operand arrives as three bf16 planes (x = x0 + x1 + x2 exactly; see kernels.hip
// "fp32 as three bf16 planes"): activations are split by their producer (LayerNorm, attention,
// the previous GEMM's epilogue), weights once at load time. Each 32x32x16 block is six
// v_mfma_f32_32x32x16_bf16 (a2b0, a1b1, a0b2, a1b0, a0b1, a0b0 — small terms first) = 192
// matrix-pipe cycles against 512 for the same block on v_mfma_f32_32x32x2_f32, with the dropped
// products (a1b2, a2b1, a2b2) at 2^-24 relative: fp32 accuracy at 2.67x the f32 MFMA rate.
//
//  * four waves in a 2x2 grid, each owning a WM x WN sub-tile (1-4 32x32 accumulators); stages of
//    BK = 32 (two MFMA k-steps) per plane;
//  * LDS images [plane][row][40] bf16: a lane's fragment A[row j][16s + 8h .. +7] is one
//    ds_read_b128; the 80-B row stride maps the rows of every ds_read_b128 lane group to distinct
//    16-B bank slots (5r mod 16 is a bijection), so reads are conflict-free;
//  * double-buffered (or single-buffered for twice the resident workgroups) with the next stage's
//    16-B global loads held in registers across the MFMAs; XCD-major tile order;
//  * fused epilogue: bias, exact GELU, residual, broadcast second residual; the result goes out
//    as fp32 and/or as three bf16 planes (split in registers) for the next x3 consumer.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <string>

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {
thread_local std::string g_err;

enum : int { EPI_NONE = 0, EPI_BIAS = 1, EPI_GELU = 2, EPI_RES = 4, EPI_RES2 = 8 };
constexpr int BK = 32, LSTR = 40;

__device__ __forceinline__ int acc_row(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }

__device__ __forceinline__ int xcd_major(int phys, int n) {
  return (n % 8 == 0) ? (phys % 8) * (n / 8) + phys / 8 : phys;
}

__device__ __forceinline__ f32x16 mfma_x3(const bf16x8& a0, const bf16x8& a1, const bf16x8& a2, const bf16x8& b0,
                                          const bf16x8& b1, const bf16x8& b2, f32x16 d) {
  d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, d, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, d, 0, 0, 0);
}

// rows x 32 bf16 per plane = rows*4 16-B chunks; chunk f = tid + 256*v -> row f/4, k offset 8*(f%4)
template <int ROWS>
struct Tile {
  static constexpr int V = ROWS * 4 / 256;  // chunks per thread per plane
};

template <int ROWS>
__device__ __forceinline__ void fetch(uint4 (&r)[3][Tile<ROWS>::V], const __bf16* __restrict__ X, size_t plane,
                                      int r0, int rmax, int K, int k0, int tid) {
#pragma unroll
  for (int v = 0; v < Tile<ROWS>::V; ++v) {
    const int f = tid + 256 * v, row = min(r0 + (f >> 2), rmax);
    const __bf16* p = X + size_t(row) * K + k0 + 8 * (f & 3);
#pragma unroll
    for (int q = 0; q < 3; ++q) r[q][v] = *reinterpret_cast<const uint4*>(p + q * plane);
  }
}

template <int ROWS>
__device__ __forceinline__ void stash(const uint4 (&r)[3][Tile<ROWS>::V], __bf16* s, int tid) {
#pragma unroll
  for (int v = 0; v < Tile<ROWS>::V; ++v) {
    const int f = tid + 256 * v;
#pragma unroll
    for (int q = 0; q < 3; ++q)
      *reinterpret_cast<uint4*>(s + q * ROWS * LSTR + (f >> 2) * LSTR + 8 * (f & 3)) = r[q][v];
  }
}

template <int WM, int WN, int NBUF>
__global__ __launch_bounds__(256, 2) void gemm_x3(const __bf16* __restrict__ A, size_t a_plane,
                                                 const __bf16* __restrict__ W, size_t w_plane,
                                                 const float* __restrict__ bias, const float* __restrict__ R,
                                                 const float* __restrict__ R2, int r2_rows, float* __restrict__ C,
                                                 __bf16* __restrict__ Cp, size_t c_plane, int M, int N, int K,
                                                 int epi) {
  constexpr int BM = 2 * WM, BN = 2 * WN;
  constexpr int TM = WM / 32, TN = WN / 32;
  __shared__ __attribute__((aligned(16))) __bf16 As[NBUF][3 * BM * LSTR];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[NBUF][3 * BN * LSTR];

  const int tiles_n = N / BN;
  const int tiles = ((M + BM - 1) / BM) * tiles_n;
  const int t = xcd_major(blockIdx.x, gridDim.x);
  if (t >= tiles) return;
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int j = lane & 31, hf = lane >> 5;

  uint4 pa[3][Tile<BM>::V], pb[3][Tile<BN>::V];
  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x16{0};

  const int nk = K / BK;
  fetch<BM>(pa, A, a_plane, m0, M - 1, K, 0, tid);
  fetch<BN>(pb, W, w_plane, n0, N - 1, K, 0, tid);
  stash<BM>(pa, As[0], tid);
  stash<BN>(pb, Bs[0], tid);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = NBUF == 2 ? (ks & 1) : 0;
    // unconditional prefetch (the last stage re-reads itself) keeps pa/pb in registers
    const int kn = min(ks + 1, nk - 1) * BK;
    fetch<BM>(pa, A, a_plane, m0, M - 1, K, kn, tid);
    fetch<BN>(pb, W, w_plane, n0, N - 1, K, kn, tid);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[TM][3], bfr[TN][3];
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int q = 0; q < 3; ++q)
          af[a][q] = *reinterpret_cast<const bf16x8*>(&As[buf][q * BM * LSTR + (wm * WM + 32 * a + j) * LSTR + 16 * s +
                                                               8 * hf]);
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int q = 0; q < 3; ++q)
          bfr[b][q] = *reinterpret_cast<const bf16x8*>(&Bs[buf][q * BN * LSTR + (wn * WN + 32 * b + j) * LSTR + 16 * s +
                                                                8 * hf]);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = mfma_x3(af[a][0], af[a][1], af[a][2], bfr[b][0], bfr[b][1], bfr[b][2], acc[a][b]);
    }
    if constexpr (NBUF == 1) {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): own fragment reads drained
      __builtin_amdgcn_s_barrier();
    }
    stash<BM>(pa, As[NBUF == 2 ? (buf ^ 1) : 0], tid);
    stash<BN>(pb, Bs[NBUF == 2 ? (buf ^ 1) : 0], tid);
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
        if (epi & EPI_RES2) v += R2[size_t(row % r2_rows) * N + col];
        if (C) C[idx] = v;
        if (Cp) {
          const __bf16 h0 = (__bf16)v;
          const float r1 = v - (float)h0;
          const __bf16 h1 = (__bf16)r1;
          Cp[idx] = h0;
          Cp[c_plane + idx] = h1;
          Cp[2 * c_plane + idx] = (__bf16)(r1 - (float)h1);
        }
      }
    }
  }
}

template <int WM, int WN, int NBUF>
int launch(const __bf16* A, size_t ap, const __bf16* W, size_t wp, const float* bias, const float* R, const float* R2,
           int r2_rows, float* C, __bf16* Cp, size_t cp, int M, int N, int K, int epi, hipStream_t s) {
  constexpr int BM = 2 * WM, BN = 2 * WN;
  if (N % BN) {
    g_err = "gemm_x3: N must be a multiple of the tile width " + std::to_string(BN);
    return -1;
  }
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  hipLaunchKernelGGL((gemm_x3<WM, WN, NBUF>), dim3(tiles), dim3(256), 0, s, A, ap, W, wp, bias, R, R2, r2_rows, C, Cp,
                     cp, M, N, K, epi);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string("gemm_x3: ") + hipGetErrorString(e);
    return int(e);
  }
  return 0;
}
}  // namespace

extern "C" {

const char* nos_gemm_x3_last_error() { return g_err.c_str(); }

// Tile configurations (BM x BN): 0 = 64x64, 1 = 128x64, 2 = 64x128, 3 = 128x128 (double-buffered
// LDS); 4 = 64x64, 5 = 128x64, 6 = 64x128 (single-buffered: half the LDS, more resident tiles).
static const int kCfgX3[7][3] = {{64, 64, 2}, {128, 64, 2}, {64, 128, 2}, {128, 128, 2},
                                 {64, 64, 1}, {128, 64, 1}, {64, 128, 1}};

int nos_gemm_x3_num_configs() { return 7; }

int nos_gemm_x3_tile(int cfg, int* bm, int* bn, int* nbuf) {
  if (cfg < 0 || cfg > 6) return -1;
  *bm = kCfgX3[cfg][0];
  *bn = kCfgX3[cfg][1];
  *nbuf = kCfgX3[cfg][2];
  return 0;
}

// C[M,N] = A[M,K] · W[N,K]^T with A and W as three bf16 planes (plane strides ap, wp elements,
// 16-B aligned), fused epilogue flags as nos_gemm_f32 (1 bias, 2 GELU, 4 + R, 8 + R2[row % r2_rows]).
// Output: fp32 C (may be null) and/or three bf16 planes Cp (plane stride cp; may be null).
// K % 32 == 0, N % BN == 0, row-major contiguous operands.
int nos_gemm_x3(const void* A, size_t ap, const void* W, size_t wp, const float* bias, const float* R,
                const float* R2, int r2_rows, float* C, void* Cp, size_t cp, int M, int N, int K, int epi, int cfg,
                void* stream) {
  if (K % BK || ap % 8 || wp % 8 || cp % 8) {
    g_err = "gemm_x3: K must be a multiple of 32 and plane strides multiples of 8 elements";
    return -1;
  }
  if (!C && !Cp) {
    g_err = "gemm_x3: no output";
    return -1;
  }
  if (((epi & EPI_BIAS) && !bias) || ((epi & EPI_RES) && !R) || ((epi & EPI_RES2) && (!R2 || r2_rows <= 0))) {
    g_err = "gemm_x3: epilogue operand missing";
    return -1;
  }
  const __bf16* a = reinterpret_cast<const __bf16*>(A);
  const __bf16* w = reinterpret_cast<const __bf16*>(W);
  __bf16* cpp = reinterpret_cast<__bf16*>(Cp);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (cfg) {
    case 0: return launch<32, 32, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 1: return launch<64, 32, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 2: return launch<32, 64, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 3: return launch<64, 64, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 4: return launch<32, 32, 1>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 5: return launch<64, 32, 1>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 6: return launch<32, 64, 1>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    default:
      g_err = "gemm_x3: unknown tile config";
      return -1;
  }
}

}  // extern "C"
