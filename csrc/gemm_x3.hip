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

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>

#include "epilogue.h"
#include "pin.h"
#include "streamk.h"

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {
thread_local std::string g_err;


enum : int { EPI_NONE = 0, EPI_BIAS = 1, EPI_GELU = 2, EPI_RES = 4, EPI_RES2 = 8 };
constexpr int BK = 32, LSTR = 40;

__device__ __forceinline__ int acc_row(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }

// Logical tile order: xcd_major_n (pin.h) deals workgroups round-robin over the XCDs (phys % nx =
// XCD, observed placement — speed only, never correctness), so XCD x gets a contiguous logical range:
// a band of whole tile rows whose A rows stay in that XCD's L2 while it sweeps the weight columns.

// Persistent grids: workgroup w's tiles are base + i*stride, i < count — the XCD's band again, dealt
// over the XCD's P/nx workgroups (nx XCDs: 8, or the pinned partition's; P % nx == 0, otherwise a
// plain w + i*P sweep).
__device__ __forceinline__ void xcd_band(int w, int P, int nx, int tiles, int& base, int& stride, int& count) {
  if (P % nx) {
    base = w, stride = P, count = w < tiles ? (tiles - w + P - 1) / P : 0;
    return;
  }
  const int x = w % nx, li = w / nx, px = P / nx, q = tiles / nx, r = tiles % nx;
  const int n = q + (x < r ? 1 : 0);
  base = x * q + min(x, r) + li, stride = px, count = li < n ? (n - li + px - 1) / px : 0;
}

// Grouped tile order: logical tile t walks GROUP tile rows down a column before moving right, so
// the tiles an XCD runs at once cover GROUP rows x (its workgroups / GROUP) columns — A and W
// slices that fit its 4 MB L2 together — instead of one row of tiles sweeping all of W. GROUP
// rides in bits 8-15 of the epilogue word (1 = plain row-major order).
__device__ __forceinline__ void tile_rc(int t, int tiles_m, int tiles_n, int group, int& mt, int& nt) {
  if (group <= 1) {
    mt = t / tiles_n, nt = t % tiles_n;
    return;
  }
  const int per = group * tiles_n, g = t / per, r0 = g * group, gs = min(tiles_m - r0, group), o = t - g * per;
  mt = r0 + o % gs, nt = o / gs;
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

template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void compute_stage(f32x16 (&acc)[WM / 32][WN / 32], const __bf16* __restrict__ as,
                                              const __bf16* __restrict__ bs, int wm, int wn, int j, int hf) {
  constexpr int TM = WM / 32, TN = WN / 32;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    bf16x8 af[TM][3], bfr[TN][3];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int q = 0; q < 3; ++q)
        af[a][q] = *reinterpret_cast<const bf16x8*>(&as[q * BM * LSTR + (wm * WM + 32 * a + j) * LSTR + 16 * s + 8 * hf]);
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int q = 0; q < 3; ++q)
        bfr[b][q] = *reinterpret_cast<const bf16x8*>(&bs[q * BN * LSTR + (wn * WN + 32 * b + j) * LSTR + 16 * s + 8 * hf]);
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
        acc[a][b] = mfma_x3(af[a][0], af[a][1], af[a][2], bfr[b][0], bfr[b][1], bfr[b][2], acc[a][b]);
  }
}

// two values of one column in adjacent rows (idx, idx + N): the plane split on packed pairs
__device__ __forceinline__ void store_pair(float v0, float v1, size_t idx, int N, float* __restrict__ C,
                                           __bf16* __restrict__ Cp, size_t c_plane) {
  if (C) C[idx] = v0, C[idx + N] = v1;
  if (Cp) {
    nos_bf2 pl[3];
    nos_split3_pair(nos_f2{v0, v1}, pl);
#pragma unroll
    for (int q = 0; q < 3; ++q) Cp[q * c_plane + idx] = pl[q].x, Cp[q * c_plane + idx + N] = pl[q].y;
  }
}

__device__ __forceinline__ void store_one(float v, size_t idx, float* __restrict__ C, __bf16* __restrict__ Cp,
                                          size_t c_plane) {
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

// Epilogue math of one 32x32 accumulator: bias, GELU, residuals (the API order). Operands are loaded for all 16
// rows at once, from clamped (always valid) rows: a per-element "if (row < M) load" becomes a
// branch and a vmcnt(0) per element (16 dependent memory round trips per accumulator).
__device__ __forceinline__ void epi_values(const f32x16& acc, float (&v)[16], int rb, int col, int hf, float bv,
                                           const float* __restrict__ R, const float* __restrict__ R2, int r2_rows,
                                           int M, int N, int epi) {
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = acc[r] + bv;
  if (epi & EPI_GELU) {
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const nos_f2 g = nos_gelu2(nos_f2{v[r], v[r + 1]});
      v[r] = g.x, v[r + 1] = g.y;
    }
  }
  if (epi & EPI_RES) {
    float rv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) rv[r] = R[size_t(min(rb + acc_row(r, hf), M - 1)) * N + col];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] += rv[r];
  }
  if (epi & EPI_RES2) {
    float rv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) rv[r] = R2[size_t(min(rb + acc_row(r, hf), M - 1) % r2_rows) * N + col];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] += rv[r];
  }
}

template <int TM, int TN>
__device__ __forceinline__ void store_tile(const f32x16 (&acc)[TM][TN], int r0, int c0, int j, int hf,
                                           const float* __restrict__ bias, const float* __restrict__ R,
                                           const float* __restrict__ R2, int r2_rows, float* __restrict__ C,
                                           __bf16* __restrict__ Cp, size_t c_plane, int M, int N, int epi) {
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int col = c0 + 32 * b + j;
    const float bv = (epi & EPI_BIAS) ? bias[col] : 0.f;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      float v[16];
      epi_values(acc[a][b], v, r0 + 32 * a, col, hf, bv, R, R2, r2_rows, M, N, epi);
      // full 32-row blocks (all but the last row of tiles) store without per-element predicates
      if (r0 + 32 * a + 32 <= M) {
        // registers r, r+1 (r even) are rows acc_row(r) and acc_row(r) + 1
#pragma unroll
        for (int r = 0; r < 16; r += 2)
          store_pair(v[r], v[r + 1], size_t(r0 + 32 * a + acc_row(r, hf)) * N + col, N, C, Cp, c_plane);
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = r0 + 32 * a + acc_row(r, hf);
          if (row < M) store_one(v[r], size_t(row) * N + col, C, Cp, c_plane);
        }
      }
    }
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
  constexpr int VA = Tile<BM>::V, VB = Tile<BN>::V;
  __shared__ __attribute__((aligned(16))) __bf16 As[NBUF][3 * BM * LSTR];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[NBUF][3 * BN * LSTR];

  const int group = (epi >> 8) & 0xff;
  const PinnedBlock pb = pinned_block(unsigned(epi >> 20) & 0xffu);
  epi &= 0xff;
  if (pb.id < 0) return;
  const int tiles_n = N / BN, tiles_m = (M + BM - 1) / BM;
  const int tiles = tiles_m * tiles_n;
  const int t = xcd_major_n(pb.id, pb.n, pb.nx);
  if (t >= tiles) return;
  int mt, nt;
  tile_rc(t, tiles_m, tiles_n, group, mt, nt);
  const int m0 = mt * BM, n0 = nt * BN;

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int j = lane & 31, hf = lane >> 5;

  uint4 pa0[3][VA], pb0[3][VB];
  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x16{0};

  const int nk = K / BK;
// past the end a load re-reads the last stage: loads stay unconditional, so the prefetch registers
// are never conditionally live (the compiler would demote them to scratch)
#define X3_LOAD(RA, RB, STAGE)                                           \
  {                                                                      \
    const int k0_ = min((STAGE), nk - 1) * BK;                           \
    fetch<BM>(RA, A, a_plane, m0, M - 1, K, k0_, tid);                   \
    fetch<BN>(RB, W, w_plane, n0, N - 1, K, k0_, tid);                   \
  }
#define X3_PUT(RA, RB, BUF)                                              \
  {                                                                      \
    if constexpr (NBUF == 1) {                                           \
      __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0) */               \
      __builtin_amdgcn_s_barrier();                                      \
    }                                                                    \
    stash<BM>(RA, As[BUF], tid);                                         \
    stash<BN>(RB, Bs[BUF], tid);                                         \
    __syncthreads();                                                     \
  }
// one stage ks: stage ks+1 is loaded into (NA, NB) across the MFMAs of stage ks, then stashed
#define X3_STEP(KS, NA, NB)                                              \
  {                                                                      \
    const int buf_ = NBUF == 2 ? ((KS) & 1) : 0;                         \
    X3_LOAD(NA, NB, (KS) + 1)                                            \
    compute_stage<BM, BN, WM, WN>(acc, As[buf_], Bs[buf_], wm, wn, j, hf); \
    X3_PUT(NA, NB, NBUF == 2 ? (buf_ ^ 1) : 0)                           \
  }

  X3_LOAD(pa0, pb0, 0)
  X3_PUT(pa0, pb0, 0)
  for (int ks = 0; ks < nk; ++ks) X3_STEP(ks, pa0, pb0)
#undef X3_STEP
#undef X3_PUT
#undef X3_LOAD

  // epilogue: acc[a][b] register r is C[m0 + wm*WM + 32a + acc_row(r, hf)][n0 + wn*WN + 32b + j]
  store_tile<TM, TN>(acc, m0 + wm * WM, n0 + wn * WN, j, hf, bias, R, R2, r2_rows, C, Cp, c_plane, M, N, epi);
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
  hipLaunchKernelGGL((gemm_x3<WM, WN, NBUF>), dim3(pinned_grid(tiles, unsigned(epi >> 20) & 0xffu)), dim3(256), 0, s, A, ap, W, wp, bias, R, R2, r2_rows, C, Cp,
                     cp, M, N, K, epi);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string("gemm_x3: ") + hipGetErrorString(e);
    return int(e);
  }
  return 0;
}

// Fused epilogue of a wave's TM x TN accumulators at rows r0.., columns c0..: register r of
// acc[a][b] is C[r0 + 32a + acc_row(r, hf)][c0 + 32b + j]; bias, exact GELU, residuals; fp32 and/or
// x3 planes out.
// ---- LDS-DMA variant ---------------------------------------------------------------------------
// Same math and epilogue; the operand tiles go global -> LDS with global_load_lds_dwordx4 (no
// register staging), S LDS buffers deep, so S-1 stages of loads are in flight behind the MFMAs at
// the cost of LDS only. The DMA writes a wave's 64 lanes x 16 B lane-linearly, so the image has
// unpadded 64-B rows [plane][row][4 chunks] and conflict-freedom comes from the lane -> chunk map
// instead: LDS slot c of row r holds k-chunk c ^ ((r >> 2) & 3); a fragment read of chunk 2s+h
// then lands, over any ds_read_b128 lane group, on 16 distinct 16-B bank slots (r mod 4 picks the
// 16-bank quarter, (r >> 2) & 3 the slot inside it). One raw s_barrier per stage: a
// __syncthreads() fence would wait for every outstanding DMA (vmcnt(0)) and serialise the pipeline;
// the per-wave "stage ks landed" wait is an explicit vmcnt(loads of the S-2 younger stages).
typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// Wait until this wave's DMA of the current stage has landed when `rem` younger stages (at most
// S-2) have been issued behind it: vmcnt needs an immediate, so the tail of the K loop (fewer
// younger stages in flight) takes the smaller waits by a wave-uniform branch.
template <int S, int NLD>
__device__ __forceinline__ void vm_wait_stage(int rem) {
  const int r = min(S - 2, rem);
  if constexpr (S > 3) {
    if (r >= 2) {
      vm_wait<2 * NLD>();
      return;
    }
  }
  if constexpr (S > 2) {
    if (r >= 1) {
      vm_wait<NLD>();
      return;
    }
  }
  vm_wait<0>();
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Stage depth BKS (32 or 64 bf16 per plane) sets the LDS row: CPR = BKS/8 16-byte chunks, so one
// wave DMA instruction (64 lanes x 16 B) covers RPI = 64/CPR rows. BKS = 64 reads whole 128-byte
// row segments: half the cache lines per byte moved of BKS = 32 (the texture-address path, not
// HBM, bounds these short-K GEMMs even when every line hits L2). Chunk c of local row r sits at
// slot c ^ swz(r), swz(r) = (r / (16/CPR)) % CPR, which makes the fragment reads (lanes j, j+32
// on rows j of a 32-row block) conflict-free for both depths.
template <int BKS, bool M16 = false>
__device__ __forceinline__ int dma_swz(int r) {
  if constexpr (M16) {
    // 16x16x32 fragment reads (lane l: row l%16, chunk l/16 of a 64-byte row): slot c ^ 2((r>>2)&1)
    // puts every ds_read_b128 lane group on 16 distinct 16-byte bank slots
    static_assert(BKS == 32, "the 16x16x32 image is defined for 32-deep stages");
    return ((r >> 2) & 1) << 1;
  } else {
    constexpr int CPR = BKS / 8;
    return (r / (16 / CPR)) % CPR;
  }
}

// Per-lane byte offsets of this wave's DMA rows inside one plane (fixed for the whole K loop):
// row groups g = wave + NW*i of RPI rows; lane -> row RPI*g + lane/CPR, chunk (lane%CPR) ^ swz(row).
template <int ROWS, int NW, int BKS = 32, bool M16 = false>
__device__ __forceinline__ void dma_offsets(uint32_t (&voff)[ROWS * BKS / 512 / NW], int r0, int rmax, int K,
                                            int wave, int lane) {
  constexpr int CPR = BKS / 8, RPI = 64 / CPR;
#pragma unroll
  for (int i = 0; i < ROWS / RPI / NW; ++i) {
    const int rl = RPI * (wave + NW * i) + lane / CPR;
    const int c = (lane % CPR) ^ dma_swz<BKS, M16>(rl);
    const int row = min(r0 + rl, rmax);
    voff[i] = uint32_t(row) * uint32_t(K) * 2u + 16u * uint32_t(c);
  }
}

// one stage of ROWS x BKS bf16 per plane for this wave (NW waves share the row groups): a wave-uniform base (plane, k0) plus the
// lane's fixed 32-bit offset, so the loads take the SGPR-base + VGPR-offset form and a stage costs
// no per-lane address arithmetic
template <int ROWS, int NW, int BKS = 32>
__device__ __forceinline__ void dma_stage(const __bf16* __restrict__ X, size_t plane,
                                          const uint32_t (&voff)[ROWS * BKS / 512 / NW], int k0, __bf16* lds,
                                          int wave) {
  constexpr int RPI = 512 / BKS;
#pragma unroll
  for (int i = 0; i < ROWS / RPI / NW; ++i) {
    const int g = wave + NW * i;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const char* src = reinterpret_cast<const char*>(X + q * plane + k0) + voff[i];
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(lds + q * ROWS * BKS + RPI * g * BKS), 16, 0, 0);
    }
  }
}

template <int BM, int BN, int WM, int WN, int BKS = 32>
__device__ __forceinline__ void compute_stage_sw(f32x16 (&acc)[WM / 32][WN / 32], const __bf16* __restrict__ as,
                                                 const __bf16* __restrict__ bs, int wm, int wn, int j, int hf) {
  constexpr int TM = WM / 32, TN = WN / 32;
  const int sw = dma_swz<BKS>(j);  // rows j and j + 32a share the swizzle
#pragma unroll
  for (int s = 0; s < BKS / 16; ++s) {
    const int ch = (2 * s + hf) ^ sw;
    bf16x8 af[TM][3], bfr[TN][3];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int q = 0; q < 3; ++q)
        af[a][q] = *reinterpret_cast<const bf16x8*>(&as[q * BM * BKS + (wm * WM + 32 * a + j) * BKS + 8 * ch]);
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int q = 0; q < 3; ++q)
        bfr[b][q] = *reinterpret_cast<const bf16x8*>(&bs[q * BN * BKS + (wn * WN + 32 * b + j) * BKS + 8 * ch]);
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
        acc[a][b] = mfma_x3(af[a][0], af[a][1], af[a][2], bfr[b][0], bfr[b][1], bfr[b][2], acc[a][b]);
  }
}

// ---- 16x16x32 variant --------------------------------------------------------------------------
// The same x3 product on v_mfma_f32_16x16x32_bf16: equal matrix-pipe cycles per FLOP, and on random
// data the smaller shape holds a higher clock when the whole chip is power-limited (the concurrent
// partitions of the bench). Fragment: lane l = row l%16, k 8(l/16)..+7 of a 32-deep stage; result:
// lane l = column l%16, rows 4(l/16)..+3 of a 16x16 block.
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ f32x4 mfma_x3_16(const bf16x8& a0, const bf16x8& a1, const bf16x8& a2, const bf16x8& b0,
                                            const bf16x8& b1, const bf16x8& b2, f32x4 d) {
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b0, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b2, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b0, d, 0, 0, 0);
  d = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b1, d, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, d, 0, 0, 0);
}

template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void compute_stage16(f32x4 (&acc)[WM / 16][WN / 16], const __bf16* __restrict__ as,
                                                const __bf16* __restrict__ bs, int wm, int wn, int lane) {
  constexpr int TM = WM / 16, TN = WN / 16;
  const int r16 = lane & 15;
  const int ch = (lane >> 4) ^ dma_swz<32, true>(r16);  // rows r16 + 16a share the swizzle
  bf16x8 af[TM][3], bfr[TN][3];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int q = 0; q < 3; ++q)
      af[a][q] = *reinterpret_cast<const bf16x8*>(&as[q * BM * 32 + (wm * WM + 16 * a + r16) * 32 + 8 * ch]);
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int q = 0; q < 3; ++q)
      bfr[b][q] = *reinterpret_cast<const bf16x8*>(&bs[q * BN * 32 + (wn * WN + 16 * b + r16) * 32 + 8 * ch]);
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
      acc[a][b] = mfma_x3_16(af[a][0], af[a][1], af[a][2], bfr[b][0], bfr[b][1], bfr[b][2], acc[a][b]);
}

template <int TM, int TN>
__device__ __forceinline__ void store_tile16(const f32x4 (&acc)[TM][TN], int r0, int c0, int lane,
                                             const float* __restrict__ bias, const float* __restrict__ R,
                                             const float* __restrict__ R2, int r2_rows, float* __restrict__ C,
                                             __bf16* __restrict__ Cp, size_t c_plane, int M, int N, int epi) {
  const int cl = lane & 15, rq = 4 * (lane >> 4);
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int col = c0 + 16 * b + cl;
    const float bv = (epi & EPI_BIAS) ? bias[col] : 0.f;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int rb = r0 + 16 * a + rq;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc[a][b][i] + bv;
      if (epi & EPI_GELU) {
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const nos_f2 g = nos_gelu2(nos_f2{v[i], v[i + 1]});
          v[i] = g.x, v[i + 1] = g.y;
        }
      }
      if (epi & EPI_RES) {
        float rv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) rv[i] = R[size_t(min(rb + i, M - 1)) * N + col];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] += rv[i];
      }
      if (epi & EPI_RES2) {
        float rv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) rv[i] = R2[size_t(min(rb + i, M - 1) % r2_rows) * N + col];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] += rv[i];
      }
      if (rb + 4 <= M) {
#pragma unroll
        for (int i = 0; i < 4; i += 2) store_pair(v[i], v[i + 1], size_t(rb + i) * N + col, N, C, Cp, c_plane);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (rb + i < M) store_one(v[i], size_t(rb + i) * N + col, C, Cp, c_plane);
      }
    }
  }
}

// BM x BN tile on a WGM x WGN grid of waves (4 or 8 waves: 8 gives each SIMD two waves of one
// workgroup, so a 128x128 tile — half the bytes per MFMA of 64x64 — still hides its load latency)
template <int BM, int BN, int WGM, int WGN, int S, int BKS = 32, bool M16 = false>
__global__ __launch_bounds__(64 * WGM * WGN, 1) void gemm_x3d(const __bf16* __restrict__ A, size_t a_plane,
                                                  const __bf16* __restrict__ W, size_t w_plane,
                                                  const float* __restrict__ bias, const float* __restrict__ R,
                                                  const float* __restrict__ R2, int r2_rows, float* __restrict__ C,
                                                  __bf16* __restrict__ Cp, size_t c_plane, int M, int N, int K,
                                                  int epi) {
  static_assert(S >= 2 && S <= 4, "2-4 LDS stages");
  constexpr int NW = WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int TM16 = WM / 16, TN16 = WN / 16;
  static_assert(!M16 || BKS == 32, "16x16x32 tiles use 32-deep stages");
  constexpr int RPI = 512 / BKS;  // rows per DMA instruction
  static_assert(BM % (RPI * NW) == 0 && BN % (RPI * NW) == 0, "row groups must divide over the waves");
  constexpr int NLD = 3 * (BM / RPI / NW) + 3 * (BN / RPI / NW);  // DMA instructions per wave per stage
  // one __shared__ object per stage buffer: the compiler's LDS-DMA wait tracking can then tell the
  // buffer being read from the buffers being filled (one array indexed by stage would make every
  // fragment read wait for ALL outstanding DMA, vmcnt(0), and serialise the pipeline)
  __shared__ __attribute__((aligned(16))) __bf16 A0[3 * BM * BKS], A1[3 * BM * BKS], A2[S > 2 ? 3 * BM * BKS : 8],
      A3[S > 3 ? 3 * BM * BKS : 8];
  __shared__ __attribute__((aligned(16))) __bf16 B0[3 * BN * BKS], B1[3 * BN * BKS], B2[S > 2 ? 3 * BN * BKS : 8],
      B3[S > 3 ? 3 * BN * BKS : 8];

  const int group = (epi >> 8) & 0xff, ablate = (epi >> 16) & 7, splits = 1 + ((epi >> 28) & 7);
  const PinnedBlock pb = pinned_block(unsigned(epi >> 20) & 0xffu);
  epi &= 0xff;
  if (pb.id < 0) return;
  const int tiles_n = N / BN, tiles_m = (M + BM - 1) / BM;
  const int tiles = tiles_m * tiles_n;
  // split-K partials (splits > 1): unit = (tile, split), a tile's splits adjacent (one XCD's L2);
  // split sp sums K stages [sp*nk/splits, (sp+1)*nk/splits) into fp32 plane sp of C [splits][M][N]
  // with no epilogue — the consumer (splitk_layernorm) adds the planes, bias and residuals
  const int u = xcd_major_n(pb.id, pb.n, pb.nx);
  if (u >= tiles * splits) return;
  const int t = u / splits, sp = u - t * splits;
  if (splits > 1) C += size_t(sp) * M * N;
  int mt, nt;
  tile_rc(t, tiles_m, tiles_n, group, mt, nt);
  const int m0 = mt * BM, n0 = nt * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS bases stay scalar
  const int wm = wave / WGN, wn = wave % WGN;
  const int j = lane & 31, hf = lane >> 5;

  f32x16 acc[M16 ? 1 : TM][M16 ? 1 : TN];
  f32x4 acc16[M16 ? TM16 : 1][M16 ? TN16 : 1];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[M16 ? 0 : a][M16 ? 0 : b] = f32x16{0};
#pragma unroll
  for (int a = 0; a < TM16; ++a)
#pragma unroll
    for (int b = 0; b < TN16; ++b) acc16[M16 ? a : 0][M16 ? b : 0] = f32x4{0};

  const int nk_all = K / BKS, kb = sp * nk_all / splits;
  const int nk = (sp + 1) * nk_all / splits - kb;
  uint32_t voff_a[BM / RPI / NW], voff_b[BN / RPI / NW];
  dma_offsets<BM, NW, BKS, M16>(voff_a, m0, M - 1, K, wave, lane);
  dma_offsets<BN, NW, BKS, M16>(voff_b, n0, N - 1, K, wave, lane);
#define X3D_A(b) ((b) == 0 ? A0 : (b) == 1 ? A1 : (b) == 2 ? A2 : A3)
#define X3D_COMPUTE(AS, BS)                                                        \
  {                                                                                \
    if constexpr (M16)                                                             \
      compute_stage16<BM, BN, WM, WN>(acc16, AS, BS, wm, wn, lane);                \
    else                                                                           \
      compute_stage_sw<BM, BN, WM, WN, BKS>(acc, AS, BS, wm, wn, j, hf);           \
  }
#define X3D_B(b) ((b) == 0 ? B0 : (b) == 1 ? B1 : (b) == 2 ? B2 : B3)
// No DMA is issued past the last stage, so when the loop ends no load can still be landing in a
// stage buffer (and no bandwidth goes to dead re-reads). The steady loop only runs while every
// issue is in range (static vmcnt, unconditional DMA); the last iterations run a tail with a
// bounds-checked issue and the smaller waits (vm_wait_stage).
#define X3D_ISSUE(STAGE, BUF)                                                      \
  {                                                                                \
    const int k0_ = (kb + (STAGE)) * BKS;                                          \
    if (!(ablate & 1)) dma_stage<BM, NW, BKS>(A, a_plane, voff_a, k0_, X3D_A(BUF), wave); \
    if (!(ablate & 2)) dma_stage<BN, NW, BKS>(W, w_plane, voff_b, k0_, X3D_B(BUF), wave); \
  }
#define X3D_ITER(KS, BUF)                                                          \
  {                                                                                \
    vm_wait<(S - 2) * NLD>(); /* this wave's DMA of stage KS has landed */         \
    raw_barrier();            /* everyone's has; stage KS-1's buffer is free */    \
    X3D_ISSUE((KS) + S - 1, ((BUF) + S - 1) % S)                                   \
    __builtin_amdgcn_sched_barrier(0); /* issue the DMA before the stage's MFMAs */ \
    X3D_COMPUTE(X3D_A(BUF), X3D_B(BUF))                                            \
  }
  for (int st = 0; st < S - 1; ++st)
    if (st < nk) X3D_ISSUE(st, st)
  int ks = 0;
  for (; ks + 2 * S - 1 <= nk; ks += S) {
    X3D_ITER(ks, 0)
    X3D_ITER(ks + 1, 1)
    if constexpr (S > 2) X3D_ITER(ks + 2, 2)
    if constexpr (S > 3) X3D_ITER(ks + 3, 3)
  }
  for (; ks < nk; ++ks) {
    const int buf = ks % S;
    vm_wait_stage<S, NLD>(nk - 1 - ks);
    raw_barrier();
    if (ks + S - 1 < nk) X3D_ISSUE(ks + S - 1, (buf + S - 1) % S)
    __builtin_amdgcn_sched_barrier(0);
    X3D_COMPUTE(X3D_A(buf), X3D_B(buf))
  }
#undef X3D_ITER
#undef X3D_COMPUTE
#undef X3D_ISSUE
#undef X3D_B
#undef X3D_A
  vm_wait<0>();  // no DMA may still target this workgroup's LDS when it retires
  // direct stores: each instruction writes whole 64/128-byte row segments of two rows. Wider
  // per-lane vectors were measured: through lane-quad DPP transposes slower; through a dedicated
  // wave-private LDS scratch (16-byte row chunks, 8x fewer store instructions for x3 planes)
  // correct run to run but no faster (qkv 27.6 vs 27.6 us, fc1 47.4 vs 46.3 on the whole GPU):
  // the plane bytes, not the instruction count, set the epilogue's time. (A scratch in the freed
  // stage buffers had given run-to-run differences with several workgroups per CU.)
  if constexpr (M16)
    store_tile16<TM16, TN16>(acc16, m0 + wm * WM, n0 + wn * WN, lane, bias, R, R2, r2_rows, C, Cp, c_plane, M, N,
                             epi);
  else
    if (!(ablate & 4))
      store_tile<TM, TN>(acc, m0 + wm * WM, n0 + wn * WN, j, hf, bias, R, R2, r2_rows, C, Cp, c_plane, M, N, epi);
}

template <int BM, int BN, int WGM, int WGN, int S, int BKS = 32, bool M16 = false>
int launch_d(const __bf16* A, size_t ap, const __bf16* W, size_t wp, const float* bias, const float* R,
             const float* R2, int r2_rows, float* C, __bf16* Cp, size_t cp, int M, int N, int K, int epi,
             hipStream_t s) {
  if (N % BN) {
    g_err = "gemm_x3: N must be a multiple of the tile width " + std::to_string(BN);
    return -1;
  }
  if (K % BKS) {
    g_err = "gemm_x3: K must be a multiple of the stage depth " + std::to_string(BKS);
    return -1;
  }
  const int tiles = ((M + BM - 1) / BM) * (N / BN) * (1 + ((epi >> 28) & 7));
  hipLaunchKernelGGL((gemm_x3d<BM, BN, WGM, WGN, S, BKS, M16>), dim3(pinned_grid(tiles, unsigned(epi >> 20) & 0xffu)),
                     dim3(64 * WGM * WGN), 0, s, A,
                     ap, W, wp, bias, R, R2, r2_rows, C, Cp, cp, M, N, K, epi);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string("gemm_x3d: ") + hipGetErrorString(e);
    return int(e);
  }
  return 0;
}

// Persistent (stream-of-stages) LDS-DMA GEMM: a grid of P workgroups, workgroup w owning tiles
// w, w+P, ...; its (tile, k-stage) pairs form one continuous stage stream, so the DMA ring keeps
// loading the next tile's first stages while the current tile's last MFMAs and its epilogue run —
// the fill/drain every short-K (K = 384: 12 stages) tile otherwise pays once per tile.
template <int BM, int BN, int WGM, int WGN, int S, int BKS = 32>
__global__ __launch_bounds__(64 * WGM * WGN, 1) void gemm_x3s(const __bf16* __restrict__ A, size_t a_plane,
                                                              const __bf16* __restrict__ W, size_t w_plane,
                                                              const float* __restrict__ bias,
                                                              const float* __restrict__ R,
                                                              const float* __restrict__ R2, int r2_rows,
                                                              float* __restrict__ C, __bf16* __restrict__ Cp,
                                                              size_t c_plane, int M, int N, int K, int epi) {
  static_assert(S >= 2 && S <= 4, "2-4 LDS stages");
  constexpr int NW = WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int RPI = 512 / BKS;
  static_assert(BM % (RPI * NW) == 0 && BN % (RPI * NW) == 0, "row groups must divide over the waves");
  constexpr int NLD = 3 * (BM / RPI / NW) + 3 * (BN / RPI / NW);
  __shared__ __attribute__((aligned(16))) __bf16 A0[3 * BM * BKS], A1[3 * BM * BKS],
      A2[S > 2 ? 3 * BM * BKS : 8], A3[S > 3 ? 3 * BM * BKS : 8];
  __shared__ __attribute__((aligned(16))) __bf16 B0[3 * BN * BKS], B1[3 * BN * BKS],
      B2[S > 2 ? 3 * BN * BKS : 8], B3[S > 3 ? 3 * BN * BKS : 8];

  const int group = (epi >> 8) & 0xff, ablate = (epi >> 16) & 7;
  const PinnedBlock pb = pinned_block(unsigned(epi >> 20) & 0xffu);
  epi &= 0xff;
  if (pb.id < 0) return;
  const int tiles_n = N / BN, tiles_m = (M + BM - 1) / BM;
  const int tiles = tiles_m * tiles_n;
  int tb, ts, tcount;
  xcd_band(pb.id, pb.n, pb.nx, tiles, tb, ts, tcount);
  if (tcount <= 0) return;
  const int nk = K / BKS;
  const int total = tcount * nk;  // this workgroup's stages

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int j = lane & 31, hf = lane >> 5;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x16{0};

#define X3S_A(b) ((b) == 0 ? A0 : (b) == 1 ? A1 : (b) == 2 ? A2 : A3)
#define X3S_B(b) ((b) == 0 ? B0 : (b) == 1 ? B1 : (b) == 2 ? B2 : B3)
// stage h of the stream (none past the end: steady loop + bounds-checked tail, as in gemm_x3d)
#define X3S_ISSUE(H, BUF)                                                                 \
  {                                                                                       \
    const int h_ = (H);                                                                   \
    const int ti_ = h_ / nk, ks_ = h_ - ti_ * nk, t_ = tb + ti_ * ts;                     \
    int mt_, nt_;                                                                         \
    tile_rc(t_, tiles_m, tiles_n, group, mt_, nt_);                                       \
    uint32_t va_[BM / RPI / NW], vb_[BN / RPI / NW];                                      \
    dma_offsets<BM, NW, BKS>(va_, mt_ * BM, M - 1, K, wave, lane);                        \
    dma_offsets<BN, NW, BKS>(vb_, nt_ * BN, N - 1, K, wave, lane);                        \
    if (!(ablate & 1)) dma_stage<BM, NW, BKS>(A, a_plane, va_, ks_ * BKS, X3S_A(BUF), wave); \
    if (!(ablate & 2)) dma_stage<BN, NW, BKS>(W, w_plane, vb_, ks_ * BKS, X3S_B(BUF), wave); \
  }
#define X3S_BODY(G, BUF)                                                                  \
  {                                                                                       \
    compute_stage_sw<BM, BN, WM, WN, BKS>(acc, X3S_A(BUF), X3S_B(BUF), wm, wn, j, hf);    \
    if (((G) + 1) % nk == 0) {                                                            \
      const int t_ = tb + ((G) / nk) * ts;                                                \
      int mt_, nt_;                                                                       \
      tile_rc(t_, tiles_m, tiles_n, group, mt_, nt_);                                     \
      if (!(ablate & 4)) store_tile<TM, TN>(acc, mt_ * BM + wm * WM, nt_ * BN + wn * WN, j, hf, bias, R, R2, \
                         r2_rows, C, Cp, c_plane, M, N, epi);                             \
      _Pragma("unroll") for (int a = 0; a < TM; ++a)                                      \
        _Pragma("unroll") for (int b = 0; b < TN; ++b) acc[a][b] = f32x16{0};             \
    }                                                                                     \
  }
#define X3S_ITER(G, BUF)                                                                  \
  {                                                                                       \
    vm_wait<(S - 2) * NLD>();                                                             \
    raw_barrier();                                                                        \
    X3S_ISSUE((G) + S - 1, ((BUF) + S - 1) % S)                                           \
    __builtin_amdgcn_sched_barrier(0); /* issue the DMA before the stage's MFMAs */         \
    X3S_BODY(G, BUF)                                                                      \
  }
  for (int st = 0; st < S - 1; ++st)
    if (st < total) X3S_ISSUE(st, st)
  int g = 0;
  for (; g + 2 * S - 1 <= total; g += S) {
    X3S_ITER(g, 0)
    X3S_ITER(g + 1, 1)
    if constexpr (S > 2) X3S_ITER(g + 2, 2)
    if constexpr (S > 3) X3S_ITER(g + 3, 3)
  }
  for (; g < total; ++g) {
    const int buf = g % S;
    vm_wait_stage<S, NLD>(total - 1 - g);
    raw_barrier();
    if (g + S - 1 < total) X3S_ISSUE(g + S - 1, (buf + S - 1) % S)
    __builtin_amdgcn_sched_barrier(0);
    X3S_BODY(g, buf)
  }
#undef X3S_BODY
#undef X3S_ITER
#undef X3S_ISSUE
#undef X3S_B
#undef X3S_A
  vm_wait<0>();
}

template <int BM, int BN, int WGM, int WGN, int S, int BKS = 32>
int launch_s(const __bf16* A, size_t ap, const __bf16* W, size_t wp, const float* bias, const float* R,
             const float* R2, int r2_rows, float* C, __bf16* Cp, size_t cp, int M, int N, int K, int epi, int grid,
             hipStream_t s) {
  if (N % BN) {
    g_err = "gemm_x3: N must be a multiple of the tile width " + std::to_string(BN);
    return -1;
  }
  if (K % BKS) {
    g_err = "gemm_x3s: K must be a multiple of the stage depth " + std::to_string(BKS);
    return -1;
  }
  const int tiles = ((M + BM - 1) / BM) * (N / BN);
  const int g = std::max(1, std::min(grid, tiles));
  hipLaunchKernelGGL((gemm_x3s<BM, BN, WGM, WGN, S, BKS>), dim3(pinned_grid(g, unsigned(epi >> 20) & 0xffu)),
                     dim3(64 * WGM * WGN), 0, s, A, ap, W, wp, bias, R, R2,
                     r2_rows, C, Cp, cp, M, N, K, epi);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string("gemm_x3s: ") + hipGetErrorString(e);
    return int(e);
  }
  return 0;
}

// ---- staggered 8-wave 16x16x32 tiles -----------------------------------------------------------
// Two waves share each SIMD in a 512-thread workgroup, and with one barrier per stage and the same
// program they run in lockstep: both issue their LDS fragment reads, wait on them and reach the
// barrier together, so neither covers the other's stall (MI355X_MICROARCH.md, "Two waves per SIMD",
// item 9). Here the second half of the workgroup (waves NW/2.., the SIMD partners of the first
// half) runs half a stage behind: in stage ks it finishes the second half of its accumulator rows
// for stage ks-1, then the first half for stage ks, so while one wave of a SIMD waits on its reads
// its partner is in the middle of its MFMAs. A stage buffer is therefore read one stage longer:
// three LDS buffers, one stage of DMA in flight (as the two-buffer tiles). Same math and epilogue
// as gemm_x3d<..., M16>; ``rows [R0, R1)`` of the wave's 16-row blocks per call.
template <int BM, int BN, int WM, int WN, int R0, int R1>
__device__ __forceinline__ void compute_rows16(f32x4 (&acc)[WM / 16][WN / 16], const __bf16* __restrict__ as,
                                               const __bf16* __restrict__ bs, int wm, int wn, int lane) {
  constexpr int TN = WN / 16;
  const int r16 = lane & 15;
  const int ch = (lane >> 4) ^ dma_swz<32, true>(r16);
  bf16x8 af[R1 - R0][3], bfr[TN][3];
#pragma unroll
  for (int a = R0; a < R1; ++a)
#pragma unroll
    for (int q = 0; q < 3; ++q)
      af[a - R0][q] = *reinterpret_cast<const bf16x8*>(&as[q * BM * 32 + (wm * WM + 16 * a + r16) * 32 + 8 * ch]);
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int q = 0; q < 3; ++q)
      bfr[b][q] = *reinterpret_cast<const bf16x8*>(&bs[q * BN * 32 + (wn * WN + 16 * b + r16) * 32 + 8 * ch]);
#pragma unroll
  for (int a = R0; a < R1; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
      acc[a][b] = mfma_x3_16(af[a - R0][0], af[a - R0][1], af[a - R0][2], bfr[b][0], bfr[b][1], bfr[b][2], acc[a][b]);
}

template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN, 1) void gemm_x3t(const __bf16* __restrict__ A, size_t a_plane,
                                                              const __bf16* __restrict__ W, size_t w_plane,
                                                              const float* __restrict__ bias,
                                                              const float* __restrict__ R,
                                                              const float* __restrict__ R2, int r2_rows,
                                                              float* __restrict__ C, __bf16* __restrict__ Cp,
                                                              size_t c_plane, int M, int N, int K, int epi) {
  constexpr int NW = WGM * WGN, BKS = 32, RPI = 16;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM16 = WM / 16, TN16 = WN / 16, HM = TM16 / 2;
  static_assert(NW == 8 && TM16 % 2 == 0, "8 waves, an even number of 16-row blocks per wave");
  static_assert(BM % (RPI * NW) == 0 && BN % (RPI * NW) == 0, "row groups must divide over the waves");
  __shared__ __attribute__((aligned(16))) __bf16 A0[3 * BM * BKS], A1[3 * BM * BKS], A2[3 * BM * BKS];
  __shared__ __attribute__((aligned(16))) __bf16 B0[3 * BN * BKS], B1[3 * BN * BKS], B2[3 * BN * BKS];

  const int group = (epi >> 8) & 0xff, ablate = (epi >> 16) & 7, splits = 1 + ((epi >> 28) & 7);
  const PinnedBlock pb = pinned_block(unsigned(epi >> 20) & 0xffu);
  epi &= 0xff;
  if (pb.id < 0) return;
  const int tiles_n = N / BN, tiles_m = (M + BM - 1) / BM;
  const int tiles = tiles_m * tiles_n;
  const int u = xcd_major_n(pb.id, pb.n, pb.nx);
  if (u >= tiles * splits) return;
  const int t = u / splits, sp = u - t * splits;
  if (splits > 1) C += size_t(sp) * M * N;
  int mt, nt;
  tile_rc(t, tiles_m, tiles_n, group, mt, nt);
  const int m0 = mt * BM, n0 = nt * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const bool lag = wave >= NW / 2;  // wave-uniform

  f32x4 acc[TM16][TN16];
#pragma unroll
  for (int a = 0; a < TM16; ++a)
#pragma unroll
    for (int b = 0; b < TN16; ++b) acc[a][b] = f32x4{0};

  const int nk_all = K / BKS, kb = sp * nk_all / splits;
  const int nk = (sp + 1) * nk_all / splits - kb;
  uint32_t voff_a[BM / RPI / NW], voff_b[BN / RPI / NW];
  dma_offsets<BM, NW, BKS, true>(voff_a, m0, M - 1, K, wave, lane);
  dma_offsets<BN, NW, BKS, true>(voff_b, n0, N - 1, K, wave, lane);
#define X3T_A(b) ((b) == 0 ? A0 : (b) == 1 ? A1 : A2)
#define X3T_B(b) ((b) == 0 ? B0 : (b) == 1 ? B1 : B2)
#define X3T_ISSUE(STAGE, BUF)                                                      \
  {                                                                                \
    const int k0_ = (kb + (STAGE)) * BKS;                                          \
    if (!(ablate & 1)) dma_stage<BM, NW, BKS>(A, a_plane, voff_a, k0_, X3T_A(BUF), wave); \
    if (!(ablate & 2)) dma_stage<BN, NW, BKS>(W, w_plane, voff_b, k0_, X3T_B(BUF), wave); \
  }
// stage KS in buffer BUF (= KS % 3): every wave's DMA of it has landed after the wait + barrier, and
// every wave is done with buffer (KS+1) % 3 (read last in stage KS-1 by the lagging half), which
// stage KS+1 then fills
#define X3T_ITER(KS, BUF)                                                          \
  {                                                                                \
    vm_wait<0>();                                                                  \
    raw_barrier();                                                                 \
    if ((KS) + 1 < nk) X3T_ISSUE((KS) + 1, ((BUF) + 1) % 3)                        \
    __builtin_amdgcn_sched_barrier(0);                                             \
    if (!lag) {                                                                    \
      compute_rows16<BM, BN, WM, WN, 0, TM16>(acc, X3T_A(BUF), X3T_B(BUF), wm, wn, lane); \
    } else {                                                                       \
      if ((KS) > 0)                                                                \
        compute_rows16<BM, BN, WM, WN, HM, TM16>(acc, X3T_A(((BUF) + 2) % 3), X3T_B(((BUF) + 2) % 3), wm, wn, lane); \
      compute_rows16<BM, BN, WM, WN, 0, HM>(acc, X3T_A(BUF), X3T_B(BUF), wm, wn, lane); \
    }                                                                              \
  }
  if (nk > 0) X3T_ISSUE(0, 0)
  for (int ks = 0; ks < nk; ks += 3) {
    X3T_ITER(ks, 0)
    if (ks + 1 < nk) X3T_ITER(ks + 1, 1)
    if (ks + 2 < nk) X3T_ITER(ks + 2, 2)
  }
  // the lagging half's last half-stage: no DMA is issued any more, so its buffer is still intact
  if (lag && nk > 0) {
    const int last = (nk - 1) % 3;
    if (last == 0)
      compute_rows16<BM, BN, WM, WN, HM, TM16>(acc, A0, B0, wm, wn, lane);
    else if (last == 1)
      compute_rows16<BM, BN, WM, WN, HM, TM16>(acc, A1, B1, wm, wn, lane);
    else
      compute_rows16<BM, BN, WM, WN, HM, TM16>(acc, A2, B2, wm, wn, lane);
  }
#undef X3T_ITER
#undef X3T_ISSUE
#undef X3T_B
#undef X3T_A
  vm_wait<0>();
  if (!(ablate & 4))
    store_tile16<TM16, TN16>(acc, m0 + wm * WM, n0 + wn * WN, lane, bias, R, R2, r2_rows, C, Cp, c_plane, M, N, epi);
}

template <int BM, int BN, int WGM, int WGN>
int launch_t(const __bf16* A, size_t ap, const __bf16* W, size_t wp, const float* bias, const float* R,
             const float* R2, int r2_rows, float* C, __bf16* Cp, size_t cp, int M, int N, int K, int epi,
             hipStream_t s) {
  if (N % BN || K % 32) {
    g_err = "gemm_x3t: N % " + std::to_string(BN) + " and K % 32 must be 0";
    return -1;
  }
  const int tiles = ((M + BM - 1) / BM) * (N / BN) * (1 + ((epi >> 28) & 7));
  hipLaunchKernelGGL((gemm_x3t<BM, BN, WGM, WGN>), dim3(pinned_grid(tiles, unsigned(epi >> 20) & 0xffu)),
                     dim3(64 * WGM * WGN), 0, s, A, ap, W, wp, bias, R, R2, r2_rows, C, Cp, cp, M, N, K, epi);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string("gemm_x3t: ") + hipGetErrorString(e);
    return int(e);
  }
  return 0;
}

// ---- fp32 A operand, split in the kernel -------------------------------------------------------
// The x3 GEMMs are bound by the latency of their operand stream (profiles/pmc_r4_gemm_spx.json:
// waves wait 40-49% of their cycles, the matrix pipe is 16-26% busy). Three bf16 planes are 6 B per
// element where fp32 is 4: here the activation operand arrives as fp32 rows and each thread splits
// its 8-value chunk into the three planes in registers (round to nearest even, the same split the
// producers use, so the planes — and the result — are bit-identical to the planes-in kernel) and
// stores them into the swizzled LDS image the 16x16x32 fragment reads expect. The weight planes
// still come by LDS-DMA. Register-staged A: the next stage's loads are issued before the MFMAs and
// stashed after them, one stage in flight, as the two-buffer tiles.
__device__ __forceinline__ void split3_8(const float4& lo, const float4& hi, bf16x8& a, bf16x8& b, bf16x8& c) {
  typedef float f32x8_t __attribute__((ext_vector_type(8)));
  const f32x8_t x = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  a = __builtin_convertvector(x, bf16x8);
  const f32x8_t r = x - __builtin_convertvector(a, f32x8_t);
  b = __builtin_convertvector(r, bf16x8);
  c = __builtin_convertvector(r - __builtin_convertvector(b, f32x8_t), bf16x8);
}

template <int BM, int BN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN, 1) void gemm_x3a(const float* __restrict__ A,
                                                              const __bf16* __restrict__ W, size_t w_plane,
                                                              const float* __restrict__ bias,
                                                              const float* __restrict__ R,
                                                              const float* __restrict__ R2, int r2_rows,
                                                              float* __restrict__ C, __bf16* __restrict__ Cp,
                                                              size_t c_plane, int M, int N, int K, int epi) {
  constexpr int NW = WGM * WGN, BKS = 32, RPI = 16;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM16 = WM / 16, TN16 = WN / 16;
  constexpr int AC = BM * 4 / (64 * NW);  // 16-B chunks (8 k-values) of the A stage per thread
  static_assert(AC >= 1 && BM * 4 % (64 * NW) == 0, "A stage chunks must divide over the threads");
  static_assert(BN % (RPI * NW) == 0, "row groups must divide over the waves");
  __shared__ __attribute__((aligned(16))) __bf16 A0[3 * BM * BKS], A1[3 * BM * BKS];
  __shared__ __attribute__((aligned(16))) __bf16 B0[3 * BN * BKS], B1[3 * BN * BKS];

  const int group = (epi >> 8) & 0xff, ablate = (epi >> 16) & 7, splits = 1 + ((epi >> 28) & 7);
  const PinnedBlock pb = pinned_block(unsigned(epi >> 20) & 0xffu);
  epi &= 0xff;
  if (pb.id < 0) return;
  const int tiles_n = N / BN, tiles_m = (M + BM - 1) / BM;
  const int tiles = tiles_m * tiles_n;
  const int u = xcd_major_n(pb.id, pb.n, pb.nx);
  if (u >= tiles * splits) return;
  const int t = u / splits, sp = u - t * splits;
  if (splits > 1) C += size_t(sp) * M * N;
  int mt, nt;
  tile_rc(t, tiles_m, tiles_n, group, mt, nt);
  const int m0 = mt * BM, n0 = nt * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;

  f32x4 acc[TM16][TN16];
#pragma unroll
  for (int a = 0; a < TM16; ++a)
#pragma unroll
    for (int b = 0; b < TN16; ++b) acc[a][b] = f32x4{0};

  const int nk_all = K / BKS, kb = sp * nk_all / splits;
  const int nk = (sp + 1) * nk_all / splits - kb;
  uint32_t voff_b[BN / RPI / NW];
  dma_offsets<BN, NW, BKS, true>(voff_b, n0, N - 1, K, wave, lane);
  // this thread's A chunks: chunk f = tid + 64*NW*v -> local row f/4, k-chunk f%4; LDS slot
  // (f%4) ^ swz(row), the layout the DMA writes for the 16x16x32 fragment reads
  const float* ap[AC];
  int aoff[AC];
#pragma unroll
  for (int v = 0; v < AC; ++v) {
    const int f = tid + 64 * NW * v, rl = f >> 2, c = f & 3;
    ap[v] = A + size_t(min(m0 + rl, M - 1)) * K + 8 * c;
    aoff[v] = rl * BKS + 8 * (c ^ dma_swz<32, true>(rl));
  }
  float4 ra[AC][2];
#define X3A_A(b) ((b) == 0 ? A0 : A1)
#define X3A_B(b) ((b) == 0 ? B0 : B1)
#define X3A_LOAD(STAGE)                                                                 \
  {                                                                                     \
    const int k0_ = (kb + (STAGE)) * BKS;                                               \
    if (!(ablate & 2)) dma_stage<BN, NW, BKS>(W, w_plane, voff_b, k0_, X3A_B((STAGE) & 1), wave); \
    _Pragma("unroll") for (int v = 0; v < AC; ++v) {                                    \
      ra[v][0] = *reinterpret_cast<const float4*>(ap[v] + k0_);                         \
      ra[v][1] = *reinterpret_cast<const float4*>(ap[v] + k0_ + 4);                     \
    }                                                                                   \
  }
#define X3A_STASH(BUF)                                                                  \
  {                                                                                     \
    __bf16* as_ = X3A_A(BUF);                                                           \
    _Pragma("unroll") for (int v = 0; v < AC; ++v) {                                    \
      bf16x8 h0, h1, h2;                                                                \
      split3_8(ra[v][0], ra[v][1], h0, h1, h2);                                         \
      *reinterpret_cast<bf16x8*>(as_ + aoff[v]) = h0;                                   \
      *reinterpret_cast<bf16x8*>(as_ + BM * BKS + aoff[v]) = h1;                        \
      *reinterpret_cast<bf16x8*>(as_ + 2 * BM * BKS + aoff[v]) = h2;                    \
    }                                                                                   \
  }
// stage KS in buffer BUF: the barrier publishes every thread's A stash and B DMA of it and frees
// buffer BUF^1 (read in stage KS-1), which stage KS+1 then fills: B by DMA, A loaded into
// registers now and stashed after this stage's MFMAs
#define X3A_ITER(KS, BUF)                                                               \
  {                                                                                     \
    vm_wait<0>();                                                                       \
    raw_barrier();                                                                      \
    const bool next_ = (KS) + 1 < nk;                                                   \
    if (next_) X3A_LOAD((KS) + 1)                                                       \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    compute_rows16<BM, BN, WM, WN, 0, TM16>(acc, X3A_A(BUF), X3A_B(BUF), wm, wn, lane); \
    if (next_) {                                                                        \
      vm_wait<0>();                                                                     \
      X3A_STASH((BUF) ^ 1)                                                              \
    }                                                                                   \
  }
  if (nk > 0) {
    X3A_LOAD(0)
    vm_wait<0>();
    X3A_STASH(0)
  }
  for (int ks = 0; ks < nk; ks += 2) {
    X3A_ITER(ks, 0)
    if (ks + 1 < nk) X3A_ITER(ks + 1, 1)
  }
#undef X3A_ITER
#undef X3A_STASH
#undef X3A_LOAD
#undef X3A_B
#undef X3A_A
  vm_wait<0>();
  if (!(ablate & 4))
    store_tile16<TM16, TN16>(acc, m0 + wm * WM, n0 + wn * WN, lane, bias, R, R2, r2_rows, C, Cp, c_plane, M, N, epi);
}

template <int BM, int BN, int WGM, int WGN>
int launch_a(const float* A, const __bf16* W, size_t wp, const float* bias, const float* R, const float* R2,
             int r2_rows, float* C, __bf16* Cp, size_t cp, int M, int N, int K, int epi, hipStream_t s) {
  if (N % BN || K % 32) {
    g_err = "gemm_x3a: N % " + std::to_string(BN) + " and K % 32 must be 0";
    return -1;
  }
  const int tiles = ((M + BM - 1) / BM) * (N / BN) * (1 + ((epi >> 28) & 7));
  hipLaunchKernelGGL((gemm_x3a<BM, BN, WGM, WGN>), dim3(pinned_grid(tiles, unsigned(epi >> 20) & 0xffu)),
                     dim3(64 * WGM * WGN), 0, s, A, W, wp, bias, R, R2, r2_rows, C, Cp, cp, M, N, K, epi);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string("gemm_x3a: ") + hipGetErrorString(e);
    return int(e);
  }
  return 0;
}

// ---- stream-K partials -------------------------------------------------------------------------
// The N = 384 GEMMs of the model (projection, fc2) have 162 tiles of 128x64 for 256 CUs: whole-tile
// grids leave a third of the chip idle (or a 27%-full second round), and split-K only moves the
// ragged edge. Here the P workgroups split the tiles' K stages evenly (streamk.h): each runs one
// continuous stage stream as gemm_x3s does (the DMA ring crosses tile boundaries), and at the end
// of every tile segment stores its raw accumulators to fp32 partial plane `segment` — no epilogue;
// the consumer (splitk_layernorm_f32 with the same SkMap) adds a tile's planes in order, then bias,
// residuals and the LayerNorm. The kernel boundary is the hand-off between workgroups (no flags).
template <int BM, int BN, int WGM, int WGN, int S, int BKS = 32>
__global__ __launch_bounds__(64 * WGM * WGN, 1) void gemm_x3k(const __bf16* __restrict__ A, size_t a_plane,
                                                              const __bf16* __restrict__ W, size_t w_plane,
                                                              float* __restrict__ C, int M, int N, int K, int P,
                                                              int ctl) {
  static_assert(S >= 2 && S <= 4, "2-4 LDS stages");
  constexpr int NW = WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int RPI = 512 / BKS;
  static_assert(BM % (RPI * NW) == 0 && BN % (RPI * NW) == 0, "row groups must divide over the waves");
  constexpr int NLD = 3 * (BM / RPI / NW) + 3 * (BN / RPI / NW);
  __shared__ __attribute__((aligned(16))) __bf16 A0[3 * BM * BKS], A1[3 * BM * BKS],
      A2[S > 2 ? 3 * BM * BKS : 8], A3[S > 3 ? 3 * BM * BKS : 8];
  __shared__ __attribute__((aligned(16))) __bf16 B0[3 * BN * BKS], B1[3 * BN * BKS],
      B2[S > 2 ? 3 * BN * BKS : 8], B3[S > 3 ? 3 * BN * BKS : 8];

  const int ablate = (ctl >> 16) & 7;
  const PinnedBlock pb = pinned_block(unsigned(ctl >> 20) & 0xffu);
  if (pb.id < 0) return;
  const int tiles_n = N / BN, tiles_m = (M + BM - 1) / BM;
  const int nk = K / BKS, U = tiles_m * tiles_n * nk;
  // logical workgroup: XCD x runs a contiguous band of ranges, so the workgroups sharing a tile
  // (neighbouring ranges) mostly share an L2 too
  const int w = xcd_major_n(pb.id, pb.n, pb.nx);
  if (w >= P) return;
  const int u0 = sk_first(w, P, U), total = sk_first(w + 1, P, U) - u0;
  const size_t plane = size_t(M) * N;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int j = lane & 31, hf = lane >> 5;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = f32x16{0};

#define X3K_A(b) ((b) == 0 ? A0 : (b) == 1 ? A1 : (b) == 2 ? A2 : A3)
#define X3K_B(b) ((b) == 0 ? B0 : (b) == 1 ? B1 : (b) == 2 ? B2 : B3)
#define X3K_ISSUE(H, BUF)                                                                 \
  {                                                                                       \
    const int u_ = u0 + (H), t_ = u_ / nk, ks_ = u_ - t_ * nk;                            \
    const int mt_ = t_ / tiles_n, nt_ = t_ - mt_ * tiles_n;                               \
    uint32_t va_[BM / RPI / NW], vb_[BN / RPI / NW];                                      \
    dma_offsets<BM, NW, BKS>(va_, mt_ * BM, M - 1, K, wave, lane);                        \
    dma_offsets<BN, NW, BKS>(vb_, nt_ * BN, N - 1, K, wave, lane);                        \
    if (!(ablate & 1)) dma_stage<BM, NW, BKS>(A, a_plane, va_, ks_ * BKS, X3K_A(BUF), wave); \
    if (!(ablate & 2)) dma_stage<BN, NW, BKS>(W, w_plane, vb_, ks_ * BKS, X3K_B(BUF), wave); \
  }
// a segment ends at its tile's last stage or at the end of this workgroup's range
#define X3K_BODY(G, BUF)                                                                  \
  {                                                                                       \
    compute_stage_sw<BM, BN, WM, WN, BKS>(acc, X3K_A(BUF), X3K_B(BUF), wm, wn, j, hf);    \
    const int u_ = u0 + (G), t_ = u_ / nk;                                                \
    if (u_ - t_ * nk == nk - 1 || (G) == total - 1) {                                     \
      const int seg_ = w - sk_owner(t_ * nk, P, U), mt_ = t_ / tiles_n, nt_ = t_ - mt_ * tiles_n; \
      if (!(ablate & 4)) store_tile<TM, TN>(acc, mt_ * BM + wm * WM, nt_ * BN + wn * WN, j, hf, nullptr, nullptr, \
                         nullptr, 0, C + size_t(seg_) * plane, nullptr, 0, M, N, 0);      \
      _Pragma("unroll") for (int a = 0; a < TM; ++a)                                      \
        _Pragma("unroll") for (int b = 0; b < TN; ++b) acc[a][b] = f32x16{0};             \
    }                                                                                     \
  }
#define X3K_ITER(G, BUF)                                                                  \
  {                                                                                       \
    vm_wait<(S - 2) * NLD>();                                                             \
    raw_barrier();                                                                        \
    X3K_ISSUE((G) + S - 1, ((BUF) + S - 1) % S)                                           \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    X3K_BODY(G, BUF)                                                                      \
  }
  for (int st = 0; st < S - 1; ++st)
    if (st < total) X3K_ISSUE(st, st)
  int g = 0;
  for (; g + 2 * S - 1 <= total; g += S) {
    X3K_ITER(g, 0)
    X3K_ITER(g + 1, 1)
    if constexpr (S > 2) X3K_ITER(g + 2, 2)
    if constexpr (S > 3) X3K_ITER(g + 3, 3)
  }
  for (; g < total; ++g) {
    const int buf = g % S;
    vm_wait_stage<S, NLD>(total - 1 - g);
    raw_barrier();
    if (g + S - 1 < total) X3K_ISSUE(g + S - 1, (buf + S - 1) % S)
    __builtin_amdgcn_sched_barrier(0);
    X3K_BODY(g, buf)
  }
#undef X3K_BODY
#undef X3K_ITER
#undef X3K_ISSUE
#undef X3K_B
#undef X3K_A
  vm_wait<0>();
}

// tile shape of stream-K config cfg (see nos_gemm_x3_streamk)
constexpr int kSkCfg[6][2] = {{64, 64}, {128, 64}, {64, 128}, {128, 64}, {64, 64}, {128, 128}};

template <int BM, int BN, int WGM, int WGN, int S, int BKS = 32>
int launch_k(const __bf16* A, size_t ap, const __bf16* W, size_t wp, float* C, int M, int N, int K, int P, int ctl,
             hipStream_t s) {
  if (N % BN || K % BKS) {
    g_err = "gemm_x3k: N % " + std::to_string(BN) + " and K % " + std::to_string(BKS) + " must be 0";
    return -1;
  }
  hipLaunchKernelGGL((gemm_x3k<BM, BN, WGM, WGN, S, BKS>), dim3(pinned_grid(P, unsigned(ctl >> 20) & 0xffu)),
                     dim3(64 * WGM * WGN), 0, s, A, ap, W, wp, C, M, N, K, P, ctl);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string("gemm_x3k: ") + hipGetErrorString(e);
    return int(e);
  }
  return 0;
}
}  // namespace

static int g_group_m = 1;
static int g_ablate = 0;  // timing studies only: 1 = skip the A operand loads, 2 = skip W (results invalid)

extern "C" {

const char* nos_gemm_x3_last_error() { return g_err.c_str(); }

int nos_gemm_x3_set_ablate(int a) {
  g_ablate = a & 7;
  return 0;
}

// grouped tile order (tile rows per group, 1..255; 1 = row-major): see tile_rc
int nos_gemm_x3_set_group(int g) {
  if (g < 1 || g > 255) {
    g_err = "gemm_x3: group must be 1..255";
    return -1;
  }
  g_group_m = g;
  return 0;
}

// Tile configurations (BM x BN, LDS buffers, load stages in flight): 0 = 64x64, 1 = 128x64,
// 2 = 64x128, 3 = 128x128 (double-buffered LDS); 4 = 64x64, 5 = 128x64, 6 = 64x128 (single-buffered:
// half the LDS, more resident tiles); 7-12 = LDS-DMA pipeline with nbuf = S stages (S-1 in
// flight): 64x64 S3/S4, 128x64 S3, 64x128 S3, 128x128 S3, 64x64 S2; 13/14 = 128x128 on 8 waves
// S3/S2; 15-17 = 2-wave 32x64 S3/S2, 64x32 S2; 18-22 = 64-deep stages (128-byte row segments):
// 64x64 S2/S3, 64x32 S2, 32x64 S2, 64x32 S3; 23/24 = 64-deep on 8 waves: 128x64 S2, 64x128 S2;
// 25/26 = 128x64 S4, 64x128 S4 (three stages in flight); 27-31 = v_mfma 16x16x32: 64x64 S2,
// 64x64 S3, 128x128 S2 (8 waves), 32x64 S2 (2 waves), 64x32 S2 (2 waves); 32-34 = 96/192-wide
// tiles (three 32-column blocks per wave), so N = 384 / 1536 split into 216 tiles at M = 3401 — one
// round on 256 CUs instead of 1.3-2.5: 128x192 S2, 64x96 S2 (2 waves), 64x192 S2 (2 waves);
// 35-37 = 8 waves of 64x64 each (a third fewer LDS fragment bytes per MFMA than 64x32 waves;
// 144 KB of LDS for two stages): 256x128 S2, 256x128 S2 on 16x16x32, 128x256 S2;
// 38 = the staggered 8-wave 16x16x32 128x128 tile (gemm_x3t, three LDS buffers).
static const int kCfgX3[39][3] = {{64, 64, 2}, {128, 64, 2}, {64, 128, 2}, {128, 128, 2},
                                  {64, 64, 1}, {128, 64, 1}, {64, 128, 1},
                                  {64, 64, 3}, {64, 64, 4}, {128, 64, 3}, {64, 128, 3},
                                  {128, 128, 3}, {64, 64, 2}, {128, 128, 3}, {128, 128, 2},
                                  {32, 64, 3}, {32, 64, 2}, {64, 32, 2},
                                  {64, 64, 2}, {64, 64, 3}, {64, 32, 2}, {32, 64, 2}, {64, 32, 3},
                                  {128, 64, 2}, {64, 128, 2}, {128, 64, 4}, {64, 128, 4},
                                  {64, 64, 2}, {64, 64, 3}, {128, 128, 2}, {32, 64, 2}, {64, 32, 2},
                                  {128, 192, 2}, {64, 96, 2}, {64, 192, 2},
                                  {256, 128, 2}, {256, 128, 2}, {128, 256, 2},
                                  {128, 128, 3}};

}  // extern "C"

static int dispatch(const __bf16* a, size_t ap, const __bf16* w, size_t wp, const float* bias, const float* R,
                    const float* R2, int r2_rows, float* C, __bf16* cpp, size_t cp, int M, int N, int K, int epi,
                    int cfg, hipStream_t s) {
  switch (cfg) {
    case 0: return launch<32, 32, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 1: return launch<64, 32, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 2: return launch<32, 64, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 3: return launch<64, 64, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 4: return launch<32, 32, 1>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 5: return launch<64, 32, 1>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 6: return launch<32, 64, 1>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 7: return launch_d<64, 64, 2, 2, 3>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 8: return launch_d<64, 64, 2, 2, 4>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 9: return launch_d<128, 64, 2, 2, 3>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 10: return launch_d<64, 128, 2, 2, 3>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 11: return launch_d<128, 128, 2, 2, 3>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 12: return launch_d<64, 64, 2, 2, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 13: return launch_d<128, 128, 2, 4, 3>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 14: return launch_d<128, 128, 2, 4, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 15: return launch_d<32, 64, 1, 2, 3>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 16: return launch_d<32, 64, 1, 2, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 17: return launch_d<64, 32, 2, 1, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 18: return launch_d<64, 64, 2, 2, 2, 64>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 19: return launch_d<64, 64, 2, 2, 3, 64>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 20: return launch_d<64, 32, 2, 1, 2, 64>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 21: return launch_d<32, 64, 1, 2, 2, 64>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 22: return launch_d<64, 32, 2, 1, 3, 64>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 23: return launch_d<128, 64, 4, 2, 2, 64>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 24: return launch_d<64, 128, 2, 4, 2, 64>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 25: return launch_d<128, 64, 2, 2, 4>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 26: return launch_d<64, 128, 2, 2, 4>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 27: return launch_d<64, 64, 2, 2, 2, 32, true>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 28: return launch_d<64, 64, 2, 2, 3, 32, true>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 29: return launch_d<128, 128, 2, 4, 2, 32, true>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 30: return launch_d<32, 64, 1, 2, 2, 32, true>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 31: return launch_d<64, 32, 2, 1, 2, 32, true>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 32: return launch_d<128, 192, 2, 2, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 33: return launch_d<64, 96, 2, 1, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 34: return launch_d<64, 192, 1, 2, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 35: return launch_d<256, 128, 4, 2, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 36: return launch_d<256, 128, 4, 2, 2, 32, true>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi,
                                                         s);
    case 37: return launch_d<128, 256, 2, 4, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 38: return launch_t<128, 128, 2, 4>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    default:
      g_err = "gemm_x3: unknown tile config";
      return -1;
  }
}

extern "C" {

int nos_gemm_x3_num_configs() { return 39; }

// Persistent stream-of-stages GEMM (same operands/epilogue as nos_gemm_x3) with an explicit grid
// (workgroups; the caller sizes it to the slice: CUs x resident workgroups per CU).
// cfg: 0 = 64x64 S3 (4 waves), 1 = 64x64 S2, 2 = 128x128 S3 (8 waves), 3 = 64x128 S3, 4 = 128x64 S3;
// 64-deep stages: 5 = 64x64 S2, 6 = 64x32 S2 (2 waves), 7 = 128x64 S2 (8 waves); 8/9 = 128x64, 64x128 S4;
// 10 = 256x128 S2 (8 waves of 64x64).
int nos_gemm_x3_persistent(const void* A, size_t ap, const void* W, size_t wp, const float* bias, const float* R,
                           const float* R2, int r2_rows, float* C, void* Cp, size_t cp, int M, int N, int K, int epi,
                           int cfg, int grid, void* stream) {
  if (K % BK || ap % 8 || wp % 8 || cp % 8 || (!C && !Cp)) {
    g_err = "gemm_x3s: K % 32 (K % 64 for 64-deep stages), plane strides % 8, and an output are required";
    return -1;
  }
  if (((epi & EPI_BIAS) && !bias) || ((epi & EPI_RES) && !R) || ((epi & EPI_RES2) && (!R2 || r2_rows <= 0))) {
    g_err = "gemm_x3s: epilogue operand missing";
    return -1;
  }
  const __bf16* a = reinterpret_cast<const __bf16*>(A);
  const __bf16* w = reinterpret_cast<const __bf16*>(W);
  __bf16* cpp = reinterpret_cast<__bf16*>(Cp);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  epi |= (g_group_m << 8) | (g_ablate << 16) | int(nos_pin_mask() << 20);
  switch (cfg) {
    case 0: return launch_s<64, 64, 2, 2, 3>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, grid, s);
    case 1: return launch_s<64, 64, 2, 2, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, grid, s);
    case 2: return launch_s<128, 128, 2, 4, 3>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, grid, s);
    case 3: return launch_s<64, 128, 2, 2, 3>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, grid, s);
    case 4: return launch_s<128, 64, 2, 2, 3>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, grid, s);
    case 5: return launch_s<64, 64, 2, 2, 2, 64>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, grid, s);
    case 6: return launch_s<64, 32, 2, 1, 2, 64>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, grid, s);
    case 7: return launch_s<128, 64, 4, 2, 2, 64>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, grid, s);
    case 8: return launch_s<128, 64, 2, 2, 4>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, grid, s);
    case 9: return launch_s<64, 128, 2, 2, 4>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, grid, s);
    case 10: return launch_s<256, 128, 4, 2, 2>(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, grid, s);
    default:
      g_err = "gemm_x3s: unknown config";
      return -1;
  }
}

// Split-K partial sums of C = A · W^T (LDS-DMA configs 7..38): plane s of C [splits][M][N] fp32
// holds the K stages [s*nk/splits, (s+1)*nk/splits); no epilogue (the consumer adds the planes in
// order, then bias and residuals: splitk_layernorm in kernels.hip). 2 <= splits <= min(8, K/stage).
int nos_gemm_x3_partials(const void* A, size_t ap, const void* W, size_t wp, float* C, int M, int N, int K, int cfg,
                         int splits, void* stream) {
  if (K % BK || ap % 8 || wp % 8 || !C) {
    g_err = "gemm_x3 partials: K % 32, plane strides % 8 and an output";
    return -1;
  }
  if (cfg < 7 || cfg > 38 || splits < 2 || splits > 8 || splits > K / BK) {
    g_err = "gemm_x3 partials: an LDS-DMA config (7..38) and 2..8 splits";
    return -1;
  }
  const int epi = (g_group_m << 8) | (g_ablate << 16) | int(nos_pin_mask() << 20) | ((splits - 1) << 28);
  return dispatch(reinterpret_cast<const __bf16*>(A), ap, reinterpret_cast<const __bf16*>(W), wp, nullptr, nullptr,
                  nullptr, 0, C, nullptr, 0, M, N, K, epi, cfg, reinterpret_cast<hipStream_t>(stream));
}

// Stream-K configs: 0 = 64x64 S3 (4 waves), 1 = 128x64 S2 64-deep (8 waves), 2 = 64x128 S2 64-deep
// (8 waves), 3 = 128x64 S3 (4 waves), 4 = 64x64 S2 64-deep (4 waves), 5 = 128x128 S3 (8 waves).
static int sk_bks(int cfg) { return (cfg == 1 || cfg == 2 || cfg == 4) ? 64 : 32; }

// The work split a stream-K launch of `P` workgroups uses (P clamped to the unit count):
// out = {P, U, nk, bm, bn, tiles_n, planes}; planes = the most segments any tile has, the depth
// of the fp32 partial buffer [planes][M][N] the launch writes.
int nos_gemm_x3_streamk_map(int M, int N, int K, int cfg, int P, int* out) {
  if (cfg < 0 || cfg > 5 || M <= 0 || P <= 0) {
    g_err = "gemm_x3k: config 0..5, M > 0 and P > 0";
    return -1;
  }
  const int bm = kSkCfg[cfg][0], bn = kSkCfg[cfg][1], bks = sk_bks(cfg);
  if (N % bn || K % bks) {
    g_err = "gemm_x3k: N % " + std::to_string(bn) + " and K % " + std::to_string(bks) + " must be 0";
    return -1;
  }
  SkMap m{0, 0, K / bks, bm, bn, N / bn};
  const long long tiles = (long long)((M + bm - 1) / bm) * m.tiles_n;
  if (tiles * m.nk > (1LL << 30) / 4096) {
    g_err = "gemm_x3k: too many units";
    return -1;
  }
  m.U = int(tiles * m.nk);
  m.P = std::min(P, m.U);
  int planes = 1;
  for (int t = 0; t < int(tiles); ++t) planes = std::max(planes, sk_segments(t, m));
  const int v[7] = {m.P, m.U, m.nk, bm, bn, m.tiles_n, planes};
  for (int i = 0; i < 7; ++i) out[i] = v[i];
  return 0;
}

// Raw partial sums of C = A · W^T, stream-K over P workgroups (P from nos_gemm_x3_streamk_map):
// C is the [planes][M][N] fp32 buffer; no epilogue (splitk_layernorm with the same map adds them).
int nos_gemm_x3_streamk(const void* A, size_t ap, const void* W, size_t wp, float* C, int M, int N, int K, int cfg,
                        int P, void* stream) {
  int m[7];
  if (nos_gemm_x3_streamk_map(M, N, K, cfg, P, m) != 0) return -1;
  if (m[0] != P || ap % 8 || wp % 8 || !C) {
    g_err = "gemm_x3k: P must be the map's (clamped) P; plane strides % 8; an output";
    return -1;
  }
  const __bf16* a = reinterpret_cast<const __bf16*>(A);
  const __bf16* w = reinterpret_cast<const __bf16*>(W);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int ctl = (g_ablate << 16) | int(nos_pin_mask() << 20);
  switch (cfg) {
    case 0: return launch_k<64, 64, 2, 2, 3>(a, ap, w, wp, C, M, N, K, P, ctl, s);
    case 1: return launch_k<128, 64, 4, 2, 2, 64>(a, ap, w, wp, C, M, N, K, P, ctl, s);
    case 2: return launch_k<64, 128, 2, 4, 2, 64>(a, ap, w, wp, C, M, N, K, P, ctl, s);
    case 3: return launch_k<128, 64, 2, 2, 3>(a, ap, w, wp, C, M, N, K, P, ctl, s);
    case 4: return launch_k<64, 64, 2, 2, 2, 64>(a, ap, w, wp, C, M, N, K, P, ctl, s);
    default: return launch_k<128, 128, 2, 4, 3>(a, ap, w, wp, C, M, N, K, P, ctl, s);
  }
}

// C = A · W^T with A as fp32 rows [M][K] (split into planes in the kernel) and W as three bf16
// planes; epilogue and outputs as nos_gemm_x3. cfg: 0 = 128x128 (8 waves, 16x16x32), 1 = 256x128.
int nos_gemm_x3_f32a(const float* A, const void* W, size_t wp, const float* bias, const float* R, const float* R2,
                     int r2_rows, float* C, void* Cp, size_t cp, int M, int N, int K, int epi, int cfg,
                     void* stream) {
  if (!A || K % 32 || wp % 8 || cp % 8 || (!C && !Cp)) {
    g_err = "gemm_x3a: an fp32 A, K % 32, plane strides % 8 and an output are required";
    return -1;
  }
  if (((epi & EPI_BIAS) && !bias) || ((epi & EPI_RES) && !R) || ((epi & EPI_RES2) && (!R2 || r2_rows <= 0))) {
    g_err = "gemm_x3a: epilogue operand missing";
    return -1;
  }
  const __bf16* w = reinterpret_cast<const __bf16*>(W);
  __bf16* cpp = reinterpret_cast<__bf16*>(Cp);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  epi |= (g_group_m << 8) | (g_ablate << 16) | int(nos_pin_mask() << 20);
  switch (cfg) {
    case 0: return launch_a<128, 128, 2, 4>(A, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    case 1: return launch_a<256, 128, 4, 2>(A, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, s);
    default:
      g_err = "gemm_x3a: unknown config";
      return -1;
  }
}

int nos_gemm_x3_tile(int cfg, int* bm, int* bn, int* nbuf) {
  if (cfg < 0 || cfg > 38) return -1;
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
  epi |= (g_group_m << 8) | (g_ablate << 16) | int(nos_pin_mask() << 20);
  return dispatch(a, ap, w, wp, bias, R, R2, r2_rows, C, cpp, cp, M, N, K, epi, cfg, s);
}

}  // extern "C"
