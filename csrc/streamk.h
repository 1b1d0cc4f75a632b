// Stream-K work split of a tiled GEMM, shared by the producer (gemm_x3k in gemm_x3.hip) and the
// consumer (splitk_layernorm_f32 in kernels.hip) so both agree on which partial plane holds what.
//
// The GEMM's work is U = tiles * nk units (one unit = one K stage of one tile, tiles row-major,
// a tile's stages consecutive); workgroup w of P owns units [w*U/P, (w+1)*U/P). A tile's stages
// are thus cut into segments, one per workgroup that touches it; segment s of tile t (s = w -
// owner(first unit of t)) goes to fp32 partial plane s. Every plane s < nseg(t) of a tile is
// written, planes at or above it are not (the consumer never reads them). P <= U keeps every range
// non-empty, so owner() is the inverse of the range split.
#pragma once

struct SkMap {
  int P;        // workgroups (0 = not stream-K: the consumer adds a fixed number of planes)
  int U;        // units = tiles * nk
  int nk;       // K stages per tile
  int bm, bn;   // tile shape
  int tiles_n;  // tiles per row of tiles (N / bn)
};

// workgroup whose range holds unit u: the largest w with floor(w*U/P) <= u
__host__ __device__ inline int sk_owner(int u, int P, int U) {
  return int(((long long)(u + 1) * P - 1) / U);
}

__host__ __device__ inline int sk_first(int w, int P, int U) { return int((long long)w * U / P); }

// segments (= partial planes) of tile t
__host__ __device__ inline int sk_segments(int t, const SkMap& m) {
  return sk_owner((t + 1) * m.nk - 1, m.P, m.U) - sk_owner(t * m.nk, m.P, m.U) + 1;
}
