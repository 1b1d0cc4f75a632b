// nos workload kernels for gfx950 (MI355X): the hot ops of the fp32 YOLOS-small fractional-GPU
// workload. Plain GEMMs stay on hipBLASLt; everything else that touches the activations is here.
//
//  * attn_fwd_f32: flash attention over a packed [B, T, 3*H*64] fp32 QKV tensor on the exact-fp32
//    matrix cores (v_mfma_f32_32x32x2_f32, 64 FLOP/clk/SIMD). One wave owns 32 queries of one head.
//    It computes S^T = K Q^T so that every lane owns ONE query column: the softmax row reductions
//    are 16 in-register ops plus a single cross-half exchange (lane l <-> l^32), no LDS. The
//    accumulator of S^T is fed straight back as the B operand of O^T += V^T P^T (accumulator-as-
//    operand, cdna_hip_programming.md §3), so P never leaves registers. Head-dim -> MFMA K-slot
//    assignment is dim = 32*half + step, which makes every lane's Q and K fragment one contiguous
//    128-byte run (8 x dwordx4). K/V of one head (3401 x 64 x 4 B x 2 = 1.7 MB) stays L2-resident
//    across the query tiles of that head. Optional key split (nsplit > 1) writes per-split
//    (O, m, l) partials that attn_combine_f32 merges, so a whole-GPU launch has enough waves for
//    1024 SIMDs while a 32-CU slice runs unsplit.
//  * layernorm_f32: one wave per row, values kept in registers (two-pass mean/variance), wave64
//    shuffles.
//  * bias_gelu_f32: in-place exact (erf) GELU(y + b) epilogue, dwordx4 vectorised.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <string>

typedef __attribute__((ext_vector_type(16))) float f32x16;

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
// LayerNorm
template <int NPL>
__global__ __launch_bounds__(256) void layernorm_f32(const float* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ b, float* __restrict__ y, int rows,
                                                     float eps) {
  constexpr int D = NPL * 64;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave;
  if (row >= rows) return;
  const float* xr = x + size_t(row) * D;
  float v[NPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    v[i] = xr[i * 64 + lane];
    s += v[i];
  }
  const float mean = wave_sum(s) * (1.0f / D);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    v[i] -= mean;
    q += v[i] * v[i];
  }
  const float rstd = rsqrtf(wave_sum(q) * (1.0f / D) + eps);
  float* yr = y + size_t(row) * D;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int c = i * 64 + lane;
    yr[c] = v[i] * rstd * w[c] + b[c];
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
constexpr int HD = 64;

__device__ __forceinline__ int key_of(int reg, int half) { return (reg & 3) + 8 * (reg >> 2) + 4 * half; }

template <bool SPLIT>
__global__ __launch_bounds__(64, 2) void attn_fwd_f32(const float* __restrict__ qkv, float* __restrict__ out,
                                                      float* __restrict__ part_o, float* __restrict__ part_ml, int T,
                                                      int H, float scale_log2e, int keys_per_split, int nsplit) {
  const int lane = threadIdx.x;
  const int j = lane & 31;   // query column owned by this lane
  const int hf = lane >> 5;  // lane half
  const int qt = blockIdx.x, head = blockIdx.y;
  const int b = SPLIT ? blockIdx.z / nsplit : blockIdx.z;
  const int split = SPLIT ? blockIdx.z % nsplit : 0;
  const int D = H * HD, ld = 3 * D;
  const float* base = qkv + size_t(b) * T * ld;
  const int q0 = qt * 32;

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

  const int k_begin = split * keys_per_split;
  const int k_end = min(T, k_begin + keys_per_split);

  f32x16 o0 = {0}, o1 = {0};
  float m = -INFINITY, l = 0.f;
  const float* kbase = base + D + head * HD + 32 * hf;
  const float* vbase = base + 2 * D + head * HD + j;

  for (int kb = k_begin; kb < k_end; kb += 32) {
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

    if (kb + 32 > k_end) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (kb + key_of(r, hf) >= k_end) s[r] = -INFINITY;
    }
    float mx = s[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s[r]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_new = fmaxf(m, mx);
    const float alpha = __builtin_amdgcn_exp2f(m - m_new);
    float psum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s[r] = __builtin_amdgcn_exp2f(s[r] - m_new);
      psum += s[r];
    }
    psum += __shfl_xor(psum, 32, 64);
    l = l * alpha + psum;
    m = m_new;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      o0[r] *= alpha;
      o1[r] *= alpha;
    }
    // O^T[d][query] += sum_key V^T[d][key] P^T[key][query]; P^T register t is key key_of(t, hf)
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      o0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v0[t], s[t], o0, 0, 0, 0);
      o1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v1[t], s[t], o1, 0, 0, 0);
    }
  }

  const int q = q0 + j;
  if (q >= T) return;
  if (!SPLIT) {
    const float inv = 1.f / l;
    float* orow = out + (size_t(b) * T + q) * D + head * HD;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = key_of(r, hf);
      orow[d] = o0[r] * inv;
      orow[32 + d] = o1[r] * inv;
    }
  } else {
    // partials: part_o[split][b][head][q][64] (unnormalised), part_ml[split][b][head][q][2] = (m, l)
    const size_t idx = ((size_t(blockIdx.z) * H + head) * T + q);
    float* po = part_o + idx * HD;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int d = key_of(r, hf);
      po[d] = o0[r];
      po[32 + d] = o1[r];
    }
    if (hf == 0) {
      part_ml[idx * 2 + 0] = m;
      part_ml[idx * 2 + 1] = l;
    }
  }
}

// merge nsplit partials: one thread per (b, head, q, d)
__global__ __launch_bounds__(256) void attn_combine_f32(const float* __restrict__ part_o,
                                                        const float* __restrict__ part_ml, float* __restrict__ out,
                                                        int B, int T, int H, int nsplit) {
  const size_t i = size_t(blockIdx.x) * 256 + threadIdx.x;
  const size_t total = size_t(B) * H * T * HD;
  if (i >= total) return;
  const int d = int(i % HD);
  size_t r = i / HD;
  const int q = int(r % T);
  r /= T;
  const int head = int(r % H);
  const int b = int(r / H);
  float mmax = -INFINITY;
  for (int s = 0; s < nsplit; ++s) {
    const size_t idx = ((size_t(b * nsplit + s) * H + head) * T + q);
    mmax = fmaxf(mmax, part_ml[idx * 2]);
  }
  float num = 0.f, den = 0.f;
  for (int s = 0; s < nsplit; ++s) {
    const size_t idx = ((size_t(b * nsplit + s) * H + head) * T + q);
    const float sc = __builtin_amdgcn_exp2f(part_ml[idx * 2] - mmax);
    num += part_o[idx * HD + d] * sc;
    den += part_ml[idx * 2 + 1] * sc;
  }
  out[(size_t(b) * T + q) * (H * HD) + head * HD + d] = num / den;
}

}  // namespace

extern "C" {

const char* nos_kernels_last_error() { return g_err.c_str(); }

int nos_layernorm_f32(const float* x, const float* w, const float* b, float* y, int rows, int D, float eps,
                      void* stream) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((rows + 3) / 4), block(256);
  switch (D) {
    case 384: hipLaunchKernelGGL(layernorm_f32<6>, grid, block, 0, s, x, w, b, y, rows, eps); break;
    case 768: hipLaunchKernelGGL(layernorm_f32<12>, grid, block, 0, s, x, w, b, y, rows, eps); break;
    case 1024: hipLaunchKernelGGL(layernorm_f32<16>, grid, block, 0, s, x, w, b, y, rows, eps); break;
    case 1536: hipLaunchKernelGGL(layernorm_f32<24>, grid, block, 0, s, x, w, b, y, rows, eps); break;
    case 2048: hipLaunchKernelGGL(layernorm_f32<32>, grid, block, 0, s, x, w, b, y, rows, eps); break;
    default:
      g_err = "layernorm: unsupported hidden size " + std::to_string(D);
      return -1;
  }
  return check_launch("layernorm_f32");
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

// keys per split (rounded to the 32-key block) and the effective split count
static void split_plan(int T, int nsplit, int* kps, int* ns) {
  *kps = ((T + nsplit - 1) / nsplit + 31) / 32 * 32;
  *ns = (T + *kps - 1) / *kps;
}

// bytes of caller-provided workspace for a split launch (0 when nsplit <= 1). The workspace comes
// from the caller's stream-ordered allocator, so concurrent slices never share scratch and a launch
// inside graph capture never allocates.
size_t nos_attention_ws_bytes(int B, int T, int H, int nsplit) {
  if (nsplit <= 1) return 0;
  int kps, ns;
  split_plan(T, nsplit, &kps, &ns);
  return size_t(ns) * B * H * T * (HD + 2) * sizeof(float);
}

int nos_attention_f32_split(const float* qkv, float* out, float* ws, int B, int T, int H, int head_dim, float scale,
                            int nsplit, void* stream) {
  if (head_dim != HD) {
    g_err = "attention: head_dim must be 64";
    return -1;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float scale_log2e = scale * 1.4426950408889634f;
  const int qtiles = (T + 31) / 32;
  if (nsplit <= 1) {
    hipLaunchKernelGGL(attn_fwd_f32<false>, dim3(qtiles, H, B), dim3(64), 0, s, qkv, out, nullptr, nullptr, T, H,
                       scale_log2e, T, 1);
    return check_launch("attn_fwd_f32");
  }
  int kps;
  split_plan(T, nsplit, &kps, &nsplit);
  if (ws == nullptr) {
    g_err = "attention: split launch needs a workspace (nos_attention_ws_bytes)";
    return -1;
  }
  float* part_o = ws;
  float* part_ml = ws + size_t(nsplit) * B * H * T * HD;
  hipLaunchKernelGGL(attn_fwd_f32<true>, dim3(qtiles, H, B * nsplit), dim3(64), 0, s, qkv, out, part_o, part_ml, T, H,
                     scale_log2e, kps, nsplit);
  if (int rc = check_launch("attn_fwd_f32<split>")) return rc;
  const size_t total = size_t(B) * H * T * HD;
  hipLaunchKernelGGL(attn_combine_f32, dim3((total + 255) / 256), dim3(256), 0, s, part_o, part_ml, out, B, T, H,
                     nsplit);
  return check_launch("attn_combine_f32");
}

int nos_attention_f32(const float* qkv, float* out, int B, int T, int H, int head_dim, float scale, void* stream) {
  return nos_attention_f32_split(qkv, out, nullptr, B, T, H, head_dim, scale, 1, stream);
}

}  // extern "C"
