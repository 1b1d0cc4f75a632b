// attn_fwd_x3w: fp32-input x3 flash attention with one wave per SIMD and two query tiles per wave
// (the "wide" kernel; kernels.hip attention_x3_launch dispatches it for fp32-input 8-tile launches
// unless nos_attention_x3_set_wide(0) / NOS_ATTN_WIDE=0).
//
// Its own translation unit because it is built with its own code generation
// (walkai_nos_amd/ops/build.py, Target.source_flags): `-mllvm -amdgpu-mfma-vgpr-form=1` makes the
// MFMAs write their accumulators to VGPRs. The default form keeps every accumulator in AGPRs, and a
// kernel whose VALU reads the scores the MFMAs just wrote (the softmax of S, the row maxima) then
// pays an AGPR -> VGPR copy per value per block: measured on the box
// (profiles/attn_wide_ab_r6.json) the wide kernel built that way only matches attn_fwd_x3p<8>; built
// with VGPR accumulators it is 4-8% faster. The flag is a backend option, not a function attribute:
// the rest of libnos_kernels (the GEMMs, whose accumulators only leave through the epilogue) keeps
// the default.
#include <hip/hip_runtime.h>

#include "pin.h"
#include "x3_common.h"

#include <utility>

namespace {

// One wave per SIMD, two query tiles per wave ("wide" x3 attention). The units, stream-K ranges and
// partial slots are attn_fwd_x3p<8>'s (a workgroup owns a 256-query group of one head; tile
// 2*wave + t is its t-th 32-query tile), so attn_sk_lds_fixup<8> merges the partials unchanged, and
// each tile's arithmetic is that kernel's in the same order: the outputs are bit-identical. What
// changes is the issue structure. In attn_fwd_x3p<8> two waves share each SIMD and fight for its
// VALU issue (the loser parks behind the winner's softmax); here one wave
// owns the SIMD and the whole register file, and carries two independent MFMA chains per phase:
// every K fragment read feeds 12 MFMAs instead of 6 and every V^T fragment 12, and the scores of
// block i+1 (48 MFMAs) issue beside block i's softmax and P split (the VALU of BOTH tiles), so the
// filler budget per MFMA gap holds without a partner wave. fp32 QKV input only (split in-kernel).
template <class F, int... Q>
__device__ __forceinline__ void x3w_slots(F& f, std::integer_sequence<int, Q...>) {
  (f(std::integral_constant<int, Q>{}), ...);
}

#ifndef NOS_X3W_FENCE
#define NOS_X3W_FENCE 1
#endif
// The k-th of mfma_x3's six products (the same order: a2b0, a1b1, a0b2, a1b0, a0b1, a0b0), so a
// chain issued one product at a time accumulates exactly as mfma_x3 does.
__device__ __forceinline__ f32x16 x3_step(int k, const bf16x8& a0, const bf16x8& a1, const bf16x8& a2,
                                          const bf16x8& b0, const bf16x8& b1, const bf16x8& b2, const f32x16& d) {
  switch (k) {
    case 0: return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, d, 0, 0, 0);
    case 1: return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, d, 0, 0, 0);
    case 2: return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, d, 0, 0, 0);
    case 3: return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, d, 0, 0, 0);
    case 4: return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, d, 0, 0, 0);
    default: return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, d, 0, 0, 0);
  }
}

template <bool FDIV = false>
__global__ __launch_bounds__(256, 1) void attn_fwd_x3w(const float* __restrict__ qkv, float* __restrict__ out,
                                                       __bf16* __restrict__ outp, float* __restrict__ part_o,
                                                       float* __restrict__ part_ml, int B, int T, int H, int h0,
                                                       int Ht, float scale_log2e, int Pk, int* __restrict__ cnt) {
  constexpr int G = 8;  // query tiles per workgroup: 4 waves x 2
  __shared__ __attribute__((aligned(16))) __bf16 lds_k[2 * 3 * XK_PLANE];
  __shared__ __attribute__((aligned(16))) __bf16 lds_v[2 * 3 * XV_PLANE];
  __shared__ int s_last;
  const int P = Pk & 0x3fffff;
  const PinnedBlock pb = pinned_block(unsigned(Pk >> 22) & 0xffu);
  if (pb.id < 0 || pb.id >= P) return;
  const int w = (Pk >> 30) ? pb.id : xcd_major_n(pb.id, P, pb.nx);
  const int NK = (T + 31) / 32, QT = NK, QG = (QT + G - 1) / G;
  const long long U = (long long)B * H * QG * NK;
  const float rP = FDIV ? 1.f / float(P) : 0.f, rNK = FDIV ? 1.f / float(NK) : 0.f;
  const float rQG = FDIV ? 1.f / float(QG) : 0.f, rH = FDIV ? 1.f / float(H) : 0.f;
  long long u = FDIV ? udiv23(w * U, P, rP) : sk_begin(w, U, P);
  const long long u1 = FDIV ? udiv23((w + 1) * U, P, rP) : sk_begin(w + 1, U, P);
  const int D = Ht * HD, ld = 3 * D;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int j = lane & 31, hf = lane >> 5;
  const int lrow = tid >> 3, lch = tid & 7;  // K/V staging: key row, 8-dim chunk
  const int gi = lane & 15, gg = lane >> 4;
  const int vtr = (4 * hf + (gi >> 2)) * XV_STR + 16 * (gg & 1) + 4 * (gi & 3);
  bool first = true;
  while (u < u1) {
    const long long grp = FDIV ? udiv23(u, NK, rNK) : u / NK;
    const int kb0 = int(u - grp * NK);
    const int kb1 = int(min<long long>(NK, kb0 + (u1 - u)));
    const int nb = kb1 - kb0;
    const long long gq = FDIV ? udiv23(grp, QG, rQG) : grp / QG;
    const int qg = int(grp - gq * QG);
    const long long bq = FDIV ? udiv23(gq, H, rH) : gq / H;
    const int head = h0 + int(gq - bq * H);
    const int b = int(bq);
    const float* basef = qkv + size_t(b) * T * ld;
    const int qtA = qg * G + 2 * wv, qtB = qtA + 1;
    const bool activeA = qtA < QT, activeB = qtB < QT;  // B active implies A active

    bf16x8 qa[3][4], qb[3][4];
    {
      const float* qpa = basef + size_t(min(qtA * 32 + j, T - 1)) * ld + head * HD + 8 * hf;
      const float* qpb = basef + size_t(min(qtB * 32 + j, T - 1)) * ld + head * HD + 8 * hf;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const f32x4 alo = *reinterpret_cast<const f32x4*>(qpa + 16 * s);
        const f32x4 ahi = *reinterpret_cast<const f32x4*>(qpa + 16 * s + 4);
        const f32x4 blo = *reinterpret_cast<const f32x4*>(qpb + 16 * s);
        const f32x4 bhi = *reinterpret_cast<const f32x4*>(qpb + 16 * s + 4);
        split3(f32x8{alo[0], alo[1], alo[2], alo[3], ahi[0], ahi[1], ahi[2], ahi[3]}, qa[0][s], qa[1][s], qa[2][s]);
        split3(f32x8{blo[0], blo[1], blo[2], blo[3], bhi[0], bhi[1], bhi[2], bhi[3]}, qb[0][s], qb[1][s], qb[2][s]);
      }
      // the Q planes only ever feed the matrix pipe: park them in AGPRs (MFMA sources may be AGPRs),
      // which leaves the VGPRs to the softmax, the P planes and the K/V staging
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int s = 0; s < 4; ++s) asm volatile("" : "+a"(qa[p][s]), "+a"(qb[p][s]));
    }
    const float* kgf = basef + D + head * HD + 8 * lch;
    const float* vgf = basef + 2 * D + head * HD + 8 * lch;
    f32x4 fk0, fk1, fv0, fv1;
    auto fetch_k = [&](int blk) {
      const size_t r = size_t(min(blk * 32 + lrow, T - 1)) * ld;
      fk0 = *reinterpret_cast<const f32x4*>(kgf + r);
      fk1 = *reinterpret_cast<const f32x4*>(kgf + r + 4);
    };
    auto fetch_v = [&](int blk) {
      const size_t r = size_t(min(blk * 32 + lrow, T - 1)) * ld;
      fv0 = *reinterpret_cast<const f32x4*>(vgf + r);
      fv1 = *reinterpret_cast<const f32x4*>(vgf + r + 4);
    };
    auto stash = [](const f32x4& lo, const f32x4& hi, __bf16* d, int pstride) {
      bf16x8 a0, a1, a2;
      split3(f32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]}, a0, a1, a2);
      *reinterpret_cast<bf16x8*>(d) = a0;
      *reinterpret_cast<bf16x8*>(d + pstride) = a1;
      *reinterpret_cast<bf16x8*>(d + 2 * pstride) = a2;
    };
    auto stash_k = [&](int buf) { stash(fk0, fk1, &lds_k[buf * 3 * XK_PLANE + lrow * XK_STR + 8 * lch], XK_PLANE); };
    auto stash_v = [&](int buf) { stash(fv0, fv1, &lds_v[buf * 3 * XV_PLANE + lrow * XV_STR + 8 * lch], XV_PLANE); };
    // S^T of both tiles for the K block in buffer BUF, one mfma_x3 per tile and k-step (prologue)
    auto qk_all = [&](f32x16& SA, f32x16& SB, int buf) {
      const __bf16* ks_ = &lds_k[buf * 3 * XK_PLANE + j * XK_STR + 8 * hf];
      SA = f32x16{0};
      SB = f32x16{0};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const bf16x8 k0 = *reinterpret_cast<const bf16x8*>(ks_ + 16 * s);
        const bf16x8 k1 = *reinterpret_cast<const bf16x8*>(ks_ + XK_PLANE + 16 * s);
        const bf16x8 k2 = *reinterpret_cast<const bf16x8*>(ks_ + 2 * XK_PLANE + 16 * s);
        SA = mfma_x3(k0, k1, k2, qa[0][s], qa[1][s], qa[2][s], SA);
        SB = mfma_x3(k0, k1, k2, qb[0][s], qb[1][s], qb[2][s], SB);
      }
    };
    auto rowmax = [&](const f32x16& S) {
      float mx = fmaxf(S[0], S[1]);
#pragma unroll
      for (int r = 2; r < 16; ++r) mx = fmaxf(mx, S[r]);
      return half_max(mx);
    };
    __syncthreads();  // the previous segment's last blocks are no longer being read
    fetch_k(kb0);
    fetch_v(kb0);
    stash_k(0);
    stash_v(0);
    fetch_k(kb0 + 1);
    stash_k(1);
    __syncthreads();
    f32x16 oa0 = {0}, oa1 = {0}, ob0 = {0}, ob1 = {0}, sca, scb, sna, snb;
    float ma = -INFINITY, la = 0.f, mb = -INFINITY, lb = 0.f;
    qk_all(sca, scb, 0);
    float mxa = rowmax(sca), mxb = rowmax(scb);  // row maxima of the current scores (before any mask)
    __syncthreads();  // iteration 0 refills K buffer 0
    // lazy rescale of one tile (wave-uniform decision, as attn_fwd_x3p)
    auto rescale = [&](float mx, float& m, float& l, f32x16& o0, f32x16& o1) {
      if (__builtin_amdgcn_ballot_w64((mx - m) * scale_log2e > 8.f)) {
        const float m_new = fmaxf(m, mx);
        const float alpha = __builtin_amdgcn_exp2f((m - m_new) * scale_log2e);
        l *= alpha;
        o0 *= alpha;
        o1 *= alpha;
        m = m_new;
      }
    };
    // One key block i as ONE basic block of 96 issue slots, each one MFMA plus its share of the
    // vector and LDS work, fenced by sched_barrier so the compiler keeps the interleave (one wave
    // per SIMD: no partner's MFMAs cover a VALU run — placed between the wave's own MFMAs, ~3
    // instructions per 32-cycle gap issue in the matrix pipe's shadow):
    //   slots  0-47  S(i+1) = K(i+1) Q^T, 4 k-steps x {tile A, tile B} x 6 products; beside them
    //                exp of P(i) (A 0-7, B 0-7, then A 8-15, B 8-15) and the plane split of keys
    //                0-15 (s2 = 0); the K fragments of each k-step and the V^T fragments of s2 = 0
    //   slots 48-71  O += V^T P^T for keys 0-15 (dh 0: A, B; dh 1: A, B); beside them the split of
    //                keys 16-31, the l updates, the row max of S(i+1) tile A, V^T reads of s2 = 1
    //   slots 72-95  the same for keys 16-31; beside them the row max of S(i+1) tile B and the
    //                split + LDS writes of the K/V blocks fetched at the top of the iteration
    // The order of every accumulation (MFMA chains, psum, l) is attn_fwd_x3p's: bit-identical.
    auto iter = [&](f32x16& SA, f32x16& SB, f32x16& NA, f32x16& NB, float& mxA, float& mxB, int i) {
      const int blk = kb0 + i;
      if (blk * 32 + 32 > T) {  // the tail block: mask keys >= T, re-take the maxima (wave-uniform)
        asm volatile("; tail block: mask keys >= T" ::: "memory");
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (blk * 32 + key_of(r, hf) >= T) SA[r] = SB[r] = -INFINITY;
        mxA = rowmax(SA);
        mxB = rowmax(SB);
      }
      rescale(mxA, ma, la, oa0, oa1);
      rescale(mxB, mb, lb, ob0, ob1);
      fetch_k(blk + 2);  // clamped rows past the segment: a harmless refill of a free buffer
      fetch_v(blk + 1);
      const float mcA = ma * scale_log2e, mcB = mb * scale_log2e;
      float psA = 0.f, psB = 0.f;
      const __bf16* ks_ = &lds_k[((i + 1) & 1) * 3 * XK_PLANE + j * XK_STR + 8 * hf];
      const __bf16* vs_ = &lds_v[(i & 1) * 3 * XV_PLANE + vtr];
      bf16x8 kf[2][3], vf[2][2][3];
      uint32_t pw[2][2][3][4];  // P planes: [tile][s2][plane][pair]
      float ra[2], rb[2];       // a pair's first residuals between its two split slots
      typedef float f32x2v __attribute__((ext_vector_type(2)));
      typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
      bf16x2v kh[3][4], vh[3][4];  // the fetched K / V chunk as planes, pair by pair
      f32x2v kr[4], vr[4];
      float mxn = 0.f;
      auto read_k = [&](int s, int slot) {
#pragma unroll
        for (int p = 0; p < 3; ++p) kf[slot][p] = *reinterpret_cast<const bf16x8*>(ks_ + p * XK_PLANE + 16 * s);
      };
      auto read_v = [&](int s2, int dh, int p) {
        const __bf16* a = vs_ + p * XV_PLANE + 16 * s2 * XV_STR + 32 * dh;
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a + 8 * XV_STR));
        vf[s2][dh][p] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      };
      // (no reference or pointer is ever selected between two arrays below: such a select keeps
      // them out of registers — every choice is a branch on a value the unrolled loop folds)
      // the exp of element r, and (a slot later, so no add waits on its transcendental) its add to
      // the row sum — in r order, so the sum is attn_fwd_x3p's
      auto expo = [&](int t, int r) {
        if (t)
          SB[r] = __builtin_amdgcn_exp2f(fmaf(SB[r], scale_log2e, -mcB));
        else
          SA[r] = __builtin_amdgcn_exp2f(fmaf(SA[r], scale_log2e, -mcA));
      };
      auto addp = [&](int t, int r) {
        if (t)
          psB += SB[r];
        else
          psA += SA[r];
      };
      // split3_trunc8 of the pair (2q, 2q+1) of keys 16*s2.., in two slots
      auto split_a = [&](int t, int s2, int q) {
        const float a = t ? SB[8 * s2 + 2 * q] : SA[8 * s2 + 2 * q];
        const float b = t ? SB[8 * s2 + 2 * q + 1] : SA[8 * s2 + 2 * q + 1];
        const uint32_t ua = __float_as_uint(a), ub = __float_as_uint(b);
        pw[t][s2][0][q] = __builtin_amdgcn_perm(ub, ua, 0x07060302u);
        ra[t] = a - __uint_as_float(ua & 0xffff0000u);
        rb[t] = b - __uint_as_float(ub & 0xffff0000u);
      };
      auto split_b = [&](int t, int s2, int q) {
        const uint32_t ura = __float_as_uint(ra[t]), urb = __float_as_uint(rb[t]);
        pw[t][s2][1][q] = __builtin_amdgcn_perm(urb, ura, 0x07060302u);
        const float sa = ra[t] - __uint_as_float(ura & 0xffff0000u), sb = rb[t] - __uint_as_float(urb & 0xffff0000u);
        pw[t][s2][2][q] = __builtin_amdgcn_perm(__float_as_uint(sb), __float_as_uint(sa), 0x07060302u);
      };
      auto pplane = [&](int t, int s2, int p) {
        return __builtin_bit_cast(bf16x8, (uint4){pw[t][s2][p][0], pw[t][s2][p][1], pw[t][s2][p][2], pw[t][s2][p][3]});
      };
      // the fetched chunk's plane split, one value pair per slot half (split3's arithmetic)
      auto stash_a = [&](bool isv, int q) {
        const f32x4 lo = isv ? fv0 : fk0, hi = isv ? fv1 : fk1;  // value selects
        const f32x2v x = q < 2 ? f32x2v{lo[2 * q], lo[2 * q + 1]} : f32x2v{hi[2 * q - 4], hi[2 * q - 3]};
        const bf16x2v h0 = __builtin_convertvector(x, bf16x2v);
        const f32x2v r = x - __builtin_convertvector(h0, f32x2v);
        if (isv) vh[0][q] = h0, vr[q] = r;
        else kh[0][q] = h0, kr[q] = r;
      };
      auto stash_b = [&](bool isv, int q) {
        const f32x2v r = isv ? vr[q] : kr[q];
        const bf16x2v h1 = __builtin_convertvector(r, bf16x2v);
        const bf16x2v h2 = __builtin_convertvector(r - __builtin_convertvector(h1, f32x2v), bf16x2v);
        if (isv) vh[1][q] = h1, vh[2][q] = h2;
        else kh[1][q] = h1, kh[2][q] = h2;
      };
      auto stash_w = [&](bool isv) {
        if (isv) {
          __bf16* d = &lds_v[((i + 1) & 1) * 3 * XV_PLANE + lrow * XV_STR + 8 * lch];
#pragma unroll
          for (int p = 0; p < 3; ++p)
            *reinterpret_cast<bf16x8*>(d + p * XV_PLANE) = bf16x8{vh[p][0][0], vh[p][0][1], vh[p][1][0], vh[p][1][1],
                                                                  vh[p][2][0], vh[p][2][1], vh[p][3][0], vh[p][3][1]};
        } else {
          __bf16* d = &lds_k[(i & 1) * 3 * XK_PLANE + lrow * XK_STR + 8 * lch];
#pragma unroll
          for (int p = 0; p < 3; ++p)
            *reinterpret_cast<bf16x8*>(d + p * XK_PLANE) = bf16x8{kh[p][0][0], kh[p][0][1], kh[p][1][0], kh[p][1][1],
                                                                  kh[p][2][0], kh[p][2][1], kh[p][3][0], kh[p][3][1]};
        }
      };
      read_k(0, 0);
      __builtin_amdgcn_sched_barrier(0);
      // slot q as a compile-time constant (a fold over 96 instantiations, not a loop the unroller
      // may decline): every array index below is constant, so every array lives in registers
      auto slot = [&](auto qc) {
        constexpr int q = decltype(qc)::value;
        // ---- the slot's MFMA
        if constexpr (q < 48) {
          constexpr int s = q / 12, t = (q / 6) & 1, k = q % 6;
          const bf16x8* kk = kf[s & 1];
          const bool init = s == 0 && k == 0;
          if (t == 0)
            NA = x3_step(k, kk[0], kk[1], kk[2], qa[0][s], qa[1][s], qa[2][s], init ? f32x16{0} : NA);
          else
            NB = x3_step(k, kk[0], kk[1], kk[2], qb[0][s], qb[1][s], qb[2][s], init ? f32x16{0} : NB);
        } else {
          const int v = q - 48, s2 = v / 24, dh = (v / 12) & 1, t = (v / 6) & 1, k = v % 6;
          const bf16x8* vv = vf[s2][dh];
          const bf16x8 p0 = pplane(t, s2, 0), p1 = pplane(t, s2, 1), p2 = pplane(t, s2, 2);
          if (dh == 0 && t == 0) oa0 = x3_step(k, vv[0], vv[1], vv[2], p0, p1, p2, oa0);
          else if (dh == 0) ob0 = x3_step(k, vv[0], vv[1], vv[2], p0, p1, p2, ob0);
          else if (t == 0) oa1 = x3_step(k, vv[0], vv[1], vv[2], p0, p1, p2, oa1);
          else ob1 = x3_step(k, vv[0], vv[1], vv[2], p0, p1, p2, ob1);
        }
        // ---- its vector work
        // the row-sum adds trail their exps by one slot (A 0-7 in slots 1-8, B 0-7 in 9-16,
        // A 8-15 in 33-40, B 8-15 in 41-48)
        if constexpr ((q >= 1 && q <= 16) || (q >= 33 && q <= 48)) {
          constexpr int e = q <= 16 ? q - 1 : q - 33;
          addp(e / 8, (q <= 16 ? 0 : 8) + e % 8);
        }
        if (q < 8) expo(0, q);
        else if (q < 16) expo(1, q - 8);
        else if (q < 32) {
          const int t = (q - 16) / 8, pq = ((q - 16) % 8) / 2;
          if (q % 2 == 0) split_a(t, 0, pq); else split_b(t, 0, pq);
        } else if (q < 40) expo(0, q - 32 + 8);
        else if (q < 48) expo(1, q - 40 + 8);
        else if (q < 64) {
          const int t = (q - 48) / 8, pq = ((q - 48) % 8) / 2;
          if (q % 2 == 0) split_a(t, 1, pq); else split_b(t, 1, pq);
        } else if (q == 64) la += half_sum(psA);
        else if (q == 65) lb += half_sum(psB);
        else if (q >= 66 && q < 70) {  // row max of S(i+1), tile A (4 x 4 values), then tile B
          const int c = q - 66;
          float m4 = fmaxf(NA[4 * c], NA[4 * c + 1]);
          m4 = fmaxf(m4, NA[4 * c + 2]);
          m4 = fmaxf(m4, NA[4 * c + 3]);
          mxn = c ? fmaxf(mxn, m4) : m4;
        } else if (q == 70) mxA = half_max(mxn);
        else if (q >= 72 && q < 76) {
          const int c = q - 72;
          float m4 = fmaxf(NB[4 * c], NB[4 * c + 1]);
          m4 = fmaxf(m4, NB[4 * c + 2]);
          m4 = fmaxf(m4, NB[4 * c + 3]);
          mxn = c ? fmaxf(mxn, m4) : m4;
        } else if (q == 76) mxB = half_max(mxn);
        else if (q >= 77 && q < 85) {
          if ((q - 77) % 2 == 0) stash_a(false, (q - 77) / 2); else stash_b(false, (q - 77) / 2);
        } else if (q >= 86 && q < 94) {
          if ((q - 86) % 2 == 0) stash_a(true, (q - 86) / 2); else stash_b(true, (q - 86) / 2);
        }
        // ---- its LDS work
        if (q == 2 || q == 14 || q == 26) read_k(q / 12 + 1, (q / 12 + 1) & 1);
        if (q >= 29 && q < 41 && (q - 29) % 2 == 0) read_v(0, (q - 29) / 6, (q - 29) / 2 % 3);
        if (q >= 50 && q < 62 && (q - 50) % 2 == 0) read_v(1, (q - 50) / 6, (q - 50) / 2 % 3);
        if (q == 85) stash_w(false);
        if (q == 94) stash_w(true);
        if (NOS_X3W_FENCE) __builtin_amdgcn_sched_barrier(0);
      };
      x3w_slots(slot, std::make_integer_sequence<int, 96>{});
    };
    // two blocks per trip (the score registers swap roles), an odd last block after the loop: one
    // back edge, so the O accumulators keep their registers across both halves
    int i = 0;
    for (; i + 1 < nb; i += 2) {
      iter(sca, scb, sna, snb, mxa, mxb, i);
      __syncthreads();
      iter(sna, snb, sca, scb, mxa, mxb, i + 1);
      __syncthreads();
    }
    if (i < nb) {
      iter(sca, scb, sna, snb, mxa, mxb, i);
      __syncthreads();
    }

    // tile t's normalised rows (a whole key range, or the merge of a split one)
    const bool whole = kb0 == 0 && kb1 == NK;
    auto store_tile = [&](int t, const f32x16& o0, const f32x16& o1, float l) {
      const int q = (qg * G + 2 * wv + t) * 32 + j;
      if (q >= T) return;
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
    };
    // the two tiles' results: whole key range -> normalised output, else a partial slot
    auto finish = [&](bool active, int t, const f32x16& o0, const f32x16& o1, float m, float l) {
      if (!active) return;
      if (whole) {
        store_tile(t, o0, o1, l);
      } else {
        const size_t slot = (size_t(w) * 2 + (first ? 0 : 1)) * G + 2 * wv + t;
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
    };
    finish(activeA, 0, oa0, oa1, ma, la);
    finish(activeB, 1, ob0, ob1, mb, lb);
    if (!whole && cnt) {
      // Stream-K merge in the kernel (cnt != nullptr): the row's contributors count themselves in
      // cnt[grp] after their partials are visible device-wide, and the LAST to arrive merges every
      // contributor's partials — in workgroup order, with attn_sk_lds_fixup's arithmetic, so the
      // result is that kernel's bit for bit — and stores the normalised tiles. Nobody waits for
      // anybody (no spin, whatever the residency), and the last arriver resets the counter, so the
      // counters are zero again when the grid has drained. Replaces the fixup launch and its re-read
      // of every partial. Opt-in (NOS_ATTN_MERGE=1): on the box it is slower than the fixup launch
      // (profiles/attn_merge_ab_r6.json); likely the device-scope release / acquire below, which
      // compile to a write-back and an invalidate of the XCD's L2 (the XCDs' L2s are not coherent).
      const long long t0 = grp * NK, t1 = t0 + NK;
      const long long wlo = ((t0 + 1) * P + U - 1) / U - 1, whi = (t1 * P + U - 1) / U - 1;
      __threadfence();  // release: this workgroup's partials before its count
      __syncthreads();
      if (tid == 0) {
        int n = 0;
        for (long long x = wlo; x <= whi; ++x) n += (x * U / P != (x + 1) * U / P) ? 1 : 0;
        const int last = atomicAdd(&cnt[grp], 1) == n - 1;
        if (last) atomicExch(&cnt[grp], 0);
        s_last = last;
      }
      __syncthreads();
      if (s_last) {
        __threadfence();  // acquire: every other contributor's partials
        auto merge = [&](int t) {
          float M = -INFINITY, L = 0.f;
          f32x16 a0 = {0}, a1 = {0};
          for (long long x = wlo; x <= whi; ++x) {
            const long long s0 = x * U / P;
            if (s0 == (x + 1) * U / P) continue;
            const size_t slot = (size_t(x) * 2 + (s0 >= t0 ? 0 : 1)) * G + 2 * wv + t;
            const float mw = part_ml[slot * 64 + j];
            if (mw == -INFINITY) continue;
            const float lw = part_ml[slot * 64 + 32 + j];
            const float* po = part_o + slot * (HD * 32);
            const float Mn = fmaxf(M, mw);
            const float so = __builtin_amdgcn_exp2f(M - Mn), sn = __builtin_amdgcn_exp2f(mw - Mn);
            L = fmaf(lw, sn, L * so);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int d = key_of(r, hf);
              a0[r] = fmaf(po[d * 32 + j], sn, a0[r] * so);
              a1[r] = fmaf(po[(32 + d) * 32 + j], sn, a1[r] * so);
            }
            M = Mn;
          }
          store_tile(t, a0, a1, L);
        };
        if (activeA) merge(0);
        if (activeB) merge(1);
      }
    }
    u += kb1 - kb0;
    first = false;
  }
}

}  // namespace

int nos_attn_x3w_launch(bool fdiv, dim3 grid, hipStream_t s, const float* qkv, float* out, __bf16* outp,
                        float* part_o, float* part_ml, int B, int T, int H, int h0, int Ht, float scale_log2e,
                        int Pk, int* cnt) {
  if (fdiv)
    hipLaunchKernelGGL(attn_fwd_x3w<true>, grid, dim3(256), 0, s, qkv, out, outp, part_o, part_ml, B, T, H, h0, Ht,
                       scale_log2e, Pk, cnt);
  else
    hipLaunchKernelGGL(attn_fwd_x3w<false>, grid, dim3(256), 0, s, qkv, out, outp, part_o, part_ml, B, T, H, h0, Ht,
                       scale_log2e, Pk, cnt);
  return int(hipPeekAtLastError());  // left set for the caller's check_launch
}

int nos_attn_x3w_occupancy() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, attn_fwd_x3w<true>, 256, 0) != hipSuccess || n <= 0) n = 1;
  return n;
}
