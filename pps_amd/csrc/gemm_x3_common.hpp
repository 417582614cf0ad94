// Pieces shared by the two bf16x3 GEMM kernels (gemm_x3.hip: register-staged;
// gemm_x3p.hip: LDS-DMA pipelined): the exact three-way bf16 split, the MFMA
// wrapper and the distance epilogue.  Both kernels apply the six product
// terms in the same order on the same 16-wide K groups, so they give
// identical bits.
#pragma once
#include "gemm_common.hpp"

namespace pps {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Two floats -> three packed bf16 pairs with x = hi + mid + lo exactly
// (round-to-nearest-even splits; each remainder is exact in f32).
__device__ inline void split2(float x0, float x1, unsigned& hi, unsigned& mid, unsigned& lo) {
  const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){x0, x1}, bf16x2));
  const float r0 = x0 - __builtin_bit_cast(float, u << 16);
  const float r1 = x1 - __builtin_bit_cast(float, u & 0xffff0000u);
  const unsigned v = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){r0, r1}, bf16x2));
  const float s0 = r0 - __builtin_bit_cast(float, v << 16);
  const float s1 = r1 - __builtin_bit_cast(float, v & 0xffff0000u);
  hi = u;
  mid = v;
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2){s0, s1}, bf16x2));
}

// Eight consecutive-K floats -> the three bf16x8 MFMA fragments.
__device__ inline void split8(const f32x4& x0, const f32x4& x1, bf16x8& fhi, bf16x8& fmid,
                              bf16x8& flo) {
  u32x4 hi, mid, lo;
  unsigned a, b, c;
  split2(x0[0], x0[1], a, b, c); hi[0] = a; mid[0] = b; lo[0] = c;
  split2(x0[2], x0[3], a, b, c); hi[1] = a; mid[1] = b; lo[1] = c;
  split2(x1[0], x1[1], a, b, c); hi[2] = a; mid[2] = b; lo[2] = c;
  split2(x1[2], x1[3], a, b, c); hi[3] = a; mid[3] = b; lo[3] = c;
  fhi = __builtin_bit_cast(bf16x8, hi);
  fmid = __builtin_bit_cast(bf16x8, mid);
  flo = __builtin_bit_cast(bf16x8, lo);
}

__device__ inline f32x16 mfma_bf16(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// The six product terms of one (A, B) fragment pair, fixed order:
//   a0b0 + a1b0 + a0b1 + a2b0 + a1b1 + a0b2
__device__ inline f32x16 mfma_x3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 c) {
  c = mfma_bf16(a[0], b[0], c);
  c = mfma_bf16(a[1], b[0], c);
  c = mfma_bf16(a[0], b[1], c);
  c = mfma_bf16(a[2], b[0], c);
  c = mfma_bf16(a[1], b[1], c);
  c = mfma_bf16(a[0], b[2], c);
  return c;
}

// The same six terms on v_mfma_f32_16x16x32_bf16 (the S = 16 tiles of
// gemm_x3p.hip and gemm_ws.hip) with the MFMA operands swapped (weights as
// the MFMA "A"): one MFMA covers a whole 32-wide K chunk, so its rounding
// differs from the 32x32x16 form -- S = 16 kernels agree bit for bit with
// each other, not with S = 32.  Transposed accumulator: lane l keeps output
// row (l & 15) and columns 4 (l >> 4) + e, e = 0..3 (one 16-byte vector per
// block).
__device__ inline f32x4 mfma16_bf16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
#ifndef PPS_X3_ORDER
#define PPS_X3_ORDER 0  // probes: 1 / 2 = weight- / activation-plane-major term order
#endif
__device__ inline f32x4 mfma16_x3t(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4 c) {
  if constexpr (PPS_X3_ORDER == 1) {
    c = mfma16_bf16(b[0], a[0], c);
    c = mfma16_bf16(b[0], a[1], c);
    c = mfma16_bf16(b[0], a[2], c);
    c = mfma16_bf16(b[1], a[0], c);
    c = mfma16_bf16(b[1], a[1], c);
    c = mfma16_bf16(b[2], a[0], c);
    return c;
  }
  if constexpr (PPS_X3_ORDER == 2) {
    c = mfma16_bf16(b[0], a[0], c);
    c = mfma16_bf16(b[1], a[0], c);
    c = mfma16_bf16(b[2], a[0], c);
    c = mfma16_bf16(b[0], a[1], c);
    c = mfma16_bf16(b[1], a[1], c);
    c = mfma16_bf16(b[0], a[2], c);
    return c;
  }
  c = mfma16_bf16(b[0], a[0], c);
  c = mfma16_bf16(b[0], a[1], c);
  c = mfma16_bf16(b[1], a[0], c);
  c = mfma16_bf16(b[0], a[2], c);
  c = mfma16_bf16(b[1], a[1], c);
  c = mfma16_bf16(b[2], a[0], c);
  return c;
}

// ---- f16x2 ("h2") arithmetic (gemm_h2.hip, and the EPI_F_H2 conv tiles of
// gemm_x3p.hip / gemm_x3c.hip): x 2^s = h0 + h1 + r with h0 = f16(x 2^s),
// h1 = f16(x 2^s - h0), |r| <= 2^-22 |x 2^s| (2^s from h2_scale_of), and a
// product from the three terms h0 h0' + h0 h1' + h1 h0' on f16 MFMAs.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

__device__ inline f32x4 mfma16_f16(const f16x8& a, const f16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// Two floats (a, b), scaled by the wave-uniform power of two S, -> their f16
// terms packed in pairs: hi = (f16(a S), f16(b S)), lo = (f16(a S - hi_a),
// f16(b S - hi_b)).  a S is exact and so is a S - hi_a (<= 24 significant
// bits), so each term is ONE rounding to f16 -- what (_Float16)(a * S) and
// (_Float16)(a * S - (float)hi) give.  Four v_fma_mix per pair: the
// compiler's own sequence (v_mul + v_cvt_pk for the hi pair, and the hi
// terms again as v_fma_mixlo for the remainders) took seven, and the split is
// the f16x2 main loops' VALU cost (an MFMA 16x16x32 gap leaves 8 issue
// cycles).
__device__ inline void h2_pair(float a, float b, float S, unsigned& hi, unsigned& lo) {
  asm("v_fma_mixlo_f16 %0, %2, %4, -0\n\t"   // (+ -0: a S exactly, its zero sign too)
      "v_fma_mixhi_f16 %0, %3, %4, -0\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(hi), "=&v"(lo)
      : "v"(a), "v"(b), "s"(S));
}

// Eight consecutive-K floats, scaled by S, -> the two f16x8 MFMA fragments
// (kept in bf16x8 storage so the bf16x3 kernels' fragment arrays hold them).
__device__ inline void split8_h2(const f32x4& x0, const f32x4& x1, float S, bf16x8& f0,
                                 bf16x8& f1) {
  unsigned h0, h1, h2, h3, l0, l1, l2, l3;
  h2_pair(x0[0], x0[1], S, h0, l0);
  h2_pair(x0[2], x0[3], S, h1, l1);
  h2_pair(x1[0], x1[1], S, h2, l2);
  h2_pair(x1[2], x1[3], S, h3, l3);
  f0 = __builtin_bit_cast(bf16x8, (u32x4){h0, h1, h2, h3});
  f1 = __builtin_bit_cast(bf16x8, (u32x4){l0, l1, l2, l3});
}

// Four outputs as f16x2 planes on the scale S (EPI_F_H2OUT): split8_h2's
// split, so a consumer reading the planes gets the fragments it would split
// from the f32 values on that scale.
__device__ inline void split4_h2(const f32x4& v, float S, u32x2& hi, u32x2& lo) {
  unsigned h0, l0, h1, l1;
  h2_pair(v[0], v[1], S, h0, l0);
  h2_pair(v[2], v[3], S, h1, l1);
  hi = (u32x2){h0, h1};
  lo = (u32x2){l0, l1};
}

// The bound B >= max|y| of an EPI_F_H2OUT conv output (GemmParams::h2o_*)
__device__ inline float h2o_bound(const GemmParams& p) {
  return p.h2o_bw * amax_read(p.h2o_in) + p.h2o_bb;
}

// The three terms with the operands swapped as in mfma16_x3t (weights as the
// MFMA "A": transposed accumulator), fixed order b0 a0, b1 a0, b0 a1.
__device__ inline f32x4 mfma16_h2t(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4 c) {
  c = mfma16_f16(__builtin_bit_cast(f16x8, b[0]), __builtin_bit_cast(f16x8, a[0]), c);
  c = mfma16_f16(__builtin_bit_cast(f16x8, b[1]), __builtin_bit_cast(f16x8, a[0]), c);
  c = mfma16_f16(__builtin_bit_cast(f16x8, b[0]), __builtin_bit_cast(f16x8, a[1]), c);
  return c;
}

// The A operand scale of an EPI_F_H2 launch: from the max of its activation
// tensor(s) (both operands of a fused-shortcut GEMM share one scale).
__device__ inline float h2_act_scale(const GemmParams& p, bool dual, float* inv) {
  float amx = amax_read(p.amax_a);
  if (dual) amx = fmaxf(amx, amax_read(p.amax_a2));
  return h2_scale_of(amx, inv);
}

// Distance epilogue from precomputed squared row norms (pps_row_sqnorm):
//   sqeuclid = (-2 q.g + |q|^2) + |g|^2 clamped at 0 [sqrt]; cosine = 1 - q.g/(|q||g|)
template <int BM, int BN, int WM, int WN>
__device__ inline void dist_epilogue(const GemmParams& p,
                                     f32x16 (&acc)[BM / WM / 32][BN / WN / 32], int m0, int n0,
                                     int wm, int wn, int r32, int h) {
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  float* __restrict__ out = p.out + (int64_t)m0 * p.ldo + n0;
  const int ldo = (int)p.ldo;
  const int mrem = p.M - m0;
  const int nrem = p.Ncol - n0;
  const float* qsq = p.norm_a + m0;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int c = wn * (BN / WN) + j * 32 + r32;
    if (c >= nrem) continue;
    const float gn = p.norm_b[n0 + c];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rb = wm * (BM / WM) + i * 32 + 4 * h;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int rr = rb + (r & 3) + 8 * (r >> 2);
        if (rr < mrem) {
          const float dot = acc[i][j][r];
          const float qn = qsq[rr];
          float v;
          if (p.metric == PPS_METRIC_COSINE) {
            const float den = fmaxf(sqrtf(qn), 1e-12f) * fmaxf(sqrtf(gn), 1e-12f);
            v = 1.f - dot / den;
          } else {
            v = fmaxf(__builtin_fmaf(-2.f, dot, qn) + gn, 0.f);
            if (p.metric == PPS_METRIC_EUCLIDEAN) v = sqrtf(v);
          }
          if (p.zero_diag && m0 + rr == n0 + c) v = 0.f;
          out[rr * ldo + c] = v;
        }
      }
    }
  }
}

}  // namespace pps
