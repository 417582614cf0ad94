// Fused ResNet stem: conv1 7x7/2 pad 3 (3 -> 64 channels, no bias) + test-mode
// SpatialBN (folded scale/shift) + ReLU + MaxPool 3x3/2 pad 1, in one kernel
// (ResNet.py:246-256 basic_bn_stem).  The 64-channel conv output, the largest
// tensor of the network (batch 64: 201 MB), never reaches HBM.
//
// Workgroup = one image x kStemPR pooled rows = 2*kStemPR + 1 conv rows (the
// row shared with the neighbouring workgroup is recomputed).  The input rows
// it needs (4*kStemPR + 7 of them, all 128 columns, zero borders) are staged
// once in LDS as bf16x3 planes, channel-planar: [channel][plane][row][col].
//
// GEMM view per conv row: M = 64 pixels, N = 64 channels, K = 7 kh x 3 c x
// 8 kw = 168 (kw = 7 has zero weight) padded to 176 = 11 chunks of 16, so a
// lane's 8 consecutive K values are 8 consecutive input columns 2*ow-3 .. 2*ow+4
// of one (kh, c) row: 4 ds_read_b32 per plane (bf16 pairs at 4-byte-aligned
// offsets), no im2col gather and no split arithmetic in the loop.  Four waves
// each own a 32-pixel x 32-channel block (v_mfma_f32_32x32x16_bf16, six
// product terms a0b0 + a1b0 + a0b1 + a2b0 + a1b1 + a0b2 as every x3 GEMM),
// their B fragments (weights, 11 chunks x 3 planes) held in VGPRs for the
// whole workgroup.
//
// Epilogue per conv row: BN + ReLU into an LDS row buffer [64 px][64 ch], then
// each thread max-pools 3 pixels x 8 channels of it horizontally and keeps the
// vertical 3-row max in registers; a finished pooled row is stored as whole
// 256-byte pixel rows.  Padding never wins: post-ReLU values are >= 0, so a
// zero stands in for a padded position exactly.
#include "gemm_x3_common.hpp"

namespace pps {

#ifndef STEM_PAIR
#define STEM_PAIR 0  // 1: two conv rows per MFMA pass (measured slower: 129 vs 122 us)
#endif
#ifndef STEM_VARIANT
#define STEM_VARIANT 0  // probes only: 1 = no epilogue/pool, 2 = no MFMA, 3 = staging only
#endif
constexpr int kStemPR = 4;                    // pooled rows per workgroup
constexpr int kStemCR = 2 * kStemPR + 1;      // conv rows per workgroup
constexpr int kStemIR = 4 * kStemPR + 7;      // input rows staged in LDS
constexpr int kStemW = 128;                   // input width (REID.SCALE width)
constexpr int kStemWc = kStemW / 2;           // conv width
constexpr int kStemWp = kStemWc / 2;          // pooled width
constexpr int kStemCols = kStemW + 8;         // staged columns: 3 zero + 128 + 5 zero
constexpr int kStemCout = 64;
constexpr int kStemK = 176;                   // 21 (kh, c) groups x 8 kw, padded
constexpr int kStemChunks = kStemK / 16;
constexpr int kStemRowLd = kStemCout + 4;     // LDS row buffer stride (floats)
constexpr int kStemPlane = kStemIR * kStemCols;  // bf16 elements per (channel, plane)
constexpr int kStemTileBytes = 3 * 3 * kStemPlane * 2;
constexpr int kStemLdsBytes = kStemTileBytes + kStemWc * kStemRowLd * 4;

__global__ void __launch_bounds__(256, 2)
stem_conv_pool_x3_kernel(const float* __restrict__ x, int H, int tiles_h,
                         const uint16_t* __restrict__ w3, const float* __restrict__ scale,
                         const float* __restrict__ shift, float* __restrict__ y, int Hc,
                         int Hp, float* __restrict__ amax) {
  extern __shared__ __attribute__((aligned(16))) unsigned char slds[];
  float amx = 0.f;  // max of this thread's pooled outputs (ReLU: >= 0)
  uint16_t* tile = reinterpret_cast<uint16_t*>(slds);
  float* rowbuf = reinterpret_cast<float*>(slds + kStemTileBytes);
  const int n = blockIdx.x / tiles_h;
  const int ph0 = (blockIdx.x - n * tiles_h) * kStemPR;
  const int r0 = 4 * ph0 - 5;  // input row of LDS row 0
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // wave (mb, nb): conv pixels 32*mb .. 32*mb + 31 (lane row r32 = pixel
  // 32*mb + r32), channels 32*nb .. 32*nb + 31
  const int mb = wave & 1, nb = wave >> 1;
  const int r32 = lane & 31, h = lane >> 5;

  // ---- stage the input rows: f32 NHWC4 -> bf16x3 planes, channel-planar ----
  // (4 staged columns per item: 4 pixel loads, one 8-byte LDS store per
  // channel and plane)
  const float* xin = x + (int64_t)n * H * kStemW * 4;
  for (int e = threadIdx.x; e < kStemIR * (kStemCols / 4); e += 256) {
    const int rr = e / (kStemCols / 4), c4 = 4 * (e - rr * (kStemCols / 4));
    const int gr = r0 + rr;
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int gc = c4 + u - 3;
      v[u] = (gr >= 0 && gr < H && gc >= 0 && gc < kStemW)
                 ? *reinterpret_cast<const f32x4*>(xin + ((int64_t)gr * kStemW + gc) * 4)
                 : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      unsigned h01, m01, l01, h23, m23, l23;
      split2(v[0][c], v[1][c], h01, m01, l01);
      split2(v[2][c], v[3][c], h23, m23, l23);
      u32x2* t = reinterpret_cast<u32x2*>(tile + c * 3 * kStemPlane + rr * kStemCols + c4);
      t[0] = (u32x2){h01, h23};
      t[kStemPlane / 4] = (u32x2){m01, m23};
      t[kStemPlane / 2] = (u32x2){l01, l23};
    }
  }
  // ---- this lane's B fragments (weights) for all chunks -------------------
  bf16x8 b[kStemChunks][3];
  {
    const int co = 32 * nb + r32;
#pragma unroll
    for (int k = 0; k < kStemChunks; ++k)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        b[k][p] = *reinterpret_cast<const bf16x8*>(w3 + ((int64_t)p * kStemCout + co) * kStemK +
                                                    16 * k + 8 * h);
  }
  const float sc = scale[32 * nb + r32], sh = shift[32 * nb + r32];
  __syncthreads();

  // pooling ownership: pooled column pw, channels cg .. cg+7
  const int pw = threadIdx.x >> 3, cg = (threadIdx.x & 7) * 8;
  f32x4 cur0 = {0.f, 0.f, 0.f, 0.f}, cur1 = cur0;
  float* yimg = y + (int64_t)n * Hp * kStemWp * kStemCout;

  // A fragment of conv row i, chunk k: staged columns 2*ow .. 2*ow + 7 of
  // one (kh, c) row = four bf16 pairs at a 4-byte-aligned offset per plane
  const int ow = 32 * mb + r32;
  auto read_a = [&](int i, int k, bf16x8 (&a)[3]) {
    int g = 2 * k + h;     // (kh, c) group of this lane's 8 K values
    g = g < 21 ? g : 20;   // the pad group: any finite values (zero weights)
    const int kh = g / 3, c = g - 3 * kh;
    const uint16_t* src = tile + c * 3 * kStemPlane + (2 * i + kh) * kStemCols + 2 * ow;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      u32x4 u;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        u[j] = *reinterpret_cast<const unsigned*>(src + p * kStemPlane + 2 * j);
      a[p] = __builtin_bit_cast(bf16x8, u);
    }
  };

  for (int i0 = 0; i0 < kStemCR; i0 += STEM_PAIR ? 2 : 1) {
    // two conv rows per pass: two independent MFMA chains whose fragment
    // reads overlap each other's MFMAs (rows past the image compute on the
    // staged zeros and are discarded below)
    const bool pair = STEM_PAIR && i0 + 1 < kStemCR;
    f32x16 acc2[2] = {{}, {}};
    if (STEM_VARIANT != 3) {
#pragma unroll
      for (int k = 0; k < kStemChunks; ++k) {
        bf16x8 a0[3], a1[3];
        read_a(i0, k, a0);
        if (pair) read_a(i0 + 1, k, a1);
        if (STEM_VARIANT != 2) {
          acc2[0] = mfma_x3(a0, b[k], acc2[0]);
          if (pair) acc2[1] = mfma_x3(a1, b[k], acc2[1]);
        } else {
          acc2[0][0] += (float)a0[0][0] + (float)a0[1][1] + (float)a0[2][2];
        }
      }
    }
    for (int ii = 0; ii < (pair ? 2 : 1); ++ii) {
    const int i = i0 + ii;
    const f32x16 acc = acc2[ii];
    const int oh = 2 * ph0 - 1 + i;
    const bool row_ok = oh >= 0 && oh < Hc;
    if (STEM_VARIANT == 3) continue;
    if (row_ok) {
      if (STEM_VARIANT == 1) {
        if (acc[0] == 12345.f && acc[15] == 1.f) y[threadIdx.x] = acc[1];
        continue;
      }
      // BN + ReLU into the row buffer: lane holds channel 32nb + r32 of 16 pixels
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int px = 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * h;
        rowbuf[px * kStemRowLd + 32 * nb + r32] = fmaxf(__builtin_fmaf(acc[r], sc, sh), 0.f);
      }
    }
    __syncthreads();
    // horizontal 3-pixel max of this conv row (padded / missing rows: zeros)
    f32x4 h0 = {0.f, 0.f, 0.f, 0.f}, h1 = h0;
    if (row_ok) {
#pragma unroll
      for (int d = -1; d <= 1; ++d) {
        const int px = 2 * pw + d;
        if (px < 0 || px >= kStemWc) continue;
        const f32x4 v0 = *reinterpret_cast<const f32x4*>(rowbuf + px * kStemRowLd + cg);
        const f32x4 v1 = *reinterpret_cast<const f32x4*>(rowbuf + px * kStemRowLd + cg + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          h0[e] = fmaxf(h0[e], v0[e]);
          h1[e] = fmaxf(h1[e], v1[e]);
        }
      }
    }
    // conv row i = 2j is the top row of pooled row j and the bottom row of
    // pooled row j - 1; i = 2j + 1 is the middle row of pooled row j
    if ((i & 1) == 0) {
      if (i > 0) {
        const int ph = ph0 + i / 2 - 1;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          cur0[e] = fmaxf(cur0[e], h0[e]);
          cur1[e] = fmaxf(cur1[e], h1[e]);
        }
        if (ph < Hp) {
          float* o = yimg + ((int64_t)ph * kStemWp + pw) * kStemCout + cg;
          *reinterpret_cast<f32x4*>(o) = cur0;
          *reinterpret_cast<f32x4*>(o + 4) = cur1;
#pragma unroll
          for (int e = 0; e < 4; ++e) amx = fmaxf(amx, fmaxf(cur0[e], cur1[e]));
        }
      }
      cur0 = h0;
      cur1 = h1;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        cur0[e] = fmaxf(cur0[e], h0[e]);
        cur1[e] = fmaxf(cur1[e], h1[e]);
      }
    }
    __syncthreads();  // the row buffer is rewritten by the next conv row
    }
  }
  if (amax) amax_commit(amax, amx);
}

// ---------------------------------------------------------------------------
// Ring-staged variant (default): no LDS epilogue and one two-wave barrier per
// conv row.  Workgroup = 2 waves = the two 32-channel halves of kRingPR
// pooled rows of one image; each wave computes WHOLE conv rows (64 pixels =
// two 32x32 MFMA blocks, same K order and term order as above -> identical
// bits), so the horizontal 3-wide max needs only the partner lane (l ^ 32)
// and the vertical one stays in registers.  The input rows live in a ring of
// kRingSlots LDS rows: while conv row i is multiplied, the two input rows
// conv row i + 1 first needs are fetched into registers, then split and
// written into the slots conv row i - 1 released.  LDS layout
// [channel][slot][plane][column] keeps the three planes of a row within the
// ds_read2 offset range: one address per (chunk, lane) serves both pixel
// blocks and all three planes.  24 KB of LDS and <= 256 VGPRs: four
// workgroups (8 waves) per CU.
#ifndef RING_ABL
#define RING_ABL 0  // probes only, bit mask: 1 = no epilogue, 2 = no ring staging, 4 = no
                    // barrier, 8 = no MFMA, 16 = no fragment reads in the K loop
#endif
// Two floats scaled by S -> their f16x2 split as two packed f16 pairs
// (h2_pair: split8_h2's arithmetic), x S = hi + lo + r, |r| <= 2^-22 |x S|.
__device__ inline void split2_h2(float x0, float x1, float S, unsigned& hi, unsigned& lo) {
  h2_pair(x0, x1, S, hi, lo);
}

// The three f16x2 terms a0 b0 + a1 b0 + a0 b1 on v_mfma_f32_32x32x16_f16
// (fragments kept in bf16x8 storage, as the x3 ring's)
__device__ inline f32x16 mfma32_h2(const bf16x8 (&a)[3], const bf16x8 (&b)[2], f32x16 c) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, a[0]), __builtin_bit_cast(h8, b[0]), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, a[1]), __builtin_bit_cast(h8, b[0]), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(h8, a[0]), __builtin_bit_cast(h8, b[1]), c, 0, 0, 0);
  return c;
}

constexpr int kRingPR = 6;                    // pooled rows per workgroup
constexpr int kRingCR = 2 * kRingPR + 1;      // conv rows per workgroup
constexpr int kRingSlots = 10;                // 7 read by row i + 1 in flight + 2 written

#ifndef RING_STREAMS
#define RING_STREAMS 2  // row streams per workgroup (2: 4-wave workgroups)
#endif
constexpr int kRingThreads = 128 * RING_STREAMS;
#ifndef RING_CLK
#define RING_CLK 0
#endif

// H2: the f16x2 arithmetic (round 6) -- the input split into two f16 planes
// on the scale of its max (amax_in: the activation-max slot of the stem's
// input), two-plane f16 weights with per-channel inverse scales w_inv, three
// product terms (v_mfma_f32_32x32x16_f16) instead of six; the scales fold
// into the BN scale of the epilogue (exact powers of two).
template <bool H2>
__global__ void __launch_bounds__(kRingThreads, 2)
stem_ring_kernel(const float* __restrict__ x, int H, int tiles_h,
                 const uint16_t* __restrict__ w3, const float* __restrict__ scale,
                 const float* __restrict__ shift, float* __restrict__ y, int Hc, int Hp,
                 float* __restrict__ amax, const float* __restrict__ amax_in,
                 const float* __restrict__ w_inv) {
  constexpr int NP = H2 ? 2 : 3;             // planes per staged row
  constexpr int RR = NP * kStemCols;         // elements per (channel, slot)
  __shared__ __attribute__((aligned(16))) uint16_t ring[RING_STREAMS * 3 * kRingSlots * RR];
  float amx = 0.f;  // max of this thread's pooled outputs (ReLU: >= 0)
  float S = 1.f, inv_a = 1.f;  // f16x2: the input's scale 2^s and 2^-s
  if (H2) S = h2_scale_of(amax_read(amax_in), &inv_a);
  const int n = blockIdx.x / tiles_h;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nb = wid & 1;        // channel half
  const int stream = wid >> 1;   // row stream: its own pooled rows and ring
  uint16_t* tile = ring + stream * (3 * kRingSlots * RR);
  const int ph0 = (blockIdx.x - n * tiles_h) * (kRingPR * RING_STREAMS) + stream * kRingPR;
  const int r0 = 4 * ph0 - 5;  // input row of ring row ri = 0
  const int lane = threadIdx.x & 63;
  const int r32 = lane & 31, h = lane >> 5;
  const float* xin = x + (int64_t)n * H * kStemW * 4;

  // staged columns 0, 1 and 132..135 (input columns -3, -2, 129..132) stay zero
  for (int e = threadIdx.x; e < RING_STREAMS * 3 * NP * kRingSlots; e += kRingThreads) {
    uint16_t* row = ring + e * kStemCols;
    *reinterpret_cast<unsigned*>(row) = 0u;
    *reinterpret_cast<u32x2*>(row + kStemW + 4) = (u32x2){0u, 0u};
  }
  // staging of ring rows (ri, ri + 1): wave nb takes row ri + nb, lane l the
  // staged columns 2l + 2, 2l + 3 (input columns 2l - 1, 2l); lane 63 also
  // columns 130, 131 (input column 127 and the zero past the edge).  The
  // loads are unconditional (clamped addresses); masks zero them on the put.
  auto fetch = [&](int ri, f32x4& a, f32x4& b, f32x4& c, int& ok) {
    const int gr = r0 + ri + nb;
    const bool rok = gr >= 0 && gr < H;
    const float* src = xin + (int64_t)(rok ? gr : 0) * kStemW * 4;
    a = *reinterpret_cast<const f32x4*>(src + (lane > 0 ? 2 * lane - 1 : 0) * 4);
    b = *reinterpret_cast<const f32x4*>(src + 2 * lane * 4);
    // (a per-lane address: a uniform one becomes a scalar load, whose
    // lgkmcnt would hold up the first LDS fragment wait)
    c = *reinterpret_cast<const f32x4*>(src + (lane == 63 ? kStemW - 1 : 2 * lane) * 4);
    ok = rok ? ((lane > 0 ? 1 : 0) | 2 | (lane == 63 ? 4 : 0)) : 0;
  };
  auto put = [&](int ri, const f32x4& a, const f32x4& b, const f32x4& c, int ok) {
    const int slot = (ri + nb) % kRingSlots;
    unsigned* t = reinterpret_cast<unsigned*>(tile + slot * RR + 2 * lane + 2);
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      unsigned* tc = t + ch * (kRingSlots * RR / 2);
      if constexpr (H2) {
        unsigned hh, ll;
        split2_h2((ok & 1) ? a[ch] : 0.f, (ok & 2) ? b[ch] : 0.f, S, hh, ll);
        tc[0] = hh;
        tc[kStemCols / 2] = ll;
        if (lane == 63) {
          split2_h2((ok & 4) ? c[ch] : 0.f, 0.f, S, hh, ll);
          tc[1] = hh;
          tc[kStemCols / 2 + 1] = ll;
        }
      } else {
        unsigned hh, mm, ll;
        split2((ok & 1) ? a[ch] : 0.f, (ok & 2) ? b[ch] : 0.f, hh, mm, ll);
        tc[0] = hh;
        tc[kStemCols / 2] = mm;
        tc[kStemCols] = ll;
        if (lane == 63) {
          split2((ok & 4) ? c[ch] : 0.f, 0.f, hh, mm, ll);
          tc[1] = hh;
          tc[kStemCols / 2 + 1] = mm;
          tc[kStemCols + 1] = ll;
        }
      }
    }
  };
  {
    f32x4 a, b, c;
    int ok;
#pragma unroll 1
    for (int ri = 0; ri < 8; ri += 2) {  // rows 0..7: conv rows 0 and 1
      fetch(ri, a, b, c, ok);
      put(ri, a, b, c, ok);
    }
  }
  // this lane's B fragments (weights) for all chunks: channel 32 nb + r32
  bf16x8 b[kStemChunks][NP];
  const int co = 32 * nb + r32;
#pragma unroll
  for (int k = 0; k < kStemChunks; ++k)
#pragma unroll
    for (int p = 0; p < NP; ++p)
      b[k][p] = *reinterpret_cast<const bf16x8*>(w3 + ((int64_t)p * kStemCout + co) * kStemK +
                                                  16 * k + 8 * h);
  // (f16x2: the product carries 2^(s_a + s_w); BN scale times 2^-(s_a + s_w)
  // is exact, so fma(acc, sc', sh) rounds as fma(acc 2^-(s_a + s_w), sc, sh))
  const float sc = H2 ? scale[co] * (inv_a * w_inv[co]) : scale[co], sh = shift[co];
  __syncthreads();

  float cur[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) cur[q] = 0.f;
  float* yimg = y + (int64_t)n * Hp * kStemWp * kStemCout + co;
#if RING_CLK
  const uint64_t clk0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
#endif

#pragma unroll 1
  for (int i = 0; i < kRingCR; ++i) {
    const int rnext = 2 * i + 8;  // ring rows conv row i + 1 (and i + 2) first need
    f32x4 pa, pb, pc;
    int pok;
    if (!(RING_ABL & 2)) fetch(rnext, pa, pb, pc, pok);
    // keep the loads here: the scheduler would otherwise sink them to their
    // use after the MFMAs and expose their latency
    __builtin_amdgcn_sched_barrier(0);
    const int rs = (2 * i) % kRingSlots;  // slot of ring row 2 i (wave-uniform)
    f32x16 acc0 = {}, acc1 = {};
    // fragment reads one half-chunk ahead of the MFMAs: block 1 of chunk k
    // is read under block 0's terms, block 0 of chunk k + 1 under block 1's
    auto src_of = [&](int k) {
      // (kh, c) group of this lane's 8 K values: g = 2k + h (pad group 21
      // reads group 20, zero weights); both candidates are wave-uniform
      const int g0 = 2 * k, g1 = 2 * k + 1 < 21 ? 2 * k + 1 : 20;
      const int kh0 = g0 / 3, c0 = g0 - 3 * kh0, kh1 = g1 / 3, c1 = g1 - 3 * kh1;
      int s0 = rs + kh0, s1 = rs + kh1;
      s0 = s0 >= kRingSlots ? s0 - kRingSlots : s0;
      s1 = s1 >= kRingSlots ? s1 - kRingSlots : s1;
      const int o0 = (c0 * kRingSlots + s0) * RR, o1 = (c1 * kRingSlots + s1) * RR;
      return tile + (h ? o1 : o0) + 2 * r32;
    };
    auto frag = [&](const uint16_t* src, int blk, bf16x8 (&a)[3]) {
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        u32x4 u;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          u[j] = *reinterpret_cast<const unsigned*>(src + p * kStemCols + 32 * 2 * blk + 2 * j);
        a[p] = __builtin_bit_cast(bf16x8, u);
      }
    };
    bf16x8 fa[3], fb[3];
    frag(src_of(0), 0, fa);
    if (RING_ABL & 16) frag(src_of(0), 1, fb);
#pragma unroll
    for (int k = 0; k < kStemChunks; ++k) {
      // (sched_barrier: the scheduler would regroup the reads behind the
      // MFMAs that free their registers, exposing the LDS latency)
      if (!(RING_ABL & 16)) frag(src_of(k), 1, fb);
      __builtin_amdgcn_sched_barrier(0);
      if (RING_ABL & 8) asm volatile("" ::"v"(fa[0]), "v"(fa[1]), "v"(fa[2]));
      else if constexpr (H2) acc0 = mfma32_h2(fa, b[k], acc0);
      else acc0 = mfma_x3(fa, b[k], acc0);
      __builtin_amdgcn_sched_barrier(0);
      if (k + 1 < kStemChunks && !(RING_ABL & 16)) frag(src_of(k + 1), 0, fa);
      __builtin_amdgcn_sched_barrier(0);
      if (RING_ABL & 8) asm volatile("" ::"v"(fb[0]), "v"(fb[1]), "v"(fb[2]));
      else if constexpr (H2) acc1 = mfma32_h2(fb, b[k], acc1);
      else acc1 = mfma_x3(fb, b[k], acc1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // the loads' unused 4th lanes stay allocated until here, so no register
    // reuse forces an early wait on them
    if (!(RING_ABL & 2)) asm volatile("" ::"v"(pa), "v"(pb), "v"(pc));
    // (unconditional, also past the last ring row: the ring invariant keeps
    // those writes in free slots, and a conditional put lets the compiler
    // sink the loads into its branch, behind the MFMAs)
    if (!(RING_ABL & 2)) put(rnext, pa, pb, pc, pok);
    if (RING_ABL & 1) {
      asm volatile("" ::"v"(acc0), "v"(acc1));
      if (!(RING_ABL & 4)) __syncthreads();
      continue;
    }

    // BN + ReLU, horizontal 3-wide max: lane (r32, h) holds pixels
    // 32 blk + 8 t + 4 h + e (r = 4 t + e); pooled column 16 blk + 4 t + 2 h
    // takes the pixel before its run from the partner lane
    const int oh = 2 * ph0 - 1 + i;
    float hp[16];
    if (oh >= 0 && oh < Hc) {
      float v[2][16], pl[2][4];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        v[0][r] = fmaxf(__builtin_fmaf(acc0[r], sc, sh), 0.f);
        v[1][r] = fmaxf(__builtin_fmaf(acc1[r], sc, sh), 0.f);
      }
#pragma unroll
      for (int blk = 0; blk < 2; ++blk)
#pragma unroll
        for (int t = 0; t < 4; ++t) pl[blk][t] = __shfl_xor(v[blk][4 * t + 3], 32);
#pragma unroll
      for (int blk = 0; blk < 2; ++blk)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const float before = t > 0 ? pl[blk][t - 1] : (blk > 0 ? pl[0][3] : 0.f);
          const float xb = h ? pl[blk][t] : before;
          hp[8 * blk + 2 * t] = fmaxf(xb, fmaxf(v[blk][4 * t], v[blk][4 * t + 1]));
          hp[8 * blk + 2 * t + 1] =
              fmaxf(v[blk][4 * t + 1], fmaxf(v[blk][4 * t + 2], v[blk][4 * t + 3]));
        }
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) hp[q] = 0.f;  // padded / missing conv rows
    }
    // vertical: conv row i = 2j closes pooled row j - 1 and opens row j
    if ((i & 1) == 0) {
      if (i > 0) {
        const int ph = ph0 + i / 2 - 1;
        if (ph < Hp) {
          float* o = yimg + (int64_t)ph * kStemWp * kStemCout;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int pw = 16 * (q >> 3) + 4 * ((q >> 1) & 3) + 2 * h + (q & 1);
            const float v = fmaxf(cur[q], hp[q]);
            o[pw * kStemCout] = v;
            amx = fmaxf(amx, v);
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) cur[q] = hp[q];
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) cur[q] = fmaxf(cur[q], hp[q]);
    }
    if (!(RING_ABL & 4)) __syncthreads();  // ring rows written above are read by the next conv row
  }
#if RING_CLK  // diagnostic build: shader clocks and 100 MHz ticks of the loop -> y
  const uint64_t clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  if (threadIdx.x == 0) {
    y[2 * blockIdx.x] = (float)(clk1 - clk0);
    y[2 * blockIdx.x + 1] = (float)(rt1 - rt0);
  }
#endif
  if (amax) amax_commit(amax, amx);
}

static int g_stem_variant = 0;  // 0: ring-staged, 1: whole-tile staged + LDS epilogue

int stem_conv_pool_x3(const float* x, int N, int H, const uint16_t* w3, const float* scale,
                      const float* shift, float* y, int Hc, int Hp, hipStream_t st,
                      float* amax) {
  if (N <= 0) return PPS_OK;
  if (g_stem_variant == 0) {
    const int tiles_h = (Hp + kRingPR * RING_STREAMS - 1) / (kRingPR * RING_STREAMS);
    hipLaunchKernelGGL(stem_ring_kernel<false>, dim3((unsigned)(N * tiles_h)), dim3(kRingThreads),
                       0, st, x, H, tiles_h, w3, scale, shift, y, Hc, Hp, amax, nullptr, nullptr);
    PPS_CHECK_LAUNCH("stem_ring_kernel<x3>");
    return PPS_OK;
  }
  const int tiles_h = (Hp + kStemPR - 1) / kStemPR;
  hipLaunchKernelGGL(stem_conv_pool_x3_kernel, dim3((unsigned)(N * tiles_h)), dim3(256),
                     kStemLdsBytes, st, x, H, tiles_h, w3, scale, shift, y, Hc, Hp, amax);
  PPS_CHECK_LAUNCH("stem_conv_pool_x3_kernel");
  return PPS_OK;
}

// f16x2 stem (ring-staged kernel only): w2 = [2][64][kStemK] f16 planes of the
// packed weights, w_inv = their per-channel inverse scales, amax_in = the
// activation-max slot of x
int stem_conv_pool_h2(const float* x, int N, int H, const uint16_t* w2, const float* w_inv,
                      const float* scale, const float* shift, float* y, int Hc, int Hp,
                      hipStream_t st, float* amax, const float* amax_in) {
  if (N <= 0) return PPS_OK;
  const int tiles_h = (Hp + kRingPR * RING_STREAMS - 1) / (kRingPR * RING_STREAMS);
  hipLaunchKernelGGL(stem_ring_kernel<true>, dim3((unsigned)(N * tiles_h)), dim3(kRingThreads), 0,
                     st, x, H, tiles_h, w2, scale, shift, y, Hc, Hp, amax, amax_in, w_inv);
  PPS_CHECK_LAUNCH("stem_ring_kernel<h2>");
  return PPS_OK;
}

// Per output channel (one wave per row of the packed [64][kStemK] f32
// weights): max |w| -> 2^s (h2_scale_of), the planes f16(w 2^s) and
// f16(w 2^s - hi), and 2^-s.
__global__ void stem_split_h2_kernel(const float* __restrict__ w, uint16_t* __restrict__ w2,
                                     float* __restrict__ w_inv) {
  const int co = blockIdx.x, lane = threadIdx.x;
  const float* r = w + (int64_t)co * kStemK;
  float mx = 0.f;
  for (int k = lane; k < kStemK; k += 64) mx = fmaxf(mx, fabsf(r[k]));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  float inv;
  const float S = h2_scale_of(mx, &inv);
  for (int k = lane; k < kStemK; k += 64) {
    const float v = r[k] * S;
    const _Float16 hi = (_Float16)v, lo = (_Float16)(v - (float)hi);
    w2[(int64_t)co * kStemK + k] = __builtin_bit_cast(uint16_t, hi);
    w2[((int64_t)kStemCout + co) * kStemK + k] = __builtin_bit_cast(uint16_t, lo);
  }
  if (lane == 0) w_inv[co] = inv;
}

int stem_split_h2(const float* w, uint16_t* w2, float* w_inv, hipStream_t st) {
  hipLaunchKernelGGL(stem_split_h2_kernel, dim3(kStemCout), dim3(64), 0, st, w, w2, w_inv);
  PPS_CHECK_LAUNCH("stem_split_h2_kernel");
  return PPS_OK;
}

}  // namespace pps

using namespace pps;

extern "C" {

int pps_stem_k(void) { return kStemK; }

int pps_stem_variant(int v) {
  const int old = g_stem_variant;
  if (v == 0 || v == 1) g_stem_variant = v;
  return old;
}

int pps_stem_conv_pool_x3(const float* x, int N, int H, int W, const uint16_t* w3,
                          const float* scale, const float* shift, float* y, int Hp, int Wp,
                          void* stream) {
  PPS_ENFORCE(x && w3 && scale && shift && y, "null pointer");
  PPS_ENFORCE(W == kStemW, "the fused stem is built for input width " +
                               std::to_string(kStemW) + ", got " + std::to_string(W));
  PPS_ENFORCE(N >= 0 && H >= 7, "bad shape");
  const int Hc = (H + 2 * 3 - 7) / 2 + 1;
  PPS_ENFORCE(Hp == (Hc + 2 - 3) / 2 + 1 && Wp == kStemWp,
              "output must be the 3x3/2 pad 1 max pool of the 7x7/2 pad 3 conv");
  PPS_ENFORCE(aligned16(x) && aligned16(w3) && aligned16(y), "16-byte aligned pointers");
  PPS_ENFORCE((int64_t)N * H * W * 4 < (1ll << 31), "input larger than 2^31 floats");
  return stem_conv_pool_x3(x, N, H, w3, scale, shift, y, Hc, Hp, as_stream(stream), nullptr);
}

int pps_stem_split_h2(const float* w, uint16_t* w2, float* w_inv, void* stream) {
  PPS_ENFORCE(w && w2 && w_inv, "null pointer");
  return stem_split_h2(w, w2, w_inv, as_stream(stream));
}

int pps_stem_conv_pool_h2(const float* x, int N, int H, int W, const uint16_t* w2,
                          const float* w_inv, const float* amax_x, const float* scale,
                          const float* shift, float* y, int Hp, int Wp, void* stream) {
  PPS_ENFORCE(x && w2 && w_inv && amax_x && scale && shift && y, "null pointer");
  PPS_ENFORCE(W == kStemW, "the fused stem is built for input width " +
                               std::to_string(kStemW) + ", got " + std::to_string(W));
  PPS_ENFORCE(N >= 0 && H >= 7, "bad shape");
  const int Hc = (H + 2 * 3 - 7) / 2 + 1;
  PPS_ENFORCE(Hp == (Hc + 2 - 3) / 2 + 1 && Wp == kStemWp,
              "output must be the 3x3/2 pad 1 max pool of the 7x7/2 pad 3 conv");
  PPS_ENFORCE(aligned16(x) && aligned16(w2) && aligned16(y), "16-byte aligned pointers");
  PPS_ENFORCE((int64_t)N * H * W * 4 < (1ll << 31), "input larger than 2^31 floats");
  return stem_conv_pool_h2(x, N, H, w2, w_inv, scale, shift, y, Hc, Hp, as_stream(stream),
                           nullptr, amax_x);
}

}  // extern "C"
