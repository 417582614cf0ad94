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
                         int Hp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char slds[];
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
}

int stem_conv_pool_x3(const float* x, int N, int H, const uint16_t* w3, const float* scale,
                      const float* shift, float* y, int Hc, int Hp, hipStream_t st) {
  if (N <= 0) return PPS_OK;
  const int tiles_h = (Hp + kStemPR - 1) / kStemPR;
  hipLaunchKernelGGL(stem_conv_pool_x3_kernel, dim3((unsigned)(N * tiles_h)), dim3(256),
                     kStemLdsBytes, st, x, H, tiles_h, w3, scale, shift, y, Hc, Hp);
  PPS_CHECK_LAUNCH("stem_conv_pool_x3_kernel");
  return PPS_OK;
}

}  // namespace pps

using namespace pps;

extern "C" {

int pps_stem_k(void) { return kStemK; }

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
  return stem_conv_pool_x3(x, N, H, w3, scale, shift, y, Hc, Hp, as_stream(stream));
}

}  // extern "C"
