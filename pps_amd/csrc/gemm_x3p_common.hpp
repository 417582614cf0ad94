// Device pieces of the LDS-DMA pipelined bf16x3 GEMMs (gemm_x3p.hip: im2col
// staged per K chunk; gemm_x3c.hip: 3x3 convs from an input patch staged
// once per channel chunk): the DMA piece, counted waits, the transposed
// six-term MFMA and the convolution epilogues.
#pragma once
#include "gemm_x3_common.hpp"

namespace pps {

typedef __attribute__((address_space(3))) void lds_void_t;

// One DMA piece: lane l's 16 bytes at buffer offset voff land at
// lds_dst + 16 * l (lds_dst wave-uniform -> M0).
__device__ inline void glds16(rsrc_t r, const unsigned char* lds_dst, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)(uintptr_t)lds_dst, 16, voff, 0, 0,
                                           0);
}

template <int N>
__device__ inline void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// The six terms with the MFMA operands swapped (weights as the MFMA "A"):
// the accumulator then holds the TRANSPOSED 32x32 block, i.e. lane l keeps
// output row (l & 31) and, in register r = 4q + e, output column
// 8q + 4(l >> 5) + e -- four consecutive columns per q, so the epilogue
// moves 16-byte vectors (4 stores per block instead of 16).  Same products,
// same term order.
__device__ inline f32x16 mfma_x3t(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 c) {
  if constexpr (PPS_X3_ORDER == 1) {
    c = mfma_bf16(b[0], a[0], c);
    c = mfma_bf16(b[0], a[1], c);
    c = mfma_bf16(b[0], a[2], c);
    c = mfma_bf16(b[1], a[0], c);
    c = mfma_bf16(b[1], a[1], c);
    c = mfma_bf16(b[2], a[0], c);
    return c;
  }
  if constexpr (PPS_X3_ORDER == 2) {
    c = mfma_bf16(b[0], a[0], c);
    c = mfma_bf16(b[1], a[0], c);
    c = mfma_bf16(b[2], a[0], c);
    c = mfma_bf16(b[0], a[1], c);
    c = mfma_bf16(b[1], a[1], c);
    c = mfma_bf16(b[0], a[2], c);
    return c;
  }
  c = mfma_bf16(b[0], a[0], c);
  c = mfma_bf16(b[0], a[1], c);
  c = mfma_bf16(b[1], a[0], c);
  c = mfma_bf16(b[0], a[2], c);
  c = mfma_bf16(b[1], a[1], c);
  c = mfma_bf16(b[2], a[0], c);
  return c;
}

// grouped tile order of the distance GEMMs: MB of query panels per group
#ifndef X3P_GM_MB
#define X3P_GM_MB 32
#endif

// Self-distance super-block: the least common multiple of the tile sides, so
// the upper triangle is enumerated by square blocks that whole tiles cover.
template <int BM, int BN>
constexpr int sym_block() {
  int a = BM, b = BN;
  while (b) { const int t = a % b; a = b; b = t; }
  return BM / a * BN;
}

template <int S> struct AccT { typedef f32x16 type; };
template <> struct AccT<16> { typedef f32x4 type; };

// Convolution epilogue on transposed accumulators (see mfma_x3t):
//   y = acc * scale + shift [+ residual] [ReLU]; DUAL: scale folded into the
//   weights; RAW: store acc; PLANES: write y as three bf16 planes (exact
//   split, 8-byte stores per plane).  Needs Ncol, ldo (and ldr) % 4 == 0
//   (x3p_eligible).
// S = MFMA block (32: 32x32x16, lane row l & 31, columns 8q + 4 (l >> 5) + e;
// 16: 16x16x32, lane row l & 15, columns 4 (l >> 4) + e); r32 = l % S,
// h = l / S.
template <int EPI, int BM, int BN, int WM, int WN, int S = 32>
__device__ inline void conv_epilogue_t(const GemmParams& p,
                                       typename AccT<S>::type (&acc)[BM / WM / S][BN / WN / S],
                                       int batch, int kslice, int m0, int n0, int wm, int wn,
                                       int r32, int h, float bnd_pre = 0.f,
                                       float inv_a_pre = 0.f) {
  constexpr int TM = BM / WM / S;
  constexpr int TN = BN / WN / S;
  constexpr int NQ = S * S / 256;  // 16-byte column groups per lane and block
  constexpr bool DUAL = (EPI & EPI_F_DUAL) != 0;
  constexpr bool HAS_RES = (EPI & EPI_F_RES) != 0;
  constexpr bool RELU = (EPI & EPI_F_RELU) != 0;
  constexpr bool RAW = (EPI & EPI_F_RAW) != 0;
  constexpr bool PLANES = (EPI & EPI_F_PLANES) != 0;
  constexpr bool H2 = (EPI & EPI_F_H2) != 0;
  constexpr bool H2O = (EPI & EPI_F_H2OUT) != 0;
  // f16x2 launches: the accumulators hold dot * 2^(s_a + s_w[col]); the
  // column scale takes 2^-(s_a + s_w) (exact: powers of two)
  float inv_a = 1.f;  // (inv_a_pre > 0: read by the kernel before its main loop)
  if (H2) {
    if (inv_a_pre > 0.f)
      inv_a = inv_a_pre;
    else
      h2_act_scale(p, DUAL, &inv_a);
  }
  float amx = 0.f;  // max |y| of this thread's outputs (p.amax_out)
  // f16x2 planes out: the bound (read by the kernel before its main loop,
  // h2o_bound) and its scale
  float so = 1.f, bnd = bnd_pre;
  if (H2O) {
    float inv;
    so = h2_scale_of(bnd, &inv);
  }
  const int64_t obase = batch * p.out_bstride + kslice * p.out_sstride + (int64_t)m0 * p.ldo + n0;
  float* __restrict__ out = (PLANES || H2O) ? nullptr : p.out + obase;
  uint16_t* __restrict__ out3 = (PLANES || H2O) ? p.out3 + obase : nullptr;
  const int ldo = (int)p.ldo;
  const int mrem = p.M - m0;
  const int nrem = p.Ncol - n0;
  const float* sc = (DUAL || RAW) ? nullptr : p.scale + batch * p.ss_bstride + n0;
  const float* sh = RAW ? nullptr : p.shift + batch * p.ss_bstride + n0;
  const float* res = HAS_RES ? p.residual + (int64_t)m0 * p.ldr + n0 : nullptr;
  const int ldr = (int)p.ldr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cb = wn * (BN / WN) + j * S + 4 * h;
    f32x4 s4[NQ], t4[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool ok = cb + 8 * q < nrem;
      s4[q] = (DUAL || RAW || !ok) ? (f32x4){1.f, 1.f, 1.f, 1.f}
                                   : *reinterpret_cast<const f32x4*>(sc + cb + 8 * q);
      t4[q] = (RAW || !ok) ? (f32x4){0.f, 0.f, 0.f, 0.f}
                           : *reinterpret_cast<const f32x4*>(sh + cb + 8 * q);
      if (H2 && ok) s4[q] = s4[q] * *reinterpret_cast<const f32x4*>(p.rs_b + n0 + cb + 8 * q) * inv_a;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rr = wm * (BM / WM) + i * S + r32;
      if (rr >= mrem) continue;
      f32x4 rv[NQ];
      if (HAS_RES) {
#pragma unroll
        for (int q = 0; q < NQ; ++q)
          rv[q] = cb + 8 * q < nrem ? *reinterpret_cast<const f32x4*>(res + rr * ldr + cb + 8 * q)
                                    : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (cb + 8 * q >= nrem) continue;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = RAW ? acc[i][j][4 * q + e] : __builtin_fmaf(acc[i][j][4 * q + e], s4[q][e], t4[q][e]);
          if (HAS_RES) v[e] += rv[q][e];
          if (RELU) v[e] = fmaxf(v[e], 0.f);
          amx = fmaxf(amx, fabsf(v[e]));
        }
        if (PLANES) {
          unsigned h0, m0_, l0, h1, m1, l1;
          split2(v[0], v[1], h0, m0_, l0);
          split2(v[2], v[3], h1, m1, l1);
          uint16_t* o = out3 + rr * ldo + cb + 8 * q;
          st_out2(o, (u32x2){h0, h1});
          st_out2(o + p.out_plane, (u32x2){m0_, m1});
          st_out2(o + 2 * p.out_plane, (u32x2){l0, l1});
        } else if (H2O) {
          u32x2 hi, lo;
          split4_h2(v, so, hi, lo);
          uint16_t* o = out3 + rr * ldo + cb + 8 * q;
          st_out2(o, hi);
          st_out2(o + p.out_plane, lo);
        } else {
          st_out4(out + rr * ldo + cb + 8 * q, v);
        }
      }
    }
  }
  if (p.amax_out) amax_commit(p.amax_out, H2O ? bnd : amx);
}

// One-launch conv split-K (EPI_F_FIX): park this K slice's raw accumulators
// as a dense [M][Ncol] partial tile, count the slice in with an agent-scope
// atomic after a release fence; the slice that arrives last (any slice) resets
// the counter, acquires, and reloads acc as part[0] + part[1] + ... in slice
// order -- the sums splitk_conv_epilogue_kernel forms, so the epilogue that
// follows gives its bits.  No workgroup waits on another (no spin), so
// residency does not matter.  Returns false in the slices that leave.
template <int BM, int BN, int WM, int WN, int S>
__device__ inline bool fix_reduce(const GemmParams& p,
                                  typename AccT<S>::type (&acc)[BM / WM / S][BN / WN / S],
                                  unsigned char* lds, int kslice, int tile_id, int m0, int n0,
                                  int wm, int wn, int r32, int h) {
  constexpr int TM = BM / WM / S, TN = BN / WN / S, NQ = S * S / 256;
  const int ld = p.Ncol;
  const int mrem = p.M - m0, nrem = p.Ncol - n0;
  float* base = p.part + (int64_t)m0 * ld + n0;
  auto each = [&](auto&& fn) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rr = wm * (BM / WM) + i * S + r32;
      if (rr >= mrem) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int cb = wn * (BN / WN) + j * S + 4 * h;
#pragma unroll
        for (int q = 0; q < NQ; ++q)
          if (cb + 8 * q < nrem) fn(i, j, q, (int64_t)rr * ld + cb + 8 * q);
      }
    }
  };
  float* mine = base + kslice * p.part_sstride;
  each([&](int i, int j, int q, int64_t o) {
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
    *reinterpret_cast<f32x4*>(mine + o) = v;
  });
#ifndef X3P_FIX_FENCE
#define X3P_FIX_FENCE 1  // probes only: 0 drops both fences (wrong results, fence cost)
#endif
  if (X3P_FIX_FENCE) __threadfence();  // release: this thread's partial stores before the count
  __syncthreads();  // every wave parked (and is done with the LDS stages)
  int* flag = reinterpret_cast<int*>(lds);
  if (threadIdx.x == 0) {
    const int old = atomicAdd(p.fix_cnt + tile_id, 1);
    const int last = old == p.splitk - 1;
    if (last) atomicExch(p.fix_cnt + tile_id, 0);  // zero for the next launch
    *flag = last;
  }
  __syncthreads();
  if (!*flag) return false;
  if (X3P_FIX_FENCE) __threadfence();  // acquire: the other slices' partials
  each([&](int i, int j, int q, int64_t o) {
    f32x4 v = *reinterpret_cast<const f32x4*>(base + o);
    for (int s = 1; s < p.splitk; ++s) v += *reinterpret_cast<const f32x4*>(base + s * p.part_sstride + o);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[i][j][4 * q + e] = v[e];
  });
  return true;
}

// The same conv epilogue staged through LDS: the waves park their
// accumulators as a [BM][BN+4] f32 tile, then the workgroup walks it row by
// row, so scale/shift, the residual and the output move as whole contiguous
// rows (16 B per lane, consecutive lanes consecutive columns) instead of the
// accumulator layout's 32-64 B row pieces.  Same per-element arithmetic in
// the same order as conv_epilogue_t (identical bits).
template <int BM, int BN>
constexpr int lds_epi_bytes() { return BM * (BN + 4) * 4; }
#ifndef X3P_PPS_ABL
#define X3P_PPS_ABL 0  // probes only: 1 = no strip pooling, 2 = no subsets, 3 = neither
#endif
#ifndef X3P_RES_PREFETCH
#define X3P_RES_PREFETCH 16  // residual vectors per thread requested early (0: off)
#endif

// HB column passes: the fused part pooling of a tile too wide for one
// [BM][BN+4] LDS image (192 x 256) parks, finishes and pools BN / HB columns
// at a time -- per element the same arithmetic in the same order.
template <int EPI, int BM, int BN, int WM, int WN, int S, int HB = 1>
__device__ inline void conv_epilogue_lds(const GemmParams& p,
                                         typename AccT<S>::type (&acc)[BM / WM / S][BN / WN / S],
                                         unsigned char* lds, int batch, int kslice, int m0,
                                         int n0, int wm, int wn, int r32, int h,
                                         float bnd_pre = 0.f, float inv_a_pre = 0.f) {
  constexpr int TM = BM / WM / S, TN = BN / WN / S, NQ = S * S / 256;
  constexpr int BNH = BN / HB;  // columns per pass
  constexpr int LD = BNH + 4;
  constexpr int NT = 64 * WM * WN;
  constexpr bool DUAL = (EPI & EPI_F_DUAL) != 0;
  constexpr bool HAS_RES = (EPI & EPI_F_RES) != 0;
  constexpr bool RELU = (EPI & EPI_F_RELU) != 0;
  constexpr bool PPS = (EPI & EPI_F_PPS) != 0;
  constexpr bool H2 = (EPI & EPI_F_H2) != 0;
  constexpr bool H2O = (EPI & EPI_F_H2OUT) != 0;
  static_assert(HB == 1 || (PPS && (BN / WN) % S == 0 && BNH % (BN / WN) == 0),
                "column passes: PPS tiles whose wave columns fall in one pass");
  static_assert(!(H2O && PPS), "f16x2 planes out: plain conv epilogues");
  float inv_a = 1.f;  // f16x2: see conv_epilogue_t
  if (H2) {
    if (inv_a_pre > 0.f)
      inv_a = inv_a_pre;
    else
      h2_act_scale(p, DUAL, &inv_a);
  }
  float amx = 0.f;
  float so = 1.f, bnd = bnd_pre;  // f16x2 planes out: see conv_epilogue_t
  if (H2O) {
    float inv;
    so = h2_scale_of(bnd, &inv);
  }
  float* t = reinterpret_cast<float*>(lds);
  const int64_t obase = batch * p.out_bstride + kslice * p.out_sstride + (int64_t)m0 * p.ldo + n0;
  const int ldo = (int)p.ldo;
  const int mrem = p.M - m0;
  const int ldr = (int)p.ldr;
  constexpr int C4 = BNH / 4;
  // the residual tile is requested before the accumulators are parked, so
  // its HBM latency overlaps the LDS round trip (up to 8 vectors per thread)
  constexpr int IT = (BM * C4) / NT;
  constexpr bool PRE = HAS_RES && (BM * C4) % NT == 0 && IT <= X3P_RES_PREFETCH;
#pragma unroll
  for (int hb = 0; hb < HB; ++hb) {
    const int c0h = hb * BNH;
    float* __restrict__ out = H2O ? nullptr : p.out + obase + c0h;
    uint16_t* __restrict__ out3 = H2O ? p.out3 + obase + c0h : nullptr;
    const int nrem = p.Ncol - n0 - c0h;
    const float* sc = DUAL ? nullptr : p.scale + batch * p.ss_bstride + n0 + c0h;
    const float* sh = p.shift + batch * p.ss_bstride + n0 + c0h;
    const float* res = HAS_RES ? p.residual + (int64_t)m0 * p.ldr + n0 + c0h : nullptr;
    f32x4 rpre[PRE ? IT : 1];
    if constexpr (PRE) {
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int idx = it * NT + threadIdx.x;
        const int row = idx / C4, col = 4 * (idx - row * C4);
        rpre[it] = (row < mrem && col < nrem)
                       ? *reinterpret_cast<const f32x4*>(res + row * ldr + col)
                       : (f32x4){0.f, 0.f, 0.f, 0.f};
      }
    }
    __syncthreads();  // every wave is done reading the last stage / the last pass
    const int wc0 = wn * (BN / WN);  // this wave's first column (wave-uniform)
    if (HB == 1 || (wc0 >= c0h && wc0 < c0h + BNH)) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int rr = wm * (BM / WM) + i * S + r32;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int cb = wc0 + j * S + 4 * h - c0h;
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
            *reinterpret_cast<f32x4*>(t + rr * LD + cb + 8 * q) = v;
          }
        }
      }
    }
    __syncthreads();
    auto finish = [&](int idx, const f32x4& rv) {
      const int row = idx / C4, col = 4 * (idx - row * C4);
      if (row >= mrem || col >= nrem) return;
      const f32x4 a = *reinterpret_cast<const f32x4*>(t + row * LD + col);
      f32x4 s4 = DUAL ? (f32x4){1.f, 1.f, 1.f, 1.f} : *reinterpret_cast<const f32x4*>(sc + col);
      if (H2) s4 = s4 * *reinterpret_cast<const f32x4*>(p.rs_b + n0 + c0h + col) * inv_a;
      const f32x4 t4 = *reinterpret_cast<const f32x4*>(sh + col);
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = __builtin_fmaf(a[e], s4[e], t4[e]);
        if (HAS_RES) v[e] += rv[e];
        if (RELU) v[e] = fmaxf(v[e], 0.f);
        amx = fmaxf(amx, fabsf(v[e]));
      }
      if (PPS) {  // the pooling below reads the tile back from LDS
        *reinterpret_cast<f32x4*>(t + row * LD + col) = v;
        if (p.pps_write_y) st_out4(out + row * ldo + col, v);
      } else if (H2O) {
        u32x2 hi, lo;
        split4_h2(v, so, hi, lo);
        st_out2(out3 + row * ldo + col, hi);
        st_out2(out3 + row * ldo + col + p.out_plane, lo);
      } else {
        st_out4(out + row * ldo + col, v);
      }
    };
    if constexpr (H2O) {
      // f16x2 planes out: eight columns per lane, so each plane leaves as
      // 16-byte stores (whole rows across the wave); no residual here
      static_assert(!HAS_RES && !PPS && C4 % 2 == 0, "f16x2 planes out: plain conv tiles");
      constexpr int C8 = C4 / 2;
      for (int idx = threadIdx.x; idx < BM * C8; idx += NT) {
        const int row = idx / C8, col = 8 * (idx - row * C8);
        if (row >= mrem || col >= nrem) continue;
        u32x4 hw, lw;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          const int c = col + 4 * g;
          const f32x4 a = *reinterpret_cast<const f32x4*>(t + row * LD + c);
          f32x4 s4 = DUAL ? (f32x4){1.f, 1.f, 1.f, 1.f} : *reinterpret_cast<const f32x4*>(sc + c);
          if (H2) s4 = s4 * *reinterpret_cast<const f32x4*>(p.rs_b + n0 + c0h + c) * inv_a;
          const f32x4 t4 = *reinterpret_cast<const f32x4*>(sh + c);
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = __builtin_fmaf(a[e], s4[e], t4[e]);
            if (RELU) v[e] = fmaxf(v[e], 0.f);
            amx = fmaxf(amx, fabsf(v[e]));
          }
          u32x2 hi, lo;
          split4_h2(v, so, hi, lo);
          hw[2 * g] = hi[0];
          hw[2 * g + 1] = hi[1];
          lw[2 * g] = lo[0];
          lw[2 * g + 1] = lo[1];
        }
        uint16_t* o = out3 + row * ldo + col;
        if (col + 4 < nrem && ((ldo | p.out_plane) & 7) == 0) {
          *reinterpret_cast<u32x4*>(o) = hw;
          *reinterpret_cast<u32x4*>(o + p.out_plane) = lw;
        } else {
          st_out2(o, (u32x2){hw[0], hw[1]});
          st_out2(o + p.out_plane, (u32x2){lw[0], lw[1]});
          if (col + 4 < nrem) {
            st_out2(o + 4, (u32x2){hw[2], hw[3]});
            st_out2(o + 4 + p.out_plane, (u32x2){lw[2], lw[3]});
          }
        }
      }
    } else if constexpr (PRE) {
#pragma unroll
      for (int it = 0; it < IT; ++it) finish(it * NT + threadIdx.x, rpre[it]);
    } else {
      for (int idx = threadIdx.x; idx < BM * C4; idx += NT) {
        f32x4 rv = {0.f, 0.f, 0.f, 0.f};
        if (HAS_RES) {
          const int row = idx / C4, col = 4 * (idx - row * C4);
          if (row < mrem && col < nrem) rv = *reinterpret_cast<const f32x4*>(res + row * ldr + col);
        }
        finish(idx, rv);
      }
    }
    if constexpr (PPS) {
      // The tile is one image (BM = Ho * Wo rows, row-major positions) x BNH
      // channels.  Per (strip, channel): sum and max over the strip's rows in
      // row-major order, then the 2^S - 1 subsets -- the arithmetic of
      // part_power_set_v3_kernel (feature_ops.hip), so the bits are the same.
      __syncthreads();
      float* s_ave = t + BM * LD;
      float* s_max = s_ave + kPpsFuseMaxStrips * BNH;
      // (work split by whole waves: the strip / subset group is wave-uniform,
      // so the strip table is read with scalar loads)
      const int W = p.Wo, NS5 = p.pps_S;
      constexpr int CB = BNH / 64;  // 64-channel slices per pass
      static_assert(BNH % 64 == 0, "fused pooling: BN / HB must be a multiple of 64");
      const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
      const int ln = threadIdx.x & 63;
      for (int it = wv; it < ((X3P_PPS_ABL & 1) ? 0 : NS5 * CB); it += NT / 64) {
        const int j = it / CB, c = (it - j * CB) * 64 + ln;
        int r0 = 0;
        for (int q = 0; q < j; ++q) r0 += p.pps_h[q];
        const int cnt = p.pps_h[j] * W;
        const float* colp = t + (r0 * W) * LD + c;
        float sum = 0.f, mx = -INFINITY;
#pragma unroll 16
        for (int e = 0; e < cnt; ++e) {
          const float v = colp[e * LD];
          sum += v;
          mx = fmaxf(mx, v);
        }
        s_ave[j * BNH + c] = sum / (float)cnt;
        s_max[j * BNH + c] = mx;
      }
      __syncthreads();
      // subsets.  S <= 5 (Market: 5 strips): one lane per channel builds all
      // 2^S - 1 subsets in increasing order, each from the subset without its
      // highest strip plus that strip -- the same ascending-order sum as the
      // standalone kernel, one add and one max per subset.  Larger S: thread
      // (channel, group of 8 subsets) with the standalone loop.
      const int img = m0 / (p.Ho * p.Wo);
      const int nsub = (1 << NS5) - 1;
      float* po = p.pps_out + (int64_t)img * p.Ncol + n0 + c0h;
      const int64_t sub_stride = (int64_t)p.pps_nimg * p.Ncol;
      if (NS5 <= 5) {
        for (int o = wv; o < ((X3P_PPS_ABL & 2) ? 0 : CB); o += NT / 64) {
          const int cc = o * 64 + ln;
          if (cc >= nrem) continue;
          float av[5], mv[5], ss[32], sm[32];
#pragma unroll
          for (int q = 0; q < 5; ++q) {
            av[q] = q < NS5 ? s_ave[q * BNH + cc] : 0.f;
            mv[q] = q < NS5 ? s_max[q * BNH + cc] : 0.f;
          }
#pragma unroll
          for (int i = 1; i < 32; ++i) {
            const int top = 31 - __builtin_clz(i), rest = i & ~(1 << top);
            ss[i] = rest ? ss[rest] + av[top] : av[top];
            sm[i] = rest ? fmaxf(sm[rest], mv[top]) : mv[top];
            if (i <= nsub) {
              const float v = p.pps_max_ave
                                  ? ss[i] * (1.f / (float)__builtin_popcount(i)) + sm[i]
                                  : 0.f;
              if (p.pps_max_ave) po[(int64_t)(i - 1) * sub_stride + cc] = v;
            }
          }
          if (!p.pps_max_ave) {  // Max-only: the max of the strip averages
            float mx[32];
#pragma unroll
            for (int i = 1; i < 32; ++i) {
              const int top = 31 - __builtin_clz(i), rest = i & ~(1 << top);
              mx[i] = rest ? fmaxf(mx[rest], av[top]) : av[top];
              if (i <= nsub) po[(int64_t)(i - 1) * sub_stride + cc] = mx[i];
            }
          }
        }
      } else {
        const int ngrp = (nsub + 7) / 8;
        for (int o = wv; o < ((X3P_PPS_ABL & 2) ? 0 : ngrp * CB); o += NT / 64) {
          const int g = o / CB, cc = (o - g * CB) * 64 + ln;
          if (cc >= nrem) continue;
          float av[kPpsFuseMaxStrips], mv[kPpsFuseMaxStrips];
#pragma unroll
          for (int q = 0; q < kPpsFuseMaxStrips; ++q) {
            av[q] = q < NS5 ? s_ave[q * BNH + cc] : 0.f;
            mv[q] = q < NS5 ? s_max[q * BNH + cc] : 0.f;
          }
          for (int i = 8 * g + 1; i <= 8 * g + 8 && i <= nsub; ++i) {
            float v;
            if (p.pps_max_ave) {
              float sm = 0.f, mx = -INFINITY;
              int k = 0;
              bool first = true;
#pragma unroll
              for (int q = 0; q < kPpsFuseMaxStrips; ++q)
                if (q < NS5 && (i & (1 << q))) {
                  sm = first ? av[q] : sm + av[q];
                  first = false;
                  mx = fmaxf(mx, mv[q]);
                  ++k;
                }
              v = sm * (1.f / (float)k) + mx;
            } else {
              float mx = -INFINITY;
#pragma unroll
              for (int q = 0; q < kPpsFuseMaxStrips; ++q)
                if (q < NS5 && (i & (1 << q))) mx = fmaxf(mx, av[q]);
              v = mx;
            }
            po[(int64_t)(i - 1) * sub_stride + cc] = v;
          }
        }
      }
    }
  }
  if (p.amax_out) amax_commit(p.amax_out, H2O ? bnd : amx);
}

// The distance epilogue staged through LDS (not for self-distance tiles,
// which also write their mirror): the dot products are parked as a
// [BM][BN+4] f32 tile and the workgroup then writes whole output rows, 16 B
// per lane with consecutive lanes on consecutive columns, so each store
// instruction covers full 64-256 B row segments instead of 16-B pieces of 16-32
// rows (PMC: the direct epilogue wrote 1.56x the matrix).  Same per-element
// formulas as dist_epilogue_t (identical bits).
template <int BM, int BN, int WM, int WN, int S>
__device__ inline void dist_epilogue_lds(const GemmParams& p,
                                         typename AccT<S>::type (&acc)[BM / WM / S][BN / WN / S],
                                         unsigned char* lds, int m0, int n0, int wm, int wn,
                                         int r32, int h) {
  constexpr int TM = BM / WM / S, TN = BN / WN / S, NQ = S * S / 256;
  constexpr int LD = BN + 4;
  constexpr int NT = 64 * WM * WN;
  float* t = reinterpret_cast<float*>(lds);
  __syncthreads();  // every wave is done reading the last stage
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rr = wm * (BM / WM) + i * S + r32;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cb = wn * (BN / WN) + j * S + 4 * h;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
        *reinterpret_cast<f32x4*>(t + rr * LD + cb + 8 * q) = v;
      }
    }
  }
  __syncthreads();
  float* __restrict__ out = p.out + (int64_t)m0 * p.ldo + n0;
  const int ldo = (int)p.ldo;
  const int mrem = p.M - m0, nrem = p.Ncol - n0;
  const bool vec = (p.ldo & 3) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  constexpr int C4 = BN / 4;
  for (int idx = threadIdx.x; idx < BM * C4; idx += NT) {
    const int row = idx / C4, col = 4 * (idx - row * C4);
    if (row >= mrem || col >= nrem) continue;
    const f32x4 a = *reinterpret_cast<const f32x4*>(t + row * LD + col);
    const float qn = p.norm_a[m0 + row];
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gn = col + e < nrem ? p.norm_b[n0 + col + e] : 0.f;
      const float dot = a[e];
      float d;
      if (p.metric == PPS_METRIC_COSINE) {
        const float den = fmaxf(sqrtf(qn), 1e-12f) * fmaxf(sqrtf(gn), 1e-12f);
        d = 1.f - dot / den;
      } else {
        d = fmaxf(__builtin_fmaf(-2.f, dot, qn) + gn, 0.f);
        if (p.metric == PPS_METRIC_EUCLIDEAN) d = sqrtf(d);
      }
      if (p.zero_diag && m0 + row == n0 + col + e) d = 0.f;
      v[e] = d;
    }
    float* o = out + row * ldo + col;
    if (vec && col + 3 < nrem) {
      *reinterpret_cast<f32x4*>(o) = v;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (col + e < nrem) o[e] = v[e];
    }
  }
}

// One distance from a dot product and the two squared norms (the formulas
// of dist_epilogue / dist_epilogue_lds, factored out for the symmetric
// epilogue: same operations in the same order).
__device__ inline float dist_value(const GemmParams& p, float dot, float qn, float gn) {
  float d;
  if (p.metric == PPS_METRIC_COSINE) {
    const float den = fmaxf(sqrtf(qn), 1e-12f) * fmaxf(sqrtf(gn), 1e-12f);
    d = 1.f - dot / den;
  } else {
    d = fmaxf(__builtin_fmaf(-2.f, dot, qn) + gn, 0.f);
    if (p.metric == PPS_METRIC_EUCLIDEAN) d = sqrtf(d);
  }
  return d;
}

// Self-distance epilogue through LDS: the tile's dot products are parked as
// [BM][BN+4]; pass 1 writes the elements on or above the diagonal (global
// row <= column) as whole row segments and leaves the finished distances in
// LDS; pass 2 writes the strictly-upper ones a second time at the mirrored
// position, walking the tile by columns so that each store is 16 bytes of
// one output row (4 consecutive tile rows).  Elements below the diagonal are
// the mirror of another tile of the same diagonal super-block.  The mirror
// is a copy, so the matrix is exactly symmetric; the upper triangle has the
// bits of the full (non-symmetric) product on the same tile.
template <int BM, int BN, int WM, int WN, int S>
__device__ inline void dist_epilogue_sym_lds(const GemmParams& p,
                                             typename AccT<S>::type (&acc)[BM / WM / S][BN / WN / S],
                                             unsigned char* lds, int m0, int n0, int wm, int wn,
                                             int r32, int h) {
  constexpr int TM = BM / WM / S, TN = BN / WN / S, NQ = S * S / 256;
  constexpr int LD = BN + 4;
  constexpr int NT = 64 * WM * WN;
  float* t = reinterpret_cast<float*>(lds);
  __syncthreads();  // every wave is done reading the last stage
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rr = wm * (BM / WM) + i * S + r32;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cb = wn * (BN / WN) + j * S + 4 * h;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][4 * q + e];
        *reinterpret_cast<f32x4*>(t + rr * LD + cb + 8 * q) = v;
      }
    }
  }
  __syncthreads();
  float* __restrict__ out = p.out;
  const int64_t ldo = p.ldo;
  const int mrem = p.M - m0, nrem = p.Ncol - n0;
  const bool vec = (ldo & 3) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
                   (m0 & 3) == 0 && (n0 & 3) == 0;
  constexpr int C4 = BN / 4;
  for (int idx = threadIdx.x; idx < BM * C4; idx += NT) {
    const int row = idx / C4, col = 4 * (idx - row * C4);
    if (row >= mrem || col >= nrem) continue;
    const int gr = m0 + row, gc = n0 + col;
    const float qn = p.norm_a[gr];
    f32x4 a = *reinterpret_cast<const f32x4*>(t + row * LD + col);
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gn = col + e < nrem ? p.norm_b[gc + e] : 0.f;
      float d = dist_value(p, a[e], qn, gn);
      if (p.zero_diag && gr == gc + e) d = 0.f;
      v[e] = d;
    }
    *reinterpret_cast<f32x4*>(t + row * LD + col) = v;  // for the mirror pass
    float* o = out + (int64_t)gr * ldo + gc;
    if (vec && col + 3 < nrem && gr <= gc) {
      *reinterpret_cast<f32x4*>(o) = v;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (col + e < nrem && gr <= gc + e) o[e] = v[e];
    }
  }
  __syncthreads();
  constexpr int R4 = BM / 4;
  for (int idx = threadIdx.x; idx < BN * R4; idx += NT) {
    const int col = idx / R4, row = 4 * (idx - col * R4);
    if (col >= nrem || row >= mrem) continue;
    const int gc = n0 + col, gr = m0 + row;
    if (gr >= gc) continue;  // nothing strictly above the diagonal here
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = t[(row + e) * LD + col];
    float* o = out + (int64_t)gc * ldo + gr;   // out[gc][gr .. gr + 3]
    if (vec && row + 3 < mrem && gr + 3 < gc) {
      *reinterpret_cast<f32x4*>(o) = v;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (row + e < mrem && gr + e < gc) o[e] = v[e];
    }
  }
}

// Distance epilogue on transposed accumulators: same formulas as
// dist_epilogue; 16-byte stores when the output rows are 16-byte aligned.
// Self-distance tiles (p.sym) write the elements on or above the diagonal
// and mirror the strictly-upper ones (per element where the tile crosses
// the diagonal).
template <int BM, int BN, int WM, int WN, int S = 32>
__device__ inline void dist_epilogue_t(const GemmParams& p,
                                       typename AccT<S>::type (&acc)[BM / WM / S][BN / WN / S],
                                       int m0, int n0, int wm, int wn, int r32, int h) {
  constexpr int TM = BM / WM / S;
  constexpr int TN = BN / WN / S;
  constexpr int NQ = S * S / 256;
  float* __restrict__ out = p.out + (int64_t)m0 * p.ldo + n0;
  // strictly-upper tile of a self-distance: every element mirrored
  const bool mirror = p.sym && m0 + BM <= n0;
  // a tile crossing the diagonal: per element, global row <= column written,
  // strictly above also mirrored
  const bool diag = p.sym && !mirror;
  const int dmn = m0 - n0;
  float* __restrict__ outT = p.out + (int64_t)n0 * p.ldo + m0;
  const int ldo = (int)p.ldo;
  const int mrem = p.M - m0;
  const int nrem = p.Ncol - n0;
  const bool vec = (p.ldo & 3) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  const float* qsq = p.norm_a + m0;
  float qn[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rr = wm * (BM / WM) + i * S + r32;
    qn[i] = rr < mrem ? qsq[rr] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cb = wn * (BN / WN) + j * S + 4 * h;
    float gn[4 * NQ];
#pragma unroll
    for (int r = 0; r < 4 * NQ; ++r) {
      const int c = cb + 8 * (r >> 2) + (r & 3);
      gn[r] = c < nrem ? p.norm_b[n0 + c] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int rr = wm * (BM / WM) + i * S + r32;
      if (rr >= mrem) continue;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int c = cb + 8 * q;
        if (c >= nrem) continue;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float dot = acc[i][j][4 * q + e];
          float d;
          if (p.metric == PPS_METRIC_COSINE) {
            const float den =
                fmaxf(sqrtf(qn[i]), 1e-12f) * fmaxf(sqrtf(gn[4 * q + e]), 1e-12f);
            d = 1.f - dot / den;
          } else {
            d = fmaxf(__builtin_fmaf(-2.f, dot, qn[i]) + gn[4 * q + e], 0.f);
            if (p.metric == PPS_METRIC_EUCLIDEAN) d = sqrtf(d);
          }
          if (p.zero_diag && m0 + rr == n0 + c + e) d = 0.f;
          v[e] = d;
        }
        float* o = out + rr * ldo + c;
        if (diag) {  // a tile on the diagonal: its upper part, mirrored
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int cc = c + e;
            if (cc < nrem && rr + dmn <= cc) {
              o[e] = v[e];
              if (rr + dmn < cc) outT[cc * ldo + rr] = v[e];
            }
          }
          continue;
        }
        if (vec && c + 3 < nrem) {
          *reinterpret_cast<f32x4*>(o) = v;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (c + e < nrem) o[e] = v[e];
        }
        if (mirror) {  // out[n0 + c + e][m0 + rr]: consecutive lanes, consecutive rows
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (c + e < nrem) outT[(c + e) * ldo + rr] = v[e];
        }
      }
    }
  }
}

}  // namespace pps
