// Weight-stationary persistent GEMM for the thin-K 1x1 convolutions of the
// bottlenecks (GEMM tile id 54, GEMM_TILE_WS): branch2c of res2-res4
// (ResNet.py:320-332, K = 64 / 128 / 256, + BN + residual Sum + ReLU), the
// res2_0 branch2c with its projection shortcut K-concatenated
// (basic_bn_shortcut, ResNet.py:203-220; K = 64 + 64), and res2 branch2a
// (K = 256 / 64).
//
// These layers move 4-10 bytes of activations per MFMA-FLOP-worth of weights:
// res2 2c reads 50 MB of input and a 201 MB residual and writes 201 MB for
// 6.4 GFLOP, with K only two 32-wide chunks.  The tiled kernels spend most of
// each tile's life in its prologue and its epilogue (0.14 of the x3 roof,
// 4 TB/s).  Here a workgroup keeps one column block of the weights -- all K,
// BN2 columns, bf16x3 planes, 96 KB -- in LDS for its whole life and walks
// its share of the row tiles: each wave loads its activation rows and its
// residual vectors straight into registers, PD tiles ahead of the one it
// computes, runs
// the 16x16x32 MFMAs against the stationary weights and streams the result
// out.  No LDS staging of activations, no barrier after the weight load.
// Each wave owns 16 rows x 64 columns of a tile (4 MFMA column blocks: 16
// accumulator registers, so several tiles' operands fit beside them); BN2 /
// 64 waves share a row group, so a tile has 16 * 512 / BN2 rows.
//
// Arithmetic: the six terms of mfma16_x3t per 32-wide K chunk, chunks in
// order, then fma(acc, scale, shift) [+ residual] [ReLU] -- the S = 16
// pipelined tiles' sequence, so this tile's results equal theirs bit for bit.
// EPI_F_H2 (round 6): the f16x2 arithmetic of the pipelined kernel's
// PPS_TILE_H2 tiles -- activations split after the load on their tensor's
// power-of-two scale (split8_h2), the two chunk-tiled f16 weight planes in
// LDS (4 B per weight instead of 6, so a 256-column block of a K = 128
// layer fits and its activation rows are read once), the three terms of
// mfma16_h2t, the column scale (scale * 2^-s_w) * 2^-s_a in the epilogue:
// bit for bit the f16x2 pipelined tiles' results.
#include <cstdlib>

#include "gemm_x3_common.hpp"

namespace pps {

constexpr int kWsCUs = 256;  // MI355X compute units (one workgroup each)
constexpr int kWsLd = 64 + 4;  // epilogue scratch row (floats): 64 columns + bank padding
template <int BN2, int W> constexpr int ws_rows() { return 16 * W / (BN2 / 64); }

// NCH: 32-wide K chunks (K = 32 NCH); BN2: the stationary column block;
// W: waves per workgroup (8: two per SIMD -- 16 waves measured no faster).
template <int NCH, int BN2, int EPI, int W>
__global__ void __launch_bounds__(64 * W)
gemm_ws_kernel(GemmParams p, int n_cb, int n_rt, int rg) {
  constexpr int kWsWaves = W;
  // tiles in flight ahead of the one computing
  constexpr int PD = NCH <= 2 ? 3 : (NCH <= 4 ? 2 : 1);
  extern __shared__ __attribute__((aligned(16))) unsigned char ws_lds[];
  constexpr int TN = 4;              // 16-column MFMA blocks per wave (64 columns)
  constexpr int WC = BN2 / 64;       // waves across the column block
  constexpr int ROWS = ws_rows<BN2, W>();
  static_assert(BN2 % 64 == 0 && kWsWaves % WC == 0, "column block");
  constexpr bool HAS_RES = (EPI & EPI_F_RES) != 0;
  constexpr bool RELU = (EPI & EPI_F_RELU) != 0;
  constexpr bool DUAL = (EPI & EPI_F_DUAL) != 0;
  constexpr bool H2 = (EPI & EPI_F_H2) != 0;
  // f16x2 planes out (PPS_TILE_H2E producer): the two f16 planes its f16x2
  // reader would split, on the scale of the output bound (conv_epilogue_t)
  constexpr bool H2O = (EPI & EPI_F_H2OUT) != 0;
  static_assert(!H2O || (H2 && !HAS_RES && !DUAL), "planes out: f16x2 conv + BN + ReLU");
  constexpr int NBP = H2 ? 2 : 3;  // weight planes
  constexpr int WBYTES = NCH * NBP * BN2 * 64;  // weights: [chunk][plane][column][32 x 2 B]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r16 = lane & 15, h = lane >> 4;
  const int wr = wave / WC, wcol = 64 * (wave - wr * WC);  // row group, first column
  // f16x2: the workgroups of one row tile's column blocks on one XCD (their
  // activation rows shared through its L2)
  const int g = H2 ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int cb = g % n_cb;
  const int n0 = cb * BN2;
  float* s_sc = reinterpret_cast<float*>(ws_lds + WBYTES);
  float* s_sh = s_sc + BN2;

  // 1) this block's weight columns [n0, n0 + BN2) and scale / shift -> LDS;
  // 16-byte slot c of a column's 64-byte chunk row lands in slot
  // c ^ sw64(col), the pipelined kernel's B swizzle (gemm_common.hpp)
  // (f16x2: chunk-tiled planes [2][col / 16][K / 32][16][32], the layout the
  // pipelined tiles stream)
  for (int u = threadIdx.x; u < NCH * NBP * BN2 * 4; u += 64 * kWsWaves) {
    const int slot = u & 3;
    const int rest = u >> 2;
    const int col = rest % BN2;
    const int pk = rest / BN2;  // chunk * NBP + plane
    const int kc = pk / NBP, pl = pk - NBP * kc;
    const int gcol = n0 + col;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (gcol < p.Ncol) {
      const int64_t e = H2 ? ((int64_t)(gcol >> 4) * (p.ldb / 32) + kc) * 512 + (gcol & 15) * 32
                           : (int64_t)gcol * p.ldb + kc * 32;
      v = *reinterpret_cast<const u32x4*>(p.b3 + pl * p.b_plane + e + slot * 8);
    }
    *reinterpret_cast<u32x4*>(ws_lds + (pk * BN2 + col) * 64 + ((slot ^ sw64(col)) << 4)) = v;
  }
  // f16x2: the activations' scale 2^s_a (and 2^-s_a for the epilogue); planes
  // out: the output bound and its scale
  float h2s = 1.f, inv_a = 1.f, bnd = 0.f, so = 1.f;
  if constexpr (H2) h2s = h2_act_scale(p, DUAL, &inv_a);
  if constexpr (H2O) {
    float inv;
    bnd = h2o_bound(p);
    so = h2_scale_of(bnd, &inv);
  }
  for (int c = threadIdx.x; c < BN2; c += 64 * kWsWaves) {
    const bool ok = n0 + c < p.Ncol;
    float sc = (ok && !DUAL) ? p.scale[n0 + c] : 1.f;
    if (H2 && ok) sc = sc * p.rs_b[n0 + c] * inv_a;  // conv_epilogue_t's order
    s_sc[c] = sc;
    s_sh[c] = ok ? p.shift[n0 + c] : 0.f;
  }
  __syncthreads();

  // the wave's epilogue scratch and its lanes' (row layout) scale / shift
  float* wsc = reinterpret_cast<float*>(ws_lds + WBYTES + 2 * BN2 * 4) + wave * 16 * kWsLd;
  const f32x4 s4r = *reinterpret_cast<const f32x4*>(s_sc + wcol + 4 * (lane & 15));
  const f32x4 t4r = *reinterpret_cast<const f32x4*>(s_sh + wcol + 4 * (lane & 15));

  // 2) row tiles rt = g / n_cb + k * rg
  const rsrc_t ra = make_rsrc(p.a, p.a_bytes);
  const rsrc_t ra2 = DUAL ? make_rsrc(p.a2, p.a2_bytes) : ra;
  const rsrc_t rres = make_rsrc(HAS_RES ? p.residual : p.a,
                                HAS_RES ? (uint32_t)((int64_t)p.M * p.ldr * 4) : 0u);
  const rsrc_t rout = H2O ? make_rsrc(p.out3, (uint32_t)((p.out_plane + (int64_t)p.M * p.ldo) * 2))
                          : make_rsrc(p.out, (uint32_t)((int64_t)p.M * p.ldo * 4));
  const int nch1 = DUAL ? p.Kloop1 / 32 : NCH;
  const int rt0 = g / n_cb;
  const int my = rt0 < n_rt ? (n_rt - rt0 + rg - 1) / rg : 0;
  const int bsw = sw64(r16);
  const int hw = p.Ho * p.Wo;

  // One tile's operands of this lane: activation vectors (chunk kc, K
  // elements [32 kc + 8h, +8) of row 16 wr + r16) and residual vectors.
  // A ring of PD + 1 sets keeps PD tiles' loads in flight while one computes
  // (the kernel is bound by how many bytes a CU has in flight: ~2.5 us of
  // HBM latency x 25 GB/s per CU).
  struct Ops {
    f32x4 a[NCH][2];
    f32x4 r[HAS_RES ? 4 : 1];
  };
  // Every memory access is a buffer op whose offset is kOOB for a row past M
  // or a tile past this workgroup's share (loads read zero, stores are
  // dropped), so the loop has no branch around a memory op and the compiler
  // counts the loads in flight exactly (a conditional load or store makes it
  // wait for everything).
  float amx = 0.f;  // max |y| of this thread's outputs (p.amax_out)
  auto load = [&](int rt, bool valid, Ops& o) {
    const int m = rt * ROWS + wr * 16 + r16;
    const bool ok = valid && m < p.M;
    const int o1 = ok ? (m * p.lda + 8 * h) * 4 : kOOB;
    int o2 = kOOB;
    if (DUAL && ok) {  // 1x1 / stride2 shortcut operand at the output pixel
      const int n = m / hw, rem = m - n * hw, oh = rem / p.Wo, ow = rem - oh * p.Wo;
      o2 = (((n * p.H2 + oh * p.stride2) * p.W2 + ow * p.stride2) * p.lda2 + 8 * h) * 4;
    }
#pragma unroll
    for (int kc = 0; kc < NCH; ++kc) {
      const bool second = DUAL && kc >= nch1;
      const rsrc_t r = second ? ra2 : ra;
      const int base = second ? o2 : o1;
      const int off = base == kOOB ? kOOB : base + (second ? (kc - nch1) : kc) * 128;
      o.a[kc][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
      o.a[kc][1] = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off == kOOB ? kOOB : off + 16, 0, 0));
    }
    if constexpr (HAS_RES) {  // row layout (see process): 4 rows x 256 B per load
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        const int mr = rt * ROWS + wr * 16 + 4 * it + (lane >> 4);
        const int ro = (valid && mr < p.M) ? (mr * p.ldr + n0 + wcol + 4 * (lane & 15)) * 4 : kOOB;
        o.r[it] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rres, ro, 0, 0));
      }
    }
  };

  auto process = [&](int rt, bool valid, const Ops& o) {
    const int m = rt * ROWS + wr * 16 + r16;
    const bool ok = valid && m < p.M;
    f32x4 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < NCH; ++kc) {
      bf16x8 fa[3];
      if (H2)
        split8_h2(o.a[kc][0], o.a[kc][1], h2s, fa[0], fa[1]);
      else
        split8(o.a[kc][0], o.a[kc][1], fa[0], fa[1], fa[2]);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bf16x8 fb[3];
        const unsigned char* bp =
            ws_lds + ((kc * NBP) * BN2 + wcol + 16 * j + r16) * 64 + ((h ^ bsw) << 4);
#pragma unroll
        for (int pl = 0; pl < NBP; ++pl)
          fb[pl] = *reinterpret_cast<const bf16x8*>(bp + pl * BN2 * 64);
        acc[j] = H2 ? mfma16_h2t(fa, fb, acc[j]) : mfma16_x3t(fa, fb, acc[j]);
      }
      // one chunk's weight fragments live at a time (the compiler would hoist
      // every chunk's LDS reads and run out of registers)
      asm volatile("" ::: "memory");
    }
    // Epilogue in row layout: the wave parks its 16 x 64 accumulator block in
    // its own LDS scratch and reads it back so that lane l holds columns
    // 4 (l & 15) .. +3 of row 4 it + (l >> 4): every residual load and
    // output store then covers 4 whole 256-byte row segments (the
    // accumulator layout would scatter 64-byte pieces over 16 rows).  Wave-
    // private: LDS ops of one wave complete in order, no barrier.
    (void)ok;
#pragma unroll
    for (int j = 0; j < TN; ++j)
      *reinterpret_cast<f32x4*>(wsc + r16 * kWsLd + 16 * j + 4 * h) = acc[j];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int row = 4 * it + (lane >> 4);
      const f32x4 a = *reinterpret_cast<const f32x4*>(wsc + row * kWsLd + 4 * (lane & 15));
      const int mr = rt * ROWS + wr * 16 + row;
      const int oo = (valid && mr < p.M) ? (mr * (int)p.ldo + n0 + wcol + 4 * (lane & 15)) * 4 : kOOB;
      f32x4 v;
      float m4 = 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = __builtin_fmaf(a[e], s4r[e], t4r[e]);
        if (HAS_RES) v[e] += o.r[it][e];
        if (RELU) v[e] = fmaxf(v[e], 0.f);
        m4 = fmaxf(m4, fabsf(v[e]));
      }
      amx = oo != kOOB ? fmaxf(amx, m4) : amx;  // rows of this launch only
      if constexpr (H2O) {  // 2-byte elements: the f32 offset halved, plane 1 a plane further
        u32x2 hi, lo;
        split4_h2(v, so, hi, lo);
        const int oh = oo == kOOB ? kOOB : oo / 2;
        __builtin_amdgcn_raw_buffer_store_b64(hi, rout, oh, 0, kStAux);
        __builtin_amdgcn_raw_buffer_store_b64(lo, rout, oh == kOOB ? kOOB : oh + (int)(p.out_plane * 2),
                                              0, kStAux);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rout, oo, 0, kStAux);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next park
  };

  Ops ring[PD + 1];
#pragma unroll
  for (int u = 0; u < PD; ++u) load(rt0 + u * rg, u < my, ring[u]);
  const int iters = (my + PD) / (PD + 1) * (PD + 1);
  for (int i = 0; i < iters; i += PD + 1) {
#pragma unroll
    for (int u = 0; u <= PD; ++u) {
      const int t = i + u;
      load(rt0 + (t + PD) * rg, t + PD < my, ring[(u + PD) % (PD + 1)]);
      process(rt0 + t * rg, t < my, ring[u]);
    }
  }
  if (p.amax_out) amax_commit(p.amax_out, H2O ? bnd : amx);
}

// Shapes this kernel takes: a 1x1 / stride-1 / unpadded conv on f32 NHWC
// rows (+ the fused shortcut operand), K = 32 NCH with NCH in {2, 4, 8},
// f32 output, the conv epilogues C [| RELU] [| RES] [| DUAL].
bool ws_eligible(const GemmParams& p, int epi, int batch) {
  if (batch != 1 || p.splitk != 1 || p.ksplit_conv || p.a3 || !p.a || !p.b3 || p.sym) return false;
  // f16x2: chunk-tiled two-plane weights, their column scales and the inputs' maxima
  if ((epi & EPI_F_H2) && (!(p.tiled & 2) || !p.rs_b || !p.amax_a ||
                           ((epi & EPI_F_DUAL) && !p.amax_a2)))
    return false;
  if (!(epi & EPI_F_H2) && (p.tiled & 2)) return false;
  if (epi & (EPI_DIST | EPI_F_RAW | EPI_F_PLANES | EPI_F_PPS)) return false;
  // f16x2 planes out: an f16x2 conv + BN + ReLU, planes within the 2 GiB a
  // buffer resource addresses
  if ((epi & EPI_F_H2OUT) &&
      (!(epi & EPI_F_H2) || (epi & (EPI_F_RES | EPI_F_DUAL)) || !p.out3 || !p.h2o_in ||
       (reinterpret_cast<uintptr_t>(p.out3) & 7) || (p.out_plane + (int64_t)p.M * p.ldo) * 2 >= kMaxBufBytes ||
       p.out_plane * 2 >= (1ll << 31)))
    return false;
  if (p.KH != 1 || p.KW != 1 || p.stride != 1 || p.pad != 0 || p.H != p.Ho || p.W != p.Wo)
    return false;
  const int K = p.Kloop;
  if (K % 32 || (K != 64 && K != 128 && K != 256) || p.kb_valid < K || p.ldb % 8) return false;
  if (p.a2 ? (p.Kloop1 % 32 || p.lda2 % 4 || p.Cin != p.Kloop1) : p.Cin != K) return false;
  if (p.lda % 4 || p.Ncol % 64 || p.ldo % 4 || (reinterpret_cast<uintptr_t>(p.out) & 15)) return false;
  if (!(epi & EPI_F_H2OUT) && !p.out) return false;
  if (p.residual && (p.ldr % 4 || (reinterpret_cast<uintptr_t>(p.residual) & 15))) return false;
  if ((int64_t)p.M * p.lda * 4 >= kMaxBufBytes || (int64_t)p.M * p.ldo * 4 >= kMaxBufBytes ||
      (p.residual && (int64_t)p.M * p.ldr * 4 >= kMaxBufBytes))
    return false;
  return true;
}

template <int NCH, int BN2, int W>
constexpr size_t ws_lds_bytes(bool h2) {
  return (size_t)NCH * (h2 ? 2 : 3) * BN2 * 64 + 2 * BN2 * sizeof(float) +
         (size_t)W * 16 * kWsLd * sizeof(float);
}

template <int NCH, int BN2, int W>
static int launch_ws_cfg(const GemmParams& p, int epi, hipStream_t stream) {
  const int n_cb = (p.Ncol + BN2 - 1) / BN2;
  const int n_rt = (p.M + ws_rows<BN2, W>() - 1) / ws_rows<BN2, W>();
  const int rg = n_cb >= kWsCUs ? 1 : (kWsCUs / n_cb < n_rt ? kWsCUs / n_cb : n_rt);
  const size_t lds = ws_lds_bytes<NCH, BN2, W>((epi & EPI_F_H2) != 0);
  if (lds > 160 * 1024) {
    set_error("weight-stationary GEMM: column block does not fit in LDS");
    return PPS_ERR_INVALID_ARG;
  }
  const dim3 grid((unsigned)(n_cb * rg)), block(64 * W);
  constexpr int C = EPI_CONV, RL = EPI_F_RELU, RS = EPI_F_RES, DU = EPI_F_DUAL;
  if (epi & EPI_F_H2) {
    constexpr int H = EPI_F_H2;
    switch (epi & ~H) {
      case C | RL: hipLaunchKernelGGL((gemm_ws_kernel<NCH, BN2, C | RL | H, W>), grid, block, lds, stream, p, n_cb, n_rt, rg); break;
      case C | RS | RL: hipLaunchKernelGGL((gemm_ws_kernel<NCH, BN2, C | RS | RL | H, W>), grid, block, lds, stream, p, n_cb, n_rt, rg); break;
      case C | RL | DU: hipLaunchKernelGGL((gemm_ws_kernel<NCH, BN2, C | RL | DU | H, W>), grid, block, lds, stream, p, n_cb, n_rt, rg); break;
      case C | RL | EPI_F_H2OUT:
        hipLaunchKernelGGL((gemm_ws_kernel<NCH, BN2, C | RL | EPI_F_H2OUT | H, W>), grid, block, lds, stream, p, n_cb, n_rt, rg);
        break;
      default:
        set_error("weight-stationary f16x2 GEMM: conv + BN + ReLU [+ residual | shortcut] only");
        return PPS_ERR_INVALID_ARG;
    }
    PPS_CHECK_LAUNCH("gemm_ws_kernel");
    return PPS_OK;
  }
  switch (epi) {
    case C: hipLaunchKernelGGL((gemm_ws_kernel<NCH, BN2, C, W>), grid, block, lds, stream, p, n_cb, n_rt, rg); break;
    case C | RL: hipLaunchKernelGGL((gemm_ws_kernel<NCH, BN2, C | RL, W>), grid, block, lds, stream, p, n_cb, n_rt, rg); break;
    case C | RS: hipLaunchKernelGGL((gemm_ws_kernel<NCH, BN2, C | RS, W>), grid, block, lds, stream, p, n_cb, n_rt, rg); break;
    case C | RS | RL: hipLaunchKernelGGL((gemm_ws_kernel<NCH, BN2, C | RS | RL, W>), grid, block, lds, stream, p, n_cb, n_rt, rg); break;
    case C | RL | DU: hipLaunchKernelGGL((gemm_ws_kernel<NCH, BN2, C | RL | DU, W>), grid, block, lds, stream, p, n_cb, n_rt, rg); break;
    case C | DU: hipLaunchKernelGGL((gemm_ws_kernel<NCH, BN2, C | DU, W>), grid, block, lds, stream, p, n_cb, n_rt, rg); break;
    default:
      set_error("weight-stationary GEMM: epilogue not built");
      return PPS_ERR_INVALID_ARG;
  }
  PPS_CHECK_LAUNCH("gemm_ws_kernel");
  return PPS_OK;
}

// The column block is the widest of 256 / 128 / 64 columns whose bf16x3
// weights (BN2 * K * 6 bytes) fit in 96 KB and that divides into Ncol.
// f16x2 (4 B per weight): the widest block whose weights and eight waves'
// epilogue scratch fit (a K = 64 layer's 256 columns: every activation row
// read once).  PPS_WS_H2_WIDE=1 (probes): also the blocks that fit only with
// four waves (K = 128: 256 columns, K = 256: 128) -- measured slower on
// res3 / res4 2c (54.7 vs 45.8 us, 49.2 vs 35.4 on the pipelined tile 45).
static bool ws_h2_wide() {
  static const bool on = [] {
    const char* e = getenv("PPS_WS_H2_WIDE");
    return e && e[0] == '1';
  }();
  return on;
}
int launch_gemm_ws(const GemmParams& p, int epi, hipStream_t stream) {
  const int K = p.Kloop;
  if (epi & EPI_F_H2) {
    if (K == 64) {
      if (p.Ncol % 256 == 0) return launch_ws_cfg<2, 256, 8>(p, epi, stream);
      if (p.Ncol % 128 == 0) return launch_ws_cfg<2, 128, 8>(p, epi, stream);
      return launch_ws_cfg<2, 64, 8>(p, epi, stream);
    }
    if (K == 128) {
      if (ws_h2_wide() && p.Ncol % 256 == 0) return launch_ws_cfg<4, 256, 4>(p, epi, stream);
      if (p.Ncol % 128 == 0) return launch_ws_cfg<4, 128, 8>(p, epi, stream);
      return launch_ws_cfg<4, 64, 8>(p, epi, stream);
    }
    if (ws_h2_wide() && p.Ncol % 128 == 0) return launch_ws_cfg<8, 128, 4>(p, epi, stream);
    return launch_ws_cfg<8, 64, 8>(p, epi, stream);
  }
  if (K == 64) {
    if (p.Ncol % 256 == 0) return launch_ws_cfg<2, 256, 8>(p, epi, stream);
    if (p.Ncol % 128 == 0) return launch_ws_cfg<2, 128, 8>(p, epi, stream);
    return launch_ws_cfg<2, 64, 8>(p, epi, stream);
  }
  if (K == 128) {
    if (p.Ncol % 128 == 0) return launch_ws_cfg<4, 128, 8>(p, epi, stream);
    return launch_ws_cfg<4, 64, 8>(p, epi, stream);
  }
  return launch_ws_cfg<8, 64, 8>(p, epi, stream);
}

}  // namespace pps
