// Patch-staged bf16x3 GEMM for the stride-1 3x3 convolutions (bottleneck
// branch2b, ResNet.py:291-306; GEMM tile ids 56-59).
//
// The pipelined kernel (gemm_x3p.hip) stages the im2col A operand per
// 32-wide K chunk, i.e. per (tap, channel chunk): every input pixel of a tile
// is fetched once per tap, nine times for a 3x3 -- from L2 or, when a
// tile's rows do not stay in its XCD's 4 MB L2 (res5: one 590 KB image per
// tile, 32 tiles per XCD), from the Infinity Cache (PMC: res5 branch2b
// fetched 6.8x its algorithmic bytes).  Here a tile is TR whole output rows of
// one image and K runs (channel chunk, tap): for channel chunk c the tile's
// input patch -- (TR + 2 dil) rows x (Wo + 2 dil) columns x 32 channels,
// padding read as zero by the buffer bounds -- lands in LDS once by LDS-DMA,
// and the nine taps read their A fragments from it at a per-tap pixel
// offset.  Only the weights still travel per chunk (the packed K index of tap
// t, channel 32 c + i is t * Cin + 32 c + i, so the weights need no
// repacking).  Patches are double-buffered: channel chunk c + 1 is requested
// during chunk c's taps, spread over its issue slots with a fixed number of
// DMA instructions per wave and slot (slots without a patch piece load zeros
// into a dummy KiB) so every chunk wait is one counted vmcnt.
//
// Arithmetic: the six terms of mfma16_x3t on 16x16x32 blocks, chunks in
// (channel chunk, tap) order -- a different K order from tiles 38-55, so
// these tiles agree bit for bit with each other, not with them (same
// f32-level error, tests/test_gpu_x3.py).
#include "gemm_x3p_common.hpp"

#ifndef X3P_PRIO
#define X3P_PRIO 0  // probes: s_setprio(1) around every MFMA cluster
#endif

namespace pps {

constexpr int kX3cTaps = 9;  // 3x3

// PMAX: patch pixels the LDS holds (>= (TR + 2 dil) * (Wo + 2 dil), checked
// on the host); NS: weight stages; A3: activations as bf16x3 planes.
template <int BM, int BN, int WM, int WN, int EPI, int NS, bool A3, int PMAX>
__global__ void __launch_bounds__(64 * WM * WN)
gemm_x3c_kernel(GemmParams p, int tiles_n) {
  constexpr int S = 16;
  constexpr int BK = 32;
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / S;
  constexpr int TN = BN / WN / S;
  constexpr int TNH = TN / 2;
  static_assert(TN % 2 == 0 && TM >= 1 && (BM / WM) % S == 0, "wave tile");
  // EPI_F_H2: f16x2 arithmetic (f32 patch split into two f16 terms after the
  // fragment read, two chunk-tiled f16 weight planes, three MFMA terms); with
  // A3 the patch is the two f16x2 activation planes (a PPS_TILE_H2E / H2P
  // edge): no split in the loop, the same fragments
  constexpr bool H2 = (EPI & EPI_F_H2) != 0;
  static_assert(!H2 || !(EPI & (EPI_F_PLANES | EPI_F_RAW)), "f16x2: plain epilogues");
  constexpr int NBP = H2 ? 2 : 3;  // weight planes
  constexpr int NAP = H2 ? 2 : 3;  // activation planes (A3)
  constexpr int B_PLANE = BN * BK * 2;
  constexpr int B_STAGE = NBP * B_PLANE;
  constexpr int NPB = BN / 16;  // weight pieces per plane and chunk
  // pieces per wave; with fewer pieces than waves the spare waves load zeros
  // into the dummy KiB, so every wave issues the same count
  constexpr int BPW = (NPB + NW - 1) / NW;
  constexpr int PXP = A3 ? 16 : 8;                    // patch pixels per DMA piece
  constexpr int PMR = (PMAX + PXP - 1) / PXP * PXP;   // pixels, whole pieces
  constexpr int PX_BYTES = A3 ? 64 : 128;             // per pixel (and plane)
  constexpr int P_PLANE = PMR * 64;                   // A3: plane stride in a buffer
  constexpr int P_BYTES = A3 ? NAP * P_PLANE : PMR * 128;
  constexpr int NPT = PMR / PXP;                      // patch pieces (per plane)
  constexpr int SL = kX3cTaps - NS + 2;               // issue slots per patch
  constexpr int NPPW = (NPT + NW * SL - 1) / (NW * SL);  // patch pieces per wave and slot
  constexpr int LA = A3 ? NAP : 1;
  constexpr int NLOAD = NBP * BPW + LA * NPPW;        // DMA instructions per wave and issue
  static_assert(NS >= 2 && NS <= 4 && NLOAD * (NS - 2) <= 63, "stages / vmcnt range");
  constexpr int OFF_P = NS * B_STAGE;                 // patch buffers
  constexpr int OFF_D = OFF_P + 2 * P_BYTES;          // dummy KiB
  constexpr int MAIN_BYTES = OFF_D + 1024;
  constexpr bool LDSEPI = !(EPI & (EPI_F_RAW | EPI_F_PLANES)) &&
                          lds_epi_bytes<BM, BN>() <= 160 * 1024;
  constexpr int LDS_BYTES =
      LDSEPI && lds_epi_bytes<BM, BN>() > MAIN_BYTES ? lds_epi_bytes<BM, BN>() : MAIN_BYTES;
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[LDS_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (X3P_PRIO == 2 && NW == 8 && wave >= 4) __builtin_amdgcn_s_setprio(1);  // probes
  const int wm = wave / WN;
  const int wn = wave - wm * WN;
  const int r32 = lane & (S - 1);
  const int h = lane / S;

  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  // consecutive ids (one XCD) share a patch, or with colmajor a weight block
  const int tiles_m = gridDim.x / tiles_n;
  const int tile_m = p.colmajor ? bid % tiles_m : bid / tiles_n;
  const int tile_n = p.colmajor ? bid / tiles_m : bid - tile_m * tiles_n;
  const int m0 = tile_m * BM;
  const int n0 = tile_n * BN;
  const int hw = p.Ho * p.Wo;
  const int img = m0 / hw;
  const int oh0 = (m0 - img * hw) / p.Wo;
  const int dil = p.dil;
  const int PW = p.Wo + 2 * dil;
  const int npix = (BM / p.Wo + 2 * dil) * PW;
  const int ncc = p.Cin / 32;
  const int nchunks = ncc * kX3cTaps;

  // ---- operand sources
  rsrc_t ra, ra1, ra2;
  if (A3) {
    ra = make_rsrc(p.a3, p.a_bytes);
    ra1 = make_rsrc(p.a3 + p.a_plane, p.a_bytes);
    ra2 = make_rsrc(p.a3 + 2 * p.a_plane, p.a_bytes);
  } else {
    ra = ra1 = ra2 = make_rsrc(p.a, p.a_bytes);
  }
  const rsrc_t rb0 = make_rsrc(p.b3, p.b_bytes);
  const rsrc_t rb1 = make_rsrc(p.b3 + p.b_plane, p.b_bytes);
  const rsrc_t rb2 = make_rsrc(p.b3 + 2 * p.b_plane, p.b_bytes);
  const int bcl = (lane & 3) ^ ((lane >> 4) & 3);
  int boff[BPW];
#pragma unroll
  for (int j = 0; j < BPW; ++j) {
    const int col = n0 + (wave * BPW + j) * 16 + (lane >> 2);
    boff[j] = (wave * BPW + j < NPB && col < p.Ncol)
                  ? ((p.tiled & 2) ? ((col >> 4) * (p.ldb / 32) * 512 + (col & 15) * 32 + bcl * 8) * 2
                                   : (col * p.ldb + bcl * 8) * 2)
                  : kOOB;
  }

  // patch piece q of channel chunk c into buffer c & 1: lane l fills pixel
  // PXP q + l / (64 / PXP) of the patch, its 16-byte physical slot holding
  // the swizzled logical slot (f32: slot ^ ((pix >> 1) & 7) of 8; planes:
  // slot ^ ((pix >> 2) & 3) of 4 -- the pipelined kernel's A swizzles)
  auto patch_piece = [&](int c, int q, bool real) {
    unsigned char* buf = lds + OFF_P + (c & 1) * P_BYTES;
    if (!real) {
#pragma unroll
      for (int pl = 0; pl < LA; ++pl) glds16(ra, lds + OFF_D, kOOB);
      return;
    }
    const int pix = q * PXP + (A3 ? (lane >> 2) : (lane >> 3));
    const int sl = A3 ? (lane & 3) : (lane & 7);
    const int lc = A3 ? (sl ^ ((pix >> 2) & 3)) : (sl ^ ((pix >> 1) & 7));
    const int pr = pix / PW, pc = pix - pr * PW;
    const int ih = oh0 - dil + pr, iw = pc - dil;
    const bool ok = pix < npix && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
    const int e = ((img * p.H + ih) * p.W + iw) * p.lda + 32 * c + (A3 ? 8 : 4) * lc;
    if (A3) {
      const int off = ok ? e * 2 : kOOB;
      unsigned char* d = buf + q * 1024;
      glds16(ra, d, off);
      glds16(ra1, d + P_PLANE, off);
      if (!H2) glds16(ra2, d + 2 * P_PLANE, off);
    } else {
      glds16(ra, buf + q * 1024, ok ? e * 4 : kOOB);
    }
  };

  // ---- request chunk kiss: its weights, and the issue slot's patch pieces.
  // Patch c (c >= 1) goes out in the issues of chunks 9 (c - 1) + NS - 1 ..
  // 9 c: the first is issued after every wave finished reading patch c - 2
  // (same buffer; the chunk NS back retired at the barrier before it), the
  // last before the barrier that opens chunk 9 c.
  int kiss = 0, siss = 0;
  int ic = 0, it = 0;  // channel chunk / tap of kiss
  auto issue = [&]() {
    const unsigned char* st = lds + siss * B_STAGE;
    const bool valid = kiss < nchunks;
    // K offset of (tap it, channels 32 ic..): row-major 2 B per element;
    // chunk-tiled weights 1 KiB per 32-wide chunk
    const int koff = (p.tiled & 2) ? (it * (p.Cin / 32) + ic) * 1024 : (it * p.Cin + 32 * ic) * 2;
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
      const int off = (valid && boff[j] != kOOB) ? boff[j] + koff : kOOB;
      const bool mine = wave * BPW + j < NPB;  // wave-uniform
      const unsigned char* d = mine ? st + (wave * BPW + j) * 1024 : lds + OFF_D;
      const int pstep = mine ? B_PLANE : 0;
      glds16(rb0, d, off);
      glds16(rb1, d + pstep, off);
      if (!H2) glds16(rb2, d + 2 * pstep, off);
    }
    int pc = -1, s = 0;  // patch chunk this issue serves, its slot
    if (it == 0) {
      pc = ic;
      s = SL - 1;
    } else if (it >= NS - 1) {
      pc = ic + 1;
      s = it - (NS - 1);
    }
    const bool any = pc >= 1 && pc < ncc;
#pragma unroll
    for (int jj = 0; jj < NPPW; ++jj) {
      const int q = (s * NW + wave) * NPPW + jj;
      patch_piece(pc, q, any && q < NPT);
    }
    ++kiss;
    if (++it == kX3cTaps) { it = 0; ++ic; }
    siss = siss + 1 == NS ? 0 : siss + 1;
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // tap (0, 0) patch pixel of each of this lane's rows
  int pbase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = wm * (BM / WM) + i * S + r32;
    const int orow = r / p.Wo;
    pbase[i] = orow * PW + (r - orow * p.Wo);
  }
  const int bsw = (r32 >> 2) & 3;
  float h2s = 1.f;  // f16x2: the activation scale 2^s_a
  float inv_a = 0.f;  // and its inverse, for the epilogue (read once, here)
  if constexpr (H2) h2s = h2_act_scale(p, false, &inv_a);

  auto chunk_barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wait_vmcnt<NLOAD * (NS - 2)>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  // A fragments of chunk (c, t) from patch buffer c & 1
  auto readA = [&](int c, int t, bf16x8 (&fa)[TM][3]) {
    const int kh = t / 3, kw = t - 3 * kh;
    const int toff = (kh * PW + kw) * dil;
    const unsigned char* buf = lds + OFF_P + (c & 1) * P_BYTES;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int pix = pbase[i] + toff;
      if (A3) {
        const unsigned char* ap = buf + pix * 64 + ((h ^ ((pix >> 2) & 3)) << 4);
#pragma unroll
        for (int pl = 0; pl < NAP; ++pl)
          fa[i][pl] = *reinterpret_cast<const bf16x8*>(ap + pl * P_PLANE);
      } else {
        const unsigned char* rp = buf + pix * PX_BYTES;
        const int sw = (pix >> 1) & 7;
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(rp + (((2 * h) ^ sw) << 4));
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(rp + (((2 * h + 1) ^ sw) << 4));
        if (H2)
          split8_h2(x0, x1, h2s, fa[i][0], fa[i][1]);
        else
          split8(x0, x1, fa[i][0], fa[i][1], fa[i][2]);
      }
    }
  };
  auto readB = [&](const unsigned char* st, int half, bf16x8 (&fb)[TNH][3]) {
#pragma unroll
    for (int jj = 0; jj < TNH; ++jj) {
      const unsigned char* bp =
          st + (wn * (BN / WN) + (half * TNH + jj) * 16 + r32) * 64 + ((h ^ bsw) << 4);
#pragma unroll
      for (int pl = 0; pl < NBP; ++pl)
        fb[jj][pl] = *reinterpret_cast<const bf16x8*>(bp + pl * B_PLANE);
    }
  };
  auto mfmas = [&](const bf16x8 (&fa)[TM][3], const bf16x8 (&fb)[TNH][3], int half) {
    if (X3P_PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int jj = 0; jj < TNH; ++jj)
        acc[i][half * TNH + jj] = H2 ? mfma16_h2t(fa[i], fb[jj], acc[i][half * TNH + jj])
                                     : mfma16_x3t(fa[i], fb[jj], acc[i][half * TNH + jj]);
    if (X3P_PRIO == 1) __builtin_amdgcn_s_setprio(0);
  };

  // prologue: patch 0 whole (older than every counted issue), then NS - 1
  // chunks of weights
  for (int q = wave; q < NPT; q += NW) patch_piece(0, q, true);
#pragma unroll
  for (int st = 0; st < NS - 1; ++st) issue();
  chunk_barrier();
  issue();

  bf16x8 fa0[TM][3], fa1[TM][3], fb0[TNH][3], fb1[TNH][3];
  int rc = 0, rt = 0;  // channel chunk / tap of the chunk read next
  auto advance = [&]() {
    if (++rt == kX3cTaps) { rt = 0; ++rc; }
  };
  readA(rc, rt, fa0);
  readB(lds, 0, fb0);
  advance();
  int scur = 0;
  auto step = [&](bf16x8 (&fc)[TM][3], bf16x8 (&fn)[TM][3]) {
    const unsigned char* st = lds + scur * B_STAGE;
    scur = scur + 1 == NS ? 0 : scur + 1;
    readB(st, 1, fb1);
    mfmas(fc, fb0, 0);
    chunk_barrier();
    issue();
    readA(rc, rt, fn);
    readB(lds + scur * B_STAGE, 0, fb0);
    advance();
    mfmas(fc, fb1, 1);
  };
  auto tail = [&](bf16x8 (&fc)[TM][3]) {
    readB(lds + scur * B_STAGE, 1, fb1);
    mfmas(fc, fb0, 0);
    mfmas(fc, fb1, 1);
  };
  int kc = 0;
  for (; kc + 2 < nchunks; kc += 2) {
    step(fa0, fa1);
    step(fa1, fa0);
  }
  if (kc + 1 < nchunks) {
    step(fa0, fa1);
    tail(fa1);
  } else {
    tail(fa0);
  }
  wait_vmcnt<0>();  // no DMA may land in LDS after the workgroup retires

  if constexpr (LDSEPI)
    conv_epilogue_lds<EPI, BM, BN, WM, WN, S, 1>(p, acc, lds, 0, 0, m0, n0, wm, wn, r32, h, 0.f,
                                                 inv_a);
  else
    conv_epilogue_t<EPI, BM, BN, WM, WN, S>(p, acc, 0, 0, m0, n0, wm, wn, r32, h, 0.f, inv_a);
}

template <int BM, int BN, int WM, int WN, int NS, bool A3, int PMAX>
static int launch_c(const GemmParams& p, int epi, hipStream_t stream) {
  constexpr int C = EPI_CONV, RL = EPI_F_RELU, RS = EPI_F_RES, PL = EPI_F_PLANES;
  const int tiles_n = (p.Ncol + BN - 1) / BN;
  const dim3 grid((p.M / BM) * tiles_n), block(64 * WM * WN);
#define X3C_CASE(E)                                                                          \
  case E:                                                                                     \
    hipLaunchKernelGGL((gemm_x3c_kernel<BM, BN, WM, WN, E, NS, A3, PMAX>), grid, block, 0,  \
                       stream, p, tiles_n);                                                   \
    break;
  switch (epi) {
    X3C_CASE(C)
    X3C_CASE(C | RL)
    X3C_CASE(C | RS)
    X3C_CASE(C | RS | RL)
    X3C_CASE(C | PL)
    X3C_CASE(C | RL | PL)
    X3C_CASE(C | RL | EPI_F_H2)
    default:
      set_error("patch-staged 3x3 GEMM: epilogue not built");
      return PPS_ERR_INVALID_ARG;
  }
#undef X3C_CASE
  PPS_CHECK_LAUNCH("gemm_x3c_kernel");
  return PPS_OK;
}

// Rows / columns / patch pixels of tiles 56-59.
static void x3c_shape(int tile, int& bm, int& bn, int& pmax) {
  switch (tile) {
    case GEMM_TILE_C16_192x128: bm = 192; bn = 128; pmax = 272; return;
    case GEMM_TILE_C16_192x64: bm = 192; bn = 64; pmax = 272; return;
    case GEMM_TILE_C16_96x128: bm = 96; bn = 128; pmax = 144; return;
    case GEMM_TILE_C16_192x64W42: bm = 192; bn = 64; pmax = 272; return;
    default: bm = bn = pmax = 0; return;
  }
}

int x3c_tile_rows(int tile) {
  int bm, bn, pm;
  x3c_shape(tile, bm, bn, pm);
  return bm;
}
int x3c_tile_cols(int tile) {
  int bm, bn, pm;
  x3c_shape(tile, bm, bn, pm);
  return bn;
}

// A stride-1 3x3 "same" conv whose tiles are whole output rows of one image
// and whose patch fits; no fused shortcut, split-K or batching.
bool x3c_eligible(const GemmParams& p, int epi, int batch, int tile) {
  int bm, bn, pmax;
  x3c_shape(tile, bm, bn, pmax);
  if (!bm || batch != 1 || p.splitk > 1 || p.ksplit_conv || p.a2 || p.sym) return false;
  constexpr int C = EPI_CONV, RL = EPI_F_RELU, RS = EPI_F_RES, PL = EPI_F_PLANES;
  if (epi != C && epi != (C | RL) && epi != (C | RS) && epi != (C | RS | RL) && epi != (C | PL) &&
      epi != (C | RL | PL) && epi != (C | RL | EPI_F_H2))
    return false;  // the epilogues launch_c builds
  if ((epi & EPI_F_H2) && (!(p.tiled & 2) || !p.rs_b || !p.amax_a)) return false;
  if (p.KH != 3 || p.KW != 3 || p.stride != 1 || p.dil < 1 || p.pad != p.dil) return false;
  if (p.Ho != p.H || p.Wo != p.W || p.Cin % 32 != 0 || p.Kloop != 9 * p.Cin) return false;
  if (bm % p.Wo != 0 || (p.Ho * p.Wo) % bm != 0 || p.M % bm != 0) return false;
  if ((bm / p.Wo + 2 * p.dil) * (p.Wo + 2 * p.dil) > pmax) return false;
  return x3p_eligible(p, epi);
}

int launch_gemm_x3c(const GemmParams& p, int epi, hipStream_t stream, int tile) {
  const bool a3 = p.a3 != nullptr;
  switch (tile) {
    case GEMM_TILE_C16_192x128:
      // 4 x 2 waves (48 x 64 each); weights in three stages (two with plane
      // activations: 104 KB of patches)
      return a3 ? launch_c<192, 128, 4, 2, 2, true, 272>(p, epi, stream)
                : launch_c<192, 128, 4, 2, 3, false, 272>(p, epi, stream);
    case GEMM_TILE_C16_192x64:
      return a3 ? launch_c<192, 64, 4, 1, 4, true, 272>(p, epi, stream)
                : launch_c<192, 64, 4, 1, 4, false, 272>(p, epi, stream);
    case GEMM_TILE_C16_96x128:
      return a3 ? launch_c<96, 128, 2, 4, 4, true, 144>(p, epi, stream)
                : launch_c<96, 128, 2, 4, 4, false, 144>(p, epi, stream);
    case GEMM_TILE_C16_192x64W42:
      // 8 waves as 4 x 2 (48 x 32 each): half the weight bytes per tile of
      // tile 57's neighbours at 256+ tiles for N = 256 (res4) / 128 (res3)
      return a3 ? launch_c<192, 64, 4, 2, 4, true, 272>(p, epi, stream)
                : launch_c<192, 64, 4, 2, 4, false, 272>(p, epi, stream);
    default:
      set_error("unknown patch-staged tile " + std::to_string(tile));
      return PPS_ERR_INVALID_ARG;
  }
}

}  // namespace pps
