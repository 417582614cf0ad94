// FP32 GEMM from bf16 MFMA for gfx950: every f32 operand is split exactly
// into three bf16 terms, x = x0 + x1 + x2 (x0 = bf16(x), x1 = bf16(x - x0),
// x2 = x - x0 - x1, each step exact in f32), and the product is summed from
// the six terms whose weight is >= 2^-16 of the leading one:
//
//   a.b ~= a0b0 + a1b0 + a0b1 + a2b0 + a1b1 + a0b2
//
// The dropped terms (a1b2, a2b1, a2b2) are below 2^-24 |ab|, i.e. under one
// f32 rounding; every product of two bf16 is exact in the f32 accumulator.  So
// the result carries f32-level error (tests/test_gpu_x3.py measures it against
// an fp64 reference next to the exact-f32 MFMA kernel) at six
// v_mfma_f32_32x32x16_bf16 (6 x 32 cycles per 32x32x16 block) instead of
// eight v_mfma_f32_32x32x2_f32 (8 x 64 cycles): 2.67x the f32 MFMA roof.
//
// Layout (same implicit-GEMM conv as gemm_f32.hip, shared AGather/epilogue):
// * A (activations, f32) is gathered exactly as in the f32 kernel, split in
//   registers while it is written to LDS as three bf16 planes.
// * B (weights) is split once at load time (pps_split_bf16x3): three bf16
//   planes [3][Ncol][ldb] per batch, 6 bytes per weight.
// * LDS rows hold BK + 8 bf16 (48 B / 80 B): the 16-byte fragment reads of a
//   32x32x16 MFMA (lane (r, h) reads k = 16g + 8h .. +8 of row r) hit 16
//   distinct 16-byte slots per 16-lane group, i.e. no bank conflicts.
// * K order is fixed (16-groups ascending, the six terms in the order above)
//   for every tile and BK, so all tile variants give identical bits.
#include "gemm_x3_common.hpp"

namespace pps {

template <int BM, int BN, int WM, int WN, int EPI, int BK, bool AF32>
__global__ void __launch_bounds__(64 * WM * WN)
gemm_x3_kernel(GemmParams p, int tiles_m, int tiles_n) {
  constexpr int T = 64 * WM * WN;
  constexpr int LSTR = BK + 8;          // LDS row stride in bf16 elements
  constexpr int V4 = BK / 4;            // 4-element slots per K chunk row
  constexpr int AL = BM * BK / 4 / T;   // A float4 loads per thread
  constexpr int BL = BN * BK / 4 / T;   // B 4-element (x3 planes) loads per thread
  constexpr int RPP = T / V4;           // rows covered per load pass
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  constexpr int APL = BM * LSTR;        // elements per A plane
  constexpr int BPL = BN * LSTR;
  // AF32: A stays f32 in LDS (rows of BK+4 floats, as in gemm_f32.hip) and is
  // split after the fragment read -- 4 B instead of 6 B per element staged
  constexpr int LSTRA = 2 * (BK + 4);   // A row stride in 16-bit units (AF32)
  constexpr int AREG = AF32 ? BM * LSTRA : 3 * APL;
  constexpr int STAGE = AREG + 3 * BPL;
  static_assert(BK == 16 || BK == 32, "BK must be 16 or 32");
  static_assert(AL >= 1 && BL >= 1 && TM >= 1 && TN >= 1, "tile too small");
  static_assert(2 * STAGE * 2 + 256 <= 160 * 1024, "LDS over 160 KB");
  constexpr bool DUAL = (EPI & EPI_F_DUAL) != 0;

  __shared__ __attribute__((aligned(16))) unsigned short lds[2 * STAGE + 128];
  int* s_tapoff = reinterpret_cast<int*>(lds + 2 * STAGE);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN;
  const int wn = wave % WN;
  const int r32 = lane & 31;
  const int h = lane >> 5;

  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tile_m = bid / tiles_n;
  const int tile_n = bid - tile_m * tiles_n;
  const int m0 = tile_m * BM;
  const int n0 = tile_n * BN;
  const int batch = blockIdx.y / p.splitk;
  const int kslice = blockIdx.y - batch * p.splitk;

  const int64_t kofs0 = (int64_t)kslice * p.Kloop;
  // one descriptor per bf16 plane: 32-bit offsets stay within a plane
  const uint16_t* b3 = p.b3 + batch * p.b_bstride + kofs0;
  const rsrc_t rb_src0 = make_rsrc(b3, p.b_bytes);
  const rsrc_t rb_src1 = make_rsrc(b3 + p.b_plane, p.b_bytes);
  const rsrc_t rb_src2 = make_rsrc(b3 + 2 * p.b_plane, p.b_bytes);
  const int c4 = tid % V4;
  const int trow = tid / V4;
  AGather<AL, RPP, BK, DUAL> ag;
  ag.init(p, batch, kofs0, m0, trow, c4, s_tapoff, tid, T);
  unsigned bbase[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int col = n0 + trow + i * RPP;
    bbase[i] = col < p.Ncol ? (unsigned)(col * p.ldb + c4 * 4) * 2u : (unsigned)kOOB;
  }

  // One register stage, two LDS stages.  Iteration kc computes on stage kc&1
  // while it writes chunk kc+1 (loaded one iteration earlier) into the other
  // stage and requests chunk kc+2; one barrier closes the iteration.  The
  // split / LDS-store work of the next chunk therefore sits between this
  // chunk's MFMAs instead of in a separate phase that every wave of the
  // block (synchronised by the barrier) would run at the same time.
  f32x4 ra[AL];
  u32x2 rb[BL][3];
  auto load_chunk = [&](int kc) {
    ag.load(p, kc, c4, s_tapoff, ra);
    const bool kok = kc * BK + c4 * 4 < p.kb_valid;
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const bool ok = kok && bbase[i] != (unsigned)kOOB;
      const unsigned o = bbase[i] + (unsigned)(kc * BK * 2);
      const int off = ok ? (int)o : kOOB;
      rb[i][0] = bload64(rb_src0, off);
      rb[i][1] = bload64(rb_src1, off);
      rb[i][2] = bload64(rb_src2, off);
    }
  };
  // registers -> LDS stage `as` (A split into planes unless AF32)
  auto store_chunk = [&](unsigned short* as) {
    unsigned short* bs = as + AREG;  // as: [3][BM][LSTR] or [BM][BK+4] f32; bs: [3][BN][LSTR]
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      if (AF32) {
        *reinterpret_cast<f32x4*>(as + (trow + i * RPP) * LSTRA + c4 * 8) = ra[i];
        continue;
      }
      unsigned h0, m0_, l0, h1, m1, l1;
      split2(ra[i][0], ra[i][1], h0, m0_, l0);
      split2(ra[i][2], ra[i][3], h1, m1, l1);
      const u32x2 hi = {h0, h1}, mid = {m0_, m1}, lo = {l0, l1};
      unsigned short* d = as + (trow + i * RPP) * LSTR + c4 * 4;
      *reinterpret_cast<u32x2*>(d) = hi;
      *reinterpret_cast<u32x2*>(d + APL) = mid;
      *reinterpret_cast<u32x2*>(d + 2 * APL) = lo;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      unsigned short* d = bs + (trow + i * RPP) * LSTR + c4 * 4;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) *reinterpret_cast<u32x2*>(d + pl * BPL) = rb[i][pl];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // MFMAs of one 16-wide K group of stage `as`
  auto compute_group = [&](const unsigned short* as, int g) {
    const unsigned short* bs = as + AREG;
    bf16x8 fa[TM][3], fb[TN][3];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * (BM / WM) + i * 32 + r32;
      if (AF32) {
        const float* s = reinterpret_cast<const float*>(as + row * LSTRA) + g * 16 + h * 8;
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(s);
        const f32x4 x1 = *reinterpret_cast<const f32x4*>(s + 4);
        u32x4 hi, mid, lo;
        unsigned a, b, c;
        split2(x0[0], x0[1], a, b, c); hi[0] = a; mid[0] = b; lo[0] = c;
        split2(x0[2], x0[3], a, b, c); hi[1] = a; mid[1] = b; lo[1] = c;
        split2(x1[0], x1[1], a, b, c); hi[2] = a; mid[2] = b; lo[2] = c;
        split2(x1[2], x1[3], a, b, c); hi[3] = a; mid[3] = b; lo[3] = c;
        fa[i][0] = __builtin_bit_cast(bf16x8, hi);
        fa[i][1] = __builtin_bit_cast(bf16x8, mid);
        fa[i][2] = __builtin_bit_cast(bf16x8, lo);
      } else {
        const unsigned short* s = as + row * LSTR + g * 16 + h * 8;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) fa[i][pl] = *reinterpret_cast<const bf16x8*>(s + pl * APL);
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const unsigned short* s = bs + (wn * (BN / WN) + j * 32 + r32) * LSTR + g * 16 + h * 8;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) fb[j][pl] = *reinterpret_cast<const bf16x8*>(s + pl * BPL);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x16 c = acc[i][j];
        c = mfma_bf16(fa[i][0], fb[j][0], c);
        c = mfma_bf16(fa[i][1], fb[j][0], c);
        c = mfma_bf16(fa[i][0], fb[j][1], c);
        c = mfma_bf16(fa[i][2], fb[j][0], c);
        c = mfma_bf16(fa[i][1], fb[j][1], c);
        c = mfma_bf16(fa[i][0], fb[j][2], c);
        acc[i][j] = c;
      }
  };

  // Loads past the last chunk are harmless: they address beyond the tap /
  // K ranges or num_records and read zero, and the stage they are written to
  // is never read.  Keeping them unconditional keeps the store work and the
  // MFMAs of an iteration in one basic block, so the scheduler interleaves them.
  const int nchunks = (p.Kloop + BK - 1) / BK;
  load_chunk(0);
  store_chunk(lds);
  load_chunk(1);
  __syncthreads();
  for (int kc = 0; kc < nchunks; ++kc) {
    const unsigned short* cur = lds + (kc & 1) * STAGE;
    unsigned short* nxt = lds + ((kc + 1) & 1) * STAGE;
    compute_group(cur, 0);
    store_chunk(nxt);
#pragma unroll
    for (int g = 1; g < BK / 16; ++g) compute_group(cur, g);
    load_chunk(kc + 2);
    __syncthreads();
  }

  if (EPI & EPI_DIST)
    dist_epilogue<BM, BN, WM, WN>(p, acc, m0, n0, wm, wn, r32, h);
  else
    conv_epilogue<EPI, BM, BN, WM, WN>(p, acc, batch, kslice, m0, n0, wm, wn, r32, h);
}

template <int BM, int BN, int WM, int WN, int EPI, int BK>
static void launch_one_x3(const GemmParams& p, int batch, hipStream_t stream, bool af32) {
  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.Ncol + BN - 1) / BN;
  if (af32)
    hipLaunchKernelGGL((gemm_x3_kernel<BM, BN, WM, WN, EPI, BK, true>),
                       dim3(tiles_m * tiles_n, batch * p.splitk), dim3(64 * WM * WN), 0, stream,
                       p, tiles_m, tiles_n);
  else
    hipLaunchKernelGGL((gemm_x3_kernel<BM, BN, WM, WN, EPI, BK, false>),
                       dim3(tiles_m * tiles_n, batch * p.splitk), dim3(64 * WM * WN), 0, stream,
                       p, tiles_m, tiles_n);
}

template <int BM, int BN, int WM, int WN, int BK>
static int launch_tile_x3(const GemmParams& p, int epi, int batch, hipStream_t stream,
                          bool af32) {
  switch (epi) {
    case EPI_DIST: launch_one_x3<BM, BN, WM, WN, EPI_DIST, BK>(p, batch, stream, af32); break;
    case EPI_CONV: launch_one_x3<BM, BN, WM, WN, EPI_CONV, BK>(p, batch, stream, af32); break;
    case EPI_CONV | EPI_F_RELU:
      launch_one_x3<BM, BN, WM, WN, EPI_CONV | EPI_F_RELU, BK>(p, batch, stream, af32); break;
    case EPI_CONV | EPI_F_RES:
      launch_one_x3<BM, BN, WM, WN, EPI_CONV | EPI_F_RES, BK>(p, batch, stream, af32); break;
    case EPI_CONV | EPI_F_RES | EPI_F_RELU:
      launch_one_x3<BM, BN, WM, WN, EPI_CONV | EPI_F_RES | EPI_F_RELU, BK>(p, batch, stream, af32);
      break;
    case EPI_CONV | EPI_F_RAW:
      launch_one_x3<BM, BN, WM, WN, EPI_CONV | EPI_F_RAW, BK>(p, batch, stream, af32); break;
    case EPI_CONV | EPI_F_RELU | EPI_F_DUAL:
      launch_one_x3<BM, BN, WM, WN, EPI_CONV | EPI_F_RELU | EPI_F_DUAL, BK>(p, batch, stream, af32);
      break;
    default:
      set_error("unknown epilogue for the bf16x3 GEMM");
      return PPS_ERR_INVALID_ARG;
  }
  PPS_CHECK_LAUNCH("gemm_x3_kernel");
  return PPS_OK;
}

int launch_gemm_x3(const GemmParams& p, int epi, int batch, hipStream_t stream) {
  if (p.M <= 0 || p.Ncol <= 0 || batch <= 0) return PPS_OK;
  if (p.splitk < 1 || !p.b3) {
    set_error("bf16x3 GEMM: splitk must be >= 1 and b3 set");
    return PPS_ERR_INVALID_ARG;
  }
  if ((epi & EPI_DIST) && (!p.norm_a || !p.norm_b)) {
    set_error("bf16x3 distance GEMM needs both squared-norm vectors");
    return PPS_ERR_INVALID_ARG;
  }
  const int epi_in = epi;
  if (p.tile == GEMM_TILE_P16_192x128W41 && !(epi & EPI_F_H2)) {
    // the f16x2-only tile: bf16x3 runs its 4 x 2-wave twin (same rounding)
    GemmParams q = p;
    q.tile = GEMM_TILE_P16_192x128W42;
    return launch_gemm_x3(q, epi, batch, stream);
  }
  if (!(epi & EPI_DIST) && !(epi & EPI_F_RAW)) {
    if (p.residual) epi |= EPI_F_RES;
    if (p.relu) epi |= EPI_F_RELU;
    if (p.a2) epi |= EPI_F_DUAL;
  }
  if ((epi & EPI_F_H2OUT) && !(epi & EPI_F_H2)) {
    // a bf16x3 producer writing f16x2 planes: pipelined tiles (the others
    // run tile 38, the pipelined 16x16x32 group)
    if (p.a3 || p.splitk != 1 || p.ksplit_conv || batch != 1 || !p.out3 || !p.h2o_in ||
        !x3p_eligible(p, epi)) {
      set_error("f16x2 planes out: f32 activations, no split-K, Cin % 32 == 0");
      return PPS_ERR_INVALID_ARG;
    }
    const int t = (p.tile < GEMM_TILE_P16_FIRST || p.tile == GEMM_TILE_WS ||
                   p.tile >= GEMM_TILE_C16_FIRST) ? GEMM_TILE_P16_FIRST : p.tile;
    return launch_gemm_x3p(p, epi, batch, stream, t - GEMM_TILE_P_FIRST);
  }
  if ((p.tiled & 2) && !(epi & EPI_F_H2) &&
      (p.tile == GEMM_TILE_WS || p.tile < GEMM_TILE_P_FIRST ||
       (p.splitk > 1 && !p.ksplit_conv))) {
    set_error("chunk-tiled weights run on the pipelined / patch tiles only");
    return PPS_ERR_INVALID_ARG;
  }
  if ((epi & EPI_F_FIX) && (!p.ksplit_conv || !p.fix_cnt || !p.part || p.tile < GEMM_TILE_P_FIRST ||
                           p.tile == GEMM_TILE_WS || p.tile >= GEMM_TILE_C16_FIRST)) {
    set_error("one-launch conv split-K needs a pipelined tile, partials and counters");
    return PPS_ERR_INVALID_ARG;
  }
  if (epi & EPI_F_H2) {
    // f16x2 convs: the patch tiles (56..59) and the weight-stationary 1x1
    // tile (54) where they apply, else the 16x16x32 pipelined tiles (38..53,
    // 55; tile 38 for the patch / weight-stationary ids' fallback and for 0)
    if (p.tile >= GEMM_TILE_C16_FIRST && x3c_eligible(p, epi, batch, p.tile))
      return launch_gemm_x3c(p, epi, stream, p.tile);
    if (p.tile == GEMM_TILE_WS && ws_eligible(p, epi, batch)) return launch_gemm_ws(p, epi, stream);
    const int t = (p.tile == 0 || p.tile == GEMM_TILE_WS ||
                   (p.tile >= GEMM_TILE_C16_FIRST && p.tile != GEMM_TILE_P16_192x128W41))
                      ? GEMM_TILE_P16_FIRST
                      : p.tile;
    if (t < GEMM_TILE_P16_FIRST || t == GEMM_TILE_WS || batch != 1 || p.splitk != 1 ||
        !x3p_eligible(p, epi)) {
      set_error("f16x2 conv: a 16x16x32 pipelined or patch tile (38..53, 55..60), no split-K, "
                "Cin % 32 == 0");
      return PPS_ERR_INVALID_ARG;
    }
    return launch_gemm_x3p(p, epi, batch, stream, t - GEMM_TILE_P_FIRST);
  }
  if (p.tile == GEMM_TILE_WS) {
    // the weight-stationary kernel where it applies, else the 128x128
    // pipelined tile of the same (16x16x32) rounding group
    if (ws_eligible(p, epi, batch)) return launch_gemm_ws(p, epi, stream);
    GemmParams q = p;
    q.tile = GEMM_TILE_P16_FIRST;
    return launch_gemm_x3(q, epi_in, batch, stream);
  }
  if (p.tile >= GEMM_TILE_C16_FIRST) {
    // patch-staged 3x3 tiles where they apply, else tile 38
    if (x3c_eligible(p, epi, batch, p.tile)) return launch_gemm_x3c(p, epi, stream, p.tile);
    GemmParams q = p;
    q.tile = GEMM_TILE_P16_FIRST;
    return launch_gemm_x3(q, epi_in, batch, stream);
  }
  if (p.ksplit_conv && (p.tile < GEMM_TILE_P_FIRST || !x3p_eligible(p, epi))) {
    set_error("conv split-K runs on the pipelined tiles only (tile >= " +
              std::to_string((int)GEMM_TILE_P_FIRST) + ", Cin % 32 == 0)");
    return PPS_ERR_INVALID_ARG;
  }
  if (p.sym) {
    // self-distance: any pipelined tile (the upper triangle is enumerated by
    // lcm(BM, BN) super-blocks, gemm_x3p.hip); tile 0 = tile 43 (128 x 256,
    // the distance matrix's winner)
    const int t = p.tile ? p.tile : GEMM_TILE_P16_FIRST + 5;
    if (!(epi & EPI_DIST) || p.M != p.Ncol || !x3p_eligible(p, epi) || t < GEMM_TILE_P_FIRST ||
        t >= GEMM_TILE_C16_FIRST || t == GEMM_TILE_WS) {
      set_error("symmetric distance: needs EPI_DIST, M == Ncol and a pipelined tile "
                "(29..53 or 55)");
      return PPS_ERR_INVALID_ARG;
    }
    return launch_gemm_x3p(p, epi, batch, stream, t - GEMM_TILE_P_FIRST);
  }
  if (p.a3 || (epi & EPI_F_PLANES)) {
    // bf16-plane activations exist only in the pipelined family
    if (!x3p_eligible(p, epi)) {
      set_error("bf16-plane activations: shape/alignment not eligible for the pipelined GEMM");
      return PPS_ERR_INVALID_ARG;
    }
    const int v = p.tile >= GEMM_TILE_P_FIRST ? p.tile - GEMM_TILE_P_FIRST
                                              : (p.M % 192 == 0 ? 1 : 0);
    return launch_gemm_x3p(p, epi, batch, stream, v);
  }
  // default for the distance matrix: the pipelined 256x128 tile on 16x16x32
  // blocks (the Market / Duke / 1M-shard autotune winner, scripts/dist_probe.py)
  int tile = p.tile ? p.tile
                    : ((epi & EPI_DIST) && x3p_eligible(p, epi) ? GEMM_TILE_P16_FIRST + 4
                                                                : pick_tile(p, batch));
  if (tile >= GEMM_TILE_P_FIRST) {
    // LDS-DMA pipelined family (gemm_x3p.hip); shapes it cannot stage
    // (Cin % 32 != 0, unaligned rows) take the heuristic register-staged tile
    if (x3p_eligible(p, epi)) return launch_gemm_x3p(p, epi, batch, stream, tile - GEMM_TILE_P_FIRST);
    tile = pick_tile(p, batch);
  }
  const bool narrow_ok = p.Cin >= 32 || (p.Cin & (p.Cin - 1)) == 0;
  const bool dual_ok = !p.a2 || p.Kloop1 % 32 == 0;
  if (tile >= GEMM_TILE_192_FIRST && tile < GEMM_TILE_P_FIRST) {
    // 192-row family (M = 12,288 / 49,152 / 196,608 at batch 64 are
    // multiples of 192: fills 256 CUs without a partial last wave of tiles)
    const int v = tile - GEMM_TILE_192_FIRST;
    const bool af = v >= 4;
    const bool k32 = (v & 2) && narrow_ok && dual_ok;
    if (v & 1)
      return k32 ? launch_tile_x3<192, 64, 2, 2, 32>(p, epi, batch, stream, af)
                 : launch_tile_x3<192, 64, 2, 2, 16>(p, epi, batch, stream, af);
    return k32 ? launch_tile_x3<192, 128, 2, 2, 32>(p, epi, batch, stream, af)
               : launch_tile_x3<192, 128, 2, 2, 16>(p, epi, batch, stream, af);
  }
  // ids 11..20: the same shapes with A kept f32 in LDS and split after the
  // fragment read (AF32); 1..10 split A while staging (three bf16 planes)
  const bool af32 = tile > GEMM_TILE_256x128_K32;
  if (af32) tile -= GEMM_TILE_256x128_K32;
  if (tile == GEMM_TILE_256x128_K32) tile = GEMM_TILE_256x128;  // 184 KB of LDS: no
  if (tile > GEMM_TILE_256x128 && (!narrow_ok || !dual_ok)) tile -= 5;
  switch (tile) {
    case GEMM_TILE_128x128: return launch_tile_x3<128, 128, 2, 2, 16>(p, epi, batch, stream, af32);
    case GEMM_TILE_128x64: return launch_tile_x3<128, 64, 4, 1, 16>(p, epi, batch, stream, af32);
    case GEMM_TILE_64x128: return launch_tile_x3<64, 128, 1, 4, 16>(p, epi, batch, stream, af32);
    case GEMM_TILE_64x64: return launch_tile_x3<64, 64, 2, 2, 16>(p, epi, batch, stream, af32);
    case GEMM_TILE_256x128: return launch_tile_x3<256, 128, 4, 2, 16>(p, epi, batch, stream, af32);
    case GEMM_TILE_128x128_K32: return launch_tile_x3<128, 128, 2, 2, 32>(p, epi, batch, stream, af32);
    case GEMM_TILE_128x64_K32: return launch_tile_x3<128, 64, 4, 1, 32>(p, epi, batch, stream, af32);
    case GEMM_TILE_64x128_K32: return launch_tile_x3<64, 128, 1, 4, 32>(p, epi, batch, stream, af32);
    case GEMM_TILE_64x64_K32: return launch_tile_x3<64, 64, 2, 2, 32>(p, epi, batch, stream, af32);
    default:
      set_error("unknown GEMM tile id " + std::to_string(tile));
      return PPS_ERR_INVALID_ARG;
  }
}

// ---- weight split: x[b][i] -> out[b][plane][i], x = hi + mid + lo ----------
__global__ void split_bf16x3_kernel(const float* __restrict__ x, int64_t n, int nbatch,
                                    unsigned short* __restrict__ out) {
  const int64_t total = n * nbatch;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / n, i = e - b * n;
    unsigned hi, mid, lo;
    split2(x[e], 0.f, hi, mid, lo);
    unsigned short* o = out + b * 3 * n + i;
    o[0] = (unsigned short)hi;
    o[n] = (unsigned short)mid;
    o[2 * n] = (unsigned short)lo;
  }
}

// Eight elements per thread: two 16-byte loads, three 16-byte plane stores
// (the scalar kernel's 2-byte stores ran the gallery split at ~4 TB/s).
// Needs n % 8 == 0 and 16-byte aligned x / out; same bits as the scalar one.
__global__ void split_bf16x3_v8_kernel(const float* __restrict__ x, int64_t n, int nbatch,
                                       unsigned short* __restrict__ out) {
  const int64_t n8 = n >> 3;
  const int64_t total = n8 * nbatch;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / n8, i = (e - b * n8) << 3;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(x + (e << 3));
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(x + (e << 3) + 4);
    u32x4 hi, mid, lo;
    unsigned a, m, l;
    split2(v0[0], v0[1], a, m, l); hi[0] = a; mid[0] = m; lo[0] = l;
    split2(v0[2], v0[3], a, m, l); hi[1] = a; mid[1] = m; lo[1] = l;
    split2(v1[0], v1[1], a, m, l); hi[2] = a; mid[2] = m; lo[2] = l;
    split2(v1[2], v1[3], a, m, l); hi[3] = a; mid[3] = m; lo[3] = l;
    unsigned short* o = out + b * 3 * n + i;
    *reinterpret_cast<u32x4*>(o) = hi;
    *reinterpret_cast<u32x4*>(o + n) = mid;
    *reinterpret_cast<u32x4*>(o + 2 * n) = lo;
  }
}

// ---- squared row norms: one wave per row, fixed lane order + xor tree -----
__global__ void row_sqnorm_kernel(const float* __restrict__ x, int64_t rows, int D, int64_t ld,
                                  float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* r = x + row * ld;
  float s = 0.f;
  for (int k = lane * 4; k < D; k += 256) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(r + k);
    s = __builtin_fmaf(v[0], v[0], s);
    s = __builtin_fmaf(v[1], v[1], s);
    s = __builtin_fmaf(v[2], v[2], s);
    s = __builtin_fmaf(v[3], v[3], s);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) out[row] = s;
}

// ---- gallery / query index in one pass: bf16x3 planes [3][rows][D] and
// squared row norms, reading x once.  The norm uses row_sqnorm_kernel's lane
// order and xor tree, the split is elementwise: bits equal to the two
// separate kernels.  TILED: the planes in the chunk-tiled layout
// [rows16 / 16][D / 32][16][32] (pps_tile_planes; rows16 = rows rounded up to
// 16, the padding rows written as zeros, D % 32 == 0).
template <bool TILED>
__global__ void split_sqnorm_kernel(const float* __restrict__ x, int64_t rows, int D, int64_t ld,
                                    unsigned short* __restrict__ out3,
                                    float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t rows16 = TILED ? (rows + 15) / 16 * 16 : rows;
  if (row >= rows16) return;
  const bool real = row < rows;
  const float* r = x + (real ? row : 0) * ld;
  const int64_t plane = rows16 * (int64_t)D;
  unsigned short* o = TILED ? out3 + (row >> 4) * 16 * (int64_t)D + (row & 15) * 32
                            : out3 + row * (int64_t)D;
  float s = 0.f;
  // kSplitU row segments of 256 per trip: their loads issue together (one
  // memory latency per trip, not per segment); the norm still accumulates
  // segment after segment, row_sqnorm_kernel's order
  constexpr int kSplitU = 4;
  for (int k0 = lane * 4; k0 < D; k0 += 256 * kSplitU) {
    f32x4 v[kSplitU];
#pragma unroll
    for (int u = 0; u < kSplitU; ++u) {
      const int k = k0 + 256 * u;
      v[u] = real && k < D ? *reinterpret_cast<const f32x4*>(r + k) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < kSplitU; ++u) {
      const int k = k0 + 256 * u;
      if (k >= D) break;
      s = __builtin_fmaf(v[u][0], v[u][0], s);
      s = __builtin_fmaf(v[u][1], v[u][1], s);
      s = __builtin_fmaf(v[u][2], v[u][2], s);
      s = __builtin_fmaf(v[u][3], v[u][3], s);
      u32x2 hi, mid, lo;
      unsigned a, m, l;
      split2(v[u][0], v[u][1], a, m, l); hi[0] = a; mid[0] = m; lo[0] = l;
      split2(v[u][2], v[u][3], a, m, l); hi[1] = a; mid[1] = m; lo[1] = l;
      const int64_t ko = TILED ? (int64_t)(k >> 5) * 512 + (k & 31) : k;
      *reinterpret_cast<u32x2*>(o + ko) = hi;
      *reinterpret_cast<u32x2*>(o + plane + ko) = mid;
      *reinterpret_cast<u32x2*>(o + 2 * plane + ko) = lo;
    }
  }
#pragma unroll
  for (int o2 = 32; o2 >= 1; o2 >>= 1) s += __shfl_xor(s, o2);
  if (lane == 0 && real) out[row] = s;
}

int split_sqnorm(const float* x, int64_t rows, int D, int64_t ld, uint16_t* out3, float* out,
                 hipStream_t stream) {
  if (rows <= 0) return PPS_OK;
  const int64_t blocks = (rows + 3) / 4;
  hipLaunchKernelGGL(split_sqnorm_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, stream, x,
                     rows, D, ld, reinterpret_cast<unsigned short*>(out3), out);
  PPS_CHECK_LAUNCH("split_sqnorm_kernel");
  return PPS_OK;
}

int split_sqnorm_tiled(const float* x, int64_t rows, int D, int64_t ld, uint16_t* out3t,
                       float* out, hipStream_t stream) {
  if (rows <= 0) return PPS_OK;
  const int64_t blocks = ((rows + 15) / 16 * 16 + 3) / 4;
  hipLaunchKernelGGL(split_sqnorm_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, stream, x,
                     rows, D, ld, reinterpret_cast<unsigned short*>(out3t), out);
  PPS_CHECK_LAUNCH("split_sqnorm_kernel");
  return PPS_OK;
}

int row_sqnorm(const float* x, int64_t rows, int D, int64_t ld, float* out, hipStream_t stream) {
  if (rows <= 0) return PPS_OK;
  const int64_t blocks = (rows + 3) / 4;
  hipLaunchKernelGGL(row_sqnorm_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, x, rows,
                     D, ld, out);
  PPS_CHECK_LAUNCH("row_sqnorm_kernel");
  return PPS_OK;
}

int split_bf16x3(const float* x, int64_t n, int nbatch, uint16_t* out, hipStream_t stream) {
  const int threads = 256;
  if (n % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0) {
    const int64_t blocks = (n / 8 * nbatch + threads - 1) / threads;
    hipLaunchKernelGGL(split_bf16x3_v8_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)),
                       dim3(threads), 0, stream, x, n, nbatch,
                       reinterpret_cast<unsigned short*>(out));
    PPS_CHECK_LAUNCH("split_bf16x3_v8_kernel");
    return PPS_OK;
  }
  const int64_t blocks = (n * nbatch + threads - 1) / threads;
  hipLaunchKernelGGL(split_bf16x3_kernel, dim3((unsigned)(blocks < 65536 ? blocks : 65536)),
                     dim3(threads), 0, stream, x, n, nbatch,
                     reinterpret_cast<unsigned short*>(out));
  PPS_CHECK_LAUNCH("split_bf16x3_kernel");
  return PPS_OK;
}

}  // namespace pps

namespace pps {
// Chunk-tiled copy of bf16x3 planes for the distance GEMM's tiled path:
// in [3][rows][ld] (plane stride ps) -> out [3][rows16 / 16][D / 32][16][32]
// with rows16 = rows rounded up to 16 (padding rows zero).  One thread per
// 16-byte vector of the output.
__global__ void tile_planes_kernel(const uint16_t* __restrict__ in, int64_t rows, int D,
                                   int64_t ld, int64_t ps, uint16_t* __restrict__ out,
                                   int64_t nvec) {
  const int64_t rows16 = (rows + 15) / 16 * 16;
  const int nkc = D / 32;
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nvec;
       v += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = v * 8;                  // output element
    const int64_t per_plane = rows16 * D;
    const int pl = (int)(e / per_plane);
    const int64_t r = e - pl * per_plane;     // within the plane
    const int64_t blk = r / 512;              // (row block, chunk)
    const int w = (int)(r - blk * 512);       // within the KiB: row * 32 + k
    const int64_t rb = blk / nkc;
    const int kc = (int)(blk - rb * nkc);
    const int64_t row = rb * 16 + (w >> 5);
    const int k = kc * 32 + (w & 31);
    uint4 x = make_uint4(0u, 0u, 0u, 0u);
    if (row < rows) x = *reinterpret_cast<const uint4*>(in + pl * ps + row * ld + k);
    *reinterpret_cast<uint4*>(out + e) = x;
  }
}
}  // namespace pps

int pps_tile_planes(const uint16_t* planes, int64_t rows, int D, int64_t ld, int64_t plane_stride,
                    uint16_t* out, void* stream) {
  using namespace pps;
  if (!planes || !out) { set_error("null pointer"); return PPS_ERR_INVALID_ARG; }
  if (rows < 0 || D <= 0 || D % 32 != 0 || ld < D || ld % 8 != 0 || plane_stride < rows * ld) {
    set_error("pps_tile_planes: bad shape (D % 32 == 0, ld % 8 == 0)");
    return PPS_ERR_INVALID_ARG;
  }
  const int64_t rows16 = (rows + 15) / 16 * 16;
  const int64_t nvec = 3 * rows16 * D / 8;
  if (nvec == 0) return PPS_OK;
  const int64_t blocks = std::min<int64_t>((nvec + 255) / 256, 8192);
  hipLaunchKernelGGL(tile_planes_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     static_cast<hipStream_t>(stream), planes, rows, D, ld, plane_stride, out, nvec);
  PPS_CHECK_LAUNCH("tile_planes_kernel");
  return PPS_OK;
}
