// Pipelined bf16x3 GEMM for gfx950: the arithmetic of gemm_x3.hip (f32
// operands split exactly into three bf16 terms, six MFMA terms per product,
// same 16-wide K groups in the same order -> identical bits), restructured
// around LDS-DMA so that several K chunks are in flight while one is
// multiplied:
//
// * both operands travel global -> LDS by `buffer_load_dwordx4 ... lds`
//   (16 B per lane, no VGPR staging, no ds_write): A as f32 rows (split into
//   bf16 terms after the fragment read), B as the three bf16 weight planes;
//   out-of-range taps / rows / K read zero in hardware (buffer bounds);
// * NS LDS stages: chunk kc+NS-1 is requested right after the barrier that
//   opens chunk kc, so up to NS-1 chunks are in flight.  The wait before the
//   barrier is a COUNTED vmcnt and the barrier a raw s_barrier (a
//   __syncthreads() would drain the DMA queue);
// * the DMA image is lane-linear (LDS address = wave base + 16 * lane), so
//   the bank-conflict swizzle goes on the per-lane SOURCE address and is
//   undone on the fragment read: A rows (128 B) keep 16-byte chunk c in slot
//   c ^ ((row >> 1) & 7), B rows (64 B) in slot c ^ ((row >> 2) & 3) -- each
//   ds_read_b128 lane group then hits 16 distinct 16-byte slots;
// * K chunk 32 and Cin % 32 == 0, so a chunk never straddles two im2col taps:
//   the tap tracker is wave-uniform (scalar) and each lane keeps only a row
//   base and a 64-bit tap-validity mask per DMA piece.
//
// Extensions on the same main loop: bf16x3 activation planes as A (A3) and
// as output (EPI_F_PLANES); 16x16x32 MFMA blocks (S = 16, their own rounding
// group); conv split-K (slices starting mid-im2col, raw partials); for the
// distance epilogue a grouped tile order (GM query panels sweep the gallery
// together) and the symmetric self-distance (upper-triangle tiles + mirror).
#include "gemm_x3p_common.hpp"

namespace pps {

// A3 = false: A is f32 NHWC, staged as 128-byte f32 rows and split after the
// fragment read.  A3 = true: A is three bf16 planes (written by a producer
// epilogue with EPI_F_PLANES), staged like B as 64-byte rows per plane --
// no split arithmetic in the main loop.
// S: MFMA block, 32 (v_mfma_f32_32x32x16_bf16, two 16-wide K groups per
// chunk) or 16 (v_mfma_f32_16x16x32_bf16, one group per chunk; the wave's
// column blocks are processed in two halves to keep the same pipeline).
#ifndef X3P_PRIO
#define X3P_PRIO 0  // probes: 1 = s_setprio(1) around every MFMA cluster, 2 = younger half raised
#endif
#ifndef X3P_ABL
#define X3P_ABL 0  // probes: 1 = no DMA after the prologue, 2 = no MFMAs (timing ablations)
#endif
#ifndef X3P_STAG
#define X3P_STAG -1  // 1 / 2: waves NW/2.. / ..NW/2-1 of 8-wave tiles multiply a chunk's two
                     // column halves before its barrier (the others: one before, one after);
                     // -1: 1 on tile 52, 0 elsewhere; 0: never (probes)
#endif
#ifndef X3P_CLK
#define X3P_CLK 0  // diagnostic builds: per-workgroup shader clocks / 100 MHz ticks
#endif
#if X3P_CLK
__device__ float g_x3p_clk[2 * 65536];
#endif

// (f16x2 128x128 8-wave tiles: four waves per SIMD -- two workgroups per CU,
// <= 128 VGPRs; HIP's second bound is waves per execution unit --
// the planes-out epilogue would otherwise tip them to 130 and one workgroup)
template <int BM, int BN, int WM, int WN, int EPI, int NS, bool A3, int S = 32>
__global__ void __launch_bounds__(64 * WM * WN,
                                  ((EPI & EPI_F_H2) && BM == 128 && BN == 128 && WM * WN == 8 &&
                                   NS == 2) ? 4 : 1)
gemm_x3p_kernel(GemmParams p, int tiles_m, int tiles_n) {
#if X3P_CLK
  const uint64_t clk0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  constexpr int BK = 32;
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / S;
  constexpr int TN = BN / WN / S;
  static_assert(S == 32 || (S == 16 && TN % 2 == 0), "MFMA block");
  // EPI_F_H2: f16x2 arithmetic -- f32 activations split into two f16 terms
  // after the fragment read (scale from their tensor's max), the weights as
  // two chunk-tiled f16 planes, three MFMA terms (mfma16_h2t)
  // With A3 the activations are two f16 planes already scaled and split
  // (pps_split_f16x2_act): no split arithmetic in the main loop, same bits.
  constexpr bool H2 = (EPI & EPI_F_H2) != 0;
  static_assert(!H2 || (S == 16 && !(EPI & (EPI_F_PLANES | EPI_F_RAW | EPI_F_FIX))),
                "f16x2 tiles: 16x16x32 blocks, plain epilogues");
  constexpr int NBP = H2 ? 2 : 3;       // weight planes
  constexpr int NAP = H2 ? 2 : 3;       // activation planes (A3)
  constexpr int A_PLANE = BM * BK * 2;  // A3: bf16 / f16 rows of 64 B per plane
  constexpr int A_BYTES = A3 ? NAP * A_PLANE : BM * BK * 4;  // else f32 rows of 128 B
  constexpr int B_PLANE = BN * BK * 2;  // bf16 rows of 64 B
  constexpr int STAGE = A_BYTES + NBP * B_PLANE;
  constexpr int AROWS = A3 ? 16 : 8;    // rows per A piece (1 KiB)
  constexpr int NPA = BM / AROWS;       // A pieces per chunk (per plane if A3)
  constexpr int NPB = BN / 16;          // B pieces (16 rows each) per plane and chunk
  // Pieces per wave.  Even tiles give every wave the same count (piece
  // q = wave * AI + i); otherwise the pieces go round-robin (q = i * NW +
  // wave) and the last slots of some waves are empty -- allowed with two
  // stages only, whose chunk wait is vmcnt(0) whatever a wave issued.
  constexpr bool AEVEN = NPA % NW == 0;
  constexpr bool BEVEN = NPB % NW == 0;
  constexpr int AI = (NPA + NW - 1) / NW;
  constexpr int BPW = (NPB + NW - 1) / NW;
  constexpr int NLOAD = (A3 ? NAP : 1) * AI + NBP * BPW;  // DMA instructions per wave and chunk
  static_assert(NPA * AROWS == BM && NPB * 16 == BN, "tile does not split into DMA pieces");
  // Uneven tiles: only a wave's last slot can be empty (round-robin), so a
  // wave issues NLOAD, NLOAD - (A3 ? 3 : 1) (A slot empty), NLOAD - 3 (B slot
  // empty) or both fewer DMA instructions per chunk; the chunk wait counts
  // its own (see chunk_barrier).
  constexpr int LA = A3 ? NAP : 1;
  static_assert(!(A3 && (EPI & EPI_F_DUAL)), "fused shortcut reads f32 activations");
  static_assert(TM >= 1 && TN >= 1 && (BM / WM) % S == 0 && (BN / WN) % S == 0, "wave tile");
  static_assert(NS >= 2 && NS <= 4 && NS * STAGE <= 160 * 1024, "LDS stages");
  static_assert(NLOAD * (NS - 2) <= 63, "vmcnt range");
  constexpr bool DUAL = (EPI & EPI_F_DUAL) != 0;

  // conv epilogue through LDS where the [BM][BN+4] tile fits the 160 KB:
  // 5-12 % faster on the epilogue-bound branch2c layers (residual + output
  // streams) for the 128-row tiles; the 8-wave 192x128 tile is faster
  // without it (scripts/gemm_probe.py --residual) except for f16x2 planes out,
  // whose 2-byte elements would leave as 32-byte row pieces
  // (scripts/probes/h2out_probe.py)
#ifndef X3P_LDSEPI
#define X3P_LDSEPI 1
#endif
  constexpr bool PPSEPI = (EPI & EPI_F_PPS) != 0;  // needs the LDS epilogue
  // PPS tiles whose [BM][BN+4] image + pooling scratch exceed the LDS (192 x
  // 256) park, finish and pool in two column passes
  constexpr int EHB = (PPSEPI && lds_epi_bytes<BM, BN>() + 2 * kPpsFuseMaxStrips * BN * 4 >
                                     160 * 1024) ? 2 : 1;
  constexpr int PPS_BYTES = PPSEPI ? 2 * kPpsFuseMaxStrips * (BN / EHB) * 4 : 0;
  static_assert(!PPSEPI || lds_epi_bytes<BM, BN / EHB>() + PPS_BYTES <= 160 * 1024,
                "part-power-set epilogue does not fit in LDS");
  constexpr bool LDSEPI = (X3P_LDSEPI || PPSEPI) &&
                          !(EPI & (EPI_DIST | EPI_F_RAW | EPI_F_PLANES)) &&
                          lds_epi_bytes<BM, BN / EHB>() <= 160 * 1024 &&
                          (PPSEPI || (EPI & EPI_F_H2OUT) != 0 ||
                           !(BM == 192 && BN == 128 && NW == 8));
#ifndef X3P_DISTLDS
#define X3P_DISTLDS 1
#endif
  constexpr bool DISTLDS = X3P_DISTLDS && (EPI & EPI_DIST) != 0 &&
                           lds_epi_bytes<BM, BN>() <= NS * STAGE;
  constexpr int LDS_BYTES =
      (LDSEPI && lds_epi_bytes<BM, BN / EHB>() + PPS_BYTES > NS * STAGE)
          ? lds_epi_bytes<BM, BN / EHB>() + PPS_BYTES
          : NS * STAGE;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[LDS_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // probes: the younger half of an 8-wave workgroup at raised priority for
  // the whole kernel (two waves per SIMD: the second-dispatched half loses
  // arbitration to the first at every segment start otherwise)
  if (X3P_PRIO == 2 && NW == 8 && wave >= 4) __builtin_amdgcn_s_setprio(1);
  const int wm = wave / WN;
  const int wn = wave - wm * WN;
  const int r32 = lane & (S - 1);  // lane's row within an MFMA block
  const int h = lane / S;          // its K slot (S = 16: 0..3) / column half (S = 32)

  const bool sym = (EPI & EPI_DIST) && p.sym;
  int tile_m, tile_n;
  if (sym) {
    // self-distance: the grid enumerates the upper triangle of SB x SB
    // super-blocks (SB = lcm(BM, BN), so non-square tiles tile them:
    // TPM x TPN tiles each), so every XCD gets an equal, contiguous share.
    // Grouped like the distance order below: GM super-block rows (~32 MB of
    // row panels) sweep their columns together (column-major inside the
    // group), so each column block is streamed once per group instead of
    // once per row panel.  The tiles of a super-block are consecutive ids
    // (one XCD after the remap).
    constexpr int SB = sym_block<BM, BN>();
    constexpr int TPM = SB / BM, TPN = SB / BN, TPS = TPM * TPN;
    const int n = (p.Ncol + SB - 1) / SB;
    const int kk = xcd_remap(blockIdx.x, TPS * (n * (n + 1) / 2));
    const int k = kk / TPS, t = kk - k * TPS;
    const int64_t panel = (int64_t)SB * p.Kloop * (A3 ? 6 : 4);
    const int64_t want = ((int64_t)X3P_GM_MB << 20) / (panel > 0 ? panel : 1);
    const int GM = (int)(want < 1 ? 1 : (want < n ? want : n));
    int g0 = 0, base = 0;
    for (;;) {  // find the group (at most n / GM + 1 steps)
      const int gm = n - g0 < GM ? n - g0 : GM;
      const int cnt = gm * (gm + 1) / 2 + gm * (n - g0 - gm);
      if (k < base + cnt || g0 + gm >= n) break;
      base += cnt;
      g0 += gm;
    }
    const int gm = n - g0 < GM ? n - g0 : GM;
    const int r = k - base;
    const int t1 = gm * (gm + 1) / 2;  // the group's own triangle, column c has c+1 blocks
    int sbm, sbn;
    if (r < t1) {
      int c = (int)((sqrt(8.0 * r + 1.0) - 1.0) * 0.5);
      while (c > 0 && c * (c + 1) / 2 > r) --c;
      while ((c + 1) * (c + 2) / 2 <= r) ++c;
      sbm = g0 + (r - c * (c + 1) / 2);
      sbn = g0 + c;
    } else {
      const int r2 = r - t1;
      sbn = g0 + gm + r2 / gm;
      sbm = g0 + r2 % gm;
    }
    tile_m = sbm * TPM + t / TPN;
    tile_n = sbn * TPN + t % TPN;
    // past the matrix (a partial last super-block), or strictly below the
    // diagonal (its mirror is written by another tile of the super-block):
    // the whole workgroup leaves before touching LDS or memory
    if (tile_m * BM >= p.M || tile_n * BN >= p.Ncol || tile_m * BM >= tile_n * BN + BN) return;
  } else {
    const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
    if (EPI & EPI_DIST) {
      // Grouped order: GM query panels sweep the gallery blocks together
      // (XCD-contiguous after the remap), GM sized so the group's panels
      // (~32 MB) stay in the Infinity Cache while every gallery block is
      // streamed once per group.  Market: GM = 7 of 14 panels, memory-side
      // traffic 5.6 -> 2.4 GB per launch and ~10 % faster than row-major
      // (which re-streams the 379 MB gallery planes once per panel).
      const int64_t panel = (int64_t)BM * p.Kloop * (A3 ? 6 : 4);
      const int64_t want = ((int64_t)X3P_GM_MB << 20) / (panel > 0 ? panel : 1);
      const int GM = (int)(want < 1 ? 1 : (want < tiles_m ? want : tiles_m));
      const int per = GM * tiles_n;
      const int grp = bid / per;
      const int first = grp * GM;
      const int gm = tiles_m - first < GM ? tiles_m - first : GM;
      const int r = bid - grp * per;
      tile_n = r / gm;
      tile_m = first + (r - tile_n * gm);
    } else if (p.colmajor) {  // consecutive ids (one XCD) share a weight block
      tile_n = bid / tiles_m;
      tile_m = bid - tile_n * tiles_m;
    } else {
      tile_m = bid / tiles_n;
      tile_n = bid - tile_m * tiles_n;
    }
  }
  const int m0 = tile_m * BM;
  const int n0 = tile_n * BN;
  const int batch = blockIdx.y / p.splitk;
  const int kslice = blockIdx.y - batch * p.splitk;
  const int64_t kofs0 = (int64_t)kslice * p.Kloop;
  const int64_t aofs0 = p.ksplit_conv ? 0 : kofs0;  // conv split: start tap instead

  // ---- A pieces: piece q = wave*AI + i covers tile rows 8q..8q+7; lane l
  // takes row 8q + (l >> 3) and fills physical chunk l & 7 with logical
  // chunk (l & 7) ^ ((row >> 1) & 7) (4 floats of the 32-wide K chunk).
  // A3: 16 rows per piece and plane, lane row 16q + (l >> 2), physical chunk
  // l & 3 holding logical chunk (l & 3) ^ ((row >> 2) & 3) (8 bf16)
  rsrc_t ra, ra1, ra2;
  if (A3) {
    const uint16_t* a3 = p.a3 + batch * p.a_bstride + aofs0;
    ra = make_rsrc(a3, p.a_bytes);
    ra1 = make_rsrc(a3 + p.a_plane, p.a_bytes);
    ra2 = make_rsrc(a3 + 2 * p.a_plane, p.a_bytes);
  } else {
    ra = make_rsrc(p.a + batch * p.a_bstride + aofs0, p.a_bytes);
    ra1 = ra;
    ra2 = DUAL ? make_rsrc(p.a2, p.a2_bytes) : ra;
  }
  // piece of slot i of this wave (>= NPA: an empty slot of an uneven tile)
  auto apiece = [&](int i) { return AEVEN ? wave * AI + i : i * NW + wave; };
  auto bpiece = [&](int j) { return BEVEN ? wave * BPW + j : j * NW + wave; };
  int abase[AI];
  uint64_t amask[AI];
  int abase2[AI];
  {
    const int hw = p.Ho * p.Wo;
    const int ntaps = p.KH * p.KW;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int rt = A3 ? apiece(i) * 16 + (lane >> 2) : apiece(i) * 8 + (lane >> 3);
      // first element (of the 32-wide K chunk) this lane fetches
      // (16x16x32 tiles: the group-aware swizzles of gemm_common.hpp)
      const int ce = A3 ? 8 * ((lane & 3) ^ (S == 16 ? sw64(rt) : ((rt >> 2) & 3)))
                        : 4 * ((lane & 7) ^ (S == 16 ? sw128(rt) : ((rt >> 1) & 7)));
      const int row = m0 + rt;
      const int rowc = row < p.M ? row : 0;
      const int n = rowc / hw;
      const int rem = rowc - n * hw;
      const int oh = rem / p.Wo;
      const int ow = rem - oh * p.Wo;
      const int ih0 = oh * p.stride - p.pad;
      const int iw0 = ow * p.stride - p.pad;
      abase[i] = ((n * p.H + ih0) * p.W + iw0) * p.lda + ce;
      if (A3 && (p.tiled & 1))  // plain rows (distance): [row / 16][K / 32][16][32]
        abase[i] = (rowc >> 4) * (p.lda / 32) * 512 + (rowc & 15) * 32 + ce;
      uint64_t m = 0;
      for (int t = 0, kh = 0, kw = 0; t < ntaps; ++t) {
        const int ih = ih0 + kh * p.dil, iw = iw0 + kw * p.dil;
        if ((unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W) m |= 1ull << t;
        if (++kw == p.KW) { kw = 0; ++kh; }
      }
      amask[i] = row < p.M ? m : 0ull;
      if (DUAL)
        abase2[i] = row < p.M ? (((n * p.H2 + oh * p.stride2) * p.W2 + ow * p.stride2) * p.lda2 +
                                 ce) * 4
                              : kOOB;
    }
  }

  // ---- B pieces: plane pl, piece q = wave*BPW + j covers tile columns
  // 16q..16q+15; lane l takes column 16q + (l >> 2) and fills physical chunk
  // l & 3 with logical chunk (l & 3) ^ ((col >> 2) & 3) = (l & 3) ^ ((l >> 4) & 3)
  // (chunk-tiled B: a 32-wide K chunk is 512 elements of a 16-column block)
  const uint16_t* b3 = p.b3 + batch * p.b_bstride + ((p.tiled & 2) ? kofs0 * 16 : kofs0);
  const rsrc_t rb0 = make_rsrc(b3, p.b_bytes);
  const rsrc_t rb1 = make_rsrc(b3 + p.b_plane, p.b_bytes);
  const rsrc_t rb2 = make_rsrc(b3 + 2 * p.b_plane, p.b_bytes);
  const int bcl = (lane & 3) ^ (S == 16 ? sw64(lane >> 2) : ((lane >> 4) & 3));
  int boff[BPW];
#pragma unroll
  for (int j = 0; j < BPW; ++j) {
    const int col = n0 + bpiece(j) * 16 + (lane >> 2);
    boff[j] = col < p.Ncol ? ((p.tiled & 2) ? ((col >> 4) * (p.ldb / 32) * 512 + (col & 15) * 32 +
                                                bcl * 8) * 2
                                             : (col * p.ldb + bcl * 8) * 2)
                           : kOOB;
  }

  // chunk strides: tiled planes advance a KiB per 32-wide chunk
  const int tcm = (A3 && (p.tiled & 1)) ? 16 : 1;
  const int bstep = (p.tiled & 2) ? 1024 : BK * 2;
  // ---- wave-uniform im2col tracker of the next chunk to request
  int tc = 0, tt = 0, tkw = 0, toff = 0;
  const int step_w = p.dil * p.lda;
  const int step_h = p.dil * p.lda * (p.W - p.KW);
  if (p.ksplit_conv && kslice) {  // this slice starts at tap t0, channel c0
    const int k0 = (int)kofs0;
    tt = k0 / p.Cin;
    tc = k0 - tt * p.Cin;
    tkw = tt % p.KW;
    toff = (tt / p.KW) * p.dil * p.lda * p.W + tkw * step_w;
  }
  const int nch1 = DUAL ? p.Kloop1 / BK : (1 << 30);
  int kiss = 0;  // next chunk to request
  int siss = 0;  // its LDS stage
  auto issue = [&]() {
    if (X3P_ABL == 1 && kiss >= NS) {  // probe: keep the counters, skip the DMA
      ++kiss;
      siss = siss + 1 == NS ? 0 : siss + 1;
      return;
    }
    const unsigned char* st = lds + siss * STAGE;
    if (DUAL && kiss >= nch1) {
      const int kofs = (kiss - nch1) * BK * 4;
#pragma unroll
      for (int i = 0; i < AI; ++i)
        if (AEVEN || apiece(i) < NPA)
          glds16(ra2, st + apiece(i) * 1024, abase2[i] == kOOB ? kOOB : abase2[i] + kofs);
    } else {
#pragma unroll
      for (int i = 0; i < AI; ++i) {
        if (!AEVEN && apiece(i) >= NPA) continue;  // wave-uniform: an empty slot
        const bool ok = tt < 64 && ((amask[i] >> tt) & 1ull);
        if (A3) {
          const int off = ok ? (abase[i] + toff + tc * tcm) * 2 : kOOB;
          const unsigned char* d = st + apiece(i) * 1024;
          glds16(ra, d, off);
          glds16(ra1, d + A_PLANE, off);
          if (!H2) glds16(ra2, d + 2 * A_PLANE, off);
        } else {
          glds16(ra, st + apiece(i) * 1024, ok ? (abase[i] + toff + tc) * 4 : kOOB);
        }
      }
      tc += BK;
      if (tc >= p.Cin) {
        tc = 0;
        ++tt;
        toff += step_w;
        if (++tkw == p.KW) { tkw = 0; toff += step_h; }
      }
    }
    const bool kok = kiss * BK + bcl * 8 < p.kb_valid;
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
      if (!BEVEN && bpiece(j) >= NPB) continue;
      const int off = (kok && boff[j] != kOOB) ? boff[j] + kiss * bstep : kOOB;
      const unsigned char* d = st + A_BYTES + bpiece(j) * 1024;
      glds16(rb0, d, off);
      glds16(rb1, d + B_PLANE, off);
      if (!H2) glds16(rb2, d + 2 * B_PLANE, off);
    }
    ++kiss;
    siss = siss + 1 == NS ? 0 : siss + 1;
  };

  typename AccT<S>::type acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < S * S / 64; ++r) acc[i][j][r] = 0.f;

  float h2s = 1.f;  // f16x2: the activation scale 2^s_a
  float inv_a = 0.f;  // and its inverse, for the epilogue (read once, here)
  if constexpr (H2) h2s = h2_act_scale(p, DUAL, &inv_a);
  // f16x2 planes out: the output bound, read now so its latency hides under
  // the main loop instead of stalling the epilogue
  float bnd_pre = 0.f;
  if constexpr ((EPI & EPI_F_H2OUT) != 0) bnd_pre = h2o_bound(p);
  // Fragment reads: the rows of this lane are r32 mod S, so both swizzles
  // are per-lane constants.
  const int asw = S == 16 ? sw128(r32) : (r32 >> 1) & 7;
  const int bsw = S == 16 ? sw64(r32) : (r32 >> 2) & 3;
  // chunk kc has landed for every wave once each wave saw its own pieces
  // retire (counted vmcnt: the NS-2 younger chunks stay in flight) and all
  // waves passed the barrier; the barrier also retires every wave's reads of
  // the stage the next request overwrites (lgkmcnt(0) before it)
  auto chunk_barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (NS == 2 || (AEVEN && BEVEN)) {
      wait_vmcnt<NLOAD * (NS - 2)>();
    } else {  // this wave's own count of younger DMA instructions
      const bool ea = !AEVEN && apiece(AI - 1) >= NPA;  // wave-uniform
      const bool eb = !BEVEN && bpiece(BPW - 1) >= NPB;
      if (!ea && !eb) wait_vmcnt<NLOAD * (NS - 2)>();
      else if (ea && !eb) wait_vmcnt<(NLOAD - LA) * (NS - 2)>();
      else if (!ea && eb) wait_vmcnt<(NLOAD - NBP) * (NS - 2)>();
      else wait_vmcnt<(NLOAD - LA - NBP) * (NS - 2)>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // Requests run NS-1 chunks ahead; requests past the last chunk read zeros
  // into stages that are never consumed, which keeps every wait count uniform.
  const int nchunks = (p.Kloop + BK - 1) / BK;
#pragma unroll
  for (int st = 0; st < NS - 1; ++st) issue();
  chunk_barrier();
  issue();
  if constexpr (S == 32) {
    // Fragment reads of one 16-wide K group g of a stage, A split into its
    // three bf16 terms.
    auto read_split = [&](const unsigned char* st, int g, bf16x8 (&fa)[TM][3],
                          bf16x8 (&fb)[TN][3]) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (A3) {
          const unsigned char* ap =
              st + (wm * (BM / WM) + i * 32 + r32) * 64 + (((2 * g + h) ^ bsw) << 4);
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            fa[i][pl] = *reinterpret_cast<const bf16x8*>(ap + pl * A_PLANE);
        } else {
          const unsigned char* rp = st + (wm * (BM / WM) + i * 32 + r32) * 128;
          const int c0 = 4 * g + 2 * h;
          const f32x4 x0 = *reinterpret_cast<const f32x4*>(rp + ((c0 ^ asw) << 4));
          const f32x4 x1 = *reinterpret_cast<const f32x4*>(rp + (((c0 + 1) ^ asw) << 4));
          split8(x0, x1, fa[i][0], fa[i][1], fa[i][2]);
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const unsigned char* bp =
            st + A_BYTES + (wn * (BN / WN) + j * 32 + r32) * 64 + (((2 * g + h) ^ bsw) << 4);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          fb[j][pl] = *reinterpret_cast<const bf16x8*>(bp + pl * B_PLANE);
      }
    };
    auto mfmas = [&](const bf16x8 (&fa)[TM][3], const bf16x8 (&fb)[TN][3]) {
      if (X3P_PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_x3t(fa[i], fb[j], acc[i][j]);
      if (X3P_PRIO == 1) __builtin_amdgcn_s_setprio(0);
    };
    // Software pipeline over 16-wide K groups (two per chunk): the reads and
    // the split of group q+1 are issued in the same basic block as the MFMAs
    // of group q, so the scheduler interleaves them.
    bf16x8 fa0[TM][3], fb0[TN][3], fa1[TM][3], fb1[TN][3];
    read_split(lds, 0, fa0, fb0);
    int scur = 0;
    for (int kc = 0; kc < nchunks - 1; ++kc) {
      const unsigned char* st = lds + scur * STAGE;
      scur = scur + 1 == NS ? 0 : scur + 1;
      read_split(st, 1, fa1, fb1);
      mfmas(fa0, fb0);
      chunk_barrier();
      issue();
      read_split(lds + scur * STAGE, 0, fa0, fb0);
      mfmas(fa1, fb1);
    }
    read_split(lds + scur * STAGE, 1, fa1, fb1);
    mfmas(fa0, fb0);
    mfmas(fa1, fb1);
  } else {
    // S = 16: a chunk is one 32-wide K group.  Its A fragments serve both
    // column halves, so A is double-buffered across chunks (fa0 / fa1
    // alternate; the loop runs two chunks per trip) and B per half.
    constexpr int TNH = TN / 2;
    auto readA16 = [&](const unsigned char* st, bf16x8 (&fa)[TM][3]) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (A3) {
          const unsigned char* ap =
              st + (wm * (BM / WM) + i * 16 + r32) * 64 + ((h ^ bsw) << 4);
#pragma unroll
          for (int pl = 0; pl < NAP; ++pl)
            fa[i][pl] = *reinterpret_cast<const bf16x8*>(ap + pl * A_PLANE);
        } else {
          const unsigned char* rp = st + (wm * (BM / WM) + i * 16 + r32) * 128;
          const f32x4 x0 = *reinterpret_cast<const f32x4*>(rp + (((2 * h) ^ asw) << 4));
          const f32x4 x1 = *reinterpret_cast<const f32x4*>(rp + (((2 * h + 1) ^ asw) << 4));
          if (H2)
            split8_h2(x0, x1, h2s, fa[i][0], fa[i][1]);
          else
            split8(x0, x1, fa[i][0], fa[i][1], fa[i][2]);
        }
      }
    };
    auto readB16 = [&](const unsigned char* st, int half, bf16x8 (&fb)[TNH][3]) {
#pragma unroll
      for (int jj = 0; jj < TNH; ++jj) {
        const unsigned char* bp = st + A_BYTES +
                                  (wn * (BN / WN) + (half * TNH + jj) * 16 + r32) * 64 +
                                  ((h ^ bsw) << 4);
#pragma unroll
        for (int pl = 0; pl < NBP; ++pl)
          fb[jj][pl] = *reinterpret_cast<const bf16x8*>(bp + pl * B_PLANE);
      }
    };
    auto mfmas16 = [&](const bf16x8 (&fa)[TM][3], const bf16x8 (&fb)[TNH][3], int half) {
      if (X3P_PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int jj = 0; jj < TNH; ++jj) {
          if (X3P_ABL == 2) {  // probe: fragments kept live, no MFMA
            asm volatile("" ::"v"(fa[i][0]), "v"(fa[i][1]), "v"(fb[jj][0]), "v"(fb[jj][1]));
            continue;
          }
          acc[i][half * TNH + jj] = H2 ? mfma16_h2t(fa[i], fb[jj], acc[i][half * TNH + jj])
                                       : mfma16_x3t(fa[i], fb[jj], acc[i][half * TNH + jj]);
        }
      if (X3P_PRIO == 1) __builtin_amdgcn_s_setprio(0);
    };
    bf16x8 fa0[TM][3], fa1[TM][3], fb0[TNH][3], fb1[TNH][3];
    readA16(lds, fa0);
    readB16(lds, 0, fb0);
    int scur = 0;
    // one chunk: MFMAs of half 0 beside the reads of half 1, barrier +
    // request, then the next chunk's A / half-0 B beside half 1's MFMAs
    auto step = [&](bf16x8 (&fc)[TM][3], bf16x8 (&fn)[TM][3]) {
      const unsigned char* st = lds + scur * STAGE;
      scur = scur + 1 == NS ? 0 : scur + 1;
      readB16(st, 1, fb1);
      mfmas16(fc, fb0, 0);
      chunk_barrier();
      issue();
      readA16(lds + scur * STAGE, fn);
      readB16(lds + scur * STAGE, 0, fb0);
      mfmas16(fc, fb1, 1);
    };
    // the same chunk with both column halves multiplied before the barrier:
    // with X3P_STAG one half of an 8-wave workgroup runs it, so the two waves
    // of a SIMD carry different amounts of MFMA work across the barrier and
    // the one that reaches it first leaves the matrix pipe to its partner
    // (MI355X_MICROARCH "try a stagger")
    auto step_pre = [&](bf16x8 (&fc)[TM][3], bf16x8 (&fn)[TM][3]) {
      const unsigned char* st = lds + scur * STAGE;
      scur = scur + 1 == NS ? 0 : scur + 1;
      readB16(st, 1, fb1);
      mfmas16(fc, fb0, 0);
      mfmas16(fc, fb1, 1);
      chunk_barrier();
      issue();
      readA16(lds + scur * STAGE, fn);
      readB16(lds + scur * STAGE, 0, fb0);
    };
    auto tail = [&](bf16x8 (&fc)[TM][3]) {
      readB16(lds + scur * STAGE, 1, fb1);
      mfmas16(fc, fb0, 0);
      mfmas16(fc, fb1, 1);
    };
    auto run = [&](auto&& stp) {
      int kc = 0;
      for (; kc + 2 < nchunks; kc += 2) {
        stp(fa0, fa1);
        stp(fa1, fa0);
      }
      if (kc + 1 < nchunks) {
        stp(fa0, fa1);
        tail(fa1);
      } else {
        tail(fa0);
      }
    };
    // tile 52 (192 x 128, 4 x 2 waves, three stages): res5 3x3 166.8 / 171.7
    // -> 155.1 / 160.0 us with the younger half staggered; the 128 x 128 8-wave
    // tile (two workgroups per CU, <= 128 VGPRs) loses 50 % with it, tiles 47
    // and 53 are level (scripts/gpu_r6_stagger.sh)
#ifndef X3P_STAG51
#define X3P_STAG51 0  // probes: 1 = the stagger on tile 51 (128 x 128, 4 x 2 waves, three stages) too
#endif
    constexpr int STAG = X3P_STAG >= 0 ? X3P_STAG
                                       : ((BM == 192 || (X3P_STAG51 && BM == 128)) && BN == 128 &&
                                          WM == 4 && WN == 2 && NS == 3);
    if (STAG != 0 && NW == 8 && (STAG == 1 ? wave >= NW / 2 : wave < NW / 2))
      run(step_pre);
    else
      run(step);
  }
  wait_vmcnt<0>();  // no DMA may land in LDS after the workgroup retires
#if X3P_CLK
  {
    const uint64_t clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    const int wg = blockIdx.x + gridDim.x * blockIdx.y;
    if (threadIdx.x == 0 && wg < 65536) {
      g_x3p_clk[2 * wg] = (float)(clk1 - clk0);
      g_x3p_clk[2 * wg + 1] = (float)(rt1 - rt0);
    }
  }
#endif

  if constexpr ((EPI & EPI_F_FIX) != 0) {
    if (!fix_reduce<BM, BN, WM, WN, S>(p, acc, lds, kslice, blockIdx.x + gridDim.x * batch, m0,
                                       n0, wm, wn, r32, h))
      return;
  }
  if constexpr (DISTLDS) {
    if (p.sym)
      dist_epilogue_sym_lds<BM, BN, WM, WN, S>(p, acc, lds, m0, n0, wm, wn, r32, h);
    else
      dist_epilogue_lds<BM, BN, WM, WN, S>(p, acc, lds, m0, n0, wm, wn, r32, h);
  } else if constexpr ((EPI & EPI_DIST) != 0)
    dist_epilogue_t<BM, BN, WM, WN, S>(p, acc, m0, n0, wm, wn, r32, h);
  else if constexpr (LDSEPI)
    conv_epilogue_lds<EPI, BM, BN, WM, WN, S, EHB>(p, acc, lds, batch, kslice, m0, n0, wm, wn, r32,
                                                  h, bnd_pre, inv_a);
  else
    conv_epilogue_t<EPI, BM, BN, WM, WN, S>(p, acc, batch, kslice, m0, n0, wm, wn, r32, h,
                                            bnd_pre, inv_a);
}

template <int BM, int BN, int WM, int WN, int NS, int EPI, bool A3, int S>
static void launch_one_p(const GemmParams& p, int batch, hipStream_t stream) {
  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.Ncol + BN - 1) / BN;
  // self-distance (M == Ncol): the tiles of the upper-triangle super-blocks
  constexpr int SB = sym_block<BM, BN>();
  const int nsb = (p.Ncol + SB - 1) / SB;
  const int nblk = ((EPI & EPI_DIST) && p.sym) ? (SB / BM) * (SB / BN) * (nsb * (nsb + 1) / 2)
                                               : tiles_m * tiles_n;
  hipLaunchKernelGGL((gemm_x3p_kernel<BM, BN, WM, WN, EPI, NS, A3, S>),
                     dim3(nblk, batch * p.splitk), dim3(64 * WM * WN), 0, stream, p, tiles_m,
                     tiles_n);
}

// f16x2 arithmetic: f32 activations, chunk-tiled two-plane weights, the
// conv epilogues of a ResNet bottleneck (16x16x32 tiles only)
template <int BM, int BN, int WM, int WN, int NSF>
static int launch_tile_h2(const GemmParams& p, int epi, int batch, hipStream_t stream) {
  constexpr int C = EPI_CONV, RL = EPI_F_RELU, RS = EPI_F_RES, H = EPI_F_H2, S = 16;
  if (!(p.tiled & 2) || !p.rs_b || !p.amax_a || ((epi & EPI_F_DUAL) && (!p.amax_a2 || p.a3))) {
    set_error("f16x2 conv: activations (f32, or f16x2 planes) with their max, chunk-tiled "
              "weights and scales; the fused shortcut reads f32");
    return PPS_ERR_INVALID_ARG;
  }
  constexpr int HO = EPI_F_H2OUT;
  if (p.a3) {   // f16x2 activation planes (pps_split_f16x2_act or a producer's EPI_F_H2OUT)
    switch (epi & ~H) {
      case C | RL: launch_one_p<BM, BN, WM, WN, NSF, C | RL | H, true, S>(p, batch, stream); break;
      case C | RL | HO:
        launch_one_p<BM, BN, WM, WN, NSF, C | RL | HO | H, true, S>(p, batch, stream); break;
      case C | RS | RL:
        launch_one_p<BM, BN, WM, WN, NSF, C | RS | RL | H, true, S>(p, batch, stream); break;
      case C | RS | RL | EPI_F_PPS:
        if constexpr (BM == 192 && BN <= 256) {
          launch_one_p<BM, BN, WM, WN, NSF, C | RS | RL | EPI_F_PPS | H, true, S>(p, batch, stream);
          break;
        } else {
          set_error("part-power-set epilogue needs a 192-row tile with at most 256 columns");
          return PPS_ERR_INVALID_ARG;
        }
      default:
        set_error("f16x2 conv on activation planes: conv + BN + ReLU [+ residual | part "
                  "pooling] only");
        return PPS_ERR_INVALID_ARG;
    }
    PPS_CHECK_LAUNCH("gemm_x3p_kernel");
    return PPS_OK;
  }
  switch (epi & ~H) {
    case C | RL: launch_one_p<BM, BN, WM, WN, NSF, C | RL | H, false, S>(p, batch, stream); break;
    case C | RL | HO:
      launch_one_p<BM, BN, WM, WN, NSF, C | RL | HO | H, false, S>(p, batch, stream); break;
    case C | RS | RL:
      launch_one_p<BM, BN, WM, WN, NSF, C | RS | RL | H, false, S>(p, batch, stream); break;
    case C | RL | EPI_F_DUAL:
      launch_one_p<BM, BN, WM, WN, NSF, C | RL | EPI_F_DUAL | H, false, S>(p, batch, stream);
      break;
    case C | RS | RL | EPI_F_PPS:
      if constexpr (BM == 192 && BN <= 256) {
        launch_one_p<BM, BN, WM, WN, NSF, C | RS | RL | EPI_F_PPS | H, false, S>(p, batch, stream);
        break;
      } else {
        set_error("part-power-set epilogue needs a 192-row tile with at most 256 columns");
        return PPS_ERR_INVALID_ARG;
      }
    default:
      set_error("f16x2 conv: conv + BN + ReLU [+ residual | shortcut | part pooling] only");
      return PPS_ERR_INVALID_ARG;
  }
  PPS_CHECK_LAUNCH("gemm_x3p_kernel");
  return PPS_OK;
}

// NSF / NSP: LDS stages with f32 / bf16-plane A operands (NSP = 0: the tile
// does not take plane activations)
// FX: also built with the one-launch split-K epilogues (EPI_F_FIX)
template <int BM, int BN, int WM, int WN, int NSF, int NSP, int S, bool FX = false>
static int launch_tile_p(const GemmParams& p, int epi, int batch, hipStream_t stream) {
  constexpr int C = EPI_CONV, RL = EPI_F_RELU, RS = EPI_F_RES, PL = EPI_F_PLANES;
  if (epi & EPI_F_H2) {
    if constexpr (S == 16) {
      return launch_tile_h2<BM, BN, WM, WN, NSF>(p, epi, batch, stream);
    } else {
      set_error("f16x2 conv needs a 16x16x32 tile (38..53, 55, 60)");
      return PPS_ERR_INVALID_ARG;
    }
  }
  if (epi & EPI_F_FIX) {
    if constexpr (FX && NSP != 0) {
      constexpr int F = EPI_F_FIX;
      const bool a3 = p.a3 != nullptr;
      switch (epi) {
        case C | RL | F:
          if (a3) launch_one_p<BM, BN, WM, WN, NSP, C | RL | F, true, S>(p, batch, stream);
          else launch_one_p<BM, BN, WM, WN, NSF, C | RL | F, false, S>(p, batch, stream);
          break;
        case C | RL | PL | F:
          if (a3) launch_one_p<BM, BN, WM, WN, NSP, C | RL | PL | F, true, S>(p, batch, stream);
          else launch_one_p<BM, BN, WM, WN, NSF, C | RL | PL | F, false, S>(p, batch, stream);
          break;
        case C | RS | RL | F:
          if (a3) launch_one_p<BM, BN, WM, WN, NSP, C | RS | RL | F, true, S>(p, batch, stream);
          else launch_one_p<BM, BN, WM, WN, NSF, C | RS | RL | F, false, S>(p, batch, stream);
          break;
        default:
          set_error("one-launch split-K: conv + BN + ReLU [+ residual | planes] only");
          return PPS_ERR_INVALID_ARG;
      }
      PPS_CHECK_LAUNCH("gemm_x3p_kernel");
      return PPS_OK;
    } else {
      set_error("tile not built for one-launch split-K");
      return PPS_ERR_INVALID_ARG;
    }
  }
  if constexpr (NSP == 0) {
    if (p.a3) {
      set_error("tile not built for bf16-plane activations");
      return PPS_ERR_INVALID_ARG;
    }
  }
  if (epi & EPI_F_PPS) {
    // the fused part-power-set epilogue: conv + BN + residual + ReLU, one
    // image per 192-row tile (Market's 24 x 8 res5 output)
    if constexpr (BM == 192 && BN <= 256) {
      if (epi != (C | RS | RL | EPI_F_PPS)) {
        set_error("part-power-set epilogue: conv + BN + residual + ReLU only");
        return PPS_ERR_INVALID_ARG;
      }
      if (p.a3) {
        if constexpr (NSP != 0) launch_one_p<BM, BN, WM, WN, NSP, C | RS | RL | EPI_F_PPS, true, S>(p, batch, stream);
        else { set_error("tile not built for bf16-plane activations"); return PPS_ERR_INVALID_ARG; }
      } else {
        launch_one_p<BM, BN, WM, WN, NSF, C | RS | RL | EPI_F_PPS, false, S>(p, batch, stream);
      }
      PPS_CHECK_LAUNCH("gemm_x3p_kernel");
      return PPS_OK;
    } else {
      set_error("part-power-set epilogue needs a 192-row tile with at most 256 columns");
      return PPS_ERR_INVALID_ARG;
    }
  }
  if constexpr (NSP != 0) {
  if (p.a3) {
    switch (epi) {
      case EPI_DIST: launch_one_p<BM, BN, WM, WN, NSP, EPI_DIST, true, S>(p, batch, stream); break;
      case C: launch_one_p<BM, BN, WM, WN, NSP, C, true, S>(p, batch, stream); break;
      case C | EPI_F_RAW:
        launch_one_p<BM, BN, WM, WN, NSP, C | EPI_F_RAW, true, S>(p, batch, stream); break;
      case C | RL: launch_one_p<BM, BN, WM, WN, NSP, C | RL, true, S>(p, batch, stream); break;
      case C | RS | RL: launch_one_p<BM, BN, WM, WN, NSP, C | RS | RL, true, S>(p, batch, stream); break;
      case C | PL: launch_one_p<BM, BN, WM, WN, NSP, C | PL, true, S>(p, batch, stream); break;
      case C | RL | PL: launch_one_p<BM, BN, WM, WN, NSP, C | RL | PL, true, S>(p, batch, stream); break;
      default:
        set_error("epilogue not built for bf16-plane activations");
        return PPS_ERR_INVALID_ARG;
    }
    PPS_CHECK_LAUNCH("gemm_x3p_kernel");
    return PPS_OK;
  }
  }
  switch (epi) {
    case EPI_DIST: launch_one_p<BM, BN, WM, WN, NSF, EPI_DIST, false, S>(p, batch, stream); break;
    case C: launch_one_p<BM, BN, WM, WN, NSF, C, false, S>(p, batch, stream); break;
    case C | RL: launch_one_p<BM, BN, WM, WN, NSF, C | RL, false, S>(p, batch, stream); break;
    case C | RS: launch_one_p<BM, BN, WM, WN, NSF, C | RS, false, S>(p, batch, stream); break;
    case C | RS | RL: launch_one_p<BM, BN, WM, WN, NSF, C | RS | RL, false, S>(p, batch, stream); break;
    case C | EPI_F_RAW:
      launch_one_p<BM, BN, WM, WN, NSF, C | EPI_F_RAW, false, S>(p, batch, stream); break;
    case C | RL | EPI_F_DUAL:
      launch_one_p<BM, BN, WM, WN, NSF, C | RL | EPI_F_DUAL, false, S>(p, batch, stream); break;
    case C | PL: launch_one_p<BM, BN, WM, WN, NSF, C | PL, false, S>(p, batch, stream); break;
    case C | RL | PL: launch_one_p<BM, BN, WM, WN, NSF, C | RL | PL, false, S>(p, batch, stream); break;
    case C | RL | EPI_F_H2OUT:
      if constexpr (S == 16) {
        launch_one_p<BM, BN, WM, WN, NSF, C | RL | EPI_F_H2OUT, false, S>(p, batch, stream);
        break;
      } else {
        set_error("f16x2 planes out: a 16x16x32 tile");
        return PPS_ERR_INVALID_ARG;
      }
    default:
      set_error("unknown epilogue for the pipelined bf16x3 GEMM");
      return PPS_ERR_INVALID_ARG;
  }
  PPS_CHECK_LAUNCH("gemm_x3p_kernel");
  return PPS_OK;
}

// The DMA pieces need 16-byte-aligned 4-float (or 8-bf16) A slots, 8-element
// B slots and a 32-wide K chunk inside one tap (and, with a fused shortcut, a
// K switch on a chunk boundary); the epilogue moves 4-column vectors.
static bool al16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }
bool x3p_eligible(const GemmParams& p, int epi) {
  if (p.Cin % 32 != 0 || p.ldb % 8 != 0) return false;
  if (p.a3 ? (p.lda % 8 != 0 || p.a2 || !al16(p.a3) || p.a_plane % 8 != 0) : p.lda % 4 != 0)
    return false;
  if (p.a2 && (p.Kloop1 % 32 != 0 || (p.Kloop - p.Kloop1) % 32 != 0 || p.lda2 % 4 != 0))
    return false;
  // 16-byte epilogue vectors (the distance epilogue falls back per row)
  if (!(epi & EPI_DIST)) {
    if (p.Ncol % 4 != 0 || p.ldo % 4 != 0) return false;
    if ((epi & (EPI_F_PLANES | EPI_F_H2OUT)) ? (!p.out3 || !al16(p.out3) || p.out_plane % 4 != 0)
                                              : !al16(p.out))
      return false;
    if (p.residual && (p.ldr % 4 != 0 || !al16(p.residual))) return false;
    if ((p.scale && !al16(p.scale)) || (p.shift && !al16(p.shift)) || p.out_bstride % 4 != 0 ||
        p.out_sstride % 4 != 0 || p.ss_bstride % 4 != 0)
      return false;
  }
  return true;
}

// variants 0..8: 32x32x16 MFMA blocks (bit-identical to gemm_x3.hip);
// 9..17: the same tiles on 16x16x32 MFMA blocks (bit-identical among
// themselves, f32-level like the others).
template <int S>
static int launch_variant(const GemmParams& p, int epi, int batch, hipStream_t stream, int v) {
  switch (v) {
    // 4-wave tiles up to 80 KB of LDS take two stages: two workgroups per CU,
    // so one's epilogue overlaps the other's loads (measured 10-30 % faster
    // than three stages at one workgroup per CU on every layer shape,
    // scripts/gemm_probe.py); 192x128 needs 96 KB for two stages anyway
    case 0: return launch_tile_p<128, 128, 2, 2, 2, 2, S>(p, epi, batch, stream);
    case 1: return launch_tile_p<192, 128, 2, 2, 3, 2, S>(p, epi, batch, stream);
    case 2: return launch_tile_p<128, 64, 2, 2, 2, 2, S>(p, epi, batch, stream);
    case 3: return launch_tile_p<192, 64, 2, 2, 2, 2, S>(p, epi, batch, stream);
    case 4: return launch_tile_p<256, 128, 4, 2, 2, 2, S>(p, epi, batch, stream);
    case 5: return launch_tile_p<128, 256, 2, 4, 2, 2, S>(p, epi, batch, stream);
    case 6:
      // 192x256 with plane A needs 168 KB for two stages, and on 16x16 blocks
      // more than the 256 VGPRs of an 8-wave workgroup: 128x256 instead
      if (p.a3 || S == 16) return launch_tile_p<128, 256, 2, 4, 2, 2, S>(p, epi, batch, stream);
      if constexpr (S == 32) return launch_tile_p<192, 256, 2, 4, 2, 0, S>(p, epi, batch, stream);
    // 8-wave versions of 128x128 / 192x128 (two waves per SIMD in one
    // workgroup; 128x128 also two workgroups per CU): res3/res4 3x3 and
    // res4 2c run 6-10 % faster on them
    case 7: return launch_tile_p<128, 128, 4, 2, 2, 2, S, S == 16>(p, epi, batch, stream);
    case 8:  // plane A: 12 pieces of 16 rows over 8 waves (uneven, two stages)
      return launch_tile_p<192, 128, 2, 4, 2, 2, S>(p, epi, batch, stream);
    default:
      set_error("unknown pipelined GEMM variant " + std::to_string(v));
      return PPS_ERR_INVALID_ARG;
  }
}

// Rows (BM) of the tile a pipelined id launches (as launch_variant /
// launch_gemm_x3p map it), 0 for a non-pipelined id.
int x3p_tile_rows(int tile, bool a3) {
  if (tile == GEMM_TILE_P16_64x128W24S4) return 64;
  if (tile == GEMM_TILE_P16_192x128W41) return 192;
  if (tile < GEMM_TILE_P_FIRST || tile >= GEMM_TILE_WS) return 0;
  if (tile == GEMM_TILE_P16_192x128W42 || tile == GEMM_TILE_P16_192x64W41 ||
      tile == GEMM_TILE_P16_192x128W42S3 || tile == GEMM_TILE_P16_192x128W41)
    return 192;
  if (tile == GEMM_TILE_P16_128x128W42S3) return 128;
  if (tile == GEMM_TILE_P16_96x128W22 || tile == GEMM_TILE_P16_96x128W24 ||
      tile == GEMM_TILE_P16_96x128W24S3)
    return 96;
  constexpr int NV = GEMM_TILE_P16_FIRST - GEMM_TILE_P_FIRST;
  const int v = (tile - GEMM_TILE_P_FIRST) % NV;
  const bool s16 = tile >= GEMM_TILE_P16_FIRST;
  switch (v) {
    case 0: case 2: case 5: case 7: return 128;
    case 1: case 3: return 192;
    case 4: return 256;
    case 6: return (a3 || s16) ? 128 : 192;
    case 8: return 192;
    default: return 0;
  }
}

// Columns (BN) of that tile.
int x3p_tile_cols(int tile, bool a3) {
  if (tile == GEMM_TILE_P16_64x128W24S4 || tile == GEMM_TILE_P16_192x128W41) return 128;
  if (tile < GEMM_TILE_P_FIRST || tile >= GEMM_TILE_WS) return 0;
  if (tile == GEMM_TILE_P16_192x128W42 || tile == GEMM_TILE_P16_96x128W22 ||
      tile == GEMM_TILE_P16_96x128W24 || tile == GEMM_TILE_P16_128x128W42S3 ||
      tile == GEMM_TILE_P16_192x128W42S3 || tile == GEMM_TILE_P16_96x128W24S3)
    return 128;
  if (tile == GEMM_TILE_P16_192x64W41) return 64;
  constexpr int NV = GEMM_TILE_P16_FIRST - GEMM_TILE_P_FIRST;
  const int v = (tile - GEMM_TILE_P_FIRST) % NV;
  (void)a3;
  switch (v) {
    case 2: case 3: return 64;
    case 5: case 6: return 256;
    default: return 128;
  }
}

int launch_gemm_x3p(const GemmParams& p, int epi, int batch, hipStream_t stream, int variant) {
  constexpr int NV = GEMM_TILE_P16_FIRST - GEMM_TILE_P_FIRST;  // variants per block size
  // plane A on the 192-row 8-wave and 96-row tiles: 12 / 6 pieces of 16 rows
  // spread unevenly over the waves (two stages)
  if (variant == GEMM_TILE_P16_192x128W42 - GEMM_TILE_P_FIRST)
    return launch_tile_p<192, 128, 4, 2, 2, 2, 16, true>(p, epi, batch, stream);
  if (variant == GEMM_TILE_P16_192x64W41 - GEMM_TILE_P_FIRST)
    return launch_tile_p<192, 64, 4, 1, 2, 2, 16, true>(p, epi, batch, stream);
  if (variant == GEMM_TILE_P16_96x128W22 - GEMM_TILE_P_FIRST)
    return launch_tile_p<96, 128, 2, 2, 2, 2, 16, true>(p, epi, batch, stream);
  // 96x128 with 8 waves as 2 x 4 (48 x 32 per wave): 256 tiles for
  // M = 12,288 x N = 256 at two waves per SIMD
  if (variant == GEMM_TILE_P16_96x128W24 - GEMM_TILE_P_FIRST)
    return launch_tile_p<96, 128, 2, 4, 2, 2, 16, true>(p, epi, batch, stream);
  // three LDS stages (two chunks in flight behind the one being consumed) on
  // the 8-wave 128x128 / 192x128 tiles, for long-K GEMMs whose operands come
  // from the Infinity Cache rather than L2 (distance matrix, res5);
  // 192-row plane A keeps two stages (uneven pieces)
#ifndef X3P_DEEP
#define X3P_DEEP 0  // probes: 1 = four LDS stages for f32 A on tiles 51 / 53
#endif
  if (variant == GEMM_TILE_P16_128x128W42S3 - GEMM_TILE_P_FIRST)
    return launch_tile_p<128, 128, 4, 2, X3P_DEEP ? 4 : 3, 3, 16>(p, epi, batch, stream);
#ifndef X3P_DEEP52
#define X3P_DEEP52 0  // probes: 1 = four LDS stages (160 KB) on tile 52
#endif
  if (variant == GEMM_TILE_P16_192x128W42S3 - GEMM_TILE_P_FIRST) {
    if (X3P_DEEP52 && (epi & EPI_F_H2)) return launch_tile_h2<192, 128, 4, 2, 4>(p, epi, batch, stream);
    return launch_tile_p<192, 128, 4, 2, 3, 2, 16>(p, epi, batch, stream);
  }
  // 96x128 as 2 x 4 waves with three stages (uneven pieces, per-wave waits)
  if (variant == GEMM_TILE_P16_96x128W24S3 - GEMM_TILE_P_FIRST)
    return launch_tile_p<96, 128, 2, 4, X3P_DEEP ? 4 : 3, 3, 16>(p, epi, batch, stream);
  // 64x128, 8 waves as 2 x 4, four stages (three chunks in flight): the
  // 64-row split-K head GEMMs, whose 8-chunk slices are all pipeline fill
  if (variant == GEMM_TILE_P16_64x128W24S4 - GEMM_TILE_P_FIRST)
    return launch_tile_p<64, 128, 2, 4, 4, 4, 16>(p, epi, batch, stream);
  // f16x2 only: 192x128 as 4 x 1 waves (48 x 128 per wave): each activation
  // fragment split once feeds eight 16x16 column blocks (the split is the
  // f16x2 kernels' VALU cost; 4 x 2 waves split every fragment twice and
  // feed four).  bf16x3 launches of this id run tile 47 (same rounding group).
  if (variant == GEMM_TILE_P16_192x128W41 - GEMM_TILE_P_FIRST) {
    if (epi & EPI_F_H2) return launch_tile_h2<192, 128, 4, 1, 2>(p, epi, batch, stream);
    return launch_tile_p<192, 128, 4, 2, 2, 2, 16, true>(p, epi, batch, stream);
  }
  if (variant >= NV) return launch_variant<16>(p, epi, batch, stream, variant - NV);
  return launch_variant<32>(p, epi, batch, stream, variant);
}

}  // namespace pps

#if X3P_CLK
extern "C" int pps_debug_x3p_clocks(float* dst, int n) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(pps::g_x3p_clk), sizeof(float) * n) == hipSuccess
             ? 0
             : -1;
}
#endif
