// f16x2 distance GEMM for gfx950 ("h2"): the query x gallery dot products of
// compute_dist (reid_dataset_evaluator.py:244-272) and the self-distances of
// re-ranking (:169-175) on f16 matrix cores with f32-level error, in three
// MFMA terms per product instead of the six of the bf16x3 kernels.
//
// Numerics.  Each feature row x is scaled by a power of two 2^s chosen per
// row so that max|x 2^s| lies in [2^14, 2^15) (far inside the f16 range), and
// split exactly as x 2^s = h0 + h1 + r with h0 = f16(x 2^s), h1 = f16(x 2^s -
// h0): the f16 significand has 11 bits, so |x 2^s - h0| <= 2^-11 |x 2^s| and
// |r| <= 2^-22 |x 2^s| (h1 is f16-subnormal only for entries below 2^-3, i.e.
// below 2^-17 of the row maximum, where |r| <= 2^-25 -- 2^-39 of the row
// maximum).  A dot product
// q.g is accumulated in f32 from h0.h0' + h0.h1' + h1.h0' (f16 x f16 products
// are exact in f32; the dropped h1.h1' and the residuals are <= ~3 x 2^-22 of
// |q_k g_k| per term) and scaled back by 2^-(s + s') -- an exact power-of-two
// multiply.  Per product that is 2^-22-level, below the f32 accumulation
// error of a 4k-term sum; the parity tests hold it to the same distance and
// near-tie bounds as the bf16x3 kernels.  Rows are independent, so the scale
// needs no global reduction.
//
// Kernel.  Both operands are chunk-tiled f16 planes [2][rows16/16][D/32][16]
// [32] (pps_split_f16x2_sqnorm_tiled), so each 16-row block of a 32-wide K
// chunk is one contiguous KiB and travels global -> LDS by one LDS-DMA
// instruction (buffer_load_dwordx4 ... lds).  Two planes instead of three let
// a 256 x 256 tile double-buffer its chunks in 128 KiB of LDS: per chunk a CU
// stages 64 KiB and issues 3 x (256/16)^2 = 768 MFMAs (v_mfma_f32_16x16x32_f16),
// the same staged bytes per MFMA as the 128 x 256 bf16x3 tile with half the
// L2 / Infinity-Cache fetch per output.  Two LDS stages: chunk c + 1 is
// requested right after the barrier that retires chunk c - 1, so it has a
// whole chunk of MFMAs to land; each wave reads its A fragments one 16-row
// block ahead of the MFMAs and the next chunk's B fragments (and first A
// block) beside the last block's MFMAs.  Tile order as in gemm_x3p.hip:
// grouped query panels for q x g, upper-triangle super-blocks + mirror for the
// self-distance.  The epilogue parks the accumulators in LDS (column passes
// when the tile's f32 image exceeds it) and writes whole row segments.
#include <type_traits>

#include "gemm_x3p_common.hpp"

namespace pps {

// The three terms with the gallery fragment as the MFMA "A" operand, so the
// accumulator is transposed like the x3p kernels': lane l keeps query row
// (l & 15) and gallery columns 4 (l >> 4) + e, e = 0..3.
__device__ inline f32x4 mfma_h2t(const f16x8& a0, const f16x8& a1, const f16x8& b0,
                                 const f16x8& b1, f32x4 c) {
#if H2_ABL == 2
  asm volatile("" ::"v"(a0), "v"(a1), "v"(b0), "v"(b1));
  return c;
#endif
  c = mfma16_f16(b0, a0, c);
  c = mfma16_f16(b1, a0, c);
  c = mfma16_f16(b0, a1, c);
  return c;
}

// Output tile of this workgroup (false: nothing to do -- a self-distance tile
// strictly below the diagonal or past the matrix).  `row_bytes` = bytes of one
// operand row over all planes (sizes the query-panel groups).
template <int BM, int BN>
__device__ inline bool dist_tile_coords(const GemmParams& p, int tiles_m, int tiles_n,
                                        int64_t row_bytes, int& tile_m, int& tile_n) {
  if (p.sym) {
    // upper triangle of SB x SB super-blocks (SB = lcm(BM, BN)), grouped: GM
    // super-block rows (~32 MB of panels) sweep their columns together
    constexpr int SB = sym_block<BM, BN>();
    constexpr int TPM = SB / BM, TPN = SB / BN, TPS = TPM * TPN;
    const int n = (p.Ncol + SB - 1) / SB;
    const int kk = xcd_remap(blockIdx.x, TPS * (n * (n + 1) / 2));
    const int k = kk / TPS, t = kk - k * TPS;
    const int64_t panel = (int64_t)SB * row_bytes;
    const int64_t want = ((int64_t)X3P_GM_MB << 20) / (panel > 0 ? panel : 1);
    const int GM = (int)(want < 1 ? 1 : (want < n ? want : n));
    int g0 = 0, base = 0;
    for (;;) {
      const int gm = n - g0 < GM ? n - g0 : GM;
      const int cnt = gm * (gm + 1) / 2 + gm * (n - g0 - gm);
      if (k < base + cnt || g0 + gm >= n) break;
      base += cnt;
      g0 += gm;
    }
    const int gm = n - g0 < GM ? n - g0 : GM;
    const int r = k - base;
    const int t1 = gm * (gm + 1) / 2;
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
    return !(tile_m * BM >= p.M || tile_n * BN >= p.Ncol || tile_m * BM >= tile_n * BN + BN);
  }
  // GM query panels (~32 MB) sweep the gallery blocks together, XCD-contiguous
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int64_t panel = (int64_t)BM * row_bytes;
  const int64_t want = ((int64_t)X3P_GM_MB << 20) / (panel > 0 ? panel : 1);
  const int GM = (int)(want < 1 ? 1 : (want < tiles_m ? want : tiles_m));
  const int per = GM * tiles_n;
  const int grp = bid / per;
  const int first = grp * GM;
  const int gm = tiles_m - first < GM ? tiles_m - first : GM;
  const int r = bid - grp * per;
  tile_n = r / gm;
  tile_m = first + (r - tile_n * gm);
  return true;
}

// Distance epilogue of the h2 kernel: the accumulators are parked in LDS
// ([BM][BN / HB + 4] f32, HB column passes), then every thread finishes
// 4-column row pieces: dot = (acc * 2^-s_q) * 2^-s_g, the metric of
// dist_value, stored as whole row segments.  Self-distance tiles write the
// elements on or above the diagonal and mirror the strictly-upper ones
// (column walk of the parked tile, 16-byte stores into the mirrored rows).
template <int BM, int BN, int WM, int WN, int HB>
__device__ inline void h2_dist_epilogue(const GemmParams& p, f32x4 (&acc)[BM / WM / 16][BN / WN / 16],
                                        unsigned char* lds, int m0, int n0, int wm, int wn,
                                        int lane) {
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16, NT = 64 * WM * WN;
  constexpr int WCOLS = BN / WN;
  constexpr int BNH = BN / HB, LD = BNH + 4, C4 = BNH / 4, R4 = BM / 4;
  static_assert(BNH % WCOLS == 0, "a wave's columns fall in one pass");
  float* t = reinterpret_cast<float*>(lds);
  const int r16 = lane & 15, h = lane >> 4;
  const int mrem = p.M - m0, nrem = p.Ncol - n0;
  const int64_t ldo = p.ldo;
  const bool sym = p.sym != 0;
  const bool vec = (ldo & 3) == 0 && (reinterpret_cast<uintptr_t>(p.out) & 15) == 0 &&
                   (m0 & 3) == 0 && (n0 & 3) == 0;
  const int wc0 = wn * WCOLS;
#pragma unroll
  for (int hb = 0; hb < HB; ++hb) {
    const int c0h = hb * BNH;
    __syncthreads();  // the stages / the previous pass are no longer read
    if (wc0 >= c0h && wc0 < c0h + BNH) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * (BM / WM) + i * 16 + r16;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wc0 - c0h + j * 16 + 4 * h;
          *reinterpret_cast<f32x4*>(t + row * LD + col) = acc[i][j];
        }
      }
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < BM * C4; idx += NT) {
      const int row = idx / C4, col = 4 * (idx - row * C4);
      const int cl = c0h + col;  // column within the tile
      if (row >= mrem || cl >= nrem) continue;
      const int gr = m0 + row, gc = n0 + cl;
      const float qn = p.norm_a[gr];
      const float ra = p.rs_a[gr];
      const f32x4 a = *reinterpret_cast<const f32x4*>(t + row * LD + col);
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = cl + e < nrem;
        const float gn = ok ? p.norm_b[gc + e] : 0.f;
        const float rb = ok ? p.rs_b[gc + e] : 0.f;
        // two exact power-of-two scalings (row scale first: no intermediate
        // underflow for rows scaled far from 1)
        v[e] = dist_value(p, (a[e] * ra) * rb, qn, gn);
      }
      float* o = p.out + (int64_t)gr * ldo + gc;
      if (sym) {
        *reinterpret_cast<f32x4*>(t + row * LD + col) = v;  // for the mirror walk
        if (vec && cl + 3 < nrem && gr <= gc) {
          *reinterpret_cast<f32x4*>(o) = v;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (cl + e < nrem && gr <= gc + e) o[e] = v[e];
        }
      } else if (vec && cl + 3 < nrem) {
        *reinterpret_cast<f32x4*>(o) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (cl + e < nrem) o[e] = v[e];
      }
    }
    if (sym) {
      __syncthreads();
      for (int idx = threadIdx.x; idx < BNH * R4; idx += NT) {
        const int col = idx / R4, row = 4 * (idx - col * R4);
        const int cl = c0h + col;
        if (cl >= nrem || row >= mrem) continue;
        const int gc = n0 + cl, gr = m0 + row;
        if (gr >= gc) continue;  // nothing strictly above the diagonal here
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = t[(row + e) * LD + col];
        float* o = p.out + (int64_t)gc * ldo + gr;  // out[gc][gr .. gr + 3]
        if (vec && row + 3 < mrem && gr + 3 < gc) {
          *reinterpret_cast<f32x4*>(o) = v;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (row + e < mrem && gr + e < gc) o[e] = v[e];
        }
      }
    }
  }
}

#ifndef H2_ABL
#define H2_ABL 0  // probes: 1 = no DMA after the prologue, 2 = no MFMAs (timing ablations)
#endif
// A blocks multiplied after the chunk barrier by waves 0 .. NW/2 - 1 (O) and
// NW/2 .. NW - 1 (Y); -1: 2 / 4 on the three-stage tiles (Market 3368 x 15913:
// tile 6 1061 / 1067 -> 1049 / 1058 us, tiles 3 / 4 1114-1130 -> 1101-1105;
// the two-stage 256-row tiles would spill), 1 / 1 on the others
#ifndef H2_STAG_O
#define H2_STAG_O -1
#endif
#ifndef H2_STAG_Y
#define H2_STAG_Y -1
#endif
#ifndef H2_SPREAD
#define H2_SPREAD 1  // DMA pieces spread over the chunk's MFMA blocks (NS >= 3 tiles); 0: a burst after the barrier
#endif

template <int BM, int BN, int WM, int WN, int NS>
__global__ void __launch_bounds__(64 * WM * WN)
gemm_h2_kernel(GemmParams p, int tiles_m, int tiles_n) {
  constexpr int BK = 32;
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int ABLK = BM / 16, BBLK = BN / 16;  // 16-row blocks per plane and chunk
  constexpr int NPIECE = 2 * (ABLK + BBLK);      // KiB DMA pieces per chunk
  // pieces per wave; uneven tiles give the last waves dummy pieces (zeros
  // into a spare KiB after the stages) so every wave's wait counts are equal
  constexpr int PPW = (NPIECE + NW - 1) / NW;
  constexpr bool EVEN = NPIECE % NW == 0;
  constexpr int STAGE = NPIECE * 1024;
  static_assert(TM % 2 == 0 && TM >= 2 && TN >= 1, "wave tile");
  static_assert(NS >= 2 && NS <= 4 && NS * STAGE <= 160 * 1024, "LDS stages");
  static_assert(PPW * (NS - 1) <= 63, "vmcnt range");
  constexpr int HB = BM * (BN + 4) * 4 <= 160 * 1024 ? 1 : 2;
  constexpr int EPI_BYTES = BM * (BN / HB + 4) * 4;
  static_assert(EPI_BYTES <= 160 * 1024, "epilogue image");
  constexpr int PIPE_BYTES = NS * STAGE + (EVEN ? 0 : 1024);
  constexpr int LDS_BYTES = PIPE_BYTES > EPI_BYTES ? PIPE_BYTES : EPI_BYTES;
  static_assert(PIPE_BYTES <= 160 * 1024, "LDS stages");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[LDS_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave - wm * WN;
  int tile_m, tile_n;
  if (!dist_tile_coords<BM, BN>(p, tiles_m, tiles_n, (int64_t)p.Kloop * 4, tile_m, tile_n))
    return;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int nkc = p.Kloop / BK;

  // ---- DMA pieces.  Piece q of a chunk: A plane q / ABLK, block q % ABLK
  // (q < 2 ABLK), else B; its LDS image is stage + q KiB.  Lane l fills row
  // l >> 2 of the 16-row block, physical 16-byte slot l & 3 with logical slot
  // (l & 3) ^ sw64(row) (bank-conflict swizzle on the source address).
  const rsrc_t ra = make_rsrc(p.a3, p.a_bytes);
  const rsrc_t rb = make_rsrc(p.b3, p.b_bytes);
  const int ablocks = (int)(p.a_plane / (16 * (int64_t)p.Kloop));
  const int bblocks = (int)(p.b_plane / (16 * (int64_t)p.Kloop));
  const int lr = lane >> 2;
  const int loff = lr * 64 + (((lane & 3) ^ sw64(lr)) << 4);
  int src[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int q = wave * PPW + i;
    int blk = 0, nblk = 0;
    int64_t pbase = 0;
    if (q >= NPIECE) {
      // dummy piece (uneven tiles): reads zeros
    } else if (q < 2 * ABLK) {
      const int pl = q / ABLK;
      blk = m0 / 16 + (q - pl * ABLK);
      nblk = ablocks;
      pbase = pl * p.a_plane * 2;
    } else {
      const int qq = q - 2 * ABLK;
      const int pl = qq / BBLK;
      blk = n0 / 16 + (qq - pl * BBLK);
      nblk = bblocks;
      pbase = pl * p.b_plane * 2;
    }
    // out-of-range blocks: an offset >= 2^31 > num_records reads zeros
    src[i] = blk < nblk ? (int)(pbase + (int64_t)blk * nkc * 1024 + loff) : (int)0x80000000;
  }
  // piece i of this wave for chunk kc into its stage
  auto issue_piece = [&](int kc, int stage, int i) {
    const unsigned char* st = lds + stage * STAGE;
    const int q = wave * PPW + i;
    if (EVEN || q < NPIECE)
      glds16(q < 2 * ABLK ? ra : rb, st + q * 1024, src[i] + kc * 1024);
    else
      glds16(rb, lds + NS * STAGE, (int)0x80000000);
  };
  auto issue = [&](int kc, int stage) {
    if (H2_ABL == 1 && kc >= NS) return;
#pragma unroll
    for (int i = 0; i < PPW; ++i) issue_piece(kc, stage, i);
  };

  // ---- fragments: lane l reads row l & 15 of a block, logical 16-byte slot
  // l >> 4 (K elements 8 (l >> 4) .. + 7), at its swizzled position
  const int r16 = lane & 15;
  const int foff = r16 * 64 + (((lane >> 4) ^ sw64(r16)) << 4);
  auto readA = [&](const unsigned char* st, int i, f16x8 (&f)[2]) {
    const unsigned char* a = st + (wm * (BM / WM / 16) + i) * 1024 + foff;
    f[0] = *reinterpret_cast<const f16x8*>(a);
    f[1] = *reinterpret_cast<const f16x8*>(a + ABLK * 1024);
  };
  auto readB = [&](const unsigned char* st, f16x8 (&fb)[TN][2]) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const unsigned char* b = st + (2 * ABLK + wn * (BN / WN / 16) + j) * 1024 + foff;
      fb[j][0] = *reinterpret_cast<const f16x8*>(b);
      fb[j][1] = *reinterpret_cast<const f16x8*>(b + BBLK * 1024);
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // Chunk c lives in stage c % NS.  The prologue requests chunks 0 .. NS-1;
  // the barrier in chunk c's tail (every wave done reading stage c % NS, and
  // chunk c + 1 landed: the NS - 2 younger chunks may stay in flight) is
  // followed by the request of chunk c + NS into the stage just freed.
  // Requests past the last chunk stay inside the operand buffers (or read
  // zeros beyond them) and are never consumed: every wait count is uniform.
#pragma unroll
  for (int c = 0; c < NS; ++c) issue(c, c);
  wait_vmcnt<PPW * (NS - 1)>();  // chunk 0 landed
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  constexpr bool SPREAD = H2_SPREAD && NS >= 3 && H2_ABL == 0;
  constexpr int SO = H2_STAG_O >= 0 ? H2_STAG_O : (NS >= 3 ? 2 : 1);
  constexpr int SY = H2_STAG_Y >= 0 ? H2_STAG_Y : (NS >= 3 ? 4 : 1);
  constexpr int DO = SO < TM ? SO : TM - 1;
  constexpr int DY = SY < TM ? SY : TM - 1;
  if constexpr (DO == 1 && DY == 1) {
    f16x8 fb0[TN][2], fb1[TN][2], fa0[2], fa1[2];
    readB(lds, fb0);
    readA(lds, 0, fa0);
    // One chunk: block i's MFMAs beside block i + 1's A reads; before the last
    // block, the barrier that retires this stage's reads and the next chunk's
    // DMA, the request two chunks ahead into this stage, and the next chunk's B
    // fragments and first A block beside the last block's MFMAs.
    int scur = 0;  // stage of chunk kc
    // SPREAD (three or more stages): chunk kc - 1 + NS goes into the stage the
    // previous chunk's barrier freed, its pieces spread over this chunk's
    // first TM - 1 blocks (an MFMA block between two DMA pieces) instead of a
    // burst right after the barrier, where both waves of a SIMD stall on
    // their DMA issue at once; all pieces are out before the chunk's wait
    auto chunk = [&](int kc, f16x8 (&fbc)[TN][2], f16x8 (&fbn)[TN][2]) {
      const unsigned char* st = lds + scur * STAGE;
      const int sprev = scur == 0 ? NS - 1 : scur - 1;
#pragma unroll
      for (int i = 0; i < TM - 1; ++i) {
        if (SPREAD && kc >= 1) {
#pragma unroll
          for (int j = i * PPW / (TM - 1); j < (i + 1) * PPW / (TM - 1); ++j)
            issue_piece(kc - 1 + NS, sprev, j);
        }
        if (i & 1) {
          readA(st, i + 1, fa0);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = mfma_h2t(fa1[0], fa1[1], fbc[j][0], fbc[j][1], acc[i][j]);
        } else {
          readA(st, i + 1, fa1);
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = mfma_h2t(fa0[0], fa0[1], fbc[j][0], fbc[j][1], acc[i][j]);
        }
      }
      if (kc + 1 < nkc) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        wait_vmcnt<PPW * (NS - 2)>();  // chunk kc + 1 landed
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (!SPREAD) issue(kc + NS, scur);
        scur = scur + 1 == NS ? 0 : scur + 1;
        const unsigned char* sn = lds + scur * STAGE;
        readB(sn, fbn);
        readA(sn, 0, fa0);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[TM - 1][j] = mfma_h2t(fa1[0], fa1[1], fbc[j][0], fbc[j][1], acc[TM - 1][j]);
    };
    int kc = 0;
    for (; kc + 1 < nkc; kc += 2) {
      chunk(kc, fb0, fb1);
      chunk(kc + 1, fb1, fb0);
    }
    if (kc < nkc) chunk(kc, fb0, fb1);
  } else {
    // One chunk, D blocks deferred: blocks 0 .. TM-1-D multiply before the
    // chunk's barrier (each beside the A read of a later block), every A block
    // of the chunk is in registers by the barrier; after it (the barrier that
    // retires this stage's reads and the next chunk's DMA), the next chunk's B
    // fragments and first A block are read beside the last D blocks' MFMAs.
    // The two halves of the workgroup run different D (H2_STAG_O for waves
    // 0 .. NW/2-1, H2_STAG_Y for the rest): the two waves of a SIMD then carry
    // different amounts of MFMA work across the barrier, so the one that
    // reaches it first leaves the matrix pipe to its partner instead of both
    // idling there together (MI355X_MICROARCH "try a stagger").
    // SPREAD (three or more stages): chunk kc - 1 + NS goes into the stage the
    // previous chunk's barrier freed, its pieces spread over this chunk's
    // pre-barrier blocks (an MFMA block between two DMA pieces) instead of a
    // burst right after the barrier, where both waves of a SIMD stall on
    // their DMA issue at once; all pieces are out before the chunk's wait
    f16x8 fb0[TN][2], fb1[TN][2];
    f16x8 fa[TM + 1][2];  // the chunk's A blocks; [TM]: the next chunk's block 0
    readB(lds, fb0);
    readA(lds, 0, fa[0]);
    int scur = 0;  // stage of chunk kc
    auto chunk = [&](auto dtag, int kc, f16x8 (&fbc)[TN][2], f16x8 (&fbn)[TN][2]) {
      constexpr int D = decltype(dtag)::value;
      constexpr int PRE = TM - D;  // blocks multiplied before the barrier
      constexpr int SPB = PRE > 0 ? PRE : 1;  // blocks the DMA pieces spread over
      const unsigned char* st = lds + scur * STAGE;
      const int sprev = scur == 0 ? NS - 1 : scur - 1;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (SPREAD && kc >= 1 && i < SPB) {
#pragma unroll
          for (int j = i * PPW / SPB; j < (i + 1) * PPW / SPB; ++j)
            issue_piece(kc - 1 + NS, sprev, j);
        }
        if (i + 1 < TM) readA(st, i + 1, fa[i + 1]);
        if (i < PRE) {
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = mfma_h2t(fa[i][0], fa[i][1], fbc[j][0], fbc[j][1], acc[i][j]);
        }
      }
      if (kc + 1 < nkc) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        wait_vmcnt<PPW * (NS - 2)>();  // chunk kc + 1 landed
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (!SPREAD) issue(kc + NS, scur);
        scur = scur + 1 == NS ? 0 : scur + 1;
        const unsigned char* sn = lds + scur * STAGE;
        readB(sn, fbn);
        readA(sn, 0, fa[TM]);
      }
#pragma unroll
      for (int i = PRE; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mfma_h2t(fa[i][0], fa[i][1], fbc[j][0], fbc[j][1], acc[i][j]);
      fa[0][0] = fa[TM][0];
      fa[0][1] = fa[TM][1];
    };
    auto loop = [&](auto dtag) {
      int kc = 0;
      for (; kc + 1 < nkc; kc += 2) {
        chunk(dtag, kc, fb0, fb1);
        chunk(dtag, kc + 1, fb1, fb0);
      }
      if (kc < nkc) chunk(dtag, kc, fb0, fb1);
    };
    if (DO == DY || wave < NW / 2)
      loop(std::integral_constant<int, DO>{});
    else
      loop(std::integral_constant<int, DY>{});
  }
  wait_vmcnt<0>();

  h2_dist_epilogue<BM, BN, WM, WN, HB>(p, acc, lds, m0, n0, wm, wn, lane);
}

template <int BM, int BN, int WM, int WN, int NS>
static int launch_h2(const GemmParams& p, hipStream_t stream) {
  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.Ncol + BN - 1) / BN;
  constexpr int SB = sym_block<BM, BN>();
  const int nsb = (p.Ncol + SB - 1) / SB;
  const int64_t nblk = p.sym ? (int64_t)(SB / BM) * (SB / BN) * (nsb * (int64_t)(nsb + 1) / 2)
                             : (int64_t)tiles_m * tiles_n;
  if (nblk <= 0) return PPS_OK;
  if (nblk >= (1ll << 31)) {
    set_error("h2 distance GEMM: grid too large");
    return PPS_ERR_INVALID_ARG;
  }
  hipLaunchKernelGGL((gemm_h2_kernel<BM, BN, WM, WN, NS>), dim3((unsigned)nblk), dim3(64 * WM * WN),
                     0, stream, p, tiles_m, tiles_n);
  PPS_CHECK_LAUNCH("gemm_h2_kernel");
  return PPS_OK;
}

// tile ids (every tile gives the same bits; speed only): 0 = default (1);
//   1 = 256 x 256, 8 waves (2 x 4: 128 x 64 per wave), two LDS stages
//   2 = 256 x 224, 8 waves (4 x 2: 64 x 112), two stages -- Market's
//       3368 x 15913 in 14 x 72 tiles, 3.94 rounds of 256 CUs
//   3 = 128 x 256, 8 waves (2 x 4), three stages
//   4 = 256 x 128, 8 waves (4 x 2), three stages
//   5 = 192 x 256, 8 waves (2 x 4), two stages
//   6 = 192 x 192, 8 waves (2 x 4: 96 x 48), three stages
//   7 = 256 x 192, 8 waves (2 x 4: 128 x 48), two stages
int launch_gemm_h2(const GemmParams& p, hipStream_t stream, int tile) {
  switch (tile) {
    case 0:
    case 1: return launch_h2<256, 256, 2, 4, 2>(p, stream);
    case 2: return launch_h2<256, 224, 4, 2, 2>(p, stream);
    case 3: return launch_h2<128, 256, 2, 4, 3>(p, stream);
    case 4: return launch_h2<256, 128, 4, 2, 3>(p, stream);
    case 5: return launch_h2<192, 256, 2, 4, 2>(p, stream);
    case 6: return launch_h2<192, 192, 2, 4, 3>(p, stream);
    case 7: return launch_h2<256, 192, 2, 4, 2>(p, stream);
    default:
      set_error("unknown h2 distance tile " + std::to_string(tile));
      return PPS_ERR_INVALID_ARG;
  }
}

// ---- the split: one wave per row.  Pass 1 sums the squared norm in
// row_sqnorm_kernel's lane order and xor tree (so the norms equal the bf16x3
// path's bit for bit) and takes max|x|; pass 2 re-reads the row (L2-warm),
// scales it by 2^s and writes the two f16 planes chunk-tiled.  Padding rows
// (rows .. rows16) are written as zeros.
__global__ void split_h2_sqnorm_kernel(const float* __restrict__ x, int64_t rows, int D,
                                       int64_t ld, _Float16* __restrict__ out2,
                                       float* __restrict__ rscale, float* __restrict__ sqnorm) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t rows16 = (rows + 15) / 16 * 16;
  if (row >= rows16) return;
  const bool real = row < rows;
  const float* r = x + (real ? row : 0) * ld;
  const int64_t plane = rows16 * (int64_t)D;
  _Float16* o = out2 + (row >> 4) * 16 * (int64_t)D + (row & 15) * 32;
  float s = 0.f, mx = 0.f;
  constexpr int U = 4;  // row segments of 256 per trip, loads issued together
  for (int k0 = lane * 4; k0 < D; k0 += 256 * U) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + 256 * u;
      v[u] = real && k < D ? *reinterpret_cast<const f32x4*>(r + k) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (k0 + 256 * u >= D) break;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s = __builtin_fmaf(v[u][e], v[u][e], s);
        mx = fmaxf(mx, fabsf(v[u][e]));
      }
    }
  }
#pragma unroll
  for (int o2 = 32; o2 >= 1; o2 >>= 1) {
    s += __shfl_xor(s, o2);
    mx = fmaxf(mx, __shfl_xor(mx, o2));
  }
  // max|x| = m 2^E with m in [0.5, 1)  ->  s = 15 - E, max|x 2^s| in [2^14, 2^15)
  float rs;
  const float S = h2_scale_of(mx, &rs);
  for (int k0 = lane * 4; k0 < D; k0 += 256 * U) {
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + 256 * u;
      v[u] = real && k < D ? *reinterpret_cast<const f32x4*>(r + k) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + 256 * u;
      if (k >= D) break;
      f16x4 h0, h1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y = v[u][e] * S;  // exact (power of two)
        h0[e] = (_Float16)y;
        h1[e] = (_Float16)(y - (float)h0[e]);  // the remainder is exact in f32
      }
      const int64_t ko = (int64_t)(k >> 5) * 512 + (k & 31);
      *reinterpret_cast<f16x4*>(o + ko) = h0;
      *reinterpret_cast<f16x4*>(o + plane + ko) = h1;
    }
  }
  if (lane == 0 && real) {
    sqnorm[row] = s;
    rscale[row] = rs;
  }
}

int split_h2_sqnorm_tiled(const float* x, int64_t rows, int D, int64_t ld, uint16_t* out2t,
                          float* rscale, float* sqnorm, hipStream_t stream) {
  if (rows <= 0) return PPS_OK;
  const int64_t blocks = ((rows + 15) / 16 * 16 + 3) / 4;
  hipLaunchKernelGGL(split_h2_sqnorm_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, x,
                     rows, D, ld, reinterpret_cast<_Float16*>(out2t), rscale, sqnorm);
  PPS_CHECK_LAUNCH("split_h2_sqnorm_kernel");
  return PPS_OK;
}

}  // namespace pps

// ---- C ABI ----------------------------------------------------------------
using namespace pps;

int pps_h2_num_tiles(void) { return kH2NumTiles; }

int pps_split_f16x2_sqnorm_tiled(const float* x, int64_t rows, int D, int64_t ld,
                                 uint16_t* out2t, float* rscale, float* sqnorm, void* stream) {
  PPS_ENFORCE(x && out2t && rscale && sqnorm, "null pointer");
  PPS_ENFORCE(rows >= 0 && D > 0 && D % 32 == 0 && ld >= D && ld % 4 == 0,
              "bad shape (D % 32 == 0, ld % 4 == 0)");
  PPS_ENFORCE(aligned16(x), "x must be 16-byte aligned");
  PPS_ENFORCE(((uintptr_t)out2t & 7) == 0, "out2t must be 8-byte aligned");
  return split_h2_sqnorm_tiled(x, rows, D, ld, out2t, rscale, sqnorm, as_stream(stream));
}

static GemmParams h2_params(const uint16_t* a2t, int64_t M, const float* asq, const float* ars,
                            const uint16_t* b2t, int64_t N, const float* bsq, const float* brs,
                            int D, int metric, float* out, int64_t ldo, int sym) {
  const int64_t Mp = (M + 15) / 16 * 16, Np = (N + 15) / 16 * 16;
  GemmParams p{};
  p.splitk = 1;
  p.tiled = 3;
  p.a3 = a2t; p.a_plane = Mp * D; p.a_bytes = (uint32_t)(2 * Mp * D * 2);
  p.M = (int)M;
  p.b3 = b2t; p.b_plane = Np * D; p.b_bytes = (uint32_t)(2 * Np * D * 2);
  p.Ncol = (int)N;
  p.Kloop = D;
  p.norm_a = asq; p.norm_b = bsq;
  p.rs_a = ars; p.rs_b = brs;
  p.out = out; p.ldo = ldo; p.metric = metric; p.sym = sym;
  return p;
}

int pps_distmat_h2_tiled(const uint16_t* q2t, int64_t Q, const float* qsq, const float* qrs,
                         const uint16_t* g2t, const float* gsq, const float* grs, int64_t G,
                         int D, int metric, float* out, int64_t ldo, int tile, void* stream) {
  PPS_ENFORCE(q2t && qsq && qrs && g2t && gsq && grs && out, "null pointer");
  PPS_ENFORCE(Q >= 0 && G >= 0 && D > 0 && D % 32 == 0, "bad shape (D % 32 == 0)");
  PPS_ENFORCE(ldo >= G, "ldo < G");
  PPS_ENFORCE(aligned16(q2t) && aligned16(g2t), "planes must be 16-byte aligned");
  PPS_ENFORCE(metric >= 0 && metric <= 2, "unknown metric");
  PPS_ENFORCE(tile >= 0 && tile < kH2NumTiles, "h2 tile must be 0.." + std::to_string(kH2NumTiles - 1));
  const int64_t Qp = (Q + 15) / 16 * 16, Gp = (G + 15) / 16 * 16;
  PPS_ENFORCE(2 * Qp * D * 2 < kMaxBufBytes && 2 * Gp * D * 2 < kMaxBufBytes,
              "planes over 2 GiB");
  if (Q == 0 || G == 0) return PPS_OK;
  const GemmParams p = h2_params(q2t, Q, qsq, qrs, g2t, G, gsq, grs, D, metric, out, ldo, 0);
  return launch_gemm_h2(p, as_stream(stream), tile);
}

int pps_distmat_h2_self_tiled(const uint16_t* x2t, int64_t N, const float* xsq, const float* xrs,
                              int D, int metric, float* out, int64_t ldo, int tile,
                              void* stream) {
  PPS_ENFORCE(x2t && xsq && xrs && out, "null pointer");
  PPS_ENFORCE(N >= 0 && D > 0 && D % 32 == 0, "D must be a positive multiple of 32");
  PPS_ENFORCE(ldo >= N, "ldo < N");
  PPS_ENFORCE(aligned16(x2t), "x2t must be 16-byte aligned");
  PPS_ENFORCE(metric >= 0 && metric <= 2, "unknown metric");
  PPS_ENFORCE(tile >= 0 && tile < kH2NumTiles, "h2 tile must be 0.." + std::to_string(kH2NumTiles - 1));
  const int64_t Np = (N + 15) / 16 * 16;
  PPS_ENFORCE(2 * Np * D * 2 < kMaxBufBytes, "planes over 2 GiB");
  PPS_ENFORCE(N * ldo < (1ll << 31), "output larger than 2^31 elements");
  if (N == 0) return PPS_OK;
  const GemmParams p = h2_params(x2t, N, xsq, xrs, x2t, N, xsq, xrs, D, metric, out, ldo, 1);
  return launch_gemm_h2(p, as_stream(stream), tile);
}
