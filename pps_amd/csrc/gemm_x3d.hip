// Distance GEMM on 256 x 256 tiles (GEMM tile id 60): the query x gallery
// dot products of compute_dist (reid_dataset_evaluator.py:244-272) with both
// operands as bf16x3 planes (queries split once, the gallery index split
// once), 32x32x16 MFMA blocks, 16-wide K chunks.
//
// What bounds the pipelined tiles here is not the MFMA pipe but how many
// bytes a CU takes in per second (PMC + timing: ~33 GB/s per CU on the
// 192x128 tile, 61 KB per 32-wide chunk; rocprof 2.0 ms for the Market
// matrix at MFMA busy 0.62).  Bytes per output element fall with the tile's
// perimeter / area: 256 x 256 needs 0.6x the bytes of 192 x 128 per
// product.  Its stages are 16 K wide to fit: (256 + 256) rows x 32 B x 3
// planes = 48 KB, three stages (two chunks in flight) = 144 KB.  8 waves
// as 2 x 4, 128 x 64 outputs each (8 accumulator blocks, 128 registers); a
// chunk's fragments (72 registers) are read once per chunk and the SIMD's
// second wave covers their latency.
//
// Arithmetic: per 16-wide K group the six terms of mfma_x3t in order, groups
// in K order -- the sequence of the 32x32x16 tiles (ids below 38), so tile
// 60 gives their bits (tests/test_gpu_retrieval.py).
#include "gemm_x3p_common.hpp"

namespace pps {

constexpr int kDBM = 256, kDBN = 256, kDWM = 2, kDWN = 4, kDBK = 16;

template <int NS>
__global__ void __launch_bounds__(64 * kDWM * kDWN)
gemm_x3d_kernel(GemmParams p, int tiles_m, int tiles_n) {
  constexpr int BM = kDBM, BN = kDBN, WM = kDWM, WN = kDWN, BK = kDBK, S = 32;
  constexpr int NW = WM * WN;
  constexpr int TM = BM / WM / S;  // 4
  constexpr int TN = BN / WN / S;  // 2
  constexpr int ROWB = BK * 2;     // bytes of one row's chunk per plane (32)
  constexpr int A_PLANE = BM * ROWB, B_PLANE = BN * ROWB;
  constexpr int STAGE = 3 * (A_PLANE + B_PLANE);
  constexpr int NPA = BM / 32;     // 1 KiB pieces (32 rows) per plane and chunk
  constexpr int NPB = BN / 32;
  static_assert(NPA == NW && NPB == NW, "one A and one B piece per wave and plane");
  constexpr int NLOAD = 6;         // DMA instructions per wave and chunk
  static_assert(NS >= 2 && NS * STAGE <= 160 * 1024 && NLOAD * (NS - 2) <= 63, "stages");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NS * STAGE];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN;
  const int wn = wave - wm * WN;
  const int r32 = lane & 31;
  const int h = lane >> 5;

  // grouped tile order (as gemm_x3p_kernel's EPI_DIST): GM query panels
  // (~32 MB of planes) sweep the gallery blocks together
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  int tile_m, tile_n;
  {
    const int64_t panel = (int64_t)BM * p.Kloop * 6;
    const int64_t want = ((int64_t)X3P_GM_MB << 20) / (panel > 0 ? panel : 1);
    const int GM = (int)(want < 1 ? 1 : (want < tiles_m ? want : tiles_m));
    const int per = GM * tiles_n;
    const int grp = bid / per;
    const int first = grp * GM;
    const int gm = tiles_m - first < GM ? tiles_m - first : GM;
    const int r = bid - grp * per;
    tile_n = r / gm;
    tile_m = first + (r - tile_n * gm);
  }
  const int m0 = tile_m * BM;
  const int n0 = tile_n * BN;

  // DMA pieces: wave w moves rows 32 w .. 32 w + 31 of A and of B, every
  // plane; lane l takes row 32 w + (l >> 1) and fills physical 16-byte slot
  // l & 1 with logical slot (l & 1) ^ ((row >> 3) & 1) (conflict-free
  // ds_read_b128 for the 32-row fragment reads)
  const rsrc_t ra0 = make_rsrc(p.a3, p.a_bytes);
  const rsrc_t ra1 = make_rsrc(p.a3 + p.a_plane, p.a_bytes);
  const rsrc_t ra2 = make_rsrc(p.a3 + 2 * p.a_plane, p.a_bytes);
  const rsrc_t rb0 = make_rsrc(p.b3, p.b_bytes);
  const rsrc_t rb1 = make_rsrc(p.b3 + p.b_plane, p.b_bytes);
  const rsrc_t rb2 = make_rsrc(p.b3 + 2 * p.b_plane, p.b_bytes);
  const int prow = 32 * wave + (lane >> 1);
  const int lslot = (lane & 1) ^ ((prow >> 3) & 1);
  const int arow = m0 + prow, brow = n0 + prow;
  const int aoff = arow < p.M ? (arow * p.lda + 8 * lslot) * 2 : kOOB;
  const int boff = brow < p.Ncol ? (brow * p.ldb + 8 * lslot) * 2 : kOOB;
  const int nchunks = (p.Kloop + BK - 1) / BK;
  int kiss = 0, siss = 0;
  auto issue = [&]() {
    unsigned char* st = lds + siss * STAGE;
    const bool ok = kiss < nchunks;
    const int ko = kiss * BK * 2;
    const int ao = ok && aoff != kOOB ? aoff + ko : kOOB;
    const int bo = ok && boff != kOOB ? boff + ko : kOOB;
    unsigned char* da = st + wave * 1024;
    unsigned char* db = st + 3 * A_PLANE + wave * 1024;
    glds16(ra0, da, ao);
    glds16(ra1, da + A_PLANE, ao);
    glds16(ra2, da + 2 * A_PLANE, ao);
    glds16(rb0, db, bo);
    glds16(rb1, db + B_PLANE, bo);
    glds16(rb2, db + 2 * B_PLANE, bo);
    ++kiss;
    siss = siss + 1 == NS ? 0 : siss + 1;
  };
  auto chunk_barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wait_vmcnt<NLOAD * (NS - 2)>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // fragment rows of this lane: r32 mod 32, so the swizzle is a lane constant
  const int fsl = (h ^ ((r32 >> 3) & 1)) << 4;
#pragma unroll
  for (int st = 0; st < NS - 1; ++st) issue();
  int scur = 0;
  for (int kc = 0; kc < nchunks; ++kc) {
    chunk_barrier();  // chunk kc landed; every wave is done with chunk kc - 1
    issue();          // chunk kc + NS - 1 into chunk kc - 1's stage
    const unsigned char* st = lds + scur * STAGE;
    scur = scur + 1 == NS ? 0 : scur + 1;
    bf16x8 fa[TM][3], fb[TN][3];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const unsigned char* ap = st + (wm * (BM / WM) + i * 32 + r32) * ROWB + fsl;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) fa[i][pl] = *reinterpret_cast<const bf16x8*>(ap + pl * A_PLANE);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const unsigned char* bp = st + 3 * A_PLANE + (wn * (BN / WN) + j * 32 + r32) * ROWB + fsl;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) fb[j][pl] = *reinterpret_cast<const bf16x8*>(bp + pl * B_PLANE);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma_x3t(fa[i], fb[j], acc[i][j]);
  }
  wait_vmcnt<0>();  // no DMA may land in LDS after the workgroup retires
  dist_epilogue_t<BM, BN, WM, WN, S>(p, acc, m0, n0, wm, wn, r32, h);
}

// Query planes x gallery planes, not the symmetric self-distance; rows
// 16-byte aligned (ld % 8) and K a multiple of 16.
bool x3d_eligible(const GemmParams& p, int epi, int batch) {
  return epi == EPI_DIST && batch == 1 && p.splitk == 1 && !p.sym && p.a3 && p.b3 && !p.a2 &&
         p.KH == 1 && p.KW == 1 && p.Kloop % kDBK == 0 && p.kb_valid >= p.Kloop &&
         p.lda % 8 == 0 && p.ldb % 8 == 0 && p.Cin == p.Kloop;
}

int launch_gemm_x3d(const GemmParams& p, hipStream_t stream) {
  const int tiles_m = (p.M + kDBM - 1) / kDBM;
  const int tiles_n = (p.Ncol + kDBN - 1) / kDBN;
  hipLaunchKernelGGL((gemm_x3d_kernel<3>), dim3(tiles_m * tiles_n), dim3(64 * kDWM * kDWN), 0,
                     stream, p, tiles_m, tiles_n);
  PPS_CHECK_LAUNCH("gemm_x3d_kernel");
  return PPS_OK;
}

}  // namespace pps
