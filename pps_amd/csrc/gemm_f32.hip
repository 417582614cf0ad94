// FP32 MFMA GEMM core for gfx950 (CDNA4): implicit-GEMM convolution over NHWC
// activations and the query x gallery distance matrix share this kernel.
//
//   C[m][n] = sum_k A[m][k] * B[n][k]       (both operands K-contiguous)
//
// * v_mfma_f32_32x32x2_f32 (exact f32 in, f32 accumulate): the only way to
//   keep the reference's fp32 numerics (SURVEY §7 "Precision vs parity").
// * Block tile BM x BN x BK (BK = 16 or 32), 64*WM*WN threads, each wave owns
//   (BM/WM) x (BN/WN) as TMxTN 32x32 accumulators (16 f32 regs each).
// * K is permuted inside each 16-group: at MFMA step s (0..7) lane half h
//   contributes k = 8h + s, so each lane reads its 8 k-values of a row with
//   two ds_read_b128 from a K-contiguous LDS row.  Row stride 20 floats
//   (80 B) makes those reads bank-conflict free for all four b128 lane groups.
// * Register-staged global->LDS pipeline, 2 LDS buffers, ONE barrier per
//   K-chunk: the loads for chunk t+1 are issued before the MFMAs on chunk t.
// * XCD-aware bijective block remap: consecutive tiles along N (sharing the
//   same A panel) land on the same XCD / L2.
// * Epilogues: EPI_CONV = per-column scale/shift (folded test-mode BN,
//   conv bias) + residual + ReLU; EPI_DIST = |q|^2 + |g|^2 - 2 q.g with the
//   squared norms accumulated from the same LDS fragments, clamp, sqrt.
#include "gemm_common.hpp"

namespace pps {

// K chunk per LDS stage is a template parameter BK (16 or 32); LDS rows hold
// BK floats + 4 pad: 80 B or 144 B, both conflict-free for the fragment reads.
template <int BM, int BN, int WM, int WN, int EPI, int BK>
__global__ void __launch_bounds__(64 * WM * WN)
gemm_f32_kernel(GemmParams p, int tiles_m, int tiles_n) {
  constexpr int T = 64 * WM * WN;
  constexpr int LSTR = BK + 4;         // LDS row stride in floats
  constexpr int V4 = BK / 4;           // float4 per LDS row
  constexpr int AL = BM * BK / 4 / T;  // f32x4 loads per thread (A)
  constexpr int BL = BN * BK / 4 / T;  // f32x4 loads per thread (B)
  constexpr int ROWS_PER_PASS = T / V4;
  static_assert(BK == 16 || BK == 32, "BK must be 16 or 32");
  constexpr int TM = BM / WM / 32;
  constexpr int TN = BN / WN / 32;
  static_assert(AL >= 1 && BL >= 1, "tile too small for thread count");
  static_assert(TM >= 1 && TN >= 1, "wave tile too small");

  // one LDS array (2 operand buffers + the 64-entry tap-offset table)
  __shared__ __attribute__((aligned(16))) float lds[2 * (BM + BN) * LSTR + 64];
  int* s_tapoff = reinterpret_cast<int*>(lds + 2 * (BM + BN) * LSTR);
  float* As = lds;                       // [2][BM][LSTR]
  float* Bs = lds + 2 * BM * LSTR;       // [2][BN][LSTR]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN;
  const int wn = wave % WN;
  const int r32 = lane & 31;
  const int h = lane >> 5;

  // ---- XCD-aware bijective remap of the flat block id -------------------
  const int bid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tile_m = bid / tiles_n;
  const int tile_n = bid - tile_m * tiles_n;
  const int m0 = tile_m * BM;
  const int n0 = tile_n * BN;
  // blockIdx.y enumerates (batch, K-slice) pairs; K-slice s covers
  // [s*Kloop, (s+1)*Kloop) of a K = splitk*Kloop reduction (raw partials)
  const int batch = blockIdx.y / p.splitk;
  const int kslice = blockIdx.y - batch * p.splitk;

  // ---- operand descriptors: buffer loads with 32-bit offsets ---------------
  // Out-of-range offsets (>= num_records) read as zero in hardware, so padding
  // taps, ragged rows/cols and K tails need no exec-mask branches.
  const int64_t kofs0 = (int64_t)kslice * p.Kloop;
  const rsrc_t rb_src = make_rsrc(p.b + batch * p.b_bstride + kofs0, p.b_bytes);
  const int c4 = tid % V4;   // float4 slot within the chunk row
  const int trow = tid / V4;
  constexpr bool DUAL = (EPI & EPI_F_DUAL) != 0;
  AGather<AL, ROWS_PER_PASS, BK, DUAL> ag;
  ag.init(p, batch, kofs0, m0, trow, c4, s_tapoff, tid, T);
  int bbase[BL];
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int col = n0 + trow + i * ROWS_PER_PASS;
    bbase[i] = col < p.Ncol ? (col * p.ldb + c4 * 4) * 4 : kOOB;
  }

  f32x4 ra[AL], rb[BL];
  auto load_chunk = [&](int kc) {
    ag.load(p, kc, c4, s_tapoff, ra);
    const int kb = kc * BK + c4 * 4;
    const bool kok = kb < p.kb_valid;
#pragma unroll
    for (int i = 0; i < BL; ++i) rb[i] = bload(rb_src, kok ? bbase[i] + kc * BK * 4 : kOOB);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float na[TM], nb[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) na[i] = 0.f;
#pragma unroll
  for (int j = 0; j < TN; ++j) nb[j] = 0.f;

  const int nchunks = (p.Kloop + BK - 1) / BK;  // zero-filled tail half-chunk
  load_chunk(0);
  int buf = 0;
  for (int kc = 0; kc < nchunks; ++kc) {
    float* as = As + buf * BM * LSTR;
    float* bs = Bs + buf * BN * LSTR;
#pragma unroll
    for (int i = 0; i < AL; ++i)
      *reinterpret_cast<f32x4*>(as + (trow + i * ROWS_PER_PASS) * LSTR + c4 * 4) = ra[i];
#pragma unroll
    for (int i = 0; i < BL; ++i)
      *reinterpret_cast<f32x4*>(bs + (trow + i * ROWS_PER_PASS) * LSTR + c4 * 4) = rb[i];
    __syncthreads();
    if (kc + 1 < nchunks) load_chunk(kc + 1);

    // K order inside every 16-wide group g: MFMA step s, lane half h uses
    // k = 16g + 8h + s.  BK=32 runs two groups per barrier with exactly the
    // accumulation order of BK=16, so every tile / BK variant is bit-identical.
#pragma unroll
    for (int g = 0; g < BK / 16; ++g) {
      f32x4 fa[TM][2], fb[TN][2];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* src = as + (wm * (BM / WM) + i * 32 + r32) * LSTR + g * 16 + h * 8;
        fa[i][0] = *reinterpret_cast<const f32x4*>(src);
        fa[i][1] = *reinterpret_cast<const f32x4*>(src + 4);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* src = bs + (wn * (BN / WN) + j * 32 + r32) * LSTR + g * 16 + h * 8;
        fb[j][0] = *reinterpret_cast<const f32x4*>(src);
        fb[j][1] = *reinterpret_cast<const f32x4*>(src + 4);
      }
      if (EPI & EPI_DIST) {
        // explicit fma chain: identical rounding for every tile configuration
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int e = 0; e < 4; ++e) na[i] = __builtin_fmaf(fa[i][u][e], fa[i][u][e], na[i]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int e = 0; e < 4; ++e) nb[j] = __builtin_fmaf(fb[j][u][e], fb[j][u][e], nb[j]);
      }
#pragma unroll
      for (int s = 0; s < 8; ++s) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const float av = (s < 4) ? fa[i][0][s] : fa[i][1][s - 4];
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const float bv = (s < 4) ? fb[j][0][s] : fb[j][1][s - 4];
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i][j], 0, 0, 0);
          }
        }
      }
    }
    buf ^= 1;
  }

  // ---- epilogue ------------------------------------------------------------
  if (!(EPI & EPI_DIST)) {
    conv_epilogue<EPI, BM, BN, WM, WN>(p, acc, batch, kslice, m0, n0, wm, wn, r32, h);
  } else {
    float* __restrict__ out = p.out + batch * p.out_bstride + (int64_t)m0 * p.ldo + n0;
    const int ldo = (int)p.ldo;
    const int mrem = p.M - m0;
    const int nrem = p.Ncol - n0;
#pragma unroll
    for (int i = 0; i < TM; ++i) na[i] += __shfl_xor(na[i], 32);
#pragma unroll
    for (int j = 0; j < TN; ++j) nb[j] += __shfl_xor(nb[j], 32);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float qn[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) qn[r] = __shfl(na[i], (r & 3) + 8 * (r >> 2) + 4 * h);
      const int rb = wm * (BM / WM) + i * 32 + 4 * h;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int c = wn * (BN / WN) + j * 32 + r32;
        if (c >= nrem) continue;
        const float gn = nb[j];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rr = rb + (r & 3) + 8 * (r >> 2);
          if (rr < mrem) {
            const float dot = acc[i][j][r];
            float v;
            if (p.metric == PPS_METRIC_COSINE) {
              const float den = fmaxf(sqrtf(qn[r]), 1e-12f) * fmaxf(sqrtf(gn), 1e-12f);
              v = 1.f - dot / den;
            } else {
              // (-2 a.b + |a|^2) + |b|^2 (reference order, fused), clamp at 0
              v = __builtin_fmaf(-2.f, dot, qn[r]) + gn;
              v = fmaxf(v, 0.f);
              if (p.metric == PPS_METRIC_EUCLIDEAN) v = sqrtf(v);
            }
            if (p.zero_diag && m0 + rr == n0 + c) v = 0.f;
            out[rr * ldo + c] = v;
          }
        }
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int EPI, int BK>
static void launch_one(const GemmParams& p, int batch, hipStream_t stream) {
  const int tiles_m = (p.M + BM - 1) / BM;
  const int tiles_n = (p.Ncol + BN - 1) / BN;
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, EPI, BK>),
                     dim3(tiles_m * tiles_n, batch * p.splitk),
                     dim3(64 * WM * WN), 0, stream, p, tiles_m, tiles_n);
}

template <int BM, int BN, int WM, int WN, int BK>
static int launch_tile(const GemmParams& p, int epi, int batch, hipStream_t stream) {
  switch (epi) {
    case EPI_DIST: launch_one<BM, BN, WM, WN, EPI_DIST, BK>(p, batch, stream); break;
    case EPI_CONV: launch_one<BM, BN, WM, WN, EPI_CONV, BK>(p, batch, stream); break;
    case EPI_CONV | EPI_F_RELU:
      launch_one<BM, BN, WM, WN, EPI_CONV | EPI_F_RELU, BK>(p, batch, stream); break;
    case EPI_CONV | EPI_F_RES:
      launch_one<BM, BN, WM, WN, EPI_CONV | EPI_F_RES, BK>(p, batch, stream); break;
    case EPI_CONV | EPI_F_RES | EPI_F_RELU:
      launch_one<BM, BN, WM, WN, EPI_CONV | EPI_F_RES | EPI_F_RELU, BK>(p, batch, stream); break;
    case EPI_CONV | EPI_F_RAW:
      launch_one<BM, BN, WM, WN, EPI_CONV | EPI_F_RAW, BK>(p, batch, stream); break;
    case EPI_CONV | EPI_F_RELU | EPI_F_DUAL:
      launch_one<BM, BN, WM, WN, EPI_CONV | EPI_F_RELU | EPI_F_DUAL, BK>(p, batch, stream); break;
    default:
      set_error("unknown epilogue");
      return PPS_ERR_INVALID_ARG;
  }
  PPS_CHECK_LAUNCH("gemm_f32_kernel");
  return PPS_OK;
}

static int ntiles(const GemmParams& p, int bm, int bn, int batch) {
  return ((p.M + bm - 1) / bm) * ((p.Ncol + bn - 1) / bn) * batch;
}

// Heuristic tile choice (tile == 0): enough workgroups to fill 256 CUs at
// >= 2 per CU, else fall back to narrower tiles.  PPSModel.autotune()
// measures every candidate per layer and passes the winner explicitly.
int pick_tile(const GemmParams& p, int batch) {
  if (p.Ncol <= 64) return GEMM_TILE_128x64;
  if (p.M <= 64) return GEMM_TILE_64x128;
  if (ntiles(p, 128, 128, batch) >= 512) return GEMM_TILE_128x128;
  if (ntiles(p, 128, 64, batch) >= 512) return GEMM_TILE_128x64;
  return GEMM_TILE_64x64;
}

int launch_gemm(const GemmParams& p, int epi, int batch, hipStream_t stream) {
  if (p.M <= 0 || p.Ncol <= 0 || batch <= 0) return PPS_OK;
  if (p.splitk < 1) {
    set_error("splitk must be >= 1");
    return PPS_ERR_INVALID_ARG;
  }
  if (!(epi & EPI_DIST) && !(epi & EPI_F_RAW)) {
    if (p.residual) epi |= EPI_F_RES;
    if (p.relu) epi |= EPI_F_RELU;
    if (p.a2) epi |= EPI_F_DUAL;
  }
  int tile = p.tile ? p.tile : pick_tile(p, batch);
  if (tile >= GEMM_TILE_P_FIRST) tile = GEMM_TILE_128x128;  // pipelined ids: bf16x3 only
  // ids 11..20 select a bf16x3 staging variant (gemm_x3.hip); the f32 kernel
  // has one variant per shape
  if (tile >= GEMM_TILE_192_FIRST && tile < GEMM_NUM_TILES) {
    const int v = tile - GEMM_TILE_192_FIRST;  // 192-row shapes -> nearest f32 shape
    tile = (v & 1) ? ((v & 2) ? GEMM_TILE_128x64_K32 : GEMM_TILE_128x64)
                   : ((v & 2) ? GEMM_TILE_128x128_K32 : GEMM_TILE_128x128);
  }
  if (tile > GEMM_TILE_256x128_K32 && tile < GEMM_TILE_192_FIRST) tile -= GEMM_TILE_256x128_K32;
  // BK=32 needs the dual operand switch on a 32-chunk boundary and, for
  // narrow inputs (Cin < 32), a power-of-two channel count
  if (tile > GEMM_TILE_256x128) {
    const bool narrow_ok = p.Cin >= 32 || (p.Cin & (p.Cin - 1)) == 0;
    const bool dual_ok = !p.a2 || p.Kloop1 % 32 == 0;
    if (!narrow_ok || !dual_ok) tile -= 5;
  }
  switch (tile) {
    case GEMM_TILE_128x128: return launch_tile<128, 128, 2, 2, 16>(p, epi, batch, stream);
    case GEMM_TILE_128x64: return launch_tile<128, 64, 4, 1, 16>(p, epi, batch, stream);
    case GEMM_TILE_64x128: return launch_tile<64, 128, 1, 4, 16>(p, epi, batch, stream);
    case GEMM_TILE_64x64: return launch_tile<64, 64, 2, 2, 16>(p, epi, batch, stream);
    case GEMM_TILE_256x128: return launch_tile<256, 128, 4, 2, 16>(p, epi, batch, stream);
    case GEMM_TILE_128x128_K32: return launch_tile<128, 128, 2, 2, 32>(p, epi, batch, stream);
    case GEMM_TILE_128x64_K32: return launch_tile<128, 64, 4, 1, 32>(p, epi, batch, stream);
    case GEMM_TILE_64x128_K32: return launch_tile<64, 128, 1, 4, 32>(p, epi, batch, stream);
    case GEMM_TILE_64x64_K32: return launch_tile<64, 64, 2, 2, 32>(p, epi, batch, stream);
    case GEMM_TILE_256x128_K32: return launch_tile<256, 128, 4, 2, 32>(p, epi, batch, stream);
    default:
      set_error("unknown GEMM tile id " + std::to_string(tile));
      return PPS_ERR_INVALID_ARG;
  }
}

}  // namespace pps
