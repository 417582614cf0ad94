// Internal helpers shared by the libpps_hip.so translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/pps_abi.h"

namespace pps {

// Thread-local ENFORCE-style error message (pps_last_error()).
void set_error(const std::string& msg);

#define PPS_ENFORCE(cond, msg)                                              \
  do {                                                                      \
    if (!(cond)) {                                                          \
      ::pps::set_error(std::string("[enforce fail at ") + __func__ + "] " + \
                       #cond + ". " + (msg));                               \
      return PPS_ERR_INVALID_ARG;                                           \
    }                                                                       \
  } while (0)

// PPS_DEBUG_SYNC=1 (debug only; breaks hipGraph capture): synchronize after
// each checked launch so an asynchronous fault is reported by the kernel
// that caused it
bool debug_sync();
#define PPS_CHECK_LAUNCH_S(name, stream)                                     \
  do {                                                                       \
    PPS_CHECK_LAUNCH(name);                                                  \
    if (::pps::debug_sync()) {                                               \
      hipError_t s_ = hipStreamSynchronize(stream);                          \
      if (s_ != hipSuccess) {                                                \
        ::pps::set_error(std::string(name) + " (sync): " + hipGetErrorString(s_)); \
        return PPS_ERR_LAUNCH;                                               \
      }                                                                      \
    }                                                                        \
  } while (0)
#define PPS_CHECK_LAUNCH(name)                                               \
  do {                                                                       \
    hipError_t e_ = hipGetLastError();                                       \
    if (e_ != hipSuccess) {                                                  \
      ::pps::set_error(std::string(name) + ": " + hipGetErrorString(e_));    \
      return PPS_ERR_LAUNCH;                                                 \
    }                                                                        \
  } while (0)

inline bool aligned16(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---- GEMM core (gemm_f32.hip) ----------------------------------------------
constexpr int64_t kMaxBufBytes = (int64_t)1 << 31;  // buffer-resource addressing limit
enum Epi {
  EPI_CONV = 0, EPI_DIST = 1, EPI_F_RELU = 2, EPI_F_RES = 4, EPI_F_DUAL = 8, EPI_F_RAW = 16,
  EPI_F_PLANES = 32,  // gemm_x3p.hip: result written as three bf16 planes (out3)
  EPI_F_PPS = 64,     // gemm_x3p.hip: + strip pooling and part power set of each image
  EPI_F_FIX = 128,    // gemm_x3p.hip conv split-K: the last K slice of a tile to finish
                      // sums the parked partials and runs the epilogue (no second pass)
  EPI_F_H2OUT = 512,  // gemm_x3p.hip conv: result written as f16x2 planes (out3) on the
                      // scale of a bound (h2o_*), the bound into amax_out
  EPI_F_H2 = 256      // gemm_x3p.hip / gemm_x3c.hip: f16x2 arithmetic (f32 activations
                      // scaled by 2^s from their tensor's max and split into two f16
                      // terms, weights as two f16 planes, three MFMA terms)
};
enum GemmTile {
  GEMM_TILE_AUTO = 0,
  GEMM_TILE_128x128 = 1,
  GEMM_TILE_128x64 = 2,
  GEMM_TILE_64x128 = 3,
  GEMM_TILE_64x64 = 4,
  GEMM_TILE_256x128 = 5,
  GEMM_TILE_128x128_K32 = 6,  // same shapes with a 32-wide K chunk per barrier
  GEMM_TILE_128x64_K32 = 7,
  GEMM_TILE_64x128_K32 = 8,
  GEMM_TILE_64x64_K32 = 9,
  GEMM_TILE_256x128_K32 = 10,
  // 11..20: ids 1..10 with the bf16x3 kernel's A operand kept f32 in LDS
  // 21..28 (bf16x3 kernel): 192x128 K16, 192x64 K16, 192x128 K32, 192x64 K32,
  // then the same four with A kept f32 in LDS
  GEMM_TILE_192_FIRST = 21,
  // 29..35 (bf16x3 only): LDS-DMA pipelined kernel (gemm_x3p.hip), K chunk 32:
  // 128x128, 192x128, 128x64, 192x64 (4 waves, 3 stages), 256x128, 128x256,
  // 192x256 (8 waves, 2 stages)
  GEMM_TILE_P_FIRST = 29,
  // 36, 37: 128x128 and 192x128 with 8 waves
  // 38..46 (bf16x3 only): ids 29..37 on 16x16x32 MFMA blocks (own rounding)
  GEMM_TILE_P16_FIRST = 38,
  // 47 (bf16x3 only, 16x16x32 rounding): 192x128 with 8 waves as 4 x 2 (48 x 64
  // per wave) -- 256 tiles for the res5 layers' M = 12,288 x N = 512
  GEMM_TILE_P16_192x128W42 = 47,
  // 48, 49 (16x16x32): 192x64 (4 x 1 waves) and 96x128 (2 x 2 waves), 48 x 64
  // per wave -- 256 tiles for M = 12,288 x N = 256 (res4 2a / 2b)
  GEMM_TILE_P16_192x64W41 = 48,
  GEMM_TILE_P16_96x128W22 = 49,
  // 50 (16x16x32): 96x128 with 8 waves as 2 x 4 (48 x 32 per wave)
  GEMM_TILE_P16_96x128W24 = 50,
  // 51, 52 (16x16x32): 128x128 and 192x128 with 8 waves as 4 x 2 and three
  // LDS stages (192x128 with plane activations: two)
  GEMM_TILE_P16_128x128W42S3 = 51,
  GEMM_TILE_P16_192x128W42S3 = 52,
  // 53 (16x16x32): 96x128 with 8 waves as 2 x 4 and three LDS stages
  GEMM_TILE_P16_96x128W24S3 = 53,
  // 54 (16x16x32 rounding): weight-stationary persistent kernel
  // (gemm_ws.hip) for 1x1 convs with K = 64 / 128 / 256; other shapes run
  // tile 38
  GEMM_TILE_WS = 54,
  // 55 (16x16x32): 64x128 with 8 waves as 2 x 4 and four LDS stages -- short
  // M (the 64-row head GEMMs: 248 split-K workgroups, three chunks in flight)
  GEMM_TILE_P16_64x128W24S4 = 55,
  // 56..59 (16x16x32, own rounding group: K in (channel chunk, tap) order):
  // patch-staged stride-1 3x3 convs (gemm_x3c.hip) -- 192x128 (8 waves), 192x64 (4 waves), 96x128 (8 waves),
  // 192x64 (8 waves); other shapes run tile 38
  GEMM_TILE_C16_FIRST = 56,
  GEMM_TILE_C16_192x128 = 56,
  GEMM_TILE_C16_192x64 = 57,
  GEMM_TILE_C16_96x128 = 58,
  GEMM_TILE_C16_192x64W42 = 59,  // 192x64 with 8 waves (4 x 2)
  // pipelined 16x16x32, 192x128 as 4 x 1 waves: f16x2 only (bf16x3 runs 47)
  GEMM_TILE_P16_192x128W41 = 60,
  GEMM_NUM_TILES = 61
};

struct GemmParams {
  // A operand: implicit im2col over an NHWC tensor (plain rows: H=1, W=M,
  // KH=KW=1).  Row m <-> output pixel (n, oh, ow).
  const float* a;
  int64_t a_bstride;
  uint32_t a_bytes;  // bytes addressable from a (+batch stride), < 2^31
  int H, W, Cin, lda;
  int KH, KW, stride, pad, dil;
  int Ho, Wo;
  int M;
  // B operand: [Ncol][ldb], K contiguous; k >= kb_valid reads as zero.
  const float* b;
  int64_t b_bstride;
  uint32_t b_bytes;  // bytes addressable from b (+batch stride), < 2^31
  int ldb, kb_valid;
  int Ncol;
  int Kloop;  // K extent iterated, multiple of 16
  // optional second A operand (1x1 conv, stride2, no padding) for K >= Kloop1
  const float* a2;
  uint32_t a2_bytes;
  int H2, W2, lda2, stride2;
  int Kloop1;
  // epilogue
  const float* scale;
  const float* shift;
  int64_t ss_bstride;
  const float* residual;
  int64_t ldr;
  float* out;
  int64_t ldo;
  int64_t out_bstride;
  int relu;
  int metric;
  int zero_diag;
  // EPI_DIST in the pipelined kernel, self-distance (A rows == B rows, square
  // tiles): strictly-lower tiles exit, strictly-upper tiles also write the
  // mirrored block out[c][r]
  int sym;
  // split-K of an implicit-GEMM conv (pipelined kernel, EPI_F_RAW partials):
  // slice s covers K elements [s*Kloop, (s+1)*Kloop) of the full im2col K
  // (tap t0 = k0 / Cin, channel k0 % Cin); the A pointer is NOT offset (the
  // plain-GEMM split-K of the heads offsets it instead)
  int ksplit_conv;
  // pipelined distance GEMM on chunk-tiled planes (pps_distmat_x3p_tiled):
  // bit 0 = A, bit 1 = B stored [rows / 16][K / 32][16][32] per plane, so a
  // 16-row DMA piece of one 32-wide K chunk is one contiguous KiB
  int tiled;
  // conv tiles: enumerate output tiles column-major (PPS_TILE_COL_ORDER)
  int colmajor;
  int tile;  // GemmTile; 0 = heuristic
  int splitk;           // >= 1; K slices enumerated with the batch on grid.y
  int64_t out_sstride;  // output stride between K slices (EPI_F_RAW)
  // bf16x3 GEMM (gemm_x3.hip): B as three bf16 planes [3][Ncol][ldb] per
  // batch, b_plane elements apart; b_bstride counts bf16 elements and b_bytes
  // the bytes addressable within ONE plane from its base
  const uint16_t* b3;
  int64_t b_plane;
  // EPI_DIST in the bf16x3 GEMM: precomputed squared norms of A rows / B rows
  const float* norm_a;
  const float* norm_b;
  // bf16x3 activation planes (gemm_x3p.hip only): A read from three bf16
  // planes a3 + k * a_plane with the NHWC indexing of `a` (x = sum of the
  // planes exactly); with EPI_F_PLANES the result is written as three planes
  // out3 + k * out_plane, indexed like `out`
  const uint16_t* a3;
  int64_t a_plane;
  uint16_t* out3;
  int64_t out_plane;
  // EPI_F_PPS (pipelined conv whose M tile is exactly one image, BM = Ho*Wo):
  // the tile's BN + residual + ReLU output is pooled per horizontal strip
  // (pps_h rows each, average and max) and combined into the 2^S - 1 part
  // subsets, written to pps_out [2^S - 1][pps_nimg][Ncol] exactly as
  // pps_part_power_set would; out is written only if pps_write_y
  float* pps_out;
  int pps_S, pps_max_ave, pps_nimg, pps_write_y;
  int pps_h[10];
  // EPI_F_FIX (conv split-K, one launch): each K slice parks its raw partial
  // tile at part + slice * part_sstride ([M][Ncol] dense); a per-tile arrival
  // counter fix_cnt[tile] (zero between launches, reset by the last arrival)
  // picks the slice that sums all partials in slice order and finishes
  float* part;
  int64_t part_sstride;
  int* fix_cnt;
  // f16x2 distance GEMM (gemm_h2.hip): per-row power-of-two inverse scales of
  // the A / B rows (the split stores x * 2^s, the dot product is scaled back);
  // f16x2 convs (EPI_F_H2): rs_b = the weight rows' (output channels') scales
  const float* rs_a;
  const float* rs_b;
  // activation maxima (f16x2 convs): amax_a / amax_a2 = max|x| of the A
  // operand tensor(s), written by their producers; amax_out (any conv
  // epilogue, may be null) receives max|y| of this launch's output by an
  // atomic max on the float bits (the caller zeroes it before the producer)
  const float* amax_a;
  const float* amax_a2;
  float* amax_out;
  // EPI_F_H2OUT (a conv + BN + ReLU producer feeding one f16x2 consumer): the
  // output y <= B = h2o_bw * max|x| + h2o_bb (h2o_bw = max_c |scale_c| |W_c|_1,
  // h2o_bb = max(0, max_c shift_c), max|x| from the input's slot h2o_in) is
  // written as two f16 planes on the power-of-two scale of B (out3 +
  // k * out_plane), and B goes to amax_out: the consumer takes its scale from
  // that slot, so it reads the same fragments its own split of y would make
  const float* h2o_in;
  float h2o_bw, h2o_bb;
};
constexpr int kPpsFuseMaxStrips = 10;
constexpr int kPpsFuseMaxCols = 256;  // widest tile the fused pooling takes (two column passes)

int launch_gemm(const GemmParams& p, int epi, int batch, hipStream_t stream);
int launch_gemm_x3(const GemmParams& p, int epi, int batch, hipStream_t stream);
bool x3p_eligible(const GemmParams& p, int epi);
int launch_gemm_x3p(const GemmParams& p, int epi, int batch, hipStream_t stream, int variant);
int x3p_tile_rows(int tile, bool a3);  // rows (BM) of a pipelined tile id, 0 if none
int x3p_tile_cols(int tile, bool a3);  // its columns (BN)
int split_bf16x3(const float* x, int64_t n, int nbatch, uint16_t* out, hipStream_t stream);
int row_sqnorm(const float* x, int64_t rows, int D, int64_t ld, float* out, hipStream_t stream);
int split_sqnorm(const float* x, int64_t rows, int D, int64_t ld, uint16_t* out3, float* out,
                 hipStream_t stream);
int split_sqnorm_tiled(const float* x, int64_t rows, int D, int64_t ld, uint16_t* out3t,
                       float* out, hipStream_t stream);
int pick_tile(const GemmParams& p, int batch);
bool ws_eligible(const GemmParams& p, int epi, int batch);
int launch_gemm_ws(const GemmParams& p, int epi, hipStream_t stream);
bool x3c_eligible(const GemmParams& p, int epi, int batch, int tile);
int launch_gemm_x3c(const GemmParams& p, int epi, hipStream_t stream, int tile);
int x3c_tile_rows(int tile);  // rows (BM) of a patch-staged tile id, 0 if none
int x3c_tile_cols(int tile);

// An activation-max slot (PPS_AMAX_SLOT_FLOATS floats, zeroed before its
// producer runs): kAmaxSubs partial maxima kAmaxStride floats (256 B) apart,
// each wave folds its max into one of them (spread by workgroup and wave, so
// thousands of same-address atomics do not queue at one memory channel); the
// tensor's max is the max of the partials.
constexpr int kAmaxSubs = 16;
constexpr int kAmaxStride = 64;
static_assert(kAmaxSubs * kAmaxStride == PPS_AMAX_SLOT_FLOATS, "amax slot layout");

// max |y| of a wave's outputs (every value >= 0: float bits compare as
// unsigned) folded into the slot.  All lanes of the wave must be converged.
__device__ inline void amax_commit(float* slot, float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  const unsigned sub = (blockIdx.x + 5u * blockIdx.y + 3u * blockIdx.z + (threadIdx.x >> 6)) &
                       (kAmaxSubs - 1);
  if ((threadIdx.x & 63) == 0)
    atomicMax(reinterpret_cast<unsigned*>(slot + sub * kAmaxStride),
              __builtin_bit_cast(unsigned, v));
}

// The tensor max a slot holds
__device__ inline float amax_read(const float* slot) {
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < kAmaxSubs; ++j) m = fmaxf(m, slot[j * kAmaxStride]);
  // the same value in every lane: kept in a scalar register (the GEMM main
  // loops carry the scales derived from it)
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, m)));
}

// f16x2 activation split: x 2^s with s = 15 - E for max|x| = m 2^E, m in
// [0.5, 1) (a zero max keeps 2^0; the exponent clamped to f32's range), so
// max|x 2^s| lies in [2^14, 2^15).  Returns 2^s; *inv = 2^-s.
__host__ __device__ inline float h2_scale_of(float amax, float* inv) {
  const unsigned ebits = (__builtin_bit_cast(unsigned, amax) >> 23) & 0xffu;
  int sh = ebits == 0 ? (amax > 0.f ? 126 : 0) : 15 - ((int)ebits - 126);
  sh = sh > 126 ? 126 : (sh < -126 ? -126 : sh);
  *inv = __builtin_bit_cast(float, (unsigned)(127 - sh) << 23);
  return __builtin_bit_cast(float, (unsigned)(127 + sh) << 23);
}

// ---- op-level implementations behind the pps_conv* / pps_stem / pps_maxpool
// entry points (abi.hip, stem.hip, feature_ops.hip), with the activation-max
// plumbing the whole-network plan uses (model.hip): amax_out (may be null)
// receives max|y| of the launch's output; w_rs != null selects the f16x2
// arithmetic (two-plane chunk-tiled weights w, per-channel scales w_rs, the
// input tensors' maxima amax_in / amax_in2)
int conv_impl(const float* x, int N, int H, int W, int Cin, int ldx, const void* w, int x3,
              int Cout, int Kpad, int KH, int KW, int stride, int pad, int dil,
              const float* scale, const float* shift, const float* residual, int relu, float* y,
              int Ho, int Wo, int ldy, int tile, void* stream, const uint16_t* x_pl,
              int64_t x_plane, uint16_t* y_pl, int64_t y_plane, int splitk, float* part,
              int* fix_cnt, int64_t n_cnt, float* amax_out, const float* w_rs,
              const float* amax_in, uint16_t* y_h2 = nullptr, int64_t y_h2_plane = 0,
              const float* h2o_in = nullptr, float h2o_bw = 0.f, float h2o_bb = 0.f);
int dual_impl(const float* x, int N, int H, int W, int Cin, int ldx, int KH, int KW, int stride,
              int pad, const float* x2, int H2, int W2, int Cin2, int ldx2, int stride2,
              const void* w, int x3, int Cout, int Kpad1, int Kpad2, const float* shift, int relu,
              float* y, int Ho, int Wo, int ldy, int tile, void* stream, float* amax_out,
              const float* w_rs, const float* amax_in, const float* amax_in2);
int conv_pps_impl(const float* x, const uint16_t* x3, int64_t x_plane, int N, int H, int W,
                  int Cin, int ldx, const uint16_t* w3, int Cout, int Kpad, int KH, int KW,
                  int stride, int pad, int dil, const float* scale, const float* shift,
                  const float* residual, float* y, int Ho, int Wo, const int32_t* splits, int S,
                  int max_ave, float* pps_out, int tile, void* stream, const float* w_rs,
                  const float* amax_in);
int stem_conv_pool_x3(const float* x, int N, int H, const uint16_t* w3, const float* scale,
                      const float* shift, float* y, int Hc, int Hp, hipStream_t st, float* amax);
int stem_conv_pool_h2(const float* x, int N, int H, const uint16_t* w2, const float* w_inv,
                      const float* scale, const float* shift, float* y, int Hc, int Hp,
                      hipStream_t st, float* amax, const float* amax_in);
int stem_split_h2(const float* w, uint16_t* w2, float* w_inv, hipStream_t st);
// image preprocessing (pps_preprocess_bgr[_ragged]); amax (may be null)
// receives max |y| (the f16x2 stem's input scale)
int preprocess_bgr(const uint8_t* img, int N, int Hi, int Wi, const int64_t* offsets,
                   const int32_t* heights, const int32_t* widths, const float* means, int Ho,
                   int Wo, float* y, hipStream_t st, float* amax = nullptr);
int maxpool2d(const float* x, int N, int H, int W, int C, int k, int stride, int pad, float* y,
              int Ho, int Wo, hipStream_t st, float* amax);
// max |x| of n floats into *amax (atomic max on the float bits; zero it first)
int split_act_h2(const float* x, int64_t n, const float* slot, uint16_t* planes, int64_t plane,
                 hipStream_t st);
int amax_of(const float* x, int64_t n, float* amax, hipStream_t st);

// ---- f16x2 distance GEMM (gemm_h2.hip) ---------------------------------------
constexpr int kH2NumTiles = 8;
int launch_gemm_h2(const GemmParams& p, hipStream_t stream, int tile);
int split_h2_sqnorm_tiled(const float* x, int64_t rows, int D, int64_t ld, uint16_t* out2t,
                          float* rscale, float* sqnorm, hipStream_t stream);

// ---- bottleneck seam (gemm_seam.hip): branch2c of block i + branch2a of block i+1
struct SeamParams {
  const float* a;        // [M][K1] branch2c input (f32 NHWC rows)
  const float* res;      // [M][N1] the block's shortcut (its input trunk)
  const uint16_t* w2c;   // [3][N1][K1] bf16x3 planes, plane stride N1 * K1
  const float* s2c;
  const float* t2c;
  float* t;              // [M][N1] trunk out
  const uint16_t* w2a;   // [3][N2][N1] planes, plane stride N2 * N1
  const float* s2a;
  const float* t2a;
  float* y;              // [M][N2] next branch2a out
  int M;
  float* amax_t = nullptr;  // max |trunk| / max |y| (atomic max, may be null)
  float* amax_y = nullptr;
};
bool seam_supported(int K1, int N1, int N2);
int launch_seam_x3(const SeamParams& p, int K1, int N1, int N2, hipStream_t st);

// ---- retrieval (rank.hip) ---------------------------------------------------
constexpr int kMergeMaxLists = 64;
// rank_count_stream / cmc_counts: gallery entries per workgroup (grid.y =
// chunks of a row, <= 65535)
#ifndef RANK_STREAM_U
#define RANK_STREAM_U 8   // float4 per thread in flight in the rank streams
#endif
constexpr int kRankStreamChunk = 256 * 4 * RANK_STREAM_U;
// rank_prepare merges R*Pmax positives in dynamic LDS (4 int arrays):
// 16 B per merged positive, 128 KiB at the cap -- within gfx950's 160 KiB
// LDS per workgroup (this library is built for gfx950 only)
constexpr int kRankMergeCap = 8192;
constexpr int kLdsBytesGfx950 = 160 * 1024;
static_assert(16 * kRankMergeCap <= kLdsBytesGfx950, "rank_prepare LDS exceeds the CU's LDS");
struct MergeOffsets {  // kernel-argument copy of the per-list global offsets
  int64_t off[kMergeMaxLists];
};
int topk_merge(const float* vals, const int32_t* idx, int R, int64_t Q, int kin,
               const MergeOffsets& offs, int kout, float* out_vals, int32_t* out_idx,
               hipStream_t st);

// ---- re-ranking (rerank.hip) -------------------------------------------------
// The concatenated distance matrix M = [[q_q, q_g], [q_g^T, g_g]]
// (reid_dataset_evaluator.py:447-452) read in place from its blocks (row
// strides ld*; qgT = q_g transposed, [G][ldT]), and for a SYMMETRIC M (q_q,
// g_g exactly symmetric) the normalised square of :452-454,
// OD[i][j] = M[j][i]^2 / colmax[i] = M[i][j]^2 / colmax[i], computed on the fly
// with the arithmetic of the OD-building kernels (rr_od).
// OD's arithmetic, float32 as NumPy does it (np.power(M, 2) then / colmax):
// a rounded square and an IEEE (correctly rounded) division -- spelled with
// the _rn intrinsics so that every kernel computing it gives the same bits
// (a plain `/` may be lowered to a reciprocal-based approximation)
// (m * m) / cm, both rounded (a product feeding a division cannot fuse)
// dynamic LDS of the Jaccard pass for a gallery of G (rerank.hip)
size_t jaccard_lds_bytes(int64_t G);

__device__ inline float rr_od(float m, float cm) { return (m * m) / cm; }

struct RrMatrix {
  const float* qg;
  const float* qq;
  const float* gg;
  const float* qgT;
  int64_t ldqg, ldqq, ldgg, ldT, Q, G;
  const float* colmax;
  __device__ float m(int64_t r, int64_t c) const {
    if (r < Q) return c < Q ? qq[r * ldqq + c] : qg[r * ldqg + (c - Q)];
    return c < Q ? qgT[(r - Q) * ldT + c] : gg[(r - Q) * ldgg + (c - Q)];
  }
  __device__ float od(int64_t i, int64_t j) const {
    return rr_od(m(i, j), colmax[i]);
  }
};
// stable (value, index) top-k of every row of OD (symmetric M, rows of N =
// Q + G >= 16384 entries, every block 16-byte aligned): the wave-streaming
// top-k reading M's blocks in place (no N x N OD buffer)
int topk_rr(const RrMatrix& M, int k, float* vals, int32_t* idx, hipStream_t st);
// symmetric M with colmax not yet known: rowmax[q] = max of row q's squares
// (= column q's), and the top-k by (OD, index) through a top-(k+8) on m * m
// (rank.hip); scratch of topk_rr_sq_scratch_bytes(N, k)
int topk_rr_sq(const RrMatrix& M, int k, float* rowmax, void* scratch, size_t scratch_bytes,
               float* vals, int32_t* idx, hipStream_t st);
size_t topk_rr_sq_scratch_bytes(int64_t N, int k);
bool topk_rr_eligible(const RrMatrix& M, int k);

}  // namespace pps
