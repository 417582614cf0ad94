/*
 * pps_abi.h -- C ABI of libpps_hip.so, the MI355X (gfx950) re-ID inference +
 * retrieval path for PPS (shenyunhang/PPS).
 *
 * Conventions:
 *   - Every buffer is caller-owned DEVICE memory (HBM), except where a
 *     parameter is documented as host memory.  No entry point allocates,
 *     frees or synchronises; all work is enqueued on `stream` (a hipStream_t
 *     passed as void*; NULL = the legacy default stream), so a caller may
 *     capture a sequence of calls into a hipGraph.
 *   - Activations are NHWC float32.  Conv weights are packed [Cout][Kpad]
 *     with K ordered (kh, kw, cin) and zero padded to Kpad (multiple of 16).
 *   - Return value: PPS_OK (0) or a negative PPS_ERR_* code.  No C++
 *     exception crosses the ABI.  pps_last_error() returns a thread-local,
 *     ENFORCE-style message for the last failing call on this thread; the
 *     Python layer raises it as RuntimeError, as Caffe2's CAFFE_ENFORCE
 *     did (reference detectron/tests/test_zero_even_op.py:48-51).
 *   - Re-entrant per stream; no global mutable state besides the
 *     thread-local error string.
 */
#ifndef PPS_ABI_H_
#define PPS_ABI_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PPS_OK 0
#define PPS_ERR_INVALID_ARG -1   /* shape / pointer / alignment check failed */
#define PPS_ERR_UNSUPPORTED -2   /* valid request outside what is built     */
#define PPS_ERR_LAUNCH -3        /* hipGetLastError after launch != success  */
#define PPS_ERR_CAPACITY -4      /* a fixed-capacity buffer was too small    */

#define PPS_METRIC_EUCLIDEAN 0   /* sqrt(max(|q|^2 + |g|^2 - 2 q.g, 0))      */
#define PPS_METRIC_SQEUCLIDEAN 1 /* max(|q|^2 + |g|^2 - 2 q.g, 0)            */
#define PPS_METRIC_COSINE 2      /* 1 - q.g / (max(|q|,eps) max(|g|,eps))    */

/* ---- library ------------------------------------------------------------ */
int pps_abi_version(void);
const char* pps_last_error(void);
/* Names of the exported operator-registry entries, ';'-separated (host). */
const char* pps_registered_ops(void);

/* GEMM tile configurations shared by pps_distmat / pps_conv2d_bn_act /
 * pps_gemm_bn_act_batched (`tile` argument): 0 = built-in heuristic,
 * 1 = 128x128 (4 waves), 2 = 128x64, 3 = 64x128, 4 = 64x64, 5 = 256x128
 * (8 waves), 6..10 = the same shapes with a 32-wide K chunk per barrier,
 * 11..20 = ids 1..10 with the `_x3` kernels' A operand kept f32 in LDS and
 * split after the fragment read (the f32 kernels treat them as 1..10),
 * 21..28 = 192-row tiles of the `_x3` kernels (192x128 / 192x64, K chunk
 * 16 / 32, A staged as planes / f32; the f32 kernels use 128-row tiles),
 * 29..37 = the `_x3` LDS-DMA pipelined tiles (128x128, 192x128, 128x64,
 * 192x64 with 4 waves; 256x128, 128x256, 192x256, 128x128, 192x128 with 8
 * waves; K chunk 32; the f32 kernels use the heuristic), 38..46 = the same
 * pipelined tiles on 16x16x32 MFMA blocks (192x256 -> 128x256), 47 =
 * 192x128 (8 waves, 4 x 2), 48 = 192x64 (4 waves), 49 = 96x128 (4 waves),
 * 50 = 96x128 (8 waves, 2 x 4), 51 / 52 = 128x128 / 192x128 (8 waves,
 * 4 x 2) with three LDS stages, 53 = tile 50 with three stages, all on
 * 16x16x32 blocks; 54 = the weight-stationary persistent kernel for 1x1
 * convs with K = 64 / 128 / 256 (stationary weight columns in LDS,
 * activations streamed to registers; other shapes run tile 38); 55 = 64x128
 * (8 waves, 2 x 4, four LDS stages: short-M split-K head GEMMs); 56 / 57 /
 * 58 / 59 = patch-staged stride-1 3x3 convs (192x128 8 waves / 192x64 4
 * waves / 96x128 8 waves / 192x64 8 waves; the tile's input patch staged once per 32-channel chunk,
 * K in (channel chunk, tap) order: their own rounding group; other shapes
 * run tile 38); 60 = 192x128 as 4 x 1 waves (48 x 128 per wave) for the
 * f16x2 entries (the bf16x3 entries run tile 47 for it).  Results
 * are identical for every tile below 38 (same per-element fp32 MFMA
 * accumulation order) and identical among the tiles from 38 on (one MFMA
 * sums a 32-wide K chunk: a different rounding
 * sequence, same f32-level error); only speed differs, so callers may
 * autotune. */
int pps_gemm_num_tiles(void);
/* Or-ed into the `tile` of pps_conv2d_bn_act_x3 / _x3p / pps_conv2d_bn_act_pps_x3p
 * (pipelined ids 29..53 and 55+): the bf16x3 weights are chunk-tiled,
 * [3][Cout16/16][Kpad/32][16][32] (pps_tile_planes over the [3][Cout][Kpad]
 * planes; Cout16 = Cout rounded up to 16, Cin % 32 == 0).  Same bits. */
#define PPS_TILE_B_TILED 0x100
/* Or-ed into the same tiles: walk the output tiles column block by column
 * block (consecutive workgroups -- one XCD -- share a weight block instead
 * of an activation panel).  Same bits. */
#define PPS_TILE_COL_ORDER 0x200
/* Whole-network plan only (pps_model_set_tile / autotune), on a bottleneck's
 * branch2c (1x1 + BN + identity residual + ReLU) whose output feeds the next
 * block's branch2a (1x1 + BN + ReLU): one launch of the bottleneck seam kernel
 * (pps_conv1x1_seam_x3) computes both -- the trunk is written for the next
 * block's residual and never re-read for its branch2a; the branch2a layer's
 * own tile is then not launched.  Base tile 54 (the same 16x16x32 rounding
 * group: same bits).  (Cin, Cout, next Cout) = (64, 256, 64) or (128, 512,
 * 128), f32 activations at both ends, no split-K. */
#define PPS_TILE_SEAM 0x400
/* Whole-network plan only, or-ed into a conv / fused-shortcut / conv_pps
 * layer's tile: run the layer in the f16x2 arithmetic of
 * pps_conv2d_bn_act_h2 (three f16 MFMA terms per product) on base tile 0,
 * 38..53, 55, 54 for a 1x1 / stride-1 conv or fused-shortcut conv with K =
 * 64 / 128 / 256 (the weight-stationary kernel with the f16x2 weight planes
 * in LDS; f32 input, no PPS_TILE_H2P / H2E) or, for stride-1 3x3 convs,
 * 56..59 (conv_pps: its 192-row tiles >= 38), optionally with
 * PPS_TILE_COL_ORDER; f32 activations at both
 * ends (no plane edge), no split-K.  The handle keeps the f16x2 weight split
 * beside the bf16x3 one; each forward zeroes its per-tensor activation maxima
 * and every producer reports max|y| from its epilogue (the f16x2 layers'
 * input scales).  On the fused stem (`stem_pool` layer) PPS_TILE_H2 alone
 * (tile 0x800) selects pps_stem_conv_pool_h2; the forward then measures its
 * input's max (pps_forward_bgr: reported by the preprocessing kernel). */
#define PPS_TILE_H2 0x800
/* With PPS_TILE_H2 on a conv / conv_pps layer: the layer's input is split
 * into f16x2 activation planes by one pass (pps_split_f16x2_act) just before
 * the conv, which then reads the planes (same bits, no split arithmetic in
 * its main loop; a workspace buffer of 4 B per input element). */
#define PPS_TILE_H2P 0x1000
/* With PPS_TILE_H2 on a conv / conv_pps layer C whose input is the output of
 * a conv + BN + ReLU layer P read by C alone (no residual, Cin % 32 == 0, not
 * the second half of a seam pair): P writes its output as f16x2 planes on
 * the scale of its output bound (pps_conv2d_bn_act_h2out; P in either
 * arithmetic, on a pipelined 16x16x32 tile) and C reads them -- no split in
 * C's main loop and no split pass, same bits as C splitting the f32 output on
 * that scale (C on a pipelined tile or, round 6, a patch tile 56-59; the same
 * for PPS_TILE_H2P). */
#define PPS_TILE_H2E 0x2000

/* ---- retrieval: distance matrix ------------------------------------------
 * Replaces reid_dataset_evaluator.py:244-272 `compute_dist(array1, array2,
 * type)` (euclidean branch; cosine is defined as a true distance, the
 * reference's cosine branch is broken).
 * out[i*ldo + j] = metric(q[i,:], g[j,:]); q is [Q][ldq], g is [G][ldg],
 * D valid columns, D % 4 == 0, ldq/ldg/ldo % 4 == 0, 16-B aligned pointers.
 * FP32 MFMA (v_mfma_f32_32x32x2_f32) tiles; squared norms fused. */
int pps_distmat(const float* q, int64_t Q, int64_t ldq,
                const float* g, int64_t G, int64_t ldg, int D, int metric,
                float* out, int64_t ldo, int tile, void* stream);

/* The distance matrix on bf16 matrix cores (same f32-level error as
 * pps_distmat, see the "x3" block below): g3 = pps_split_bf16x3(g) as planes
 * [3][G][ldg]; qsq / gsq = pps_row_sqnorm of q / g (a gallery index is
 * split and normed once, then scored against any number of query batches). */
int pps_row_sqnorm(const float* x, int64_t rows, int D, int64_t ld, float* out,
                   void* stream);
/* Both in one read of x (a gallery index or a query batch): out3 =
 * pps_split_bf16x3 planes [3][rows][D] (row stride D, plane stride rows*D),
 * sqnorm = pps_row_sqnorm; bit-identical to the two calls.  D % 4 == 0,
 * ld % 4 == 0, x 16-byte and out3 8-byte aligned. */
int pps_split_bf16x3_sqnorm(const float* x, int64_t rows, int D, int64_t ld,
                            uint16_t* out3, float* sqnorm, void* stream);
int pps_distmat_x3(const float* q, int64_t Q, int64_t ldq, const float* qsq,
                   const uint16_t* g3, const float* gsq, int64_t G, int64_t ldg, int D,
                   int metric, float* out, int64_t ldo, int tile, void* stream);
/* pps_distmat_x3 with the queries ALSO pre-split into bf16x3 planes
 * q3 [3][Q][ldq] (pps_split_bf16x3; plane stride Q*ldq): both operands are
 * then staged by pure DMA.  Same bits as pps_distmat_x3.  Pipelined tiles
 * only (tile 0 or >= 29); D % 32 == 0, ldq % 8 == 0, ldg % 8 == 0. */
int pps_distmat_x3p(const uint16_t* q3, int64_t Q, int64_t ldq, const float* qsq,
                    const uint16_t* g3, const float* gsq, int64_t G, int64_t ldg,
                    int D, int metric, float* out, int64_t ldo, int tile,
                    void* stream);
/* Chunk-tiled planes (experimental layout for the distance GEMM): planes
 * [3][rows][ld] (plane stride plane_stride) -> out [3][rows16/16][D/32][16][32],
 * rows16 = rows rounded up to 16, padding rows zero; D % 32 == 0.  out holds
 * 3 * rows16 * D bf16. */
int pps_tile_planes(const uint16_t* planes, int64_t rows, int D, int64_t ld,
                    int64_t plane_stride, uint16_t* out, void* stream);
/* pps_split_bf16x3_sqnorm writing the planes chunk-tiled (the layout of
 * pps_tile_planes; out3t holds 3 * rows16 * D bf16, padding rows zero):
 * one read of x, the same bits. */
int pps_split_bf16x3_sqnorm_tiled(const float* x, int64_t rows, int D, int64_t ld,
                                  uint16_t* out3t, float* sqnorm, void* stream);
/* pps_distmat_x3p on tiled query and gallery planes (pps_tile_planes): each
 * 16-row DMA piece of a 32-wide K chunk is one contiguous KiB.  Same bits as
 * pps_distmat_x3p on the same tile; pipelined tiles 29..53 (0 = 43, 128 x 256). */
int pps_distmat_x3p_tiled(const uint16_t* q3t, int64_t Q, const float* qsq,
                          const uint16_t* g3t, const float* gsq, int64_t G, int D,
                          int metric, float* out, int64_t ldo, int tile, void* stream);
/* Self-distance of one feature set x [N][ld] (the reference's
 * compute_dist(g, g) / compute_dist(q, q) of re-ranking and multi-query,
 * reid_dataset_evaluator.py:169-175, 195-206): out [N][N] from the tiles of
 * the upper triangle only (enumerated by lcm(BM, BN) super-blocks), each
 * writing its elements on or above the diagonal and mirroring the strictly-
 * upper ones (half the MFMA work).  x3 = pps_split_bf16x3(x) planes, xsq =
 * pps_row_sqnorm(x).  Any pipelined tile (29..53, 55; 0 = 43, 128 x 256);
 * D % 32 == 0.  Entry (i, j), i <= j, equals pps_distmat_x3's on the same
 * tile; the lower triangle holds exact copies (a symmetric matrix, unlike
 * the rounding-asymmetric full product). */
int pps_distmat_x3_self(const float* x, int64_t N, int64_t ld, const float* xsq,
                        const uint16_t* x3, int D, int metric, float* out,
                        int64_t ldo, int tile, void* stream);

/* pps_distmat_x3_self from chunk-tiled planes x3t [3][N16/16][D/32][16][32]
 * (pps_split_bf16x3_sqnorm_tiled: planes + xsq in one pass): both operands
 * staged by pure DMA, as pps_distmat_x3p_tiled.  Same bits as
 * pps_distmat_x3_self on the same tile. */
int pps_distmat_x3_self_tiled(const uint16_t* x3t, int64_t N, const float* xsq, int D,
                              int metric, float* out, int64_t ldo, int tile, void* stream);

/* ---- f16x2 distance GEMM ("h2", round 5) -----------------------------------
 * The same distances as pps_distmat_x3p_tiled / pps_distmat_x3_self_tiled in
 * THREE f16 MFMA terms per product instead of six bf16 ones.  Each row x is
 * scaled by a power of two 2^s (per row: max|x 2^s| in [2^14, 2^15)) and
 * split x 2^s = h0 + h1 + r, h0 = f16(x 2^s), h1 = f16(x 2^s - h0),
 * |r| <= 2^-22 |x 2^s|; q.g = 2^-(s_q + s_g) (h0.h0' + h0.h1' + h1.h0') with
 * f32 accumulation (csrc/gemm_h2.hip states the error bound).  Same metric
 * formulas and squared norms as the x3 path.
 *
 * pps_split_f16x2_sqnorm_tiled: one read of x [rows][ld] -> out2t, the two
 * f16 planes chunk-tiled [2][rows16/16][D/32][16][32] (rows16 = rows rounded
 * up to 16, padding rows zero; 2 * rows16 * D f16), rscale[r] = 2^-s_r and
 * sqnorm[r] = pps_row_sqnorm's value (same bits).  D % 32 == 0. */
int pps_split_f16x2_sqnorm_tiled(const float* x, int64_t rows, int D, int64_t ld,
                                 uint16_t* out2t, float* rscale, float* sqnorm, void* stream);
/* Query x gallery distances from two such splits.  tile: 0 = default
 * (256 x 256, 8 waves), 1..pps_h2_num_tiles()-1 the alternatives listed in
 * csrc/gemm_h2.hip (speed only: every tile gives the same bits). */
int pps_distmat_h2_tiled(const uint16_t* q2t, int64_t Q, const float* qsq, const float* qrs,
                         const uint16_t* g2t, const float* gsq, const float* grs, int64_t G,
                         int D, int metric, float* out, int64_t ldo, int tile, void* stream);
/* Self-distance of one split (upper-triangle tiles + mirror: an exactly
 * symmetric matrix whose upper triangle has the bits of pps_distmat_h2_tiled
 * on the same operands). */
int pps_distmat_h2_self_tiled(const uint16_t* x2t, int64_t N, const float* xsq, const float* xrs,
                              int D, int metric, float* out, int64_t ldo, int tile,
                              void* stream);
int pps_h2_num_tiles(void);

/* An activation-max slot: PPS_AMAX_SLOT_FLOATS device floats, zeroed before
 * its producer runs.  Producers fold max|y| into it by atomic maxima on the
 * float bits, spread over 16 partial maxima 64 floats (256 B) apart; the
 * tensor's max is the max of slot[0], slot[64], ..., slot[960]. */
#define PPS_AMAX_SLOT_FLOATS 1024

/* ---- f16x2 convolutions ("h2", round 5) ---------------------------------
 * The conv entry points above in the f16x2 arithmetic of pps_distmat_h2_*:
 * three f16 MFMA terms per product instead of six bf16 ones.  Weights: the
 * packed [Cout][Kpad] f32 weights split per output channel by
 * pps_split_f16x2_sqnorm_tiled (w2t chunk-tiled [2][Cout16/16][Kpad/32][16]
 * [32], wrs[c] = 2^-s_c).  Activations stay f32 NHWC; the kernel scales them
 * by the power of two 2^s_a with max|x 2^s_a| in [2^14, 2^15), taken from
 * the activation-max slot amax_x (above; e.g. filled by the producer of x
 * through its amax_y, or by pps_amax), and splits them into two f16 terms
 * after the LDS fragment read.  amax_y (a zeroed slot or NULL) receives
 * max|y|.  Cin % 32 == 0,
 * Kpad == KH*KW*Cin; tile 0 (= 38), the 16x16x32 pipelined tiles 38..53, 55,
 * the weight-stationary tile 54 (1x1 / stride 1 / K = 64, 128, 256; other
 * shapes run 38) and the patch tiles 56..59, or-ed with PPS_TILE_COL_ORDER;
 * no planes, no split-K.  Every tile gives the same bits; the same f32-level
 * error as the x3 entries (tests/test_gpu_h2_conv.py). */
int pps_conv2d_bn_act_h2(const float* x, int N, int H, int W, int Cin, int ldx,
                         const uint16_t* w2t, const float* wrs, int Cout, int Kpad, int KH,
                         int KW, int stride, int pad, int dil, const float* scale,
                         const float* shift, const float* residual, int relu, float* y, int Ho,
                         int Wo, int ldy, const float* amax_x, float* amax_y, int tile,
                         void* stream);
/* pps_conv2d_dual_bn_act_x3 (projection shortcut K-concatenated) in f16x2:
 * both inputs share the scale of max(*amax_x, *amax_x2); Cin2 % 32 == 0;
 * tiles 0, 38..55 (54: the weight-stationary kernel when K = Cin + Cin2 is
 * 64, 128 or 256) or 60. */
int pps_conv2d_dual_bn_act_h2(const float* x, int N, int H, int W, int Cin, int ldx, int KH,
                              int KW, int stride, int pad, const float* x2, int H2, int W2,
                              int Cin2, int ldx2, int stride2, const uint16_t* w2t,
                              const float* wrs, int Cout, int Kpad1, int Kpad2,
                              const float* shift, int relu, float* y, int Ho, int Wo, int ldy,
                              const float* amax_x, const float* amax_x2, float* amax_y, int tile,
                              void* stream);
/* pps_conv2d_bn_act_pps_x3p (last conv + part pooling) in f16x2. */
int pps_conv2d_bn_act_pps_h2(const float* x, int N, int H, int W, int Cin, int ldx,
                             const uint16_t* w2t, const float* wrs, int Cout, int Kpad, int KH,
                             int KW, int stride, int pad, int dil, const float* scale,
                             const float* shift, const float* residual, float* y, int Ho, int Wo,
                             const int32_t* splits, int S, int max_ave, float* pps_out,
                             const float* amax_x, int tile, void* stream);
/* f16x2 activation planes: planes [2][plane] f16 (int16 storage) =
 * f16(x 2^s), f16(x 2^s - hi) with 2^s from the slot amax -- the split the
 * f16x2 conv kernels make after an f32 fragment read, done once per element.
 * n % 8 == 0, plane >= n, 16-byte aligned.  The _planes conv entries take
 * them in place of x (same bits as the f32 entries on x with that max). */
int pps_split_f16x2_act(const float* x, int64_t n, const float* amax, uint16_t* planes,
                        int64_t plane, void* stream);
int pps_conv2d_bn_act_h2_planes(const uint16_t* x2, int64_t x_plane, int N, int H, int W,
                                int Cin, int ldx, const uint16_t* w2t, const float* wrs, int Cout,
                                int Kpad, int KH, int KW, int stride, int pad, int dil,
                                const float* scale, const float* shift, const float* residual,
                                int relu, float* y, int Ho, int Wo, int ldy, const float* amax_x,
                                float* amax_y, int tile, void* stream);
int pps_conv2d_bn_act_pps_h2_planes(const uint16_t* x2, int64_t x_plane, int N, int H, int W,
                                    int Cin, int ldx, const uint16_t* w2t, const float* wrs,
                                    int Cout, int Kpad, int KH, int KW, int stride, int pad,
                                    int dil, const float* scale, const float* shift,
                                    const float* residual, float* y, int Ho, int Wo,
                                    const int32_t* splits, int S, int max_ave, float* pps_out,
                                    const float* amax_x, int tile, void* stream);
/* A conv + BN + ReLU producer whose output feeds one f16x2 conv: the
 * output is written as f16x2 planes y2 [2][y_plane] on the power-of-two
 * scale of the bound B = bound_w * max|x| + bound_b >= max|y| (max|x| from
 * the slot bound_in; bound_w / bound_b from pps_h2_out_bound on the packed
 * f32 weights, BN scale and shift), and B goes to the slot bound_out -- the
 * consumer's activation slot, so it takes the same scale and reads the
 * fragments it would split from the f32 output (same bits as the f32 path
 * given that slot).  w: bf16x3 planes (wrs NULL; pipelined 16x16x32 tiles,
 * f32 x) or chunk-tiled f16x2 weights with wrs (x or planes x2 [2][x_plane]
 * with amax_x, as pps_conv2d_bn_act_h2[_planes]).  No residual, no split-K,
 * Cin % 32 == 0. */
int pps_conv2d_bn_act_h2out(const float* x, const uint16_t* x2, int64_t x_plane, int N, int H,
                            int W, int Cin, int ldx, const void* w, const float* wrs, int Cout,
                            int Kpad, int KH, int KW, int stride, int pad, int dil,
                            const float* scale, const float* shift, uint16_t* y2, int64_t y_plane,
                            int Ho, int Wo, int ldy, const float* amax_x, const float* bound_in,
                            float bound_w, float bound_b, float* bound_out, int tile,
                            void* stream);
/* out2 (HOST) = {max_c |scale_c| * sum_k |w[c][k]|, max(0, max_c shift_c)}
 * of packed f32 conv weights w [Cout][Kpad] (scale may be NULL: 1), padded
 * up by 2^-20 relative: the bound constants of pps_conv2d_bn_act_h2out.
 * Synchronous; the same value on every call. */
int pps_h2_out_bound(const float* w, int Cout, int Kpad, const float* scale, const float* shift,
                     float* out2, void* stream);
/* max |x| over n floats into the activation-max slot amax (zero it first):
 * the input scale the f16x2 entries take, for a tensor whose producer did
 * not report it. */
int pps_amax(const float* x, int64_t n, float* amax, void* stream);
/* Caffe2 operator `PairWiseDistance` (detectron/ops/pairwise_distance_op.cu
 * :9-21,26-41): Z[p,q] = sum_d (X[p,d]-X[q,d])^2, X [N][D], Z [N][N].
 * The diagonal is exactly 0 as in the reference's difference form. */
int pps_pairwise_distance(const float* X, int N, int D, float* Z,
                          void* stream);

/* ---- retrieval: rank / evaluation ----------------------------------------
 * Count-based mAP/CMC (reid_dataset_evaluator.py:283-363 `cmc`, :366-439
 * `mean_ap`): identical to sorting each row with a stable (distance, index)
 * order, without materialising the sort.  Gallery may be a shard
 * [g_offset, g_offset+G) of a global gallery.
 *
 * 1) pps_collect_positives: for each query row, list the gallery entries that
 *    are true matches (gid == qid && gcam != qcam), as (distance, global
 *    gallery index), in index order.  pos_cnt[q] may exceed Pmax, in which
 *    case only Pmax entries are stored and the caller must retry larger. */
int pps_collect_positives(const float* dist, int64_t Q, int64_t G,
                          int64_t ldd, const int32_t* qid,
                          const int32_t* qcam, const int32_t* gid,
                          const int32_t* gcam, int64_t g_offset, int Pmax,
                          float* pos_d, int32_t* pos_idx, int32_t* pos_cnt,
                          void* stream);
/* 2) pps_rank_counts: R positive lists ([R][Q][Pmax] entries, counts
 *    [R][Q]) are merged and sorted per query by (distance, index) into
 *    sorted_d [Q][R*Pmax] / sorted_idx (padding +inf / -1; pos_total[q] =
 *    merged count); then for every valid gallery entry of
 *    THIS shard (not same id & same cam) its distance is binned against the
 *    sorted positives: hist[q][p] += 1 where p = first positive with
 *    d_p >= d_i, and before[q] counts entries ordered before the first
 *    positive.  hist / before are ADDITIVE over gallery shards (sum with an
 *    all-reduce), and must be zeroed by the caller.  Capacity: R*Pmax <=
 *    2048 (LDS), else PPS_ERR_CAPACITY -- the streaming entry points below
 *    have no such limit and are what the Python evaluator uses. */
int pps_rank_counts(const float* dist, int64_t Q, int64_t G, int64_t ldd,
                    const int32_t* qid, const int32_t* qcam,
                    const int32_t* gid, const int32_t* gcam, int64_t g_offset,
                    int R, int Pmax, const float* pos_d,
                    const int32_t* pos_idx, const int32_t* pos_cnt,
                    float* sorted_d, int32_t* sorted_idx, int32_t* pos_total,
                    int32_t* hist, int32_t* before, void* stream);
/* 3) pps_ap_finalize: per query AP (sklearn >= 0.19 step-wise definition,
 *    tie-grouped), validity flag and first-match rank from the summed
 *    counts.  ap is float64 [Q]; first_rank int32 [Q] (-1 when invalid). */
int pps_ap_finalize(int64_t Q, int Ptot, const float* sorted_d,
                    const int32_t* pos_total, const int32_t* hist,
                    const int32_t* before, double* ap, int32_t* valid,
                    int32_t* first_rank, void* stream);

/* Streaming evaluation (the product path): the same counts as 1)-2) from a
 * per-identity gallery index, with one pure stream over the distance row.
 *
 * a) pps_collect_matches: members = the shard's LOCAL gallery indices sorted
 *    by (id, index) (a CSR over identities, built once per gallery from the
 *    ids); query q's identity occupies members[q_beg[q], q_end[q]).  Lists
 *    its positives (other camera) as pps_collect_positives does, and its junk
 *    entries (same id, same camera, reid_dataset_evaluator.py:427-428) as
 *    junk_d / junk_idx [Q][Jmax] with exact counts junk_cnt -- O(matches)
 *    per query instead of a scan of G ids.
 * b) pps_rank_prepare: merge R shards' lists [R][Q][Pmax] and sort by
 *    (distance, global index) -> sorted_d / sorted_idx [Q][R*Pmax] (padding
 *    +inf / -1), pos_total [Q], and the query's bin-lookup cells
 *    [Q][pps_rank_cells()] (int32, 16-byte aligned) that c) reads.
 *    Up to R*Pmax = 8192 merged positives per query the merge sort runs in
 *    LDS (16 B per positive, 128 KiB of gfx950's 160 KiB); beyond, the
 *    query's lists are sorted in place in its sorted_d / sorted_idx row in
 *    global memory (same order; slower, for identities with thousands of
 *    gallery entries per shard).  No capacity limit (R*Pmax < 2^30).
 * c) pps_rank_count_stream: for this shard's rows, hist[q][p] += #entries
 *    with p = first positive d_p >= d, before[q] += #entries ordered before
 *    the first positive, over all entries of the row minus this shard's junk
 *    entries -- the same additive counts as pps_rank_counts (caller zeroes
 *    hist / before; sum over shards), then pps_ap_finalize.  Rows are read
 *    as 16-byte vectors when 16-byte aligned (ldd % 4 == 0).  No capacity
 *    limit on Ptot (long positive lists are searched in L2). */
int pps_collect_matches(const float* dist, int64_t Q, int64_t G, int64_t ldd,
                        const int32_t* qcam, const int32_t* gcam, const int32_t* members,
                        const int32_t* q_beg, const int32_t* q_end, int64_t g_offset,
                        int Pmax, float* pos_d, int32_t* pos_idx, int32_t* pos_cnt, int Jmax,
                        float* junk_d, int32_t* junk_idx, int32_t* junk_cnt, void* stream);
int pps_rank_cells(void);
int pps_rank_prepare(int R, int64_t Q, int Pmax, const float* pos_d, const int32_t* pos_idx,
                     const int32_t* pos_cnt, float* sorted_d, int32_t* sorted_idx,
                     int32_t* pos_total, int32_t* cells, void* stream);
int pps_rank_count_stream(const float* dist, int64_t Q, int64_t G, int64_t ldd,
                          int64_t g_offset, int Ptot, const float* sorted_d,
                          const int32_t* sorted_idx, const int32_t* pos_total,
                          const int32_t* cells, int Jmax, const float* junk_d,
                          const int32_t* junk_idx, const int32_t* junk_cnt, int32_t* hist,
                          int32_t* before, void* stream);

/* CMC beyond the Market protocol (reid_dataset_evaluator.py:283-363 `cmc`
 * with its defaults first_match_break=False, topk=100, and with
 * separate_camera_set=True).  pps_cmc_counts bins every valid entry of this
 * shard's rows by the number of positives whose (distance, global index) key
 * is below its own: hist[q][b] += 1 (b < pos_total[q]; caller zeroes hist,
 * sums over shards).  Valid = not junk (junk lists of pps_collect_matches),
 * or with qcam / gcam given (separate_camera_set; gcam = this shard's LOCAL
 * cams) = not from the query's camera.  pps_cmc_finalize then writes the
 * reference's per-query CMC row after its cumsum, ret [Q][topk] float64
 * (the j-th positive at valid position k adds 1/P at k - j, or 1 once with
 * first_match_break), and valid [Q].  Exact under the stable (distance,
 * index) order. */
int pps_cmc_counts(const float* dist, int64_t Q, int64_t G, int64_t ldd, int64_t g_offset,
                   int Ptot, const float* sorted_d, const int32_t* sorted_idx,
                   const int32_t* pos_total, const int32_t* qcam, const int32_t* gcam,
                   int Jmax, const float* junk_d, const int32_t* junk_idx,
                   const int32_t* junk_cnt, int32_t* hist, void* stream);
int pps_cmc_finalize(int64_t Q, int Ptot, const int32_t* pos_total, const int32_t* hist,
                     int topk, int first_match_break, double* ret, int32_t* valid,
                     void* stream);

/* CMC with single_gallery_shot=True (reid_dataset_evaluator.py:334-346,
 * `_unique_sample` :275-280).  Identities are dense (gid in [0, U); qid in
 * [0, U) or -1 when absent from the gallery).  The random draws stay with the
 * caller's NumPy RNG; these three steps do the rest on the device:
 *  - pps_sgs_keys: keys [Q][G] = gid of the p-th entry of order (the stable
 *    rank list of pps_argsort_rows, [Q][ldo]) when it is valid for the query
 *    (different identity or camera; with separate_camera_set also a different
 *    camera), else U;
 *  - pps_argsort_rows(keys, .., perm, vals=sorted keys): the caller's;
 *  - pps_sgs_groups: per query the identities' groups of perm in the order
 *    the reference's `ids_dict` meets them (by first ranked position):
 *    gstart / glen [Q][U] (entries t < nids[q]), nids [Q], qt [Q] = the
 *    query identity's group (-1: no valid entry of it, the query is skipped);
 *  - (caller) draws [nr][repeat][ldd], draws[i][r][t] in [0, glen[q][t]) for
 *    the listed queries rows[i] -- np.random.randint(0, tile(glen, repeat))
 *    is the reference's np.random.choice stream, call for call;
 *  - pps_sgs_ranks: k [nr][repeat] = the number of drawn entries ranked
 *    before the query identity's draw (the reference's one hit per repeat).
 * G <= pps_argsort_rows_cap(), U <= 16384, 8 U + 8 ceil(G / 32) <= 160 KiB. */
int pps_sgs_keys(const int32_t* order, int64_t Q, int64_t G, int64_t ldo, const int32_t* gid,
                 const int32_t* gcam, const int32_t* qid, const int32_t* qcam,
                 int separate_camera_set, int U, float* keys, void* stream);
int pps_sgs_groups(const float* sorted_keys, const int32_t* perm, int64_t Q, int64_t G, int U,
                   const int32_t* qid, int32_t* gstart, int32_t* glen, int32_t* nids,
                   int32_t* qt, void* stream);
int pps_sgs_ranks(const int32_t* perm, int64_t Q, int64_t G, const int32_t* rows, int64_t nr,
                  const int32_t* gstart, const int32_t* glen, const int32_t* nids,
                  const int32_t* qt, int U, int repeat, const int32_t* draws, int64_t ldd,
                  int32_t* k, void* stream);

/* The whole rank list: idx [Q][ldi] int32, row q = every gallery column in
 * (distance, index) order -- np.argsort(distmat, axis=1, kind='stable'), the
 * reference's `indices = np.argsort(distmat, axis=1)`
 * (reid_dataset_evaluator.py:319,420) with ties in index order; vals
 * (optional, [Q][ldv]) the sorted distances.  One row per workgroup:
 * rows up to 18,432 columns sorted in LDS in one pass (equalised bucket map
 * of the row's own range, one sorting network per bucket), longer rows in
 * segments of <= 7,168 words cut by exact word ranges.  G <=
 * pps_argsort_rows_cap() (458,752), else PPS_ERR_INVALID_ARG. */
int pps_argsort_rows(const float* dist, int64_t Q, int64_t G, int64_t ldd, int32_t* idx,
                     int64_t ldi, float* vals, int64_t ldv, void* stream);
int pps_argsort_rows_cap(void);
/* Stable per-row top-k (k <= 1024) of a distance matrix, ascending, ties by
 * gallery index.  Replaces the `np.argsort(distmat, axis=1)[:, :k]` rank
 * list (reid_dataset_evaluator.py:319,420). */
int pps_topk(const float* dist, int64_t Q, int64_t G, int64_t ldd, int k,
             float* vals, int32_t* idx, void* stream);

/* Global rank list of a gallery-sharded search (per-shard
 * stable top-k, all-gather of Q*k*8 B, k-way merge).  vals / idx are R lists
 * [R][Q][k_in] as pps_topk writes them (ascending, ties by index; LOCAL
 * indices, idx < 0 marks a pad entry), list r's global offset
 * list_offsets[r] (HOST array); out_vals / out_idx [Q][k_out] = the stable
 * (distance, global index) top-k_out of the union, padded with (+inf, -1)
 * when it holds fewer entries.  Equals pps_topk over the concatenated
 * shards.  R <= 64, R * k_in <= 8192. */
int pps_topk_merge(const float* vals, const int32_t* idx, int R, int64_t Q, int k_in,
                   const int64_t* list_offsets, int k_out, float* out_vals,
                   int32_t* out_idx, void* stream);

/* k-reciprocal re-ranking (reid_dataset_evaluator.py:442-519): out [Q][G] =
 * re_ranking(q_g, q_q, g_g, k1, k2, lambda) with the reference's float32
 * operand order for V, V_qe and the Jaccard sums; ties in the initial rank use
 * the stable (distance, index) order.  q_g [Q][G], q_q [Q][Q], g_g [G][G]
 * (euclidean distances, as compute_dist returns them).  Workspace: a caller
 * device buffer of pps_rerank_workspace_bytes(Q, G, k1, k2) bytes
 * (dominated by the dense N x N normalised distance, N = Q + G; G <= 38400). */
int64_t pps_rerank_workspace_bytes(int64_t Q, int64_t G, int k1, int k2);
int pps_re_ranking(const float* q_g, const float* q_q, const float* g_g, int64_t Q,
                   int64_t G, int k1, int k2, double lambda_value, void* workspace,
                   int64_t ws_bytes, float* out, void* stream);
/* The same with flags.  PPS_RERANK_SYMMETRIC: the caller guarantees q_q and
 * g_g are exactly symmetric (q_q[a][b] == q_q[b][a] bit for bit -- e.g. both
 * from the mirrored self-distance GEMM, pps_distmat_x3_self), so the N x N
 * matrix is built from M's rows and only its q_g^T block is transposed.  Same
 * result as pps_re_ranking on such inputs. */
#define PPS_RERANK_SYMMETRIC 1
int pps_re_ranking_flags(const float* q_g, const float* q_q, const float* g_g, int64_t Q,
                         int64_t G, int k1, int k2, double lambda_value, int flags,
                         void* workspace, int64_t ws_bytes, float* out, void* stream);
/* The same with row strides (e.g. the 16-byte-aligned rows of padded
 * distance buffers).  With PPS_RERANK_SYMMETRIC, N = Q + G >= 16384 and
 * every block's rows 16-byte aligned (ld % 4 == 0; ld_qq >= Q rounded up to
 * 4), the N x N normalised distance is never built: its top-k (the
 * wave-streaming kernel), the V weights and the Jaccard blend read the
 * blocks in place and compute M[i][j]^2 / colmax[i] on the fly (the same
 * float32 operations); only q_g^T is materialised (in the workspace).
 * Results equal the dense path's bit for bit. */
/* PPS_RERANK_WHOLE (with PPS_RERANK_SYMMETRIC, pps_re_ranking_ld): the three
 * blocks are views of ONE exactly symmetric N x N matrix [[q_q, q_g],
 * [q_g^T, g_g]] with one row stride (q_g = q_q + Q, g_g = q_q + Q * ld + Q;
 * e.g. the mirrored self-distance of the concatenated [queries; gallery]
 * features): q_g^T is read from its lower-left block, not transposed. */
/* Workspace bytes of one pps_re_ranking_ld call with these blocks and flags:
 * the in-place path (see above) reserves only q_g^T -- nothing with
 * PPS_RERANK_WHOLE -- plus N ints of top-k scratch instead of the N x N
 * normalised distance; calls that take the dense path get the dense size
 * (= pps_rerank_workspace_bytes).  A call handed fewer bytes than its path
 * needs fails with PPS_ERR_CAPACITY. */
int64_t pps_rerank_workspace_bytes_ld(const float* q_g, int64_t ld_qg, const float* q_q,
                                      int64_t ld_qq, const float* g_g, int64_t ld_gg, int64_t Q,
                                      int64_t G, int k1, int k2, int flags);
#define PPS_RERANK_WHOLE 2
int pps_re_ranking_ld(const float* q_g, int64_t ld_qg, const float* q_q, int64_t ld_qq,
                      const float* g_g, int64_t ld_gg, int64_t Q, int64_t G, int k1, int k2,
                      double lambda_value, int flags, void* workspace, int64_t ws_bytes,
                      float* out, void* stream);

/* ---- feature extractor ----------------------------------------------------
 * Implicit-GEMM convolution + test-mode SpatialBN + optional residual Sum +
 * optional ReLU, fused (ResNet.py:246-256 stem conv, :276-333 bottleneck,
 * :203-220 shortcut; detector.py:82-84,419-447 ConvAffine; reid_heads.py
 * :42-76 head conv+bias+BN+ReLU via shift).
 * y[p, co] = act(acc[p, co] * scale[co] + shift[co] (+ res[p, co])).
 * x NHWC [N][H][W][ldx] (Cin valid channels, Cin % 4 == 0),
 * w [Cout][Kpad], Kpad % 16 == 0, Kpad >= KH*KW*Cin,
 * y NHWC [N][Ho][Wo][ldy] written at column offset 0. */
int pps_conv2d_bn_act(const float* x, int N, int H, int W, int Cin, int ldx,
                      const float* w, int Cout, int Kpad, int KH, int KW,
                      int stride, int pad, int dil, const float* scale,
                      const float* shift, const float* residual, int relu,
                      float* y, int Ho, int Wo, int ldy, int tile,
                      void* stream);

/* Fused bottleneck tail with projection shortcut (first block of a stage):
 * y = relu?(conv_KHxKW(x; W1') + conv_1x1_stride2(x2; W2') + shift), where the
 * BN scales are pre-multiplied into W1' (branch2c) and W2' (branch1) and
 * shift = shift_2c + shift_1; i.e. ResNet.py:186-195 Sum + Relu of
 * bottleneck branch2c (:320-332) and basic_bn_shortcut (:203-220) as ONE
 * implicit GEMM over the concatenated K (no shortcut tensor in HBM).
 * w [Cout][Kpad1 + Kpad2]; x2 NHWC [N][H2][W2][ldx2], Kpad2 == Cin2 % 16 == 0. */
int pps_conv2d_dual_bn_act(const float* x, int N, int H, int W, int Cin,
                           int ldx, int KH, int KW, int stride, int pad,
                           const float* x2, int H2, int W2, int Cin2, int ldx2,
                           int stride2, const float* w, int Cout, int Kpad1,
                           int Kpad2, const float* shift, int relu, float* y,
                           int Ho, int Wo, int ldy, int tile, void* stream);

/* Batched variant for the 31 PPS head convs (reid_heads.py:42-79):
 * for b in [0,B): Y[:, b*Cout:(b+1)*Cout] = relu?(X_b W_b^T * scale_b +
 * shift_b); X_b = x + b*x_bstride ([M][K]), W_b = w + b*w_bstride
 * ([Cout][K]), scale/shift + b*Cout, Y row stride ldy. */
int pps_gemm_bn_act_batched(const float* x, int64_t x_bstride, int M, int K,
                            const float* w, int64_t w_bstride, int Cout,
                            const float* scale, const float* shift, int relu,
                            float* y, int ldy, int B, int tile, void* stream);

/* Split-K form of the batched head GEMM: raw partial products
 * part[s][m][b*Cout + c] = sum_{k in slice s} X_b[m][k] W_b[c][k] for the
 * `splitk` equal K slices (K % (16*splitk) == 0); x [B][M][K], w [B][Cout][K],
 * part [splitk][M][B*Cout].  Fills the chip at small batch (M = images). */
int pps_gemm_splitk_batched(const float* x, int M, int K, const float* w, int Cout,
                            int B, int splitk, float* part, int tile, void* stream);
/* ---- f32 GEMMs on bf16 matrix cores ("x3") --------------------------------
 * Same operations as pps_conv2d_bn_act / pps_conv2d_dual_bn_act /
 * pps_gemm_splitk_batched, with the weights pre-split by pps_split_bf16x3
 * into three bf16 planes (w = hi + mid + lo exactly) and the activations
 * split the same way on the fly; products are summed from the six terms
 * above 2^-24 relative weight on v_mfma_f32_32x32x16_bf16, so results carry
 * f32-level error (not bf16) at 2.67x the f32-MFMA peak.  Identical bits for
 * every tile; not bit-identical to the exact-f32 kernels (different
 * rounding sequence).  Weight layouts: conv [3][Cout][Kpad], dual
 * [3][Cout][Kpad1+Kpad2], split-K [B][3][Cout][K]. */
int pps_split_bf16x3(const float* x, int64_t n, int nbatch, uint16_t* out,
                     void* stream); /* x [nbatch][n] -> out [nbatch][3][n] */
int pps_conv2d_bn_act_x3(const float* x, int N, int H, int W, int Cin, int ldx,
                         const uint16_t* w3, int Cout, int Kpad, int KH, int KW,
                         int stride, int pad, int dil, const float* scale,
                         const float* shift, const float* residual, int relu,
                         float* y, int Ho, int Wo, int ldy, int tile,
                         void* stream);
/* pps_conv2d_bn_act_x3 with bf16x3 ACTIVATION planes on either side
 * (pipelined tiles only: tile 0 or >= 29).  Exactly one of x (f32 NHWC) /
 * x3 (planes [3][N][H][W][ldx], plane stride x_plane elements) and one of
 * y / y3 (planes [3][N][Ho][Wo][ldy], stride y_plane) is non-null.  A
 * producer writes y = hi + mid + lo split exactly as the x3 GEMMs split an
 * f32 operand, so a consumer reading x3 computes the same bits as from the
 * f32 tensor while skipping the split in its K loop.  Used between the
 * bottleneck convs branch2a -> 2b -> 2c (ResNet.py:276-333), whose
 * intermediates have no other reader.  Needs Cin % 32 == 0, ldx % 8 == 0,
 * Cout % 4 == 0, 16-byte aligned planes. */
int pps_conv2d_bn_act_x3p(const float* x, const uint16_t* x3, int64_t x_plane,
                          int N, int H, int W, int Cin, int ldx,
                          const uint16_t* w3, int Cout, int Kpad, int KH, int KW,
                          int stride, int pad, int dil, const float* scale,
                          const float* shift, const float* residual, int relu,
                          float* y, uint16_t* y3, int64_t y_plane, int Ho,
                          int Wo, int ldy, int tile, void* stream);
/* pps_conv2d_bn_act_x3p with split-K: the K = KH*KW*Cin reduction is cut
 * into `splitk` slices (whole 32-wide chunks, Kpad % (32*splitk) == 0) that
 * run as separate workgroups writing raw partial sums part
 * [splitk][N*Ho*Wo][Cout] (caller-owned), then one pass sums them in slice
 * order and applies scale/shift [+ residual] [ReLU] to y (f32) or y3
 * (planes).  For layers whose output tiles alone under-fill the 256 CUs
 * (res4 at batch 64: 12288 x 256).  A separate rounding group (the slices
 * are summed at the end), same f32-level error. */
int pps_conv2d_bn_act_x3p_splitk(const float* x, const uint16_t* x3, int64_t x_plane,
                                 int N, int H, int W, int Cin, int ldx,
                                 const uint16_t* w3, int Cout, int Kpad, int KH,
                                 int KW, int stride, int pad, int dil,
                                 const float* scale, const float* shift,
                                 const float* residual, int relu, float* y,
                                 uint16_t* y3, int64_t y_plane, int Ho, int Wo,
                                 int ldy, int splitk, float* part, int tile,
                                 void* stream);
/* The same split-K in ONE launch (no summing pass): each slice parks its
 * raw partial tile in part [splitk][N*Ho*Wo][Cout] and bumps a per-tile
 * arrival counter; the last slice of a tile to arrive sums the partials in
 * slice order and applies the epilogue -- the bits of
 * pps_conv2d_bn_act_x3p_splitk at the same tile id (tile 0 means tile 45
 * in both entries, so the defaults agree too).  counters: n_counters >= output tiles of
 * the tile shape, all zero on entry, zero again on return (so a captured
 * graph may replay it).  ReLU epilogues only (+ residual with f32 y, or
 * y3 planes); tiles 45 / 47 / 48 / 49 / 50, PPS_TILE_B_TILED allowed.
 * Same layer as pps_conv2d_bn_act_x3p: a bottleneck conv + AffineChannel
 * [+ Sum] + Relu (ResNet.py:276-333). */
int pps_conv2d_bn_act_x3p_splitk_fused(const float* x, const uint16_t* x3, int64_t x_plane,
                                       int N, int H, int W, int Cin, int ldx,
                                       const uint16_t* w3, int Cout, int Kpad, int KH,
                                       int KW, int stride, int pad, int dil,
                                       const float* scale, const float* shift,
                                       const float* residual, int relu, float* y,
                                       uint16_t* y3, int64_t y_plane, int Ho, int Wo,
                                       int ldy, int splitk, float* part, int* counters,
                                       int64_t n_counters, int tile, void* stream);
/* The bottleneck seam (ResNet.py:276-333): branch2c of an identity block and
 * branch2a of the next block in one launch, for the 1x1 stride-1 shapes of
 * res2 / res3, (K1, N1, N2) = (64, 256, 64) or (128, 512, 128):
 *   trunk [M][N1] = relu(x [M][K1] . w2c^T * scale2c + shift2c + residual)
 *   y     [M][N2] = relu(trunk . w2a^T * scale2a + shift2a)
 * w2c / w2a: bf16x3 planes [3][N1][K1] / [3][N2][N1] (pps_split_bf16x3 of
 * the packed weights).  trunk is written (the next block's shortcut) but
 * not read back.  Both outputs equal two pps_conv2d_bn_act_x3p calls on a
 * 16x16x32-block tile (ids 38-55) bit for bit. */
int pps_conv1x1_seam_x3(const float* x, int64_t M, int K1, const uint16_t* w2c, int N1,
                        const float* scale2c, const float* shift2c, const float* residual,
                        float* trunk, const uint16_t* w2a, int N2, const float* scale2a,
                        const float* shift2a, float* y, void* stream);
int pps_conv2d_dual_bn_act_x3(const float* x, int N, int H, int W, int Cin,
                              int ldx, int KH, int KW, int stride, int pad,
                              const float* x2, int H2, int W2, int Cin2,
                              int ldx2, int stride2, const uint16_t* w3,
                              int Cout, int Kpad1, int Kpad2, const float* shift,
                              int relu, float* y, int Ho, int Wo, int ldy,
                              int tile, void* stream);
int pps_gemm_splitk_batched_x3(const float* x, int M, int K, const uint16_t* w3,
                               int Cout, int B, int splitk, float* part,
                               int tile, void* stream);

/* y[m][j] = relu?(sum_s part[s][m][j] * scale[j] + shift[j]) (fixed order),
 * then, if normalize, Caffe2 Normalize along axis 1: y[m] /= max(|y[m]|,1e-12)
 * (reid_heads.py:58-76 BN + Relu, :96-127 Concat + Normalize). */
int pps_splitk_bn_act_normalize(const float* part, int splitk, int M, int N,
                                const float* scale, const float* shift, int relu,
                                int normalize, float* y, void* stream);

/* Fused ResNet stem (ResNet.py:246-256 basic_bn_stem): conv1 7x7/2 pad 3
 * (3 -> 64 channels) + test-mode BN (scale/shift) + ReLU + MaxPool 3x3/2 pad
 * 1 in one kernel, the conv output kept on chip.  x NHWC4 [N][H][128][4]
 * (BGR + zero, as pps_preprocess_bgr writes it); w3 = pps_split_bf16x3 of
 * the [64][pps_stem_k()] weight (K index (kh*3 + c)*8 + kw, kw = 7 and the
 * tail zero); y NHWC [N][Hp][32][64].  f32 products as six bf16 MFMA terms
 * (the "x3" arithmetic).  W must be 128. */
int pps_stem_k(void);
/* Stem kernel choice (process-wide): 0 = ring-staged input rows, whole conv
 * rows per wave, no LDS epilogue (default); 1 = whole input tile staged, LDS
 * row-buffer epilogue.  Identical bits.  Returns the previous choice; other
 * values only query. */
int pps_stem_variant(int v);
int pps_stem_conv_pool_x3(const float* x, int N, int H, int W, const uint16_t* w3,
                          const float* scale, const float* shift, float* y, int Hp, int Wp,
                          void* stream);
/* The same stem in the f16x2 arithmetic (round 6): the input split into two
 * f16 planes on the power-of-two scale of its max (amax_x: an activation-max
 * slot, PPS_AMAX_SLOT_FLOATS floats, as pps_amax fills it), the weights as
 * pps_stem_split_h2 leaves them (w2 [2][64][pps_stem_k()] f16, w_inv [64] the
 * per-channel 2^-s), three f16 MFMA terms per product; f32 accumulation. */
int pps_stem_split_h2(const float* w, uint16_t* w2, float* w_inv, void* stream);
int pps_stem_conv_pool_h2(const float* x, int N, int H, int W, const uint16_t* w2,
                          const float* w_inv, const float* amax_x, const float* scale,
                          const float* shift, float* y, int Hp, int Wp, void* stream);

/* The last res5 conv with the part pooling fused into its epilogue
 * (ResNet.py:276-333 res5_2 branch2c + Sum + Relu feeding bpm_heads.py:18-55
 * and pps_heads.py:38-80): conv + BN (scale/shift) + residual + ReLU on a
 * pipelined bf16x3 tile whose rows are exactly one image (Ho*Wo rows, <= 256
 * columns, the 192x256 tile pooling in two column passes; pps_x3p_tile_shape tells a tile's rows/columns); every tile pools
 * its image's S horizontal strips (heights `splits`, average and max) and
 * writes the 2^S - 1 part subsets to pps_out [2^S - 1][N][Cout] with
 * pps_part_power_set's arithmetic (same bits).  Exactly one of x (f32 NHWC)
 * or x3 (bf16x3 activation planes, x_plane apart) is given; y (the conv
 * output, NHWC) may be NULL and is then not written.  tile 0 = default. */
int pps_conv2d_bn_act_pps_x3p(const float* x, const uint16_t* x3, int64_t x_plane, int N,
                              int H, int W, int Cin, int ldx, const uint16_t* w3, int Cout,
                              int Kpad, int KH, int KW, int stride, int pad, int dil,
                              const float* scale, const float* shift, const float* residual,
                              float* y, int Ho, int Wo, const int32_t* splits, int S,
                              int max_ave, float* pps_out, int tile, void* stream);
/* Rows and columns of the tile a pipelined GEMM id launches (0 if none);
 * planes != 0: with bf16x3-plane activations. */
int pps_x3p_tile_shape(int tile, int planes, int* rows, int* cols);

/* MaxPool kernel k, stride s, pad p (padding never wins), NHWC
 * (ResNet.py:255 `pool1`). */
int pps_maxpool2d(const float* x, int N, int H, int W, int C, int k,
                  int stride, int pad, float* y, int Ho, int Wo,
                  void* stream);

/* Part power set (bpm_heads.py:18-55 + pps_heads.py:38-80): split H into
 * `nstrip` strips of heights `splits` (HOST array), global ave + max pool per
 * strip, then for every non-empty subset i = 1..2^S-1 (bit j => strip j):
 * out[i-1][n][c] = mean_{j in i}(ave_j) + max_{j in i}(max_j)
 * (max_ave = 1) or max_{j in i}(ave_j) (max_ave = 0, reference :70-76).
 * x NHWC [N][H][W][C]; out [2^S-1][N][C]. */
int pps_part_power_set(const float* x, int N, int H, int W, int C,
                       const int32_t* splits, int nstrip, int max_ave,
                       float* out, void* stream);

/* Caffe2 `Normalize` along axis 1 (triplet_loss.py:17-19):
 * y = x / max(||x||_2, 1e-12).  x, y [N][D] (may alias). */
int pps_l2_normalize(const float* x, int64_t N, int D, float* y,
                     void* stream);

/* Multi-query pooling (reid_dataset_evaluator.py:132-143, pool_type
 * 'average'): out[g][:] = mean of x[members[offsets[g]..offsets[g+1])][:],
 * summed in member order (device arrays; every group non-empty). */
int pps_group_mean(const float* x, int D, const int32_t* offsets,
                   const int32_t* members, int ngroups, float* out, void* stream);

/* ---- unfused Caffe2 operators (op-by-op net execution) --------------------
 * The product forward runs the recorded test net compiled into fused GEMM
 * epilogues; these stand-alone forms back the operator registry's eager
 * mode (pps_amd/net.py) for the remaining op names of the graph.
 * pps_spatial_bn: Caffe2 SpatialBN, is_test (detector.py:419-447,
 *   ResNet.py:252-253): y = (x - rm[c]) * (s[c] / sqrt(riv[c] + eps)) + b[c]
 *   (+ ReLU if relu) over NHWC [M][C].
 * pps_eltwise: n-ary elementwise over n floats, inputs = HOST array of k
 *   device pointers (k <= 32): op 0 = Sum / Add (input order), 1 = Max,
 *   2 = Mean (Sum * (1/k), pps_heads.py:58-68), 3 = Relu (k = 1).
 * pps_global_pool: AveragePool / MaxPool with global_pooling
 *   (bpm_heads.py:50-53): x image n at x + n*n_stride holds H*W*C values
 *   (a Split strip is such a view); mode 0 = mean, 1 = max; y [N][C]. */
int pps_spatial_bn(const float* x, int64_t M, int C, const float* s, const float* b,
                   const float* rm, const float* riv, float eps, int relu, float* y,
                   void* stream);
int pps_eltwise(const float* const* inputs, int k, int64_t n, int op, float* y,
                void* stream);
int pps_global_pool(const float* x, int N, int H, int W, int C, int64_t n_stride,
                    int mode, float* y, void* stream);

/* Image preprocessing (utils/blob.py:97-117 prep_im_for_blob,
 * :65-94 im_list_to_blob): uint8 BGR HWC images [N][Hi][Wi][3] (device) ->
 * subtract pixel means (HOST float[3]) -> bicubic resize (a = -0.75,
 * half-pixel centres, border replicate, as cv2.INTER_CUBIC) to Ho x Wo ->
 * NHWC float32 with 4 channels (4th = 0), the stem's packed layout. */
int pps_preprocess_bgr(const uint8_t* img, int N, int Hi, int Wi,
                       const float* pixel_means, int Ho, int Wo, float* y,
                       void* stream);
/* Same for a ragged batch of images of different sizes packed in one device
 * blob: image n starts at byte offsets[n] and is heights[n] x widths[n] x 3
 * (offsets / heights / widths are DEVICE arrays). */
int pps_preprocess_bgr_ragged(const uint8_t* blob, int N, const int64_t* offsets,
                              const int32_t* heights, const int32_t* widths,
                              const float* pixel_means, int Ho, int Wo, float* y,
                              void* stream);

/* ---- whole network ---------------------------------------------------------
 * The PPS test net as one handle (SURVEY §8(b) "pps_forward + model
 * create/destroy from a weights blob map").  Replaces the reference's
 * `workspace.RunNet(model.net.Proto().name)` of the test net, fed with the
 * `data` blob and fetching `reid_feature_concat_norm`
 * (detectron/core/test.py:155-165, test_engine.py:282-315), and the
 * net build it runs (model_builder.py build_generic_reid_model: ResNet.py
 * add_ResNet50_conv5_body, pps_heads.py add_pps_part_head, reid_heads.py
 * add_reid_outputs).  The handle owns the packed / bf16x3-split weights, the
 * activation buffers per batch size and the per-layer GEMM tile, activation-
 * plane and split-K table; every launch of a forward is the op-level entry
 * point above with the same arguments pps_amd/model.py uses, so both
 * orchestrators give identical bits for the same table.
 *
 * Unlike the op-level entry points, the handle allocates device memory:
 * pps_model_create (weights) and pps_model_reserve (activations for batch N,
 * ~62 MB per image at 384x128).  pps_forward itself never allocates or
 * synchronises once N is reserved, so it can be captured into a hipGraph.
 * One forward at a time per handle (the activation buffers are shared); use
 * one handle per concurrent stream. */
#define PPS_MATH_X3 0   /* f32 products as six bf16 MFMA terms (default)   */
#define PPS_MATH_F32 1  /* exact f32 MFMA (v_mfma_f32_32x32x2_f32)         */
#define PPS_AUTOTUNE_NO_PLANES 1  /* keep the plane edges as they are     */
#define PPS_AUTOTUNE_SPLITK 2     /* also try conv split-K 2..4           */
#define PPS_AUTOTUNE_NO_SEAM 4    /* do not try PPS_TILE_SEAM pairs       */
#define PPS_AUTOTUNE_NO_H2 8      /* do not try PPS_TILE_H2 (f16x2) tiles */
#define PPS_AUTOTUNE_NO_H2E 16    /* do not try PPS_TILE_H2E planes edges */
#define PPS_AUTOTUNE_NO_GROUPS 32 /* skip the in-forward pass over layers of
                                     one shape (each layer keeps its own pick) */

typedef struct PpsBlob {     /* one Detectron blob, HOST float32 memory   */
  const char* name;          /* e.g. "res2_0_branch2a_w", "pps01_bn_riv"  */
  const float* data;
  int ndim;
  int64_t shape[4];
} PpsBlob;

typedef struct PpsModelConfig {  /* reference cfg keys (core/config.py)   */
  int struct_size;               /* = sizeof(PpsModelConfig)               */
  int height, width;             /* REID.SCALE[1], REID.SCALE[0]: 384, 128 */
  int strip_num;                 /* REID.BPM_STRIP_NUM                     */
  int bpm_dim;                   /* REID.BPM_DIM                           */
  int num_groups, width_per_group, stride_1x1; /* RESNETS.*               */
  int res5_stride, res5_dilation;
  int fpn_on, fpn_dim;           /* FPN.FPN_ON, FPN.DIM                    */
  int max_ave;                   /* REID.MAX_AVE_FEATURE                   */
  int normalize;                 /* REID.NORMALIZE_FEATURE                 */
  int math;                      /* PPS_MATH_*                             */
  int fused_stem, fused_pps, act_planes;  /* x3 fusions (1 = on)          */
  float pixel_means[3];          /* PIXEL_MEANS (BGR), pps_forward_bgr     */
} PpsModelConfig;

typedef struct PpsLayerInfo {
  const char* name;   /* tuning key: conv name, or the output blob        */
  const char* op;     /* conv, conv_dual, stem_pool, conv_pps, heads, ...  */
  int tile, splitk, planes_in, planes_out;
  int gemm;           /* an MFMA launch (counted in the conv roofline)     */
  double flops;       /* algorithmic FLOP at batch N                       */
  double bytes;       /* algorithmic HBM bytes at batch N                  */
  int64_t out_shape[4];
  const char* output; /* the output blob (pps_model_tensor's name)        */
} PpsLayerInfo;

typedef struct PpsModel PpsModel;

/* The reference's PPS Market-1501 test configuration. */
int pps_model_config_default(PpsModelConfig* cfg);
/* Build the net from `nblobs` host blobs (every parameter of the test net;
 * `<prefix>_conv_b` head biases optional), fold BN, pack and split the
 * weights on the current device.  Synchronous. */
int pps_model_create(const PpsBlob* blobs, int nblobs, const PpsModelConfig* cfg,
                     PpsModel** model);
int pps_model_destroy(PpsModel* model);
int pps_model_feat_dim(const PpsModel* model);
int pps_model_num_layers(const PpsModel* model);
int pps_model_layer_info(const PpsModel* model, int layer, int N, PpsLayerInfo* info);
/* Tuning table (results do not depend on it beyond the MFMA block group, see
 * pps_gemm_num_tiles).  Autotune results of pps_model_autotune or of
 * pps_amd/model.py (tiles JSON) are applied by name. */
int pps_model_set_tile(PpsModel* model, const char* layer, int tile);
int pps_model_set_splitk(PpsModel* model, const char* layer, int splitk);
int pps_model_num_plane_edges(const PpsModel* model);
int pps_model_plane_edge(const PpsModel* model, int edge, const char** producer,
                         const char** consumer, int* on);
int pps_model_set_planes(PpsModel* model, const char* producer, int on);
/* Time every tile per layer on this device (then plane edges, optionally
 * split-K, seams, f16x2-plane edges) with x [N][H][W][4] as input; last, the
 * layers of one shape (e.g. the five res4 3x3 convs) are tried on each of
 * their members' three best tiles inside whole forwards, with their f16x2-plane
 * edges all on and all off, and a layer of its own shape on its three best
 * variants, so the pick holds where the layer actually runs (isolated
 * repeats of one launch can rank near-equal tiles differently).  Not
 * capturable. */
int pps_model_autotune(PpsModel* model, const float* x, int N, int flags, void* stream);
/* Allocate (synchronously) the activation buffers for batch N and pin them:
 * from here on they are never reallocated, so a hipGraph captured around
 * pps_forward stays valid.  A later pps_model_set_splitk / set_tile /
 * autotune that would need larger split-K buffers for batch N fails with
 * PPS_ERR instead of freeing memory a captured graph still addresses:
 * pps_model_release(N), pps_model_reserve(N) and recapture. */
int pps_model_reserve(PpsModel* model, int N);
int pps_model_release(PpsModel* model, int N);   /* N <= 0: all */
/* An intermediate tensor of the last forward at batch N (debug / parity):
 * device pointer, planes flag (bf16x3 [3][...]) and its 4-D shape. */
int pps_model_tensor(const PpsModel* model, int N, const char* blob, void** ptr,
                     int* planes, int64_t* shape4);
/* (*planes == 2: f16x2 planes [2][...] of the PPS_TILE_H2E edge, on the
 * power-of-two scale of the bound pps_model_tensor_amax reports.) */
/* The activation max max|t| its producer reported for tensor `blob` in the
 * last forward at batch N (the f16x2 layers' input scales; debug / parity),
 * copied to *out (HOST).  Synchronous. */
int pps_model_tensor_amax(const PpsModel* model, int N, const char* blob, float* out);
/* feat [N][feat_dim] = reid_feature_concat_norm of x NHWC4 [N][H][W][4]
 * (pps_preprocess_bgr's layout: BGR minus PIXEL_MEANS, 4th channel 0). */
int pps_forward(const PpsModel* model, const float* nhwc4, int N, float* feat,
                void* stream);
/* Layers [first, last) only (per-layer timing); the intermediates persist
 * in the handle, the last layer writes feat.  With first > 0 the activation
 * maxima of the tensors the range reads but does not produce are measured
 * afresh (pps_amax) before it runs. */
int pps_forward_layers(const PpsModel* model, const float* nhwc4, int N, float* feat,
                       int first, int last, void* stream);
/* The same with flags.  PPS_FWD_KEEP_AMAX: the activation maxima are kept as
 * the previous call left them (no re-measure, no reset) -- for timing a range
 * whose inputs have not changed since the forward that reported them. */
#define PPS_FWD_KEEP_AMAX 1
int pps_forward_layers_flags(const PpsModel* model, const float* nhwc4, int N, float* feat,
                             int first, int last, int flags, void* stream);
/* The reference's `data` blob as it is: NCHW [N][3][H][W] float32. */
int pps_forward_nchw(const PpsModel* model, const float* nchw, int N, float* feat,
                     void* stream);
/* uint8 BGR images [N][Hi][Wi][3] (device) -> preprocess -> forward. */
int pps_forward_bgr(const PpsModel* model, const uint8_t* img, int N, int Hi, int Wi,
                    float* feat, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PPS_ABI_H_ */
