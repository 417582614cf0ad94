// extern "C" entry points of libpps_hip.so (declared in include/pps_abi.h).
// Each entry point validates shapes/alignment ENFORCE-style, fills the
// launch parameters and enqueues on the caller's stream.  No allocation, no
// synchronisation: every entry point is hipGraph-capturable.
#include <algorithm>
#include <cstdlib>
#include <string>

#include "pps_internal.hpp"

namespace pps {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
bool debug_sync() {
  static const bool on = [] {
    const char* e = getenv("PPS_DEBUG_SYNC");
    return e && e[0] == '1';
  }();
  return on;
}

int part_power_set(const float*, int, int, int, int, const int32_t*, int, int, float*,
                   hipStream_t);
int l2_normalize(const float*, int64_t, int, float*, hipStream_t);
int group_mean(const float*, int, const int32_t*, const int32_t*, int, float*, hipStream_t);
int collect_positives(const float*, int64_t, int64_t, int64_t, const int32_t*,
                      const int32_t*, const int32_t*, const int32_t*, int64_t, int, float*,
                      int32_t*, int32_t*, hipStream_t);
int rank_counts(const float*, int64_t, int64_t, int64_t, const int32_t*, const int32_t*,
                const int32_t*, const int32_t*, int64_t, int, int, const float*,
                const int32_t*, const int32_t*, float*, int32_t*, int32_t*, int32_t*,
                int32_t*, hipStream_t);
int ap_finalize(int64_t, int, const float*, const int32_t*, const int32_t*,
                const int32_t*, double*, int32_t*, int32_t*, hipStream_t);
int topk(const float*, int64_t, int64_t, int64_t, int, float*, int32_t*, hipStream_t);
int argsort_rows(const float*, int64_t, int64_t, int64_t, int32_t*, int64_t, float*, int64_t,
                 hipStream_t);
int argsort_rows_cap();
int sgs_keys(const int32_t*, int64_t, int64_t, int64_t, const int32_t*, const int32_t*,
             const int32_t*, const int32_t*, int, int, float*, hipStream_t);
int sgs_groups(const float*, const int32_t*, int64_t, int64_t, int, const int32_t*, int32_t*,
               int32_t*, int32_t*, int32_t*, hipStream_t);
int sgs_ranks(const int32_t*, int64_t, const int32_t*, int64_t, const int32_t*, const int32_t*,
              const int32_t*, const int32_t*, int, int, const int32_t*, int64_t, int32_t*,
              hipStream_t);
size_t sgs_groups_lds_bytes(int64_t, int);
int cmc_counts(const float*, int64_t, int64_t, int64_t, int64_t, int, const float*,
               const int32_t*, const int32_t*, const int32_t*, const int32_t*, int,
               const float*, const int32_t*, const int32_t*, int32_t*, hipStream_t);
int cmc_finalize(int64_t, int, const int32_t*, const int32_t*, int, int, double*, int32_t*,
                 hipStream_t);
int collect_matches(const float*, int64_t, int64_t, const int32_t*, const int32_t*,
                    const int32_t*, const int32_t*, const int32_t*, int64_t, int, float*,
                    int32_t*, int32_t*, int, float*, int32_t*, int32_t*, hipStream_t);
int rank_prepare(int, int64_t, int, const float*, const int32_t*, const int32_t*, float*,
                 int32_t*, int32_t*, int32_t*, hipStream_t);
int rank_count_stream(const float*, int64_t, int64_t, int64_t, int64_t, int, const float*,
                      const int32_t*, const int32_t*, const int32_t*, int, const float*,
                      const int32_t*, const int32_t*, int32_t*, int32_t*, hipStream_t);
int rerank(const float*, int64_t, const float*, int64_t, const float*, int64_t, int64_t, int64_t,
           int, int, double, void*, size_t, float*, hipStream_t, int);
size_t rerank_workspace_bytes(int64_t, int64_t, int, int);
size_t rerank_workspace_bytes_for(const float*, int64_t, const float*, int64_t, const float*,
                                  int64_t, int64_t, int64_t, int, int, int);
int splitk_bn_act_normalize(const float*, int, int64_t, int, int, const float*,
                            const float*, int, int, float*, hipStream_t);
int splitk_conv_epilogue(const float*, int, int64_t, int, const float*, const float*,
                         const float*, int, float*, uint16_t*, int64_t, hipStream_t, float*);

}  // namespace pps

using namespace pps;

extern "C" {

int pps_abi_version(void) { return 1; }

const char* pps_last_error(void) { return g_last_error.c_str(); }

const char* pps_registered_ops(void) {
  // the reference's Caffe2 op names of the test net (pps_amd/net.py OPS) and
  // the fused / retrieval entry points the product path runs
  return "Conv;SpatialBN;Relu;Sum;Add;Max;Mean;MaxPool;AveragePool;Split;FC;Concat;"
         "Reshape;Normalize;PairWiseDistance;"
         "Conv+SpatialBN+Sum+Relu;PartPowerSet;ComputeDist;RankCounts;CMC;TopK;TopKMerge;"
         "ReRanking;PrepImForBlob";
}

int pps_gemm_num_tiles(void) { return GEMM_NUM_TILES - 1; }

int pps_distmat(const float* q, int64_t Q, int64_t ldq, const float* g, int64_t G,
                int64_t ldg, int D, int metric, float* out, int64_t ldo, int tile,
                void* stream) {
  PPS_ENFORCE(q && g && out, "null pointer");
  PPS_ENFORCE(Q >= 0 && G >= 0 && D > 0, "bad shape");
  PPS_ENFORCE(D % 4 == 0, "D must be a multiple of 4, got " + std::to_string(D));
  PPS_ENFORCE(ldq % 4 == 0 && ldg % 4 == 0 && ldq >= D && ldg >= D, "bad leading dims");
  PPS_ENFORCE(ldo >= G, "ldo < G");
  PPS_ENFORCE(aligned16(q) && aligned16(g), "q/g must be 16-byte aligned");
  PPS_ENFORCE(metric >= 0 && metric <= 2, "unknown metric");
  PPS_ENFORCE(ldq * 4 < kMaxBufBytes && ldg * 4 < kMaxBufBytes, "rows too long");
  // operands are addressed through 32-bit buffer offsets: split Q and G into
  // blocks of < 2 GiB each (one launch per block pair, same results)
  const int64_t qblk = std::min<int64_t>(Q, (kMaxBufBytes - 1) / (ldq * 4));
  const int64_t gblk = std::min<int64_t>(G, (kMaxBufBytes - 1) / (ldg * 4));
  for (int64_t q0 = 0; q0 < Q; q0 += qblk) {
    for (int64_t g0 = 0; g0 < G; g0 += gblk) {
      const int64_t qn = std::min(qblk, Q - q0), gn = std::min(gblk, G - g0);
      GemmParams p{};
  p.splitk = 1;
      p.a = q + q0 * ldq; p.a_bytes = (uint32_t)(qn * ldq * 4);
      p.H = 1; p.W = (int)qn; p.Cin = D; p.lda = (int)ldq;
      p.KH = p.KW = 1; p.stride = 1; p.pad = 0; p.dil = 1; p.Ho = 1; p.Wo = (int)qn;
      p.M = (int)qn;
      p.b = g + g0 * ldg; p.b_bytes = (uint32_t)(gn * ldg * 4);
      p.ldb = (int)ldg; p.kb_valid = D; p.Ncol = (int)gn;
      p.Kloop = (D + 15) / 16 * 16;
      p.out = out + q0 * ldo + g0; p.ldo = ldo; p.metric = metric; p.tile = tile;
      const int rc = launch_gemm(p, EPI_DIST, 1, as_stream(stream));
      if (rc != PPS_OK) return rc;
    }
  }
  return PPS_OK;
}

int pps_row_sqnorm(const float* x, int64_t rows, int D, int64_t ld, float* out,
                   void* stream) {
  PPS_ENFORCE(x && out, "null pointer");
  PPS_ENFORCE(rows >= 0 && D > 0 && D % 4 == 0 && ld >= D && ld % 4 == 0, "bad shape");
  PPS_ENFORCE(aligned16(x), "x must be 16-byte aligned");
  return row_sqnorm(x, rows, D, ld, out, as_stream(stream));
}

int pps_split_bf16x3_sqnorm(const float* x, int64_t rows, int D, int64_t ld, uint16_t* out3,
                            float* sqnorm, void* stream) {
  PPS_ENFORCE(x && out3 && sqnorm, "null pointer");
  PPS_ENFORCE(rows >= 0 && D > 0 && D % 4 == 0 && ld >= D && ld % 4 == 0, "bad shape");
  PPS_ENFORCE(aligned16(x), "x must be 16-byte aligned");
  PPS_ENFORCE(((uintptr_t)out3 & 7) == 0, "out3 must be 8-byte aligned");
  return split_sqnorm(x, rows, D, ld, out3, sqnorm, as_stream(stream));
}

int pps_split_bf16x3_sqnorm_tiled(const float* x, int64_t rows, int D, int64_t ld,
                                  uint16_t* out3t, float* sqnorm, void* stream) {
  PPS_ENFORCE(x && out3t && sqnorm, "null pointer");
  PPS_ENFORCE(rows >= 0 && D > 0 && D % 32 == 0 && ld >= D && ld % 4 == 0,
              "bad shape (D % 32 == 0)");
  PPS_ENFORCE(aligned16(x), "x must be 16-byte aligned");
  PPS_ENFORCE(((uintptr_t)out3t & 7) == 0, "out3t must be 8-byte aligned");
  return split_sqnorm_tiled(x, rows, D, ld, out3t, sqnorm, as_stream(stream));
}

int pps_distmat_x3(const float* q, int64_t Q, int64_t ldq, const float* qsq,
                   const uint16_t* g3, const float* gsq, int64_t G, int64_t ldg, int D,
                   int metric, float* out, int64_t ldo, int tile, void* stream) {
  PPS_ENFORCE(q && qsq && g3 && gsq && out, "null pointer");
  PPS_ENFORCE(Q >= 0 && G >= 0 && D > 0, "bad shape");
  PPS_ENFORCE(D % 4 == 0, "D must be a multiple of 4, got " + std::to_string(D));
  PPS_ENFORCE(ldq % 4 == 0 && ldg % 4 == 0 && ldq >= D && ldg >= D, "bad leading dims");
  PPS_ENFORCE(ldo >= G, "ldo < G");
  PPS_ENFORCE(aligned16(q) && aligned16(g3), "q/g3 must be 16-byte aligned");
  PPS_ENFORCE(metric >= 0 && metric <= 2, "unknown metric");
  PPS_ENFORCE(ldq * 4 < kMaxBufBytes && ldg * 2 < kMaxBufBytes, "rows too long");
  const int64_t qblk = std::min<int64_t>(Q, (kMaxBufBytes - 1) / (ldq * 4));
  const int64_t gblk = std::min<int64_t>(G, (kMaxBufBytes - 1) / (ldg * 2));
  for (int64_t q0 = 0; q0 < Q; q0 += qblk) {
    for (int64_t g0 = 0; g0 < G; g0 += gblk) {
      const int64_t qn = std::min(qblk, Q - q0), gn = std::min(gblk, G - g0);
      GemmParams p{};
      p.splitk = 1;
      p.a = q + q0 * ldq; p.a_bytes = (uint32_t)(qn * ldq * 4);
      p.H = 1; p.W = (int)qn; p.Cin = D; p.lda = (int)ldq;
      p.KH = p.KW = 1; p.stride = 1; p.pad = 0; p.dil = 1; p.Ho = 1; p.Wo = (int)qn;
      p.M = (int)qn;
      p.b3 = g3 + g0 * ldg; p.b_plane = G * ldg; p.b_bytes = (uint32_t)(gn * ldg * 2);
      p.ldb = (int)ldg; p.kb_valid = D; p.Ncol = (int)gn;
      p.Kloop = (D + 15) / 16 * 16;
      p.norm_a = qsq + q0; p.norm_b = gsq + g0;
      p.out = out + q0 * ldo + g0; p.ldo = ldo; p.metric = metric; p.tile = tile;
      const int rc = launch_gemm_x3(p, EPI_DIST, 1, as_stream(stream));
      if (rc != PPS_OK) return rc;
    }
  }
  return PPS_OK;
}

int pps_distmat_x3p(const uint16_t* q3, int64_t Q, int64_t ldq, const float* qsq,
                    const uint16_t* g3, const float* gsq, int64_t G, int64_t ldg, int D,
                    int metric, float* out, int64_t ldo, int tile, void* stream) {
  PPS_ENFORCE(q3 && qsq && g3 && gsq && out, "null pointer");
  PPS_ENFORCE(Q >= 0 && G >= 0 && D > 0, "bad shape");
  PPS_ENFORCE(D % 32 == 0, "D must be a multiple of 32, got " + std::to_string(D));
  PPS_ENFORCE(ldq % 8 == 0 && ldg % 8 == 0 && ldq >= D && ldg >= D, "bad leading dims");
  PPS_ENFORCE(ldo >= G, "ldo < G");
  PPS_ENFORCE(aligned16(q3) && aligned16(g3), "q3/g3 must be 16-byte aligned");
  PPS_ENFORCE(metric >= 0 && metric <= 2, "unknown metric");
  PPS_ENFORCE(tile == 0 || tile >= GEMM_TILE_P_FIRST,
              "query planes need a pipelined tile (0 or >= " +
                  std::to_string((int)GEMM_TILE_P_FIRST) + ")");
  PPS_ENFORCE(ldq * 2 < kMaxBufBytes && ldg * 2 < kMaxBufBytes, "rows too long");
  const int64_t qblk = std::min<int64_t>(Q, (kMaxBufBytes - 1) / (ldq * 2));
  const int64_t gblk = std::min<int64_t>(G, (kMaxBufBytes - 1) / (ldg * 2));
  for (int64_t q0 = 0; q0 < Q; q0 += qblk) {
    for (int64_t g0 = 0; g0 < G; g0 += gblk) {
      const int64_t qn = std::min(qblk, Q - q0), gn = std::min(gblk, G - g0);
      GemmParams p{};
      p.splitk = 1;
      p.a3 = q3 + q0 * ldq; p.a_plane = Q * ldq; p.a_bytes = (uint32_t)(qn * ldq * 2);
      p.H = 1; p.W = (int)qn; p.Cin = D; p.lda = (int)ldq;
      p.KH = p.KW = 1; p.stride = 1; p.pad = 0; p.dil = 1; p.Ho = 1; p.Wo = (int)qn;
      p.M = (int)qn;
      p.b3 = g3 + g0 * ldg; p.b_plane = G * ldg; p.b_bytes = (uint32_t)(gn * ldg * 2);
      p.ldb = (int)ldg; p.kb_valid = D; p.Ncol = (int)gn;
      p.Kloop = D;
      p.norm_a = qsq + q0; p.norm_b = gsq + g0;
      p.out = out + q0 * ldo + g0; p.ldo = ldo; p.metric = metric;
      p.tile = tile ? tile : GEMM_TILE_P16_FIRST + 4;  // as pps_distmat_x3's default
      const int rc = launch_gemm_x3(p, EPI_DIST, 1, as_stream(stream));
      if (rc != PPS_OK) return rc;
    }
  }
  return PPS_OK;
}

// Both operands' planes chunk-tiled ([rows16 / 16][D / 32][16][32] per
// plane, rows padded to a multiple of 16 with zeros: pps_tile_planes).
int pps_distmat_x3p_tiled(const uint16_t* q3t, int64_t Q, const float* qsq,
                          const uint16_t* g3t, const float* gsq, int64_t G, int D, int metric,
                          float* out, int64_t ldo, int tile, void* stream) {
  PPS_ENFORCE(q3t && qsq && g3t && gsq && out, "null pointer");
  PPS_ENFORCE(Q >= 0 && G >= 0 && D > 0 && D % 32 == 0, "bad shape (D % 32 == 0)");
  PPS_ENFORCE(ldo >= G, "ldo < G");
  PPS_ENFORCE(aligned16(q3t) && aligned16(g3t), "planes must be 16-byte aligned");
  PPS_ENFORCE(metric >= 0 && metric <= 2, "unknown metric");
  PPS_ENFORCE(tile == 0 || (tile >= GEMM_TILE_P_FIRST && tile < GEMM_TILE_WS),
              "tiled planes need a pipelined tile (0 or 29..53)");
  const int64_t Qp = (Q + 15) / 16 * 16, Gp = (G + 15) / 16 * 16;
  PPS_ENFORCE(Qp * D * 2 < kMaxBufBytes && Gp * D * 2 < kMaxBufBytes, "planes over 2 GiB");
  if (Q == 0 || G == 0) return PPS_OK;
  GemmParams p{};
  p.splitk = 1;
  p.tiled = 3;
  p.a3 = q3t; p.a_plane = Qp * D; p.a_bytes = (uint32_t)(Qp * D * 2);
  p.H = 1; p.W = (int)Q; p.Cin = D; p.lda = D;
  p.KH = p.KW = 1; p.stride = 1; p.pad = 0; p.dil = 1; p.Ho = 1; p.Wo = (int)Q;
  p.M = (int)Q;
  p.b3 = g3t; p.b_plane = Gp * D; p.b_bytes = (uint32_t)(Gp * D * 2);
  p.ldb = D; p.kb_valid = D; p.Ncol = (int)G;
  p.Kloop = D;
  p.norm_a = qsq; p.norm_b = gsq;
  p.out = out; p.ldo = ldo; p.metric = metric;
  // default 128 x 256 (tile 43): Market 1.81 ms vs 2.05 on 256 x 128, Duke's
  // query x gallery the same either way (scripts/probes/dist_default_tile_probe.py)
  p.tile = tile ? tile : GEMM_TILE_P16_FIRST + 5;
  return launch_gemm_x3(p, EPI_DIST, 1, as_stream(stream));
}

int pps_distmat_x3_self(const float* x, int64_t N, int64_t ld, const float* xsq,
                        const uint16_t* x3, int D, int metric, float* out, int64_t ldo,
                        int tile, void* stream) {
  PPS_ENFORCE(x && xsq && x3 && out, "null pointer");
  PPS_ENFORCE(N >= 0 && D > 0 && D % 32 == 0, "D must be a positive multiple of 32");
  PPS_ENFORCE(ld % 8 == 0 && ld >= D, "bad leading dim");
  PPS_ENFORCE(ldo >= N, "ldo < N");
  PPS_ENFORCE(aligned16(x) && aligned16(x3), "x/x3 must be 16-byte aligned");
  PPS_ENFORCE(metric >= 0 && metric <= 2, "unknown metric");
  PPS_ENFORCE(N * ld * 4 < kMaxBufBytes, "self-distance operand larger than 2 GiB");
  PPS_ENFORCE(N * ldo < (1ll << 31), "output larger than 2^31 elements");
  GemmParams p{};
  p.splitk = 1;
  p.a = x; p.a_bytes = (uint32_t)(N * ld * 4);
  p.H = 1; p.W = (int)N; p.Cin = D; p.lda = (int)ld;
  p.KH = p.KW = 1; p.stride = 1; p.pad = 0; p.dil = 1; p.Ho = 1; p.Wo = (int)N;
  p.M = (int)N;
  p.b3 = x3; p.b_plane = N * ld; p.b_bytes = (uint32_t)(N * ld * 2);
  p.ldb = (int)ld; p.kb_valid = D; p.Ncol = (int)N;
  p.Kloop = D;
  p.norm_a = xsq; p.norm_b = xsq;
  p.out = out; p.ldo = ldo; p.metric = metric; p.sym = 1; p.tile = tile;
  return launch_gemm_x3(p, EPI_DIST, 1, as_stream(stream));
}

// The same from chunk-tiled planes (pps_split_bf16x3_sqnorm_tiled /
// pps_tile_planes layout): both operands are the one tiled copy, staged by
// pure DMA like pps_distmat_x3p_tiled.
int pps_distmat_x3_self_tiled(const uint16_t* x3t, int64_t N, const float* xsq, int D,
                              int metric, float* out, int64_t ldo, int tile, void* stream) {
  PPS_ENFORCE(x3t && xsq && out, "null pointer");
  PPS_ENFORCE(N >= 0 && D > 0 && D % 32 == 0, "D must be a positive multiple of 32");
  PPS_ENFORCE(ldo >= N, "ldo < N");
  PPS_ENFORCE(aligned16(x3t), "x3t must be 16-byte aligned");
  PPS_ENFORCE(metric >= 0 && metric <= 2, "unknown metric");
  const int64_t Np = (N + 15) / 16 * 16;
  PPS_ENFORCE(Np * D * 2 < kMaxBufBytes, "planes over 2 GiB");
  PPS_ENFORCE(N * ldo < (1ll << 31), "output larger than 2^31 elements");
  PPS_ENFORCE(tile == 0 || (tile >= GEMM_TILE_P_FIRST && tile < GEMM_TILE_C16_FIRST &&
                            tile != GEMM_TILE_WS),
              "tiled self-distance needs a pipelined tile (0, 29..53 or 55)");
  if (N == 0) return PPS_OK;
  GemmParams p{};
  p.splitk = 1;
  p.tiled = 3;
  p.a3 = x3t; p.a_plane = Np * D; p.a_bytes = (uint32_t)(Np * D * 2);
  p.H = 1; p.W = (int)N; p.Cin = D; p.lda = D;
  p.KH = p.KW = 1; p.stride = 1; p.pad = 0; p.dil = 1; p.Ho = 1; p.Wo = (int)N;
  p.M = (int)N;
  p.b3 = x3t; p.b_plane = Np * D; p.b_bytes = (uint32_t)(Np * D * 2);
  p.ldb = D; p.kb_valid = D; p.Ncol = (int)N;
  p.Kloop = D;
  p.norm_a = xsq; p.norm_b = xsq;
  p.out = out; p.ldo = ldo; p.metric = metric; p.sym = 1;
  p.tile = tile ? tile : GEMM_TILE_P16_FIRST + 5;  // 128 x 256 (the distance matrix's)
  return launch_gemm_x3(p, EPI_DIST, 1, as_stream(stream));
}

int pps_pairwise_distance(const float* X, int N, int D, float* Z, void* stream) {
  PPS_ENFORCE(X && Z, "null pointer");
  PPS_ENFORCE(N >= 0 && D > 0 && D % 4 == 0, "X must be 2-D [N][D] with D % 4 == 0");
  PPS_ENFORCE(aligned16(X), "X must be 16-byte aligned");
  GemmParams p{};
  p.splitk = 1;
  PPS_ENFORCE((int64_t)N * D * 4 < kMaxBufBytes, "X larger than 2 GiB");
  p.a = X; p.H = 1; p.W = N; p.Cin = D; p.lda = D; p.a_bytes = (uint32_t)((int64_t)N * D * 4);
  p.KH = p.KW = 1; p.stride = 1; p.dil = 1; p.Ho = 1; p.Wo = N; p.M = N;
  p.b = X; p.ldb = D; p.kb_valid = D; p.Ncol = N; p.b_bytes = p.a_bytes;
  p.Kloop = (D + 15) / 16 * 16;
  p.out = Z; p.ldo = N; p.metric = PPS_METRIC_SQEUCLIDEAN; p.zero_diag = 1;
  return launch_gemm(p, EPI_DIST, 1, as_stream(stream));
}

int pps_collect_positives(const float* dist, int64_t Q, int64_t G, int64_t ldd,
                          const int32_t* qid, const int32_t* qcam, const int32_t* gid,
                          const int32_t* gcam, int64_t g_offset, int Pmax, float* pos_d,
                          int32_t* pos_idx, int32_t* pos_cnt, void* stream) {
  PPS_ENFORCE(dist && qid && qcam && gid && gcam && pos_d && pos_idx && pos_cnt,
              "null pointer");
  PPS_ENFORCE(Q >= 0 && G >= 0 && ldd >= G && Pmax > 0, "bad shape");
  return collect_positives(dist, Q, G, ldd, qid, qcam, gid, gcam, g_offset, Pmax, pos_d,
                           pos_idx, pos_cnt, as_stream(stream));
}

int pps_rank_counts(const float* dist, int64_t Q, int64_t G, int64_t ldd,
                    const int32_t* qid, const int32_t* qcam, const int32_t* gid,
                    const int32_t* gcam, int64_t g_offset, int R, int Pmax,
                    const float* pos_d, const int32_t* pos_idx, const int32_t* pos_cnt,
                    float* sorted_d, int32_t* sorted_idx, int32_t* pos_total,
                    int32_t* hist, int32_t* before, void* stream) {
  PPS_ENFORCE(dist && qid && qcam && gid && gcam && pos_d && pos_idx && pos_cnt &&
                  sorted_d && sorted_idx && pos_total && hist && before,
              "null pointer");
  PPS_ENFORCE(Q >= 0 && G >= 0 && ldd >= G, "bad shape");
  PPS_ENFORCE(R >= 1 && R <= 64, "R must be in [1, 64]");
  if ((int64_t)R * Pmax > 2048) {
    set_error("merged positives per query R*Pmax=" + std::to_string((int64_t)R * Pmax) +
              " exceeds the LDS capacity 2048");
    return PPS_ERR_CAPACITY;
  }
  return rank_counts(dist, Q, G, ldd, qid, qcam, gid, gcam, g_offset, R, Pmax, pos_d,
                     pos_idx, pos_cnt, sorted_d, sorted_idx, pos_total, hist, before,
                     as_stream(stream));
}

int pps_collect_matches(const float* dist, int64_t Q, int64_t G, int64_t ldd,
                        const int32_t* qcam, const int32_t* gcam, const int32_t* members,
                        const int32_t* q_beg, const int32_t* q_end, int64_t g_offset,
                        int Pmax, float* pos_d, int32_t* pos_idx, int32_t* pos_cnt, int Jmax,
                        float* junk_d, int32_t* junk_idx, int32_t* junk_cnt, void* stream) {
  PPS_ENFORCE(dist && qcam && gcam && members && q_beg && q_end && pos_d && pos_idx &&
                  pos_cnt && junk_d && junk_idx && junk_cnt,
              "null pointer");
  PPS_ENFORCE(Q >= 0 && G >= 0 && ldd >= G && Pmax > 0 && Jmax > 0, "bad shape");
  PPS_ENFORCE(G < (1ll << 31) && g_offset + G < (1ll << 31), "gallery indices must fit int32");
  return collect_matches(dist, Q, ldd, qcam, gcam, members, q_beg, q_end, g_offset, Pmax,
                         pos_d, pos_idx, pos_cnt, Jmax, junk_d, junk_idx, junk_cnt,
                         as_stream(stream));
}

int pps_rank_cells(void) { return 1024; }

int pps_rank_prepare(int R, int64_t Q, int Pmax, const float* pos_d, const int32_t* pos_idx,
                     const int32_t* pos_cnt, float* sorted_d, int32_t* sorted_idx,
                     int32_t* pos_total, int32_t* cells, void* stream) {
  PPS_ENFORCE(pos_d && pos_idx && pos_cnt && sorted_d && sorted_idx && pos_total && cells,
              "null pointer");
  PPS_ENFORCE(((uintptr_t)cells & 15) == 0, "cells must be 16-byte aligned");
  PPS_ENFORCE(R >= 1 && R <= kMergeMaxLists, "R must be in [1, 64]");
  PPS_ENFORCE(Q >= 0 && Pmax > 0, "bad shape");
  // beyond kRankMergeCap merged positives the lists are sorted in place in
  // global memory (rank_prepare_global_kernel): no capacity limit
  PPS_ENFORCE((int64_t)R * Pmax < (1ll << 30), "R * Pmax must be < 2^30");
  return rank_prepare(R, Q, Pmax, pos_d, pos_idx, pos_cnt, sorted_d, sorted_idx, pos_total,
                      cells, as_stream(stream));
}

int pps_rank_count_stream(const float* dist, int64_t Q, int64_t G, int64_t ldd,
                          int64_t g_offset, int Ptot, const float* sorted_d,
                          const int32_t* sorted_idx, const int32_t* pos_total,
                          const int32_t* cells, int Jmax, const float* junk_d,
                          const int32_t* junk_idx, const int32_t* junk_cnt, int32_t* hist,
                          int32_t* before, void* stream) {
  PPS_ENFORCE(dist && sorted_d && sorted_idx && pos_total && cells && junk_d && junk_idx &&
                  junk_cnt && hist && before,
              "null pointer");
  PPS_ENFORCE(((uintptr_t)cells & 15) == 0, "cells must be 16-byte aligned");
  PPS_ENFORCE(Q >= 0 && G >= 0 && ldd >= G && Ptot > 0 && Jmax > 0, "bad shape");
  PPS_ENFORCE((G + kRankStreamChunk - 1) / kRankStreamChunk <= 65535,
              "G too large for the chunk grid (65535 chunks of " +
                  std::to_string(kRankStreamChunk) + ")");
  return rank_count_stream(dist, Q, G, ldd, g_offset, Ptot, sorted_d, sorted_idx, pos_total,
                           cells, Jmax, junk_d, junk_idx, junk_cnt, hist, before,
                           as_stream(stream));
}

int pps_ap_finalize(int64_t Q, int Ptot, const float* sorted_d, const int32_t* pos_total,
                    const int32_t* hist, const int32_t* before, double* ap,
                    int32_t* valid, int32_t* first_rank, void* stream) {
  PPS_ENFORCE(sorted_d && pos_total && hist && before && ap && valid && first_rank,
              "null pointer");
  PPS_ENFORCE(Q >= 0 && Ptot >= 0, "bad shape");
  return ap_finalize(Q, Ptot, sorted_d, pos_total, hist, before, ap, valid, first_rank,
                     as_stream(stream));
}

int pps_cmc_counts(const float* dist, int64_t Q, int64_t G, int64_t ldd, int64_t g_offset,
                   int Ptot, const float* sorted_d, const int32_t* sorted_idx,
                   const int32_t* pos_total, const int32_t* qcam, const int32_t* gcam, int Jmax,
                   const float* junk_d, const int32_t* junk_idx, const int32_t* junk_cnt,
                   int32_t* hist, void* stream) {
  PPS_ENFORCE(dist && sorted_d && sorted_idx && pos_total && hist, "null pointer");
  PPS_ENFORCE((qcam == nullptr) == (gcam == nullptr),
              "qcam and gcam are given together (separate_camera_set) or not at all");
  PPS_ENFORCE(gcam || (junk_d && junk_idx && junk_cnt && Jmax > 0),
              "without separate_camera_set the junk lists are required");
  PPS_ENFORCE(Q >= 0 && G >= 0 && ldd >= G && Ptot > 0, "bad shape");
  PPS_ENFORCE(G < (1ll << 31) && g_offset + G < (1ll << 31), "gallery indices must fit int32");
  PPS_ENFORCE((G + kRankStreamChunk - 1) / kRankStreamChunk <= 65535,
              "G too large for the chunk grid");
  return cmc_counts(dist, Q, G, ldd, g_offset, Ptot, sorted_d, sorted_idx, pos_total, qcam,
                    gcam, Jmax, junk_d, junk_idx, junk_cnt, hist, as_stream(stream));
}

int pps_cmc_finalize(int64_t Q, int Ptot, const int32_t* pos_total, const int32_t* hist,
                     int topk, int first_match_break, double* ret, int32_t* valid,
                     void* stream) {
  PPS_ENFORCE(pos_total && hist && ret && valid, "null pointer");
  PPS_ENFORCE(Q >= 0 && Ptot > 0 && topk >= 1, "bad shape");
  return cmc_finalize(Q, Ptot, pos_total, hist, topk, first_match_break ? 1 : 0, ret, valid,
                      as_stream(stream));
}

int pps_topk(const float* dist, int64_t Q, int64_t G, int64_t ldd, int k, float* vals,
             int32_t* idx, void* stream) {
  PPS_ENFORCE(dist && vals && idx, "null pointer");
  PPS_ENFORCE(k >= 1 && k <= 1024, "k must be in [1, 1024], got " + std::to_string(k));
  PPS_ENFORCE(G >= k && ldd >= G, "need G >= k");
  PPS_ENFORCE(G < (1ll << 31), "G must fit int32");
  return topk(dist, Q, G, ldd, k, vals, idx, as_stream(stream));
}

int pps_argsort_rows(const float* dist, int64_t Q, int64_t G, int64_t ldd, int32_t* idx,
                     int64_t ldi, float* vals, int64_t ldv, void* stream) {
  PPS_ENFORCE(dist && idx, "null pointer");
  PPS_ENFORCE(Q >= 0 && G >= 0 && ldd >= G && ldi >= G && (!vals || ldv >= G), "bad shape");
  PPS_ENFORCE(G <= argsort_rows_cap(), "rows longer than " + std::to_string(argsort_rows_cap()) +
                                           " entries (pps_argsort_rows_cap): use pps_topk");
  return argsort_rows(dist, Q, G, ldd, idx, ldi, vals, ldv, as_stream(stream));
}

int pps_argsort_rows_cap(void) { return argsort_rows_cap(); }

int pps_sgs_keys(const int32_t* order, int64_t Q, int64_t G, int64_t ldo, const int32_t* gid,
                 const int32_t* gcam, const int32_t* qid, const int32_t* qcam,
                 int separate_camera_set, int U, float* keys, void* stream) {
  PPS_ENFORCE(order && gid && gcam && qid && qcam && keys, "null pointer");
  PPS_ENFORCE(Q >= 0 && G >= 0 && ldo >= G, "bad shape");
  PPS_ENFORCE(U >= 1 && U <= 16384, "U (distinct gallery identities) must be in [1, 16384]");
  return sgs_keys(order, Q, G, ldo, gid, gcam, qid, qcam, separate_camera_set ? 1 : 0, U, keys,
                  as_stream(stream));
}

int pps_sgs_groups(const float* sorted_keys, const int32_t* perm, int64_t Q, int64_t G, int U,
                   const int32_t* qid, int32_t* gstart, int32_t* glen, int32_t* nids,
                   int32_t* qt, void* stream) {
  PPS_ENFORCE(sorted_keys && perm && qid && gstart && glen && nids && qt, "null pointer");
  PPS_ENFORCE(Q >= 0 && G >= 1 && G <= argsort_rows_cap(), "G must be in [1, " +
                                                               std::to_string(argsort_rows_cap()) +
                                                               "]");
  PPS_ENFORCE(U >= 1 && U <= 16384, "U (distinct gallery identities) must be in [1, 16384]");
  PPS_ENFORCE(sgs_groups_lds_bytes(G, U) <= 160 * 1024, "groups do not fit in LDS");
  return sgs_groups(sorted_keys, perm, Q, G, U, qid, gstart, glen, nids, qt, as_stream(stream));
}

int pps_sgs_ranks(const int32_t* perm, int64_t Q, int64_t G, const int32_t* rows, int64_t nr,
                  const int32_t* gstart, const int32_t* glen, const int32_t* nids,
                  const int32_t* qt, int U, int repeat, const int32_t* draws, int64_t ldd,
                  int32_t* k, void* stream) {
  PPS_ENFORCE(perm && gstart && glen && nids && qt && k && (nr == 0 || (rows && draws)),
              "null pointer");
  PPS_ENFORCE(Q >= 0 && G >= 1 && nr >= 0 && repeat >= 1 && ldd >= 1, "bad shape");
  PPS_ENFORCE(U >= 1 && U <= 16384 && ldd <= U, "ldd must be in [1, U]");
  return sgs_ranks(perm, G, rows, nr, gstart, glen, nids, qt, U, repeat, draws, ldd, k,
                   as_stream(stream));
}

int pps_topk_merge(const float* vals, const int32_t* idx, int R, int64_t Q, int k_in,
                   const int64_t* list_offsets, int k_out, float* out_vals,
                   int32_t* out_idx, void* stream) {
  PPS_ENFORCE(vals && idx && list_offsets && out_vals && out_idx, "null pointer");
  PPS_ENFORCE(R >= 1 && R <= kMergeMaxLists,
              "R must be in [1, " + std::to_string(kMergeMaxLists) + "]");
  PPS_ENFORCE(Q >= 0 && k_in >= 1 && k_out >= 1, "bad shape");
  PPS_ENFORCE((int64_t)R * k_in <= 8192,
              "R * k_in must be <= 8192 (LDS), got " + std::to_string((int64_t)R * k_in));
  MergeOffsets offs{};
  for (int r = 0; r < R; ++r) {
    PPS_ENFORCE(list_offsets[r] >= 0 && list_offsets[r] + k_in <= (int64_t)INT32_MAX,
                "list offset out of the int32 index range");
    offs.off[r] = list_offsets[r];
  }
  return topk_merge(vals, idx, R, Q, k_in, offs, k_out, out_vals, out_idx,
                    as_stream(stream));
}

int64_t pps_rerank_workspace_bytes(int64_t Q, int64_t G, int k1, int k2) {
  if (Q < 0 || G < 0 || k1 < 1 || k2 < 1) return -1;
  return (int64_t)rerank_workspace_bytes(Q, G, k1, k2);
}

int64_t pps_rerank_workspace_bytes_ld(const float* q_g, int64_t ld_qg, const float* q_q,
                                      int64_t ld_qq, const float* g_g, int64_t ld_gg, int64_t Q,
                                      int64_t G, int k1, int k2, int flags) {
  if (Q < 0 || G < 0 || k1 < 1 || k2 < 1) return -1;
  return (int64_t)rerank_workspace_bytes_for(q_g, ld_qg, q_q, ld_qq, g_g, ld_gg, Q, G, k1, k2,
                                             flags);
}

int pps_re_ranking_ld(const float* q_g, int64_t ld_qg, const float* q_q, int64_t ld_qq,
                      const float* g_g, int64_t ld_gg, int64_t Q, int64_t G, int k1, int k2,
                      double lambda_value, int flags, void* workspace, int64_t ws_bytes,
                      float* out, void* stream) {
  PPS_ENFORCE(q_g && q_q && g_g && workspace && out, "null pointer");
  PPS_ENFORCE(Q > 0 && G > 0, "bad shape");
  PPS_ENFORCE(ld_qg >= G && ld_qq >= Q && ld_gg >= G, "leading dims smaller than the rows");
  PPS_ENFORCE(k1 >= 1 && k1 + 1 <= 64, "k1 + 1 must be <= 64");
  PPS_ENFORCE(k2 >= 1 && k2 <= k1 + 1, "k2 must be in [1, k1 + 1]");
  const int K1 = k1 + 1, Kh = (int)lrint(k1 / 2.0) + 1;
  PPS_ENFORCE(K1 + K1 * Kh <= 1024, "expansion bound (k1+1)(round(k1/2)+2) must be <= 1024");
  PPS_ENFORCE(k2 * (K1 + K1 * Kh <= 256 ? 256 : (K1 + K1 * Kh <= 512 ? 512 : 1024)) <= 4096,
              "k2 * V row capacity must be <= 4096");
  PPS_ENFORCE(jaccard_lds_bytes(G) + 2048 <= 160 * 1024,
              "G must be <= 38400 (the Jaccard pass keeps a gallery row in LDS)");
  PPS_ENFORCE((Q + G) >= K1, "need Q + G >= k1 + 1");
  PPS_ENFORCE((flags & ~(PPS_RERANK_SYMMETRIC | PPS_RERANK_WHOLE)) == 0,
              "unknown re-ranking flags");
  PPS_ENFORCE(!(flags & PPS_RERANK_WHOLE) ||
                  ((flags & PPS_RERANK_SYMMETRIC) && ld_qg == ld_qq && ld_gg == ld_qq &&
                   q_g == q_q + Q && g_g == q_q + Q * ld_qq + Q),
              "PPS_RERANK_WHOLE: q_q, q_g and g_g must be the blocks of one symmetric matrix "
              "(one row stride, q_g = q_q + Q, g_g = q_q + Q * ld + Q) and PPS_RERANK_SYMMETRIC set");
  return rerank(q_g, ld_qg, q_q, ld_qq, g_g, ld_gg, Q, G, k1, k2, lambda_value, workspace,
                (size_t)ws_bytes, out, as_stream(stream), flags);
}

int pps_re_ranking_flags(const float* q_g, const float* q_q, const float* g_g, int64_t Q,
                         int64_t G, int k1, int k2, double lambda_value, int flags,
                         void* workspace, int64_t ws_bytes, float* out, void* stream) {
  return pps_re_ranking_ld(q_g, G, q_q, Q, g_g, G, Q, G, k1, k2, lambda_value, flags, workspace,
                           ws_bytes, out, stream);
}

int pps_re_ranking(const float* q_g, const float* q_q, const float* g_g, int64_t Q,
                   int64_t G, int k1, int k2, double lambda_value, void* workspace,
                   int64_t ws_bytes, float* out, void* stream) {
  return pps_re_ranking_flags(q_g, q_q, g_g, Q, G, k1, k2, lambda_value, 0, workspace,
                              ws_bytes, out, stream);
}

int pps_conv1x1_seam_x3(const float* x, int64_t M, int K1, const uint16_t* w2c, int N1,
                        const float* scale2c, const float* shift2c, const float* residual,
                        float* trunk, const uint16_t* w2a, int N2, const float* scale2a,
                        const float* shift2a, float* y, void* stream) {
  PPS_ENFORCE(x && w2c && scale2c && shift2c && residual && trunk && w2a && scale2a && shift2a &&
                  y,
              "null pointer");
  PPS_ENFORCE(M >= 0 && M * N1 * 4 < kMaxBufBytes, "bad M");
  PPS_ENFORCE(seam_supported(K1, N1, N2),
              "bottleneck seam: (K1, N1, N2) must be (64, 256, 64) or (128, 512, 128), got (" +
                  std::to_string(K1) + ", " + std::to_string(N1) + ", " + std::to_string(N2) + ")");
  PPS_ENFORCE(aligned16(x) && aligned16(w2c) && aligned16(residual) && aligned16(trunk) &&
                  aligned16(w2a) && aligned16(y) && aligned16(scale2c) && aligned16(shift2c) &&
                  aligned16(scale2a) && aligned16(shift2a),
              "seam operands must be 16-byte aligned");
  SeamParams p{x, residual, w2c, scale2c, shift2c, trunk, w2a, scale2a, shift2a, y, (int)M};
  return launch_seam_x3(p, K1, N1, N2, as_stream(stream));
}

// weights either f32 [Cout][Kpad] (x3 = 0) or bf16x3 planes [3][Cout][Kpad]
// x3p: bf16x3 activation planes (x_pl / y_pl, plane strides in elements)
// instead of f32 x / y -- gemm_x3p.hip tiles only
}  // extern "C"
namespace pps {
int conv_impl(const float* x, int N, int H, int W, int Cin, int ldx,
                      const void* w, int x3, int Cout, int Kpad, int KH, int KW, int stride,
                      int pad, int dil, const float* scale, const float* shift,
                      const float* residual, int relu, float* y, int Ho, int Wo, int ldy,
                      int tile, void* stream, const uint16_t* x_pl = nullptr,
                      int64_t x_plane = 0, uint16_t* y_pl = nullptr, int64_t y_plane = 0,
                      int splitk = 1, float* part = nullptr, int* fix_cnt = nullptr,
                      int64_t n_cnt = 0, float* amax_out = nullptr,
                      const float* w_rs = nullptr, const float* amax_in = nullptr,
                      uint16_t* y_h2, int64_t y_h2_plane, const float* h2o_in, float h2o_bw,
                      float h2o_bb) {
  // y_h2: the output as f16x2 planes on the scale of the bound
  // h2o_bw * max|x| + h2o_bb (EPI_F_H2OUT; the bound goes to amax_out)
  PPS_ENFORCE((x != nullptr) != (x_pl != nullptr) &&
                  (int)(y != nullptr) + (int)(y_pl != nullptr) + (int)(y_h2 != nullptr) == 1,
              "exactly one of x / x planes and one of y / y planes / y f16x2 planes must be given");
  if (y_h2) {
    PPS_ENFORCE(relu && !residual && splitk == 1 && h2o_in && amax_out && x3 &&
                    y_h2_plane >= (int64_t)N * Ho * Wo * ldy && Cin % 32 == 0 &&
                    Kpad == KH * KW * Cin && h2o_bw >= 0.f && h2o_bb >= 0.f,
                "f16x2 planes out: conv + BN + ReLU (no residual, no split-K), Cin % 32 == 0, "
                "the input's slot, an output slot, a plane stride >= N*Ho*Wo*ldy");
    y = reinterpret_cast<float*>(y_h2);  // for the shared checks below
  }
  // PPS_TILE_B_TILED or-ed into tile: the bf16x3 weights are chunk-tiled;
  // PPS_TILE_COL_ORDER: column-major tile order
  const bool wtiled = tile > 0 && (tile & PPS_TILE_B_TILED) != 0;
  const bool colmajor = tile > 0 && (tile & PPS_TILE_COL_ORDER) != 0;
  tile &= ~(PPS_TILE_B_TILED | PPS_TILE_COL_ORDER);
  if (wtiled) {
    PPS_ENFORCE(x3 && (splitk == 1 || fix_cnt), "tiled weights: bf16x3 weights, no two-pass split-K");
    PPS_ENFORCE(Kpad % 32 == 0 && Cin % 32 == 0, "tiled weights need Cin % 32 == 0");
    PPS_ENFORCE((tile >= GEMM_TILE_P_FIRST && tile < GEMM_TILE_WS) ||
                    (tile > GEMM_TILE_WS && tile < GEMM_NUM_TILES),
                "tiled weights need a pipelined tile (29..53, 55+)");
  }
  if (x_pl || y_pl) {
    PPS_ENFORCE(x3, "activation planes need the bf16x3 weights");
    PPS_ENFORCE(tile == 0 || tile >= GEMM_TILE_P_FIRST,
                "activation planes need a pipelined tile (0 or >= " +
                    std::to_string((int)GEMM_TILE_P_FIRST) + ")");
    if (x_pl) x = reinterpret_cast<const float*>(x_pl);  // for the shared checks below
    if (y_pl) y = reinterpret_cast<float*>(y_pl);
    PPS_ENFORCE(!x_pl || x_plane >= (int64_t)N * H * W * ldx, "x plane stride too small");
    PPS_ENFORCE(!y_pl || y_plane >= (int64_t)N * Ho * Wo * ldy, "y plane stride too small");
  }
  PPS_ENFORCE(x && w && scale && shift && y, "null pointer");
  PPS_ENFORCE(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0, "bad shape");
  PPS_ENFORCE(Cin % 4 == 0 && ldx % 4 == 0 && ldx >= Cin,
              "input channels must be a multiple of 4 (pad NHWC), got " +
                  std::to_string(Cin));
  PPS_ENFORCE(Kpad % 16 == 0 && Kpad >= KH * KW * Cin, "Kpad must be >= KH*KW*Cin, %16");
  PPS_ENFORCE(stride >= 1 && dil >= 1 && pad >= 0, "bad stride/pad/dilation");
  PPS_ENFORCE(Ho == (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1 &&
                  Wo == (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1,
              "output size does not match conv arithmetic");
  PPS_ENFORCE(ldy >= Cout, "ldy < Cout");
  PPS_ENFORCE(aligned16(x) && aligned16(w), "x/w must be 16-byte aligned");
  PPS_ENFORCE((int64_t)N * Ho * Wo < (1ll << 31), "too many output pixels");
  GemmParams p{};
  p.splitk = 1;
  PPS_ENFORCE(KH * KW <= 64, "at most 64 filter taps");
  PPS_ENFORCE(Cin >= 16 || ((Cin & (Cin - 1)) == 0 && Kpad <= 64 * Cin),
              "channels < 16 must be a power of two with Kpad <= 64*Cin");
  PPS_ENFORCE((int64_t)N * H * W * ldx * 4 < kMaxBufBytes, "input larger than 2 GiB");
  PPS_ENFORCE((int64_t)Cout * Kpad * 6 < kMaxBufBytes, "weights larger than 2 GiB");
  p.a = x; p.H = H; p.W = W; p.Cin = Cin; p.lda = ldx;
  p.a_bytes = (uint32_t)((int64_t)N * H * W * ldx * 4);
  p.b_bytes = (uint32_t)((int64_t)Cout * Kpad * 4);
  p.KH = KH; p.KW = KW; p.stride = stride; p.pad = pad; p.dil = dil;
  p.Ho = Ho; p.Wo = Wo; p.M = N * Ho * Wo;
  p.ldb = Kpad; p.kb_valid = Kpad; p.Ncol = Cout; p.Kloop = Kpad;
  p.scale = scale; p.shift = shift; p.residual = residual; p.ldr = ldy;
  p.out = y; p.ldo = ldy; p.relu = relu; p.tile = tile;
  p.colmajor = colmajor ? 1 : 0;
  p.amax_out = amax_out;
  int h2o = 0;
  if (y_h2) {
    p.out = nullptr; p.out3 = y_h2; p.out_plane = y_h2_plane;
    p.h2o_in = h2o_in; p.h2o_bw = h2o_bw; p.h2o_bb = h2o_bb;
    h2o = EPI_F_H2OUT;
  }
  if (w_rs) {
    // f16x2 (pps_conv2d_bn_act_h2, the whole-network plan's PPS_TILE_H2):
    // f32 activations scaled by their tensor's max, chunk-tiled two-plane
    // weights [2][Cout16 / 16][Kpad / 32][16][32] with per-channel scales
    // x_pl: f16x2 activation planes [2][x_plane] (pps_split_f16x2_act of x
    // with the same max): same bits as the f32 input, no split in the loop
    PPS_ENFORCE(!y_pl && splitk == 1, "f16x2 conv: f32 output, no split-K");
    PPS_ENFORCE(amax_in != nullptr, "f16x2 conv: the input tensor's max (amax_x) is required");
    PPS_ENFORCE(Cin % 32 == 0 && Kpad == KH * KW * Cin,
                "f16x2 conv: Cin % 32 == 0 and Kpad == KH*KW*Cin");
    PPS_ENFORCE(tile == 0 || (tile >= GEMM_TILE_P16_FIRST && tile < GEMM_NUM_TILES),
                "f16x2 conv: tile 0 or 38..60 (54: the weight-stationary 1x1 where it "
                "applies, else 38)");
    p.b3 = static_cast<const uint16_t*>(w);
    p.b_plane = (int64_t)(Cout + 15) / 16 * 16 * Kpad;
    p.b_bytes = (uint32_t)(p.b_plane * 2);
    p.tiled = 2;
    p.rs_b = w_rs;
    p.amax_a = amax_in;
    if (x_pl) {
      p.a = nullptr; p.a3 = x_pl; p.a_plane = x_plane;
      p.a_bytes = (uint32_t)((int64_t)N * H * W * ldx * 2);
    }
    return launch_gemm_x3(p, EPI_CONV | EPI_F_H2 | h2o, 1, as_stream(stream));
  }
  if (x_pl) {
    p.a = nullptr; p.a3 = x_pl; p.a_plane = x_plane;
    p.a_bytes = (uint32_t)((int64_t)N * H * W * ldx * 2);
  }
  if (splitk > 1) {
    // conv split-K: raw partial sums of K slices [splitk][M][Cout] on the
    // pipelined kernel, then one pass that sums them in slice order and
    // applies BN [+ residual] [ReLU] (f32 or bf16x3-plane output)
    PPS_ENFORCE(x3 && part, "split-K needs the bf16x3 weights and a partials buffer");
    PPS_ENFORCE(Cin % 32 == 0 && Kpad % (32 * splitk) == 0 && Kpad == KH * KW * Cin,
                "split-K needs Cin % 32 == 0 and Kpad % (32 * splitk) == 0");
    PPS_ENFORCE(ldy == Cout && Cout % 4 == 0 && aligned16(part), "split-K: dense output");
    PPS_ENFORCE(tile == 0 || tile >= GEMM_TILE_P_FIRST, "split-K needs a pipelined tile");
    const int64_t M = (int64_t)N * Ho * Wo;
    p.splitk = splitk; p.ksplit_conv = 1;
    p.Kloop = Kpad / splitk; p.kb_valid = p.Kloop;
    p.b3 = static_cast<const uint16_t*>(w); p.b_plane = (int64_t)Cout * Kpad;
    p.b_bytes = (uint32_t)(p.b_plane * 2);
    if (fix_cnt) {
      // one launch: the last K slice of each tile to finish sums the parked
      // partials (slice order) and runs BN [+ residual] + ReLU [-> planes]
      PPS_ENFORCE(relu, "one-launch split-K: conv + BN + ReLU epilogues only");
      PPS_ENFORCE(!(residual && y_pl), "one-launch split-K: residual with f32 output only");
      const int t = tile ? tile : GEMM_TILE_P16_FIRST + 7;
      const int bm = x3p_tile_rows(t, x_pl != nullptr), bn = x3p_tile_cols(t, x_pl != nullptr);
      PPS_ENFORCE(bm > 0 && bn > 0, "one-launch split-K needs a pipelined tile");
      const int64_t ntile = ((M + bm - 1) / bm) * ((Cout + bn - 1) / bn);
      PPS_ENFORCE(n_cnt >= ntile, "one-launch split-K: " + std::to_string(ntile) +
                                      " tile counters needed, " + std::to_string(n_cnt) + " given");
      if (wtiled) {
        p.b_plane = (int64_t)(Cout + 15) / 16 * 16 * Kpad;
        p.tiled = 2;
        p.b_bytes = (uint32_t)(p.b_plane * 2);
      }
      p.tile = t;
      p.part = part; p.part_sstride = M * Cout; p.fix_cnt = fix_cnt;
      p.out_sstride = 0;
      if (y_pl) { p.out = nullptr; p.out3 = y_pl; p.out_plane = y_plane; }
      return launch_gemm_x3(p, (y_pl ? EPI_CONV | EPI_F_PLANES : EPI_CONV) | EPI_F_FIX, 1,
                            as_stream(stream));
    }
    p.out = part; p.out3 = nullptr; p.ldo = Cout; p.out_sstride = M * Cout;
    p.residual = nullptr; p.relu = 0;
    // tile 0: tile 45, the one-launch entry's default (same rounding group,
    // so both entries give the same bits at tile 0 as at any equal id)
    p.tile = tile ? tile : GEMM_TILE_P16_FIRST + 7;
    const int rc = launch_gemm_x3(p, EPI_CONV | EPI_F_RAW, 1, as_stream(stream));
    if (rc != PPS_OK) return rc;
    return splitk_conv_epilogue(part, splitk, M, Cout, scale, shift, residual, relu,
                                y_pl ? nullptr : y, y_pl, y_plane, as_stream(stream), amax_out);
  }
  if (y_pl) { p.out = nullptr; p.out3 = y_pl; p.out_plane = y_plane; }
  if (x3) {
    p.b3 = static_cast<const uint16_t*>(w); p.b_plane = (int64_t)Cout * Kpad;
    if (wtiled) {  // [3][Cout16 / 16][Kpad / 32][16][32]
      p.b_plane = (int64_t)(Cout + 15) / 16 * 16 * Kpad;
      p.tiled = 2;
    }
    p.b_bytes = (uint32_t)(p.b_plane * 2);
    PPS_ENFORCE(!h2o || !x_pl, "f16x2 planes out from a bf16x3 conv: f32 activations in");
    return launch_gemm_x3(p, (y_pl ? EPI_CONV | EPI_F_PLANES : EPI_CONV) | h2o, 1,
                          as_stream(stream));
  }
  p.b = static_cast<const float*>(w);
  return launch_gemm(p, EPI_CONV, 1, as_stream(stream));
}
}  // namespace pps
extern "C" {

int pps_conv2d_bn_act(const float* x, int N, int H, int W, int Cin, int ldx,
                      const float* w, int Cout, int Kpad, int KH, int KW, int stride,
                      int pad, int dil, const float* scale, const float* shift,
                      const float* residual, int relu, float* y, int Ho, int Wo, int ldy,
                      int tile, void* stream) {
  return conv_impl(x, N, H, W, Cin, ldx, w, 0, Cout, Kpad, KH, KW, stride, pad, dil, scale,
                   shift, residual, relu, y, Ho, Wo, ldy, tile, stream);
}

int pps_conv2d_bn_act_x3(const float* x, int N, int H, int W, int Cin, int ldx,
                         const uint16_t* w3, int Cout, int Kpad, int KH, int KW, int stride,
                         int pad, int dil, const float* scale, const float* shift,
                         const float* residual, int relu, float* y, int Ho, int Wo, int ldy,
                         int tile, void* stream) {
  return conv_impl(x, N, H, W, Cin, ldx, w3, 1, Cout, Kpad, KH, KW, stride, pad, dil, scale,
                   shift, residual, relu, y, Ho, Wo, ldy, tile, stream);
}

int pps_conv2d_bn_act_x3p_splitk(const float* x, const uint16_t* x3, int64_t x_plane, int N,
                                 int H, int W, int Cin, int ldx, const uint16_t* w3, int Cout,
                                 int Kpad, int KH, int KW, int stride, int pad, int dil,
                                 const float* scale, const float* shift, const float* residual,
                                 int relu, float* y, uint16_t* y3, int64_t y_plane, int Ho,
                                 int Wo, int ldy, int splitk, float* part, int tile,
                                 void* stream) {
  PPS_ENFORCE(splitk >= 1 && splitk <= 16, "splitk must be in [1, 16]");
  return conv_impl(x, N, H, W, Cin, ldx, w3, 1, Cout, Kpad, KH, KW, stride, pad, dil, scale,
                   shift, residual, relu, y, Ho, Wo, ldy, tile, stream, x3, x_plane, y3,
                   y_plane, splitk, part);
}

int pps_conv2d_bn_act_x3p_splitk_fused(const float* x, const uint16_t* x3, int64_t x_plane,
                                       int N, int H, int W, int Cin, int ldx, const uint16_t* w3,
                                       int Cout, int Kpad, int KH, int KW, int stride, int pad,
                                       int dil, const float* scale, const float* shift,
                                       const float* residual, int relu, float* y, uint16_t* y3,
                                       int64_t y_plane, int Ho, int Wo, int ldy, int splitk,
                                       float* part, int* counters, int64_t n_counters, int tile,
                                       void* stream) {
  PPS_ENFORCE(splitk >= 2 && splitk <= 16, "splitk must be in [2, 16]");
  PPS_ENFORCE(counters != nullptr, "null tile counters");
  return conv_impl(x, N, H, W, Cin, ldx, w3, 1, Cout, Kpad, KH, KW, stride, pad, dil, scale,
                   shift, residual, relu, y, Ho, Wo, ldy, tile, stream, x3, x_plane, y3,
                   y_plane, splitk, part, counters, n_counters);
}

int pps_conv2d_bn_act_x3p(const float* x, const uint16_t* x3, int64_t x_plane, int N, int H,
                          int W, int Cin, int ldx, const uint16_t* w3, int Cout, int Kpad,
                          int KH, int KW, int stride, int pad, int dil, const float* scale,
                          const float* shift, const float* residual, int relu, float* y,
                          uint16_t* y3, int64_t y_plane, int Ho, int Wo, int ldy, int tile,
                          void* stream) {
  return conv_impl(x, N, H, W, Cin, ldx, w3, 1, Cout, Kpad, KH, KW, stride, pad, dil, scale,
                   shift, residual, relu, y, Ho, Wo, ldy, tile, stream, x3, x_plane, y3,
                   y_plane);
}

int pps_x3p_tile_shape(int tile, int planes, int* rows, int* cols) {
  PPS_ENFORCE(rows && cols, "null pointer");
  *rows = x3p_tile_rows(tile, planes != 0);
  *cols = x3p_tile_cols(tile, planes != 0);
  return PPS_OK;
}

// The last res5 conv with the part pooling fused into its epilogue
// (ResNet.py:276-333 res5_2 branch2c + Sum + Relu, then bpm_heads.py:18-55 /
// pps_heads.py:38-80): conv + BN + residual + ReLU on a pipelined tile whose
// rows are exactly one image (Ho * Wo); each tile pools its image's strips
// and writes the 2^S - 1 part subsets into pps_out [2^S - 1][N][Cout] as
// pps_part_power_set does (same bits).  y (the conv output) may be null: it
// is then never written.
}  // extern "C"
namespace pps {
int conv_pps_impl(const float* x, const uint16_t* x3, int64_t x_plane, int N,
                              int H, int W, int Cin, int ldx, const uint16_t* w3, int Cout,
                              int Kpad, int KH, int KW, int stride, int pad, int dil,
                              const float* scale, const float* shift, const float* residual,
                              float* y, int Ho, int Wo, const int32_t* splits, int S,
                              int max_ave, float* pps_out, int tile, void* stream,
                              const float* w_rs, const float* amax_in) {
  PPS_ENFORCE((x != nullptr) != (x3 != nullptr), "exactly one of x / x planes must be given");
  PPS_ENFORCE(w3 && scale && shift && residual && pps_out && splits, "null pointer");
  PPS_ENFORCE(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && Cout % 4 == 0, "bad shape");
  PPS_ENFORCE(Cin % 32 == 0 && ldx % 8 == 0 && ldx >= Cin && Kpad == KH * KW * Cin,
              "pipelined conv: Cin % 32 == 0, Kpad == KH*KW*Cin");
  PPS_ENFORCE(KH * KW <= 64 && stride >= 1 && dil >= 1 && pad >= 0, "bad filter");
  PPS_ENFORCE(Ho == (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1 &&
                  Wo == (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1,
              "output size does not match conv arithmetic");
  PPS_ENFORCE(S >= 1 && S <= kPpsFuseMaxStrips, "1..10 strips");
  int hsum = 0;
  for (int j = 0; j < S; ++j) {
    PPS_ENFORCE(splits[j] > 0, "strip heights must be positive");
    hsum += splits[j];
  }
  PPS_ENFORCE(hsum == Ho, "strip heights must sum to the output height");
  const bool pl = x3 != nullptr;
  // chunk-tiled weights (always for f16x2: two planes, per-channel scales)
  const bool wtiled = w_rs != nullptr || (tile > 0 && (tile & PPS_TILE_B_TILED) != 0);
  PPS_ENFORCE(!w_rs || amax_in, "f16x2: the activations' max is required");
  const bool colmajor = tile > 0 && (tile & PPS_TILE_COL_ORDER) != 0;
  tile &= ~(PPS_TILE_B_TILED | PPS_TILE_COL_ORDER);
  if (tile == 0) tile = pl ? GEMM_TILE_P16_FIRST + 1 : GEMM_TILE_P16_192x128W42;
  PPS_ENFORCE(!w_rs || tile >= GEMM_TILE_P16_FIRST, "f16x2: a 16x16x32 tile (38+)");
  PPS_ENFORCE(x3p_tile_rows(tile, pl) == Ho * Wo && x3p_tile_cols(tile, pl) <= kPpsFuseMaxCols,
              "the fused pooling needs a pipelined tile of exactly Ho*Wo = " +
                  std::to_string(Ho * Wo) + " rows and <= 256 columns, tile " +
                  std::to_string(tile) + " has " + std::to_string(x3p_tile_rows(tile, pl)));
  PPS_ENFORCE((int64_t)N * H * W * ldx * (pl ? 2 : 4) < kMaxBufBytes, "input larger than 2 GiB");
  PPS_ENFORCE((int64_t)(1 << S) * N * Cout < (1ll << 31), "part output too large");
  PPS_ENFORCE(aligned16(pl ? (const void*)x3 : (const void*)x) && aligned16(w3) &&
                  aligned16(scale) && aligned16(shift) && aligned16(residual) &&
                  (!y || aligned16(y)),
              "16-byte aligned pointers");
  PPS_ENFORCE(!pl || x_plane >= (int64_t)N * H * W * ldx, "x plane stride too small");
  GemmParams p{};
  p.splitk = 1;
  p.a = x; p.H = H; p.W = W; p.Cin = Cin; p.lda = ldx;
  p.a_bytes = (uint32_t)((int64_t)N * H * W * ldx * (pl ? 2 : 4));
  if (pl) { p.a = nullptr; p.a3 = x3; p.a_plane = x_plane; }
  p.KH = KH; p.KW = KW; p.stride = stride; p.pad = pad; p.dil = dil;
  p.Ho = Ho; p.Wo = Wo; p.M = N * Ho * Wo;
  p.ldb = Kpad; p.kb_valid = Kpad; p.Ncol = Cout; p.Kloop = Kpad;
  p.b3 = w3; p.b_plane = (int64_t)(wtiled ? (Cout + 15) / 16 * 16 : Cout) * Kpad;
  p.b_bytes = (uint32_t)(p.b_plane * 2);
  p.tiled = wtiled ? 2 : 0;
  p.colmajor = colmajor ? 1 : 0;
  p.scale = scale; p.shift = shift; p.residual = residual; p.ldr = Cout;
  p.out = y; p.ldo = Cout; p.relu = 1; p.tile = tile;
  p.pps_out = pps_out; p.pps_S = S; p.pps_max_ave = max_ave ? 1 : 0; p.pps_nimg = N;
  p.pps_write_y = y ? 1 : 0;
  for (int j = 0; j < S; ++j) p.pps_h[j] = splits[j];
  PPS_ENFORCE(x3p_eligible(p, EPI_CONV | EPI_F_RES | EPI_F_RELU), "shape not eligible for the pipelined GEMM");
  const int h2 = w_rs ? EPI_F_H2 : 0;
  p.rs_b = w_rs;
  p.amax_a = amax_in;
  return launch_gemm_x3p(p, EPI_CONV | EPI_F_RES | EPI_F_RELU | EPI_F_PPS | h2, 1,
                         as_stream(stream), tile - GEMM_TILE_P_FIRST);
}
}  // namespace pps
extern "C" {

int pps_conv2d_bn_act_pps_x3p(const float* x, const uint16_t* x3, int64_t x_plane, int N,
                              int H, int W, int Cin, int ldx, const uint16_t* w3, int Cout,
                              int Kpad, int KH, int KW, int stride, int pad, int dil,
                              const float* scale, const float* shift, const float* residual,
                              float* y, int Ho, int Wo, const int32_t* splits, int S,
                              int max_ave, float* pps_out, int tile, void* stream) {
  return conv_pps_impl(x, x3, x_plane, N, H, W, Cin, ldx, w3, Cout, Kpad, KH, KW, stride, pad,
                       dil, scale, shift, residual, y, Ho, Wo, splits, S, max_ave, pps_out, tile,
                       stream, nullptr, nullptr);
}

// ---- f16x2 convolutions (include/pps_abi.h "f16x2 convolutions") ----------
int pps_conv2d_bn_act_h2(const float* x, int N, int H, int W, int Cin, int ldx,
                         const uint16_t* w2t, const float* wrs, int Cout, int Kpad, int KH,
                         int KW, int stride, int pad, int dil, const float* scale,
                         const float* shift, const float* residual, int relu, float* y, int Ho,
                         int Wo, int ldy, const float* amax_x, float* amax_y, int tile,
                         void* stream) {
  PPS_ENFORCE(wrs != nullptr, "null weight scales");
  return conv_impl(x, N, H, W, Cin, ldx, w2t, 1, Cout, Kpad, KH, KW, stride, pad, dil, scale,
                   shift, residual, relu, y, Ho, Wo, ldy, tile, stream, nullptr, 0, nullptr, 0, 1,
                   nullptr, nullptr, 0, amax_y, wrs, amax_x);
}

int pps_conv2d_dual_bn_act_h2(const float* x, int N, int H, int W, int Cin, int ldx, int KH,
                              int KW, int stride, int pad, const float* x2, int H2, int W2,
                              int Cin2, int ldx2, int stride2, const uint16_t* w2t,
                              const float* wrs, int Cout, int Kpad1, int Kpad2,
                              const float* shift, int relu, float* y, int Ho, int Wo, int ldy,
                              const float* amax_x, const float* amax_x2, float* amax_y, int tile,
                              void* stream) {
  PPS_ENFORCE(wrs != nullptr, "null weight scales");
  return dual_impl(x, N, H, W, Cin, ldx, KH, KW, stride, pad, x2, H2, W2, Cin2, ldx2, stride2,
                   w2t, 1, Cout, Kpad1, Kpad2, shift, relu, y, Ho, Wo, ldy, tile, stream, amax_y,
                   wrs, amax_x, amax_x2);
}

int pps_conv2d_bn_act_h2_planes(const uint16_t* x2, int64_t x_plane, int N, int H, int W,
                                int Cin, int ldx, const uint16_t* w2t, const float* wrs, int Cout,
                                int Kpad, int KH, int KW, int stride, int pad, int dil,
                                const float* scale, const float* shift, const float* residual,
                                int relu, float* y, int Ho, int Wo, int ldy, const float* amax_x,
                                float* amax_y, int tile, void* stream) {
  PPS_ENFORCE(wrs != nullptr && x2 != nullptr, "null pointer");
  return conv_impl(nullptr, N, H, W, Cin, ldx, w2t, 1, Cout, Kpad, KH, KW, stride, pad, dil,
                   scale, shift, residual, relu, y, Ho, Wo, ldy, tile, stream, x2, x_plane,
                   nullptr, 0, 1, nullptr, nullptr, 0, amax_y, wrs, amax_x);
}

int pps_conv2d_bn_act_h2out(const float* x, const uint16_t* x2, int64_t x_plane, int N, int H,
                            int W, int Cin, int ldx, const void* w, const float* wrs, int Cout,
                            int Kpad, int KH, int KW, int stride, int pad, int dil,
                            const float* scale, const float* shift, uint16_t* y2, int64_t y_plane,
                            int Ho, int Wo, int ldy, const float* amax_x, const float* bound_in,
                            float bound_w, float bound_b, float* bound_out, int tile,
                            void* stream) {
  PPS_ENFORCE(w && y2 && bound_in && bound_out, "null pointer");
  PPS_ENFORCE(!x2 || wrs, "f16x2 activation planes in: f16x2 weights (wrs) only");
  return conv_impl(x2 ? nullptr : x, N, H, W, Cin, ldx, w, 1, Cout, Kpad, KH, KW, stride, pad,
                   dil, scale, shift, nullptr, 1, nullptr, Ho, Wo, ldy, tile, stream, x2, x_plane,
                   nullptr, 0, 1, nullptr, nullptr, 0, bound_out, wrs, wrs ? amax_x : nullptr, y2,
                   y_plane, bound_in, bound_w, bound_b);
}

int pps_conv2d_bn_act_pps_h2_planes(const uint16_t* x2, int64_t x_plane, int N, int H, int W,
                                    int Cin, int ldx, const uint16_t* w2t, const float* wrs,
                                    int Cout, int Kpad, int KH, int KW, int stride, int pad,
                                    int dil, const float* scale, const float* shift,
                                    const float* residual, float* y, int Ho, int Wo,
                                    const int32_t* splits, int S, int max_ave, float* pps_out,
                                    const float* amax_x, int tile, void* stream) {
  PPS_ENFORCE(wrs != nullptr && x2 != nullptr, "null pointer");
  return conv_pps_impl(nullptr, x2, x_plane, N, H, W, Cin, ldx, w2t, Cout, Kpad, KH, KW, stride,
                       pad, dil, scale, shift, residual, y, Ho, Wo, splits, S, max_ave, pps_out,
                       tile, stream, wrs, amax_x);
}

int pps_conv2d_bn_act_pps_h2(const float* x, int N, int H, int W, int Cin, int ldx,
                             const uint16_t* w2t, const float* wrs, int Cout, int Kpad, int KH,
                             int KW, int stride, int pad, int dil, const float* scale,
                             const float* shift, const float* residual, float* y, int Ho, int Wo,
                             const int32_t* splits, int S, int max_ave, float* pps_out,
                             const float* amax_x, int tile, void* stream) {
  PPS_ENFORCE(wrs != nullptr, "null weight scales");
  return conv_pps_impl(x, nullptr, 0, N, H, W, Cin, ldx, w2t, Cout, Kpad, KH, KW, stride, pad,
                       dil, scale, shift, residual, y, Ho, Wo, splits, S, max_ave, pps_out, tile,
                       stream, wrs, amax_x);
}

}  // extern "C"
namespace pps {
int dual_impl(const float* x, int N, int H, int W, int Cin, int ldx,
                           int KH, int KW, int stride, int pad, const float* x2, int H2,
                           int W2, int Cin2, int ldx2, int stride2, const void* w, int x3,
                           int Cout, int Kpad1, int Kpad2, const float* shift, int relu,
                           float* y, int Ho, int Wo, int ldy, int tile, void* stream,
                           float* amax_out, const float* w_rs, const float* amax_in,
                           const float* amax_in2) {
  PPS_ENFORCE(x && x2 && w && shift && y, "null pointer");
  PPS_ENFORCE(N > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && Cin2 > 0, "bad shape");
  const bool wtiled = tile > 0 && (tile & PPS_TILE_B_TILED) != 0;  // chunk-tiled weights
  const bool colmajor = tile > 0 && (tile & PPS_TILE_COL_ORDER) != 0;
  tile &= ~(PPS_TILE_B_TILED | PPS_TILE_COL_ORDER);
  if (wtiled)
    PPS_ENFORCE(x3 && (Kpad1 + Kpad2) % 32 == 0 &&
                    ((tile >= GEMM_TILE_P_FIRST && tile < GEMM_TILE_WS) ||
                     (tile > GEMM_TILE_WS && tile < GEMM_NUM_TILES)),
                "tiled weights: bf16x3, K % 32 == 0, a pipelined tile");
  PPS_ENFORCE(Cin % 4 == 0 && ldx % 4 == 0 && Cin2 % 16 == 0 && ldx2 % 4 == 0,
              "channel counts must be multiples of 4 (second operand: 16)");
  PPS_ENFORCE(Kpad1 % 16 == 0 && Kpad1 >= KH * KW * Cin && Kpad2 == Cin2,
              "Kpad1 >= KH*KW*Cin (%16), Kpad2 == Cin2");
  PPS_ENFORCE(KH * KW <= 64, "at most 64 filter taps");
  PPS_ENFORCE(Ho == (H + 2 * pad - (KH - 1) - 1) / stride + 1 &&
                  Wo == (W + 2 * pad - (KW - 1) - 1) / stride + 1,
              "output size does not match conv arithmetic");
  PPS_ENFORCE(Ho == (H2 - 1) / stride2 + 1 && Wo == (W2 - 1) / stride2 + 1,
              "second operand (1x1, stride2) does not map onto the output grid");
  PPS_ENFORCE((int64_t)N * H * W * ldx * 4 < kMaxBufBytes &&
                  (int64_t)N * H2 * W2 * ldx2 * 4 < kMaxBufBytes,
              "input larger than 2 GiB");
  PPS_ENFORCE(aligned16(x) && aligned16(x2) && aligned16(w), "16-byte alignment");
  GemmParams p{};
  p.splitk = 1;
  p.a = x; p.H = H; p.W = W; p.Cin = Cin; p.lda = ldx;
  p.a_bytes = (uint32_t)((int64_t)N * H * W * ldx * 4);
  p.KH = KH; p.KW = KW; p.stride = stride; p.pad = pad; p.dil = 1;
  p.Ho = Ho; p.Wo = Wo; p.M = N * Ho * Wo;
  p.a2 = x2; p.a2_bytes = (uint32_t)((int64_t)N * H2 * W2 * ldx2 * 4);
  p.H2 = H2; p.W2 = W2; p.lda2 = ldx2; p.stride2 = stride2; p.Kloop1 = Kpad1;
  p.ldb = Kpad1 + Kpad2; p.kb_valid = Kpad1 + Kpad2; p.Ncol = Cout;
  p.Kloop = Kpad1 + Kpad2;
  p.scale = nullptr; p.shift = shift; p.out = y; p.ldo = ldy; p.relu = relu; p.tile = tile;
  p.colmajor = colmajor ? 1 : 0;
  PPS_ENFORCE((int64_t)Cout * (Kpad1 + Kpad2) * 6 < kMaxBufBytes, "weights larger than 2 GiB");
  p.amax_out = amax_out;
  if (w_rs) {  // f16x2: both operands share their maxima's scale (conv_impl)
    PPS_ENFORCE(amax_in && amax_in2, "f16x2 conv: both inputs' maxima are required");
    PPS_ENFORCE(Cin % 32 == 0 && Kpad1 == KH * KW * Cin && Kpad2 % 32 == 0,
                "f16x2 conv: Cin % 32 == 0, Kpad1 == KH*KW*Cin, Cin2 % 32 == 0");
    PPS_ENFORCE(tile == 0 || tile == GEMM_TILE_P16_192x128W41 ||
                    (tile >= GEMM_TILE_P16_FIRST && tile < GEMM_TILE_C16_FIRST),
                "f16x2 fused-shortcut conv: tile 0, 38..55 or 60");
    p.b3 = static_cast<const uint16_t*>(w);
    p.b_plane = (int64_t)(Cout + 15) / 16 * 16 * (Kpad1 + Kpad2);
    p.b_bytes = (uint32_t)(p.b_plane * 2);
    p.tiled = 2;
    p.rs_b = w_rs;
    p.amax_a = amax_in;
    p.amax_a2 = amax_in2;
    return launch_gemm_x3(p, EPI_CONV | EPI_F_H2, 1, as_stream(stream));
  }
  if (x3) {
    p.b3 = static_cast<const uint16_t*>(w);
    p.b_plane = (int64_t)(wtiled ? (Cout + 15) / 16 * 16 : Cout) * (Kpad1 + Kpad2);
    p.b_bytes = (uint32_t)(p.b_plane * 2);
    p.tiled = wtiled ? 2 : 0;
    return launch_gemm_x3(p, EPI_CONV, 1, as_stream(stream));
  }
  p.b = static_cast<const float*>(w);
  p.b_bytes = (uint32_t)((int64_t)Cout * (Kpad1 + Kpad2) * 4);
  return launch_gemm(p, EPI_CONV, 1, as_stream(stream));
}
}  // namespace pps
extern "C" {

int pps_conv2d_dual_bn_act(const float* x, int N, int H, int W, int Cin, int ldx,
                           int KH, int KW, int stride, int pad, const float* x2, int H2,
                           int W2, int Cin2, int ldx2, int stride2, const float* w,
                           int Cout, int Kpad1, int Kpad2, const float* shift, int relu,
                           float* y, int Ho, int Wo, int ldy, int tile, void* stream) {
  return dual_impl(x, N, H, W, Cin, ldx, KH, KW, stride, pad, x2, H2, W2, Cin2, ldx2, stride2,
                   w, 0, Cout, Kpad1, Kpad2, shift, relu, y, Ho, Wo, ldy, tile, stream, nullptr,
                   nullptr, nullptr, nullptr);
}

int pps_conv2d_dual_bn_act_x3(const float* x, int N, int H, int W, int Cin, int ldx,
                              int KH, int KW, int stride, int pad, const float* x2, int H2,
                              int W2, int Cin2, int ldx2, int stride2, const uint16_t* w3,
                              int Cout, int Kpad1, int Kpad2, const float* shift, int relu,
                              float* y, int Ho, int Wo, int ldy, int tile, void* stream) {
  return dual_impl(x, N, H, W, Cin, ldx, KH, KW, stride, pad, x2, H2, W2, Cin2, ldx2, stride2,
                   w3, 1, Cout, Kpad1, Kpad2, shift, relu, y, Ho, Wo, ldy, tile, stream, nullptr,
                   nullptr, nullptr, nullptr);
}

int pps_gemm_bn_act_batched(const float* x, int64_t x_bstride, int M, int K,
                            const float* w, int64_t w_bstride, int Cout,
                            const float* scale, const float* shift, int relu, float* y,
                            int ldy, int B, int tile, void* stream) {
  PPS_ENFORCE(x && w && scale && shift && y, "null pointer");
  PPS_ENFORCE(M > 0 && K > 0 && Cout > 0 && B > 0, "bad shape");
  PPS_ENFORCE(K % 16 == 0, "K must be a multiple of 16");
  PPS_ENFORCE(x_bstride % 4 == 0 && w_bstride % 4 == 0, "batch strides must be %4");
  PPS_ENFORCE(ldy >= B * Cout, "ldy < B*Cout");
  PPS_ENFORCE(aligned16(x) && aligned16(w), "x/w must be 16-byte aligned");
  GemmParams p{};
  p.splitk = 1;
  PPS_ENFORCE((int64_t)M * K * 4 < kMaxBufBytes && (int64_t)Cout * K * 4 < kMaxBufBytes,
              "operands larger than 2 GiB");
  p.a = x; p.a_bstride = x_bstride; p.H = 1; p.W = M; p.Cin = K; p.lda = K;
  p.a_bytes = (uint32_t)((int64_t)M * K * 4);
  p.b_bytes = (uint32_t)((int64_t)Cout * K * 4);
  p.KH = p.KW = 1; p.stride = 1; p.dil = 1; p.Ho = 1; p.Wo = M; p.M = M;
  p.b = w; p.b_bstride = w_bstride; p.ldb = K; p.kb_valid = K; p.Ncol = Cout;
  p.Kloop = K;
  p.scale = scale; p.shift = shift; p.ss_bstride = Cout;
  p.out = y; p.ldo = ldy; p.out_bstride = Cout; p.relu = relu; p.tile = tile;
  return launch_gemm(p, EPI_CONV, B, as_stream(stream));
}

static int splitk_impl(const float* x, int M, int K, const void* w, int x3, int Cout, int B,
                            int splitk, float* part, int tile, void* stream) {
  PPS_ENFORCE(x && w && part, "null pointer");
  PPS_ENFORCE(M > 0 && K > 0 && Cout > 0 && B > 0 && splitk >= 1, "bad shape");
  PPS_ENFORCE(K % (16 * splitk) == 0, "K must be a multiple of 16*splitk");
  PPS_ENFORCE((int64_t)M * K * 4 < kMaxBufBytes && (int64_t)Cout * K * 4 < kMaxBufBytes,
              "operands larger than 2 GiB");
  PPS_ENFORCE(aligned16(x) && aligned16(w), "x/w must be 16-byte aligned");
  GemmParams p{};
  p.splitk = splitk;
  p.a = x; p.a_bstride = (int64_t)M * K; p.H = 1; p.W = M; p.Cin = K / splitk; p.lda = K;
  p.a_bytes = (uint32_t)((int64_t)M * K * 4);
  p.KH = p.KW = 1; p.stride = 1; p.dil = 1; p.Ho = 1; p.Wo = M; p.M = M;
  p.ldb = K; p.kb_valid = K / splitk; p.Ncol = Cout;
  p.Kloop = K / splitk;
  p.out = part; p.ldo = (int64_t)B * Cout; p.out_bstride = Cout;
  p.out_sstride = (int64_t)M * B * Cout; p.tile = tile;
  if (x3) {
    PPS_ENFORCE((int64_t)Cout * K * 6 < kMaxBufBytes, "weights larger than 2 GiB");
    p.b3 = static_cast<const uint16_t*>(w); p.b_plane = (int64_t)Cout * K;
    p.b_bstride = 3 * p.b_plane; p.b_bytes = (uint32_t)(p.b_plane * 2);
    return launch_gemm_x3(p, EPI_CONV | EPI_F_RAW, B, as_stream(stream));
  }
  p.b = static_cast<const float*>(w); p.b_bstride = (int64_t)Cout * K;
  p.b_bytes = (uint32_t)((int64_t)Cout * K * 4);
  return launch_gemm(p, EPI_CONV | EPI_F_RAW, B, as_stream(stream));
}

int pps_gemm_splitk_batched(const float* x, int M, int K, const float* w, int Cout, int B,
                            int splitk, float* part, int tile, void* stream) {
  return splitk_impl(x, M, K, w, 0, Cout, B, splitk, part, tile, stream);
}

int pps_gemm_splitk_batched_x3(const float* x, int M, int K, const uint16_t* w3, int Cout,
                               int B, int splitk, float* part, int tile, void* stream) {
  return splitk_impl(x, M, K, w3, 1, Cout, B, splitk, part, tile, stream);
}

int pps_split_bf16x3(const float* x, int64_t n, int nbatch, uint16_t* out, void* stream) {
  PPS_ENFORCE(x && out, "null pointer");
  PPS_ENFORCE(n > 0 && nbatch > 0, "bad shape");
  return split_bf16x3(x, n, nbatch, out, as_stream(stream));
}

int pps_splitk_bn_act_normalize(const float* part, int splitk, int M, int N,
                                const float* scale, const float* shift, int relu,
                                int normalize, float* y, void* stream) {
  PPS_ENFORCE(part && scale && shift && y, "null pointer");
  PPS_ENFORCE(splitk >= 1 && M >= 0 && N > 0, "bad shape");
  return splitk_bn_act_normalize(part, splitk, (int64_t)M * N, M, N, scale, shift, relu,
                                 normalize, y, as_stream(stream));
}

int pps_maxpool2d(const float* x, int N, int H, int W, int C, int k, int stride, int pad,
                  float* y, int Ho, int Wo, void* stream) {
  PPS_ENFORCE(x && y, "null pointer");
  PPS_ENFORCE(C % 4 == 0, "C must be a multiple of 4");
  PPS_ENFORCE(Ho == (H + 2 * pad - k) / stride + 1 && Wo == (W + 2 * pad - k) / stride + 1,
              "output size does not match pooling arithmetic (floor)");
  PPS_ENFORCE(aligned16(x) && aligned16(y), "x/y must be 16-byte aligned");
  return maxpool2d(x, N, H, W, C, k, stride, pad, y, Ho, Wo, as_stream(stream), nullptr);
}

int pps_part_power_set(const float* x, int N, int H, int W, int C, const int32_t* splits,
                       int nstrip, int max_ave, float* out, void* stream) {
  PPS_ENFORCE(x && splits && out, "null pointer");
  PPS_ENFORCE(nstrip >= 1 && nstrip <= 10, "nstrip must be in [1, 10]");
  int sum = 0;
  for (int j = 0; j < nstrip; ++j) {
    PPS_ENFORCE(splits[j] > 0, "split heights must be positive");
    sum += splits[j];
  }
  PPS_ENFORCE(sum == H, "split heights must sum to H (Split axis=2)");
  return part_power_set(x, N, H, W, C, splits, nstrip, max_ave, out, as_stream(stream));
}

int pps_group_mean(const float* x, int D, const int32_t* offsets, const int32_t* members,
                   int ngroups, float* out, void* stream) {
  PPS_ENFORCE(x && offsets && members && out && D > 0 && ngroups >= 0, "bad arguments");
  return group_mean(x, D, offsets, members, ngroups, out, as_stream(stream));
}

int pps_l2_normalize(const float* x, int64_t N, int D, float* y, void* stream) {
  PPS_ENFORCE(x && y && D > 0 && N >= 0, "bad arguments");
  return l2_normalize(x, N, D, y, as_stream(stream));
}

int pps_preprocess_bgr(const uint8_t* img, int N, int Hi, int Wi, const float* means,
                       int Ho, int Wo, float* y, void* stream) {
  PPS_ENFORCE(img && means && y, "null pointer");
  PPS_ENFORCE(N >= 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, "bad shape");
  PPS_ENFORCE(aligned16(y), "y must be 16-byte aligned");
  return preprocess_bgr(img, N, Hi, Wi, nullptr, nullptr, nullptr, means, Ho, Wo, y,
                        as_stream(stream));
}

int pps_preprocess_bgr_ragged(const uint8_t* blob, int N, const int64_t* offsets,
                              const int32_t* heights, const int32_t* widths,
                              const float* means, int Ho, int Wo, float* y, void* stream) {
  PPS_ENFORCE(blob && offsets && heights && widths && means && y, "null pointer");
  PPS_ENFORCE(N >= 0 && Ho > 0 && Wo > 0, "bad shape");
  PPS_ENFORCE(aligned16(y), "y must be 16-byte aligned");
  return preprocess_bgr(blob, N, 0, 0, offsets, heights, widths, means, Ho, Wo, y,
                        as_stream(stream));
}

}  // extern "C"
