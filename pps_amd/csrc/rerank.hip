// k-reciprocal re-ranking on the GPU (Zhong et al., CVPR 2017), as the
// reference evaluator applies it: reid_dataset_evaluator.py:442-519
// `re_ranking(q_g_dist, q_q_dist, g_g_dist, k1=20, k2=6, lambda_value=0.3)`.
//
// The reference materialises four N x N matrices (N = Q + G) and walks them
// with Python loops.  Here only the normalised squared-distance matrix OD is
// dense; the k-reciprocal weights V are sparse rows (at most (k1+1)(r+2)
// entries, r = round(k1/2)), the query-expanded V_qe rows are merges of k2
// sparse rows, and the Jaccard term is accumulated per query in LDS through
// an inverted (column) index of V_qe, in the same column order as the
// reference, so every float32 sum has the reference's operand order.
//
//  1. rerank_colmax_sq / rowmax_sq / build_od : OD[i][j] = M[j][i]^2 / max_r M[r][i]^2
//     with M = [[qq, qg], [qg^T, gg]]                          (:447-454)
//  2. pps_topk (rank.hip) on OD, k = k1 + 1 -> initial_rank      (:456)
//  3. rerank_v_rows  : k-reciprocal sets, expansion, exp weights  (:462-488)
//  4. rerank_vqe     : V_qe[i] = mean of V rows initial_rank[i,:k2] (:490-494)
//  5. rerank_csc_*   : inverted index of V_qe                     (:497-499)
//  6. rerank_jaccard : temp_min, jaccard, lambda blend, [Q][G] out (:501-518)
#include <vector>

#include "pps_internal.hpp"

// NumPy rounds every float32 product and sum on its own; hipcc's default
// fp-contract=fast would fuse e.g. the final blend jac * (1 - l) + od * l
// into an FMA (one rounding fewer), differently in each instantiation --
// off for the whole file (re-ranking is memory-bound; no FMA is needed).
// The pragma governs operators written in this file only: the __fmul_rn /
// __fadd_rn header helpers are plain operators compiled under the default
// contract setting and DO fuse after inlining, so they are not used here.
#pragma clang fp contract(off)

namespace pps {

// PPS_RERANK_INPLACE=0: keep the dense OD path (A/B runs)
static bool getenv_flag_off(const char* name) {
  const char* e = getenv(name);
  return e && e[0] == '0';
}

// M[r][c] of the concatenated distance matrix (before squaring), blocks with
// row strides (q_g^T read from q_g's columns)
struct RrIn {
  const float* qg;
  const float* qq;
  const float* gg;
  int64_t ldqg, ldqq, ldgg;
};
__device__ inline float rr_m(const RrIn& in, int64_t Q, int64_t r, int64_t c) {
  if (r < Q) return c < Q ? in.qq[r * in.ldqq + c] : in.qg[r * in.ldqg + (c - Q)];
  return c < Q ? in.qg[c * in.ldqg + (r - Q)] : in.gg[(r - Q) * in.ldgg + (c - Q)];
}

// OD rows are padded to a multiple of 4 floats: 16-byte aligned rows let the
// top-k over OD take its 16-byte-load kernels (the wave-streaming one at
// Duke size, N >= 16384)
static int64_t od_stride(int64_t N) { return (N + 3) / 4 * 4; }

// The column maxima of M^2 by blocks: column c of M is column c of qq plus
// row c of qg (c < Q), or column c-Q of qg plus column c-Q of gg (c >= Q).
// Squares are >= 0, so their float bits order as unsigned integers and an
// integer atomicMax into a zeroed vector is an exact, order-free max.  A
// thread owns one column of a kCmRows-row block and keeps kCmBatch loads in
// flight (one load at a time left the 1.2 GB of Duke's blocks at ~2.3 TB/s).
constexpr int kCmRows = 256;   // rows per block of the column-max kernel
constexpr int kCmBatch = 16;   // loads in flight per thread
__global__ void rerank_colmax_sq_kernel(const float* __restrict__ x, int64_t R, int64_t C,
                                        int64_t ld, unsigned* __restrict__ out) {
  const int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (c >= C) return;
  const int64_t r0 = blockIdx.y * (int64_t)kCmRows;
  const int64_t r1 = r0 + kCmRows < R ? r0 + kCmRows : R;
  float m = 0.f;
  int64_t r = r0;
  for (; r + kCmBatch <= r1; r += kCmBatch) {
    float v[kCmBatch];
#pragma unroll
    for (int u = 0; u < kCmBatch; ++u) v[u] = __builtin_nontemporal_load(x + (r + u) * ld + c);
#pragma unroll
    for (int u = 0; u < kCmBatch; ++u) m = fmaxf(m, v[u] * v[u]);
  }
  for (; r < r1; ++r) {
    const float v = x[r * ld + c];
    m = fmaxf(m, v * v);
  }
  atomicMax(out + c, __float_as_uint(m));
}

// max over row r of x^2 (one block per row)
__global__ void rerank_rowmax_sq_kernel(const float* __restrict__ x, int64_t C, int64_t ld,
                                        unsigned* __restrict__ out) {
  const int64_t r = blockIdx.x;
  const float* row = x + r * ld;
  float m = 0.f;
  int64_t c = threadIdx.x;
  for (; c + (kCmBatch - 1) * (int64_t)blockDim.x < C; c += kCmBatch * (int64_t)blockDim.x) {
    float v[kCmBatch];
#pragma unroll
    for (int u = 0; u < kCmBatch; ++u) v[u] = row[c + u * (int64_t)blockDim.x];
#pragma unroll
    for (int u = 0; u < kCmBatch; ++u) m = fmaxf(m, v[u] * v[u]);
  }
  for (; c < C; c += blockDim.x) {
    const float v = row[c];
    m = fmaxf(m, v * v);
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(out + r, __float_as_uint(m));
}

// OD[i][j] = M[j][i]^2 / colmax[i], via T x T LDS tiles (the transpose of
// :454).  256 threads; a wave moves T/64 consecutive 256-byte pieces of a
// tile row per access round, so HBM sees T*4-byte row segments both ways.
#ifndef PPS_OD_TILE
#define PPS_OD_TILE 64
#endif
template <int T>
__global__ void __launch_bounds__(256)
rerank_build_od_kernel(RrIn in, int64_t Q, int64_t G, const float* __restrict__ colmax,
                       float* __restrict__ od, int64_t ldo, int64_t i_min, int64_t j_max) {
  // writes OD[i][j] for i >= i_min, j < j_max (tiles cover that window)
  constexpr int H = T / 64;
  __shared__ float tile[T][T + 1];
  const int64_t N = Q + G;
  const int64_t i0 = (i_min / T) * T + blockIdx.y * (int64_t)T, j0 = blockIdx.x * (int64_t)T;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 256 threads: ty 0..3
  if (i0 + T <= Q && j0 >= Q) {
    // query rows x gallery columns: M[j][i] = qg[i][j - Q], i.e. OD here is
    // qg itself (squared, scaled) -- read it row-wise, no transpose (the
    // generic path below would read qg down its columns, stride G)
    for (int k = ty; k < T; k += 4) {
      const int64_t i = i0 + k;
      const float cm = colmax[i];
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const int64_t j = j0 + tx + 64 * h;
        if (j < N && j < j_max && i >= i_min) {
          const float m = in.qg[i * in.ldqg + (j - Q)];
          od[i * ldo + j] = rr_od(m, cm);
        }
      }
    }
    return;
  }
  for (int k = ty; k < T; k += 4) {  // read M[j0+k][i0+tx..] (row j, col i)
    const int64_t r = j0 + k;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const int64_t c = i0 + tx + 64 * h;
      float v = 0.f;
      if (r < N && c < N) {
        const float m = rr_m(in, Q, r, c);
        v = m;
      }
      tile[k][tx + 64 * h] = v;
    }
  }
  __syncthreads();
  for (int k = ty; k < T; k += 4) {  // write OD[i0+k][j0+tx..] = tile[tx..][k] / colmax
    const int64_t i = i0 + k;
    if (i >= N || i < i_min) continue;
    const float cm = colmax[i];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const int64_t j = j0 + tx + 64 * h;
      if (j < N && j < j_max) od[i * ldo + j] = rr_od(tile[tx + 64 * h][k], cm);
    }
  }
}

// Symmetric q_q and g_g (both self-distances from the mirrored GEMM, exactly
// symmetric): M is symmetric, so OD[i][j] = M[j][i]^2 / colmax[i] =
// M[i][j]^2 / colmax[i] is a row-major scaled copy of M's rows -- except the
// block i >= Q, j < Q, which is qg^T and keeps the tiled transpose above.
// One block streams kOdRowChunk entries of one OD row, 8 loads in flight per
// thread; same arithmetic (rr_od) as the transposing kernel.
constexpr int kOdRowChunk = 2048;
__global__ void __launch_bounds__(256)
rerank_build_od_rows_kernel(RrIn in, int64_t Q, int64_t G, const float* __restrict__ colmax,
                            float* __restrict__ od, int64_t ldo) {
  const int64_t N = Q + G;
  const int64_t i = blockIdx.y;
  // row i's sources: [0, Q) from qq (i < Q) -- none for i >= Q (qg^T, tiled
  // kernel); [Q, N) from qg (i < Q) or gg (i >= Q)
  const int64_t jlo = i < Q ? 0 : Q;
  const int64_t j0 = jlo + blockIdx.x * (int64_t)kOdRowChunk;
  if (j0 >= N) return;
  const float cm = colmax[i];
  float* orow = od + i * ldo;
  float m[kOdRowChunk / 256];
#pragma unroll
  for (int u = 0; u < kOdRowChunk / 256; ++u) {
    const int64_t j = j0 + u * 256 + threadIdx.x;
    m[u] = 0.f;
    if (j < N)
      m[u] = j < Q ? in.qq[i * in.ldqq + j]
                   : (i < Q ? in.qg[i * in.ldqg + (j - Q)] : in.gg[(i - Q) * in.ldgg + (j - Q)]);
  }
#pragma unroll
  for (int u = 0; u < kOdRowChunk / 256; ++u) {
    const int64_t j = j0 + u * 256 + threadIdx.x;
    if (j < N) orow[j] = rr_od(m[u], cm);
  }
}

// q_g^T [G][ldT] for the in-place path (the one block of M that is not a
// row of an input): 64 x 64 tiles through LDS, 256-byte row pieces both ways
__global__ void __launch_bounds__(256)
rerank_transpose_kernel(const float* __restrict__ qg, int64_t ldqg, int64_t Q, int64_t G,
                        float* __restrict__ qgT, int64_t ldT) {
  __shared__ float tile[64][65];
  const int64_t q0 = blockIdx.y * 64ll, g0 = blockIdx.x * 64ll;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int k = ty; k < 64; k += 4) {
    const int64_t q = q0 + k, g = g0 + tx;
    tile[k][tx] = (q < Q && g < G) ? qg[q * ldqg + g] : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 64; k += 4) {
    const int64_t g = g0 + k, q = q0 + tx;
    if (g < G && q < Q) qgT[g * ldT + q] = tile[tx][k];
  }
}

// OD[i][j]: the dense buffer, or (OTF) computed from M in place
template <bool OTF>
__device__ inline float od_at(const float* od, int64_t ldo, const RrMatrix& M, int64_t i,
                              int64_t j) {
  return OTF ? M.od(i, j) : od[i * ldo + j];
}

// ---- 3) V rows -----------------------------------------------------------------
// One 64-lane wave per row i.  rank: [N][K1] (K1 = k1 + 1 <= 64), rank[i][0..K1).

// true if x is among rank[row][0, len): every load issued before the first
// compare (indices clamped to len - 1, a repeat of an entry inside the
// list), so a check costs one memory latency per 16 entries, not one per entry
__device__ inline bool in_row(const int32_t* rank, int K1, int row, int len, int x) {
  const int32_t* r = rank + (int64_t)row * K1;
  bool f = false;
  for (int t0 = 0; t0 < len; t0 += 16) {
    int32_t v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = r[min(t0 + u, len - 1)];
#pragma unroll
    for (int u = 0; u < 16; ++u) f |= v[u] == x;
  }
  return f;
}

// NumPy's float32 np.sum of a contiguous vector (pairwise_sum, PW_BLOCKSIZE
// 128: eight strided accumulators per block of <= 128, halves split at a
// multiple of 8) -- the same rounding sequence as the reference's
// np.sum(weight) (reid_dataset_evaluator.py:487).  D bounds the recursion.
template <int D>
__device__ float np_pairwise_sum(const float* a, int n) {
  if (n < 8) {
    float r = 0.f;
    for (int t = 0; t < n; ++t) r = r + a[t];
    return r;
  }
  if (n <= 128 || D == 0) {
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int t = 8;
    for (; t < n - (n % 8); t += 8)
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = r[j] + a[t + j];
    float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; t < n; ++t) res = res + a[t];
    return res;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  return np_pairwise_sum<(D > 0 ? D - 1 : 0)>(a, n2) +
         np_pairwise_sum<(D > 0 ? D - 1 : 0)>(a + n2, n - n2);
}

// Dynamic LDS (ints) of the V-row kernel: the expansion list (E2 = the
// expansion bound K1 + K1 * Kh rounded up to a power of two, the bitonic
// length), then the candidate table [K1][Kh] aliased afterwards by the unique
// list and its weights (2 * E2).  ~3 KB at k1 = 20: many rows per CU in flight.
struct VRowsLds {
  int E2, tab;
  VRowsLds(int K1, int Kh) {
    E2 = 1;
    while (E2 < K1 + K1 * Kh) E2 <<= 1;
    tab = K1 * Kh > 2 * E2 ? K1 * Kh : 2 * E2;
  }
  size_t bytes() const { return sizeof(int32_t) * (size_t)(E2 + tab); }
};

template <bool OTF>
__global__ void __launch_bounds__(64)
rerank_v_rows_kernel(const float* __restrict__ od, int64_t N, int64_t ldo,
                     const int32_t* __restrict__ rank, int K1, int Kh, int vcap, int E2,
                     int32_t* __restrict__ v_idx, float* __restrict__ v_val,
                     int32_t* __restrict__ v_cnt, RrMatrix M) {
  extern __shared__ int32_t vr_lds[];
  int32_t* exp_ = vr_lds;   // [E2] expansion list
  // candidate table [nR][Kh]: the candidate's forward neighbour, or -1 when
  // that neighbour does not list the candidate back; afterwards the unique
  // expansion entries and their weights
  int32_t* tab = vr_lds + E2;
  __shared__ int32_t R[64];
  int32_t* uq = tab;
  float* wv = reinterpret_cast<float*>(tab + E2);
  const int64_t i = blockIdx.x;
  const int lane = threadIdx.x;
  const unsigned long long below = (1ull << lane) - 1ull;
  // k-reciprocal neighbours of i: forward k1+1 list, kept if i is in their list
  const int f = lane < K1 ? rank[i * K1 + lane] : -1;
  const bool rec = lane < K1 && in_row(rank, K1, f, K1, (int)i);
  const unsigned long long bal = __ballot(rec);
  const int nR = __popcll(bal);
  if (rec) {
    R[__popcll(bal & below)] = f;
    exp_[__popcll(bal & below)] = f;
  }
  __syncthreads();
  // every candidate's reciprocal test at once (all loads in flight together)
  const int nc = nR * Kh;
  for (int e = lane; e < nc; e += 64) {
    const int jc = e / Kh, t = e - jc * Kh;
    const int cand = R[jc];
    const int cf = rank[(int64_t)cand * K1 + t];
    tab[e] = in_row(rank, K1, cf, Kh, cand) ? cf : -1;
  }
  __syncthreads();
  // expansion, candidate by candidate (the reference's order): a candidate's
  // set joins if more than 2/3 of it lies in R
  int s_n = nR;
  for (int jc = 0; jc < nR; ++jc) {
    const int cf = lane < Kh ? tab[jc * Kh + lane] : -1;
    const bool crec = cf >= 0;
    const unsigned long long cb = __ballot(crec);
    const int ncr = __popcll(cb);
    bool inR = false;
    if (crec)
      for (int t = 0; t < nR; ++t) inR |= (R[t] == cf);
    const int inter = __popcll(__ballot(crec && inR));
    if (3 * inter > 2 * ncr) {  // len(intersect) > 2/3 * len(candidate set)
      const int p = s_n + __popcll(cb & below);
      if (crec && p < E2) exp_[p] = cf;
      s_n += ncr;
    }
  }
  __syncthreads();
  const int n = min(s_n, E2);   // s_n <= K1 + K1 * Kh <= E2
  // np.unique: sort (bitonic over the next power of two) and drop repeats
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  for (int t = n + lane; t < n2; t += 64) exp_[t] = 0x7fffffff;
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = lane; t < n2 / 2; t += 64) {
        const int a = 2 * stride * (t / stride) + (t % stride), b = a + stride;
        const bool up = (a & size) == 0;
        const int x = exp_[a], y = exp_[b];
        if ((x > y) == up) { exp_[a] = y; exp_[b] = x; }
      }
      __syncthreads();
    }
  // compact the unique entries (a ballot per 64) and weight them in parallel
  int u = 0;
  for (int b0 = 0; b0 < n; b0 += 64) {
    const int t = b0 + lane;
    const int x = t < n ? exp_[t] : 0;
    const bool first = t < n && (t == 0 || exp_[t - 1] != x);
    const unsigned long long fb = __ballot(first);
    if (first) uq[u + __popcll(fb & below)] = x;
    u += __popcll(fb);
  }
  __syncthreads();
  // weight = exp(-OD[i, idx]); V = weight / np.sum(weight) (float32, index order)
  for (int t = lane; t < u; t += 64) wv[t] = expf(-od_at<OTF>(od, ldo, M, i, uq[t]));
  __syncthreads();
  float wsum = lane == 0 ? np_pairwise_sum<4>(wv, u) : 0.f;
  wsum = __shfl(wsum, 0);
  const int cap = min(u, vcap);
  for (int t = lane; t < cap; t += 64) {
    v_idx[i * vcap + t] = uq[t];
    v_val[i * vcap + t] = wv[t] / wsum;
  }
  if (lane == 0) v_cnt[i] = u;
}

// ---- 4) V_qe rows: mean of k2 sparse rows (row order = initial_rank order) ----
constexpr int kQeCap = 4096;
constexpr int kQeSmall = 512;   // rows with <= this many concatenated entries: one wave

// One wave per row whose k2 V rows hold <= kQeSmall entries together (the
// common case; 10 KB of LDS, so many rows per CU are in flight).  Same merge
// and the same column sums in row order t as rerank_vqe_kernel below, which
// takes the longer rows.
__global__ void __launch_bounds__(64)
rerank_vqe_wave_kernel(int64_t N, const int32_t* __restrict__ rank, int K1, int k2,
                       const int32_t* __restrict__ v_idx, const float* __restrict__ v_val,
                       const int32_t* __restrict__ v_cnt, int vcap, int qcap,
                       int32_t* __restrict__ q_idx, float* __restrict__ q_val,
                       int32_t* __restrict__ q_cnt, int32_t* __restrict__ col_cnt,
                       int32_t* __restrict__ ovf_rows, int32_t* __restrict__ ovf_n) {
  // the merged row: kcol[pos] / val[pos] at each entry's final position
  // (column, then row order t); 4-byte columns keep the block at ~8 KB of
  // LDS, so ~19 rows per CU are in flight
  __shared__ int32_t kcol[kQeSmall];
  __shared__ float val[kQeSmall];
  __shared__ int32_t lc[kQeSmall];
  __shared__ int s_off[65], s_row[64];
  const int64_t i = blockIdx.x;
  const int lane = threadIdx.x;
  const unsigned long long below = (1ull << lane) - 1ull;
  // row offsets: a wave prefix sum over the k2 (<= 64) rows
  const int r = lane < k2 ? rank[i * K1 + lane] : 0;
  const int len = lane < k2 ? min(v_cnt[r], vcap) : 0;
  int incl = len;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  const int n = __shfl(incl, 63);
  if (n > kQeSmall) {   // rerank_vqe_kernel's row
    if (lane == 0) ovf_rows[atomicAdd(ovf_n, 1)] = (int32_t)i;
    return;
  }
  if (lane < k2) {
    s_row[lane] = r;
    s_off[lane] = incl - len;
  }
  if (lane == 0) s_off[k2] = n;
  __syncthreads();
  auto list_of = [&](int e) {
    int t = 0;
    while (t + 1 < k2 && s_off[t + 1] <= e) ++t;
    return t;
  };
  for (int e = lane; e < n; e += 64) {
    const int t = list_of(e);
    lc[e] = v_idx[(int64_t)s_row[t] * vcap + (e - s_off[t])];
  }
  __syncthreads();
  for (int e = lane; e < n; e += 64) {
    const int t = list_of(e);
    const int32_t c = lc[e];
    int pos = e - s_off[t];
    for (int t2 = 0; t2 < k2; ++t2) {
      if (t2 == t) continue;
      int lo = s_off[t2], hi = s_off[t2 + 1];
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        const bool before = t2 < t ? lc[mid] <= c : lc[mid] < c;
        if (before) lo = mid + 1; else hi = mid;
      }
      pos += lo - s_off[t2];
    }
    kcol[pos] = c;
    val[pos] = v_val[(int64_t)s_row[t] * vcap + (e - s_off[t])];
  }
  __syncthreads();
  // a column's entries are consecutive in merged order; the lane at a segment's
  // first entry sums it left to right (row order t) and writes output slot =
  // the number of segment starts before it
  int u = 0;
  for (int b0 = 0; b0 < n; b0 += 64) {
    const int e = b0 + lane;
    const int32_t col = e < n ? kcol[e] : 0;
    const bool st = e < n && (e == 0 || kcol[e - 1] != col);
    const unsigned long long sb = __ballot(st);
    if (st) {
      float sum = val[e];
      for (int f = e + 1; f < n && kcol[f] == col; ++f) sum += val[f];
      const int slot = u + __popcll(sb & below);
      if (slot < qcap) {
        const float qv = sum / (float)k2;
        q_idx[i * qcap + slot] = (int32_t)col;
        q_val[i * qcap + slot] = qv;
        if (qv != 0.f) atomicAdd(&col_cnt[col], 1);   // the inverted index's column sizes
      }
    }
    u += __popcll(sb);
  }
  if (lane == 0) q_cnt[i] = u;
}

__device__ void vqe_row_long(int64_t i, const int32_t* __restrict__ rank, int K1, int k2,
                             const int32_t* __restrict__ v_idx,
                             const float* __restrict__ v_val,
                             const int32_t* __restrict__ v_cnt, int vcap, int qcap,
                             int32_t* __restrict__ q_idx, float* __restrict__ q_val,
                             int32_t* __restrict__ q_cnt, int32_t* __restrict__ col_cnt);

__global__ void rerank_vqe_kernel(int64_t N, const int32_t* __restrict__ rank, int K1, int k2,
                                  const int32_t* __restrict__ v_idx,
                                  const float* __restrict__ v_val,
                                  const int32_t* __restrict__ v_cnt, int vcap, int qcap,
                                  int32_t* __restrict__ q_idx, float* __restrict__ q_val,
                                  int32_t* __restrict__ q_cnt, int32_t* __restrict__ col_cnt,
                                  const int32_t* __restrict__ ovf_rows,
                                  const int32_t* __restrict__ ovf_n) {
  // the rows rerank_vqe_wave_kernel left: ovf_rows[0, *ovf_n), a block each
  for (int r = blockIdx.x; r < *ovf_n; r += gridDim.x) {
    __syncthreads();   // LDS reuse across rows
    vqe_row_long(ovf_rows[r], rank, K1, k2, v_idx, v_val, v_cnt, vcap, qcap, q_idx, q_val,
                 q_cnt, col_cnt);
  }
}

__device__ void vqe_row_long(int64_t i, const int32_t* __restrict__ rank, int K1, int k2,
                             const int32_t* __restrict__ v_idx,
                             const float* __restrict__ v_val,
                             const int32_t* __restrict__ v_cnt, int vcap, int qcap,
                             int32_t* __restrict__ q_idx, float* __restrict__ q_val,
                             int32_t* __restrict__ q_cnt, int32_t* __restrict__ col_cnt) {
  __shared__ unsigned long long key[kQeCap];  // (column << 32) | (t << 16) | slot
  __shared__ float val[kQeCap];
  __shared__ int32_t lc[kQeCap];              // the k2 rows' columns, concatenated
  __shared__ int s_off[65], s_row[64];
  const int tid = threadIdx.x, nt = blockDim.x;
  if (tid == 0) {
    int o = 0;
    for (int t = 0; t < k2; ++t) {
      const int r = rank[i * K1 + t];
      s_row[t] = r;
      s_off[t] = o;
      o += min(v_cnt[r], vcap);
    }
    s_off[k2] = o;
  }
  __syncthreads();
  const int n = min(s_off[k2], kQeCap);
  auto list_of = [&](int e) {   // the row t holding concatenated entry e
    int t = 0;
    while (t + 1 < k2 && s_off[t + 1] <= e) ++t;
    return t;
  };
  for (int e = tid; e < n; e += nt) {
    const int t = list_of(e);
    lc[e] = v_idx[(int64_t)s_row[t] * vcap + (e - s_off[t])];
  }
  __syncthreads();
  // Each V row is sorted by column (np.unique), so the (column, t) order of
  // all entries is a k2-way merge: an entry's position is its index in its
  // own row plus, in every other row t2, the entries with a smaller column
  // (or the same column and t2 < t) -- binary searches in LDS, no sort.
  for (int e = tid; e < n; e += nt) {
    const int t = list_of(e);
    const int32_t c = lc[e];
    int pos = e - s_off[t];
    for (int t2 = 0; t2 < k2; ++t2) {
      if (t2 == t) continue;
      int lo = s_off[t2], hi = min(s_off[t2 + 1], n);
      while (lo < hi) {   // first entry of row t2 with column > c (t2 < t) / >= c (t2 > t)
        const int mid = (lo + hi) >> 1;
        const bool before = t2 < t ? lc[mid] <= c : lc[mid] < c;
        if (before) lo = mid + 1; else hi = mid;
      }
      pos += lo - s_off[t2];
    }
    key[pos] = ((unsigned long long)(uint32_t)c << 32) | ((unsigned long long)t << 16) |
               (unsigned)pos;
    val[pos] = v_val[(int64_t)s_row[t] * vcap + (e - s_off[t])];
  }
  __syncthreads();
  // segmented sums per column in row order t (key order), then / k2.  Each
  // thread owns a contiguous run of entries; a segment is summed left to
  // right by the thread owning its first entry (the serial order), at the
  // output slot given by a block scan of the segment starts.
  __shared__ int s_scan[1024];
  const int per = (n + nt - 1) / nt;
  const int e0 = tid * per, e1 = min(n, e0 + per);
  auto is_start = [&](int e) {
    return e == 0 || (uint32_t)(key[e] >> 32) != (uint32_t)(key[e - 1] >> 32);
  };
  int cnt = 0;
  for (int e = e0; e < e1; ++e) cnt += is_start(e);
  s_scan[tid] = cnt;
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int t = 0; t < nt; ++t) {
      const int v = s_scan[t];
      s_scan[t] = run;
      run += v;
    }
    q_cnt[i] = run;
  }
  __syncthreads();
  int u = s_scan[tid];
  for (int e = e0; e < e1; ++e) {
    if (!is_start(e)) continue;
    const uint32_t col = (uint32_t)(key[e] >> 32);
    float sum = val[key[e] & 0xffff];
    for (int f = e + 1; f < n && (uint32_t)(key[f] >> 32) == col; ++f)
      sum += val[key[f] & 0xffff];
    if (u < qcap) {
      const float qv = sum / (float)k2;
      q_idx[i * qcap + u] = (int32_t)col;
      q_val[i * qcap + u] = qv;
      if (qv != 0.f) atomicAdd(&col_cnt[col], 1);
    }
    ++u;
  }
}

// ---- 5) inverted index (CSC) of V_qe ------------------------------------------
__global__ void rerank_csc_count_kernel(int64_t N, const int32_t* __restrict__ q_idx,
                                        const float* __restrict__ q_val,
                                        const int32_t* __restrict__ q_cnt, int qcap,
                                        int32_t* __restrict__ col_cnt) {
  const int64_t i = blockIdx.x;
  const int c = min(q_cnt[i], qcap);
  for (int e = threadIdx.x; e < c; e += blockDim.x)
    if (q_val[i * qcap + e] != 0.f) atomicAdd(&col_cnt[q_idx[i * qcap + e]], 1);
}

// single-block exclusive scan over tiles of 1024 x kScanU counts: a thread's
// kScanU consecutive counts are loaded together (one memory latency per tile,
// not one per count), summed, and the 1024 sums scanned by wave shuffles and
// the 16 wave totals; the tile total carries into the next tile
constexpr int kScanU = 8;
__global__ void __launch_bounds__(1024)
rerank_scan_kernel(int64_t N, const int32_t* __restrict__ cnt, int32_t* __restrict__ start) {
  __shared__ int32_t wtot[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int32_t carry = 0;
  for (int64_t base = 0; base < N; base += 1024 * kScanU) {
    const int64_t e0 = base + (int64_t)tid * kScanU;
    int32_t v[kScanU];
#pragma unroll
    for (int u = 0; u < kScanU; ++u) v[u] = e0 + u < N ? cnt[e0 + u] : 0;
    int32_t s = 0;
#pragma unroll
    for (int u = 0; u < kScanU; ++u) s += v[u];
    int32_t incl = s;
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t y = __shfl_up(incl, o);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    int32_t wb = 0, tot = 0;
    for (int w = 0; w < 16; ++w) {
      const int32_t x = wtot[w];
      if (w < wave) wb += x;
      tot += x;
    }
    int32_t run = carry + wb + incl - s;
#pragma unroll
    for (int u = 0; u < kScanU; ++u) {
      if (e0 + u < N) start[e0 + u] = run;
      run += v[u];
    }
    carry += tot;
    __syncthreads();   // wtot is rewritten by the next tile
  }
  if (tid == 0) start[N] = carry;
}

__global__ void rerank_csc_fill_kernel(int64_t N, const int32_t* __restrict__ q_idx,
                                       const float* __restrict__ q_val,
                                       const int32_t* __restrict__ q_cnt, int qcap,
                                       const int32_t* __restrict__ start,
                                       int32_t* __restrict__ fill, int32_t* __restrict__ csc_row,
                                       float* __restrict__ csc_val) {
  const int64_t i = blockIdx.x;
  const int c = min(q_cnt[i], qcap);
  for (int e = threadIdx.x; e < c; e += blockDim.x) {
    const float v = q_val[i * qcap + e];
    if (v == 0.f) continue;
    const int col = q_idx[i * qcap + e];
    const int slot = start[col] + atomicAdd(&fill[col], 1);
    csc_row[slot] = (int32_t)i;
    csc_val[slot] = v;
  }
}

// ---- 6) Jaccard + blend for the query rows ------------------------------------
// One block per query row i: temp_min over the gallery rows j >= Q (the only
// columns the result keeps, :518) accumulates min(V_qe[i][col], V_qe[j][col])
// column by column in increasing column order -- the reference's loop order
// (:503-510), so every tm[j] sums in the same sequence.  The inverted index's
// entries are staged into LDS kJacStage at a time (all loads of a stage in
// flight together); the per-column pass then only touches LDS, one barrier
// per column.
// 16 waves per block (two blocks per CU, the LDS row): the per-column pass
// and the blend are latency chains, so more waves in flight is what helps --
// Duke re-ranking 906 -> 845 (512 threads) -> 818 us (1024) vs 256 threads
constexpr int kJacThreads = 1024;
constexpr int kJacCols = 128;    // column metadata loaded per batch
constexpr int kJacStage = 1024;  // staged (row, value) entries
size_t jaccard_lds_bytes(int64_t G) {
  return sizeof(float) * (size_t)G + (sizeof(int32_t) + sizeof(float)) * kJacStage;
}
template <bool OTF>
__global__ void __launch_bounds__(kJacThreads)
rerank_jaccard_kernel(int64_t Q, int64_t N, const float* __restrict__ od, int64_t ldo,
                      RrMatrix M, const int32_t* __restrict__ q_idx,
                      const float* __restrict__ q_val, const int32_t* __restrict__ q_cnt,
                      int qcap, const int32_t* __restrict__ start,
                      const int32_t* __restrict__ csc_row, const float* __restrict__ csc_val,
                      float lam, float one_m_lam, float* __restrict__ out) {
  extern __shared__ float tm[];  // [G] temp_min of the gallery rows, then the stage
  const int64_t G = N - Q;
  int32_t* srow = reinterpret_cast<int32_t*>(tm + G);
  float* sval = reinterpret_cast<float*>(srow + kJacStage);
  __shared__ int m_off[kJacCols + 1], m_s0[kJacCols];
  __shared__ float m_a[kJacCols];
  __shared__ int s_wtot;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t i = blockIdx.x;
  for (int64_t j = tid; j < G; j += kJacThreads) tm[j] = 0.f;
  const int c = min(q_cnt[i], qcap);
  for (int e0 = 0; e0 < c; e0 += kJacCols) {
    const int nb = min(kJacCols, c - e0);
    // batch metadata: value, first entry and entry count of each column
    // (zero-valued columns contribute nothing: count 0), offsets by a scan
    int len = 0;
    if (tid < kJacCols) {
      float av = 0.f;
      int s0 = 0;
      if (tid < nb) {
        av = q_val[i * qcap + e0 + tid];
        if (av != 0.f) {
          const int col = q_idx[i * qcap + e0 + tid];
          s0 = start[col];
          len = start[col + 1] - s0;
        }
      }
      m_a[tid] = av;
      m_s0[tid] = s0;
      int incl = len;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      if (wave == 0 && lane == 63) s_wtot = incl;
      m_off[tid + 1] = incl;   // wave 1 adds wave 0's total below
    }
    __syncthreads();
    if (tid >= 64 && tid < kJacCols) m_off[tid + 1] += s_wtot;
    if (tid == 0) m_off[0] = 0;
    __syncthreads();
    int ca = 0;
    while (ca < nb) {
      // the longest run of columns [ca, cb) whose entries fit the stage
      int lo = ca, hi = nb;   // largest cb with m_off[cb] - m_off[ca] <= kJacStage
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (m_off[mid] - m_off[ca] <= kJacStage) lo = mid; else hi = mid - 1;
      }
      const int cb = lo;
      if (cb == ca) {   // one column longer than the stage: straight from memory
        const float av = m_a[ca];
        const int s0 = m_s0[ca], s1 = s0 + (m_off[ca + 1] - m_off[ca]);
        for (int s = s0 + tid; s < s1; s += kJacThreads) {
          const int64_t r = csc_row[s] - Q;
          if (r >= 0) tm[r] = tm[r] + fminf(av, csc_val[s]);
        }
        __syncthreads();
        ++ca;
        continue;
      }
      const int base = m_off[ca], tot = m_off[cb] - base;
      for (int f = tid; f < tot; f += kJacThreads) {
        int l2 = ca, h2 = cb - 1;   // column holding staged entry f: last m_off <= base + f
        while (l2 < h2) {
          const int mid = (l2 + h2 + 1) >> 1;
          if (m_off[mid] <= base + f) l2 = mid; else h2 = mid - 1;
        }
        const int s = m_s0[l2] + (base + f - m_off[l2]);
        srow[f] = csc_row[s];
        sval[f] = csc_val[s];
      }
      __syncthreads();
      for (int k = ca; k < cb; ++k) {   // column order
        const float av = m_a[k];
        for (int f = m_off[k] - base + tid; f < m_off[k + 1] - base; f += kJacThreads) {
          const int64_t r = srow[f] - Q;
          if (r >= 0) tm[r] = tm[r] + fminf(av, sval[f]);   // one row per column entry
        }
        __syncthreads();
      }
      ca = cb;
    }
  }
  __syncthreads();
  for (int64_t j = Q + tid; j < N; j += kJacThreads) {
    const float t = tm[j - Q];
    const float jac = 1.f - t / (2.f - t);
    const float wj = jac * one_m_lam;                          // rounded
    const float wo = od_at<OTF>(od, ldo, M, i, j) * lam;       // rounded
    out[i * (N - Q) + (j - Q)] = wj + wo;
  }
}

int topk(const float*, int64_t, int64_t, int64_t, int, float*, int32_t*, hipStream_t);

namespace {
struct RrLayout {  // V-row capacities of a (k1, k2) configuration
  int K1, Kh, vcap, qcap;
  RrLayout(int k1, int k2) {
    K1 = k1 + 1;
    Kh = (int)lrint(k1 / 2.0) + 1;  // int(np.around(k1 / 2.)) + 1
    const int vbound = K1 + K1 * Kh;
    vcap = vbound <= 256 ? 256 : (vbound <= 512 ? 512 : 1024);
    qcap = k2 * vcap;
  }
};
}  // namespace

// The N x N OD region of a call: the dense normalised distance, or in place
// (symmetric, N >= 16384, 16-byte block rows) only q_g^T ([G][Q rounded up to
// 4]; none with PPS_RERANK_WHOLE, where it is M's lower-left block) plus the
// squared top-k's scratch.  The OD region is the workspace's first carve, so
// its base is the workspace's (256-B aligned) and decides nothing here.
static bool rr_inplace(const float* qg, int64_t ldqg, const float* qq, int64_t ldqq,
                       const float* gg, int64_t ldgg, int64_t Q, int64_t G, int K1, int flags,
                       float* od) {
  const bool whole = (flags & PPS_RERANK_WHOLE) != 0;
  const RrMatrix M{qg, qq, gg, whole ? qq + Q * ldqq : od, ldqg, ldqq, ldgg,
                   whole ? ldqq : (Q + 3) / 4 * 4, Q, G, nullptr};
  return (flags & PPS_RERANK_SYMMETRIC) && topk_rr_eligible(M, K1) &&
         getenv_flag_off("PPS_RERANK_INPLACE") == false;
}

static size_t rr_od_bytes(bool inplace, bool whole, int64_t Q, int64_t G, int K1) {
  const int64_t N = Q + G;
  if (!inplace) return sizeof(float) * (size_t)(N * od_stride(N));
  const size_t tb = whole ? 0 : (sizeof(float) * (size_t)(G * ((Q + 3) / 4 * 4)) + 255) / 256 * 256;
  return tb + topk_rr_sq_scratch_bytes(N, K1);
}

// Everything past the OD region
static size_t rr_rest_bytes(int64_t Q, int64_t G, int k1, int k2) {
  const int64_t N = Q + G;
  const RrLayout L(k1, k2);
  const int64_t K1 = L.K1, vcap = L.vcap, qcap = L.qcap;
  auto r = [](size_t b) { return (b + 255) / 256 * 256; };
  size_t s = r(4 * N) + r(4 * N * K1) * 2 + r(4 * N * vcap) * 2 + r(4 * N);
  s += r(4 * N * qcap) * 2 + r(4 * N) + r(4 * (N + 1)) * 3 + r(4 * N * qcap) * 2;
  s += r(4 * N) + r(4);   // V_qe overflow rows + count
  return s;
}

int rerank(const float* qg, int64_t ldqg, const float* qq, int64_t ldqq, const float* gg,
           int64_t ldgg, int64_t Q, int64_t G, int k1, int k2, double lambda, void* ws,
           size_t ws_bytes, float* out, hipStream_t st, int flags) {
  // NumPy (NEP 50) casts the Python-float factors to float32: lambda and 1-lambda
  const float lam = (float)lambda, one_m_lam = (float)(1.0 - lambda);
  const int64_t N = Q + G;
  const int64_t ldo = od_stride(N);
  const RrLayout L(k1, k2);
  const int K1 = L.K1, Kh = L.Kh, vcap = L.vcap, qcap = L.qcap;
  const int64_t ldT = (Q + 3) / 4 * 4;
  const bool whole = (flags & PPS_RERANK_WHOLE) != 0;
  const bool inplace = rr_inplace(qg, ldqg, qq, ldqq, gg, ldgg, Q, G, K1, flags,
                                  reinterpret_cast<float*>(ws));
  const size_t odb = rr_od_bytes(inplace, whole, Q, G, K1);
  // workspace carve-up (all 256-B aligned)
  char* p = reinterpret_cast<char*>(ws);
  auto take = [&](size_t bytes) {
    char* r = p;
    p += (bytes + 255) / 256 * 256;
    return r;
  };
  float* od = reinterpret_cast<float*>(take(odb));
  float* colmax = reinterpret_cast<float*>(take(sizeof(float) * N));
  float* topv = reinterpret_cast<float*>(take(sizeof(float) * N * K1));
  int32_t* rank = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * N * K1));
  int32_t* v_idx = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * N * vcap));
  float* v_val = reinterpret_cast<float*>(take(sizeof(float) * N * vcap));
  int32_t* v_cnt = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * N));
  int32_t* q_idx = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * N * qcap));
  float* q_val = reinterpret_cast<float*>(take(sizeof(float) * N * qcap));
  int32_t* q_cnt = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * N));
  int32_t* col_cnt = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (N + 1)));
  int32_t* start = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (N + 1)));
  int32_t* fill = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * (N + 1)));
  int32_t* csc_row = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * N * qcap));
  float* csc_val = reinterpret_cast<float*>(take(sizeof(float) * N * qcap));
  int32_t* ovf_rows = reinterpret_cast<int32_t*>(take(sizeof(int32_t) * N));
  int32_t* ovf_n = reinterpret_cast<int32_t*>(take(sizeof(int32_t)));
  if ((size_t)(p - reinterpret_cast<char*>(ws)) > ws_bytes) {
    set_error("rerank workspace too small: need " +
              std::to_string((size_t)(p - reinterpret_cast<char*>(ws))) + " bytes");
    return PPS_ERR_CAPACITY;
  }
  const RrIn in{qg, qq, gg, ldqg, ldqq, ldgg};
  // In place (symmetric M, long rows, 16-byte rows): no N x N OD buffer --
  // its top-k, the V weights and the Jaccard blend read M's blocks and
  // compute (m * m) / colmax on the fly; q_g^T (the block that is nobody's
  // row) goes where OD would start.
  // PPS_RERANK_WHOLE: q_g^T is the matrix's own lower-left block
  RrMatrix M{qg, qq, gg, whole ? qq + Q * ldqq : od, ldqg, ldqq, ldgg, whole ? ldqq : ldT,
             Q, G, colmax};
  // colmax = np.max(M^2, axis=0) (:453), from the four blocks of M (in place:
  // the top-k pass computes it, = the row maxima of the symmetric M)
  unsigned* cm = reinterpret_cast<unsigned*>(colmax);
  if (!inplace) (void)hipMemsetAsync(cm, 0, sizeof(unsigned) * N, st);
  auto colmax_sq = [&](const float* x, int64_t R, int64_t C, int64_t ld, unsigned* o) {
    if (R <= 0 || C <= 0 || inplace) return;
    hipLaunchKernelGGL(rerank_colmax_sq_kernel,
                       dim3((unsigned)((C + 255) / 256), (unsigned)((R + kCmRows - 1) / kCmRows)),
                       dim3(256), 0, st, x, R, C, ld, o);
  };
  colmax_sq(qq, Q, Q, ldqq, cm);      // columns c < Q: rows r < Q
  colmax_sq(qg, Q, G, ldqg, cm + Q);  // columns c >= Q: rows r < Q
  colmax_sq(gg, G, G, ldgg, cm + Q);  // columns c >= Q: rows r >= Q
  if (!inplace)
    hipLaunchKernelGGL(rerank_rowmax_sq_kernel, dim3((unsigned)Q), dim3(256), 0, st, qg, G, ldqg,
                       cm);       // columns c < Q: rows r >= Q (qg^T)
  PPS_CHECK_LAUNCH_S("rerank_colmax_sq_kernel", st);
  constexpr int T = PPS_OD_TILE;
  if (inplace) {
    if (!whole) {
      hipLaunchKernelGGL(rerank_transpose_kernel,
                         dim3((unsigned)((G + 63) / 64), (unsigned)((Q + 63) / 64)), dim3(256), 0,
                         st, qg, ldqg, Q, G, od, ldT);
      PPS_CHECK_LAUNCH_S("rerank_transpose_kernel", st);
    }
    // scratch for the squared top-k: the OD region past q_g^T
    const size_t tb = whole ? 0 : (sizeof(float) * (size_t)(G * ldT) + 255) / 256 * 256;
    const int rc = topk_rr_sq(M, K1, colmax, reinterpret_cast<char*>(od) + tb, odb - tb, topv,
                              rank, st);
    if (rc != PPS_OK) return rc;
  } else {
    if (flags & PPS_RERANK_SYMMETRIC) {
      // rows streamed from M's rows; only the qg^T block (i >= Q, j < Q) is
      // transposed
      hipLaunchKernelGGL(rerank_build_od_rows_kernel,
                         dim3((unsigned)((N + kOdRowChunk - 1) / kOdRowChunk), (unsigned)N),
                         dim3(256), 0, st, in, Q, G, colmax, od, ldo);
      PPS_CHECK_LAUNCH_S("rerank_build_od_rows_kernel", st);
      const int64_t ti = (N + T - 1) / T - Q / T;   // row tiles covering [Q, N)
      hipLaunchKernelGGL(rerank_build_od_kernel<T>, dim3((unsigned)((Q + T - 1) / T), (unsigned)ti),
                         dim3(256), 0, st, in, Q, G, colmax, od, ldo, Q, Q);
    } else {
      hipLaunchKernelGGL(rerank_build_od_kernel<T>, dim3((unsigned)((N + T - 1) / T),
                                                         (unsigned)((N + T - 1) / T)),
                         dim3(256), 0, st, in, Q, G, colmax, od, ldo, (int64_t)0, N);
    }
    PPS_CHECK_LAUNCH_S("rerank_build_od_kernel", st);
    const int rc = topk(od, N, N, ldo, K1, topv, rank, st);
    if (rc != PPS_OK) return rc;
  }
  PPS_CHECK_LAUNCH_S("rerank topk", st);
  if (debug_sync()) {  // every neighbour index must address a row of OD
    std::vector<int32_t> h((size_t)(N * K1));
    (void)hipMemcpy(h.data(), rank, h.size() * sizeof(int32_t), hipMemcpyDeviceToHost);
    for (size_t t = 0; t < h.size(); ++t)
      if (h[t] < 0 || h[t] >= N) {
        set_error("rerank topk: rank[" + std::to_string(t / K1) + "][" +
                  std::to_string(t % K1) + "] = " + std::to_string(h[t]));
        return PPS_ERR_LAUNCH;
      }
  }
  const VRowsLds vl(K1, Kh);
  if (inplace)
    hipLaunchKernelGGL(rerank_v_rows_kernel<true>, dim3((unsigned)N), dim3(64), vl.bytes(), st, od,
                       N, ldo, rank, K1, Kh, vcap, vl.E2, v_idx, v_val, v_cnt, M);
  else
    hipLaunchKernelGGL(rerank_v_rows_kernel<false>, dim3((unsigned)N), dim3(64), vl.bytes(), st,
                       od, N, ldo, rank, K1, Kh, vcap, vl.E2, v_idx, v_val, v_cnt, M);
  PPS_CHECK_LAUNCH_S("rerank_v_rows_kernel", st);
  // the V_qe kernels also count the inverted index's column sizes
  (void)hipMemsetAsync(col_cnt, 0, sizeof(int32_t) * (N + 1), st);
  if (k2 != 1) {
    (void)hipMemsetAsync(ovf_n, 0, sizeof(int32_t), st);
    hipLaunchKernelGGL(rerank_vqe_wave_kernel, dim3((unsigned)N), dim3(64), 0, st, N, rank, K1,
                       k2, v_idx, v_val, v_cnt, vcap, qcap, q_idx, q_val, q_cnt, col_cnt,
                       ovf_rows, ovf_n);
    PPS_CHECK_LAUNCH_S("rerank_vqe_wave_kernel", st);
    hipLaunchKernelGGL(rerank_vqe_kernel, dim3(256), dim3(256), 0, st, N, rank, K1, k2, v_idx,
                       v_val, v_cnt, vcap, qcap, q_idx, q_val, q_cnt, col_cnt, ovf_rows, ovf_n);
    PPS_CHECK_LAUNCH_S("rerank_vqe_kernel", st);
  } else {
    (void)hipMemcpyAsync(q_idx, v_idx, sizeof(int32_t) * N * vcap, hipMemcpyDeviceToDevice, st);
    (void)hipMemcpyAsync(q_val, v_val, sizeof(float) * N * vcap, hipMemcpyDeviceToDevice, st);
    (void)hipMemcpyAsync(q_cnt, v_cnt, sizeof(int32_t) * N, hipMemcpyDeviceToDevice, st);
  }
  const int qc = k2 != 1 ? qcap : vcap;
  (void)hipMemsetAsync(fill, 0, sizeof(int32_t) * (N + 1), st);
  if (k2 == 1) {   // V_qe = V: count here
    hipLaunchKernelGGL(rerank_csc_count_kernel, dim3((unsigned)N), dim3(256), 0, st, N, q_idx,
                       q_val, q_cnt, qc, col_cnt);
    PPS_CHECK_LAUNCH_S("rerank_csc_count_kernel", st);
  }
  hipLaunchKernelGGL(rerank_scan_kernel, dim3(1), dim3(1024), 0, st, N, col_cnt, start);
  PPS_CHECK_LAUNCH_S("rerank_scan_kernel", st);
  hipLaunchKernelGGL(rerank_csc_fill_kernel, dim3((unsigned)N), dim3(256), 0, st, N, q_idx,
                     q_val, q_cnt, qc, start, fill, csc_row, csc_val);
  PPS_CHECK_LAUNCH_S("rerank_csc_fill_kernel", st);
  const size_t jac_lds = jaccard_lds_bytes(G);
  if (inplace)
    hipLaunchKernelGGL(rerank_jaccard_kernel<true>, dim3((unsigned)Q), dim3(kJacThreads), jac_lds,
                       st, Q, N, od, ldo, M, q_idx, q_val, q_cnt, qc, start, csc_row, csc_val, lam,
                       one_m_lam, out);
  else
    hipLaunchKernelGGL(rerank_jaccard_kernel<false>, dim3((unsigned)Q), dim3(kJacThreads), jac_lds,
                       st, Q, N, od, ldo, M, q_idx, q_val, q_cnt, qc, start, csc_row, csc_val, lam,
                       one_m_lam, out);
  PPS_CHECK_LAUNCH_S("rerank_jaccard_kernel", st);
  return PPS_OK;
}

size_t rerank_workspace_bytes(int64_t Q, int64_t G, int k1, int k2) {
  // the dense path's size: enough for every call with these shapes
  return (rr_od_bytes(false, false, Q, G, k1 + 1) + 255) / 256 * 256 + rr_rest_bytes(Q, G, k1, k2);
}

size_t rerank_workspace_bytes_for(const float* qg, int64_t ldqg, const float* qq, int64_t ldqq,
                                  const float* gg, int64_t ldgg, int64_t Q, int64_t G, int k1,
                                  int k2, int flags) {
  // the OD region's base is 256-B aligned: any such pointer stands in for it
  float* od_probe = reinterpret_cast<float*>((uintptr_t)256);
  const bool inplace = rr_inplace(qg, ldqg, qq, ldqq, gg, ldgg, Q, G, k1 + 1, flags, od_probe);
  const size_t odb = rr_od_bytes(inplace, (flags & PPS_RERANK_WHOLE) != 0, Q, G, k1 + 1);
  return (odb + 255) / 256 * 256 + rr_rest_bytes(Q, G, k1, k2);
}

}  // namespace pps
