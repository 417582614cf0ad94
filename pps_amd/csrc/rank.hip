// Retrieval ranking and evaluation kernels.
//
// The reference sorts every query row (np.argsort, reid_dataset_evaluator.py
// :319,:420) and then walks it in Python.  mAP and CMC only need, for each
// true match p of a query, how many valid gallery entries rank before it, so
// these kernels compute exactly that by counting against the (few) positives'
// distances -- one streaming read of the distance row, no sort.  The result
// equals a stable (distance, gallery index) sort; counts are additive over
// gallery shards, which is what the multi-GPU path all-reduces.
#include <cstdlib>

#include "gemm_common.hpp"

namespace pps {

constexpr int kEvalThreads = 256;
constexpr int kPosCap = 2048;  // max merged positives per query in LDS

// ---- 1) collect positives ------------------------------------------------------
// One block per query; wave w scans its own contiguous quarter of the gallery
// (count, then write at its offset), compacting with ballots -- no block
// barrier inside the scan.  The list keeps ascending gallery order.  The id /
// cam arrays are L2-resident, so the scan is bound by load latency: each
// thread issues kCpU groups' loads before testing any, and the first pass
// keeps its 64-entry ballot masks in LDS (up to kMaskCap groups per wave) so
// the writing pass re-reads ids only beyond that.
constexpr int kCpU = 4;
constexpr int kMaskCap = 256;
__global__ void collect_positives_kernel(const float* __restrict__ dist, int64_t G,
                                         int64_t ldd, const int32_t* __restrict__ qid,
                                         const int32_t* __restrict__ qcam,
                                         const int32_t* __restrict__ gid,
                                         const int32_t* __restrict__ gcam,
                                         int64_t g_offset, int Pmax,
                                         float* __restrict__ pos_d,
                                         int32_t* __restrict__ pos_idx,
                                         int32_t* __restrict__ pos_cnt) {
  const int64_t q = blockIdx.x;
  const int qi = qid[q], qc = qcam[q];
  const float* row = dist + q * ldd;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int W = kEvalThreads / 64;
  __shared__ int wtot[W];
  __shared__ unsigned long long masks[W][kMaskCap];
  const int64_t chunk = ((G + W - 1) / W + 63) / 64 * 64;
  const int64_t beg = wave * chunk;
  const int64_t end = beg + chunk < G ? beg + chunk : G;
  const unsigned long long below = (1ull << lane) - 1ull;
  // buffer loads: entries at or past G read 0 without a branch (masked below)
  const rsrc_t rid = make_rsrc(gid, (uint32_t)(G * 4));
  const rsrc_t rcam = make_rsrc(gcam, (uint32_t)(G * 4));
  auto group_flags = [&](int64_t t0, bool* f) {
    int a[kCpU], c[kCpU];
#pragma unroll
    for (int u = 0; u < kCpU; ++u) {
      const int off = (int)((t0 + 64 * u + lane) * 4);
      a[u] = __builtin_amdgcn_raw_buffer_load_b32(rid, off, 0, 0);
      c[u] = __builtin_amdgcn_raw_buffer_load_b32(rcam, off, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kCpU; ++u)
      f[u] = (t0 + 64 * u + lane < end) && a[u] == qi && c[u] != qc;
  };
  int cnt = 0;
  for (int64_t t0 = beg, g = 0; t0 < end; t0 += 64 * kCpU, g += kCpU) {
    bool f[kCpU];
    group_flags(t0, f);
#pragma unroll
    for (int u = 0; u < kCpU; ++u) {
      const unsigned long long bal = __ballot(f[u]);
      if (g + u < kMaskCap && lane == 0) masks[wave][g + u] = bal;
      cnt += __popcll(bal);
    }
  }
  if (lane == 0) wtot[wave] = cnt;
  __syncthreads();
  int slot = 0, total = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    slot += w < wave ? wtot[w] : 0;
    total += wtot[w];
  }
  if (slot < Pmax && cnt > 0) {
    for (int64_t t0 = beg, g = 0; t0 < end && slot < Pmax; t0 += 64 * kCpU, g += kCpU) {
      unsigned long long bal[kCpU];
      if (g + kCpU <= kMaskCap) {
#pragma unroll
        for (int u = 0; u < kCpU; ++u) bal[u] = masks[wave][g + u];
      } else {
        bool f[kCpU];
        group_flags(t0, f);
#pragma unroll
        for (int u = 0; u < kCpU; ++u) bal[u] = __ballot(f[u]);
      }
#pragma unroll
      for (int u = 0; u < kCpU; ++u) {
        const int64_t i = t0 + 64 * u + lane;
        const bool flag = (bal[u] >> lane) & 1ull;
        const int s = slot + __popcll(bal[u] & below);
        if (flag && s < Pmax) {
          pos_d[q * Pmax + s] = row[i];
          pos_idx[q * Pmax + s] = (int32_t)(g_offset + i);
        }
        slot += __popcll(bal[u]);
      }
    }
  }
  if (threadIdx.x == 0) pos_cnt[q] = total;
}

int collect_positives(const float* dist, int64_t Q, int64_t G, int64_t ldd,
                      const int32_t* qid, const int32_t* qcam, const int32_t* gid,
                      const int32_t* gcam, int64_t g_offset, int Pmax, float* pos_d,
                      int32_t* pos_idx, int32_t* pos_cnt, hipStream_t st) {
  if (Q <= 0) return PPS_OK;
  hipLaunchKernelGGL(collect_positives_kernel, dim3((unsigned)Q), dim3(kEvalThreads), 0,
                     st, dist, G, ldd, qid, qcam, gid, gcam, g_offset, Pmax, pos_d,
                     pos_idx, pos_cnt);
  PPS_CHECK_LAUNCH("collect_positives_kernel");
  return PPS_OK;
}

// ---- 2) rank counts -------------------------------------------------------------
__device__ inline bool key_less(float da, int ia, float db, int ib) {
  return da < db || (da == db && ia < ib);
}

__global__ void rank_counts_kernel(const float* __restrict__ dist, int64_t Q, int64_t G,
                                   int64_t ldd, const int32_t* __restrict__ qid,
                                   const int32_t* __restrict__ qcam,
                                   const int32_t* __restrict__ gid,
                                   const int32_t* __restrict__ gcam, int64_t g_offset,
                                   int R, int Pmax, const float* __restrict__ pos_d,
                                   const int32_t* __restrict__ pos_idx,
                                   const int32_t* __restrict__ pos_cnt,
                                   float* __restrict__ sorted_d,
                                   int32_t* __restrict__ sorted_idx,
                                   int32_t* __restrict__ pos_total,
                                   int32_t* __restrict__ hist,
                                   int32_t* __restrict__ before) {
  const int64_t q = blockIdx.x;
  const int Ptot = R * Pmax;
  const int qi = qid[q], qc = qcam[q];
  // positive lists in dynamic LDS sized to R*Pmax (<= kPosCap): tens of
  // entries on real splits, so several blocks share a CU and keep enough
  // row loads in flight (a fixed 40 KB allowed three)
  extern __shared__ int dyn_lds[];
  float* ud = reinterpret_cast<float*>(dyn_lds);
  int* ui = dyn_lds + Ptot;
  float* sd = reinterpret_cast<float*>(dyn_lds + 2 * Ptot);
  int* si = dyn_lds + 3 * Ptot;
  int* hs = dyn_lds + 4 * Ptot;
  __shared__ int offs[65];
  __shared__ int red[kEvalThreads / 64];
  // merged list layout: list r occupies [offs[r], offs[r+1])
  if (threadIdx.x == 0) {
    int o = 0;
    for (int r = 0; r < R; ++r) {
      offs[r] = o;
      const int c = pos_cnt[(int64_t)r * Q + q];
      o += c < Pmax ? c : Pmax;
    }
    offs[R] = o;
  }
  __syncthreads();
  const int P = offs[R];
  for (int r = 0; r < R; ++r) {
    const int n = offs[r + 1] - offs[r];
    for (int p = threadIdx.x; p < n; p += blockDim.x) {
      ud[offs[r] + p] = pos_d[((int64_t)r * Q + q) * Pmax + p];
      ui[offs[r] + p] = pos_idx[((int64_t)r * Q + q) * Pmax + p];
    }
  }
  for (int p = threadIdx.x; p < P; p += blockDim.x) hs[p] = 0;
  __syncthreads();
  // rank-by-counting sort of the positives (P is small: tens per query)
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    const float d = ud[p];
    const int ix = ui[p];
    int rk = 0;
    for (int o = 0; o < P; ++o) rk += key_less(ud[o], ui[o], d, ix) ? 1 : 0;
    sd[rk] = d;
    si[rk] = ix;
  }
  __syncthreads();
  for (int p = threadIdx.x; p < Ptot; p += blockDim.x) {
    sorted_d[q * Ptot + p] = p < P ? sd[p] : INFINITY;
    sorted_idx[q * Ptot + p] = p < P ? si[p] : -1;
  }
  if (threadIdx.x == 0) pos_total[q] = P;
  const float df = P > 0 ? sd[0] : 0.f;
  const int64_t idf = P > 0 ? si[0] : 0;
  const float* row = dist + q * ldd;
  int nbefore = 0;
  if (P > 0) {
    // Entries farther than the farthest positive change neither the histogram
    // (their bin would be P) nor the first-match count: only the closer ones
    // (a few % of a row) are searched against the positives.
    const float dmax = sd[P - 1];
    auto visit = [&](int64_t i, float d) {
      if (d > dmax) return;
      if (gid[i] == qi && gcam[i] == qc) return;  // junk: same id, same cam
      int lo = 0, hi = P;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sd[mid] < d) lo = mid + 1; else hi = mid;
      }
      if (lo < P) atomicAdd(&hs[lo], 1);
      nbefore += (d < df || (d == df && g_offset + i < idf)) ? 1 : 0;
    };
    // The row is streamed as 16-byte vectors: a scalar head up to the first
    // 16-byte boundary (rows of odd length start unaligned), U float4 loads
    // in flight per thread, a scalar tail.  visit() only accumulates
    // order-free counts, so the visiting order does not matter.
    const int64_t head0 = (int64_t)(((16 - ((uintptr_t)row & 15)) & 15) >> 2);
    const int64_t head = head0 < G ? head0 : G;
    const int64_t nb = (G - head) >> 2;
    if (threadIdx.x < head) visit(threadIdx.x, row[threadIdx.x]);
    const float4* body = reinterpret_cast<const float4*>(row + head);
    // ids / cams of the same entries are fetched together with the distances
    // (buffer loads: L2-resident arrays, past-the-end reads return 0): with
    // 64 lanes nearly every element slot of a wave has an entry closer than
    // the farthest positive, and a dependent id fetch per slot made the scan
    // latency-bound (242 -> 115 -> this)
    const rsrc_t rid = make_rsrc(gid, (uint32_t)(G * 4));
    const rsrc_t rcam = make_rsrc(gcam, (uint32_t)(G * 4));
    auto binned = [&](int64_t i, float d, int id, int cam) {
      if (d > dmax || (id == qi && cam == qc)) return;
      int lo = 0, hi = P;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sd[mid] < d) lo = mid + 1; else hi = mid;
      }
      if (lo < P) atomicAdd(&hs[lo], 1);
      nbefore += (d < df || (d == df && g_offset + i < idf)) ? 1 : 0;
    };
    constexpr int U = 4;
    const int64_t step = (int64_t)blockDim.x * U;
    for (int64_t j0 = threadIdx.x; j0 < nb; j0 += step) {
      float4 v[U];
      int id[U][4], cam[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t j = j0 + (int64_t)u * blockDim.x;
        v[u] = j < nb ? body[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        const int off = (int)((head + 4 * j) * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          id[u][e] = __builtin_amdgcn_raw_buffer_load_b32(rid, off + 4 * e, 0, 0);
          cam[u][e] = __builtin_amdgcn_raw_buffer_load_b32(rcam, off + 4 * e, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t j = j0 + (int64_t)u * blockDim.x;
        if (j < nb) {
          const int64_t i = head + 4 * j;
          binned(i, v[u].x, id[u][0], cam[u][0]);
          binned(i + 1, v[u].y, id[u][1], cam[u][1]);
          binned(i + 2, v[u].z, id[u][2], cam[u][2]);
          binned(i + 3, v[u].w, id[u][3], cam[u][3]);
        }
      }
    }
    const int64_t t = head + 4 * nb + threadIdx.x;
    if (t < G) visit(t, row[t]);
  }
  for (int o = 32; o > 0; o >>= 1) nbefore += __shfl_xor(nbefore, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = nbefore;
  __syncthreads();
  for (int p = threadIdx.x; p < P; p += blockDim.x) hist[q * Ptot + p] += hs[p];
  if (threadIdx.x == 0) {
    int s = 0;
    for (int w = 0; w < kEvalThreads / 64; ++w) s += red[w];
    before[q] += s;
  }
}

int rank_counts(const float* dist, int64_t Q, int64_t G, int64_t ldd, const int32_t* qid,
                const int32_t* qcam, const int32_t* gid, const int32_t* gcam,
                int64_t g_offset, int R, int Pmax, const float* pos_d,
                const int32_t* pos_idx, const int32_t* pos_cnt, float* sorted_d,
                int32_t* sorted_idx, int32_t* pos_total, int32_t* hist, int32_t* before,
                hipStream_t st) {
  if (Q <= 0) return PPS_OK;
  if ((int64_t)R * Pmax > kPosCap) return PPS_ERR_CAPACITY;  // abi.hip reports it
  const size_t lds = (size_t)5 * R * Pmax * sizeof(int);
  hipLaunchKernelGGL(rank_counts_kernel, dim3((unsigned)Q), dim3(kEvalThreads), lds, st,
                     dist, Q, G, ldd, qid, qcam, gid, gcam, g_offset, R, Pmax, pos_d,
                     pos_idx, pos_cnt, sorted_d, sorted_idx, pos_total, hist, before);
  PPS_CHECK_LAUNCH("rank_counts_kernel");
  return PPS_OK;
}

// ---- streaming evaluation from a per-identity gallery index ---------------------
// The product path (v2).  A CSR index of the gallery (host-built once from the
// ids: `members` = local gallery indices sorted by (id, index); the query's
// identity occupies members[q_beg[q], q_end[q])) lets every query list its
// true matches directly -- tens of gathers instead of a scan of all G ids and
// cams -- split into positives (other camera) and junk (same camera,
// reid_dataset_evaluator.py:427-428).  The counting pass then needs no ids at
// all: it bins EVERY entry of the distance row against the sorted positives
// and afterwards takes the junk entries (known, few) back out, so the row is
// one pure 16-byte-vector stream of distances.
//
// a) collect_matches: one wave per query.
constexpr int kMatchWaves = 4;
__global__ void __launch_bounds__(64 * kMatchWaves)
collect_matches_kernel(const float* __restrict__ dist, int64_t Q, int64_t ldd,
                       const int32_t* __restrict__ qcam, const int32_t* __restrict__ gcam,
                       const int32_t* __restrict__ members,
                       const int32_t* __restrict__ q_beg, const int32_t* __restrict__ q_end,
                       int64_t g_offset, int Pmax, float* __restrict__ pos_d,
                       int32_t* __restrict__ pos_idx, int32_t* __restrict__ pos_cnt, int Jmax,
                       float* __restrict__ junk_d, int32_t* __restrict__ junk_idx,
                       int32_t* __restrict__ junk_cnt) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * kMatchWaves + (threadIdx.x >> 6);
  if (q >= Q) return;
  const int beg = q_beg[q], end = q_end[q], qc = qcam[q];
  const float* row = dist + q * ldd;
  const unsigned long long below = (1ull << lane) - 1ull;
  int np = 0, nj = 0;
  for (int m0 = beg; m0 < end; m0 += 64) {
    const int m = m0 + lane;
    const bool in = m < end;
    const int idx = in ? members[m] : 0;
    const bool pos = in && gcam[idx] != qc;
    const bool junk = in && !pos;
    const float d = in ? row[idx] : 0.f;
    const unsigned long long bp = __ballot(pos), bj = __ballot(junk);
    const int sp = np + __popcll(bp & below), sj = nj + __popcll(bj & below);
    if (pos && sp < Pmax) {
      pos_d[q * Pmax + sp] = d;
      pos_idx[q * Pmax + sp] = (int32_t)(g_offset + idx);
    }
    if (junk && sj < Jmax) {
      junk_d[q * Jmax + sj] = d;
      junk_idx[q * Jmax + sj] = (int32_t)(g_offset + idx);
    }
    np += __popcll(bp);
    nj += __popcll(bj);
  }
  if (lane == 0) {
    pos_cnt[q] = np;
    junk_cnt[q] = nj;
  }
}

int collect_matches(const float* dist, int64_t Q, int64_t ldd, const int32_t* qcam,
                    const int32_t* gcam, const int32_t* members, const int32_t* q_beg,
                    const int32_t* q_end, int64_t g_offset, int Pmax, float* pos_d,
                    int32_t* pos_idx, int32_t* pos_cnt, int Jmax, float* junk_d,
                    int32_t* junk_idx, int32_t* junk_cnt, hipStream_t st) {
  if (Q <= 0) return PPS_OK;
  const unsigned grid = (unsigned)((Q + kMatchWaves - 1) / kMatchWaves);
  hipLaunchKernelGGL(collect_matches_kernel, dim3(grid), dim3(64 * kMatchWaves), 0, st, dist,
                     Q, ldd, qcam, gcam, members, q_beg, q_end, g_offset, Pmax, pos_d, pos_idx,
                     pos_cnt, Jmax, junk_d, junk_idx, junk_cnt);
  PPS_CHECK_LAUNCH("collect_matches_kernel");
  return PPS_OK;
}

// Bin-lookup cells of a query (used by c)): (df, dmax] of its sorted positives
// cut into kStreamCells equal cells by a monotone map; cells[c] = the number
// of positives whose cell is below c, | kCellDirty if a positive lies in c.
constexpr int kStreamCells = 1024;
constexpr int kCellDirty = 1 << 30;
__device__ inline float cell_scale(float df, float dmax) {
  const float span = dmax - df;
  const float inv = span > 0.f ? (float)kStreamCells / span : 0.f;
  return isfinite(inv) ? inv : 0.f;  // a denormal span: one cell
}
__device__ inline int cell_of(float d, float df, float inv) {
  const float t = (d - df) * inv;
  const int c = t < (float)(kStreamCells - 1) ? (int)t : kStreamCells - 1;
  return c > 0 ? c : 0;
}

// b) rank_prepare: merge the R shards' positive lists of a query and sort
// them by (distance, global index) -- rank by counting in LDS (one block per
// query; tens of entries on real splits) -- and build its bin-lookup cells.
__global__ void rank_prepare_kernel(int R, int64_t Q, int Pmax, const float* __restrict__ pos_d,
                                    const int32_t* __restrict__ pos_idx,
                                    const int32_t* __restrict__ pos_cnt,
                                    float* __restrict__ sorted_d,
                                    int32_t* __restrict__ sorted_idx,
                                    int32_t* __restrict__ pos_total,
                                    int32_t* __restrict__ cells) {
  const int64_t q = blockIdx.x;
  const int Ptot = R * Pmax;
  extern __shared__ int plds[];
  float* ud = reinterpret_cast<float*>(plds);
  int* ui = plds + Ptot;
  float* sd = reinterpret_cast<float*>(plds + 2 * Ptot);
  int* ct = plds + 3 * Ptot;
  __shared__ int offs[kMergeMaxLists + 1];
  if (threadIdx.x == 0) {
    int o = 0;
    for (int r = 0; r < R; ++r) {
      offs[r] = o;
      const int c = pos_cnt[(int64_t)r * Q + q];
      o += c < Pmax ? c : Pmax;
    }
    offs[R] = o;
  }
  __syncthreads();
  const int P = offs[R];
  for (int r = 0; r < R; ++r) {
    const int n = offs[r + 1] - offs[r];
    for (int p = threadIdx.x; p < n; p += blockDim.x) {
      ud[offs[r] + p] = pos_d[((int64_t)r * Q + q) * Pmax + p];
      ui[offs[r] + p] = pos_idx[((int64_t)r * Q + q) * Pmax + p];
    }
  }
  __syncthreads();
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    const float d = ud[p];
    const int ix = ui[p];
    int rk = 0;
    for (int o = 0; o < P; ++o) rk += key_less(ud[o], ui[o], d, ix) ? 1 : 0;
    sorted_d[q * Ptot + rk] = d;
    sorted_idx[q * Ptot + rk] = ix;
    sd[rk] = d;
  }
  for (int p = P + threadIdx.x; p < Ptot; p += blockDim.x) {
    sorted_d[q * Ptot + p] = INFINITY;
    sorted_idx[q * Ptot + p] = -1;
  }
  if (threadIdx.x == 0) pos_total[q] = P;
  if (P == 0) return;  // uniform: the count pass skips this query
  __syncthreads();
  const float df = sd[0], inv = cell_scale(df, sd[P - 1]);
  for (int p = threadIdx.x; p < P; p += blockDim.x) ct[p] = cell_of(sd[p], df, inv);
  __syncthreads();
  for (int c = threadIdx.x; c < kStreamCells; c += blockDim.x) {
    int lo = 0, hi = P;  // first positive whose cell is >= c (ct is non-decreasing)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (ct[mid] < c) lo = mid + 1; else hi = mid;
    }
    cells[q * kStreamCells + c] = lo | ((lo < P && ct[lo] == c) ? kCellDirty : 0);
  }
}

// b') rank_prepare for merged lists longer than the LDS merge holds (R*Pmax
// > kRankMergeCap: an identity with thousands of gallery entries per shard).
// The query's lists are copied into its output row (sorted_d / sorted_idx,
// padding +inf / -1 past P) and sorted there in place by the block: a
// bitonic network for any length -- the first compare of each merge step
// mirrors inside the block (i <-> block end - 1 - i), the rest are half-
// cleaners, every compare puts the smaller (distance, index) key first and
// partners at or past P are skipped (they act as +inf at the end) -- over
// the L2-resident row, one block barrier per stage.  Keys are unique
// (global indices), so the order is the LDS path's.  Then the bin-lookup
// cells from the sorted row (the positive's cell computed on the fly).
__global__ void rank_prepare_global_kernel(int R, int64_t Q, int Pmax,
                                           const float* __restrict__ pos_d,
                                           const int32_t* __restrict__ pos_idx,
                                           const int32_t* __restrict__ pos_cnt,
                                           float* __restrict__ sorted_d,
                                           int32_t* __restrict__ sorted_idx,
                                           int32_t* __restrict__ pos_total,
                                           int32_t* __restrict__ cells) {
  const int64_t q = blockIdx.x;
  const int64_t Ptot = (int64_t)R * Pmax;
  __shared__ int offs[kMergeMaxLists + 1];
  if (threadIdx.x == 0) {
    int o = 0;
    for (int r = 0; r < R; ++r) {
      offs[r] = o;
      const int c = pos_cnt[(int64_t)r * Q + q];
      o += c < Pmax ? c : Pmax;
    }
    offs[R] = o;
  }
  __syncthreads();
  const int P = offs[R];
  float* gd = sorted_d + q * Ptot;
  int32_t* gi = sorted_idx + q * Ptot;
  for (int r = 0; r < R; ++r) {
    const int n = offs[r + 1] - offs[r];
    for (int p = threadIdx.x; p < n; p += blockDim.x) {
      gd[offs[r] + p] = pos_d[((int64_t)r * Q + q) * Pmax + p];
      gi[offs[r] + p] = pos_idx[((int64_t)r * Q + q) * Pmax + p];
    }
  }
  for (int64_t p = P + threadIdx.x; p < Ptot; p += blockDim.x) {
    gd[p] = INFINITY;
    gi[p] = -1;
  }
  if (threadIdx.x == 0) pos_total[q] = P;
  if (P == 0) return;  // uniform
  __syncthreads();
  auto cas = [&](int i, int j) {  // i < j: the smaller key to i
    const float di = gd[i], dj = gd[j];
    const int ii = gi[i], ij = gi[j];
    if (key_less(dj, ij, di, ii)) {
      gd[i] = dj; gi[i] = ij;
      gd[j] = di; gi[j] = ii;
    }
  };
  int n2 = 1;
  while (n2 < P) n2 <<= 1;
  for (int size = 2; size <= n2; size <<= 1) {
    const int half = size >> 1;
    for (int t = threadIdx.x; t < n2 / 2; t += blockDim.x) {  // mirror step
      const int b = t / half, o = t - b * half;
      const int i = b * size + o, j = b * size + size - 1 - o;
      if (j < P) cas(i, j);
    }
    __syncthreads();
    for (int stride = half >> 1; stride > 0; stride >>= 1) {  // half-cleaners
      for (int t = threadIdx.x; t < n2 / 2; t += blockDim.x) {
        const int b = t / stride, o = t - b * stride;
        const int i = 2 * b * stride + o, j = i + stride;
        if (j < P) cas(i, j);
      }
      __syncthreads();
    }
  }
  const float df = gd[0], inv = cell_scale(df, gd[P - 1]);
  for (int c = threadIdx.x; c < kStreamCells; c += blockDim.x) {
    int lo = 0, hi = P;  // first positive whose cell is >= c (non-decreasing in p)
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cell_of(gd[mid], df, inv) < c) lo = mid + 1; else hi = mid;
    }
    cells[q * kStreamCells + c] = lo | ((lo < P && cell_of(gd[lo], df, inv) == c) ? kCellDirty : 0);
  }
}

int rank_prepare(int R, int64_t Q, int Pmax, const float* pos_d, const int32_t* pos_idx,
                 const int32_t* pos_cnt, float* sorted_d, int32_t* sorted_idx,
                 int32_t* pos_total, int32_t* cells, hipStream_t st) {
  if (Q <= 0) return PPS_OK;
  if ((int64_t)R * Pmax > kRankMergeCap) {
    hipLaunchKernelGGL(rank_prepare_global_kernel, dim3((unsigned)Q), dim3(kEvalThreads), 0, st,
                       R, Q, Pmax, pos_d, pos_idx, pos_cnt, sorted_d, sorted_idx, pos_total,
                       cells);
    PPS_CHECK_LAUNCH("rank_prepare_global_kernel");
    return PPS_OK;
  }
  const size_t lds = (size_t)4 * R * Pmax * sizeof(int);
  hipLaunchKernelGGL(rank_prepare_kernel, dim3((unsigned)Q), dim3(kEvalThreads), lds, st, R,
                     Q, Pmax, pos_d, pos_idx, pos_cnt, sorted_d, sorted_idx, pos_total, cells);
  PPS_CHECK_LAUNCH("rank_prepare_kernel");
  return PPS_OK;
}

// c) rank_count_stream: grid (query, row chunk).  Each block streams its chunk
// of the row as 16-byte vectors (kStreamU in flight per thread), bins the
// entries closer than the farthest positive against the sorted positives
// (binary search, LDS histogram), counts the entries ordered before the
// first positive, takes this shard's junk entries back out (chunk 0), and
// adds its counts to hist / before with one global atomic per non-empty bin.
// KLDS = false: positive lists too long for LDS are searched in global memory
// (L2) and binned with global atomics -- no capacity limit.
#ifndef RANK_STREAM_VARIANT
#define RANK_STREAM_VARIANT 0  // probes only (scripts/rank_probe.py): 1 = stream + compare,
                               // 2 = + binary search, no histogram atomics
#endif
constexpr int kStreamThreads = 256;
constexpr int kStreamU = RANK_STREAM_U;                      // float4 per thread in flight
constexpr int kStreamChunk = kStreamThreads * kStreamU * 4;  // 8192 entries per block
static_assert(kStreamChunk == kRankStreamChunk, "pps_internal.hpp kRankStreamChunk");
constexpr int kStreamLdsCap = 6144;                          // positives held in LDS

template <bool KLDS>
__global__ void __launch_bounds__(kStreamThreads)
rank_count_stream_kernel(const float* __restrict__ dist, int64_t G, int64_t ldd,
                         int64_t g_offset, int Ptot, const float* __restrict__ sorted_d,
                         const int32_t* __restrict__ sorted_idx,
                         const int32_t* __restrict__ pos_total,
                         const int32_t* __restrict__ cells, int Jmax,
                         const float* __restrict__ junk_d,
                         const int32_t* __restrict__ junk_idx,
                         const int32_t* __restrict__ junk_cnt, int32_t* __restrict__ hist,
                         int32_t* __restrict__ before) {
  const int64_t q = blockIdx.x;
  const int P = pos_total[q];
  if (P == 0) return;
  extern __shared__ int slds[];
  const float* gsd = sorted_d + q * Ptot;
  int32_t* ghist = hist + q * Ptot;
  const int Pa = (P + 3) & ~3;  // keeps the cell arrays 16-byte aligned
  float* sd = reinterpret_cast<float*>(slds);
  int* hs = slds + (KLDS ? Pa : 0);
  int* cs = slds + (KLDS ? 2 * Pa : 0);  // bin-lookup cells (rank_prepare)
  int* cc = cs + kStreamCells;          // per-cell entry counts (clean cells)
  __shared__ int red[kStreamThreads / 64];
  const float df = gsd[0], dmax = gsd[P - 1];
  // Binning without a per-entry binary search: a "clean" cell holds no
  // positive, so every entry in it has bin cs[c] exactly and only bumps the
  // cell's counter cc[c] (1024 addresses: a wave's LDS atomics rarely collide;
  // with one counter per positive they serialised).  A cell holding
  // positives finishes the lower_bound with a short forward scan from cs[c].
  // The clean-cell counts are folded into the positives' bins once per block.
  const float inv = cell_scale(df, dmax);
  if (KLDS) {
    for (int p = threadIdx.x; p < P; p += kStreamThreads) {
      sd[p] = gsd[p];
      hs[p] = 0;
    }
    const int4* gc = reinterpret_cast<const int4*>(cells + q * kStreamCells);
    for (int c = threadIdx.x; c < kStreamCells / 4; c += kStreamThreads) {
      reinterpret_cast<int4*>(cs)[c] = gc[c];
      reinterpret_cast<int4*>(cc)[c] = make_int4(0, 0, 0, 0);
    }
    __syncthreads();
  }
  const float* S = KLDS ? sd : gsd;
  const int64_t idf = sorted_idx[q * Ptot];
  auto bin = [&](float d) {  // lower_bound(S, d) for d <= dmax: < P
    int lo = 0, hi = P;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (S[mid] < d) lo = mid + 1; else hi = mid;
    }
    return lo;
  };
  auto add = [&](int b, int v) {
    if (KLDS) atomicAdd(&hs[b], v); else atomicAdd(&ghist[b], v);
  };
  int nb = 0;
  auto visit = [&](int64_t i, float d) {
    if (d <= dmax) {
#if RANK_STREAM_VARIANT == 1
      nb += 1;
#elif RANK_STREAM_VARIANT == 2
      nb += bin(d);
#else
      if (d <= df) {  // bin 0; the only entries that can precede the first positive
        add(0, 1);
        nb += (d < df || g_offset + i < idf) ? 1 : 0;
      } else if (KLDS) {
        const int c = cell_of(d, df, inv);
        const int e = cs[c];
        if (e & kCellDirty) {
          int b = e & (kCellDirty - 1);
          while (S[b] < d) ++b;
          atomicAdd(&hs[b], 1);
        } else {
          atomicAdd(&cc[c], 1);
        }
      } else {
        add(bin(d), 1);
      }
#endif
    }
  };
  const int64_t c0 = (int64_t)blockIdx.y * kStreamChunk;
  const int64_t c1 = c0 + kStreamChunk < G ? c0 + kStreamChunk : G;
  const float* row = dist + q * ldd;
  if (((reinterpret_cast<uintptr_t>(row) & 15) == 0)) {
    // 16-byte rows: the chunk [c0, c1) starts on a vector boundary
    const f32x4* v4 = reinterpret_cast<const f32x4*>(row + c0);
    const int nv = (int)((c1 - c0) >> 2);
    f32x4 v[kStreamU];
#pragma unroll
    for (int u = 0; u < kStreamU; ++u) {
      const int j = threadIdx.x + u * kStreamThreads;
      // streamed once: non-temporal, so the row does not evict useful L2 lines
      v[u] = j < nv ? __builtin_nontemporal_load(v4 + j) : f32x4{INFINITY, INFINITY, INFINITY,
                                                                  INFINITY};
    }
#pragma unroll
    for (int u = 0; u < kStreamU; ++u) {
      const int64_t i = c0 + 4 * (int64_t)(threadIdx.x + u * kStreamThreads);
      visit(i, v[u].x);
      visit(i + 1, v[u].y);
      visit(i + 2, v[u].z);
      visit(i + 3, v[u].w);
    }
    const int64_t t = c0 + 4 * (int64_t)nv + threadIdx.x;
    if (t < c1) visit(t, row[t]);
  } else {
    float v[4 * kStreamU];
#pragma unroll
    for (int u = 0; u < 4 * kStreamU; ++u) {
      const int64_t i = c0 + threadIdx.x + (int64_t)u * kStreamThreads;
      v[u] = i < c1 ? row[i] : INFINITY;
    }
#pragma unroll
    for (int u = 0; u < 4 * kStreamU; ++u)
      visit(c0 + threadIdx.x + (int64_t)u * kStreamThreads, v[u]);
  }
  if (blockIdx.y == 0) {  // junk entries of this shard were binned above: take them out
    const int nj = junk_cnt[q] < Jmax ? junk_cnt[q] : Jmax;
    for (int j = threadIdx.x; j < nj; j += kStreamThreads) {
      const float d = junk_d[q * Jmax + j];
      if (d <= dmax) {
        add(bin(d), -1);
        nb -= (d < df || (d == df && (int64_t)junk_idx[q * Jmax + j] < idf)) ? 1 : 0;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) nb += __shfl_xor(nb, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = nb;
  __syncthreads();
  if (KLDS) {
    for (int c = threadIdx.x; c < kStreamCells; c += kStreamThreads)
      if (cc[c]) atomicAdd(&hs[cs[c] & (kCellDirty - 1)], cc[c]);
    __syncthreads();
    for (int p = threadIdx.x; p < P; p += kStreamThreads)
      if (hs[p]) atomicAdd(&ghist[p], hs[p]);
  }
  if (threadIdx.x == 0) {
    int s = 0;
    for (int w = 0; w < kStreamThreads / 64; ++w) s += red[w];
    if (s) atomicAdd(&before[q], s);
  }
}

int rank_count_stream(const float* dist, int64_t Q, int64_t G, int64_t ldd, int64_t g_offset,
                      int Ptot, const float* sorted_d, const int32_t* sorted_idx,
                      const int32_t* pos_total, const int32_t* cells, int Jmax, const float* junk_d,
                      const int32_t* junk_idx, const int32_t* junk_cnt, int32_t* hist,
                      int32_t* before, hipStream_t st) {
  if (Q <= 0 || G <= 0) return PPS_OK;
  const int64_t nchunk = (G + kStreamChunk - 1) / kStreamChunk;
  for (int64_t q0 = 0; q0 < Q; q0 += 65535) {  // grid.x limit
    const int64_t qn = Q - q0 < 65535 ? Q - q0 : 65535;
    const dim3 grid((unsigned)qn, (unsigned)nchunk);
    const float* d = dist + q0 * ldd;
    if (Ptot <= kStreamLdsCap) {
      hipLaunchKernelGGL(rank_count_stream_kernel<true>, grid, dim3(kStreamThreads),
                         (size_t)(2 * ((Ptot + 3) & ~3) + 2 * kStreamCells) * sizeof(int), st,
                         d, G, ldd,
                         g_offset, Ptot,
                         sorted_d + q0 * Ptot, sorted_idx + q0 * Ptot, pos_total + q0,
                         cells + q0 * kStreamCells, Jmax, junk_d + q0 * Jmax, junk_idx + q0 * Jmax, junk_cnt + q0,
                         hist + q0 * Ptot, before + q0);
    } else {
      hipLaunchKernelGGL(rank_count_stream_kernel<false>, grid, dim3(kStreamThreads), 0, st, d,
                         G, ldd, g_offset, Ptot, sorted_d + q0 * Ptot, sorted_idx + q0 * Ptot,
                         pos_total + q0, cells + q0 * kStreamCells, Jmax, junk_d + q0 * Jmax, junk_idx + q0 * Jmax,
                         junk_cnt + q0, hist + q0 * Ptot, before + q0);
    }
    PPS_CHECK_LAUNCH("rank_count_stream_kernel");
  }
  return PPS_OK;
}

// ---- 3) AP / first-match finalisation -----------------------------------------
// One wave per query.  le[p] = prefix sum of hist (valid entries with
// d <= d_p); pos_le[p] = #positives with d <= d_p (upper bound, so tied
// positives share the precision at the end of their tie group, as sklearn's
// precision_recall_curve does on distinct thresholds).
__global__ void ap_finalize_kernel(int64_t Q, int Ptot, const float* __restrict__ sorted_d,
                                   const int32_t* __restrict__ pos_total,
                                   const int32_t* __restrict__ hist,
                                   const int32_t* __restrict__ before,
                                   double* __restrict__ ap, int32_t* __restrict__ valid,
                                   int32_t* __restrict__ first_rank) {
  const int64_t q = blockIdx.x;
  const int lane = threadIdx.x;
  const int P = pos_total[q];
  const float* sd = sorted_d + q * Ptot;
  const int32_t* hq = hist + q * Ptot;
  double acc = 0.0;
  int carry = 0;
  for (int p0 = 0; p0 < P; p0 += 64) {
    const int p = p0 + lane;
    int v = p < P ? hq[p] : 0;
    // inclusive wave scan
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(v, o);
      if (lane >= o) v += t;
    }
    const int le = carry + v;
    carry += __shfl(v, 63);
    if (p < P) {
      const float d = sd[p];
      int lo = p, hi = P;  // upper_bound of d in sd[p..P)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (sd[mid] <= d) lo = mid + 1; else hi = mid;
      }
      acc += (double)lo / (double)le;
    }
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) {
    ap[q] = P > 0 ? acc / (double)P : 0.0;
    valid[q] = P > 0 ? 1 : 0;
    first_rank[q] = P > 0 ? before[q] : -1;
  }
}

int ap_finalize(int64_t Q, int Ptot, const float* sorted_d, const int32_t* pos_total,
                const int32_t* hist, const int32_t* before, double* ap, int32_t* valid,
                int32_t* first_rank, hipStream_t st) {
  if (Q <= 0) return PPS_OK;
  hipLaunchKernelGGL(ap_finalize_kernel, dim3((unsigned)Q), dim3(64), 0, st, Q, Ptot,
                     sorted_d, pos_total, hist, before, ap, valid, first_rank);
  PPS_CHECK_LAUNCH("ap_finalize_kernel");
  return PPS_OK;
}

// ---- 4) CMC beyond the Market protocol (reid_dataset_evaluator.py:283-363) -------
// The reference's cmc defaults to first_match_break=False: for the j-th true
// match (in rank order) at position k among the valid entries it adds
// 1/#matches to ret[k - j], k - j = the number of valid NON-matches ranked
// before it (:349-356); separate_camera_set=True also drops every gallery
// entry from the query's camera (:329-331).  Both need, per positive p, the
// exact count of valid entries ordered before it.  Entry e is binned at
// b(e) = #positives whose (distance, global index) key is below e's, so
// H[p] = sum_{b <= p} hist[b] counts the valid entries ranked before positive
// p plus the positives 0..p: k - j = H[p] - p - 1.  Exact under the stable
// (distance, index) order, ties included; additive over gallery shards.
constexpr int kCmcLdsCap = 4096;

template <bool KLDS, bool SEP>
__global__ void __launch_bounds__(kStreamThreads)
cmc_count_kernel(const float* __restrict__ dist, int64_t G, int64_t ldd, int64_t g_offset,
                 int Ptot, const float* __restrict__ sorted_d,
                 const int32_t* __restrict__ sorted_idx, const int32_t* __restrict__ pos_total,
                 const int32_t* __restrict__ qcam, const int32_t* __restrict__ gcam, int Jmax,
                 const float* __restrict__ junk_d, const int32_t* __restrict__ junk_idx,
                 const int32_t* __restrict__ junk_cnt, int32_t* __restrict__ hist) {
  const int64_t q = blockIdx.x;
  const int P = pos_total[q];
  if (P == 0) return;
  extern __shared__ int slds[];
  float* sd = reinterpret_cast<float*>(slds);
  int* si = slds + (KLDS ? P : 0);
  int* hs = slds + (KLDS ? 2 * P : 0);
  const float* gsd = sorted_d + q * Ptot;
  const int32_t* gsi = sorted_idx + q * Ptot;
  int32_t* ghist = hist + q * Ptot;
  if (KLDS) {
    for (int p = threadIdx.x; p < P; p += kStreamThreads) {
      sd[p] = gsd[p];
      si[p] = gsi[p];
      hs[p] = 0;
    }
    __syncthreads();
  }
  const float* S = KLDS ? sd : gsd;
  const int32_t* I = KLDS ? si : gsi;
  const float dmax = S[P - 1];
  // b = #positives with key < (d, gi); entries ordered after every positive
  // (b == P) do not count
  auto key_bin = [&](float d, int64_t gi) {
    int lo = 0, hi = P;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (S[mid] < d || (S[mid] == d && (int64_t)I[mid] < gi)) lo = mid + 1; else hi = mid;
    }
    return lo;
  };
  auto add = [&](int b, int v) {
    if (b < P) {
      if (KLDS) atomicAdd(&hs[b], v); else atomicAdd(&ghist[b], v);
    }
  };
  const int qc = SEP ? qcam[q] : 0;
  const int64_t c0 = (int64_t)blockIdx.y * kStreamChunk;
  const int64_t c1 = c0 + kStreamChunk < G ? c0 + kStreamChunk : G;
  const float* row = dist + q * ldd;
  for (int64_t i = c0 + threadIdx.x; i < c1; i += kStreamThreads) {
    const float d = row[i];
    if (d > dmax) continue;
    if (SEP && gcam[i] == qc) continue;  // same camera: never valid
    add(key_bin(d, g_offset + i), 1);
  }
  if (!SEP && blockIdx.y == 0) {  // this shard's junk (same id, same camera) back out
    const int nj = junk_cnt[q] < Jmax ? junk_cnt[q] : Jmax;
    for (int j = threadIdx.x; j < nj; j += kStreamThreads) {
      const float d = junk_d[q * Jmax + j];
      if (d <= dmax) add(key_bin(d, (int64_t)junk_idx[q * Jmax + j]), -1);
    }
  }
  if (KLDS) {
    __syncthreads();
    for (int p = threadIdx.x; p < P; p += kStreamThreads)
      if (hs[p]) atomicAdd(&ghist[p], hs[p]);
  }
}

int cmc_counts(const float* dist, int64_t Q, int64_t G, int64_t ldd, int64_t g_offset, int Ptot,
               const float* sorted_d, const int32_t* sorted_idx, const int32_t* pos_total,
               const int32_t* qcam, const int32_t* gcam, int Jmax, const float* junk_d,
               const int32_t* junk_idx, const int32_t* junk_cnt, int32_t* hist,
               hipStream_t st) {
  if (Q <= 0 || G <= 0) return PPS_OK;
  const int64_t nchunk = (G + kStreamChunk - 1) / kStreamChunk;
  const bool lds = Ptot <= kCmcLdsCap, sep = gcam != nullptr;
  const size_t shm = lds ? (size_t)3 * Ptot * sizeof(int) : 0;
  for (int64_t q0 = 0; q0 < Q; q0 += 65535) {  // grid.x limit
    const int64_t qn = Q - q0 < 65535 ? Q - q0 : 65535;
    const dim3 grid((unsigned)qn, (unsigned)nchunk);
    auto launch = [&](auto kernel) {
      hipLaunchKernelGGL(kernel, grid, dim3(kStreamThreads), shm, st, dist + q0 * ldd, G, ldd,
                         g_offset, Ptot, sorted_d + q0 * Ptot, sorted_idx + q0 * Ptot,
                         pos_total + q0, sep ? qcam + q0 : nullptr, gcam, Jmax,
                         junk_d + q0 * Jmax, junk_idx + q0 * Jmax, junk_cnt + q0,
                         hist + q0 * Ptot);
    };
    if (lds && sep) launch(cmc_count_kernel<true, true>);
    else if (lds) launch(cmc_count_kernel<true, false>);
    else if (sep) launch(cmc_count_kernel<false, true>);
    else launch(cmc_count_kernel<false, false>);
    PPS_CHECK_LAUNCH("cmc_count_kernel");
  }
  return PPS_OK;
}

// Per query (one wave): ret[q][0..topk) = the reference's CMC row after its
// cumsum (:358-360): for positives p = 0.. in rank order, c = H[p] - p - 1;
// stop at c >= topk; first_match_break adds 1 once, else 1/P each, summed in
// the reference's order (float64, same rounding).  valid[q] = P > 0.
__global__ void cmc_finalize_kernel(int Ptot, const int32_t* __restrict__ pos_total,
                                    const int32_t* __restrict__ hist, int topk, int fmb,
                                    double* __restrict__ ret, int32_t* __restrict__ valid) {
  const int64_t q = blockIdx.x;
  const int P = pos_total[q];
  double* r = ret + q * topk;
  for (int t = threadIdx.x; t < topk; t += 64) r[t] = 0.0;
  __syncthreads();
  if (threadIdx.x == 0) {
    valid[q] = P > 0 ? 1 : 0;
    if (P > 0) {
      const int32_t* h = hist + q * Ptot;
      const double delta = 1.0 / (double)P;
      int64_t H = 0;
      for (int p = 0; p < P; ++p) {
        H += h[p];
        const int64_t c = H - p - 1;
        if (c >= topk) break;
        if (fmb) {
          r[c] += 1.0;
          break;
        }
        r[c] += delta;
      }
      for (int t = 1; t < topk; ++t) r[t] += r[t - 1];
    }
  }
}

int cmc_finalize(int64_t Q, int Ptot, const int32_t* pos_total, const int32_t* hist, int topk,
                 int fmb, double* ret, int32_t* valid, hipStream_t st) {
  if (Q <= 0) return PPS_OK;
  hipLaunchKernelGGL(cmc_finalize_kernel, dim3((unsigned)Q), dim3(64), 0, st, Ptot, pos_total,
                     hist, topk, fmb, ret, valid);
  PPS_CHECK_LAUNCH("cmc_finalize_kernel");
  return PPS_OK;
}

// ---- stable per-row top-k ---------------------------------------------------------
// Radix select (4 x 8-bit digits of the order-preserving key) finds the k-th
// smallest key K*; entries with key < K*, then entries == K* in index order,
// are compacted into LDS and bitonic-sorted as 64-bit (key << 32 | index).
__device__ inline uint32_t float_key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float key_float(uint32_t k) {
  const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

constexpr int kTopkThreads = 256;
constexpr int kTopkCap = 1024;      // max k
constexpr int kTopkBuf = 4096;      // candidate buffer (64-bit entries) in LDS
constexpr int kTopkUnroll = 8;      // row elements per thread per chunk
static_assert(kTopkCap + kTopkThreads * kTopkUnroll <= kTopkBuf,
              "a cut buffer plus one chunk must fit");

// Bitonic sort (ascending) of buf[0, n2), n2 a power of two, by the block.
__device__ inline void block_bitonic(unsigned long long* buf, int n2) {
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < n2 / 2; t += blockDim.x) {
        const int i = 2 * stride * (t / stride) + (t % stride);
        const int j = i + stride;
        const bool up = (i & size) == 0;
        const unsigned long long a = buf[i], b = buf[j];
        if ((a > b) == up) { buf[i] = b; buf[j] = a; }
      }
      __syncthreads();
    }
  }
}

// cut: keep the k best of the n candidates cand[0, n) at the front (block-
// wide).  The k-th best packed key T is found by an 8-pass radix select
// (8-bit digits from the top; packed keys are unique, so exactly k entries
// are <= T) and the k entries are compacted to the front -- a full bitonic
// sort of the buffer (78 LDS-bound stages for 4096 entries, shared by the
// CU's blocks) cost ~150 us per row block on short rows.  Only the final
// cut sorts, and only those k entries.  Returns T (~0 when n <= k).
struct TopkSmem {
  unsigned hist[256];
  unsigned long long pref;
  int rank, cnt;
};
__device__ unsigned long long block_cut(unsigned long long* cand, int n, int k, bool final,
                                        TopkSmem& sm) {
  constexpr int kPerThr = kTopkBuf / kTopkThreads;
  unsigned long long T = ~0ull;
  int keep = n;
  if (n > k) {
    if (threadIdx.x == 0) { sm.pref = 0ull; sm.rank = k; }
    for (int pass = 0; pass < 8; ++pass) {
      const int shift = 56 - 8 * pass;
      for (int i = threadIdx.x; i < 256; i += blockDim.x) sm.hist[i] = 0u;
      __syncthreads();
      const unsigned long long pre = sm.pref;
      for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const unsigned long long v = cand[i];
        if (pass == 0 || (v >> (shift + 8)) == pre)
          atomicAdd(&sm.hist[(unsigned)(v >> shift) & 255u], 1u);
      }
      __syncthreads();
      if (threadIdx.x < 64) {  // one wave: the bin holding rank sm.rank
        const int l = threadIdx.x;
        unsigned h[4], sum = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) { h[b] = sm.hist[4 * l + b]; sum += h[b]; }
        unsigned incl = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const unsigned t = __shfl_up(incl, o);
          if (l >= o) incl += t;
        }
        const unsigned r = (unsigned)sm.rank;
        const unsigned long long hit = __ballot(incl >= r);
        const int hl = __ffsll((long long)hit) - 1;
        if (l == hl) {
          unsigned before = incl - sum;
          int b = 0;
          while (b < 3 && before + h[b] < r) before += h[b++];
          sm.pref = (pre << 8) | (unsigned long long)(4 * l + b);
          sm.rank = (int)(r - before);
        }
      }
      __syncthreads();
    }
    T = sm.pref;  // the k-th best packed key
    unsigned long long mine[kPerThr];
#pragma unroll
    for (int j = 0; j < kPerThr; ++j) {
      const int i = threadIdx.x + j * kTopkThreads;
      mine[j] = i < n ? cand[i] : ~0ull;
    }
    if (threadIdx.x == 0) sm.cnt = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kPerThr; ++j)
      if (mine[j] <= T) cand[atomicAdd(&sm.cnt, 1)] = mine[j];
    __syncthreads();
    keep = k;
  }
  if (final) {
    int n2 = 1;
    while (n2 < keep) n2 <<= 1;
    for (int i = keep + threadIdx.x; i < n2; i += blockDim.x) cand[i] = ~0ull;
    __syncthreads();
    block_bitonic(cand, n2);
  }
  return T;
}

// One pass over the row.  Entries are packed as (order-preserving key << 32 |
// index), so comparing packed values is the stable (distance, index) order.
// An entry enters the LDS candidate buffer only if it beats the current
// threshold = the k-th best packed value among the candidates kept so far;
// when the buffer could overflow in the next chunk it is cut back to its k
// best (rare after the first chunks: ~k*ln(G/k) insertions per row).
// V4: 16-byte rows -- each thread takes two float4 per chunk (dwordx4 buffer
// loads, 4x fewer load instructions) and the loads run two chunks ahead, so
// a block keeps 16 KB of its row in flight instead of 8 KB (the kernel is
// latency-bound at 5 blocks per CU).  Which thread sees which entry does
// not matter: candidates are ordered by their packed (key, index) value.
template <bool V4>
__global__ void __launch_bounds__(kTopkThreads)
topk_kernel(const float* __restrict__ dist, int64_t G, int64_t ldd, int k,
            float* __restrict__ vals, int32_t* __restrict__ idx) {
  const int64_t q = blockIdx.x;
  const float* row = dist + q * ldd;
  __shared__ unsigned long long cand[kTopkBuf];
  __shared__ int s_n;
  __shared__ unsigned long long s_thr;
  if (threadIdx.x == 0) { s_n = 0; s_thr = ~0ull; }
  __syncthreads();
  const int64_t chunk = (int64_t)blockDim.x * kTopkUnroll;
  __shared__ TopkSmem sm;
  auto cut = [&](int n, bool final) {
    const unsigned long long T = block_cut(cand, n, k, final, sm);
    if (threadIdx.x == 0) {
      s_n = n > k ? k : n;
      if (n > k) s_thr = T;
    }
    __syncthreads();
  };
  // the next chunk's row values are requested before this chunk is
  // processed; the chunk-closing barrier is a raw s_barrier after an LDS-only
  // wait, so those loads stay in flight across it (__syncthreads() would
  // drain them with vmcnt(0))
  auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  // buffer loads: the row tail past G reads zero without exec-mask branches,
  // which keeps the loads countable (a branchy guard makes hipcc wait vmcnt(0))
  // V4: the vector loop covers the first GV = G & ~3 entries (its descriptor
  // ends there, so no 16-byte load straddles G); the last G - GV entries
  // are taken after the loop by scalar loads.
  const int64_t GV = V4 ? (G & ~(int64_t)3) : G;
  const rsrc_t rrow = make_rsrc(row, (uint32_t)(GV * 4));
  auto ld = [&](int64_t i) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rrow, (int)(i * 4), 0, 0));
  };
  // entry u of this thread in the chunk at c0
  auto ent = [&](int64_t c0, int u) -> int64_t {
    return V4 ? c0 + 4 * ((int64_t)(u >> 2) * kTopkThreads + threadIdx.x) + (u & 3)
              : c0 + (int64_t)u * kTopkThreads + threadIdx.x;
  };
  auto load_chunk = [&](int64_t c0, float (&dst)[kTopkUnroll]) {
    if (V4) {
#pragma unroll
      for (int j = 0; j < kTopkUnroll / 4; ++j) {
        const f32x4 v = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rrow, (int)(ent(c0, 4 * j) * 4), 0, 0));
        dst[4 * j] = v.x;
        dst[4 * j + 1] = v.y;
        dst[4 * j + 2] = v.z;
        dst[4 * j + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int u = 0; u < kTopkUnroll; ++u) dst[u] = ld(ent(c0, u));
    }
  };
  float d[kTopkUnroll], dn[kTopkUnroll];
  load_chunk(0, d);
  if (V4) load_chunk(chunk, dn);
  for (int64_t c0 = 0; c0 < GV; c0 += chunk) {
    // every wave must take the same cut decision: snapshot the count, then
    // a barrier so that no wave's insertions of this chunk (atomicAdd on
    // s_n) can land before a slower wave has read it
    const int n_now = s_n;
    lds_barrier();
    // the first chunk enters unfiltered: cut it at once (a 2048-entry select
    // instead of a 4096-entry one a chunk later) so the next chunks filter
    if (n_now + chunk > kTopkBuf || (c0 == chunk && n_now > k)) cut(n_now, false);
    const unsigned long long thr = s_thr;
    float dn2[kTopkUnroll];
    load_chunk(c0 + (V4 ? 2 : 1) * chunk, dn2);
#pragma unroll
    for (int u = 0; u < kTopkUnroll; ++u) {
      const int64_t i = ent(c0, u);
      const unsigned long long packed =
          ((unsigned long long)float_key(d[u]) << 32) | (uint32_t)i;
      const bool take = i < GV && packed < thr;
      const unsigned long long bal = __ballot(take);  // one LDS atomic per wave
      if (bal) {
        int base = 0;
        if (lane == 0) base = atomicAdd(&s_n, __popcll(bal));
        base = __shfl(base, 0);
        if (take) cand[base + __popcll(bal & below)] = packed;
      }
    }
#pragma unroll
    for (int u = 0; u < kTopkUnroll; ++u) {
      if (V4) {
        d[u] = dn[u];
        dn[u] = dn2[u];
      } else {
        d[u] = dn2[u];
      }
    }
    lds_barrier();
  }
  if (V4 && GV < G) {  // the < 4 entries past the vector loop
    const int n_now = s_n;
    lds_barrier();
    if (n_now + 4 > kTopkBuf) cut(n_now, false);
    const unsigned long long thr = s_thr;
    if (threadIdx.x < G - GV) {
      const int64_t i = GV + threadIdx.x;
      const unsigned long long packed = ((unsigned long long)float_key(row[i]) << 32) | (uint32_t)i;
      if (packed < thr) cand[atomicAdd(&s_n, 1)] = packed;
    }
    __syncthreads();
  }
  cut(s_n, true);
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    const unsigned long long v = cand[i];
    vals[q * k + i] = key_float((uint32_t)(v >> 32));
    idx[q * k + i] = (int32_t)(v & 0xffffffffu);
  }
}

// Long rows (the 1M-gallery shards: 125k entries per row): every WAVE streams
// its own contiguous quarter of the row with its own threshold and its own
// candidate buffer in LDS, so the streaming loop has no block barrier and no
// LDS atomic (a wave appends at its own uniform count).  When the next
// iteration could overflow the buffer (and once right after the first
// iteration, so the rest of the row is filtered against a real threshold) the
// wave cuts it back to between k and k + kTkwSlack entries; at the end to
// exactly its k best.  Wave 0 then selects the row's k best of the four lists
// and the block sorts them.  Same result as topk_kernel (the stable
// (distance, index) top-k is unique).
//
// Selection is a bisection on the packed value with the buffer held in
// registers: each step is one compare per register, a ballot and a scalar
// popcount -- no LDS atomics.  (A radix select's LDS histogram serialises
// here: after the first cut the buffered keys share their top bytes, so 64
// lanes add into one bin.)
#ifndef PPS_TKW_U
#define PPS_TKW_U 2
#endif
#ifndef PPS_TKW_D
#define PPS_TKW_D 2   // iterations loaded ahead of the one filtering
#endif
#ifndef PPS_TKW_PROBE
#define PPS_TKW_PROBE 0
#endif
constexpr int kTkwU = PPS_TKW_U;            // float4 per lane per iteration
constexpr int kTkwIter = 64 * 4 * kTkwU;    // row entries per wave iteration (512)
constexpr int kTkwWaves = kTopkThreads / 64;
constexpr int kTkwMinRow = 16384;           // rows at least this long take this kernel
constexpr int kTkwMaxK = 256;
constexpr int kTkwSlack = 64;               // a streaming cut keeps k .. k + slack entries
// per-wave buffer: what a cut keeps + one iteration's worst-case inflow
__host__ __device__ constexpr int tkw_cap(int k) { return (k + kTkwSlack + kTkwIter + 63) / 64 * 64; }
// registers per lane for a wave's buffer / the four merged lists, for k <= KM
template <int KM> constexpr int tkw_j() { return tkw_cap(KM) / 64; }
template <int KM> constexpr int tkw_merge_j() { return kTkwWaves * KM / 64 + 1; }

__device__ inline void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ inline unsigned long long wave_min_u64(unsigned long long x) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_xor(x, o);
    x = y < x ? y : x;
  }
  return x;
}
__device__ inline unsigned long long wave_max_u64(unsigned long long x) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_xor(x, o);
    x = y > x ? y : x;
  }
  return x;
}
template <int J>
__device__ inline int wave_count_le(const unsigned long long (&v)[J], unsigned long long t) {
  int c = 0;
#pragma unroll
  for (int j = 0; j < J; ++j) c += __popcll(__ballot(v[j] <= t));
  return c;
}

// v[j] holds entry j*64 + lane of a wave's n > k unique packed values (~0ull
// past n; no real entry is ~0ull: indices are < 2^31).  Returns a T with
// k <= count(v <= T) <= k + slack; slack 0 gives the k-th smallest value.
// Invariant count(<= lo) < k <= count(<= hi); every value is wave-uniform.
template <int J>
__device__ unsigned long long wave_select(const unsigned long long (&v)[J], int k, int slack) {
  unsigned long long mn = ~0ull, mx = 0ull;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    mn = v[j] < mn ? v[j] : mn;
    mx = (v[j] != ~0ull && v[j] > mx) ? v[j] : mx;
  }
  mn = wave_min_u64(mn);
  mx = wave_max_u64(mx);
  if (k <= 1) return mn;
  unsigned long long lo = mn, hi = mx;   // count(<= mn) = 1 < k
  while (hi - lo > 1) {
    const unsigned long long mid = lo + ((hi - lo) >> 1);
    const int c = wave_count_le(v, mid);
    if (c >= k && c <= k + slack) return mid;
    if (c < k) lo = mid; else hi = mid;
  }
  return hi;
}

// Cuts a wave's buffer buf[0, n) to the entries <= T of wave_select: reads
// it into registers, selects, writes the kept entries back to the front.
// Returns T; n becomes the kept count.
template <int J>
__device__ unsigned long long wave_cut(unsigned long long* buf, int& n, int k, int slack) {
  const int lane = threadIdx.x & 63;
  unsigned long long v[J];
#pragma unroll
  for (int j = 0; j < J; ++j) v[j] = j * 64 + lane < n ? buf[j * 64 + lane] : ~0ull;
  const unsigned long long T = wave_select(v, k, slack);
  int m = 0;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const bool keep = v[j] <= T;
    const unsigned long long bal = __ballot(keep);
    if (keep) buf[m + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u))] = v[j];
    m += __popcll(bal);
  }
  wave_lds_sync();
  n = m;
  return T;
}

// RR (re-ranking, rerank.hip): row q is row q of OD for a symmetric M read
// in place -- a virtual row of the M row's first block (Q entries, padded to
// naq = Q rounded up to 4 with +inf, never selected) followed by its second
// block (G entries), each entry transformed to rr_od(m, colmax[q]) before the
// filter; packed indices are the global column (virtual index with the pad
// taken out: a monotone map, so the order is the same).
//
// WPR (waves per row) 1: every wave streams a whole row of its own (a block
// holds four rows) -- for many rows of moderate length (re-ranking's N rows
// of N), where four waves per row would each cut their short segment three or
// four times and then merge: one wave per row cuts ~log(row / 512) times in
// all and sorts its own k, no block barrier.
//
// rows (WPR 1): the rows to process are rows[0, *rows_n) (a device list).
template <int KM, bool RR, int WPR = kTkwWaves>
__global__ void __launch_bounds__(kTopkThreads) __attribute__((amdgpu_waves_per_eu(6)))
topk_wave_kernel(const float* __restrict__ dist, int64_t G, int64_t ldd, int k, int cap,
                 float* __restrict__ vals, int32_t* __restrict__ idx, RrMatrix rr,
                 int64_t nrows, const int32_t* __restrict__ rows = nullptr,
                 const int32_t* __restrict__ rows_n = nullptr) {
  static_assert(WPR == 1 || WPR == kTkwWaves, "one wave or the whole block per row");
  extern __shared__ unsigned long long tkw[];  // [waves][cap] buffers
  // wave-uniform: segment bounds, buffer base and counts live in SGPRs
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  unsigned long long* buf = tkw + wave * cap;
  constexpr int RPB = kTkwWaves / WPR;   // rows per block
  const int wseg = wave % WPR;           // this wave's segment of its row
  int64_t q = (int64_t)blockIdx.x * RPB + wave / WPR;
  if (WPR == 1 && rows) {
    if (q >= *rows_n) return;
    q = rows[q];
  }
  if (WPR == 1 && q >= nrows) return;   // (WPR = 1 has no block barrier)
  const float* row = RR ? nullptr : dist + q * ldd;
  // RR: the two blocks of M's row q
  const int64_t na = RR ? rr.Q : 0, naq = RR ? (rr.Q + 3) / 4 * 4 : 0;
  const float* rowA = RR ? (q < rr.Q ? rr.qq + q * rr.ldqq : rr.qgT + (q - rr.Q) * rr.ldT) : nullptr;
  const float* rowB = RR ? (q < rr.Q ? rr.qg + q * rr.ldqg : rr.gg + (q - rr.Q) * rr.ldgg) : nullptr;
  const float cm = RR ? rr.colmax[q] : 1.f;
  if (RR) G = naq + rr.G;  // virtual row length
  // virtual index -> column of OD
  auto col = [&](uint32_t i) -> uint32_t {
    return RR ? (i < (uint32_t)naq ? i : i - (uint32_t)(naq - na)) : i;
  };
  // one loaded entry -> its OD value (RR) / itself
  auto xf = [&](float m, int64_t i) -> float {
    if (!RR) return m;
    return (i >= na && i < naq) ? __builtin_huge_valf() : rr_od(m, cm);
  };
  // this wave's segment [s0, s1): whole float4s of the 16-byte-aligned row
  const int64_t GV = G & ~(int64_t)3;
  const int64_t per = ((GV / 4 + WPR - 1) / WPR) * 4;
  const int64_t s0 = min(GV, (int64_t)wseg * per), s1 = min(GV, s0 + per);
  const rsrc_t rrow = make_rsrc(RR ? rowA : row, (uint32_t)(GV * 4));  // past GV: reads zero (masked)
  const unsigned long long below = (1ull << lane) - 1ull;
  auto load = [&](int64_t it, f32x4 (&dst)[kTkwU]) {
#pragma unroll
    for (int u = 0; u < kTkwU; ++u) {
      const int64_t i = s0 + it * kTkwIter + 4 * (u * 64 + lane);
      if (RR) {  // per-lane block select; past the segment a harmless in-row address
        const float* a = i >= s1 ? rowA : (i < naq ? rowA + i : rowB + (i - naq));
        dst[u] = *reinterpret_cast<const f32x4*>(a);
      } else {
        dst[u] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(rrow, (int)(i < s1 ? i * 4 : GV * 4), 0, 0));
      }
    }
  };
  const int64_t niter = (s1 - s0 + kTkwIter - 1) / kTkwIter;
  int n = 0;
  unsigned long long thr = ~0ull;   // inclusive: entries <= thr stay candidates
  // Float pre-filter: an entry can only be <= thr if its distance is not
  // above thr's distance, !(e > thr_f) -- a superset of the exact test (NaN
  // entries and the initial NaN threshold pass it).  One compare per entry;
  // the append runs only for the entry slots where some lane passed.
  float thr_f = key_float((uint32_t)(thr >> 32));
  // one iteration: refill `nxt` (consumed by the previous iteration) with
  // iteration it + PPS_TKW_D, then filter `cur`.  Named buffers in a loop
  // unrolled by the rotation length: a rotating a = b, b = c would make the
  // compiler copy the registers at the end of every iteration and so wait for
  // the load it had just issued (vmcnt(0)).
  auto step = [&](int64_t it, const f32x4 (&cur)[kTkwU], f32x4 (&nxt)[kTkwU]) {
    if (n + kTkwIter > cap || (it == 1 && n > k + kTkwSlack)) {
      thr = wave_cut<tkw_j<KM>()>(buf, n, k, kTkwSlack);
      thr_f = key_float((uint32_t)(thr >> 32));
#if PPS_TKW_PROBE
      thr_f = -__builtin_huge_valf();   // timing probe only: stream, take nothing
#endif
    }
    // keep each step's refill in its step: a load hoisted above the previous
    // step's filter would overlap `nxt` with live buffers, and the loop head
    // would then wait for every load in flight
    asm volatile("" ::: "memory");
    load(it + PPS_TKW_D, nxt);
    unsigned long long m[kTkwU][4], any = 0ull;
    float ev[kTkwU][4];
#pragma unroll
    for (int u = 0; u < kTkwU; ++u) {
      const int64_t iv = s0 + it * kTkwIter + 4 * (u * 64 + lane);
      const float e[4] = {cur[u].x, cur[u].y, cur[u].z, cur[u].w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        ev[u][t] = xf(e[t], iv + t);
        m[u][t] = __ballot(!(ev[u][t] > thr_f));
        any |= m[u][t];
      }
    }
    if (!any) return;
    if ((it + 1) * kTkwIter > s1 - s0) {   // the segment's last iteration: exact, bounded
#pragma unroll
      for (int u = 0; u < kTkwU; ++u) {
        const int64_t i0 = s0 + it * kTkwIter + 4 * (u * 64 + lane);
        const float* e = ev[u];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (!m[u][t]) continue;
          const int64_t i = i0 + t;
          const unsigned long long packed = ((unsigned long long)float_key(e[t]) << 32) | col((uint32_t)i);
          const bool take = i < s1 && packed <= thr;
          const unsigned long long bal = __ballot(take);
          if (take) buf[n + __popcll(bal & below)] = packed;
          n += __popcll(bal);
        }
      }
      return;
    }
    // inside the segment every pre-filter passer is appended: an entry with
    // thr's distance but a larger index is a harmless extra candidate (cuts
    // rank packed values), so the slot costs the key, the lane's rank in the
    // pass mask and one LDS store
#pragma unroll
    for (int u = 0; u < kTkwU; ++u) {
      const uint32_t i0 = (uint32_t)(s0 + it * kTkwIter) + 4u * (uint32_t)(u * 64 + lane);
      const float* e = ev[u];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const unsigned long long mm = m[u][t];
        if (!mm) continue;
        if (!(e[t] > thr_f)) {
          const uint32_t ub = __float_as_uint(e[t]);
          const uint32_t key = ub ^ ((uint32_t)((int32_t)ub >> 31) | 0x80000000u);
          const int pos = n + (int)__builtin_amdgcn_mbcnt_hi(
                                  (uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
          buf[pos] = ((unsigned long long)key << 32) | col(i0 + (uint32_t)t);
        }
        n += __popcll(mm);
      }
    }
  };
  // Whole rounds: the iterations past the segment read zeros (buffer loads
  // past GV) and take nothing (i >= s1).
#if PPS_TKW_D == 3
  f32x4 a[kTkwU], b[kTkwU], c[kTkwU], d4[kTkwU];
  load(0, a);
  load(1, b);
  load(2, c);
  for (int64_t it = 0; it < niter; it += 4) {
    step(it, a, d4);
    step(it + 1, b, a);
    step(it + 2, c, b);
    step(it + 3, d4, c);
  }
#else
  f32x4 a[kTkwU], b[kTkwU], c[kTkwU];
  load(0, a);
  asm volatile("" ::: "memory");   // issue order a, b: the first step waits for a only
  load(1, b);
  for (int64_t it = 0; it < niter; it += 3) {
    step(it, a, c);
    step(it + 1, b, a);
    step(it + 2, c, b);
  }
#endif
  if (n > k) wave_cut<tkw_j<KM>()>(buf, n, k, 0);
  // the < 4 entries past the last float4: segment 0 takes them (scalar loads)
  if (wseg == 0 && GV < G) {
    const int64_t i = GV + lane;
    const bool take = i < G;
    const float e = RR ? (take ? xf(rowB[i - naq], i) : 0.f) : row[take ? i : 0];
    const unsigned long long packed =
        take ? (((unsigned long long)float_key(e) << 32) | col((uint32_t)i)) : ~0ull;
    const unsigned long long bal = __ballot(take);
    if (take) buf[n + __popcll(bal & below)] = packed;
    n += __popcll(bal);
  }
  if (WPR == 1) {   // the wave's own list is the row's: exact k, then sorted
    if (n > k) wave_cut<tkw_j<KM>()>(buf, n, k, 0);
    int n2 = 1;
    while (n2 < k) n2 <<= 1;
    for (int i = n + lane; i < n2; i += 64) buf[i] = ~0ull;
    wave_lds_sync();
    for (int size = 2; size <= n2; size <<= 1)
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int t = lane; t < n2 / 2; t += 64) {
          const int i = 2 * stride * (t / stride) + (t % stride), j = i + stride;
          const bool up = (i & size) == 0;
          const unsigned long long a = buf[i], b = buf[j];
          if ((a > b) == up) { buf[i] = b; buf[j] = a; }
        }
        wave_lds_sync();
      }
    for (int i = lane; i < k; i += 64) {
      const unsigned long long v = buf[i];
      vals[q * k + i] = key_float((uint32_t)(v >> 32));
      idx[q * k + i] = (int32_t)(v & 0xffffffffu);
    }
    return;
  }
  // merge: wave 0 reads the four lists (<= k + 3 entries each) and keeps the
  // row's k best at the front of the LDS; the block sorts them
  __shared__ int s_cnt[kTkwWaves];
  if (lane == 0) s_cnt[wave] = n;
  __syncthreads();
  if (wave == 0) {
    constexpr int MJ = tkw_merge_j<KM>();
    unsigned long long v[MJ];
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int p = j * 64 + lane;   // merged position
      int ww = 0, off = p;
      for (; ww < kTkwWaves && off >= s_cnt[ww]; ++ww) off -= s_cnt[ww];
      v[j] = ww < kTkwWaves ? tkw[ww * cap + off] : ~0ull;
    }
    int total = 0;
    for (int ww = 0; ww < kTkwWaves; ++ww) total += s_cnt[ww];
    const unsigned long long T = total > k ? wave_select(v, k, 0) : ~0ull - 1;
    wave_lds_sync();
    int m = 0;
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const bool keep = v[j] <= T;
      const unsigned long long bal = __ballot(keep);
      if (keep) tkw[m + __popcll(bal & below)] = v[j];
      m += __popcll(bal);
    }
    // pad to the sort length
    int n2 = 1;
    while (n2 < k) n2 <<= 1;
    for (int i = m + lane; i < n2; i += 64) tkw[i] = ~0ull;
  }
  __syncthreads();
  int n2 = 1;
  while (n2 < k) n2 <<= 1;
  block_bitonic(tkw, n2);
  __syncthreads();
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    const unsigned long long v = tkw[i];
    vals[q * k + i] = key_float((uint32_t)(v >> 32));
    idx[q * k + i] = (int32_t)(v & 0xffffffffu);
  }
}

// PPS_TOPK_WAVE=0: keep long rows on topk_kernel (A/B runs)
static bool topk_wave_enabled() {
  static const bool on = [] {
    const char* e = getenv("PPS_TOPK_WAVE");
    return !(e && e[0] == '0');
  }();
  return on;
}

int topk(const float* dist, int64_t Q, int64_t G, int64_t ldd, int k, float* vals,
         int32_t* idx, hipStream_t st) {
  if (Q <= 0) return PPS_OK;
  const bool v4 = (reinterpret_cast<uintptr_t>(dist) & 15) == 0 && (ldd & 3) == 0;
  if (v4 && G >= kTkwMinRow && k <= kTkwMaxK && topk_wave_enabled()) {
    const int cap = tkw_cap(k);
    const size_t lds = (size_t)kTkwWaves * cap * 8;
    const RrMatrix none{};
    if (k <= 128)
      hipLaunchKernelGGL((topk_wave_kernel<128, false>), dim3((unsigned)Q), dim3(kTopkThreads),
                         lds, st, dist, G, ldd, k, cap, vals, idx, none, Q, nullptr,
                         nullptr);
    else
      hipLaunchKernelGGL((topk_wave_kernel<kTkwMaxK, false>), dim3((unsigned)Q),
                         dim3(kTopkThreads), lds, st, dist, G, ldd, k, cap, vals, idx, none, Q, nullptr,
                         nullptr);
  } else if (v4)
    hipLaunchKernelGGL(topk_kernel<true>, dim3((unsigned)Q), dim3(kTopkThreads), 0, st, dist, G,
                       ldd, k, vals, idx);
  else
    hipLaunchKernelGGL(topk_kernel<false>, dim3((unsigned)Q), dim3(kTopkThreads), 0, st, dist,
                       G, ldd, k, vals, idx);
  PPS_CHECK_LAUNCH("topk_kernel");
  return PPS_OK;
}

bool topk_rr_eligible(const RrMatrix& M, int k) {
  auto a16 = [](const float* p, int64_t ld) { return aligned16(p) && (ld & 3) == 0; };
  return M.Q + M.G >= kTkwMinRow && k <= kTkwMaxK && topk_wave_enabled() &&
         a16(M.qq, M.ldqq) && a16(M.qg, M.ldqg) && a16(M.gg, M.ldgg) && a16(M.qgT, M.ldT) &&
         M.ldT >= (M.Q + 3) / 4 * 4 && M.ldqq >= (M.Q + 3) / 4 * 4 && M.Q + M.G < (1ll << 31);
}

int topk_rr(const RrMatrix& M, int k, float* vals, int32_t* idx, hipStream_t st) {
  const int64_t N = M.Q + M.G;
  if (!topk_rr_eligible(M, k)) {
    set_error("topk_rr: needs N >= 16384, k <= 256 and 16-byte aligned block rows");
    return PPS_ERR_INVALID_ARG;
  }
  const int cap = tkw_cap(k);
  const size_t lds = (size_t)kTkwWaves * cap * 8;
  // one wave per row (PPS_TOPK_RR_WPR=4: the block per row, A/B runs)
  static const bool wpr4 = [] {
    const char* e = getenv("PPS_TOPK_RR_WPR");
    return e && e[0] == '4';
  }();
  const unsigned rows_grid = (unsigned)((N + kTkwWaves - 1) / kTkwWaves);
  if (wpr4 && k <= 128)
    hipLaunchKernelGGL((topk_wave_kernel<128, true>), dim3((unsigned)N), dim3(kTopkThreads), lds,
                       st, nullptr, (int64_t)0, (int64_t)0, k, cap, vals, idx, M, N, nullptr, nullptr);
  else if (wpr4)
    hipLaunchKernelGGL((topk_wave_kernel<kTkwMaxK, true>), dim3((unsigned)N), dim3(kTopkThreads),
                       lds, st, nullptr, (int64_t)0, (int64_t)0, k, cap, vals, idx, M, N, nullptr, nullptr);
  else if (k <= 128)
    hipLaunchKernelGGL((topk_wave_kernel<128, true, 1>), dim3(rows_grid), dim3(kTopkThreads),
                       lds, st, nullptr, (int64_t)0, (int64_t)0, k, cap, vals, idx, M, N, nullptr, nullptr);
  else
    hipLaunchKernelGGL((topk_wave_kernel<kTkwMaxK, true, 1>), dim3(rows_grid),
                       dim3(kTopkThreads), lds, st, nullptr, (int64_t)0, (int64_t)0, k, cap,
                       vals, idx, M, N, nullptr, nullptr);
  PPS_CHECK_LAUNCH("topk_wave_kernel<rr>");
  return PPS_OK;
}

// Re-ranking's first pass over a symmetric M (rerank.hip, in place): per row
// q the top-k' by (m * m, index) over M's row -- its first block (qq or
// q_g^T, Q entries) then its second (q_g or g_g, G entries), column = Q +
// position in the second -- and rowmax[q] = the max of the row's squares,
// which for a symmetric M is colmax[q] (:453).  OD = (m * m) / colmax is a
// monotone map of m * m, so rerank_rank_fix_kernel gets the top-k by (OD,
// index) from this list.  One wave per row (four rows per block) streams the
// two blocks as two segments through the same candidate buffer and threshold
// (topk_wave_kernel's filter / cut / select); per entry one product, one
// compare and one max, 32-bit offsets into buffer descriptors.
//
// The list's fix-up runs in the same wave once the row max is known: OD of
// each of the k' = kp entries, and when the kp-th entry's OD is above the
// k-th's (so every entry outside the list has OD above the k-th too) the
// top-k by (OD, index) is the list's k smallest (OD, index) pairs -- written
// to vals (OD) / idx.  Otherwise (an equal-OD run longer than the slack) the
// row goes to fb_rows for the exact OD pass.
template <int KM>
__global__ void __launch_bounds__(kTopkThreads) __attribute__((amdgpu_waves_per_eu(6)))
topk_rr_sq_kernel(RrMatrix rr, int k, int kp, int cap, float* __restrict__ vals,
                  int32_t* __restrict__ idx, float* __restrict__ rowmax,
                  int32_t* __restrict__ fb_rows, int32_t* __restrict__ fb_n) {
  extern __shared__ unsigned long long tkw[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  unsigned long long* buf = tkw + wave * cap;
  const int64_t q = (int64_t)blockIdx.x * kTkwWaves + wave;
  if (q >= rr.Q + rr.G) return;
  const float* rowA = q < rr.Q ? rr.qq + q * rr.ldqq : rr.qgT + (q - rr.Q) * rr.ldT;
  const float* rowB = q < rr.Q ? rr.qg + q * rr.ldqg : rr.gg + (q - rr.Q) * rr.ldgg;
  const unsigned long long below = (1ull << lane) - 1ull;
  int n = 0, cuts = 0;
  unsigned long long thr = ~0ull;
  float thr_f = key_float((uint32_t)(thr >> 32));   // NaN: everything passes
  float mx = 0.f;
  auto cut = [&]() {
    thr = wave_cut<tkw_j<KM>()>(buf, n, kp, kTkwSlack);
    thr_f = key_float((uint32_t)(thr >> 32));
    ++cuts;
  };
  auto segment = [&](const float* base, uint32_t L, uint32_t col0) {
    const uint32_t V = L & ~3u;
    const rsrc_t rs = make_rsrc(base, V * 4u);
    const uint32_t niter = (V + kTkwIter - 1) / kTkwIter;
    auto load = [&](uint32_t it, f32x4 (&dst)[kTkwU]) {
#pragma unroll
      for (int u = 0; u < kTkwU; ++u)
        dst[u] = __builtin_bit_cast(
            f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                       rs, (int)((it * kTkwIter + 4u * (uint32_t)(u * 64 + lane)) * 4u), 0, 0));
    };
    auto step = [&](uint32_t it, const f32x4 (&cur)[kTkwU], f32x4 (&nxt)[kTkwU]) {
      if (n + kTkwIter > cap || (cuts == 0 && n > kp + kTkwSlack)) cut();
      asm volatile("" ::: "memory");
      load(it + PPS_TKW_D, nxt);
      const uint32_t i0 = it * kTkwIter;
      const bool last = i0 + kTkwIter > V;   // wave-uniform: the only partial iteration
      float sq[kTkwU][4];
      unsigned long long m[kTkwU][4], any = 0ull;
#pragma unroll
      for (int u = 0; u < kTkwU; ++u) {
        const float e[4] = {cur[u].x, cur[u].y, cur[u].z, cur[u].w};
        const uint32_t iv = i0 + 4u * (uint32_t)(u * 64 + lane);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          sq[u][t] = e[t] * e[t];
          const bool valid = !last || iv + t < V;
          mx = valid ? fmaxf(mx, sq[u][t]) : mx;
          m[u][t] = __ballot(valid && !(sq[u][t] > thr_f));
          any |= m[u][t];
        }
      }
      if (!any) return;
#pragma unroll
      for (int u = 0; u < kTkwU; ++u) {
        const uint32_t iv = i0 + 4u * (uint32_t)(u * 64 + lane);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const unsigned long long mm = m[u][t];
          if (!mm) continue;
          if ((mm >> lane) & 1ull) {
            const uint32_t ub = __float_as_uint(sq[u][t]);
            const uint32_t key = ub ^ ((uint32_t)((int32_t)ub >> 31) | 0x80000000u);
            const int pos = n + (int)__builtin_amdgcn_mbcnt_hi(
                                    (uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
            buf[pos] = ((unsigned long long)key << 32) | (col0 + iv + (uint32_t)t);
          }
          n += __popcll(mm);
        }
      }
    };
    f32x4 a[kTkwU], b[kTkwU], c[kTkwU];
    load(0, a);
    asm volatile("" ::: "memory");
    load(1, b);
    for (uint32_t it = 0; it < niter; it += 3) {
      step(it, a, c);
      if (it + 1 < niter) step(it + 1, b, a);
      if (it + 2 < niter) step(it + 2, c, b);
    }
    // the < 4 entries past the last float4
    if (V < L) {
      if (n + 4 > cap) cut();
      const bool take = lane < (int)(L - V);
      const float e = take ? base[V + lane] : 0.f;
      const float s2 = e * e;
      if (take) mx = fmaxf(mx, s2);
      const unsigned long long packed =
          ((unsigned long long)float_key(s2) << 32) | (col0 + V + (uint32_t)lane);
      const bool keep = take && packed <= thr;
      const unsigned long long bal = __ballot(keep);
      if (keep) buf[n + __popcll(bal & below)] = packed;
      n += __popcll(bal);
    }
    wave_lds_sync();
  };
  segment(rowA, (uint32_t)rr.Q, 0u);
  segment(rowB, (uint32_t)rr.G, (uint32_t)rr.Q);
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if (lane == 0) rowmax[q] = mx;
  if (n > kp) wave_cut<tkw_j<KM>()>(buf, n, kp, 0);   // exactly the kp best (row >= kp)
  // fix-up: one list entry per lane (kp <= 64)
  const unsigned long long v = lane < kp ? buf[lane] : ~0ull;
  const float od = key_float((uint32_t)(v >> 32)) / mx;   // rr_od's (m * m) / colmax
  int ps = 0;   // position in (m * m, index) order
  for (int t = 0; t < kp; ++t) ps += __shfl(v, t) < v ? 1 : 0;
  const unsigned long long at_k = __ballot(lane < kp && ps == k - 1);
  const unsigned long long at_l = __ballot(lane < kp && ps == kp - 1);
  const float vk = __shfl(od, (int)__builtin_ctzll(at_k)), vl = __shfl(od, (int)__builtin_ctzll(at_l));
  if (!(vl > vk)) {
    if (lane == 0) fb_rows[atomicAdd(fb_n, 1)] = (int32_t)q;
    return;
  }
  const unsigned long long packed =
      lane < kp ? (((unsigned long long)float_key(od) << 32) | (v & 0xffffffffu)) : ~0ull;
  int pos = 0;
  for (int t = 0; t < kp; ++t) pos += __shfl(packed, t) < packed ? 1 : 0;
  if (lane < kp && pos < k) {
    vals[q * k + pos] = od;
    idx[q * k + pos] = (int32_t)(v & 0xffffffffu);
  }
}

int topk_rr_sq(const RrMatrix& M, int k, float* rowmax, void* scratch, size_t scratch_bytes,
               float* vals, int32_t* idx, hipStream_t st) {
  const int64_t N = M.Q + M.G;
  const int kp = k + 8 < 64 ? k + 8 : 64;
  if (!topk_rr_eligible(M, kp)) {
    set_error("topk_rr_sq: needs N >= 16384, k <= 256 and 16-byte aligned block rows");
    return PPS_ERR_INVALID_ARG;
  }
  if (scratch_bytes < topk_rr_sq_scratch_bytes(N, k)) {
    set_error("topk_rr_sq: scratch too small");
    return PPS_ERR_CAPACITY;
  }
  int32_t* fb_n = reinterpret_cast<int32_t*>(scratch);
  int32_t* fb_rows = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(scratch) + 256);
  (void)hipMemsetAsync(fb_n, 0, sizeof(int32_t), st);
  const unsigned grid = (unsigned)((N + kTkwWaves - 1) / kTkwWaves);
  const int capp = tkw_cap(kp);
  hipLaunchKernelGGL(topk_rr_sq_kernel<128>, dim3(grid), dim3(kTopkThreads),
                     (size_t)kTkwWaves * capp * 8, st, M, k, kp, capp, vals, idx, rowmax, fb_rows,
                     fb_n);
  PPS_CHECK_LAUNCH("topk_rr_sq_kernel");
  // the exact OD pass over the rows the list could not settle (grid for all
  // rows; waves past *fb_n return at once)
  RrMatrix Mc = M;
  Mc.colmax = rowmax;
  const int cap = tkw_cap(k);
  hipLaunchKernelGGL((topk_wave_kernel<128, true, 1>), dim3(grid), dim3(kTopkThreads),
                     (size_t)kTkwWaves * cap * 8, st, nullptr, (int64_t)0, (int64_t)0, k, cap,
                     vals, idx, Mc, N, fb_rows, fb_n);
  PPS_CHECK_LAUNCH("topk_wave_kernel<rr, rows>");
  return PPS_OK;
}

size_t topk_rr_sq_scratch_bytes(int64_t N, int) {
  return 256 + (sizeof(int32_t) * N + 255) / 256 * 256;
}

// ---- k-way merge of per-shard top-k lists ------------------------
// R gallery shards each hold a stable ascending top-k_in list per query
// (local indices; list r's global offset off[r]).  The global stable top-k_out
// is their merge by the packed (order-preserving key << 32 | global index)
// value.  Packed values are unique (global indices are), so an entry's output
// position is exactly its position in its own list plus, for every other list,
// the number of that list's entries below it (a binary search in LDS): every
// entry is placed independently, no sort and no serial merge.  Pad entries
// (index < 0, e.g. shards shorter than k_in) pack to ~0 and are never placed;
// output positions past the number of real entries get (+inf, -1).
constexpr int kMergeThreads = 256;

__global__ void topk_merge_kernel(const float* __restrict__ vals,
                                  const int32_t* __restrict__ idx, int R, int64_t Q,
                                  int kin, MergeOffsets offs, int kout,
                                  float* __restrict__ out_vals,
                                  int32_t* __restrict__ out_idx) {
  const int64_t q = blockIdx.x;
  extern __shared__ unsigned long long mkeys[];
  __shared__ int s_real;
  const int n = R * kin;
  if (threadIdx.x == 0) s_real = 0;
  __syncthreads();
  int real = 0;
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    const int r = t / kin, p = t - r * kin;
    const int64_t src = ((int64_t)r * Q + q) * kin + p;
    const int32_t li = idx[src];
    unsigned long long key = ~0ull;
    if (li >= 0) {
      key = ((unsigned long long)float_key(vals[src]) << 32) |
            (uint32_t)(offs.off[r] + li);
      ++real;
    }
    mkeys[t] = key;
  }
  atomicAdd(&s_real, real);
  __syncthreads();
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    const unsigned long long key = mkeys[t];
    if (key == ~0ull) continue;
    const int r = t / kin;
    int pos = t - r * kin;
    for (int o = 0; o < R && pos < kout; ++o) {
      if (o == r) continue;
      const unsigned long long* L = mkeys + o * kin;
      int lo = 0, hi = kin;  // lower_bound: entries of list o below key
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (L[mid] < key) lo = mid + 1; else hi = mid;
      }
      pos += lo;
    }
    if (pos < kout) {
      out_vals[q * kout + pos] = key_float((uint32_t)(key >> 32));
      out_idx[q * kout + pos] = (int32_t)(key & 0xffffffffu);
    }
  }
  for (int p = s_real + threadIdx.x; p < kout; p += blockDim.x) {
    out_vals[q * kout + p] = INFINITY;
    out_idx[q * kout + p] = -1;
  }
}

int topk_merge(const float* vals, const int32_t* idx, int R, int64_t Q, int kin,
               const MergeOffsets& offs, int kout, float* out_vals, int32_t* out_idx,
               hipStream_t st) {
  if (Q <= 0) return PPS_OK;
  const size_t lds = (size_t)R * kin * sizeof(unsigned long long);
  hipLaunchKernelGGL(topk_merge_kernel, dim3((unsigned)Q), dim3(kMergeThreads), lds, st,
                     vals, idx, R, Q, kin, offs, kout, out_vals, out_idx);
  PPS_CHECK_LAUNCH("topk_merge_kernel");
  return PPS_OK;
}

}  // namespace pps
