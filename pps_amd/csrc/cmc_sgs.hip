// CMC with single_gallery_shot=True (reid_dataset_evaluator.py:334-346):
// every valid query repeats 100 times "draw one valid gallery entry per
// identity (`_unique_sample`, :275-280), find the rank of the query
// identity's draw among the draws".  The draws themselves stay with the
// caller's NumPy RNG (the reference's np.random.choice stream, reproduced
// exactly by one vectorised randint per query); these kernels do everything
// around them on the device, from the stable rank order of pps_argsort_rows:
//
//  1. sgs_keys: key[q][p] = dense identity of the p-th ranked gallery entry
//     of query q, or U (sorts last) when the entry is not valid for q (same
//     identity and camera; with separate_camera_set also any same camera).
//  2. pps_argsort_rows of the keys (caller) -> perm[q][j]: the valid ranked
//     positions grouped by identity, ascending inside a group -- exactly the
//     reference's `ids_dict[x]` lists (:335-339).
//  3. sgs_groups: per query, each identity's group start / length and its
//     insertion rank (the order in which `ids_dict` first meets it = by the
//     group's first position), so that a group's draws are addressed in the
//     order the reference makes them.
//  4. (host) draws[r][t] = randint(0, glen[t]) for r < repeat, t < nids.
//  5. sgs_ranks: per query and repeat, pick[t] = perm[gstart[t] + draw[t]];
//     k = #{t : pick[t] < pick[query identity]} = the reference's
//     `np.nonzero(matches[i, sampled])[0]` (one hit per repeat).
#include "pps_internal.hpp"

namespace pps {

namespace {

constexpr int kSgsThreads = 1024;

__global__ void sgs_keys_kernel(const int32_t* __restrict__ order, int64_t Q, int G, int64_t ldo,
                                const int32_t* __restrict__ gid, const int32_t* __restrict__ gcam,
                                const int32_t* __restrict__ qid, const int32_t* __restrict__ qcam,
                                int sep, int U, float* __restrict__ keys) {
  const int64_t n = Q * G;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = e / G;
    const int p = (int)(e - q * G);
    const int g = order[q * ldo + p];
    const int x = gid[g], c = gcam[g], cq = qcam[q];
    bool valid = x != qid[q] || c != cq;   // :323-325
    if (sep) valid = valid && c != cq;     // :327-328
    keys[e] = valid ? (float)x : (float)U;
  }
}

// One workgroup per query (persistent).  LDS: gs[U], ge[U] (group bounds in
// perm), bits[W] (first positions of the groups), pre[W] (exclusive
// popcount prefix of bits).
__global__ void __launch_bounds__(kSgsThreads)
sgs_groups_kernel(const float* __restrict__ skeys, const int32_t* __restrict__ perm, int64_t Q,
                  int G, int U, const int32_t* __restrict__ qid, int32_t* __restrict__ gstart,
                  int32_t* __restrict__ glen, int32_t* __restrict__ nids, int32_t* __restrict__ qt) {
  extern __shared__ int32_t sg_lds[];
  const int W = (G + 31) / 32;
  int32_t* gs = sg_lds;
  int32_t* ge = gs + U;
  uint32_t* bits = reinterpret_cast<uint32_t*>(ge + U);
  int32_t* pre = reinterpret_cast<int32_t*>(bits + W);
  __shared__ int32_t wsum[kSgsThreads / 64];
  const int t = threadIdx.x;
  for (int64_t q = blockIdx.x; q < Q; q += gridDim.x) {
    for (int i = t; i < U; i += kSgsThreads) gs[i] = ge[i] = 0;
    for (int i = t; i < W; i += kSgsThreads) bits[i] = 0u;
    __syncthreads();
    const float* krow = skeys + q * G;
    const int32_t* prow = perm + q * G;
    for (int j = t; j < G; j += kSgsThreads) {
      const int x = (int)krow[j];
      if (x >= U) continue;   // invalid entries sort last
      if (j == 0 || (int)krow[j - 1] != x) {
        gs[x] = j;
        const int p = prow[j];   // the group's first (smallest) ranked position
        atomicOr(&bits[p >> 5], 1u << (p & 31));
      }
      if (j + 1 == G || (int)krow[j + 1] != x) ge[x] = j + 1;
    }
    __syncthreads();
    // exclusive prefix of the popcounts: thread t owns words [t * PW, t * PW + PW)
    const int PW = (W + kSgsThreads - 1) / kSgsThreads;
    int c = 0;
    for (int j = 0; j < PW; ++j) {
      const int wd = t * PW + j;
      if (wd < W) c += __popc(bits[wd]);
    }
    int v = c;
    const int lane = t & 63, wv = t >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(v, o, 64);
      if (lane >= o) v += y;
    }
    if (lane == 63) wsum[wv] = v;
    __syncthreads();
    int base = 0;
    for (int w = 0; w < wv; ++w) base += wsum[w];
    int run = base + v - c;
    for (int j = 0; j < PW; ++j) {
      const int wd = t * PW + j;
      if (wd < W) { pre[wd] = run; run += __popc(bits[wd]); }
    }
    if (t == kSgsThreads - 1) nids[q] = base + v;
    __syncthreads();
    int32_t* gsq = gstart + q * U;
    int32_t* glq = glen + q * U;
    const int xq = qid[q];
    for (int x = t; x < U; x += kSgsThreads) {
      if (ge[x] <= gs[x]) {
        if (x == xq) qt[q] = -1;   // no valid entry of the query identity
        continue;
      }
      const int p = prow[gs[x]];
      const int r = pre[p >> 5] + __popc(bits[p >> 5] & ((1u << (p & 31)) - 1u));
      gsq[r] = gs[x];
      glq[r] = ge[x] - gs[x];
      if (x == xq) qt[q] = r;
    }
    if (t == 0 && (xq < 0 || xq >= U)) qt[q] = -1;
    __syncthreads();
  }
}

// One workgroup per listed query (persistent); draws [nr][repeat][ldd].
__global__ void __launch_bounds__(256)
sgs_ranks_kernel(const int32_t* __restrict__ perm, int G, const int32_t* __restrict__ rows,
                 int64_t nr, const int32_t* __restrict__ gstart, const int32_t* __restrict__ glen,
                 const int32_t* __restrict__ nids, const int32_t* __restrict__ qt, int U,
                 int repeat, const int32_t* __restrict__ draws, int64_t ldd,
                 int32_t* __restrict__ kout) {
  __shared__ int32_t s_pq;
  __shared__ int32_t s_red[4];
  const int t = threadIdx.x;
  for (int64_t i = blockIdx.x; i < nr; i += gridDim.x) {
    const int64_t q = rows[i];
    const int n = nids[q], tq = qt[q];
    const int32_t* prow = perm + q * G;
    const int32_t* gsq = gstart + q * U;
    const int32_t* glq = glen + q * U;
    for (int r = 0; r < repeat; ++r) {
      const int32_t* d = draws + (i * repeat + r) * ldd;
      auto pick = [&](int u) {
        int k = d[u];
        const int l = glq[u];
        k = k < 0 ? 0 : (k >= l ? l - 1 : k);   // a bad draw cannot leave the group
        return prow[gsq[u] + k];
      };
      if (t == 0) s_pq = tq >= 0 ? pick(tq) : -1;
      __syncthreads();
      const int pq = s_pq;
      int c = 0;
      for (int u = t; u < n; u += 256) c += pick(u) < pq;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
      if ((t & 63) == 0) s_red[t >> 6] = c;
      __syncthreads();
      if (t == 0) kout[i * repeat + r] = tq >= 0 ? s_red[0] + s_red[1] + s_red[2] + s_red[3] : -1;
    }
  }
}

int sgs_grid(int64_t work, int per_cu) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t cap = (int64_t)cus * per_cu;
  return (int)(work < cap ? (work > 0 ? work : 1) : cap);
}

}  // namespace

size_t sgs_groups_lds_bytes(int64_t G, int U) {
  return (size_t)8 * U + (size_t)8 * ((G + 31) / 32);
}

int sgs_keys(const int32_t* order, int64_t Q, int64_t G, int64_t ldo, const int32_t* gid,
             const int32_t* gcam, const int32_t* qid, const int32_t* qcam, int sep, int U,
             float* keys, hipStream_t st) {
  if (Q <= 0 || G <= 0) return PPS_OK;
  const int64_t blocks = (Q * G + 255) / 256;
  hipLaunchKernelGGL(sgs_keys_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256),
                     0, st, order, Q, (int)G, ldo, gid, gcam, qid, qcam, sep, U, keys);
  PPS_CHECK_LAUNCH_S("sgs_keys_kernel", st);
  return PPS_OK;
}

int sgs_groups(const float* skeys, const int32_t* perm, int64_t Q, int64_t G, int U,
               const int32_t* qid, int32_t* gstart, int32_t* glen, int32_t* nids, int32_t* qt,
               hipStream_t st) {
  if (Q <= 0) return PPS_OK;
  hipLaunchKernelGGL(sgs_groups_kernel, dim3(sgs_grid(Q, 1)), dim3(kSgsThreads),
                     sgs_groups_lds_bytes(G, U), st, skeys, perm, Q, (int)G, U, qid, gstart, glen,
                     nids, qt);
  PPS_CHECK_LAUNCH_S("sgs_groups_kernel", st);
  return PPS_OK;
}

int sgs_ranks(const int32_t* perm, int64_t G, const int32_t* rows, int64_t nr,
              const int32_t* gstart, const int32_t* glen, const int32_t* nids, const int32_t* qt,
              int U, int repeat, const int32_t* draws, int64_t ldd, int32_t* kout,
              hipStream_t st) {
  if (nr <= 0 || repeat <= 0) return PPS_OK;
  hipLaunchKernelGGL(sgs_ranks_kernel, dim3(sgs_grid(nr, 8)), dim3(256), 0, st, perm, (int)G,
                     rows, nr, gstart, glen, nids, qt, U, repeat, draws, ldd, kout);
  PPS_CHECK_LAUNCH_S("sgs_ranks_kernel", st);
  return PPS_OK;
}

}  // namespace pps
