// Full stable argsort of every distance row: idx[q][j] = the j-th gallery
// column in (distance, index) order -- the reference's rank list
// `np.argsort(distmat, axis=1)` (reid_dataset_evaluator.py:319, :420) for
// callers that need all G columns (writing ranked lists), not only the top-k
// pps_topk gives.  np.argsort's default quicksort leaves ties in an
// unspecified order; this is the stable order (= kind='stable').
//
// One workgroup per row at a time (persistent over rows), the row held in
// LDS as packed 64-bit (order-preserving key << 32 | column) values:
//  1. the row's entries are loaded (the NEXT row's loads are issued before
//     this row is sorted, so HBM latency hides under the sort), keyed, and
//     their min / max key found;
//  2. a bucket per entry from a monotone map of its key onto kSortBuckets
//     equal ranges of [min, max] (the distances' own range, so a row of
//     values that share their exponent still spreads); LDS histogram,
//     exclusive scan, and a scatter by per-bucket atomic cursors (the order
//     inside a bucket is arbitrary: the packed key decides it below);
//  3. an entry's final position = its bucket's start + the number of packed
//     keys in its bucket below its own (a handful per bucket on distance
//     rows) -- written straight to the row of idx; buckets holding more than
//     kSortSmall entries (ties, degenerate rows) are sorted in place by one
//     wave with a bitonic network and written in order.
// Algorithmic bytes per row: G * 4 read + G * 4 written (+ G * 4 with vals).
#include "pps_internal.hpp"

namespace pps {

namespace {

constexpr int kSortThreads = 512;
constexpr int kSortBuckets = 4096;
constexpr int kSortSmall = 64;   // larger buckets: one wave's bitonic sort
constexpr int kSortBigMax = 18432 / kSortSmall;   // buckets that can exceed kSortSmall
// LDS: packed row (8 B per entry) + bucket offsets + the large-bucket list,
// within 160 KiB
constexpr int kSortCap = (160 * 1024 - 4 * kSortBuckets - 4 * kSortBigMax - 256) / 8 / 64 * 64;
constexpr int kSortU = (kSortCap + kSortThreads - 1) / kSortThreads;            // entries per thread

#ifdef PPS_SORT_PROBE
// phase cycle counts of workgroup 0 (scripts/probes/argsort_phases.py)
__device__ unsigned long long g_sort_phase[16];
#define SORT_PHASE(k)                                  \
  do {                                                 \
    if (t == 0 && blockIdx.x == 0) {                   \
      const unsigned long long c = clock64();          \
      ph[k] += c - ph_last;                            \
      ph_last = c;                                     \
    }                                                  \
  } while (0)
#else
#define SORT_PHASE(k) do {} while (0)
#endif

// -0.0 is keyed as +0.0 (they compare equal, so NumPy's stable sort keeps
// them in index order)
__device__ inline uint32_t sort_key(float f) {
  const uint32_t u = __float_as_uint(f + 0.0f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ inline float sort_key_float(uint32_t k) {
  const uint32_t u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

__global__ void __launch_bounds__(kSortThreads)
argsort_rows_kernel(const float* __restrict__ dist, int64_t Q, int G, int64_t ldd,
                    int32_t* __restrict__ idx, int64_t ldi, float* __restrict__ vals,
                    int64_t ldv) {
  __shared__ unsigned long long pk[kSortCap];
  __shared__ unsigned off[kSortBuckets];
  __shared__ uint32_t red_min[kSortThreads / 64], red_max[kSortThreads / 64];
  __shared__ int big[kSortBigMax];   // buckets over kSortSmall entries
  __shared__ int s_nbig;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  constexpr int NW = kSortThreads / 64;
  float cur[kSortU], nxt[kSortU];
  auto load = [&](int64_t q, float (&dst)[kSortU]) {
    const float* row = dist + q * ldd;
#pragma unroll
    for (int u = 0; u < kSortU; ++u) {
      const int i = t + u * kSortThreads;
      dst[u] = (q < Q && i < G) ? __builtin_nontemporal_load(row + i) : 0.f;
    }
  };
#ifdef PPS_SORT_PROBE
  unsigned long long ph[16] = {}, ph_last = clock64();
#endif
  int64_t q = blockIdx.x;
  load(q, cur);
  for (; q < Q; q += gridDim.x) {
    SORT_PHASE(0);
    load(q + gridDim.x, nxt);   // the next row's loads fly under this row's sort
    // 1) keys, min / max
    uint32_t kmn = 0xffffffffu, kmx = 0u;
#pragma unroll
    for (int u = 0; u < kSortU; ++u) {
      const int i = t + u * kSortThreads;
      if (i < G) {
        const uint32_t k = sort_key(cur[u]);
        kmn = k < kmn ? k : kmn;
        kmx = k > kmx ? k : kmx;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t a = __shfl_xor(kmn, o), b = __shfl_xor(kmx, o);
      kmn = a < kmn ? a : kmn;
      kmx = b > kmx ? b : kmx;
    }
    if (lane == 0) { red_min[wave] = kmn; red_max[wave] = kmx; }
    for (int b = t; b < kSortBuckets; b += kSortThreads) off[b] = 0u;
    __syncthreads();
    SORT_PHASE(1);
    kmn = red_min[0];
    kmx = red_max[0];
    for (int w = 1; w < NW; ++w) {
      kmn = red_min[w] < kmn ? red_min[w] : kmn;
      kmx = red_max[w] > kmx ? red_max[w] : kmx;
    }
    // monotone bucket map: float conversion, product and truncation never
    // reverse the order of two keys
    const float fscale = (float)kSortBuckets / ((float)(kmx - kmn) + 1.0f);
    auto bucket = [&](uint32_t k) {
      const int b = (int)((float)(k - kmn) * fscale);
      return b < kSortBuckets - 1 ? b : kSortBuckets - 1;
    };
    // 2) histogram, exclusive scan, scatter
#pragma unroll
    for (int u = 0; u < kSortU; ++u) {
      const int i = t + u * kSortThreads;
      if (i < G) atomicAdd(&off[bucket(sort_key(cur[u]))], 1u);
    }
    __syncthreads();
    SORT_PHASE(2);
    {  // block exclusive scan of off[] (kSortBuckets / kSortThreads per thread)
      constexpr int PER = kSortBuckets / kSortThreads;
      unsigned v[PER], s = 0;
#pragma unroll
      for (int j = 0; j < PER; ++j) { v[j] = off[t * PER + j]; s += v[j]; }
      unsigned incl = s;
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      __syncthreads();
      if (lane == 63) red_min[wave] = incl;   // wave totals (reuses the scratch)
      __syncthreads();
      unsigned base = 0;
      for (int w = 0; w < wave; ++w) base += red_min[w];
      unsigned run = base + incl - s;
#pragma unroll
      for (int j = 0; j < PER; ++j) { off[t * PER + j] = run; run += v[j]; }
    }
    __syncthreads();
    SORT_PHASE(3);
#pragma unroll
    for (int u = 0; u < kSortU; ++u) {
      const int i = t + u * kSortThreads;
      if (i < G) {
        const uint32_t k = sort_key(cur[u]);
        const unsigned pos = atomicAdd(&off[bucket(k)], 1u);   // off[b] ends at bucket b's end
        pk[pos] = ((unsigned long long)k << 32) | (uint32_t)i;
      }
    }
    __syncthreads();
    SORT_PHASE(4);
    // 3) the buckets holding more than kSortSmall entries (ties, degenerate
    // rows): a list in LDS, found by every thread over its own buckets
    if (t == 0) s_nbig = 0;
    __syncthreads();
    for (int b = t; b < kSortBuckets; b += kSortThreads) {
      const int s = b ? (int)off[b - 1] : 0, e = (int)off[b];
      if (e - s > kSortSmall) big[atomicAdd(&s_nbig, 1)] = b;
    }
    // 4) small buckets: every entry's rank among its bucket's packed keys,
    // then (after the barrier: the ranks read the unsorted bucket) written
    // to its final slot -- pk ends up sorted
    unsigned long long sv[kSortU];
    int sp[kSortU];
#pragma unroll
    for (int u = 0; u < kSortU; ++u) {
      const int p = t + u * kSortThreads;
      sp[u] = -1;
      if (p < G) {
        const unsigned long long v = pk[p];
        const int b = bucket((uint32_t)(v >> 32));
        const int s = b ? (int)off[b - 1] : 0, e = (int)off[b];
        if (e - s <= kSortSmall) {
          // the bucket's first 8 entries in one batch of loads (the bucket
          // holds this entry, so s + min(k, n - 1) is in it), the rest after:
          // one LDS latency per entry instead of one per compare
          const int n = e - s;
          unsigned long long w[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) w[k] = pk[s + (k < n ? k : n - 1)];
          int r = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k) r += (k < n && w[k] < v) ? 1 : 0;
          for (int j = s + 8; j < e; ++j) r += pk[j] < v ? 1 : 0;
          sv[u] = v;
          sp[u] = s + r;
        }
      }
    }
    __syncthreads();
    SORT_PHASE(5);
#pragma unroll
    for (int u = 0; u < kSortU; ++u)
      if (sp[u] >= 0) pk[sp[u]] = sv[u];
    SORT_PHASE(6);
    // large buckets: one wave each, bitonic network for any length in place
    // (mirror step, then half-cleaners; partners past the end are skipped)
    for (int bi = wave; bi < s_nbig; bi += NW) {
      const int b = big[bi];
      const int s = b ? (int)off[b - 1] : 0, e = (int)off[b];
      const int n = e - s;
      unsigned long long* a = pk + s;
      int n2 = 1;
      while (n2 < n) n2 <<= 1;
      for (int size = 2; size <= n2; size <<= 1) {
        const int half = size >> 1;
        for (int x = lane; x < n2 / 2; x += 64) {
          const int bb = x / half, o = x - bb * half;
          const int i = bb * size + o, j = bb * size + size - 1 - o;
          if (j < n) {
            const unsigned long long ai = a[i], aj = a[j];
            if (aj < ai) { a[i] = aj; a[j] = ai; }
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int stride = half >> 1; stride > 0; stride >>= 1) {
          for (int x = lane; x < n2 / 2; x += 64) {
            const int bb = x / stride, o = x - bb * stride;
            const int i = 2 * bb * stride + o, j = i + stride;
            if (j < n) {
              const unsigned long long ai = a[i], aj = a[j];
              if (aj < ai) { a[i] = aj; a[j] = ai; }
            }
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
      }
    }
    __syncthreads();
    SORT_PHASE(7);
    // 5) the sorted row out, coalesced
    int32_t* orow = idx + q * ldi;
    float* vrow = vals ? vals + q * ldv : nullptr;
    for (int p = t; p < G; p += kSortThreads) {
      const unsigned long long v = pk[p];
      orow[p] = (int32_t)(uint32_t)v;
      if (vrow) vrow[p] = sort_key_float((uint32_t)(v >> 32));
    }
    __syncthreads();   // pk / off are rebuilt for the next row
    SORT_PHASE(8);
#pragma unroll
    for (int u = 0; u < kSortU; ++u) cur[u] = nxt[u];
    SORT_PHASE(9);
  }
#ifdef PPS_SORT_PROBE
  if (t == 0 && blockIdx.x == 0) {
    ph[15] = 1;
    for (int k = 0; k < 16; ++k) g_sort_phase[k] = ph[k];
  }
#endif
}

}  // namespace

int argsort_rows_cap() { return kSortCap; }

#ifdef PPS_SORT_PROBE
extern "C" int pps_sort_probe_read(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sort_phase), sizeof(g_sort_phase)) == hipSuccess
             ? 0 : -1;
}
#endif

int argsort_rows(const float* dist, int64_t Q, int64_t G, int64_t ldd, int32_t* idx,
                 int64_t ldi, float* vals, int64_t ldv, hipStream_t st) {
  if (Q <= 0 || G <= 0) return PPS_OK;
  if (G > kSortCap) {
    set_error("argsort_rows: rows of " + std::to_string(G) + " entries exceed the " +
              std::to_string(kSortCap) + " an LDS row holds (use pps_topk for the first k)");
    return PPS_ERR_CAPACITY;
  }
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t grid = Q < cus ? Q : cus;   // one resident workgroup per CU (LDS)
  hipLaunchKernelGGL(argsort_rows_kernel, dim3((unsigned)grid), dim3(kSortThreads), 0, st, dist,
                     Q, (int)G, ldd, idx, ldi, vals, ldv);
  PPS_CHECK_LAUNCH("argsort_rows_kernel");
  return PPS_OK;
}

}  // namespace pps
