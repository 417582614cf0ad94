// Full stable argsort of every distance row: idx[q][j] = the j-th gallery
// column in (distance, index) order -- the reference's rank list
// `np.argsort(distmat, axis=1)` (reid_dataset_evaluator.py:319, :420) for
// callers that need all G columns (writing ranked lists, CMC
// single_gallery_shot), not only the top-k pps_topk gives.  np.argsort's
// default quicksort leaves ties in an unspecified order; this is the stable
// order (= kind='stable').
//
// Every entry is one unique 64-bit word (order-preserving key << 32 |
// column), so any sort of the words is the stable order.  The sort core
// (sort_core) orders n words of a known range [lo, hi] in LDS:
//  1. a coarse histogram over kNC equal slices of the range (a monotone
//     float map of word - lo) of every kSample-th word;
//  2. equalisation: coarse slice c gets 1 + cnt_c (kNF - kNC) / n of the kNF
//     fine buckets, split evenly over its own sub-range -- dense regions of
//     a row (distances pile up around the typical non-match distance) get
//     proportionally more buckets, so fine buckets hold ~n / kNF words;
//  3. fine histogram (16-bit counters, two per LDS word: n < 65536), scan,
//     scatter by per-bucket cursors;
//  4. every fine bucket sorted by one lane with a sorting network in
//     registers (<= 8 or <= 16 words), the rare larger buckets by a wave's
//     bitonic network in LDS.
// Rows up to kSortCap columns run the core once, the row held in registers
// (the next row's loads in flight under the sort; argsort_rows_kernel).
// Longer rows (argsort_rows_big_kernel) are cut into segments of at most
// kSeg words by exact word ranges (histograms of the row over the range,
// refined where a bucket is still too full), and each segment is selected
// from the row (L2-resident between passes), sorted by the core and
// written at its offset.
// Algorithmic bytes per row: G * 4 read + G * 4 written (+ G * 4 with vals).
#include "pps_internal.hpp"

namespace pps {

namespace {

typedef unsigned long long u64;

constexpr int kT = 1024;     // threads per workgroup (16 waves)
constexpr int kW = kT / 64;
#ifndef PPS_SORT_NC
#define PPS_SORT_NC 512
#endif
constexpr int kNC = PPS_SORT_NC;   // coarse slices (equalisation)
constexpr int kNF = 6144;    // fine buckets (16-bit counters, two per word)
constexpr int kNF2 = kNF / 2;
#ifndef PPS_SORT_SAMPLE
#define PPS_SORT_SAMPLE 2
#endif
constexpr int kSample = PPS_SORT_SAMPLE;   // the coarse histogram counts every kSample-th word
constexpr int kNet = 16;     // buckets up to this size: one lane's sorting network
constexpr int kLds = 160 * 1024;
constexpr int kFixed = 4 * (kNC + 1) + 4 * kNF2 + 8 * 2 * kW + 64;
constexpr int kSortU = (kLds - kFixed) / 8 / kT;   // row entries per thread
constexpr int kSortCap = kSortU * kT;              // longest row of the one-pass kernel
// long rows: segments of <= kSeg words (src + dst in LDS), grouped by
// kHalf-word histogram prefixes, at most kSegCap per row
constexpr int kSeg = 7168;
constexpr int kHalf = kSeg / 2;
constexpr int kSegCap = 256;
constexpr int kNH = 7168;    // segmentation histogram buckets (aliases src / dst)
constexpr int kBigMax = kSegCap / 2 * kHalf;       // 458,752 columns
static_assert(4 * (kNH + 1) <= kSeg * 8 && 8 * kNH <= kSeg * 8,
              "segmentation histogram must fit the segment buffers");

#ifdef PPS_SORT_PROBE
// phase cycle counts of workgroup 0 (scripts/probes/argsort_phases.py)
__device__ unsigned long long g_sort_phase[16];
#define SORT_PHASE(k)                                  \
  do {                                                 \
    if (threadIdx.x == 0 && blockIdx.x == 0) {         \
      const unsigned long long c_ = clock64();         \
      ph[k] += c_ - ph_last;                           \
      ph_last = c_;                                    \
    }                                                  \
  } while (0)
#define PROBE_ARGS , ph, ph_last
#define PROBE_PARAMS , unsigned long long (&ph)[16], unsigned long long& ph_last
#else
#define SORT_PHASE(k) do {} while (0)
#define PROBE_ARGS
#define PROBE_PARAMS
#endif

// Workgroup barrier ordering LDS only: __syncthreads()'s fences also wait
// for every outstanding global load, which stalls the sort on the next row's
// prefetch at its first barrier.
__device__ inline void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

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
__device__ inline u64 word_of(float d, int col) {
  return ((u64)sort_key(d) << 32) | (uint32_t)col;
}

// exclusive scan of a[0, n) in place; returns the total.  Ends with a
// barrier (a[] final, red[] reusable).
__device__ unsigned block_scan_excl(unsigned* a, int n, unsigned* red) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int per = (n + kT - 1) / kT;
  const int b0 = t * per;
  unsigned s = 0;
  for (int j = 0; j < per; ++j)
    if (b0 + j < n) s += a[b0 + j];
  unsigned incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) red[wave] = incl;
  lds_barrier();
  unsigned base = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kW; ++w) {
    const unsigned r = red[w];
    base += w < wave ? r : 0u;
    total += r;
  }
  unsigned run = base + incl - s;
  for (int j = 0; j < per; ++j)
    if (b0 + j < n) {
      const unsigned v = a[b0 + j];
      a[b0 + j] = run;
      run += v;
    }
  lds_barrier();
  return total;
}

// exclusive scan of the kNF 16-bit counters packed two per word (bucket f
// in word f / 2, half f % 2) in place; totals < 65536.  Ends with a barrier.
__device__ void block_scan_packed(unsigned* a, unsigned* red) {
  constexpr int per = kNF2 / kT;
  static_assert(kNF2 % kT == 0, "packed scan: whole words per thread");
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int b0 = t * per;
  unsigned w[per], s = 0;
#pragma unroll
  for (int j = 0; j < per; ++j) {
    w[j] = a[b0 + j];
    s += (w[j] & 0xffffu) + (w[j] >> 16);
  }
  unsigned incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) red[wave] = incl;
  lds_barrier();
  unsigned base = 0;
#pragma unroll
  for (int w2 = 0; w2 < kW; ++w2) base += w2 < wave ? red[w2] : 0u;
  unsigned run = base + incl - s;
#pragma unroll
  for (int j = 0; j < per; ++j) {
    const unsigned lo = run, hi = run + (w[j] & 0xffffu);
    a[b0 + j] = lo | (hi << 16);
    run = hi + (w[j] >> 16);
  }
  lds_barrier();
}
__device__ inline int packed_get(const unsigned* a, int f) {
  const unsigned w = a[f >> 1];
  return (int)((f & 1) ? w >> 16 : w & 0xffffu);
}
// cursor of bucket f: its current value, then + 1
__device__ inline int packed_take(unsigned* a, int f) {
  const unsigned old = atomicAdd(&a[f >> 1], (f & 1) ? 0x10000u : 1u);
  return (int)((f & 1) ? old >> 16 : old & 0xffffu);
}

// min / max of the threads' values over the workgroup (red: 2 * kW words)
__device__ void block_minmax(u64& mn, u64& mx, u64* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const u64 a = __shfl_xor(mn, o), b = __shfl_xor(mx, o);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  if (lane == 0) { red[wave] = mn; red[kW + wave] = mx; }
  lds_barrier();
  mn = red[0];
  mx = red[kW];
#pragma unroll
  for (int w = 1; w < kW; ++w) {
    mn = red[w] < mn ? red[w] : mn;
    mx = red[kW + w] > mx ? red[kW + w] : mx;
  }
  lds_barrier();
}

// monotone maps of words in [lo, hi] onto kNC coarse slices and each slice
// c onto its fine buckets [cb[c], cb[c + 1]): the conversion to float, the
// product and the truncation never reverse the order of two words
struct FineMap {
  u64 lo;
  float cscale;
  const unsigned* cb;
  __device__ FineMap(u64 lo_, u64 hi_, const unsigned* cb_)
      : lo(lo_), cscale((float)kNC / ((float)(hi_ - lo_) + 1.0f)), cb(cb_) {}
  __device__ int coarse(u64 v, float* frac) const {
    const float x = (float)(v - lo) * cscale;
    int c = (int)x;
    c = c < kNC - 1 ? c : kNC - 1;
    *frac = x - (float)c;
    return c;
  }
  __device__ int fine(u64 v) const {
    float fr;
    const int c = coarse(v, &fr);
    const int b = (int)cb[c], ns = (int)cb[c + 1] - b;
    int s = (int)(fr * (float)ns);
    s = s < ns - 1 ? s : ns - 1;
    return b + s;
  }
};

__device__ inline void ce(u64& a, u64& b) {
  const u64 x = a < b ? a : b, y = a < b ? b : a;
  a = x;
  b = y;
}

#define CE(i, j) ce(r[i], r[j])
__device__ inline void net8(u64 (&r)[kNet]) {
  CE(0, 2); CE(1, 3); CE(4, 6); CE(5, 7); CE(0, 4); CE(1, 5); CE(2, 6); CE(3, 7);
  CE(0, 1); CE(2, 3); CE(4, 5); CE(6, 7); CE(2, 4); CE(3, 5); CE(1, 4); CE(3, 6);
  CE(1, 2); CE(3, 4); CE(5, 6);
}

// Batcher's odd-even merge sort, 63 comparators
__device__ inline void net16(u64 (&r)[kNet]) {
  CE(0, 1); CE(2, 3); CE(0, 2); CE(1, 3); CE(1, 2); CE(4, 5); CE(6, 7); CE(4, 6);
  CE(5, 7); CE(5, 6); CE(0, 4); CE(2, 6); CE(2, 4); CE(1, 5); CE(3, 7); CE(3, 5);
  CE(1, 2); CE(3, 4); CE(5, 6); CE(8, 9); CE(10, 11); CE(8, 10); CE(9, 11); CE(9, 10);
  CE(12, 13); CE(14, 15); CE(12, 14); CE(13, 15); CE(13, 14); CE(8, 12); CE(10, 14);
  CE(10, 12); CE(9, 13); CE(11, 15); CE(11, 13); CE(9, 10); CE(11, 12); CE(13, 14);
  CE(0, 8); CE(4, 12); CE(4, 8); CE(2, 10); CE(6, 14); CE(6, 10); CE(2, 4); CE(6, 8);
  CE(10, 12); CE(1, 9); CE(5, 13); CE(5, 9); CE(3, 11); CE(7, 15); CE(7, 11); CE(3, 5);
  CE(7, 9); CE(11, 13); CE(1, 2); CE(3, 4); CE(5, 6); CE(7, 8); CE(9, 10); CE(11, 12);
  CE(13, 14);
}
#undef CE

// one wave: bitonic network in place over a[0, n) (any n; mirror step, then
// half-cleaners; partners past the end skipped)
__device__ void wave_bitonic(u64* a, int n) {
  const int lane = threadIdx.x & 63;
  int n2 = 1;
  while (n2 < n) n2 <<= 1;
  for (int size = 2; size <= n2; size <<= 1) {
    const int half = size >> 1;
    for (int x = lane; x < n2 / 2; x += 64) {
      const int bb = x / half, o = x - bb * half;
      const int i = bb * size + o, j = bb * size + size - 1 - o;
      if (j < n) {
        const u64 ai = a[i], aj = a[j];
        if (aj < ai) { a[i] = aj; a[j] = ai; }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int stride = half >> 1; stride > 0; stride >>= 1) {
      for (int x = lane; x < n2 / 2; x += 64) {
        const int bb = x / stride, o = x - bb * stride;
        const int i = 2 * bb * stride + o, j = i + stride;
        if (j < n) {
          const u64 ai = a[i], aj = a[j];
          if (aj < ai) { a[i] = aj; a[j] = ai; }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
}

// The sort core: the n words the workgroup's threads hold (each(f, k) calls
// f(word) for the calling thread's words; every k-th of them when k > 1) in
// range [lo, hi] -> dst[0, n) ascending (n < 65536).  cb: kNC + 1 words,
// off: kNF2 words, red: 2 * kW words.
template <class Each, class After>
__device__ void sort_core(Each each, int n, u64 lo, u64 hi, u64* dst, unsigned* cb,
                          unsigned* off, unsigned* red, After after_scatter PROBE_PARAMS) {
  const int t = threadIdx.x;
  for (int i = t; i <= kNC; i += kT) cb[i] = 0u;
  for (int i = t; i < kNF2; i += kT) off[i] = 0u;
  lds_barrier();
  const FineMap fm(lo, hi, cb);
  // 1) coarse histogram of a sample (every kSample-th word of a thread)
  each([&](u64 v) {
    float fr;
    atomicAdd(&cb[fm.coarse(v, &fr)], 1u);
  }, kSample);
  lds_barrier();
  SORT_PHASE(1);
  // 2) fine buckets per coarse slice in proportion to its sampled count (sum
  //    <= kNF), their bases
  {
    __shared__ unsigned s_ns;
    if (t == 0) s_ns = 0;
    lds_barrier();
    unsigned part = 0;
    for (int c = t; c < kNC; c += kT) part += cb[c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
    if ((t & 63) == 0 && part) atomicAdd(&s_ns, part);
    lds_barrier();
    const unsigned ns = s_ns > 0 ? s_ns : 1u;
    for (int c = t; c < kNC; c += kT) cb[c] = 1u + cb[c] * (unsigned)(kNF - kNC) / ns;
    lds_barrier();
  }
  block_scan_excl(cb, kNC + 1, red);
  SORT_PHASE(2);
  // 3) fine histogram, scan, scatter (bucket f's counter then ends at its end)
  each([&](u64 v) {
    const int f = fm.fine(v);
    atomicAdd(&off[f >> 1], (f & 1) ? 0x10000u : 1u);
  }, 1);
  lds_barrier();
  block_scan_packed(off, red);
  SORT_PHASE(3);
  each([&](u64 v) { dst[packed_take(off, fm.fine(v))] = v; }, 1);
  lds_barrier();
  after_scatter();   // the caller's words are in LDS now (their registers free)
  SORT_PHASE(4);
  // 4) buckets of <= kNet words, one lane each.  Buckets hold ~2.6 words on
  //    average: the 2..4-word ones take a 5-comparator network in place;
  //    the 5..kNet-word ones (~12 %) are listed per wave (in cb, free after
  //    the scatter) and sorted in batches of up to kList, one per lane -- so
  //    a wave runs the 8- / 16-input networks once per batch instead of once
  //    per 64 buckets with most lanes idle (the per-bucket branches used to
  //    diverge inside every wave).  Larger buckets (ties, words the float
  //    map cannot separate) are sorted by a wave's bitonic network.
  constexpr int kList = (kNC + 1) / kW;   // per-wave list entries (s | m << 16)
  static_assert(kList >= 32, "medium-bucket lists");
  const int lane = t & 63, wave = t >> 6;
  unsigned* wl = cb + wave * kList;
  auto sort_listed = [&](int n) {   // lanes j < n: listed bucket j
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane < n) {
      const unsigned e = wl[lane];
      const int s = (int)(e & 0xffffu), m = (int)(e >> 16);
      u64 r[kNet];
      if (m <= 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = j < m ? dst[s + j] : ~0ull;
        net8(r);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < m) dst[s + j] = r[j];
      } else {
#pragma unroll
        for (int j = 0; j < kNet; ++j) r[j] = j < m ? dst[s + j] : ~0ull;
        net16(r);
#pragma unroll
        for (int j = 0; j < kNet; ++j)
          if (j < m) dst[s + j] = r[j];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };
  int nl = 0;   // listed, not yet sorted (wave-uniform)
  for (int base = wave * 64; base < kNF; base += kT) {
    const int f = base + lane;
    const int s = f ? packed_get(off, f - 1) : 0, m = packed_get(off, f) - s;
    if (m >= 2 && m <= 4) {
      u64 r0 = dst[s], r1 = dst[s + 1], r2 = m > 2 ? dst[s + 2] : ~0ull,
          r3 = m > 3 ? dst[s + 3] : ~0ull;
      ce(r0, r1); ce(r2, r3); ce(r0, r2); ce(r1, r3); ce(r1, r2);
      dst[s] = r0;
      dst[s + 1] = r1;
      if (m > 2) dst[s + 2] = r2;
      if (m > 3) dst[s + 3] = r3;
    }
    const bool med = m > 4 && m <= kNet;
    const unsigned long long mb = __ballot(med);
    // up to 64 new entries: list them in order, sorting each full batch
    // (a batch never takes more than kList; pre < 0 once a lane is listed)
    int cnt = __popcll(mb), pre = med ? __popcll(mb & ((1ull << lane) - 1ull)) : -1;
    while (cnt) {   // wave-uniform
      if (nl == kList) {   // the batch is full: sort it first
        sort_listed(nl);
        nl = 0;
      }
      const int take = cnt < kList - nl ? cnt : kList - nl;
      if (pre >= 0 && pre < take) wl[nl + pre] = (unsigned)s | ((unsigned)m << 16);
      nl += take;
      cnt -= take;
      pre = pre >= take ? pre - take : -1;
    }
    unsigned long long big = __ballot(m > kNet);
    while (big) {
      const int j = __builtin_ctzll(big);
      big &= big - 1;
      wave_bitonic(dst + __shfl(s, j), __shfl(m, j));
    }
  }
  if (nl) sort_listed(nl);
  SORT_PHASE(5);
  lds_barrier();
  SORT_PHASE(6);
}

__global__ void __launch_bounds__(kT)
argsort_rows_kernel(const float* __restrict__ dist, int64_t Q, int G, int64_t ldd,
                    int32_t* __restrict__ idx, int64_t ldi, float* __restrict__ vals,
                    int64_t ldv) {
  __shared__ u64 pk[kSortCap];
  __shared__ unsigned cb[kNC + 1];
  __shared__ unsigned off[kNF2];
  __shared__ u64 red64[2 * kW];
  unsigned* red = reinterpret_cast<unsigned*>(red64);
  const int t = threadIdx.x;
#ifdef PPS_SORT_PROBE
  unsigned long long ph[16] = {}, ph_last = clock64();
#endif
  float cur[kSortU], nxt[kSortU];
  auto load = [&](int64_t q, float (&d)[kSortU]) {
    const float* row = dist + q * ldd;
#pragma unroll
    for (int u = 0; u < kSortU; ++u) {
      const int i = t + u * kT;
      d[u] = (q < Q && i < G) ? __builtin_nontemporal_load(row + i) : 0.f;
    }
  };
  int64_t q = blockIdx.x;
  load(q, cur);
  for (; q < Q; q += gridDim.x) {
    SORT_PHASE(0);
    // the row's word range (min / max key; columns 0 .. G - 1)
    u64 mn = ~0ull, mx = 0ull;
#pragma unroll
    for (int u = 0; u < kSortU; ++u) {
      const int i = t + u * kT;
      if (i < G) {
        const u64 k = (u64)sort_key(cur[u]);
        mn = k < mn ? k : mn;
        mx = k > mx ? k : mx;
      }
    }
    block_minmax(mn, mx, red64);
    auto each = [&](auto f, int k) {
#pragma unroll
      for (int u = 0; u < kSortU; ++u) {
        const int i = t + u * kT;
        if (i < G && u % k == 0) f(word_of(cur[u], i));
      }
    };
    // the next row's loads fly under this row's bucket sort, issued once
    // this row's values are scattered: the two never hold registers at once
    // (the kernel is at the 128-VGPR cap of 16 waves per CU)
    sort_core(each, G, mn << 32, (mx << 32) | (u64)(G - 1), pk, cb, off, red,
              [&] { load(q + gridDim.x, nxt); } PROBE_ARGS);
    // the sorted row out, coalesced
    int32_t* orow = idx + q * ldi;
    float* vrow = vals ? vals + q * ldv : nullptr;
    for (int p = t; p < G; p += kT) {
      const u64 v = pk[p];
      orow[p] = (int32_t)(uint32_t)v;
      if (vrow) vrow[p] = sort_key_float((uint32_t)(v >> 32));
    }
    lds_barrier();   // pk is rebuilt for the next row
    SORT_PHASE(7);
#pragma unroll
    for (int u = 0; u < kSortU; ++u) cur[u] = nxt[u];
  }
#ifdef PPS_SORT_PROBE
  if (t == 0 && blockIdx.x == 0) {
    ph[15] = 1;
    for (int k = 0; k < 16; ++k) g_sort_phase[k] = ph[k];
  }
#endif
}

// Rows longer than kSortCap: segments of <= kSeg words by exact word ranges,
// each selected from the row, sorted by the core and written at its offset.
__global__ void __launch_bounds__(kT)
argsort_rows_big_kernel(const float* __restrict__ dist, int64_t Q, int G, int64_t ldd,
                        int32_t* __restrict__ idx, int64_t ldi, float* __restrict__ vals,
                        int64_t ldv) {
  __shared__ u64 buf[2 * kSeg];   // src | dst; the segmentation histogram aliases it
  __shared__ unsigned cb[kNC + 1];
  __shared__ unsigned off[kNF2];
  __shared__ u64 red64[2 * kW];
  __shared__ u64 seg_lo[kSegCap], seg_hi[kSegCap];
  __shared__ int seg_n[kSegCap];
  __shared__ u64 new_lo[kSegCap];
  __shared__ int new_pre[kSegCap + 1];
  __shared__ int s_nseg, s_ref, s_nnew, s_cnt;
  unsigned* red = reinterpret_cast<unsigned*>(red64);
  u64* src = buf;
  u64* dst = buf + kSeg;
  unsigned* hcnt = reinterpret_cast<unsigned*>(buf);   // [kNH + 1]
  u64* hmin = buf + kSeg;                               // [kNH]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
#ifdef PPS_SORT_PROBE
  unsigned long long ph[16] = {}, ph_last = clock64();
#endif
  for (int64_t q = blockIdx.x; q < Q; q += gridDim.x) {
    const float* row = dist + q * ldd;
    // min / max of the row's words in [lo, hi]
    auto range_of = [&](u64 lo, u64 hi, u64& mn, u64& mx) {
      mn = ~0ull;
      mx = 0ull;
      for (int i = t; i < G; i += kT) {
        const u64 v = word_of(row[i], i);
        if (v >= lo && v <= hi) {
          mn = v < mn ? v : mn;
          mx = v > mx ? v : mx;
        }
      }
      block_minmax(mn, mx, red64);
    };
    u64 amn, amx;
    range_of(0ull, ~0ull, amn, amx);
    if (t == 0) {
      s_nseg = 1;
      seg_lo[0] = amn;
      seg_hi[0] = amx;
      seg_n[0] = G;
    }
    lds_barrier();
    // refine every segment of more than kSeg words: a histogram of its words
    // over their exact range, cut at kHalf-word prefix boundaries
    for (int iter = 0;; ++iter) {
      if (t == 0) {
        s_ref = -1;
        for (int j = 0; j < s_nseg; ++j)
          if (seg_n[j] > kSeg) { s_ref = j; break; }
        if (s_ref >= 0 && iter >= 4 * kSegCap) {   // no progress: give up on the row
          s_ref = -1;
          s_nseg = -1;
        }
      }
      lds_barrier();
      const int r = s_ref;
      if (r < 0) break;
      u64 lo, hi;
      range_of(seg_lo[r], seg_hi[r], lo, hi);
      for (int i = t; i <= kNH; i += kT) hcnt[i] = 0u;
      for (int i = t; i < kNH; i += kT) hmin[i] = ~0ull;
      lds_barrier();
      const float hs = (float)kNH / ((float)(hi - lo) + 1.0f);
      for (int i = t; i < G; i += kT) {
        const u64 v = word_of(row[i], i);
        if (v >= lo && v <= hi) {
          int b = (int)((float)(v - lo) * hs);
          b = b < kNH - 1 ? b : kNH - 1;
          atomicAdd(&hcnt[b], 1u);
          atomicMin(&hmin[b], v);
        }
      }
      lds_barrier();
      block_scan_excl(hcnt, kNH + 1, red);   // hcnt[b] = words before bucket b
      // new segments: the first non-empty bucket of each kHalf-prefix group;
      // a bucket of more than kHalf words is a segment of its own (refined
      // over its own, narrower range next).  One wave walks the buckets 64 at
      // a time, carrying the last non-empty bucket's group and size.
      if (wave == 0) {
        int carry = -1, nn = 0;
        bool carry_big = false;
        for (int b0 = 0; b0 < kNH; b0 += 64) {
          const int b = b0 + lane;
          const int pre = (int)hcnt[b], cnt = (int)hcnt[b + 1] - pre;
          const int g = pre / kHalf;
          const bool big = cnt > kHalf;
          const unsigned long long ne = __ballot(cnt > 0);
          const unsigned long long below = ne & ((1ull << lane) - 1ull);
          const int pl = below ? 63 - __builtin_clzll(below) : -1;
          const int gp = __shfl(g, pl < 0 ? 0 : pl);
          const bool bigp = __shfl((int)big, pl < 0 ? 0 : pl) != 0;
          const bool first = cnt > 0 && (big || (pl < 0 ? (g != carry || carry_big)
                                                          : (g != gp || bigp)));
          const unsigned long long fm = __ballot(first);
          if (first) {
            const int k = nn + __popcll(fm & ((1ull << lane) - 1ull));
            if (k < kSegCap) {
              new_lo[k] = hmin[b];
              new_pre[k] = pre;
            }
          }
          nn += __popcll(fm);
          if (ne) {
            const int hl = 63 - __builtin_clzll(ne);
            carry = __shfl(g, hl);
            carry_big = __shfl((int)big, hl) != 0;
          }
        }
        if (lane == 0) {
          s_nnew = nn;
          if (nn <= kSegCap) new_pre[nn] = (int)hcnt[kNH];
        }
      }
      lds_barrier();
      if (t == 0) {
        const int nn = s_nnew, tail = s_nseg - r - 1;
        if (nn < 1 || s_nseg - 1 + nn > kSegCap) {
          s_nseg = -1;   // over capacity (the host bounds G so that it is not)
        } else {
          for (int j = tail - 1; j >= 0; --j) {   // the tail moves by nn - 1
            seg_lo[r + nn + j] = seg_lo[r + 1 + j];
            seg_hi[r + nn + j] = seg_hi[r + 1 + j];
            seg_n[r + nn + j] = seg_n[r + 1 + j];
          }
          const u64 rhi = seg_hi[r];
          for (int k = 0; k < nn; ++k) {
            seg_lo[r + k] = new_lo[k];
            seg_hi[r + k] = k + 1 < nn ? new_lo[k + 1] - 1 : rhi;
            seg_n[r + k] = new_pre[k + 1] - new_pre[k];
          }
          s_nseg += nn - 1;
        }
      }
      lds_barrier();
      if (s_nseg < 0) break;
    }
    const int nseg = s_nseg;   // < 0: the row is left unwritten (unreachable by the bounds)
    lds_barrier();
    // each segment: select its words from the row, sort, write at its offset
    int out0 = 0;
    for (int k = 0; k < nseg; ++k) {
      const u64 lo = seg_lo[k], hi = seg_hi[k];
      const int n = seg_n[k];
      if (t == 0) s_cnt = 0;
      lds_barrier();
      u64 mn = ~0ull, mx = 0ull;
      for (int i = t; i < G; i += kT) {
        const u64 v = word_of(row[i], i);
        if (v >= lo && v <= hi) {
          src[atomicAdd(&s_cnt, 1)] = v;
          mn = v < mn ? v : mn;
          mx = v > mx ? v : mx;
        }
      }
      block_minmax(mn, mx, red64);
      auto each = [&](auto f, int k) {
        for (int i = t; i < n; i += kT * k) f(src[i]);
      };
      sort_core(each, n, mn, mx, dst, cb, off, red, [] {} PROBE_ARGS);
      int32_t* orow = idx + q * ldi + out0;
      float* vrow = vals ? vals + q * ldv + out0 : nullptr;
      for (int p = t; p < n; p += kT) {
        const u64 v = dst[p];
        orow[p] = (int32_t)(uint32_t)v;
        if (vrow) vrow[p] = sort_key_float((uint32_t)(v >> 32));
      }
      out0 += n;
      lds_barrier();
    }
  }
}

int cus_of_device() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return cus;
}

}  // namespace

int argsort_rows_cap() { return kBigMax; }

#ifdef PPS_SORT_PROBE
extern "C" int pps_sort_probe_read(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sort_phase), sizeof(g_sort_phase)) == hipSuccess
             ? 0 : -1;
}
#endif

int argsort_rows(const float* dist, int64_t Q, int64_t G, int64_t ldd, int32_t* idx,
                 int64_t ldi, float* vals, int64_t ldv, hipStream_t st) {
  if (Q <= 0 || G <= 0) return PPS_OK;
  if (G > kBigMax) {
    set_error("argsort_rows: rows of " + std::to_string(G) + " entries exceed " +
              std::to_string(kBigMax) + " (use pps_topk for the first k)");
    return PPS_ERR_CAPACITY;
  }
  const int64_t cus = cus_of_device();
  const int64_t grid = Q < cus ? Q : cus;   // one resident workgroup per CU (LDS)
  if (G <= kSortCap) {
    hipLaunchKernelGGL(argsort_rows_kernel, dim3((unsigned)grid), dim3(kT), 0, st, dist, Q,
                       (int)G, ldd, idx, ldi, vals, ldv);
    PPS_CHECK_LAUNCH("argsort_rows_kernel");
  } else {
    hipLaunchKernelGGL(argsort_rows_big_kernel, dim3((unsigned)grid), dim3(kT), 0, st, dist, Q,
                       (int)G, ldd, idx, ldi, vals, ldv);
    PPS_CHECK_LAUNCH("argsort_rows_big_kernel");
  }
  return PPS_OK;
}

}  // namespace pps
