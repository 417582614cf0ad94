// Memory-bound feature-extractor kernels (HBM / L2 bound, no MFMA):
//   max pooling (stem pool1), part-power-set strip pooling + subset combine,
//   row L2 normalisation, image preprocessing (mean-subtract + bicubic).
// All NHWC float32, 16-B vectorised along channels where the layout allows.
#include <algorithm>

#include "pps_internal.hpp"
#include "gemm_x3_common.hpp"

namespace pps {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---- MaxPool k x k / s, pad p (ResNet.py:255) --------------------------------
// One thread per (n, oh, ow, 4 channels).  Padding never wins (Caffe2 / cuDNN
// max pooling ignores padded taps).  Index type IDX: 32-bit unsigned when the
// element count allows it (the stem's 3.1M threads), so the index split is not
// three 64-bit divisions per thread.
template <typename IDX>
__global__ void maxpool_nhwc_kernel(const float* __restrict__ x, int N, int H, int W,
                                    int C, int k, int s, int pad,
                                    float* __restrict__ y, int Ho, int Wo,
                                    float* __restrict__ amax) {
  float amx = 0.f;
  const IDX C4 = (IDX)(C >> 2);
  const IDX total = (IDX)N * (IDX)Ho * (IDX)Wo * C4;
  for (IDX t = (IDX)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (IDX)gridDim.x * blockDim.x) {
    const int c4 = (int)(t % C4);
    IDX r = t / C4;
    const int ow = (int)(r % (IDX)Wo);
    r /= (IDX)Wo;
    const int oh = (int)(r % (IDX)Ho);
    const int n = (int)(r / (IDX)Ho);
    f32x4 m = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    const int h0 = oh * s - pad, w0 = ow * s - pad;
    for (int kh = 0; kh < k; ++kh) {
      const int ih = h0 + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int iw = w0 + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        const f32x4 v = *reinterpret_cast<const f32x4*>(
            x + (((int64_t)n * H + ih) * W + iw) * C + c4 * 4);
        m.x = fmaxf(m.x, v.x);
        m.y = fmaxf(m.y, v.y);
        m.z = fmaxf(m.z, v.z);
        m.w = fmaxf(m.w, v.w);
      }
    }
    *reinterpret_cast<f32x4*>(y + (((int64_t)n * Ho + oh) * Wo + ow) * C + c4 * 4) = m;
    amx = fmaxf(amx, fmaxf(fmaxf(fabsf(m.x), fabsf(m.y)), fmaxf(fabsf(m.z), fabsf(m.w))));
  }
  if (amax) amax_commit(amax, amx);
}

int maxpool2d(const float* x, int N, int H, int W, int C, int k, int stride, int pad,
              float* y, int Ho, int Wo, hipStream_t st, float* amax) {
  const int64_t total = (int64_t)N * Ho * Wo * (C / 4);
  const int block = 256;
  const int64_t want = (total + block - 1) / block;
  if (want == 0) return PPS_OK;
  if (total < (int64_t)1 << 31) {
    // one thread per output vector (no grid-stride loop)
    hipLaunchKernelGGL(maxpool_nhwc_kernel<uint32_t>, dim3((unsigned)want), dim3(block), 0, st,
                       x, N, H, W, C, k, stride, pad, y, Ho, Wo, amax);
  } else {
    const int grid = (int)(want < 8192 ? want : 8192);
    hipLaunchKernelGGL(maxpool_nhwc_kernel<int64_t>, dim3(grid), dim3(block), 0, st, x, N, H,
                       W, C, k, stride, pad, y, Ho, Wo, amax);
  }
  PPS_CHECK_LAUNCH("maxpool_nhwc_kernel");
  return PPS_OK;
}

// ---- Part power set (bpm_heads.py:18-55, pps_heads.py:38-80) ---------------
// Per (n, c): strip-wise global average and max over the strip's rows x W,
// then every non-empty subset i (bit j <=> strip j):
//   max_ave: out = Mean(ave_j, j in i) + Max(max_j, j in i)
//   else   : out = Max(ave_j, j in i)
// Mean follows Caffe2's Mean op: sum in input order, then * (1/n).
constexpr int kMaxStrips = 10;
struct Splits {
  int h[kMaxStrips];
};

constexpr int kPpsC_fwd = 64;
__global__ void part_power_set_v2_kernel(const float* __restrict__ x, int N, int H, int W,
                                         int C, Splits sp, int S, int max_ave,
                                         float* __restrict__ out);

constexpr int kPpsC4 = 256;  // channels per block of the vectorized variant
__global__ void part_power_set_v3_kernel(const float* __restrict__ x, int N, int H, int W,
                                         int C, Splits sp, int S, int max_ave,
                                         float* __restrict__ out);

int part_power_set(const float* x, int N, int H, int W, int C, const int32_t* splits,
                   int S, int max_ave, float* out, hipStream_t st) {
  Splits sp;
  for (int j = 0; j < kMaxStrips; ++j) sp.h[j] = j < S ? splits[j] : 0;
  if (C % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    hipLaunchKernelGGL(part_power_set_v3_kernel, dim3((C + kPpsC4 - 1) / kPpsC4, N),
                       dim3(kPpsC4 / 4 * S), 0, st, x, N, H, W, C, sp, S, max_ave, out);
    PPS_CHECK_LAUNCH("part_power_set_v3_kernel");
    return PPS_OK;
  }
  dim3 block(kPpsC_fwd * S), grid((C + kPpsC_fwd - 1) / kPpsC_fwd, N);
  hipLaunchKernelGGL(part_power_set_v2_kernel, grid, block, 0, st, x, N, H, W, C, sp, S,
                     max_ave, out);
  PPS_CHECK_LAUNCH("part_power_set_v2_kernel");
  return PPS_OK;
}

// ---- split-K conv epilogue ---------------------------------------------------
// y = relu?(sum_s part[s] * scale + shift [+ residual]) over the S partial
// slices in fixed order (deterministic), written as f32 or as bf16x3 planes
// (y3 + k * plane: the exact split of the pipelined GEMM's EPI_F_PLANES).
__global__ void splitk_conv_epilogue_kernel(const float* __restrict__ part, int S,
                                            int64_t sstride, int64_t total4, int N4,
                                            const float* __restrict__ scale,
                                            const float* __restrict__ shift,
                                            const float* __restrict__ res, int relu,
                                            float* __restrict__ y, uint16_t* __restrict__ y3,
                                            int64_t plane, float* __restrict__ amax) {
  float amx = 0.f;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total4;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int c4 = (int)(t % N4);
    f32x4 v = reinterpret_cast<const f32x4*>(part)[t];
    for (int s = 1; s < S; ++s) {
      const f32x4 w = reinterpret_cast<const f32x4*>(part + s * sstride)[t];
      v += w;
    }
    const f32x4 sc = reinterpret_cast<const f32x4*>(scale)[c4];
    const f32x4 sh = reinterpret_cast<const f32x4*>(shift)[c4];
    const f32x4 rv = res ? reinterpret_cast<const f32x4*>(res)[t] : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = __builtin_fmaf(v[e], sc[e], sh[e]);
      if (res) v[e] += rv[e];
      if (relu) v[e] = fmaxf(v[e], 0.f);
      amx = fmaxf(amx, fabsf(v[e]));
    }
    if (y3) {
      unsigned h0, m0, l0, h1, m1, l1;
      split2(v[0], v[1], h0, m0, l0);
      split2(v[2], v[3], h1, m1, l1);
      typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
      reinterpret_cast<u32x2_t*>(y3)[t] = (u32x2_t){h0, h1};
      reinterpret_cast<u32x2_t*>(y3 + plane)[t] = (u32x2_t){m0, m1};
      reinterpret_cast<u32x2_t*>(y3 + 2 * plane)[t] = (u32x2_t){l0, l1};
    } else {
      reinterpret_cast<f32x4*>(y)[t] = v;
    }
  }
  if (amax) amax_commit(amax, amx);
}

int splitk_conv_epilogue(const float* part, int S, int64_t M, int N, const float* scale,
                         const float* shift, const float* res, int relu, float* y,
                         uint16_t* y3, int64_t plane, hipStream_t st, float* amax) {
  const int64_t total4 = M * N / 4;
  if (total4 == 0) return PPS_OK;
  const int64_t want = (total4 + 255) / 256;
  hipLaunchKernelGGL(splitk_conv_epilogue_kernel, dim3((unsigned)(want < 16384 ? want : 16384)),
                     dim3(256), 0, st, part, S, M * N, total4, N / 4, scale, shift, res, relu,
                     y, y3, plane, amax);
  PPS_CHECK_LAUNCH("splitk_conv_epilogue_kernel");
  return PPS_OK;
}

// ---- Normalize (triplet_loss.py:17-19 -> Caffe2 Normalize) -------------------
__global__ void l2_normalize_kernel(const float* __restrict__ x, int D,
                                    float* __restrict__ y) {
  const int64_t row = blockIdx.x;
  const float* xr = x + row * D;
  float s = 0.f;
  for (int i = threadIdx.x; i < D; i += blockDim.x) s += xr[i] * xr[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  __shared__ float red[16];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = threadIdx.x < (blockDim.x >> 6) ? red[threadIdx.x] : 0.f;
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if (threadIdx.x == 0) red[0] = t;
  }
  __syncthreads();
  const float inv = 1.f / fmaxf(sqrtf(red[0]), 1e-12f);
  float* yr = y + row * D;
  for (int i = threadIdx.x; i < D; i += blockDim.x) yr[i] = xr[i] * inv;
}

int l2_normalize(const float* x, int64_t N, int D, float* y, hipStream_t st) {
  if (N <= 0) return PPS_OK;
  hipLaunchKernelGGL(l2_normalize_kernel, dim3((unsigned)N), dim3(256), 0, st, x, D, y);
  PPS_CHECK_LAUNCH("l2_normalize_kernel");
  return PPS_OK;
}

// ---- split-K reduce + BN + ReLU + Normalize (reid_heads.py:42-127) ---------
// One block per feature row: y[m][j] = relu(sum_s part[s][m][j] * scale[j] +
// shift[j]) over the S partial GEMM slices in fixed order (deterministic),
// then optionally y[m] /= max(||y[m]||, 1e-12) (Caffe2 Normalize axis 1).
__global__ void splitk_bn_act_normalize_kernel(const float* __restrict__ part, int S,
                                               int64_t sstride, int N,
                                               const float* __restrict__ scale,
                                               const float* __restrict__ shift, int relu,
                                               int normalize, float* __restrict__ y) {
  const int64_t m = blockIdx.x;
  float* yr = y + m * N;
  float ss = 0.f;
  for (int j = threadIdx.x; j < N; j += blockDim.x) {
    float v = part[m * N + j];
    for (int s = 1; s < S; ++s) v += part[s * sstride + m * N + j];
    v = __builtin_fmaf(v, scale[j], shift[j]);
    if (relu) v = fmaxf(v, 0.f);
    yr[j] = v;
    ss += v * v;
  }
  if (!normalize) return;
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  __shared__ float red[16];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x < 64) {
    float t = threadIdx.x < (blockDim.x >> 6) ? red[threadIdx.x] : 0.f;
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
    if (threadIdx.x == 0) red[0] = t;
  }
  __syncthreads();
  const float inv = 1.f / fmaxf(sqrtf(red[0]), 1e-12f);
  for (int j = threadIdx.x; j < N; j += blockDim.x) yr[j] *= inv;
}

// Vectorised single-pass form for N % 4 == 0, N <= 4096: one float4 column
// group per thread, kept in registers between the norm and the scaling.
// SC > 0: the slice count as a constant, so all SC partial loads are issued
// before the first add (a runtime-count loop waits for each load in turn).
template <int SC>
__global__ void __launch_bounds__(1024)
splitk_bn_act_normalize_v4_kernel(const float* __restrict__ part, int S, int64_t sstride,
                                  int N, const float* __restrict__ scale,
                                  const float* __restrict__ shift, int relu, int normalize,
                                  float* __restrict__ y) {
  const int64_t m = blockIdx.x;
  const int j = threadIdx.x * 4;
  const bool on = j < N;
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (on) {
    if constexpr (SC > 0) {
      f32x4 ps[SC];
#pragma unroll
      for (int s = 0; s < SC; ++s)
        ps[s] = __builtin_nontemporal_load(
            reinterpret_cast<const f32x4*>(part + s * sstride + m * N + j));
      v = ps[0];
#pragma unroll
      for (int s = 1; s < SC; ++s) v += ps[s];
    } else {
      v = *reinterpret_cast<const f32x4*>(part + m * N + j);
      for (int s = 1; s < S; ++s)
        v += *reinterpret_cast<const f32x4*>(part + s * sstride + m * N + j);
    }
    const f32x4 sc = *reinterpret_cast<const f32x4*>(scale + j);
    const f32x4 sh = *reinterpret_cast<const f32x4*>(shift + j);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = __builtin_fmaf(v[e], sc[e], sh[e]);
      v[e] = relu ? fmaxf(t, 0.f) : t;
    }
  }
  float inv = 1.f;
  if (normalize) {
    float ss = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    __shared__ float red[16];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    if (threadIdx.x < 64) {
      float t = threadIdx.x < (blockDim.x >> 6) ? red[threadIdx.x] : 0.f;
      for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
      if (threadIdx.x == 0) red[0] = t;
    }
    __syncthreads();
    inv = 1.f / fmaxf(sqrtf(red[0]), 1e-12f);
  }
  if (on) *reinterpret_cast<f32x4*>(y + m * N + j) = v * inv;
}

int splitk_bn_act_normalize(const float* part, int S, int64_t sstride, int M, int N,
                            const float* scale, const float* shift, int relu, int normalize,
                            float* y, hipStream_t st) {
  if (M <= 0) return PPS_OK;
  if (N % 4 == 0 && N <= 4096 && ((reinterpret_cast<uintptr_t>(part) |
                                   reinterpret_cast<uintptr_t>(y) |
                                   reinterpret_cast<uintptr_t>(scale) |
                                   reinterpret_cast<uintptr_t>(shift)) & 15) == 0) {
    const int threads = ((N / 4 + 63) / 64) * 64;
    if (S == 8)
      hipLaunchKernelGGL(splitk_bn_act_normalize_v4_kernel<8>, dim3(M), dim3(threads), 0, st,
                         part, S, sstride, N, scale, shift, relu, normalize, y);
    else
      hipLaunchKernelGGL(splitk_bn_act_normalize_v4_kernel<0>, dim3(M), dim3(threads), 0, st,
                         part, S, sstride, N, scale, shift, relu, normalize, y);
    PPS_CHECK_LAUNCH("splitk_bn_act_normalize_v4_kernel");
    return PPS_OK;
  }
  hipLaunchKernelGGL(splitk_bn_act_normalize_kernel, dim3(M), dim3(256), 0, st, part, S,
                     sstride, N, scale, shift, relu, normalize, y);
  PPS_CHECK_LAUNCH("splitk_bn_act_normalize_kernel");
  return PPS_OK;
}

// ---- part power set, strip-parallel variant ----------------------------------
// Block = (image n, 64 channels); thread (strip j, channel c) reduces its
// strip (rows x W values) -> LDS; then all threads emit the 2^S-1 subsets.
constexpr int kPpsC = 64;
__global__ void part_power_set_v2_kernel(const float* __restrict__ x, int N, int H, int W,
                                         int C, Splits sp, int S, int max_ave,
                                         float* __restrict__ out) {
  __shared__ float s_ave[kMaxStrips][kPpsC];
  __shared__ float s_max[kMaxStrips][kPpsC];
  const int n = blockIdx.y;
  const int c0 = blockIdx.x * kPpsC;
  const int cl = threadIdx.x % kPpsC;
  const int j = threadIdx.x / kPpsC;
  const int c = c0 + cl;
  if (j < S && c < C) {
    int r0 = 0;
    for (int t = 0; t < j; ++t) r0 += sp.h[t];
    const float* base = x + (((int64_t)n * H + r0) * W) * C + c;
    float sum = 0.f, m = -INFINITY;
    const int cnt = sp.h[j] * W;
    for (int e = 0; e < cnt; ++e) {  // rows of the strip, row-major: (hh, ww)
      const float v = base[(int64_t)e * C];
      sum += v;
      m = fmaxf(m, v);
    }
    s_ave[j][cl] = sum / (float)cnt;
    s_max[j][cl] = m;
  }
  __syncthreads();
  const int nsub = (1 << S) - 1;
  for (int o = threadIdx.x; o < nsub * kPpsC; o += blockDim.x) {
    const int i = o / kPpsC + 1, cc = o % kPpsC;
    if (c0 + cc >= C) continue;
    float v;
    if (max_ave) {
      float s = 0.f, m = -INFINITY;
      int k = 0;
      bool first = true;
      for (int t = 0; t < S; ++t)
        if (i & (1 << t)) {
          s = first ? s_ave[t][cc] : s + s_ave[t][cc];
          first = false;
          m = fmaxf(m, s_max[t][cc]);
          ++k;
        }
      v = s * (1.f / (float)k) + m;
    } else {
      float m = -INFINITY;
      for (int t = 0; t < S; ++t)
        if (i & (1 << t)) m = fmaxf(m, s_ave[t][cc]);
      v = m;
    }
    out[((int64_t)(i - 1) * N + n) * C + c0 + cc] = v;
  }
}

// Vectorized variant (C % 4 == 0): thread (strip j, 4 channels) reduces its
// strip with 16-byte loads, 8 independent loads in flight; per channel the
// summation order is v2's (rows of the strip in row-major order), so the
// results are bit-identical.  Block = (image n, 256 channels).
__global__ void __launch_bounds__(kPpsC4 / 4 * kMaxStrips)
part_power_set_v3_kernel(const float* __restrict__ x, int N, int H, int W, int C, Splits sp,
                         int S, int max_ave, float* __restrict__ out) {
  __shared__ float s_ave[kMaxStrips][kPpsC4];
  __shared__ float s_max[kMaxStrips][kPpsC4];
  const int n = blockIdx.y;
  const int c0 = blockIdx.x * kPpsC4;
  const int q = threadIdx.x % (kPpsC4 / 4);
  const int j = threadIdx.x / (kPpsC4 / 4);
  const int c = c0 + 4 * q;
  if (j < S && c < C) {
    int r0 = 0;
    for (int t = 0; t < j; ++t) r0 += sp.h[t];
    const f32x4* base = reinterpret_cast<const f32x4*>(x + (((int64_t)n * H + r0) * W) * C + c);
    const int64_t st4 = C / 4;
    f32x4 sum = {0.f, 0.f, 0.f, 0.f};
    f32x4 m = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    const int cnt = sp.h[j] * W;
    int e = 0;
    for (; e + 8 <= cnt; e += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = base[(int64_t)(e + u) * st4];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          sum[k] += v[u][k];
          m[k] = fmaxf(m[k], v[u][k]);
        }
      }
    }
    for (; e < cnt; ++e) {
      const f32x4 v = base[(int64_t)e * st4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        sum[k] += v[k];
        m[k] = fmaxf(m[k], v[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      s_ave[j][4 * q + k] = sum[k] / (float)cnt;
      s_max[j][4 * q + k] = m[k];
    }
  }
  __syncthreads();
  const int nsub = (1 << S) - 1;
  for (int o = threadIdx.x; o < nsub * kPpsC4; o += blockDim.x) {
    const int i = o / kPpsC4 + 1, cc = o % kPpsC4;
    if (c0 + cc >= C) continue;
    float v;
    if (max_ave) {
      float s = 0.f, mx = -INFINITY;
      int k = 0;
      bool first = true;
      for (int t = 0; t < S; ++t)
        if (i & (1 << t)) {
          s = first ? s_ave[t][cc] : s + s_ave[t][cc];
          first = false;
          mx = fmaxf(mx, s_max[t][cc]);
          ++k;
        }
      v = s * (1.f / (float)k) + mx;
    } else {
      float mx = -INFINITY;
      for (int t = 0; t < S; ++t)
        if (i & (1 << t)) mx = fmaxf(mx, s_ave[t][cc]);
      v = mx;
    }
    out[((int64_t)(i - 1) * N + n) * C + c0 + cc] = v;
  }
}

// ---- multi-query pooling (reid_dataset_evaluator.py:132-143) ------------------
// out[g] = mean of rows members[offsets[g] .. offsets[g+1]) of x, summed in
// member order then divided by the count (np.mean over axis 0, float32).
__global__ void group_mean_kernel(const float* __restrict__ x, int D,
                                  const int32_t* __restrict__ offsets,
                                  const int32_t* __restrict__ members,
                                  float* __restrict__ out) {
  const int g = blockIdx.x;
  const int a = offsets[g], b = offsets[g + 1];
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = x[(int64_t)members[a] * D + d];
    for (int m = a + 1; m < b; ++m) s += x[(int64_t)members[m] * D + d];
    out[(int64_t)g * D + d] = s / (float)(b - a);
  }
}

int group_mean(const float* x, int D, const int32_t* offsets, const int32_t* members,
               int ngroups, float* out, hipStream_t st) {
  if (ngroups <= 0) return PPS_OK;
  hipLaunchKernelGGL(group_mean_kernel, dim3(ngroups), dim3(256), 0, st, x, D, offsets,
                     members, out);
  PPS_CHECK_LAUNCH("group_mean_kernel");
  return PPS_OK;
}

// ---- Preprocess (utils/blob.py:97-117) ---------------------------------------
// u8 BGR HWC -> float, minus PIXEL_MEANS, bicubic resize (cv2.INTER_CUBIC:
// a = -0.75, src = (dst + 0.5) * scale - 0.5, replicate border) -> NHWC4.
__device__ inline void cubic_coeffs(float x, float w[4]) {
  const float A = -0.75f;
  w[0] = ((A * (x + 1.f) - 5.f * A) * (x + 1.f) + 8.f * A) * (x + 1.f) - 4.f * A;
  w[1] = ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f;
  w[2] = ((A + 2.f) * (1.f - x) - (A + 3.f)) * (1.f - x) * (1.f - x) + 1.f;
  w[3] = 1.f - w[0] - w[1] - w[2];
}

struct Means {
  float m[3];
};

// One thread per output pixel.  Images are either a dense [N][Hi][Wi][3]
// batch (offsets == nullptr) or a ragged blob described per image by a byte
// offset and its own height / width (device arrays), as decoded JPEGs of a
// dataset with mixed sizes (DukeMTMC-reID) arrive.
__global__ void __launch_bounds__(128)
preprocess_bgr_kernel(const uint8_t* __restrict__ blob, int N, int Hi0, int Wi0,
                      const int64_t* __restrict__ offsets, const int32_t* __restrict__ heights,
                      const int32_t* __restrict__ widths, Means mean, int Ho, int Wo,
                      float* __restrict__ y) {
  // block = (output row n*Ho + oy, 128 output columns): no 64-bit index math
  const int row = blockIdx.x;
  const int ox = blockIdx.y * blockDim.x + threadIdx.x;
  const int n = row / Ho;
  const int oy = row - n * Ho;
  int Hi = Hi0, Wi = Wi0;
  const uint8_t* img;
  if (offsets) {
    Hi = heights[n];
    Wi = widths[n];
    img = blob + offsets[n];
  } else {
    img = blob + (int64_t)n * Hi * Wi * 3;
  }
  // source coordinate in double, then float (cv::resize computes its tap
  // tables the same way: fy = (float)((dy + 0.5) * scale - 0.5))
  const float fy = (float)((oy + 0.5) * ((double)Hi / (double)Ho) - 0.5);
  const int y0 = (int)floorf(fy);
  int yy[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) yy[j] = min(max(y0 - 1 + j, 0), Hi - 1);
  const int rb = Wi * 3;
  if (ox >= Wo) return;
  const float fx = (float)((ox + 0.5) * ((double)Wi / (double)Wo) - 0.5);
  const int x0 = (int)floorf(fx);
  float wx[4], wy[4];
  cubic_coeffs(fx - x0, wx);
  cubic_coeffs(fy - y0, wy);
  int xo[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) xo[i] = min(max(x0 - 1 + i, 0), Wi - 1) * 3;
  float acc[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint8_t* rowp = img + (int64_t)yy[j] * rb;
    float rowv[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint8_t* px = rowp + xo[i];
#pragma unroll
      for (int c = 0; c < 3; ++c) rowv[c] += wx[i] * ((float)px[c] - mean.m[c]);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) acc[c] += wy[j] * rowv[c];
  }
  *reinterpret_cast<f32x4*>(y + ((int64_t)row * Wo + ox) * 4) = f32x4{acc[0], acc[1], acc[2], 0.f};
}

// Separable variant: block = (image n, band of kPrepRows output rows).  Pass
// 1 filters the band's source rows horizontally into LDS (each source row
// once, not once per output row that uses it), pass 2 filters vertically --
// the same sums in the same order as the direct kernel above (row sums over
// i, then acc over j).  A band whose source rows exceed the LDS cap (strong
// downscaling) is computed directly.
constexpr int kPrepRows = 16;
__global__ void __launch_bounds__(256)
preprocess_sep_kernel(const uint8_t* __restrict__ blob, int N, int Hi0, int Wi0,
                      const int64_t* __restrict__ offsets, const int32_t* __restrict__ heights,
                      const int32_t* __restrict__ widths, Means mean, int Ho, int Wo, int kcap,
                      float* __restrict__ y, float* __restrict__ amax) {
  extern __shared__ float hrow[];  // [kcap][Wo][3]
  float amx = 0.f;  // max |y| of this thread's outputs (amax: the f16x2 stem's input scale)
  const int nb = (Ho + kPrepRows - 1) / kPrepRows;
  const int n = blockIdx.x / nb;
  const int oy0 = (blockIdx.x - n * nb) * kPrepRows;
  const int oy1 = min(Ho, oy0 + kPrepRows);
  int Hi = Hi0, Wi = Wi0;
  const uint8_t* img;
  if (offsets) {
    Hi = heights[n];
    Wi = widths[n];
    img = blob + offsets[n];
  } else {
    img = blob + (int64_t)n * Hi * Wi * 3;
  }
  const double sy = (double)Hi / (double)Ho, sx = (double)Wi / (double)Wo;
  const int rb = Wi * 3;
  auto src_y0 = [&](int oy) { return (int)floorf((float)((oy + 0.5) * sy - 0.5)); };
  const int ys = min(max(src_y0(oy0) - 1, 0), Hi - 1);
  const int ye = min(max(src_y0(oy1 - 1) + 2, 0), Hi - 1);
  const int nr = ye - ys + 1;
  const int nout = (oy1 - oy0) * Wo;
  if (nr > kcap) {  // direct
    for (int t = threadIdx.x; t < nout; t += blockDim.x) {
      const int oy = oy0 + t / Wo, ox = t - (t / Wo) * Wo;
      const float fy = (float)((oy + 0.5) * sy - 0.5);
      const float fx = (float)((ox + 0.5) * sx - 0.5);
      const int y0 = (int)floorf(fy), x0 = (int)floorf(fx);
      float wx[4], wy[4];
      cubic_coeffs(fx - x0, wx);
      cubic_coeffs(fy - y0, wy);
      float acc[3] = {0.f, 0.f, 0.f};
      for (int j = 0; j < 4; ++j) {
        const uint8_t* rowp = img + (int64_t)min(max(y0 - 1 + j, 0), Hi - 1) * rb;
        float rowv[3] = {0.f, 0.f, 0.f};
        for (int i = 0; i < 4; ++i) {
          const uint8_t* px = rowp + min(max(x0 - 1 + i, 0), Wi - 1) * 3;
          for (int c = 0; c < 3; ++c) rowv[c] += wx[i] * ((float)px[c] - mean.m[c]);
        }
        for (int c = 0; c < 3; ++c) acc[c] += wy[j] * rowv[c];
      }
      *reinterpret_cast<f32x4*>(y + (((int64_t)n * Ho + oy) * Wo + ox) * 4) =
          f32x4{acc[0], acc[1], acc[2], 0.f};
      amx = fmaxf(amx, fmaxf(fabsf(acc[0]), fmaxf(fabsf(acc[1]), fabsf(acc[2]))));
    }
    if (amax) amax_commit(amax, amx);
    return;
  }
  // pass 1: horizontal filter of source rows ys..ye
  for (int t = threadIdx.x; t < nr * Wo; t += blockDim.x) {
    const int r = t / Wo, ox = t - r * Wo;
    const float fx = (float)((ox + 0.5) * sx - 0.5);
    const int x0 = (int)floorf(fx);
    float wx[4];
    cubic_coeffs(fx - x0, wx);
    const uint8_t* rowp = img + (int64_t)(ys + r) * rb;
    float rowv[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint8_t* px = rowp + min(max(x0 - 1 + i, 0), Wi - 1) * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) rowv[c] += wx[i] * ((float)px[c] - mean.m[c]);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) hrow[t * 3 + c] = rowv[c];
  }
  __syncthreads();
  // pass 2: vertical filter
  for (int t = threadIdx.x; t < nout; t += blockDim.x) {
    const int oyl = t / Wo, ox = t - oyl * Wo;
    const int oy = oy0 + oyl;
    const float fy = (float)((oy + 0.5) * sy - 0.5);
    const int y0 = (int)floorf(fy);
    float wy[4];
    cubic_coeffs(fy - y0, wy);
    float acc[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = min(max(y0 - 1 + j, 0), Hi - 1) - ys;
      const float* h = hrow + (r * Wo + ox) * 3;
#pragma unroll
      for (int c = 0; c < 3; ++c) acc[c] += wy[j] * h[c];
    }
    *reinterpret_cast<f32x4*>(y + (((int64_t)n * Ho + oy) * Wo + ox) * 4) =
        f32x4{acc[0], acc[1], acc[2], 0.f};
    amx = fmaxf(amx, fmaxf(fabsf(acc[0]), fmaxf(fabsf(acc[1]), fabsf(acc[2]))));
  }
  if (amax) amax_commit(amax, amx);
}

int preprocess_bgr(const uint8_t* img, int N, int Hi, int Wi, const int64_t* offsets,
                   const int32_t* heights, const int32_t* widths, const float* means,
                   int Ho, int Wo, float* y, hipStream_t st, float* amax) {
  Means m;
  for (int c = 0; c < 3; ++c) m.m[c] = means[c];
  if ((int64_t)N * Ho == 0 || Wo == 0) return PPS_OK;
  if ((int64_t)N * Ho >= (1ll << 31)) {
    set_error("preprocess: N * Ho must be < 2^31");
    return PPS_ERR_INVALID_ARG;
  }
  // separable two-pass kernel when a band's horizontally filtered rows fit
  // 48 KB of LDS (Wo <= 256 with the 16-row cap); the direct kernel otherwise
  const int kcap = (int)std::min<int64_t>(kPrepRows, (48 * 1024) / ((int64_t)Wo * 12));
  if (kcap >= 8) {
    const int64_t nblk = (int64_t)N * ((Ho + kPrepRows - 1) / kPrepRows);
    hipLaunchKernelGGL(preprocess_sep_kernel, dim3((unsigned)nblk), dim3(256),
                       (size_t)kcap * Wo * 12, st, img, N, Hi, Wi, offsets, heights, widths, m,
                       Ho, Wo, kcap, y, amax);
    PPS_CHECK_LAUNCH("preprocess_sep_kernel");
    return PPS_OK;
  }
  if (amax) {  // (wide outputs: the direct kernel, then a max pass)
    hipLaunchKernelGGL(preprocess_bgr_kernel, dim3((unsigned)(N * Ho), (Wo + 127) / 128),
                       dim3(128), 0, st, img, N, Hi, Wi, offsets, heights, widths, m, Ho, Wo, y);
    PPS_CHECK_LAUNCH("preprocess_bgr_kernel");
    return amax_of(y, (int64_t)N * Ho * Wo * 4, amax, st);
  }
  hipLaunchKernelGGL(preprocess_bgr_kernel, dim3((unsigned)(N * Ho), (Wo + 127) / 128),
                     dim3(128), 0, st, img, N, Hi, Wi, offsets, heights, widths, m, Ho, Wo, y);
  PPS_CHECK_LAUNCH("preprocess_bgr_kernel");
  return PPS_OK;
}

}  // namespace pps

namespace pps {
// ---- max |x| of a tensor (f16x2 activation scales, when the producer did not
// report it; also the reference for the producers' in-epilogue maxima) -------
__global__ void amax_kernel(const float* __restrict__ x, int64_t n, int vec,
                            float* __restrict__ amax) {
  float m = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t n4 = vec ? n / 4 : 0;
  for (int64_t i = t0; i < n4; i += stride) {
    const f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
  for (int64_t i = 4 * n4 + t0; i < n; i += stride) m = fmaxf(m, fabsf(x[i]));
  amax_commit(amax, m);
}

// f16x2 activation planes: planes[0][i] = f16(x[i] 2^s), planes[1][i] =
// f16(x[i] 2^s - planes[0][i]) with 2^s from the slot's max -- exactly the
// split the f16x2 conv kernels apply after an f32 fragment read (split8_h2),
// done once per element instead of once per wave and column tile.  8
// elements per thread.
__global__ void split_act_h2_kernel(const float* __restrict__ x, int64_t n8,
                                    const float* __restrict__ slot, uint16_t* __restrict__ out,
                                    int64_t plane) {
  float inv;
  const float S = h2_scale_of(amax_read(slot), &inv);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += stride) {
    const f32x4 x0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x) + 2 * i);
    const f32x4 x1 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x) + 2 * i + 1);
    bf16x8 f0, f1;
    split8_h2(x0, x1, S, f0, f1);
    *reinterpret_cast<bf16x8*>(out + 8 * i) = f0;
    *reinterpret_cast<bf16x8*>(out + plane + 8 * i) = f1;
  }
}

int split_act_h2(const float* x, int64_t n, const float* slot, uint16_t* planes, int64_t plane,
                 hipStream_t st) {
  if (n <= 0) return PPS_OK;
  const int64_t n8 = n / 8;
  const int64_t want = (n8 + 255) / 256;
  hipLaunchKernelGGL(split_act_h2_kernel, dim3((unsigned)(want < 8192 ? want : 8192)), dim3(256),
                     0, st, x, n8, slot, planes, plane);
  PPS_CHECK_LAUNCH("split_act_h2_kernel");
  return PPS_OK;
}

// The constants of an f16x2-planes-out conv's output bound (EPI_F_H2OUT):
// out[0] = max_c |scale_c| * sum_k |w[c][k]| (k in order, one thread per
// channel), out[1] = max(0, max_c shift_c).  One workgroup; max is
// order-free, so the value is the same on every launch.
__global__ void __launch_bounds__(256)
h2_out_bound_kernel(const float* __restrict__ w, int Cout, int Kpad,
                    const float* __restrict__ scale, const float* __restrict__ shift,
                    float* __restrict__ out) {
  __shared__ float s_w[256], s_b[256];
  float mw = 0.f, mb = 0.f;
  for (int c = threadIdx.x; c < Cout; c += 256) {
    float a = 0.f;
    for (int k = 0; k < Kpad; ++k) a += fabsf(w[(int64_t)c * Kpad + k]);
    mw = fmaxf(mw, fabsf(scale ? scale[c] : 1.f) * a);
    mb = fmaxf(mb, shift[c]);
  }
  s_w[threadIdx.x] = mw;
  s_b[threadIdx.x] = mb;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 256; ++i) {
      mw = fmaxf(mw, s_w[i]);
      mb = fmaxf(mb, s_b[i]);
    }
    // one ulp of headroom per 2^20 (the f32 sum is not an upper bound of the
    // exact one by itself)
    out[0] = mw * (1.f + 0x1p-20f);
    out[1] = mb * (1.f + 0x1p-20f);
  }
}

int amax_of(const float* x, int64_t n, float* amax, hipStream_t st) {
  if (n <= 0) return PPS_OK;
  const int vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  const int64_t want = ((vec ? n / 4 : n) + 255) / 256;
  hipLaunchKernelGGL(amax_kernel, dim3((unsigned)(want < 2048 ? (want > 0 ? want : 1) : 2048)),
                     dim3(256), 0, st, x, n, vec, amax);
  PPS_CHECK_LAUNCH("amax_kernel");
  return PPS_OK;
}
}  // namespace pps

int pps_amax(const float* x, int64_t n, float* amax, void* stream) {
  using namespace pps;
  PPS_ENFORCE(x && amax, "null pointer");
  PPS_ENFORCE(n >= 0, "n must be >= 0");
  return amax_of(x, n, amax, as_stream(stream));
}

int pps_h2_out_bound(const float* w, int Cout, int Kpad, const float* scale, const float* shift,
                     float* out2, void* stream) {
  using namespace pps;
  PPS_ENFORCE(w && shift && out2, "null pointer");
  PPS_ENFORCE(Cout > 0 && Kpad > 0, "bad shape");
  const hipStream_t st = as_stream(stream);
  float* d = nullptr;
  PPS_ENFORCE(hipMallocAsync(&d, 2 * sizeof(float), st) == hipSuccess, "hipMallocAsync");
  hipLaunchKernelGGL(h2_out_bound_kernel, dim3(1), dim3(256), 0, st, w, Cout, Kpad, scale, shift,
                     d);
  const hipError_t e1 = hipMemcpyAsync(out2, d, 2 * sizeof(float), hipMemcpyDeviceToHost, st);
  const hipError_t e2 = hipStreamSynchronize(st);
  (void)hipFreeAsync(d, st);
  PPS_ENFORCE(e1 == hipSuccess && e2 == hipSuccess, "h2_out_bound_kernel");
  return PPS_OK;
}

int pps_split_f16x2_act(const float* x, int64_t n, const float* amax, uint16_t* planes,
                        int64_t plane, void* stream) {
  using namespace pps;
  PPS_ENFORCE(x && amax && planes, "null pointer");
  PPS_ENFORCE(n >= 0 && n % 8 == 0 && plane >= n && plane % 8 == 0,
              "n % 8 == 0 and plane >= n, plane % 8 == 0");
  PPS_ENFORCE(aligned16(x) && aligned16(planes), "16-byte aligned x / planes");
  return split_act_h2(x, n, amax, planes, plane, as_stream(stream));
}
