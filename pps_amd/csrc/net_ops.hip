// Stand-alone (unfused) forms of the Caffe2 operators of the reference's test
// net, for op-by-op execution through the operator registry
// (pps_amd/net.py, `Net.run_eager`): the compatibility surface behind
// `model.net.<OpName>(...)`.  The product forward never calls these -- it runs
// the same graph compiled into fused GEMM epilogues (model.py) -- but every
// op name of the recorded graph (tests/golden/pps_graph_market1501.json) has a
// HIP implementation here or in the GEMM / feature kernels.
//
//   SpatialBN (is_test)  detector.py:419-447 / Caffe2 spatial_batch_norm_op
//   Relu, Sum, Add, Max, Mean (elementwise, n-ary; Mean = sum * 1/n)
//   AveragePool / MaxPool with global_pooling (bpm_heads.py:50-53)
//
// All are HBM-streaming: one read of each input, one write.  NHWC float32.
#include "pps_internal.hpp"

namespace pps {

constexpr int kNetThreads = 256;

// y[m][c] = (x[m][c] - rm[c]) * (s[c] / sqrt(riv[c] + eps)) + b[c]
__global__ void spatial_bn_kernel(const float* __restrict__ x, int64_t n, int C,
                                  const float* __restrict__ s, const float* __restrict__ b,
                                  const float* __restrict__ rm,
                                  const float* __restrict__ riv, float eps, int relu,
                                  float* __restrict__ y) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int c = (int)(i % C);
    const float inv = s[c] / sqrtf(riv[c] + eps);
    float v = (x[i] - rm[c]) * inv + b[c];
    if (relu) v = fmaxf(v, 0.f);
    y[i] = v;
  }
}

int spatial_bn(const float* x, int64_t M, int C, const float* s, const float* b,
               const float* rm, const float* riv, float eps, int relu, float* y,
               hipStream_t st) {
  const int64_t n = M * C;
  if (n <= 0) return PPS_OK;
  const int64_t want = (n + kNetThreads - 1) / kNetThreads;
  const int grid = (int)(want < 65536 ? want : 65536);
  hipLaunchKernelGGL(spatial_bn_kernel, dim3(grid), dim3(kNetThreads), 0, st, x, n, C, s,
                     b, rm, riv, eps, relu, y);
  PPS_CHECK_LAUNCH("spatial_bn_kernel");
  return PPS_OK;
}

// n-ary elementwise: op 0 Sum (in input order), 1 Max, 2 Mean (Sum * (1/k),
// Caffe2's Mean), 3 Relu (k = 1).  Inputs by value in the kernel arguments.
constexpr int kEltMaxIn = 32;
struct EltInputs {
  const float* p[kEltMaxIn];
};

__global__ void eltwise_kernel(EltInputs in, int k, int64_t n, int op,
                               float* __restrict__ y) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float v = in.p[0][i];
    if (op == 3) {
      v = fmaxf(v, 0.f);
    } else {
      for (int j = 1; j < k; ++j) {
        const float u = in.p[j][i];
        v = op == 1 ? fmaxf(v, u) : v + u;
      }
      if (op == 2) v = v * (1.f / (float)k);
    }
    y[i] = v;
  }
}

int eltwise(const float* const* xs, int k, int64_t n, int op, float* y, hipStream_t st) {
  if (n <= 0) return PPS_OK;
  EltInputs in{};
  for (int j = 0; j < k; ++j) in.p[j] = xs[j];
  const int64_t want = (n + kNetThreads - 1) / kNetThreads;
  const int grid = (int)(want < 65536 ? want : 65536);
  hipLaunchKernelGGL(eltwise_kernel, dim3(grid), dim3(kNetThreads), 0, st, in, k, n, op, y);
  PPS_CHECK_LAUNCH("eltwise_kernel");
  return PPS_OK;
}

// Global pooling of a (possibly row-strided) NHWC tensor: image n starts at
// x + n * n_stride and holds H*W*C contiguous values (a Split strip of a
// taller tensor is a view with n_stride = H_full*W*C).  One thread per (n, c):
// mode 0 = mean (sum in (h, w) order, / (H*W)), 1 = max.
__global__ void global_pool_kernel(const float* __restrict__ x, int N, int HW, int C,
                                   int64_t n_stride, int mode, float* __restrict__ y) {
  const int n = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float* p = x + (int64_t)n * n_stride + c;
  float acc = mode ? -INFINITY : 0.f;
  for (int i = 0; i < HW; ++i) {
    const float v = p[(int64_t)i * C];
    acc = mode ? fmaxf(acc, v) : acc + v;
  }
  y[(int64_t)n * C + c] = mode ? acc : acc / (float)HW;
}

int global_pool(const float* x, int N, int H, int W, int C, int64_t n_stride, int mode,
                float* y, hipStream_t st) {
  if (N <= 0 || C <= 0) return PPS_OK;
  dim3 grid((C + kNetThreads - 1) / kNetThreads, N);
  hipLaunchKernelGGL(global_pool_kernel, grid, dim3(kNetThreads), 0, st, x, N, H * W, C,
                     n_stride, mode, y);
  PPS_CHECK_LAUNCH("global_pool_kernel");
  return PPS_OK;
}

}  // namespace pps

using namespace pps;

extern "C" {

int pps_spatial_bn(const float* x, int64_t M, int C, const float* s, const float* b,
                   const float* rm, const float* riv, float eps, int relu, float* y,
                   void* stream) {
  PPS_ENFORCE(x && s && b && rm && riv && y, "null pointer");
  PPS_ENFORCE(M >= 0 && C > 0, "bad shape");
  PPS_ENFORCE(eps >= 0.f, "epsilon must be >= 0");
  return spatial_bn(x, M, C, s, b, rm, riv, eps, relu, y, as_stream(stream));
}

int pps_eltwise(const float* const* inputs, int k, int64_t n, int op, float* y,
                void* stream) {
  PPS_ENFORCE(inputs && y, "null pointer");
  PPS_ENFORCE(k >= 1 && k <= kEltMaxIn,
              "number of inputs must be in [1, " + std::to_string(kEltMaxIn) + "]");
  PPS_ENFORCE(op >= 0 && op <= 3, "unknown elementwise op " + std::to_string(op));
  PPS_ENFORCE(op != 3 || k == 1, "Relu takes one input");
  PPS_ENFORCE(n >= 0, "bad size");
  for (int j = 0; j < k; ++j) PPS_ENFORCE(inputs[j], "null input pointer");
  return eltwise(inputs, k, n, op, y, as_stream(stream));
}

int pps_global_pool(const float* x, int N, int H, int W, int C, int64_t n_stride,
                    int mode, float* y, void* stream) {
  PPS_ENFORCE(x && y, "null pointer");
  PPS_ENFORCE(N >= 0 && H > 0 && W > 0 && C > 0, "bad shape");
  PPS_ENFORCE(n_stride >= (int64_t)H * W * C, "n_stride < H*W*C");
  PPS_ENFORCE(mode == 0 || mode == 1, "mode must be 0 (average) or 1 (max)");
  return global_pool(x, N, H, W, C, n_stride, mode, y, as_stream(stream));
}

}  // extern "C"
