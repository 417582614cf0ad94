// Whole-network entry points of libpps_hip.so (include/pps_abi.h, "feature
// extractor as one call"): pps_model_create builds the PPS test net from a
// Detectron weights blob map, owns its packed / bf16x3-split weights, the
// activation buffers per batch size and the per-layer tile / plane / split-K
// table; pps_forward enqueues the whole forward on one stream.
//
// The plan is built by the same builders the reference uses, with the same
// blob and parameter names (mirrored one for one by pps_amd/model.py):
//   add_ResNet50_conv5_body  detectron/modeling/ResNet.py:39-40,91-126
//     basic_bn_stem          ResNet.py:246-256
//     add_stage              ResNet.py:60-88
//     add_residual_block     ResNet.py:153-195 (stride rule :169-171)
//     bottleneck_transformation ResNet.py:276-333 (STRIDE_1X1 :290)
//     basic_bn_shortcut      ResNet.py:203-220
//   FPN coarsest level       detectron/modeling/FPN_reid.py:160-174 (gated)
//   add_pps_part_head        detectron/modeling/pps_heads.py:38-96
//     add_uniform_partition  detectron/modeling/bpm_heads.py:18-55
//   add_reid_outputs         detectron/modeling/reid_heads.py:34-127
// and compiled into the fused launches of the op-level ABI (test-mode BN
// folded into conv epilogues, projection shortcuts K-concatenated into their
// branch2c GEMM, stem conv + pool fused, part pooling in the last conv's
// epilogue, 31 heads as one split-K batched GEMM + one BN/ReLU/Normalize
// pass).  Each launch goes through the same pps_* entry point, with the same
// arguments, as the Python orchestrator (pps_amd/model.py PPSModel), so the
// two give identical bits for the same tile / plane / split-K table.
//
// This replaces the reference's `workspace.RunNet(model.net)` of the test net
// (detectron/core/test.py:163-165) behind a C ABI.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "pps_internal.hpp"

namespace pps {
namespace {

constexpr double kBnEps = 1e-5;  // Caffe2 SpatialBN default epsilon (pytorch v1.0.1)
constexpr int kHeadSplitK = 8;   // K = 2048 head GEMMs cut 8 ways (pps_amd/model.py HEAD_SPLITK)
constexpr int kMaxSplitK = 4;    // conv split-K factors the autotune tries

enum class Op { Conv, ConvDual, MaxPool, StemPool, Pps, ConvPps, Heads, Normalize };

const char* op_name(Op op) {
  switch (op) {
    case Op::Conv: return "conv";
    case Op::ConvDual: return "conv_dual";
    case Op::MaxPool: return "maxpool";
    case Op::StemPool: return "stem_pool";
    case Op::Pps: return "pps";
    case Op::ConvPps: return "conv_pps";
    case Op::Heads: return "heads";
    case Op::Normalize: return "normalize";
  }
  return "?";
}

struct ModelError : std::runtime_error {
  int code;
  ModelError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
#define PPS_MCHECK(cond, msg)                                                         \
  do {                                                                                \
    if (!(cond))                                                                      \
      throw ModelError(PPS_ERR_INVALID_ARG, std::string("[enforce fail at ") +       \
                                                __func__ + "] " + #cond + ". " + (msg)); \
  } while (0)

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw ModelError(PPS_ERR_LAUNCH, std::string(what) + ": " + hipGetErrorString(e));
}
void rc_check(int rc) {  // an op-level entry point failed: its message is already set
  if (rc != PPS_OK) throw ModelError(rc, pps_last_error());
}

// ---- plan (structure only) -------------------------------------------------
struct PlanLayer {
  Op op;
  std::string name, bn, input, output, residual;
  int cin = 0, cout = 0, k = 1, stride = 1, pad = 0, dil = 1;
  bool relu = false;
  std::vector<int> split;  // pps
  bool max_ave = false;
  std::vector<std::string> prefixes;
  int dim = 0, dim_inner = 0;
};

struct Plan {
  std::vector<PlanLayer> layers;
  std::map<std::string, std::vector<int64_t>> params;
  std::string output;
  int feat_dim = 0;

  std::string conv(const std::string& in, const std::string& prefix, int din, int dout, int k,
                   int stride, int pad, int dil = 1, bool relu = false,
                   const std::string& residual = "", const std::string& out = "",
                   bool bias = false, const std::string& bn_name = "") {
    params[prefix + "_w"] = {dout, din, k, k};
    if (bias) params[prefix + "_b"] = {dout};
    const std::string bn = bn_name.empty() ? prefix + "_bn" : bn_name;
    for (const char* s : {"_s", "_b", "_rm", "_riv"}) params[bn + s] = {dout};
    PlanLayer L;
    L.op = Op::Conv; L.name = prefix; L.bn = bn; L.input = in;
    L.output = out.empty() ? bn : out;
    L.cin = din; L.cout = dout; L.k = k; L.stride = stride; L.pad = pad; L.dil = dil;
    L.relu = relu; L.residual = residual;
    layers.push_back(L);
    return L.output;
  }
};

// model.py basic_bn_stem (ResNet.py:246-256)
std::string basic_bn_stem(Plan& p) {
  const std::string c = p.conv("data", "conv1", 3, 64, 7, 2, 3, 1, true, "", "", false, "res_conv1_bn");
  PlanLayer L;
  L.op = Op::MaxPool; L.input = c; L.output = "pool1"; L.k = 3; L.stride = 2; L.pad = 1;
  p.layers.push_back(L);
  return "pool1";
}

// ResNet.py:276-333 (+ the Sum/Relu of add_residual_block :186-195)
std::string bottleneck(Plan& p, const PpsModelConfig& c, const std::string& in, int din, int dout,
                       int stride, const std::string& prefix, int dinner, int dil,
                       const std::string& shortcut, const std::string& out) {
  const int s1 = c.stride_1x1 ? stride : 1, s3 = c.stride_1x1 ? 1 : stride;
  std::string cur = p.conv(in, prefix + "_branch2a", din, dinner, 1, s1, 0, 1, true);
  cur = p.conv(cur, prefix + "_branch2b", dinner, dinner, 3, s3, dil, dil, true);
  return p.conv(cur, prefix + "_branch2c", dinner, dout, 1, 1, 0, 1, true, shortcut, out);
}

// ResNet.py:153-195 with basic_bn_shortcut :203-220
std::string residual_block(Plan& p, const PpsModelConfig& c, const std::string& prefix,
                           const std::string& in, int din, int dout, int dinner, int dil,
                           int stride_init, bool inplace_sum) {
  const int stride = (din != dout && din != 64 && dil == 1) ? stride_init : 1;
  std::string sc = in;
  if (din != dout) sc = p.conv(in, prefix + "_branch1", din, dout, 1, stride, 0);
  const std::string out = prefix + (inplace_sum ? "_branch2c_bn" : "_sum");
  return bottleneck(p, c, in, din, dout, stride, prefix, dinner, dil, sc, out);
}

// ResNet.py:60-88
std::string add_stage(Plan& p, const PpsModelConfig& c, const std::string& prefix,
                      std::string in, int n, int& din, int dout, int dinner, int dil,
                      int stride_init) {
  for (int i = 0; i < n; ++i) {
    in = residual_block(p, c, prefix + "_" + std::to_string(i), in, din, dout, dinner, dil,
                        stride_init, i < n - 1);
    din = dout;
  }
  return in;
}

// bpm_heads.py:18-35: strip heights along H
std::vector<int> uniform_partition_split(const PpsModelConfig& c, double spatial_scale) {
  static const std::map<int, std::vector<int>> table = {
      {7, {3, 3, 4, 4, 4, 3, 3}}, {5, {5, 5, 4, 5, 5}},
      {9, {2, 3, 3, 3, 3, 3, 3, 2, 2}}, {10, {2, 2, 2, 3, 3, 3, 3, 2, 2, 2}}};
  std::vector<int> out;
  auto it = table.find(c.strip_num);
  if (it != table.end() && c.height == 16 * 24) {
    const double scale = 16 * spatial_scale;
    for (int s : it->second) out.push_back((int)(s * scale));
    return out;
  }
  const int h = (int)(c.height * spatial_scale / c.strip_num);
  out.assign(c.strip_num, h);
  return out;
}

Plan build_plan(const PpsModelConfig& c) {
  Plan p;
  std::string s = basic_bn_stem(p);
  int din = 64;
  const int db = c.num_groups * c.width_per_group;
  s = add_stage(p, c, "res2", s, 3, din, 256, db, 1, 2);
  s = add_stage(p, c, "res3", s, 4, din, 512, db * 2, 1, 2);
  s = add_stage(p, c, "res4", s, 6, din, 1024, db * 4, 1, 2);
  s = add_stage(p, c, "res5", s, 3, din, 2048, db * 8, c.res5_dilation, c.res5_stride);
  const double scale = 1. / 16. * c.res5_dilation / c.res5_stride;
  int dim = din;
  if (c.fpn_on && dim != c.fpn_dim) {  // FPN_reid.py:160-174 (coarsest level only)
    s = p.conv(s, "fpn_inner_" + s, dim, c.fpn_dim, 1, 1, 0, 1, true, "", "", true,
               "fpn_inner_" + s + "_bn");
    dim = c.fpn_dim;
  }
  // pps_heads.py:38-96: subset i = bits of i; blob prefix pps + digits
  PlanLayer P;
  P.op = Op::Pps; P.input = s; P.output = "pps_pool2_all"; P.dim = dim;
  P.split = uniform_partition_split(c, scale);
  P.max_ave = c.max_ave != 0;
  for (int i = 1; i < (1 << c.strip_num); ++i) {
    std::string pre = "pps";
    for (int j = 0; j < c.strip_num; ++j)
      if (i & (1 << j)) pre += std::to_string(j);
    P.prefixes.push_back(pre);
  }
  p.layers.push_back(P);
  // reid_heads.py:34-127 (test branch; the unused FC logits are not built)
  for (const auto& pre : P.prefixes) {
    p.params[pre + "_conv_w"] = {c.bpm_dim, dim, 1, 1};
    p.params[pre + "_conv_b"] = {c.bpm_dim};
    for (const char* sfx : {"_s", "_b", "_rm", "_riv"}) p.params[pre + "_bn" + sfx] = {c.bpm_dim};
  }
  PlanLayer H;
  H.op = Op::Heads; H.input = P.output; H.prefixes = P.prefixes; H.dim = dim;
  H.dim_inner = c.bpm_dim; H.output = "reid_feature_concat";
  p.layers.push_back(H);
  p.output = H.output;
  if (c.normalize) {
    PlanLayer N;
    N.op = Op::Normalize; N.input = H.output; N.output = "reid_feature_concat_norm";
    p.layers.push_back(N);
    p.output = N.output;
  }
  p.feat_dim = (int)P.prefixes.size() * c.bpm_dim;
  return p;
}

// ---- device memory ------------------------------------------------------------
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  explicit DevBuf(size_t n) : bytes(n) {
    if (n) hip_check(hipMalloc(&p, n), "hipMalloc");
  }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};
using Buf = std::shared_ptr<DevBuf>;

Buf upload(const std::vector<float>& h, hipStream_t st) {
  auto b = std::make_shared<DevBuf>(h.size() * sizeof(float));
  hip_check(hipMemcpyAsync(b->p, h.data(), b->bytes, hipMemcpyHostToDevice, st), "hipMemcpyAsync");
  hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");  // h may die after return
  return b;
}

// f32 weights -> bf16x3 planes [nbatch][3][n] (pps_split_bf16x3)
Buf split3(const Buf& w, int64_t n, int nbatch, hipStream_t st) {
  auto b = std::make_shared<DevBuf>((size_t)n * nbatch * 3 * sizeof(uint16_t));
  rc_check(pps_split_bf16x3(w->as<float>(), n, nbatch, b->as<uint16_t>(), st));
  hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
  return b;
}

// f32 weights [rows][K] -> the f16x2 split (pps_split_f16x2_sqnorm_tiled):
// chunk-tiled planes [2][rows16 / 16][K / 32][16][32] and per-row scales
void split_h2w(const Buf& w, int rows, int64_t K, Buf& w2, Buf& wrs, hipStream_t st) {
  const int64_t r16 = (rows + 15) / 16 * 16;
  w2 = std::make_shared<DevBuf>((size_t)2 * r16 * K * sizeof(uint16_t));
  wrs = std::make_shared<DevBuf>((size_t)rows * sizeof(float));
  DevBuf sq((size_t)rows * sizeof(float));
  rc_check(pps_split_f16x2_sqnorm_tiled(w->as<float>(), rows, (int)K, K, w2->as<uint16_t>(),
                                        wrs->as<float>(), sq.as<float>(), st));
  hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
}

// ---- weights (host) -------------------------------------------------------------
struct Blob {
  const float* data;
  std::vector<int64_t> shape;
  int64_t numel() const {
    int64_t n = 1;
    for (auto s : shape) n *= s;
    return n;
  }
};

// model.py fold_bn: test-mode SpatialBN y = (x - rm) * s / sqrt(riv + eps) + b as
// y = x * scale + shift, in float64 then rounded to float32 (conv bias in shift)
void fold_bn(const std::map<std::string, Blob>& blobs, const std::string& bn, const Blob* bias,
             std::vector<float>& scale, std::vector<float>& shift) {
  const Blob& s = blobs.at(bn + "_s");
  const Blob& b = blobs.at(bn + "_b");
  const Blob& rm = blobs.at(bn + "_rm");
  const Blob& riv = blobs.at(bn + "_riv");
  const int64_t n = s.numel();
  scale.resize(n);
  shift.resize(n);
  for (int64_t i = 0; i < n; ++i) {
    const double sc = (double)s.data[i] / std::sqrt((double)riv.data[i] + kBnEps);
    const double cb = bias ? (double)bias->data[i] : 0.0;
    scale[i] = (float)sc;
    shift[i] = (float)((cb - (double)rm.data[i]) * sc + (double)b.data[i]);
  }
}

// [Cout][Cin][KH][KW] -> [Cout][Kpad], K ordered (kh, kw, cin), Kpad % 16 == 0
std::vector<float> pack_conv(const Blob& w, int cin_pad, int& kpad) {
  const int64_t co = w.shape[0], ci = w.shape[1], kh = w.shape[2], kw = w.shape[3];
  const int64_t cp = std::max<int64_t>(cin_pad, ci);
  const int64_t k = kh * kw * cp;
  kpad = (int)((k + 15) / 16 * 16);
  std::vector<float> out((size_t)co * kpad, 0.f);
  for (int64_t o = 0; o < co; ++o)
    for (int64_t y = 0; y < kh; ++y)
      for (int64_t x = 0; x < kw; ++x)
        for (int64_t c = 0; c < ci; ++c)
          out[o * kpad + (y * kw + x) * cp + c] = w.data[((o * ci + c) * kh + y) * kw + x];
  return out;
}

// conv1 [64][3][7][7] -> the fused stem's [64][pps_stem_k()] layout: K index
// (kh * 3 + c) * 8 + kw, kw = 7 and the tail zero (stem.hip, model.py pack_stem_weight)
std::vector<float> pack_stem(const Blob& w) {
  const int K = pps_stem_k();
  std::vector<float> out((size_t)64 * K, 0.f);
  for (int o = 0; o < 64; ++o)
    for (int kh = 0; kh < 7; ++kh)
      for (int c = 0; c < 3; ++c)
        for (int kw = 0; kw < 7; ++kw)
          out[(size_t)o * K + (kh * 3 + c) * 8 + kw] = w.data[((o * 3 + c) * 7 + kh) * 7 + kw];
  return out;
}

// ---- compiled layers ----------------------------------------------------------
struct Layer {
  Op op;
  std::string name;  // tuning key: conv name, or the output blob for heads / pooling
  std::string input, input2, output, residual, conv_output;
  int cin = 0, cout = 0, k = 1, stride = 1, pad = 0, dil = 1, stride2 = 1;
  bool relu = false;
  int cin_eff = 0, kpad = 0, shortcut_cin = 0;
  Buf w, scale, shift;  // w: f32 [Cout][Kpad] or bf16x3 planes
  Buf wt;               // x3 plain convs with Kpad % 32 == 0: the planes chunk-tiled
                        // (pps_tile_planes), used when tile carries PPS_TILE_B_TILED
  float h2o_bw = 0.f, h2o_bb = 0.f;  // output bound constants (pps_h2_out_bound; 0: none)
  Buf w2, wrs;          // the f16x2 split (PPS_TILE_H2): two chunk-tiled f16 planes
                        // [2][Cout16/16][K/32][16][32] and per-channel scales [Cout]
  std::vector<int> split;
  bool max_ave = false, normalize = false;
  int nsub = 0, dim = 0, dim_inner = 0;
  int tile = 0, splitk = 1;
  bool planes_in = false, planes_out = false;
  int seam_next = -1;   // the next layer a PPS_TILE_SEAM launch also computes
};

struct Shape {
  int64_t d[4] = {0, 0, 0, 0};
  int64_t numel() const { return d[0] * d[1] * d[2] * d[3]; }
};

struct Workspace {
  int N = 0;
  std::map<std::string, Shape> shapes;
  std::map<std::string, Buf> bufs;  // plane-capable tensors hold 6 B per element
  Buf part;                         // conv split-K partials
  size_t part_floats = 0;
  Buf h2p;                          // f16x2 activation planes of a PPS_TILE_H2P layer's input
  size_t h2p_elems = 0;
  Buf cnt;                          // one-launch split-K tile counters (zero between launches)
  size_t cnt_ints = 0;
  Buf nhwc4;                        // input staging for pps_forward_nchw / _bgr
  Buf amax;                         // per-tensor max |x| (PpsModel::slot), zeroed per forward
  std::vector<char> amax_need;      // slots this forward reports (set by forward_range)
  // set by pps_model_reserve: a graph captured afterwards may hold these
  // buffers' addresses, so they are never reallocated until pps_model_release
  bool pinned = false;
};

}  // namespace
}  // namespace pps

struct PpsModel {
  PpsModelConfig cfg;
  pps::Plan plan;
  std::vector<pps::Layer> layers;
  std::vector<std::pair<int, int>> edges;  // plane-eligible (producer, consumer) layer indices
  std::set<std::string> plane_capable;     // outputs of edge producers
  bool x3 = true, fused_stem = false, fused_pps = false, act_planes = false;
  std::map<std::string, int> slot;         // activation tensor -> its max |x| slot
  // every producer reports its maximum (autotune: any layer may try an f16x2
  // tile; env PPS_AMAX_ALL=1), else only the inputs of PPS_TILE_H2 layers
  mutable bool amax_all = false;
  mutable std::map<int, pps::Workspace> ws;
  mutable std::vector<std::string> names;  // storage for pps_model_layer_info
};

namespace pps {
namespace {

int conv_out(int h, int pad, int dil, int k, int stride) {
  return (h + 2 * pad - dil * (k - 1) - 1) / stride + 1;
}

int count_readers(const PpsModel& m, const std::string& blob, bool all_keys) {
  int n = 0;
  for (const auto& L : m.layers) {
    if (L.input == blob) ++n;
    if (all_keys && (L.input2 == blob || L.residual == blob)) ++n;
  }
  return n;
}

void compile(PpsModel& m, const std::map<std::string, Blob>& blobs, hipStream_t st) {
  const Plan& plan = m.plan;
  // projection shortcuts fused into their block's branch2c GEMM (K concat)
  std::map<std::string, const PlanLayer*> shortcut_of;
  for (const auto& L : plan.layers)
    if (L.op == Op::Conv && L.name.size() > 8 &&
        L.name.compare(L.name.size() - 8, 8, "_branch1") == 0 && L.k == 1)
      shortcut_of[L.output] = &L;
  auto bias_of = [&](const std::string& n) -> const Blob* {
    auto it = blobs.find(n);
    return it == blobs.end() ? nullptr : &it->second;
  };
  for (const auto& P : plan.layers) {
    Layer L;
    L.op = P.op; L.name = P.name.empty() ? P.output : P.name;
    L.input = P.input; L.output = P.output; L.residual = P.residual;
    L.cin = P.cin; L.cout = P.cout; L.k = P.k; L.stride = P.stride; L.pad = P.pad; L.dil = P.dil;
    L.relu = P.relu;
    if (P.op == Op::Conv && shortcut_of.count(P.output)) continue;  // inside its branch2c
    if (P.op == Op::Conv && shortcut_of.count(P.residual)) {
      const PlanLayer& S = *shortcut_of.at(P.residual);
      int kpad1 = 0, kpad2 = 0;
      std::vector<float> w1 = pack_conv(blobs.at(P.name + "_w"), 0, kpad1);
      std::vector<float> w2 = pack_conv(blobs.at(S.name + "_w"), 0, kpad2);
      PPS_MCHECK(kpad1 == P.cin && kpad2 == S.cin, "fused shortcut needs Cin % 16 == 0");
      std::vector<float> s1, h1, s2, h2;
      fold_bn(blobs, P.bn, nullptr, s1, h1);
      fold_bn(blobs, S.bn, nullptr, s2, h2);
      const int K = kpad1 + kpad2;
      std::vector<float> w((size_t)P.cout * K), sh(P.cout);
      for (int o = 0; o < P.cout; ++o) {
        for (int k = 0; k < kpad1; ++k) w[(size_t)o * K + k] = w1[(size_t)o * kpad1 + k] * s1[o];
        for (int k = 0; k < kpad2; ++k)
          w[(size_t)o * K + kpad1 + k] = w2[(size_t)o * kpad2 + k] * s2[o];
        sh[o] = h1[o] + h2[o];
      }
      L.op = Op::ConvDual;
      L.w = upload(w, st); L.shift = upload(sh, st);
      L.kpad = kpad1; L.cin_eff = P.cin;
      L.input2 = S.input; L.stride2 = S.stride; L.residual.clear(); L.shortcut_cin = S.cin;
      m.layers.push_back(L);
      continue;
    }
    if (P.op == Op::Conv) {
      const int cin_pad = P.cin == 3 ? 4 : 0;
      std::vector<float> w = pack_conv(blobs.at(P.name + "_w"), cin_pad, L.kpad);
      std::vector<float> sc, sh;
      fold_bn(blobs, P.bn, bias_of(P.name + "_b"), sc, sh);
      L.w = upload(w, st); L.scale = upload(sc, st); L.shift = upload(sh, st);
      L.cin_eff = cin_pad ? cin_pad : P.cin;
    } else if (P.op == Op::Heads) {
      const int nb = (int)P.prefixes.size();
      std::vector<float> w((size_t)nb * P.dim_inner * P.dim), sc, sh, s1, h1;
      for (int b = 0; b < nb; ++b) {
        const Blob& wb = blobs.at(P.prefixes[b] + "_conv_w");
        std::copy(wb.data, wb.data + (size_t)P.dim_inner * P.dim,
                  w.begin() + (size_t)b * P.dim_inner * P.dim);
        fold_bn(blobs, P.prefixes[b] + "_bn", bias_of(P.prefixes[b] + "_conv_b"), s1, h1);
        sc.insert(sc.end(), s1.begin(), s1.end());
        sh.insert(sh.end(), h1.begin(), h1.end());
      }
      L.w = upload(w, st); L.scale = upload(sc, st); L.shift = upload(sh, st);
      L.dim = P.dim; L.dim_inner = P.dim_inner; L.nsub = nb;
    } else if (P.op == Op::Pps) {
      L.split = P.split; L.max_ave = P.max_ave; L.nsub = (int)P.prefixes.size();
    } else if (P.op == Op::Normalize && !m.layers.empty() && m.layers.back().op == Op::Heads) {
      // heads as split-K partials + one reduce/BN/ReLU/Normalize pass
      m.layers.back().normalize = true;
      m.layers.back().output = P.output;
      m.layers.back().name = P.output;
      continue;
    }
    m.layers.push_back(L);
  }
  if (m.x3) {
    for (auto& L : m.layers) {
      // the f16x2 split beside the bf16x3 one where an f16x2 tile can run
      // the layer (PPS_TILE_H2: Cin % 32 == 0, no K padding)
      if ((L.op == Op::Conv || L.op == Op::ConvDual) && L.cin_eff % 32 == 0 &&
          L.kpad == L.k * L.k * L.cin_eff && (L.op == Op::Conv || L.shortcut_cin % 32 == 0))
        split_h2w(L.w, L.cout, L.op == Op::ConvDual ? L.kpad + L.shortcut_cin : L.kpad, L.w2,
                  L.wrs, st);
      // a conv + BN + ReLU that may write f16x2 planes for its consumer
      // (PPS_TILE_H2E): the bound constants, from the f32 weights
      if (L.op == Op::Conv && L.relu && L.residual.empty() && L.cin_eff % 32 == 0 &&
          L.kpad == L.k * L.k * L.cin_eff && L.scale && L.shift) {
        float b2[2];
        rc_check(pps_h2_out_bound(L.w->as<float>(), L.cout, L.kpad, L.scale->as<float>(),
                                  L.shift->as<float>(), b2, st));
        L.h2o_bw = b2[0];
        L.h2o_bb = b2[1];
      }
      if (L.op == Op::Conv || L.op == Op::ConvDual)
        L.w = split3(L.w, (int64_t)L.cout * (L.op == Op::ConvDual ? L.kpad + L.shortcut_cin : L.kpad), 1, st);
      const int64_t kt = L.op == Op::ConvDual ? L.kpad + L.shortcut_cin : L.kpad;
      if ((L.op == Op::Conv || L.op == Op::ConvDual) && kt % 32 == 0 && L.cin_eff % 32 == 0) {
        const int64_t c16 = (L.cout + 15) / 16 * 16;
        L.wt = std::make_shared<DevBuf>((size_t)3 * c16 * kt * sizeof(uint16_t));
        rc_check(pps_tile_planes(L.w->as<uint16_t>(), L.cout, (int)kt, kt, (int64_t)L.cout * kt,
                                 L.wt->as<uint16_t>(), st));
        hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
      }
      else if (L.op == Op::Heads)
        L.w = split3(L.w, (int64_t)L.dim_inner * L.dim, L.nsub, st);
    }
  }
  // conv1 + BN + ReLU + pool1 as one kernel (x3, input width 128 only)
  if (m.fused_stem) {
    bool done = false;
    for (size_t i = 0; i + 1 < m.layers.size() && !done; ++i) {
      Layer& L = m.layers[i];
      const Layer& P = m.layers[i + 1];
      if (L.op == Op::Conv && L.input == "data" && L.k == 7 && L.stride == 2 && L.pad == 3 &&
          L.dil == 1 && L.cin == 3 && L.cout == 64 && L.relu && L.residual.empty() &&
          P.op == Op::MaxPool && P.input == L.output && P.k == 3 && P.stride == 2 && P.pad == 1 &&
          count_readers(m, L.output, false) == 1) {
        Layer F = L;
        F.op = Op::StemPool; F.output = P.output; F.conv_output = L.output;
        const Buf wf = upload(pack_stem(blobs.at(L.name + "_w")), st);
        F.w = split3(wf, 64LL * pps_stem_k(), 1, st);
        // and the f16x2 split (PPS_TILE_H2 on the stem): [2][64][K] f16 + 2^-s per channel
        F.w2 = std::make_shared<DevBuf>((size_t)2 * 64 * pps_stem_k() * sizeof(uint16_t));
        F.wrs = std::make_shared<DevBuf>((size_t)64 * sizeof(float));
        rc_check(stem_split_h2(wf->as<float>(), F.w2->as<uint16_t>(), F.wrs->as<float>(), st));
        hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
        m.layers[i] = F;
        m.layers.erase(m.layers.begin() + i + 1);
        done = true;
      }
    }
    m.fused_stem = done;
  }
  // the last conv (+ residual + ReLU) and the part pooling that is its only
  // reader as one conv_pps layer (x3)
  if (m.fused_pps) {
    bool done = false;
    for (size_t i = 0; i + 1 < m.layers.size() && !done; ++i) {
      Layer& L = m.layers[i];
      const Layer& P = m.layers[i + 1];
      if (L.op == Op::Conv && !L.residual.empty() && L.relu && P.op == Op::Pps &&
          P.input == L.output && L.output != m.plan.output && L.cin_eff % 32 == 0 &&
          L.kpad == L.k * L.k * L.cin_eff && count_readers(m, L.output, true) == 1) {
        Layer F = L;
        F.op = Op::ConvPps; F.output = P.output; F.conv_output = L.output;
        F.split = P.split; F.max_ave = P.max_ave; F.nsub = P.nsub;
        m.layers[i] = F;
        m.layers.erase(m.layers.begin() + i + 1);
        done = true;
      }
    }
    m.fused_pps = done;
  }
  // (producer, consumer) conv pairs whose tensor may travel as bf16x3 planes:
  // one reader, a plain conv / conv_pps taking it as main input, Cin % 32 == 0
  if (m.act_planes) {
    for (size_t i = 0; i < m.layers.size(); ++i) {
      const Layer& L = m.layers[i];
      if (L.op != Op::Conv || L.cin_eff % 4 || L.cout % 4 || L.output == m.plan.output) continue;
      int nread = 0, j = -1;
      bool main_input = false;
      for (size_t r = 0; r < m.layers.size(); ++r) {
        const Layer& R = m.layers[r];
        if (R.input == L.output) { ++nread; j = (int)r; main_input = true; }
        if (R.input2 == L.output) { ++nread; j = (int)r; main_input = false; }
        if (R.residual == L.output) { ++nread; j = (int)r; main_input = false; }
      }
      if (nread == 1 && main_input &&
          (m.layers[j].op == Op::Conv || m.layers[j].op == Op::ConvPps) &&
          m.layers[j].cin_eff % 32 == 0) {
        m.edges.emplace_back((int)i, j);
        m.plane_capable.insert(L.output);
      }
    }
    // heuristic before any autotune: the 3x3 consumers with Cin >= 256
    for (auto& e : m.edges) {
      const Layer& C = m.layers[e.second];
      const bool on = C.k > 1 && C.cin >= 256;
      m.layers[e.first].planes_out = m.layers[e.second].planes_in = on;
    }
  }
  // one activation-max slot per tensor (the input and every layer output):
  // each producer reports max |y| there, the f16x2 layers scale by it
  m.slot["data"] = 0;
  for (const auto& L : m.layers)
    for (const std::string* t : {&L.output, &L.conv_output})
      if (!t->empty() && !m.slot.count(*t)) {
        const int n = (int)m.slot.size();
        m.slot[*t] = n;
      }
}

// ---- shapes / workspaces ------------------------------------------------------
std::map<std::string, Shape> infer_shapes(const PpsModel& m, int N) {
  std::map<std::string, Shape> s;
  s["data"] = Shape{{N, m.cfg.height, m.cfg.width, 4}};
  for (const auto& L : m.layers) {
    const Shape& x = s.at(L.input);
    switch (L.op) {
      case Op::Conv: case Op::ConvDual:
        s[L.output] = Shape{{x.d[0], conv_out((int)x.d[1], L.pad, L.dil, L.k, L.stride),
                             conv_out((int)x.d[2], L.pad, L.dil, L.k, L.stride), L.cout}};
        break;
      case Op::MaxPool:
        s[L.output] = Shape{{x.d[0], (x.d[1] + 2 * L.pad - L.k) / L.stride + 1,
                             (x.d[2] + 2 * L.pad - L.k) / L.stride + 1, x.d[3]}};
        break;
      case Op::StemPool: {
        const int64_t hc = (x.d[1] - 1) / 2 + 1, wc = (x.d[2] - 1) / 2 + 1;
        s[L.output] = Shape{{x.d[0], (hc - 1) / 2 + 1, (wc - 1) / 2 + 1, L.cout}};
        break;
      }
      case Op::Pps:
        s[L.output] = Shape{{L.nsub, x.d[0], x.d[3], 1}};
        break;
      case Op::ConvPps:
        s[L.conv_output] = Shape{{x.d[0], conv_out((int)x.d[1], L.pad, L.dil, L.k, L.stride),
                                  conv_out((int)x.d[2], L.pad, L.dil, L.k, L.stride), L.cout}};
        s[L.output] = Shape{{L.nsub, x.d[0], L.cout, 1}};
        break;
      case Op::Heads:
        s[L.output] = Shape{{N, (int64_t)L.nsub * L.dim_inner, 1, 1}};
        s[L.output + "_partials"] = Shape{{kHeadSplitK, N, (int64_t)L.nsub * L.dim_inner, 1}};
        break;
      case Op::Normalize:
        s[L.output] = x;
        break;
    }
  }
  return s;
}

std::vector<int> pps_tiles(const PpsModel& m, const Layer& L, const Shape& conv_shape) {
  std::vector<int> out;
  const int rows = (int)(conv_shape.d[1] * conv_shape.d[2]);
  for (int t = GEMM_TILE_P_FIRST; t < GEMM_NUM_TILES; ++t) {
    const int r = x3p_tile_rows(t, L.planes_in), c = x3p_tile_cols(t, L.planes_in);
    if (r == rows && c > 0 && c <= kPpsFuseMaxCols) out.push_back(t);
  }
  (void)m;
  return out;
}

// f16x2 activation planes of the largest PPS_TILE_H2P input (2 x int16 per element)
size_t h2p_need(const PpsModel& m, const std::map<std::string, Shape>& shapes) {
  size_t need = 0;
  for (const auto& L : m.layers)
    if ((L.tile & PPS_TILE_H2P) && (L.tile & PPS_TILE_H2))
      need = std::max(need, (size_t)shapes.at(L.input).numel());
  return need;
}

size_t part_need(const PpsModel& m, const std::map<std::string, Shape>& shapes) {
  size_t need = 0;
  for (const auto& L : m.layers)
    if (L.op == Op::Conv && L.splitk > 1)
      need = std::max(need, (size_t)L.splitk * (size_t)shapes.at(L.output).numel());
  return need;
}

// tiles built with the one-launch split-K epilogue (gemm_x3p.hip FX)
// A branch2c -> next branch2a pair the seam kernel covers (structure only;
// seam_ok adds the table's conditions)
bool seam_pair(const PpsModel& m, size_t i) {
  if (!m.x3 || i + 1 >= m.layers.size()) return false;
  const Layer& L = m.layers[i];
  const Layer& X = m.layers[i + 1];
  auto plain1x1 = [](const Layer& A) {
    return A.op == Op::Conv && A.k == 1 && A.stride == 1 && A.pad == 0 && A.relu &&
           A.kpad == A.cin_eff && A.w;
  };
  return plain1x1(L) && plain1x1(X) && !L.residual.empty() && X.residual.empty() &&
         X.input == L.output && X.cin_eff == L.cout && seam_supported(L.cin_eff, L.cout, X.cout);
}
bool seam_ok(const PpsModel& m, const Layer& L) {
  if (L.seam_next < 0) return false;
  const Layer& X = m.layers[L.seam_next];
  return !L.planes_in && !L.planes_out && !X.planes_out && L.splitk == 1 && X.splitk == 1;
}

// A layer the f16x2 weight-stationary kernel takes (gemm_ws.hip ws_eligible):
// a 1x1 / stride-1 / unpadded conv, or the fused shortcut conv, whose K =
// Cin (+ the shortcut's Cin) is 64, 128 or 256
bool ws_h2_layer(const Layer& L) {
  if (L.op != Op::Conv && L.op != Op::ConvDual) return false;
  if (L.k != 1 || L.stride != 1 || L.pad != 0 || L.kpad != L.cin_eff) return false;
  const int K = L.cin_eff + (L.op == Op::ConvDual ? L.shortcut_cin : 0);
  return (K == 64 || K == 128 || K == 256) && L.cout % 64 == 0;
}

// A PPS_TILE_H2 tile this layer can run (structure only; planes and split-K
// are checked at run time, since they may change after the tile is set)
bool h2_tile_ok(const Layer& L, int tile) {
  const int base = tile & 0xff;
  if (!L.w2 || (tile & PPS_TILE_SEAM)) return false;
  // the fused stem: its own kernel, no tile id, no planes at either end
  if (L.op == Op::StemPool) return tile == PPS_TILE_H2;
  // activation planes: plain convs and conv_pps (the fused shortcut reads f32)
  if ((tile & (PPS_TILE_H2P | PPS_TILE_H2E)) && L.op == Op::ConvDual) return false;
  if ((tile & PPS_TILE_H2P) && (tile & PPS_TILE_H2E)) return false;
  if (L.op != Op::Conv && L.op != Op::ConvDual && L.op != Op::ConvPps) return false;
  if (!L.relu && L.op == Op::Conv) return false;  // the f16x2 epilogues end in a ReLU
  if (base == 0) return true;
  if (base == GEMM_TILE_WS)  // the weight-stationary 1x1 (f32 input, K = 64 / 128 / 256)
    return ws_h2_layer(L) && !(tile & (PPS_TILE_H2P | PPS_TILE_H2E));
  if (base < GEMM_TILE_P16_FIRST || base >= GEMM_NUM_TILES) return false;
  return L.op == Op::Conv || base < GEMM_TILE_C16_FIRST || base == GEMM_TILE_P16_192x128W41;
}

// The producer whose f16x2-planes output a PPS_TILE_H2E layer C reads
// (structure only; planes / split-K at run time), or -1
int h2e_producer(const PpsModel& m, const Layer& C) {
  if (C.op != Op::Conv && C.op != Op::ConvPps) return -1;
  for (size_t i = 0; i < m.layers.size(); ++i) {
    const Layer& P = m.layers[i];
    if (P.output != C.input) continue;
    if (P.op != Op::Conv || !P.relu || !P.residual.empty() || P.h2o_bw <= 0.f) return -1;
    if (count_readers(m, P.output, true) != 1) return -1;
    if (i > 0 && m.layers[i - 1].seam_next == (int)i) return -1;  // a seam pair's second half
    return (int)i;
  }
  return -1;
}

bool fix_tile(int tile) {
  const int t = tile & 0xff;
  return t == GEMM_TILE_P16_FIRST + 7 ||
         (t >= GEMM_TILE_P16_192x128W42 && t <= GEMM_TILE_P16_96x128W24);
}

// tile counters for the one-launch split-K: an upper bound on the output
// tiles of any split conv (the smallest FIX tile is 96 x 128 / 192 x 64)
size_t cnt_need(const PpsModel& m, const std::map<std::string, Shape>& shapes) {
  size_t need = 0;
  for (const auto& L : m.layers)
    if (L.op == Op::Conv && L.splitk > 1) {
      const Shape& y = shapes.at(L.output);
      const size_t M = (size_t)(y.d[0] * y.d[1] * y.d[2]);
      need = std::max(need, ((M + 95) / 96) * (((size_t)L.cout + 63) / 64));
    }
  return need;
}

void grow_counters(Workspace& w, size_t need, hipStream_t st) {
  if (need <= w.cnt_ints) return;
  w.cnt = std::make_shared<DevBuf>(need * sizeof(int));
  hip_check(hipMemsetAsync(w.cnt->p, 0, need * sizeof(int), st), "hipMemsetAsync");
  w.cnt_ints = need;
}

bool capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return false;
  return cs != hipStreamCaptureStatusNone;
}

Workspace& workspace(const PpsModel& m, int N, hipStream_t st, bool allow_alloc) {
  auto it = m.ws.find(N);
  if (it != m.ws.end()) {
    Workspace& w = it->second;
    const size_t need = part_need(m, w.shapes);
    const std::string pinned_msg =
        "the buffers of batch " + std::to_string(N) +
        " are pinned by pps_model_reserve (a captured graph may hold them) and the tuning "
        "table now needs larger split-K ";
    if (need > w.part_floats) {
      PPS_MCHECK(!w.pinned, pinned_msg + "partials: pps_model_release, reserve again, recapture");
      PPS_MCHECK(allow_alloc && !capturing(st),
                 "split-K partials grew after pps_model_reserve: reserve again outside capture");
      w.part = std::make_shared<DevBuf>(need * sizeof(float));
      w.part_floats = need;
    }
    const size_t hneed = h2p_need(m, w.shapes);
    if (hneed > w.h2p_elems) {
      PPS_MCHECK(!w.pinned, "the buffers of batch " + std::to_string(N) +
                                " are pinned by pps_model_reserve and the tuning table now needs "
                                "larger f16x2 activation planes: pps_model_release, reserve "
                                "again, recapture");
      PPS_MCHECK(allow_alloc && !capturing(st),
                 "f16x2 activation planes grew after pps_model_reserve: reserve again outside "
                 "capture");
      w.h2p = std::make_shared<DevBuf>(hneed * 2 * sizeof(uint16_t));
      w.h2p_elems = hneed;
    }
    const size_t cneed = cnt_need(m, w.shapes);
    if (cneed > w.cnt_ints) {
      PPS_MCHECK(!w.pinned, pinned_msg + "counters: pps_model_release, reserve again, recapture");
      PPS_MCHECK(allow_alloc && !capturing(st),
                 "split-K counters grew after pps_model_reserve: reserve again outside capture");
      grow_counters(w, cneed, st);
    }
    return w;
  }
  PPS_MCHECK(allow_alloc && !capturing(st),
             "no workspace for batch " + std::to_string(N) +
                 ": call pps_model_reserve before capturing pps_forward");
  Workspace w;
  w.N = N;
  w.shapes = infer_shapes(m, N);
  bool need_conv_out = false;
  for (const auto& L : m.layers)
    if (L.op == Op::ConvPps && pps_tiles(m, L, w.shapes.at(L.conv_output)).empty())
      need_conv_out = true;
  for (const auto& kv : w.shapes) {
    if (kv.first == "data") continue;
    bool fused_away = false;
    for (const auto& L : m.layers)
      if (L.op == Op::ConvPps && L.conv_output == kv.first && !need_conv_out) fused_away = true;
    if (fused_away) continue;
    const size_t esz = m.plane_capable.count(kv.first) ? 6 : 4;
    w.bufs[kv.first] = std::make_shared<DevBuf>((size_t)kv.second.numel() * esz);
  }
  w.part_floats = part_need(m, w.shapes);
  if (w.part_floats) w.part = std::make_shared<DevBuf>(w.part_floats * sizeof(float));
  w.h2p_elems = h2p_need(m, w.shapes);
  if (w.h2p_elems) w.h2p = std::make_shared<DevBuf>(w.h2p_elems * 2 * sizeof(uint16_t));
  grow_counters(w, cnt_need(m, w.shapes), st);
  w.amax = std::make_shared<DevBuf>(m.slot.size() * PPS_AMAX_SLOT_FLOATS * sizeof(float));
  hip_check(hipMemsetAsync(w.amax->p, 0, w.amax->bytes, st), "hipMemsetAsync");
  return m.ws.emplace(N, std::move(w)).first->second;
}

float* nhwc4_buffer(const PpsModel& m, Workspace& w, hipStream_t st) {
  if (!w.nhwc4) {
    PPS_MCHECK(!capturing(st), "input staging buffer: call pps_model_reserve before capture");
    w.nhwc4 = std::make_shared<DevBuf>((size_t)w.N * m.cfg.height * m.cfg.width * 4 * sizeof(float));
  }
  return w.nhwc4->as<float>();
}

// ---- one layer ----------------------------------------------------------------
const float* fbuf_of(const Workspace& w, const std::string& name) {
  return w.bufs.at(name)->as<float>();
}

struct Act {  // an activation operand: f32 NHWC or bf16x3 planes
  const float* f = nullptr;
  const uint16_t* pl = nullptr;
  int64_t plane = 0;
  Shape s;
};

bool getenv_flag_on(const char* name) {
  const char* v = std::getenv(name);
  return v && v[0] && std::strcmp(v, "0") != 0;
}

void run_layer(const PpsModel& m, const Layer& L, Workspace& w, const float* x, float* feat,
               bool last, int tile, int sk, hipStream_t st) {
  auto act = [&](const std::string& name, bool planes) {
    Act a;
    a.s = w.shapes.at(name);
    if (name == "data") { a.f = x; return a; }
    void* p = w.bufs.at(name)->p;
    if (planes) { a.pl = static_cast<const uint16_t*>(p); a.plane = a.s.numel(); }
    else a.f = static_cast<const float*>(p);
    return a;
  };
  auto fbuf = [&](const std::string& name) { return w.bufs.at(name)->as<float>(); };
  // activation-max slot of a tensor an f16x2 layer reads (its producer
  // reports max |y| there), else null
  auto slotp = [&](const std::string& t) -> float* {
    auto it = m.slot.find(t);
    return it == m.slot.end() || it->second >= (int)w.amax_need.size() || !w.amax_need[it->second]
               ? nullptr
               : w.amax->as<float>() + (size_t)it->second * PPS_AMAX_SLOT_FLOATS;
  };
  // PPS_TILE_H2: the f16x2 arithmetic on the base tile (weights always the
  // chunk-tiled f16x2 split; COL_ORDER kept)
  const bool h2 = (tile & PPS_TILE_H2) != 0;
  const bool h2p = h2 && (tile & PPS_TILE_H2P) != 0;
  const bool h2e = h2 && (tile & PPS_TILE_H2E) != 0;
  if (h2) {
    PPS_MCHECK(L.w2 && !L.planes_in && !L.planes_out && sk == 1,
               "layer '" + L.name + "': PPS_TILE_H2 needs the f16x2 weights, f32 activations "
               "at both ends and no split-K");
    tile &= ~(PPS_TILE_H2 | PPS_TILE_H2P | PPS_TILE_H2E | PPS_TILE_B_TILED | PPS_TILE_SEAM);
  }
  // PPS_TILE_H2E on the layer that reads this one's output: write it as
  // f16x2 planes on the output bound's scale (the bound into the slot)
  const Layer* h2e_c = nullptr;
  if (L.op == Op::Conv && L.h2o_bw > 0.f)
    for (const Layer& C : m.layers)
      if (C.input == L.output && (C.tile & PPS_TILE_H2E) && (C.tile & PPS_TILE_H2)) h2e_c = &C;
  if (h2e_c) {
    PPS_MCHECK(h2e_producer(m, *h2e_c) == (int)(&L - &m.layers[0]) && !L.planes_in &&
                   !L.planes_out && sk == 1 && !(tile & PPS_TILE_SEAM),
               "layer '" + h2e_c->name + "': PPS_TILE_H2E needs its producer '" + L.name +
                   "' to be a conv + BN + ReLU read by it alone, f32 input, no split-K");
    tile &= ~(PPS_TILE_B_TILED | PPS_TILE_SEAM);
  }
  // PPS_TILE_H2E: this layer's input, as f16x2 planes its producer wrote
  auto h2e_input = [&](const Act& a, int64_t* plane) -> const uint16_t* {
    *plane = a.s.numel();
    return w.bufs.at(L.input)->as<uint16_t>();
  };
  // PPS_TILE_H2P: the input's f16x2 planes, split once (same bits)
  auto h2_planes = [&](const Act& a, int64_t* plane) -> const uint16_t* {
    if (h2e) return h2e_input(a, plane);
    const int64_t n = a.s.numel();
    PPS_MCHECK(w.h2p && (size_t)n <= w.h2p_elems, "layer '" + L.name +
                                                     "': no f16x2 activation-plane workspace");
    uint16_t* pl = w.h2p->as<uint16_t>();
    rc_check(split_act_h2(a.f, n, slotp(L.input), pl, n, st));
    *plane = n;
    return pl;
  };
  // split convs run in one launch on the FIX tiles (same bits as the
  // two-pass split-K), else raw partials + the summing pass (plain weights)
  const bool fused_sk = sk > 1 && L.op == Op::Conv && fix_tile(tile) && L.relu &&
                        !(L.planes_out && !L.residual.empty());
  if (sk > 1 && !fused_sk) tile &= ~PPS_TILE_B_TILED;
  // PPS_TILE_B_TILED in the tile: the chunk-tiled weight copy (plain convs)
  const bool wtiled = tile > 0 && (tile & PPS_TILE_B_TILED) && L.wt;
  if (L.op == Op::Heads) tile &= ~PPS_TILE_COL_ORDER;
  if (!wtiled) tile &= ~PPS_TILE_B_TILED;
  const uint16_t* w3 = m.x3 && L.w ? (wtiled ? L.wt->as<uint16_t>() : L.w->as<uint16_t>()) : nullptr;
  const float* wf = !m.x3 && L.w ? L.w->as<float>() : nullptr;
  const float* sc = L.scale ? L.scale->as<float>() : nullptr;
  const float* sh = L.shift ? L.shift->as<float>() : nullptr;
  const int N = w.N;
  if (L.op == Op::Conv && (tile & PPS_TILE_SEAM)) {
    PPS_MCHECK(seam_ok(m, L), "layer '" + L.name + "': PPS_TILE_SEAM needs f32 activations "
                              "at both ends and no split-K");
    const Layer& X = m.layers[L.seam_next];
    const Act a = act(L.input, false);
    const int64_t M = a.s.d[0] * a.s.d[1] * a.s.d[2];
    // pps_conv1x1_seam_x3 with the two outputs' maxima reported
    SeamParams sp{a.f, fbuf(L.residual), L.w->as<uint16_t>(), sc, sh, fbuf(L.output),
                  X.w->as<uint16_t>(), X.scale->as<float>(), X.shift->as<float>(),
                  fbuf(X.output), (int)M};
    sp.amax_t = slotp(L.output);
    sp.amax_y = slotp(X.output);
    rc_check(launch_seam_x3(sp, L.cin_eff, L.cout, X.cout, st));
    return;
  }
  switch (L.op) {
    case Op::Conv: {
      const Act a = act(L.input, L.planes_in);
      const Shape ys = w.shapes.at(L.output);
      const float* res = L.residual.empty() ? nullptr : fbuf(L.residual);
      const int n = (int)a.s.d[0], H = (int)a.s.d[1], W = (int)a.s.d[2], ldx = (int)a.s.d[3];
      const int Ho = (int)ys.d[1], Wo = (int)ys.d[2];
      // the op-level entry points' implementation (same arguments as
      // pps_conv2d_bn_act_x3p[_splitk[_fused]] / _x3 / _h2), reporting max |y|
      float* amo = slotp(L.output);
      // f16x2 planes out (the consumer's PPS_TILE_H2E): the output buffer
      // holds the two planes, the bound goes to the output's slot
      uint16_t* yh2 = h2e_c ? w.bufs.at(L.output)->as<uint16_t>() : nullptr;
      const int64_t yh2_plane = ys.numel();
      if (h2e_c)
        PPS_MCHECK(amo && slotp(L.input), "layer '" + L.name + "': f16x2 planes out needs the "
                                          "input's and the output's activation slots");
      if (h2) {
        int64_t xpl = 0;
        const uint16_t* xp = (h2p || h2e) ? h2_planes(a, &xpl) : nullptr;
        rc_check(conv_impl(xp ? nullptr : a.f, n, H, W, L.cin_eff, ldx, L.w2->as<uint16_t>(), 1,
                           L.cout, L.kpad, L.k, L.k, L.stride, L.pad, L.dil, sc, sh, res, L.relu,
                           yh2 ? nullptr : fbuf(L.output), Ho, Wo, L.cout, tile, st, xp, xpl,
                           nullptr, 0, 1, nullptr, nullptr, 0, amo, L.wrs->as<float>(),
                           slotp(L.input), yh2, yh2_plane, slotp(L.input), L.h2o_bw, L.h2o_bb));
      } else if (yh2) {   // bf16x3 arithmetic, f16x2 planes out
        rc_check(conv_impl(a.f, n, H, W, L.cin_eff, ldx, w3, 1, L.cout, L.kpad, L.k, L.k,
                           L.stride, L.pad, L.dil, sc, sh, res, L.relu, nullptr, Ho, Wo, L.cout,
                           tile, st, nullptr, 0, nullptr, 0, 1, nullptr, nullptr, 0, amo, nullptr,
                           nullptr, yh2, yh2_plane, slotp(L.input), L.h2o_bw, L.h2o_bb));
      } else if (m.x3 && (L.planes_in || L.planes_out || sk > 1)) {
        const int t = tile >= GEMM_TILE_P_FIRST ? tile : 0;
        float* yf = L.planes_out ? nullptr : fbuf(L.output);
        uint16_t* y3 = L.planes_out ? w.bufs.at(L.output)->as<uint16_t>() : nullptr;
        const int64_t ypl = L.planes_out ? ys.numel() : 0;
        if (fused_sk)
          rc_check(conv_impl(a.f, n, H, W, L.cin_eff, ldx, w3, 1, L.cout, L.kpad, L.k, L.k,
                             L.stride, L.pad, L.dil, sc, sh, res, L.relu, yf, Ho, Wo, L.cout, t,
                             st, a.pl, a.plane, y3, ypl, sk, w.part->as<float>(),
                             w.cnt->as<int>(), (int64_t)w.cnt_ints, amo, nullptr, nullptr));
        else
          rc_check(conv_impl(a.f, n, H, W, L.cin_eff, ldx, w3, 1, L.cout, L.kpad, L.k, L.k,
                             L.stride, L.pad, L.dil, sc, sh, res, L.relu, yf, Ho, Wo, L.cout, t,
                             st, a.pl, a.plane, y3, ypl, sk, sk > 1 ? w.part->as<float>() : nullptr,
                             nullptr, 0, amo, nullptr, nullptr));
      } else if (m.x3) {
        rc_check(conv_impl(a.f, n, H, W, L.cin_eff, ldx, w3, 1, L.cout, L.kpad, L.k, L.k,
                           L.stride, L.pad, L.dil, sc, sh, res, L.relu, fbuf(L.output), Ho, Wo,
                           L.cout, tile, st, nullptr, 0, nullptr, 0, 1, nullptr, nullptr, 0, amo,
                           nullptr, nullptr));
      } else {
        rc_check(pps_conv2d_bn_act(a.f, n, H, W, L.cin_eff, ldx, wf, L.cout, L.kpad, L.k, L.k,
                                   L.stride, L.pad, L.dil, sc, sh, res, L.relu, fbuf(L.output),
                                   Ho, Wo, L.cout, tile, st));
      }
      return;
    }
    case Op::ConvDual: {
      const Act a = act(L.input, false), b = act(L.input2, false);
      const Shape ys = w.shapes.at(L.output);
      const int C2 = (int)b.s.d[3];
      if (m.x3)
        rc_check(dual_impl(a.f, (int)a.s.d[0], (int)a.s.d[1], (int)a.s.d[2], L.cin_eff,
                           (int)a.s.d[3], L.k, L.k, L.stride, L.pad, b.f, (int)b.s.d[1],
                           (int)b.s.d[2], C2, C2, L.stride2,
                           h2 ? L.w2->as<uint16_t>() : w3, 1, L.cout, L.kpad, C2, sh, L.relu,
                           fbuf(L.output), (int)ys.d[1], (int)ys.d[2], L.cout, tile, st,
                           slotp(L.output), h2 ? L.wrs->as<float>() : nullptr,
                           h2 ? slotp(L.input) : nullptr, h2 ? slotp(L.input2) : nullptr));
      else
        rc_check(pps_conv2d_dual_bn_act(a.f, (int)a.s.d[0], (int)a.s.d[1], (int)a.s.d[2],
                                        L.cin_eff, (int)a.s.d[3], L.k, L.k, L.stride, L.pad, b.f,
                                        (int)b.s.d[1], (int)b.s.d[2], C2, C2, L.stride2, wf,
                                        L.cout, L.kpad, C2, sh, L.relu, fbuf(L.output),
                                        (int)ys.d[1], (int)ys.d[2], L.cout, tile, st));
      return;
    }
    case Op::MaxPool: {
      const Act a = act(L.input, false);
      const Shape ys = w.shapes.at(L.output);
      PPS_MCHECK(a.s.d[3] % 4 == 0, "max pooling needs C % 4 == 0");
      rc_check(maxpool2d(a.f, (int)a.s.d[0], (int)a.s.d[1], (int)a.s.d[2], (int)a.s.d[3], L.k,
                         L.stride, L.pad, fbuf(L.output), (int)ys.d[1], (int)ys.d[2], st,
                         slotp(L.output)));
      return;
    }
    case Op::StemPool: {
      const Act a = act(L.input, false);
      const Shape ys = w.shapes.at(L.output);
      // pps_stem_conv_pool_x3 (shapes checked when the stem was fused), max |y| reported
      const int Hin = (int)a.s.d[1];
      if (h2) {  // pps_stem_conv_pool_h2: the input's max from its slot
        PPS_MCHECK(slotp(L.input), "layer '" + L.name + "': the f16x2 stem needs its input's "
                                   "activation-max slot");
        rc_check(stem_conv_pool_h2(a.f, (int)a.s.d[0], Hin, L.w2->as<uint16_t>(),
                                   L.wrs->as<float>(), sc, sh, fbuf(L.output),
                                   (Hin + 2 * 3 - 7) / 2 + 1, (int)ys.d[1], st, slotp(L.output),
                                   slotp(L.input)));
        return;
      }
      rc_check(stem_conv_pool_x3(a.f, (int)a.s.d[0], Hin, w3, sc, sh, fbuf(L.output),
                                 (Hin + 2 * 3 - 7) / 2 + 1, (int)ys.d[1], st, slotp(L.output)));
      return;
    }
    case Op::Pps: {
      const Act a = act(L.input, false);
      rc_check(pps_part_power_set(a.f, (int)a.s.d[0], (int)a.s.d[1], (int)a.s.d[2],
                                  (int)a.s.d[3], L.split.data(), (int)L.split.size(), L.max_ave,
                                  fbuf(L.output), st));
      return;
    }
    case Op::ConvPps: {
      const Act a = act(L.input, L.planes_in);
      const Shape cs = w.shapes.at(L.conv_output);
      const float* res = fbuf(L.residual);
      const std::vector<int> ok = pps_tiles(m, L, cs);
      const int n = (int)a.s.d[0], H = (int)a.s.d[1], W = (int)a.s.d[2], ldx = (int)a.s.d[3];
      if (h2) {  // f16x2: the 192-row tiles on 16x16x32 blocks
        std::vector<int> ok16;
        for (int t : ok)
          if (t >= GEMM_TILE_P16_FIRST) ok16.push_back(t);
        PPS_MCHECK(!ok16.empty(), "layer '" + L.name + "': no f16x2 tile holds one image");
        const int tb = tile & ~PPS_TILE_COL_ORDER;
        int t = std::find(ok16.begin(), ok16.end(), tb) != ok16.end() ? tb : ok16[0];
        t |= tile & PPS_TILE_COL_ORDER;
        int64_t xpl = 0;
        const uint16_t* xp = (h2p || h2e) ? h2_planes(a, &xpl) : nullptr;
        rc_check(conv_pps_impl(xp ? nullptr : a.f, xp, xpl, n, H, W, L.cin_eff, ldx,
                               L.w2->as<uint16_t>(),
                               L.cout, L.kpad, L.k, L.k, L.stride, L.pad, L.dil, sc, sh, res,
                               nullptr, (int)cs.d[1], (int)cs.d[2], L.split.data(),
                               (int)L.split.size(), L.max_ave, fbuf(L.output), t, st,
                               L.wrs->as<float>(), slotp(L.input)));
      } else if (!ok.empty()) {
        const int tb = tile & ~(PPS_TILE_B_TILED | PPS_TILE_COL_ORDER);
        int t = std::find(ok.begin(), ok.end(), tb) != ok.end() ? tb : ok[0];
        t |= tile & PPS_TILE_COL_ORDER;
        if (wtiled) t |= PPS_TILE_B_TILED;
        rc_check(pps_conv2d_bn_act_pps_x3p(a.f, a.pl, a.plane, n, H, W, L.cin_eff, ldx, w3,
                                           L.cout, L.kpad, L.k, L.k, L.stride, L.pad, L.dil, sc,
                                           sh, res, nullptr, (int)cs.d[1], (int)cs.d[2],
                                           L.split.data(), (int)L.split.size(), L.max_ave,
                                           fbuf(L.output), t, st));
      } else {  // no tile holds exactly one image: conv, then the pooling kernel
        float* y = fbuf(L.conv_output);
        rc_check(pps_conv2d_bn_act_x3p(a.f, a.pl, a.plane, n, H, W, L.cin_eff, ldx, w3, L.cout,
                                       L.kpad, L.k, L.k, L.stride, L.pad, L.dil, sc, sh, res, 1,
                                       y, nullptr, 0, (int)cs.d[1], (int)cs.d[2], L.cout,
                                       tile >= GEMM_TILE_P_FIRST ? tile | (wtiled ? PPS_TILE_B_TILED : 0) : 0, st));
        rc_check(pps_part_power_set(y, n, (int)cs.d[1], (int)cs.d[2], L.cout, L.split.data(),
                                    (int)L.split.size(), L.max_ave, fbuf(L.output), st));
      }
      return;
    }
    case Op::Heads: {
      float* part = fbuf(L.output + "_partials");
      const float* xin = fbuf(L.input);
      if (m.x3)
        rc_check(pps_gemm_splitk_batched_x3(xin, N, L.dim, w3, L.dim_inner, L.nsub, kHeadSplitK,
                                            part, tile, st));
      else
        rc_check(pps_gemm_splitk_batched(xin, N, L.dim, wf, L.dim_inner, L.nsub, kHeadSplitK,
                                         part, tile, st));
      float* y = last ? feat : fbuf(L.output);
      rc_check(pps_splitk_bn_act_normalize(part, kHeadSplitK, N, L.nsub * L.dim_inner, sc, sh, 1,
                                           L.normalize ? 1 : 0, y, st));
      return;
    }
    case Op::Normalize: {
      const Act a = act(L.input, false);
      rc_check(pps_l2_normalize(a.f, a.s.d[0], (int)a.s.d[1], last ? feat : fbuf(L.output), st));
      return;
    }
  }
}

// pre (whole forwards only): writes x before the layers run -- the
// preprocessing of pps_forward_bgr -- and reports max|x| into the slot it is
// given (null when no f16x2 layer reads the input)
void forward_range(const PpsModel& m, const float* x, int N, float* feat, int first, int last,
                   hipStream_t st, bool keep_amax = false,
                   const std::function<void(float*)>* pre = nullptr) {
  Workspace& w = workspace(m, N, st, true);
  // the tensors whose maxima this forward needs
  const bool all = m.amax_all || getenv_flag_on("PPS_AMAX_ALL");
  w.amax_need.assign(m.slot.size(), all ? 1 : 0);
  if (!all)
    for (const Layer& L : m.layers)
      if (L.tile & PPS_TILE_H2) {
        for (const std::string* t : {&L.input, &L.input2})
          if (!t->empty() && m.slot.count(*t)) w.amax_need[m.slot.at(*t)] = 1;
        // PPS_TILE_H2E: the producer's bound reads its own input's max
        const int pi = (L.tile & PPS_TILE_H2E) ? h2e_producer(m, L) : -1;
        if (pi >= 0 && m.slot.count(m.layers[pi].input))
          w.amax_need[m.slot.at(m.layers[pi].input)] = 1;
      }
  if (first == 0 && !keep_amax) {
    // a forward: every producer reports its output's max afresh, and the
    // input's max is measured when an f16x2 layer (the stem) reads it
    hip_check(hipMemsetAsync(w.amax->p, 0, w.amax->bytes, st), "hipMemsetAsync");
    const auto ds = m.slot.find("data");
    float* dslot = ds != m.slot.end() && ds->second < (int)w.amax_need.size() &&
                           w.amax_need[ds->second]
                       ? w.amax->as<float>() + (size_t)ds->second * PPS_AMAX_SLOT_FLOATS
                       : nullptr;
    if (pre) (*pre)(dslot);  // the producer of x reports its max
    else if (dslot) rc_check(amax_of(x, w.shapes.at("data").numel(), dslot, st));
  } else if (!keep_amax) {
    // a layer range: the f32 tensors it reads but does not produce are
    // measured afresh (their producers ran in an earlier call)
    std::set<std::string> made, done;
    for (int i = first; i < last; ++i) {
      const Layer& L = m.layers[i];
      for (const std::string* t : {&L.input, &L.input2}) {
        if (t->empty() || made.count(*t) || done.count(*t) || !m.slot.count(*t) ||
            !w.amax_need[m.slot.at(*t)])
          continue;
        bool planes = false;
        for (const auto& P : m.layers)
          if (P.output == *t && P.planes_out) planes = true;
        // an f16x2-planes edge (PPS_TILE_H2E): its slot keeps the producer's bound
        if (L.input == *t && (L.tile & PPS_TILE_H2E) && (L.tile & PPS_TILE_H2)) planes = true;
        const float* src = *t == "data" ? x : (w.bufs.count(*t) ? fbuf_of(w, *t) : nullptr);
        if (planes || !src) continue;
        float* slot = w.amax->as<float>() + (size_t)m.slot.at(*t) * PPS_AMAX_SLOT_FLOATS;
        hip_check(hipMemsetAsync(slot, 0, PPS_AMAX_SLOT_FLOATS * sizeof(float), st),
                  "hipMemsetAsync");
        rc_check(amax_of(src, w.shapes.at(*t).numel(), slot, st));
        done.insert(*t);
      }
      made.insert(L.output);
      if (!L.conv_output.empty()) made.insert(L.conv_output);
      if (L.seam_next >= 0 && (L.tile & PPS_TILE_SEAM)) made.insert(m.layers[L.seam_next].output);
    }
    // and the tensors it produces start from zero, as in a whole forward:
    // their producers combine into the slot with atomicMax, so a larger max
    // left by an earlier call would otherwise set a stale scale
    for (const std::string& t : made) {
      if (!m.slot.count(t)) continue;
      float* slot = w.amax->as<float>() + (size_t)m.slot.at(t) * PPS_AMAX_SLOT_FLOATS;
      hip_check(hipMemsetAsync(slot, 0, PPS_AMAX_SLOT_FLOATS * sizeof(float), st),
                "hipMemsetAsync");
    }
  }
  for (int i = first; i < last; ++i) {
    const Layer& L = m.layers[i];
    // computed by the previous layer's seam launch (when that ran here too)
    if (i > first && (m.layers[i - 1].tile & PPS_TILE_SEAM) && m.layers[i - 1].seam_next == i)
      continue;
    run_layer(m, L, w, x, feat, i + 1 == (int)m.layers.size(), L.tile & ~(i + 1 == last ? PPS_TILE_SEAM : 0),
              L.splitk, st);
  }
}

bool tunable(const Layer& L) {
  return L.op == Op::Conv || L.op == Op::ConvDual || L.op == Op::Heads || L.op == Op::ConvPps;
}

double layer_flops(const PpsModel& m, const Layer& L, const std::map<std::string, Shape>& s, int N) {
  switch (L.op) {
    case Op::StemPool: {
      const Shape& x = s.at(L.input);
      const double hc = (double)((x.d[1] - 1) / 2 + 1), wc = (double)((x.d[2] - 1) / 2 + 1);
      return 2.0 * N * hc * wc * L.cout * L.k * L.k * L.cin;  // true Cin = 3
    }
    case Op::Conv: case Op::ConvDual: case Op::ConvPps: {
      const Shape& y = s.at(L.op == Op::ConvPps ? L.conv_output : L.output);
      return 2.0 * y.d[0] * y.d[1] * y.d[2] * y.d[3] * ((double)L.k * L.k * L.cin + L.shortcut_cin);
    }
    case Op::Heads:
      return 2.0 * N * L.nsub * L.dim_inner * L.dim;
    default:
      return 0.0;
  }
  (void)m;
}

// algorithmic HBM bytes per launch: every operand read once, the output
// written once (model.py PPSModel._alloc)
double layer_bytes(const PpsModel& m, const Layer& L, const std::map<std::string, Shape>& s, int N) {
  const double wb = m.x3 && !(L.tile & PPS_TILE_H2) ? 6.0 : 4.0;  // f16x2 weights: 4 B
  switch (L.op) {
    case Op::StemPool:
      return 4.0 * s.at(L.input).numel() + 4.0 * s.at(L.output).numel() +
             wb * L.cout * pps_stem_k();
    case Op::Conv: case Op::ConvDual: {
      const Shape& y = s.at(L.output);
      const double pix = (double)y.d[0] * y.d[1] * y.d[2];
      // a 1x1 (k < stride) conv reads only the pixels under its taps: one
      // input pixel per output position and tap, not the whole tensor
      const double in = L.k < L.stride ? 4.0 * pix * L.k * L.k * L.cin
                                       : 4.0 * s.at(L.input).numel();
      double b = in + 4.0 * y.numel() + wb * L.cout * ((double)L.k * L.k * L.cin + L.shortcut_cin);
      if (!L.residual.empty()) b += 4.0 * y.numel();
      if (L.op == Op::ConvDual)  // the 1x1 shortcut, stride2
        b += L.stride2 > 1 ? 4.0 * pix * L.shortcut_cin : 4.0 * s.at(L.input2).numel();
      return b;
    }
    case Op::ConvPps: {
      const Shape& y = s.at(L.conv_output);
      return 4.0 * s.at(L.input).numel() + 4.0 * y.numel() +
             wb * L.cout * (double)L.k * L.k * L.cin + 4.0 * s.at(L.output).numel();
    }
    case Op::Heads:
      return 4.0 * s.at(L.input).numel() + wb * L.nsub * L.dim_inner * L.dim +
             4.0 * kHeadSplitK * N * L.nsub * L.dim_inner;
    default:
      return 0.0;
  }
}

// ---- autotune (the reference's cudnn_exhaustive_search analogue,
// modeling/detector.py:58; same procedure as PPSModel.autotune) --------------
struct Timer {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  Timer() {
    hip_check(hipEventCreate(&e0), "hipEventCreate");
    hip_check(hipEventCreate(&e1), "hipEventCreate");
  }
  ~Timer() {
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
};

float time_forward(const PpsModel& m, const float* x, int N, float* feat, int reps,
                   hipStream_t st, Timer& t) {
  forward_range(m, x, N, feat, 0, (int)m.layers.size(), st);
  hip_check(hipEventRecord(t.e0, st), "hipEventRecord");
  for (int i = 0; i < reps; ++i) forward_range(m, x, N, feat, 0, (int)m.layers.size(), st);
  hip_check(hipEventRecord(t.e1, st), "hipEventRecord");
  hip_check(hipEventSynchronize(t.e1), "hipEventSynchronize");
  float ms = 0.f;
  hip_check(hipEventElapsedTime(&ms, t.e0, t.e1), "hipEventElapsedTime");
  return ms / reps;
}

// The in-forward pass of pps_model_autotune over layers of one shape: the
// members' three best distinct tiles (their own f16x2-plane flags kept), each
// applied to the whole group, and the group's planes edges all on (each
// reader on its best planes variant, h2e_best) or all off (pre_h2e), timed
// as whole forwards in interleaved rounds; the group moves to the best
// assignment if it beats the current one by > 0.5 %.  A layer of its own
// shape tries its three best variants as they are.  Seam pairs keep their
// launch.
void group_pass(PpsModel& m, Workspace& w, const float* x, int N,
                const std::map<const Layer*, std::vector<std::pair<float, int>>>& ranked,
                const std::map<const Layer*, int>& pre_h2e,
                const std::map<const Layer*, int>& h2e_best, hipStream_t st, Timer& t) {
  constexpr int kKeep = PPS_TILE_H2E | PPS_TILE_H2P;
  std::map<std::string, std::vector<int>> groups;
  for (size_t i = 0; i < m.layers.size(); ++i) {
    const Layer& L = m.layers[i];
    if (!ranked.count(&L) || (L.tile & PPS_TILE_SEAM) || L.op == Op::Heads) continue;
    if (i > 0 && (m.layers[i - 1].tile & PPS_TILE_SEAM) && m.layers[i - 1].seam_next == (int)i)
      continue;
    const Shape& s = w.shapes.at(L.input);
    std::string key = std::to_string((int)L.op);
    for (int v : {L.cin_eff, L.cout, L.kpad, L.k, L.stride, L.pad, L.dil, L.shortcut_cin,
                  (int)L.relu, (int)L.residual.empty(), (int)L.planes_in, (int)L.planes_out,
                  L.splitk})
      key += "," + std::to_string(v);
    for (int d = 0; d < 4; ++d) key += "," + std::to_string(s.d[d]);
    groups[key].push_back((int)i);
  }
  DevBuf feat((size_t)N * m.plan.feat_dim * sizeof(float));
  constexpr int reps = 6, rounds = 3;
  for (const auto& g : groups) {
    const std::vector<int>& mem = g.second;
    const bool single = mem.size() == 1;
    std::vector<int> save;
    for (int i : mem) save.push_back(m.layers[i].tile);
    // candidate assignments (one tile per member); [0] = the current one
    std::vector<std::vector<int>> cands{save};
    auto add = [&](const std::vector<int>& a) {
      if (std::find(cands.begin(), cands.end(), a) == cands.end()) cands.push_back(a);
    };
    std::vector<int> bases;
    for (int i : mem) {
      int taken = 0;
      for (const auto& r : ranked.at(&m.layers[i])) {
        const int c = single ? r.second : r.second & ~kKeep;
        if (std::find(bases.begin(), bases.end(), c) == bases.end()) bases.push_back(c);
        if (++taken == 3) break;
      }
    }
    for (int c : bases) {   // one tile for the whole group (members' plane flags kept)
      std::vector<int> a(mem.size());
      for (size_t j = 0; j < mem.size(); ++j) {
        const Layer& L = m.layers[mem[j]];
        int tl = single ? c : c | ((c & PPS_TILE_H2) ? (save[j] & kKeep) : 0);
        if ((tl & PPS_TILE_H2P) && !h2_tile_ok(L, tl)) tl &= ~PPS_TILE_H2P;
        if ((tl & PPS_TILE_H2E) && !h2_tile_ok(L, tl)) tl &= ~PPS_TILE_H2E;
        a[j] = tl;
      }
      add(a);
    }
    // the f16x2-planes edges into the group: every reader on its best planes
    // variant, and every reader back on its pick without them
    std::vector<int> on = save, off = save;
    for (size_t j = 0; j < mem.size(); ++j) {
      const Layer* L = &m.layers[mem[j]];
      if (h2e_best.count(L)) on[j] = h2e_best.at(L);
      if (pre_h2e.count(L) && (save[j] & PPS_TILE_H2E)) off[j] = pre_h2e.at(L);
    }
    add(on);
    add(off);
    if (cands.size() < 2) continue;
    auto apply = [&](const std::vector<int>& a) {
      for (size_t j = 0; j < mem.size(); ++j) m.layers[mem[j]].tile = a[j];
    };
    std::vector<float> tmin(cands.size(), 1e30f);
    for (int r = 0; r < rounds; ++r)
      for (size_t v = 0; v < cands.size(); ++v) {
        apply(cands[v]);
        tmin[v] = std::min(tmin[v], time_forward(m, x, N, feat.as<float>(), reps, st, t));
      }
    size_t best = 0;
    for (size_t v = 1; v < cands.size(); ++v)
      if (tmin[v] < tmin[best]) best = v;
    apply(best > 0 && tmin[best] < 0.995f * tmin[0] ? cands[best] : save);
  }
}

// The bottleneck seams judged inside whole forwards too: each seam-capable
// branch2c with its launch toggled (on: the seam tile; off: its best tile of
// its own, ranked), kept if the forward gets > 0.5 % faster.  The seam pass
// before it judged the pair's two isolated launches.
void seam_forward_pass(PpsModel& m, Workspace& w, const float* x, int N,
                       const std::map<const Layer*, std::vector<std::pair<float, int>>>& ranked,
                       hipStream_t st, Timer& t) {
  DevBuf feat((size_t)N * m.plan.feat_dim * sizeof(float));
  constexpr int reps = 6, rounds = 3;
  for (Layer& L : m.layers) {
    if (!seam_ok(m, L) || !ranked.count(&L)) continue;
    const int save = L.tile;
    int alt = GEMM_TILE_WS | PPS_TILE_SEAM;
    if (save & PPS_TILE_SEAM) {   // off: the layer's best variant of its own
      alt = -1;
      for (const auto& r : ranked.at(&L))
        if (!(r.second & PPS_TILE_SEAM)) { alt = r.second; break; }
      if (alt < 0) continue;
    }
    float t0 = 1e30f, t1 = 1e30f;
    for (int r = 0; r < rounds; ++r) {
      L.tile = save;
      t0 = std::min(t0, time_forward(m, x, N, feat.as<float>(), reps, st, t));
      L.tile = alt;
      t1 = std::min(t1, time_forward(m, x, N, feat.as<float>(), reps, st, t));
    }
    L.tile = t1 < 0.995f * t0 ? alt : save;
  }
}

float time_layer(const PpsModel& m, const Layer& L, Workspace& w, const float* x, int tile,
                 int sk, int reps, hipStream_t st, Timer& t) {
  for (int i = 0; i < 2; ++i) run_layer(m, L, w, x, nullptr, false, tile, sk, st);
  hip_check(hipEventRecord(t.e0, st), "hipEventRecord");
  for (int i = 0; i < reps; ++i) run_layer(m, L, w, x, nullptr, false, tile, sk, st);
  hip_check(hipEventRecord(t.e1, st), "hipEventRecord");
  hip_check(hipEventSynchronize(t.e1), "hipEventSynchronize");
  float ms = 0.f;
  hip_check(hipEventElapsedTime(&ms, t.e0, t.e1), "hipEventElapsedTime");
  return ms / reps;
}

}  // namespace
}  // namespace pps

using namespace pps;

namespace {
template <class F> int guarded(F&& f) {
  try {
    f();
    return PPS_OK;
  } catch (const ModelError& e) {
    set_error(e.what());
    return e.code;
  } catch (const std::exception& e) {
    set_error(std::string("pps model: ") + e.what());
    return PPS_ERR_INVALID_ARG;
  }
}

Layer* find_layer(PpsModel* m, const char* name) {
  PPS_MCHECK(m && name, "null argument");
  for (auto& L : m->layers)
    if (L.name == name) return &L;
  throw ModelError(PPS_ERR_INVALID_ARG, std::string("no layer named '") + name + "'");
}

__global__ void nchw_to_nhwc4_kernel(const float* __restrict__ x, int64_t npix_img, int64_t total,
                                     float4* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = i / npix_img, p = i - n * npix_img;
    const float* src = x + n * 3 * npix_img + p;
    y[i] = make_float4(src[0], src[npix_img], src[2 * npix_img], 0.f);
  }
}
}  // namespace

extern "C" {

int pps_model_config_default(PpsModelConfig* c) {
  if (!c) return PPS_ERR_INVALID_ARG;
  std::memset(c, 0, sizeof(*c));
  c->struct_size = (int)sizeof(PpsModelConfig);
  // configs/market1501/pps_crm_triplet_R-50_1x.yaml (the reference's PPS
  // Market-1501 test configuration)
  c->height = 384; c->width = 128;
  c->strip_num = 5; c->bpm_dim = 128;
  c->num_groups = 1; c->width_per_group = 64; c->stride_1x1 = 1;
  c->res5_stride = 1; c->res5_dilation = 1;
  c->fpn_on = 0; c->fpn_dim = 256;
  c->max_ave = 1; c->normalize = 1;
  c->math = PPS_MATH_X3;
  c->fused_stem = 1; c->fused_pps = 1; c->act_planes = 1;
  c->pixel_means[0] = 102.9801f; c->pixel_means[1] = 115.9465f; c->pixel_means[2] = 122.7717f;
  return PPS_OK;
}

int pps_model_create(const PpsBlob* blobs, int nblobs, const PpsModelConfig* cfg,
                     PpsModel** out) {
  return guarded([&] {
    PPS_MCHECK(out && cfg && (blobs || nblobs == 0) && nblobs >= 0, "null argument");
    PPS_MCHECK(cfg->struct_size == (int)sizeof(PpsModelConfig),
               "PpsModelConfig.struct_size mismatch (use pps_model_config_default)");
    *out = nullptr;
    const PpsModelConfig& c = *cfg;
    PPS_MCHECK(c.height > 0 && c.width > 0 && c.strip_num >= 1 && c.strip_num <= 10 &&
                   c.bpm_dim > 0 && c.num_groups > 0 && c.width_per_group > 0 &&
                   c.res5_stride >= 1 && c.res5_dilation >= 1 && c.fpn_dim > 0,
               "bad config");
    PPS_MCHECK(c.math == PPS_MATH_X3 || c.math == PPS_MATH_F32, "math must be PPS_MATH_X3 or _F32");
    auto m = std::make_unique<PpsModel>();
    m->cfg = c;
    m->plan = build_plan(c);
    m->x3 = c.math == PPS_MATH_X3;
    m->fused_stem = m->x3 && c.fused_stem && c.width == 128;  // the fused stem's kernel is W = 128
    m->fused_pps = m->x3 && c.fused_pps;
    m->act_planes = m->x3 && c.act_planes;
    std::map<std::string, Blob> bmap;
    for (int i = 0; i < nblobs; ++i) {
      const PpsBlob& b = blobs[i];
      PPS_MCHECK(b.name && (b.data || b.ndim == 0) && b.ndim >= 0 && b.ndim <= 4, "bad blob entry");
      Blob B{b.data, std::vector<int64_t>(b.shape, b.shape + b.ndim)};
      bmap[b.name] = B;
    }
    std::vector<std::string> missing;
    for (const auto& kv : m->plan.params) {
      auto it = bmap.find(kv.first);
      const bool optional = kv.first.size() > 7 &&
                            kv.first.compare(kv.first.size() - 7, 7, "_conv_b") == 0;
      if (it == bmap.end()) {
        if (!optional) missing.push_back(kv.first);
        continue;
      }
      int64_t want = 1;
      for (auto s : kv.second) want *= s;
      PPS_MCHECK(it->second.numel() == want,
                 "blob " + kv.first + " has " + std::to_string(it->second.numel()) +
                     " elements, the net needs " + std::to_string(want));
      it->second.shape = kv.second;
    }
    PPS_MCHECK(missing.empty(), "weights missing " + std::to_string(missing.size()) +
                                    " blobs, e.g. " + (missing.empty() ? "" : missing[0]));
    hipStream_t st = nullptr;
    hip_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
    try {
      compile(*m, bmap, st);
    } catch (...) {
      (void)hipStreamDestroy(st);
      throw;
    }
    hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
    (void)hipStreamDestroy(st);
    for (size_t i = 0; i < m->layers.size(); ++i)
      if (seam_pair(*m, i)) m->layers[i].seam_next = (int)i + 1;
    *out = m.release();
  });
}

int pps_model_destroy(PpsModel* m) {
  return guarded([&] {
    if (!m) return;
    (void)hipDeviceSynchronize();  // no launch of this model may still read its buffers
    delete m;
  });
}

int pps_model_feat_dim(const PpsModel* m) { return m ? m->plan.feat_dim : -1; }
int pps_model_num_layers(const PpsModel* m) { return m ? (int)m->layers.size() : -1; }

int pps_model_layer_info(const PpsModel* m, int i, int N, PpsLayerInfo* info) {
  return guarded([&] {
    PPS_MCHECK(m && info, "null argument");
    PPS_MCHECK(i >= 0 && i < (int)m->layers.size(), "layer index out of range");
    PPS_MCHECK(N > 0, "N must be positive");
    const Layer& L = m->layers[i];
    const auto shapes = infer_shapes(*m, N);
    std::memset(info, 0, sizeof(*info));
    info->name = L.name.c_str();
    info->op = op_name(L.op);
    info->tile = L.tile;
    info->splitk = L.splitk;
    info->planes_in = L.planes_in;
    info->planes_out = L.planes_out;
    info->gemm = tunable(L) || L.op == Op::StemPool;
    info->flops = layer_flops(*m, L, shapes, N);
    info->bytes = layer_bytes(*m, L, shapes, N);
    const Shape& y = shapes.at(L.op == Op::ConvPps ? L.output : L.output);
    for (int d = 0; d < 4; ++d) info->out_shape[d] = y.d[d];
    info->output = L.output.c_str();
  });
}

int pps_model_set_tile(PpsModel* m, const char* layer, int tile) {
  return guarded([&] {
    Layer* L = find_layer(m, layer);
    // the fused stem takes 0 (bf16x3) or PPS_TILE_H2 (f16x2) only
    if (L->op == Op::StemPool) {
      PPS_MCHECK(tile == 0 || (tile == PPS_TILE_H2 && h2_tile_ok(*L, tile)),
                 std::string("stem '") + layer + "': tile 0 or PPS_TILE_H2 (f16x2) only");
      L->tile = tile;
      return;
    }
    PPS_MCHECK(tunable(*L), std::string("layer '") + layer + "' has no GEMM tile");
    const int base = tile & ~(PPS_TILE_B_TILED | PPS_TILE_COL_ORDER | PPS_TILE_SEAM | PPS_TILE_H2 |
                              PPS_TILE_H2P | PPS_TILE_H2E);
    PPS_MCHECK(tile >= 0 && base < GEMM_NUM_TILES, "tile out of range");
    PPS_MCHECK(!(tile & PPS_TILE_H2) || h2_tile_ok(*L, tile),
               std::string("PPS_TILE_H2: '") + layer +
                   "' has no f16x2 weights (Cin % 32 == 0) or the base tile is not 0, 38..53, "
                   "55, 60 or (convs) 56..59; PPS_TILE_H2P: plain convs and conv_pps only");
    PPS_MCHECK(!(tile & PPS_TILE_H2P) || (tile & PPS_TILE_H2),
               "PPS_TILE_H2P goes with PPS_TILE_H2");
    PPS_MCHECK(!(tile & PPS_TILE_H2E) || ((tile & PPS_TILE_H2) && h2e_producer(*m, *L) >= 0),
               std::string("PPS_TILE_H2E: '") + layer + "' needs PPS_TILE_H2 and a producer "
               "that is a conv + BN + ReLU read by it alone (Cin % 32 == 0)");
    PPS_MCHECK(!(tile & PPS_TILE_SEAM) ||
                   (L->seam_next >= 0 && base == GEMM_TILE_WS &&
                    !(tile & (PPS_TILE_B_TILED | PPS_TILE_COL_ORDER))),
               std::string("PPS_TILE_SEAM: '") + layer +
                   "' is not a branch2c feeding a seam-capable branch2a (base tile 54)");
    PPS_MCHECK(!(tile & PPS_TILE_B_TILED) ||
                   (L->wt && base >= GEMM_TILE_P_FIRST && base != GEMM_TILE_WS),
               "PPS_TILE_B_TILED: x3 conv with Cin % 32 == 0 on a pipelined tile only");
    PPS_MCHECK(!(tile & PPS_TILE_COL_ORDER) ||
                   (L->op != Op::Heads && base >= GEMM_TILE_P_FIRST && base != GEMM_TILE_WS),
               "PPS_TILE_COL_ORDER: conv layers on a pipelined tile only");
    L->tile = tile;
  });
}

int pps_model_set_splitk(PpsModel* m, const char* layer, int splitk) {
  return guarded([&] {
    Layer* L = find_layer(m, layer);
    PPS_MCHECK(L->op == Op::Conv, std::string("split-K applies to plain convs, not '") + layer + "'");
    PPS_MCHECK(splitk == 1 || !(L->tile & PPS_TILE_H2),
               std::string("'") + layer + "' runs an f16x2 tile: no split-K");
    PPS_MCHECK(splitk >= 1 && splitk <= kMaxSplitK, "splitk must be in [1, 4]");
    PPS_MCHECK(splitk == 1 || (m->x3 && L->cin_eff % 32 == 0 && L->kpad == L->k * L->k * L->cin_eff &&
                               L->kpad % (32 * splitk) == 0),
               "split-K " + std::to_string(splitk) + " not possible for " + layer);
    L->splitk = splitk;
  });
}

int pps_model_num_plane_edges(const PpsModel* m) { return m ? (int)m->edges.size() : -1; }

int pps_model_plane_edge(const PpsModel* m, int i, const char** producer, const char** consumer,
                         int* on) {
  return guarded([&] {
    PPS_MCHECK(m && producer && consumer && on, "null argument");
    PPS_MCHECK(i >= 0 && i < (int)m->edges.size(), "edge index out of range");
    const Layer& P = m->layers[m->edges[i].first];
    *producer = P.name.c_str();
    *consumer = m->layers[m->edges[i].second].name.c_str();
    *on = P.planes_out;
  });
}

int pps_model_set_planes(PpsModel* m, const char* producer, int on) {
  return guarded([&] {
    PPS_MCHECK(m && producer, "null argument");
    for (auto& e : m->edges)
      if (m->layers[e.first].name == producer) {
        PPS_MCHECK(!on || !((m->layers[e.first].tile | m->layers[e.second].tile) & PPS_TILE_H2),
                   std::string("plane edge '") + producer + "': an f16x2 (PPS_TILE_H2) layer "
                   "takes and writes f32 activations");
        m->layers[e.first].planes_out = m->layers[e.second].planes_in = on != 0;
        return;
      }
    throw ModelError(PPS_ERR_INVALID_ARG,
                     std::string("not a plane-eligible producer: '") + producer + "'");
  });
}

int pps_model_reserve(PpsModel* m, int N) {
  return guarded([&] {
    PPS_MCHECK(m && N > 0, "bad arguments");
    Workspace& w = workspace(*m, N, nullptr, true);
    nhwc4_buffer(*m, w, nullptr);
    w.pinned = true;
  });
}

int pps_model_release(PpsModel* m, int N) {
  return guarded([&] {
    PPS_MCHECK(m, "null argument");
    (void)hipDeviceSynchronize();
    if (N > 0) m->ws.erase(N);
    else m->ws.clear();
  });
}

int pps_model_tensor(const PpsModel* m, int N, const char* blob, void** ptr, int* planes,
                     int64_t* shape4) {
  return guarded([&] {
    PPS_MCHECK(m && blob && ptr && planes && shape4, "null argument");
    auto it = m->ws.find(N);
    PPS_MCHECK(it != m->ws.end(), "no workspace for this batch size (pps_model_reserve)");
    auto b = it->second.bufs.find(blob);
    PPS_MCHECK(b != it->second.bufs.end(), std::string("no device tensor '") + blob + "'");
    *ptr = b->second->p;
    *planes = 0;
    for (const auto& L : m->layers) {
      if (L.output == blob && L.planes_out) *planes = 1;
      // read by a PPS_TILE_H2E layer: f16x2 planes on the slot's scale
      if (L.input == blob && (L.tile & PPS_TILE_H2E) && (L.tile & PPS_TILE_H2) &&
          h2e_producer(*m, L) >= 0)
        *planes = 2;
    }
    const Shape& s = it->second.shapes.at(blob);
    for (int d = 0; d < 4; ++d) shape4[d] = s.d[d];
  });
}

int pps_model_tensor_amax(const PpsModel* m, int N, const char* blob, float* out) {
  return guarded([&] {
    PPS_MCHECK(m && blob && out, "null argument");
    auto it = m->ws.find(N);
    PPS_MCHECK(it != m->ws.end(), "no workspace for this batch size (pps_model_reserve)");
    auto s = m->slot.find(blob);
    PPS_MCHECK(s != m->slot.end(), std::string("no activation-max slot for '") + blob + "'");
    float h[PPS_AMAX_SLOT_FLOATS];
    hip_check(hipMemcpy(h, it->second.amax->as<float>() + (size_t)s->second * PPS_AMAX_SLOT_FLOATS,
                        sizeof(h), hipMemcpyDeviceToHost),
              "hipMemcpy");
    float mx = 0.f;
    for (int j = 0; j < kAmaxSubs; ++j) mx = std::max(mx, h[j * kAmaxStride]);
    *out = mx;
  });
}

int pps_forward_layers_flags(const PpsModel* m, const float* x, int N, float* feat, int first,
                             int last, int flags, void* stream) {
  return guarded([&] {
    PPS_MCHECK(m && x && feat, "null pointer");
    PPS_MCHECK(N > 0, "N must be positive");
    PPS_MCHECK(0 <= first && first <= last && last <= (int)m->layers.size(), "bad layer range");
    PPS_MCHECK(aligned16(x) && aligned16(feat), "x / feat must be 16-byte aligned");
    PPS_MCHECK((flags & ~PPS_FWD_KEEP_AMAX) == 0, "unknown pps_forward_layers flags");
    forward_range(*m, x, N, feat, first, last, as_stream(stream), (flags & PPS_FWD_KEEP_AMAX) != 0);
  });
}

int pps_forward_layers(const PpsModel* m, const float* x, int N, float* feat, int first,
                       int last, void* stream) {
  return pps_forward_layers_flags(m, x, N, feat, first, last, 0, stream);
}

int pps_forward(const PpsModel* m, const float* nhwc4, int N, float* feat, void* stream) {
  return pps_forward_layers(m, nhwc4, N, feat, 0, m ? (int)m->layers.size() : 0, stream);
}

int pps_forward_nchw(const PpsModel* m, const float* nchw, int N, float* feat, void* stream) {
  return guarded([&] {
    PPS_MCHECK(m && nchw && feat, "null pointer");
    PPS_MCHECK(N > 0, "N must be positive");
    const hipStream_t st = as_stream(stream);
    Workspace& w = workspace(*m, N, st, true);
    float* x = nhwc4_buffer(*m, w, st);
    const int64_t npix = (int64_t)m->cfg.height * m->cfg.width, total = npix * N;
    const int64_t blocks = std::min<int64_t>((total + 255) / 256, 65535);
    hipLaunchKernelGGL(nchw_to_nhwc4_kernel, dim3((unsigned)blocks), dim3(256), 0, st, nchw, npix,
                       total, reinterpret_cast<float4*>(x));
    hip_check(hipGetLastError(), "nchw_to_nhwc4_kernel");
    forward_range(*m, x, N, feat, 0, (int)m->layers.size(), st);
  });
}

int pps_forward_bgr(const PpsModel* m, const uint8_t* img, int N, int Hi, int Wi, float* feat,
                    void* stream) {
  return guarded([&] {
    PPS_MCHECK(m && img && feat, "null pointer");
    PPS_MCHECK(N > 0, "N must be positive");
    const hipStream_t st = as_stream(stream);
    Workspace& w = workspace(*m, N, st, true);
    float* x = nhwc4_buffer(*m, w, st);
    PPS_MCHECK(Hi > 0 && Wi > 0, "bad image shape");
    // preprocessing inside the forward, after the maxima slots are zeroed:
    // it reports max|x| for an f16x2 stem (no separate pass over x)
    const std::function<void(float*)> pre = [&](float* slot) {
      rc_check(preprocess_bgr(img, N, Hi, Wi, nullptr, nullptr, nullptr, m->cfg.pixel_means,
                              m->cfg.height, m->cfg.width, x, st, slot));
    };
    forward_range(*m, x, N, feat, 0, (int)m->layers.size(), st, false, &pre);
  });
}

int pps_model_autotune(PpsModel* m, const float* x, int N, int flags, void* stream) {
  return guarded([&] {
    PPS_MCHECK(m && x, "null pointer");
    PPS_MCHECK(N > 0, "N must be positive");
    const hipStream_t st = as_stream(stream);
    PPS_MCHECK(!capturing(st), "autotune cannot run inside a graph capture");
#ifndef PPS_TUNE_FINALISTS
#define PPS_TUNE_FINALISTS 4  // probes: more screened tiles into the interleaved final rounds
#endif
    const int reps = 3, finalists = PPS_TUNE_FINALISTS, final_reps = 10, final_rounds = 3;
    Workspace* w = &workspace(*m, N, st, true);
    // every candidate may be an f16x2 tile: all producers report maxima
    struct AmaxAll {
      const PpsModel* m;
      ~AmaxAll() { m->amax_all = false; }
    } amax_guard{m};
    m->amax_all = true;
    std::vector<float> scratch((size_t)N * m->plan.feat_dim);
    DevBuf feat(scratch.size() * sizeof(float));
    forward_range(*m, x, N, feat.as<float>(), 0, (int)m->layers.size(), st);
    hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
    Timer t;
    // f16x2 candidates (PPS_TILE_H2) beside the bf16x3 tiles of a layer with
    // f32 activations at both ends and no split-K
    const bool try_h2 = m->x3 && !(flags & PPS_AUTOTUNE_NO_H2);
    if (try_h2) {   // planes workspace for the PPS_TILE_H2P candidates
      size_t hneed = 0;
      for (const Layer& L : m->layers)
        if (L.w2 && (L.op == Op::Conv || L.op == Op::ConvPps))
          hneed = std::max(hneed, (size_t)w->shapes.at(L.input).numel());
      if (hneed > w->h2p_elems) {
        PPS_MCHECK(!w->pinned, "autotune: the batch's buffers are pinned (pps_model_reserve); "
                               "release them first");
        w->h2p = std::make_shared<DevBuf>(hneed * 2 * sizeof(uint16_t));
        w->h2p_elems = hneed;
      }
    }
    auto cands_of = [&](const Layer& L) {
      std::vector<int> c;
      const bool h2ok = try_h2 && L.w2 && !L.planes_in && !L.planes_out && L.splitk == 1;
      if (L.op == Op::ConvPps) {
        c = pps_tiles(*m, L, w->shapes.at(L.conv_output));
        if (h2ok) {
          const size_t n = c.size();
          for (size_t i = 0; i < n; ++i)
            if (c[i] >= GEMM_TILE_P16_FIRST) c.push_back(c[i] | PPS_TILE_H2);
        }
      } else {
        const bool pipelined_only = L.planes_in || L.planes_out;
        for (int tl = pipelined_only ? GEMM_TILE_P_FIRST : 1; tl < GEMM_NUM_TILES; ++tl)
          if (tl != GEMM_TILE_P16_192x128W41) c.push_back(tl);   // (f16x2 only)
        // (PPS_AUTOTUNE_NO_WSH2=1, A/B runs: no f16x2 weight-stationary tile)
        static const bool no_wsh2 = getenv_flag_on("PPS_AUTOTUNE_NO_WSH2");
        if (h2ok)
          for (int tl = GEMM_TILE_P16_FIRST; tl < GEMM_NUM_TILES; ++tl)
            if (h2_tile_ok(L, tl | PPS_TILE_H2) && !(no_wsh2 && tl == GEMM_TILE_WS) &&
                !(tl >= GEMM_TILE_C16_FIRST && tl != GEMM_TILE_P16_192x128W41 &&
                  (L.k != 3 || L.stride != 1)))
              c.push_back(tl | PPS_TILE_H2);
      }
      if (c.empty()) c.push_back(0);
      return c;
    };
    // every tuned layer's finalists, best first, and an f16x2-planes reader's
    // pick before the planes (the in-forward group pass)
    std::map<const Layer*, std::vector<std::pair<float, int>>> ranked;
    std::map<const Layer*, int> pre_h2e, h2e_best;   // (h2e_best: kept or not)
    // extra: flags or-ed into every candidate (PPS_TILE_H2E: the f16x2 tiles
    // only, reading the planes the producer wrote)
    auto tune = [&](Layer& L, int extra = 0) {
      std::vector<std::pair<float, int>> screen;
      for (int tl : cands_of(L)) {
        if (extra && !((tl & PPS_TILE_H2) && h2_tile_ok(L, tl | extra))) continue;
        tl |= extra;
        screen.emplace_back(time_layer(*m, L, *w, x, tl, L.splitk, reps, st, t), tl);
      }
      std::sort(screen.begin(), screen.end());
      // finalists, each also on the chunk-tiled weight copy and / or in
      // column-major tile order; timed in interleaved rounds (min per
      // variant), so a drifting clock does not favour whichever ran first
      std::vector<int> var;
      for (int i = 0; i < (int)screen.size() && i < finalists; ++i) {
        const int tl = screen[i].second;
        var.push_back(tl);
        // f16x2 finalists also with the input split once into planes
        if ((tl & PPS_TILE_H2) && h2_tile_ok(L, tl | PPS_TILE_H2P)) var.push_back(tl | PPS_TILE_H2P);
        // (base tile: the flags of an f16x2 candidate are or-ed in already;
        // the weight-stationary kernel has no tile order to choose)
        const int tb = tl & 0xff;
        if (L.splitk == 1 && L.op != Op::Heads && tb >= GEMM_TILE_P_FIRST && tb != GEMM_TILE_WS)
          for (int f : {PPS_TILE_B_TILED, PPS_TILE_COL_ORDER,
                        PPS_TILE_B_TILED | PPS_TILE_COL_ORDER})
            if (!(f & PPS_TILE_B_TILED) || (L.wt && !(tl & PPS_TILE_H2))) var.push_back(tl | f);
      }
      std::vector<float> tmin(var.size(), 1e30f);
      for (int r = 0; r < final_rounds; ++r)
        for (size_t v = 0; v < var.size(); ++v)
          tmin[v] = std::min(tmin[v], time_layer(*m, L, *w, x, var[v], L.splitk, final_reps, st, t));
      float best = 1e30f;
      auto& rk = ranked[&L];
      rk.clear();
      for (size_t v = 0; v < var.size(); ++v) {
        rk.emplace_back(tmin[v], var[v]);
        if (tmin[v] < best) { best = tmin[v]; L.tile = var[v]; }
      }
      std::sort(rk.begin(), rk.end());
      return best;
    };
    const bool tune_planes = (flags & PPS_AUTOTUNE_NO_PLANES) == 0 && m->act_planes;
    if (tune_planes)
      for (auto& e : m->edges) m->layers[e.first].planes_out = m->layers[e.second].planes_in = false;
    std::vector<float> cost(m->layers.size(), 0.f);
    for (size_t i = 0; i < m->layers.size(); ++i)
      if (tunable(m->layers[i])) cost[i] = tune(m->layers[i]);
    // the fused stem: f16x2 (plus the pass that measures the input's max, run
    // by every forward that takes it) against bf16x3, interleaved rounds
    for (Layer& L : m->layers)
      if (L.op == Op::StemPool) L.tile = 0;
    if (try_h2)
      for (Layer& L : m->layers) {
        if (L.op != Op::StemPool || !h2_tile_ok(L, PPS_TILE_H2) || !m->slot.count("data")) continue;
        float* ds = w->amax->as<float>() + (size_t)m->slot.at("data") * PPS_AMAX_SLOT_FLOATS;
        const int64_t n = w->shapes.at("data").numel();
        float tx = 1e30f, th = 1e30f, ta = 1e30f;
        for (int r = 0; r < final_rounds; ++r) {
          tx = std::min(tx, time_layer(*m, L, *w, x, 0, 1, final_reps, st, t));
          th = std::min(th, time_layer(*m, L, *w, x, PPS_TILE_H2, 1, final_reps, st, t));
          hip_check(hipEventRecord(t.e0, st), "hipEventRecord");
          for (int i = 0; i < final_reps; ++i) rc_check(amax_of(x, n, ds, st));  // same max again
          hip_check(hipEventRecord(t.e1, st), "hipEventRecord");
          hip_check(hipEventSynchronize(t.e1), "hipEventSynchronize");
          float ms = 0.f;
          hip_check(hipEventElapsedTime(&ms, t.e0, t.e1), "hipEventElapsedTime");
          ta = std::min(ta, ms / final_reps);
        }
        L.tile = th + ta < 0.98f * tx ? PPS_TILE_H2 : 0;
      }
    if (tune_planes) {
      for (auto& e : m->edges) {
        Layer& P = m->layers[e.first];
        Layer& C = m->layers[e.second];
        const float before = cost[e.first] + cost[e.second];
        const int tp = P.tile, tc = C.tile;
        P.planes_out = C.planes_in = true;
        const float cp = tune(P), cc = tune(C);
        if (cp + cc < 0.98f * before) {
          cost[e.first] = cp; cost[e.second] = cc;
        } else {
          P.planes_out = C.planes_in = false;
          P.tile = tp; C.tile = tc;
        }
      }
    }
    if (m->x3 && (flags & PPS_AUTOTUNE_SPLITK)) {
      for (size_t i = 0; i < m->layers.size(); ++i) {
        Layer& L = m->layers[i];
        if (L.op != Op::Conv || L.cin_eff % 32 || L.kpad != L.k * L.k * L.cin_eff) continue;
        std::vector<std::pair<float, std::pair<int, int>>> screen;
        for (int sk = 2; sk <= kMaxSplitK; ++sk) {
          if (L.kpad % (32 * sk)) continue;
          const int save = L.splitk;
          L.splitk = sk;
          w = &workspace(*m, N, st, true);  // grow the partials buffer
          L.splitk = save;
          // the one-launch split-K tiles, on plain and chunk-tiled weights
          for (int tl = GEMM_TILE_P16_FIRST + 7; tl <= GEMM_TILE_P16_96x128W24; ++tl) {
            if (!fix_tile(tl)) continue;
            for (int f : {0, PPS_TILE_B_TILED})
              if (!f || L.wt)
                screen.push_back({time_layer(*m, L, *w, x, tl | f, sk, reps, st, t), {tl | f, sk}});
          }
        }
        if (screen.empty()) continue;
        std::sort(screen.begin(), screen.end());
        float best = 1e30f;
        std::pair<int, int> pick{0, 1};
        for (int j = 0; j < (int)screen.size() && j < finalists; ++j) {
          const auto o = screen[j].second;
          const float ms = time_layer(*m, L, *w, x, o.first, o.second, final_reps, st, t);
          if (ms < best) { best = ms; pick = o; }
        }
        if (best < 0.98f * cost[i]) {
          L.tile = pick.first; L.splitk = pick.second; cost[i] = best;
        }
      }
    }
    if (!(flags & PPS_AUTOTUNE_NO_SEAM)) {
      // bottleneck seams: branch2c + the next branch2a in one launch, kept
      // if > 2 % faster than the two tuned launches
      for (size_t i = 0; i < m->layers.size(); ++i) {
        Layer& L = m->layers[i];
        if (!seam_ok(*m, L)) continue;
        const int save = L.tile;
        float ts = 1e30f;
        for (int r = 0; r < final_rounds; ++r)
          ts = std::min(ts, time_layer(*m, L, *w, x, GEMM_TILE_WS | PPS_TILE_SEAM, 1, final_reps,
                                       st, t));
        const float sep = cost[i] + cost[L.seam_next];
        if (ts < 0.98f * sep) {
          L.tile = GEMM_TILE_WS | PPS_TILE_SEAM;
          cost[i] = ts;
          cost[L.seam_next] = 0.f;
        } else {
          L.tile = save;
        }
      }
    }
    if (try_h2 && !(flags & PPS_AUTOTUNE_NO_H2E)) {
      // f16x2 planes from the producer's epilogue (PPS_TILE_H2E): the
      // consumer re-tuned over the f16x2 tiles reading them (the planes
      // input favours other tiles than f32 does), kept if the producer +
      // consumer pair is > 2 % faster
      for (size_t ci = 0; ci < m->layers.size(); ++ci) {
        Layer& C = m->layers[ci];
        // (a seam launch keeps its pair: its cost also holds the next layer's)
        if (!C.w2 || C.planes_in || C.planes_out || C.splitk != 1 || (C.tile & PPS_TILE_SEAM))
          continue;
        const int pi = h2e_producer(*m, C);
        if (pi < 0) continue;
        Layer& P = m->layers[pi];
        if (P.planes_in || P.planes_out || P.splitk != 1 || (P.tile & PPS_TILE_SEAM)) continue;
        int first = -1;   // an f16x2 tile of C, so P writes the planes from here on
        for (int tl : cands_of(C))
          if ((tl & PPS_TILE_H2) && h2_tile_ok(C, tl | PPS_TILE_H2E)) { first = tl; break; }
        if (first < 0) continue;
        const int save = C.tile;
        const auto save_rank = ranked[&C];
        C.tile = first | PPS_TILE_H2E;
        run_layer(*m, P, *w, x, nullptr, false, P.tile, 1, st);
        const float tc = tune(C, PPS_TILE_H2E);
        h2e_best[&C] = C.tile;
        float tp = 1e30f;
        for (int r = 0; r < final_rounds; ++r)
          tp = std::min(tp, time_layer(*m, P, *w, x, P.tile, 1, final_reps, st, t));
        if (tp + tc < 0.98f * (cost[pi] + cost[ci])) {
          cost[pi] = tp;
          cost[ci] = tc;
          pre_h2e[&C] = save;
        } else {
          C.tile = save;
          ranked[&C] = save_rank;
          run_layer(*m, P, *w, x, nullptr, false, P.tile, 1, st);   // f32 output again
        }
      }
    }
    if (!(flags & PPS_AUTOTUNE_NO_GROUPS)) {
      group_pass(*m, *w, x, N, ranked, pre_h2e, h2e_best, st, t);
      if (!(flags & PPS_AUTOTUNE_NO_SEAM)) seam_forward_pass(*m, *w, x, N, ranked, st, t);
    }
    hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
  });
}

}  // extern "C"
