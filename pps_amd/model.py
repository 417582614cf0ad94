"""PPS feature extractor on MI355X: ResNet-50 (stride-1 res5) + part power set
+ 31 reid heads, executed as hand-written HIP kernels through libpps_hip.so.

The layer plan is produced by builders that mirror the reference graph
builders one for one, with the same blob and parameter names:

  add_ResNet50_conv5_body   detectron/modeling/ResNet.py:39-40,91-126
    basic_bn_stem           ResNet.py:246-256
    add_stage               ResNet.py:60-88
    add_residual_block      ResNet.py:153-195 (stride rule :169-171)
    bottleneck_transformation ResNet.py:276-333 (STRIDE_1X1 :290)
    basic_bn_shortcut       ResNet.py:203-220
  add_pps_part_head         detectron/modeling/pps_heads.py:38-96
    add_uniform_partition   detectron/modeling/bpm_heads.py:18-55
  add_reid_outputs          detectron/modeling/reid_heads.py:34-127

Differences by design: NHWC activations; test-mode
SpatialBN folded into the conv epilogue as per-channel scale/shift; residual
Sum and ReLU fused into branch2c's epilogue; the 31 head convs run as one
batched GEMM; the unused FC logits (reid_heads.py:84-90) are not computed;
batch N instead of the reference's batch-1 Reshape([1,-1]).
"""
import os

import numpy as np
import torch

from . import ops
from .config import cfg

BN_EPS = 1e-5  # Caffe2 SpatialBN default epsilon (pytorch v1.0.1)
HEAD_SPLITK = 8  # K=2048 head GEMMs split 8 ways: 31 x 8 x 2 workgroups at batch 64


# ---------------------------------------------------------------------------
# Plan builders (structure only; no device work)
# ---------------------------------------------------------------------------
class Plan(object):
    def __init__(self):
        self.layers = []       # dicts, executed in order
        self.params = {}       # name -> shape (Detectron naming)

    def conv(self, blob_in, prefix, dim_in, dim_out, k, stride, pad, dilation=1,
             relu=False, residual=None, out=None, bias=False, bn=None):
        self.params[prefix + '_w'] = (dim_out, dim_in, k, k)
        if bias:
            self.params[prefix + '_b'] = (dim_out,)
        bn = bn or prefix + '_bn'
        for s in ('_s', '_b', '_rm', '_riv'):
            self.params[bn + s] = (dim_out,)
        out = out or bn
        self.layers.append(dict(op='conv', name=prefix, bn=bn, input=blob_in,
                                output=out, cin=dim_in, cout=dim_out, k=k,
                                stride=stride, pad=pad, dil=dilation, relu=relu,
                                residual=residual))
        return out


def basic_bn_stem(plan, data):
    """ResNet.py:246-256: conv1 7x7/2 -> res_conv1_bn -> Relu -> pool1."""
    p = plan.conv(data, 'conv1', 3, 64, 7, 2, 3, relu=True, bn='res_conv1_bn')
    plan.layers.append(dict(op='maxpool', input=p, output='pool1', k=3, stride=2,
                            pad=1))
    return 'pool1', 64


def bottleneck_transformation(plan, blob_in, dim_in, dim_out, stride, prefix,
                              dim_inner, dilation=1, shortcut=None, out=None):
    """ResNet.py:276-333 (+ the Sum/Relu of add_residual_block :186-195)."""
    str1x1, str3x3 = (stride, 1) if cfg.RESNETS.STRIDE_1X1 else (1, stride)
    cur = plan.conv(blob_in, prefix + '_branch2a', dim_in, dim_inner, 1, str1x1,
                    0, relu=True)
    cur = plan.conv(cur, prefix + '_branch2b', dim_inner, dim_inner, 3, str3x3,
                    dilation, dilation=dilation, relu=True)
    cur = plan.conv(cur, prefix + '_branch2c', dim_inner, dim_out, 1, 1, 0,
                    relu=True, residual=shortcut, out=out)
    return cur


def basic_bn_shortcut(plan, prefix, blob_in, dim_in, dim_out, stride):
    """ResNet.py:203-220."""
    if dim_in == dim_out:
        return blob_in
    return plan.conv(blob_in, prefix + '_branch1', dim_in, dim_out, 1, stride, 0)


def add_residual_block(plan, prefix, blob_in, dim_in, dim_out, dim_inner,
                       dilation, stride_init=2, inplace_sum=False):
    """ResNet.py:153-195."""
    stride = stride_init if (dim_in != dim_out and dim_in != 64 and
                             dilation == 1) else 1
    sc = basic_bn_shortcut(plan, prefix, blob_in, dim_in, dim_out, stride)
    # :190-193 -- in-place Sum into branch2c_bn except for a stage's last block
    out = prefix + ('_branch2c_bn' if inplace_sum else '_sum')
    return bottleneck_transformation(plan, blob_in, dim_in, dim_out, stride,
                                     prefix, dim_inner, dilation, shortcut=sc,
                                     out=out)


def add_stage(plan, prefix, blob_in, n, dim_in, dim_out, dim_inner, dilation,
              stride_init=2):
    """ResNet.py:60-88."""
    for i in range(n):
        blob_in = add_residual_block(plan, '{}_{}'.format(prefix, i), blob_in,
                                     dim_in, dim_out, dim_inner, dilation,
                                     stride_init, inplace_sum=i < n - 1)
        dim_in = dim_out
    return blob_in, dim_in


def add_ResNet50_conv5_body(plan):
    """ResNet.py:39-40 -> add_ResNet_convX_body :91-126."""
    p, dim_in = basic_bn_stem(plan, 'data')
    dim_b = cfg.RESNETS.NUM_GROUPS * cfg.RESNETS.WIDTH_PER_GROUP
    s, dim_in = add_stage(plan, 'res2', p, 3, dim_in, 256, dim_b, 1)
    s, dim_in = add_stage(plan, 'res3', s, 4, dim_in, 512, dim_b * 2, 1)
    s, dim_in = add_stage(plan, 'res4', s, 6, dim_in, 1024, dim_b * 4, 1)
    s, dim_in = add_stage(plan, 'res5', s, 3, dim_in, 2048, dim_b * 8,
                          cfg.RESNETS.RES5_DILATION,
                          stride_init=cfg.RESNETS.RES5_STRIDE)
    return s, dim_in, 1. / 16. * cfg.RESNETS.RES5_DILATION / cfg.RESNETS.RES5_STRIDE


def uniform_partition_split(spatial_scale):
    """bpm_heads.py:18-35: strip heights along H."""
    strip_num = cfg.REID.BPM_STRIP_NUM
    table = {7: [3, 3, 4, 4, 4, 3, 3], 5: [5, 5, 4, 5, 5],
             9: [2, 3, 3, 3, 3, 3, 3, 2, 2], 10: [2, 2, 2, 3, 3, 3, 3, 2, 2, 2]}
    if strip_num in table and cfg.REID.SCALE[1] == 16 * 24:
        scale = 16 * spatial_scale
        return [int(s * scale) for s in table[strip_num]]
    strip_h = int(cfg.REID.SCALE[1] * spatial_scale / strip_num)
    return [strip_h] * strip_num


def subset_prefixes(strip_num, preprefix='pps'):
    """pps_heads.py:47-64: subset i = bits of i; blob prefix pps + digits."""
    out = []
    for i in range(1, 1 << strip_num):
        comb = [j for j in range(strip_num) if i & (1 << j)]
        out.append(preprefix + ''.join(str(c) for c in comb))
    return out


def add_pps_part_head(plan, blob_in, dim_in, spatial_scale, preprefix='pps'):
    """pps_heads.py:38-96 (+ bpm_heads.add_uniform_partition)."""
    split = uniform_partition_split(spatial_scale)
    prefixes = subset_prefixes(cfg.REID.BPM_STRIP_NUM, preprefix)
    plan.layers.append(dict(op='pps', input=blob_in, output=preprefix + '_pool2_all',
                            split=split, max_ave=bool(cfg.REID.MAX_AVE_FEATURE),
                            prefixes=prefixes, dim=dim_in))
    return prefixes, dim_in


def add_reid_outputs(plan, prefixes, dim, preprefix='reid'):
    """reid_heads.py:34-127 (test branch; FC logits skipped, never fetched)."""
    dim_inner = cfg.REID.BPM_DIM
    for p in prefixes:
        plan.params[p + '_conv_w'] = (dim_inner, dim, 1, 1)
        plan.params[p + '_conv_b'] = (dim_inner,)
        for s in ('_s', '_b', '_rm', '_riv'):
            plan.params[p + '_bn' + s] = (dim_inner,)
    out = preprefix + '_feature_concat'
    plan.layers.append(dict(op='heads', input=plan.layers[-1]['output'],
                            prefixes=prefixes, dim=dim, dim_inner=dim_inner,
                            output=out))
    if cfg.REID.NORMALIZE_FEATURE:
        plan.layers.append(dict(op='normalize', input=out,
                                output=preprefix + '_feature_concat_norm'))
        out = preprefix + '_feature_concat_norm'
    return out


def add_fpn_coarsest_level(plan, blob, dim):
    """FPN_reid.py:117-174 add_fpn, restricted to what the test net consumes:
    with FPN_ON the PPS head reads only blob_in[0] (pps_heads.py:88-96), the
    coarsest level = Conv 1x1 (bias) -> SpatialBN -> Relu on res5_2_sum
    ('fpn_inner_res5_2_sum_bn').  The reference also computes the top-down /
    lateral levels at test, whose outputs are never read;
    they are not built here.  No P6 level: max FPN level = 5 unless
    MULTILEVEL_RPN/ROIS (FPN_reid.py:375-390, :272-283)."""
    fpn_dim = cfg.FPN.DIM
    if dim == fpn_dim:
        return blob, dim
    out = plan.conv(blob, 'fpn_inner_' + blob, dim, fpn_dim, 1, 1, 0, relu=True, bias=True,
                    bn='fpn_inner_' + blob + '_bn')
    return out, fpn_dim


def build_plan():
    """model_builder.py:242 build_generic_reid_model (test, single GPU)."""
    plan = Plan()
    blob, dim, scale = add_ResNet50_conv5_body(plan)
    if cfg.FPN.FPN_ON:
        assert 'FPN_reid.add_fpn_ResNet50_conv5_body' in cfg.MODEL.CONV_BODY, \
            'FPN_ON: only FPN_reid.add_fpn_ResNet50_conv5_body is built'
        blob, dim = add_fpn_coarsest_level(plan, blob, dim)
    prefixes, d = add_pps_part_head(plan, blob, dim, scale)
    plan.output = add_reid_outputs(plan, prefixes, d)
    plan.spatial_scale = scale
    plan.feat_dim = len(prefixes) * cfg.REID.BPM_DIM
    return plan


# ---------------------------------------------------------------------------
# Weights
# ---------------------------------------------------------------------------
def synthetic_weights(plan, seed=0):
    """Seeded Detectron-format weights: He-normal convs, BN
    _s ~ U(0.5,1.5), _b ~ N(0,0.1), _rm ~ N(0,0.1), _riv ~ U(0.5,1.5).  The
    branch2c / branch1 BN scales are drawn smaller (U(0.05,0.15)) so that the
    residual stream stays O(1) through 16 blocks with untrained weights."""
    rng = np.random.RandomState(seed)
    blobs = {}
    for name in sorted(plan.params):
        shape = plan.params[name]
        if name.endswith('_w') and len(shape) == 4:
            fan_in = shape[1] * shape[2] * shape[3]
            blobs[name] = (rng.randn(*shape) * np.sqrt(2.0 / fan_in)).astype(np.float32)
        elif name.endswith('_conv_b'):
            blobs[name] = (0.01 * rng.randn(*shape)).astype(np.float32)
        elif name.endswith('_s'):
            lo, hi = (0.05, 0.15) if ('branch2c' in name or 'branch1' in name) else (0.5, 1.5)
            blobs[name] = rng.uniform(lo, hi, size=shape).astype(np.float32)
        elif name.endswith('_riv'):
            blobs[name] = rng.uniform(0.5, 1.5, size=shape).astype(np.float32)
        elif name.endswith('_rm') or name.endswith('_b'):
            blobs[name] = (0.1 * rng.randn(*shape)).astype(np.float32)
        else:
            raise KeyError(name)
    return blobs


def fold_bn(blobs, bn, conv_bias=None):
    """Test-mode SpatialBN y = (x - rm) * s / sqrt(riv + eps) + b as
    y = x * scale + shift (conv bias folded into shift)."""
    s = blobs[bn + '_s'].astype(np.float64)
    b = blobs[bn + '_b'].astype(np.float64)
    rm = blobs[bn + '_rm'].astype(np.float64)
    riv = blobs[bn + '_riv'].astype(np.float64)
    scale = s / np.sqrt(riv + BN_EPS)
    cb = 0.0 if conv_bias is None else conv_bias.astype(np.float64)
    shift = (cb - rm) * scale + b
    return scale.astype(np.float32), shift.astype(np.float32)


def pack_stem_weight(w):
    """conv1 [64][3][7][7] -> the fused stem's [64][176] layout: K index
    (kh * 3 + c) * 8 + kw, kw = 7 and the last 8 columns zero (stem.hip)."""
    cout, cin, kh_, kw_ = w.shape
    assert (cin, kh_, kw_) == (3, 7, 7), w.shape
    out = np.zeros((cout, ops.stem_k()), np.float32)
    for kh in range(7):
        for c in range(3):
            g = kh * 3 + c
            out[:, g * 8:g * 8 + 7] = w[:, c, kh, :]
    return out


def pack_conv_weight(w, cin_pad=None):
    """[Cout][Cin][KH][KW] -> [Cout][Kpad], K ordered (kh, kw, cin), Kpad % 16."""
    cout, cin, kh, kw = w.shape
    cin_p = cin_pad or cin
    t = np.zeros((cout, kh, kw, cin_p), np.float32)
    t[..., :cin] = w.transpose(0, 2, 3, 1)
    k = kh * kw * cin_p
    kpad = (k + 15) // 16 * 16
    out = np.zeros((cout, kpad), np.float32)
    out[:, :k] = t.reshape(cout, k)
    return out, kpad


# ---------------------------------------------------------------------------
# Device model
# ---------------------------------------------------------------------------
MAX_SPLITK = 4  # conv split-K factors autotune tries (2..MAX_SPLITK)
GEMM_OPS = ('conv', 'conv_dual', 'heads', 'stem_pool', 'conv_pps')  # MFMA layers of a forward


class PPSModel(object):
    """Device-resident PPS extractor.  forward(x_nhwc4) -> [N, 3968] features.

    x_nhwc4: float32 [N, H, W, 4] (BGR minus PIXEL_MEANS, 4th channel zero)
    on the current CUDA device, H x W = REID.SCALE[::-1].
    """

    def __init__(self, blobs, device='cuda', plan=None, fuse_shortcut=True, math=None,
                 act_planes=None, fused_stem=None, fused_pps=None):
        """math: 'x3' (default; f32 products on bf16 matrix cores, weights
        split once into three bf16 planes -- gemm_x3.hip) or 'f32' (exact
        f32 MFMA, gemm_f32.hip).  Env PPS_MATH overrides the default.

        act_planes (x3 only; default on, env PPS_ACT_PLANES=0 disables):
        a bottleneck intermediate read only by the next conv (branch2a ->
        2b -> 2c) may be written by its producer's epilogue as bf16x3 planes
        and read as such (ops.conv2d_bn_act_x3p), so the consumer's K loop
        skips the operand split at the price of 6 instead of 4 bytes per
        element.  Which edges use planes is a speed choice made per edge by
        autotune() (heuristic before that: the 3x3 convs with Cin >= 256);
        the bits are the same either way.

        fused_stem / fused_pps (x3 only; default on, env PPS_FUSED_STEM=0 /
        PPS_FUSED_PPS=0 disable): conv1 + BN + ReLU + pool1 as one kernel;
        the last res5 conv with the part pooling in its epilogue (its 100 MB
        output is then never written -- `res5_2_sum` is not in buffers()).
        Both give the bits of the unfused pair on the same GEMM tile."""
        self.math = math or ops.default_math()
        if self.math not in ('x3', 'f32'):
            raise ValueError("math must be 'x3' or 'f32', got %r" % self.math)
        self.plan = plan or build_plan()
        self.device = torch.device(device)
        missing = [n for n in self.plan.params if n not in blobs
                   and not n.endswith('_conv_b')]
        if missing:
            raise KeyError('weights missing %d blobs, e.g. %s' % (len(missing), missing[:5]))
        self.layers = []
        dev = self.device
        # projection shortcuts fused into their block's branch2c GEMM (K concat)
        shortcut_of = {}
        if fuse_shortcut:
            for L in self.plan.layers:
                if L['op'] == 'conv' and L['name'].endswith('_branch1') and L['k'] == 1:
                    shortcut_of[L['output']] = L
        for L in self.plan.layers:
            L = dict(L)
            if L['op'] == 'conv' and L['output'] in shortcut_of:
                continue  # computed inside the consuming branch2c
            if L['op'] == 'conv' and L.get('residual') in shortcut_of:
                sc_L = shortcut_of[L['residual']]
                w1, kpad1 = pack_conv_weight(blobs[L['name'] + '_w'])
                s1, h1 = fold_bn(blobs, L['bn'])
                w2, kpad2 = pack_conv_weight(blobs[sc_L['name'] + '_w'])
                s2, h2 = fold_bn(blobs, sc_L['bn'])
                assert kpad2 == sc_L['cin'] and kpad1 == L['cin']
                w = np.concatenate([w1 * s1[:, None], w2 * s2[:, None]], axis=1)
                L.update(op='conv_dual', w=torch.from_numpy(w.astype(np.float32)).to(dev),
                         kpad=kpad1, shift=torch.from_numpy((h1 + h2).astype(np.float32)).to(dev),
                         cin_eff=L['cin'], input2=sc_L['input'], stride2=sc_L['stride'],
                         residual=None, fused_shortcut=sc_L['name'],
                         shortcut_cin=sc_L['cin'])
                self.layers.append(L)
                continue
            if L['op'] == 'conv':
                cin_pad = 4 if L['cin'] == 3 else None
                w, kpad = pack_conv_weight(blobs[L['name'] + '_w'], cin_pad)
                sc, sh = fold_bn(blobs, L['bn'], blobs.get(L['name'] + '_b'))
                L.update(w=torch.from_numpy(w).to(dev), kpad=kpad,
                         scale=torch.from_numpy(sc).to(dev),
                         shift=torch.from_numpy(sh).to(dev),
                         cin_eff=cin_pad or L['cin'])
            elif L['op'] == 'heads':
                ws, scs, shs = [], [], []
                for p in L['prefixes']:
                    w = blobs[p + '_conv_w'].reshape(L['dim_inner'], L['dim'])
                    sc, sh = fold_bn(blobs, p + '_bn', blobs.get(p + '_conv_b'))
                    ws.append(w)
                    scs.append(sc)
                    shs.append(sh)
                L.update(w=torch.from_numpy(np.stack(ws).astype(np.float32)).to(dev),
                         scale=torch.from_numpy(np.concatenate(scs)).to(dev),
                         shift=torch.from_numpy(np.concatenate(shs)).to(dev))
            elif L['op'] == 'pps':
                L['split_arr'] = np.array(L['split'], np.int32)
            elif L['op'] == 'normalize' and self.layers and self.layers[-1]['op'] == 'heads':
                # heads GEMM as split-K partials + one reduce/BN/ReLU/Normalize pass
                H = self.layers[-1]
                H['normalize'] = True
                H['output'] = L['output']
                continue
            self.layers.append(L)
        if self.math == 'x3':
            for L in self.layers:
                if L['op'] in ('conv', 'conv_dual'):
                    L['w32'] = L['w']   # the f16x2 split is taken from it on first use
                if L['op'] in ('conv', 'conv_dual', 'heads'):
                    L['w'] = ops.split_bf16x3(L['w'], batched=L['op'] == 'heads')
        if fused_stem is None:
            fused_stem = os.environ.get('PPS_FUSED_STEM', '1') != '0'
        self.fused_stem = bool(fused_stem) and self.math == 'x3'
        if self.fused_stem:
            self._fuse_stem(blobs)
        if fused_pps is None:
            fused_pps = os.environ.get('PPS_FUSED_PPS', '1') != '0'
        self.fused_pps = bool(fused_pps) and self.math == 'x3' and self._fuse_pps()
        if act_planes is None:
            act_planes = os.environ.get('PPS_ACT_PLANES', '1') != '0'
        self.act_planes = bool(act_planes) and self.math == 'x3'
        self._bufs = {}
        self._edges = self._plane_edges() if self.act_planes else []
        self.set_planes([P['name'] for P, C in self._edges
                         if C['k'] > 1 and C['cin'] >= 256])
        self.feat_dim = self.plan.feat_dim
        self._batch = None
        self._h2e_slot = {}   # PPS_TILE_H2E edges of the last forward: blob -> bound slot

    def _fuse_stem(self, blobs):
        """Replace the stem conv + maxpool pair by one 'stem_pool' layer (its
        kernel takes 128-wide inputs: REID.SCALE[0] == 128, else the conv and
        maxpool stay separate)."""
        if int(cfg.REID.SCALE[0]) != ops.STEM_WIDTH:
            return
        for i, L in enumerate(self.layers[:-1]):
            P = self.layers[i + 1]
            if (L['op'] == 'conv' and L['input'] == 'data' and L['k'] == 7 and
                    L['stride'] == 2 and L['pad'] == 3 and L['dil'] == 1 and L['cin'] == 3 and
                    L['cout'] == 64 and L['relu'] and not L['residual'] and
                    P['op'] == 'maxpool' and P['input'] == L['output'] and P['k'] == 3 and
                    P['stride'] == 2 and P['pad'] == 1 and
                    sum(1 for M in self.layers if M.get('input') == L['output']) == 1):
                w = pack_stem_weight(blobs[L['name'] + '_w'])
                wd = torch.from_numpy(w).to(self.device)
                F = dict(L, op='stem_pool', output=P['output'], conv_output=L['output'],
                         w=ops.split_bf16x3(wd), w32s=wd)
                self.layers[i:i + 2] = [F]
                return

    def _fuse_pps(self):
        """Replace the last conv (+ residual + ReLU) and the part pooling that
        is its only reader by one 'conv_pps' layer (pooling in the GEMM
        epilogue).  Returns whether a pair was fused."""
        for i, L in enumerate(self.layers[:-1]):
            P = self.layers[i + 1]
            if (L['op'] == 'conv' and L.get('residual') and L['relu'] and
                    P['op'] == 'pps' and P['input'] == L['output'] and
                    L['output'] != self.plan.output and L['cin_eff'] % 32 == 0 and
                    L['kpad'] == L['k'] ** 2 * L['cin_eff'] and
                    sum(1 for M in self.layers for key in ('input', 'input2', 'residual')
                        if M.get(key) == L['output']) == 1):
                F = dict(L, op='conv_pps', output=P['output'], conv_output=L['output'],
                         split_arr=P['split_arr'], max_ave=P['max_ave'],
                         prefixes=P['prefixes'], pps_name=P.get('name', P['output']))
                self.layers[i:i + 2] = [F]
                return True
        return False

    def pps_tiles(self, L):
        """Tiles the fused conv + pooling can run on: pipelined, exactly one
        image (Ho x Wo rows) per tile, <= 256 columns (empty: unfused fallback)."""
        n, ho, wo, co = self._shapes[L['conv_output']]
        planes = bool(L.get('planes_in'))
        key = (ho * wo, planes)
        cache = L.setdefault('_pps_tiles', {})
        if key not in cache:
            cache[key] = [t for t in range(ops.TILE_P_FIRST, ops.num_tiles() + 1)
                          if ops.tile_shape(t, planes)[0] == ho * wo and
                          0 < ops.tile_shape(t, planes)[1] <= ops.PPS_FUSE_MAX_COLS]
        return cache[key]

    def _plane_edges(self):
        """(producer, consumer) conv pairs whose tensor may travel as bf16x3
        planes: the producer's output has exactly one reader, a plain conv
        taking it as its main input with Cin % 32 == 0 (the pipelined GEMM's
        staging unit) -- never a residual, shortcut or pooling input."""
        readers = {}
        for L in self.layers:
            for key in ('input', 'input2', 'residual'):
                if L.get(key):
                    readers.setdefault(L[key], []).append((L, key))
        edges = []
        for L in self.layers:
            rs = readers.get(L['output'], [])
            if (L['op'] == 'conv' and L['cin_eff'] % 4 == 0 and L['cout'] % 4 == 0
                    and L['output'] != self.plan.output and len(rs) == 1
                    and rs[0][0]['op'] in ('conv', 'conv_pps') and rs[0][1] == 'input'
                    and rs[0][0]['cin_eff'] % 32 == 0):
                edges.append((L, rs[0][0]))
        return edges

    def _set_edge(self, P, C, on):
        P['planes_out'] = C['planes_in'] = bool(on)
        name = P['output']
        if name in self._bufs:  # swap the one buffer if already allocated
            old = self._bufs[name]
            shape = tuple(old.shape[1:]) if old.dtype == torch.int16 else tuple(old.shape)
            is_pl = old.dtype == torch.int16
            if is_pl != bool(on):
                self._bufs[name] = (ops.act_planes(shape, self.device) if on else
                                    torch.empty(shape, dtype=torch.float32, device=self.device))

    def planes(self):
        """Names of the conv layers whose output travels as bf16x3 planes."""
        return [P['name'] for P, C in self._edges if P.get('planes_out')]

    def set_planes(self, producers):
        names = set(producers)
        known = {P['name'] for P, C in self._edges}
        if names - known:
            raise ValueError('not a plane-eligible producer: %s' % sorted(names - known)[:3])
        for P, C in self._edges:
            self._set_edge(P, C, P['name'] in names)

    # -- activation buffers (allocated once per batch size) -----------------
    def _alloc(self, N, H, W):
        shapes = {'data': (N, H, W, 4)}
        for L in self.layers:
            if L['op'] in ('conv', 'conv_dual'):
                n, h, w, _ = shapes[L['input']]
                ho = (h + 2 * L['pad'] - L['dil'] * (L['k'] - 1) - 1) // L['stride'] + 1
                wo = (w + 2 * L['pad'] - L['dil'] * (L['k'] - 1) - 1) // L['stride'] + 1
                shapes[L['output']] = (n, ho, wo, L['cout'])
            elif L['op'] == 'maxpool':
                n, h, w, c = shapes[L['input']]
                ho = (h + 2 * L['pad'] - L['k']) // L['stride'] + 1
                wo = (w + 2 * L['pad'] - L['k']) // L['stride'] + 1
                shapes[L['output']] = (n, ho, wo, c)
            elif L['op'] == 'stem_pool':
                n, h, w, _ = shapes[L['input']]
                hc, wc = (h - 1) // 2 + 1, (w - 1) // 2 + 1
                L['conv_hw'] = (hc, wc)
                shapes[L['output']] = (n, (hc - 1) // 2 + 1, (wc - 1) // 2 + 1, L['cout'])
            elif L['op'] == 'pps':
                n, h, w, c = shapes[L['input']]
                shapes[L['output']] = (len(L['prefixes']), n, c)
            elif L['op'] == 'conv_pps':
                n, h, w, _ = shapes[L['input']]
                ho = (h + 2 * L['pad'] - L['dil'] * (L['k'] - 1) - 1) // L['stride'] + 1
                wo = (w + 2 * L['pad'] - L['dil'] * (L['k'] - 1) - 1) // L['stride'] + 1
                shapes[L['conv_output']] = (n, ho, wo, L['cout'])
                shapes[L['output']] = (len(L['prefixes']), n, L['cout'])
            elif L['op'] == 'heads':
                shapes[L['output']] = (N, len(L['prefixes']) * L['dim_inner'])
                shapes[L['output'] + '_partials'] = (HEAD_SPLITK, N,
                                                     len(L['prefixes']) * L['dim_inner'])
            elif L['op'] == 'normalize':
                shapes[L['output']] = shapes[L['input']]
        self._shapes = shapes
        # algorithmic FLOPs per launch (2*M*Cout*K with the TRUE Cin: the
        # stem's 4th packed channel is not counted) -- SURVEY §8(d)
        for L in self.layers:
            if L['op'] == 'stem_pool':
                hc, wc = L['conv_hw']
                L['flops'] = 2.0 * N * hc * wc * L['cout'] * L['k'] * L['k'] * L['cin']
            elif L['op'] in ('conv', 'conv_dual', 'conv_pps'):
                n, ho, wo, co = shapes[L.get('conv_output', L['output'])]
                L['flops'] = 2.0 * n * ho * wo * co * (L['k'] * L['k'] * L['cin'] +
                                                      L.get('shortcut_cin', 0))
            elif L['op'] == 'heads':
                L['flops'] = 2.0 * N * len(L['prefixes']) * L['dim_inner'] * L['dim']
            else:
                L['flops'] = 0.0
        # algorithmic HBM bytes per launch: every operand read once, the output
        # written once (f32 activations; weights in the format the GEMM reads)
        wbytes = 6 if self.math == 'x3' else 4
        for L in self.layers:
            if L['op'] == 'stem_pool':
                L['bytes'] = float(4 * np.prod(shapes[L['input']]) +
                                   4 * np.prod(shapes[L['output']]) +
                                   wbytes * L['cout'] * ops.stem_k())
            elif L['op'] in ('conv', 'conv_dual'):
                n, ho, wo, co = shapes[L['output']]
                # a 1x1 (k < stride) conv reads only the pixels under its taps
                if L['k'] < L['stride']:
                    b = 4 * n * ho * wo * L['k'] * L['k'] * L['cin']
                else:
                    b = 4 * np.prod(shapes[L['input']])
                b += 4 * n * ho * wo * co
                b += wbytes * co * (L['k'] * L['k'] * L['cin'] + L.get('shortcut_cin', 0))
                if L.get('residual'):
                    b += 4 * n * ho * wo * co
                if L['op'] == 'conv_dual':   # the 1x1 shortcut at stride2
                    b += (4 * n * ho * wo * L['shortcut_cin'] if L['stride2'] > 1 else
                          4 * np.prod(shapes[L['input2']]))
                L['bytes'] = float(b)
            elif L['op'] == 'conv_pps':
                # input + residual + weights read, the part subsets written (the
                # conv output itself never leaves the chip)
                n, ho, wo, co = shapes[L['conv_output']]
                b = 4 * np.prod(shapes[L['input']]) + 4 * n * ho * wo * co
                b += wbytes * co * L['k'] * L['k'] * L['cin'] + 4 * np.prod(shapes[L['output']])
                L['bytes'] = float(b)
            elif L['op'] == 'heads':
                nb = len(L['prefixes'])
                L['bytes'] = float(4 * np.prod(shapes[L['input']]) +
                                   wbytes * nb * L['dim_inner'] * L['dim'] +
                                   4 * HEAD_SPLITK * N * nb * L['dim_inner'])
            else:
                L['bytes'] = 0.0
        planes = {L['output'] for L in self.layers if L.get('planes_out')}
        self._bufs = {k: (ops.act_planes(v, self.device) if k in planes else
                          torch.empty(v, dtype=torch.float32, device=self.device))
                      for k, v in shapes.items() if k != 'data'}
        self._part = None  # split-K partial sums, grown on first use (_part_for)
        self._batch = (N, H, W)

    def buffers(self):
        return self._bufs

    def flops_per_forward(self, kinds=GEMM_OPS):
        return sum(L['flops'] for L in self.layers if L['op'] in kinds)

    def bytes_per_forward(self, kinds=GEMM_OPS):
        """Algorithmic HBM bytes of the GEMM launches of one forward."""
        return sum(L['bytes'] for L in self.layers if L['op'] in kinds)

    def h2_capable(self, L):
        """Whether PPS_TILE_H2 can run the layer (the C plan's h2_tile_ok):
        a conv / fused-shortcut conv / conv_pps with Cin % 32 == 0 and no K
        padding, ending in a ReLU."""
        return (self.math == 'x3' and L['op'] in ('conv', 'conv_dual', 'conv_pps') and
                'w32' in L and L['cin_eff'] % 32 == 0 and
                L['kpad'] == L['k'] ** 2 * L['cin_eff'] and
                (L['op'] != 'conv_dual' or L['shortcut_cin'] % 32 == 0) and
                (L['op'] != 'conv' or L['relu']))

    @staticmethod
    def ws_h2_layer(L):
        """The layers the f16x2 weight-stationary tile (54) takes (the C
        plan's ws_h2_layer): a 1x1 / stride-1 / unpadded conv or fused
        shortcut conv with K = 64, 128 or 256 and Cout % 64 == 0."""
        if L['op'] not in ('conv', 'conv_dual'):
            return False
        if L['k'] != 1 or L['stride'] != 1 or L['pad'] != 0 or L['kpad'] != L['cin_eff']:
            return False
        K = L['cin_eff'] + (L.get('shortcut_cin', 0) if L['op'] == 'conv_dual' else 0)
        return K in (64, 128, 256) and L['cout'] % 64 == 0

    def _run_h2(self, L, bufs, tile):
        """PPS_TILE_H2: the layer in f16x2 arithmetic (ops.conv2d_bn_act_h2 and
        siblings); the input's max comes from ops.amax (the C plan's producers
        report the same value from their epilogues, so the scale and the bits
        agree)."""
        if L.get('planes_in') or L.get('planes_out') or L.get('splitk', 1) > 1:
            raise RuntimeError("layer '%s': PPS_TILE_H2 needs f32 activations at both ends "
                               "and no split-K" % L.get('name', L['output']))
        if '_w2' not in L:
            L['_w2'] = ops.split_weights_h2(L['w32'])
        w2, wrs = L['_w2']
        base = tile & ~(ops.TILE_H2 | ops.TILE_H2P | ops.TILE_H2E | ops.TILE_B_TILED |
                        ops.TILE_SEAM | ops.TILE_COL_ORDER)
        flags = tile & ops.TILE_COL_ORDER
        x = bufs[L['input']]
        op = L['op']
        if tile & ops.TILE_H2E:   # the producer wrote f16x2 planes and their bound's slot
            amx = self._h2e_slot.get(L['input'])
            if amx is None:
                raise RuntimeError("layer '%s': PPS_TILE_H2E but the producer wrote no f16x2 "
                                   "planes" % L['name'])
            xin = self._h2e_view(L['input'], bufs)
        else:
            amx = self._in_slot(L['input'], x)
            xin = ops.split_act_h2(x, amx) if tile & ops.TILE_H2P else x   # PPS_TILE_H2P
        if op == 'conv':
            res = bufs[L['residual']] if L['residual'] else None
            ops.conv2d_bn_act_h2(xin, L['cin_eff'], w2, wrs, L['kpad'], L['k'], L['stride'],
                                 L['pad'], L['dil'], L['scale'], L['shift'], res, L['relu'],
                                 bufs[L['output']], amx, tile=base | flags)
        elif op == 'conv_dual':
            x2 = bufs[L['input2']]
            ops.conv2d_dual_bn_act_h2(x, L['cin_eff'], L['k'], L['stride'], L['pad'], x2,
                                      L['stride2'], w2, wrs, L['kpad'], L['shift'], L['relu'],
                                      bufs[L['output']], amx, ops.amax(x2), tile=base | flags)
        else:   # conv_pps
            ok = [t for t in self.pps_tiles(L) if t >= ops.TILE_P16_FIRST]
            if not ok:
                raise RuntimeError("layer '%s': no f16x2 tile holds one image" % L['name'])
            t = (base if base in ok else ok[0]) | flags
            ops.conv2d_bn_act_pps_h2(xin, L['cin_eff'], w2, wrs, L['kpad'], L['k'], L['stride'],
                                     L['pad'], L['dil'], L['scale'], L['shift'],
                                     bufs[L['residual']], L['split_arr'], L['max_ave'],
                                     bufs[L['output']], amx, y=None, tile=t)

    def _h2e_view(self, blob, bufs):
        """The f16x2 planes [2, N, H, W, C] (int16) an H2E edge's f32 buffer holds
        (the two planes numel() apart, as the C plan writes them)."""
        b = bufs[blob]
        return b.view(-1).view(torch.int16).view((2,) + tuple(b.shape))

    def _in_slot(self, blob, x):
        """The activation-max slot an f16x2 layer reads for its input: the
        bound slot of an H2E edge, else max|x| measured here (the C plan's
        producers report the same value from their epilogues)."""
        s = self._h2e_slot.get(blob)
        return s if s is not None else ops.amax(x)

    def h2e_producer(self, C):
        """Index of the conv + BN + ReLU whose output layer C may read as f16x2
        planes (PPS_TILE_H2E; the C plan's h2e_producer), or -1."""
        if C['op'] not in ('conv', 'conv_pps'):
            return -1
        for i, P in enumerate(self.layers):
            if P['output'] != C['input']:
                continue
            if (P['op'] != 'conv' or not P['relu'] or P['residual'] or 'w32' not in P or
                    P['cin_eff'] % 32 or P['kpad'] != P['k'] ** 2 * P['cin_eff']):
                return -1
            readers = sum((Q['input'] == P['output']) + (Q.get('input2') == P['output']) +
                          (Q.get('residual') == P['output']) for Q in self.layers)
            if readers != 1 or (i > 0 and self._seam_pair(i - 1)):
                return -1
            return i
        return -1

    def _seam_pair(self, i):
        """Layers i, i + 1 are a seam-capable branch2c + branch2a (seam_pair)."""
        if self.math != 'x3' or i + 1 >= len(self.layers):
            return False
        L, X = self.layers[i], self.layers[i + 1]

        def plain1x1(A):
            return (A['op'] == 'conv' and A['k'] == 1 and A['stride'] == 1 and
                    A['pad'] == 0 and A['relu'] and A['kpad'] == A['cin_eff'])
        return bool(plain1x1(L) and plain1x1(X) and L.get('residual') and
                    not X.get('residual') and X['input'] == L['output'] and
                    X['cin_eff'] == L['cout'] and
                    (L['cin_eff'], L['cout'], X['cout']) in ((64, 256, 64), (128, 512, 128)))

    def _h2e_consumer(self, L):
        for C in self.layers:
            if (C['input'] == L['output'] and C.get('tile', 0) & ops.TILE_H2E and
                    C.get('tile', 0) & ops.TILE_H2):
                return C
        return None

    def _run_h2out(self, L, bufs, tile):
        """Producer of a PPS_TILE_H2E edge: conv + BN + ReLU writing f16x2
        planes on the scale of the bound bw * max|x| + bb (its arithmetic as
        its own tile says), the bound into the edge's slot."""
        if L.get('planes_in') or L.get('planes_out') or L.get('splitk', 1) > 1:
            raise RuntimeError("layer '%s': f16x2 planes out needs an f32 input and no split-K"
                               % L['name'])
        if '_h2o' not in L:
            L['_h2o'] = ops.h2_out_bound(L['w32'], L['scale'], L['shift'])
        x = bufs[L['input']]
        base = tile & ~(ops.TILE_H2 | ops.TILE_H2P | ops.TILE_H2E | ops.TILE_B_TILED |
                        ops.TILE_SEAM)
        in_slot = self._in_slot(L['input'], x) if not tile & ops.TILE_H2E else \
            self._h2e_slot[L['input']]
        out_slot = ops.amax_slot(x.device)
        y2 = self._h2e_view(L['output'], bufs)
        if tile & ops.TILE_H2:
            if '_w2' not in L:
                L['_w2'] = ops.split_weights_h2(L['w32'])
            w, wrs = L['_w2']
            if tile & ops.TILE_H2E:
                xin = self._h2e_view(L['input'], bufs)
            else:
                xin = ops.split_act_h2(x, in_slot) if tile & ops.TILE_H2P else x
            amx = in_slot
        else:
            w, wrs, xin, amx = L['w'], None, x, None
        ops.conv2d_bn_act_h2out(xin, L['cin_eff'], w, wrs, L['kpad'], L['k'], L['stride'],
                                L['pad'], L['dil'], L['scale'], L['shift'], y2, amx, in_slot,
                                L['_h2o'], out_slot, tile=base)
        self._h2e_slot[L['output']] = out_slot

    def _run(self, L, bufs, out=None, tile=None, splitk=None):
        op = L['op']
        tile = L.get('tile', 0) if tile is None else tile
        tile &= ~ops.TILE_SEAM   # one layer alone (forward() runs the seam pairs)
        if op == 'conv' and self._h2e_consumer(L) is not None:
            return self._run_h2out(L, bufs, tile)
        if op == 'stem_pool' and tile & ops.TILE_H2:   # f16x2 stem, the input's max measured here
            if '_w2s' not in L:
                L['_w2s'] = ops.stem_split_h2(L['w32s'])
            w2, winv = L['_w2s']
            x = bufs[L['input']]
            return ops.stem_conv_pool_h2(x, w2, winv, ops.amax(x), L['scale'], L['shift'],
                                         bufs[L['output']])
        if tile & ops.TILE_H2:
            return self._run_h2(L, bufs, tile)
        sk = L.get('splitk', 1) if splitk is None else splitk
        w = L.get('w')
        # split convs run in one launch on the FIX tiles (same bits as the
        # two-pass split-K, which takes plain weights only)
        fused_sk = (op == 'conv' and sk > 1 and (tile & 0xff) in ops.FIX_TILES and L['relu']
                    and not (L.get('planes_out') and L['residual']))
        if sk > 1 and not fused_sk:
            tile &= ~ops.TILE_B_TILED
        if op in ('conv', 'conv_dual', 'conv_pps') and tile > 0 and tile & ops.TILE_B_TILED:
            # the chunk-tiled weight copy (pps_model_autotune may pick it)
            if '_wt' not in L:
                L['_wt'] = ops.tile_planes(L['w'])
            w = L['_wt']
        if op == 'conv' and (L.get('planes_in') or L.get('planes_out') or sk > 1):
            tile = tile if tile >= ops.TILE_P_FIRST else 0  # pipelined tiles only
            res = bufs[L['residual']] if L['residual'] else None
            ops.conv2d_bn_act_x3p(bufs[L['input']], L['cin_eff'], w, L['kpad'], L['k'],
                                  L['stride'], L['pad'], L['dil'], L['scale'], L['shift'],
                                  res, L['relu'], bufs[L['output']], tile=tile, splitk=sk,
                                  part=self._part_for(sk * np.prod(self._shapes[L['output']]))
                                  if sk > 1 else None,
                                  counters=self._cnt_for(np.prod(self._shapes[L['output']][:3]),
                                                         L['cout']) if fused_sk else None)
        elif op == 'conv':
            res = bufs[L['residual']] if L['residual'] else None
            ops.conv2d_bn_act(bufs[L['input']], L['cin_eff'], w, L['kpad'], L['k'],
                              L['stride'], L['pad'], L['dil'], L['scale'], L['shift'],
                              res, L['relu'], bufs[L['output']], tile=tile)
        elif op == 'conv_dual':
            ops.conv2d_dual_bn_act(bufs[L['input']], L['cin_eff'], L['k'], L['stride'],
                                   L['pad'], bufs[L['input2']], L['stride2'], w,
                                   L['kpad'], L['shift'], L['relu'], bufs[L['output']],
                                   tile=tile)
        elif op == 'maxpool':
            ops.maxpool2d(bufs[L['input']], L['k'], L['stride'], L['pad'],
                          bufs[L['output']])
        elif op == 'stem_pool':
            ops.stem_conv_pool_x3(bufs[L['input']], L['w'], L['scale'], L['shift'],
                                  bufs[L['output']])
        elif op == 'pps':
            ops.part_power_set(bufs[L['input']], L['split_arr'], L['max_ave'],
                               bufs[L['output']])
        elif op == 'conv_pps':
            res = bufs[L['residual']]
            ok = self.pps_tiles(L)
            if ok:
                flags = tile & (ops.TILE_B_TILED | ops.TILE_COL_ORDER)
                tb = tile & ~flags
                t = (tb if tb in ok else ok[0]) | flags
                ops.conv2d_bn_act_pps(bufs[L['input']], L['cin_eff'], w, L['kpad'], L['k'],
                                      L['stride'], L['pad'], L['dil'], L['scale'], L['shift'],
                                      res, L['split_arr'], L['max_ave'], bufs[L['output']],
                                      y=None, tile=t)
            else:   # no tile holds exactly one image: conv, then the pooling kernel
                ops.conv2d_bn_act_x3p(bufs[L['input']], L['cin_eff'], w, L['kpad'],
                                      L['k'], L['stride'], L['pad'], L['dil'], L['scale'],
                                      L['shift'], res, True, bufs[L['conv_output']],
                                      tile=tile if tile >= ops.TILE_P_FIRST else 0)
                ops.part_power_set(bufs[L['conv_output']], L['split_arr'], L['max_ave'],
                                   bufs[L['output']])
        elif op == 'heads':
            y = bufs[L['output']] if out is None or self.layers[-1] is not L else out
            part = bufs[L['output'] + '_partials']
            ops.gemm_splitk_batched(bufs[L['input']], L['w'], HEAD_SPLITK, part, tile=tile)
            ops.splitk_bn_act_normalize(part, L['scale'], L['shift'], True,
                                        L.get('normalize', False), y)
            bufs[L['output']] = y
        elif op == 'normalize':
            y = out if out is not None else bufs[L['output']]
            ops.l2_normalize(bufs[L['input']], y)
            bufs[L['output']] = y

    def forward(self, x, out=None, timer=None, timer_external=False):
        """Run the plan.  `timer`, if a list, receives (layer, op, flops,
        start_event, end_event) per layer, recorded on the current stream
        (timer_external: events that may be recorded inside a hipGraph
        capture, so a graph replay times each launch)."""
        assert x.dtype == torch.float32 and x.is_contiguous() and x.dim() == 4
        assert x.shape[3] == 4, 'input must be NHWC with 4 channels (see preprocess)'
        N, H, W, _ = x.shape
        if self._batch != (N, H, W):
            self._alloc(N, H, W)
        bufs = dict(self._bufs)
        bufs['data'] = x
        self._h2e_slot = {}   # f16x2-planes edges (PPS_TILE_H2E): blob -> bound slot
        fused = None   # the branch2a the previous seam launch computed
        for i, L in enumerate(self.layers):
            if L is fused:
                continue
            if timer is not None:
                ev0 = torch.cuda.Event(enable_timing=True, external=timer_external)
                ev1 = torch.cuda.Event(enable_timing=True, external=timer_external)
                ev0.record()
            if L['op'] == 'conv' and L.get('tile', 0) & ops.TILE_SEAM:
                # PPS_TILE_SEAM (set by the C autotune): this branch2c and the
                # next block's branch2a in one launch, as the C plan runs them
                fused = self.layers[i + 1]
                if (L.get('planes_in') or L.get('planes_out') or fused.get('planes_out') or
                        L.get('splitk', 1) > 1 or fused.get('splitk', 1) > 1):
                    raise RuntimeError("layer '%s': PPS_TILE_SEAM needs f32 activations at "
                                       "both ends and no split-K" % L['name'])
                ops.conv1x1_seam(bufs[L['input']], L['w'], L['scale'], L['shift'],
                                 bufs[L['residual']], bufs[L['output']], fused['w'],
                                 fused['scale'], fused['shift'], bufs[fused['output']])
            else:
                self._run(L, bufs, out)
            if timer is not None:
                ev1.record()
                timer.append((L.get('name', L['output']), L['op'], L['flops'], ev0, ev1))
        return bufs[self.plan.output]

    def autotune(self, x, reps=3, tiles=None, finalists=4, final_reps=10, planes=True,
                 splitk=False):
        """Pick the fastest GEMM tile per conv layer by timing every candidate
        on this device (the cudnn_exhaustive_search analogue of the
        reference's DetectionModelHelper, detector.py:58): a screening pass
        over all tiles, then the `finalists` best re-timed with `final_reps`
        launches each.  Then (x3 with act_planes) each plane-eligible edge,
        in forward order, is switched to bf16x3 planes and kept if its two
        layers, re-tuned, get > 2 % faster; last (x3, splitk=True) each conv
        tries split-K 2..MAX_SPLITK on the pipelined tiles, kept if > 2 %
        faster -- off by default: at batch 64 it wins 7-8 % on isolated res5
        layers (scripts/probes/splitk_probe.py) but never inside the forward, where
        the extra partial-sum pass eats the gain.  Results do not depend on the
        tile or the plane choice (same per-element accumulation order)."""
        self.forward(x)
        torch.cuda.synchronize()
        cands = list(tiles or range(1, ops.num_tiles() + 1))

        def time_tile(L, t, n):
            bufs = dict(self._bufs)
            bufs['data'] = x
            for _ in range(2):
                self._run(L, bufs, tile=t)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                self._run(L, bufs, tile=t)
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) / n

        def tune(L):
            lc = cands
            if L.get('planes_in') or L.get('planes_out'):
                lc = [t for t in cands if t >= ops.TILE_P_FIRST] or [0]
            if L['op'] == 'conv_pps':
                lc = [t for t in cands if t in self.pps_tiles(L)] or [0]
            times = {t: time_tile(L, t, reps) for t in lc}
            best = sorted(times, key=times.get)[:finalists]
            final = {t: time_tile(L, t, final_reps) for t in best}
            L['tile'] = min(final, key=final.get)
            return final[L['tile']], times

        tune_planes = planes and self.act_planes
        if tune_planes:
            self.set_planes([])
        report, cost = {}, {}
        for L in self.layers:
            if L['op'] not in ('conv', 'conv_dual', 'heads', 'conv_pps'):
                continue
            cost[id(L)], times = tune(L)
            report[L.get('name', L['output'])] = (L['tile'], times)
        if tune_planes:
            for P, C in self._edges:
                before = cost[id(P)] + cost[id(C)]
                saved = P['tile'], C['tile']
                self._set_edge(P, C, True)
                (cp, tp), (cc, tc) = tune(P), tune(C)
                if cp + cc < 0.98 * before:
                    cost[id(P)], cost[id(C)] = cp, cc
                    report[P['name']] = (P['tile'], tp)
                    report[C['name']] = (C['tile'], tc)
                else:
                    self._set_edge(P, C, False)
                    P['tile'], C['tile'] = saved
        if self.math == 'x3' and splitk:
            # split-K (conv_bn_act_x3p_splitk) where it beats the one-pass
            # kernel by > 2 % -- the res5 3x3/1x1 layers at batch 64
            ptiles = [t for t in cands if ops.TILE_P_FIRST <= t < ops.TILE_C16_FIRST]

            def time_split(L, t, sk, n):
                bufs = dict(self._bufs)
                bufs['data'] = x
                for _ in range(2):
                    self._run(L, bufs, tile=t, splitk=sk)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(n):
                    self._run(L, bufs, tile=t, splitk=sk)
                e1.record()
                e1.synchronize()
                return e0.elapsed_time(e1) / n

            for L in self.layers:
                if L['op'] != 'conv' or L['cin_eff'] % 32 or L['kpad'] != L['k'] ** 2 * L['cin_eff']:
                    continue
                opts = [(t, sk) for sk in range(2, MAX_SPLITK + 1) if L['kpad'] % (32 * sk) == 0
                        for t in ptiles]
                if not opts:
                    continue
                times = {o: time_split(L, o[0], o[1], reps) for o in opts}
                best = sorted(times, key=times.get)[:finalists]
                final = {o: time_split(L, o[0], o[1], final_reps) for o in best}
                o = min(final, key=final.get)
                if final[o] < 0.98 * cost[id(L)]:
                    L['tile'], L['splitk'] = o
                    cost[id(L)] = final[o]
                    report[L['name']] = (L['tile'], times)
        return report

    def _part_for(self, n):
        """Split-K partials buffer of >= n floats, shared by the layers (grown
        outside graph capture: autotune / the first eager forward)."""
        if self._part is None or self._part.numel() < n:
            self._part = torch.empty((int(n),), dtype=torch.float32, device=self.device)
        return self._part

    def _cnt_for(self, M, cout):
        """Zeroed tile counters of the one-launch split-K (>= the output tiles
        of the smallest FIX tile; the kernel leaves them zero)."""
        n = -(-int(M) // 96) * -(-int(cout) // 64)
        if getattr(self, '_cnt', None) is None or self._cnt.numel() < n:
            self._cnt = torch.zeros((n,), dtype=torch.int32, device=self.device)
        return self._cnt

    def splitks(self):
        """{layer name: split-K factor} of the conv layers that use split-K."""
        return {L['name']: int(L['splitk']) for L in self.layers if L.get('splitk', 1) > 1}

    def set_splitks(self, sks):
        """Apply a splitks() mapping; a factor must cut K into whole 32-wide
        chunks of a Cin % 32 == 0 conv (bf16x3 math)."""
        for L in self.layers:
            if L['op'] != 'conv':
                continue
            sk = int(sks.get(L['name'], 1))
            if sk > 1 and (self.math != 'x3' or L['cin_eff'] % 32 or sk > MAX_SPLITK or
                           L['kpad'] != L['k'] ** 2 * L['cin_eff'] or L['kpad'] % (32 * sk)):
                raise ValueError('split-K %d not possible for %s (K = %d)'
                                 % (sk, L['name'], L['kpad']))
            L['splitk'] = sk

    def tiles(self):
        """{layer name: tile id} of the GEMM layers (0 = heuristic)."""
        return {L.get('name', L['output']): int(L.get('tile', 0)) for L in self.layers
                if L['op'] in ('conv', 'conv_dual', 'heads', 'conv_pps', 'stem_pool')}

    def _check_tile(self, i, tile):
        """The C plan's set_tile / seam_ok / h2_tile_ok conditions: a table
        the C plan refuses is refused here too (a stale or hand-edited table
        must not run a wrong launch silently)."""
        L = self.layers[i]
        name = L.get('name', L['output'])
        if L['op'] == 'stem_pool':   # 0 (bf16x3) or PPS_TILE_H2 (f16x2) only
            if tile not in (0, ops.TILE_H2) or (tile and 'w32s' not in L):
                raise ValueError("stem '%s': tile 0 or PPS_TILE_H2 (f16x2) only" % name)
            return
        if tile & ops.TILE_SEAM:
            X = self.layers[i + 1] if i + 1 < len(self.layers) else None

            def plain1x1(A):
                return (A['op'] == 'conv' and A['k'] == 1 and A['stride'] == 1 and
                        A['pad'] == 0 and A['relu'] and A['kpad'] == A['cin_eff'])
            ok = (self.math == 'x3' and X is not None and plain1x1(L) and plain1x1(X) and
                  L.get('residual') and not X.get('residual') and X['input'] == L['output'] and
                  X['cin_eff'] == L['cout'] and
                  (L['cin_eff'], L['cout'], X['cout']) in ((64, 256, 64), (128, 512, 128)) and
                  (tile & ~ops.TILE_SEAM) == ops.TILE_WS)
            if not ok:
                raise ValueError("PPS_TILE_SEAM: '%s' is not a branch2c feeding a seam-capable "
                                 "branch2a (base tile 54)" % name)
        if tile & ops.TILE_H2E and (not tile & ops.TILE_H2 or tile & ops.TILE_H2P or
                                    self.h2e_producer(L) < 0):
            raise ValueError("PPS_TILE_H2E: '%s' needs PPS_TILE_H2 (not H2P) and a producer that "
                             "is a conv + BN + ReLU read by it alone" % name)
        if tile & ops.TILE_H2P and (not tile & ops.TILE_H2 or L['op'] == 'conv_dual'):
            raise ValueError("PPS_TILE_H2P: '%s' needs PPS_TILE_H2 on a plain conv or conv_pps"
                             % name)
        if tile & ops.TILE_H2:
            base = tile & 0xff
            if base == ops.TILE_WS:   # the weight-stationary 1x1, f32 input (h2_tile_ok)
                ok = (self.ws_h2_layer(L) and
                      not tile & (ops.TILE_H2P | ops.TILE_H2E))
            else:
                ok = base == 0 or (ops.TILE_P16_FIRST <= base <= ops.num_tiles() and
                                   (L['op'] == 'conv' or base < ops.TILE_C16_FIRST or
                                    base == ops.TILE_H2_WIDE))
            if not self.h2_capable(L) or not ok:
                raise ValueError("PPS_TILE_H2: '%s' has no f16x2 arithmetic or the base tile "
                                 "%d is not 0, 38..55, 60, (convs) 56..59 or 54 on a "
                                 "weight-stationary 1x1" % (name, base))

    def set_tiles(self, tiles):
        """Apply a tiles() mapping (e.g. a saved autotune result).  Seam and
        f16x2 flags are validated as the C plan does."""
        for i, L in enumerate(self.layers):
            k = L.get('name', L['output'])
            if k in tiles:
                self._check_tile(i, int(tiles[k]))
                L['tile'] = int(tiles[k])
