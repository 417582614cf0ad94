"""The reference's test net, executed by name: operator registry + net
executor over libpps_hip.so.

The reference builds its test net with Caffe2 operators called by name
(`model.net.Conv(...)`, `model.net.Sum(...)`, `model.net.PairWiseDistance`;
detectron/modeling/ResNet.py, pps_heads.py, bpm_heads.py, reid_heads.py,
triplet_loss.py:145) from the registry the ops libraries fill
(`dyndep.InitOpsLibrary`, utils/c2.py:41-50) and runs it with
`workspace.RunNet` (core/test.py:163-185).  Here the same net -- the op list
recorded from the reference's own builders, tests/golden/pps_graph_*.json --
runs two ways:

* `Net.run_eager(x)`: op by op through `OPS`, the registry of the reference's
  op names (Conv, SpatialBN, Relu, Sum, Add, Max, Mean, MaxPool, AveragePool,
  Split, FC, Concat, Reshape, Normalize, PairWiseDistance), each a HIP kernel
  (Concat / Reshape / Split are layout only: views and one copy).  Blobs are
  NHWC device tensors; NCHW axis arguments are translated.
* `Net.forward(x)`: `compile_graph` fuses the op list into the product plan
  -- Conv+SpatialBN(+Sum)+Relu into one implicit-GEMM launch, the projection
  shortcut into its block's branch2c GEMM, Split + 10 global pools + 31
  Mean/Max/Add into the part-power-set kernel, the 31 head Conv+SpatialBN+Relu
  + Concat + Reshape + Normalize into one split-K GEMM + one epilogue pass --
  and runs it on PPSModel.  The compiled plan equals `model.build_plan()`
  layer for layer, so `forward` is bit-identical to PPSModel.

Layout: NHWC activations; the graph input 'data' is NHWC with 4 channels
(BGR minus means, 4th zero), as ops.preprocess_bgr writes it.
"""
import json
import weakref

import numpy as np
import torch

from . import model as pmodel
from . import ops

NCHW_TO_NHWC = {0: 0, 1: 3, 2: 1, 3: 2}


# ---------------------------------------------------------------------------
# Operator registry (reference Caffe2 op names)
# ---------------------------------------------------------------------------
def _host(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


# packed device copies per weight object: id(w) -> (weakref to w, {cin:
# (version, packed, kpad)}).  The weakref's callback drops the entry when the
# weight dies, and an in-place change of a torch weight (its version
# counter) repacks it.
_PACKED = {}


def _packed_conv(w, cin):
    """Caffe2 conv weight [Cout][Cin][k][k] -> the GEMM layout [Cout][Kpad]
    (K ordered kh, kw, cin; cin padded to the input's channels), cached per
    weight tensor."""
    version = getattr(w, '_version', 0)
    key = id(w)
    entry = _PACKED.get(key)
    if entry is not None and entry[0]() is not w:
        entry = None
    hit = entry[1].get(cin) if entry is not None else None
    if hit is not None and hit[0] == version:
        return hit[1], hit[2]
    wn = _host(w).astype(np.float32)
    packed, kpad = pmodel.pack_conv_weight(wn, cin if cin != wn.shape[1] else None)
    dev = torch.from_numpy(packed).cuda()
    if entry is None:
        entry = (weakref.ref(w, lambda _r, k=key: _PACKED.pop(k, None)), {})
        _PACKED[key] = entry
    entry[1][cin] = (version, dev, kpad)
    return dev, kpad


def op_conv(inputs, kernel=1, stride=1, pad=0, dilation=1, group=1, **_):
    x, w = inputs[0], inputs[1]
    if group != 1:
        raise RuntimeError('Conv: group != 1 is not built')
    N, H, W, C = x.shape
    cout, cin, kh, kw = w.shape
    if kh != kernel or kw != kernel or cin > C:
        raise RuntimeError('Conv: weight %s does not match kernel %d / input channels %d'
                           % (tuple(w.shape), kernel, C))
    wp, kpad = _packed_conv(w, C)
    ho = (H + 2 * pad - dilation * (kernel - 1) - 1) // stride + 1
    wo = (W + 2 * pad - dilation * (kernel - 1) - 1) // stride + 1
    y = torch.empty((N, ho, wo, cout), dtype=torch.float32, device=x.device)
    one = torch.ones(cout, dtype=torch.float32, device=x.device)
    bias = inputs[2].contiguous() if len(inputs) > 2 else \
        torch.zeros(cout, dtype=torch.float32, device=x.device)
    ops.conv2d_bn_act(x.contiguous(), C, wp, kpad, kernel, stride, pad, dilation, one, bias,
                      None, False, y)
    return [y]


def op_spatial_bn(inputs, epsilon=1e-5, is_test=1, **_):
    if not is_test:
        raise RuntimeError('SpatialBN: only is_test=1 (inference) is built')
    x, s, b, rm, riv = inputs
    return [ops.spatial_bn(x.contiguous(), s, b, rm, riv, epsilon)]


def _eltwise(name):
    def run(inputs, **_):
        return [ops.eltwise(name, [t.contiguous() for t in inputs])]
    return run


def _pool(mode):
    def run(inputs, kernel=None, stride=1, pad=0, global_pooling=False, **_):
        x = inputs[0]
        if global_pooling:
            N, _, _, C = x.shape
            return [ops.global_pool(x, 'ave' if mode == 'ave' else 'max')
                    .view(N, 1, 1, C)]
        if mode != 'max':
            raise RuntimeError('AveragePool: only global_pooling is built')
        N, H, W, C = x.shape
        ho = (H + 2 * pad - kernel) // stride + 1
        wo = (W + 2 * pad - kernel) // stride + 1
        y = torch.empty((N, ho, wo, C), dtype=torch.float32, device=x.device)
        return [ops.maxpool2d(x.contiguous(), kernel, stride, pad, y)]
    return run


def op_split(inputs, split=None, axis=1, **_):
    x = inputs[0]
    ax = NCHW_TO_NHWC[axis]
    return list(torch.split(x, list(split), dim=ax))   # views: no data movement


def op_fc(inputs, **_):
    x, w, b = inputs
    N = x.shape[0]
    x2 = x.reshape(N, -1).contiguous()
    cout, K = w.shape[0], int(np.prod(w.shape[1:]))
    if x2.shape[1] != K:
        raise RuntimeError('FC: input width %d != weight K %d' % (x2.shape[1], K))
    y = torch.empty((N, cout), dtype=torch.float32, device=x.device)
    one = torch.ones(cout, dtype=torch.float32, device=x.device)
    ops.gemm_bn_act_batched(x2.view(1, N, K), w.reshape(1, cout, K).contiguous(), one,
                            b.contiguous(), False, y)
    return [y]


def op_concat(inputs, axis=1, **_):
    ax = NCHW_TO_NHWC[axis] if inputs[0].dim() == 4 else axis
    y = torch.cat([t for t in inputs], dim=ax)     # layout: one copy
    info = torch.tensor([t.shape[ax] for t in inputs], dtype=torch.int32)
    return [y, info]


def op_reshape(inputs, shape=None, **_):
    x = inputs[0]
    # reid_heads.py:110-115 Reshape [1, -1] of a batch-1 blob: kept per image
    # (batch N) -- SURVEY Appendix A.7
    if list(shape) == [1, -1]:
        y = x.reshape(x.shape[0], -1)
    else:
        y = x.reshape(tuple(shape))
    return [y, torch.tensor(list(x.shape), dtype=torch.int64)]


def op_normalize(inputs, axis=1, **_):
    x = inputs[0]
    if axis != 1 or x.dim() != 2:
        raise RuntimeError('Normalize: only axis=1 on 2-D input is built')
    return [ops.l2_normalize(x.contiguous())]


def op_pairwise_distance(inputs, **_):
    (x,) = inputs
    return [ops.pairwise_distance(x)]


OPS = {
    'Conv': op_conv,
    'SpatialBN': op_spatial_bn,
    'Relu': _eltwise('Relu'),
    'Sum': _eltwise('Sum'),
    'Add': _eltwise('Add'),
    'Max': _eltwise('Max'),
    'Mean': _eltwise('Mean'),
    'MaxPool': _pool('max'),
    'AveragePool': _pool('ave'),
    'Split': op_split,
    'FC': op_fc,
    'Concat': op_concat,
    'Reshape': op_reshape,
    'Normalize': op_normalize,
    'PairWiseDistance': op_pairwise_distance,
}


def run_op(name, inputs, **args):
    """Look up an operator by its reference (Caffe2) name and run it."""
    if name not in OPS:
        raise RuntimeError('Operator %s is not registered in pps_amd (have: %s)'
                           % (name, ', '.join(sorted(OPS))))
    return OPS[name](inputs, **args)


# ---------------------------------------------------------------------------
# Graph compiler: op list -> fused plan
# ---------------------------------------------------------------------------
def live_ops(graph):
    """The ops the output depends on (backward liveness over the op list;
    in-place ops keep their producer chain).  Drops what the reference
    computes at test and never reads: the FC logits (reid_heads.py:84-120)
    and, with FPN on, the top-down levels (pps_heads.py:88-96)."""
    need = {graph['output']}
    keep = []
    for o in reversed(graph['ops']):
        if any(b in need for b in o['outputs']):
            keep.append(o)
            need.difference_update(o['outputs'])
            need.update(o['inputs'])
    return keep[::-1]


def compile_graph(graph):
    """Fuse the recorded op list into the layer plan PPSModel runs (same
    layers, names and parameters as model.build_plan() for that config)."""
    ops_ = live_ops(graph)
    shapes = {k: tuple(v) for k, v in graph['params'].items()}
    plan = pmodel.Plan()
    pending = {}     # BN output -> conv spec awaiting its Sum (shortcut / branch2c)
    n, i = len(ops_), 0

    def conv_spec(c, bn):
        w = c['inputs'][1]
        cout, cin, k, _ = shapes[w]
        a = c['args']
        return dict(blob_in=c['inputs'][0], prefix=c['outputs'][0], dim_in=cin,
                    dim_out=cout, k=k, stride=a['stride'], pad=a['pad'],
                    dilation=a.get('dilation', 1), bias=len(c['inputs']) > 2,
                    bn=bn['outputs'][0])

    def emit(spec, relu=False, residual=None, out=None):
        return plan.conv(spec['blob_in'], spec['prefix'], spec['dim_in'], spec['dim_out'],
                         spec['k'], spec['stride'], spec['pad'], spec['dilation'],
                         relu=relu, residual=residual, out=out, bias=spec['bias'],
                         bn=spec['bn'])

    def is_(j, t, inp=None):
        return j < n and ops_[j]['type'] == t and (inp is None or ops_[j]['inputs'][0] == inp)

    pooled = set()   # the part-power-set outputs (<prefix>_pool2)
    while i < n:
        o = ops_[i]
        t = o['type']
        if t == 'Conv' and o['inputs'][0] in pooled:
            break        # the reid heads: handled below
        if t == 'Conv' and is_(i + 1, 'SpatialBN', o['outputs'][0]):
            bn = ops_[i + 1]
            spec = conv_spec(o, bn)
            bout = bn['outputs'][0]
            if is_(i + 2, 'Relu', bout) and ops_[i + 2]['outputs'][0] == bout:
                emit(spec, relu=True)
                i += 3
            else:
                pending[bout] = spec
                i += 2
            continue
        if t == 'Sum':
            a, b = o['inputs']
            out = o['outputs'][0]
            relu = is_(i + 1, 'Relu', out) and ops_[i + 1]['outputs'][0] == out
            if b in pending:      # projection shortcut, placed where build_plan has it:
                sc = pending.pop(b)   # before its block's first conv (ResNet.py:186-195)
                emit(sc)
                L = plan.layers.pop()
                j = next(k for k, M in enumerate(plan.layers) if M['input'] == sc['blob_in'])
                plan.layers.insert(j, L)
            emit(pending.pop(a), relu=relu, residual=b, out=out)
            i += 2 if relu else 1
            continue
        if t == 'MaxPool' and not o['args'].get('global_pooling'):
            a = o['args']
            plan.layers.append(dict(op='maxpool', input=o['inputs'][0], output=o['outputs'][0],
                                    k=a['kernel'], stride=a['stride'], pad=a.get('pad', 0)))
            i += 1
            continue
        if t == 'Split':
            # uniform partition + part power set (bpm_heads.py:18-55, pps_heads.py:38-80)
            src = o['inputs'][0]
            strips = o['outputs']
            preprefix = strips[0][:-len('0_strip')]
            j = i + 1
            has_max = False
            prefixes = []
            while j < n and ops_[j]['type'] in ('AveragePool', 'MaxPool', 'Mean', 'Max', 'Add'):
                if ops_[j]['type'] == 'MaxPool':
                    has_max = True
                if ops_[j]['type'] == 'Add':
                    prefixes.append(ops_[j]['outputs'][0][:-len('_pool2')])
                if ops_[j]['type'] == 'Max' and not has_max:
                    # Max-only variant (MAX_AVE_FEATURE off, pps_heads.py:70-76)
                    prefixes.append(ops_[j]['outputs'][0][:-len('_pool2')])
                j += 1
            dim = shapes[prefixes[0] + '_conv_w'][1]
            pooled.update(p + '_pool2' for p in prefixes)
            plan.layers.append(dict(op='pps', input=src, output=preprefix + '_pool2_all',
                                    split=list(o['args']['split']), max_ave=has_max,
                                    prefixes=prefixes, dim=dim))
            i = j
            continue
        if t in ('Concat', 'Reshape', 'Normalize', 'FC'):
            break
        raise RuntimeError('compile_graph: no fusion rule for op %s at %d (%s)'
                           % (t, i, o['outputs']))
    if pending:
        raise RuntimeError('compile_graph: conv+BN without consumer: %s' % sorted(pending))
    # reid heads (reid_heads.py:34-127): Conv(bias)+BN+Relu[+FC] per prefix,
    # Concat of the *_bn blobs, Reshape, Normalize
    pps = [L for L in plan.layers if L['op'] == 'pps'][-1]
    prefixes, dim_inner, out, norm = [], None, None, None
    while i < n:
        o = ops_[i]
        t = o['type']
        if t == 'Conv':
            p = o['outputs'][0][:-len('_conv')]
            prefixes.append(p)
            dim_inner = shapes[o['inputs'][1]][0]
            for s in ('_w', '_b'):
                plan.params[p + '_conv' + s] = shapes[p + '_conv' + s]
            for s in ('_s', '_b', '_rm', '_riv'):
                plan.params[p + '_bn' + s] = shapes[p + '_bn' + s]
        elif t == 'Reshape':
            out = o['outputs'][0]
        elif t == 'Normalize':
            norm = o
        i += 1
    if prefixes != pps['prefixes']:
        raise RuntimeError('compile_graph: head order %s != part subsets %s'
                           % (prefixes[:3], pps['prefixes'][:3]))
    plan.layers.append(dict(op='heads', input=pps['output'], prefixes=prefixes,
                            dim=pps['dim'], dim_inner=dim_inner, output=out))
    if norm is not None:
        plan.layers.append(dict(op='normalize', input=norm['inputs'][0],
                                output=norm['outputs'][0]))
    plan.output = graph['output']
    plan.spatial_scale = graph.get('spatial_scale')
    plan.feat_dim = len(prefixes) * dim_inner
    return plan


# ---------------------------------------------------------------------------
# Net
# ---------------------------------------------------------------------------
class Net(object):
    """A recorded reference test net + its weights on the device."""

    def __init__(self, graph, blobs, device='cuda'):
        if isinstance(graph, str):
            with open(graph) as f:
                graph = json.load(f)
        self.graph = graph
        self.blobs = blobs
        self.device = torch.device(device)
        self._dev_params = None
        self._model = None

    def compile(self):
        return compile_graph(self.graph)

    def forward(self, x, out=None):
        """Fused execution (the product path): bit-identical to PPSModel."""
        if self._model is None:
            self._model = pmodel.PPSModel(self.blobs, device=self.device, plan=self.compile())
        return self._model.forward(x, out=out)

    def run_eager(self, x, keep=(), skip_fc=True):
        """Op-by-op execution through OPS (unfused, exact-f32 GEMMs)."""
        if self._dev_params is None:
            self._dev_params = {k: torch.from_numpy(np.ascontiguousarray(v, np.float32))
                                .to(self.device) for k, v in self.blobs.items()}
        ws = dict(self._dev_params)
        ws['data'] = x
        kept = {}
        for o in self.graph['ops']:
            t = o['type']
            if skip_fc and (t == 'FC' or (t in ('Concat', 'Reshape')
                                          and o['outputs'][0].startswith('reid_fc'))):
                continue    # logits never fetched at test (reid_heads.py:84-120)
            outs = run_op(t, [ws[name] for name in o['inputs']], **o['args'])
            for name, val in zip(o['outputs'], outs):
                ws[name] = val
                if name in keep:
                    kept[name] = val
        out = ws[self.graph['output']]
        return (out, kept) if keep else out
