"""ORACLE (test infrastructure only) -- CPU fp32 restatement of the
reference's PPS test-time forward.

It interprets the op graph that tests/golden/record_graph.py recorded by
driving the reference's own graph builders (ResNet.py, pps_heads.py,
bpm_heads.py, reid_heads.py), so the STRUCTURE (op order, blob names, Split
sizes, subset order, conv args, param names) is the reference's.  Each op is
restated with the Caffe2 (pytorch v1.0.1) NCHW semantics the reference ran on
(third-party arithmetic, parity unpinned by any reference test: SURVEY §8(c)):

  Conv         zero padding, cross-correlation, optional bias
  SpatialBN    is_test: (x - rm) * s / sqrt(riv + eps) + b, eps = 1e-5
  Relu, Sum, Add, Max (elementwise), Mean (sum in input order, * 1/n)
  MaxPool      kernel/stride/pad, floor output size; global_pooling
  AveragePool  global_pooling = mean over H x W
  Split        axis 2 by `split`
  FC           x W^T + b        Concat axis 1        Reshape [1,-1] -> [N,-1]
  Normalize    x / max(||x||_2, 1e-12) along axis 1
  UpsampleNearest  integer nearest-neighbour upsampling (FPN top-down path)

torch on CPU is used as the fp32 array library.  Only tests/, smoke() and
bench.py's cpu_baseline may use this module.
"""
import json
import os

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
GRAPH = os.path.join(HERE, '..', 'tests', 'golden', 'pps_graph_market1501.json')


def load_graph(path=GRAPH):
    with open(path) as f:
        return json.load(f)


class GraphForward(object):
    def __init__(self, blobs, graph=None, skip_fc=True, threads=None):
        self.g = graph or load_graph()
        self.params = {k: torch.from_numpy(np.ascontiguousarray(v, np.float32))
                       for k, v in blobs.items()}
        self.skip_fc = skip_fc
        if threads:
            torch.set_num_threads(threads)

    def __call__(self, data_nchw, keep=()):
        """data_nchw: float32 [N,3,H,W] (BGR minus means).  Returns the output
        blob (and any blobs named in `keep`)."""
        ws = {'data': torch.as_tensor(data_nchw, dtype=torch.float32)}
        ws.update(self.params)
        kept = {}
        with torch.no_grad():
            for op in self.g['ops']:
                t = op['type']
                if t == 'FC' and self.skip_fc:
                    continue  # logits never fetched at test (reid_heads.py:84-120)
                if t == 'Concat' and op['outputs'][0].startswith('reid_fc'):
                    continue
                if t == 'Reshape' and op['outputs'][0].startswith('reid_fc'):
                    continue
                outs = self._run(t, [ws[i] for i in op['inputs']], op['args'])
                for name, val in zip(op['outputs'], outs):
                    ws[name] = val
                    if name in keep:
                        kept[name] = val.clone()
        out = ws[self.g['output']]
        return (out, kept) if keep else out

    @staticmethod
    def _run(t, x, a):
        if t == 'Conv':
            b = x[2] if len(x) > 2 else None
            return [F.conv2d(x[0], x[1], b, stride=a['stride'], padding=a['pad'],
                             dilation=a['dilation'], groups=a['group'])]
        if t == 'SpatialBN':
            inp, s, b, rm, riv = x
            inv = s / torch.sqrt(riv + a.get('epsilon', 1e-5))
            shape = (1, -1) + (1,) * (inp.dim() - 2)
            return [(inp - rm.view(shape)) * inv.view(shape) + b.view(shape)]
        if t == 'Relu':
            return [torch.clamp_min(x[0], 0)]
        if t in ('Sum', 'Add'):
            acc = x[0]
            for v in x[1:]:
                acc = acc + v
            return [acc]
        if t == 'Max':
            acc = x[0]
            for v in x[1:]:
                acc = torch.maximum(acc, v)
            return [acc]
        if t == 'Mean':
            acc = x[0]
            for v in x[1:]:
                acc = acc + v
            return [acc * (1.0 / len(x))]
        if t == 'MaxPool':
            if a.get('global_pooling'):
                return [torch.amax(x[0], dim=(2, 3), keepdim=True)]
            return [F.max_pool2d(x[0], a['kernel'], a['stride'], a.get('pad', 0))]
        if t == 'AveragePool':
            assert a.get('global_pooling')
            return [torch.mean(x[0], dim=(2, 3), keepdim=True)]
        if t == 'Split':
            return list(torch.split(x[0], a['split'], dim=a['axis']))
        if t == 'FC':
            inp = x[0].reshape(x[0].shape[0], -1)
            return [inp @ x[1].t() + x[2]]
        if t == 'Concat':
            cat = torch.cat(x, dim=a['axis'])
            return [cat, torch.tensor([v.shape[a['axis']] for v in x])]
        if t == 'Reshape':
            return [x[0].reshape(x[0].shape[0], -1), torch.tensor(a['shape'])]
        if t == 'UpsampleNearest':
            return [F.interpolate(x[0], scale_factor=a['scale'], mode='nearest')]
        if t == 'Normalize':
            v = x[0]
            n = torch.sqrt(torch.sum(v * v, dim=1, keepdim=True))
            return [v / torch.clamp_min(n, 1e-12)]
        raise NotImplementedError(t)


def param_shapes(graph=None):
    g = graph or load_graph()
    return {k: tuple(v) for k, v in g['params'].items()}
