"""Record the reference's PPS test-time net as a JSON op graph.

Run in the build container only (needs /root/reference):

    python tests/golden/record_graph.py

The reference's own graph builders are imported UNCHANGED from
/root/reference/detectron (ResNet.py, pps_heads.py, bpm_heads.py,
reid_heads.py, core/config.py) and driven with a *recording model*: an object
that exposes the model-helper methods those builders call
(Conv / SpatialBN / Relu / MaxPool / AveragePool / FC / ConvAffine /
AffineChannel, and `net.<OpName>(...)`), and that appends one record per op.

Caffe2 is not installed here, so caffe2.*, cv2 and a few
detectron.utils modules are stubbed; the stubs only satisfy imports.  The
ConvAffine / AffineChannel methods restate detector.py:82-84,419-447 (with
MODEL.USE_BN the affine becomes a test-mode SpatialBN).  Caffe2 parameter
naming (`<blob>_w`, `<blob>_b`; BN `<blob>_{s,b,rm,riv}`) follows the
brew helpers, matching tools/pickle_caffe_blobs_keep_bn.py:75-88,141-159.

Output: tests/golden/pps_graph_<cfgname>.json = {cfg, ops: [...], params: {...},
output}.  It pins STRUCTURE (op types, order, blob names, args, param shapes),
not arithmetic.
"""
import json
import os
import sys
import types

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))


def _stub(name, **attrs):
    m = sys.modules.get(name) or types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def install_stubs():
    import yaml
    _stub('future')
    _stub('future.utils', iteritems=lambda d: iter(d.items()))
    _stub('cv2')
    for n in ['caffe2', 'caffe2.python', 'caffe2.proto']:
        _stub(n)
    _stub('caffe2.python.workspace')
    _stub('caffe2.python.core')
    _stub('caffe2.proto.caffe2_pb2')
    sys.modules['caffe2.python'].workspace = sys.modules['caffe2.python.workspace']
    sys.modules['caffe2.python'].core = sys.modules['caffe2.python.core']
    sys.modules['caffe2.proto'].caffe2_pb2 = sys.modules['caffe2.proto.caffe2_pb2']
    sys.path.insert(0, REF)
    import detectron  # noqa: F401  (the real package dir)
    import detectron.utils  # noqa: F401
    _stub('detectron.utils.net', get_group_gn=lambda d: 32)
    _stub('detectron.utils.c2', const_fill=lambda v: ('ConstantFill', {'value': v}),
          gauss_fill=lambda s: ('GaussianFill', {'std': s}),
          UnscopeName=lambda s: s.split('/')[-1])
    _stub('detectron.utils.boxes')
    _stub('detectron.modeling.generate_anchors', generate_anchors=lambda **k: None)
    import detectron.utils.env as envu
    envu.yaml_load = lambda s: yaml.load(s, Loader=yaml.Loader)


class Net(object):
    def __init__(self, rec):
        self._rec = rec

    def __getattr__(self, op):
        def fn(inputs, outputs, **args):
            return self._rec.add(op, inputs, outputs, args)
        return fn


class RecordingModel(object):
    def __init__(self, num_classes):
        self.train = False
        self.num_classes = num_classes
        self.ops = []
        self.params = {}
        self.net = Net(self)

    # -- generic op record --------------------------------------------------
    def add(self, op, inputs, outputs, args):
        ins = [str(i) for i in (inputs if isinstance(inputs, (list, tuple)) else [inputs])]
        outs = [str(o) for o in (outputs if isinstance(outputs, (list, tuple)) else [outputs])]
        clean = {}
        for k, v in args.items():
            if isinstance(v, tuple):
                v = list(v)
            if isinstance(v, (int, float, str, bool, list)) or v is None:
                clean[k] = v
        self.ops.append(dict(type=op, inputs=ins, outputs=outs, args=clean))
        return outs[0] if len(outs) == 1 else tuple(outs)

    def param(self, name, shape):
        self.params[name] = list(shape)
        return name

    # -- model-helper surface used by the builders ---------------------------
    def Conv(self, blob_in, blob_out, dim_in, dim_out, kernel, stride=1, pad=0,
             dilation=1, group=1, no_bias=0, weight_init=None, bias_init=None,
             **kw):
        w = self.param(blob_out + '_w', [dim_out, dim_in // group, kernel, kernel])
        ins = [blob_in, w]
        if not no_bias:
            ins.append(self.param(blob_out + '_b', [dim_out]))
        return self.add('Conv', ins, blob_out,
                        dict(kernel=kernel, stride=stride, pad=pad,
                             dilation=dilation, group=group))

    def SpatialBN(self, blob_in, blob_out, dim, is_test=True, **kw):
        ps = [self.param(blob_out + s, [dim]) for s in ('_s', '_b', '_rm', '_riv')]
        return self.add('SpatialBN', [blob_in] + ps, blob_out,
                        dict(is_test=1, epsilon=kw.get('epsilon', 1e-5)))

    def AffineChannel(self, blob_in, blob_out, dim, inplace=False):
        # detector.py:82-84 -- MODEL.USE_BN => SpatialBN(is_test)
        return self.SpatialBN(blob_in, blob_out, dim, is_test=True)

    def ConvAffine(self, blob_in, prefix, dim_in, dim_out, kernel, stride, pad,
                   group=1, dilation=1, weight_init=None, bias_init=None,
                   suffix='_bn', inplace=False):
        # detector.py:419-447
        c = self.Conv(blob_in, prefix, dim_in, dim_out, kernel, stride=stride,
                      pad=pad, group=group, dilation=dilation, no_bias=1)
        return self.AffineChannel(c, prefix + suffix, dim_out, inplace=inplace)

    def Relu(self, blob_in, blob_out):
        return self.add('Relu', [blob_in], blob_out, {})

    def MaxPool(self, blob_in, blob_out, **args):
        return self.add('MaxPool', [blob_in], blob_out, args)

    def AveragePool(self, blob_in, blob_out, **args):
        return self.add('AveragePool', [blob_in], blob_out, args)

    def FC(self, blob_in, blob_out, dim_in, dim_out, weight_init=None,
           bias_init=None, **kw):
        w = self.param(blob_out + '_w', [dim_out, dim_in])
        b = self.param(blob_out + '_b', [dim_out])
        return self.add('FC', [blob_in, w, b], blob_out, {})

    def DropoutIfTraining(self, blob_in, dropout_rate):
        return blob_in

    def StopGradient(self, blob_in, blob_out):
        return blob_out


def record(cfg_file, overrides=()):
    from detectron.core.config import cfg, merge_cfg_from_file, merge_cfg_from_list
    merge_cfg_from_file(cfg_file)
    if overrides:
        merge_cfg_from_list(list(overrides))
    import detectron.modeling.ResNet as ResNet
    import detectron.modeling.pps_heads as pps_heads
    import detectron.modeling.reid_heads as reid_heads
    reid_heads.feature_list[:] = []
    reid_heads.fc_list[:] = []
    m = RecordingModel(cfg.MODEL.NUM_CLASSES)
    import io
    import contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        if cfg.FPN.FPN_ON:
            import detectron.modeling.FPN_reid as FPN_reid
            body = cfg.MODEL.CONV_BODY.split('.')[-1]
            blob, dim, scale = getattr(FPN_reid, body)(m)
        else:
            blob, dim, scale = ResNet.add_ResNet50_conv5_body(m)
        blobs, dims = pps_heads.add_pps_part_head(m, blob, dim, scale)
        reid_heads.add_reid_outputs(m, blobs, dims)
    out = 'reid_feature_concat_norm' if cfg.REID.NORMALIZE_FEATURE else 'reid_feature_concat'
    keys = dict(
        SCALE=list(cfg.REID.SCALE), BPM_STRIP_NUM=cfg.REID.BPM_STRIP_NUM,
        BPM_DIM=cfg.REID.BPM_DIM, MAX_AVE_FEATURE=bool(cfg.REID.MAX_AVE_FEATURE),
        NORMALIZE_FEATURE=bool(cfg.REID.NORMALIZE_FEATURE),
        RES5_STRIDE=cfg.RESNETS.RES5_STRIDE, STRIDE_1X1=bool(cfg.RESNETS.STRIDE_1X1),
        USE_BN=bool(cfg.MODEL.USE_BN), NUM_CLASSES=cfg.MODEL.NUM_CLASSES,
        PIXEL_MEANS=[float(v) for v in cfg.PIXEL_MEANS.ravel()],
        FPN_ON=bool(cfg.FPN.FPN_ON))
    keys['CONV_BODY'] = cfg.MODEL.CONV_BODY
    keys['FPN_DIM'] = cfg.FPN.DIM
    return dict(cfg_file=os.path.relpath(cfg_file, REF), cfg=keys, ops=m.ops,
                params=m.params, output=out,
                spatial_scale=scale if not isinstance(scale, (list, tuple)) else list(scale),
                overrides=list(overrides))


def main():
    install_stubs()
    from collections import Counter
    from detectron.core.config import cfg
    import copy
    pristine = copy.deepcopy(cfg)
    cases = [('pps_graph_market1501.json', ()),
             # config-gated FPN_reid variant; not in a shipped config
             ('pps_graph_market1501_fpn.json',
              ('FPN.FPN_ON', 'True', 'MODEL.CONV_BODY', 'FPN_reid.add_fpn_ResNet50_conv5_body'))]
    for name, over in cases:
        cfg.clear()
        cfg.update(copy.deepcopy(pristine))
        g = record(os.path.join(REF, 'configs/market1501/pps_crm_triplet_R-50_1x.yaml'), over)
        path = os.path.join(HERE, name)
        with open(path, 'w') as f:
            json.dump(g, f, indent=0, sort_keys=True)
        c = Counter(o['type'] for o in g['ops'])
        print(path, len(g['ops']), 'ops', dict(c), len(g['params']), 'params')


if __name__ == '__main__':
    main()
