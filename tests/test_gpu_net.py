"""The reference's recorded test net through the operator registry
(pps_amd/net.py): every registered op vs the oracle's restatement of the
Caffe2 op (oracle/forward.py) on random inputs; the whole net op by op
(unfused, eager) vs the oracle forward; and the compiled net bit-identical
to PPSModel."""
import json
import os

import numpy as np
import pytest
import torch

from oracle.forward import GraphForward

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def _cuda(x):
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()


def _nhwc(x):
    return _cuda(np.asarray(x).transpose(0, 2, 3, 1))


def _nchw(t):
    return t.cpu().numpy().transpose(0, 3, 1, 2)


def _ref(op, xs, **a):
    return [v.numpy() for v in GraphForward._run(op, [torch.from_numpy(np.asarray(x))
                                                      for x in xs], a)]


def test_registry_conv_spatialbn_relu_sum():
    from pps_amd import net
    rng = np.random.RandomState(0)
    x = rng.randn(2, 32, 9, 7).astype(np.float32)
    w = (rng.randn(24, 32, 3, 3) / 17).astype(np.float32)
    b = rng.randn(24).astype(np.float32)
    y = net.run_op('Conv', [_nhwc(x), _cuda(w), _cuda(b)], kernel=3, stride=2, pad=1,
                   dilation=1, group=1)[0]
    ref = _ref('Conv', [x, w, b], kernel=3, stride=2, pad=1, dilation=1, group=1)[0]
    np.testing.assert_allclose(_nchw(y), ref, rtol=1e-5, atol=1e-5)
    s, bb, rm = (rng.randn(24).astype(np.float32) for _ in range(3))
    riv = rng.uniform(0.5, 1.5, 24).astype(np.float32)
    z = net.run_op('SpatialBN', [y, _cuda(s), _cuda(bb), _cuda(rm), _cuda(riv)],
                   epsilon=1e-5, is_test=1)[0]
    zr = _ref('SpatialBN', [_nchw(y), s, bb, rm, riv], epsilon=1e-5)[0]
    np.testing.assert_allclose(_nchw(z), zr, rtol=1e-6, atol=1e-6)
    r = net.run_op('Relu', [z])[0]
    np.testing.assert_array_equal(_nchw(r), np.maximum(_nchw(z), 0))
    for op in ('Sum', 'Add', 'Max', 'Mean'):
        xs = [rng.randn(3, 5, 2, 2).astype(np.float32) for _ in range(3)]
        got = net.run_op(op, [_nhwc(v) for v in xs])[0]
        want = _ref(op, xs)[0]
        np.testing.assert_allclose(_nchw(got), want, rtol=0, atol=1e-6, err_msg=op)


def test_registry_pools_split_fc_concat_normalize():
    from pps_amd import net
    rng = np.random.RandomState(1)
    x = rng.randn(2, 16, 24, 8).astype(np.float32)
    strips = net.run_op('Split', [_nhwc(x)], axis=2, split=[5, 5, 4, 5, 5])
    rs = _ref('Split', [x], axis=2, split=[5, 5, 4, 5, 5])
    for s, r in zip(strips, rs):
        for op in ('AveragePool', 'MaxPool'):
            got = net.run_op(op, [s], global_pooling=True)[0]
            want = _ref(op, [r], global_pooling=True)[0]
            np.testing.assert_allclose(_nchw(got), want, rtol=1e-6, atol=1e-6)
    mp = net.run_op('MaxPool', [_nhwc(x)], kernel=3, stride=2, pad=1)[0]
    np.testing.assert_array_equal(_nchw(mp), _ref('MaxPool', [x], kernel=3, stride=2, pad=1)[0])
    f = rng.randn(4, 64, 1, 1).astype(np.float32)
    w = rng.randn(10, 64).astype(np.float32)
    b = rng.randn(10).astype(np.float32)
    got = net.run_op('FC', [_nhwc(f), _cuda(w), _cuda(b)])[0]
    np.testing.assert_allclose(got.cpu().numpy(), _ref('FC', [f, w, b])[0], rtol=1e-5,
                               atol=1e-5)
    parts = [rng.randn(4, 8, 1, 1).astype(np.float32) for _ in range(3)]
    cat, info = net.run_op('Concat', [_nhwc(p) for p in parts], axis=1)
    flat = net.run_op('Reshape', [cat], shape=[1, -1])[0]
    want = _ref('Reshape', [_ref('Concat', parts, axis=1)[0]], shape=[1, -1])[0]
    np.testing.assert_array_equal(flat.cpu().numpy(), want)
    assert info.tolist() == [8, 8, 8]
    nrm = net.run_op('Normalize', [flat], axis=1)[0]
    np.testing.assert_allclose(nrm.cpu().numpy(), _ref('Normalize', [want], axis=1)[0],
                               rtol=1e-6, atol=1e-7)


def _setup(seed=0, n=2):
    from pps_amd import config, model
    config.merge_cfg_from_file(os.path.join(GOLDEN, '..', '..', 'configs', 'market1501',
                                            'pps_crm_triplet_R-50_1x.yaml'))
    with open(os.path.join(GOLDEN, 'pps_graph_market1501.json')) as f:
        g = json.load(f)
    blobs = model.synthetic_weights(model.build_plan(), seed=seed)
    rng = np.random.RandomState(seed)
    x = (rng.randn(n, 3, 384, 128) * 50).astype(np.float32)
    xin = np.zeros((n, 384, 128, 4), np.float32)
    xin[..., :3] = x.transpose(0, 2, 3, 1)
    return g, blobs, x, _cuda(xin)


def test_compiled_net_bit_identical_to_ppsmodel():
    from pps_amd import model, net
    g, blobs, _, xin = _setup()
    a = net.Net(g, blobs).forward(xin).clone()
    b = model.PPSModel(blobs).forward(xin)
    assert torch.equal(a, b)


def test_eager_net_vs_oracle():
    """The recorded net op by op through the registry (384 live ops, exact
    f32 GEMMs, SpatialBN as its own pass) vs the oracle forward."""
    from pps_amd import net
    g, blobs, x, xin = _setup(seed=1)
    out, kept = net.Net(g, blobs).run_eager(xin, keep=('res5_2_sum', 'pps013_pool2'))
    ref, rk = GraphForward(blobs)(x, keep=('res5_2_sum', 'pps013_pool2'))
    for name in ('res5_2_sum', 'pps013_pool2'):
        got, want = _nchw(kept[name]), rk[name].numpy()
        err = np.abs(got - want).max() / max(1e-6, np.abs(want).max())
        print('eager net %s max|err| / max|ref| = %.3g' % (name, err))
        assert err < 1e-5, (name, err)
    err = float(np.abs(out.cpu().numpy() - ref.numpy()).max())
    print('eager net forward max|err| vs oracle %.3g' % err)
    assert err <= 1e-6
