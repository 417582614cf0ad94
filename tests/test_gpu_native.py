"""The whole-network C entry point (pps_model_create / pps_forward, include/
pps_abi.h) against the Python orchestrator (bit for bit, same tuning table)
and the CPU oracle (tight bound): the forward a C/C++ caller gets through the
ABI with no pps_amd/model.py orchestration."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FWD_ATOL = 1e-6   # normalised features vs the oracle (observed ~6e-8)


def _market_cfg():
    from tests.test_gpu_forward import _market_cfg as f
    return f()


def _models(seed=0, **kw):
    from pps_amd import model, native
    _market_cfg()
    plan = model.build_plan()
    blobs = model.synthetic_weights(plan, seed=seed)
    return blobs, model.PPSModel(blobs, plan=plan, **kw), native.NativeModel(blobs, **kw)


def _input(N, seed=0):
    rng = np.random.RandomState(seed)
    x = (rng.randn(N, 3, 384, 128) * 50).astype(np.float32)
    xin = np.zeros((N, 384, 128, 4), np.float32)
    xin[..., :3] = x.transpose(0, 2, 3, 1)
    return x, torch.from_numpy(xin).cuda()


def test_native_plan_matches_python():
    """Same layers, names, ops, FLOPs, bytes and default plane edges as the
    Python orchestrator (both mirror the reference builders)."""
    _, pm, nm = _models()
    _, x = _input(2)
    pm.forward(x)
    nl = nm.layers(N=2)
    assert [L.get('name', L['output']) for L in pm.layers] == [L['name'] for L in nl]
    assert [L['op'] for L in pm.layers] == [L['op'] for L in nl]
    for a, b in zip(pm.layers, nl):
        assert a['flops'] == pytest.approx(b['flops'], rel=1e-12), b['name']
        assert a['bytes'] == pytest.approx(b['bytes'], rel=1e-12), b['name']
    assert sorted(pm.planes()) == sorted(nm.planes())
    assert len(nm.plane_edges()) == len(pm._edges)
    assert nm.feat_dim == pm.feat_dim == 3968


@pytest.mark.parametrize('math', ['x3', 'f32'])
def test_native_forward_bit_identical_and_vs_oracle(math):
    from oracle.forward import GraphForward
    blobs, pm, nm = _models(math=math)
    x, xd = _input(3)
    a = pm.forward(xd).cpu().numpy()
    b = nm.forward(xd).cpu().numpy()
    assert np.array_equal(a, b)
    ref = GraphForward(blobs)(x).numpy()
    err = float(np.abs(b - ref).max())
    print('native forward (%s) max|err| vs oracle %.3g' % (math, err))
    assert err <= FWD_ATOL


def test_native_fused_splitk_layers():
    """Split-K on FIX tiles (one launch, tile counters in the workspace,
    plain and chunk-tiled weights, plane edges in and out) in the C plan
    equals the Python orchestrator bit for bit, and a captured graph replays
    it to the same bits (the counters come back to zero every launch)."""
    from pps_amd import ops
    _, pm, nm = _models()
    _, x = _input(4, seed=3)
    base = nm.forward(x).cpu().numpy()
    tiles, sks = {}, {}
    fix = [t for t in ops.FIX_TILES]
    for i, L in enumerate(pm.layers):
        if L['op'] == 'conv' and L['name'][:4] in ('res4', 'res5') and L['relu']:
            sk = 2 if L['kpad'] % 64 == 0 else 1
            if sk == 1:
                continue
            sks[L['name']] = sk
            tiles[L['name']] = fix[i % len(fix)] | (ops.TILE_B_TILED if i % 2 else 0)
    assert sks
    pm.set_tiles(tiles)
    pm.set_planes([n for n in ('res4_1_branch2a', 'res5_1_branch2a') if n in sks])
    pm.set_splitks(sks)
    nm.apply_table(pm)
    assert nm.splitks() == sks
    a = pm.forward(x).cpu().numpy()
    b = nm.forward(x).cpu().numpy()
    assert np.array_equal(a, b)
    np.testing.assert_allclose(b, base, rtol=0, atol=2e-5)
    nm.reserve(4)
    out = torch.empty((4, nm.feat_dim), device='cuda')
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        nm.forward(x, out=out)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), b)


def test_native_graph_capture():
    """pps_forward is stream-ordered and capturable once N is reserved."""
    _, pm, nm = _models()
    _, x = _input(4, seed=1)
    nm.reserve(4)
    out = torch.empty((4, nm.feat_dim), device='cuda')
    nm.forward(x, out=out)
    torch.cuda.synchronize()
    want = out.clone()
    out.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        nm.forward(x, out=out)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, want)


def test_native_autotune_then_python_twin():
    """The C autotune fills the table; the Python orchestrator given that
    table computes the same bits."""
    _, pm, nm = _models(seed=1)
    _, x = _input(2, seed=2)
    tiles = nm.autotune(x)
    from pps_amd import ops
    assert all(0 <= (t & ~ops.TILE_FLAGS) <= ops.num_tiles()
               for t in tiles.values())
    assert any(t != 0 for t in tiles.values())
    pm.set_tiles(tiles)
    pm.set_planes(nm.planes())
    assert np.array_equal(pm.forward(x).cpu().numpy(), nm.forward(x).cpu().numpy())


def test_native_intermediate_tensor_and_layer_range():
    _, pm, nm = _models(fused_pps=False)
    _, x = _input(2, seed=3)
    pm.forward(x)
    nm.forward(x)
    torch.cuda.synchronize()
    for name in ('pool1', 'res3_3_sum', 'res5_2_sum'):
        assert np.array_equal(pm.buffers()[name].cpu().numpy(), nm.tensor(2, name)), name
    # layers [0, n) in two ranges == one forward
    n = len(nm.layers())
    a = nm.forward(x).clone()
    nm.forward_layers(x, 0, n // 2)
    b = nm.forward_layers(x, n // 2, n)
    assert torch.equal(a, b)


def test_native_fpn_variant_bit_identical():
    from pps_amd import config, model, native
    _market_cfg()
    config.merge_cfg_from_list(['FPN.FPN_ON', 'True', 'MODEL.CONV_BODY',
                                'FPN_reid.add_fpn_ResNet50_conv5_body'])
    try:
        plan = model.build_plan()
        blobs = model.synthetic_weights(plan, seed=3)
        pm = model.PPSModel(blobs, plan=plan)
        nm = native.NativeModel(blobs)
        _, x = _input(2, seed=4)
        assert [L['name'] for L in nm.layers()][-3].startswith('fpn_inner_')
        assert np.array_equal(pm.forward(x).cpu().numpy(), nm.forward(x).cpu().numpy())
    finally:
        config.merge_cfg_from_list(['FPN.FPN_ON', 'False', 'MODEL.CONV_BODY',
                                    'ResNet.add_ResNet50_conv5_body'])


def test_native_errors_are_enforce_style():
    from pps_amd import model, native
    _market_cfg()
    plan = model.build_plan()
    blobs = model.synthetic_weights(plan, seed=0)
    bad = dict(blobs)
    bad['res2_0_branch2a_w'] = bad['res2_0_branch2a_w'][:10]
    with pytest.raises(RuntimeError, match='res2_0_branch2a_w has'):
        native.NativeModel(bad)
    missing = dict(blobs)
    del missing['res4_3_branch2b_bn_riv']
    with pytest.raises(RuntimeError, match='weights missing 1 blobs'):
        native.NativeModel(missing)
    nm = native.NativeModel(blobs)
    with pytest.raises(RuntimeError, match='no layer named'):
        native.call('pps_model_set_tile', nm.handle, b'res9_branch2a', 3)
    with pytest.raises(RuntimeError, match='not a plane-eligible producer'):
        native.call('pps_model_set_planes', nm.handle, b'res2_0_branch2c', 1)
    with pytest.raises(ValueError, match='not a plane-eligible producer'):
        nm.set_planes(['res2_0_branch2c'])


def test_reserved_buffers_are_pinned():
    """after pps_model_reserve(N) a tuning change that needs
    larger split-K buffers must fail (a captured graph may still address the
    old ones) instead of reallocating; release + reserve re-enables it."""
    _, pm, nm = _models()
    _, x = _input(2, seed=5)
    nm.reserve(2)
    nm.forward(x)
    torch.cuda.synchronize()
    L = next(L for L in nm.layers(N=2) if L['op'] == 'conv' and L['name'].startswith('res5')
             and L['name'].endswith('branch2b'))
    nm.set_splitks({L['name']: 2})
    with pytest.raises(RuntimeError, match='pinned by pps_model_reserve'):
        nm.forward(x)
    nm.release(2)
    nm.reserve(2)
    out = nm.forward(x)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(out).all())


def test_bottleneck_seam_in_the_plan():
    """PPS_TILE_SEAM on res2_1 / res3_1 branch2c: one launch computes it and
    the next block's branch2a -- the same bits as the two layers on the
    16x16x32 group tiles (54 and 38), in the C plan and the Python twin; the
    flag is refused on a layer that is not such a pair, and eager ranges
    that split a pair still compute both layers."""
    from pps_amd import ops
    _, pm, nm = _models()
    _, x = _input(2)
    base = dict(nm.tiles())
    base.update({'res2_1_branch2c': 54, 'res2_2_branch2a': 38,
                 'res3_1_branch2c': 54, 'res3_2_branch2a': 38})
    nm.set_tiles(base)
    pm.set_tiles(base)
    ref = nm.forward(x).cpu().numpy()
    seam = dict(base)
    for k in ('res2_1_branch2c', 'res3_1_branch2c'):
        seam[k] = 54 | ops.TILE_SEAM
    nm.set_tiles(seam)
    pm.set_tiles(seam)
    assert nm.tiles()['res2_1_branch2c'] == 54 | ops.TILE_SEAM
    assert np.array_equal(nm.forward(x).cpu().numpy(), ref)
    assert np.array_equal(pm.forward(x).cpu().numpy(), ref)
    # a range ending at the seam layer, then one starting at its branch2a
    names = [L['name'] for L in nm.layers(2)]
    i = names.index('res2_1_branch2c')
    out = torch.empty((2, nm.feat_dim), dtype=torch.float32, device='cuda')
    nm.forward_layers(x, 0, i + 1, out=out)
    nm.forward_layers(x, i + 1, len(names), out=out)
    assert np.array_equal(out.cpu().numpy(), ref)
    with pytest.raises(RuntimeError, match='PPS_TILE_SEAM'):
        nm.set_tiles({'res2_0_branch2c': 54 | ops.TILE_SEAM})   # projection block (dual)
    with pytest.raises(RuntimeError, match='PPS_TILE_SEAM'):
        nm.set_tiles({'res4_1_branch2c': 54 | ops.TILE_SEAM})   # (256, 1024, 256): no kernel
