"""The f16x2 ("h2") convolutions (EPI_F_H2 tiles of gemm_x3p.hip / gemm_x3c.hip,
include/pps_abi.h "f16x2 convolutions"):

* error: against an fp64 reference the h2 kernels' max error stays within
  H2_VS_X3 x the bf16x3 kernel's on the same data (the x3 kernels are held
  to 4x the exact-f32 MFMA kernel's in test_gpu_x3.py) -- f32-level, far
  from f16 (~5e-4) -- also for inputs scaled by 1e-20 / 1e20 (the per-tensor
  power-of-two scale keeps them inside the f16 range);
* every tile of a rounding group gives the same bits (16x16x32 pipelined
  38..55; patch tiles 56..59 run K in (channel chunk, tap) order);
* amax_y is max|y| exactly, and the activation max every producer reports
  (x3 tiles, the weight-stationary tile, the fused stem, max pooling) equals
  max|y| of its output.
"""
import numpy as np
from _tiles import check_tile_bits
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

H2_VS_X3 = 3.0       # max error of h2 <= H2_VS_X3 * max error of x3 (+ floor)
ERR_FLOOR = 2e-7     # relative to max |ref|


def _cuda(x):
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()


def _rel_err(got, ref):
    return float(np.abs(got.astype(np.float64) - ref).max() / max(1e-30, np.abs(ref).max()))


def _h2_tiles():
    # (54: the weight-stationary 1x1 kernel where it applies, else tile 38)
    from pps_amd import ops
    return [0] + list(range(ops.TILE_P16_FIRST, ops.num_tiles() + 1))


_SHAPES = [
    (2, 24, 8, 256, 256, 3, 1, 1),     # res4 branch2b (patch tiles apply)
    (1, 24, 8, 512, 512, 3, 1, 1),     # res5 branch2b
    (2, 24, 8, 1024, 256, 1, 1, 0),    # res4 branch2a
    (2, 48, 16, 256, 128, 1, 2, 0),    # strided 1x1 (STRIDE_1X1 branch2a)
    (2, 96, 32, 64, 64, 3, 1, 1),      # res2 branch2b
    (3, 7, 5, 64, 40, 3, 1, 1),        # ragged M and N
    # the f16x2 weight-stationary 1x1 shapes (tile 54): res2 2c / 2a, res3 2c,
    # res4 2c, and a ragged row count
    (1, 96, 32, 64, 256, 1, 1, 0),
    (1, 96, 32, 256, 64, 1, 1, 0),
    (2, 48, 16, 128, 512, 1, 1, 0),
    (2, 24, 8, 256, 1024, 1, 1, 0),
    (3, 7, 5, 128, 192, 1, 1, 0),
]
# every shape with and without the residual at unit magnitude, plus the
# magnitude sweep (inputs x 1e-20 and x 1e20) on the res4 3x3 shape
_CASES = [sh + (res, 1.0) for sh in _SHAPES for res in (False, True)] + \
    [_SHAPES[0] + (False, mag) for mag in (1e-20, 1e20)]


@pytest.mark.parametrize('N,H,W,Cin,Cout,k,s,p,residual,mag', _CASES)
def test_conv_h2_error_tiles_amax(N, H, W, Cin, Cout, k, s, p, residual, mag):
    from pps_amd import model, ops
    rng = np.random.RandomState(N + H + Cin + Cout + k)
    x = (rng.randn(N, Cin, H, W) * mag).astype(np.float32)
    w = (rng.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)).astype(np.float32)
    scale = rng.uniform(0.5, 1.5, Cout).astype(np.float32)
    shift = (rng.randn(Cout) * 0.1 * mag).astype(np.float32)
    ref = F.conv2d(torch.from_numpy(x).double(), torch.from_numpy(w).double(), stride=s,
                   padding=p)
    ref = ref * torch.from_numpy(scale).double()[None, :, None, None] + \
        torch.from_numpy(shift).double()[None, :, None, None]
    res = None
    if residual:
        res_np = (rng.randn(*ref.shape) * mag).astype(np.float32)
        ref = ref + torch.from_numpy(res_np).double()
        res = _cuda(res_np.transpose(0, 2, 3, 1))
    ref = torch.clamp_min(ref, 0).numpy().transpose(0, 2, 3, 1)
    wp, kpad = model.pack_conv_weight(w)
    xd = _cuda(x.transpose(0, 2, 3, 1))
    y = torch.empty(ref.shape, dtype=torch.float32, device='cuda')
    ops.conv2d_bn_act(xd, Cin, ops.split_bf16x3(_cuda(wp)), kpad, k, s, p, 1, _cuda(scale),
                      _cuda(shift), res, True, y, tile=ops.TILE_P16_FIRST)
    e_x3 = _rel_err(y.cpu().numpy(), ref)
    w2, wrs = ops.split_weights_h2(_cuda(wp))
    amx = ops.amax(xd)
    assert ops.amax_value(amx) == float(np.abs(x).max())
    tiles = _h2_tiles()
    outs = []
    for tile in tiles:
        y = torch.full(ref.shape, float('nan'), dtype=torch.float32, device='cuda')
        ay = ops.amax_slot()
        ops.conv2d_bn_act_h2(xd, Cin, w2, wrs, kpad, k, s, p, 1, _cuda(scale), _cuda(shift), res,
                             True, y, amx, ay, tile=tile)
        yn = y.cpu().numpy()
        assert ops.amax_value(ay) == float(np.abs(yn).max()), tile
        outs.append(yn)
    for t, o in zip(tiles, outs):
        e_h2 = _rel_err(o, ref)
        assert e_h2 <= H2_VS_X3 * e_x3 + ERR_FLOOR, (t, e_h2, e_x3)
    print('conv h2 err %.3g  x3 err %.3g' % (_rel_err(outs[0], ref), e_x3))
    check_tile_bits(tiles, outs, ops.TILE_P16_FIRST)


@pytest.mark.parametrize('N,H,W,C1,C2,Cout,s2', [(2, 24, 8, 128, 256, 512, 2),
                                                 (1, 24, 8, 512, 1024, 2048, 1),
                                                 (2, 96, 32, 64, 64, 256, 1),
                                                 (1, 12, 8, 32, 32, 64, 2)])
def test_conv_dual_h2(N, H, W, C1, C2, Cout, s2):
    """The fused projection shortcut: both operands scaled by the larger of
    their two maxima (here 100x apart), one K-concatenated f16x2 GEMM."""
    from pps_amd import model, ops
    rng = np.random.RandomState(C1 + Cout)
    x = rng.randn(N, C1, H, W).astype(np.float32)
    x2 = (rng.randn(N, C2, (H - 1) * s2 + 1, (W - 1) * s2 + 1) * 100).astype(np.float32)
    w1 = (rng.randn(Cout, C1, 1, 1) / np.sqrt(C1)).astype(np.float32)
    w2 = (rng.randn(Cout, C2, 1, 1) / np.sqrt(C2) / 100).astype(np.float32)
    sh = rng.randn(Cout).astype(np.float32)
    p1, k1 = model.pack_conv_weight(w1)
    p2, _ = model.pack_conv_weight(w2)
    w = np.concatenate([p1, p2], 1)
    ref = F.conv2d(torch.from_numpy(x).double(), torch.from_numpy(w1).double()) + \
        F.conv2d(torch.from_numpy(x2).double(), torch.from_numpy(w2).double(), stride=s2) + \
        torch.from_numpy(sh).double()[:, None, None]
    ref = torch.clamp_min(ref, 0).numpy().transpose(0, 2, 3, 1)
    xd, x2d = _cuda(x.transpose(0, 2, 3, 1)), _cuda(x2.transpose(0, 2, 3, 1))
    y = torch.empty(ref.shape, device='cuda')
    ops.conv2d_dual_bn_act(xd, C1, 1, 1, 0, x2d, s2, ops.split_bf16x3(_cuda(w)), k1, _cuda(sh),
                           True, y, tile=ops.TILE_P16_FIRST)
    e_x3 = _rel_err(y.cpu().numpy(), ref)
    wq, wrs = ops.split_weights_h2(_cuda(w))
    tiles = [0] + list(range(ops.TILE_P16_FIRST, 56)) + [60]
    outs = []
    for tile in tiles:
        y = torch.full(ref.shape, float('nan'), device='cuda')
        ay = ops.amax_slot()
        ops.conv2d_dual_bn_act_h2(xd, C1, 1, 1, 0, x2d, s2, wq, wrs, k1, _cuda(sh), True, y,
                                  ops.amax(xd), ops.amax(x2d), ay, tile=tile)
        yn = y.cpu().numpy()
        assert ops.amax_value(ay) == float(np.abs(yn).max())
        outs.append(yn)
    for t, o in zip(tiles, outs):
        assert _rel_err(o, ref) <= H2_VS_X3 * e_x3 + ERR_FLOOR, (t, _rel_err(o, ref), e_x3)
    check_tile_bits(tiles, outs, ops.TILE_P16_FIRST)


def test_conv_pps_h2_equals_conv_then_pooling():
    """The last conv with the part pooling fused (f16x2): the pooled subsets
    equal part_power_set of the same tile group's conv output bit for bit."""
    from pps_amd import model, ops
    rng = np.random.RandomState(5)
    N, H, W, Cin, Cout = 2, 24, 8, 512, 256
    x = np.maximum(rng.randn(N, H, W, Cin), 0).astype(np.float32)
    w = (rng.randn(Cout, Cin, 1, 1) / np.sqrt(Cin)).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, Cout).astype(np.float32)
    sh = (rng.randn(Cout) * 0.1).astype(np.float32)
    res = np.maximum(rng.randn(N, H, W, Cout), 0).astype(np.float32)
    wp, kpad = model.pack_conv_weight(w)
    w2, wrs = ops.split_weights_h2(_cuda(wp))
    xd = _cuda(x)
    amx = ops.amax(xd)
    split = [5, 5, 5, 5, 4]
    y = torch.empty((N, H, W, Cout), device='cuda')
    ops.conv2d_bn_act_h2(xd, Cin, w2, wrs, kpad, 1, 1, 0, 1, _cuda(sc), _cuda(sh), _cuda(res),
                         True, y, amx, tile=ops.TILE_P16_FIRST)
    want = torch.empty((31, N, Cout), device='cuda')
    ops.part_power_set(y, split, True, want)
    for tile in (39, 46, 47, 52):
        got = torch.full((31, N, Cout), float('nan'), device='cuda')
        y2 = torch.full((N, H, W, Cout), float('nan'), device='cuda')
        ops.conv2d_bn_act_pps_h2(xd, Cin, w2, wrs, kpad, 1, 1, 0, 1, _cuda(sc), _cuda(sh),
                                 _cuda(res), split, True, got, amx, y=y2, tile=tile)
        assert torch.equal(got, want), tile
        assert torch.equal(y2, y), tile


def test_conv_h2_enforces():
    from pps_amd import model, ops
    x = torch.zeros((1, 8, 8, 64), device='cuda')
    w = np.zeros((64, 64, 1, 1), np.float32)
    wp, kpad = model.pack_conv_weight(w)
    w2, wrs = ops.split_weights_h2(_cuda(wp))
    y = torch.empty((1, 8, 8, 64), device='cuda')
    one = torch.ones((64,), device='cuda')
    with pytest.raises(RuntimeError, match='relu|ReLU'):   # f16x2 epilogues end in a ReLU
        ops.conv2d_bn_act_h2(x, 64, w2, wrs, kpad, 1, 1, 0, 1, one, one, None, False, y,
                             ops.amax(x))
    with pytest.raises(RuntimeError, match='tile'):
        ops.conv2d_bn_act_h2(x, 64, w2, wrs, kpad, 1, 1, 0, 1, one, one, None, True, y,
                             ops.amax(x), tile=30)


@pytest.mark.parametrize('N,H,W,Cin,Cout,k,s,p', [
    (2, 24, 8, 256, 256, 3, 1, 1),     # res4 branch2b
    (2, 24, 8, 1024, 256, 1, 1, 0),    # res4 branch2a
    (2, 48, 16, 256, 128, 1, 2, 0),    # strided 1x1
    (3, 7, 5, 64, 40, 3, 1, 1),        # ragged M and N
    (2, 48, 16, 128, 512, 1, 1, 0),    # a weight-stationary shape (tile 54 -> 38 on planes)
])
@pytest.mark.parametrize('residual', [False, True])
def test_conv_h2_activation_planes_same_bits(N, H, W, Cin, Cout, k, s, p, residual):
    """f16x2 activation planes (pps_split_f16x2_act, once per element) in
    place of the f32 input: the same fragments reach the MFMAs, so every tile
    gives the f32-input kernel's bits, and the same max|y| -- the patch tiles
    56-59 too (round 6: their planes patch; stride-1 3x3 shapes, no residual)."""
    from pps_amd import model, ops
    rng = np.random.RandomState(Cin + Cout + k + s)
    x = rng.randn(N, H, W, Cin).astype(np.float32)
    x[0, 0, 0, :5] = [1e-30, -3e-8, 0.0, -0.0, 7.5e4]   # subnormal f16 parts, a large max
    w = (rng.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)).astype(np.float32)
    wp, kpad = model.pack_conv_weight(w)
    w2, wrs = ops.split_weights_h2(_cuda(wp))
    sc, sh = _cuda(rng.uniform(0.5, 1.5, Cout)), _cuda(rng.randn(Cout) * 0.1)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    res = _cuda(rng.randn(N, Ho, Wo, Cout)) if residual else None
    xd = _cuda(x)
    amx = ops.amax(xd)
    planes = ops.split_act_h2(xd, amx)
    for tile in (0, 38, 45, 47, 52, 60, 56, 57, 58, 59):
        y1 = torch.full((N, Ho, Wo, Cout), float('nan'), device='cuda')
        y2 = torch.full((N, Ho, Wo, Cout), float('nan'), device='cuda')
        a1, a2 = ops.amax_slot(), ops.amax_slot()
        ops.conv2d_bn_act_h2(xd, Cin, w2, wrs, kpad, k, s, p, 1, sc, sh, res, True, y1, amx, a1,
                             tile=tile)
        ops.conv2d_bn_act_h2(planes, Cin, w2, wrs, kpad, k, s, p, 1, sc, sh, res, True, y2, amx,
                             a2, tile=tile)
        assert torch.equal(y1, y2), tile
        assert ops.amax_value(a1) == ops.amax_value(a2), tile


def test_conv_pps_h2_activation_planes_same_bits():
    from pps_amd import model, ops
    rng = np.random.RandomState(6)
    N, H, W, Cin, Cout = 2, 24, 8, 512, 256
    x = np.maximum(rng.randn(N, H, W, Cin), 0).astype(np.float32)
    w = (rng.randn(Cout, Cin, 1, 1) / np.sqrt(Cin)).astype(np.float32)
    wp, kpad = model.pack_conv_weight(w)
    w2, wrs = ops.split_weights_h2(_cuda(wp))
    sc, sh = _cuda(rng.uniform(0.5, 1.5, Cout)), _cuda(rng.randn(Cout) * 0.1)
    res = _cuda(np.maximum(rng.randn(N, H, W, Cout), 0))
    xd = _cuda(x)
    amx = ops.amax(xd)
    planes = ops.split_act_h2(xd, amx)
    split = [5, 5, 5, 5, 4]
    for tile in (47, 52, 60):
        a = torch.full((31, N, Cout), float('nan'), device='cuda')
        b = torch.full((31, N, Cout), float('nan'), device='cuda')
        ops.conv2d_bn_act_pps_h2(xd, Cin, w2, wrs, kpad, 1, 1, 0, 1, sc, sh, res, split, True, a,
                                 amx, tile=tile)
        ops.conv2d_bn_act_pps_h2(planes, Cin, w2, wrs, kpad, 1, 1, 0, 1, sc, sh, res, split,
                                 True, b, amx, tile=tile)
        assert torch.equal(a, b), tile


@pytest.mark.parametrize('N,H,W,Cin,Cout,k,s,p', [
    (2, 24, 8, 512, 512, 1, 1, 0),     # res5 branch2a -> 2b
    (2, 24, 8, 256, 256, 3, 1, 1),     # res4 branch2b -> 2c
    (2, 48, 16, 256, 128, 1, 2, 0),    # strided 1x1
    (3, 7, 5, 64, 96, 3, 1, 1),        # ragged M (N and the consumer's K: multiples of 32)
])
@pytest.mark.parametrize('arith', ['x3', 'h2', 'h2_planes_in'])
def test_conv_h2out_planes_equal_split_of_f32_output(N, H, W, Cin, Cout, k, s, p, arith):
    """A producer writing f16x2 planes on its output bound's scale
    (pps_conv2d_bn_act_h2out): the planes equal pps_split_f16x2_act of the same
    conv's f32 output with the bound in the slot, the bound is >= max|y|, and
    a consumer f16x2 conv reading the planes gives the bits of one reading the
    f32 output with that slot."""
    from pps_amd import model, ops
    rng = np.random.RandomState(Cin + Cout + k)
    x = np.maximum(rng.randn(N, H, W, Cin), 0).astype(np.float32)
    w = (rng.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)).astype(np.float32)
    wp, kpad = model.pack_conv_weight(w)
    wpd = _cuda(wp)
    sc, sh = _cuda(rng.uniform(0.5, 1.5, Cout)), _cuda(rng.randn(Cout) * 0.1)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    xd = _cuda(x)
    ax = ops.amax(xd)
    bound = ops.h2_out_bound(wpd, sc, sh)
    y = torch.empty((N, Ho, Wo, Cout), device='cuda')
    y2 = torch.full((2, N, Ho, Wo, Cout), -1, dtype=torch.int16, device='cuda')
    by = ops.amax_slot()
    tile = ops.TILE_P16_FIRST
    if arith == 'x3':
        w3 = ops.split_bf16x3(wpd)
        ops.conv2d_bn_act(xd, Cin, w3, kpad, k, s, p, 1, sc, sh, None, True, y, tile=tile)
        ops.conv2d_bn_act_h2out(xd, Cin, w3, None, kpad, k, s, p, 1, sc, sh, y2, None, ax, bound,
                                by, tile=tile)
    else:
        w2, wrs = ops.split_weights_h2(wpd)
        xin = ops.split_act_h2(xd, ax) if arith == 'h2_planes_in' else xd
        ops.conv2d_bn_act_h2(xd, Cin, w2, wrs, kpad, k, s, p, 1, sc, sh, None, True, y, ax,
                             tile=tile)
        ops.conv2d_bn_act_h2out(xin, Cin, w2, wrs, kpad, k, s, p, 1, sc, sh, y2, ax, ax, bound,
                                by, tile=tile)
    B = ops.amax_value(by)
    assert B >= float(y.abs().max())
    assert B == np.float32(bound[0]) * np.float32(ops.amax_value(ax)) + np.float32(bound[1]) or \
        abs(B - (bound[0] * ops.amax_value(ax) + bound[1])) <= 1e-6 * B
    want = ops.split_act_h2(y, by)
    assert torch.equal(y2, want)
    # a consumer (1x1 to 96 channels): planes in == f32 in with the bound slot
    w_c = (rng.randn(96, Cout, 1, 1) / np.sqrt(Cout)).astype(np.float32)
    wpc, kpc = model.pack_conv_weight(w_c)
    w2c, wrsc = ops.split_weights_h2(_cuda(wpc))
    one, zero = torch.ones(96, device='cuda'), torch.zeros(96, device='cuda')
    z1 = torch.empty((N, Ho, Wo, 96), device='cuda')
    z2 = torch.empty((N, Ho, Wo, 96), device='cuda')
    ops.conv2d_bn_act_h2(y, Cout, w2c, wrsc, kpc, 1, 1, 0, 1, one, zero, None, True, z1, by,
                         tile=tile)
    ops.conv2d_bn_act_h2(y2, Cout, w2c, wrsc, kpc, 1, 1, 0, 1, one, zero, None, True, z2, by,
                         tile=tile)
    assert torch.equal(z1, z2)
