"""The bf16x3 GEMM path (pps_amd/csrc/gemm_x3.hip): f32 products on bf16
matrix cores.

* the weight split is exact: hi + mid + lo == w bit for bit (fp64 sum);
* results carry f32-level error: measured against an fp64 reference, the
  x3 kernel's max error stays within 4x the exact-f32 MFMA kernel's max error
  on the same data (tolerance written below), far from bf16 (~4e-3);
* every tile configuration gives identical bits.
"""
import numpy as np
from _tiles import check_tile_bits
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

X3_VS_F32 = 4.0      # max error of x3 <= X3_VS_F32 * max error of exact f32 (+ floor)
ERR_FLOOR = 2e-7     # relative to max |ref|: one f32 ulp order of magnitude


def _cuda(x):
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()


def _rel_err(got, ref):
    return float(np.abs(got.astype(np.float64) - ref).max() / max(1e-30, np.abs(ref).max()))


def test_split_bf16x3_exact():
    from pps_amd import ops
    rng = np.random.RandomState(0)
    x = np.concatenate([rng.randn(4096), rng.randn(4096) * 1e-20, rng.randn(4096) * 1e20,
                        [0.0, -0.0, 1.0, -1.0, 3.0e38, 1.17549435e-38]]).astype(np.float32)
    planes = ops.split_bf16x3(_cuda(x))
    assert planes.shape == (3, x.size) and planes.dtype == torch.int16
    parts = planes.view(torch.bfloat16).double().cpu().numpy()
    np.testing.assert_array_equal(parts.sum(0), x.astype(np.float64))
    # the leading plane is round-to-nearest bf16 of x
    np.testing.assert_array_equal(parts[0], torch.from_numpy(x).bfloat16().double().numpy())
    hb = ops.split_bf16x3(_cuda(x[:12288].reshape(3, 64, 64)), batched=True)
    assert hb.shape == (3, 3, 64, 64)
    np.testing.assert_array_equal(hb.view(torch.bfloat16).double().sum(1).cpu().numpy(),
                                  x[:12288].reshape(3, 64, 64))
    # 8-wide vector kernel (n % 8 == 0, 16-byte aligned) == scalar kernel
    # (same data at a 4-byte offset, which forces the scalar path)
    xd = _cuda(np.concatenate([[0.0], x[:12288]]).astype(np.float32))
    p_scalar = ops.split_bf16x3(xd[1:])
    p_vector = ops.split_bf16x3(xd[1:].clone())
    assert xd[1:].data_ptr() % 16 != 0 and p_vector.shape == (3, 12288)
    assert torch.equal(p_scalar, p_vector)


@pytest.mark.parametrize('R,D', [(1, 4), (7, 132), (33, 2048), (130, 3968)])
def test_split_sqnorm_fused_equals_separate(R, D):
    """pps_split_bf16x3_sqnorm (gallery index / query planes in one read)
    gives the bits of pps_split_bf16x3 + pps_row_sqnorm."""
    from pps_amd import ops
    rng = np.random.RandomState(R + D)
    x = _cuda(rng.randn(R, D).astype(np.float32))
    planes, sq = ops.split_sqnorm(x)
    assert planes.shape == (3, R, D)
    assert torch.equal(planes, ops.split_bf16x3(x))
    assert torch.equal(sq, ops.row_sqnorm(x))
    idx = ops.GalleryIndex(x)
    assert torch.equal(idx.planes, planes) and torch.equal(idx.sqnorm, sq)


@pytest.mark.parametrize('N,H,W,Cin,Cout,k,s,p', [
    (2, 96, 32, 64, 64, 1, 1, 0),
    (2, 96, 32, 64, 64, 3, 1, 1),
    (2, 48, 16, 256, 128, 1, 2, 0),
    (1, 24, 8, 512, 512, 3, 1, 1),
    (3, 7, 5, 32, 40, 3, 1, 1),        # ragged M and N
    (1, 11, 9, 16, 33, 3, 2, 1),       # ragged, strided, Cin < 32 (BK32 falls back)
    (1, 9, 7, 20, 24, 3, 1, 1),        # Cin not a power of two and < 32
    (2, 384, 128, 4, 64, 7, 2, 3),     # stem conv1 (Cin 3 packed to 4)
    # the weight-stationary tile 54 (1x1, K = 64 / 128 / 256): res2 / res3 /
    # res4 branch2c shapes, ragged M, Cout < the column block
    (2, 96, 32, 64, 256, 1, 1, 0),
    (1, 48, 16, 128, 512, 1, 1, 0),
    (2, 24, 8, 256, 1024, 1, 1, 0),
    (3, 7, 5, 64, 128, 1, 1, 0),
    (1, 9, 9, 128, 64, 1, 1, 0),
])
@pytest.mark.parametrize('residual', [False, True])
def test_conv_x3_error_and_tiles(N, H, W, Cin, Cout, k, s, p, residual):
    from pps_amd import model, ops
    rng = np.random.RandomState(N + H + Cin + Cout + k)
    x = rng.randn(N, Cin, H, W).astype(np.float32)
    if Cin == 4:
        x[:, 3] = 0
    w = (rng.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)).astype(np.float32)
    scale = rng.uniform(0.5, 1.5, Cout).astype(np.float32)
    shift = rng.randn(Cout).astype(np.float32) * 0.1
    ref = F.conv2d(torch.from_numpy(x).double(), torch.from_numpy(w).double(), stride=s,
                   padding=p)
    ref = ref * torch.from_numpy(scale).double()[None, :, None, None] + \
        torch.from_numpy(shift).double()[None, :, None, None]
    res = None
    if residual:
        res_np = rng.randn(*ref.shape).astype(np.float32)
        ref = ref + torch.from_numpy(res_np).double()
        res = _cuda(res_np.transpose(0, 2, 3, 1))
    ref = ref.numpy().transpose(0, 2, 3, 1)
    wp, kpad = model.pack_conv_weight(w)
    xd = _cuda(x.transpose(0, 2, 3, 1))
    y = torch.empty(ref.shape, dtype=torch.float32, device='cuda')
    ops.conv2d_bn_act(xd, Cin, _cuda(wp), kpad, k, s, p, 1, _cuda(scale), _cuda(shift), res,
                      False, y)
    e_f32 = _rel_err(y.cpu().numpy(), ref)
    w3 = ops.split_bf16x3(_cuda(wp))
    outs = []
    for tile in range(0, ops.num_tiles() + 1):
        y = torch.full(ref.shape, float('nan'), dtype=torch.float32, device='cuda')
        ops.conv2d_bn_act(xd, Cin, w3, kpad, k, s, p, 1, _cuda(scale), _cuda(shift), res,
                          False, y, tile=tile)
        outs.append(y.cpu().numpy())
    for o in (outs[0], outs[ops.TILE_P16_FIRST]):
        e_x3 = _rel_err(o, ref)
        print('conv x3 err %.3g  f32 err %.3g' % (e_x3, e_f32))
        assert e_x3 <= X3_VS_F32 * e_f32 + ERR_FLOOR, (e_x3, e_f32)
    check_tile_bits(range(0, ops.num_tiles() + 1), outs, ops.TILE_P16_FIRST)


@pytest.mark.parametrize('N,H,W,C1,C2,Cout,s2', [(2, 24, 8, 128, 256, 512, 2),
                                                 (1, 24, 8, 512, 1024, 2048, 1),
                                                 (3, 5, 7, 16, 32, 40, 1),
                                                 (2, 96, 32, 64, 64, 256, 1),   # res2_0 (tile 54)
                                                 (1, 12, 8, 32, 32, 64, 2)])
def test_conv_dual_x3(N, H, W, C1, C2, Cout, s2):
    from pps_amd import model, ops
    rng = np.random.RandomState(C1 + Cout)
    x = rng.randn(N, C1, H, W).astype(np.float32)
    x2 = rng.randn(N, C2, (H - 1) * s2 + 1, (W - 1) * s2 + 1).astype(np.float32)
    w1 = (rng.randn(Cout, C1, 1, 1) / np.sqrt(C1)).astype(np.float32)
    w2 = (rng.randn(Cout, C2, 1, 1) / np.sqrt(C2)).astype(np.float32)
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
    ops.conv2d_dual_bn_act(xd, C1, 1, 1, 0, x2d, s2, _cuda(w), k1, _cuda(sh), True, y)
    e_f32 = _rel_err(y.cpu().numpy(), ref)
    w3 = ops.split_bf16x3(_cuda(w))
    outs = []
    for tile in range(0, ops.num_tiles() + 1):
        y = torch.full(ref.shape, float('nan'), device='cuda')
        ops.conv2d_dual_bn_act(xd, C1, 1, 1, 0, x2d, s2, w3, k1, _cuda(sh), True, y,
                               tile=tile)
        outs.append(y.cpu().numpy())
    for o in (outs[0], outs[ops.TILE_P16_FIRST]):
        e_x3 = _rel_err(o, ref)
        assert e_x3 <= X3_VS_F32 * e_f32 + ERR_FLOOR, (e_x3, e_f32)
    check_tile_bits(range(0, ops.num_tiles() + 1), outs, ops.TILE_P16_FIRST)


@pytest.mark.parametrize('splitk', [1, 8])
def test_heads_splitk_x3(splitk):
    from pps_amd import ops
    rng = np.random.RandomState(7)
    B, M, K, C = 31, 6, 2048, 128
    x = rng.randn(B, M, K).astype(np.float32)
    w = (rng.randn(B, C, K) / 45).astype(np.float32)
    ref = np.einsum('bmk,bck->mbc', x.astype(np.float64), w).reshape(M, B * C)
    part = torch.empty((splitk, M, B * C), device='cuda')
    ops.gemm_splitk_batched(_cuda(x), _cuda(w), splitk, part)
    e_f32 = _rel_err(part.sum(0).cpu().numpy(), ref)
    ops.gemm_splitk_batched(_cuda(x), ops.split_bf16x3(_cuda(w), batched=True), splitk, part)
    e_x3 = _rel_err(part.sum(0).cpu().numpy(), ref)
    assert e_x3 <= X3_VS_F32 * e_f32 + ERR_FLOOR, (e_x3, e_f32)



def _planes_of(t):
    """f32 NHWC tensor -> bf16x3 activation planes [3, N, H, W, C]."""
    from pps_amd import ops
    return ops.split_bf16x3(t.contiguous().view(-1)).view((3,) + tuple(t.shape))


@pytest.mark.parametrize('N,H,W,Cin,Cout,k,s,p', [
    (2, 96, 32, 64, 64, 3, 1, 1),      # res2 branch2b
    (2, 24, 8, 512, 2048, 1, 1, 0),    # res5 branch2c
    (1, 24, 8, 512, 512, 3, 1, 1),     # res5 branch2b
    (3, 7, 5, 32, 40, 3, 1, 1),        # ragged M and N
    (1, 11, 9, 64, 36, 3, 2, 1),       # ragged, strided
])
@pytest.mark.parametrize('residual', [False, True])
def test_conv_x3_activation_planes(N, H, W, Cin, Cout, k, s, p, residual):
    """pps_conv2d_bn_act_x3p: planes in and/or out give the same bits as the
    f32-activation call, on every pipelined tile; written planes sum exactly
    to the f32 output."""
    from pps_amd import model, ops
    rng = np.random.RandomState(7 + N + H + Cin + Cout + k)
    x = _cuda(rng.randn(N, H, W, Cin))
    w = (rng.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)).astype(np.float32)
    wp, kpad = model.pack_conv_weight(w)
    w3 = ops.split_bf16x3(_cuda(wp))
    scale = _cuda(rng.uniform(0.5, 1.5, Cout))
    shift = _cuda(rng.randn(Cout) * 0.1)
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    res = _cuda(rng.randn(N, Ho, Wo, Cout)) if residual else None
    y = torch.empty((N, Ho, Wo, Cout), dtype=torch.float32, device='cuda')
    xp = _planes_of(x)
    for tile in [0] + list(range(ops.TILE_P_FIRST, ops.num_tiles() + 1)):
        # f32-activation call on the same tile (same rounding group)
        ops.conv2d_bn_act(x, Cin, w3, kpad, k, s, p, 1, scale, shift, res, True, y,
                          tile=tile or ops.TILE_P_FIRST)
        want = y.cpu().numpy()
        yo = torch.full_like(y, float('nan'))
        ops.conv2d_bn_act_x3p(xp, Cin, w3, kpad, k, s, p, 1, scale, shift, res, True, yo,
                              tile=tile)
        np.testing.assert_array_equal(yo.cpu().numpy(), want, err_msg='planes in, tile %d' % tile)
        if residual:
            continue  # plane outputs feed convs only (no residual epilogue with planes)
        for src in (x, xp):
            yp = ops.act_planes(y.shape, 'cuda').fill_(-1)
            ops.conv2d_bn_act_x3p(src, Cin, w3, kpad, k, s, p, 1, scale, shift, None, True,
                                  yp, tile=tile)
            got = yp.view(torch.bfloat16).double().sum(0).cpu().numpy()
            np.testing.assert_array_equal(got, want.astype(np.float64),
                                          err_msg='planes out, tile %d' % tile)
            np.testing.assert_array_equal(yp.cpu().numpy(), _planes_of(y).cpu().numpy())


def test_conv_x3_planes_rejects_register_tiles():
    from pps_amd import ops
    x = torch.zeros((1, 4, 4, 32), device='cuda')
    w3 = torch.zeros((3, 32, 32), dtype=torch.int16, device='cuda')
    v = torch.zeros(32, device='cuda')
    y = ops.act_planes((1, 4, 4, 32), 'cuda')
    with pytest.raises(RuntimeError, match='pipelined tile'):
        ops.conv2d_bn_act_x3p(x, 32, w3, 32, 1, 1, 0, 1, v, v, None, False, y, tile=1)


def test_forward_act_planes_same_bits():
    """The whole forward with bottleneck intermediates as planes equals the
    f32-intermediate forward bit for bit."""
    from pps_amd import config, model
    cfg = config.cfg
    cfg.MODEL.NUM_CLASSES = 752
    cfg.MODEL.USE_BN = True
    cfg.RESNETS.RES5_STRIDE = 1
    cfg.REID.SCALE = (128, 384)
    cfg.REID.BPM_STRIP_NUM = 5
    cfg.REID.BPM_DIM = 128
    cfg.REID.NORMALIZE_FEATURE = True
    cfg.REID.MAX_AVE_FEATURE = True
    plan = model.build_plan()
    blobs = model.synthetic_weights(plan, seed=1)
    rng = np.random.RandomState(1)
    x = np.zeros((4, 384, 128, 4), np.float32)
    x[..., :3] = rng.randn(4, 384, 128, 3) * 50
    xd = _cuda(x)
    m_pl = model.PPSModel(blobs, math='x3', act_planes=True)
    m_f = model.PPSModel(blobs, math='x3', act_planes=False)
    m_pl.set_planes([P['name'] for P, C in m_pl._edges])
    # 2a and 2b of every bottleneck but the 2b's feeding a fused shortcut
    assert len(m_pl.planes()) == 28, m_pl.planes()
    a = m_pl.forward(xd).cpu().numpy()
    b = m_f.forward(xd).cpu().numpy()
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize('Q,G,D', [(300, 1000, 3968), (37, 501, 64), (1, 7, 2048)])
def test_distmat_query_planes_same_bits(Q, G, D):
    """pps_distmat_x3p (queries pre-split into planes) == pps_distmat_x3 bit
    for bit on every pipelined tile, and within 1e-4 of the f32 formula."""
    from oracle import evaluator as ev
    from pps_amd import ops
    rng = np.random.RandomState(Q + G)
    qn = rng.randn(Q, D).astype(np.float32)
    gn = rng.randn(G, D).astype(np.float32)
    q, idx = _cuda(qn), ops.GalleryIndex(_cuda(gn), math='x3')
    for tile in [0] + list(range(ops.TILE_P_FIRST, ops.num_tiles() + 1)):
        want = ops.compute_dist(q, idx, q_planes=False,
                                tile=tile or ops.TILE_P16_FIRST + 4).cpu().numpy()
        got = ops.compute_dist(q, idx, q_planes=True, tile=tile).cpu().numpy()
        np.testing.assert_array_equal(got, want, err_msg='tile %d' % tile)
    np.testing.assert_allclose(want, ev.compute_dist(qn, gn), rtol=0, atol=1e-4 * np.sqrt(D / 64))


@pytest.mark.parametrize('N,D', [(1000, 3968), (2500, 3968), (301, 64), (129, 2048), (17, 32)])
@pytest.mark.parametrize('metric', ['euclidean', 'cosine'])
def test_self_distance_symmetric(N, D, metric):
    """compute_dist(x, x) from the upper-triangle tiles + mirror: symmetric,
    upper-triangle tiles bit-equal to the full product on the same tile, and
    within the f32 tolerance of the NumPy formula everywhere."""
    from oracle import evaluator as ev
    from pps_amd import ops
    rng = np.random.RandomState(N + D)
    xn = rng.randn(N, D).astype(np.float32)
    xn /= np.linalg.norm(xn, axis=1, keepdims=True)  # re-ID features are L2-normalised
    x = _cuda(xn)
    ref = ev.compute_dist(xn, xn, metric) if metric == 'euclidean' else None
    for tile in ops.SELF_TILES:
        d = ops.compute_dist(x, x, metric=metric, tile=tile, math='x3').cpu().numpy()
        full = ops.compute_dist(x, x, metric=metric, tile=tile or ops.TILE_P16_FIRST,
                                symmetric=False, math='x3').cpu().numpy()
        np.testing.assert_array_equal(d, d.T, err_msg='tile %d' % tile)
        iu = np.triu_indices(N)           # the upper triangle is the full product's
        np.testing.assert_array_equal(d[iu], full[iu], err_msg='tile %d' % tile)
        if ref is not None:
            # off the diagonal within the f32 tolerance; ON it both sides take
            # the sqrt of a cancelled |x|^2 + |x|^2 - 2 x.x, i.e. of f32
            # rounding noise (~sqrt(D) * 2^-24 ~ 4e-6 for |x| = 1 -> ~2e-3),
            # whose value depends on the summation order (NumPy: 0 .. 5e-4)
            off = ~np.eye(N, dtype=bool)
            np.testing.assert_allclose(d[off], ref[off], rtol=0, atol=1e-4)
            assert np.abs(np.diag(d) - np.diag(ref)).max() < 5e-3
        else:
            np.testing.assert_allclose(d, full, rtol=0, atol=1e-5)


@pytest.mark.parametrize('N,H,W,Cin,Cout,k,s,p', [
    (2, 24, 8, 256, 256, 3, 1, 1),     # res4 branch2b
    (2, 24, 8, 1024, 256, 1, 1, 0),    # res4 branch2a
    (3, 7, 5, 64, 40, 3, 1, 1),        # ragged M and N
])
@pytest.mark.parametrize('splitk', [2, 3, 4])
@pytest.mark.parametrize('mode', ['f32', 'planes_in', 'planes_out', 'residual'])
def test_conv_x3_splitk(N, H, W, Cin, Cout, k, s, p, splitk, mode):
    """Conv split-K (raw slice partials + one summing BN/residual/ReLU pass):
    within the f32-level bound of the fp64 reference, like the one-pass
    kernel, for f32 / plane inputs and outputs and with a residual."""
    from pps_amd import model, ops
    Kpad = k * k * Cin
    if Kpad % (32 * splitk):
        pytest.skip('K does not split into whole 32-wide chunks')
    rng = np.random.RandomState(Cin + Cout + splitk)
    xn = rng.randn(N, H, W, Cin).astype(np.float32)
    w = (rng.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, Cout).astype(np.float32)
    sh = (rng.randn(Cout) * 0.1).astype(np.float32)
    ref = F.conv2d(torch.from_numpy(xn.transpose(0, 3, 1, 2)).double(),
                   torch.from_numpy(w).double(), stride=s, padding=p)
    ref = ref * torch.from_numpy(sc).double()[None, :, None, None] + \
        torch.from_numpy(sh).double()[None, :, None, None]
    ref = ref.numpy().transpose(0, 2, 3, 1)
    res = None
    if mode == 'residual':
        rn = rng.randn(*ref.shape).astype(np.float32)
        ref = ref + rn
        res = _cuda(rn)
    ref = np.maximum(ref, 0)
    wp, kpad = model.pack_conv_weight(w)
    w3 = ops.split_bf16x3(_cuda(wp))
    x = _cuda(xn)
    xin = _planes_of(x) if mode == 'planes_in' else x
    y1 = torch.empty(ref.shape, dtype=torch.float32, device='cuda')
    ops.conv2d_bn_act_x3p(xin, Cin, w3, kpad, k, s, p, 1, _cuda(sc), _cuda(sh), res, True, y1,
                          tile=ops.TILE_P_FIRST)
    part = torch.empty(splitk * y1.numel(), device='cuda')
    for tile in (ops.TILE_P_FIRST, ops.TILE_P_FIRST + 8, ops.TILE_P16_FIRST + 7):
        if mode == 'planes_out':
            yp = ops.act_planes(ref.shape, 'cuda')
            ops.conv2d_bn_act_x3p(xin, Cin, w3, kpad, k, s, p, 1, _cuda(sc), _cuda(sh), res,
                                  True, yp, tile=tile, splitk=splitk, part=part)
            y = yp.view(torch.bfloat16).double().sum(0).float()
        else:
            y = torch.full(ref.shape, float('nan'), device='cuda')
            ops.conv2d_bn_act_x3p(xin, Cin, w3, kpad, k, s, p, 1, _cuda(sc), _cuda(sh), res,
                                  True, y, tile=tile, splitk=splitk, part=part)
        e_split = _rel_err(y.cpu().numpy(), ref)
        e_one = _rel_err(y1.cpu().numpy(), ref)
        assert e_split <= X3_VS_F32 * e_one + ERR_FLOOR, (tile, e_split, e_one)


@pytest.mark.parametrize('N,H,W,Cin,Cout,k,s,p', [
    (64, 24, 8, 256, 256, 3, 1, 1),    # res4 branch2b at the bench batch
    (4, 24, 8, 1024, 256, 1, 1, 0),    # res4 branch2a
    (3, 7, 5, 64, 40, 3, 1, 1),        # ragged M and N
])
@pytest.mark.parametrize('splitk', [2, 3, 4])
@pytest.mark.parametrize('mode', ['f32', 'planes_in', 'planes_out', 'residual', 'tiled_w'])
def test_conv_x3_splitk_fused_bits(N, H, W, Cin, Cout, k, s, p, splitk, mode):
    """One-launch split-K (last arriving K slice sums the parked partials)
    gives the bits of the two-pass split-K on every FIX tile, for f32 / plane
    inputs and outputs, a residual and chunk-tiled weights, and leaves the
    tile counters zero (a replayed graph starts clean).  Repeated launches
    give the same bits (the arrival order does not change the sum order)."""
    from pps_amd import model, ops
    Kpad = k * k * Cin
    if Kpad % (32 * splitk):
        pytest.skip('K does not split into whole 32-wide chunks')
    rng = np.random.RandomState(Cin + Cout + splitk + 7)
    xn = rng.randn(N, H, W, Cin).astype(np.float32)
    w = (rng.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)).astype(np.float32)
    sc = _cuda(rng.uniform(0.5, 1.5, Cout).astype(np.float32))
    sh = _cuda((rng.randn(Cout) * 0.1).astype(np.float32))
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    shape = (N, Ho, Wo, Cout)
    res = _cuda(rng.randn(*shape).astype(np.float32)) if mode == 'residual' else None
    wp, kpad = model.pack_conv_weight(w)
    w3 = ops.split_bf16x3(_cuda(wp))
    x = _cuda(xn)
    xin = _planes_of(x) if mode == 'planes_in' else x
    part = torch.empty(splitk * N * Ho * Wo * Cout, device='cuda')
    cnt = torch.zeros(4096, dtype=torch.int32, device='cuda')

    def out():
        if mode == 'planes_out':
            return ops.act_planes(shape, 'cuda')
        return torch.full(shape, float('nan'), device='cuda')

    for tile in (45, 47, 48, 49, 50):
        ref = out()
        ops.conv2d_bn_act_x3p(xin, Cin, w3, kpad, k, s, p, 1, sc, sh, res, True, ref,
                              tile=tile, splitk=splitk, part=part)
        wf, tf = w3, tile
        if mode == 'tiled_w':
            wf, tf = ops.tile_planes(w3), tile | ops.TILE_B_TILED
        for rep in range(2):
            y = out()
            ops.conv2d_bn_act_x3p(xin, Cin, wf, kpad, k, s, p, 1, sc, sh, res, True, y,
                                  tile=tf, splitk=splitk, part=part, counters=cnt)
            torch.cuda.synchronize()
            assert torch.equal(y.view(torch.int32), ref.view(torch.int32)) if mode != 'planes_out' \
                else torch.equal(y, ref), (tile, rep)
            assert int(cnt.abs().sum()) == 0, (tile, rep)
    with pytest.raises(RuntimeError):  # tile counters too few
        ops.conv2d_bn_act_x3p(xin, Cin, w3, kpad, k, s, p, 1, sc, sh, res, True, out(),
                              tile=45, splitk=splitk, part=part, counters=cnt[:0])


def test_forward_splitk_layers():
    """The model with split-K on the res5 convs (and plane edges) gives the
    one-pass features within the f32 forward tolerance."""
    from pps_amd import config, model
    cfg = config.cfg
    cfg.MODEL.NUM_CLASSES = 752
    cfg.MODEL.USE_BN = True
    cfg.RESNETS.RES5_STRIDE = 1
    cfg.REID.SCALE = (128, 384)
    cfg.REID.BPM_STRIP_NUM = 5
    cfg.REID.BPM_DIM = 128
    cfg.REID.NORMALIZE_FEATURE = True
    cfg.REID.MAX_AVE_FEATURE = True
    plan = model.build_plan()
    blobs = model.synthetic_weights(plan, seed=2)
    rng = np.random.RandomState(2)
    x = np.zeros((4, 384, 128, 4), np.float32)
    x[..., :3] = rng.randn(4, 384, 128, 3) * 50
    xd = _cuda(x)
    m = model.PPSModel(blobs, math='x3')
    base = m.forward(xd).cpu().numpy()
    sks = {}
    for i, L in enumerate(m.layers):
        if L['op'] == 'conv' and L['name'].startswith('res5'):
            sk = 2 + (i % 3)
            sks[L['name']] = sk if L['kpad'] % (32 * sk) == 0 else 2
    with pytest.raises(ValueError):
        m.set_splitks({'res5_1_branch2c': 3})  # K = 512: not whole 32-wide chunks
    m.set_splitks(sks)
    assert m.splitks() == sks
    got = m.forward(xd).cpu().numpy()
    np.testing.assert_allclose(got, base, rtol=0, atol=2e-5)


@pytest.mark.parametrize('N,H,W,Cin,Cout,k,planes', [(1, 24, 8, 512, 512, 3, True),
                                                     (2, 24, 8, 256, 256, 3, False),
                                                     (1, 24, 8, 1024, 256, 1, False),
                                                     (3, 7, 5, 64, 40, 1, False)])
def test_conv_tiled_weights_bits(N, H, W, Cin, Cout, k, planes):
    """Chunk-tiled bf16x3 weights (PPS_TILE_B_TILED, ops.tile_planes over the
    [3][Cout][Kpad] planes) give the row-major weights' bits on every
    pipelined and patch tile, and the other tiles refuse them."""
    from pps_amd import model, ops
    rng = np.random.RandomState(Cin + Cout + k)
    x = _cuda(rng.randn(N, H, W, Cin).astype(np.float32))
    w = (rng.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)).astype(np.float32)
    wp, kpad = model.pack_conv_weight(w)
    w3 = ops.split_bf16x3(_cuda(wp))
    w3t = ops.tile_planes(w3)
    sc = _cuda(rng.uniform(0.5, 1.5, Cout).astype(np.float32))
    sh = _cuda(rng.randn(Cout).astype(np.float32))
    p = (k - 1) // 2
    xin = ops.split_bf16x3(x.reshape(-1, Cin)).reshape(3, N, H, W, Cin) if planes else x
    tiles = [t for t in range(ops.TILE_P_FIRST, ops.num_tiles() + 1) if t != 54]
    for t in tiles:
        ya = torch.empty((N, H, W, Cout), device='cuda')
        yb = torch.full((N, H, W, Cout), float('nan'), device='cuda')
        ops.conv2d_bn_act_x3p(xin, Cin, w3, kpad, k, 1, p, 1, sc, sh, None, True, ya, tile=t)
        ops.conv2d_bn_act_x3p(xin, Cin, w3t, kpad, k, 1, p, 1, sc, sh, None, True, yb,
                              tile=t | 0x100)
        assert torch.equal(ya, yb), 'tile %d' % t
        # column-major tile order (PPS_TILE_COL_ORDER), either weight layout
        for f, wl in ((0x200, w3), (0x300, w3t)):
            yb.fill_(float('nan'))
            ops.conv2d_bn_act_x3p(xin, Cin, wl, kpad, k, 1, p, 1, sc, sh, None, True, yb,
                                  tile=t | f)
            assert torch.equal(ya, yb), 'tile %d flags %#x' % (t, f)
    for t in (1, 28, 54):
        with pytest.raises(RuntimeError):
            ops.conv2d_bn_act_x3p(xin, Cin, w3t, kpad, k, 1, p, 1, sc, sh, None, True, yb,
                                  tile=t | 0x100)


@pytest.mark.parametrize('N,H,W,C1,C2,Cout,s2', [(1, 24, 8, 512, 1024, 2048, 1),
                                                 (2, 24, 8, 128, 256, 512, 2)])
def test_conv_dual_tiled_weights_bits(N, H, W, C1, C2, Cout, s2):
    """The K-concatenated shortcut conv on chunk-tiled weights (the
    [3][Cout][Kpad1 + Cin2] planes through ops.tile_planes) equals the
    row-major run bit for bit on the pipelined tiles."""
    from pps_amd import model, ops
    rng = np.random.RandomState(C1 + C2)
    x = _cuda(rng.randn(N, H, W, C1).astype(np.float32))
    x2 = _cuda(rng.randn(N, (H - 1) * s2 + 1, (W - 1) * s2 + 1, C2).astype(np.float32))
    w1 = (rng.randn(Cout, C1, 1, 1) / np.sqrt(C1)).astype(np.float32)
    w2 = (rng.randn(Cout, C2, 1, 1) / np.sqrt(C2)).astype(np.float32)
    p1, k1 = model.pack_conv_weight(w1)
    p2, _ = model.pack_conv_weight(w2)
    w3 = ops.split_bf16x3(_cuda(np.concatenate([p1, p2], axis=1)))
    w3t = ops.tile_planes(w3)
    sh = _cuda(rng.randn(Cout).astype(np.float32))
    for t in (29, 35, 36, 38, 42, 47, 52):
        ya = torch.empty((N, H, W, Cout), device='cuda')
        yb = torch.full((N, H, W, Cout), float('nan'), device='cuda')
        ops.conv2d_dual_bn_act(x, C1, 1, 1, 0, x2, s2, w3, k1, sh, True, ya, tile=t)
        ops.conv2d_dual_bn_act(x, C1, 1, 1, 0, x2, s2, w3t, k1, sh, True, yb, tile=t | 0x100)
        assert torch.equal(ya, yb), 'tile %d' % t
