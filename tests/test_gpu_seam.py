"""The bottleneck seam kernel (pps_conv1x1_seam_x3, csrc/gemm_seam.hip):
branch2c of an identity block + branch2a of the next block in one launch
(ResNet.py:276-333).  Both outputs must equal the two convolutions run
separately on 16x16x32-block tiles (their rounding group) bit for bit, and
be within f32 tolerance of a float64 reference."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cuda(x):
    return torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda()


@pytest.mark.parametrize('N,H,W,K1', [(2, 96, 32, 64), (1, 7, 9, 64), (2, 48, 16, 128),
                                      (3, 5, 7, 128), (64, 96, 32, 64)])
def test_seam_equals_two_convs(N, H, W, K1):
    from pps_amd import model, ops
    N1, N2 = 4 * K1, K1
    rng = np.random.RandomState(N * H + K1)
    x = np.maximum(rng.randn(N, H, W, K1), 0).astype(np.float32)        # post-ReLU 2b output
    res = np.maximum(rng.randn(N, H, W, N1), 0).astype(np.float32)      # the block's trunk
    w2c = (rng.randn(N1, K1, 1, 1) / np.sqrt(K1)).astype(np.float32)
    w2a = (rng.randn(N2, N1, 1, 1) / np.sqrt(N1)).astype(np.float32)
    s2c, t2c = rng.uniform(0.5, 1.5, N1).astype(np.float32), (0.1 * rng.randn(N1)).astype(np.float32)
    s2a, t2a = rng.uniform(0.5, 1.5, N2).astype(np.float32), (0.1 * rng.randn(N2)).astype(np.float32)
    pc, kc = model.pack_conv_weight(w2c)
    pa, ka = model.pack_conv_weight(w2a)
    assert kc == K1 and ka == N1
    w2c3, w2a3 = ops.split_bf16x3(_cuda(pc)), ops.split_bf16x3(_cuda(pa))
    xd, rd = _cuda(x), _cuda(res)
    dev = dict(s2c=_cuda(s2c), t2c=_cuda(t2c), s2a=_cuda(s2a), t2a=_cuda(t2a))
    trunk = torch.full((N, H, W, N1), float('nan'), device='cuda')
    y = torch.full((N, H, W, N2), float('nan'), device='cuda')
    ops.conv1x1_seam(xd, w2c3, dev['s2c'], dev['t2c'], rd, trunk, w2a3, dev['s2a'], dev['t2a'], y)
    # the two layers separately, on tiles of the 16x16x32 group
    for tile in (ops.TILE_P16_FIRST, 54, ops.TILE_P16_FIRST + 9):
        t2 = torch.full_like(trunk, float('nan'))
        y2 = torch.full_like(y, float('nan'))
        ops.conv2d_bn_act_x3p(xd, K1, w2c3, kc, 1, 1, 0, 1, dev['s2c'], dev['t2c'], rd, True, t2,
                              tile=tile)
        ops.conv2d_bn_act_x3p(t2, N1, w2a3, ka, 1, 1, 0, 1, dev['s2a'], dev['t2a'], None, True,
                              y2, tile=tile)
        assert torch.equal(trunk, t2), 'trunk vs tile %d' % tile
        assert torch.equal(y, y2), 'y vs tile %d' % tile
    # float64 reference
    t64 = np.maximum(x.astype(np.float64) @ pc.astype(np.float64).T * s2c + t2c + res, 0)
    y64 = np.maximum(t64 @ pa.astype(np.float64).T * s2a + t2a, 0)
    tn, yn = trunk.cpu().numpy(), y.cpu().numpy()
    assert np.abs(tn - t64).max() <= 1e-5 * max(1.0, np.abs(t64).max())
    assert np.abs(yn - y64).max() <= 1e-5 * max(1.0, np.abs(y64).max())


def test_seam_rejects_other_shapes():
    from pps_amd import ops
    z = torch.zeros((4, 96), device='cuda')
    w = torch.zeros((3, 96, 96), dtype=torch.int16, device='cuda')
    s = torch.ones(96, device='cuda')
    with pytest.raises(RuntimeError, match='bottleneck seam'):
        ops.conv1x1_seam(z, w, s, s, torch.zeros((4, 96), device='cuda'),
                         torch.zeros((4, 96), device='cuda'), w, s, s, torch.zeros((4, 96),
                                                                                   device='cuda'))
