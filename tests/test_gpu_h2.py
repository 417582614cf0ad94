"""GPU parity of the f16x2 ("h2") distance path (csrc/gemm_h2.hip), the
default arithmetic of compute_dist since round 5:

* the split is exact where it must be: rscale is a power of two per row,
  max|x 2^s| in [2^14, 2^15), (h0 + h1) 2^-s reproduces x within 2^-22 of
  the row maximum, padding rows are zero, the squared norms are
  row_sqnorm's bits, and the chunk-tiled layout is [p][r//16][k//32][r%16][k%32];
* distances vs the reference's goldens and the oracle within the same bounds
  as the bf16x3 kernel (1e-4 absolute, north_star; typically ~1e-6), every
  metric, ragged shapes, every h2 tile bit-identical;
* the self-distance is exactly symmetric and its upper triangle has the bits
  of the full product;
* degenerate rows (zeros, huge and tiny magnitudes) stay finite and within
  the f32 bound of the NumPy formula.
Market-scale ranking parity (near-tie-exact top-k, mAP/CMC) is
tests/test_gpu_market_scale.py with math='h2'."""
import numpy as np
import pytest
import torch

from oracle import evaluator as ev

pytestmark = pytest.mark.gpu


def _cuda(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).cuda()


def _untile(t, R, D):
    """[2, R16, D] chunk-tiled int16 planes -> [2, R, D] f16 planes."""
    r16 = t.shape[1]
    u = t.reshape(2, r16 // 16, D // 32, 16, 32).permute(0, 1, 3, 2, 4).reshape(2, r16, D)
    return u.view(torch.float16)[:, :R], u.view(torch.float16)[:, R:]


@pytest.mark.parametrize('R,D', [(1, 32), (37, 96), (300, 2048), (33, 3968)])
def test_h2_split_exact(R, D):
    from pps_amd import ops
    rng = np.random.RandomState(R + D)
    xn = rng.randn(R, D).astype(np.float32) * np.exp(rng.uniform(-20, 20, (R, 1))).astype(
        np.float32)
    x = _cuda(xn)
    planes, rs, sq = ops.split_h2_tiled(x)
    assert planes.shape == (2, (R + 15) // 16 * 16, D)
    assert torch.equal(sq, ops.row_sqnorm(x))
    h, pad = _untile(planes, R, D)
    assert not bool(pad.float().abs().sum())
    rsn = rs.cpu().numpy().astype(np.float64)
    m, e = np.frexp(rsn)
    assert np.all(m == 0.5), 'rscale must be a power of two'
    h0 = h[0].float().cpu().numpy().astype(np.float64)
    h1 = h[1].float().cpu().numpy().astype(np.float64)
    y = xn.astype(np.float64) / rsn[:, None]          # x 2^s (exact)
    amax = np.abs(y).max(1)
    assert np.all((amax >= 2 ** 14) & (amax < 2 ** 15)), amax
    assert np.all(h0 == np.float16(y).astype(np.float64))   # round to nearest
    resid = np.abs(y - h0 - h1)
    assert np.all(resid <= 2.0 ** -22 * np.abs(y) + 2.0 ** -25), resid.max()


@pytest.mark.parametrize('case', ['market_small', 'full_dim'])
def test_h2_distmat_vs_golden(golden, case):
    from pps_amd import ops
    g = golden(case)
    if g['qf'].shape[1] % 32:
        pytest.skip('h2 needs D % 32 == 0 (compute_dist runs x3 otherwise)')
    d = ops.compute_dist(_cuda(g['qf']), _cuda(g['gf']), math='h2').cpu().numpy()
    np.testing.assert_allclose(d, g['dist'], rtol=0, atol=1e-4)
    assert np.abs(d - g['dist']).max() < 5e-6


@pytest.mark.parametrize('Q,G,D', [(1, 1, 32), (3, 5, 64), (33, 65, 96), (127, 129, 160),
                                   (200, 300, 2048), (64, 1000, 3968), (300, 257, 3968),
                                   (33, 65, 20)])
@pytest.mark.parametrize('metric', ['euclidean', 'sqeuclidean', 'cosine'])
def test_h2_ragged_shapes_all_tiles(Q, G, D, metric):
    """Every h2 tile: within the f32 bound of the oracle and bit-identical to
    the others (one K order, one term order).  D % 32 != 0 falls back to x3."""
    from pps_amd import ops
    rng = np.random.RandomState(Q * 7 + G + D)
    q = rng.randn(Q, D).astype(np.float32)
    g = rng.randn(G, D).astype(np.float32)
    ref = ev.compute_dist(q, g, metric)
    scale = max(1.0, float(np.abs(ref).max()))
    base = None
    for tile in range(ops.h2_num_tiles()):
        d = ops.compute_dist(_cuda(q), _cuda(g), metric=metric, tile=tile, math='h2')
        d = d.cpu().numpy()
        np.testing.assert_allclose(d, ref, rtol=0, atol=2e-5 * scale * np.sqrt(D / 128.0),
                                   err_msg='tile %d' % tile)
        if base is None:
            base = d
        np.testing.assert_array_equal(d, base, err_msg='tile %d' % tile)


def test_h2_gallery_index_and_padded_output():
    """A prepared h2 GalleryIndex scores any query batch with the bits of the
    one-call path, into dense and row-padded outputs and a row-strided block."""
    from pps_amd import ops
    rng = np.random.RandomState(3)
    q = _cuda(rng.randn(70, 256))
    g = _cuda(rng.randn(301, 256))
    idx = ops.GalleryIndex(g, math='h2')
    assert idx.math == 'h2'
    a = ops.compute_dist(q, idx)
    b = ops.compute_dist(q, g, math='h2', pad_rows=True)
    full = torch.zeros((70, 400), device='cuda')
    c = ops.compute_dist(q, idx, out=full[:, 50:351])
    assert torch.equal(a, b) and torch.equal(a, c)
    assert float(full[:, :50].abs().sum()) == 0 and float(full[:, 351:].abs().sum()) == 0


def test_h2_strided_gallery_and_math_mismatch():
    """A row-strided raw gallery (big[:, :D], D % 32 == 0) takes the h2 path
    with the bits of its contiguous copy (it used to reach the h2 GEMM with
    no h2 index); an explicit math that disagrees with a GalleryIndex's split
    is an error, not silently overridden."""
    from pps_amd import ops
    rng = np.random.RandomState(11)
    q = _cuda(rng.randn(40, 96))
    big = _cuda(rng.randn(130, 160))
    g = big[:, :96]
    assert not g.is_contiguous()
    a = ops.compute_dist(q, g, math='h2')
    b = ops.compute_dist(q, g.contiguous(), math='h2')
    assert torch.equal(a, b)
    ref = ev.compute_dist(q.cpu().numpy(), g.cpu().numpy())
    assert np.abs(a.cpu().numpy() - ref).max() < 1e-4
    idx = ops.GalleryIndex(g.contiguous(), math='h2')
    with pytest.raises(RuntimeError, match='GalleryIndex'):
        ops.compute_dist(q, idx, math='x3')
    assert torch.equal(ops.compute_dist(q, idx, math='h2'), a)
    # f32 reads the index's features as they are
    f = ops.compute_dist(q, idx, math='f32').cpu().numpy()
    assert np.abs(f - ref).max() < 1e-4


@pytest.mark.parametrize('N,D', [(1000, 3968), (700, 256), (301, 64), (17, 32), (513, 2048)])
@pytest.mark.parametrize('metric', ['euclidean', 'cosine'])
def test_h2_self_distance_symmetric(N, D, metric):
    from pps_amd import ops
    rng = np.random.RandomState(N + D)
    xn = rng.randn(N, D).astype(np.float32)
    xn /= np.linalg.norm(xn, axis=1, keepdims=True)
    x = _cuda(xn)
    ref = ev.compute_dist(xn, xn, metric) if metric == 'euclidean' else None
    for tile in range(ops.h2_num_tiles()):
        dt = ops.compute_dist(x, x, metric=metric, tile=tile, math='h2')
        assert getattr(dt, '_pps_symmetric', False)
        d = dt.cpu().numpy()
        full = ops.compute_dist(x, x, metric=metric, tile=tile, symmetric=False,
                                math='h2').cpu().numpy()
        np.testing.assert_array_equal(d, d.T, err_msg='tile %d' % tile)
        iu = np.triu_indices(N)
        np.testing.assert_array_equal(d[iu], full[iu], err_msg='tile %d' % tile)
        if ref is not None:   # the diagonal: sqrt of cancelled rounding noise (test_gpu_x3)
            off = ~np.eye(N, dtype=bool)
            np.testing.assert_allclose(d[off], ref[off], rtol=0, atol=1e-4)
            assert np.abs(np.diag(d) - np.diag(ref)).max() < 5e-3


def test_h2_degenerate_rows():
    """Zero rows, rows of magnitude 1e17 and 1e-30 (per-row scales reach the
    ends of the f32 exponent range): finite, and within the f32 bound of the
    float64 formula relative to the operands' magnitudes."""
    from pps_amd import ops
    rng = np.random.RandomState(9)
    D = 128
    q = rng.randn(6, D).astype(np.float32)
    q[1] = 0
    q[2] *= 1e17
    q[3] *= 1e-30
    q[4, :] = 0
    q[4, 7] = 3.0          # one non-zero entry
    g = rng.randn(9, D).astype(np.float32)
    g[0] = 0
    g[3] *= 1e-30
    g[5] *= 1e17
    d = ops.compute_dist(_cuda(q), _cuda(g), metric='sqeuclidean', math='h2').cpu().numpy()
    assert np.all(np.isfinite(d))
    qd, gd = q.astype(np.float64), g.astype(np.float64)
    ref = (qd ** 2).sum(1)[:, None] + (gd ** 2).sum(1)[None] - 2 * qd @ gd.T
    mag = (np.abs(qd) ** 2).sum(1)[:, None] + (np.abs(gd) ** 2).sum(1)[None]
    assert np.all(np.abs(d - np.maximum(ref, 0)) <= 1e-5 * mag + 1e-30)


def test_h2_enforces_shapes():
    from pps_amd import ops
    x = torch.zeros((4, 64), device='cuda')
    p, rs, sq = ops.split_h2_tiled(x)
    out = torch.empty((4, 4), device='cuda')
    with pytest.raises(RuntimeError, match='h2 tile'):
        ops.call('pps_distmat_h2_tiled', p.data_ptr(), 4, sq.data_ptr(), rs.data_ptr(),
                 p.data_ptr(), sq.data_ptr(), rs.data_ptr(), 4, 64, 0, out.data_ptr(), 4,
                 ops.h2_num_tiles(), ops._stream())
    with pytest.raises(RuntimeError, match='D % 32'):
        ops.call('pps_split_f16x2_sqnorm_tiled', x.data_ptr(), 4, 48, 64, p.data_ptr(),
                 rs.data_ptr(), sq.data_ptr(), ops._stream())
