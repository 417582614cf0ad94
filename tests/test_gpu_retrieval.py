"""GPU parity: distance matrix, PairWiseDistance, count-based mAP/CMC and top-k
against the oracle and the reference's golden vectors.

Tolerances: distances within 1e-4 absolute (north_star), typically ~1e-6;
AP per query within 1e-9 when no rank flips (fp32 accumulation order differs
from NumPy's sgemm, so near-tied distances may order differently: asserted
bit-exact where the golden distance gap exceeds 1e-5)."""
import numpy as np
from _tiles import check_tile_bits
import pytest
import torch

from oracle import evaluator as ev

pytestmark = pytest.mark.gpu


def _cuda(x, dtype=torch.float32):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dtype).cuda()


@pytest.mark.parametrize('math', ['x3', 'f32'])
@pytest.mark.parametrize('case', ['market_small', 'full_dim'])
def test_distmat_vs_golden(golden, case, math):
    from pps_amd import ops
    g = golden(case)
    d = ops.compute_dist(_cuda(g['qf']), _cuda(g['gf']), math=math).cpu().numpy()
    np.testing.assert_allclose(d, g['dist'], rtol=0, atol=1e-4)
    assert np.abs(d - g['dist']).max() < 5e-6


@pytest.mark.parametrize('Q,G,D', [(1, 1, 4), (3, 5, 8), (33, 65, 20), (127, 129, 132),
                                   (200, 300, 2048), (64, 1000, 3968)])
@pytest.mark.parametrize('metric', ['euclidean', 'sqeuclidean', 'cosine'])
@pytest.mark.parametrize('math', ['x3', 'f32'])
def test_distmat_ragged_shapes(Q, G, D, metric, math):
    from pps_amd import ops
    rng = np.random.RandomState(Q * 7 + G)
    q = rng.randn(Q, D).astype(np.float32)
    g = rng.randn(G, D).astype(np.float32)
    ref = ev.compute_dist(q, g, metric)
    scale = max(1.0, float(np.abs(ref).max()))
    outs = []
    for tile in range(0, ops.num_tiles() + 1):
        d = ops.compute_dist(_cuda(q), _cuda(g), metric=metric, tile=tile,
                             math=math).cpu().numpy()
        np.testing.assert_allclose(d, ref, rtol=0, atol=2e-5 * scale * np.sqrt(D / 128.0),
                                   err_msg='tile %d' % tile)
        outs.append(d)
    check_tile_bits(range(0, ops.num_tiles() + 1), outs, ops.TILE_P16_FIRST)


def test_gallery_index_matches_plain_x3():
    from pps_amd import ops
    rng = np.random.RandomState(11)
    q = _cuda(rng.randn(70, 256).astype(np.float32))
    g = _cuda(rng.randn(300, 256).astype(np.float32))
    idx = ops.GalleryIndex(g, math='x3')
    a = ops.compute_dist(q, idx).cpu().numpy()
    b = ops.compute_dist(q, g, math='x3').cpu().numpy()
    np.testing.assert_array_equal(a, b)
    sq = ops.row_sqnorm(g).cpu().numpy()
    np.testing.assert_allclose(sq, (g.double() ** 2).sum(1).cpu().numpy(), rtol=2e-6)


@pytest.mark.parametrize('R,D', [(1, 32), (37, 96), (300, 2048), (33, 3968)])
def test_tiled_planes_layout(R, D):
    """split_sqnorm_tiled == tile_planes(split_sqnorm) bit for bit; the tiled
    layout holds element (r, k) of plane p at [p][r // 16][k // 32][r % 16]
    [k % 32] and zeros in the padding rows."""
    from pps_amd import ops
    x = _cuda(np.random.RandomState(R + D).randn(R, D).astype(np.float32))
    planes, sq = ops.split_sqnorm(x)
    t1 = ops.tile_planes(planes)
    t2, sq2 = ops.split_sqnorm_tiled(x)
    assert torch.equal(t1, t2) and torch.equal(sq, sq2)
    r16 = (R + 15) // 16 * 16
    want = torch.zeros((3, r16, D), dtype=torch.int16, device='cuda')
    want[:, :R] = planes
    want = want.reshape(3, r16 // 16, 16, D // 32, 32).permute(0, 1, 3, 2, 4).reshape(3, r16, D)
    assert torch.equal(t2, want)


@pytest.mark.parametrize('Q,G,D', [(45, 77, 96), (64, 1000, 3968), (3, 17, 32)])
@pytest.mark.parametrize('metric', ['euclidean', 'cosine'])
def test_distmat_tiled_planes_bits(Q, G, D, metric):
    """compute_dist(q_planes=True) streams chunk-tiled planes of both operands
    (pps_distmat_x3p_tiled); it equals the row-major planes GEMM
    (pps_distmat_x3p) bit for bit on every tile, and the tiles keep their
    rounding groups."""
    from pps_amd import ops
    rng = np.random.RandomState(Q + G)
    q = _cuda(rng.randn(Q, D).astype(np.float32))
    g = _cuda(rng.randn(G, D).astype(np.float32))
    idx = ops.GalleryIndex(g, math='x3')
    q3, qsq = ops.split_sqnorm(q)
    tiles = [0] + list(range(ops.TILE_P_FIRST, ops.num_tiles() + 1))
    outs = []
    for tile in tiles:
        a = ops.compute_dist(q, g, metric=metric, tile=tile, q_planes=True, pad_rows=True,
                             math='x3')
        b = ops.dist_buffer(Q, G, 'cuda')
        ops.call('pps_distmat_x3p', ops._dev(q3, 'q3', torch.int16), Q, D, ops._dev(qsq, 'qsq'),
                 ops._dev(idx.planes, 'g3', torch.int16), ops._dev(idx.sqnorm, 'gsq'), G, D, D,
                 ops.METRICS[metric], ops._dev_rows(b, 'out'), ops._ld(b),
                 ops._tiled_tile(tile), ops._stream())
        assert torch.equal(a, b), 'tile %d' % tile
        outs.append(a.cpu().numpy())
    check_tile_bits(tiles, outs, ops.TILE_P16_FIRST)


def test_distmat_enforces_shapes():
    from pps_amd import ops
    with pytest.raises(RuntimeError):
        ops.compute_dist(torch.zeros(3, 6, device='cuda'), torch.zeros(4, 6, device='cuda'))
    with pytest.raises(RuntimeError):
        ops.compute_dist(torch.zeros(3, 8, device='cuda'), torch.zeros(4, 4, device='cuda'))


def test_pairwise_distance_op():
    from pps_amd import ops
    rng = np.random.RandomState(1)
    X = rng.randn(64, 128).astype(np.float32)   # PPS triplet shape (P=8,K=8)
    Z = ops.run_op('PairWiseDistance', [_cuda(X)])[0].cpu().numpy()
    ref = ev.pairwise_distance(X)
    np.testing.assert_allclose(Z, ref, rtol=1e-5, atol=1e-4)
    assert np.all(np.diag(Z) == 0)
    with pytest.raises(RuntimeError, match='X.dim'):
        ops.run_op('PairWiseDistance', [torch.zeros(4, device='cuda')])


@pytest.mark.parametrize('case', ['market_small', 'full_dim', 'ties'])
def test_rank_eval_vs_golden(golden, case):
    from pps_amd import reid_dataset_evaluator as gev
    g = golden(case)
    # use the reference's own float32 distances as input: isolates the ranking
    ap, valid, first = gev.rank_eval(g['dist'], g['qid'], g['gid'], g['qcam'], g['gcam'])
    ap, valid = ap.cpu().numpy(), valid.cpu().numpy()
    np.testing.assert_array_equal(valid, g['valid_ap'])
    np.testing.assert_allclose(ap, g['aps'], rtol=0, atol=1e-12)
    if 'cmc_all' in g:
        ret, v2 = gev.cmc(g['dist'], g['qid'], g['gid'], g['qcam'], g['gcam'], topk=10,
                          first_match_break=True, average=False)
        np.testing.assert_array_equal(ret, g['cmc_all'])
        m = gev.mean_ap(g['dist'], g['qid'], g['gid'], g['qcam'], g['gcam'])
        assert abs(m - float(g['mAP'])) < 1e-12


def test_rank_eval_edge_cases():
    from pps_amd import reid_dataset_evaluator as gev
    rng = np.random.RandomState(3)
    Q, G = 9, 40
    dist = rng.rand(Q, G).astype(np.float32)
    qid = np.arange(Q)
    qcam = np.ones(Q, int)
    gid = rng.randint(0, Q, size=G)
    gcam = rng.randint(1, 3, size=G)
    gid[:5] = 0
    gcam[:5] = 1            # query 0: all same-id gallery entries are junk
    gid[gid == 0] = 0
    ap, valid, first = gev.rank_eval(dist, qid, gid, qcam, gcam)
    ref_ap, ref_valid = ev.mean_ap(dist, qid, gid, qcam, gcam, average=False)
    np.testing.assert_array_equal(valid.cpu().numpy(), ref_valid)
    np.testing.assert_allclose(ap.cpu().numpy(), ref_ap, atol=1e-12)
    ret, _ = ev.cmc(dist, qid, gid, qcam, gcam, topk=G, first_match_break=True,
                    average=False)
    f = first.cpu().numpy()
    for i in range(Q):
        if ref_valid[i]:
            assert ret[i].argmax() == f[i]
        else:
            assert f[i] == -1


def test_rank_eval_more_positives_than_first_guess():
    """A query with more true matches than rank_eval's first positive-list
    capacity (64) is re-collected at the exact size: same AP / first match."""
    from pps_amd import reid_dataset_evaluator as gev
    rng = np.random.RandomState(5)
    Q, G = 4, 700
    dist = rng.rand(Q, G).astype(np.float32)
    qid = np.array([1, 2, 3, 4])
    qcam = np.array([1, 1, 2, 2])
    gid = rng.randint(2, 9, size=G)
    gid[:300] = 1                          # query 0: ~250 positives + junk
    gcam = rng.randint(1, 7, size=G)
    ap, valid, first = gev.rank_eval(dist, qid, gid, qcam, gcam)
    ref_ap, ref_valid = ev.mean_ap(dist, qid, gid, qcam, gcam, average=False)
    np.testing.assert_array_equal(valid.cpu().numpy(), ref_valid)
    np.testing.assert_allclose(ap.cpu().numpy(), ref_ap, atol=1e-12)
    ret, _ = ev.cmc(dist, qid, gid, qcam, gcam, topk=G, first_match_break=True,
                    average=False)
    f = first.cpu().numpy()
    for i in range(Q):
        assert (ret[i].argmax() == f[i]) if ref_valid[i] else (f[i] == -1)


def test_rank_eval_exact_ties_stable_order():
    """Tied distances: CMC uses the stable (distance, index) order."""
    from pps_amd import reid_dataset_evaluator as gev
    dist = np.array([[0.5, 0.5, 0.5, 0.2, 0.5]], np.float32)
    qid, qcam = np.array([7]), np.array([1])
    gid = np.array([3, 7, 7, 4, 7])
    gcam = np.array([2, 2, 1, 2, 3])          # index 2 is junk (same id, same cam)
    ap, valid, first = gev.rank_eval(dist, qid, gid, qcam, gcam)
    ref_ap, _ = ev.mean_ap(dist, qid, gid, qcam, gcam, average=False)
    assert abs(float(ap[0]) - ref_ap[0]) < 1e-12
    ret, _ = ev.cmc(dist, qid, gid, qcam, gcam, topk=5, first_match_break=True,
                    average=False)
    assert int(first[0]) == int(ret[0].argmax()) == 2


@pytest.mark.parametrize('k', [1, 10, 100, 457])
def test_topk_stable(golden, k):
    from pps_amd import ops
    g = golden('market_small')
    d = _cuda(g['dist'])
    vals, idx = ops.topk(d, k)
    order = g['order_stable'][:, :k]
    np.testing.assert_array_equal(idx.cpu().numpy(), order)
    np.testing.assert_array_equal(vals.cpu().numpy(),
                                  np.take_along_axis(g['dist'], order, axis=1))


def test_topk_ties_and_negatives():
    from pps_amd import ops
    rng = np.random.RandomState(0)
    d = rng.randint(-3, 4, size=(5, 3000)).astype(np.float32)
    vals, idx = ops.topk(_cuda(d), 50)
    ref = np.argsort(d, axis=1, kind='stable')[:, :50]
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)


@pytest.mark.parametrize('k', [21, 100])
def test_topk_many_rows_odd_stride(k):
    """Re-ranking shapes (DukeMTMC: N = Q + G = 19,889 rows of OD, odd row
    stride, k = k1 + 1 = 21): every row's stable top-k equals NumPy's.  Many
    blocks per CU exercise the candidate-count snapshot (all waves must take
    the same cut decision in every chunk)."""
    from pps_amd import ops
    rng = np.random.RandomState(k)
    Q, G = 1536, 19889
    d = rng.rand(Q, G).astype(np.float32)
    d[::7, ::5] = 0.25  # ties
    vals, idx = ops.topk(_cuda(d), k)
    ref = np.argsort(d, axis=1, kind='stable')[:, :k]
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)
    np.testing.assert_array_equal(vals.cpu().numpy(), np.take_along_axis(d, ref, axis=1))


@pytest.mark.parametrize('G', [1, 3, 4, 4097, 8190, 16387, 19889])
def test_topk_padded_rows_vector_path(G):
    """16-byte rows (ops.dist_buffer pads the stride to 4 floats) take the
    dwordx4 path with two chunks of lookahead; the < 4 entries past the last
    full vector are taken by the scalar tail.  Stable order vs NumPy, with
    ties and negative distances."""
    from pps_amd import ops
    rng = np.random.RandomState(G)
    Q = 300
    d = rng.randint(-50, 50, size=(Q, G)).astype(np.float32) / 8
    d[:, -1] = -100.0  # the very last entry is every row's best
    buf = ops.dist_buffer(Q, G, 'cuda')
    assert buf.stride(0) % 4 == 0
    buf.copy_(torch.from_numpy(d))
    for k in (1, 21, 100):
        kk = min(k, G)
        vals, idx = ops.topk(buf, kk)
        ref = np.argsort(d, axis=1, kind='stable')[:, :kk]
        np.testing.assert_array_equal(idx.cpu().numpy(), ref)
        np.testing.assert_array_equal(vals.cpu().numpy(), np.take_along_axis(d, ref, axis=1))


def test_evaluate_vs_golden(golden):
    from pps_amd import reid_dataset_evaluator as gev
    from pps_amd.config import cfg
    cfg.REID.RERANK = False
    g = golden('evaluate')
    mAP, cmc, mq, _ = gev.evaluate_arrays(g['feat'], g['ids'], g['cams'], g['marks'],
                                          verbose=False)
    assert abs(mAP - float(g['mAP'])) < 1e-9
    np.testing.assert_allclose(cmc, g['cmc'], atol=1e-12)


def test_re_ranking_vs_golden(golden):
    """k-reciprocal re-ranking on the GPU vs the reference's own output."""
    from pps_amd import reid_dataset_evaluator as gev
    g = golden('rerank')
    rr = gev.re_ranking(g['q_g'], g['q_q'], g['g_g'], k1=20, k2=6, lambda_value=0.3)
    np.testing.assert_allclose(rr, g['rerank'], rtol=0, atol=1e-5)
    m = gev.mean_ap(rr, g['qid'], g['gid'], g['qcam'], g['gcam'])
    assert abs(m - float(g['mAP'])) < 1e-6


@pytest.mark.parametrize('k1,k2', [(20, 6), (10, 1), (6, 3), (24, 8)])
def test_re_ranking_vs_oracle_params(k1, k2):
    from pps_amd import reid_dataset_evaluator as gev
    rng = np.random.RandomState(k1 + k2)
    x = rng.randn(150, 32).astype(np.float32)
    q, g = x[:30], x[30:]
    qg, qq, gg = ev.compute_dist(q, g), ev.compute_dist(q, q), ev.compute_dist(g, g)
    ref = ev.re_ranking(qg, qq, gg, k1=k1, k2=k2, lambda_value=0.3)
    rr = gev.re_ranking(qg, qq, gg, k1=k1, k2=k2, lambda_value=0.3)
    np.testing.assert_allclose(rr, ref, rtol=0, atol=1e-5)


@pytest.mark.parametrize('Q,G,metric', [(300, 1700, 'cosine'), (77, 2100, 'euclidean')])
def test_re_ranking_symmetric_path_bit_identical(Q, G, metric):
    """PPS_RERANK_SYMMETRIC (row-streamed N x N build, only q_g^T transposed)
    gives the same bits as the transposing build on the mirrored self-distance
    GEMM's exactly symmetric q_q / g_g, and both match the oracle."""
    from pps_amd import ops
    rng = np.random.RandomState(Q)
    x = rng.randn(Q + G, 64).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    xd = torch.from_numpy(x).cuda()
    q, g = xd[:Q].contiguous(), xd[Q:].contiguous()
    qg = ops.compute_dist(q, g, metric=metric)
    qq = ops.compute_dist(q, q, metric=metric)
    gg = ops.compute_dist(g, g, metric=metric)
    assert getattr(qq, '_pps_symmetric', False) and getattr(gg, '_pps_symmetric', False)
    assert torch.equal(gg, gg.t()) and torch.equal(qq, qq.t())
    sym = ops.re_ranking(qg, qq, gg)
    asym = ops.re_ranking(qg, qq, gg, symmetric=False)
    assert torch.equal(sym, asym)
    ref = ev.re_ranking(qg.cpu().numpy(), qq.cpu().numpy(), gg.cpu().numpy(), k1=20, k2=6,
                        lambda_value=0.3)
    np.testing.assert_allclose(sym.cpu().numpy(), ref, rtol=0, atol=1e-5)


def test_evaluate_with_rerank_vs_oracle(golden):
    from pps_amd import reid_dataset_evaluator as gev
    from pps_amd.config import cfg
    g = golden('evaluate')
    cfg.REID.RERANK = True
    mAP, cmc, _, _ = gev.evaluate_arrays(g['feat'], g['ids'], g['cams'], g['marks'],
                                         verbose=False)
    ref = ev.evaluate_arrays(g['feat'], g['ids'], g['cams'], g['marks'], rerank=True)
    assert abs(mAP - ref[0]) < 1e-6
    np.testing.assert_allclose(cmc, ref[1], atol=1e-9)


def test_multi_query_pooling_vs_oracle():
    """marks == 2 (multi-query): per-(id, cam) mean features, then scores."""
    from pps_amd import reid_dataset_evaluator as gev
    from pps_amd.config import cfg
    cfg.REID.RERANK = False
    rng = np.random.RandomState(9)
    x = rng.randn(200, 64).astype(np.float32)
    ids = rng.randint(1, 15, 200)
    cams = rng.randint(1, 4, 200)
    marks = rng.choice([0, 1, 1, 2], 200)
    res = gev.evaluate_arrays(x, ids, cams, marks, verbose=False)
    ref = ev.evaluate_arrays(x, ids, cams, marks)
    assert abs(res[0] - ref[0]) < 1e-9 and abs(res[2] - ref[2]) < 1e-9
    np.testing.assert_allclose(res[3], ref[3], atol=1e-12)


def test_rank_eval_long_positive_lists_and_unaligned_rows():
    """The streaming count pass with a positive list too long for LDS (the
    global-memory path: 7000 matches) and rows that are not 16-byte aligned
    (odd G: the scalar path), plus junk entries removed after the stream."""
    from pps_amd import reid_dataset_evaluator as gev
    rng = np.random.RandomState(8)
    Q, G = 6, 20001
    dist = rng.rand(Q, G).astype(np.float32)
    dist[:, ::97] = 0.5                                   # ties
    qid = np.array([1, 2, 3, 1, 5, 9])
    qcam = np.array([1, 2, 1, 3, 1, 1])
    gid = rng.randint(2, 50, size=G)
    gid[:7500] = 1
    gcam = rng.randint(1, 7, size=G)
    ap, valid, first = gev.rank_eval(dist, qid, gid, qcam, gcam)
    ref_ap, ref_valid = ev.mean_ap(dist, qid, gid, qcam, gcam, average=False)
    np.testing.assert_array_equal(valid.cpu().numpy(), ref_valid)
    np.testing.assert_allclose(ap.cpu().numpy(), ref_ap, rtol=0, atol=1e-12)
    np.testing.assert_array_equal(first.cpu().numpy(),
                                  ev.first_match_rank(dist, qid, gid, qcam, gcam))


def test_rank_eval_padded_rows_view(golden):
    """A [Q, G] view of a wider, 16-byte-padded buffer (row stride > G): the
    same per-query results as the dense matrix."""
    from pps_amd import reid_dataset_evaluator as gev
    g = golden('market_small')
    d = g['dist']
    Q, G = d.shape
    buf = torch.full((Q, G + 3), float('nan'), device='cuda')
    buf[:, :G] = _cuda(d)
    view = buf[:, :G]
    a1 = [t.cpu().numpy() for t in gev.rank_eval(view, g['qid'], g['gid'], g['qcam'], g['gcam'])]
    a2 = [t.cpu().numpy() for t in gev.rank_eval(d, g['qid'], g['gid'], g['qcam'], g['gcam'])]
    for x, y in zip(a1, a2):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_allclose(a1[0], g['aps'], rtol=0, atol=1e-12)


@pytest.mark.parametrize('tag', ['market_small', 'dense'])
def test_cmc_all_modes_vs_reference_golden(golden, tag):
    """The reference `cmc` with its own defaults (topk=100, fractional
    first_match_break=False) and with separate_camera_set=True, on the
    reference's distances (cmc_modes.npz): per-query rows bit-exact."""
    from pps_amd import reid_dataset_evaluator as gev
    g = golden('cmc_modes')
    d, qid, gid = g[tag + '_dist'], g[tag + '_qid'], g[tag + '_gid']
    qcam, gcam = g[tag + '_qcam'], g[tag + '_gcam']
    for sep in (0, 1):
        for fmb in (0, 1):
            key = '%s_sep%d_fmb%d' % (tag, sep, fmb)
            ret, valid = gev.cmc(d, qid, gid, qcam, gcam, separate_camera_set=bool(sep),
                                 first_match_break=bool(fmb), average=False)
            np.testing.assert_array_equal(valid, g[key + '_valid'], err_msg=key)
            np.testing.assert_array_equal(ret, g[key + '_all'], err_msg=key)
            avg = gev.cmc(d, qid, gid, qcam, gcam, separate_camera_set=bool(sep),
                          first_match_break=bool(fmb))
            np.testing.assert_array_equal(avg, g[key], err_msg=key)
    np.testing.assert_array_equal(gev.cmc(d, qid, gid, qcam, gcam), g[tag + '_default'])
    np.testing.assert_array_equal(gev.cmc(d, qid, gid, qcam, gcam, topk=5,
                                          separate_camera_set=True),
                                  g[tag + '_sep1_fmb0_top5'])


SGS_CASES = ((0, False, False, 100), (1, True, False, 100), (2, False, True, 20),
             (3, True, True, 10))


def test_cmc_single_gallery_shot_vs_reference_golden(golden):
    """cmc(single_gallery_shot=True) against the reference's own output
    (cmc_sgs.npz: the reference cmc run after np.random.seed(s)): the same
    global-RNG draws in the same order -> per-query rows and averages
    bit-exact, and the RNG left in the same state."""
    from pps_amd import reid_dataset_evaluator as gev
    g = golden('cmc_sgs')
    d, qid, gid, qcam, gcam = g['dist'], g['qid'], g['gid'], g['qcam'], g['gcam']
    for seed, sep, fmb, topk in SGS_CASES:
        key = 'seed%d_sep%d_fmb%d_top%d' % (seed, sep, fmb, topk)
        kw = dict(topk=topk, separate_camera_set=sep, single_gallery_shot=True,
                  first_match_break=fmb)
        np.random.seed(seed)
        ret, valid = gev.cmc(d, qid, gid, qcam, gcam, average=False, **kw)
        np.testing.assert_array_equal(valid, g[key + '_valid'], err_msg=key)
        np.testing.assert_array_equal(ret, g[key + '_all'], err_msg=key)
        np.random.seed(seed)
        np.testing.assert_array_equal(gev.cmc(d, qid, gid, qcam, gcam, **kw), g[key],
                                      err_msg=key)
        assert np.random.randint(1 << 30) == g[key + '_next_draw'], key


@pytest.mark.parametrize('Q,G,n_ids,seed', [(40, 3000, 100, 0), (25, 700, 12, 1),
                                            (7, 1, 1, 2), (30, 18240, 40, 3)])
def test_cmc_single_gallery_shot_vs_oracle(Q, G, n_ids, seed):
    """Larger / ragged cases vs the oracle (the reference's loop with a
    RandomState): many identities, few identities with long groups, a
    one-entry gallery, and the argsort cap; query identities missing from the
    gallery (skipped, no draws), junk ids, repeated cameras."""
    from pps_amd import reid_dataset_evaluator as gev
    rng = np.random.RandomState(seed)
    d = rng.rand(Q, G).astype(np.float32)
    gid = rng.randint(-1, n_ids, size=G)
    qid = rng.randint(0, n_ids + 3, size=Q)
    qcam = rng.randint(1, 4, size=Q)
    gcam = rng.randint(1, 4, size=G)
    for sep in (False, True):
        for fmb in (False, True):
            kw = dict(topk=50, separate_camera_set=sep, single_gallery_shot=True,
                      first_match_break=fmb, average=False)
            try:
                want = ev.cmc(d, qid, gid, qcam, gcam, rng=np.random.RandomState(seed + 10), **kw)
            except RuntimeError:   # no valid query
                with pytest.raises(RuntimeError, match='No valid query'):
                    gev.cmc(d, qid, gid, qcam, gcam, rng=np.random.RandomState(seed + 10), **kw)
                continue
            got = gev.cmc(d, qid, gid, qcam, gcam, rng=np.random.RandomState(seed + 10), **kw)
            np.testing.assert_array_equal(got[1], want[1])
            np.testing.assert_array_equal(got[0], want[0])


def test_cmc_single_gallery_shot_many_identities():
    """Thousands of gallery identities (the groups kernel's LDS holds two
    ints per identity: ~80 KB here) vs the oracle, one mode."""
    from pps_amd import reid_dataset_evaluator as gev
    rng = np.random.RandomState(7)
    Q, G, n_ids = 3, 12000, 5000
    d = rng.rand(Q, G).astype(np.float32)
    gid = rng.randint(0, n_ids, size=G)
    qid = gid[rng.randint(0, G, size=Q)]
    qcam = rng.randint(1, 4, size=Q)
    gcam = rng.randint(1, 4, size=G)
    kw = dict(topk=100, single_gallery_shot=True, average=False)
    want = ev.cmc(d, qid, gid, qcam, gcam, rng=np.random.RandomState(3), **kw)
    got = gev.cmc(d, qid, gid, qcam, gcam, rng=np.random.RandomState(3), **kw)
    np.testing.assert_array_equal(got[1], want[1])
    np.testing.assert_array_equal(got[0], want[0])


def test_cmc_counts_sharded_equal_unsharded(golden):
    """pps_cmc_counts is additive over gallery shards (global indices)."""
    from pps_amd import ops
    g = golden('cmc_modes')
    d = torch.from_numpy(g['dense_dist']).cuda()
    qid, gid, qcam, gcam = g['dense_qid'], g['dense_gid'], g['dense_qcam'], g['dense_gcam']
    G = d.shape[1]
    full_idx = ops.MatchIndex(qid, qcam, gid, gcam)
    pd, pi, pc, junk = ops.collect_matches(d, full_idx)
    sp = ops.rank_prepare(pd[None], pi[None], pc[None])
    want = ops.cmc_counts(d, 0, sp, junk)
    cuts = [0, G // 3, G]
    lists, shards = [], []
    for a, b in zip(cuts[:-1], cuts[1:]):
        ds = d[:, a:b].contiguous()
        idx = ops.MatchIndex(qid, qcam, gid[a:b], gcam[a:b])
        p = ops.collect_matches(ds, idx, a, full_idx.capacity)
        lists.append(p[:3])
        shards.append((ds, a, p[3]))
    sp2 = ops.rank_prepare(torch.stack([l[0] for l in lists]), torch.stack([l[1] for l in lists]),
                           torch.stack([l[2] for l in lists]))
    hist = None
    for ds, a, junk_s in shards:
        hist = ops.cmc_counts(ds, a, sp2, junk_s, hist=hist)
    r1, v1 = ops.cmc_finalize(sp.pos_total, want, 100, False)
    r2, v2 = ops.cmc_finalize(sp2.pos_total, hist, 100, False)
    assert torch.equal(v1, v2) and torch.equal(r1, r2)


@pytest.mark.parametrize('G,k', [(16384, 1), (40003, 100), (40000, 256), (125001, 100),
                                 (20001, 257)])
def test_topk_long_rows_wave_kernel(G, k):
    """Long rows (>= 16384 entries, k <= 256: the per-wave streaming kernel of
    the 1M-gallery shards; k = 257 stays on the block kernel): the stable
    (distance, index) top-k equals NumPy's, with heavy ties, negative values,
    the < 4-entry tail (odd G, padded rows), and adversarial rows whose
    values only decrease (every entry beats the running threshold, so every
    iteration cuts)."""
    from pps_amd import ops
    rng = np.random.RandomState(G + k)
    Q = 24
    d = rng.randint(-40, 40, size=(Q, G)).astype(np.float32) / 4   # many ties
    d[1] = rng.rand(G).astype(np.float32)
    d[2] = -np.arange(G, dtype=np.float32)                            # strictly decreasing
    d[3] = 1.0                                                        # all tied
    d[4, -1] = -1e9                                                   # best entry in the tail
    d[5, :G // 2] = np.linspace(1, 0, G // 2, dtype=np.float32)       # decreasing first half
    buf = ops.dist_buffer(Q, G, 'cuda')
    buf.copy_(torch.from_numpy(d))
    vals, idx = ops.topk(buf, k)
    ref = np.argsort(d, axis=1, kind='stable')[:, :k]
    np.testing.assert_array_equal(idx.cpu().numpy(), ref)
    np.testing.assert_array_equal(vals.cpu().numpy(), np.take_along_axis(d, ref, axis=1))


@pytest.mark.parametrize('case', ['market_small', 'full_dim'])
def test_sharded_evaluator_tiled_query_planes(golden, case):
    """The distance paths bench.py tunes inside the evaluator (h2 tiles;
    x3 with queries and gallery as chunk-tiled bf16x3 planes,
    pps_distmat_x3p_tiled): every tile of one arithmetic gives the same
    distance bits, all are within 1e-5 of the default path, and every run
    reproduces the mAP of the reference's own evaluation."""
    from pps_amd import distributed as pdist
    g = golden(case)
    if 'qid' not in g:
        pytest.skip('no ids in this fixture')
    qf, gf = _cuda(g['qf']), _cuda(g['gf'])
    ev_ = pdist.ShardedEvaluator(g['qid'], g['qcam'], g['gid'], g['gcam'], 0, 1)
    be = pdist.HipBackend
    saved = (be.distmat_math, be.distmat_tile, be.distmat_qplanes)
    outs = []
    runs = ((None, 0, False), ('x3', 52, True), ('x3', 47, True), ('h2', 1, False),
            ('h2', 5, False))
    try:
        for math, tile, qp in runs:
            be.distmat_math, be.distmat_tile, be.distmat_qplanes = math, tile, qp
            outs.append(ev_.run(qf, gf, keep_dist=True))
    finally:
        be.distmat_math, be.distmat_tile, be.distmat_qplanes = saved
    if g['qf'].shape[1] % 32 == 0:
        assert torch.equal(outs[1]['dist'], outs[2]['dist'])
        assert torch.equal(outs[3]['dist'], outs[4]['dist'])
        assert torch.equal(outs[0]['dist'], outs[3]['dist'])   # the default is h2
    for o in outs[1:]:
        np.testing.assert_allclose(o['dist'].cpu().numpy(), outs[0]['dist'].cpu().numpy(),
                                   rtol=0, atol=1e-5)
    for o in outs:
        assert abs(o['mAP'] - float(g['mAP'])) < 1e-6
        # CMC of every arithmetic (the default h2 included) vs the reference's
        # own evaluation (the golden cmc covers topk = 10 here too)
        np.testing.assert_allclose(o['cmc'], np.asarray(g['cmc'])[:len(o['cmc'])], rtol=0,
                                   atol=1e-9)
    # runs of one arithmetic on the same bits: identical scores
    for a, b in ((outs[1], outs[2]), (outs[3], outs[4]), (outs[0], outs[3])):
        if torch.equal(a['dist'], b['dist']):
            assert a['mAP'] == b['mAP']
            np.testing.assert_array_equal(a['cmc'], b['cmc'])


def test_rank_prepare_beyond_lds_merge_cap():
    """four gallery shards, one identity with 3000 entries
    in every shard -- R * Pmax = 12000 merged positives, past the LDS merge
    (8192): pps_rank_prepare sorts in global memory.  AP, validity and the
    first-match rank of every query equal the oracle's mean_ap / the stable
    argsort on the same float32 distances (reid_dataset_evaluator.py:366-439),
    sharded and unsharded alike."""
    from pps_amd import ops
    R, Gs, big, D = 4, 4000, 3000, 32
    rng = np.random.RandomState(11)
    gid = np.concatenate([np.concatenate([np.full(big, 7), rng.randint(100, 600, Gs - big)])
                          for _ in range(R)])
    gcam = rng.randint(1, 7, R * Gs)
    Q = 48
    qid = np.concatenate([np.full(12, 7), rng.randint(100, 600, Q - 12)])
    qcam = rng.randint(1, 7, Q)
    f = rng.randn(Q + R * Gs, D).astype(np.float32)
    d = ev.compute_dist(f[:Q], f[Q:])
    dd = _cuda(d)
    ref_ap, ref_valid = ev.mean_ap(d, qid, gid, qcam, gcam, average=False)
    ref_valid = np.asarray(ref_valid).astype(bool)
    for shards in (1, R):
        cuts = [r * (R * Gs) // shards for r in range(shards + 1)]
        lists, parts = [], []
        for a, b in zip(cuts[:-1], cuts[1:]):
            ds = dd[:, a:b].contiguous()
            idx = ops.MatchIndex(qid, qcam, gid[a:b], gcam[a:b])
            p = ops.collect_matches(ds, idx, a, big * R // shards + 16)
            lists.append(p[:3])
            parts.append((ds, a, p[3]))
        sp = ops.rank_prepare(torch.stack([l[0] for l in lists]),
                              torch.stack([l[1] for l in lists]),
                              torch.stack([l[2] for l in lists]))
        assert sp.sorted_d.shape[1] > 8192
        hist = before = None
        for ds, a, junk in parts:
            hist, before = ops.rank_count_stream(ds, a, sp, junk, hist, before)
        ap, valid, first = ops.ap_finalize(sp.sorted_d, sp.pos_total, hist, before)
        ap, valid, first = ap.cpu().numpy(), valid.cpu().numpy(), first.cpu().numpy()
        np.testing.assert_array_equal(valid.astype(bool), ref_valid)
        np.testing.assert_allclose(ap[ref_valid], np.asarray(ref_ap)[ref_valid], rtol=0, atol=1e-12)
        # first match: valid entries (not same id + same camera) before the
        # first true match in the stable (distance, index) order
        for q in range(Q):
            order = np.lexsort((np.arange(d.shape[1]), d[q]))
            junk = (gid[order] == qid[q]) & (gcam[order] == qcam[q])
            o = order[~junk]
            hit = np.nonzero(gid[o] == qid[q])[0]
            assert first[q] == (hit[0] if len(hit) else -1), q
        # the merged rows are the positives in (distance, index) order
        q = 0
        P = int(sp.pos_total[q])
        assert P > 8192
        sd = sp.sorted_d[q, :P].cpu().numpy()
        si = sp.sorted_idx[q, :P].cpu().numpy()
        pos = np.nonzero((gid == qid[q]) & (gcam != qcam[q]))[0]
        want = pos[np.lexsort((pos, d[q, pos]))]
        np.testing.assert_array_equal(si, want)
        np.testing.assert_array_equal(sd, d[q, want])


@pytest.mark.parametrize('Q,G,kind', [(3368, 15913, 'market'), (64, 17661, 'ties'),
                                      (37, 1, 'plain'), (5, 4099, 'degenerate'),
                                      (40, 18432, 'plain'), (300, 19889, 'market'),
                                      (24, 19889, 'ties'), (5, 30001, 'degenerate'),
                                      (12, 125000, 'market'), (6, 125000, 'ties'),
                                      (48, 15913, 'groups'), (12, 30001, 'groups')])
def test_argsort_rows_equals_stable_argsort(Q, G, kind):
    """pps_argsort_rows == np.argsort(kind='stable') on every row (VERDICT
    r03 item 8): Market-sized rows of L2 distances (the reference's full rank
    list, reid_dataset_evaluator.py:319,420), rows with heavy ties and
    negative zeros, all-equal and two-valued rows (one bucket: the wave
    bitonic path), the one-pass kernel's longest row (18,432), and longer
    rows through the segmented kernel: Duke-plus (19,889) and a 1M-config
    gallery shard (125,000).  'groups': every value repeated 5..16 times
    (row q: 5 + q % 12), so most buckets hold 5..16 words -- the per-wave
    lists of those buckets fill several times per step (over 32 new entries
    in one 64-bucket step, the case that once overran a list)."""
    from pps_amd import ops
    rng = np.random.RandomState(G + Q)
    if kind == 'market':
        d = np.sqrt(rng.chisquare(50, size=(Q, G)).astype(np.float32) / 25)
    elif kind == 'ties':
        d = (rng.randint(0, 300, (Q, G)) / 16).astype(np.float32)
        d[1] = -0.0
        d[2, ::3] = 0.0
        d[3] = np.float32(np.inf)
        d[3, 7] = 1.0
    elif kind == 'groups':
        d = np.stack([(rng.permutation(G) // (5 + q % 12)).astype(np.float32)
                      for q in range(Q)])
    elif kind == 'degenerate':
        d = np.ones((Q, G), np.float32)
        d[1, ::2] = 2.0
        d[2] = rng.rand(G).astype(np.float32) * 1e-30
        d[3] = np.float32(3.0) + np.arange(G, dtype=np.float32) * 1e-7
    else:
        d = rng.randn(Q, G).astype(np.float32)
    buf = ops.dist_buffer(Q, G, 'cuda')
    buf.copy_(torch.from_numpy(d))
    idx, vals = ops.argsort_rows(buf, with_values=True)
    want = np.argsort(d, axis=1, kind='stable')
    got = idx.cpu().numpy()
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(vals.cpu().numpy(), np.take_along_axis(d, want, 1))


def test_argsort_rows_capacity_error():
    """Rows past the segmented kernel's capacity (458,752 columns) are refused
    with a pointer to pps_topk."""
    from pps_amd import ops
    cap = ops._lib.lib().pps_argsort_rows_cap()
    assert cap >= 400000
    with pytest.raises(RuntimeError, match='pps_topk'):
        ops.argsort_rows(torch.zeros((1, cap + 1), device='cuda'))
