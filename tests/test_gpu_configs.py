"""The other BASELINE.json configs on the HIP path, each checked against the
oracle:

* DukeMTMC-reID (configs[2]): k-reciprocal re-ranking
  (reid_dataset_evaluator.py:442-519) vs the oracle at Q=500, G=3000 on the
  same input distances, then near-tie-aware mAP/CMC parity on the re-ranked
  matrices; and the full 2228 x 17661 cosine + re-ranking run checked by
  properties: finite, lambda=1 reduces to the normalised original distance
  (:452-454, :518), lambda=0 is a Jaccard distance in [0, 1], and the GPU
  ranking of the re-ranked matrix equals the oracle's on the same matrix.
* CUHK03-detected (configs[3], 4 GPUs gallery-sharded): the 1400 x 5332
  gallery cut into 4 shards in one process; per-shard positive lists, counts
  summed as the all-reduce does, rank lists merged (pps_topk_merge) --
  identical to the one-shard results and near-tie-exact vs the oracle.
* Synthetic 1M x 10k (configs[4], 8 GPUs): one GPU's share (10k x 125k,
  D=2048) with the stable top-100 checked against NumPy on 64 sampled query
  rows; and the 8-shard k-way merge at 512 queries x 1M gallery equal to the
  top-100 of the whole matrix.
"""
import numpy as np
import pytest
import torch
from _parity import check_rank_metrics, check_topk, tie_eps

from oracle import evaluator as ev

ev_compute_dist = ev.compute_dist
from oracle.rank_counts import merge_topk

pytestmark = pytest.mark.gpu

DIST_TILE = 0    # the default h2 tile (every h2 tile gives the same bits)


def _feats(n_ids, ids, D, gen, noise=4.0):
    cent = torch.randn((n_ids + 1, D), generator=gen, device='cuda')
    x = cent[torch.from_numpy(np.asarray(ids)).cuda()] + \
        noise * torch.randn((len(ids), D), generator=gen, device='cuda')
    return (x / x.norm(dim=1, keepdim=True)).contiguous()


# ---------------------------------------------------------------- top-k merge
@pytest.mark.parametrize('R,kin,kout', [(1, 5, 5), (4, 100, 100), (8, 100, 100),
                                        (3, 7, 20), (8, 1024, 1024), (64, 16, 10)])
def test_topk_merge_kernel(R, kin, kout):
    from pps_amd import ops
    rng = np.random.RandomState(R * 1000 + kin)
    Q = 37
    vals = np.sort(rng.randint(0, 50, (R, Q, kin)).astype(np.float32) / 8, axis=2)
    idx = np.zeros((R, Q, kin), np.int32)
    for r in range(R):
        for q in range(Q):   # ascending indices inside equal values: a stable list
            idx[r, q] = np.sort(rng.choice(5000, kin, replace=False))
            idx[r, q] = idx[r, q][np.lexsort((idx[r, q], vals[r, q]))]
    if R > 1:
        idx[1, :3, kin // 2:] = -1    # short shard: pads
        vals[1, :3, kin // 2:] = np.inf
    offs = np.arange(R) * 5000
    v, i = ops.topk_merge(torch.from_numpy(vals).cuda(), torch.from_numpy(idx).cuda(),
                          offs, kout)
    rv, ri = merge_topk(vals, idx, offs, kout)
    np.testing.assert_array_equal(i.cpu().numpy(), ri)
    np.testing.assert_array_equal(v.cpu().numpy(), rv)


def test_topk_merge_enforces_limits():
    from pps_amd import ops
    z = torch.zeros((2, 3, 8192), device='cuda')
    with pytest.raises(RuntimeError, match='8192'):
        ops.topk_merge(z, z.to(torch.int32), [0, 1], 5)
    with pytest.raises(RuntimeError, match='one offset per list'):
        ops.topk_merge(z[:, :, :4], z[:, :, :4].to(torch.int32), [0], 5)


# ---------------------------------------------------------------- CUHK03
def test_cuhk03_four_shards_in_process():
    """BASELINE configs[3]: 1400 queries x 5332 gallery, 4 gallery shards as
    the 4 ranks hold them, through the product sharded kernels exactly as
    ShardedEvaluator.run drives them (pps_amd/distributed.py:253-276):
    per rank collect_matches on its shard, the lists "all-gathered"
    (stacked), rank_prepare + rank_count_stream per rank, hist / before
    summed as the all-reduce does, ap_finalize.  Equal to the one-shard
    rank_eval and near-tie-exact vs the oracle; the merged top-100 rank list
    equals the whole matrix's."""
    from pps_amd import ops
    from pps_amd import reid_dataset_evaluator as gev
    from pps_amd.distributed import HipBackend, ShardedEvaluator
    Q, G, D, R = 1400, 5332, 3968, 4
    rng = np.random.RandomState(3)
    qid = rng.randint(1, 701, Q)
    gid = rng.randint(1, 701, G)
    qcam = rng.randint(1, 3, Q)
    gcam = rng.randint(1, 3, G)
    gen = torch.Generator(device='cuda')
    gen.manual_seed(3)
    f = _feats(700, np.concatenate([qid, gid]), D, gen)
    qf, gf = f[:Q].contiguous(), f[Q:].contiguous()
    full = ops.compute_dist(qf, gf, tile=DIST_TILE)
    evs = [ShardedEvaluator(qid, qcam, gid, gcam, r, R) for r in range(R)]
    be = HipBackend
    blocks, lists, junks, states = [], [], [], []
    for ev in evs:   # each rank: its shard's distances and lists
        a, b = ev.g_ranges[ev.rank]
        blk = be.distmat(qf, gf[a:b].contiguous(), ev.metric)
        assert torch.equal(blk, full[:, a:b])   # a shard block = that slice of the matrix
        st = be.prepare(ev)
        pd, pi, pc, junk = be.collect(blk, ev, st, ev.pmax)
        blocks.append(blk)
        lists.append((pd, pi, pc))
        junks.append(junk)
        states.append(st)
    # the all-gather of the lists (ShardedEvaluator._gather_lists)
    pos_d = torch.stack([l[0] for l in lists])
    pos_i = torch.stack([l[1] for l in lists])
    pos_c = torch.stack([l[2] for l in lists])
    hist = before = None
    for ev, blk, st, junk in zip(evs, blocks, states, junks):
        sd, _, ptot, h, bf = be.counts(blk, ev, st, pos_d, pos_i, pos_c, junk)
        hist = h if hist is None else hist + h      # the all-reduce(SUM)
        before = bf if before is None else before + bf
    ap, valid, first = be.finalize(sd, ptot, hist, before)
    ap1, valid1, first1 = gev.rank_eval(full, qid, gid, qcam, gcam)
    np.testing.assert_array_equal(valid.cpu().numpy(), valid1.cpu().numpy())
    np.testing.assert_array_equal(first.cpu().numpy(), first1.cpu().numpy())
    np.testing.assert_allclose(ap.cpu().numpy(), ap1.cpu().numpy(), rtol=0, atol=1e-12)
    # merged rank list == top-k of the whole matrix
    ranges = [ev.g_ranges[ev.rank] for ev in evs]
    tops = [ops.topk(blk, 100) for blk in blocks]
    mv, mi = ops.topk_merge(torch.stack([t[0] for t in tops]),
                            torch.stack([t[1] for t in tops]), [a for a, _ in ranges], 100)
    fv, fi = ops.topk(full, 100)
    assert torch.equal(mi, fi) and torch.equal(mv, fv)
    # vs the oracle (NumPy distances, stable argsort, mean_ap / cmc)
    qn, gn = qf.cpu().numpy(), gf.cpu().numpy()
    ref = ev_compute_dist(qn, gn)
    dn = full.cpu().numpy()
    eps = tie_eps(dn, ref)
    flips = check_topk(mi.cpu().numpy(), ref, 100, eps)
    r = check_rank_metrics(ap.cpu().numpy(), valid.cpu().numpy(), first.cpu().numpy(), ref,
                           qid, gid, qcam, gcam, eps)
    print('CUHK03 4 shards: top-100 flips %d, %s' % (flips, r))


# ---------------------------------------------------------------- 1M x 10k
def test_synthetic_1m_shard_top100_sampled():
    """BASELINE configs[4], one GPU's share: 10k queries x 125k gallery
    shard, D=2048, L2 on normalised Gaussian features (seed 0)."""
    from pps_amd import ops
    Q, G, D, k = 10000, 125000, 2048, 100
    gen = torch.Generator(device='cuda')
    gen.manual_seed(0)
    q = torch.randn(Q, D, generator=gen, device='cuda')
    q /= q.norm(dim=1, keepdim=True)
    g = torch.randn(G, D, generator=gen, device='cuda')
    g /= g.norm(dim=1, keepdim=True)
    d = ops.compute_dist(q, ops.GalleryIndex(g))
    vals, idx = ops.topk(d, k)
    rows = np.random.RandomState(1).choice(Q, 64, replace=False)
    rows_t = torch.from_numpy(rows).cuda()
    ref = ev.compute_dist(q[rows_t].cpu().numpy(), g.cpu().numpy())
    dsub = d[rows_t].cpu().numpy()
    assert np.abs(dsub - ref).max() < 1e-4
    eps = tie_eps(dsub, ref)
    flips = check_topk(idx[rows_t].cpu().numpy(), ref, k, eps)
    np.testing.assert_array_equal(vals[rows_t].cpu().numpy(),
                                  np.take_along_axis(dsub, idx[rows_t].cpu().numpy()
                                                     .astype(np.int64), axis=1))
    print('1M shard: %d of %d sampled top-%d positions differ (near-ties, eps %.3g)'
          % (flips, 64 * k, k, eps))


def test_synthetic_1m_eight_shard_merge():
    """The 8-GPU global rank list at 512 queries x 1M gallery: per-shard
    top-100 of each 125k block, merged == top-100 of the whole matrix."""
    from pps_amd import ops
    from pps_amd.distributed import shard_range
    Q, G, D, R, k = 512, 1000000, 2048, 8, 100
    gen = torch.Generator(device='cuda')
    gen.manual_seed(5)
    q = torch.randn(Q, D, generator=gen, device='cuda')
    q /= q.norm(dim=1, keepdim=True)
    full = torch.empty((Q, G), device='cuda')
    tv, ti, offs = [], [], []
    for r in range(R):
        a, b = shard_range(G, r, R)
        g = torch.randn(b - a, D, generator=gen, device='cuda')
        g /= g.norm(dim=1, keepdim=True)
        blk = full[:, a:b]                    # row-strided view: ldo = G
        ops.compute_dist(q, ops.GalleryIndex(g), out=blk, tile=DIST_TILE)
        v, i = ops.topk(blk, k)
        tv.append(v)
        ti.append(i)
        offs.append(a)
        del g
    mv, mi = ops.topk_merge(torch.stack(tv), torch.stack(ti), offs, k)
    fv, fi = ops.topk(full, k)
    assert torch.equal(mi, fi) and torch.equal(mv, fv)


# ---------------------------------------------------------------- Duke
def test_duke_rerank_vs_oracle_500x3000():
    from pps_amd import ops
    from pps_amd import reid_dataset_evaluator as gev
    Q, G, D = 500, 3000, 256
    rng = np.random.RandomState(2)
    qid = rng.randint(1, 200, Q)
    gid = rng.randint(1, 200, G)
    qcam = rng.randint(1, 9, Q)
    gcam = rng.randint(1, 9, G)
    cent = rng.randn(200, D).astype(np.float32)
    f = cent[np.concatenate([qid, gid])] + 2.5 * rng.randn(Q + G, D).astype(np.float32)
    f = (f / np.linalg.norm(f, axis=1, keepdims=True)).astype(np.float32)
    qg = ev.compute_dist(f[:Q], f[Q:])
    qq = ev.compute_dist(f[:Q], f[:Q])
    gg = ev.compute_dist(f[Q:], f[Q:])
    ref = ev.re_ranking(qg, qq, gg, k1=20, k2=6, lambda_value=0.3)
    rr = ops.re_ranking(*(torch.from_numpy(np.ascontiguousarray(x)).cuda()
                          for x in (qg, qq, gg)), 20, 6, 0.3)
    rrn = rr.cpu().numpy()
    err = np.abs(rrn - ref).max()
    assert err < 1e-5, err
    ap, valid, first = gev.rank_eval(rr, qid, gid, qcam, gcam)
    r = check_rank_metrics(ap.cpu().numpy(), valid.cpu().numpy(), first.cpu().numpy(), ref,
                           qid, gid, qcam, gcam, tie_eps(rrn, ref))
    print("Duke 500x3000 re-ranking: max|err| %.3g, %s" % (err, r))
    assert 0.3 < r["mAP"] < 0.8   # non-trivial regime (plain mAP ~0.28, re-ranked ~0.50)


def test_rerank_long_rows_vs_oracle():
    """Q + G = 16500 >= 16384: the OD rows are long enough for the wave-
    streaming top-k (topk_wave_kernel) inside pps_re_ranking (VERDICT r03
    item 5).  Same float32 distances into both; the checker is the oracle's
    sparse restatement (pinned equal to oracle.re_ranking,
    tests/test_oracle_golden.py)."""
    from pps_amd import ops
    from pps_amd import reid_dataset_evaluator as gev
    Q, G, D = 1000, 15500, 256
    rng = np.random.RandomState(7)
    qid = rng.randint(1, 700, Q)
    gid = rng.randint(1, 700, G)
    qcam = rng.randint(1, 9, Q)
    gcam = rng.randint(1, 9, G)
    cent = rng.randn(700, D).astype(np.float32)
    f = cent[np.concatenate([qid, gid])] + 2.5 * rng.randn(Q + G, D).astype(np.float32)
    f = (f / np.linalg.norm(f, axis=1, keepdims=True)).astype(np.float32)
    qg = ev.compute_dist(f[:Q], f[Q:])
    # exactly symmetric self-distances (upper triangle mirrored, as the GPU's
    # self-distance GEMM returns them), so the in-place path runs: N >= 16384,
    # 16-byte rows (Q, G % 4 == 0), PPS_RERANK_SYMMETRIC
    sym = lambda d: np.triu(d) + np.triu(d, 1).T
    qq = sym(ev.compute_dist(f[:Q], f[:Q]))
    gg = sym(ev.compute_dist(f[Q:], f[Q:]))
    ref = ev.re_ranking_sparse(qg, qq, gg, k1=20, k2=6, lambda_value=0.3)
    dev = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (qg, qq, gg)]
    rr = ops.re_ranking(*dev, k1=20, k2=6, lambda_value=0.3, symmetric=True)
    dense = ops.re_ranking(*dev, k1=20, k2=6, lambda_value=0.3, symmetric=False)
    assert torch.equal(rr, dense)   # in place == the dense N x N path, bit for bit
    rrn = rr.cpu().numpy()
    err = float(np.abs(rrn - ref).max())
    ap, valid, first = gev.rank_eval(rr, qid, gid, qcam, gcam)
    r = check_rank_metrics(ap.cpu().numpy(), valid.cpu().numpy(), first.cpu().numpy(), ref,
                           qid, gid, qcam, gcam, tie_eps(rrn, ref))
    print('re-ranking 1000 x 15500 (long rows): max|err| %.3g, %s' % (err, r))
    assert err < 1e-5, err


def test_rerank_inplace_equals_dense_duke_shape():
    """Duke shape (2228 + 17661, odd G): the padded blocks from
    compute_dist(pad_rows=True) take the in-place path (no N x N buffer); the
    same blocks copied dense take the dense OD path -- identical bits, also
    against the non-symmetric (transposing) OD path."""
    from pps_amd import ops
    Q, G, D = 2228, 17661, 256
    gen = torch.Generator(device='cuda')
    gen.manual_seed(3)
    rng = np.random.RandomState(3)
    x = _feats(300, rng.randint(1, 301, Q + G), D, gen, noise=2.5)
    qf, gf = x[:Q].contiguous(), x[Q:].contiguous()
    q_g = ops.compute_dist(qf, gf, metric='cosine', pad_rows=True)
    q_q = ops.compute_dist(qf, qf, metric='cosine', pad_rows=True)
    g_g = ops.compute_dist(gf, gf, metric='cosine', pad_rows=True)
    assert q_g.stride(0) % 4 == 0 and g_g.stride(0) % 4 == 0
    a = ops.re_ranking(q_g, q_q, g_g, 20, 6, 0.3)
    b = ops.re_ranking(q_g.contiguous(), q_q.contiguous(), g_g.contiguous(), 20, 6, 0.3,
                       symmetric=True)
    c = ops.re_ranking(q_g.contiguous(), q_q.contiguous(), g_g.contiguous(), 20, 6, 0.3,
                       symmetric=False)
    assert torch.equal(a, b) and torch.equal(a, c)


def test_rerank_inplace_tied_rows_take_exact_pass():
    """Gallery features repeated 24 times: every row's k1+1 = 21st and
    (k1+9)-th neighbours lie in one run of equal distances, so the in-place
    top-k on m * m cannot settle the (OD, index) order from its k+8 list and
    hands the rows to the exact OD pass -- same bits as the dense path."""
    from pps_amd import ops
    Q, reps, U, D = 1000, 24, 700, 64
    gen = torch.Generator(device='cuda')
    gen.manual_seed(5)
    rng = np.random.RandomState(5)
    base = _feats(200, rng.randint(1, 201, Q + U), D, gen, noise=2.5)
    qf = base[:Q].contiguous()
    gf = base[Q:].repeat_interleave(reps, dim=0).contiguous()   # G = 16800
    q_g = ops.compute_dist(qf, gf, metric='cosine', pad_rows=True)
    q_q = ops.compute_dist(qf, qf, metric='cosine', pad_rows=True)
    g_g = ops.compute_dist(gf, gf, metric='cosine', pad_rows=True)
    a = ops.re_ranking(q_g, q_q, g_g, 20, 6, 0.3)
    c = ops.re_ranking(q_g.contiguous(), q_q.contiguous(), g_g.contiguous(), 20, 6, 0.3,
                       symmetric=False)
    assert torch.equal(a, c)


def test_duke_full_size_cosine_rerank_properties():
    from pps_amd import ops
    from pps_amd import reid_dataset_evaluator as gev
    Q, G, D = 2228, 17661, 3968
    rng = np.random.RandomState(0)
    qid = rng.randint(1, 703, Q)
    gid = rng.randint(1, 703, G)
    qcam = rng.randint(1, 9, Q)
    gcam = rng.randint(1, 9, G)
    gen = torch.Generator(device='cuda')
    gen.manual_seed(0)
    x = _feats(702, np.concatenate([qid, gid]), D, gen)
    qf, gf = x[:Q].contiguous(), x[Q:].contiguous()
    q_g = ops.compute_dist(qf, gf, metric='cosine')
    q_q = ops.compute_dist(qf, qf, metric='cosine')
    g_g = ops.compute_dist(gf, gf, metric='cosine')
    assert torch.equal(g_g, g_g.t())                  # symmetric self-distance
    rr = ops.re_ranking(q_g, q_q, g_g, 20, 6, 0.3)
    assert tuple(rr.shape) == (Q, G) and bool(torch.isfinite(rr).all())
    # lambda = 1: the normalised original distance, od[i][j] = M[i][j]^2 /
    # max_r M[r][i]^2 with M symmetric (:452-454, :518)
    r1 = ops.re_ranking(q_g, q_q, g_g, 20, 6, 1.0)
    colmax = torch.maximum((q_q * q_q).max(dim=1).values, (q_g * q_g).max(dim=1).values)
    od = (q_g * q_g) / colmax[:, None]
    torch.testing.assert_close(r1, od, rtol=2e-6, atol=0)
    # lambda = 0: Jaccard distance 1 - t / (2 - t) with t in [0, 1]
    r0 = ops.re_ranking(q_g, q_q, g_g, 20, 6, 0.0)
    assert float(r0.min()) >= 0.0 and float(r0.max()) <= 1.0 + 1e-6
    # rr = 0.7 * r0 + 0.3 * r1 (the reference's final combination, :518)
    torch.testing.assert_close(rr, r0 * 0.7 + r1 * 0.3, rtol=0, atol=2e-6)
    # the GPU ranking of the re-ranked matrix == the oracle's on the same matrix
    rrn = rr.cpu().numpy()
    ap, valid, first = gev.rank_eval(rr, qid, gid, qcam, gcam)
    r = check_rank_metrics(ap.cpu().numpy(), valid.cpu().numpy(), first.cpu().numpy(), rrn,
                           qid, gid, qcam, gcam, 0.0)
    assert r['ap_differs'] == 0 and r['first_differs'] == 0, r
    print('Duke full size: re-ranked %s' % r)


@pytest.mark.parametrize('Q', [1000, 1001])
def test_rerank_whole_matrix_blocks(Q):
    """re-ranking inputs as the blocks of ONE mirrored self-distance of
    [queries; gallery] (ops.self_distance_blocks, PPS_RERANK_WHOLE: q_g^T read
    from the matrix's lower-left block, no transpose): the blocks equal the
    three separate compute_dist calls bit for bit, and so does the re-ranked
    result (Q = 1000: in place, N >= 16384, with a workspace that holds no
    N x N region; Q = 1001: q_g's rows are not 16-byte aligned, the dense
    path runs on the dense workspace); the flag is refused on separate
    buffers, and the ranking of the (possibly misaligned) q_g view equals
    that of its contiguous copy."""
    from pps_amd import _lib, ops
    from pps_amd import reid_dataset_evaluator as gev
    G, D = 15500, 64
    gen = torch.Generator(device='cuda')
    gen.manual_seed(11)
    rng = np.random.RandomState(11)
    x = _feats(300, rng.randint(1, 301, Q + G), D, gen, noise=2.5)
    qf, gf = x[:Q], x[Q:]
    M, q_g, q_q, g_g = ops.self_distance_blocks(x, Q, metric='cosine')
    assert torch.equal(M[Q:, :Q], M[:Q, Q:].t())   # the mirror: q_g^T in place
    sq_g = ops.compute_dist(qf, gf, metric='cosine', pad_rows=True)
    sq_q = ops.compute_dist(qf.contiguous(), qf.contiguous(), metric='cosine', pad_rows=True)
    sg_g = ops.compute_dist(gf.contiguous(), gf.contiguous(), metric='cosine', pad_rows=True)
    assert torch.equal(q_g, sq_g) and torch.equal(q_q, sq_q) and torch.equal(g_g, sg_g)
    a = ops.re_ranking(q_g, q_q, g_g, 20, 6, 0.3, symmetric=True, whole=True)
    b = ops.re_ranking(sq_g, sq_q, sg_g, 20, 6, 0.3)
    assert torch.equal(a, b)
    with pytest.raises(RuntimeError, match='PPS_RERANK_WHOLE'):
        ops.re_ranking(sq_g, sq_q, sg_g, 20, 6, 0.3, symmetric=True, whole=True)
    L = _lib.lib()
    dense = L.pps_rerank_workspace_bytes(Q, G, 20, 6)
    need = L.pps_rerank_workspace_bytes_ld(q_g.data_ptr(), M.stride(0), q_q.data_ptr(),
                                           M.stride(0), g_g.data_ptr(), M.stride(0), Q, G, 20,
                                           6, ops.RERANK_SYMMETRIC | ops.RERANK_WHOLE)
    N = Q + G
    if Q % 4 == 0:
        assert need < dense - 4 * N * N + 4 * N * 64, (need, dense)   # no N x N region
    else:
        assert need == dense
    rng2 = np.random.RandomState(12)
    qid, gid = rng2.randint(0, 300, Q), rng2.randint(0, 300, G)
    qcam, gcam = rng2.randint(0, 6, Q), rng2.randint(0, 6, G)
    r1 = gev.rank_eval(q_g, qid, gid, qcam, gcam)
    r2 = gev.rank_eval(q_g.contiguous(), qid, gid, qcam, gcam)
    for u, v in zip(r1, r2):
        assert torch.equal(u, v)
