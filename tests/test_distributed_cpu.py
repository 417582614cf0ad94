"""Gallery-sharded retrieval (pps_amd/distributed.py) with torch.distributed
gloo, world_size 2 and 3, on CPU: the sharded results must equal the
single-process reference evaluator (the golden-pinned oracle) exactly --
single-query mAP/CMC, the merged global rank list, multi-query pooling and
re-ranking (reid_dataset_evaluator.py:29-209)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)


def _worker(rank, world, port, data, k, out):
    _init(rank, world, port)
    from oracle.rank_counts import CpuBackend
    from pps_amd import distributed as pdist
    qf, gf, qid, qcam, gid, gcam = data
    qa, qb = pdist.shard_range(len(qid), rank, world)
    ga, gb = pdist.shard_range(len(gid), rank, world)
    ev = pdist.ShardedEvaluator(qid, qcam, gid, gcam, rank, world, backend=CpuBackend)
    res = ev.run(torch.from_numpy(qf[qa:qb]), torch.from_numpy(gf[ga:gb]))
    vals, idx = ev.rank_list(torch.from_numpy(qf[qa:qb]), torch.from_numpy(gf[ga:gb]), k=k)
    out[rank] = (res['mAP'], res['cmc'].tolist(), res['ap'].tolist(),
                 res['first_rank'].tolist(), idx.numpy().tolist(), vals.numpy().tolist(),
                 ev.pmax)
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [1, 2, 3])
def test_sharded_eval_matches_single_process(golden, world):
    from oracle import evaluator as ev
    g = golden('market_small')
    data = (g['qf'], g['gf'], g['qid'], g['qcam'], g['gid'], g['gcam'])
    k = 50
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), data, k, out), nprocs=world, join=True)
    ref_ap, ref_valid = ev.mean_ap(g['dist'], g['qid'], g['gid'], g['qcam'], g['gcam'],
                                   average=False)
    order = g['order_stable'][:, :k]
    for r in range(world):
        mAP, cmc, ap, first, idx, vals, pmax = out[r]
        np.testing.assert_allclose(ap, ref_ap, atol=1e-12)
        assert abs(mAP - float(g['mAP'])) < 1e-12
        np.testing.assert_allclose(cmc, g['cmc'], atol=1e-12)
        # merged global rank list == stable argsort of the full matrix
        np.testing.assert_array_equal(np.array(idx), order)
        np.testing.assert_array_equal(np.array(vals, np.float32),
                                      np.take_along_axis(g['dist'], order, axis=1))


def _eval_worker(rank, world, port, data, rerank, out):
    _init(rank, world, port)
    from oracle.rank_counts import CpuBackend
    from pps_amd import distributed as pdist
    feat, ids, cams, marks = data
    parts = []
    for m in (0, 1, 2):
        rows = np.nonzero(marks == m)[0]
        a, b = pdist.shard_range(len(rows), rank, world)
        parts.append(torch.from_numpy(feat[rows[a:b]]))
    res = pdist.evaluate_sharded(parts[0], parts[1], parts[2], ids, cams, marks, rank, world,
                                 backend=CpuBackend, rerank=rerank)
    out[rank] = (res[0], list(res[1]), res[2], list(res[3]))
    dist.destroy_process_group()


@pytest.mark.parametrize('rerank,world', [(False, 2), (True, 2), (True, 1)])
def test_sharded_evaluate_multi_query_and_rerank(rerank, world):
    """evaluate() with marks 0/1/2 over 2 ranks == the oracle's one-process
    evaluate_arrays (single query, multi-query pooling, re-ranking of both).
    World size 1 runs every collective on a one-rank group."""
    from oracle import evaluator as ev
    rng = np.random.RandomState(9)
    n = 240
    ids = rng.randint(1, 16, n)
    cams = rng.randint(1, 4, n)
    marks = rng.choice([0, 1, 1, 2], n)
    cent = rng.randn(16, 64).astype(np.float32)
    feat = (cent[ids] + 0.8 * rng.randn(n, 64)).astype(np.float32)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_eval_worker, args=(world, _free_port(), (feat, ids, cams, marks), rerank, out),
             nprocs=world, join=True)
    ref = ev.evaluate_arrays(feat, ids, cams, marks, rerank=rerank)
    for r in range(world):
        mAP, cmc, mq_mAP, mq_cmc = out[r]
        assert abs(mAP - ref[0]) < 1e-12, (mAP, ref[0])
        np.testing.assert_allclose(cmc, ref[1], atol=1e-12)
        assert abs(mq_mAP - ref[2]) < 1e-12, (mq_mAP, ref[2])
        np.testing.assert_allclose(mq_cmc, ref[3], atol=1e-12)


def test_merge_topk_semantics():
    """oracle merge: pads dropped, (distance, global index) order, short
    output padded with (+inf, -1)."""
    from oracle.rank_counts import merge_topk
    vals = np.array([[[0.1, 0.5, np.inf]], [[0.1, 0.2, 0.3]]], np.float32)
    idx = np.array([[[4, 0, -1]], [[1, 2, 0]]], np.int32)
    v, i = merge_topk(vals, idx, [0, 10], 7)
    np.testing.assert_array_equal(i[0], [4, 11, 12, 10, 0, -1, -1])
    np.testing.assert_array_equal(v[0], np.array([0.1, 0.1, 0.2, 0.3, 0.5, np.inf, np.inf],
                                                 np.float32))


def test_shard_range_is_array_split():
    from pps_amd.distributed import shard_range
    for n in (0, 1, 7, 15913):
        for w in (1, 2, 3, 8):
            parts = np.array_split(np.arange(n), w)
            assert [shard_range(n, r, w) for r in range(w)] == \
                [(int(p[0]) if len(p) else sum(len(x) for x in parts[:i]),
                  (int(p[-1]) + 1) if len(p) else sum(len(x) for x in parts[:i]))
                 for i, p in enumerate(parts)]


_LEG_CUHK = dict(nq=60, ng=300, n_distractors=0, n_ids=20, dim=64)
_LEG_1M = dict(nq=24, ng=500, dim=32, k=10)


def _legs_worker(rank, world, port, out):
    if world > 1:
        _init(rank, world, port)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from oracle.rank_counts import CpuBackend
    c = bench.config_cuhk03(rank, world, reps=1, backend=CpuBackend, device='cpu',
                            sizes=_LEG_CUHK)
    m = bench.config_1m(rank, world, reps=1, backend=CpuBackend, device='cpu', sizes=_LEG_1M,
                        keep=True)
    mv, mi = m.pop('merged')
    out[rank] = (c['mAP_synthetic'], c['cmc'], c['G_local_rank0'], mv.numpy().tolist(),
                 mi.numpy().tolist(), m['G_local_rank0'], sorted(c), sorted(m))
    if world > 1:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [1, 2])
def test_bench_sharded_legs_rehearsal(world):
    """bench.py's config_cuhk03 / config_1m legs (BASELINE configs[3] and
    [4], run by the driver's N > 1 benches) driven through their collective
    code on CPU with gloo and the oracle backend, at reduced sizes: the
    sharded mAP / CMC equal the one-process oracle evaluation of the same
    features, and the merged top-k of the 1M leg equals the stable argsort of
    the unsharded matrix."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from oracle import evaluator as ev
    mgr = mp.Manager()
    out = mgr.dict()
    if world > 1:
        mp.spawn(_legs_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    else:
        _legs_worker(0, 1, None, out)
    s = _LEG_CUHK
    qid, gid, qcam, gcam, f = bench.retrieval_inputs(s['nq'], s['ng'], s['n_distractors'],
                                                     s['n_ids'], s['dim'], 'cpu')
    f = f.numpy()
    d = ev.compute_dist(f[:s['nq']], f[s['nq']:])
    ref_map = ev.mean_ap(d, qid, gid, qcam, gcam)
    ref_cmc = ev.cmc(d, qid, gid, qcam, gcam, topk=10, first_match_break=True)
    t = _LEG_1M
    q = bench.synth_rows(0, t['nq'], t['dim'], 1, 'cpu').numpy()
    g = bench.synth_rows(0, t['ng'], t['dim'], 2, 'cpu').numpy()
    full = ev.compute_dist(q, g)
    order = np.argsort(full, axis=1, kind='stable')[:, :t['k']]
    for r in range(world):
        mAP, cmc, gl, mv, mi, gl1, ckeys, mkeys = out[r]
        assert gl == s['ng'] // world + (1 if r < s['ng'] % world else 0)   # this rank's shard
        assert gl1 == t['ng'] // world + (1 if r < t['ng'] % world else 0)
        assert abs(mAP - ref_map) < 1e-9, (mAP, ref_map)
        np.testing.assert_allclose(cmc, ref_cmc, atol=1e-12)
        np.testing.assert_array_equal(np.array(mi), order)
        np.testing.assert_allclose(np.array(mv, np.float32), np.take_along_axis(full, order, 1),
                                   rtol=0, atol=1e-6)
        assert {'distmat_ms', 'query_allgather_ms', 'retrieval_ms', 'mAP_synthetic'} <= set(ckeys)
        assert {'distmat_ms', 'topk_ms', 'list_allgather_merge_ms', 'total_ms'} <= set(mkeys)


def test_synth_rows_do_not_depend_on_sharding():
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from pps_amd.distributed import shard_range
    full = bench.synth_rows(0, 1000, 16, 7, 'cpu', chunk=96)
    for w in (1, 3, 8):
        parts = [bench.synth_rows(*shard_range(1000, r, w), 16, 7, 'cpu', chunk=96)
                 for r in range(w)]
        assert torch.equal(torch.cat(parts), full)
