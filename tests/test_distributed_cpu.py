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
