"""Gallery-sharded retrieval (pps_amd/distributed.py) with torch.distributed
gloo, world_size 2 and 3, on CPU: the sharded result must equal the
single-process reference evaluator (the golden-pinned oracle) exactly."""
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


def _worker(rank, world, port, data, out):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from oracle.rank_counts import CpuBackend
    from pps_amd import distributed as pdist
    qf, gf, qid, qcam, gid, gcam = data
    qa, qb = pdist.shard_range(len(qid), rank, world)
    ga, gb = pdist.shard_range(len(gid), rank, world)
    ev = pdist.ShardedEvaluator(qid, qcam, gid, gcam, rank, world, backend=CpuBackend)
    res = ev.run(torch.from_numpy(qf[qa:qb]), torch.from_numpy(gf[ga:gb]))
    out[rank] = (res['mAP'], res['cmc'].tolist(), res['ap'].tolist(),
                 res['first_rank'].tolist())
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_sharded_eval_matches_single_process(golden, world):
    from oracle import evaluator as ev
    g = golden('market_small')
    data = (g['qf'], g['gf'], g['qid'], g['qcam'], g['gid'], g['gcam'])
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), data, out), nprocs=world, join=True)
    ref_ap, ref_valid = ev.mean_ap(g['dist'], g['qid'], g['gid'], g['qcam'], g['gcam'],
                                   average=False)
    ret, _ = ev.cmc(g['dist'], g['qid'], g['gid'], g['qcam'], g['gcam'], topk=10,
                    first_match_break=True, average=False)
    for r in range(world):
        mAP, cmc, ap, first = out[r]
        np.testing.assert_allclose(ap, ref_ap, atol=1e-12)
        assert abs(mAP - float(g['mAP'])) < 1e-12
        np.testing.assert_allclose(cmc, g['cmc'], atol=1e-12)


def test_shard_range_is_array_split():
    from pps_amd.distributed import shard_range
    for n in (0, 1, 7, 15913):
        for w in (1, 2, 3, 8):
            parts = np.array_split(np.arange(n), w)
            assert [shard_range(n, r, w) for r in range(w)] == \
                [(int(p[0]) if len(p) else sum(len(x) for x in parts[:i]),
                  (int(p[-1]) + 1) if len(p) else sum(len(x) for x in parts[:i]))
                 for i, p in enumerate(parts)]
