"""The multi-GPU retrieval path over RCCL (torch.distributed 'nccl') with
device tensors: a one-rank communicator on this box's GPU runs every
collective of distributed.py (all-gather of queries and positive lists,
SUM all-reduce of the counts, the rank-list gather, the rerank broadcast,
barrier and max-over-ranks) on HIP buffers, and must give the same results
as the same code with no process group (the N>1 RCCL run is
the driver's 8-GPU bench)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(seed=4, n=3000, d=256, n_ids=150):
    rng = np.random.RandomState(seed)
    ids = rng.randint(1, n_ids + 1, n)
    cams = rng.randint(1, 7, n)
    marks = rng.choice([0, 1, 1, 1, 1, 2], n)
    cent = rng.randn(n_ids + 1, d).astype(np.float32)
    feat = (cent[ids] + 3.0 * rng.randn(n, d)).astype(np.float32)
    feat /= np.linalg.norm(feat, axis=1, keepdims=True)
    return feat, ids, cams, marks


def _run(feat, ids, cams, marks, rank, world):
    from pps_amd import distributed as pdist
    parts = []
    for m in (0, 1, 2):
        rows = np.nonzero(marks == m)[0]
        a, b = pdist.shard_range(len(rows), rank, world)
        parts.append(torch.from_numpy(feat[rows[a:b]]).cuda())
    sc = pdist.evaluate_sharded(parts[0], parts[1], parts[2], ids, cams, marks, rank, world,
                                rerank=True)
    q, g = marks == 0, marks == 1
    ev = pdist.ShardedEvaluator(ids[q], cams[q], ids[g], cams[g], rank, world)
    res = ev.run(parts[0], parts[1])
    vals, idx = ev.rank_list(parts[0], parts[1], k=100)
    t = pdist.max_over_ranks(1.5 + rank, world)
    pdist.barrier(world)
    return (sc[0], list(sc[1]), sc[2], list(sc[3]), res['ap'].tolist(),
            res['first_rank'].tolist(), idx.cpu().numpy(), vals.cpu().numpy(), t)


def _worker(rank, world, port, data, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK='0')
    torch.cuda.set_device(0)
    torch.distributed.init_process_group('nccl', device_id=torch.device('cuda', 0))
    assert torch.distributed.get_backend() == 'nccl'
    out[rank] = _run(*data, rank=rank, world=world)
    torch.distributed.destroy_process_group()


def test_rccl_one_rank_group_matches_no_group():
    data = _data()
    ref = _run(*data, rank=0, world=1)      # no process group: collectives skipped
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(1, _free_port(), data, out), nprocs=1, join=True)
    got = out[0]
    for a, b in zip(got[:6], ref[:6]):
        np.testing.assert_array_equal(np.asarray(a), np.asarray(b))
    np.testing.assert_array_equal(got[6], ref[6])
    np.testing.assert_array_equal(got[7], ref[7])
    assert got[8] == 1.5
    assert 0.05 < ref[0] < 0.999 and 0.05 < ref[2] < 0.999, (ref[0], ref[2])
