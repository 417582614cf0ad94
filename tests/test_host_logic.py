"""Host-side logic of the retrieval path (no GPU): the per-identity gallery
index the match collection reads, the exact list capacity of the sharded
evaluator, multi-query grouping (reid_dataset_evaluator.py:136-143)."""
import os

import numpy as np

from pps_amd import distributed as pdist
from pps_amd import ops


def test_match_index_lists_every_same_id_entry_in_index_order():
    rng = np.random.RandomState(0)
    gid = rng.randint(0, 40, 500)
    gcam = rng.randint(1, 7, 500)
    qid = np.concatenate([rng.randint(0, 40, 60), [99]])      # 99: no gallery entry
    qcam = rng.randint(1, 7, len(qid))
    idx = ops.MatchIndex(qid, qcam, gid, gcam, device='cpu')
    members = idx.members.numpy()
    beg, end = idx.q_beg.numpy(), idx.q_end.numpy()
    for q in range(len(qid)):
        got = members[beg[q]:end[q]]
        np.testing.assert_array_equal(got, np.nonzero(gid == qid[q])[0])
    assert idx.capacity == max(1, max(int((gid == i).sum()) for i in qid))
    assert end[-1] == beg[-1]


def test_max_same_id_is_exact_per_shard():
    rng = np.random.RandomState(1)
    gid = rng.randint(0, 30, 1000)
    qid = rng.randint(0, 35, 200)
    for r in range(3):
        a, b = pdist.shard_range(len(gid), r, 3)
        want = max([1] + [int((gid[a:b] == i).sum()) for i in qid])
        assert pdist.max_same_id(qid, gid[a:b]) == want
    assert pdist.max_same_id([], gid) == 1 and pdist.max_same_id(qid, []) == 1


def test_mq_groups_first_appearance_order():
    keys, groups = pdist.mq_groups([5, 3, 5, 3, 5], [1, 2, 1, 1, 1])
    assert keys.tolist() == [[5, 1], [3, 2], [3, 1]]
    assert groups == [[0, 2, 4], [1], [3]]


def _bench(args, env=None):
    import json
    import subprocess
    import sys
    from tests.conftest import ROOT
    e = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    e.update(env or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=e,
                       capture_output=True, text=True, timeout=240)
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    return p.returncode, [json.loads(l) for l in lines], p.stderr


def test_bench_gpus_flag_launches_ranks():
    """`bench.py --gpus 2` starts two ranks (torch.distributed.run child,
    no GPU touched by the launcher) and rank 0 prints ONE line with n_gpus 2
    (--dry-run: the rendezvous / max-over-ranks / report path, gloo)."""
    rc, lines, err = _bench(['--gpus', '2', '--dry-run', '--steps', '2'])
    assert rc == 0, err[-2000:]
    assert len(lines) == 1 and lines[0]['n_gpus'] == 2 and lines[0]['dry_run'], lines


def test_bench_gpus_must_match_world_size():
    """Under a launcher (WORLD_SIZE set) --gpus must agree with it."""
    rc, lines, err = _bench(['--gpus', '4', '--dry-run'], env={'WORLD_SIZE': '2'})
    assert rc != 0 and not lines and '--gpus 4 but WORLD_SIZE=2' in err
