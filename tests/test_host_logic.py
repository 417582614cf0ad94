"""Host-side logic of the retrieval path (no GPU): the per-identity gallery
index the match collection reads, the exact list capacity of the sharded
evaluator, multi-query grouping (reid_dataset_evaluator.py:136-143)."""
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
