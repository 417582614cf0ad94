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


def test_decode_pool_matches_in_process_decode(tmp_path):
    """The decode processes return exactly what decode_bgr returns in the
    calling process (BGR uint8, source shapes kept), in order."""
    from PIL import Image
    from pps_amd import decode_pool
    rng = np.random.RandomState(7)
    paths = []
    for i, (h, w) in enumerate([(128, 64), (97, 41), (128, 64), (200, 90), (64, 32)]):
        p = str(tmp_path / ('%d.jpg' % i))
        Image.fromarray(rng.randint(0, 256, (h, w, 3)).astype(np.uint8)).save(p, quality=90)
        paths.append(p)
    try:
        pool = decode_pool.start(2)
        assert decode_pool.workers() == 2 and decode_pool.start(3) is pool
        got = [im for c in pool.map(decode_pool.decode_many, [paths[:2], paths[2:]]) for im in c]
    finally:
        decode_pool.stop()
    assert decode_pool.pool() is None
    for p, g in zip(paths, got):
        want = decode_pool.decode_bgr(p)
        assert g.dtype == np.uint8 and g.shape == want.shape and np.array_equal(g, want)
    assert decode_pool.default_workers(share=1000) == 1


def test_h2_inv_scale_mirrors_the_kernel_scale():
    """native.h2_inv_scale (the f16x2-planes decode of NativeModel.tensor)
    follows pps_internal.hpp h2_scale_of: normal maxima land in [2^14, 2^15)
    after scaling, a zero max keeps scale 1, a denormal max takes 2^126, and
    the shift is clamped to [-126, 126]."""
    from pps_amd.native import h2_inv_scale
    rng = np.random.RandomState(0)
    for a in np.exp(rng.uniform(-70, 80, 200)).astype(np.float32):
        s = a / h2_inv_scale(a)
        assert 2.0 ** 14 <= s < 2.0 ** 15, (a, s)
    assert h2_inv_scale(0.0) == 1.0
    assert h2_inv_scale(np.float32(1e-40)) == 2.0 ** -126      # denormal
    assert h2_inv_scale(np.float32(1e-37)) == 2.0 ** -126      # shift clamped
    assert h2_inv_scale(np.float32(3e38)) == 2.0 ** 113
