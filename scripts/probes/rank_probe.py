"""Probe: rank_count_stream variants on the Market-size distance matrix.
  PPS_LIB_PATH=_variants/libpps_hip_X.so python scripts/rank_probe.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', os.path.join(os.path.dirname(__file__), '..', '..')))
import bench  # noqa: E402
from pps_amd import distributed as pdist  # noqa: E402
from pps_amd import ops  # noqa: E402

Q, G = bench.Q_MARKET, bench.G_MARKET
rng = np.random.RandomState(0)
qid = rng.randint(1, 751, Q)
gid = np.concatenate([rng.randint(1, 751, G - 2793), np.zeros(2793, int)])
qcam, gcam = rng.randint(1, 7, Q), rng.randint(1, 7, G)
gen = torch.Generator(device='cuda')
gen.manual_seed(0)
f = bench.synth_features(Q + G, torch.from_numpy(np.concatenate([qid, gid])).cuda(), gen)
d = ops.compute_dist(f[:Q].contiguous(), f[Q:].contiguous(), pad_rows=True)
ev = pdist.ShardedEvaluator(qid, qcam, gid, gcam, 0, 1)
r = bench.rank_roofline(ev, d, reps=50)
frac = float((d <= 0).float().mean())
print(os.path.basename(os.environ.get('PPS_LIB_PATH', 'default')), 'us %.2f' % r['avg_launch_us'],
      'GB/s %.0f' % r['achieved'], 'pmax', ev.pmax, flush=True)
