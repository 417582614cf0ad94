"""Probe: the stem at batch 64 (384x128): fused conv+BN+ReLU+pool kernel vs
the two-kernel path (implicit-GEMM conv + maxpool), per-launch HIP events."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', os.path.join(os.path.dirname(__file__), '..', '..')))
import bench  # noqa: E402
from pps_amd import model, ops  # noqa: E402

bench.market_cfg()
plan = model.build_plan()
blobs = model.synthetic_weights(plan, seed=0)
x = torch.randn(64, 384, 128, 4, device='cuda') * 50
x[..., 3] = 0
cases = [(True, 0), (True, 1)] + ([] if os.environ.get('FUSED_ONLY') else [(False, 0)])
for fused, variant in cases * 2:
    ops.stem_variant(variant)
    m = model.PPSModel(blobs, fused_stem=fused)
    m.forward(x)
    if not fused:
        m.autotune(x, tiles=None)
    t = {}
    for rep in range(5):
        timer = []
        m.forward(x, timer=timer)
        torch.cuda.synchronize()
        for name, op, f, e0, e1 in timer:
            if op in ('stem_pool', 'maxpool') or name == 'conv1':
                t.setdefault((name, op), []).append(e0.elapsed_time(e1) * 1e3)
    print('fused v%d' % variant if fused else 'two-kernel',
          {'%s/%s' % k: round(float(np.median(v)), 1) for k, v in t.items()},
          'total us %.1f' % sum(float(np.median(v)) for v in t.values()), flush=True)
