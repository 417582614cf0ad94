"""Top-k on long rows (1M-gallery shard rows): time + check vs torch.sort
(stable) on a few rows.  PPS_LIB_PATH selects a variant build."""
import os
import sys
import torch
sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '.'))
from pps_amd import ops


def t(d, k, reps=5):
    for _ in range(2):
        ops.topk(d, k)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        ops.topk(d, k)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


R, C = 10000, 125000
g = torch.Generator(device='cuda')
g.manual_seed(0)
for name in ('uniform', 'clustered'):
    if name == 'uniform':
        d = torch.rand((R, C), generator=g, device='cuda')
    else:   # distances of L2 features to identity centroids: a heavy low tail
        d = 2.0 - 2.0 * torch.rand((R, C), generator=g, device='cuda').pow(0.02)
    for k in (100,):
        ms = t(d, k)
        v, i = ops.topk(d, k)
        s, si = torch.sort(d[:64], dim=1, stable=True)
        ok = torch.equal(v[:64], s[:, :k]) and torch.equal(i[:64].long(), si[:, :k])
        print('%s %dx%d k=%d %.3f ms %.0f GB/s exact=%s' % (name, R, C, k, ms, R * C * 4 / ms / 1e6, ok),
              flush=True)
    if name == 'uniform':
        for _ in range(2):
            d.sum(dim=1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            d.sum(dim=1)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 5
        print('torch row-sum read %.3f ms %.0f GB/s' % (ms, R * C * 4 / ms / 1e6), flush=True)
    del d
