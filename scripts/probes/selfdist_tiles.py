"""Mirrored self-distance (re-ranking's [queries; gallery] x itself, Duke
sizes N = 2228 + 17661, D = 3968, cosine) on each h2 distance tile:
python scripts/probes/selfdist_tiles.py [tiles...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import ops  # noqa: E402


def main():
    tiles = [int(t) for t in sys.argv[1:]] or list(range(0, 8))
    N, D = 2228 + 17661, 3968
    gen = torch.Generator(device='cuda')
    gen.manual_seed(0)
    x = torch.nn.functional.normalize(torch.randn(N, D, generator=gen, device='cuda'), dim=1)
    out = ops.dist_buffer(N, N, 'cuda')
    ref = None
    for t in tiles:
        ops.compute_dist(x, x, metric='cosine', out=out, tile=t, symmetric=True)
    torch.cuda.synchronize()
    res = {t: [] for t in tiles}
    for _ in range(3):
        for t in tiles:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                ops.compute_dist(x, x, metric='cosine', out=out, tile=t, symmetric=True)
            e1.record()
            e1.synchronize()
            res[t].append(e0.elapsed_time(e1) / 3)
            if ref is None:
                ref = out.clone()
            else:
                assert torch.equal(out, ref), t   # every tile: the same bits
    fl = 2.0 * N * N * D / 2   # the upper triangle
    for t in tiles:
        ms = min(res[t])
        print('self-distance tile %d: %.3f ms  %.1f TF (triangle)' % (t, ms, fl / ms / 1e9), flush=True)


if __name__ == '__main__':
    main()
