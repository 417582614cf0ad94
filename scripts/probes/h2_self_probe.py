"""f16x2 mirrored self-distance (pps_distmat_h2_self_tiled) at the Duke
re-ranking size (19,889 = 2,228 + 17,661 rows x 3968) on every f16x2 tile.
TF counted on the work the mirrored mode does: N (N + 1) / 2 dot products."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import ops  # noqa: E402


def main():
    N, D = (int(v) for v in os.environ.get('SHAPE', '19889,3968').split(','))
    x = torch.nn.functional.normalize(torch.randn(N, D, device='cuda'), dim=1)
    half = 2.0 * N * (N + 1) / 2 * D
    out = None

    def t(tile):
        nonlocal out
        for _ in range(2):
            out = ops.compute_dist(x, x, metric='cosine', tile=tile, symmetric=True, math='h2',
                                   pad_rows=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            out = ops.compute_dist(x, x, metric='cosine', tile=tile, symmetric=True, math='h2',
                                   pad_rows=True)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / 3

    res = []
    for tile in range(0, ops.h2_num_tiles()):
        ms = t(tile)
        res.append((ms, tile))
        print('h2 sym tile %d  %.3f ms (%.0f TF on the half, %.3f of the h2 roof)' % (
            tile, ms, half / ms / 1e9, half / ms / 1e9 / 838.9), flush=True)
    print('best: tile %d %.3f ms' % (min(res)[1], min(res)[0]))


if __name__ == '__main__':
    main()
