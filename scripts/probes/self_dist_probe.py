"""Self-distance timing at the Duke gallery size (17661 x 3968): the full
product on the distance matrix's tiles vs the symmetric mode (upper-triangle
super-blocks + mirror, chunk-tiled planes) on every pipelined tile.  TF are
counted on the work the symmetric mode must do: N (N + 1) / 2 dot products."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import ops  # noqa: E402


def main():
    N, D = (int(v) for v in os.environ.get('SHAPE', '17661,3968').split(','))
    x = torch.nn.functional.normalize(torch.randn(N, D, device='cuda'), dim=1)
    idx = ops.GalleryIndex(x, tiled=True)
    out = torch.empty(N, N, device='cuda')
    half = 2.0 * N * (N + 1) / 2 * D

    def t(**kw):
        for _ in range(2):
            ops.compute_dist(x, idx, out=out, metric='cosine', **kw)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            ops.compute_dist(x, idx, out=out, metric='cosine', **kw)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / 3

    for tile in [int(v) for v in os.environ.get('FULL', '43').split(',') if v]:
        ms = t(tile=tile, symmetric=False)
        print('full  tile %d  %.3f ms (%.0f TF, %.0f TF on the half)' % (
            tile, ms, 2 * half / ms / 1e9, half / ms / 1e9), flush=True)
    tiles = [int(v) for v in os.environ['TILES'].split(',')] if os.environ.get('TILES') \
        else ops.SELF_TILES[1:]
    res = []
    for tile in tiles:
        ms = t(tile=tile, symmetric=True)
        res.append((ms, tile))
        print('sym   tile %d  %.3f ms (%.0f TF on the half, %.3f of the x3 roof)' % (
            tile, ms, half / ms / 1e9, half / ms / 1e9 / 419.5), flush=True)
    print('best sym: tile %d %.3f ms' % (min(res)[1], min(res)[0]))


if __name__ == '__main__':
    main()
