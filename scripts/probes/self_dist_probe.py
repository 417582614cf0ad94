"""Self-distance timing at the Duke gallery size (17661 x 3968): the full
product on its best tiles vs the symmetric (upper-triangle + mirror) mode on
the square tiles."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import ops  # noqa: E402


def main():
    N, D = (int(v) for v in os.environ.get('SHAPE', '17661,3968').split(','))
    x = torch.nn.functional.normalize(torch.randn(N, D, device='cuda'), dim=1)
    idx = ops.GalleryIndex(x)
    out = torch.empty(N, N, device='cuda')
    flops = 2.0 * N * N * D

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

    for tile in (ops.TILE_P16_FIRST + 4, ops.TILE_P_FIRST + 4):
        ms = t(tile=tile, symmetric=False)
        print('full  tile %d  %.3f ms (%.0f TF)' % (tile, ms, flops / ms / 1e9), flush=True)
    for tile in ops.SELF_TILES[1:]:
        ms = t(tile=tile, symmetric=True)
        print('sym   tile %d  %.3f ms (%.0f TF-equivalent)' % (tile, ms, flops / ms / 1e9),
              flush=True)


if __name__ == '__main__':
    main()
