"""Market distance GEMM (3368 x 15913 x 3968, f16x2) per tile, operands
prepared once: python scripts/probes/dist_tiles_time.py  (PPS_LIB_PATH
selects a library build for A/B runs)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import ops  # noqa: E402


def main():
    Q, G, D = 3368, 15913, 3968
    torch.manual_seed(0)
    q = torch.nn.functional.normalize(torch.randn(Q, D, device='cuda'), dim=1)
    g = torch.nn.functional.normalize(torch.randn(G, D, device='cuda'), dim=1)
    gidx = ops.GalleryIndex(g, math='h2')
    q2, qrs, qsq = ops.split_h2_tiled(q)
    out = ops.dist_buffer(Q, G, 'cuda')
    fl = 2.0 * Q * G * D
    tag = os.path.basename(os.environ.get('PPS_LIB_PATH', 'in-tree'))
    for t in [int(v) for v in os.environ.get('TILES', '0,6,7').split(',')]:
        run = lambda: ops.distmat_h2(q2, qrs, qsq, gidx, out, tile=t)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1) / 10)
        print('%s tile %d %.1f us %.0f TF' % (tag, t, best * 1e3, fl / best / 1e9), flush=True)


if __name__ == '__main__':
    main()
