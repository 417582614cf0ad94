"""Which pipelined tile should pps_distmat_x3p_tiled default to?  Times the
tiled distance GEMM (queries and gallery as chunk-tiled bf16x3 planes, what
compute_dist(..., q_planes=True) on a GalleryIndex(tiled=True) runs) on the
Market and Duke query x gallery shapes for the candidate tiles."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))


def main():
    from pps_amd import ops
    D = 3968
    for name, Q, G in (('market', 3368, 15913), ('duke', 2228, 17661)):
        q = torch.nn.functional.normalize(torch.randn(Q, D, device='cuda'), dim=1)
        g = torch.nn.functional.normalize(torch.randn(G, D, device='cuda'), dim=1)
        idx = ops.GalleryIndex(g, tiled=True)
        qt, qsq = ops.split_sqnorm_tiled(q)
        out = ops.dist_buffer(Q, G, 'cuda')
        res = []
        for tile in (42, 43, 44, 47, 51, 52, 53):
            def run():
                ops.distmat_planes(None, qsq, idx, out, 'euclidean', tile, q_tiled=qt, Q=Q, D=D)
            for _ in range(2):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(8):
                run()
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / 8
            res.append((ms, tile))
            print('%s tile %d: %.3f ms  %.1f TF' % (name, tile, ms, 2.0 * Q * G * D / ms / 1e9),
                  flush=True)
        print(name, 'best', min(res), flush=True)


if __name__ == '__main__':
    main()
