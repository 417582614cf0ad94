"""Grouped tile order (X3P_GM_MB) A/B: Duke [queries; gallery] self-distance
and the Market tiled distance GEMM (tile 43) with the library in
PPS_LIB_PATH (builds with -DX3P_GM_MB=<MB>)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))


def timed(fn, n=4):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    from pps_amd import ops
    D = 3968
    x = torch.nn.functional.normalize(torch.randn(2228 + 17661, D, device='cuda'), dim=1)
    sd = timed(lambda: ops.self_distance_blocks(x, 2228, metric='cosine'))
    del x
    Q, G = 3368, 15913
    q = torch.nn.functional.normalize(torch.randn(Q, D, device='cuda'), dim=1)
    g = torch.nn.functional.normalize(torch.randn(G, D, device='cuda'), dim=1)
    idx = ops.GalleryIndex(g, tiled=True)
    qt, qsq = ops.split_sqnorm_tiled(q)
    out = ops.dist_buffer(Q, G, 'cuda')
    dm = timed(lambda: ops.distmat_planes(None, qsq, idx, out, 'euclidean', 43, q_tiled=qt,
                                          Q=Q, D=D), 8)
    print('%s: duke self-distance %.3f ms, market distmat %.3f ms'
          % (os.path.basename(os.environ.get('PPS_LIB_PATH', 'default(32)')), sd, dm), flush=True)


if __name__ == '__main__':
    main()
