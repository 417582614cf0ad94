"""Distance GEMM on chunk-tiled planes (pps_tile_planes + pps_distmat_x3p_tiled)
vs the row-major planes (pps_distmat_x3p), same tile, same box: bits and
time.  SHAPE=Q,G,D (default Market 3368,15913,3968), TILES=47,42."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import ops  # noqa: E402
from pps_amd.ops import _dev, _dev_rows, _ld, _stream, call  # noqa: E402


def tiled(planes, rows, D):
    r16 = (rows + 15) // 16 * 16
    out = torch.empty(3 * r16 * D, dtype=torch.int16, device='cuda')
    call('pps_tile_planes', _dev(planes, 'planes', torch.int16), rows, D, D, rows * D,
         _dev(out, 'out', torch.int16), _stream())
    return out


def timed(fn, n=5):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    Q, G, D = (int(v) for v in os.environ.get('SHAPE', '3368,15913,3968').split(','))
    q = torch.nn.functional.normalize(torch.randn(Q, D, device='cuda'), dim=1)
    g = torch.nn.functional.normalize(torch.randn(G, D, device='cuda'), dim=1)
    idx = ops.GalleryIndex(g)
    q3, qsq = ops.split_sqnorm(q)
    qt, gt = tiled(q3, Q, D), tiled(idx.planes, G, D)
    out = ops.dist_buffer(Q, G, 'cuda')
    out2 = ops.dist_buffer(Q, G, 'cuda')
    flops = 2.0 * Q * G * D
    for t in [int(v) for v in os.environ.get('TILES', '47,42').split(',')]:
        base = lambda: ops.distmat_planes(q3, qsq, idx, out, tile=t)  # noqa: E731
        til = lambda: call('pps_distmat_x3p_tiled', _dev(qt, 'qt', torch.int16), Q,  # noqa: E731
                           _dev(qsq, 'qsq'), _dev(gt, 'gt', torch.int16), _dev(idx.sqnorm, 'gsq'),
                           G, D, 0, _dev_rows(out2, 'out'), _ld(out2), t, _stream())
        mb, mt = timed(base), timed(til)
        same = torch.equal(out, out2)
        print('tile %d  row-major %.3f ms (%.0f TF)  tiled %.3f ms (%.0f TF)  bits equal %s'
              % (t, mb, flops / mb / 1e9, mt, flops / mt / 1e9, same), flush=True)
        if not same:
            sys.exit(1)


if __name__ == '__main__':
    main()
