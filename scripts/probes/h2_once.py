"""The h2 distance GEMM alone at the Market shape (or the Duke self-distance),
`--reps` launches after one warm-up, for rocprofv3 passes:
  python scripts/probes/h2_once.py [--tile T] [--reps N] [--self] [--x3]"""
import argparse
import sys

import torch

sys.path.insert(0, '.')
from pps_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tile', type=int, default=0)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--self', action='store_true', help='Duke self-distance (N = 19889)')
    ap.add_argument('--x3', action='store_true', help='the bf16x3 kernel instead')
    a = ap.parse_args()
    D = 3968
    gen = torch.Generator(device='cuda')
    gen.manual_seed(0)
    if a.self:
        N = 2228 + 17661
        x = torch.randn((N, D), generator=gen, device='cuda')
        x = (x / x.norm(dim=1, keepdim=True)).contiguous()
        out = ops.dist_buffer(N, N, 'cuda')
        if a.x3:
            xt, sq = ops.split_sqnorm_tiled(x)
            run = lambda: ops.call('pps_distmat_x3_self_tiled', xt.data_ptr(), N, sq.data_ptr(), D,
                                   2, out.data_ptr(), out.stride(0), a.tile, ops._stream())
        else:
            x2, rs, sq = ops.split_h2_tiled(x)
            run = lambda: ops.call('pps_distmat_h2_self_tiled', x2.data_ptr(), N, sq.data_ptr(),
                                   rs.data_ptr(), D, 2, out.data_ptr(), out.stride(0), a.tile,
                                   ops._stream())
    else:
        Q, G = 3368, 15913
        q = torch.randn((Q, D), generator=gen, device='cuda')
        q = (q / q.norm(dim=1, keepdim=True)).contiguous()
        g = torch.randn((G, D), generator=gen, device='cuda')
        g = (g / g.norm(dim=1, keepdim=True)).contiguous()
        out = ops.dist_buffer(Q, G, 'cuda')
        if a.x3:
            idx = ops.GalleryIndex(g, tiled=True, math='x3')
            qt, qsq = ops.split_sqnorm_tiled(q)
            run = lambda: ops.distmat_planes(None, qsq, idx, out, tile=a.tile or 43, q_tiled=qt,
                                             Q=Q, D=D)
        else:
            idx = ops.GalleryIndex(g, math='h2')
            q2, qrs, qsq = ops.split_h2_tiled(q)
            run = lambda: ops.distmat_h2(q2, qrs, qsq, idx, out, tile=a.tile)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        run()
    e1.record()
    e1.synchronize()
    print('avg %.3f ms over %d launches' % (e0.elapsed_time(e1) / a.reps, a.reps), flush=True)


if __name__ == '__main__':
    main()
