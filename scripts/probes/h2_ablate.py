"""Distance-GEMM timing ablation (gemm_h2.hip H2_ABL builds): the Market
shape (3368 x 15913 x 3968) on the given h2 tiles with whatever library
PPS_LIB_PATH names -- the product build, one without main-loop DMA
(H2_ABL=1) and one without MFMAs (H2_ABL=2) tell which side bounds the
kernel.  python scripts/probes/h2_ablate.py [tiles...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import ops  # noqa: E402


def main():
    tiles = [int(t) for t in sys.argv[1:]] or [1, 5]
    Q, G, D = 3368, 15913, 3968
    gen = torch.Generator(device='cuda')
    gen.manual_seed(0)
    q = torch.nn.functional.normalize(torch.randn(Q, D, generator=gen, device='cuda'), dim=1)
    g = torch.nn.functional.normalize(torch.randn(G, D, generator=gen, device='cuda'), dim=1)
    idx = ops.GalleryIndex(g, math='h2')
    q2, qrs, qsq = ops.split_h2_tiled(q)
    out = ops.dist_buffer(Q, G, 'cuda')
    lib = os.path.basename(os.environ.get('PPS_LIB_PATH', 'libpps_hip.so'))
    for _ in range(2):
        for t in tiles:
            ops.distmat_h2(q2, qrs, qsq, idx, out, tile=t)
    torch.cuda.synchronize()
    res = {t: [] for t in tiles}
    for _ in range(3):   # interleaved rounds
        for t in tiles:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                ops.distmat_h2(q2, qrs, qsq, idx, out, tile=t)
            e1.record()
            e1.synchronize()
            res[t].append(e0.elapsed_time(e1) * 1e3 / 5)
    fl = 2.0 * Q * G * D
    for t in tiles:
        us = min(res[t])
        print('%s tile %d: %.1f us  %.1f TF  frac %.3f' % (lib, t, us, fl / us / 1e6,
                                                         fl / us / 1e6 / (2516.8 / 3)), flush=True)


if __name__ == '__main__':
    main()
