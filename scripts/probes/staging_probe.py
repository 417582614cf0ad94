"""Do the mid-size 1x1 convs scale with the bytes they stage into LDS?
res4 2a (M = 12288, K = 1024, N = 256) and res4 2c (K = 256, N = 1024) at
batch 64, on the pipelined tiles, with the activation operand as f32 rows
(4 B / element staged) and as bf16x3 planes (6 B): if the planes input is
slower by about its extra staged bytes, the layer is bound by the LDS fill,
not by the MFMAs or the split arithmetic."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))


def bench(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def main():
    from pps_amd import ops
    g = torch.Generator(device='cuda')
    g.manual_seed(0)
    for name, K, N in (('res4_2a', 1024, 256), ('res4_2c', 256, 1024)):
        x = torch.randn((64, 24, 8, K), generator=g, device='cuda')
        w = torch.randn((N, K), generator=g, device='cuda') * 0.03
        w3 = ops.split_bf16x3(w)
        sc = torch.ones(N, device='cuda')
        sh = torch.zeros(N, device='cuda')
        y = torch.empty((64, 24, 8, N), device='cuda')
        xp = ops.act_planes(x.shape, 'cuda')
        ops.conv2d_bn_act_x3p(x, K, w3, K, 1, 1, 0, 1, sc, sh, None, False, xp, tile=38)
        for tile in (36, 40, 45, 47, 49, 50, 51, 53):
            try:
                tf = bench(lambda: ops.conv2d_bn_act_x3p(x, K, w3, K, 1, 1, 0, 1, sc, sh, None,
                                                         True, y, tile=tile))
                tp = bench(lambda: ops.conv2d_bn_act_x3p(xp, K, w3, K, 1, 1, 0, 1, sc, sh, None,
                                                         True, y, tile=tile))
            except RuntimeError as e:
                print(name, tile, 'n/a', str(e)[:60], flush=True)
                continue
            bm, bn = ops.tile_shape(tile)
            print('%s tile %d (%dx%d): f32 A %.1f us, planes A %.1f us (x%.2f)'
                  % (name, tile, bm, bn, tf, tp, tp / tf), flush=True)


if __name__ == '__main__':
    main()
