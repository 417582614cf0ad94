"""Tile sweep of one conv layer shape of the batch-64 forward (one process):
  python scripts/probes/conv_sweep.py SHAPE MATH [TILES...]   (MATH: h2, h2p, x3)
Shapes as scripts/probes/conv_once.py."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import model, ops  # noqa: E402
from scripts.probes.conv_once import SHAPES  # noqa: E402


def main():
    shape, math = sys.argv[1], sys.argv[2]
    tiles = [int(t) for t in sys.argv[3:]] or [0] + list(range(38, 54)) + [55, 56, 57, 58, 59, 60]
    N = 64
    H, W, Cin, Cout, k = SHAPES[shape]
    rng = np.random.RandomState(0)
    x = torch.from_numpy(np.maximum(rng.randn(N, H, W, Cin), 0).astype(np.float32)).cuda()
    w = (rng.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)).astype(np.float32)
    wp, kpad = model.pack_conv_weight(w)
    wp = torch.from_numpy(wp).cuda()
    sc = torch.ones(Cout, device='cuda')
    sh = torch.zeros(Cout, device='cuda')
    y = torch.empty((N, H, W, Cout), device='cuda')
    p = k // 2
    fl = 2.0 * N * H * W * Cout * Cin * k * k
    if math.startswith('h2'):
        w2, wrs = ops.split_weights_h2(wp)
        amx = ops.amax(x)
        xin = ops.split_act_h2(x, amx) if math == 'h2p' else x
    else:
        w3 = ops.split_bf16x3(wp)
    for tile in tiles:
        if tile == 54 or (tile >= 56 and tile <= 59 and k != 3):
            continue
        if math.startswith('h2'):
            run = lambda: ops.conv2d_bn_act_h2(xin, Cin, w2, wrs, kpad, k, 1, p, 1, sc, sh, None,
                                               True, y, amx, tile=tile)
        else:
            run = lambda: ops.conv2d_bn_act(x, Cin, w3, kpad, k, 1, p, 1, sc, sh, None, True, y,
                                            tile=tile)
        try:
            run()
        except RuntimeError as e:
            print('%s %s tile %d: %s' % (shape, math, tile, str(e)[:60]))
            continue
        torch.cuda.synchronize()
        best = 1e30
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 100.0)
        print('%s %s tile %d: %.1f us, %.1f TF' % (shape, math, tile, best, fl / best / 1e6),
              flush=True)


if __name__ == '__main__':
    main()
