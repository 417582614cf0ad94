"""One conv layer of the batch-64 forward, alone, for profiling
(scripts/probes/conv_pmc.sh):  python scripts/probes/conv_once.py SHAPE MATH TILE [--reps N]
SHAPE: res5b (3x3 512->512, 24x8), res5a (1x1 2048->512), res5c (1x1 512->2048),
res4b (3x3 256->256), res4a (1x1 1024->256), res4c (1x1 256->1024), res3b, res2b,
res2a0 (res2_0_branch2a: 1x1 64->64 on 96x32)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import model, ops  # noqa: E402

SHAPES = {   # H, W, Cin, Cout, k
    'res5b': (24, 8, 512, 512, 3), 'res5a': (24, 8, 2048, 512, 1),
    'res5c': (24, 8, 512, 2048, 1), 'res4b': (24, 8, 256, 256, 3),
    'res4a': (24, 8, 1024, 256, 1), 'res4c': (24, 8, 256, 1024, 1),
    'res3b': (48, 16, 128, 128, 3), 'res2b': (96, 32, 64, 64, 3),
    'res3c': (48, 16, 128, 512, 1), 'res2c': (96, 32, 64, 256, 1),
    'res2a': (96, 32, 256, 64, 1), 'res3a': (48, 16, 512, 128, 1),
    'res2a0': (96, 32, 64, 64, 1),
}


def main():
    shape, math, tile = sys.argv[1], sys.argv[2], int(sys.argv[3])
    reps = int(sys.argv[sys.argv.index('--reps') + 1]) if '--reps' in sys.argv else 20
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
    if math in ('h2', 'h2p'):
        w2, wrs = ops.split_weights_h2(wp)
        amx = ops.amax(x)
        xin = ops.split_act_h2(x, amx) if math == 'h2p' else x
        run = lambda: ops.conv2d_bn_act_h2(xin, Cin, w2, wrs, kpad, k, 1, p, 1, sc, sh, None, True,
                                           y, amx, tile=tile)
        if math == 'h2p':   # the split pass, timed separately
            pl = torch.empty_like(xin)
            ops.split_act_h2(x, amx, out=pl)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                ops.split_act_h2(x, amx, out=pl)
            e1.record()
            torch.cuda.synchronize()
            print('split pass: %.1f us' % (e0.elapsed_time(e1) * 1e3 / reps))
    else:
        w3 = ops.split_bf16x3(wp)
        run = lambda: ops.conv2d_bn_act(x, Cin, w3, kpad, k, 1, p, 1, sc, sh, None, True, y,
                                        tile=tile)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    fl = 2.0 * N * H * W * Cout * Cin * k * k
    nb = 4.0 * N * H * W * (Cin + Cout)
    print('%s %s tile %d: %.1f us, %.1f TF, %.2f TB/s in + out' % (shape, math, tile, us,
                                                                 fl / us / 1e6, nb / us / 1e6))


if __name__ == '__main__':
    main()
