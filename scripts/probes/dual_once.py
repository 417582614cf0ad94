"""A branch2c fused-shortcut conv of the batch-64 forward, alone, f16x2:
python scripts/probes/dual_once.py TILE [--reps N] [--shape res2|res5]
res2: 1x1 64 -> 256 on res2_0_branch2b's output + the 1x1 64 -> 256
projection of pool1 (K = 128; PPS_WS_H2_WIDE=1: the 256-column
weight-stationary block); res5: 1x1 512 -> 2048 + the stride-1 1024 -> 2048
projection of res4's output on 24 x 8 (K = 1536)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import model, ops  # noqa: E402


def main():
    tile = int(sys.argv[1])
    reps = int(sys.argv[sys.argv.index('--reps') + 1]) if '--reps' in sys.argv else 20
    shape = sys.argv[sys.argv.index('--shape') + 1] if '--shape' in sys.argv else 'res2'
    N, H, W, C1, C2, Cout = {'res2': (64, 96, 32, 64, 64, 256),
                             'res5': (64, 24, 8, 512, 1024, 2048)}[shape]
    rng = np.random.RandomState(0)
    x = torch.from_numpy(np.maximum(rng.randn(N, H, W, C1), 0).astype(np.float32)).cuda()
    x2 = torch.from_numpy(np.maximum(rng.randn(N, H, W, C2), 0).astype(np.float32)).cuda()
    w1 = (rng.randn(Cout, C1, 1, 1) / 8).astype(np.float32)
    w2 = (rng.randn(Cout, C2, 1, 1) / 8).astype(np.float32)
    p1, k1 = model.pack_conv_weight(w1)
    p2, _ = model.pack_conv_weight(w2)
    wq, wrs = ops.split_weights_h2(torch.from_numpy(np.concatenate([p1, p2], 1)).cuda())
    sh = torch.zeros(Cout, device='cuda')
    y = torch.empty((N, H, W, Cout), device='cuda')
    a1, a2 = ops.amax(x), ops.amax(x2)
    run = lambda: ops.conv2d_dual_bn_act_h2(x, C1, 1, 1, 0, x2, 1, wq, wrs, k1, sh, True, y,  # noqa
                                           a1, a2, tile=tile)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    byt = 4.0 * N * H * W * (C1 + C2 + Cout)
    fl = 2.0 * N * H * W * Cout * (C1 + C2)
    print('dual %s tile %d (wide %s, GM %s): %.1f us, %.2f TB/s algorithmic, %.1f TF'
          % (shape, tile, os.environ.get('PPS_WS_H2_WIDE', '0'), os.environ.get('PPS_CONV_GM', '0'),
             us, byt / us / 1e6, fl / us / 1e6))


if __name__ == '__main__':
    main()
