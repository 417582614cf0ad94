"""Timing of the bottleneck seam (pps_conv1x1_seam_x3) at batch 64 against
the two unfused 1x1 layers on their usual tiles (res2: WS tile 54 for both;
res3: 2c on tile 54, 2a on tile 47 | tiled weights), and the algorithmic HBM
rate of each."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import model, ops  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    for name, H, W, K1, t2c, t2a in (('res2', 96, 32, 64, 54, 54), ('res3', 48, 16, 128, 54, 47)):
        if os.environ.get('ONLY') and os.environ['ONLY'] != name:
            continue
        N = 64
        N1, N2 = 4 * K1, K1
        rng = np.random.RandomState(0)
        x = torch.relu(torch.randn(N, H, W, K1, device='cuda'))
        res = torch.relu(torch.randn(N, H, W, N1, device='cuda'))
        pc, kc = model.pack_conv_weight((rng.randn(N1, K1, 1, 1) / np.sqrt(K1)).astype(np.float32))
        pa, ka = model.pack_conv_weight((rng.randn(N2, N1, 1, 1) / np.sqrt(N1)).astype(np.float32))
        w2c3 = ops.split_bf16x3(torch.from_numpy(pc).cuda())
        w2a3 = ops.split_bf16x3(torch.from_numpy(pa).cuda())
        s1, s2 = torch.ones(N1, device='cuda'), torch.ones(N2, device='cuda')
        z1, z2 = torch.zeros(N1, device='cuda'), torch.zeros(N2, device='cuda')
        trunk = torch.empty(N, H, W, N1, device='cuda')
        y = torch.empty(N, H, W, N2, device='cuda')
        M = N * H * W
        fused = timeit(lambda: ops.conv1x1_seam(x, w2c3, s1, z1, res, trunk, w2a3, s2, z2, y))
        c = timeit(lambda: ops.conv2d_bn_act_x3p(x, K1, w2c3, kc, 1, 1, 0, 1, s1, z1, res, True,
                                                 trunk, tile=t2c))
        a = timeit(lambda: ops.conv2d_bn_act_x3p(trunk, N1, w2a3, ka, 1, 1, 0, 1, s2, z2, None,
                                                 True, y, tile=t2a))
        fb = M * (K1 + 2 * N1 + N2) * 4
        print('%s M=%d: seam %.1f us (%.2f TB/s on %.0f MB) | 2c %.1f + 2a %.1f = %.1f us'
              % (name, M, fused, fb / fused / 1e6, fb / 1e6, c, a, c + a), flush=True)


if __name__ == '__main__':
    main()
