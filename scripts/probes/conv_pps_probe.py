"""Probe: the last res5 conv (1x1 512 -> 2048 + BN + residual + ReLU, batch
64, 24 x 8) alone vs with the part pooling fused into its epilogue, per
eligible tile; plus the standalone pooling kernel."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from pps_amd import model, ops  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


rng = np.random.RandomState(0)
N, H, W, Cin, Cout = 64, 24, 8, 512, 2048
x = torch.randn(N, H, W, Cin, device='cuda').relu()
w = (rng.randn(Cout, Cin, 1, 1) / np.sqrt(Cin)).astype(np.float32)
wp, kpad = model.pack_conv_weight(w)
w3 = ops.split_bf16x3(torch.from_numpy(wp).cuda())
sc = torch.ones(Cout, device='cuda')
sh = torch.zeros(Cout, device='cuda')
res = torch.randn(N, H, W, Cout, device='cuda')
y = torch.empty(N, H, W, Cout, device='cuda')
out = torch.empty(31, N, Cout, device='cuda')
split = [5, 5, 4, 5, 5]
print('pooling kernel alone: %.1f us' % timeit(lambda: ops.part_power_set(y, split, True, out)))
for t in (36, 42, 43):
    print('tile %d conv: %.1f us' % (t, timeit(lambda: ops.conv2d_bn_act_x3p(
        x, Cin, w3, kpad, 1, 1, 0, 1, sc, sh, res, True, y, tile=t))))
for t in range(ops.TILE_P_FIRST, ops.num_tiles() + 1):
    r, c = ops.tile_shape(t)
    if r != H * W or c > 128:
        continue
    a = timeit(lambda: ops.conv2d_bn_act_x3p(x, Cin, w3, kpad, 1, 1, 0, 1, sc, sh, res, True, y,
                                             tile=t))
    b = timeit(lambda: ops.conv2d_bn_act_pps(x, Cin, w3, kpad, 1, 1, 0, 1, sc, sh, res, split,
                                             True, out, tile=t))
    c2 = timeit(lambda: ops.conv2d_bn_act_pps(x, Cin, w3, kpad, 1, 1, 0, 1, sc, sh, res, split,
                                              True, out, y=y, tile=t))
    print('tile %d (%dx%d): conv %.1f us, conv+pooling %.1f us (writing y too: %.1f us)'
          % (t, r, c, a, b, c2), flush=True)
