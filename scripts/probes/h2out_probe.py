"""Producer cost of f16x2 planes out (EPI_F_H2OUT) vs the f32 output, one
1x1 / 3x3 conv + BN + ReLU of the batch-64 forward, f16x2 and bf16x3 arithmetic:
  python scripts/probes/h2out_probe.py [--reps N]
Prints us per launch for each (shape, math, tile, output) cell."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import model, ops  # noqa: E402

SHAPES = {   # H, W, Cin, Cout, k
    'res2a': (96, 32, 256, 64, 1), 'res3a': (48, 16, 512, 128, 1),
    'res3b': (48, 16, 128, 128, 3), 'res4a': (24, 8, 1024, 256, 1),
    'res5a': (24, 8, 2048, 512, 1), 'res5b': (24, 8, 512, 512, 3),
}


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    reps = int(sys.argv[sys.argv.index('--reps') + 1]) if '--reps' in sys.argv else 50
    N = 64
    rng = np.random.RandomState(0)
    for name, (H, W, Cin, Cout, k) in SHAPES.items():
        x = torch.from_numpy(np.maximum(rng.randn(N, H, W, Cin), 0).astype(np.float32)).cuda()
        w = (rng.randn(Cout, Cin, k, k) / np.sqrt(Cin * k * k)).astype(np.float32)
        wp, kpad = model.pack_conv_weight(w)
        wp = torch.from_numpy(wp).cuda()
        sc = torch.ones(Cout, device='cuda')
        sh = torch.zeros(Cout, device='cuda')
        y = torch.empty((N, H, W, Cout), device='cuda')
        y2 = torch.empty((2, N, H, W, Cout), dtype=torch.int16, device='cuda')
        p = k // 2
        w2, wrs = ops.split_weights_h2(wp)
        w3 = ops.split_bf16x3(wp)
        amx = ops.amax(x)
        bnd = ops.h2_out_bound(wp, sc, sh)
        bout = ops.amax_slot()
        for tile in (38, 45, 47, 47 | ops.TILE_COL_ORDER, 49, 60):
            if tile == 60 and False:
                continue
            cells = []
            try:
                cells.append(timed(lambda: ops.conv2d_bn_act_h2(
                    x, Cin, w2, wrs, kpad, k, 1, p, 1, sc, sh, None, True, y, amx, tile=tile), reps))
                cells.append(timed(lambda: ops.conv2d_bn_act_h2out(
                    x, Cin, w2, wrs, kpad, k, 1, p, 1, sc, sh, y2, amx, amx, bnd, bout,
                    tile=tile), reps))
            except RuntimeError as e:
                cells += [float('nan')] * (2 - len(cells))
                print('  h2 tile %d: %s' % (tile, str(e)[:80]))
            if tile != 60:
                cells.append(timed(lambda: ops.conv2d_bn_act(
                    x, Cin, w3, kpad, k, 1, p, 1, sc, sh, None, True, y, tile=tile), reps))
                cells.append(timed(lambda: ops.conv2d_bn_act_h2out(
                    x, Cin, w3, None, kpad, k, 1, p, 1, sc, sh, y2, None, amx, bnd, bout,
                    tile=tile), reps))
            print('%-6s tile %#5x  h2 f32 %7.1f  h2 planes %7.1f  | x3 f32 %s  x3 planes %s' % (
                name, tile, cells[0], cells[1],
                '%7.1f' % cells[2] if len(cells) > 2 else '   -', '%7.1f' % cells[3]
                if len(cells) > 3 else '   -'), flush=True)


if __name__ == '__main__':
    main()
