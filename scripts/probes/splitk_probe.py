"""Conv split-K timing on the under-filled res4 shapes (batch 64):
one-pass pipelined tiles vs split-K 2/3/4 on the same tiles."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import model, ops  # noqa: E402

LAYERS = {'res4b': (64, 24, 8, 256, 256, 3), 'res4a': (64, 24, 8, 1024, 256, 1),
          'res4c': (64, 24, 8, 256, 1024, 1), 'res5a': (64, 24, 8, 2048, 512, 1),
          'res5b': (64, 24, 8, 512, 512, 3), 'res3b': (64, 48, 16, 128, 128, 3)}


def main():
    for name, (N, H, W, Cin, Cout, k) in LAYERS.items():
        x = torch.randn(N, H, W, Cin, device='cuda').clamp_min(0)
        w = np.random.RandomState(0).randn(Cout, Cin, k, k).astype(np.float32) / np.sqrt(Cin * k * k)
        wp, kpad = model.pack_conv_weight(w)
        w3 = ops.split_bf16x3(torch.from_numpy(wp).cuda())
        sc = torch.ones(Cout, device='cuda')
        sh = torch.zeros(Cout, device='cuda')
        y = torch.empty(N, H, W, Cout, device='cuda')
        part = torch.empty(4 * y.numel(), device='cuda')
        flops = 2.0 * N * H * W * Cout * k * k * Cin
        res = []
        for tile in (ops.TILE_P_FIRST, ops.TILE_P_FIRST + 7, ops.TILE_P_FIRST + 8,
                     ops.TILE_P16_FIRST + 7):
            for sk in (1, 2, 3, 4):
                if kpad % (32 * sk):
                    continue
                def run():
                    ops.conv2d_bn_act_x3p(x, Cin, w3, kpad, k, 1, k // 2, 1, sc, sh, None, True, y,
                                          tile=tile, splitk=sk, part=part)
                for _ in range(3):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    run()
                e1.record()
                e1.synchronize()
                ms = e0.elapsed_time(e1) / 20
                res.append('%d/s%d:%.3f(%.0f)' % (tile, sk, ms, flops / ms / 1e9))
        print('%-6s %s' % (name, ' '.join(res)), flush=True)


if __name__ == '__main__':
    main()
