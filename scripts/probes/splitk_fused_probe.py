"""One-launch split-K (EPI_F_FIX) vs the one-pass kernel on the res4 / res5
bottleneck shapes at batch 64, with the bench's operand formats (planes
into branch2b, planes out of branch2a, residual on branch2c) and plain /
chunk-tiled weights.  Prints us per launch (event-timed, 30 reps)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import model, ops  # noqa: E402

# name: N, H, W, Cin, Cout, k, planes_in, planes_out, residual
LAYERS = {'res4a': (64, 24, 8, 1024, 256, 1, False, True, False),
          'res4b': (64, 24, 8, 256, 256, 3, True, False, False),
          'res4c': (64, 24, 8, 256, 1024, 1, False, False, True),
          'res5a': (64, 24, 8, 2048, 512, 1, False, True, False),
          'res5b': (64, 24, 8, 512, 512, 3, True, False, False),
          'res3b': (64, 48, 16, 128, 128, 3, True, False, False)}


def planes_of(x):
    return ops.split_bf16x3(x.reshape(-1)).reshape((3,) + tuple(x.shape))


def main():
    for name, (N, H, W, Cin, Cout, k, pin, pout, hres) in LAYERS.items():
        x = torch.randn(N, H, W, Cin, device='cuda').clamp_min(0)
        xin = planes_of(x) if pin else x
        w = np.random.RandomState(0).randn(Cout, Cin, k, k).astype(np.float32) / np.sqrt(Cin * k * k)
        wp, kpad = model.pack_conv_weight(w)
        w3 = ops.split_bf16x3(torch.from_numpy(wp).cuda())
        wt = ops.tile_planes(w3)
        sc = torch.ones(Cout, device='cuda')
        sh = torch.zeros(Cout, device='cuda')
        res = torch.randn(N, H, W, Cout, device='cuda') if hres else None
        y = ops.act_planes((N, H, W, Cout), 'cuda') if pout else torch.empty(N, H, W, Cout, device='cuda')
        part = torch.empty(4 * N * H * W * Cout, device='cuda')
        cnt = torch.zeros(65536, dtype=torch.int32, device='cuda')
        out = []
        for tile in ops.FIX_TILES:
            for tiled in (False, True):
                for sk in (1, 2, 3, 4):
                    if kpad % (32 * sk):
                        continue
                    wf, tf = (wt, tile | ops.TILE_B_TILED) if tiled else (w3, tile)

                    def run():
                        ops.conv2d_bn_act_x3p(xin, Cin, wf, kpad, k, 1, k // 2, 1, sc, sh, res,
                                              True, y, tile=tf, splitk=sk,
                                              part=part if sk > 1 else None,
                                              counters=cnt if sk > 1 else None)
                    for _ in range(3):
                        run()
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(30):
                        run()
                    e1.record()
                    e1.synchronize()
                    out.append((e0.elapsed_time(e1) / 30 * 1e3, '%d%s/s%d' % (tile, 't' if tiled else '', sk)))
        out.sort()
        one = min(u for u, s in out if s.endswith('/s1'))
        fused = [(u, s) for u, s in out if not s.endswith('/s1')]
        print('%-6s best one-pass %.1f us | fused %s' % (name, one, ' '.join('%s:%.1f' % (s, u) for u, s in fused[:6])),
              flush=True)


if __name__ == '__main__':
    main()
