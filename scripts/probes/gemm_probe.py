"""Time single implicit-GEMM conv launches (x3 and f32 kernels) on PPS layer
shapes, one tile at a time -- the unit used when tuning gemm_x3.hip /
gemm_f32.hip and for PMC passes (scripts/pmc.sh CMD="python3 scripts/gemm_probe.py").

  python scripts/gemm_probe.py [--layers res5b,res4b,...] [--tiles 1,5] [--math x3,f32]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))

# name: (N, H, W, Cin, Cout, k, stride, pad) at batch 64, 384x128 input
LAYERS = {
    'res5b': (64, 24, 8, 512, 512, 3, 1, 1),
    'res5a': (64, 24, 8, 2048, 512, 1, 1, 0),
    'res5c': (64, 24, 8, 512, 2048, 1, 1, 0),
    'res4b': (64, 24, 8, 256, 256, 3, 1, 1),
    'res3b': (64, 48, 16, 128, 128, 3, 1, 1),
    'res2b': (64, 96, 32, 64, 64, 3, 1, 1),
    'res2c': (64, 96, 32, 64, 256, 1, 1, 0),
    'stem': (64, 384, 128, 4, 64, 7, 2, 3),
    'res3c': (64, 48, 16, 128, 512, 1, 1, 0),
    'res4c': (64, 24, 8, 256, 1024, 1, 1, 0),
    'res4a': (64, 24, 8, 1024, 256, 1, 1, 0),
    'res2a': (64, 96, 32, 256, 64, 1, 1, 0),
    'res3a': (64, 48, 16, 512, 128, 1, 1, 0),
    'stemgemm': (64, 192, 64, 224, 64, 1, 1, 0),  # the stem as a plain K=224 GEMM
    # full-chip shapes (thousands of tiles): the kernel's own ceiling
    'big3x3': (64, 64, 64, 512, 512, 3, 1, 1),
    'big1x1': (64, 32, 32, 2048, 2048, 1, 1, 0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--layers', default='res5b,res5a,res4b,res2b')
    ap.add_argument('--tiles', default='1,2,3,4,5,6,7,8,9')
    ap.add_argument('--math', default='x3,f32')
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--residual', action='store_true', help='conv + BN + residual Sum + ReLU')
    ap.add_argument('--planes', action='store_true',
                    help='x3 only: input as bf16x3 activation planes (conv2d_bn_act_x3p)')
    ap.add_argument('--wtiled', action='store_true',
                    help='x3 only: also time chunk-tiled weights (tile | PPS_TILE_B_TILED) and '
                         'check their bits against the row-major run')
    a = ap.parse_args()
    from pps_amd import model, ops
    for name in a.layers.split(','):
        N, H, W, Cin, Cout, k, s, p = LAYERS[name]
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(N, H, W, Cin, device='cuda')
        w = np.random.RandomState(0).randn(Cout, Cin, k, k).astype(np.float32) / np.sqrt(Cin * k * k)
        wp, kpad = model.pack_conv_weight(w)
        wf = torch.from_numpy(wp).cuda()
        w3 = ops.split_bf16x3(wf)
        w3t = ops.tile_planes(w3) if a.wtiled else None
        sc = torch.ones(Cout, device='cuda')
        sh = torch.zeros(Cout, device='cuda')
        y = torch.empty(N, Ho, Wo, Cout, device='cuda')
        resid = torch.randn(N, Ho, Wo, Cout, device="cuda") if a.residual else None
        if a.planes:
            xp = ops.split_bf16x3(x.reshape(-1, Cin)).reshape(3, N, H, W, Cin)
        flops = 2.0 * N * Ho * Wo * Cout * k * k * Cin
        for math in a.math.split(','):
            wt = w3 if math == 'x3' else wf
            res = []
            def launch(tile, tiled=False):
                wl = w3t if tiled else (w3 if a.planes else wt)
                tl = tile | 0x100 if tiled else tile
                if a.planes:
                    ops.conv2d_bn_act_x3p(xp, Cin, wl, kpad, k, s, p, 1, sc, sh, resid, True, y,
                                          tile=tl)
                else:
                    ops.conv2d_bn_act(x, Cin, wl, kpad, k, s, p, 1, sc, sh, resid, True, y,
                                      tile=tl)
            for tile in [int(t) for t in a.tiles.split(',')]:
                launch(tile)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    launch(tile)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                res.append('%d:%.3f(%.0f)' % (tile, ms, flops / ms / 1e9))
                if a.wtiled and math == 'x3':
                    ref = y.clone()
                    launch(tile, True)
                    torch.cuda.synchronize()
                    same = torch.equal(ref, y)
                    e0.record()
                    for _ in range(a.reps):
                        launch(tile, True)
                    e1.record()
                    torch.cuda.synchronize()
                    mt = e0.elapsed_time(e1) / a.reps
                    res.append('t%d:%.3f%s' % (tile, mt, '' if same else '(BITS DIFFER)'))
            print('%-6s %-4s M=%d N=%d K=%d  %s' % (name, math, N * Ho * Wo, Cout, k * k * Cin,
                                                    ' '.join(res)), flush=True)


if __name__ == '__main__':
    main()
