"""The 31 head GEMMs at batch 64 (x [31, 64, 2048] -> [64, 31 x 128], bf16x3
weights) + the reduce / BN / ReLU / Normalize pass, per split-K factor and
tile: is the K = 2048 split of 8 (model.py HEAD_SPLITK) the right one?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import ops  # noqa: E402


def timed(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best * 1e3


def main():
    B, M, K, C = 31, 64, 2048, 128
    torch.manual_seed(0)
    x = torch.rand(B, M, K, device='cuda')
    w = ops.split_bf16x3(torch.randn(B, C, K, device='cuda') / 45.0, batched=True)
    sc = torch.ones(B * C, device='cuda')
    sh = torch.zeros(B * C, device='cuda')
    y = torch.empty(M, B * C, device='cuda')
    for s in (4, 8, 16, 32):
        part = torch.empty(s, M, B * C, device='cuda')
        res = []
        for t in (0, 36, 45, 55):
            try:
                us = timed(lambda: (ops.gemm_splitk_batched(x, w, s, part, tile=t),
                                    ops.splitk_bn_act_normalize(part, sc, sh, True, True, y)))
                res.append('t%d %.1f' % (t, us))
            except RuntimeError as e:
                res.append('t%d -' % t)
        print('splitk %2d: %s' % (s, '  '.join(res)), flush=True)


if __name__ == '__main__':
    main()
