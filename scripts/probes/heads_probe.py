"""Time the 31 head GEMMs (reid_heads.py:42-79: [64 x 2048] x [2048 x 128]
per head, split-K raw partials) per tile and split, and the reduce / BN /
ReLU / Normalize pass, at batch 64."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import ops  # noqa: E402


def timed(fn, n=50):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    B, M, K, C = 31, 64, 2048, 128
    x = torch.randn(B, M, K, device='cuda').clamp_min(0)
    w = torch.randn(B, C, K, device='cuda') / 45.0
    w3 = ops.split_bf16x3(w, batched=True)  # [B][3][C][K]
    sc = torch.ones(B * C, device='cuda')
    sh = torch.zeros(B * C, device='cuda')
    y = torch.empty(M, B * C, device='cuda')
    for sk in (4, 8, 16):
        part = torch.empty(sk, M, B * C, device='cuda')
        row = []
        for t in (36, 38, 45, 51, 55):
            us = timed(lambda: ops.gemm_splitk_batched(x, w3, sk, part, tile=t))
            row.append('%d:%.1f' % (t, us))
        red = timed(lambda: ops.splitk_bn_act_normalize(part, sc, sh, True, True, y))
        print('splitk %2d  gemm us %s  reduce %.1f us' % (sk, ' '.join(row), red), flush=True)


if __name__ == '__main__':
    main()
