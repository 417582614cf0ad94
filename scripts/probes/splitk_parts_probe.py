"""Split-K anatomy on the under-filled res4/res5 shapes (batch 64): per
(layer, tile, splitk) run, the main GEMM and the partial-sum pass are
launched REPS times; run under `rocprofv3 --kernel-trace` and pass the
trace CSV to --parse to split each run's time into the two kernels
(the point: how much of split-K's cost is the separate summing pass)."""
import argparse
import csv
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

LAYERS = {'res4a': (64, 24, 8, 1024, 256, 1), 'res4b': (64, 24, 8, 256, 256, 3),
          'res4c': (64, 24, 8, 256, 1024, 1), 'res5a': (64, 24, 8, 2048, 512, 1),
          'res5b': (64, 24, 8, 512, 512, 3), 'res3a': (64, 48, 16, 512, 128, 1)}
TILES = (45, 48, 50)
SPLITS = (1, 2, 3, 4)
REPS = 20


def runs():
    for name, (N, H, W, Cin, Cout, k) in LAYERS.items():
        for tile in TILES:
            for sk in SPLITS:
                if (k * k * Cin) % (32 * sk) == 0:
                    yield name, tile, sk


def main():
    import torch
    from pps_amd import model, ops
    for name, (N, H, W, Cin, Cout, k) in LAYERS.items():
        x = torch.randn(N, H, W, Cin, device='cuda').clamp_min(0)
        w = np.random.RandomState(0).randn(Cout, Cin, k, k).astype(np.float32) / np.sqrt(Cin * k * k)
        wp, kpad = model.pack_conv_weight(w)
        w3 = ops.split_bf16x3(torch.from_numpy(wp).cuda())
        sc = torch.ones(Cout, device='cuda')
        sh = torch.zeros(Cout, device='cuda')
        res = torch.randn(N, H, W, Cout, device='cuda')
        y = torch.empty(N, H, W, Cout, device='cuda')
        part = torch.empty(4 * y.numel(), device='cuda')
        for ln, tile, sk in runs():
            if ln != name:
                continue
            for _ in range(REPS):
                ops.conv2d_bn_act_x3p(x, Cin, w3, kpad, k, 1, k // 2, 1, sc, sh, res, True, y,
                                      tile=tile, splitk=sk, part=part)
        torch.cuda.synchronize()
    print('done', flush=True)


def parse(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r['Kernel_Name']
            if 'gemm_x3p_kernel' in n or 'splitk_conv' in n:
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), n))
    rows.sort()
    i = 0
    for name, tile, sk in runs():
        nk = 1 if sk == 1 else 2
        mains, reds = [], []
        for _ in range(REPS):
            mains.append(rows[i][1] - rows[i][0])
            if nk == 2:
                reds.append(rows[i + 1][1] - rows[i + 1][0])
            i += nk
        mains, reds = sorted(mains)[2:-2], sorted(reds)[2:-2]
        m = np.mean(mains) / 1e3
        r = np.mean(reds) / 1e3 if reds else 0.0
        print('%-6s tile %2d sk %d  main %7.1f us  sum %6.1f us  total %7.1f us'
              % (name, tile, sk, m, r, m + r))
    assert i == len(rows), (i, len(rows))


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--parse', default=None)
    a = ap.parse_args()
    if a.parse:
        parse(a.parse)
    else:
        main()
