"""Probe: part power set pooling (pps_part_power_set) at batch 64 on the res5
output [64, 24, 8, 2048] (split [5,5,4,5,5], MAX_AVE): launch time and read
rate; PPS_LIB_PATH selects a build (PPS_C4 / PPS_U variants)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from pps_amd import ops  # noqa: E402

x = torch.rand(64, 24, 8, 2048, device='cuda')
out = torch.empty(31, 64, 2048, device='cuda')
split = np.array([5, 5, 4, 5, 5], np.int32)
for _ in range(3):
    ops.part_power_set(x, split, True, out)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    ops.part_power_set(x, split, True, out)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 50 * 1e3
print('%s  %.1f us  %.2f TB/s  checksum %.6f' % (os.environ.get('PPS_LIB_PATH', 'default'), us,
                                                  x.numel() * 4 / us / 1e6, out.double().sum().item()))
