"""Probe: shader clock inside the ring stem (diagnostic build with
-DRING_CLK=1: each workgroup writes its loop's s_memtime / s_memrealtime
deltas into y).  PPS_LIB_PATH selects the build."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', os.path.join(os.path.dirname(__file__), '..', '..')))
from pps_amd import model, ops  # noqa: E402

x = torch.randn(64, 384, 128, 4, device='cuda') * 50
x[..., 3] = 0
w = (np.random.RandomState(0).randn(64, 3, 7, 7) / np.sqrt(147)).astype(np.float32)
w3 = ops.split_bf16x3(torch.from_numpy(model.pack_stem_weight(w)).cuda())
sc = torch.ones(64, device='cuda')
sh = torch.zeros(64, device='cuda')
y = torch.empty(64, 96, 32, 64, device='cuda')
for _ in range(3):
    ops.stem_conv_pool_x3(x, w3, sc, sh, y)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    ops.stem_conv_pool_x3(x, w3, sc, sh, y)
e1.record()
torch.cuda.synchronize()
v = y.flatten()[:2 * 1024].cpu().numpy().reshape(-1, 2)
ghz = v[:, 0] / v[:, 1] * 0.1
print('us %.1f  loop clocks median %.0f  ticks median %.0f (%.1f us)  shader GHz median %.3f min %.3f max %.3f'
      % (e0.elapsed_time(e1) / 20 * 1e3, np.median(v[:, 0]), np.median(v[:, 1]),
         np.median(v[:, 1]) / 100, np.median(ghz), ghz.min(), ghz.max()))
