"""One Market-shape distance matrix (3368 x 15913 x 3968) on a given tile,
for PMC passes: python scripts/dist_once.py [tile]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import ops  # noqa: E402

tile = int(sys.argv[1]) if len(sys.argv) > 1 else 0
q = torch.nn.functional.normalize(torch.randn(3368, 3968, device='cuda'), dim=1)
g = torch.nn.functional.normalize(torch.randn(15913, 3968, device='cuda'), dim=1)
idx = ops.GalleryIndex(g)
out = torch.empty(3368, 15913, device='cuda')
for _ in range(3):
    ops.compute_dist(q, idx, out=out, tile=tile)
torch.cuda.synchronize()
