"""Distance-matrix tile / operand-format timing at the Market shape
(3368 x 15913 x 3968): every pipelined tile with the queries split on the fly
(f32 A) and pre-split into bf16x3 planes (q_planes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import ops  # noqa: E402


def main():
    Q, G, D = (int(v) for v in os.environ.get('SHAPE', '3368,15913,3968').split(','))
    q = torch.nn.functional.normalize(torch.randn(Q, D, device='cuda'), dim=1)
    g = torch.nn.functional.normalize(torch.randn(G, D, device='cuda'), dim=1)
    idx = ops.GalleryIndex(g)
    out = ops.dist_buffer(Q, G, 'cuda') if os.environ.get('PAD', '1') == '1' else \
        torch.empty(Q, G, device='cuda')
    flops = 2.0 * Q * G * D
    tiles = [int(t) for t in os.environ['TILES'].split(',')] if os.environ.get('TILES') else \
        range(ops.TILE_P_FIRST, ops.num_tiles() + 1)
    for tile in tiles:
        row = []
        for qp in (False, True):
            for _ in range(2):
                ops.compute_dist(q, idx, out=out, tile=tile, q_planes=qp)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                ops.compute_dist(q, idx, out=out, tile=tile, q_planes=qp)
            e1.record()
            e1.synchronize()
            ms = e0.elapsed_time(e1) / 5
            row.append('%s %.3f ms (%.0f TF)' % ('planes' if qp else 'f32A  ', ms,
                                                 flops / ms / 1e9))
        print('tile %d  %s' % (tile, '   '.join(row)), flush=True)


if __name__ == '__main__':
    main()
