"""Duke distance stage, same box: ONE mirrored [queries; gallery]
self-distance (self_distance_blocks) vs three calls on a shared tiled
gallery index (q_g tiled GEMM + q_q and g_g mirrored self-distances).

r04, one box: whole 7.58 / 7.36 ms, three 7.33 / 7.35 ms -- a tie within
box noise; the whole matrix keeps the evaluator's q_g^T block for free
(no transpose in re-ranking), so it stays the evaluator's path."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))


def timed(fn, n=4):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    from pps_amd import ops
    Q, G, D = 2228, 17661, 3968
    x = torch.nn.functional.normalize(torch.randn(Q + G, D, device='cuda'), dim=1)
    qf, gf = x[:Q], x[Q:]

    def whole():
        return ops.self_distance_blocks(x, Q, metric='cosine')

    def three():
        gidx = ops.GalleryIndex(gf, tiled=True)
        q_g = ops.compute_dist(qf, gidx, metric='cosine', pad_rows=True, q_planes=True)
        q_q = ops.compute_dist(qf, qf, metric='cosine', pad_rows=True)
        g_g = ops.compute_dist(gf, gidx, metric='cosine', pad_rows=True)
        return q_g, q_q, g_g
    for _ in range(2):
        print('whole %.3f ms   three %.3f ms' % (timed(whole), timed(three)), flush=True)


if __name__ == '__main__':
    main()
