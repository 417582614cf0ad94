"""Time one re-ranking call at Duke size (whole mirrored matrix, in place)
for library A/B runs (PPS_LIB_PATH)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))


def main():
    from pps_amd import ops
    Q, G, D = 2228, 17661, 3968
    g = torch.Generator(device='cuda')
    g.manual_seed(0)
    ids = torch.randint(0, 703, (Q + G,), generator=g, device='cuda')
    cent = torch.randn((703, D), generator=g, device='cuda')
    x = cent[ids] + 4.0 * torch.randn((Q + G, D), generator=g, device='cuda')
    x = x / x.norm(dim=1, keepdim=True)
    _, q_g, q_q, g_g = ops.self_distance_blocks(x, Q, metric='cosine')
    del x
    run = lambda: ops.re_ranking(q_g, q_q, g_g, 20, 6, 0.3, symmetric=True, whole=True)
    run()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            run()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 200.0)
    print('%s rerank %.1f us' % (os.path.basename(os.environ.get('PPS_LIB_PATH', 'in-tree')), best),
          flush=True)


if __name__ == '__main__':
    main()
