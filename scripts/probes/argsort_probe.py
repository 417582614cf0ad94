"""Full stable row argsort (pps_argsort_rows) on the Market distance shape:
3368 x 15913 float32 distances (synthetic, the distmat's value range) ->
int32 indices (+ optional sorted values).  HBM roofline: Q*G*4 read + Q*G*4
written (+ Q*G*4 with values).  KIND=market: distances of unit features
(mostly near sqrt(2), a few close matches; argsort_phases.py's rows)
instead of uniform ones."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))


def main():
    from pps_amd import ops
    Q, G = 3368, 15913
    g = torch.Generator(device='cuda')
    g.manual_seed(0)
    if os.environ.get('KIND', 'uniform') == 'market':
        d = 1.3 + 0.08 * torch.randn((Q, G), generator=g, device='cuda')
        d[:, :20] -= 0.6
        d = d.contiguous()
    else:
        d = (0.6 + 0.8 * torch.rand((Q, G), generator=g, device='cuda')).contiguous()
    for vals in (False, True):
        for _ in range(2):
            ops.argsort_rows(d, with_values=vals)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            ops.argsort_rows(d, with_values=vals)
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 100.0
        nb = Q * G * 4 * (3 if vals else 2)
        print('argsort %s values=%s  %.1f us  %.2f TB/s  %.3f of 8 TB/s' %
              (os.environ.get('KIND', 'uniform'), vals, us, nb / us / 1e6, nb / us / 1e6 / 8.0), flush=True)
    idx = ops.argsort_rows(d)
    ref = torch.sort(d[:64], dim=1, stable=True).indices.to(torch.int32)
    assert torch.equal(idx[:64], ref)
    print('ok')


if __name__ == '__main__':
    main()
