"""Does splitting the 64-image step into S concurrent sub-batches on S HIP
streams (one hipGraph) beat one 64-image chain?  Each sub-batch runs its own
PPSModel (weights shared on the device, activations separate), so the
sub-chains' GEMM waves can fill CUs the other chain leaves idle (wave
quantisation at M = 12,288) -- at the price of smaller GEMMs.

  python scripts/stream_split_probe.py [--splits 1,2,4] [--steps 20]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--splits', default='1,2,4')
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--batch', type=int, default=64)
    a = ap.parse_args()
    import bench
    from pps_amd import model
    bench.market_cfg()
    plan = model.build_plan()
    blobs = model.synthetic_weights(plan, seed=0)
    B = a.batch
    x = torch.randn(B, 384, 128, 4, device='cuda') * 50
    x[..., 3] = 0
    feat = torch.empty(B, 3968, device='cuda')
    for S in [int(s) for s in a.splits.split(',')]:
        b = B // S
        models = [model.PPSModel(blobs) for _ in range(S)]
        xs = [x[i * b:(i + 1) * b].contiguous() for i in range(S)]
        outs = [feat[i * b:(i + 1) * b] for i in range(S)]
        for m, xi in zip(models, xs):
            m.autotune(xi)
        streams = [torch.cuda.Stream() for _ in range(S)]
        def step():
            main = torch.cuda.current_stream()
            for m, xi, o, st in zip(models, xs, outs, streams):
                st.wait_stream(main)
                with torch.cuda.stream(st):
                    o.copy_(m.forward(xi))
            for st in streams:
                main.wait_stream(st)

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            g.replay()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.steps
        print('splits %d: %.3f ms/step  %.0f img/s' % (S, ms, B / ms * 1e3), flush=True)
        del models, g


if __name__ == '__main__':
    main()
