"""Batch 64 as one forward vs two concurrent 32-image forwards on two streams
(two handles, each autotuned at 32): does running two half batches side by
side fill the CUs the under-sized layers leave idle?  Eager and hipGraph."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best


def main():
    from pps_amd import native
    nm64, blobs, imgs, x64 = bench.build_bench_model(64)
    out64 = torch.empty((64, nm64.feat_dim), device='cuda')
    halves = []
    for h in range(2):
        nm = native.NativeModel(blobs)
        xs = x64[32 * h:32 * (h + 1)]
        nm.autotune(xs, 0)
        halves.append((nm, xs, torch.empty((32, nm.feat_dim), device='cuda')))
    s = [torch.cuda.Stream(), torch.cuda.Stream()]

    def one():
        nm64.forward(x64, out=out64)

    def two():
        cur = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(cur)
        for (nm, xs, o), st in zip(halves, s):
            st.wait_event(ev)
            with torch.cuda.stream(st):
                nm.forward(xs, out=o)
        for st in s:
            e = torch.cuda.Event()
            e.record(st)
            cur.wait_event(e)

    def serial32():
        for nm, xs, o in halves:
            nm.forward(xs, out=o)

    print('eager: one 64 %.3f ms, two 32 on two streams %.3f ms, two 32 serial %.3f ms' % (
        timed(one), timed(two), timed(serial32)), flush=True)
    nm64.reserve(64)
    for nm, _, _ in halves:
        nm.reserve(32)
    g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    one()
    two()
    torch.cuda.synchronize()
    with torch.cuda.graph(g1):
        one()
    with torch.cuda.graph(g2):
        two()
    print('graph: one 64 %.3f ms, two 32 on two streams %.3f ms' % (
        timed(g1.replay), timed(g2.replay)), flush=True)
    a = torch.cat([o for _, _, o in halves])
    print('max |two - one| %.3g' % float((a - out64).abs().max()))


if __name__ == '__main__':
    main()
