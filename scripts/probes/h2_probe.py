"""f16x2 ("h2") distance GEMM vs the bf16x3 kernel: parity at Market size
(vs the oracle's NumPy compute_dist; near-tie flips counted as in
tests/_parity.py) and timing of every h2 tile against the x3 default, in
interleaved rounds on one process; then the Duke self-distance both ways."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from pps_amd import ops  # noqa: E402

Q, G, D = 3368, 15913, 3968


def feats(seed=0):
    rng = np.random.RandomState(seed)
    qid = rng.randint(1, 751, Q)
    gid = np.concatenate([rng.randint(1, 751, G - 2793), np.zeros(2793, int)])
    cent = rng.randn(751, D).astype(np.float32)
    f = cent[np.concatenate([qid, gid])] + 4.0 * rng.randn(Q + G, D).astype(np.float32)
    f /= np.linalg.norm(f, axis=1, keepdims=True)
    return f.astype(np.float32)


def timed(fn, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    f = feats()
    qf = torch.from_numpy(f[:Q]).cuda()
    gf = torch.from_numpy(f[Q:]).cuda()
    t0 = time.time()
    ref = (np.sum(f[:Q] ** 2, 1)[:, None] + np.sum(f[Q:] ** 2, 1)[None] -
           2 * f[:Q] @ f[Q:].T)
    ref = np.sqrt(np.maximum(ref, 0)).astype(np.float32)
    print('oracle %.1f s' % (time.time() - t0), flush=True)
    from _parity import check_topk, tie_eps
    order = np.argsort(ref, axis=1, kind='stable')[:, :100]
    for math in ('x3', 'h2'):
        d = ops.compute_dist(qf, gf, math=math)
        dn = d.cpu().numpy()
        err = float(np.abs(dn - ref).max())
        eps = tie_eps(dn, ref)
        _, idx = ops.topk(d, 100)
        flips = check_topk(idx.cpu().numpy(), ref, 100, eps, order)
        print('%s: max err %.3g, eps %.3g, top-100 flips %d' % (math, err, eps, flips), flush=True)
    d3 = ops.compute_dist(qf, gf, math='x3').cpu().numpy()
    d2 = ops.compute_dist(qf, gf, math='h2').cpu().numpy()
    print('h2 vs x3 max diff %.3g' % float(np.abs(d3 - d2).max()), flush=True)
    # cosine and sqeuclidean, a few tiles, bits equal across tiles
    for metric in ('sqeuclidean', 'cosine'):
        base = None
        for t in range(ops.h2_num_tiles()):
            d = ops.compute_dist(qf, gf, math='h2', metric=metric, tile=t).cpu().numpy()
            if base is None:
                base = d
            assert np.array_equal(base, d), (metric, t)
        print('%s: all h2 tiles bit-identical' % metric, flush=True)

    # timing: GEMM alone, index + query split prepared once
    gidx3 = ops.GalleryIndex(gf, tiled=True, math='x3')
    qt, qsq = ops.split_sqnorm_tiled(qf)
    gidx2 = ops.GalleryIndex(gf, math='h2')
    q2, qrs, qsq2 = ops.split_h2_tiled(qf)
    out = ops.dist_buffer(Q, G, 'cuda')
    arms = {'x3_t43': lambda: ops.distmat_planes(None, qsq, gidx3, out, tile=43, q_tiled=qt, Q=Q,
                                                 D=D)}
    for t in range(1, ops.h2_num_tiles()):
        arms['h2_t%d' % t] = (lambda t=t: ops.distmat_h2(q2, qrs, qsq2, gidx2, out, tile=t))
    for a in arms.values():
        a()
    torch.cuda.synchronize()
    res = {k: [] for k in arms}
    for _ in range(4):
        for k, a in arms.items():
            res[k].append(timed(a, 10))
    flops = 2.0 * Q * G * D
    for k, v in res.items():
        ms = min(v)
        print('%-8s min %.3f ms  med %.3f ms  %.1f f32-TF' % (k, ms, float(np.median(v)),
                                                           flops / ms / 1e9), flush=True)
    # split cost
    print('split h2 (gallery) %.3f ms, split x3 tiled %.3f ms' % (
        timed(lambda: ops.split_h2_tiled(gf), 5), timed(lambda: ops.split_sqnorm_tiled(gf), 5)))

    # Duke self-distance (N = 19889, cosine)
    N = 2228 + 17661
    x = torch.randn((N, D), device='cuda')
    x = (x / x.norm(dim=1, keepdim=True)).contiguous()
    m3 = ops.dist_buffer(N, N, 'cuda')
    x3t, xsq = ops.split_sqnorm_tiled(x)
    x2, xrs, xsq2 = ops.split_h2_tiled(x)
    arms = {'x3_self_t43': lambda: ops.call('pps_distmat_x3_self_tiled', x3t.data_ptr(), N,
                                            xsq.data_ptr(), D, 2, m3.data_ptr(), m3.stride(0), 0,
                                            ops._stream())}
    for t in range(1, ops.h2_num_tiles()):
        arms['h2_self_t%d' % t] = (lambda t=t: ops.call(
            'pps_distmat_h2_self_tiled', x2.data_ptr(), N, xsq2.data_ptr(), xrs.data_ptr(), D, 2,
            m3.data_ptr(), m3.stride(0), t, ops._stream()))
    for a in arms.values():
        a()
    torch.cuda.synchronize()
    res = {k: [] for k in arms}
    for _ in range(3):
        for k, a in arms.items():
            res[k].append(timed(a, 3))
    for k, v in res.items():
        print('%-12s min %.3f ms  med %.3f ms' % (k, min(v), float(np.median(v))), flush=True)
    # symmetric and equal to the full product's upper triangle on a sample
    arms['h2_self_t1']()
    full = ops.compute_dist(x[:512], x, math='h2', metric='cosine', symmetric=False)
    s = m3[:512].cpu().numpy()
    fu = full.cpu().numpy()
    iu = np.triu_indices(512, 0, N)
    print('self upper == full:', bool(np.array_equal(s[iu], fu[iu])),
          ' symmetric:', bool(np.array_equal(m3[:512, :512].cpu().numpy(),
                                             m3[:512, :512].cpu().numpy().T)), flush=True)


if __name__ == '__main__':
    main()
