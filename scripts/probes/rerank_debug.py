"""Debug: the in-place re-ranking path vs the dense OD path on the same
symmetric inputs -- compare the workspace intermediates region by region."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import evaluator as ev  # noqa: E402
from pps_amd import ops, _lib  # noqa: E402
from pps_amd._lib import call  # noqa: E402


def main():
    Q, G, D = 1000, 15500, 64
    rng = np.random.RandomState(7)
    f = rng.randn(Q + G, D).astype(np.float32)
    f /= np.linalg.norm(f, axis=1, keepdims=True)
    qg = ev.compute_dist(f[:Q], f[Q:])
    sym = lambda d: np.triu(d) + np.triu(d, 1).T
    qq = sym(ev.compute_dist(f[:Q], f[:Q]))
    gg = sym(ev.compute_dist(f[Q:], f[Q:]))
    dev = [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (qg, qq, gg)]
    k1, k2 = 20, 6
    N = Q + G
    nbytes = _lib.lib().pps_rerank_workspace_bytes(Q, G, k1, k2)
    outs, wss = [], []
    lam = float(os.environ.get('LAM', '0.3'))
    for flags in (1, 0, 1):
        ws = torch.zeros((int(nbytes),), dtype=torch.uint8, device='cuda')
        out = torch.empty((Q, G), device='cuda')
        call('pps_re_ranking_ld', dev[0].data_ptr(), G, dev[1].data_ptr(), Q, dev[2].data_ptr(), G,
             Q, G, k1, k2, lam, flags, ws.data_ptr(), int(nbytes), out.data_ptr(),
             torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy())
        wss.append(ws.cpu().numpy())
    r = lambda b: (b + 255) // 256 * 256
    ldo = (N + 3) // 4 * 4
    K1 = k1 + 1
    off = r(4 * N * ldo)
    regions = []
    for name, nb, dt in (('colmax', 4 * N, np.float32), ('topv', 4 * N * K1, np.float32),
                         ('rank', 4 * N * K1, np.int32), ('v_idx', 4 * N * 256, np.int32),
                         ('v_val', 4 * N * 256, np.float32), ('v_cnt', 4 * N, np.int32),
                         ('q_idx', 4 * N * 1536, np.int32), ('q_val', 4 * N * 1536, np.float32),
                         ('q_cnt', 4 * N, np.int32)):
        regions.append((name, off, nb, dt))
        off += r(nb)
    for name, o, nb, dt in regions:
        a = wss[0][o:o + nb].view(dt)
        b = wss[1][o:o + nb].view(dt)
        diff = np.nonzero(a != b)[0]
        print('%-7s differ at %d of %d' % (name, len(diff), a.size), diff[:5],
              a[diff[:5]] if len(diff) else '', b[diff[:5]] if len(diff) else '', flush=True)
    rank_a = wss[0][regions[2][1]:regions[2][1] + 4 * N * K1].view(np.int32).reshape(N, K1)
    rank_b = wss[1][regions[2][1]:regions[2][1] + 4 * N * K1].view(np.int32).reshape(N, K1)
    rows = np.nonzero((rank_a != rank_b).any(1))[0]
    print('rows with different ranks:', len(rows), rows[:10])
    if len(rows):
        i = rows[0]
        print('row', i, 'inplace', rank_a[i], '\ndense  ', rank_b[i])
    d = np.abs(outs[0] - outs[1])
    print('lambda', lam, 'out max diff', d.max(), 'count', int((d > 0).sum()))
    d2 = np.abs(outs[0] - outs[2])
    print('in-place run to run: max diff', d2.max(), 'count', int((d2 > 0).sum()))
    ref = ev.re_ranking_sparse(qg, qq, gg, k1=k1, k2=k2, lambda_value=lam)
    for nm, o in (('inplace', outs[0]), ('dense', outs[1])):
        e = np.abs(o - ref)
        print(nm, 'vs oracle max', e.max(), 'exact', int((e == 0).sum()), 'of', e.size)


if __name__ == '__main__':
    main()
