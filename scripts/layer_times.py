"""Per-layer HIP-event timing of one PPS forward (batch 64), for tuning."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pps_amd import model  # noqa: E402


def main():
    B = int(os.environ.get('BATCH', '64'))
    bench.market_cfg()
    plan = model.build_plan()
    m = model.PPSModel(model.synthetic_weights(plan, 0))
    x = torch.randn((B, 384, 128, 4), device='cuda') * 50
    x[..., 3] = 0
    tf = os.environ.get('TILES_FILE')
    if tf:
        with open(tf) as f:
            saved = json.load(f)
        m.set_tiles(saved)
        m.set_planes(saved.get('__planes__', m.planes()))
        m.set_splitks(saved.get('__splitk__', {}))
    elif not os.environ.get('NO_AUTOTUNE'):
        rep = m.autotune(x)
        for k, (t, ts) in rep.items():
            print('%-22s tile %d  %s' % (k, t, ' '.join('%d:%.3f' % kv for kv in sorted(ts.items()))))
    for _ in range(3):
        m.forward(x)
    agg = {}
    for _ in range(5):
        t = []
        m.forward(x, timer=t)
        torch.cuda.synchronize()
        for name, op, f, e0, e1 in t:
            agg.setdefault(name, [op, f, []])[2].append(e0.elapsed_time(e1))
    tot = 0
    rows = []
    for L in m.layers:
        name = L.get('name', L['output'])
        op, f, ts = agg[name]
        ms = float(np.median(ts))
        tot += ms
        shp = ''
        if op == 'conv':
            n, ho, wo, co = m._shapes[L['output']]
            shp = 'M=%d N=%d K=%d' % (n * ho * wo, co, L['k'] * L['k'] * L['cin'])
        if L.get('planes_in') or L.get('planes_out'):
            op += '/p' + ('i' if L.get('planes_in') else '') + ('o' if L.get('planes_out') else '')
        op += ' t%d' % L.get('tile', 0) if op != 'pps' and op != 'maxpool' else ''
        if L.get('splitk', 1) > 1:
            op += 's%d' % L['splitk']
        rows.append((name, op, shp, ms, f / (ms * 1e-3) / 1e12 if f else 0))
    for r in rows:
        print('%-22s %-15s %-26s %8.3f ms %7.1f TF' % r)
    print('total %.3f ms' % tot)


if __name__ == '__main__':
    main()
