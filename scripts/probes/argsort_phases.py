"""Phase cycle counts of pps_argsort_rows (workgroup 0, clock64 deltas summed
over its rows) on the Market distance shape; needs the PPS_SORT_PROBE
variant: scripts/build_variant.sh sortprobe rowsort -DPPS_SORT_PROBE=1, then
PPS_LIB_PATH=_variants/libpps_hip_sortprobe.so python scripts/probes/argsort_phases.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pps_amd import _lib, ops  # noqa: E402

NAMES = ['cur<-nxt', 'minmax..coarse hist', 'fine alloc', 'fine hist+scan', 'scatter',
         'networks', 'big buckets', 'out']


def main():
    Q, G = int(os.environ.get('Q', 3368)), int(os.environ.get('G', 15913))
    kind = os.environ.get('KIND', 'market')
    g = torch.Generator(device='cuda')
    g.manual_seed(0)
    if kind == 'market':
        # distances of unit features: mostly near sqrt(2), a few close matches
        d = 1.3 + 0.08 * torch.randn((Q, G), generator=g, device='cuda')
        d[:, :20] -= 0.6
    else:
        d = torch.rand((Q, G), generator=g, device='cuda')
    L = _lib.lib()
    fn = getattr(L, 'pps_sort_probe_read')
    buf = (ctypes.c_ulonglong * 16)()
    for _ in range(2):
        ops.argsort_rows(d)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.argsort_rows(d)
    e1.record()
    torch.cuda.synchronize()
    assert fn(buf) == 0
    ph = np.array(list(buf[:8]), dtype=np.float64)
    rows = (Q + 255) // 256
    print('Q %d G %d %s: %.1f us; workgroup 0 rows %d, cycles/row %.0f' %
          (Q, G, kind, e0.elapsed_time(e1) * 1e3, rows, ph.sum() / rows))
    for n, v in zip(NAMES, ph):
        print('  %-14s %8.0f cycles/row  %5.1f %%' % (n, v / rows, 100 * v / ph.sum()))


if __name__ == '__main__':
    main()
