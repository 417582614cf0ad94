"""Per-phase shader clocks of pps_argsort_rows' workgroup 0 (a build with
-DARGSORT_CLK=1, loaded through PPS_LIB_PATH) on the Market shape."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))


def main():
    from pps_amd import ops, _lib
    Q, G = 3368, 15913
    g = torch.Generator(device='cuda')
    g.manual_seed(0)
    d = (0.6 + 0.8 * torch.rand((Q, G), generator=g, device='cuda')).contiguous()
    ops.argsort_rows(d)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 8)()
    _lib.lib().pps_debug_sort_clocks(buf)
    names = ['-', 'load wait + min/max', 'histogram', 'scan', 'scatter', 'ranks',
             'write back + big buckets', 'stream out']
    tot = sum(buf[1:])
    rows = (Q + 255) // 256
    for k in range(1, 8):
        print('%-26s %10d ticks  %5.1f %%' % (names[k], buf[k], 100.0 * buf[k] / max(tot, 1)))
    print('total %d ticks over %d rows (s_memtime ticks: 100 MHz)' % (tot, rows))


if __name__ == '__main__':
    main()
