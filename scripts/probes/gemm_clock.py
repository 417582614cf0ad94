"""Probe: shader clock inside the pipelined x3 GEMM (diagnostic build with
-DX3P_CLK=1, scripts/build_variant.sh; PPS_LIB_PATH selects it).  Per layer
and tile: launch time, median in-kernel clock (s_memtime / s_memrealtime x
100 MHz over the workgroups of the last launch) and the MFMA issue share of
the launch's cycles at that clock (6 x M N K / 512 MAC per cycle per SIMD,
1024 SIMDs).

  PPS_LIB_PATH=_variants/libpps_hip_clk.so python scripts/probes/gemm_clock.py res5b:43,res4b:36
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..'))
from pps_amd import _lib, model, ops  # noqa: E402
from gemm_probe import LAYERS  # noqa: E402


def main():
    spec = sys.argv[1] if len(sys.argv) > 1 else 'res5b:43,res4b:36,res3b:42,res2b:40,big3x3:42'
    lib = _lib.lib()
    fn = lib.pps_debug_x3p_clocks
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for item in spec.split(','):
        name, tile = item.split(':')
        tile = int(tile)
        N, H, W, Cin, Cout, k, s, p = LAYERS[name]
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(N, H, W, Cin, device='cuda')
        w = np.random.RandomState(0).randn(Cout, Cin, k, k).astype(np.float32) / np.sqrt(Cin * k * k)
        wp, kpad = model.pack_conv_weight(w)
        w3 = ops.split_bf16x3(torch.from_numpy(wp).cuda())
        sc = torch.ones(Cout, device='cuda')
        sh = torch.zeros(Cout, device='cuda')
        y = torch.empty(N, Ho, Wo, Cout, device='cuda')
        M, K = N * Ho * Wo, k * k * Cin
        run = lambda: ops.conv2d_bn_act(x, Cin, w3, kpad, k, s, p, 1, sc, sh, None, True, y,  # noqa: E731
                                        tile=tile)
        for _ in range(200):   # ~steady clock before the timed launches
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        buf = np.zeros(2 * 65536, np.float32)
        assert fn(buf.ctypes.data, buf.size) == 0
        v = buf.reshape(-1, 2)
        v = v[v[:, 1] > 0]
        ghz = np.median(v[:, 0] / v[:, 1] * 0.1)
        mfma_cycles = 6.0 * M * Cout * K / 512 / 1024
        print('%-7s tile %2d  M=%d N=%d K=%d  %.1f us  clock %.3f GHz  MFMA issue %.0f %% of '
              'cycles at that clock (%.0f %% at 2.4 GHz)' % (
                  name, tile, M, Cout, K, us, ghz, 100 * mfma_cycles / (us * 1e3 * ghz),
                  100 * mfma_cycles / (us * 1e3 * 2.4)), flush=True)


if __name__ == '__main__':
    main()
