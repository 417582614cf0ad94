"""Per-layer roofline table of the forward's MFMA launches:
GFLOP, algorithmic MB, us, TF, fraction of the x3 roof, MFMA busy (over the
launch's trace duration at 2.4 GHz: a lower bound; no GRBM-derived clock, see
pmc_traffic.py), memory-side FETCH/WRITE MB per launch.

  python scripts/layer_table.py <layers.json (bench.py PPS_BENCH_LAYERS)> <pmcb dir> > table.md

layers.json holds the bench's per-launch HIP-event times in forward order;
pmcb/p1..p3 are the PMC passes of scripts/gpu_profile.sh (FETCH_SIZE;
WRITE_SIZE; GRBM_GUI_ACTIVE + SQ_VALU_MFMA_BUSY_CYCLES) whose last forward's
MFMA launches are matched to the layers by position."""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import epi_of, load, load_all  # noqa: E402

PEAK_X3 = 2516.8 / 6  # bf16 dense MFMA peak / 6 product terms (bench.py)
PEAK_H2 = 2516.8 / 3  # f16 dense MFMA peak / 3 product terms (PPS_TILE_H2 layers)
H2 = 0x800


def is_mfma(nm):
    return ('gemm_x3_kernel<' in nm or 'gemm_x3p_kernel<' in nm or 'gemm_x3c_kernel<' in nm or
            'gemm_ws_kernel<' in nm or 'seam_kernel<' in nm or
            ('stem_conv_pool_x3_kernel' in nm or 'stem_ring_x3_kernel' in nm)) and epi_of(nm) != 1


def main():
    layers = json.load(open(sys.argv[1]))
    d = sys.argv[2]
    gemm = [(k, v) for k, v in layers.items() if v['op'] in
            ('conv', 'conv_dual', 'heads', 'stem_pool', 'conv_pps', 'seam')]
    n = len(gemm)
    f = [v for nm, v in load(glob.glob(os.path.join(d, 'p1', '*counter_collection.csv'))[0],
                             'FETCH_SIZE') if is_mfma(nm)][-n:]
    w = [v for nm, v in load(glob.glob(os.path.join(d, 'p2', '*counter_collection.csv'))[0],
                             'WRITE_SIZE') if is_mfma(nm)][-n:]
    p3 = [r for r in load_all(glob.glob(os.path.join(d, 'p3', '*counter_collection.csv'))[0])
          if is_mfma(r[0]) and 'SQ_VALU_MFMA_BUSY_CYCLES' in r[1]][-n:]
    print('| layer | op | tile | math | GFLOP | alg. MB | us | TF | frac of its roof | frac of x3 '
          'roof | MFMA busy at 2.4 GHz | LDS conflict Mcyc | fetch MB | write MB | traffic / alg. |')
    print('|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|')
    tot = dict(fl=0.0, ms=0.0, by=0.0, tr=0.0, roof_ms=0.0)
    for i, (name, v) in enumerate(gemm):
        fl, ms, by = v['flops'], v['ms'], v['bytes']
        tf = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        fb = 2 * 1024 * f[i] if i < len(f) else float('nan')
        wb = 1024 * w[i] if i < len(w) else float('nan')
        if i < len(p3):
            nm, c, dur = p3[i]
            busy = c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0) / (1024.0 * dur * 2.4) if dur else 0.0
            lcf = c.get('SQ_LDS_BANK_CONFLICT', float('nan')) / 1e6
        else:
            busy = lcf = float('nan')
        h2 = bool(v.get('tile', 0) & H2)
        peak = PEAK_H2 if h2 else PEAK_X3
        tot['fl'] += fl
        tot['ms'] += ms
        tot['by'] += by
        tot['tr'] += fb + wb
        tot['roof_ms'] += fl / (peak * 1e12) * 1e3
        print('| %s | %s | %#x | %s | %.2f | %.1f | %.1f | %.1f | %.3f | %.3f | %.3f | %.2f | %.1f '
              '| %.1f | %.2f |' % (name, v['op'], v.get('tile', 0), 'f16x2' if h2 else 'bf16x3',
                                   fl / 1e9, by / 1e6, ms * 1e3, tf, tf / peak, tf / PEAK_X3,
                                   busy, lcf, fb / 1e6, wb / 1e6,
                                   (fb + wb) / by if by else float('nan')))
    tf = tot['fl'] / (tot['ms'] * 1e-3) / 1e12
    print('| **all %d** | | | | %.1f | %.1f | %.1f | %.1f | %.3f | %.3f | | | | | %.2f |'
          % (n, tot['fl'] / 1e9, tot['by'] / 1e6, tot['ms'] * 1e3, tf,
             tot['roof_ms'] / tot['ms'], tf / PEAK_X3, tot['tr'] / tot['by']))


if __name__ == '__main__':
    main()
