"""HBM traffic per launch of the bench's dominant kernels from two rocprofv3
PMC passes (FETCH_SIZE, WRITE_SIZE; separate passes, --kernel-trace only):

  rocprofv3 --kernel-trace --pmc FETCH_SIZE -d <dir>/p1 -o run --output-format csv -- python3 bench.py ...
  rocprofv3 --kernel-trace --pmc WRITE_SIZE -d <dir>/p2 -o run --output-format csv -- python3 bench.py ...
  python scripts/pmc_traffic.py <dir> <math> <batch> <launches per forward> [tiles.json]
      [--clock-from <bench log>] > profiles/rNN/pmc_traffic.json

<math> is the model's base arithmetic (bench.py looks the entry up by it:
`model_math`); with the bench's tiles file the conv entry's `math` names the
arithmetic the launches actually run (f16x2 / bf16x3 launch counts).

Clock: GRBM_GUI_ACTIVE counts over the profiler's counter window, which is
longer than the kernel's trace duration (it brackets the dispatch), so
GRBM_GUI_ACTIVE / duration over-reads the clock (2.3-3.3 GHz on the round-5
layers, above the part's 2.4 GHz maximum) and is not used.  MFMA busy is
reported against the trace duration at 2.4 GHz (a lower bound on the busy
fraction) and, with --clock-from, at the DPM clock the bench sampled during
its timed loop (gpu_clock.median).

gfx950 corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE (KB) counts half of
the bytes of wide streaming reads -> x2; WRITE_SIZE (KB) is exact for 16-B
stores.  Infinity-Cache hits are counted too, so this is memory-side
traffic, an upper bound on HBM bytes.  conv = the last forward's implicit-GEMM
launches (the bench's conv_roofline forward; bf16x3 and f16x2 tiles alike),
conv_splits = that forward's f16x2 activation-split passes
(split_act_h2_kernel, PPS_TILE_H2P); distmat = the last distance launch
(gemm_h2_kernel, or gemm_x3p_kernel with EPI_DIST); rank = the last
rank_count_stream launch (the rank roofline's kernel).
"""
import csv
import glob
import json
import os
import sys


def load(path, counter):
    rows = {}
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] != counter:
            continue
        rows[int(r['Dispatch_Id'])] = (r['Kernel_Name'], float(r['Counter_Value']))
    return [rows[k] for k in sorted(rows)]


def load_all(path):
    """[(kernel name, {counter: value}, duration ns)] in dispatch order."""
    rows = {}
    for r in csv.DictReader(open(path)):
        e = rows.setdefault(int(r['Dispatch_Id']),
                            [r['Kernel_Name'], {},
                             int(r['End_Timestamp']) - int(r['Start_Timestamp'])])
        e[1][r['Counter_Name']] = float(r['Counter_Value'])
    return [tuple(rows[k]) for k in sorted(rows)]


def epi_of(name):
    if '<' not in name or 'seam_kernel<' in name:
        return 0   # the fused stem: a conv epilogue
    args = name.split('<', 1)[1].split('>', 1)[0].split(',')
    if 'gemm_ws_kernel' in name:   # <NCH, BN2, EPI, W>
        return int(args[2])
    return int(args[4])


def arith_label(tiles_file):
    """'f16x2 x N + bf16x3 x M' from the bench's tiles file (PPS_TILE_H2 =
    0x800 on a layer's tile), or None."""
    if not tiles_file:
        return None
    t = json.load(open(tiles_file))
    layers = {k: v for k, v in t.items() if not k.startswith('__') and isinstance(v, int)}
    h2 = sum(1 for v in layers.values() if v & 0x800)
    return 'f16x2 x %d + bf16x3 x %d layers (tiles file)' % (h2, len(layers) - h2)


def dpm_clock(log):
    """gpu_clock.median (MHz) of the last JSON line of a bench log, or None."""
    if not log:
        return None
    try:
        for line in reversed(open(log).read().splitlines()):
            if line.startswith('{'):
                return (json.loads(line).get('gpu_clock') or {}).get('median')
    except (OSError, ValueError):
        pass
    return None


def busy_fields(busy, dur_ns, mhz):
    out = dict(mfma_busy_frac_at_2p4GHz=round(busy / (1024.0 * dur_ns * 2.4), 4))
    if mhz:
        out.update(dpm_clock_MHz=mhz,
                   mfma_busy_frac_at_dpm_clock=round(busy / (1024.0 * dur_ns * mhz * 1e-3), 4))
    return out


def main():
    args = [a for a in sys.argv[1:]]
    clock_log = None
    if '--clock-from' in args:
        i = args.index('--clock-from')
        clock_log = args[i + 1]
        del args[i:i + 2]
    d, math, batch, nconv = args[0], args[1], int(args[2]), int(args[3])
    tiles_file = args[4] if len(args) > 4 else None
    mhz = dpm_clock(clock_log)
    fetch = load(glob.glob(os.path.join(d, 'p1', '*counter_collection.csv'))[0], 'FETCH_SIZE')
    write = load(glob.glob(os.path.join(d, 'p2', '*counter_collection.csv'))[0], 'WRITE_SIZE')
    # the x3 path launches both the register-staged and the pipelined family
    knames = ('gemm_x3_kernel', 'gemm_x3p_kernel', 'gemm_x3c_kernel', 'gemm_ws_kernel') if math == 'x3' \
        else ('gemm_f32_kernel',)

    def is_gemm(nm):   # the forward's MFMA launches (the fused stem included)
        return any(k + '<' in nm for k in knames + ('seam_kernel',)) or (
            'stem_conv_pool_x3_kernel' in nm or 'stem_ring_x3_kernel' in nm)

    def is_dist(nm):
        return 'gemm_h2_kernel<' in nm or (is_gemm(nm) and epi_of(nm) == 1)

    def is_conv(nm):
        return is_gemm(nm) and epi_of(nm) != 1
    out = dict(source='rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE (separate passes) '
                      'of bench.py; bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per launch')
    dmath = 'h2' if any('gemm_h2_kernel<' in nm for nm, _ in fetch) else math
    for key, sel, n in (('conv', is_conv, nconv), ('distmat', is_dist, 1)):
        f = [v for nm, v in fetch if sel(nm)][-n:]
        w = [v for nm, v in write if sel(nm)][-n:]
        if len(f) < n or len(w) < n:
            continue
        fb = 2 * 1024 * sum(f)
        wb = 1024 * sum(w)
        out[key] = dict(math=dmath, launches=n, fetch_bytes=fb,
                        write_bytes=wb, bytes_per_launch=round((fb + wb) / n))
        if key == 'conv':
            out[key].update(batch=batch, model_math=math,
                            math=arith_label(tiles_file) or math)
    # the activation-split passes of the same forward (those after its first conv)
    if 'conv' in out:
        idx = [i for i, (nm, _) in enumerate(fetch) if is_conv(nm)]
        if len(idx) >= nconv:
            lo, hi = idx[-nconv], idx[-1]
            fs = [v for nm, v in fetch[lo:hi] if 'split_act_h2_kernel' in nm]
            wi = [i for i, (nm, _) in enumerate(write) if is_conv(nm)]
            ws = [v for nm, v in write[wi[-nconv]:wi[-1]] if 'split_act_h2_kernel' in nm] \
                if len(wi) >= nconv else []
            if fs and len(fs) == len(ws):
                out['conv_splits'] = dict(launches=len(fs), fetch_bytes=2 * 1024 * sum(fs),
                                          write_bytes=1024 * sum(ws))
    f = [v for nm, v in fetch if 'rank_count_stream_kernel' in nm][-1:]
    w = [v for nm, v in write if 'rank_count_stream_kernel' in nm][-1:]
    if f and w:
        fb, wb = 2 * 1024 * f[0], 1024 * w[0]
        out['rank'] = dict(math=math, launches=1, fetch_bytes=fb, write_bytes=wb,
                           bytes_per_launch=round(fb + wb))
    # optional third pass: GRBM_GUI_ACTIVE + SQ_VALU_MFMA_BUSY_CYCLES -> the
    # fraction of SIMD cycles (1024 SIMDs) the MFMA pipe was busy over the
    # launches' trace durations (module docstring: no GRBM-derived clock)
    p3 = glob.glob(os.path.join(d, 'p3', '*counter_collection.csv'))
    if p3:
        rows = [(nm, c, dur) for nm, c, dur in load_all(p3[0])
                if is_conv(nm) and 'SQ_VALU_MFMA_BUSY_CYCLES' in c][-nconv:]
        if len(rows) == nconv:
            dur = sum(r[2] for r in rows)
            busy = sum(r[1].get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0) for r in rows)
            lds_cf = sum(r[1].get('SQ_LDS_BANK_CONFLICT', 0.0) for r in rows)
            out['conv_mfma'] = dict(
                math=out.get('conv', {}).get('math', math), model_math=math, batch=batch,
                launches=nconv, duration_us=round(dur / 1e3, 1),
                lds_bank_conflict_cycles_per_forward=lds_cf,
                source='rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES (third pass)',
                **busy_fields(busy, dur, mhz))
        # the same for the last distance-matrix launch (the distmat roofline's kernel)
        rows = [(nm, c, dur) for nm, c, dur in load_all(p3[0])
                if is_dist(nm) and 'SQ_VALU_MFMA_BUSY_CYCLES' in c][-1:]
        if rows:
            nm, c, dur = rows[0]
            out['distmat_mfma'] = dict(
                math=dmath, duration_us=round(dur / 1e3, 1),
                source='rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES (third pass)',
                **busy_fields(c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0.0), dur, mhz))
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
