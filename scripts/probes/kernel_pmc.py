"""Average rocprofv3 PMC counters per kernel (name substring) over the
dispatches of every pass directory under ROOT, and derive clock, MFMA busy
and wait fractions:  python scripts/probes/kernel_pmc.py ROOT SUBSTR [SKIP]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root, sub = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    ctr = defaultdict(list)
    durs = []
    for f in sorted(glob.glob(os.path.join(root, '*', '*counter_collection.csv'))):
        disp = {}
        for r in csv.DictReader(open(f)):
            if sub not in r['Kernel_Name']:
                continue
            k = int(r['Dispatch_Id'])
            e = disp.setdefault(k, dict(dur=int(r['End_Timestamp']) - int(r['Start_Timestamp']),
                                        c={}))
            e['c'][r['Counter_Name']] = float(r['Counter_Value'])
        for k in sorted(disp)[skip:]:
            durs.append(disp[k]['dur'])
            for n, v in disp[k]['c'].items():
                ctr[n].append((v, disp[k]['dur']))
    if not durs:
        print('no dispatch of', sub)
        return
    avg = {n: sum(v for v, _ in l) / len(l) for n, l in ctr.items()}
    dur = sum(durs) / len(durs)
    print('%s: %d dispatches, avg %.1f us' % (sub, len(durs), dur / 1e3))
    for n in sorted(avg):
        print('  %-28s %.4g' % (n, avg[n]))
    if 'GRBM_GUI_ACTIVE' in ctr:
        l = ctr['GRBM_GUI_ACTIVE']
        act = sum(v for v, _ in l) / len(l) / 8.0
        d = sum(t for _, t in l) / len(l)
        print('  clock %.3f GHz' % (act / d))
        if 'SQ_VALU_MFMA_BUSY_CYCLES' in avg:
            print('  MFMA busy %.3f of SIMD cycles (%.3f at 2.4 GHz)' % (
                avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * act),
                avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * d * 2.4)))
    wc = avg.get('SQ_WAVE_CYCLES')
    if wc:
        for n in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_WAIT_INST_LDS',
                  'SQ_ACTIVE_INST_MFMA' if False else 'SQ_ACTIVE_INST_VALU'):
            if n in avg:
                print('  %s / WAVE_CYCLES %.3f' % (n, avg[n] / wc))
    if 'FETCH_SIZE' in avg:
        print('  FETCH_SIZE x2 = %.1f MB per launch' % (2 * avg['FETCH_SIZE'] / 1024))
    if 'WRITE_SIZE' in avg:
        print('  WRITE_SIZE = %.1f MB per launch' % (avg['WRITE_SIZE'] / 1024))


if __name__ == '__main__':
    main()
