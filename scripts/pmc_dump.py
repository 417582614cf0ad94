"""Dump rocprofv3 PMC passes per GEMM dispatch (scripts/pmc.sh output):
duration, raw counters and a few derived ratios.

  python scripts/pmc_dump.py [gpurun_out/pmc] [kernel-substring]
"""
import csv
import glob
import os
import sys
from collections import OrderedDict

root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/pmc'
pat = sys.argv[2] if len(sys.argv) > 2 else 'gemm'
merged = OrderedDict()
for path in sorted(glob.glob(os.path.join(root, 'p*/run_counter_collection.csv'))):
    seen = OrderedDict()
    for r in csv.DictReader(open(path)):
        if pat not in r['Kernel_Name']:
            continue
        k = int(r['Dispatch_Id'])
        e = seen.setdefault(k, dict(name=r['Kernel_Name'], ctr={},
                                    dur=int(r['End_Timestamp']) - int(r['Start_Timestamp'])))
        e['ctr'][r['Counter_Name']] = float(r['Counter_Value'])
    # dispatches are replayed in the same order in every pass: key by ordinal
    for i, e in enumerate(seen.values()):
        m = merged.setdefault(i, dict(name=e['name'], dur=e['dur'], ctr={}))
        m['ctr'].update(e['ctr'])
for i, e in merged.items():
    c = e['ctr']
    nm = e['name'].split('(')[0].replace('void pps::', '')[:60]
    dur_cyc = e['dur'] * 2.4  # ns -> cycles at 2.4 GHz nominal
    out = ['%3d %-60s %8.1fus' % (i, nm, e['dur'] / 1e3)]
    if 'SQ_VALU_MFMA_BUSY_CYCLES' in c:
        out.append('mfma_busy/SIMD %.1f%%' % (100 * c['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * dur_cyc)))
    wc = c.get('SQ_WAVE_CYCLES')
    if wc:
        for k in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_WAIT_INST_LDS'):
            if k in c:
                out.append('%s %.1f%%' % (k.replace('SQ_', '').lower(), 100 * c[k] / wc))
    if 'SQ_LDS_IDX_ACTIVE' in c and c['SQ_LDS_IDX_ACTIVE']:
        out.append('lds_conflict %.1f%%' % (100 * c.get('SQ_LDS_BANK_CONFLICT', 0) /
                                            c['SQ_LDS_IDX_ACTIVE']))
    if 'FETCH_SIZE' in c:
        out.append('fetch %.1fMB' % (2 * c['FETCH_SIZE'] / 1024))
    if 'WRITE_SIZE' in c:
        out.append('write %.1fMB' % (c['WRITE_SIZE'] / 1024))
    print('  '.join(out))
    print('      ', {k: round(v) for k, v in sorted(c.items())})
