"""Join rocprofv3 PMC passes (gpurun_out/pmc/p*/run_counter_collection.csv)
per dispatch and print per-layer metrics for the last forward."""
import csv
import glob
import os
import sys
from collections import OrderedDict, defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/pmc'
passes = []
for d in sorted(glob.glob(os.path.join(root, 'p*/run_counter_collection.csv'))):
    disp = OrderedDict()
    for r in csv.DictReader(open(d)):
        k = int(r['Dispatch_Id'])
        e = disp.setdefault(k, dict(name=r['Kernel_Name'], ctr={}, dur=int(r['End_Timestamp']) - int(r['Start_Timestamp']),
                                    grid=int(r['Grid_Size']), wg=int(r['Workgroup_Size']), vgpr=r['VGPR_Count'], agpr=r['Accum_VGPR_Count'], lds=r['LDS_Block_Size']))
        e['ctr'][r['Counter_Name']] = float(r['Counter_Value'])
    passes.append(list(disp.values()))
# find last forward: last maxpool kernel index in pass 0
def fwd(lst):
    idx = [i for i, e in enumerate(lst) if 'maxpool' in e['name']]
    s = idx[-1] - 1
    return lst[s:s + 58]
rows = [fwd(p) for p in passes]
names = [l.strip() for l in open(os.environ.get('LAYERS', '/dev/null'))] if os.environ.get('LAYERS') else None
hdr = '%-4s %-40s %9s %6s %6s %6s %6s %7s %8s %8s' % ('#', 'kernel', 'dur_us', 'mfma%', 'wait%', 'winst%', 'act%', 'GHz', 'fetchMB', 'writeMB')
print(hdr)
for i in range(len(rows[0])):
    c = {}
    for p in rows:
        c.update(p[i]['ctr'])
    e = rows[0][i]
    dur = e['dur'] / 1e3
    wc = c.get('SQ_WAVE_CYCLES', 0) or 1
    busy = c.get('SQ_BUSY_CYCLES', 0) or 1
    # MFMA busy: cycles over (CUs * 4 SIMDs)? report per SQ busy cycle
    mf = c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0)
    ghz = c.get('GRBM_GUI_ACTIVE', 0) / 8 / (rows[1][i]['dur'] if len(rows) > 1 else e['dur'])
    nm = e['name'].split('(')[0].replace('void pps::', '').replace('pps::', '')[:40]
    print('%-4d %-40s %9.1f %6.1f %6.1f %6.1f %6.1f %7.2f %8.1f %8.1f' % (
        i, nm, dur, 100 * mf / (busy * 4 * 256 / 32) if busy else 0,
        100 * c.get('SQ_WAIT_ANY', 0) / wc, 100 * c.get('SQ_WAIT_INST_ANY', 0) / wc,
        100 * c.get('SQ_ACTIVE_INST_ANY', 0) / wc, ghz,
        2 * c.get('FETCH_SIZE', 0) / 1024, c.get('WRITE_SIZE', 0) / 1024))
    if i < 3:
        print('     ', {k: round(v) for k, v in c.items()})
