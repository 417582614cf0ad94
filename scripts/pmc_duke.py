"""Memory-side traffic per call of the Duke leg's two rooflined stages from
two rocprofv3 PMC passes of scripts/bench_duke_rerank.py (FETCH_SIZE,
WRITE_SIZE; separate passes, --kernel-trace only; scripts/gpu_duke_pmc.sh):

  python scripts/pmc_duke.py <dir with p1/ p2/> <dist math> > profiles/rNN/pmc_duke.json

rerank = every kernel of pps_re_ranking_ld (topk_rr_sq_kernel and the
rerank_* kernels), per call (calls counted by rerank_jaccard_kernel);
selfdist = the plane split + norms and the mirrored triangle GEMM of
ops.self_distance_blocks, per call (calls counted by the GEMM launches).
Bytes = 2 x FETCH_SIZE (gfx950 counts half of wide streaming reads) +
WRITE_SIZE, KB -> B; Infinity-Cache hits included (memory-side traffic, an
upper bound on HBM bytes)."""
import csv
import glob
import json
import os
import sys


def per_kernel(path, counter):
    out = []
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] == counter:
            out.append((int(r['Dispatch_Id']), r['Kernel_Name'], float(r['Counter_Value'])))
    return [(k, v) for _, k, v in sorted(out)]


def main():
    d, math = sys.argv[1], sys.argv[2]
    fetch = per_kernel(glob.glob(os.path.join(d, 'p1', '*counter_collection.csv'))[0], 'FETCH_SIZE')
    write = per_kernel(glob.glob(os.path.join(d, 'p2', '*counter_collection.csv'))[0], 'WRITE_SIZE')
    is_rr = lambda nm: 'rerank_' in nm or 'topk_rr_sq_kernel' in nm
    gemm = 'gemm_h2_kernel<' if math == 'h2' else 'gemm_x3p_kernel<'
    split = 'split_h2_sqnorm_kernel' if math == 'h2' else 'split_sqnorm_kernel'
    is_sd = lambda nm: gemm in nm or split in nm
    out = dict(source='rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE (separate passes) '
                      'of scripts/bench_duke_rerank.py; bytes = 2*FETCH_SIZE*1024 + '
                      'WRITE_SIZE*1024 per call', math=math)
    for key, sel, counter in (('rerank', is_rr, 'rerank_jaccard_kernel'), ('selfdist', is_sd, gemm)):
        n = sum(1 for nm, _ in fetch if counter in nm)
        nw = sum(1 for nm, _ in write if counter in nm)
        if not n or n != nw:
            continue
        fb = 2 * 1024 * sum(v for nm, v in fetch if sel(nm)) / n
        wb = 1024 * sum(v for nm, v in write if sel(nm)) / n
        out[key] = dict(calls=n, fetch_bytes=round(fb), write_bytes=round(wb),
                        bytes_per_call=round(fb + wb))
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
