#!/bin/bash
# Duke configuration (BASELINE configs[2]): timing JSON, then its per-kernel
# rocprofv3 summary -> gpurun_out/duke_prof/.  Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
mkdir -p $OUT
timeout -k 10 300 python -u scripts/bench_duke_rerank.py > $OUT/duke.log 2>&1 || { tail -5 $OUT/duke.log; exit 1; }
tail -1 $OUT/duke.log
rm -rf $OUT/duke_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/duke_prof -o duke --output-format csv -- python3 scripts/bench_duke_rerank.py --reps 2 > $OUT/duke_prof.log 2>&1 || { tail -5 $OUT/duke_prof.log; exit 1; }
f=$(ls $OUT/duke_prof/*/duke_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | cut -c1-200 | head -25
exit 0
