#!/bin/bash
# PMC passes over the Duke configuration (scripts/bench_duke_rerank.py):
# FETCH_SIZE, WRITE_SIZE (separate runs, --kernel-trace only) ->
# profiles/r06/pmc_duke.json (scripts/pmc_duke.py), which the Duke leg reads
# for its roofline traffic.  Each GPU step under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/duke_pmc
R=${ROUND_DIR:-profiles/r06}
rm -rf $OUT && mkdir -p $OUT $R
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/p1 -o run --output-format csv -- python3 scripts/bench_duke_rerank.py --reps 1 > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/p2 -o run --output-format csv -- python3 scripts/bench_duke_rerank.py --reps 1 > $OUT/p2.log 2>&1 || { tail -5 $OUT/p2.log; exit 1; }
python3 scripts/pmc_duke.py $OUT ${DIST_MATH:-h2} > $R/pmc_duke.json || exit 1
cat $R/pmc_duke.json
