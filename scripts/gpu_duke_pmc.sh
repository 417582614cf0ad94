#!/bin/bash
# PMC passes over the Duke configuration (re-ranking kernels): instruction
# mix / stall cycles, then HBM fetch.  One counter set per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/duke_pmc
rm -rf $OUT && mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $OUT/p1 -o run --output-format csv -- python3 scripts/bench_duke_rerank.py --reps 1 > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- python3 scripts/bench_duke_rerank.py --reps 1 > $OUT/p2.log 2>&1 || { tail -5 $OUT/p2.log; exit 1; }
ls -R $OUT | head -20
