#!/bin/bash
# GPU suite + GEMM probe of the uneven-piece tiles (47/49 with plane input,
# 50) on the res4/res5 shapes + one bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probes/gemm_probe.py --layers res4b,res5b --math x3 --planes --tiles 36,37,45,46,47,48,49,50 > $OUT/probe.log 2>&1 || { tail -5 $OUT/probe.log; exit 1; }
timeout -k 10 300 python scripts/probes/gemm_probe.py --layers res4b,res5b,res4a,res5a --math x3 --tiles 36,45,47,48,49,50 >> $OUT/probe.log 2>&1 || { tail -5 $OUT/probe.log; exit 1; }
cat $OUT/probe.log
timeout -k 10 300 python bench.py --no-cpu-baseline --tiles-file $OUT/tiles_new.json > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
