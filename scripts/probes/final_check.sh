#!/bin/bash
# Round-end evidence on one box: the whole GPU suite, smoke(), one default
# bench line and the Duke configuration, each step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 300 python scripts/bench_duke_rerank.py > $OUT/duke.log 2>&1 || { tail -5 $OUT/duke.log; exit 1; }
tail -1 $OUT/duke.log | cut -c1-200
bash scripts/probes/bench_n2_rehearsal.sh > $OUT/n2.log 2>&1 || { tail -5 $OUT/n2.log; exit 1; }
tail -1 $OUT/bench_n2_gloo.log | cut -c1-200
