#!/bin/bash
# Tiles 54-55 (three-stage 192x64 4-wave, 128x64 8-wave):
# tile-loop GPU tests, GEMM probes, forward tuned over 1..53 vs all, alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p $OUT/s5
rm -f $OUT/s5/*.json
timeout -k 10 500 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_forward.py tests/test_gpu_retrieval.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest_s5.log 2>&1
rc=$?; tail -2 $OUT/pytest_s5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probes/gemm_probe.py --layers res5b,res5a,res3b --math x3 --tiles 36,48,29,53,54,55 2>/dev/null || exit 1
timeout -k 10 300 python scripts/probes/gemm_probe.py --layers res5b,res5b --math x3 --planes --tiles 48,53,54,55 2>/dev/null || exit 1
run() { timeout -k 10 300 python bench.py --no-cpu-baseline --tiles-file "$@" 2>/dev/null | tail -1 | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["config"]["act_plane_edges"],d["roofline"]["forward_graph_ms"],d["distmat_ms"])'; }
for i in 1 2 3; do
  echo -n "m53: "; PPS_AUTOTUNE_MAXTILE=53 run $OUT/s5/m52.json || exit 1
  echo -n "all:   "; run $OUT/s5/all.json || exit 1
done
