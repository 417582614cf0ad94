#!/bin/bash
# Three-stage tiles 51/52: tile-loop GPU tests, distance + GEMM probes, then
# the forward tuned with candidates 1..50 vs all (same library), alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p $OUT/s3
rm -f $OUT/s3/*.json
timeout -k 10 500 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_forward.py tests/test_gpu_retrieval.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest_s3.log 2>&1
rc=$?; tail -2 $OUT/pytest_s3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probes/dist_probe.py 2>/dev/null | grep -E "tile (4[2-9]|5[0-2])" || exit 1
timeout -k 10 300 python scripts/probes/gemm_probe.py --layers res5b,res5a,res4b --math x3 --tiles 45,47,51,52 2>/dev/null || exit 1
timeout -k 10 300 python scripts/probes/gemm_probe.py --layers res5b,res4b --math x3 --planes --tiles 45,47,50,51,52 2>/dev/null || exit 1
run() { timeout -k 10 300 python bench.py --no-cpu-baseline --tiles-file "$@" 2>/dev/null | tail -1 | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["config"]["act_plane_edges"],d["roofline"]["forward_graph_ms"],d["distmat_ms"],d["roofline_distmat"]["kernel"][-40:])'; }
for i in 1 2 3; do
  echo -n "max50: "; PPS_AUTOTUNE_MAXTILE=50 run $OUT/s3/m50.json || exit 1
  echo -n "all:   "; run $OUT/s3/all.json || exit 1
done
