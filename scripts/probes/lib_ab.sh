#!/bin/bash
# Same-box A/B of two library builds: the baseline (_variants/libpps_hip_base.so,
# PPS_LIB_PATH) vs the in-tree one, alternated, each a full bench run with
# its own autotune (tiles saved on the first run of each, reused after).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/libab
mkdir -p $OUT
rm -f $OUT/*.json
BASE=${BASE:-$PWD/_variants/libpps_hip_base.so}
run() { timeout -k 10 300 python bench.py --no-cpu-baseline --tiles-file "$@" 2>/dev/null | tail -1 | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["config"]["act_plane_edges"],d["roofline"]["forward_graph_ms"],d["distmat_ms"])'; }
for i in 1 2 3; do
  echo -n "base: "; PPS_LIB_PATH=$BASE run $OUT/base.json || exit 1
  echo -n "new:  "; run $OUT/new.json || exit 1
done
