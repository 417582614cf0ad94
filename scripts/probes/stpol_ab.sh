#!/bin/bash
# Same-box A/B of the layer-output store cache policy (PPS_STPOL builds in
# _variants/): base (plain) vs nt vs sc1, one tiles table (tuned on base).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/stpol
mkdir -p $OUT
rm -f $OUT/*.json
run() { timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --tiles-file $OUT/tiles.json 2>/dev/null | tail -1 | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["roofline"]["forward_graph_ms"],d["distmat_ms"])'; }
echo -n "tune base: "; PPS_LIB_PATH=$PWD/_variants/libpps_hip_base.so run || exit 1
for i in 1 2 3; do
  for v in base pol1 pol2; do
    echo -n "$v: "; PPS_LIB_PATH=$PWD/_variants/libpps_hip_$v.so run || exit 1
  done
done
