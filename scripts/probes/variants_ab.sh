#!/bin/bash
# Same-box A/B of library builds in _variants/ (libpps_hip_<name>.so),
# alternated ROUNDS times on one tiles table tuned on the first variant:
#   VARIANTS="base ord1 ord2" bash scripts/probes/variants_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/ab
mkdir -p $OUT
rm -f $OUT/tiles.json
VARIANTS=${VARIANTS:-base}
ROUNDS=${ROUNDS:-3}
first=${VARIANTS%% *}
run() { timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --tiles-file $OUT/tiles.json 2>/dev/null | tail -1 | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["roofline"]["forward_graph_ms"],d["distmat_ms"])'; }
echo -n "tune $first: "; PPS_LIB_PATH=$PWD/_variants/libpps_hip_$first.so run || exit 1
for i in $(seq $ROUNDS); do
  for v in $VARIANTS; do
    echo -n "$v: "; PPS_LIB_PATH=$PWD/_variants/libpps_hip_$v.so run || exit 1
  done
done
