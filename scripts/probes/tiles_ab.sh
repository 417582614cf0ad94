#!/bin/bash
# Same-box A/B of tile choices: a fresh autotune vs the committed tiles file
# (profiles/r02/tiles_v4.json), alternated, each a full bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/ab
mkdir -p $OUT
rm -f $OUT/tA.json
REF=${REF:-profiles/r02/tiles_v4.json}
run() { timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2>/dev/null | tail -1 | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["config"]["act_plane_edges"],d["roofline"]["forward_graph_ms"],d["distmat_ms"])'; }
echo "fresh autotune:"; run --tiles-file $OUT/tA.json || exit 1
echo "ref tiles:";      run --tiles-file $REF || exit 1
echo "fresh tiles A:";  run --tiles-file $OUT/tA.json || exit 1
echo "ref tiles:";      run --tiles-file $REF || exit 1
echo "fresh autotune 2:"; run --tiles-file $OUT/tB.json || exit 1
