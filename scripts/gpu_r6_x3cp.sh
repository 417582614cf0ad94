#!/bin/bash
# Patch tiles (56-59) reading f16x2 activation planes (round 6): the planes
# == f32-input bit tests and the f16x2 plan tests, the 3x3 shapes on planes
# input per tile, then the default bench twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_h2_conv.py tests/test_gpu_h2_model.py tests/test_gpu_bench_table.py -x -q --timeout 300 --timeout-method thread \
    > $OUT/r6_x3cp_pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" $OUT/r6_x3cp_pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
L=$OUT/r6_x3cp.log
: > $L
for shape in res2b res3b res4b res5b; do
  for t in 40 47 48 52 53 56 57 58 59; do
    timeout -k 10 120 python -u scripts/probes/conv_once.py $shape h2p $t --reps 30 >> $L 2>&1 || { tail -5 $L; exit 1; }
  done
done
grep -E "tile" $L
for r in 1 2; do
  timeout -k 10 600 python -u bench.py --no-e2e --no-cpu-baseline --no-duke --tiles-file $OUT/tiles_x3cp_$r.json > $OUT/r6_bench_x3cp_$r.log 2>&1 || { tail -20 $OUT/r6_bench_x3cp_$r.log; exit 1; }
  tail -1 $OUT/r6_bench_x3cp_$r.log | cut -c1-160
  python -c "
import json; t = json.load(open('$OUT/tiles_x3cp_$r.json'))
print({k: hex(v) for k, v in t.items() if isinstance(v, int) and 56 <= (v & 0xff) <= 59})"
done
