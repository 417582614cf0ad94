#!/bin/bash
# Round-6 check: the f16x2 stem, the staggered tiles (52, three-stage h2
# distance tiles), the plans that use them; then the default bench twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
T="${TESTS:-tests/test_gpu_forward.py tests/test_gpu_h2_model.py tests/test_gpu_h2.py tests/test_gpu_h2_conv.py tests/test_gpu_bench_table.py tests/test_gpu_native.py}"
timeout -k 10 900 python -u -m pytest $T -x -q --timeout 300 --timeout-method thread \
    > $OUT/r6_check2.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" $OUT/r6_check2.log | tail -5
[ $rc -eq 0 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
for r in 1 2; do
  timeout -k 10 600 python -u bench.py --no-e2e --no-cpu-baseline --tiles-file $OUT/tiles_c2_$r.json \
      > $OUT/r6_bench_c2_$r.log 2>&1 || { tail -20 $OUT/r6_bench_c2_$r.log; exit 1; }
  tail -1 $OUT/r6_bench_c2_$r.log | cut -c1-330
  python -c "import json; t=json.load(open('$OUT/tiles_c2_$r.json')); print('stem', t.get('conv1'))"
done
