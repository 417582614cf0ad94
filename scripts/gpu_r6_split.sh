#!/bin/bash
# The hand-scheduled f16x2 split (h2_pair): the f16x2 conv / stem / plan
# tests (bit equality across tiles, H2P / H2E planes == in-loop split, C plan
# == twin), then layer probes and the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_h2_conv.py tests/test_gpu_h2_model.py tests/test_gpu_bench_table.py tests/test_gpu_forward.py -k "h2 or stem or bench_table or H2" -x -q --timeout 300 --timeout-method thread \
    > $OUT/r6_split_pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" $OUT/r6_split_pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
L=$OUT/r6_split.log
: > $L
for cfg in "res4a h2 45" "res5c h2 45" "res5a h2 47" "res3b h2 47" "res5b h2 52" "res4b h2 53"; do
  timeout -k 10 120 python -u scripts/probes/conv_once.py $cfg --reps 30 >> $L 2>&1 || { tail -5 $L; exit 1; }
done
timeout -k 10 120 python -u scripts/probes/dual_once.py 45 --shape res5 >> $L 2>&1 || { tail -5 $L; exit 1; }
grep -E "tile" $L
for r in 1 2; do
  timeout -k 10 600 python -u bench.py --no-e2e --no-cpu-baseline --no-duke > $OUT/r6_bench_split_$r.log 2>&1 || { tail -20 $OUT/r6_bench_split_$r.log; exit 1; }
  tail -1 $OUT/r6_bench_split_$r.log | cut -c1-200
done
