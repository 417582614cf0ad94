#!/bin/bash
# The f16x2 tests touched by the weight-stationary tile, then an A/B of the
# bench on one box: autotune with and without the f16x2 ws candidates.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_h2_conv.py tests/test_gpu_h2_model.py \
    tests/test_gpu_native.py tests/test_gpu_bench_table.py -x -q --timeout 300 --timeout-method thread > $OUT/r6_ab_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/r6_ab_pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
for arm in ws nows ws2 nows2; do
  case $arm in nows*) export PPS_AUTOTUNE_NO_WSH2=1 ;; *) unset PPS_AUTOTUNE_NO_WSH2 ;; esac
  PPS_BENCH_LAYERS=$OUT/layers_$arm.json timeout -k 10 600 python -u bench.py --tiles-file $OUT/tiles_$arm.json \
      --no-cpu-baseline --no-e2e --no-duke > $OUT/bench_$arm.log 2>&1 || { tail -20 $OUT/bench_$arm.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/bench_$arm.log').read().splitlines()[-1]); print('$arm', d['value'], d['roofline']['forward_graph_ms'], d['gpu_clock'].get('median'))"
done
