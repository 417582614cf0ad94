#!/bin/bash
# Round-6 first check: the tests this round touched, then the bench with the
# sharded legs at N = 1 (config_cuhk03 / config_1m), no e2e / Duke / CPU leg.
# Each GPU step under its own time limit, chained: stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
mkdir -p $OUT
T="${TESTS:-tests/test_gpu_h2.py tests/test_gpu_h2_model.py tests/test_gpu_h2_conv.py tests/test_gpu_native.py::test_native_plan_matches_python tests/test_gpu_retrieval.py::test_sharded_evaluator_tiled_query_planes}"
timeout -k 10 900 python -u -m pytest $T -x -v --timeout 300 --timeout-method thread \
    > $OUT/r6_pytest.log 2>&1
rc=$?
grep -E "passed|failed|PASSED|FAILED|ERROR" $OUT/r6_pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python -u bench.py --sharded-legs --no-e2e --no-duke --no-cpu-baseline \
    ${BENCH_ARGS} > $OUT/r6_bench.log 2>&1 || { tail -20 $OUT/r6_bench.log; exit 1; }
tail -1 $OUT/r6_bench.log | cut -c1-600
