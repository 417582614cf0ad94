#!/bin/bash
# Row argsort with the medium buckets batched per wave: the stable-argsort
# tests, then the Market-shape timing against the previous core
# (probe_libs/libpps_hip_rsold.so: the library linked with rowsort.hip of
# the commit before the batching; made by hand, not tracked), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_retrieval.py tests/test_gpu_market_scale.py tests/test_gpu_configs.py -k "argsort or sgs or single_gallery or cmc" -x -q --timeout 300 --timeout-method thread \
    > $OUT/r6_argsort_pytest.log 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR" $OUT/r6_argsort_pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
L=$OUT/r6_argsort.log
: > $L
for r in 1 2; do
  for lib in "" probe_libs/libpps_hip_rsold.so; do
    echo "lib=${lib:-product}" >> $L
    PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/argsort_probe.py >> $L 2>&1 || { tail -5 $L; exit 1; }
  done
done
grep -E "lib=|argsort" $L
