#!/bin/bash
# Mutation check of the grouped-ties argsort rows: the library built with the
# old per-wave list append (probe_libs/libpps_hip_oldlist.so: rowsort.hip with
# a 64-lane ballot appended past a 32-entry list; made by hand, not tracked)
# must FAIL them; the product library passes them (gpu_r6_argsort_groups.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
PPS_LIB_PATH=probe_libs/libpps_hip_oldlist.so timeout -k 10 300 python -u -m pytest tests/test_gpu_retrieval.py \
    -k "argsort and (groups or market)" -v --timeout 200 --timeout-method thread > $OUT/r6_mutation.log 2>&1
echo "pytest rc=$?"
grep -E "PASSED|FAILED|Mismatched|passed|failed" $OUT/r6_mutation.log | tail -20
exit 0
