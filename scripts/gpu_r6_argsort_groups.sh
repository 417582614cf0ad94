#!/bin/bash
# Row argsort regression: the grouped-ties rows (most buckets 5..16 words,
# per-wave lists filling several times per step) plus the other stable-
# argsort cases.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_retrieval.py -k "argsort" -v --timeout 300 --timeout-method thread \
    > $OUT/r6_argsort_groups.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/r6_argsort_groups.log | tail -20
exit $rc
