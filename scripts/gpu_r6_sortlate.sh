#!/bin/bash
# Row argsort with the next row's loads issued after this row's scatter
# (the row's and the next row's values never hold registers together; the
# kernel is at the 128-VGPR cap): the argsort / CMC tests on the product,
# then interleaved timings against probe_libs/libpps_hip_head.so (the
# previous commit's rowsort.hip, made by hand, not tracked).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_retrieval.py tests/test_gpu_market_scale.py tests/test_gpu_configs.py -k "argsort or sgs or single_gallery or cmc" -x -q --timeout 300 --timeout-method thread \
    > $OUT/r6_sortlate_pytest.log 2>&1
rc=$?
tail -2 $OUT/r6_sortlate_pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Mismatch" $OUT/r6_sortlate_pytest.log | head; exit $rc; }
L=$OUT/r6_sortlate.log
: > $L
for r in 1 2; do
  for kind in uniform market; do
    for lib in "" probe_libs/libpps_hip_head.so; do
      echo "lib=${lib:-product}" >> $L
      KIND=$kind PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/argsort_probe.py >> $L 2>&1 || { tail -5 $L; exit 1; }
    done
  done
done
grep -E "lib=|argsort " $L
