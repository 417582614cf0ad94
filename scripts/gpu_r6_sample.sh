#!/bin/bash
# Row argsort: coarse-histogram sample density (probe_libs/libpps_hip_sN.so =
# PPS_SORT_SAMPLE=N builds, made by hand, not tracked; product = every 4th
# word).  Tests per library, then interleaved timings on uniform and
# Market-like rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
L=$OUT/r6_sample.log
: > $L
LIBS="probe_libs/libpps_hip_s1.so probe_libs/libpps_hip_s2.so probe_libs/libpps_hip_s3.so"
for lib in $LIBS; do
  echo "tests lib=$lib" >> $L
  PPS_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_retrieval.py -k "argsort" -q \
      --timeout 200 --timeout-method thread >> $L 2>&1 || { tail -20 $L; exit 1; }
done
for r in 1 2; do
  for kind in uniform market; do
    for lib in "" $LIBS; do
      echo "lib=${lib:-product}" >> $L
      KIND=$kind PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/argsort_probe.py >> $L 2>&1 || { tail -5 $L; exit 1; }
    done
  done
done
grep -E "lib=|argsort |passed|failed" $L
