#!/bin/bash
# Row argsort parameter A/B: probe_libs/ builds made by hand with
# scripts/build_variant.sh, not tracked -- libpps_hip_sN.so = PPS_SORT_SAMPLE=N
# (coarse histogram of every N-th word), libpps_hip_ncN.so = PPS_SORT_NC=N
# coarse slices; LIBS picks them (default: the sample-density set).  Tests per
# library, then interleaved timings on uniform and Market-like rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
L=$OUT/r6_${TAG:-sample}.log
: > $L
LIBS=${LIBS:-"probe_libs/libpps_hip_s1.so probe_libs/libpps_hip_s2.so probe_libs/libpps_hip_s3.so"}
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
