#!/bin/bash
# Row argsort variants (probe_libs/, made by hand, not tracked): head = the
# committed single-list core, split = 5..8- and 9..16-word buckets in two
# lists (PPS_SORT_SPLIT=1), s8 = coarse histogram of every 8th word
# (PPS_SORT_SAMPLE=8), splits8 = both; product = the refactored single list.
# Each: the stable-argsort tests, then two interleaved timing rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
L=$OUT/r6_sortvar.log
: > $L
for lib in "" probe_libs/libpps_hip_head.so probe_libs/libpps_hip_split.so probe_libs/libpps_hip_s8.so probe_libs/libpps_hip_splits8.so; do
  echo "tests lib=${lib:-product}" >> $L
  PPS_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_retrieval.py -k "argsort" -q \
      --timeout 200 --timeout-method thread >> $L 2>&1 || { tail -20 $L; exit 1; }
done
for r in 1 2; do
  for lib in "" probe_libs/libpps_hip_head.so probe_libs/libpps_hip_split.so probe_libs/libpps_hip_s8.so probe_libs/libpps_hip_splits8.so; do
    echo "lib=${lib:-product}" >> $L
    PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/argsort_probe.py >> $L 2>&1 || { tail -5 $L; exit 1; }
  done
done
grep -E "lib=|argsort values|passed|failed" $L
