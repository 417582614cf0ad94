#!/bin/bash
# A/B: four LDS stages on tiles 51 / 53 (X3P_DEEP=1 variant library in
# probe_libs/) against the product build, whole-forward bench (autotuned
# each run), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
for r in 1 2; do
  for lib in "" probe_libs/libpps_hip_deep.so; do
    PPS_LIB_PATH=$lib timeout -k 10 600 python -u bench.py --no-e2e --no-cpu-baseline --no-duke \
        > $OUT/r6_deep_$r.log 2>&1 || { tail -20 $OUT/r6_deep_$r.log; exit 1; }
    echo "lib=${lib:-product} $(tail -1 $OUT/r6_deep_$r.log | cut -c1-160)"
  done
done
