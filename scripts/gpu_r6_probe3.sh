#!/bin/bash
# A/B probes: distance GEMM with spread DMA pieces (H2_SPREAD=1) and the
# res5 3x3 on a four-stage tile 52 (X3P_DEEP52=1), product build beside each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
L=$OUT/r6_probe3.log
: > $L
for r in 1 2; do
  for lib in "" probe_libs/libpps_hip_spread.so; do
    PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/h2_ablate.py 3 4 6 >> $L 2>&1 || { tail -5 $L; exit 1; }
  done
  for lib in "" probe_libs/libpps_hip_deep52.so; do
    echo "lib=${lib:-product}" >> $L
    PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/conv_once.py res5b h2p 52 --reps 30 >> $L 2>&1 || { tail -5 $L; exit 1; }
    PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/conv_once.py res5b h2 52 --reps 30 >> $L 2>&1 || { tail -5 $L; exit 1; }
  done
done
grep -E "tile|lib=" $L
