#!/bin/bash
# Tile 51 (128 x 128, 4 x 2 waves, three stages, one workgroup per CU) with
# the staggered halves (X3P_STAG51=1 variant in probe_libs/) against tile 45
# (two workgroups per CU) on the shapes tile 45 serves; then whole forwards.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
L=$OUT/r6_stag51.log
: > $L
for lib in "" probe_libs/libpps_hip_stg51.so; do
  for cfg in "res4a h2 45" "res4a h2 51" "res4c h2 45" "res4c h2 51" "res5c h2 45" "res5c h2 51"; do
    echo "lib=${lib:-product} $cfg" >> $L
    PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/conv_once.py $cfg --reps 30 >> $L 2>&1 || { tail -5 $L; exit 1; }
  done
  for t in 45 51; do
    echo "lib=${lib:-product} dual $t" >> $L
    PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/dual_once.py $t --shape res5 >> $L 2>&1 || { tail -5 $L; exit 1; }
  done
done
grep -A2 "^lib=" $L | grep -v amdgpu.ids | grep -v "^--"
for r in 1 2; do
  for lib in "" probe_libs/libpps_hip_stg51.so; do
    PPS_LIB_PATH=$lib timeout -k 10 600 python -u bench.py --no-e2e --no-cpu-baseline --no-duke \
        > $OUT/r6_stag51_$r.log 2>&1 || { tail -20 $OUT/r6_stag51_$r.log; exit 1; }
    echo "lib=${lib:-product} $(tail -1 $OUT/r6_stag51_$r.log | cut -c1-160)"
  done
done
