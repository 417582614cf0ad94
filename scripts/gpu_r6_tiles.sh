#!/bin/bash
# Per-shape tile sweep of the mid-size 1x1 layers (f32 and planes input),
# product build and the four-stage variant (X3P_DEEP=1: tiles 51 / 53).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
L=$OUT/r6_tiles.log
: > $L
for lib in "" probe_libs/libpps_hip_deep.so; do
  for shape in res4a res4c res5c res5a; do
    for m in h2 h2p; do
      for t in ${TILES:-45 47 51 52 53 55}; do
        echo "lib=${lib:-product} $shape $m $t" >> $L
        PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/conv_once.py $shape $m $t --reps 30 >> $L 2>&1 || { tail -5 $L; exit 1; }
      done
    done
  done
done
grep -v amdgpu.ids $L | grep -v "^lib=" 
