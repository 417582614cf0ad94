#!/bin/bash
# Probes of the f16x2 weight-stationary shapes, then the bench (autotune,
# tiles saved, per-layer times) without the CPU / e2e legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
L=$OUT/r6_ws2.log
: > $L
for cfg in ${CFGS:-"res3c h2 54" "res3c h2 45" "res4c h2 54" "res4c h2 45"}; do
  echo "$cfg" >> $L
  timeout -k 10 120 python -u scripts/probes/conv_once.py $cfg --reps 30 >> $L 2>&1 || { tail -5 $L; exit 1; }
done
grep "tile" $L
TAG=${TAG:-a}
PPS_BENCH_LAYERS=$OUT/layers_$TAG.json timeout -k 10 900 python -u bench.py --tiles-file $OUT/tiles_$TAG.json --no-cpu-baseline --no-e2e \
    > $OUT/bench_$TAG.log 2>&1 || { tail -20 $OUT/bench_$TAG.log; exit 1; }
tail -1 $OUT/bench_$TAG.log | cut -c1-700
