#!/bin/bash
# bench two fixed tile tables A / B interleaved (no autotune): tiles_file_ab.sh A.json B.json
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --no-e2e --no-cpu-baseline --no-duke"
for r in 1 2; do
  for v in A B; do
    f=$1; [ $v = B ] && f=$2
    PPS_BENCH_LAYERS=gpurun_out/layers_$v$r.json timeout -k 10 300 $B --tiles-file $f > gpurun_out/ab_$v$r.log 2>&1 || exit $?
  done
done
