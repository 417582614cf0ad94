#!/bin/bash
# A/B of PPS_TILE_H2E on one box: autotune with and without the planes-edge
# trials, interleaved twice (clock drift shows as a spread between repeats)
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --no-e2e --no-cpu-baseline --no-duke"
for r in 1 2; do
  PPS_BENCH_LAYERS=gpurun_out/layers_h2e_$r.json timeout -k 10 300 $B > gpurun_out/ab_h2e_$r.log 2>&1 || exit $?
  PPS_AUTOTUNE_NO_H2E=1 PPS_BENCH_LAYERS=gpurun_out/layers_noh2e_$r.json timeout -k 10 300 $B > gpurun_out/ab_noh2e_$r.log 2>&1 || exit $?
done
