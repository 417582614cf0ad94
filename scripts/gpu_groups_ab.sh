#!/bin/bash
# A/B of the autotune's in-forward group pass (PPS_AUTOTUNE_NO_GROUPS) on one
# box, interleaved twice
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --no-e2e --no-cpu-baseline --no-duke"
for r in 1 2; do
  PPS_BENCH_LAYERS=gpurun_out/layers_grp_$r.json timeout -k 10 300 $B --tiles-file gpurun_out/tiles_grp_$r.json > gpurun_out/ab_grp_$r.log 2>&1 || exit $?
  PPS_AUTOTUNE_NO_GROUPS=1 PPS_BENCH_LAYERS=gpurun_out/layers_nogrp_$r.json timeout -k 10 300 $B > gpurun_out/ab_nogrp_$r.log 2>&1 || exit $?
done
