#!/bin/bash
# A/B of the conv stack: autotune with f16x2 candidates vs without, per-layer
# times dumped (PPS_BENCH_LAYERS) for scripts/layer_times compare
set -o pipefail
mkdir -p gpurun_out
B="python -u bench.py --no-e2e --no-cpu-baseline --no-duke"
PPS_BENCH_LAYERS=gpurun_out/layers_h2.json timeout -k 10 300 $B > gpurun_out/ab_h2.log 2>&1 || exit $?
PPS_AUTOTUNE_NO_H2=1 PPS_BENCH_LAYERS=gpurun_out/layers_x3.json timeout -k 10 300 $B > gpurun_out/ab_x3.log 2>&1 || exit $?
