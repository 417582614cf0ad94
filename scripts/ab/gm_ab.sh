#!/bin/bash
# distance GEMM grouped-order size (X3P_GM_MB) A/B: in-tree (32 MB) vs variants
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  TILES=6,7 timeout -k 10 120 python -u scripts/probes/dist_tiles_time.py >> gpurun_out/gm_ab.log 2>&1 || exit $?
  for g in 8 16 64 128; do
    PPS_LIB_PATH=$PWD/pps_amd/variant_gm$g.so TILES=6,7 timeout -k 10 120 python -u scripts/probes/dist_tiles_time.py >> gpurun_out/gm_ab.log 2>&1 || exit $?
  done
done
