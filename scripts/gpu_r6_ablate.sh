#!/bin/bash
# Timing ablations of the distance GEMM (gemm_h2.hip H2_ABL) and the conv
# main loop (gemm_x3p.hip X3P_ABL): product build vs no main-loop DMA vs no
# MFMAs, on the shapes the bench runs.  Variant libraries in probe_libs/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
L=$OUT/r6_ablate.log
: > $L
for lib in "" probe_libs/libpps_hip_h2abl1.so probe_libs/libpps_hip_h2abl2.so; do
  PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/h2_ablate.py 1 5 3 6 >> $L 2>&1 || { tail -5 $L; exit 1; }
done
for lib in "" probe_libs/libpps_hip_x3pabl1.so probe_libs/libpps_hip_x3pabl2.so; do
  for cfg in "res5b h2p 52" "res4b h2p 53" "res4a h2 45" "res5c h2 45" "res3b h2 47"; do
    echo "lib=${lib:-product} $cfg" >> $L
    PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/conv_once.py $cfg >> $L 2>&1 || { tail -5 $L; exit 1; }
  done
done
cat $L
