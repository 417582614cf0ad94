#!/bin/bash
# Weight-stationary 1x1 kernel, activation tiles in flight: probe_libs/ builds
# made by hand with scripts/build_variant.sh from a gemm_ws.hip whose PD
# took a WS_PD_ADD define (not kept, not tracked) -- pdA = WS_PD_ADD=1 on every kernel without a residual / dual input, pdB = the
# same for K <= 128 only.  res2_1_branch2a (K = 256) and res2_0_branch2a
# (K = 64), f16x2 on tile 54, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
L=$OUT/r6_wspd.log
: > $L
for r in 1 2 3; do
  for lib in "" probe_libs/libpps_hip_pdA.so probe_libs/libpps_hip_pdB.so; do
    echo "lib=${lib:-product}" >> $L
    for sh in res2a res2a0; do
      PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/conv_once.py $sh h2 54 --reps 50 >> $L 2>&1 || { tail -5 $L; exit 1; }
    done
  done
done
cat $L | grep -v amdgpu.ids
