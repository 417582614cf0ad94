#!/bin/bash
# Staggered chunk schedules: the h2 distance GEMM (H2_STAG_O / H2_STAG_Y:
# A blocks multiplied after the chunk barrier by the older / younger half of
# the workgroup) and the conv GEMM (X3P_STAG 1 / 2: the younger / older half
# multiplies both column halves before the barrier).  Variant libraries in
# probe_libs/ timed beside the product build; then parity tests on one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
L=$OUT/r6_stagger.log
: > $L
for r in 1 2; do
  for lib in "" probe_libs/libpps_hip_stg13.so probe_libs/libpps_hip_stg03.so probe_libs/libpps_hip_stg14.so probe_libs/libpps_hip_stg24.so probe_libs/libpps_hip_stg02.so probe_libs/libpps_hip_stg12.so; do
    PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/h2_ablate.py 3 4 6 >> $L 2>&1 || { tail -5 $L; exit 1; }
  done
  for lib in "" probe_libs/libpps_hip_stgx1.so probe_libs/libpps_hip_stgx2.so; do
    for cfg in "res5b h2p 52" "res4b h2p 53" "res4a h2 45" "res5c h2 45" "res3b h2 47" "res5a h2 47"; do
      echo "lib=${lib:-product} $cfg" >> $L
      PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/conv_once.py $cfg >> $L 2>&1 || { tail -5 $L; exit 1; }
    done
    echo "lib=${lib:-product} dual" >> $L
    PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/dual_once.py 45 --shape res5 >> $L 2>&1 || { tail -5 $L; exit 1; }
  done
done
grep tile $L | grep -v "^lib=" | sort -k3,3n -k1,1
grep -A3 "^lib=" $L | grep -v amdgpu.ids | grep -v "split pass"
PPS_LIB_PATH=${CHECK_LIB:-probe_libs/libpps_hip_stg13.so} timeout -k 10 600 python -u -m pytest tests/test_gpu_h2.py -x -q --timeout 300 --timeout-method thread > $OUT/r6_stagger_pytest.log 2>&1
rc=$?; tail -3 $OUT/r6_stagger_pytest.log; exit $rc
