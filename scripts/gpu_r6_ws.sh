#!/bin/bash
# f16x2 weight-stationary tile (54 | PPS_TILE_H2): the h2 conv tests, then
# per-shape timings of tile 54 against the pipelined picks, then the
# three/four-stage sweep of the mid-size 1x1 shapes (probe_libs/ variant).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_h2_conv.py tests/test_gpu_h2_model.py \
    tests/test_gpu_native.py -x -q --timeout 300 --timeout-method thread > $OUT/r6_ws_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/r6_ws_pytest.log | tail -5
[ $rc -eq 0 ] || exit $rc
L=$OUT/r6_ws.log
: > $L
for cfg in "res2c h2 54" "res2c h2 43" "res2a h2 54" "res2a h2 48" "res3c h2 54" "res3c h2 45" \
           "res4c h2 54" "res4c h2 45" "res2c x3 54"; do
  echo "$cfg" >> $L
  timeout -k 10 120 python -u scripts/probes/conv_once.py $cfg --reps 30 >> $L 2>&1 || { tail -5 $L; exit 1; }
done
for lib in "" probe_libs/libpps_hip_deep.so; do
  for shape in res4a res5c res5a res3a; do
    for t in 45 51 52 53; do
      echo "lib=${lib:-product} $shape h2 $t" >> $L
      PPS_LIB_PATH=$lib timeout -k 10 120 python -u scripts/probes/conv_once.py $shape h2 $t --reps 30 >> $L 2>&1 || { tail -5 $L; exit 1; }
    done
  done
done
grep -v amdgpu.ids $L | grep -v "^lib=\|^res[0-9][a-z] "
