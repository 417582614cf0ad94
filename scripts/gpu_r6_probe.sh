#!/bin/bash
# Layer / distance-GEMM timings of the current build (the shapes of
# scripts/gpu_r6_ablate.sh), then the GPU test suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
L=$OUT/r6_probe.log
: > $L
timeout -k 10 120 python -u scripts/probes/h2_ablate.py 1 5 3 6 >> $L 2>&1 || { tail -5 $L; exit 1; }
for cfg in "res5b h2p 52" "res4b h2p 53" "res4a h2 45" "res5c h2 45" "res3b h2 47" ${EXTRA_CFGS}; do
  echo "$cfg" >> $L
  timeout -k 10 120 python -u scripts/probes/conv_once.py $cfg >> $L 2>&1 || { tail -5 $L; exit 1; }
done
grep -v amdgpu.ids $L
[ -n "$NO_TESTS" ] && exit 0
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/r6_pytest_full.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/r6_pytest_full.log | head; tail -3 $OUT/r6_pytest_full.log
exit $rc
