#!/bin/bash
# Round-6 measurement session: the GPU suite, the profile session
# (scripts/gpu_profile.sh: bench-tune, rocprofv3 stats, PMC passes, bench
# with traffic, layer table), the Duke PMC passes.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > $OUT/r6_pytest_full.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" $OUT/r6_pytest_full.log | head; tail -2 $OUT/r6_pytest_full.log
  [ $rc -eq 0 ] || exit $rc
fi
bash scripts/gpu_profile.sh || exit 1
bash scripts/gpu_duke_pmc.sh || exit 1
