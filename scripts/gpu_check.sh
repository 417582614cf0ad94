#!/bin/bash
# One GPU session: parity tests -> bench -> rocprofv3 kernel stats.
# Stops at the first crash/timeout (exit codes >1 from pytest, any nonzero
# from bench/rocprof); plain test failures (pytest rc=1) still run the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-20}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
if [ $rc -gt 1 ]; then echo "pytest crashed/timed out; stopping"; exit $rc; fi
if [ -n "$SKIP_BENCH" ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps $STEPS > $OUT/bench.log 2>&1
brc=$?
echo "bench rc=$brc"; tail -3 $OUT/bench.log
if [ $brc -ne 0 ]; then exit $brc; fi
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o bench --output-format csv -- python3 bench.py --steps 10 --no-cpu-baseline > $OUT/prof.log 2>&1
  prc=$?
  echo "rocprof rc=$prc"; tail -3 $OUT/prof.log
  exit $prc
fi
