#!/bin/bash
# Round-end rehearsal on the final build: the GPU suite, smoke(), and the
# driver's bench command (all legs: e2e, Duke, CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/r6_final_pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/r6_final_pytest.log | head; tail -2 $OUT/r6_final_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/r6_final_smoke.log 2>&1 || { tail -5 $OUT/r6_final_smoke.log; exit 1; }
tail -2 $OUT/r6_final_smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/r6_final_bench.log 2>&1 || { tail -10 $OUT/r6_final_bench.log; exit 1; }
tail -1 $OUT/r6_final_bench.log | cut -c1-300
