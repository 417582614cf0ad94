#!/bin/bash
# Whole GPU suite + smoke() + top-k A/B vs the base build + one default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
BASE=$PWD/_variants/libpps_hip_base.so
for i in 1 2; do
  echo "base topk:"; PPS_LIB_PATH=$BASE timeout -k 10 200 python scripts/probes/topk_probe.py 2>/dev/null || exit 1
  echo "new topk:"; timeout -k 10 200 python scripts/probes/topk_probe.py 2>/dev/null || exit 1
done
bash scripts/probes/rank_u_ab.sh || exit 1
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
