#!/bin/bash
# rank_count_stream: retrieval GPU tests, then base vs in-tree library, alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_retrieval.py tests/test_gpu_market_scale.py tests/test_gpu_configs.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest_rank.log 2>&1
rc=$?; tail -2 $OUT/pytest_rank.log; [ $rc -eq 0 ] || exit $rc
BASE=$PWD/_variants/libpps_hip_base.so
for i in 1 2 3; do
  echo -n "base: "; PPS_LIB_PATH=$BASE timeout -k 10 120 python scripts/probes/rank_probe.py 2>/dev/null | tail -1 || exit 1
  echo -n "new:  "; timeout -k 10 120 python scripts/probes/rank_probe.py 2>/dev/null | tail -1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_retrieval.py -x -q -k topk --timeout 240 --timeout-method thread > $OUT/pytest_topk.log 2>&1
rc=$?; tail -2 $OUT/pytest_topk.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  echo "base topk:"; PPS_LIB_PATH=$BASE timeout -k 10 200 python scripts/probes/topk_probe.py 2>/dev/null || exit 1
  echo "new topk:"; timeout -k 10 200 python scripts/probes/topk_probe.py 2>/dev/null || exit 1
done
