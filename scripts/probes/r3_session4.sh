set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_retrieval.py tests/test_gpu_x3.py -x -q --timeout 240 --timeout-method thread > gpurun_out/x3d_tests.log 2>&1; rc=$?; tail -3 gpurun_out/x3d_tests.log; [ $rc -eq 0 ] || exit 1
echo "== dist market"; TILES=42,47,52,60 timeout -k 10 120 python scripts/probes/dist_probe.py || exit 1
echo "== dist 1M shard"; SHAPE=10000,125000,2048 TILES=47,60 timeout -k 10 120 python scripts/probes/dist_probe.py || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench4.log 2>&1; tail -1 gpurun_out/bench4.log | cut -c1-200
