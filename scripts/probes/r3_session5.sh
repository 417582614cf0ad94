set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_retrieval.py -x -q --timeout 240 --timeout-method thread > gpurun_out/x3d_tests.log 2>&1; rc=$?; tail -2 gpurun_out/x3d_tests.log; [ $rc -eq 0 ] || exit 1
echo "== dist market"; TILES=47,60 timeout -k 10 120 python scripts/probes/dist_probe.py || exit 1
echo "== dist 1M shard"; SHAPE=10000,125000,2048 TILES=47,60 timeout -k 10 120 python scripts/probes/dist_probe.py || exit 1
