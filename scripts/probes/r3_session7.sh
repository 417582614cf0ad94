set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_retrieval.py -x -q --timeout 240 --timeout-method thread > gpurun_out/tiled_tests.log 2>&1; rc=$?; tail -3 gpurun_out/tiled_tests.log; [ $rc -eq 0 ] || exit 1
echo "== market"; TILES=47,42,52 timeout -k 10 120 python scripts/probes/dist_tiled_probe.py || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench7.log 2>&1; tail -1 gpurun_out/bench7.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["distmat_ms"],d["retrieval_ms"],json.dumps(d["roofline_distmat"]))'
