set -o pipefail
mkdir -p gpurun_out
echo "== heads"; timeout -k 10 120 python scripts/probes/heads_probe.py || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_native.py -x -q --timeout 240 --timeout-method thread > gpurun_out/native_tests.log 2>&1; rc=$?; tail -2 gpurun_out/native_tests.log; [ $rc -le 1 ] || exit $rc
bash scripts/gpu_profile.sh
