set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -x -q -k "conv_x3_error" --timeout 240 --timeout-method thread > gpurun_out/x3c_tests.log 2>&1; rc=$?; tail -2 gpurun_out/x3c_tests.log; [ $rc -eq 0 ] || exit 1
echo "== patch probe f32"; timeout -k 10 180 python scripts/probes/gemm_probe.py --layers res2b,res3b,res4b,res5b --tiles 48,52,53,56,57,59 --math x3 || exit 1
echo "== patch probe planes"; timeout -k 10 180 python scripts/probes/gemm_probe.py --layers res3b,res4b,res5b --tiles 50,52,53,56,58,59 --math x3 --planes || exit 1
PYTEST_ARGS="--timeout 300 --timeout-method thread" STEPS=20 bash scripts/gpu_check.sh || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
