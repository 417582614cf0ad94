set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -x -q -k "conv_x3_error" --timeout 240 --timeout-method thread > gpurun_out/x3c_tests.log 2>&1; rc=$?; tail -3 gpurun_out/x3c_tests.log; [ $rc -le 1 ] || exit $rc
echo "== patch probe f32"; timeout -k 10 180 python scripts/probes/gemm_probe.py --layers res2b,res3b,res4b,res5b --tiles 38,48,50,52,53,56,57,58 --math x3 || exit 1
echo "== patch probe planes"; timeout -k 10 180 python scripts/probes/gemm_probe.py --layers res4b,res5b --tiles 47,50,52,53,56,57,58 --math x3 --planes || exit 1
for L in base deep; do echo "== $L"; PPS_LIB_PATH=$PWD/_variants/libpps_hip_$L.so timeout -k 10 120 python scripts/probes/gemm_probe.py --layers res4a,res4c,res4b,res3a,res3c --tiles 50,51,53 --math x3 || exit 1; done
PYTEST_ARGS="--timeout 300 --timeout-method thread" STEPS=20 bash scripts/gpu_check.sh || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
VARIANTS="base pol2 ord1" ROUNDS=2 bash scripts/probes/variants_ab.sh
