set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 240 --timeout-method thread 2>&1 | tail -2; [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
echo "== f32"; timeout -k 10 180 python scripts/probes/gemm_probe.py --layers res2b,res3b,res4b,res5b --tiles 48,52,53,56,57,60 --math x3 --wtiled || exit 1
echo "== planes"; timeout -k 10 180 python scripts/probes/gemm_probe.py --layers res3b,res4b,res5b --tiles 50,53,56,59,60 --math x3 --planes --wtiled || exit 1
