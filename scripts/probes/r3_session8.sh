set -o pipefail
echo "== f32 A"; timeout -k 10 240 python scripts/probes/gemm_probe.py --layers res5b,res4b,res3b,res5a,res4a,res4c,res5c,res3a --tiles 36,48,50,52,53,56 --math x3 --wtiled || exit 1
echo "== planes A"; timeout -k 10 240 python scripts/probes/gemm_probe.py --layers res5b,res4b --tiles 52,53,56,59 --math x3 --wtiled --planes || exit 1
