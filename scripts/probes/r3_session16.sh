set -o pipefail
for v in base gm16 gm64 prio; do echo "== $v"; PPS_LIB_PATH=$PWD/_variants/libpps_hip_$v.so TILES=43,47,52 timeout -k 10 120 python scripts/probes/dist_tiled_probe.py || exit 1; done
for v in base prio; do echo "== conv $v"; PPS_LIB_PATH=$PWD/_variants/libpps_hip_$v.so timeout -k 10 180 python scripts/probes/gemm_probe.py --layers res5b,res4b,res3b,res5a,res4a,res4c,res5c --tiles 36,47,52,53 --math x3 || exit 1; done
