set -o pipefail
for v in base vf; do echo "== $v"; PPS_LIB_PATH=$PWD/_variants/libpps_hip_$v.so timeout -k 10 180 python scripts/probes/gemm_probe.py --layers res5b,res4b,res3b,res5a,res4a,res4c,res5c,res2b --tiles 36,48,50,52,53,56 --math x3 || exit 1; done
mkdir -p gpurun_out/ab
run() { PPS_LIB_PATH=$PWD/_variants/libpps_hip_$1.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --tiles-file gpurun_out/ab/t.json 2>/dev/null | tail -1 | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["roofline"]["forward_graph_ms"],d["roofline"]["frac"],d["distmat_ms"])'; }
cp profiles/r03/tiles_v5.json gpurun_out/ab/t.json
for i in 1 2 3; do for v in base vf; do echo -n "$v: "; run $v || exit 1; done; done
