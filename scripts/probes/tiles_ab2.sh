# same-box A/B of two committed tiles tables (no autotune): img/s, forward ms
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/tab
run() { cp "$1" gpurun_out/tab/t.json; timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --tiles-file gpurun_out/tab/t.json 2>/dev/null | tail -1 | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["roofline"]["forward_graph_ms"],d["roofline"]["frac"])'; }
for i in 1 2 3; do
  for t in $TABLES; do echo -n "$t: "; run $t || exit 1; done
done
