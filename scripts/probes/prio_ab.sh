cd $GRAFT_REPO_ROOT
T=profiles/r04/tiles_v2.json
run() { timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --tiles-file $T 2>/dev/null | tail -1 | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"],d["roofline"]["forward_graph_ms"],d["distmat_ms"],d["roofline_distmat"]["avg_launch_us"],d["gpu_clock"]["median"])'; }
for i in 1 2; do
  echo -n "base: "; run || exit 1
  echo -n "prio: "; PPS_LIB_PATH=$PWD/_variants/libpps_prio.so run || exit 1
done
