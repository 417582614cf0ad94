cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "self_distance or re_ranking or rerank or duke or distributed or evaluate or rank_prepare or cmc or rank_eval or argsort" > gpurun_out/pytest_sym.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_sym.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/probes/self_dist_probe.py > gpurun_out/self_dist_probe.log 2>&1 || exit 1
cat gpurun_out/self_dist_probe.log
timeout -k 10 300 python -u scripts/bench_duke_rerank.py > gpurun_out/duke.log 2>&1 || exit 1
tail -1 gpurun_out/duke.log
