cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "seam or self_distance or re_ranking or rerank or duke or distributed or evaluate or rank_prepare or cmc or rank_eval or argsort" > gpurun_out/pytest_r4.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_r4.log | grep -v PASSED | head -20; tail -3 gpurun_out/pytest_r4.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/probes/seam_probe.py > gpurun_out/seam_probe.log 2>&1 || exit 1
cat gpurun_out/seam_probe.log
timeout -k 10 300 python -u scripts/probes/self_dist_probe.py > gpurun_out/self_dist_probe.log 2>&1 || exit 1
tail -5 gpurun_out/self_dist_probe.log
timeout -k 10 300 python -u scripts/bench_duke_rerank.py > gpurun_out/duke.log 2>&1 || exit 1
tail -1 gpurun_out/duke.log
