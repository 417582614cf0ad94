# Full GPU test suite, then the default bench and the Duke config bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; brc=$?
echo "bench rc=$brc"; tail -1 gpurun_out/bench.log | cut -c1-400
[ $brc -eq 0 ] || exit $brc
timeout -k 10 300 python -u scripts/bench_duke_rerank.py > gpurun_out/duke.log 2>&1 || { tail -5 gpurun_out/duke.log; exit 1; }
tail -1 gpurun_out/duke.log
exit $rc
