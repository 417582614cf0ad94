cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; brc=$?
echo "bench rc=$brc"; tail -1 gpurun_out/bench.log | cut -c1-600
exit $brc
