cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/probes/rerank_debug.py > gpurun_out/rerank_debug.log 2>&1; rc=$?
tail -14 gpurun_out/rerank_debug.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_seam.py -x -q --timeout 120 --timeout-method thread > gpurun_out/seam_test.log 2>&1 || { tail -20 gpurun_out/seam_test.log; exit 1; }
tail -2 gpurun_out/seam_test.log
timeout -k 10 120 python -u scripts/probes/seam_probe.py > gpurun_out/seam_probe.log 2>&1 || exit 1
PPS_SEAM_W3=4 ONLY=res3 timeout -k 10 120 python -u scripts/probes/seam_probe.py >> gpurun_out/seam_probe.log 2>&1 || exit 1
cat gpurun_out/seam_probe.log
