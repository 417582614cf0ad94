cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lam in 0.3 1.0 0.0; do
LAM=$lam timeout -k 10 300 python -u scripts/probes/rerank_debug.py > gpurun_out/rerank_debug_$lam.log 2>&1 || { tail -5 gpurun_out/rerank_debug_$lam.log; exit 1; }
tail -8 gpurun_out/rerank_debug_$lam.log
done
