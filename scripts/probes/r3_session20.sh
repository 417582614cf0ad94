set -o pipefail
mkdir -p gpurun_out/skp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/skp -o skp -- python3 scripts/probes/splitk_parts_probe.py > gpurun_out/skp.log 2>&1 || { tail -5 gpurun_out/skp.log; exit 1; }
f=$(ls gpurun_out/skp/*kernel_trace.csv gpurun_out/skp/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/probes/splitk_parts_probe.py --parse "$f" | tee gpurun_out/skp_table.txt
