cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for k in market uniform; do
KIND=$k PPS_LIB_PATH=probe_libs/libpps_hip_sortprobe.so timeout -k 10 120 python -u scripts/probes/argsort_phases.py > gpurun_out/argsort_phases_$k.log 2>&1 || exit 1
cat gpurun_out/argsort_phases_$k.log
done
