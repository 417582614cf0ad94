set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python bench.py --no-e2e --no-cpu-baseline > gpurun_out/fin4_$i.log 2>&1 || { tail -5 gpurun_out/fin4_$i.log; exit 1; }
echo "fin4: $(tail -1 gpurun_out/fin4_$i.log | cut -c90-130)"
PPS_LIB_PATH=_variants/libpps_hip_fin7.so timeout -k 10 300 python bench.py --no-e2e --no-cpu-baseline > gpurun_out/fin7_$i.log 2>&1 || { tail -5 gpurun_out/fin7_$i.log; exit 1; }
echo "fin7: $(tail -1 gpurun_out/fin7_$i.log | cut -c90-130)"
done
