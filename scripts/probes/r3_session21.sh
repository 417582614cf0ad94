set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3.py -x -q -k "splitk" --timeout 300 --timeout-method thread > gpurun_out/sk_tests.log 2>&1; rc=$?; tail -3 gpurun_out/sk_tests.log; [ $rc -eq 0 ] || exit 1
rm -f gpurun_out/tiles_sk.json
PPS_AUTOTUNE_SPLITK=1 timeout -k 10 600 python bench.py --tiles-file gpurun_out/tiles_sk.json --no-e2e --no-cpu-baseline > gpurun_out/bench_sk_tuned.log 2>&1 || { tail -5 gpurun_out/bench_sk_tuned.log; exit 1; }
tail -1 gpurun_out/bench_sk_tuned.log | cut -c1-300
python -c "import json; d=json.load(open('gpurun_out/tiles_sk.json')); print(d['__splitk__']); print({k: v for k, v in d.items() if k in d['__splitk__']})"
for i in 1 2; do
timeout -k 10 300 python bench.py --tiles-file profiles/r03/tiles_v5.json --no-e2e --no-cpu-baseline > gpurun_out/bench_v5_$i.log 2>&1 || { tail -5 gpurun_out/bench_v5_$i.log; exit 1; }
echo "v5: $(tail -1 gpurun_out/bench_v5_$i.log | cut -c1-200)"
timeout -k 10 300 python bench.py --tiles-file gpurun_out/tiles_sk.json --no-e2e --no-cpu-baseline > gpurun_out/bench_sk_$i.log 2>&1 || { tail -5 gpurun_out/bench_sk_$i.log; exit 1; }
echo "sk: $(tail -1 gpurun_out/bench_sk_$i.log | cut -c1-200)"
done
