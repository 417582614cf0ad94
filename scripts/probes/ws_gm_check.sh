mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 300 --timeout-method thread -k "error_and_tiles or dual_x3" > gpurun_out/t_ws.log 2>&1 || { tail -30 gpurun_out/t_ws.log; exit 1; }
tail -2 gpurun_out/t_ws.log
timeout -k 10 200 python -u scripts/probes/gemm_probe.py --layers res2c,res3c,res4c,res2a --tiles 36,54 --math x3 --residual > gpurun_out/ws_probe.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/probes/gemm_probe.py --layers res2a,res3c --tiles 36,48,54 --math x3 >> gpurun_out/ws_probe.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ws_probe.log
for v in base gm8 gm16 gm64; do
  if [ $v = base ]; then L=""; else L=_variants/libpps_hip_$v.so; fi
  echo "== $v"
  PPS_LIB_PATH=$L TILES=42,43,44,47,52 timeout -k 10 200 python -u scripts/probes/dist_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
