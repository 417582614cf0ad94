#!/bin/bash
# rank_count_stream float4-per-thread unroll (RANK_STREAM_U) variants, alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for i in 1 2 3; do
  for v in default u12 u16; do
    if [ $v = default ]; then L=""; else L=$PWD/_variants/libpps_hip_$v.so; fi
    echo -n "$v: "; PPS_LIB_PATH=$L timeout -k 10 120 python scripts/probes/rank_probe.py 2>/dev/null | tail -1 || exit 1
  done
done
