#!/bin/bash
# res2_0 fused-shortcut conv on the f16x2 tiles (ws narrow / wide), and the
# res2 3x3 on the pipelined and patch tiles (f32 input and planes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
L=$OUT/r6_probe2.log
: > $L
for t in 43 47 54; do
  timeout -k 10 120 python -u scripts/probes/dual_once.py $t --reps 30 >> $L 2>&1 || { tail -5 $L; exit 1; }
done
PPS_WS_H2_WIDE=1 timeout -k 10 120 python -u scripts/probes/dual_once.py 54 --reps 30 >> $L 2>&1 || { tail -5 $L; exit 1; }
for cfg in "res2b h2 40" "res2b h2 48" "res2b h2 57" "res2b h2 59" "res2b h2 56" "res2b h2p 40" "res2b h2p 57" "res2b h2p 59" \
           "res3b h2 47" "res3b h2 56" "res3b h2 58" "res3b h2p 47" "res3b h2p 56"; do
  timeout -k 10 120 python -u scripts/probes/conv_once.py $cfg --reps 30 >> $L 2>&1 || { tail -5 $L; exit 1; }
done
grep -E "us" $L
