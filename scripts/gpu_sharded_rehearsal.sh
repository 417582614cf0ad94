#!/bin/bash
# CUHK03 config (BASELINE configs[3]) retrieval: one rank, then 4 ranks over
# gloo sharing this box's GPU (rehearsal of the 4-GPU gallery-sharded path;
# mAP/CMC must match the single rank exactly).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 300 python scripts/bench_retrieval_sharded.py --dataset cuhk03 > $OUT/cuhk03_n1.log 2>&1 || { tail -5 $OUT/cuhk03_n1.log; exit 1; }
tail -1 $OUT/cuhk03_n1.log
PPS_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29511 scripts/bench_retrieval_sharded.py --dataset cuhk03 \
  > $OUT/cuhk03_n4_gloo.log 2>&1 || { tail -5 $OUT/cuhk03_n4_gloo.log; exit 1; }
tail -1 $OUT/cuhk03_n4_gloo.log
timeout -k 10 300 python scripts/bench_retrieval_sharded.py --dataset duke > $OUT/duke_n1.log 2>&1 || { tail -5 $OUT/duke_n1.log; exit 1; }
tail -1 $OUT/duke_n1.log
