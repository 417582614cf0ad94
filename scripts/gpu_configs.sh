#!/bin/bash
# BASELINE configs beside the bench line, one GPU: configs[4] one 1M-gallery
# shard (10k x 125k, top-100), configs[2] Duke cosine + re-ranking, configs[3]
# CUHK03 retrieval one rank and 4 gloo ranks sharing the GPU.  Logs ->
# gpurun_out/cfg_*.log.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 400 "$@" > $OUT/cfg_$name.log 2>&1 || { tail -5 $OUT/cfg_$name.log; exit 1; }; tail -1 $OUT/cfg_$name.log | cut -c1-400; }
run shard_1m python scripts/bench_shard_1m.py
run duke_rerank python scripts/bench_duke_rerank.py
run cuhk03_n1 python scripts/bench_retrieval_sharded.py --dataset cuhk03
PPS_DIST_BACKEND=gloo run cuhk03_n4_gloo python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29517 \
  scripts/bench_retrieval_sharded.py --dataset cuhk03
