#!/bin/bash
# bench.py's N > 1 path (the driver's scaling run) rehearsed with 2 gloo ranks
# sharing this box's one GPU: barrier + max-over-ranks timing, the
# PCIe-inclusive leg, gallery-sharded retrieval.  Rank 0 prints the line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p $OUT
PPS_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 10 --warmup 2 \
  > $OUT/bench_n2_gloo.log 2>&1 || { tail -20 $OUT/bench_n2_gloo.log; exit 1; }
tail -1 $OUT/bench_n2_gloo.log | cut -c1-700
