#!/bin/bash
# Evaluate every epoch snapshot of a PPS training run, as the reference's
# scripts/test_reid.sh:51-55 does (ITER = 1, 11, ..., 171), on MI355X.
#   scripts/test_reid.sh <cfg.yaml> <snapshot_dir> [NUM_GPUS]
set -e
CFG=$1
SNAP=$2
NGPU=${3:-1}
cd "$(dirname "$0")/.."
for ITER in $(seq 1 10 171); do
  W=$SNAP/model_epoch${ITER}.npz
  [ -f "$W" ] || continue
  if [ "$NGPU" -gt 1 ]; then
    python -m torch.distributed.run --nnodes=1 --nproc-per-node $NGPU \
      --master-addr 127.0.0.1 --master-port 29511 \
      tools/test_net.py --cfg $CFG --multi-gpu-testing --wait False TEST.WEIGHTS $W
  else
    python tools/test_net.py --cfg $CFG --wait False TEST.WEIGHTS $W
  fi
done
