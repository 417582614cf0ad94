#!/bin/bash
# Evaluate every epoch snapshot of a PPS training run on MI355X, with the
# reference's calling convention (scripts/test_reid.sh:7-55):
#
#   scripts/test_reid.sh ARGS... <snapshot_dir>
#
# ARGS are tools/test_net.py arguments (--cfg X, KEY VALUE overrides); the
# value after OUTPUT_DIR names the experiment directory, and the output is
# tee'd into "${EXP_DIR}/../_logs/<basename> test_reid.sh <args> <date>.log".
# For ITER = 1, 11, ..., 171 the snapshot <snapshot_dir>/model_epoch${ITER}.pkl
# is tested with --multi-gpu-testing (one process per GPU; NUM_GPUS from the
# ARGS, default 1).  A Detectron .pkl is a pickle: it is only read when the
# caller declares the snapshots trusted with PPS_TRUSTED_WEIGHTS=1 (then
# --trusted-weights is passed); a converted model_epoch${ITER}.npz
# (tools/convert_weights.py) next to it is used without that.
set -e
export PYTHONUNBUFFERED="True"

array=( "$@" )
len=${#array[@]}
if [ "$len" -lt 1 ]; then
  echo "usage: $0 ARGS... <snapshot_dir>" >&2
  exit 2
fi
ARGS=( "${array[@]:0:$len-1}" )
ARGS_SLUG="${ARGS[*]}"
ARGS_SLUG=${ARGS_SLUG//\//_}
LAST_ARG=${array[$len-1]}

EXP_DIR=""
NGPU=1
is_next=""
for var in "${ARGS[@]}"; do
  case "$is_next" in
    out) EXP_DIR=$var ;;
    ngpu) NGPU=$var ;;
  esac
  is_next=""
  [ "$var" == "OUTPUT_DIR" ] && is_next=out
  [ "$var" == "NUM_GPUS" ] && is_next=ngpu
done
EXP_DIR=${EXP_DIR:-./output}

mkdir -p "${EXP_DIR}"
mkdir -p "${EXP_DIR}/../_logs"
BASENAME=$(basename "${EXP_DIR}")
LOG="${EXP_DIR}/../_logs/${BASENAME} ${0##*/} ${ARGS_SLUG} $(date +'%Y-%m-%d_%H-%M-%S').log"
exec &> >(tee -a "$LOG")
echo Logging output to "$LOG"
echo ---------------------------------------------------------------------
git -C "$(dirname "$0")/.." log -1 2>/dev/null || true
echo ---------------------------------------------------------------------

ROOT="$(cd "$(dirname "$0")/.." && pwd)"
RUN=""
[ "${PPS_DRY_RUN:-0}" == "1" ] && RUN=echo   # print the commands only (tests)
ITERS=180
for ((ITER = 1; ITER <= ITERS; ITER = ITER + 10)); do
  PKL=${LAST_ARG}/model_epoch${ITER}.pkl
  NPZ=${LAST_ARG}/model_epoch${ITER}.npz
  EXTRA=()
  if [ -f "$NPZ" ]; then
    W=$NPZ
  elif [ -f "$PKL" ]; then
    if [ "${PPS_TRUSTED_WEIGHTS:-0}" != "1" ]; then
      echo "ERROR: $PKL is a pickle; set PPS_TRUSTED_WEIGHTS=1 if the snapshots are" \
           "trusted, or convert it with tools/convert_weights.py --trusted-weights" >&2
      exit 1
    fi
    W=$PKL
    EXTRA=(--trusted-weights)
  else
    W=$PKL   # test_net.py waits for it (--wait True), as the reference does
  fi
  if [ "$NGPU" -gt 1 ]; then
    $RUN python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPU" \
      --master-addr 127.0.0.1 --master-port "${MASTER_PORT:-29511}" \
      "$ROOT/tools/test_net.py" --multi-gpu-testing "${EXTRA[@]}" "${ARGS[@]}" TEST.WEIGHTS "$W"
  else
    $RUN python "$ROOT/tools/test_net.py" --multi-gpu-testing "${EXTRA[@]}" "${ARGS[@]}" \
      TEST.WEIGHTS "$W"
  fi
done
