#!/bin/bash
# rocprofv3 PMC passes over one conv layer (scripts/probes/conv_once.py ARGS);
# summary by kernel_pmc.py.  Each GPU step under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/convpmc${TAG}
rm -rf $OUT; mkdir -p $OUT
ARGS="$*"
K=${KNAME:-gemm_x3}
i=0
for set in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $OUT/pmc/p$i -o run --output-format csv -- python3 scripts/probes/conv_once.py $ARGS --reps 5 > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/probes/kernel_pmc.py $OUT/pmc $K
