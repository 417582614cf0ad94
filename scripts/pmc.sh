#!/bin/bash
# PMC passes (counters only with --kernel-trace; never with sys/runtime traces).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmc
mkdir -p $OUT
CMD=${CMD:-"python3 scripts/layer_times.py"}
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- $CMD > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
