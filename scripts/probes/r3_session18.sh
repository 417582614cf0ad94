set -o pipefail
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/pmcw
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
grep -oE "SQ_[A-Z_]+" $OUT/counters.txt | sort -u > $OUT/sq_names.txt || true
wc -l $OUT/sq_names.txt
CMD="python3 scripts/probes/gemm_probe.py --layers res4a,res5b --tiles 48,52 --math x3 --reps 5"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU -d $OUT/p1 -o run --output-format csv -- $CMD > $OUT/p1.log 2>&1; echo "rc=$?"; tail -3 $OUT/p1.log
