#!/bin/bash
# One GPU session that produces the round's measurement artefacts:
#   1. bench (autotune; tiles saved)            -> gpurun_out/bench_tuned.log
#   2. rocprofv3 --kernel-trace --stats (same tiles, no e2e stage: its ragged
#      last batch would be the "last forward") -> gpurun_out/prof/
#   3. PMC passes FETCH_SIZE / WRITE_SIZE / MFMA busy (same tiles)
#      -> gpurun_out/pmc_traffic.json
#   4. bench again (same tiles, traffic filled)  -> gpurun_out/bench_final.log
# Each GPU step has its own time limit; the script stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$PWD/gpurun_out
R=${ROUND_DIR:-profiles/r06}
mkdir -p $OUT $R
TILES=$OUT/tiles.json
rm -f $TILES
# TILES_IN=<committed table>: skip the tuning run, profile that table
if [ -n "$TILES_IN" ]; then cp "$TILES_IN" $TILES; fi
MATH=${PPS_MATH:-x3}
step() { echo "== $1"; }
step bench-tune
[ -n "$TILES_IN" ] || timeout -k 10 600 python bench.py --tiles-file $TILES > $OUT/bench_tuned.log 2>&1 || { tail -5 $OUT/bench_tuned.log; exit 1; }
[ -n "$TILES_IN" ] || tail -1 $OUT/bench_tuned.log | cut -c1-300
step stats
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 bench.py --tiles-file $TILES --no-cpu-baseline --no-e2e --no-duke > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
step pmc
rm -rf $OUT/pmcb
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/pmcb/p1 -o run --output-format csv -- python3 bench.py --tiles-file $TILES --no-cpu-baseline --no-e2e --no-duke --steps 2 --warmup 1 --dist-reps 1 > $OUT/pmc1.log 2>&1 || { tail -5 $OUT/pmc1.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/pmcb/p2 -o run --output-format csv -- python3 bench.py --tiles-file $TILES --no-cpu-baseline --no-e2e --no-duke --steps 2 --warmup 1 --dist-reps 1 > $OUT/pmc2.log 2>&1 || { tail -5 $OUT/pmc2.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d $OUT/pmcb/p3 -o run --output-format csv -- python3 bench.py --tiles-file $TILES --no-cpu-baseline --no-e2e --no-duke --steps 2 --warmup 1 --dist-reps 1 > $OUT/pmc3.log 2>&1 || { tail -5 $OUT/pmc3.log; exit 1; }
# MFMA launches per forward: 50 layers, one fewer per bottleneck seam pair
NCONV=$(python -c "import json; t = json.load(open('$TILES')); print(50 - sum(1 for k, v in t.items() if not k.startswith('__') and isinstance(v, int) and v & 0x400))")
CLK=$OUT/bench_tuned.log; [ -f $CLK ] || CLK=$OUT/prof.log
python scripts/pmc_traffic.py $OUT/pmcb $MATH 64 $NCONV $TILES --clock-from $CLK > $OUT/pmc_traffic.json || exit 1
cat $OUT/pmc_traffic.json
cp $OUT/pmc_traffic.json $R/pmc_traffic.json   # bench-final reads it (box copy)
step bench-final
PPS_BENCH_LAYERS=$OUT/layers.json timeout -k 10 600 python bench.py --tiles-file $TILES > $OUT/bench_final.log 2>&1 || { tail -5 $OUT/bench_final.log; exit 1; }
tail -1 $OUT/bench_final.log
python scripts/layer_table.py $OUT/layers.json $OUT/pmcb > $OUT/layer_table.md || exit 1
