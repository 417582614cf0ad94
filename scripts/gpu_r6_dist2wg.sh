#!/bin/bash
# Distance GEMM tiles 8 / 9 / 10 of a build not kept (128 x 128, two stages,
# two workgroups per CU: 8 waves 2 x 4 / 4 x 2, 4 waves 2 x 2):
# the h2 distance tests (every tile, plain and mirrored), then Market
# 3368 x 15913 and Duke's self-distance per tile, against tiles 0 / 6.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_h2.py -x -q --timeout 300 --timeout-method thread \
    > $OUT/r6_dist2wg_pytest.log 2>&1
rc=$?
tail -2 $OUT/r6_dist2wg_pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/r6_dist2wg_pytest.log | head; exit $rc; }
L=$OUT/r6_dist2wg.log
: > $L
for r in 1 2; do
  TILES=6,10,8,0 timeout -k 10 200 python -u scripts/probes/dist_tiles_time.py >> $L 2>&1 || { tail -5 $L; exit 1; }
done
timeout -k 10 300 python -u scripts/probes/selfdist_tiles.py 0 6 10 >> $L 2>&1 || { tail -5 $L; exit 1; }
grep -v amdgpu.ids $L
