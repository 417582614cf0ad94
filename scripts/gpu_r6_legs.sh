#!/bin/bash
# The sharded legs (config_cuhk03 / config_1m) at N = 1 on the GPU: what the
# driver's N > 1 runs execute per rank.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$PWD/gpurun_out
mkdir -p $OUT
timeout -k 10 900 python -u bench.py --sharded-legs --no-e2e --no-duke --no-cpu-baseline \
    > $OUT/r6_legs.log 2>&1 || { tail -20 $OUT/r6_legs.log; exit 1; }
tail -1 $OUT/r6_legs.log | python -c "
import json, sys
d = json.loads(sys.stdin.read())
print(d['value'], d['ms_per_step'])
for k in ('config_cuhk03', 'config_1m'):
    print(k, json.dumps(d.get(k))[:600])
"
