#!/bin/bash
# r03ai: default bench line on the final tree (config-5 entries at 200 / 100 timed steps)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03ai}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
python -c "
import json; j=json.load(open('$OUT/bench.json'))
print('headline', j['value'], j['roofline']['frac'])
for k,v in j['configs'].items(): print(k, v['ms_per_step'], v.get('wall_s'))
"
