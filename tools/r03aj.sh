#!/bin/bash
# r03aj: fp64 (the reference dtype) config-5 step after the reverse-pass rework (parallel
# flush, sibling tables; eager launches): B = 16 / 128 / 1024
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03aj}; mkdir -p $OUT
export TMPDIR=/tmp
: > $OUT/f64.jsonl
for b in 16 128 1024; do
  timeout -k 10 300 python bench.py --mode train --dtype f64 --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
  grep '^{' $OUT/b.log | tail -1 >> $OUT/f64.jsonl
done
python -c "
import json
for l in open('$OUT/f64.jsonl'):
    j=json.loads(l); print(j['config']['global_batch'], round(j['ms_per_step'],4), round(j['roofline']['frac'],4))
"
