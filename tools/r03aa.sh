#!/bin/bash
# r03aa: release tree after the small-batch rework: default bench line (all configs), rocprofv3
# kernel traces of the config-5 step at B = 16 and 128, and the training curve
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03aa}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
for b in 16 128; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_B$b -o run --output-format csv -- python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/prof_B$b.log 2>&1 || { tail $OUT/prof_B$b.log; exit 1; }
done
: > $OUT/curve.jsonl
for b in 16 128 256 1024 2048 8192; do
  timeout -k 10 300 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
  grep '^{' $OUT/b.log | tail -1 >> $OUT/curve.jsonl
done
echo done
