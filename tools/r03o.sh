#!/bin/bash
# r03o: reverse-pass workgroup shapes (GNND_TRAIN_THREADS) at B = 128 / 8192, config-5 step
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03o}; mkdir -p $OUT
export TMPDIR=/tmp
: > $OUT/ab.txt
for rep in 1 2; do
for shape in 1024 512 5122; do
  for b in 128 8192; do
    GNND_TRAIN_THREADS=$shape timeout -k 10 200 python bench.py --mode train --batch $b --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$shape', $b, round(j['ms_per_step'],4))" >> $OUT/ab.txt
  done
done
done
cat $OUT/ab.txt
