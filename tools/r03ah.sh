#!/bin/bash
# r03ah: forward unit split of the small-batch training step after the gather / readout
# rework: US = 2 / 4 (default) / 8 (GNND_V24_SPLIT) at B = 16 and 128; reverse-pass shape 1024 (16
# waves, default below 2 x CUs rows) vs 512 (8 waves, 256 VGPRs) (GNND_TRAIN_THREADS)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03ah}; mkdir -p $OUT
export TMPDIR=/tmp
: > $OUT/ab.txt
for rep in 1 2; do
for us in 4 8 2; do
  export GNND_V24_SPLIT=$us
  for b in 16 128; do
    timeout -k 10 200 python bench.py --mode train --batch $b --steps 40 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('US=$us', $b, round(j['ms_per_step'],4))" >> $OUT/ab.txt
  done
done
done
cat $OUT/ab.txt
unset GNND_V24_SPLIT
for rep in 1 2; do
for th in 1024 512; do
  export GNND_TRAIN_THREADS=$th
  for b in 16 128; do
    timeout -k 10 200 python bench.py --mode train --batch $b --steps 40 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('bwd threads $th', $b, round(j['ms_per_step'],4))" >> $OUT/ab.txt
  done
done
done
cat $OUT/ab.txt
