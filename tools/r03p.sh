#!/bin/bash
# r03p: reverse-pass workgroup shapes incl. 2564, and the batch-dependent default
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03p}; mkdir -p $OUT
export TMPDIR=/tmp
: > $OUT/ab.txt
for shape in default 2564 5122; do
  for b in 128 1024 8192; do
    if [ $shape = default ]; then unset GNND_TRAIN_THREADS; else export GNND_TRAIN_THREADS=$shape; fi
    timeout -k 10 200 python bench.py --mode train --batch $b --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$shape', $b, round(j['ms_per_step'],4), round(j['roofline']['frac'],4))" >> $OUT/ab.txt
  done
done
unset GNND_TRAIN_THREADS
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_split.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log
cat $OUT/ab.txt
exit $rc
