#!/bin/bash
# r03m: fused weighted-BP training (NBP, V22) tests + step timing
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03m}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_wbp.py tests/test_gpu_train_v30.py tests/test_v22.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
: > $OUT/curve.jsonl
for m in "v22 --code toric_6" "nbp --code toric_4" "v30 --code toric_8"; do
  for b in 128 1024; do
    timeout -k 10 200 python bench.py --mode train --model $m --dtype f64 --batch $b --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 >> $OUT/curve.jsonl
  done
done
echo done
