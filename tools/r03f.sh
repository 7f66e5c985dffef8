#!/bin/bash
# r03f: split rule (B < CUs) + the reverse-pass workgroup-shape A/B; issue-cost micro
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03f}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 ./tools/micro/issue_cost > $OUT/issue_cost.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_training.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -le 1 ] || exit $rc
: > $OUT/curve.jsonl; : > $OUT/curve_5122.jsonl
for b in 16 64 128 200 256 512 1024 2048 4096 8192; do
  timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/b$b.log 2>&1 || exit 1; grep '^{' $OUT/b$b.log | tail -1 >> $OUT/curve.jsonl
done
for b in 512 1024 8192; do
  GNND_TRAIN_THREADS=5122 timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/x_b$b.log 2>&1 || exit 1; grep '^{' $OUT/x_b$b.log | tail -1 >> $OUT/curve_5122.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_b8192 -o run --output-format csv -- python bench.py --mode train --batch 8192 --steps 10 --warmup 2 --cpu-seconds 0 > $OUT/prof_b8192.log 2>&1 || exit 1
bash tools/pmc_train.sh $OUT/pmc8192 --batch 8192 > $OUT/pmc8192.log 2>&1 || { tail $OUT/pmc8192.log; exit 1; }
echo done
