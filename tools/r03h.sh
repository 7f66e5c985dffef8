#!/bin/bash
# r03h: fp64 V24 MLP trims + reverse-pass W2 factoring: tests, full bench line, curve, profiles
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03h}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_training.py tests/test_gpu_dist_decode.py tests/test_gpu_parity.py tests/test_gpu_at_size.py -k "v24 or split or train or fused or decode_counts or loss" -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
: > $OUT/curve.jsonl
for b in 16 128 256 1024 8192; do
  timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/b$b.log 2>&1 || exit 1; grep '^{' $OUT/b$b.log | tail -1 >> $OUT/curve.jsonl
done
bash tools/pmc_classes.sh $OUT/pmc_v24f64 --model v24 --code toric_5 --dtype f64 --batch 16384 > $OUT/pmc_v24f64.log 2>&1 || { tail $OUT/pmc_v24f64.log; exit 1; }
for b in 128 8192; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_b$b -o run --output-format csv -- python bench.py --mode train --batch $b --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/prof_b$b.log 2>&1 || exit 1
done
echo done
