#!/bin/bash
# r03d: split/fused-loss/update/dist tests, config-5 A/B (16 vs 8 waves in the reverse pass),
# rocprof of the B=128 step, and the full default bench line (headline + nested configs).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03d}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_training.py tests/test_gpu_dist_decode.py tests/test_gpu_parity.py tests/test_gpu_at_size.py -k "v24 or split or train or fused or decode_counts or loss" -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -le 1 ] || exit $rc
: > $OUT/curve.jsonl
for b in 16 128 1024; do
  timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/b$b.log 2>&1 || exit 1; grep '^{' $OUT/b$b.log | tail -1 >> $OUT/curve.jsonl
  GNND_TRAIN_THREADS=512 timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/w8_b$b.log 2>&1 || exit 1; grep '^{' $OUT/w8_b$b.log | tail -1 >> $OUT/curve.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_b128 -o run --output-format csv -- python bench.py --mode train --batch 128 --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/prof_b128.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
echo done
