#!/bin/bash
# r03z: v6 = v5 + check-row variable table, four-wide logical rows and early per-edge loads in the
# fused loss setup, readout MLP weights re-read per codeword; v6n = v6 without the re-read
# v7 = v6 + slot words and check feature held in registers in the gathered forward (base = release = v5)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03y}; mkdir -p $OUT
export TMPDIR=/tmp
GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_v7.so timeout -k 10 900 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_split.py tests/test_gpu_train_v30.py tests/test_gpu_at_size.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_v7.log 2>&1; rc=$?; tail -2 $OUT/pytest_v7.log
[ $rc -eq 0 ] || exit $rc
true
: > $OUT/ab.txt
for rep in 1 2; do
for lib in base v6 v6n v7; do
  if [ $lib = base ]; then unset GNND_LIB; else export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_$lib.so; fi
  for b in 16 128 1024; do
    timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib train', $b, round(j['ms_per_step'],4), round(j['roofline']['frac'],4))" >> $OUT/ab.txt
  done
done
done
cat $OUT/ab.txt
