#!/bin/bash
# r03r: A/B of the reverse pass with four consecutive edges per wave step (ds_read_b128, row
# stores, pass-local partials) = libgnnd_b128, against the release library
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03r}; mkdir -p $OUT
export TMPDIR=/tmp
: > $OUT/ab.txt
for rep in 1 2; do
for lib in base b128; do
  if [ $lib = base ]; then unset GNND_LIB; else export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_b128.so; fi
  for b in 128 1024 8192; do
    timeout -k 10 200 python bench.py --mode train --batch $b --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib', $b, round(j['ms_per_step'],4), round(j['roofline']['frac'],4))" >> $OUT/ab.txt
  done
done
done
export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_b128.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_split.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_b128.log 2>&1; tail -2 $OUT/pytest_b128.log
cat $OUT/ab.txt
