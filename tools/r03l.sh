#!/bin/bash
# r03l: fused decoder_v3_0 training tests + V30 step timing; A/B of the headline kernel
# variants (MLP batch interleave, variable-step priority)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03l}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_v30.py tests/test_v30.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for b in 128 1024; do
  timeout -k 10 200 python bench.py --mode train --model v30 --code toric_5 --dtype f64 --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/v30_b$b.log 2>&1 || { tail $OUT/v30_b$b.log; exit 1; }
  grep '^{' $OUT/v30_b$b.log | tail -1 >> $OUT/v30_curve.jsonl
done
: > $OUT/ab.txt
for rep in 1 2; do
  for lib in base mlpb prio; do
    if [ $lib = base ]; then unset GNND_LIB; else export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_$lib.so; fi
    timeout -k 10 120 python bench.py --cpu-seconds 0 --configs off > $OUT/ab_b.log 2>&1 || { tail $OUT/ab_b.log; exit 1; }
    grep '^{' $OUT/ab_b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib', round(j['value']/1e6,2), round(j['roofline']['kernel_ms'],4), round(j['roofline']['frac'],4))" >> $OUT/ab.txt
  done
done
unset GNND_LIB
cat $OUT/ab.txt
echo done
