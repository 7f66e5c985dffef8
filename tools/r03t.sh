#!/bin/bash
# r03t: A/B of the V24 fp32 streaming kernel with the linear parts passed by value (no
# scratch round trip, no vmcnt(0) behind the tape stores) = libgnnd_$1, against the release
# library: config-5 training steps and the fp32 V24 decode
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
V=${1:-nos}
OUT=gpurun_out/${2:-r03t}; mkdir -p $OUT
export TMPDIR=/tmp
: > $OUT/ab.txt
for rep in 1 2; do
for lib in base $V; do
  if [ $lib = base ]; then unset GNND_LIB; else export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_$V.so; fi
  for b in 128 1024 8192; do
    timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib train', $b, round(j['ms_per_step'],4), round(j['roofline']['frac'],4))" >> $OUT/ab.txt
  done
  timeout -k 10 200 python bench.py --model v24 --code toric_5 --batch 65536 --dtype f32 --steps 20 --warmup 3 --cpu-seconds 0 --configs off > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
  grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib v24f32', round(j['value']/1e6,3), j['roofline']['kernel_ms'])" >> $OUT/ab.txt
done
done
cat $OUT/ab.txt
export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_$V.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_split.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$V.log 2>&1; tail -2 $OUT/pytest_$V.log
