#!/bin/bash
# r03y: libgnnd_v5 = v3 + batched setup loads and the wave-parallel linear parts in the V24
# streaming forward: GPU tests, A/B against release and v3 (training steps, fp32 V24 decode),
# phase profile (libgnnd_prof5)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03y}; mkdir -p $OUT
export TMPDIR=/tmp
GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_v5.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_v5.log 2>&1; rc=$?; tail -2 $OUT/pytest_v5.log
[ $rc -eq 0 ] || exit $rc
bash tools/r03u.sh ${1:-r03y}_prof prof5 || exit 1
: > $OUT/ab.txt
for rep in 1 2; do
for lib in base v3 v5; do
  if [ $lib = base ]; then unset GNND_LIB; else export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_$lib.so; fi
  for b in 16 128 1024 8192; do
    timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib train', $b, round(j['ms_per_step'],4), round(j['roofline']['frac'],4))" >> $OUT/ab.txt
  done
  timeout -k 10 200 python bench.py --model v24 --code toric_5 --batch 65536 --dtype f32 --steps 20 --warmup 3 --cpu-seconds 0 --configs off > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
  grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib v24f32', round(j['value']/1e6,3), j['roofline']['kernel_ms'])" >> $OUT/ab.txt
done
done
cat $OUT/ab.txt
