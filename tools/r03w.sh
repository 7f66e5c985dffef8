#!/bin/bash
# r03w: A/B/C of the small-batch training step: release | libgnnd_v3 (parallel flush, gathered
# variable sums, unit-split readout, sibling tables in the reverse pass) | libgnnd_v3ng (v3
# without the gathered variable sums); phase profile of v3 (libgnnd_prof3)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03w}; mkdir -p $OUT
export TMPDIR=/tmp
GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_v3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_split.py tests/test_gpu_at_size.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_v3.log 2>&1; rc=$?; tail -2 $OUT/pytest_v3.log
[ $rc -eq 0 ] || exit $rc
bash tools/r03u.sh ${1:-r03w}_prof prof3 || exit 1
: > $OUT/ab.txt
for rep in 1 2; do
for lib in base v3 v3ng; do
  if [ $lib = base ]; then unset GNND_LIB; else export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_$lib.so; fi
  for b in 16 128 1024; do
    timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib train', $b, round(j['ms_per_step'],4), round(j['roofline']['frac'],4))" >> $OUT/ab.txt
  done
done
done
cat $OUT/ab.txt
