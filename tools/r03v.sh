#!/bin/bash
# r03v: libgnnd_$1 (parallel gradient flush, gathered variable sums and unit-split readout in
# the small-batch forward) — GPU suite on it, A/B against the release library, phase profile
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
V=${1:-v2}
OUT=gpurun_out/${2:-r03v}; mkdir -p $OUT
export TMPDIR=/tmp
GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_$V.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$V.log 2>&1; rc=$?; tail -3 $OUT/pytest_$V.log
[ $rc -eq 0 ] || exit $rc
bash tools/r03u.sh ${2:-r03v}_prof prof || exit 1
: > $OUT/ab.txt
for rep in 1 2; do
for lib in base $V; do
  if [ $lib = base ]; then unset GNND_LIB; else export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_$V.so; fi
  for b in 16 128 1024 8192; do
    timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib train', $b, round(j['ms_per_step'],4), round(j['roofline']['frac'],4))" >> $OUT/ab.txt
  done
done
done
cat $OUT/ab.txt
