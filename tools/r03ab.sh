#!/bin/bash
# r03ab: libgnnd_v8 = release + the reverse pass's last partial round of 4-edge groups run as
# half steps over more SIMDs: training GPU tests on it, A/B against release
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03ab}; mkdir -p $OUT
export TMPDIR=/tmp
V=${2:-v8}
GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_$V.so timeout -k 10 900 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_split.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$V.log 2>&1; rc=$?; tail -2 $OUT/pytest_$V.log
[ $rc -eq 0 ] || exit $rc
: > $OUT/ab.txt
for rep in 1 2 3; do
for lib in base $V; do
  if [ $lib = base ]; then unset GNND_LIB; else export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_$lib.so; fi
  for b in 16 128 1024 8192; do
    [ $rep -eq 3 ] && [ $b -ne 128 ] && continue
    timeout -k 10 200 python bench.py --mode train --batch $b --steps 40 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib train', $b, round(j['ms_per_step'],4), round(j['roofline']['frac'],4))" >> $OUT/ab.txt
  done
done
done
cat $OUT/ab.txt
