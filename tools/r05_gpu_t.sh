#!/bin/bash
# r05t: the fp64 config-5 forward's unit split (GNND_V24_SPLIT = 1 / 2 vs the default 4) on the
# B = 128 training step.  usage: tools/r05_gpu_t.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05t}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
T5="--mode train --model v24 --code toric_7 --batch 128 --steps 200 --warmup 5 --configs off --cpu-seconds 0 --dtype f64"
for rep in 1 2; do
  for s in 0 2 1; do
    if [ $s = 0 ]; then env timeout -k 10 300 python bench.py $T5 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 3; }
    else env GNND_V24_SPLIT=$s timeout -k 10 300 python bench.py $T5 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 3; }; fi
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); r=j['roofline'] or {}; print('split$s', '%.4g' % j['value'], 'ms', j['ms_per_step'], 'kernel_ms', r.get('kernel_ms'))" | tee -a $OUT/ab.txt
  done
done
echo done
