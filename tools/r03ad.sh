#!/bin/bash
# r03ad: bench --launch auto (eager stream launches for the fused trainer, loss buffer not
# cloned) on the release tree: training curve, trace of the B = 128 step, training GPU tests
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03ad}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_split.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
: > $OUT/curve.jsonl
for rep in 1 2; do
for b in 16 128 256 1024 2048 8192; do
  [ $rep -eq 2 ] && [ $b -ne 128 ] && [ $b -ne 1024 ] && continue
  timeout -k 10 300 python bench.py --mode train --batch $b --steps 40 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
  grep '^{' $OUT/b.log | tail -1 >> $OUT/curve.jsonl
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_B128 -o run --output-format csv -- python bench.py --mode train --batch 128 --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_B16 -o run --output-format csv -- python bench.py --mode train --batch 16 --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/prof16.log 2>&1 || { tail $OUT/prof16.log; exit 1; }
python -c "
import json
for l in open('$OUT/curve.jsonl'):
    j=json.loads(l); print(j['config']['global_batch'], round(j['ms_per_step'],4), j['config']['hip_graph'])
"
