#!/bin/bash
# r03ag: final tree of the round: full GPU suite, smoke, default bench line (every config) and
# its rocprofv3 kernel summary, config-5 curve
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03ag}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -2 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 > $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --configs off --cpu-seconds 0 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
: > $OUT/curve.jsonl
for b in 16 128 256 1024 2048 8192; do
  timeout -k 10 300 python bench.py --mode train --batch $b --steps 40 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
  grep '^{' $OUT/b.log | tail -1 >> $OUT/curve.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_B128 -o run --output-format csv -- python bench.py --mode train --batch 128 --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/prof128.log 2>&1 || { tail $OUT/prof128.log; exit 1; }
echo done
