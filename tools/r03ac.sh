#!/bin/bash
# r03ac: config-5 step at B = 16 / 128 / 1024 with the fused trainer's HIP graph vs eager
# stream launches (bench --no-graph); the rocprof trace shows ~9 us between consecutive graph
# replays (fwd 78 + bwd 122 + update 5 us of kernels in a 214 us step)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03ac}; mkdir -p $OUT
export TMPDIR=/tmp
: > $OUT/ab.txt
for rep in 1 2; do
for mode in graph eager; do
  extra=""; [ $mode = eager ] && extra="--no-graph"
  for b in 16 128 1024; do
    timeout -k 10 200 python bench.py --mode train --batch $b --steps 40 --warmup 3 --cpu-seconds 0 $extra > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$mode train', $b, round(j['ms_per_step'],4), 'host', round(j.get('host_issue_ms_per_step',0),4))" >> $OUT/ab.txt
  done
done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_eager -o run --output-format csv -- python bench.py --mode train --batch 128 --steps 20 --warmup 3 --cpu-seconds 0 --no-graph > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
cat $OUT/ab.txt
