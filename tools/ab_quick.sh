#!/bin/bash
# Quick A/B: default libgnnd.so vs a tuning build gnn-decode_amd/gnndecode/libgnnd_$1.so on one
# bench workload, alternating, $3 reps.  usage: tools/ab_quick.sh NAME "bench args" [reps]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
name=$1; args=$2; reps=${3:-2}
mkdir -p gpurun_out/ab
for rep in $(seq $reps); do
  for lib in base $name; do
    if [ $lib = base ]; then unset GNND_LIB; else export GNND_LIB=$ROOT/gnn-decode_amd/gnndecode/libgnnd_$name.so; fi
    timeout -k 10 120 python bench.py $args --cpu-seconds 0 > gpurun_out/ab/b.log 2>&1 || { tail -5 gpurun_out/ab/b.log; exit 3; }
    grep '^{' gpurun_out/ab/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); r=j['roofline'] or {}; print('$lib', j['config']['workload'][:40], round(j['value']/1e6,2), 'M/s kernel_ms', r.get('kernel_ms'))"
  done
done
