#!/bin/bash
# A/B/C of the default libgnnd.so against tuning builds libgnnd_<name>.so (GNND_LIB) on
# several bench workloads, alternating processes.  usage: tools/ab_multi.sh "v1 v2" REPS "args1" "args2" ...
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
names=$1; reps=$2; shift 2
mkdir -p gpurun_out/ab
for args in "$@"; do
  for rep in $(seq $reps); do
    for lib in base $names; do
      if [ $lib = base ]; then unset GNND_LIB; else export GNND_LIB=$ROOT/gnn-decode_amd/gnndecode/libgnnd_$lib.so; fi
      timeout -k 10 120 python bench.py $args --cpu-seconds 0 > gpurun_out/ab/b.log 2>&1 || { tail -5 gpurun_out/ab/b.log; exit 3; }
      grep '^{' gpurun_out/ab/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); r=j['roofline'] or {}; print('$lib', j['config']['workload'][:40], round(j['value']/1e6,2), 'M/s kernel_ms', round(r.get('kernel_ms') or 0, 4))"
    done
  done
done
