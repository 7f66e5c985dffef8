#!/bin/bash
# r03u: per-phase shader-clock cycles of the config-5 forward (tape) and reverse pass, one wave
# of workgroup 0 (libgnnd_prof: -DGNND_PHASE_PROF), at B = 128 and 1 024
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03u}; mkdir -p $OUT
export TMPDIR=/tmp
export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_${2:-prof}.so
for b in 128 1024; do
  timeout -k 10 200 python bench.py --mode train --batch $b --steps 4 --warmup 1 --cpu-seconds 0 > $OUT/prof_B$b.log 2>&1 || { tail $OUT/prof_B$b.log; exit 1; }
  grep PHASE $OUT/prof_B$b.log | tail -4
done
