#!/bin/bash
# r05j: A/B of the unit-pass issue-fairness priorities (libgnnd_fair.so: -DGNND_BWD_FAIR=1) on the
# config-5 step (fp32 and fp64, B = 128), then the config-3 PMC (tools/r05_gpu_i.sh).
# usage: tools/r05_gpu_j.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05j}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
T5="--mode train --model v24 --code toric_7 --batch 128 --steps 200 --warmup 5 --configs off"
bash tools/ab_var.sh fair "" "$T5 --dtype f32" 3 > $OUT/ab_fair_t5_f32.txt 2>&1 || exit 3
bash tools/ab_var.sh fair "" "$T5 --dtype f64" 3 > $OUT/ab_fair_t5_f64.txt 2>&1 || exit 3
cat $OUT/ab_*.txt
bash tools/r05_gpu_i.sh $TAG || exit 3
echo done
