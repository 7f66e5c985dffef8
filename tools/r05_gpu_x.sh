#!/bin/bash
# r05x: the headline's variable-step issue priority (GNND_VAR_PRIO 1 / 3 vs the default 2).
# usage: tools/r05_gpu_x.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05x}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/ab_var.sh vp1 "" "--configs off --steps 200" 3 > $OUT/ab_vp1.txt 2>&1 || exit 1
bash tools/ab_var.sh vp3 "" "--configs off --steps 200" 3 > $OUT/ab_vp3.txt 2>&1 || exit 1
cat $OUT/ab_*.txt
echo done
