#!/bin/bash
# r05l: A/B of the interleaved two-variable sums of the resident kernel's variable step
# (libgnnd_varpair.so: -DGNND_VAR_PAIR=1) on the headline and config 4.  usage: tools/r05_gpu_l.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05l}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/ab_var.sh varpair "" "--configs off --steps 200" 3 > $OUT/ab_varpair.txt 2>&1 || exit 3
bash tools/ab_var.sh varpair "" "--code ldpc_648_324 --batch 131072 --steps 30 --configs off" 2 > $OUT/ab_varpair_ldpc.txt 2>&1 || exit 3
PYTEST="tests/test_gpu_parity.py tests/test_gpu_at_size.py -k cgnni" bash tools/ab_var.sh varpair "" "--configs off --steps 50" 1 > $OUT/ab_varpair_tests.txt 2>&1
cat $OUT/ab_*.txt
echo done
