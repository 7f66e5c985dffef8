#!/bin/bash
# r05w: resident-plan Q sweep (tools/variant_sweep.sh) on config 4 (LDPC) and the headline with
# the final kernels (five cached variable entries for the light plans).  usage: tools/r05_gpu_w.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05w}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/variant_sweep.sh --code ldpc_648_324 --batch 131072 --configs off > $OUT/sweep_ldpc.txt 2>&1 || exit 3
bash tools/variant_sweep.sh --configs off > $OUT/sweep_bch.txt 2>&1 || exit 3
cat $OUT/sweep_*.txt
echo done
