#!/bin/bash
# r05g: GPU suite with the signed fp64 Softplus table (kSgTab), then same-box A/Bs against the
# kSpTab form (libgnnd_sptab.so: -DGNND_F64_SGTAB=0) on config 3 (toric-5 decoder_v2_4 fp64
# decode) and the fp64 config-5 training step.  usage: tools/r05_gpu_g.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05g}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit $rc; fi
C3="--model v24 --code toric_5 --dtype f64 --steps 10 --warmup 2 --configs off"
T5="--mode train --model v24 --code toric_7 --batch 128 --dtype f64 --steps 200 --warmup 5 --configs off"
bash tools/ab_var.sh sptab "" "$C3" 3 > $OUT/ab_sptab_c3.txt 2>&1 || exit 3
bash tools/ab_var.sh sptab "" "$T5" 2 > $OUT/ab_sptab_t5.txt 2>&1 || exit 3
cat $OUT/ab_*.txt
echo done
