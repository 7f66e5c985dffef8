#!/bin/bash
# r05n: A/B of five cached variable entries for the fp32 resident plans with <= 64 item-state
# VGPRs (libgnnd_vc5.so: -DGNND_VAR_CACHE_NL=5) on config 4 (LDPC CGNNI), toric QGNNI / QBP and
# the headline (unchanged plan), then the resident-kernel parity tests on the variant.
# usage: tools/r05_gpu_n.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05n}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/ab_var.sh vc5 "" "--code ldpc_648_324 --batch 131072 --steps 30 --configs off" 3 > $OUT/ab_vc5_ldpc.txt 2>&1 || exit 3
bash tools/ab_var.sh vc5 "" "--model qgnni --code toric_5 --steps 100 --configs off" 2 > $OUT/ab_vc5_qgnni.txt 2>&1 || exit 3
bash tools/ab_var.sh vc5 "" "--model qbp --code toric_5 --steps 100 --configs off" 2 > $OUT/ab_vc5_qbp.txt 2>&1 || exit 3
bash tools/ab_var.sh vc5 "" "--configs off --steps 200" 1 > $OUT/ab_vc5_bch.txt 2>&1 || exit 3
PYTEST="tests/test_gpu_parity.py tests/test_gpu_at_size.py tests/test_gpu_resident.py" bash tools/ab_var.sh vc5 "" "--configs off --steps 20" 1 > $OUT/ab_vc5_tests.txt 2>&1
cat $OUT/ab_*.txt
echo done
