#!/bin/bash
# r05d: headline / LDPC A/Bs of the message-MLP forms (base = one-asm + pruning; noprune = one-asm;
# noasm = r04 form; vcache = one-asm + cached var_ord entries)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out/r05d; mkdir -p $OUT
L="--code ldpc_648_324 --batch 131072 --steps 30 --configs off"
bash tools/ab_var.sh noprune "" "--configs off --steps 200" 2 > $OUT/bch_noprune.txt 2>&1 || exit 3
bash tools/ab_var.sh noasm "" "--configs off --steps 200" 2 > $OUT/bch_noasm.txt 2>&1 || exit 3
bash tools/ab_var.sh vcache "" "--configs off --steps 200" 3 > $OUT/bch_vcache.txt 2>&1 || exit 3
bash tools/ab_var.sh noprune "" "$L" 2 > $OUT/ldpc_noprune.txt 2>&1 || exit 3
bash tools/ab_var.sh noasm "" "$L" 2 > $OUT/ldpc_noasm.txt 2>&1 || exit 3
cat $OUT/*.txt
