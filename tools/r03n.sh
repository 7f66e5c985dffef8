#!/bin/bash
# r03n: PMC of the config-5 training step at B = 8192 (reverse pass efficiency)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03n}; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/pmc_train.sh $OUT/pmc --batch 8192 > $OUT/pmc.log 2>&1 || { tail $OUT/pmc.log; exit 1; }
BENCH=(python bench.py --mode train --steps 5 --warmup 2 --cpu-seconds 0 --batch 8192)
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT -d $OUT/pmc/cls -o run --output-format csv -- "${BENCH[@]}" > $OUT/cls.log 2>&1 || { tail $OUT/cls.log; exit 1; }
python tools/pmc_kernels.py $OUT/pmc $OUT/summary.json v24_bwd decode_kernel > /dev/null
cat $OUT/summary.json
echo done
