#!/bin/bash
# VALU instruction-class counters (gfx950 SQ_INSTS_VALU_*) of a bench workload, two passes, for
# the cycle-weighted issue model (bench.py issue_model).  usage: tools/pmc_classes.sh OUT [bench args]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$1"; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH=(python bench.py --steps 3 --warmup 1 --prewarm-s 0 --cpu-seconds 0 --configs off "$@")
pass() {
  local name=$1; shift
  echo "=== pmc $name: $*"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- "${BENCH[@]}" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "--- pmc $name exit $rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi
}
pass c1 SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64
pass c2 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_LDS SQ_WAVES
pass c3 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM
python tools/pmc_kernels.py "$OUT" "$OUT/summary.json" decode > /dev/null
echo "=== pmc done"
