#!/bin/bash
# PMC passes over the config-5 training step (bench.py --mode train), every kernel of the step.
# usage: tools/pmc_train.sh OUTDIR [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$1"; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH=(python bench.py --mode train --steps 5 --warmup 2 --cpu-seconds 0 "$@")
pass() {  # name counters...
  local name=$1; shift
  echo "=== pmc $name: $*"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- "${BENCH[@]}" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "--- pmc $name exit $rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi
}
pass sq1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY
pass sq2 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE
python tools/pmc_kernels.py "$OUT" "$OUT/summary.json" > /dev/null
echo "=== pmc done"
