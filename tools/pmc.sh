#!/bin/bash
# rocprofv3 PMC passes for the bench workload (one counter group per pass, --pmc only
# with --kernel-trace: never combined with sys/runtime/hip traces).
# usage: tools/pmc.sh OUTDIR [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$1"; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH=(python bench.py --steps 5 --warmup 1 --cpu-seconds 0 "$@")
pass() {  # name counters...
  local name=$1; shift
  echo "=== pmc $name: $*"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- "${BENCH[@]}" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "--- pmc $name exit $rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY
pass sq2 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE
echo "=== pmc done"
