#!/bin/bash
# PMC passes (tools/pmc.sh) on the fp64 decoder_v2_4 toric-5 decode (config 3 at reference
# precision), per-launch means into OUTDIR/pmc_v24_f64.json.  usage: tools/pmc_v24_f64.sh OUTDIR
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$1"; mkdir -p "$OUT"
bash tools/pmc.sh "$OUT/pmc" --model v24 --code toric_5 --dtype f64 --batch 16384 --steps 3 --warmup 1 > "$OUT/pmc.log" 2>&1 || { tail -20 "$OUT/pmc.log"; exit 1; }
python tools/pmc_summary.py "$OUT/pmc" v24_toric5_B16384_f64 "$OUT/pmc_v24_f64.json" > "$OUT/pmc_summary.log" 2>&1 || { tail -20 "$OUT/pmc_summary.log"; exit 1; }
echo done
