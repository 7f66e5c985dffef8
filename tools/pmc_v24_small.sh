#!/bin/bash
# PMC passes (sq1/sq2 of tools/pmc.sh) on the fp32 decoder_v2_4 toric-5 decode at B = 128,
# unit split off (GNND_V24_SPLIT=1) and on (4).  usage: tools/pmc_v24_small.sh OUTDIR
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
for us in 1 4; do
  export GNND_V24_SPLIT=$us
  bash tools/pmc.sh "$OUT/us$us" --model v24 --code toric_5 --batch 128 --steps 20 --warmup 2 > "$OUT/us$us.log" 2>&1 || { tail -20 "$OUT/us$us.log"; exit 1; }
done
echo done
