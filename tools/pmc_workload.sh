#!/bin/bash
# PMC evidence for one decode workload: the VALU-class passes (tools/pmc_classes.sh ->
# pmc_classes_<CTAG>.json, read by bench.py's issue model) and the traffic / LDS / wait passes
# (tools/pmc.sh -> pmc_<PTAG>.json, bench.py's roofline.traffic).
# usage: tools/pmc_workload.sh OUT CTAG PTAG KERNEL_SUBSTRING BATCH E T [bench args...]
#   e.g. tools/pmc_workload.sh gpurun_out/x cbp_bch_63_45_T25_f32 cbp_bch_63_45_B65536_T25_f32 \
#          "decode_resident_kernel<4, float" 65536 432 25 --model cbp
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=$1; CTAG=$2; PTAG=$3; KSUB=$4; B=$5; E=$6; T=$7; shift 7
mkdir -p "$OUT"
SRC="rocprofv3 --kernel-trace --pmc passes (tools/pmc_workload.sh), $(basename "$OUT")"
bash tools/pmc_classes.sh "$OUT/cls_$CTAG" --batch "$B" "$@" || exit 3
python tools/pmc_classes_json.py "$OUT/cls_$CTAG/summary.json" "$KSUB" "$B" "$CTAG" "$SRC" \
    "$OUT/pmc_classes_$CTAG.json" "$E" "$T" || exit 3
bash tools/pmc.sh "$OUT/pmc_$PTAG" --batch "$B" --configs off "$@" || exit 3
python tools/pmc_summary.py "$OUT/pmc_$PTAG" "$PTAG" "$OUT/pmc_$PTAG.json" > "$OUT/pmc_$PTAG.log" 2>&1
echo "pmc_workload $CTAG done"
