#!/bin/bash
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03e}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 ./tools/micro/issue_cost > $OUT/issue_cost.txt 2>&1 || exit 1
bash tools/pmc_classes.sh $OUT/pmc_cgnni > $OUT/pmc_cgnni.log 2>&1 || { tail $OUT/pmc_cgnni.log; exit 1; }
bash tools/pmc_classes.sh $OUT/pmc_v24f64 --model v24 --code toric_5 --dtype f64 --batch 16384 > $OUT/pmc_v24f64.log 2>&1 || { tail $OUT/pmc_v24f64.log; exit 1; }
bash tools/pmc_classes.sh $OUT/pmc_v24f32 --model v24 --code toric_5 --dtype f32 --batch 65536 > $OUT/pmc_v24f32.log 2>&1 || { tail $OUT/pmc_v24f32.log; exit 1; }
echo done
