#!/bin/bash
# r05i: config-3 PMC on the signed-table fp64 kernel: VALU classes for bench.py's issue model
# (tools/pmc_classes.sh at B = 16 384) and HBM traffic / LDS conflicts (tools/pmc.sh at the
# bench size).  usage: tools/r05_gpu_i.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05i}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
C3="--model v24 --code toric_5 --dtype f64"
bash tools/pmc_classes.sh $OUT/pmc_classes $C3 --batch 16384 || exit 3
python tools/pmc_classes_json.py $OUT/pmc_classes/summary.json "decode_kernel<0, double, 1, false, 1>" 16384 v24_toric_5_T15_f64 "rocprofv3 --kernel-trace --pmc, three passes (tools/pmc_classes.sh), $TAG (signed one-read kSgTab Softplus, 3 workgroups per CU)" $OUT/pmc_classes_v24_toric_5_T15_f64.json 192 15
bash tools/pmc.sh $OUT/pmc $C3 --configs off || exit 3
python tools/pmc_summary.py $OUT/pmc v24_toric_5_B65536_T15_f64 $OUT/pmc_v24_toric_5_B65536_T15_f64.json > $OUT/pmc_summary.log 2>&1
tail -5 $OUT/pmc_summary.log
echo done
