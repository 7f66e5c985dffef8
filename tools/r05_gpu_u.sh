#!/bin/bash
# r05u: PMC refresh on the final kernels: VALU classes (tools/pmc_classes.sh) and HBM traffic /
# LDS conflicts (tools/pmc.sh) for the headline, config 4 (LDPC) and config 3 (toric-5 fp64,
# 512-lane workgroups).  usage: tools/r05_gpu_u.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05u}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
SRC="rocprofv3 --kernel-trace --pmc, three passes (tools/pmc_classes.sh), $TAG"
bash tools/pmc_classes.sh $OUT/cls_bch || exit 3
python tools/pmc_classes_json.py $OUT/cls_bch/summary.json "decode_resident_kernel<3, float, 8, 3, 9, 0" 65536 cgnni_bch_63_45_T25_f32 "$SRC" $OUT/pmc_classes_cgnni_bch_63_45_T25_f32.json 432 25
bash tools/pmc.sh $OUT/pmc_bch --configs off || exit 3
python tools/pmc_summary.py $OUT/pmc_bch cgnni_bch_63_45_B65536_T25_f32 $OUT/pmc_cgnni_bch_63_45_B65536_T25_f32.json > $OUT/pmc_bch.log 2>&1
L="--code ldpc_648_324 --batch 131072"
bash tools/pmc_classes.sh $OUT/cls_ldpc $L || exit 3
python tools/pmc_classes_json.py $OUT/cls_ldpc/summary.json "decode_resident_kernel<3, float, 2, 4, 6, 1" 131072 cgnni_ldpc_648_324_T25_f32 "$SRC" $OUT/pmc_classes_cgnni_ldpc_648_324_T25_f32.json 2376 25
bash tools/pmc.sh $OUT/pmc_ldpc $L --configs off || exit 3
python tools/pmc_summary.py $OUT/pmc_ldpc cgnni_ldpc_648_324_B131072_T25_f32 $OUT/pmc_cgnni_ldpc_648_324_B131072_T25_f32.json > $OUT/pmc_ldpc.log 2>&1
C3="--model v24 --code toric_5 --dtype f64"
bash tools/pmc_classes.sh $OUT/cls_c3 $C3 --batch 16384 || exit 3
python tools/pmc_classes_json.py $OUT/cls_c3/summary.json "decode_kernel<0, double, 1, false, 1, 2>" 16384 v24_toric_5_T15_f64 "$SRC (signed one-read kSgTab Softplus, 512-lane workgroups, 2 per CU)" $OUT/pmc_classes_v24_toric_5_T15_f64.json 192 15
bash tools/pmc.sh $OUT/pmc_c3 $C3 --configs off || exit 3
python tools/pmc_summary.py $OUT/pmc_c3 v24_toric_5_B65536_T15_f64 $OUT/pmc_v24_toric_5_B65536_T15_f64.json > $OUT/pmc_c3.log 2>&1
ls $OUT/*.json
echo done
