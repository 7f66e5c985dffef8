#!/bin/bash
# r05 GPU round on the final MLP forms: GPU suite, LDPC quick check, default bench + same-run
# rocprofv3 (tools/gpu_round.sh), headline PMC: VALU classes (tools/pmc_classes.sh) and HBM
# traffic (FETCH_SIZE / WRITE_SIZE passes).  usage: tools/r05_gpu_e.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05e}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit $rc; fi
STEPS="bench_default prof_default" bash tools/gpu_round.sh $TAG || exit 3
bash tools/pmc_classes.sh $OUT/pmc_classes || exit 3
python tools/pmc_classes_json.py $OUT/pmc_classes/summary.json "decode_resident_kernel<3, float, 8, 3, 9, 0" 65536 cgnni_bch_63_45_T25_f32 "rocprofv3 --kernel-trace --pmc, three passes (tools/pmc_classes.sh), $TAG" $OUT/pmc_classes_cgnni_bch_63_45_T25_f32.json 432 25
bash tools/pmc.sh $OUT/pmc --configs off || exit 3
python tools/pmc_summary.py $OUT/pmc cgnni_bch_63_45_B65536_T25_f32 $OUT/pmc_cgnni_bch_63_45_B65536_T25_f32.json > $OUT/pmc_summary.log 2>&1
tail -5 $OUT/pmc_summary.log
echo done
