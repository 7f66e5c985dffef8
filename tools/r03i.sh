#!/bin/bash
# r03i: fp64 V24 (degree-3 exp) parity + config-3 line + class counters
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03i}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_at_size.py tests/test_gpu_training.py tests/test_v30.py tests/test_v22.py -k "v24 or f64 or float64" -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --model v24 --code toric_5 --dtype f64 --steps 10 --warmup 2 --cpu-seconds 4 --configs off > $OUT/c3.log 2>&1 || { tail $OUT/c3.log; exit 1; }
grep '^{' $OUT/c3.log | tail -1 > $OUT/c3.json
bash tools/pmc_classes.sh $OUT/pmc_v24f64 --model v24 --code toric_5 --dtype f64 --batch 16384 > $OUT/pmc_v24f64.log 2>&1 || { tail $OUT/pmc_v24f64.log; exit 1; }
echo done
