#!/bin/bash
# r05k: GPU suite with the reverse pass's fairness priorities on, an A/B of the same idea in the
# unit-split forwards (libgnnd_fwdfair.so: -DGNND_FWD_FAIR=1) on the config-5 step, then the
# default bench + same-run rocprofv3 (tools/gpu_round.sh).  usage: tools/r05_gpu_k.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05k}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit $rc; fi
T5="--mode train --model v24 --code toric_7 --batch 128 --steps 200 --warmup 5 --configs off"
bash tools/ab_var.sh fwdfair "" "$T5 --dtype f32" 3 > $OUT/ab_fwdfair_t5_f32.txt 2>&1 || exit 3
bash tools/ab_var.sh fwdfair "" "$T5 --dtype f64" 3 > $OUT/ab_fwdfair_t5_f64.txt 2>&1 || exit 3
cat $OUT/ab_*.txt
STEPS="bench_default prof_default" bash tools/gpu_round.sh $TAG || exit 3
echo done
