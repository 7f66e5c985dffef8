#!/bin/bash
# r05f: GPU suite after the variable-cache fix, then workgroup-size A/Bs (512 / 1024 threads) on
# the headline and LDPC, and the default bench + same-run rocprofv3.  usage: tools/r05_gpu_f.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05f}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit $rc; fi
L="--code ldpc_648_324 --batch 131072 --steps 30 --configs off"
bash tools/ab_var.sh blk512 "GNND_LDS_TARGET=81920" "--configs off --steps 200" 2 > $OUT/ab_blk512.txt 2>&1 || exit 3
bash tools/ab_var.sh blk1024 "GNND_LDS_TARGET=163840" "--configs off --steps 200" 2 > $OUT/ab_blk1024.txt 2>&1 || exit 3
bash tools/ab_var.sh blk512 "GNND_LDS_TARGET=81920" "$L" 2 > $OUT/ab_blk512_ldpc.txt 2>&1 || exit 3
bash tools/ab_var.sh blk1024 "GNND_LDS_TARGET=163840" "$L" 2 > $OUT/ab_blk1024_ldpc.txt 2>&1 || exit 3
cat $OUT/ab_*.txt
STEPS="bench_default prof_default" bash tools/gpu_round.sh $TAG || exit 3
echo done
