#!/bin/bash
# r05h: GPU suite with the signed table in the fp64 reverse pass too, a same-box A/B against the
# kSpTab reverse pass (libgnnd_spbwd.so) on the fp64 config-5 step, and per-wave phase profiles of
# the config-5 step (libgnnd_prof.so: -DGNND_PHASE_PROF -DGNND_PPROF_ALLWAVES=1, fp32 and fp64).
# usage: tools/r05_gpu_h.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05h}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit $rc; fi
T5="--mode train --model v24 --code toric_7 --batch 128 --dtype f64 --steps 200 --warmup 5 --configs off"
bash tools/ab_var.sh spbwd "" "$T5" 3 > $OUT/ab_spbwd_t5.txt 2>&1 || exit 3
for dt in f32 f64; do
  GNND_LIB=$ROOT/gnn-decode_amd/gnndecode/libgnnd_prof.so timeout -k 10 300 python bench.py --mode train --model v24 --code toric_7 --batch 128 --dtype $dt --steps 3 --warmup 1 --configs off --cpu-seconds 0 > $OUT/prof_$dt.log 2>&1 || { tail -5 $OUT/prof_$dt.log; exit 3; }
  grep PHASE $OUT/prof_$dt.log | tail -40 > $OUT/phase_$dt.txt
done
cat $OUT/ab_*.txt
echo done
