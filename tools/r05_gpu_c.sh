#!/bin/bash
# r05 GPU round: the GPU suite, the headline pruning A/B (libgnnd_noprune.so), config-5 step times
# f32/f64 at B = 16/128/1024, then the driver's default bench and the same command under rocprofv3
# (tools/gpu_round.sh steps bench_default / prof_default).  usage: tools/r05_gpu_c.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05c}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit $rc; fi
if [ -f gnn-decode_amd/gnndecode/libgnnd_noprune.so ]; then
  bash tools/ab_var.sh noprune "" "--configs off --steps 200" 3 > $OUT/ab_noprune.txt 2>&1 || exit 3
  cat $OUT/ab_noprune.txt
fi
for dt in f32 f64; do
  for b in 16 128 1024; do
    st=200; [ $b = 1024 ] && st=50
    timeout -k 10 200 python bench.py --mode train --dtype $dt --batch $b --steps $st --warmup 5 --cpu-seconds 0 > $OUT/t.log 2>&1 || { echo "train fail"; tail -5 $OUT/t.log; exit 3; }
    grep '^{' $OUT/t.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$dt', $b, 'ms', j['ms_per_step'], 'kernel_ms', (j.get('roofline') or {}).get('kernel_ms'))" | tee -a $OUT/train.txt
  done
done
STEPS="bench_default prof_default" bash tools/gpu_round.sh $TAG
echo done
