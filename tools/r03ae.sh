#!/bin/bash
# r03ae: syndrome loss in the unit-split forward's epilogue (gnnd_train_fwd_loss): split /
# training GPU tests, then the config-5 step with it (release default) vs the reverse pass's
# loss (GNND_LOSS_IN_FORWARD=0)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03ae}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_training.py tests/test_gpu_at_size.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
: > $OUT/ab.txt
for rep in 1 2 3; do
for lif in 1 0; do
  export GNND_LOSS_IN_FORWARD=$lif
  for b in 16 128 1024; do
    [ $rep -eq 3 ] && [ $b -eq 16 ] && continue
    timeout -k 10 200 python bench.py --mode train --batch $b --steps 40 --warmup 3 --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 1; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('loss_in_forward=$lif', $b, round(j['ms_per_step'],4))" >> $OUT/ab.txt
  done
done
done
unset GNND_LOSS_IN_FORWARD
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_B128 -o run --output-format csv -- python bench.py --mode train --batch 128 --steps 30 --warmup 3 --cpu-seconds 0 > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
cat $OUT/ab.txt
