#!/bin/bash
# r05b: the GPU suite on the new tree, then A/Bs: headline MLP-asm / 128-thread variants,
# config-5 unit-pair forward (GNND_V24_UPAIR=0 vs default), config 3 after the sp_poly change
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/r05b; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit $rc; fi
ab_train() {  # tag env args
  for rep in 1 2; do
    for mode in base var; do
      if [ $mode = var ]; then e="$2"; else e=""; fi
      env $e timeout -k 10 200 python bench.py --mode train --cpu-seconds 0 $3 > $OUT/t.log 2>&1 || { echo "train fail"; tail -5 $OUT/t.log; return 3; }
      grep '^{' $OUT/t.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$1', '$mode', j['config']['workload'][:50], 'ms', j['ms_per_step'])" | tee -a $OUT/ab_train.txt
    done
  done
}
ab_train b128 "GNND_V24_UPAIR=0" "--batch 128 --steps 200 --warmup 5" || exit 3
ab_train b16 "GNND_V24_UPAIR=0" "--batch 16 --steps 200 --warmup 5" || exit 3
ab_train b1024 "GNND_V24_UPAIR=0" "--batch 1024 --steps 50 --warmup 3" || exit 3
bash tools/ab_var.sh oneasm "" "--configs off --steps 200" 3 > $OUT/ab_oneasm.txt 2>&1 || exit 3
cat $OUT/ab_oneasm.txt
bash tools/ab_var.sh blk128 "GNND_LDS_TARGET=20480" "--configs off --steps 200" 2 > $OUT/ab_blk128.txt 2>&1 || exit 3
cat $OUT/ab_blk128.txt
timeout -k 10 300 python bench.py --model v24 --code toric_5 --dtype f64 --steps 10 --warmup 2 --prewarm-s 0.3 --configs off --cpu-seconds 0 > $OUT/c3.log 2>&1 && grep '^{' $OUT/c3.log | tail -1 | cut -c1-300
echo done
