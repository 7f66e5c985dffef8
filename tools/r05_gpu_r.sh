#!/bin/bash
# r05r: config 3 (toric-5 decoder_v2_4 fp64, B = 65 536) with wide workgroups
# (GNND_V24F64_WIDE = 2: 512 item lanes, 2 per CU; 4: 1 024 lanes, 1 per CU) vs the default
# (256 lanes, 3 per CU), then the fp64 decoder_v2_4 GPU tests under each setting.
# usage: tools/r05_gpu_r.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05r}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
C3="--model v24 --code toric_5 --dtype f64 --steps 10 --warmup 2 --configs off --cpu-seconds 0"
for rep in 1 2 3; do
  for w in 1 2 4; do
    GNND_V24F64_WIDE=$w timeout -k 10 300 python bench.py $C3 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 3; }
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); r=j['roofline'] or {}; print('wide$w', j['config']['workload'][:40], '%.4g' % j['value'], 'kernel_ms', r.get('kernel_ms'), 'cw/wg', j['config'].get('codewords_per_workgroup'), 'lds', j['config'].get('lds_bytes_per_workgroup'))" | tee -a $OUT/ab.txt
  done
done
for w in 2 4; do
  GNND_V24F64_WIDE=$w timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_at_size.py -k "v24" > $OUT/pytest_wide$w.txt 2>&1
  echo "wide$w pytest rc=$?"; tail -2 $OUT/pytest_wide$w.txt
done
echo done
