#!/bin/bash
# r05m: GPU suite, default bench + same-run rocprofv3 (tools/gpu_round.sh), and the config-5
# step's PMC (tools/pmc_train.sh, fp32 and fp64, B = 128) on the round's final kernels.
# usage: tools/r05_gpu_m.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05m}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit $rc; fi
STEPS="bench_default prof_default" bash tools/gpu_round.sh $TAG || exit 3
for dt in f32 f64; do
  bash tools/pmc_train.sh $OUT/pmc_train_$dt --model v24 --code toric_7 --batch 128 --dtype $dt --configs off || exit 3
  python - "$OUT/pmc_train_$dt/summary.json" "$OUT/pmc_train_v24_B128_${dt}_$TAG.json" "$dt" "$TAG" <<'PY'
import json, sys
src, dst, dt, tag = sys.argv[1:5]
d = json.load(open(src))
json.dump({'tag': f'train_v24_toric7_B128_{dt}',
           'command': f'tools/pmc_train.sh OUT --model v24 --code toric_7 --batch 128 --dtype {dt} --configs off ({tag})',
           'per_dispatch_mean': d}, open(dst, 'w'), indent=1, sort_keys=True)
for k, v in d.items():
    if 'v24_bwd' in k or 'decode_kernel' in k:
        print(dt, k[:60], {c: round(x, 3) for c, x in v.items() if c.startswith('frac')})
PY
done
echo done
