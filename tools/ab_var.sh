#!/bin/bash
# A/B of a tuning library (gnndecode/libgnnd_$NAME.so, tools/build_variant_tu.sh) with optional
# extra environment, alternating with the release library over $REPS reps on one bench workload;
# then (PYTEST set) the named GPU tests on the variant.
# usage: [PYTEST="tests/x.py -k y"] tools/ab_var.sh NAME "ENV=V ..." "bench args" [reps]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
name=$1; envs=$2; args=$3; reps=${4:-2}
OUT=gpurun_out/ab_$name; mkdir -p $OUT
for rep in $(seq $reps); do
  for lib in base $name; do
    if [ $lib = base ]; then
      timeout -k 10 300 python bench.py $args --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 3; }
    else
      env GNND_LIB=$ROOT/gnn-decode_amd/gnndecode/libgnnd_$name.so $envs timeout -k 10 300 python bench.py $args --cpu-seconds 0 > $OUT/b.log 2>&1 || { tail -5 $OUT/b.log; exit 3; }
    fi
    grep '^{' $OUT/b.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); r=j['roofline'] or {}; print('$lib', j['config']['workload'][:44], '%.4g' % j['value'], 'kernel_ms', r.get('kernel_ms'), 'frac', r.get('frac'))" | tee -a $OUT/ab.txt
  done
done
if [ -n "${PYTEST:-}" ]; then
  env GNND_LIB=$ROOT/gnn-decode_amd/gnndecode/libgnnd_$name.so $envs timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $PYTEST > $OUT/pytest.log 2>&1
  rc=$?; tail -3 $OUT/pytest.log; exit $rc
fi
