#!/bin/bash
# Compare decoder plan variants (env overrides) on one workload in fresh processes.
# usage: tools/variant_sweep.sh [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {
  echo -n "$1  "
  env $1 timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 10 "${@:2}" | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(round(j['value']/1e6,3),'M cw/s  kernel_ms', round(j['roofline']['kernel_ms'],3), 'frac', j['roofline'].get('frac'))" || exit $?
}
run GNND_DEFAULT=1 "$@"
run GNND_NO_RESIDENT=1 "$@"
run GNND_RESIDENT_Q=3 "$@"
run GNND_RESIDENT_Q=6 "$@"
run GNND_RESIDENT_Q=9 "$@"
run GNND_RESIDENT_Q=12 "$@"
