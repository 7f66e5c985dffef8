#!/bin/bash
# Compare tuning builds (GNND_LIB=...) x resident plan overrides on one workload.
# usage: tools/lib_sweep.sh "ENV1" "ENV2" ... -- [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cfgs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do cfgs+=("$1"); shift; done
[ "$1" == "--" ] && shift
for c in "${cfgs[@]}"; do
  echo -n "$c  "
  env $c timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 10 "$@" | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(round(j['value']/1e6,3),'M cw/s  cw/wg', j['config']['codewords_per_workgroup'], 'kernel_ms', round(j['roofline']['kernel_ms'],3))" || exit $?
done
