#!/bin/bash
# Sweep the decoder's per-workgroup LDS budget (codewords per workgroup) on one workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for t in 16384 24576 32768 40960 53248 81920; do
  echo -n "LDS_TARGET=$t  "
  GNND_LDS_TARGET=$t timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 10 "$@" | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(round(j['value']/1e6,3),'M cw/s  cw/wg', j['config']['codewords_per_workgroup'], 'kernel_ms', round(j['roofline']['kernel_ms'],3))" || exit $?
done
