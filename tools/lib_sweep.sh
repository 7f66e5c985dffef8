#!/bin/bash
# Compare tuning builds (GNND_LIB) x resident plan overrides on one workload.
# usage: tools/lib_sweep.sh [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {
  echo -n "$1  "
  env $1 timeout -k 10 120 python bench.py --cpu-seconds 0 --steps 10 "${@:2}" | python -c "import json,sys; j=json.loads(sys.stdin.read()); print(round(j['value']/1e6,3),'M cw/s  cw/wg', j['config']['codewords_per_workgroup'], 'kernel_ms', round(j['roofline']['kernel_ms'],3), 'err', j['config']['hard_decision_error_rate'])" || exit $?
}
L=gnn-decode_amd/gnndecode
run "GNND_DEFAULT=1" "$@"
for q in 3 6 9; do run "GNND_RESIDENT_Q=$q" "$@"; done
for q in 6 9 12; do run "GNND_LIB=$L/libgnnd_w3.so GNND_RESIDENT_Q=$q" "$@"; done
for q in 6 9 12; do run "GNND_LIB=$L/libgnnd_w3.so GNND_RESIDENT_Q=$q GNND_LDS_TARGET=53000" "$@"; done
for q in 9 12; do run "GNND_LIB=$L/libgnnd_w2.so GNND_RESIDENT_Q=$q GNND_LDS_TARGET=80000" "$@"; done
