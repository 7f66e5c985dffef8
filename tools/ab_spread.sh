#!/bin/bash
# Same-box A/B of the x-layout slot spreading (gnnd_graph.hip spread_check_slots) on the
# headline decode: alternating runs with and without GNND_NO_SLOT_SPREAD=1.
# usage: tools/ab_spread.sh OUT [reps] [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=$1; REPS=${2:-3}; shift 2 || shift $#
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for i in $(seq "$REPS"); do
  for mode in spread nospread; do
    if [ $mode = nospread ]; then export GNND_NO_SLOT_SPREAD=1; else unset GNND_NO_SLOT_SPREAD; fi
    timeout -k 10 300 python bench.py --configs off --cpu-seconds 0 "$@" > /tmp/ab.json 2> /tmp/ab.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "bench failed rc $rc"; tail -5 /tmp/ab.err; exit $rc; fi
    python -c "import json,sys; j=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1]); print('$mode', j['config']['workload'], round(j['value']/1e6,3), 'M', round(j['roofline']['kernel_ms'],4), 'ms', round(j['roofline']['frac'],4))" >> "$OUT"
  done
done
unset GNND_NO_SLOT_SPREAD
cat "$OUT"
