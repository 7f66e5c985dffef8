#!/bin/bash
# Same-box A/B of the resident kernel's LDS layout searches (gnnd_graph.hip): slot spreading
# (spread_check_slots, off with GNND_NO_SLOT_SPREAD=1) and T-row placement (place_t_rows, off
# with GNND_NO_TPERM=1), alternating runs of one decode workload.
# usage: tools/ab_spread.sh OUT [reps] [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=$1; REPS=${2:-3}; shift 2 || shift $#
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for i in $(seq "$REPS"); do
  for mode in both none spread tperm; do
    case $mode in
      both)   S=0; P=0;;
      none)   S=1; P=1;;
      spread) S=0; P=1;;
      tperm)  S=1; P=0;;
    esac
    GNND_NO_SLOT_SPREAD=$S GNND_NO_TPERM=$P timeout -k 10 300 python bench.py --configs off --cpu-seconds 0 "$@" > /tmp/ab.json 2> /tmp/ab.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "bench failed rc $rc"; tail -5 /tmp/ab.err; exit $rc; fi
    python -c "import json; j=json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1]); print('$mode', j['config']['workload'], round(j['value']/1e6,3), 'M', round(j['roofline']['kernel_ms'],4), 'ms', round(j['roofline']['frac'],4))" >> "$OUT"
  done
done
cat "$OUT"
