#!/bin/bash
# Compact bench summaries on the GPU box: each argument is one quoted bench.py argument set
# (decode lines, or "--mode train ..."); one summary line each (value, ms/step, roofline frac,
# BER, oracle-sample parity).  Stops at the first failing run.
# usage: tools/quick_lines.sh OUTDIR "--model cbp" "--mode train --dtype f64 --batch 128" ...
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=$1; shift
mkdir -p "$OUT"
i=0
for a in "$@"; do
  i=$((i + 1))
  timeout -k 10 300 python bench.py $a --cpu-seconds ${CPU_SECONDS:-2} --configs off > "$OUT/line_$i.txt" 2>&1 || { echo "FAIL: $a"; tail -5 "$OUT/line_$i.txt"; exit 3; }
  grep '^{' "$OUT/line_$i.txt" | tail -1 | python -c "
import json, sys
d = json.loads(sys.stdin.read()); r = d.get('roofline') or {}; c = d.get('config') or {}; cb = d.get('cpu_baseline') or {}
par = d.get('parity') or {}
print('%-55s %-4s %12.6g %s ms %8.5f frac %s %s ber %s par %s/%s %s' % (c.get('workload', '')[:55], d['dtype'], d['value'], d['unit'], d['ms_per_step'],
      r.get('bound'), r.get('frac'), c.get('hard_decision_error_rate'), par.get('mismatches', cb.get('parity_hard_decision_mismatches')),
      par.get('bits', cb.get('parity_bits_compared')), par.get('max_abs_err', cb.get('parity_max_abs_err'))))
" | tee -a "$OUT/lines.txt"
done
