#!/bin/bash
# Run a list of bench.py configurations (one per line of $2, or the default list below),
# appending each JSON line (tagged with its args) to $1.  Each run has its own timeout; a
# crash / timeout ends the script.  usage: tools/bench_lines.sh OUT.jsonl [ARGS_FILE]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=$1
mkdir -p "$(dirname "$OUT")"
if [ $# -ge 2 ]; then mapfile -t RUNS < "$2"; else RUNS=(
  "--steps 200"
  "--dtype bf16 --steps 200"
  "--model cbp --steps 100"
  "--model cgnni --code ldpc_648_324 --batch 131072 --steps 20"
  "--model v24 --code toric_5 --steps 10"
  "--model v24 --code toric_5 --dtype f64 --steps 3 --warmup 1"
  "--model v30 --code toric_5 --dtype f64 --steps 5 --warmup 1"
  "--model v30 --code toric_5 --steps 10"
  "--mode sample --code ldpc_648_324 --batch 131072 --steps 50"
  "--mode sample --code toric_5 --dtype f64 --steps 50"
); fi
for args in "${RUNS[@]}"; do
  [ -z "$args" ] && continue
  echo "=== $args ($(date +%T))"
  timeout -k 10 300 python bench.py $args > "$OUT.tmp" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "FAIL rc=$rc: $args"; tail -5 "$OUT.tmp"; exit $rc; fi
  grep '^{' "$OUT.tmp" | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['args']='$args'; print(json.dumps(d))" >> "$OUT"
  tail -1 "$OUT" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline') or {}; c=d.get('cpu_baseline') or {}; print('   ', '%.4g' % d['value'], d['unit'], 'frac', r.get('frac'), 'kernel_ms', r.get('kernel_ms'), 'ber', d['config'].get('hard_decision_error_rate'), 'cpu', c.get('value'), 'mism', c.get('parity_hard_decision_mismatches'))"
done
rm -f "$OUT.tmp"
echo "=== done"
