#!/bin/bash
# fp64 decoder_v2_4 (config 3 at reference precision): V24 GPU parity tests (release and debug
# builds), then the toric-5 B=65536 and toric-7 B=16384 fp64 decode lines and a rocprofv3
# kernel summary of the toric-5 line.  usage: tools/v24_f64_check.sh OUTDIR
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
fail() { echo "FAIL $1 rc $2"; tail -20 "$OUT/$1.log"; exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "v24 or V24 or debug" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || fail pytest $rc
line() {  # tag args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$tag.log" 2>&1 || fail "$tag" $?
  grep '^{' "$OUT/$tag.log" | tail -1 > "$OUT/$tag.json"
  python -c "import json; d=json.load(open('$OUT/$tag.json')); print('$tag', '%.4g' % d['value'], round(d['ms_per_step'], 3), d['roofline'] and d['roofline'].get('frac'), (d.get('cpu_baseline') or {}).get('hard_decision_mismatches'))"
}
line c3_v24_toric5_f64 --model v24 --code toric_5 --dtype f64 --steps 10 --warmup 2 --cpu-seconds 20
line v24_toric7_f64 --model v24 --code toric_7 --dtype f64 --batch 16384 --steps 10 --warmup 2 --cpu-seconds 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --model v24 --code toric_5 --dtype f64 --steps 10 --warmup 2 --cpu-seconds 0 > "$OUT/prof.log" 2>&1 || fail prof $?
echo done
