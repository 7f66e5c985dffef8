#!/bin/bash
# A/B of one environment knob on the decode bench: for each workload, bench with the knob
# unset and set (one JSON line each, tagged), e.g.  tools/ab_env.sh OUT GNND_NO_VLAYOUT=1
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
# the knobs are read by the tuning build only (make -C gnn-decode_amd tuning)
export GNND_LIB="$ROOT/gnn-decode_amd/gnndecode/libgnnd_tuning.so"
OUT="$1"; KNOB="$2"; mkdir -p "$OUT"
: > "$OUT/ab.jsonl"
run() {  # tag args...
  local tag=$1; shift
  for mode in base knob; do
    if [ $mode = knob ]; then env "$KNOB" timeout -k 10 300 python bench.py --cpu-seconds 0 "$@" > "$OUT/$tag.$mode.log" 2>&1
    else timeout -k 10 300 python bench.py --cpu-seconds 0 "$@" > "$OUT/$tag.$mode.log" 2>&1; fi
    local rc=$?
    if [ $rc -ne 0 ]; then echo "FAIL $tag $mode rc $rc"; tail -5 "$OUT/$tag.$mode.log"; exit $rc; fi
    python -c "import json,sys; d=json.loads([l for l in open('$OUT/$tag.$mode.log') if l.startswith('{')][-1]); print('$tag', '$mode', '%.4g' % d['value'], d['roofline'] and d['roofline'].get('kernel_ms'), d['config'].get('codewords_per_workgroup'))" | tee -a "$OUT/ab.txt"
    grep '^{' "$OUT/$tag.$mode.log" | sed "s/^{/{\"ab\": \"$tag.$mode\", /" >> "$OUT/ab.jsonl"
  done
}
if [ "${3:-f32}" = f64 ]; then
  for m in qbp qgnni nbp v10; do run ${m}_toric5_f64 --model $m --code toric_5 --dtype f64 --steps 10 --warmup 2; done
  run cbp_bch_f64 --model cbp --dtype f64 --steps 10 --warmup 2
  run cgnni_bch_f64 --dtype f64 --steps 10 --warmup 2
else
  run cgnni_bch --steps 100
  run cbp_bch --model cbp --steps 100
  run cgnni_ldpc --code ldpc_648_324 --batch 131072 --steps 30
  run cbp_ldpc --model cbp --code ldpc_648_324 --batch 131072 --steps 30
  run qbp_toric5 --model qbp --code toric_5 --steps 100
  run qgnni_toric5 --model qgnni --code toric_5 --steps 100
fi
echo done
