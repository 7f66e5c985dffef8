#!/bin/bash
# fp32 decoder_v2_4 unit split (decode_kernel US = 2 / 4 at one codeword per workgroup):
# parity tests of the V24 paths, then the training step and small/large decodes with the
# default split against GNND_V24_SPLIT=1, and a rocprofv3 kernel summary of the B = 128 step.
# usage: tools/v24_split_ab.sh OUTDIR
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
fail() { echo "FAIL $1 rc $2"; tail -20 "$OUT/$1.log"; exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "(v24 or V24 or train or Train) and not debug" > "$OUT/pytest_v24.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_v24.log"; [ $rc -eq 0 ] || fail pytest_v24 $rc
: > "$OUT/ab.jsonl"
line() {  # tag knob args...
  local tag=$1 knob=$2; shift 2
  env $knob timeout -k 10 300 python bench.py --cpu-seconds 0 "$@" > "$OUT/$tag.log" 2>&1 || fail "$tag" $?
  grep '^{' "$OUT/$tag.log" | tail -1 | sed "s/^{/{\"ab\": \"$tag\", /" >> "$OUT/ab.jsonl"
  python -c "import json; d=json.loads(open('$OUT/ab.jsonl').readlines()[-1]); print('$tag', '%.4g' % d['value'], round(d['ms_per_step'], 4))"
}
for b in 16 128 256 512; do
  line train_b${b}_split GNND_V24_SPLIT=0 --mode train --batch $b --steps 30 --warmup 3
  line train_b${b}_nosplit GNND_V24_SPLIT=1 --mode train --batch $b --steps 30 --warmup 3
done
line dec_t5_b128_split GNND_V24_SPLIT=0 --model v24 --code toric_5 --batch 128 --steps 50 --warmup 5
line dec_t5_b128_nosplit GNND_V24_SPLIT=1 --model v24 --code toric_5 --batch 128 --steps 50 --warmup 5
line dec_t5_b65536 GNND_V24_SPLIT=0 --model v24 --code toric_5 --steps 10 --warmup 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --mode train --batch 128 --steps 30 --warmup 3 --cpu-seconds 0 > "$OUT/prof.log" 2>&1 || fail prof $?
echo done
