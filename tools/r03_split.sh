#!/bin/bash
# r03: component split + fused epilogue: GPU tests, then the config-5 step curve (split and,
# for reference, GNND_NO_SPLIT=1) and a rocprof summary of the B=16 / B=128 steps.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG="${1:-r03a}"
OUT="gpurun_out/$TAG"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_training.py tests/test_gpu_at_size.py tests/test_gpu_parity.py -k "v24 or split or train or fused" -m gpu -v \
  --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -le 1 ] || exit $rc
: > "$OUT/curve.jsonl"; : > "$OUT/curve_nosplit.jsonl"
for b in 16 32 64 128 256 512 1024 2048 4096 8192; do
  timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > "$OUT/b$b.log" 2>&1 || { tail -5 "$OUT/b$b.log"; exit 1; }
  grep '^{' "$OUT/b$b.log" | tail -1 >> "$OUT/curve.jsonl"
done
for b in 16 128 1024; do
  GNND_NO_SPLIT=1 timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > "$OUT/ns_b$b.log" 2>&1 || { tail -5 "$OUT/ns_b$b.log"; exit 1; }
  grep '^{' "$OUT/ns_b$b.log" | tail -1 >> "$OUT/curve_nosplit.jsonl"
done
for b in 16 128; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_b$b" -o run --output-format csv -- python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > "$OUT/prof_b$b.log" 2>&1 || { tail -5 "$OUT/prof_b$b.log"; exit 1; }
done
echo done
