#!/bin/bash
# config-5 single-GPU step-time curve (tools/runs/train_curve.txt: B = 16 ... 1024, plus 2048,
# 4096, 8192), one JSON line per batch into OUT/train_curve.jsonl.  usage: tools/train_curve.sh OUT
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$1"; mkdir -p "$OUT"; : > "$OUT/train_curve.jsonl"
for b in 16 32 64 128 256 512 1024 2048 4096 8192; do
  timeout -k 10 200 python bench.py --mode train --batch $b --steps 30 --warmup 3 --cpu-seconds 0 > "$OUT/b$b.log" 2>&1 || { tail -5 "$OUT/b$b.log"; exit 1; }
  grep '^{' "$OUT/b$b.log" | tail -1 >> "$OUT/train_curve.jsonl"
done
echo done
