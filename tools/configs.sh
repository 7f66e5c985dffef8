#!/bin/bash
# One bench.py line per BASELINE.json config (1 GPU), each with roofline + cpu_baseline.
# usage: tools/configs.sh OUTDIR
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$1"; mkdir -p "$OUT"
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$to" python bench.py "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  grep '^{' "$OUT/$name.log" >> "$OUT/configs.jsonl"
  echo "--- $name exit $rc"; tail -2 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
}
: > "$OUT/configs.jsonl"
# config 2 (headline): BCH(63,45) CGNNI, B=65536, fp32 (bench default) and classical BP
run c2_cgnni_bch 600
run c2_cbp_bch 600 --model cbp
run c2_cgnni_bch_bf16 600 --dtype bf16
# config 3: toric d=5 decoder_v2_4, B=65536: fp32 perf mode, fp64 parity mode
run c3_v24_toric5_f32 600 --model v24 --code toric_5 --steps 50
run c3_v24_toric5_f64 900 --model v24 --code toric_5 --dtype f64 --steps 10 --warmup 2 --cpu-seconds 20
# config 4: LDPC(648,324) per-GPU shard of the 1M-codeword job (131072 per GPU), CGNNI and BP
run c4_cgnni_ldpc 600 --code ldpc_648_324 --batch 131072 --steps 50
run c4_cbp_ldpc 600 --model cbp --code ldpc_648_324 --batch 131072 --steps 50
# quantum BP / QGNNI (quantum/BP.py, quantum/QGNNI.py) on toric d=5: fp32 and the reference fp64
run qbp_toric5_f32 600 --model qbp --code toric_5 --steps 100
run qbp_toric5_f64 600 --model qbp --code toric_5 --dtype f64 --steps 20 --cpu-seconds 5
run qgnni_toric5_f32 600 --model qgnni --code toric_5 --steps 100
run qgnni_toric5_f64 600 --model qgnni --code toric_5 --dtype f64 --steps 20 --cpu-seconds 5
# weighted (neural) BP, quantum/neural_BP.py at the reference L = 4 and at L = 5
run nbp_toric4_f32 600 --model nbp --code toric_4 --steps 50
run nbp_toric5_f64 600 --model nbp --code toric_5 --dtype f64 --steps 20 --cpu-seconds 5
# edge-type weighted BP with per-layer readout (quantum/decoder_v2_2.py: L = 6, Nc = 25)
run v22_toric6_f64 600 --model v22 --code toric_6 --dtype f64 --steps 20 --cpu-seconds 5
run v22_toric6_f32 600 --model v22 --code toric_6 --steps 50 --cpu-seconds 5
# GRU edge-state decoder (quantum/decoder_v3_0.py) on toric d=5
run v30_toric5_f64 600 --model v30 --code toric_5 --dtype f64 --steps 20 --cpu-seconds 5
# config 5: toric d=7 decoder_v2_4 training step (1 GPU shard)
run c5_train_v24_toric7 600 --mode train --batch 128 --steps 20 --warmup 3
run train_nbp_toric4 600 --mode train --model nbp --code toric_4 --batch 128 --steps 20 --warmup 3
echo "=== configs done"
