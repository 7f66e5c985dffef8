#!/bin/bash
# Config-3 (toric-5 fp64 decoder_v2_4 decode, B = 65 536) workgroup shapes: the default plan
# (one codeword group per 256-thread workgroup, 80 KB LDS: 2 per CU), GNND_LDS_TARGET=27000 (54 KB:
# 3 per CU), GNND_V24F64_US=2 / 4 (the MLP units split over 2 / 4 waves too).  Two runs each.
set -u
mkdir -p gpurun_out/ab
A="--model v24 --code toric_5 --batch 65536 --dtype f64 --steps 10 --warmup 2 --configs off --cpu-seconds 0"
for rep in 1 2; do
  for v in base t27 us2 us4; do
    unset GNND_LDS_TARGET GNND_V24F64_US
    case $v in t27) export GNND_LDS_TARGET=27000;; us2) export GNND_V24F64_US=2;; us4) export GNND_V24F64_US=4;; esac
    timeout -k 10 180 python bench.py $A > gpurun_out/ab/c3.log 2>&1 || exit $?
    tail -1 gpurun_out/ab/c3.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$v', j['value'], round(j['ms_per_step'],4), (j.get('roofline') or {}).get('kernel_ms'), (j.get('parity') or {}).get('hard_decision_mismatches'))"
  done
done
