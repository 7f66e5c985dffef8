#!/bin/bash
# A/B of the fp64 decoder_v2_4 Softplus forms: the default build (one-read kSpTab table) against
# libgnnd_sp0.so (tools/build_variant.sh sp0 "-DGNND_F64_SPTAB=0": exp + log1p tables), two runs
# each, on config 3 (toric-5 fp64 decode, B = 65 536) and the config-5 fp64 training step (B = 128).
set -u
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for lib in base sp0; do
    if [ $lib = sp0 ]; then export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_$lib.so; else unset GNND_LIB; fi
    for a in "--model v24 --code toric_5 --batch 65536 --dtype f64 --steps 10 --warmup 2" \
             "--mode train --model v24 --dtype f64 --batch 128 --steps 50 --warmup 3" \
             "--mode train --model v24 --dtype f64 --batch 1024 --steps 20 --warmup 2"; do
      timeout -k 10 180 python bench.py $a --configs off --cpu-seconds 0 > gpurun_out/ab/b.log 2>&1 || exit $?
      tail -1 gpurun_out/ab/b.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib', j['config']['workload'][:40], j['value'], round(j['ms_per_step'],4), (j.get('roofline') or {}).get('kernel_ms'))"
    done
  done
done
