#!/bin/bash
# A/B of the default libgnnd.so against a tuning build (tools/build_variant.sh NAME FLAGS ->
# gnn-decode_amd/gnndecode/libgnnd_NAME.so, loaded through GNND_LIB), two runs each, on the
# workloads below.  usage: tools/build_variant.sh nopf "-DGNND_NO_PAIR_PREFETCH ..." &&
#                          tools/ab_lib.sh   (variant name nopf hard-wired below)
set -u
mkdir -p gpurun_out/ab
for a in "--model cgnni" "--model qgnni --code toric_5" "--model cgnni --code ldpc_648_324 --batch 131072 --steps 40" "--model cbp"; do
  for rep in 1 2; do
    for lib in base nopf; do
      if [ $lib = nopf ]; then export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_nopf.so; else unset GNND_LIB; fi
      timeout -k 10 120 python bench.py $a --cpu-seconds 0 > gpurun_out/ab/b.log 2>&1 || exit $?
      tail -1 gpurun_out/ab/b.log | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('$lib', j['config']['workload'][:30], round(j['value']/1e6,2))"
    done
  done
done
