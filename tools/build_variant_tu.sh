#!/bin/bash
# Tuning variant that recompiles only the named translation units with extra flags and links
# them with the release objects in build/ (make first).
# usage: tools/build_variant_tu.sh NAME "TU1 TU2" "-DFLAG ..."  -> gnndecode/libgnnd_NAME.so
set -e
cd "$(dirname "$0")/../gnn-decode_amd"
name=$1; tus=$2; flags=$3
mkdir -p build_$name
cp build/*.o build_$name/
pids=()
for t in $tus; do
  x=""
  case $t in gnnd_decode_cgnni|gnnd_decode_qgnni|gnnd_decode_cbp|gnnd_decode_qbp|gnnd_decode_nbp|gnnd_decode_v10|gnnd_decode_v22) x=-fno-slp-vectorize;; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DGNND_TUNING $x $flags -c csrc/$t.hip -o build_$name/$t.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build_$name/*.o -o gnndecode/libgnnd_$name.so
rm -rf build_$name
echo gnndecode/libgnnd_$name.so
