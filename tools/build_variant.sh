#!/bin/bash
# Build a tuning variant of libgnnd.so with extra compile flags (for GNND_LIB sweeps).
# usage: tools/build_variant.sh NAME "-DFLAG ..."   -> gnn-decode_amd/gnndecode/libgnnd_NAME.so
set -e
cd "$(dirname "$0")/../gnn-decode_amd"
name=$1; shift
mkdir -p build_$name
pids=()
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $* -c $f -o build_$name/$(basename $f .hip).o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build_$name/*.o -o gnndecode/libgnnd_$name.so
rm -rf build_$name
echo gnndecode/libgnnd_$name.so
