#!/bin/bash
# Build a tuning variant of libgnnd.so with extra compile flags (for GNND_LIB sweeps).
# usage: tools/build_variant.sh NAME "-DFLAG ..."   -> gnn-decode_amd/gnndecode/libgnnd_NAME.so
set -e
cd "$(dirname "$0")/../gnn-decode_amd"
name=$1; shift
mkdir -p build_$name
pids=()
for f in csrc/*.hip; do
  x=""   # the Makefile's per-TU flags (XFLAGS_*)
  case $(basename $f .hip) in gnnd_decode_cgnni|gnnd_decode_qgnni|gnnd_decode_cbp|gnnd_decode_qbp|gnnd_decode_nbp|gnnd_decode_v10|gnnd_decode_v22) x=-fno-slp-vectorize;; esac
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DGNND_TUNING $x $* -c $f -o build_$name/$(basename $f .hip).o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 build_$name/*.o -o gnndecode/libgnnd_$name.so
rm -rf build_$name
echo gnndecode/libgnnd_$name.so
