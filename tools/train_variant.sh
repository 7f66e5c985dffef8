#!/bin/bash
# Variant of libgnnd.so with gnnd_train.hip rebuilt under extra flags (the other objects from
# build/): tools/train_variant.sh NAME "-DFLAG=.." -> gnn-decode_amd/gnndecode/libgnnd_NAME.so
set -e
cd "$(dirname "$0")/../gnn-decode_amd"
name=$1; shift
mkdir -p build_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $* -c csrc/gnnd_train.hip -o build_$name/gnnd_train.o
objs=$(ls build/*.o | grep -v gnnd_train.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build_$name/gnnd_train.o -o gnndecode/libgnnd_$name.so
rm -rf build_$name
echo gnndecode/libgnnd_$name.so
