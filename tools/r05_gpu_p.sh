#!/bin/bash
# r05p: A/B of the software-pipelined fp64 decoder_v2_4 MLP (libgnnd_pipe.so: -DGNND_F64_PIPE=1)
# on config 3, then the decoder_v2_4 GPU tests on the variant.  usage: tools/r05_gpu_p.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05p}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
C3="--model v24 --code toric_5 --dtype f64 --steps 10 --warmup 2 --configs off"
bash tools/ab_var.sh pipe "" "$C3" 3 > $OUT/ab_pipe_c3.txt 2>&1 || exit 3
PYTEST="tests/test_gpu_parity.py tests/test_gpu_at_size.py -k v24" bash tools/ab_var.sh pipe "" "$C3" 1 > $OUT/ab_pipe_tests.txt 2>&1
cat $OUT/ab_*.txt
echo done
