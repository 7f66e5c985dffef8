#!/bin/bash
# r05 headline A/Bs: 128-thread workgroups (blk128), the one-asm-block message MLP (oneasm);
# then the CGNNI parity tests on each variant
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
bash tools/ab_var.sh oneasm "" "--configs off --steps 200" 3 || exit $?
bash tools/ab_var.sh blk128 "GNND_LDS_TARGET=20480" "--configs off --steps 200" 2 || exit $?
PYTEST="tests/test_gpu_parity.py tests/test_gpu_at_size.py -k cgnni" bash tools/ab_var.sh oneasm "" "--configs off --steps 20" 1 || exit $?
PYTEST="tests/test_gpu_parity.py tests/test_gpu_at_size.py -k cgnni" bash tools/ab_var.sh blk128 "GNND_LDS_TARGET=20480" "--configs off --steps 20" 1
