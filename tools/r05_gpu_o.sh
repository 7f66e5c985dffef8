#!/bin/bash
# r05o: the round's final tree: GPU suite, smoke(), default bench + same-run rocprofv3.
# usage: tools/r05_gpu_o.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05o}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -5 $OUT/smoke.txt; exit 3; }
tail -3 $OUT/smoke.txt
STEPS="bench_default prof_default" bash tools/gpu_round.sh $TAG || exit 3
echo done
