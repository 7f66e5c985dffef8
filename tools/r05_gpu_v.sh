#!/bin/bash
# r05v: the default bench + same-run rocprofv3 with the refreshed PMC files in profiles/.
# usage: tools/r05_gpu_v.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05v}
export TMPDIR=/tmp
STEPS="bench_default prof_default" bash tools/gpu_round.sh $TAG || exit 3
echo done
