#!/bin/bash
# r05q: rehearsal of the driver's N-rank flow on the one-GPU box with this round's bench.py:
# torchrun --nproc-per-node 2 bench.py --gpus 2 over gloo (RCCL refuses two ranks on one GPU),
# both ranks on the same MI355X.  usage: tools/r05_gpu_q.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r05q}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
GNND_BENCH_BACKEND=gloo GNND_BENCH_FULL=$OUT/rehearsal_full.json timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 > $OUT/rehearsal.log 2>&1
rc=$?
tail -c 7000 $OUT/rehearsal.log | tail -1 > $OUT/rehearsal_line.json
python -c "
import json; d=json.load(open('$OUT/rehearsal_line.json'))
print('n_gpus', d['n_gpus'], 'value', d['value'], 'len', len(json.dumps(d)), 'dist', d.get('dist'))
for k, v in d['configs'].items(): print(k, v.get('value'), v.get('ms_per_step'))
"
echo "rc=$rc"
exit $rc
