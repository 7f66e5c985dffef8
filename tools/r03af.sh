#!/bin/bash
# r03af: why gnnd_train_fwd_loss declines toric-7 B=16 (debug build prints the plan)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03af}; mkdir -p $OUT
export GNND_LIB=$PWD/gnn-decode_amd/gnndecode/libgnnd_dbg.so
timeout -k 10 200 python - > $OUT/dbg.log 2>&1 <<'PY'
import sys, torch
sys.path.insert(0, 'gnn-decode_amd')
import gnndecode as gd
H = gd.codes.toric_code(7)
m = gd.MODELS['v24'](6, H).to('cuda')
g = m.graph('cuda')
lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H)).to('cuda')
x, y = gd.data.toric_batch(H, 16, seed=16, device='cuda')
prep = gd.ops.prepare_weights('v24', m.packed_weights().detach().contiguous())
r = gd.ops.train_forward_loss(g, 'v24', x, prep, 6, y, lf.logical_mask(x.device), lf.logical_rows.size(0), False)
print('result', None if r is None else [t.shape for t in r])
PY
cat $OUT/dbg.log
