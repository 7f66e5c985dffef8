#!/bin/bash
# r03g: reverse-pass phase breakdown (timing-only builds, tools/train_variant.sh bexpN) at B=128/8192
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${1:-r03g}; mkdir -p $OUT
export TMPDIR=/tmp
: > $OUT/ab.txt
for b in 128 8192; do
  for lib in base bexp1 bexp2 bexp3; do
    if [ $lib = base ]; then unset GNND_LIB; else export GNND_LIB=$ROOT/gnn-decode_amd/gnndecode/libgnnd_$lib.so; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/p_${lib}_$b -o run --output-format csv -- python bench.py --mode train --batch $b --steps 20 --warmup 3 --cpu-seconds 0 > $OUT/${lib}_$b.log 2>&1 || exit 1
    python - "$OUT/p_${lib}_$b" "$lib" "$b" >> $OUT/ab.txt <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
r = {x['Name'][:40]: float(x['AverageNs']) / 1e3 for x in csv.DictReader(open(f))}
print(sys.argv[2], sys.argv[3], {k: round(v, 1) for k, v in r.items() if 'bwd' in k or 'decode_kernel' in k})
PY
  done
done
unset GNND_LIB
cat $OUT/ab.txt
echo done
