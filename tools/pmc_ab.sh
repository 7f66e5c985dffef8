#!/bin/bash
# PMC instruction/stall counters of the bench kernel with and without an env knob.
# usage: tools/pmc_ab.sh OUTDIR KNOB=VALUE [bench args...]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT="$1"; KNOB="$2"; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
for mode in base knob; do
  for grp in "sq1:SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY" \
             "sq2:SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"; do
    name=${grp%%:*}; ctrs=${grp#*:}
    if [ $mode = knob ]; then export "$KNOB"; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/$mode.$name" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-seconds 0 "$@" > "$OUT/$mode.$name.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "FAIL $mode $name rc $rc"; tail -5 "$OUT/$mode.$name.log"; exit $rc; fi
    if [ $mode = knob ]; then unset "${KNOB%%=*}"; fi
  done
done
python - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for mode in ('base', 'knob'):
    acc = collections.defaultdict(list)
    for f in glob.glob(f'{out}/{mode}.*/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'decode' not in r.get('Kernel_Name', ''): continue
            acc[(r['Counter_Name'], r.get('Dispatch_Id'))].append(float(r['Counter_Value']))
    tot = collections.defaultdict(list)
    for (c, d), v in acc.items(): tot[c].append(sum(v))
    print(mode, {c: '%.4g' % (sum(v) / len(v)) for c, v in sorted(tot.items())})
PY
