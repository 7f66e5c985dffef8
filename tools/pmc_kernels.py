#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc passes (counter_collection.csv files under PMCDIR):
mean per dispatch of every counter (summed over XCD/SE instances of one dispatch), by kernel
(name truncated at the template arguments' first 60 characters).
usage: tools/pmc_kernels.py PMCDIR [OUTJSON] [name-substring ...]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    out_path = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2].endswith('.json') else None
    keep = [a for a in sys.argv[2:] if not a.endswith('.json')]
    vals = defaultdict(float)                     # (kernel, dispatch, counter) -> sum
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get('Kernel_Name', '')
                if keep and not any(s in k for s in keep):
                    continue
                vals[(k[:90], f + ':' + row['Dispatch_Id'], row['Counter_Name'])] += float(row['Counter_Value'])
    per = defaultdict(lambda: defaultdict(list))
    for (k, disp, c), v in vals.items():
        per[k][c].append(v)
    res = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}
    for k, cs in res.items():
        if 'SQ_WAVE_CYCLES' in cs and cs['SQ_WAVE_CYCLES']:
            for c in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU'):
                if c in cs:
                    cs['frac_' + c] = cs[c] / cs['SQ_WAVE_CYCLES']
        if 'SQ_LDS_IDX_ACTIVE' in cs and cs['SQ_LDS_IDX_ACTIVE']:
            cs['frac_lds_bank_conflict'] = cs.get('SQ_LDS_BANK_CONFLICT', 0) / cs['SQ_LDS_IDX_ACTIVE']
    txt = json.dumps(res, indent=1, sort_keys=True)
    if out_path:
        with open(out_path, 'w') as f:
            f.write(txt)
    print(txt)


if __name__ == '__main__':
    main()
