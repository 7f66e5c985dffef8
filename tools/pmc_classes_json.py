#!/usr/bin/env python3
"""Per-codeword VALU-class counters of one decode kernel for bench.py's issue model, from a
tools/pmc_classes.sh run (its summary.json: per-dispatch means of every counter).

usage: pmc_classes_json.py SUMMARY.json KERNEL_SUBSTRING BATCH TAG SOURCE OUT.json [E T]

Writes {tag, kernel, batch, command, source, per_codeword{counter: value / batch}} — the file
bench.py load_pmc_classes() reads as profiles/pmc_classes_<tag>.json — and prints the wave64
VALU instructions per edge-iteration when E (edges) and T (iterations) are given.
"""
import json
import sys


def main():
    summ, sub, batch, tag, source, out = sys.argv[1:7]
    batch = float(batch)
    data = json.load(open(summ))
    ks = [k for k in data if sub in k]
    if len(ks) != 1:
        raise SystemExit(f'kernel substring {sub!r} matches {ks}')
    cs = data[ks[0]]
    per = {c: v / batch for c, v in cs.items() if c.startswith('SQ_') and not c.startswith('frac_')}
    res = {'tag': tag, 'kernel': ks[0], 'batch': int(batch),
           'command': 'tools/pmc_classes.sh OUT (bench args of the tag)', 'source': source,
           'per_codeword': per,
           'frac_of_wave_cycles': {c: v for c, v in cs.items() if c.startswith('frac_')}}
    if len(sys.argv) > 8:
        E, T = float(sys.argv[7]), float(sys.argv[8])
        res['valu_per_edge_iteration'] = per['SQ_INSTS_VALU'] * 64 / (E * T)
        print('VALU per edge-iteration', res['valu_per_edge_iteration'])
    with open(out, 'w') as f:
        json.dump(res, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
