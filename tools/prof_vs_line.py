#!/usr/bin/env python3
"""Cross-check a bench line against the rocprofv3 kernel trace of the SAME run (VERDICT r04
item 3).

usage: prof_vs_line.py <run_kernel_trace.csv> <bench_full.json> [out.json]

bench.py records every timed region's CLOCK_MONOTONIC window (`timed_region_ns`, the clock
rocprofv3 stamps kernels with).  For the headline and each nested config this selects the
kernels that ran inside that window and reports, per kernel, launches, average duration and
time per step; the rule checked is that the dominant kernel's time per step (and the sum over
all kernels per step) does not exceed the line's `ms_per_step`.
"""
import csv
import json
import sys


def load_trace(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    return rows


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0] if '(' in n else n


def window(rows, t0, t1, steps, ms_per_step):
    sel = [(s, e, n) for s, e, n in rows if s >= t0 and e <= t1]
    by = {}
    for s, e, n in sel:
        k = short(n)
        c, tot = by.get(k, (0, 0))
        by[k] = (c + 1, tot + (e - s))
    kern = sorted(({'kernel': k, 'launches': c, 'avg_us': tot / c / 1e3,
                    'ms_per_step': tot / steps / 1e6} for k, (c, tot) in by.items()),
                  key=lambda d: -d['ms_per_step'])
    busy = sum(d['ms_per_step'] for d in kern)
    dom = kern[0] if kern else None
    return {'steps': steps, 'line_ms_per_step': ms_per_step,
            'kernels_ms_per_step': busy,
            'dominant': dom,
            'dominant_le_step': bool(dom and dom['ms_per_step'] <= ms_per_step),
            'all_kernels_le_step': busy <= ms_per_step,
            'gpu_busy_frac': busy / ms_per_step if ms_per_step else None,
            'kernels': kern}


def main():
    rows = load_trace(sys.argv[1])
    full = json.load(open(sys.argv[2]))
    entries = {'headline': full}
    entries.update(full.get('configs') or {})
    out = {}
    for name, r in entries.items():
        w = r.get('timed_region_ns')
        if not w or not w[0]:
            continue
        out[name] = window(rows, w[0], w[1], r['steps'], r['ms_per_step'])
    for name, d in out.items():
        dom = d['dominant']
        print(f"{name:44s} line {d['line_ms_per_step']:.4f} ms/step | kernels {d['kernels_ms_per_step']:.4f}"
              f" | dominant {dom['kernel'] if dom else '-'}: {dom['ms_per_step'] if dom else 0:.4f}"
              f" ms/step, {dom['launches'] if dom else 0} launches, avg {dom['avg_us'] if dom else 0:.1f} us"
              f" | ok={d['dominant_le_step'] and d['all_kernels_le_step']}")
    if len(sys.argv) > 3:
        with open(sys.argv[3], 'w') as f:
            json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
