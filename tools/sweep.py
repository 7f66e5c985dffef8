#!/usr/bin/env python3
"""Run bench.py over several (model, code, dtype, batch) workloads; print a table.
usage: python tools/sweep.py [--steps K]"""
import json
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [
    ('cgnni', 'bch_63_45', 'f32', 65536),
    ('cbp', 'bch_63_45', 'f32', 65536),
    ('v24', 'toric_5', 'f32', 65536),
    ('v24', 'toric_7', 'f32', 16384),
    ('qbp', 'toric_5', 'f32', 65536),
    ('qgnni', 'toric_5', 'f32', 65536),
    ('cgnni', 'ldpc_648_324', 'f32', 16384),
    ('cbp', 'ldpc_648_324', 'f32', 16384),
    ('v24', 'toric_5', 'f64', 8192),
]


def main():
    steps = sys.argv[sys.argv.index('--steps') + 1] if '--steps' in sys.argv else '5'
    for model, code, dt, B in CASES:
        cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--model', model, '--code', code,
               '--dtype', dt, '--batch', str(B), '--steps', steps, '--warmup', '2',
               '--cpu-seconds', '0']
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        line = [l for l in r.stdout.splitlines() if l.startswith('{')]
        if r.returncode != 0 or not line:
            print(f'{model:6s} {code:14s} {dt} B={B}: FAILED rc={r.returncode}\n{r.stderr[-2000:]}', flush=True)
            if r.returncode < 0 or r.returncode >= 124:
                sys.exit(r.returncode)
            continue
        j = json.loads(line[-1])
        rf = j['roofline']
        print(f"{model:6s} {code:14s} {dt} B={B:6d}: {j['value']/1e6:9.3f} M cw/s  kernel {rf['kernel_ms']:8.3f} ms  "
              f"{rf['achieved']:7.2f} TFLOP/s ({100*rf['frac']:5.1f}%)  cw/wg={j['config']['codewords_per_workgroup']} "
              f"err={j['config']['hard_decision_error_rate']:.4f}", flush=True)


if __name__ == '__main__':
    main()
