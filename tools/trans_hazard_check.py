#!/usr/bin/env python3
"""Scan gfx950 device assembly (hipcc --cuda-device-only -S) for a transcendental result
(v_exp/v_log/v_rcp/... _f32) read by the very next instruction without an s_nop.

The compiler's hazard recognizer inserts the TRANS -> VALU-use wait state for its own
instructions, but an inline-asm consumer can slip through: a `v_max_f32` asm reading a
`__builtin_amdgcn_logf` result right after the v_log read a stale register in some lanes
(wrong training gradients, caught by tests/test_gpu_training.py).  Every kernel in csrc/
must report 0 immediate uses.
usage: tools/trans_hazard_check.py file.s ...   (exit 1 if any immediate use is found)"""
import re
import sys


def scan(fn):
    lines = open(fn).read().split('\n')
    bad = tot = 0
    for i, line in enumerate(lines):
        m = re.match(r'\s+v_(log|exp|rcp|rsq|sqrt|sin|cos)_f32\S*\s+(v\d+),', line)
        if not m:
            continue
        reg, tot = m.group(2), tot + 1
        j = i + 1
        while j < len(lines) and (lines[j].strip().startswith(';') or not lines[j].strip()):
            j += 1
        nxt = lines[j].strip() if j < len(lines) else ''
        if nxt.startswith('s_nop'):
            continue
        parts = nxt.split(None, 1)
        srcs = parts[1].split(',', 1)[1] if len(parts) > 1 and ',' in parts[1] else ''
        if re.search(r'\b' + reg + r'\b', srcs):
            bad += 1
            print(f'{fn}: {line.strip()}  ->  {nxt}')
    print(f'{fn}: {tot} transcendental ops, {bad} immediate uses')
    return bad


if __name__ == '__main__':
    sys.exit(1 if sum(scan(f) for f in sys.argv[1:]) else 0)
