#!/usr/bin/env python3
"""Static instruction mix of device kernels in a hipcc -S assembly file: per kernel whose
mangled name matches REGEX, counts of VALU / packed / transcendental / LDS / SALU ops.
usage: tools/asm_stats.py file.s REGEX [file2.s]   (two files: side-by-side totals)"""
import re
import sys


def kernels(path):
    s = open(path).read()
    out = {}
    for m in re.finditer(r'^(_Z[^:\s]+):', s, re.M):
        name = m.group(1)
        end = s.find('.Lfunc_end', m.end())
        body = s[m.end():end]
        ins = [l.split()[0] for l in body.split('\n')
               if l.startswith('\t') and l.strip() and not l.strip().startswith(('.', ';'))]
        out[name] = ins
    return out


def classify(ins):
    c = {'valu': 0, 'pk': 0, 'trans': 0, 'ds_read': 0, 'ds_write': 0, 'salu': 0, 'dpp': 0, 'total': len(ins)}
    for op in ins:
        if op.startswith('v_'):
            c['valu'] += 1
            if op.startswith('v_pk_'):
                c['pk'] += 1
            if re.match(r'v_(exp|log|rcp|rsq|sqrt|sin|cos)_f32', op):
                c['trans'] += 1
            if '_dpp' in op:
                c['dpp'] += 1
        elif op.startswith('ds_read'):
            c['ds_read'] += 1
        elif op.startswith('ds_write'):
            c['ds_write'] += 1
        elif op.startswith('s_'):
            c['salu'] += 1
    return c


def main():
    pat = re.compile(sys.argv[2])
    files = [sys.argv[1]] + sys.argv[3:]
    ks = [kernels(f) for f in files]
    for name in sorted(ks[0]):
        if not pat.search(name):
            continue
        row = [classify(k.get(name, [])) for k in ks]
        print(name[:110])
        for f, c in zip(files, row):
            print('   ', f, c)


if __name__ == '__main__':
    main()
