#!/usr/bin/env python3
"""LDS bank-conflict model of decode_resident_kernel (csrc/gnnd_decode_impl.h) for one graph.

Rebuilds the host plan of csrc/gnnd_graph.hip (check-group slot plan with ties to the larger
R, degree-ordered variables, the padded variable-major message layout) and of make_plan
(codewords per workgroup CW, items per lane Q), then walks every LDS wave-instruction of one
decode iteration of one workgroup and prices it with the CDNA4 banking rules of
MI355X_MICROARCH.md §LDS:

  ds_read_b64 (the {S_v, x_v} gathers)  2 groups of 32 lanes, bank = (a/4) mod 64, 8-B access
  ds_read_b32 / ds_read2_b32 (variable sums, per dword)  2 x 32 lanes, bank = (a/4) mod 32
  ds_write_b32 (message and S_v stores)  2 x 32 lanes, bank = (a/4) mod 32

cycles of a group = the largest number of DISTINCT dword addresses on one bank (identical
addresses broadcast); conflict cycles = cycles - 1 per group, summed (SQ_LDS_BANK_CONFLICT);
IDX_ACTIVE ~ all cycles.  Used to choose layouts on the CPU before spending GPU time; the
PMC counters on the box are the arbiter.

usage: python tools/lds_bank_model.py [code] [--sx-stride N] [--e1 N]
"""
import argparse
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gnn-decode_amd'))

BLOCK = 256


def plan(H):
    H = np.asarray(H)
    V, C = H.shape
    v, c = np.nonzero(H)
    E = v.size
    vdeg = np.bincount(v, minlength=V)
    cdeg = np.bincount(c, minlength=C)
    max_dc = cdeg.max()
    best = None
    for R in range(1, 5):                        # ties -> larger R (resident plan)
        need = -(-max_dc // R)
        G = 1
        while G < need:
            G <<= 1
        if G > 64:
            continue
        slots = C * G * R
        if best is None or slots <= best[0]:
            best = (slots, G, R)
    _, G, R = best
    chk_edges = [np.nonzero(c == k)[0] for k in range(C)]   # increasing e (= increasing v)
    slot_e = np.full(C * G * R, -1)
    for k in range(C):
        for i, e in enumerate(chk_edges[k]):
            slot_e[k * G * R + i] = e
    vord = sorted(range(V), key=lambda a: vdeg[a])           # stable by degree
    return dict(V=V, C=C, E=E, G=G, R=R, v=v, c=c, vdeg=vdeg, slot_e=slot_e, vord=vord)


def layout(p, gs):
    """padded variable-major positions for wave groups of gs var_ord entries"""
    V, vord, vdeg = p['V'], p['vord'], p['vdeg']
    vptr = np.concatenate([[0], np.cumsum(vdeg)])
    epos = np.zeros(p['E'], int)
    vstart = np.zeros(V, int)
    vpad = np.zeros(V, int)
    pos = 0
    for j0 in range(0, V, gs):
        grp = vord[j0:j0 + gs]
        dpad = max(vdeg[a] for a in grp)
        for a in grp:
            vstart[a] = pos
            vpad[a] = dpad
            for e in range(vptr[a], vptr[a + 1]):
                epos[e] = pos + e - vptr[a]
            pos += dpad
    return epos, vstart, vpad, pos


def conflicts(addr_dw, mod, groups=((0, 32), (32, 64))):
    """(cycles, conflict cycles) of one wave instruction; addr_dw: dword address per lane
    (None = inactive lane)"""
    cyc = conf = 0
    for lo, hi in groups:
        banks = defaultdict(set)
        for a in addr_dw[lo:hi]:
            if a is not None:
                banks[a % mod].add(a)
        if not banks:
            continue
        m = max(len(s) for s in banks.values())
        cyc += m
        conf += m - 1
    return cyc, conf


def model(H, Q=None, CW=None, sx_stride=None, e1=None, nw=62, pr=print):
    p = plan(H)
    V, C, E, G, R = p['V'], p['C'], p['E'], p['G'], p['R']
    IC = C * G
    if CW is None:   # make_plan for BCH-like graphs: the best-utilisation (CW, Q)
        best = (0, 0, 0)
        for q in (3, 6, 9, 12):
            if q * (2 * R + 2) > 88:
                continue
            cw = min(64, q * BLOCK // IC)
            if cw < 1:
                continue
            u = cw * IC / (q * BLOCK)
            if u > best[0] + 1e-9 or (abs(u - best[0]) < 1e-9 and cw > best[1]):
                best = (u, cw, q)
        _, CW, Q = best
    gs = max(1, 64 // CW)
    epos, vstart, vpad, P = layout(p, gs)
    E1 = e1 if e1 else (P + 1) | 1
    VS = sx_stride if sx_stride else V
    # byte offsets (align16 blocks as the kernel)
    a16 = lambda n: (n + 15) & ~15
    off_m = a16(nw * 4) + a16(V * 8)
    off_sx = off_m + 4 * ((CW * E1 + 1) & ~1)
    dw_m = off_m // 4
    dw_sx = off_sx // 4
    tot = defaultdict(lambda: [0, 0, 0])          # kind -> [instructions, cycles, conflicts]

    def acc(kind, addrs, mod):
        cy, cf = conflicts(addrs, mod)
        t = tot[kind]
        t[0] += 1
        t[1] += cy
        t[2] += cf

    kLogG = G.bit_length() - 1
    for w in range(BLOCK // 64):
        lanes = range(w * 64, w * 64 + 64)
        for q in range(Q):
            for r in range(R):
                rd, wr = [], []
                for t in lanes:
                    f = t + q * BLOCK
                    gi = f >> kLogG
                    cc, b = gi // CW, gi % CW
                    if cc >= C:
                        rd.append(None)
                        wr.append(None)
                        continue
                    e = p['slot_e'][(cc * G + (f & (G - 1))) * R + r]
                    var = p['v'][e] if e >= 0 else 0
                    rd.append(dw_sx + 2 * (b * VS + var))           # 8-B SumX
                    wr.append(dw_m + b * E1 + (epos[e] if e >= 0 else P))
                # ds_read_b64: bank = dword mod 64, each 8-B access spans 2 banks: price by
                # the even dword (a pair of banks behaves as one wide bank)
                acc('sx_read_b64', [None if a is None else a // 2 for a in rd], 32)
                acc('m_write_b32', wr, 32)
        # variable sums (vuni path): vb = t % CW, vi = t // CW, stride 256/CW
        vstep = BLOCK // CW
        for i0 in range(0, V, vstep):
            rows = []
            for t in lanes:
                vb, vi = t % CW, t // CW + i0
                rows.append((vb, p['vord'][vi]) if vi < V else None)
            if all(r is None for r in rows):
                continue
            dp = max(vpad[r[1]] for r in rows if r is not None)
            for k in range(dp):
                acc('vsum_read_b32', [None if r is None else dw_m + r[0] * E1 + vstart[r[1]] + k
                                      for r in rows], 32)
            acc('sx_write_b32', [None if r is None else dw_sx + 2 * (r[0] * VS + r[1]) for r in rows], 32)
    allc = sum(t[1] for t in tot.values())
    allf = sum(t[2] for t in tot.values())
    pr(f'G={G} R={R} Q={Q} CW={CW} gs={gs} P={P} E1={E1} VS={VS}')
    for k, (n, cy, cf) in sorted(tot.items()):
        pr(f'  {k:14s} {n:6d} instr  {cy:7d} cycles  {cf:7d} conflict ({cf / max(cy, 1):.0%})')
    pr(f'  total cycles {allc}  conflict {allf} ({allf / allc:.1%}) per workgroup-iteration')
    return tot, allc, allf


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('code', nargs='?', default='bch_63_45')
    ap.add_argument('--sx-stride', type=int, default=None)
    ap.add_argument('--e1', type=int, default=None)
    a = ap.parse_args()
    from gnndecode import codes
    model(codes.get_code(a.code), sx_stride=a.sx_stride, e1=a.e1)


if __name__ == '__main__':
    main()
