#!/usr/bin/env python3
"""Prototype of the T-layout permutation search for decode_resident_kernel (kTX: fp32 GNN / BP
models): LDS bank model of the per-iteration accesses that depend on where T_v lives
(s_t[b * S + pi(v)]) and on which lane/slot of its check each edge sits in:

  T gathers     ds_read_b32 per (item round q, slot r): lanes (codeword b, group lane g) read
                s_t[b S + pi(v)] of the check's edge at (g, r)
  msg writes    ds_write_b32 per (q, r): s_m[b E1 + pos(e)]
  T writes      ds_write_b32 per variable-step row: 256 / CW consecutive var_ord entries x CW
                codewords write s_t[b S + pi(v)]

A half-wave (32 lanes) is one LDS group; its cost = the largest number of distinct dword
addresses on one bank (a / 4 mod 32).  Searches pi (positions in [0, S)) and per-check slot
permutations by simulated annealing; prints cycles per workgroup-iteration for the identity
layout (S = V) and the best found.  usage: tools/t_perm.py [code] [--S N] [--iters N]"""
import argparse
import math
import os
import random
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gnn-decode_amd'))


def resident_plan(H):
    """(G, R, per-check sorted variable lists, CW, Q) as gnnd_graph / make_plan choose them."""
    H = np.asarray(H)
    V, C = H.shape
    v, c = np.nonzero(H)
    order = np.lexsort((c, v))
    v, c = v[order], c[order]
    cdeg = np.bincount(c, minlength=C)
    best = None
    for R in range(1, 5):
        need = -(-cdeg.max() // R)
        G = 1
        while G < need:
            G <<= 1
        if G > 64:
            continue
        if best is None or C * G * R <= best[0]:
            best = (C * G * R, G, R)
    _, G, R = best
    chk = [list(v[c == k]) for k in range(C)]
    IC = C * G
    bu, CW, Q = 0, 0, 0
    for q in (3, 6, 9, 12):
        if q * (2 * R + 2) > 88:
            continue
        cw = min(64, q * 256 // IC)
        if cw < 1:
            continue
        u = cw * IC / (q * 256)
        if u > bu + 1e-9 or (abs(u - bu) < 1e-9 and cw > CW):
            bu, CW, Q = u, cw, q
    return V, C, G, R, chk, CW, Q, v


def half_cost(addrs):
    banks = {}
    for a in addrs:
        banks.setdefault(a % 32, set()).add(a)
    return max(len(s) for s in banks.values()) if banks else 0


class Model:
    def __init__(self, H, S):
        self.V, self.C, self.G, self.R, self.chk, self.CW, self.Q, ev = resident_plan(H)
        self.S = S
        assert 32 % self.G == 0 or self.G >= 32
        # half-wave groups of the gathers: codeword quads (32 / G consecutive codewords of one check)
        self.nb = max(1, 32 // self.G)
        self.deg = np.bincount(ev, minlength=self.V)

    def gather_cost(self, pi, slots_c):
        """sum over (check, slot r) of the half-wave cost x the number of codeword groups"""
        G, R, nb, S = self.G, self.R, self.nb, self.S
        tot = 0
        for sl in slots_c:
            for r in range(R):
                vs = [sl[g * R + r] for g in range(G) if g * R + r < len(sl)]
                tot += half_cost([b * S + pi[x] for b in range(nb) for x in vs])
        return tot * (self.CW // nb)


def anneal(m, iters, seed=0, S=None):
    rnd = random.Random(seed)
    V, G, R, nb = m.V, m.G, m.R, m.nb
    S = m.S
    pos = list(range(V))            # pi: variable -> position
    free = list(range(V, S))        # unused positions
    slots = [list(x) for x in m.chk]
    # per-(check, r) cost cache
    def cost_cr(c, r):
        sl = slots[c]
        vs = [sl[g * R + r] for g in range(G) if g * R + r < len(sl)]
        return half_cost([b * S + pos[x] for b in range(nb) for x in vs])
    vchecks = [[] for _ in range(V)]
    for c, sl in enumerate(slots):
        for x in sl:
            vchecks[x].append(c)
    cache = {(c, r): cost_cr(c, r) for c in range(m.C) for r in range(R)}
    cur = sum(cache.values())
    start = cur
    T0 = 1.0
    for it in range(iters):
        T = T0 * (1 - it / iters) + 1e-3
        kind = rnd.random()
        if kind < 0.5:
            # swap two slots of one check
            c = rnd.randrange(m.C)
            n = len(slots[c])
            i, j = rnd.randrange(n), rnd.randrange(n)
            if i % R == j % R:
                continue
            slots[c][i], slots[c][j] = slots[c][j], slots[c][i]
            keys = [(c, i % R), (c, j % R)]
            undo = lambda: slots[c].__setitem__(slice(None), slots[c])
            old = sum(cache[k] for k in keys)
            new = {k: cost_cr(*k) for k in keys}
            d = sum(new.values()) - old
            if d <= 0 or rnd.random() < math.exp(-d / T):
                cache.update(new)
                cur += d
            else:
                slots[c][i], slots[c][j] = slots[c][j], slots[c][i]
        else:
            a = rnd.randrange(V)
            if free and rnd.random() < 0.3:
                k = rnd.randrange(len(free))
                old_p = pos[a]
                pos[a], free[k] = free[k], old_p
                keys = {(c, r) for c in vchecks[a] for r in range(R)}
                oldc = sum(cache[kk] for kk in keys)
                new = {kk: cost_cr(*kk) for kk in keys}
                d = sum(new.values()) - oldc
                if d <= 0 or rnd.random() < math.exp(-d / T):
                    cache.update(new)
                    cur += d
                else:
                    free[k], pos[a] = pos[a], old_p
            else:
                b = rnd.randrange(V)
                if a == b:
                    continue
                pos[a], pos[b] = pos[b], pos[a]
                keys = {(c, r) for c in vchecks[a] + vchecks[b] for r in range(R)}
                oldc = sum(cache[kk] for kk in keys)
                new = {kk: cost_cr(*kk) for kk in keys}
                d = sum(new.values()) - oldc
                if d <= 0 or rnd.random() < math.exp(-d / T):
                    cache.update(new)
                    cur += d
                else:
                    pos[a], pos[b] = pos[b], pos[a]
    return start, cur, pos, slots


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('code', nargs='?', default='bch_63_45')
    ap.add_argument('--S', type=int, nargs='*', default=None)
    ap.add_argument('--iters', type=int, default=200000)
    a = ap.parse_args()
    from gnndecode import codes
    H = codes.get_code(a.code)
    V = H.shape[0]
    for S in (a.S or [V]):
        m = Model(H, S)
        ideal = m.C * m.R
        s0, s1, pos, slots = anneal(m, a.iters, S=S)
        print(f'{a.code} G={m.G} R={m.R} CW={m.CW} Q={m.Q} S={S} (S mod 32 = {S % 32}): '
              f'gather half-wave cycles per (check, slot): identity {s0 / ideal:.3f} -> '
              f'{s1 / ideal:.3f} (1.0 = conflict-free)', flush=True)


if __name__ == '__main__':
    main()
