#!/usr/bin/env python3
"""LDS bank model of the headline kernel's T_v gathers (decode_resident_kernel, BCH(63,45)
CGNNI fp32: G = 8 lanes x R = 3 slots per check, CW = 16 codewords per workgroup, Q = 9 items
per lane): for every item round q, slot r and half-wave, the ds_read_b32 addresses
b * stride + v (4-byte words) of the 32 lanes, banks (a / 4) mod 32 (MI355X_MICROARCH.md
LDS table); prints the mean cycles per half-wave group (1.0 = conflict-free) per codeword
stride.  usage: tools/lds_stride_sweep.py [min_stride max_stride]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gnn-decode_amd'))
import gnndecode as gd  # noqa: E402

G, R, CW, Q = 8, 3, 16, 9


def checks():
    H = np.asarray(gd.codes.bch_63_45())
    H = H.T if H.shape[0] > H.shape[1] else H          # [C, V]
    return [sorted(np.nonzero(H[c])[0]) for c in range(H.shape[0])]


def cycles(chk, stride):
    C = len(chk)
    tot = groups = 0
    for w in range(4):
        for q in range(Q):
            for r in range(R):
                for half in range(2):
                    banks = {}
                    for lane in range(32 * half, 32 * half + 32):
                        f = 64 * w + lane + 256 * q        # item -> (check, codeword, lane)
                        gi = f >> 3
                        c, b = gi // CW, gi % CW
                        k = (f & 7) * R + r
                        if c >= C or k >= len(chk[c]):
                            continue
                        a = b * stride + chk[c][k]
                        banks.setdefault(a % 32, set()).add(a)
                    if banks:
                        tot += max(len(s) for s in banks.values())
                        groups += 1
    return tot / groups


if __name__ == '__main__':
    lo, hi = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (63, 100)
    chk = checks()
    for s in range(lo, hi + 1):
        print(s, round(cycles(chk, s), 3))
