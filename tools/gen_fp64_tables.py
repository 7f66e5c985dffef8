#!/usr/bin/env python3
"""Tables of the table-driven fp64 exp / log1p used by the fp64 Softplus (gnnd_common.h,
kExpTab / kLogTab).  Values are computed with 60-digit decimal arithmetic and rounded to
the nearest double (float(Decimal) rounds correctly); printed as C hex-float literals.

  kExpTab[j] = 2^(j/256),                   j = 0..255
  kLogTab[2j] = r_j = RN(1 / (1 + j/256)),  kLogTab[2j+1] = RN(-ln r_j)   (exact r_j), j = 0..256
  kSpTab[2j] = RN(ln(1 + e^-a_j)), kSpTab[2j+1] = RN(1 / (1 + e^a_j)),   a_j = j/64, j = 0..2048;
      entry 2049 = (0, 0)  (the fp64 decoder_v2_4 Softplus: softplus_sp / sp_and_grad_n)

usage: python tools/gen_fp64_tables.py   (prints the two C arrays)"""
from decimal import Decimal, getcontext

getcontext().prec = 60


def main():
    exp_tab = [float(Decimal(2) ** (Decimal(j) / 256)) for j in range(256)]
    log_tab = []
    for j in range(257):
        c = Decimal(1) + Decimal(j) / 256
        r = float(Decimal(1) / c)                    # the double r_j
        lr = -(Decimal(r).ln())                      # -ln of the EXACT double r_j
        log_tab += [r, float(lr)]
    print('__constant__ static const double kExpTab[256] = {')
    for i in range(0, 256, 4):
        print('    ' + ', '.join(v.hex() for v in exp_tab[i:i + 4]) + ',')
    print('};')
    print('__constant__ static const double kLogTab[514] = {')
    for i in range(0, 514, 4):
        print('    ' + ', '.join(v.hex() for v in log_tab[i:i + 4]) + ',')
    print('};')
    sp = []
    for j in range(2049):
        ea = (Decimal(j) / 64).exp()
        sp += [float((Decimal(1) + Decimal(1) / ea).ln()), float(Decimal(1) / (Decimal(1) + ea))]
    sp += [0.0, 0.0]
    print('__constant__ static const double kSpTab[4100] = {')
    for i in range(0, 4100, 4):
        print('    ' + ', '.join(v.hex() for v in sp[i:i + 4]) + ',')
    print('};')


if __name__ == '__main__':
    main()
