#!/usr/bin/env python3
"""Tables of the table-driven fp64 exp / log1p used by the fp64 Softplus (gnnd_common.h,
kExpTab / kLogTab).  Values are computed with 60-digit decimal arithmetic and rounded to
the nearest double (float(Decimal) rounds correctly); printed as C hex-float literals.

  kExpTab[j] = 2^(j/256),                   j = 0..255
  kLogTab[2j] = r_j = RN(1 / (1 + j/256)),  kLogTab[2j+1] = RN(-ln r_j)   (exact r_j), j = 0..256
  kSpTab[2j] = RN(ln(1 + e^-a_j)), kSpTab[2j+1] = RN(1 / (1 + e^a_j)),   a_j = j/64, j = 0..2048;
      entry 2049 = (0, 0)  (the fp64 decoder_v2_4 reverse pass: sp_and_grad_n)
  kSgTab[2i] = RN(g(c_j)), kSgTab[2i+1] = RN(1/2 - sigmoid(c_j)),  g(h) = softplus(h) - h/2,
      c_j = j * kSgStep (exact real product), j = i - 1281 = -1280..799; entry j = 800 (h >= 20:
      torch's threshold, Softplus = h) = {RN(c/2), -1/2}, entry j = -1281 (h < -32.03) =
      {RN(-c/2), 1/2}  (the fp64 decoder_v2_4 forward: softplus_sg)

usage: python tools/gen_fp64_tables.py   (prints the two C arrays)"""
from decimal import Decimal, getcontext

getcontext().prec = 60

# kSgTab's index scale: the double just below 799.5 / 20, so that round(h * scale) is 799 at
# h = 20 and 800 just above it (torch's Softplus threshold is an entry boundary)
SG_SCALE = float.fromhex("0x1.3fcccccccccccp+5")
SG_LO, SG_HI = -1281, 800


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
    step = Decimal(1 / SG_SCALE)                 # the double kSgStep, exactly
    sg = []
    for j in range(SG_LO, SG_HI + 1):
        c = Decimal(j) * step
        if j == SG_HI:
            sg += [float(c / 2), -0.5]
        elif j == SG_LO:
            sg += [float(-c / 2), 0.5]
        else:
            sg += [float((Decimal(1) + c.exp()).ln() - c / 2),
                   float(Decimal(1) / 2 - Decimal(1) / (Decimal(1) + (-c).exp()))]
    n = len(sg)
    print(f'__constant__ static const double kSgTab[{n}] = {{')
    for i in range(0, n, 4):
        print('    ' + ', '.join(v.hex() for v in sg[i:i + 4]) + ',')
    print('};')


if __name__ == '__main__':
    main()
