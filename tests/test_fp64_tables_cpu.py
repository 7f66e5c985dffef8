"""The fp64 Softplus tables compiled into the kernels (gnnd_common.h kExpTab, kLogTab, kSpTab)
are exactly the generator's output (tools/gen_fp64_tables.py: 60-digit decimal arithmetic,
correctly rounded doubles), and the one-read table's entries are {ln(1 + e^-a), 1/(1 + e^a)}
at a = j/64 to within an ulp of the float64 libm values."""
import math
from fractions import Fraction
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, 'gnn-decode_amd', 'csrc', 'gnnd_common.h')


def _arrays(text):
    out = {}
    for m in re.finditer(r'static const double (kExpTab|kLogTab|kSpTab|kSgTab)\[(\d+)\] = \{(.*?)\};', text, re.S):
        vals = [float.fromhex(v) for v in re.findall(r'-?0x[0-9a-fA-F.]+p[-+]?\d+', m.group(3))]
        assert len(vals) == int(m.group(2)), m.group(1)
        out[m.group(1)] = vals
    return out


def test_tables_match_generator():
    gen = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'gen_fp64_tables.py')],
                         check=True, capture_output=True, text=True).stdout
    g, h = _arrays(gen), _arrays(open(HDR).read())
    for name in ('kExpTab', 'kLogTab', 'kSpTab', 'kSgTab'):
        assert g[name] == h[name], name


def test_softplus_table_entries():
    sp = _arrays(open(HDR).read())['kSpTab']
    assert sp[-2:] == [0.0, 0.0]                         # the zero entry (threshold, |x| > 32)
    for j in range(0, 2049, 7):
        a = j / 64
        f, s = sp[2 * j], sp[2 * j + 1]
        assert abs(f - math.log1p(math.exp(-a))) <= 2 * math.ulp(f)
        assert abs(s - 1.0 / (1.0 + math.exp(a))) <= 2 * math.ulp(s)


def test_signed_softplus_table_entries():
    """kSgTab: {softplus(c) - c/2, 1/2 - sigmoid(c)} at c = j * step, j = -1280..799, between the
    two linear clamp entries (h < -32.03: -h/2; h > 20: h/2, slope -sig = -+1/2, t = 0)."""
    sg = _arrays(open(HDR).read())['kSgTab']
    scale = float.fromhex('0x1.3fcccccccccccp+5')
    step = 1.0 / scale
    # (exact products, as the index FMA forms them before its one rounding)
    half = Fraction(1599, 2)
    assert Fraction(20) * Fraction(scale) < half < Fraction(math.nextafter(20.0, 30.0)) * Fraction(scale)
    n = len(sg) // 2
    assert n == 2082
    assert sg[1] == 0.5 and sg[-1] == -0.5
    for i in range(1, n - 1, 5):
        c = (i - 1281) * step
        f, s = sg[2 * i], sg[2 * i + 1]
        ref = math.log1p(math.exp(-abs(c))) + abs(c) / 2
        assert abs(f - ref) <= 4 * math.ulp(ref)
        assert abs(s - (0.5 - 1.0 / (1.0 + math.exp(-c)))) <= 3e-16
