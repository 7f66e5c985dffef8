"""The fp64 Softplus tables compiled into the kernels (gnnd_common.h kExpTab, kLogTab, kSpTab)
are exactly the generator's output (tools/gen_fp64_tables.py: 60-digit decimal arithmetic,
correctly rounded doubles), and the one-read table's entries are {ln(1 + e^-a), 1/(1 + e^a)}
at a = j/64 to within an ulp of the float64 libm values."""
import math
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, 'gnn-decode_amd', 'csrc', 'gnnd_common.h')


def _arrays(text):
    out = {}
    for m in re.finditer(r'static const double (kExpTab|kLogTab|kSpTab)\[(\d+)\] = \{(.*?)\};', text, re.S):
        vals = [float.fromhex(v) for v in re.findall(r'-?0x[0-9a-fA-F.]+p[-+]?\d+', m.group(3))]
        assert len(vals) == int(m.group(2)), m.group(1)
        out[m.group(1)] = vals
    return out


def test_tables_match_generator():
    gen = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'gen_fp64_tables.py')],
                         check=True, capture_output=True, text=True).stdout
    g, h = _arrays(gen), _arrays(open(HDR).read())
    for name in ('kExpTab', 'kLogTab', 'kSpTab'):
        assert g[name] == h[name], name


def test_softplus_table_entries():
    sp = _arrays(open(HDR).read())['kSpTab']
    assert sp[-2:] == [0.0, 0.0]                         # the zero entry (threshold, |x| > 32)
    for j in range(0, 2049, 7):
        a = j / 64
        f, s = sp[2 * j], sp[2 * j + 1]
        assert abs(f - math.log1p(math.exp(-a))) <= 2 * math.ulp(f)
        assert abs(s - 1.0 / (1.0 + math.exp(a))) <= 2 * math.ulp(s)
