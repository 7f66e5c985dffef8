"""BASELINE config 2 as written: BCH(63,45) decode with bf16 storage (x and the decoded
probabilities in bf16 in HBM, fp32 weights, every operation fp32; GNND_BF16).

* exactness: the bf16 kernel computes exactly what the fp32 kernel computes on the
  bf16-widened inputs, then rounds each output to bf16 (round to nearest even);
* SURVEY.md §8(d) parity rule (2): at every SNR point 1..6 dB the bf16 BER lies inside the
  95 % binomial confidence interval of the fp32 BER on the same codewords (the hard-decision
  disagreement rate between the two is reported in the assertion message)."""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cgnni():
    import gnndecode as gd
    z = np.load(os.path.join(ROOT, 'gnn-decode_amd', 'gnndecode', 'weights', 'cgnni_bch_63_45.npz'))
    H = gd.codes.bch_63_45()
    m = gd.MODELS['cgnni'](25, H)
    m.load_state_dict({k: torch.as_tensor(np.array(z[k])) for k in z.files})
    return m.to(DEV).eval(), H


def _decode(m, x):
    import gnndecode as gd
    with torch.no_grad():
        return m(gd.data.make_batch(x, m.graph(x.device)))


@pytest.mark.parametrize('model', ['cgnni', 'cbp'])
def test_bf16_storage_equals_fp32_math_on_widened_inputs(model):
    import gnndecode as gd
    if model == 'cgnni':
        m, H = _cgnni()
    else:
        H = gd.codes.bch_63_45()
        m = gd.MODELS['cbp'](25, H).to(DEV).eval()
    x32, _ = gd.data.awgn_batch(H, 8192, seed=31, device=DEV, codewords='random')
    xb = x32.bfloat16()
    ob = _decode(m, xb)
    assert ob.dtype == torch.bfloat16 and ob.shape == (8192 * 63, 1)
    of = _decode(m, xb.float())
    assert torch.equal(ob, of.bfloat16())


def test_bf16_ber_inside_fp32_confidence_interval_per_snr():
    import gnndecode as gd
    m, H = _cgnni()
    B, V = 65536, 63
    snrs = (1, 2, 3, 4, 5, 6)
    x32, lab = gd.data.awgn_batch(H, B, snrs=snrs, seed=32, device=DEV, codewords='random')
    d32 = (_decode(m, x32) > 0.5).view(B, V)
    d16 = (_decode(m, x32.bfloat16()).float() > 0.5).view(B, V)
    truth = (lab > 0.5).view(B, V)
    for k, snr in enumerate(snrs):
        rows = torch.arange(k, B, len(snrs), device=DEV)
        n = rows.numel() * V
        e32 = (d32[rows] != truth[rows]).sum().item() / n
        e16 = (d16[rows] != truth[rows]).sum().item() / n
        dis = (d32[rows] != d16[rows]).sum().item() / n
        half = 1.96 * math.sqrt(max(e32 * (1 - e32), 1.0 / n) / n)
        assert abs(e16 - e32) <= half, (snr, e32, e16, half, dis)
