"""On-device input synthesis (gnnd_sample_toric / gnnd_sample_awgn) vs the
reference generators: quantum/error_generate.py:252-278 (gen_syn) and classical/CGNNI.py:
125-147 (Gen_Data.AWGN / get_post).  The random streams differ from the reference's numpy /
torch CPU draws by construction, so parity is exact where the reference is deterministic
(layout, prior values, syndrome = (-1)^(H^T e), codewords in the code, LLR = 2 y'/sigma^2)
and statistical (5-sigma bounds) for the draws themselves."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _split(x, V, C):
    x = x.reshape(-1, V + C)
    return x[:, :V], x[:, V:]


@pytest.mark.parametrize('dtype', [torch.float64, torch.float32])
def test_toric_sampler_exact_structure_and_rates(golden, dtype):
    from gnndecode import codes, data
    H = codes.toric_code(5)
    V, C = H.shape
    ps = (0.01, 0.05, 0.1)                                   # the reference fixture's grid
    B = 200000
    x, y = data.toric_batch(H, B, ps=ps, seed=5, device=DEV, dtype=dtype)
    assert x.dtype == dtype and tuple(x.shape) == (B * (V + C), 1) and tuple(y.shape) == (B * V, 1)
    xv, xc = _split(x.double().cpu().numpy(), V, C)
    yv = y.cpu().numpy().reshape(B, V).astype(np.int64)
    # exact: one prior per codeword from the grid, syndrome (-1)^(H^T e) (gen_syn :270-273)
    priors = np.array([math.log((1 - p) / p) for p in ps], np.float64).astype(
        np.float32 if dtype == torch.float32 else np.float64)
    assert (xv == xv[:, :1]).all()
    assert np.isin(xv[:, 0], priors.astype(np.float64)).all()
    np.testing.assert_array_equal(xc, 1 - 2 * ((yv @ H.astype(np.int64)) % 2))
    # the reference's own draws have the same value sets
    ref = golden('toric_L5_gen_syn')
    rx, _ = _split(ref['x'], V, C)
    assert np.isin(np.unique(rx), np.array([math.log((1 - p) / p) for p in ps])).all()
    # statistical: uniform grid choice, Bernoulli(p) flips per qubit
    pi = np.abs(xv[:, :1] - priors.astype(np.float64)[None, :]).argmin(1)
    for k, p in enumerate(ps):
        sel = pi == k
        n = int(sel.sum())
        assert abs(n / B - 1 / len(ps)) < 5 * math.sqrt((1 / 3) * (2 / 3) / B)
        rate = yv[sel].mean()
        assert abs(rate - p) < 5 * math.sqrt(p * (1 - p) / (n * V)), (p, rate)
        # qubit columns are exchangeable: no column deviates beyond 6 sigma
        col = yv[sel].mean(0)
        assert np.abs(col - p).max() < 6 * math.sqrt(p * (1 - p) / n)


def test_samplers_shard_consistently():
    """Data-parallel shards (offset = shard start) reproduce the global draw bit for bit."""
    from gnndecode import codes, data
    H = codes.toric_code(5)
    B = 10000
    x, y = data.toric_batch(H, B, seed=9, device=DEV)
    parts = [data.toric_batch(H, e - s, seed=9, device=DEV, offset=s) for s, e in
             ((0, 3333), (3333, 6667), (6667, B))]
    assert torch.equal(torch.cat([p[0] for p in parts]), x)
    assert torch.equal(torch.cat([p[1] for p in parts]), y)
    Hb = codes.bch_63_45()
    xa, ya = data.awgn_batch(Hb, B, seed=4, device=DEV, codewords='random')
    pa = [data.awgn_batch(Hb, e - s, seed=4, device=DEV, codewords='random', offset=s)
          for s, e in ((0, 5001), (5001, B))]
    assert torch.equal(torch.cat([p[0] for p in pa]), xa)
    assert torch.equal(torch.cat([p[1] for p in pa]), ya)


def test_awgn_fixed_word_llr_moments_and_tails():
    from gnndecode import codes, data
    H = codes.bch_63_45()
    V, C = H.shape
    snrs = (1, 3, 6)
    B = 300000
    x, lab = data.awgn_batch(H, B, snrs=snrs, codeword_bit=0, seed=11, device=DEV)
    xv, xc = _split(x.double().cpu().numpy(), V, C)
    assert (xc == 0).all() and (lab.cpu().numpy() == 0).all()
    for k, snr in enumerate(snrs):
        rows = xv[k::len(snrs)]
        sig2 = 10 ** (-snr / 10)
        mean, var = 2 / sig2, 4 / sig2                     # LLR = 2 (1 + n) / sigma^2
        n = rows.size
        assert abs(rows.mean() - mean) < 5 * math.sqrt(var / n)
        assert abs(rows.var() / var - 1) < 5 * math.sqrt(2 / n)
        z = (rows - mean) / math.sqrt(var)                 # standard normal draws
        for t, q in ((1.0, 0.3173105), (2.0, 0.0455003), (3.0, 0.0026998)):
            f = (np.abs(z) > t).mean()
            assert abs(f - q) < 5 * math.sqrt(q * (1 - q) / n), (snr, t, f)
    x1, lab1 = data.awgn_batch(H, 6000, snrs=(6,), codeword_bit=1, seed=12, device=DEV)
    assert (lab1.cpu().numpy() == 1).all()
    assert x1.reshape(-1, V + C)[:, :V].mean().item() < 0          # BPSK of the all-ones word


@pytest.mark.parametrize('code', ['bch_63_45', 'ldpc_648_324'])
def test_awgn_random_codewords_are_codewords(code):
    from gnndecode import codes, data
    H = codes.get_code(code)
    V, C = H.shape
    B = 20000
    x, lab = data.awgn_batch(H, B, snrs=(2,), seed=13, device=DEV, codewords='random')
    c = lab.cpu().numpy().reshape(B, V).astype(np.int64)
    assert not ((c @ H.astype(np.int64)) % 2).any()                 # every word is in the code
    ones = c.mean(0)
    assert np.abs(ones - 0.5).max() < 6 * math.sqrt(0.25 / B)       # uniform over the code
    xv, _ = _split(x.double().cpu().numpy(), V, C)
    sig2 = 10 ** (-2 / 10)
    m1 = xv[c == 1].mean()
    assert abs(m1 + 2 / sig2) < 5 * math.sqrt(4 / sig2 / (c == 1).sum())


def test_awgn_fp64_output_is_the_fp32_draw():
    from gnndecode import codes, data
    H = codes.bch_63_45()
    a, la = data.awgn_batch(H, 1000, seed=3, device=DEV, dtype=torch.float32, codewords='random')
    b, lb = data.awgn_batch(H, 1000, seed=3, device=DEV, dtype=torch.float64, codewords='random')
    assert torch.equal(a.double(), b) and torch.equal(la.double(), lb)


def test_sampler_config4_size_and_determinism():
    """Config 4's per-GPU shard size (LDPC(648,324), 131 072 codewords per GPU of 1 M) draws
    identically twice; the per-codeword SNR follows the global index."""
    from gnndecode import codes, data
    H = codes.get_code('ldpc_648_324')
    V, C = H.shape
    B = 131072
    a = data.awgn_batch(H, B, snrs=(1, 2, 3), seed=21, device=DEV, codewords='random', offset=B)
    b = data.awgn_batch(H, B, snrs=(1, 2, 3), seed=21, device=DEV, codewords='random', offset=B)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    xv = a[0].reshape(B, V + C)[:, :V].double()
    c = a[1].reshape(B, V).double()
    s = 1 - 2 * c
    for k, snr in enumerate((1, 2, 3)):
        sel = (torch.arange(B, device=DEV) + B) % 3 == k              # SNR by global index
        sig2 = 10 ** (-snr / 10)
        z = (xv[sel] * sig2 / 2 - s[sel]) / math.sqrt(sig2)           # recovered noise
        n = z.numel()
        assert abs(z.mean().item()) < 5 / math.sqrt(n)
        assert abs(z.var().item() - 1) < 5 * math.sqrt(2 / n)
