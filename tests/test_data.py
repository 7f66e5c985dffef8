"""On-device input synthesis vs the reference's generators, checked
statistically (the distributions must match, not the random streams).  Runs the same torch
code on CPU generators.

* toric: quantum/error_generate.py:252-278 `gen_syn` (fixture `toric_L5_gen_syn.npz` = seeded
  reference draws): priors log((1-p)/p) on the variable rows, syndrome (-1)^(H^T e) on the
  check rows, labels e ~ Bernoulli(p) per qubit.
* AWGN: classical/CGNNI.py:125-147 `Gen_Data`: BPSK 1 - 2c, sigma^2 = 10^(-SNR/10),
  LLR = 2 y / sigma^2.
"""
import math

import numpy as np
import torch

from gnndecode import codes, data


def _split(x, V, C):
    x = x.reshape(-1, V + C)
    return x[:, :V], x[:, V:]


def test_toric_sampler_layout_matches_reference_draws(golden):
    H = codes.toric_code(5)
    V, C = H.shape
    ref = golden('toric_L5_gen_syn')
    rx, _ = _split(ref['x'], V, C)
    ry = ref['y'].reshape(-1, V)
    ps = (0.01, 0.05, 0.1)                                   # the fixture's grid
    x, y = data.toric_batch(H, 4096, ps=ps, seed=3, device='cpu')
    xv, xc = _split(x.numpy(), V, C)
    yv = y.numpy().reshape(-1, V)
    # same row layout and value sets as the reference: one prior per codeword from the grid,
    # syndrome entries +-1 consistent with the labels
    prior_set = {round(math.log((1 - p) / p), 9) for p in ps}
    assert {round(float(v), 9) for v in np.unique(rx)} <= prior_set
    assert {round(float(v), 9) for v in np.unique(xv)} <= prior_set
    assert (xv == xv[:, :1]).all() and (rx == rx[:, :1]).all()
    assert set(np.unique(xc)) <= {-1.0, 1.0}
    for xs, ys in ((xc, yv), (_split(ref['x'], V, C)[1], ry)):
        syn = (ys.astype(np.int64) @ H.astype(np.int64)) % 2
        np.testing.assert_array_equal(xs, 1 - 2 * syn)


def test_toric_sampler_flip_rates_per_p():
    H = codes.toric_code(5)
    V, C = H.shape
    ps = (0.01, 0.05, 0.1)
    B = 20000
    x, y = data.toric_batch(H, B, ps=ps, seed=7, device='cpu')
    xv, _ = _split(x.numpy(), V, C)
    yv = y.numpy().reshape(-1, V)
    p_row = 1.0 / (1.0 + np.exp(xv[:, 0]))                  # invert the prior
    for p in ps:
        sel = np.isclose(p_row, p)
        n = sel.sum()
        assert abs(n / B - 1 / len(ps)) < 5 * math.sqrt((1 / 3) * (2 / 3) / B)   # uniform grid
        rate = yv[sel].mean()
        assert abs(rate - p) < 5 * math.sqrt(p * (1 - p) / (n * V)), (p, rate)


def test_awgn_llr_moments_match_gen_data():
    H = codes.bch_63_45()
    V, C = H.shape
    snrs = (1, 3, 6)
    B = 6000
    x, lab = data.awgn_batch(H, B, snrs=snrs, codeword_bit=0, seed=11, device='cpu')
    xv, xc = _split(x.numpy().astype(np.float64), V, C)
    assert (xc == 0).all() and (lab.numpy() == 0).all()
    for k, snr in enumerate(snrs):
        rows = xv[k::len(snrs)]
        sig2 = 10 ** (-snr / 10)
        mean, var = 2 / sig2, 4 / sig2                     # LLR = 2 (1 + n) / sigma^2
        n = rows.size
        assert abs(rows.mean() - mean) < 5 * math.sqrt(var / n)
        assert abs(rows.var() / var - 1) < 5 * math.sqrt(2 / n)
    # codeword bit 1 flips the BPSK sign (classical/CGNNI.py:195 uses the all-ones word)
    x1, lab1 = data.awgn_batch(H, 600, snrs=(6,), codeword_bit=1, seed=12, device='cpu')
    assert (lab1.numpy() == 1).all()
    assert _split(x1.numpy(), V, C)[0].mean() < 0


def test_random_codewords_satisfy_parity_checks():
    """codewords='random': labels are codewords of H (c H = 0 mod 2), about half ones, and
    the LLR signs follow the bits at high SNR."""
    H = codes.bch_63_45()
    G = codes.gf2_generator(H)
    assert G.shape == (45, 63) and codes.gf2_rank(G) == 45
    assert not ((G.astype(np.int64) @ H) % 2).any()
    B = 400
    x, lab = data.awgn_batch(H, B, snrs=(12,), seed=4, device='cpu', codewords='random')
    c = lab.view(B, 63).numpy().astype(np.int64)
    assert not ((c @ H) % 2).any()
    assert 0.4 < c.mean() < 0.6
    llr = x.view(B, 81)[:, :63].numpy()
    assert ((llr < 0) == (c == 1)).mean() > 0.999
