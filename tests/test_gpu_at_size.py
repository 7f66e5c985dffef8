"""Every BASELINE.json config's kernel instantiation, decoded at its OWN batch size on the
GPU, compared with the oracle on a sample of its codewords (SURVEY.md §8(d) parity rule 1),
plus the reference-pinned FER rule on the device metric kernel.

The fused decoder picks its kernel from (model, dtype, graph, batch): BCH CGNNI runs
decode_resident_kernel<CGNNI, f32, G=8, R=3, Q=9>, LDPC CGNNI <G=2, R=4, Q=6>, toric V24
the streaming decode_kernel (R = 4, fp32 paired or fp64 scalar).  Small-batch golden tests
do not reach every one of those tile shapes and tile counts, so each config is run here at
the size the bench quotes and a seeded sample of 128 codewords (first, last, random) is
re-decoded by the oracle.

Tolerances (written per test): fp64 soft outputs rtol 1e-10 with bit-exact hard decisions;
fp32 rtol 1e-4 / atol 2e-5 with identical decisions except bits within 1e-6 of 0.5
(CGNNI); the fp32 kernel on the fp64 quantum model |dp| <= 1e-4 with identical decisions
outside |p - 0.5| < 1e-3; fp32 classical BP by the conditioning bound of
tests/test_gpu_parity.py (fp32 BP is ill-conditioned at its 1 - 1e-7 clamp).
"""
import os

import numpy as np
import pytest
import torch

import gnn_oracle as O
from conftest import weights_of

pytestmark = pytest.mark.gpu

DEV = 'cuda'
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _sample(B, n=128, seed=0):
    rng = np.random.default_rng(seed)
    mid = rng.choice(np.arange(1, B - 1), n - 2, replace=False)
    return np.sort(np.concatenate([[0, B - 1], mid]))


def _model(name, code, T, weights=None, dtype=torch.float32):
    import gnndecode as gd
    H = gd.codes.get_code(code)
    m = gd.MODELS[name](T, H)
    if weights is not None:
        m.load_state_dict({k: torch.as_tensor(np.array(v)) for k, v in weights.items()})
    return m.to(DEV).eval(), H


def _shipped(name):
    z = np.load(os.path.join(ROOT, 'gnn-decode_amd', 'gnndecode', 'weights', f'{name}.npz'))
    return {k: z[k] for k in z.files}


def _decode(m, x):
    import gnndecode as gd
    g = m.graph(x.device)
    w = m.prepared_weights(x.dtype, x.device)
    out = gd.ops.decode(g, m.kind, x, m.Nc, w)
    torch.cuda.synchronize()
    return g, out


def _rows(t, B, width, pick):
    return t.view(B, width)[torch.as_tensor(pick, device=t.device)].cpu().numpy()


def test_config2_bch_cgnni_B65536_plan_and_parity():
    """Config 2: BCH(63,45) CGNNI, B = 65 536, shipped trained weights, random codewords."""
    import gnndecode as gd
    w = _shipped('cgnni_bch_63_45')
    m, H = _model('cgnni', 'bch_63_45', 25, w)
    B = 65536
    x, _ = gd.data.awgn_batch(H, B, codewords='random', seed=21, device=DEV)
    g, out = _decode(m, x)
    plan = gd.ops.decode_plan(g, 'cgnni', torch.float32)
    assert plan['kernel'] == 'decode_resident_kernel'
    pick = _sample(B)
    xs = _rows(x, B, g.N, pick).reshape(-1, 1)
    ref = O.decode('cgnni', H, xs, 25, w).reshape(len(pick), g.V)
    got = _rows(out, B, g.V, pick)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=2e-5)
    far = np.abs(ref - 0.5) >= 1e-6
    assert ((got > 0.5) == (ref > 0.5))[far].all()


def test_config4_ldpc_cgnni_B131072_plan_and_parity():
    """Config 4's per-GPU shard: LDPC(648,324) CGNNI at B = 131 072 (trained weights)."""
    import gnndecode as gd
    w = _shipped('cgnni_ldpc_648_324')
    m, H = _model('cgnni', 'ldpc_648_324', 25, w)
    B = 131072
    x, _ = gd.data.awgn_batch(H, B, codewords='fixed', codeword_bit=0, seed=22, device=DEV)
    g, out = _decode(m, x)
    plan = gd.ops.decode_plan(g, 'cgnni', torch.float32)
    assert plan['kernel'] == 'decode_resident_kernel'
    pick = _sample(B)
    xs = _rows(x, B, g.N, pick).reshape(-1, 1)
    ref = O.decode('cgnni', H, xs, 25, w).reshape(len(pick), g.V)
    got = _rows(out, B, g.V, pick)
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=2e-5)
    far = np.abs(ref - 0.5) >= 1e-6
    assert ((got > 0.5) == (ref > 0.5))[far].all()
    del x, out


def test_config4_ldpc_cbp_B131072_conditioning_bound():
    """Config 4 with classical BP (classical/BP.py) at B = 131 072: the sampled GPU decisions
    disagree with the fp32 oracle no more than the fp32 oracle disagrees with the fp64 one
    (+ slack), soft outputs agree to 1e-3 away from the clamp region."""
    import gnndecode as gd
    m, H = _model('cbp', 'ldpc_648_324', 25)
    B = 131072
    x, _ = gd.data.awgn_batch(H, B, seed=23, device=DEV)
    g, out = _decode(m, x)
    pick = _sample(B, 64)
    xs = _rows(x, B, g.N, pick).reshape(-1, 1)
    got = _rows(out, B, g.V, pick).reshape(-1)
    o32 = O.decode('cbp', H, xs.astype(np.float32), 25).reshape(-1)
    o64 = O.decode('cbp', H, xs.astype(np.float64), 25).reshape(-1)
    gpu_vs_32 = int(((got > 0.5) != (o32 > 0.5)).sum())
    f32_vs_64 = int(((o32 > 0.5) != (o64 > 0.5)).sum())
    assert gpu_vs_32 <= 2 * f32_vs_64 + 10, (gpu_vs_32, f32_vs_64)
    del x, out


@pytest.mark.parametrize('dtype', [torch.float64, torch.float32])
def test_config3_toric5_v24_B65536(dtype):
    """Config 3: toric d = 5 decoder_v2_4 (reference epoch-67 checkpoint), B = 65 536, in the
    reference's fp64 (bit-exact decisions, rtol 1e-10) and in the fp32 perf mode."""
    import gnndecode as gd
    w = _shipped('v24_toric_5')
    m, H = _model('v24', 'toric_5', 15, w)
    B = 65536
    x, _ = gd.data.toric_batch(H, B, seed=24, device=DEV, dtype=dtype)
    g, out = _decode(m, x)
    pick = _sample(B)
    xs = _rows(x, B, g.N, pick).reshape(-1, 1).astype(np.float64)
    ref = O.decode('v24', H, xs, 15, w).reshape(len(pick), g.V)
    got = _rows(out, B, g.V, pick).astype(np.float64)
    if dtype == torch.float64:
        np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-13)
        assert ((got > 0.5) == (ref > 0.5)).all()
    else:
        assert np.abs(got - ref).max() <= 1e-4
        far = np.abs(ref - 0.5) >= 1e-3
        assert ((got > 0.5) == (ref > 0.5))[far].all()


def test_config3_toric5_v24_B65536_prior_tables():
    """Config 3 as the bench runs it: fp64 decoder_v2_4 at B = 65 536 with the batch's channel
    priors registered (the variable-side and readout MLPs from the prepared tables) -- rtol
    1e-10 and bit-exact decisions against the oracle on sampled codewords."""
    import gnndecode as gd
    w = _shipped('v24_toric_5')
    m, H = _model('v24', 'toric_5', 15, w)
    B = 65536
    x, _ = gd.data.toric_batch(H, B, seed=26, device=DEV, dtype=torch.float64)
    g = m.graph(x.device)
    pri = gd.ops.channel_priors(g, x)
    assert len(pri) == 10
    m.set_channel_priors(pri)
    g, out = _decode(m, x)
    m.set_channel_priors(())
    pick = _sample(B)
    xs = _rows(x, B, g.N, pick).reshape(-1, 1)
    ref = O.decode('v24', H, xs, 15, w).reshape(len(pick), g.V)
    got = _rows(out, B, g.V, pick)
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-13)
    assert ((got > 0.5) == (ref > 0.5)).all()


def test_config5_toric7_v24_decode_B16384_fp64():
    """Config 5's architecture (decoder_v2_4 at L = 7, seeded reference init) decoded at
    B = 16 384 in fp64: bit-exact decisions on 64 sampled codewords."""
    import gnndecode as gd
    H = gd.codes.get_code('toric_7')
    torch.manual_seed(7)
    m = gd.MODELS['v24'](15, H).double()
    w = {k: v.detach().numpy() for k, v in m.state_dict().items()}
    m = m.to(DEV).eval()
    B = 16384
    x, _ = gd.data.toric_batch(H, B, seed=25, device=DEV, dtype=torch.float64)
    g, out = _decode(m, x)
    pick = _sample(B, 64)
    xs = _rows(x, B, g.N, pick).reshape(-1, 1)
    ref = O.decode('v24', H, xs, 15, w).reshape(len(pick), g.V)
    got = _rows(out, B, g.V, pick)
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-13)
    assert ((got > 0.5) == (ref > 0.5)).all()


# ------------------------------------------------------------------------------------
# the FER rule of quantum/neural_BP.py:338-348, pinned by the reference LossFunc(train=0)
# ------------------------------------------------------------------------------------
@pytest.mark.parametrize('dtype', [torch.float64, torch.float32])
@pytest.mark.parametrize('L', [5, 7])
def test_decision_errors_kernel_matches_reference_fer(golden, L, dtype):
    import gnndecode as gd
    z = golden('fer_rule')
    gz = golden(f'toric_L{L}_graph')
    g = gd.TannerGraph(gz['H'], device=DEV)
    lg = torch.as_tensor(gz['logical'].astype(np.int32), device=DEV)
    pred = torch.as_tensor(z[f'L{L}/pred'], device=DEV).to(dtype)
    y = torch.as_tensor(z[f'L{L}/y'], device=DEV).to(dtype)
    c = gd.ops.decision_errors(g, lg, pred, y).cpu().tolist()
    assert c[2] + c[3] == int(z[f'L{L}/count'])
    assert c[2] > 0 and c[3] > 0


def test_decision_errors_kernel_on_decoder_outputs(golden):
    import gnndecode as gd
    z = golden('v24_toric5')
    gz = golden('toric_L5_graph')
    g = gd.TannerGraph(gz['H'], device=DEV)
    lg = torch.as_tensor(gz['logical'].astype(np.int32), device=DEV)
    c = gd.ops.decision_errors(g, lg, torch.as_tensor(z['out_B32_T15'], device=DEV),
                               torch.as_tensor(z['y_B32'], device=DEV)).cpu().tolist()
    assert c[2] + c[3] == int(golden('fer_rule')['v24_B32/count'])


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
def test_v24_unit_split_192_lane_rounds_bit_identical(dtype):
    """toric-7 (a component-codeword holds 192 edges): the unit split runs 192-lane rounds
    (decode_kernel IW3: US = 4 at B*ncomp <= 256, US = 2 at <= 512) -- slices decoded alone give
    the same bits as the B = 1 024 decode (US = 1, whole graph)."""
    import gnndecode as gd
    H = gd.codes.get_code('toric_7')
    torch.manual_seed(7)
    m = gd.MODELS['v24'](15, H).to(DEV).eval()
    if dtype == torch.float64:
        m = m.double()
    B = 1024
    x, _ = gd.data.toric_batch(H, B, seed=8, device=DEV, dtype=dtype)
    _, full = _decode(m, x)
    full = full.view(B, -1)
    xb = x.view(B, -1)
    for b0, n in ((0, 128), (128, 200), (700, 77), (1023, 1)):
        _, part = _decode(m, xb[b0:b0 + n].reshape(-1, 1).contiguous())
        assert torch.equal(part.view(n, -1), full[b0:b0 + n]), (b0, n)


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
def test_v24_unit_split_bit_identical(dtype):
    """decoder_v2_4 small-batch unit split: decode_kernel runs US = 4 (B*ncomp <= 256), 2
    (<= 512) waves per item wave at one codeword per workgroup (fp32 also US = 8 when a
    component-codeword's items fit 128 lanes) and US = 1 above (the toric graph is split into its
    two components below one codeword per CU, B*ncomp = 2B).  fp32 runs the R = 2 slot table below
    B = 4096, fp64 (the reference dtype) the default plan (toric: one slot per lane).  The 128
    hidden units are summed in one fixed chain order (gnnd_decode_impl.h mlp128_chains: 8 chains,
    mlp128d_chains: 4 chains in fp64), so every codeword decodes to the SAME BITS under every
    split and tile: slices decoded alone (US = 4 / 2) equal the B = 1024 decode (US = 1)."""
    import gnndecode as gd
    w = _shipped('v24_toric_5')
    m, H = _model('v24', 'toric_5', 15, w)
    if dtype == torch.float64:
        m = m.double()
    B = 1024
    x, _ = gd.data.toric_batch(H, B, seed=5, device=DEV, dtype=dtype)
    _, full = _decode(m, x)
    full = full.view(B, -1)
    xb = x.view(B, -1)
    for b0, n in ((0, 128), (128, 300), (700, 256), (1000, 24), (1023, 1)):
        _, part = _decode(m, xb[b0:b0 + n].reshape(-1, 1).contiguous())
        assert torch.equal(part.view(n, -1), full[b0:b0 + n]), (b0, n)
