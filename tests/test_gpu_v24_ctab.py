"""decoder_v2_4's check-side MLP through the fp64 decoder's per-launch table (build_ctab /
ctab_eval in gnnd_decode_impl.h, exposed as gnnd_v24_check_mlp_table).

ggc2.mlp (Linear(1,128) -> Softplus -> Linear(128,1), quantum/decoder_v2_4.py:241-243,
:253-257) is evaluated on ONE scalar u = S_c(tanh(m/2)) - tanh(m_e/2) in [-(dc-1), dc-1]
(:135-136), so the fp64 prepared weights carry it tabulated (degree-11 Taylor polynomials
about j/8, built by gnnd_prepare_weights and after every fused optimizer step).
Held here against torch's own fp64 MLP (the reference module, Softplus threshold 20 included)
at 1e-13 absolute over the whole input range; weights whose unit range crosses the Softplus
threshold make the table invalid and the decoder falls back to the per-unit MLP (decode
still equal to the oracle, rtol 1e-10, bit-exact decisions).
"""
import os

import numpy as np
import pytest
import torch

import gnn_oracle as O

pytestmark = pytest.mark.gpu

DEV = 'cuda'
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = 1e-13


def _model(L=5, weights='shipped', seed=0):
    import gnndecode as gd
    H = gd.codes.toric_code(L)
    torch.manual_seed(seed)
    m = gd.MODELS['v24'](15, H)
    if weights == 'shipped':
        z = np.load(os.path.join(ROOT, 'gnn-decode_amd', 'gnndecode', 'weights', 'v24_toric_5.npz'))
        m.load_state_dict({k: torch.from_numpy(z[k]) for k in z.files})
    return m.to(DEV).double().eval(), H


def _torch_mlp(m, u):
    with torch.no_grad():
        return m.ggc2.mlp(u.view(-1, 1)).view(-1)


def _inputs(R):
    u = torch.linspace(-R, R, 24001, dtype=torch.float64, device=DEV)
    g = torch.Generator(device='cpu').manual_seed(1)
    extra = (torch.rand(4000, generator=g, dtype=torch.float64) * 2 - 1).to(DEV) * R
    return torch.cat([u, extra, torch.tensor([-R, R, 0.0, 1 / 64, -1 / 64], dtype=torch.float64, device=DEV)])


@pytest.mark.parametrize('weights', ['shipped', 'random'])
def test_table_matches_reference_mlp(weights):
    import gnndecode as gd
    m, H = _model(weights=weights)
    g = m.graph(torch.device(DEV))
    R = g.max_chk_degree - 1
    assert R == 3
    u = _inputs(R)
    y, ok = gd.ops.v24_check_mlp_table(g, m.packed_weights().double(), u)
    assert ok
    err = float((y - _torch_mlp(m, u)).abs().max())
    assert err <= TOL, err


def test_threshold_crossing_unit_disables_table_and_decode_stays_exact():
    """A unit whose pre-activation range over [-R, R] crosses torch's Softplus threshold (20):
    the table is reported invalid, and the decoder's per-unit path still matches the oracle."""
    import gnndecode as gd
    m, H = _model(weights='shipped')
    with torch.no_grad():
        m.ggc2.mlp[0].weight[5, 0] = 2.0      # h = 2 u + 17 spans [11, 23] over u in [-3, 3]
        m.ggc2.mlp[0].bias[5] = 17.0
    g = m.graph(torch.device(DEV))
    u = _inputs(3)
    _, ok = gd.ops.v24_check_mlp_table(g, m.packed_weights().double(), u)
    assert not ok
    # the same weights on a graph whose range stops short of the crossing (toric: R = 3; a
    # unit crossing 20 at |u| = 3.5): valid
    with torch.no_grad():
        m.ggc2.mlp[0].bias[5] = 13.0           # h = 2 u + 13 reaches 20 at u = 3.5
    _, ok = gd.ops.v24_check_mlp_table(g, m.packed_weights().double(), u)
    assert ok
    with torch.no_grad():
        m.ggc2.mlp[0].bias[5] = 17.0
    x, _ = gd.data.toric_batch(H, 64, seed=3, device=torch.device(DEV), dtype=torch.float64)
    out = gd.ops.decode(g, 'v24', x, m.Nc, m.prepared_weights(torch.float64, torch.device(DEV)))
    w = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    ref = O.decode('v24', H, x.cpu().numpy(), m.Nc, w)
    got = out.cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-12)
    assert ((got > 0.5) == (ref > 0.5)).all()


def test_large_weights_fail_the_remainder_bound():
    """sum |W2| |W1|^12 large enough that the Taylor remainder bound exceeds 1e-13: invalid."""
    import gnndecode as gd
    m, H = _model(weights='shipped')
    with torch.no_grad():
        m.ggc2.mlp[0].weight[7, 0] = 9.0       # |W1|^12 = 2.8e11: bound 1.8e-10; h stays below 20
        m.ggc2.mlp[0].bias[7] = -10.0
        m.ggc2.mlp[2].weight[0, 7] = 1.0
    g = m.graph(torch.device(DEV))
    _, ok = gd.ops.v24_check_mlp_table(g, m.packed_weights().double(), _inputs(3))
    assert not ok


def test_prepared_layout_and_trainer_rebuild():
    """gnnd_prepare_weights (fp64 V24) = [plain weights | bound, R limit, pad | table | prior
    header (0 tables)]; the
    fused trainer's epilogue (gnnd_train_update) rebuilds the table of the updated weights, so
    its prepared buffer equals a fresh gnnd_prepare_weights of its parameters after each step."""
    import gnndecode as gd
    m, H = _model(L=5)
    flat = m.packed_weights().double().detach().contiguous()
    prep = gd.ops.prepare_weights('v24', flat)
    assert prep.numel() == gd.ops.prepared_count('v24', torch.float64) == 7264
    assert torch.equal(prep[:1283], flat)
    assert 0 < float(prep[1283]) < 1e-13 and float(prep[1284]) > 3
    assert gd.ops.prepared_count('v24', torch.float32) == 7264          # (fp32: the same table in fp32)
    assert float(prep[7252:7264].abs().sum()) == 0.0                    # (no channel-prior tables)
    lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H)).to(DEV)
    tr = gd.train.FusedV24Trainer(m, lf, graph=False)
    x, y = gd.data.toric_batch(H, 32, seed=2, device=torch.device(DEV), dtype=torch.float64)
    for _ in range(2):
        tr.step(gd.data.make_batch(x, m.graph(x.device)), y)
        torch.cuda.synchronize()
        ref = gd.ops.prepare_weights('v24', tr.flat)
        assert torch.equal(tr.prepared, ref)


def test_huge_priors_take_the_safe_softplus_index():
    """the fp64 Softplus table index (sg_index) wraps for |h| >= 2^31 / 40; a wave
    whose MLP pre-activation bound reaches 2^25 evaluates its units with sg_index_safe.  Priors of
    +-1e8 on some codewords (h up to ~4e8): the decode still equals the oracle (rtol 1e-10)."""
    import warnings
    import gnndecode as gd
    m, H = _model(weights='shipped')
    x, _ = gd.data.toric_batch(H, 32, seed=4, device=torch.device(DEV), dtype=torch.float64)
    N, V = H.shape[0] + H.shape[1], H.shape[0]
    xv = x.view(32, N)
    xv[::3, :V] *= 1e8 / xv[::3, :V].abs().clamp_min(1e-300)
    g = m.graph(x.device)
    out = gd.ops.decode(g, 'v24', x, m.Nc, m.prepared_weights(torch.float64, x.device))
    w = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')               # (exp overflow inside the oracle's where)
        ref = O.decode('v24', H, x.cpu().numpy(), m.Nc, w)
    got = out.cpu().numpy()
    assert np.isfinite(got).all()
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-12)
