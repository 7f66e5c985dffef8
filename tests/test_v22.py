"""decoder_v2_2 (quantum/decoder_v2_2.py:272-380: neural BP with weights shared by the 8 edge
types of H_prime, residual m_p @ sigmoid(weight), one readout per layer) — oracle, edge
types and loss vs the reference-generated goldens (CPU), and the HIP path through the C ABI
vs the goldens and the oracle (`-m gpu`).

The script's module top level cannot run against the shipped error_generate (see
tests/golden/make_golden.py gen_v22); the goldens run its own classes with `feat_onehot`
built from the reference's own 8-type H_prime.

Tolerances: fp64 (the script's dtype) soft outputs rtol 1e-10 with identical hard decisions;
fp32 kernels |dp| <= 1e-4 with identical decisions outside |p - 0.5| < 1e-3; training
gradients 1e-8 relative to the largest reference gradient (fp64)."""
import numpy as np
import pytest
import torch

import gnn_oracle as O
from conftest import weights_of

DEV = 'cuda'
CASES = [(B, T) for B in (1, 8) for T in (1, 2, 25)]


def _w(z):
    w = weights_of(z)
    w['edge_types'] = z['edge_types']
    return w


# ------------------------------------------------------------------------------------
# CPU
# ------------------------------------------------------------------------------------
@pytest.mark.parametrize('B,T', CASES)
def test_oracle_v22_matches_reference(golden, B, T):
    z = golden('v22_toric4')
    H = golden('toric_L4_graph')['H']
    outs = O.decode('v22', H, z[f'x_B{B}'], T, _w(z))
    ref = z[f'out_B{B}_T{T}']
    assert len(outs) == T == ref.shape[0]
    got = np.stack([o.reshape(-1) for o in outs])
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-14)
    assert ((got > 0.5) == (ref > 0.5)).all()


def test_edge_types_match_reference_h_prime(golden):
    """codes.toric_edge_types restates error_generate.py's H_prime labels; the golden holds
    the labels computed by the reference function itself."""
    import gnndecode as gd
    z = golden('v22_toric4')
    assert np.array_equal(gd.codes.toric_edge_types(4), z['edge_types'])
    assert np.array_equal(gd.codes.toric_code(4), golden('toric_L4_graph')['H'])


def test_v22_state_dict_keys_and_packing(golden):
    import gnndecode as gd
    z = golden('v22_toric4')
    H = golden('toric_L4_graph')['H']
    m = gd.DecoderV22(25, H)
    assert sorted(m.state_dict().keys()) == sorted(weights_of(z).keys())
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()})
    E = int(H.sum())
    flat = m.packed_weights()
    assert flat.numel() == 2 * E * 25 + 2 * E + 1
    t = torch.from_numpy(z['edge_types'])
    w0 = torch.from_numpy(z['w/layers.0.W']).reshape(-1)
    assert torch.equal(flat[:E], w0[t])
    assert float(flat[-1]) == float(torch.sigmoid(torch.from_numpy(z['w/weight'])).reshape(()))


def test_v22_explicit_edge_types_validated(golden):
    import gnndecode as gd
    H = golden('toric_L4_graph')['H']
    with pytest.raises(ValueError):
        gd.DecoderV22(2, H, edge_types=np.zeros(3, np.int64))
    with pytest.raises(ValueError):
        gd.DecoderV22(2, H, edge_types=np.full(int(H.sum()), 8))
    with pytest.raises(ValueError):                       # not a toric H: types required
        gd.DecoderV22(2, gd.codes.bch_63_45())
    m = gd.DecoderV22(2, gd.codes.bch_63_45(), edge_types=np.arange(432) % 8)
    assert m.packed_weights().numel() == 2 * 432 * 2 + 2 * 432 + 1


def test_per_layer_loss_matches_reference_lossfunc(golden):
    """PerLayerLoss (reference formula path) on the reference's own per-layer predictions
    reproduces the reference LossFunc(train=1) value."""
    import gnndecode as gd
    z = golden('train_v22_L4')
    H = golden('toric_L4_graph')['H']
    lf = gd.loss.PerLayerLoss(H, gd.codes.toric_logicals(H), fused=False)
    preds = [torch.from_numpy(p).unsqueeze(1) for p in z['pred']]
    loss = lf(preds, torch.from_numpy(z['y']))
    assert abs(loss.item() - float(z['loss'])) <= 1e-10 * max(1.0, abs(float(z['loss'])))


# ------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------
def _model(golden, T):
    import gnndecode as gd
    z = golden('v22_toric4')
    m = gd.DecoderV22(T, golden('toric_L4_graph')['H'])
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()
                       if not k.startswith('layers.') or int(k.split('.')[1]) < 2 * T})
    return z, m.to(DEV).eval()


def _fused(m, x):
    import gnndecode as gd
    with torch.no_grad():
        return m(gd.data.make_batch(x, m.graph(x.device)))


@pytest.mark.gpu
@pytest.mark.parametrize('B,T', CASES)
def test_v22_fused_decode_fp64(golden, B, T):
    z, m = _model(golden, T)
    import gnndecode as gd
    assert gd.ops.decode_plan(m.graph(DEV), 'v22', torch.float64)['kernel'] == 'decode_resident_kernel'
    x = torch.from_numpy(z[f'x_B{B}']).to(DEV)
    out = _fused(m, x)
    assert isinstance(out, list) and len(out) == T
    got = torch.stack([o.reshape(-1) for o in out]).cpu().numpy()
    ref = z[f'out_B{B}_T{T}']
    assert got.dtype == ref.dtype
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-12)
    assert ((got > 0.5) == (ref > 0.5)).all()


@pytest.mark.gpu
@pytest.mark.parametrize('B', (1, 8))
def test_v22_fused_decode_fp32(golden, B):
    z, m = _model(golden, 25)
    x = torch.from_numpy(z[f'x_B{B}']).to(DEV).float()
    out = _fused(m, x)
    got = torch.stack([o.reshape(-1) for o in out]).double().cpu().numpy()
    ref = z[f'out_B{B}_T25']
    assert np.abs(got - ref).max() <= 1e-4
    far = np.abs(ref - 0.5) >= 1e-3
    assert ((got > 0.5) == (ref > 0.5))[far].all()


@pytest.mark.gpu
@pytest.mark.parametrize('B,T', [c for c in CASES if c[1] <= 2 or c[0] == 1])
def test_v22_layerwise_operator_path(golden, B, T):
    """The reference's layer-by-layer loop on the device operator (NBP propagate bodies)."""
    import gnndecode as gd
    z, m = _model(golden, T)
    x = torch.from_numpy(z[f'x_B{B}']).to(DEV)
    with torch.no_grad():
        out = m.forward_layers(x, gd.data.make_batch(x, m.graph(x.device)).edge_index)
    got = torch.stack([o.reshape(-1) for o in out]).cpu().numpy()
    np.testing.assert_allclose(got, z[f'out_B{B}_T{T}'], rtol=1e-9, atol=1e-11)


@pytest.mark.gpu
def test_v22_training_step_gradients_match_reference(golden):
    """Layer path (HIP propagate forward/backward kernels) + PerLayerLoss + backward vs the
    reference's own autograd gradients of every parameter."""
    import gnndecode as gd
    z = golden('train_v22_L4')
    H = golden('toric_L4_graph')['H']
    m = gd.DecoderV22(int(z['T']), H)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()})
    m = m.to(DEV).train()
    x = torch.from_numpy(z['x']).to(DEV)
    y = torch.from_numpy(z['y']).to(DEV)
    lf = gd.loss.PerLayerLoss(H, gd.codes.toric_logicals(H)).to(DEV)
    pred = m(gd.data.make_batch(x, m.graph(x.device)))
    assert pred[0].requires_grad and len(pred) == int(z['T'])
    got = torch.stack([p.detach().reshape(-1) for p in pred]).cpu().numpy()
    np.testing.assert_allclose(got, z['pred'], rtol=1e-9, atol=1e-11)
    loss = lf(pred, y)
    assert abs(loss.item() - float(z['loss'])) <= 1e-9 * max(1, abs(float(z['loss'])))
    loss.backward()
    for name, p in m.named_parameters():
        key = 'g/' + name
        if key not in z.files:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, name
            continue
        ref = z[key]
        got = p.grad.detach().cpu().numpy()
        scale = max(np.abs(ref).max(), 1e-30)
        assert np.abs(got - ref).max() <= 1e-8 * scale, (name, np.abs(got - ref).max(), scale)


@pytest.mark.gpu
def test_v22_at_size_sampled_oracle_and_batch_independence(golden):
    """B = 65 536 fp64 decode vs the oracle on 32 sampled codewords (every layer's readout);
    the same codewords decoded alone give identical bits."""
    import gnndecode as gd
    z, m = _model(golden, 25)
    H = golden('toric_L4_graph')['H']
    B, T = 65536, 25
    x, _ = gd.data.toric_batch(torch.from_numpy(H), B, seed=22, device=DEV, dtype=torch.float64)
    out = torch.stack(_fused(m, x))                            # [T, B*V, 1]
    g = m.graph(DEV)
    rng = np.random.default_rng(22)
    pick = np.sort(np.concatenate([[0, B - 1], rng.choice(np.arange(1, B - 1), 30, replace=False)]))
    idx = torch.as_tensor(pick, device=DEV)
    xs = x.view(B, g.N)[idx]
    ref = np.stack([o.reshape(-1, g.V) for o in
                    O.decode('v22', H, xs.cpu().numpy().reshape(-1, 1), T, _w(z))])
    got = out.view(T, B, g.V)[:, idx].cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-12)
    assert ((got > 0.5) == (ref > 0.5)).all()
    alone = torch.stack(_fused(m, xs.reshape(-1, 1).contiguous())).view(T, -1, g.V).cpu()
    assert torch.equal(alone, torch.from_numpy(got))


@pytest.mark.gpu
def test_v22_empty_batch_and_zero_iterations(golden):
    import gnndecode as gd
    _, m = _model(golden, 25)
    g = m.graph(DEV)
    x = torch.empty(0, 1, dtype=torch.float64, device=DEV)
    out = gd.ops.decode(g, 'v22', x, 25, m.prepared_weights(torch.float64, DEV))
    assert out.numel() == 0
    m0 = gd.DecoderV22(0, golden('toric_L4_graph')['H']).to(DEV).eval()
    z = golden('v22_toric4')
    assert _fused(m0, torch.from_numpy(z['x_B1']).to(DEV)) == []
