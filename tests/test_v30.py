"""decoder_v3_0 (quantum/decoder_v3_0.py:199-335: GRU edge states, two-output readout) —
oracle and loss vs the reference-generated goldens (CPU), and the HIP path through the C ABI
vs the goldens and the oracle (`-m gpu`).

Tolerances: fp64 (the script's dtype) soft outputs rtol 1e-10 with identical hard decisions;
fp32 kernels |dp| <= 1e-4 with identical decisions outside |p - 0.5| < 1e-3; training
gradients 1e-8 relative to the largest reference gradient (fp64)."""
import numpy as np
import pytest
import torch

import gnn_oracle as O
from conftest import weights_of

DEV = 'cuda'
CASES = [(B, T) for B in (1, 4) for T in (1, 2, 15)]


# ------------------------------------------------------------------------------------
# CPU: oracle and loss restatements vs the reference
# ------------------------------------------------------------------------------------
@pytest.mark.parametrize('B,T', CASES)
def test_oracle_v30_matches_reference(golden, B, T):
    z = golden('v30_toric5')
    H = golden('toric_L5_graph')['H']
    o0, o1 = O.decode('v30', H, z[f'x_B{B}'], T, weights_of(z))
    for got, key in ((o0, f'out0_B{B}_T{T}'), (o1, f'out1_B{B}_T{T}')):
        ref = z[key]
        assert got.shape == ref.shape
        np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-14)


def test_v30_loss_matches_reference_lossfunc(golden):
    """V30Loss on the reference outputs reproduces the reference LossFunc value (including
    its stride-V column slicing and first-codeword y)."""
    import gnndecode as gd
    z = golden('train_v30_L5')
    H = golden('toric_L5_graph')['H']
    lf = gd.loss.V30Loss(torch.from_numpy(H.astype(np.float64)))
    preds = [torch.from_numpy(z['pred0']), torch.from_numpy(z['pred1'])]
    loss = lf(preds, torch.from_numpy(z['y']), torch.from_numpy(z['x']))
    assert abs(loss.item() - float(z['loss'])) <= 1e-12 * max(1.0, abs(float(z['loss'])))


def test_v30_state_dict_keys_match_reference(golden):
    import gnndecode as gd
    z = golden('v30_toric5')
    m = gd.DecoderV30(15, golden('toric_L5_graph')['H'])
    assert sorted(m.state_dict().keys()) == sorted(weights_of(z).keys())
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()})
    assert m.packed_weights().numel() == 137


# ------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------
def _model(golden, T, dtype=torch.float64):
    import gnndecode as gd
    z = golden('v30_toric5')
    m = gd.DecoderV30(T, golden('toric_L5_graph')['H'])
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()})
    return z, m.to(DEV).eval()


def _fused(m, x):
    import gnndecode as gd
    with torch.no_grad():
        return m(gd.data.make_batch(x, m.graph(x.device)))


@pytest.mark.gpu
@pytest.mark.parametrize('B,T', CASES)
def test_v30_fused_decode_fp64(golden, B, T):
    z, m = _model(golden, T)
    x = torch.from_numpy(z[f'x_B{B}']).to(DEV)
    out = _fused(m, x)
    assert isinstance(out, list) and len(out) == 2
    for got, key in zip(out, (f'out0_B{B}_T{T}', f'out1_B{B}_T{T}')):
        ref = z[key]
        got = got.cpu().numpy()
        assert got.shape == ref.shape and got.dtype == ref.dtype
        np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-12)
        assert ((got > 0.5) == (ref > 0.5)).all()


@pytest.mark.gpu
@pytest.mark.parametrize('B,T', [c for c in CASES if c[1] == 15])
def test_v30_fused_decode_fp32(golden, B, T):
    z, m = _model(golden, T)
    x = torch.from_numpy(z[f'x_B{B}']).to(DEV).float()
    out = _fused(m, x)
    for got, key in zip(out, (f'out0_B{B}_T{T}', f'out1_B{B}_T{T}')):
        ref = z[key]
        got = got.double().cpu().numpy()
        assert np.abs(got - ref).max() <= 1e-4
        far = np.abs(ref - 0.5) >= 1e-3
        assert ((got > 0.5) == (ref > 0.5))[far].all()


@pytest.mark.gpu
@pytest.mark.parametrize('B,T', [c for c in CASES if c[0] <= 4])
def test_v30_layerwise_operator_path(golden, B, T):
    """The reference's layer-by-layer loop: propagate on the device operator + torch GRUCell."""
    import gnndecode as gd
    z, m = _model(golden, T)
    x = torch.from_numpy(z[f'x_B{B}']).to(DEV)
    with torch.no_grad():
        out = m.forward_layers(x, gd.data.make_batch(x, m.graph(x.device)).edge_index)
    for got, key in zip(out, (f'out0_B{B}_T{T}', f'out1_B{B}_T{T}')):
        np.testing.assert_allclose(got.cpu().numpy(), z[key], rtol=1e-9, atol=1e-11)


@pytest.mark.gpu
def test_v30_training_step_gradients_match_reference(golden):
    """Forward (layer path, HIP propagate forward/backward kernels, torch GRUCell autograd)
    + reference LossFunc + backward vs the reference's own autograd gradients."""
    import gnndecode as gd
    z = golden('train_v30_L5')
    H = golden('toric_L5_graph')['H']
    m = gd.DecoderV30(int(z['T']), H)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()})
    m = m.to(DEV).train()
    x = torch.from_numpy(z['x']).to(DEV)
    y = torch.from_numpy(z['y']).to(DEV)
    lf = gd.loss.V30Loss(torch.from_numpy(H.astype(np.float64))).to(DEV)
    pred = m(gd.data.make_batch(x, m.graph(x.device)))
    assert pred[0].requires_grad
    np.testing.assert_allclose(pred[0].detach().cpu().numpy(), z['pred0'], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(pred[1].detach().cpu().numpy(), z['pred1'], rtol=1e-10, atol=1e-12)
    loss = lf(pred, y, x)
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
def test_v30_trainer_step_runs_with_input_aware_loss(golden):
    """Trainer passes x to losses that need it (V30Loss) — eager and HIP-graph replay agree."""
    import gnndecode as gd
    z = golden('train_v30_L5')
    H = golden('toric_L5_graph')['H']
    res = []
    for graph in (False, True):
        m = gd.DecoderV30(5, H)
        m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()})
        m = m.to(DEV)
        lf = gd.loss.V30Loss(torch.from_numpy(H.astype(np.float64))).to(DEV)
        tr = gd.train.Trainer(m, lf, graph=graph, warmup=1, capturable=True)
        x = torch.from_numpy(z['x']).to(DEV)
        y = torch.from_numpy(z['y']).to(DEV)
        data = gd.data.make_batch(x, m.graph(x.device))
        res.append([float(tr.step(data, y)) for _ in range(3)])
    assert all(abs(a - b) <= 1e-9 * max(1, abs(a)) for a, b in zip(*res)), res


@pytest.mark.gpu
def test_v30_at_size_sampled_oracle_and_batch_independence(golden):
    """B = 65 536 (config-3 size) fp64 decode vs the oracle on 32 sampled codewords; the
    same codewords decoded alone give identical bits."""
    import gnndecode as gd
    z, m = _model(golden, 15)
    H = golden('toric_L5_graph')['H']
    B = 65536
    x, _ = gd.data.toric_batch(torch.from_numpy(H), B, seed=30, device=DEV, dtype=torch.float64)
    out = _fused(m, x)
    g = m.graph(DEV)
    rng = np.random.default_rng(3)
    pick = np.sort(np.concatenate([[0, B - 1], rng.choice(np.arange(1, B - 1), 30, replace=False)]))
    xs = x.view(B, g.N)[torch.as_tensor(pick, device=DEV)]
    r0, r1 = O.decode('v30', H, xs.cpu().numpy().reshape(-1, 1), 15, weights_of(z))
    got0 = out[0].view(B, g.N)[torch.as_tensor(pick, device=DEV)].cpu().numpy().reshape(-1, 1)
    got1 = out[1].view(B, g.N)[torch.as_tensor(pick, device=DEV)].cpu().numpy().reshape(-1, 1)
    np.testing.assert_allclose(got0, r0, rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(got1, r1, rtol=1e-10, atol=1e-12)
    alone = _fused(m, xs.reshape(-1, 1).contiguous())
    assert torch.equal(alone[0].cpu(), torch.from_numpy(got0))
    assert torch.equal(alone[1].cpu(), torch.from_numpy(got1))


@pytest.mark.gpu
def test_v30_empty_batch(golden):
    import gnndecode as gd
    _, m = _model(golden, 15)
    g = m.graph(DEV)
    x = torch.empty(0, 1, dtype=torch.float64, device=DEV)
    out = gd.ops.decode(g, 'v30', x, 15, m.prepared_weights(torch.float64, DEV))
    assert out.numel() == 0


def test_v30_loss_and_grad_matches_autograd_cpu():
    """V30Loss.loss_and_grad (the fused trainer's loss: the check term through SyndromeLoss,
    the BCE term and its gradient by formula, gathered rows of out1 and x) equals torch
    autograd of the reference LossFunc restatement, on a view with a storage offset (CPU: the
    check term takes SyndromeLoss's reference formula there)."""
    import gnndecode as gd
    H = torch.as_tensor(gd.codes.toric_code(5), dtype=torch.float64)
    lf = gd.loss.V30Loss(H)
    a, b = lf.a, lf.b
    N, B = a + b, 6
    g = torch.Generator().manual_seed(0)
    base = torch.rand(2 * B * N + 7, 1, generator=g, dtype=torch.float64) * 0.9 + 0.05
    out = base[7:]
    y = (torch.rand(B * a, 1, generator=g) < 0.1).double()
    x = torch.rand(B * N, 1, generator=g, dtype=torch.float64)
    x.view(B, N)[:, a:] = (torch.rand(B, b, generator=g) < 0.5).double()
    n = B * N
    o = out.detach().clone().requires_grad_(True)
    ref = lf([o[:n], o[n:]], y, x)
    (dref,) = torch.autograd.grad(ref, o)
    loss, d = lf.loss_and_grad(out, y, x)
    assert abs(loss.item() - ref.item()) <= 1e-12 * abs(ref.item())
    assert (d - dref).abs().max().item() <= 1e-12 * dref.abs().max().item()
