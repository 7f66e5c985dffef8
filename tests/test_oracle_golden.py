"""Pin the oracle (oracle/gnn_oracle.py) to golden vectors produced by the reference's own
class definitions (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

import gnn_oracle as O
from conftest import weights_of

# (fixture, model, code graph fixture)
DECODERS = [
    ('cgnni_bch', 'cgnni', 'bch_63_45_graph'),
    ('cgnni_bch_randinit', 'cgnni', 'bch_63_45_graph'),
    ('bp_bch', 'cbp', 'bch_63_45_graph'),
    ('bp_toric4', 'qbp', 'toric_L4_graph'),
    ('qgnni_toric4', 'qgnni', 'toric_L4_graph'),
    ('v24_toric5', 'v24', 'toric_L5_graph'),
    ('v24_toric7', 'v24', 'toric_L7_graph'),
    ('nbp_toric4', 'nbp', 'toric_L4_graph'),
    ('v10_toric4', 'v10', 'toric_L4_graph'),
    ('cgnni_ldpc', 'cgnni', 'ldpc_648_324_graph'),
    ('cgnni_ldpc_randinit', 'cgnni', 'ldpc_648_324_graph'),
    ('bp_ldpc', 'cbp', 'ldpc_648_324_graph'),
]


def _cases():
    for fx, model, gfx in DECODERS:
        z = np.load(f'tests/golden/{fx}.npz')
        for k in z.files:
            if k.startswith('out_'):
                _, b, t = k.split('_')
                yield pytest.param(fx, model, gfx, int(b[1:]), int(t[1:]), id=f'{fx}-{b}-{t}')


@pytest.mark.parametrize('fx,model,gfx,B,T', list(_cases()))
def test_oracle_decoder_matches_reference(golden, fx, model, gfx, B, T):
    z = golden(fx)
    H = golden(gfx)['H']
    out = O.decode(model, H, z[f'x_B{B}'], T, weights_of(z))
    ref = z[f'out_B{B}_T{T}']
    assert out.shape == ref.shape and out.dtype == ref.dtype
    if ref.dtype == np.float32:
        np.testing.assert_allclose(out, ref, rtol=2e-5, atol=2e-6)
    else:
        np.testing.assert_allclose(out, ref, rtol=1e-10, atol=1e-13)
    assert ((out > 0.5) == (ref > 0.5)).all()


def _prop_cases():
    for fx in ('propagate_ops', 'propagate_ops_nbp', 'propagate_ops_v30'):
        z = np.load(f'tests/golden/{fx}.npz')
        for k in z.files:
            parts = k.split('/')
            if len(parts) >= 3:
                yield pytest.param(fx, k, id=f'{fx}:{k}')


@pytest.mark.parametrize('fx,key', list(_prop_cases()))
def test_oracle_propagate_matches_reference(golden, fx, key):
    z = golden(fx)
    tag, flow, aggr = key.split('/')[:3]
    extra = None if key.endswith('nopost') else z[f'{tag}/extra']
    out = O.propagate(tag, flow, aggr, z[f'{tag}/edge_index'], z[f'{tag}/msg'], extra,
                      z[f'{tag}/extra'].shape[0])
    ref = z[key]
    assert out.shape == ref.shape
    tol = dict(rtol=1e-5, atol=5e-6) if ref.dtype == np.float32 else dict(rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(out, ref, **tol)


def test_toric_failure_metric_counts(golden):
    """Hard FER rule (quantum/neural_BP.py:338-348) on the v2_4 fixture outputs."""
    z = golden('v24_toric5')
    g = golden('toric_L5_graph')
    bad_syn, bad_log = O.toric_failures(g['H'], g['logical'], z['y_B32'], z['out_B32_T15'])
    assert 0 <= bad_syn <= 32 and 0 <= bad_log <= 32
    # predicting the true error exactly is a perfect decode
    y = z['y_B32']
    assert O.toric_failures(g['H'], g['logical'], y, y.astype(np.float64)) == (0, 0)
    # predicting no error fails exactly on the codewords with a non-zero syndrome
    nz = int((golden('v24_toric5')['x_B32'].reshape(32, -1)[:, 100:] < 0).any(axis=1).sum())
    assert O.toric_failures(g['H'], g['logical'], y, np.zeros_like(y))[0] == nz


@pytest.mark.parametrize('L', [5, 7])
def test_toric_failure_rule_matches_reference_lossfunc(golden, L):
    """The oracle's hard FER rule == the reference's own LossFunc(train=0) count
    (quantum/neural_BP.py:338-348) on crafted decodes: syndrome failures, pure logical
    failures, stabiliser-equivalent successes, exact-0.5 ties (tests/golden/make_golden.py
    gen_fer)."""
    z = golden('fer_rule')
    g = golden(f'toric_L{L}_graph')
    syn, lg = O.toric_failures(g['H'], g['logical'], z[f'L{L}/y'], z[f'L{L}/pred'])
    assert syn + lg == int(z[f'L{L}/count'])
    assert syn > 0 and lg > 0


def test_toric_failure_rule_on_decoder_outputs(golden):
    z = golden('v24_toric5')
    g = golden('toric_L5_graph')
    syn, lg = O.toric_failures(g['H'], g['logical'], z['y_B32'], z['out_B32_T15'])
    assert syn + lg == int(golden('fer_rule')['v24_B32/count'])


def test_ldpc_graph_matches_framework_code(golden):
    import gnndecode as gd
    np.testing.assert_array_equal(golden('ldpc_648_324_graph')['H'], gd.codes.wifi_ldpc_648())


@pytest.mark.parametrize('L', [5, 7])
def test_torch_training_restatement_matches_reference_gradients(golden, L):
    """oracle/torch_train.py (the train-mode CPU baseline) reproduces the reference's own
    forward, LossFunc and parameter gradients (tests/golden/train_v24_L*.npz)."""
    import torch
    import torch_train
    z = golden(f'train_v24_L{L}')
    g = golden(f'toric_L{L}_graph')
    st = torch_train.V24Step(g['H'], g['logical'], weights_of(z), int(z['T']))
    pred = st.forward(torch.from_numpy(z['x']))
    np.testing.assert_allclose(pred.detach().numpy().reshape(-1, 1), z['pred'], rtol=1e-10, atol=1e-13)
    loss = st.loss(pred, torch.from_numpy(z['y']))
    assert abs(loss.item() - float(z['loss'])) <= 1e-9 * abs(float(z['loss']))
    loss.backward()
    for k, p in st.p.items():
        np.testing.assert_allclose(p.grad.numpy(), z['g/' + k], rtol=1e-8, atol=1e-11)
