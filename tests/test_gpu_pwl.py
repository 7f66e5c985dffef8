"""CGNNI / QGNNI message MLP as the piecewise-linear table of the fp32 resident decoder
(pwl_build_kernel / pwl_stage / pwl_eval in gnnd_decode_impl.h, built by
gnnd_prepare_weights into the prepared layout).

The MLP (Linear(1,10) -> ReLU -> Linear(10,1), classical/CGNNI.py:238-242,
quantum/QGNNI.py:207-214) is linear between its knots; the table holds it exactly (up to fp32
rounding).  Checked here: the prepared header of the shipped weights (valid, K <= 32 cells),
and decodes through the table against the numpy oracle (fp32: rtol 1e-4 / atol 2e-5,
identical hard decisions except bits within 1e-6 of 0.5) -- also for weights whose knots
crowd beyond two per cell at any K <= 32, where the decoder keeps the 10-unit MLP.
"""
import os

import numpy as np
import pytest
import torch

import gnn_oracle as O

pytestmark = pytest.mark.gpu


def _pwl_built():
    import gnndecode as gd
    return gd.ops.prepared_count('cgnni', torch.float32) == 328


# (GNND_MLP_PWL is off in release builds -- measured slower, gnnd_decode_impl.h; these tests run
# against a library built with -DGNND_MLP_PWL=1, loaded through GNND_LIB)
needs_pwl = pytest.mark.skipif('not _pwl_built()', reason='library built without GNND_MLP_PWL')

DEV = 'cuda'
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model(model, code, wfile):
    import gnndecode as gd
    H = gd.codes.get_code(code)
    m = gd.MODELS[model](gd.DEFAULT_ITERS[model], H)
    z = np.load(os.path.join(ROOT, 'gnn-decode_amd', 'gnndecode', 'weights', wfile))
    m.load_state_dict({k: torch.from_numpy(z[k]) for k in z.files})
    return m.to(DEV).eval(), H


def _check(m, H, model, B=96, seed=5):
    import gnndecode as gd
    if model == 'cgnni':
        x, _ = gd.data.awgn_batch(H, B, codewords='random', seed=seed, device=torch.device(DEV))
    else:
        x, _ = gd.data.toric_batch(H, B, seed=seed, device=torch.device(DEV), dtype=torch.float32)
    g = m.graph(x.device)
    assert gd.ops.decode_plan(g, model, torch.float32)['kernel'] == 'decode_resident_kernel'
    out = gd.ops.decode(g, model, x, m.Nc, m.prepared_weights(torch.float32, x.device))
    w = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    ref = O.decode(model, H, x.cpu().numpy(), m.Nc, w)
    got = out.cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=2e-5)
    far = np.abs(ref - 0.5) > 1e-6
    assert ((got > 0.5) == (ref > 0.5))[far].all()


@needs_pwl
@pytest.mark.parametrize('model,code,wfile', [('cgnni', 'bch_63_45', 'cgnni_bch_63_45.npz'),
                                              ('cgnni', 'ldpc_648_324', 'cgnni_ldpc_648_324.npz'),
                                              ('qgnni', 'toric_5', 'qgnni_toric_5.npz')])
def test_prepared_table_valid_and_decode_matches_oracle(model, code, wfile):
    import gnndecode as gd
    m, H = _model(model, code, wfile)
    prep = m.prepared_weights(torch.float32, torch.device(DEV))
    assert prep.numel() == gd.ops.prepared_count(model, torch.float32) == 328
    assert torch.equal(prep[:62], m.packed_weights().float().to(DEV))
    hdr = prep[64:72].cpu()
    assert hdr[0] == 1 and 1 <= hdr[1] <= 32
    _check(m, H, model)


@needs_pwl
def test_crowded_knots_keep_the_unit_mlp():
    """Three units with one knot: no cells hold it with at most two knots each, the table is
    marked invalid and the decoder evaluates the 10 units (still the oracle's function)."""
    m, H = _model('cgnni', 'bch_63_45', 'cgnni_bch_63_45.npz')
    with torch.no_grad():
        W1 = m.ggc2.mlp2[0].weight
        for k in range(3):                    # knots -b1/W1 = 0.25 (inside |u| <= 23)
            W1[k, 0] = 1.0 if k % 2 else -1.0
            m.ggc2.mlp2[0].bias[k] = -W1[k, 0] * 0.25
    prep = m.prepared_weights(torch.float32, torch.device(DEV))
    assert prep[64].item() == 0
    _check(m, H, 'cgnni')
