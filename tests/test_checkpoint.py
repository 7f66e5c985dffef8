"""Reference-checkpoint loading (weights_only) and the .npz form.  CPU only."""
import numpy as np
import torch

import gnndecode as gd
from conftest import weights_of


def test_reference_state_dict_roundtrip(golden, tmp_path):
    z = golden('v24_toric5')                     # weights of quantum/new_model/...epoch67.pkl
    sd = {k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()}
    pkl = tmp_path / 'decoder_parameters_epoch67.pkl'
    torch.save(sd, pkl)                           # the reference's torch.save(state_dict)
    m = gd.DecoderV24(15, golden('toric_L5_graph')['H'])
    gd.checkpoint.load_into(m, str(pkl))
    for k, v in m.state_dict().items():
        np.testing.assert_array_equal(v.numpy(), sd[k].numpy())
    npz = tmp_path / 'w.npz'
    gd.checkpoint.save_npz(m.state_dict(), npz)
    m2 = gd.DecoderV24(15, golden('toric_L5_graph')['H'])
    gd.checkpoint.load_into(m2, str(npz))
    assert all(torch.equal(a, b) for a, b in zip(m.state_dict().values(), m2.state_dict().values()))


def test_weighted_bp_takes_leading_layers(golden):
    z = golden('nbp_toric4')
    sd = {k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()}
    m = gd.NeuralBP(2, golden('toric_L4_graph')['H'])
    gd.checkpoint.load_into(m, sd)
    np.testing.assert_array_equal(m.layers[3].W_p.detach().numpy(), sd['layers.3.W_p'].numpy())
    np.testing.assert_array_equal(m.W.detach().numpy(), sd['W'].numpy())
