"""Reference checkpoints <-> gnndecode models.

The reference saves `decoder.state_dict()` with `torch.save` (e.g.
quantum/decoder_v2_4.py:344, classical/CGNNI.py `./model/decoder_parameters_epoch%d.pkl`),
often from CUDA tensors.  Those files are read here with `torch.load(weights_only=True,
map_location='cpu')` only (no unpickling of code), and the gnndecode models keep the
reference's attribute names, so the state_dict loads unchanged.  `.npz` is the portable
form (one array per state_dict key), used by the golden fixtures and by the C-ABI users
that pack weights themselves.
"""
import numpy as np
import torch


def load_reference(path):
    """state_dict of a reference checkpoint (.pkl/.pt via torch.load weights_only, or .npz)."""
    if str(path).endswith('.npz'):
        with np.load(path, allow_pickle=False) as z:
            return {k: torch.from_numpy(np.array(z[k])) for k in z.files}
    sd = torch.load(path, map_location='cpu', weights_only=True)
    if not isinstance(sd, dict):
        raise TypeError(f'{path}: expected a state_dict, got {type(sd).__name__}')
    return {k: v.detach().cpu() for k, v in sd.items()}


def save_npz(state, path):
    np.savez(path, **{k: v.detach().cpu().numpy() for k, v in state.items()})


def load_into(model, path_or_state, strict=True):
    """Load a reference checkpoint into a gnndecode model.  Weighted-BP decoders built with
    fewer layers than the checkpoint take its first 2 Nc layers (the reference's per-layer
    tables are indexed by iteration)."""
    state = load_reference(path_or_state) if isinstance(path_or_state, str) else dict(path_or_state)
    nlayers = getattr(model, 'layers', None)
    if nlayers is not None:
        n = len(nlayers)
        state = {k: v for k, v in state.items()
                 if not k.startswith('layers.') or int(k.split('.')[1]) < n}
    own = model.state_dict()
    state = {k: v.to(own[k].dtype) if k in own else v for k, v in state.items()}
    return model.load_state_dict(state, strict=strict)
