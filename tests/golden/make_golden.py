"""Golden-vector generator (container-only; NOT shipped, NOT run on the GPU box).

Runs the reference's OWN class definitions on CPU to produce small seeded input/output
fixtures (`tests/golden/*.npz`) that pin the oracle (`oracle/gnn_oracle.py`) and, through
it, the HIP path.  Nothing from the reference is copied into the repo: at generation time
this script reads the reference files under /root/reference as text, keeps only the named
FunctionDef/ClassDef nodes (SURVEY.md Appendix C recipe) and `exec`s them against:

* a `torch_scatter` 1.x shim: `scatter_add` = `zeros(dim_size).index_add_(0, idx, src)`
  (sequential edge-order accumulation, as CPU torch_scatter) and `scatter_max` =
  `full(fill).scatter_reduce('amax', include_self=True)`;
* a PyG-1.x `scatter_` equal to the local replica at quantum/decoder_v2_4.py:34-51
  (fill 0 for add/mean, -1e9 for max, fill mapped back to 0 for max);
* `torch.Tensor.cuda = identity`, injected globals `rows`, `cols`, `BATCH_SIZE`, `H`;
* PyG `Batch` collation restated: `edge_index` tiled with `b*N` node offsets.

Checkpoints are read with `torch.load(..., weights_only=True)` only.
Seeds are explicit (the reference sets none).

Usage:  python tests/golden/make_golden.py      (writes tests/golden/*.npz)
"""
import ast
import math
import os
import random
import sys
import types
import inspect

import numpy as np
import torch

REF = '/root/reference/GNN-decode'
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------------------
# shims for the absent third-party packages (torch_scatter 1.x, torch_geometric <= 1.5)
# --------------------------------------------------------------------------------------
def _ts_scatter_add(src, index, dim=-1, out=None, dim_size=None, fill_value=0):
    assert dim == 0
    if dim_size is None:
        dim_size = int(index.max()) + 1
    res = torch.full((dim_size,) + tuple(src.shape[1:]), float(fill_value), dtype=src.dtype)
    return res.index_add_(0, index, src)


def _ts_scatter_max(src, index, dim=-1, out=None, dim_size=None, fill_value=None):
    assert dim == 0
    if dim_size is None:
        dim_size = int(index.max()) + 1
    fill = -1e9 if fill_value is None else float(fill_value)
    res = torch.full((dim_size,) + tuple(src.shape[1:]), fill, dtype=src.dtype)
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    res = res.scatter_reduce(0, idx, src, reduce='amax', include_self=True)
    return res, None


def _ts_scatter_mean(src, index, dim=-1, out=None, dim_size=None, fill_value=0):
    s = _ts_scatter_add(src, index, dim, out, dim_size, fill_value)
    c = _ts_scatter_add(torch.ones_like(src), index, dim, None, s.size(0), 0)
    return s / c.clamp(min=1)


torch_scatter = types.ModuleType('torch_scatter')
torch_scatter.scatter_add = _ts_scatter_add
torch_scatter.scatter_max = _ts_scatter_max
torch_scatter.scatter_mean = _ts_scatter_mean


def pyg_scatter_(name, src, index, dim_size=None):
    """PyG-1.x utils.scatter_ (same rule as the local replica at decoder_v2_4.py:34-51)."""
    assert name in ['add', 'mean', 'max']
    op = getattr(torch_scatter, 'scatter_{}'.format(name))
    fill_value = -1e9 if name == 'max' else 0
    out = op(src, index, 0, None, dim_size, fill_value)
    if isinstance(out, tuple):
        out = out[0]
    if name == 'max':
        out[out == fill_value] = 0
    return out


torch.Tensor.cuda = lambda self, *a, **k: self


def load_ref(relpath, names, **globs):
    path = os.path.join(REF, relpath)
    tree = ast.parse(open(path).read(), path)
    keep = []
    for node in tree.body:
        if isinstance(node, (ast.FunctionDef, ast.ClassDef)) and node.name in names:
            keep.append(node)
        elif isinstance(node, ast.Assign) and any(
                isinstance(t, ast.Name) and t.id in ('special_args', '__size_error_msg__')
                for t in node.targets):
            keep.append(node)
    ns = dict(torch=torch, math=math, inspect=inspect, np=np,
              Variable=torch.autograd.Variable, F=torch.nn.functional,
              torch_scatter=torch_scatter, scatter_add=_ts_scatter_add,
              scatter_=pyg_scatter_)
    ns.update(globs)
    exec(compile(ast.Module(body=keep, type_ignores=[]), path, 'exec'), ns)
    return ns


def single_edge_index(H):
    """H [V, C]; reference: `H.to_sparse()._indices()` (coalesced, sorted by (v, c))."""
    return H.to_sparse()._indices()


def batch_edge_index(ei, B, N):
    """PyG-1.x collation: concatenate per-graph edge_index adding b*N (Batch.from_data_list)."""
    E = ei.size(1)
    off = torch.arange(B).repeat_interleave(E) * N
    return ei.repeat(1, B) + off.unsqueeze(0)


def set_seed(s):
    random.seed(s)
    np.random.seed(s)
    torch.manual_seed(s)


def bch_H():
    Hm = np.loadtxt(os.path.join(REF, 'classical', 'BCH(63,45).txt'))   # [18, 63]
    return torch.from_numpy(Hm).float().t()                                # [63, 18] as CGNNI.py:181


def awgn_llr(B, n, codeword_bit, seed, snrs=(1, 2, 3, 4, 5, 6)):
    """BPSK/AWGN LLRs following Gen_Data (classical/CGNNI.py:125-147): sigma^2 = 10^(-SNR/10),
    y = (1-2c) + N(0, sigma^2), LLR = 2 y / sigma^2 (float32).  SNR cycles over the grid."""
    g = torch.Generator().manual_seed(seed)
    snr = torch.tensor([snrs[b % len(snrs)] for b in range(B)], dtype=torch.float32)
    sigma = (1 / (10 ** (snr / 10))) ** 0.5
    xm = 1 - 2 * float(codeword_bit)
    noise = torch.normal(0.0, sigma.unsqueeze(1).repeat(1, n), generator=g)
    y = xm + noise
    llr = 2 * y * (1 / (sigma ** 2)).unsqueeze(1)
    return llr.float(), snr


def classical_x(llr, C):
    """CustomDataset (classical/CGNNI.py:157-161): x = [LLR (V); zeros (C)] per codeword."""
    B, V = llr.shape
    x = torch.cat([llr, torch.zeros(B, C)], dim=1)
    return x.reshape(B * (V + C), 1)


def run_model(ns, H, x, B, T, state=None, dtype=torch.float32):
    V, C = H.size(0), H.size(1)
    N = V + C
    ns['rows'], ns['cols'], ns['BATCH_SIZE'], ns['H'] = V, C, B, H
    ei = batch_edge_index(single_edge_index(H), B, N)
    model = ns['GNNI'](T)
    if state is not None:
        model.load_state_dict(state)
    data = types.SimpleNamespace(x=x, edge_index=ei)
    with torch.no_grad():
        out = model(data)
    return out, model


def sd_to_np(state):
    return {'w/' + k: v.detach().cpu().numpy() for k, v in state.items()}


def save(name, **arrays):
    path = os.path.join(OUT, name + '.npz')
    np.savez_compressed(path, **arrays)
    print('wrote', path, sum(a.nbytes for a in arrays.values()), 'bytes')


# --------------------------------------------------------------------------------------
def gen_classical():
    H = bch_H()
    V, C = H.shape
    ei = single_edge_index(H)
    save('bch_63_45_graph', H=H.numpy().astype(np.uint8), edge_index=ei.numpy())

    # ---- CGNNI (classical/CGNNI.py), epoch-18 checkpoint, all-ones codeword
    ns = load_ref('classical/CGNNI.py', {'MessagePassing', 'GatedGraphConv', 'GNNI'})
    sd = torch.load(os.path.join(REF, 'classical/model/decoder_parameters_epoch18.pkl'),
                    map_location='cpu', weights_only=True)
    arrays = dict(sd_to_np(sd))
    for B, seed in ((1, 11), (4, 12), (32, 13)):
        llr, snr = awgn_llr(B, V, 1, seed)
        x = classical_x(llr, C)
        arrays[f'x_B{B}'] = x.numpy()
        for T in (1, 2, 25):
            out, _ = run_model(ns, H, x, B, T, sd)
            arrays[f'out_B{B}_T{T}'] = out.numpy()
    save('cgnni_bch', **arrays)

    # CGNNI with seeded random init (different weights exercise other MLP regions)
    set_seed(101)
    ns['rows'], ns['cols'], ns['BATCH_SIZE'], ns['H'] = V, C, 8, H
    m0 = ns['GNNI'](25)
    sd_r = {k: v.clone() for k, v in m0.state_dict().items()}
    arrays = dict(sd_to_np(sd_r))
    llr, _ = awgn_llr(8, V, 0, 14)
    x = classical_x(llr, C)
    arrays['x_B8'] = x.numpy()
    for T in (1, 25):
        out, _ = run_model(ns, H, x, 8, T, sd_r)
        arrays[f'out_B8_T{T}'] = out.numpy()
    save('cgnni_bch_randinit', **arrays)

    # ---- classical BP (classical/BP.py), all-zeros codeword
    ns = load_ref('classical/BP.py', {'MessagePassing', 'GatedGraphConv', 'GNNI'})
    arrays = {}
    for B, seed in ((1, 21), (32, 22)):
        llr, snr = awgn_llr(B, V, 0, seed)
        x = classical_x(llr, C)
        arrays[f'x_B{B}'] = x.numpy()
        for T in (1, 2, 25):
            out, _ = run_model(ns, H, x, B, T)
            arrays[f'out_B{B}_T{T}'] = out.numpy()
    save('bp_bch', **arrays)


def toric_inputs(eg, H, L, P, run, seed):
    set_seed(seed)
    ds = eg.gen_syn(P, L, H, run)
    xs = torch.cat([ds[i].t() for i in range(0, len(ds), 2)], dim=0)      # [B*N, 1]
    ys = torch.cat([ds[i + 1].t() for i in range(0, len(ds), 2)], dim=0)  # [B*V, 1]
    return xs.double(), ys.double()


def gen_quantum():
    sys.path.insert(0, os.path.join(REF, 'quantum'))
    import error_generate as eg

    # ---- toric code construction fixtures (quantum/error_generate.py)
    for L in (4, 5, 7):
        Hnp, _ = eg.generate_PCM(2 * L * L - 2, L)
        H = torch.from_numpy(Hnp).t()
        h_prep = eg.H_Prep(H.t())
        H_prep = torch.from_numpy(h_prep.get_H_Prep())
        logical, stab = h_prep.get_logical(H_prep)
        save(f'toric_L{L}_graph', H=H.numpy().astype(np.uint8),
             edge_index=single_edge_index(H).numpy(),
             logical=logical.numpy().astype(np.uint8))

    def toric_H(L):
        Hnp, _ = eg.generate_PCM(2 * L * L - 2, L)
        return torch.from_numpy(Hnp).t()

    # seeded sampler draws (distribution reference for the on-device sampler)
    H5 = toric_H(5)
    xs, ys = toric_inputs(eg, H5, 5, [0.01, 0.05, 0.1], 64, 31)
    save('toric_L5_gen_syn', x=xs.numpy(), y=ys.numpy())

    # ---- quantum BP (quantum/BP.py), L = 4, T = 10
    H4 = toric_H(4)
    ns = load_ref('quantum/BP.py', {'MessagePassing', 'GatedGraphConv', 'GNNI'})
    arrays = {}
    for B, seed in ((1, 41), (32, 42)):
        x, y = toric_inputs(eg, H4, 4, [0.05, 0.1], B, seed)
        arrays[f'x_B{B}'], arrays[f'y_B{B}'] = x.numpy(), y.numpy()
        for T in (1, 2, 10):
            out, _ = run_model(ns, H4, x, B, T)
            arrays[f'out_B{B}_T{T}'] = out.numpy()
    save('bp_toric4', **arrays)

    # ---- QGNNI (quantum/QGNNI.py), L = 4, T = 25, seeded default init
    ns = load_ref('quantum/QGNNI.py', {'MessagePassing', 'GraphConv', 'GNNI'})
    set_seed(51)
    ns['rows'], ns['cols'], ns['BATCH_SIZE'], ns['H'] = H4.size(0), H4.size(1), 1, H4
    sd = {k: v.clone() for k, v in ns['GNNI'](25).state_dict().items()}
    arrays = dict(sd_to_np(sd))
    for B, seed in ((1, 52), (32, 53)):
        x, y = toric_inputs(eg, H4, 4, [0.05, 0.1], B, seed)
        arrays[f'x_B{B}'], arrays[f'y_B{B}'] = x.numpy(), y.numpy()
        for T in (1, 2, 25):
            out, _ = run_model(ns, H4, x, B, T, sd)
            arrays[f'out_B{B}_T{T}'] = out.numpy()
    save('qgnni_toric4', **arrays)

    # ---- decoder_v2_4 (quantum/decoder_v2_4.py), L = 5, T = 15, epoch-67 checkpoint
    names = {'scatter_mean', 'scatter_', 'MessagePassing', 'GraphConv', 'GNNI',
             'init_weights', 'init_weights_2'}
    ns = load_ref('quantum/decoder_v2_4.py', names)
    sd = torch.load(os.path.join(REF, 'quantum/new_model/decoder_parameters_epoch67.pkl'),
                    map_location='cpu', weights_only=True)
    arrays = dict(sd_to_np(sd))
    for B, seed in ((1, 61), (4, 62), (32, 63)):
        x, y = toric_inputs(eg, H5, 5, [0.01, 0.05, 0.1], B, seed)
        arrays[f'x_B{B}'], arrays[f'y_B{B}'] = x.numpy(), y.numpy()
        for T in (1, 2, 15):
            out, _ = run_model(ns, H5, x, B, T, sd)
            arrays[f'out_B{B}_T{T}'] = out.numpy()
    save('v24_toric5', **arrays)

    # decoder_v2_4 architecture at L = 7 (config 5), seeded Kaiming init as the reference
    H7 = toric_H(7)
    set_seed(71)
    ns['rows'], ns['cols'], ns['BATCH_SIZE'], ns['H'] = H7.size(0), H7.size(1), 1, H7
    sd7 = {k: v.clone() for k, v in ns['GNNI'](15).state_dict().items()}
    arrays = dict(sd_to_np(sd7))
    x, y = toric_inputs(eg, H7, 7, [0.01, 0.05, 0.1], 8, 72)
    arrays['x_B8'], arrays['y_B8'] = x.numpy(), y.numpy()
    out, _ = run_model(ns, H7, x, 8, 15, sd7)
    arrays['out_B8_T15'] = out.numpy()
    save('v24_toric7', **arrays)

    # ---- operator-level fixtures: one bare `propagate` call per script variant, with the
    # base class's identity `update`, on random per-edge messages.
    gen_propagate(eg, H5, H4)


def gen_propagate(eg, H5, H4):
    arrays = {}
    B = 3
    specs = [
        # (tag, script, H, dtype, flows, aggrs, second-arg name)
        ('v24', 'quantum/decoder_v2_4.py', H5, torch.float64, ('add', 'mean', 'max'), 'extra'),
        ('qgnni', 'quantum/QGNNI.py', H4, torch.float64, ('add',), 'extra'),
        ('qbp', 'quantum/BP.py', H4, torch.float64, ('add',), 'extra'),
        ('cgnni', 'classical/CGNNI.py', bch_H(), torch.float32, ('add',), 'post'),
        ('cbp', 'classical/BP.py', bch_H(), torch.float32, ('add',), 'extra'),
    ]
    g = torch.Generator().manual_seed(81)
    for tag, script, H, dt, aggrs, argname in specs:
        names = {'MessagePassing'}
        if 'decoder_v2_4' in script:
            names |= {'scatter_mean', 'scatter_'}
        ns = load_ref(script, names)
        V, C = H.shape
        N = V + C
        ei = batch_edge_index(single_edge_index(H), B, N)
        ei = torch.stack([ei[0], ei[1] + V])                      # GNNI.forward's shift
        E = ei.size(1)
        arrays[f'{tag}/edge_index'] = ei.numpy()
        m = (torch.randn(E, 1, generator=g) * 3).to(dt)
        xv = (torch.randn(B, V, generator=g) * 2)
        xc = torch.where(torch.rand(B, C, generator=g) < 0.3, -1.0, 1.0)
        extra = torch.cat([xv, xc], dim=1).reshape(B * N, 1).to(dt)
        arrays[f'{tag}/msg'] = m.numpy()
        arrays[f'{tag}/extra'] = extra.numpy()
        for flow in ('source_to_target', 'target_to_source'):
            for aggr in aggrs:
                mp = ns['MessagePassing'](aggr, flow)
                with torch.no_grad():
                    kw = {argname: extra}
                    out = mp.propagate(edge_index=ei, size=(N * B, N * B), x=m, **kw)
                arrays[f'{tag}/{flow}/{aggr}'] = out.numpy()
                if tag == 'cgnni':           # classical CGNNI also calls it with post=None (c->v)
                    with torch.no_grad():
                        out = mp.propagate(edge_index=ei, post=None, size=(N * B, N * B), x=m)
                    arrays[f'{tag}/{flow}/{aggr}/nopost'] = out.numpy()
    save('propagate_ops', **arrays)


def grads_of(model):
    return {'g/' + k: p.grad.detach().numpy().copy() for k, p in model.named_parameters()
            if p.grad is not None}


def gen_training():
    """One forward + reference LossFunc + backward per trainable model: loss value and
    parameter gradients (pins the training path)."""
    sys.path.insert(0, os.path.join(REF, 'quantum'))
    import error_generate as eg

    def toric(L):
        Hnp, _ = eg.generate_PCM(2 * L * L - 2, L)
        H = torch.from_numpy(Hnp).t()
        hp = eg.H_Prep(H.t())
        H_prep = torch.from_numpy(hp.get_H_Prep())
        logical, _ = hp.get_logical(H_prep)
        return H, H_prep, logical

    # decoder_v2_4 at L = 5 (epoch-67 weights) and L = 7 (seeded init, config 5 shape)
    for L, ckpt, B, T, seed in ((5, 'quantum/new_model/decoder_parameters_epoch67.pkl', 4, 15, 91),
                                (7, None, 2, 15, 92)):
        H, H_prep, logical = toric(L)
        names = {'scatter_mean', 'scatter_', 'MessagePassing', 'GraphConv', 'GNNI',
                 'init_weights', 'init_weights_2', 'LossFunc'}
        ns = load_ref('quantum/decoder_v2_4.py', names, logical=logical)
        x, y = toric_inputs(eg, H, L, [0.05, 0.1], B, seed)
        V, C = H.shape
        ns['rows'], ns['cols'], ns['BATCH_SIZE'], ns['H'] = V, C, B, H
        set_seed(seed + 1)
        model = ns['GNNI'](T)
        if ckpt:
            model.load_state_dict(torch.load(os.path.join(REF, ckpt), map_location='cpu',
                                             weights_only=True))
        sd = {k: v.clone() for k, v in model.state_dict().items()}
        ei = batch_edge_index(single_edge_index(H), B, V + C)
        data = types.SimpleNamespace(x=x, edge_index=ei, y=y)
        pred = model(data)
        loss = ns['LossFunc'](H, H_prep)(pred, data)
        loss.backward()
        save(f'train_v24_L{L}', x=x.numpy(), y=y.numpy(), loss=np.array(loss.item()),
             pred=pred.detach().numpy(),
             T=np.array(T), **sd_to_np(sd), **grads_of(model))

    # QGNNI at L = 4 (logical-only loss)
    H, H_prep, logical = toric(4)
    ns = load_ref('quantum/QGNNI.py', {'MessagePassing', 'GraphConv', 'GNNI', 'LossFunc'},
                  logical=logical)
    B, T = 4, 25
    x, y = toric_inputs(eg, H, 4, [0.05, 0.1], B, 93)
    V, C = H.shape
    ns['rows'], ns['cols'], ns['BATCH_SIZE'], ns['H'] = V, C, B, H
    set_seed(94)
    model = ns['GNNI'](T)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    data = types.SimpleNamespace(x=x, edge_index=batch_edge_index(single_edge_index(H), B, V + C), y=y)
    pred = model(data)
    loss = ns['LossFunc'](H, H_prep)(pred, data)
    loss.backward()
    save('train_qgnni_L4', x=x.numpy(), y=y.numpy(), loss=np.array(loss.item()), T=np.array(T),
         pred=pred.detach().numpy(),
         **sd_to_np(sd), **grads_of(model))

    # CGNNI on BCH(63,45) (epoch-18 weights), train-mode loss with lambda = 0.8
    H = bch_H()
    V, C = H.shape
    ns = load_ref('classical/CGNNI.py', {'MessagePassing', 'GatedGraphConv', 'GNNI', 'LossFunc'},
                  lambda_a=0.8)
    B, T = 8, 25
    llr, _ = awgn_llr(B, V, 1, 95)
    x = classical_x(llr, C)
    y = torch.ones(B * V, 1)
    ns['rows'], ns['cols'], ns['BATCH_SIZE'], ns['H'] = V, C, B, H
    model = ns['GNNI'](T)
    model.load_state_dict(torch.load(os.path.join(REF, 'classical/model/decoder_parameters_epoch18.pkl'),
                                     map_location='cpu', weights_only=True))
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    data = types.SimpleNamespace(x=x, edge_index=batch_edge_index(single_edge_index(H), B, V + C), y=y)
    pred = model(data)
    loss = ns['LossFunc'](H)(pred, data.y, 1)
    loss.backward()
    save('train_cgnni_bch', x=x.numpy(), y=y.numpy(), loss=np.array(loss.item()), T=np.array(T),
         pred=pred.detach().numpy(),
         **sd_to_np(sd), **grads_of(model))


def gen_neural_bp():
    """Weighted ("neural") BP decoders on the same operator:
    quantum/neural_BP.py (per-layer per-edge W, W_p on the v->c step; readout W, W_p;
    residual alpha) and quantum/decoder_v1_0.py (per-layer per-edge W on the c->v input;
    residual alpha).  Toric L = 4, T = 15 (the scripts' Nc), fp64.  The scripts initialise
    every weight to 1 (0.5 for the readout W_p, 0 for alpha): the fixtures perturb them
    (seeded) so that every weight path is exercised.  The shipped checkpoints under
    quantum/neural_BP/ belong to an orphaned revision (ggc1/ggc2, 4 edge types, per-variable
    W_p) that matches neither script and are not used.  Also: a bare propagate() per flow,
    and one training step (reference LossFunc, train=1) with parameter gradients."""
    sys.path.insert(0, os.path.join(REF, 'quantum'))
    import error_generate as eg
    L = 4
    Hnp, _ = eg.generate_PCM(2 * L * L - 2, L)
    H = torch.from_numpy(Hnp).t()
    hp = eg.H_Prep(H.t())
    H_prep = torch.from_numpy(hp.get_H_Prep())
    logical, _ = hp.get_logical(H_prep)
    V, C = H.shape
    N = V + C
    specs = (('nbp', 'quantum/neural_BP.py', 201), ('v10', 'quantum/decoder_v1_0.py', 301))
    prop = {}
    for tag, script, seed in specs:
        ns = load_ref(script, {'MessagePassing', 'GraphConv', 'GNNI', 'LossFunc'},
                      logical=logical)
        ns['rows'], ns['cols'], ns['BATCH_SIZE'], ns['H'] = V, C, 1, H
        set_seed(seed)
        model = ns['GNNI'](15)
        with torch.no_grad():
            for k, p in model.named_parameters():
                if k == 'alpha':
                    p.fill_(0.3)
                else:
                    p.mul_(1 + 0.25 * torch.randn(p.shape, dtype=p.dtype))
        sd = {k: v.clone() for k, v in model.state_dict().items()}
        arrays = dict(sd_to_np(sd))
        for B, xs in ((1, seed + 1), (32, seed + 2)):
            x, y = toric_inputs(eg, H, L, [0.05, 0.1], B, xs)
            arrays[f'x_B{B}'], arrays[f'y_B{B}'] = x.numpy(), y.numpy()
            for T in (1, 2, 15):
                out, _ = run_model(ns, H, x, B, T, {k: v for k, v in sd.items()
                                                    if not k.startswith('layers.') or
                                                    int(k.split('.')[1]) < 2 * T})
                arrays[f'out_B{B}_T{T}'] = out.numpy()
        save(f'{tag}_toric4', **arrays)

        # one training step at B = 4 (reference LossFunc, train=1: sum-of-|sin| syndrome +
        # logical loss), gradients of every parameter
        B = 4
        x, y = toric_inputs(eg, H, L, [0.05, 0.1], B, seed + 3)
        ns['BATCH_SIZE'] = B
        model = ns['GNNI'](15)
        model.load_state_dict(sd)
        data = types.SimpleNamespace(x=x, edge_index=batch_edge_index(single_edge_index(H), B, N), y=y)
        pred = model(data)
        loss = ns['LossFunc'](H, H_prep)(pred, data, 1)
        loss.backward()
        save(f'train_{tag}_L4', x=x.numpy(), y=y.numpy(), loss=np.array(loss.item()),
             pred=pred.detach().numpy(), T=np.array(15), **sd_to_np(sd), **grads_of(model))

        # bare propagate() per flow on random messages (identity message/update)
        B = 3
        ei = batch_edge_index(single_edge_index(H), B, N)
        ei = torch.stack([ei[0], ei[1] + V])
        g = torch.Generator().manual_seed(seed + 4)
        E = ei.size(1)
        m = (torch.randn(E, 1, generator=g) * 3).double()
        m[::7] *= 8                                   # saturate some tanh(x/2) below 1e-15
        xv = torch.randn(B, V, generator=g) * 2
        xc = torch.where(torch.rand(B, C, generator=g) < 0.3, -1.0, 1.0)
        extra = torch.cat([xv, xc], dim=1).reshape(B * N, 1).double()
        prop[f'{tag}/edge_index'] = ei.numpy()
        prop[f'{tag}/msg'] = m.numpy()
        prop[f'{tag}/extra'] = extra.numpy()
        for flow in ('source_to_target', 'target_to_source'):
            mp = ns['MessagePassing']('add', flow)
            with torch.no_grad():
                out = mp.propagate(edge_index=ei, size=(N * B, N * B), x=m, extra=extra)
            prop[f'{tag}/{flow}/add'] = out.numpy()
    save('propagate_ops_nbp', **prop)


def _repo_codes():
    """This framework's code constructions (the LDPC H has no reference counterpart: the
    reference swaps H by hand, classical/CGNNI.py:180-189)."""
    pkg = os.path.join(os.path.dirname(os.path.dirname(OUT)), 'gnn-decode_amd')
    if pkg not in sys.path:
        sys.path.insert(0, pkg)
    from gnndecode import codes
    return codes


def gen_ldpc():
    """Config 4's code: 802.11n LDPC(648,324) through the reference's
    own CGNNI (classical/CGNNI.py) and classical BP (classical/BP.py) classes, H swapped in
    the way classical/CGNNI.py:180-189 swaps H_BCH for H_LDPC.  CGNNI runs with this
    framework's trained LDPC weights (gnndecode/weights/cgnni_ldpc_648_324.npz: plain arrays,
    the reference state_dict keys) and with a seeded default init."""
    codes = _repo_codes()
    H = torch.from_numpy(codes.wifi_ldpc_648().astype(np.float32))          # [648, 324]
    V, C = H.shape
    save('ldpc_648_324_graph', H=H.numpy().astype(np.uint8),
         edge_index=single_edge_index(H).numpy())
    wz = np.load(os.path.join(os.path.dirname(codes.__file__), 'weights', 'cgnni_ldpc_648_324.npz'))
    trained = {k: torch.from_numpy(wz[k]) for k in wz.files}
    ns = load_ref('classical/CGNNI.py', {'MessagePassing', 'GatedGraphConv', 'GNNI'})
    set_seed(401)
    ns['rows'], ns['cols'], ns['BATCH_SIZE'], ns['H'] = V, C, 1, H
    rand = {k: v.clone() for k, v in ns['GNNI'](25).state_dict().items()}
    for tag, sd, bit in (('cgnni_ldpc', trained, 0), ('cgnni_ldpc_randinit', rand, 1)):
        arrays = dict(sd_to_np(sd))
        for B, seed in ((2, 402), (6, 403)):
            llr, _ = awgn_llr(B, V, bit, seed + (7 if bit else 0))
            x = classical_x(llr, C)
            arrays[f'x_B{B}'] = x.numpy()
            for T in (1, 2, 25):
                out, _ = run_model(ns, H, x, B, T, sd)
                arrays[f'out_B{B}_T{T}'] = out.numpy()
        save(tag, **arrays)
    ns = load_ref('classical/BP.py', {'MessagePassing', 'GatedGraphConv', 'GNNI'})
    arrays = {}
    for B, seed in ((2, 404), (6, 405)):
        llr, _ = awgn_llr(B, V, 0, seed, snrs=(1, 2, 3))
        x = classical_x(llr, C)
        arrays[f'x_B{B}'] = x.numpy()
        for T in (1, 25):
            out, _ = run_model(ns, H, x, B, T)
            arrays[f'out_B{B}_T{T}'] = out.numpy()
    save('bp_ldpc', **arrays)


def _gf2_null_space(A):
    """Basis [k, n] of {v : A v = 0 (mod 2)} for A [m, n] (Gauss-Jordan over GF(2))."""
    M = (np.asarray(A) % 2).astype(np.int64)
    m, n = M.shape
    piv, r = [], 0
    for c in range(n):
        p = next((i for i in range(r, m) if M[i, c]), None)
        if p is None:
            continue
        M[[r, p]] = M[[p, r]]
        for i in range(m):
            if i != r and M[i, c]:
                M[i] ^= M[r]
        piv.append(c)
        r += 1
    basis = []
    for f in (c for c in range(n) if c not in piv):
        v = np.zeros(n, np.int64)
        v[f] = 1
        for i, c in enumerate(piv):
            v[c] = M[i, f]
        basis.append(v)
    return np.array(basis)


def gen_fer():
    """The hard-decision frame-failure count of quantum/neural_BP.py:322-348 (LossFunc with
    train=0: codewords with a non-zero residual syndrome H^T(y + e_hat) plus codewords with a
    zero residual syndrome and an odd overlap with some logical row), run with the
    reference's own LossFunc on (a) the decoder_v2_4 fixture outputs and (b) crafted
    predictions at L = 5 and L = 7 mixing correct decodes, syndrome failures, zero-syndrome
    decodes (y + a random vector of the GF(2) null space of H^T: a logical failure when it
    overlaps a logical row oddly under the reference's plain product, else a success),
    all-zero predictions and exact-0.5 ties.  The fixture stores pred, y and the count."""
    sys.path.insert(0, os.path.join(REF, 'quantum'))
    import error_generate as eg
    arrays = {}
    for L, B, seed in ((5, 600, 501), (7, 300, 502)):
        Hnp, _ = eg.generate_PCM(2 * L * L - 2, L)
        H = torch.from_numpy(Hnp).t()
        hp = eg.H_Prep(H.t())
        H_prep = torch.from_numpy(hp.get_H_Prep())
        logical, _ = hp.get_logical(H_prep)
        V, C = H.shape
        ns = load_ref('quantum/neural_BP.py', {'LossFunc'}, logical=logical, H=H)
        lf = ns['LossFunc'](H, H_prep)
        g = torch.Generator().manual_seed(seed)
        y = (torch.rand(B, V, generator=g, dtype=torch.float64) < 0.06).double()
        kind = torch.randint(0, 6, (B,), generator=g)
        pred = y.clone()
        null = torch.from_numpy(_gf2_null_space(H.t().numpy())).double()   # H^T n = 0 (mod 2)
        for b in range(B):
            k = int(kind[b])
            if k == 1:                                    # random flips (mostly syndrome failures)
                f = (torch.rand(V, generator=g) < 0.03).double()
                pred[b] = (pred[b] + f) % 2
            elif k in (2, 3):                             # + a zero-syndrome pattern: a pure
                # logical failure when it overlaps some logical row oddly, else a success
                sel = torch.rand(null.size(0), generator=g) < 0.5
                pred[b] = (pred[b] + null[sel].sum(0)) % 2
            elif k == 4:                                  # predict no error
                pred[b] = 0
        soft = torch.where(pred > 0.5, 0.75, 0.25).double()
        tie = torch.rand(B, V, generator=g) < 0.002       # p == 0.5 is a 0 decision (not > 0.5)
        soft[tie] = 0.5
        data = types.SimpleNamespace(y=y.reshape(B * V, 1))
        with torch.no_grad():
            cnt = lf(soft.reshape(B * V, 1), data, 0)
        arrays[f'L{L}/pred'] = soft.reshape(B * V, 1).numpy()
        arrays[f'L{L}/y'] = y.reshape(B * V, 1).numpy()
        arrays[f'L{L}/count'] = np.array(float(cnt))
    # (a) the decoder_v2_4 fixture outputs at B = 32
    z = np.load(os.path.join(OUT, 'v24_toric5.npz'))
    L = 5
    Hnp, _ = eg.generate_PCM(2 * L * L - 2, L)
    H = torch.from_numpy(Hnp).t()
    hp = eg.H_Prep(H.t())
    H_prep = torch.from_numpy(hp.get_H_Prep())
    logical, _ = hp.get_logical(H_prep)
    ns = load_ref('quantum/neural_BP.py', {'LossFunc'}, logical=logical, H=H)
    data = types.SimpleNamespace(y=torch.from_numpy(z['y_B32']))
    with torch.no_grad():
        cnt = ns['LossFunc'](H, H_prep)(torch.from_numpy(z['out_B32_T15']), data, 0)
    arrays['v24_B32/count'] = np.array(float(cnt))
    save('fer_rule', **arrays)


def gen_v30():
    """quantum/decoder_v3_0.py (GRU edge states, two-output readout) at toric L = 5.  The
    script's module top level is not run (load_ref keeps only the named classes); GNNI.forward
    reads the module globals rows, cols, BATCH_SIZE and Nc (the iteration whose ggc1 output
    is kept as m_p), injected here with Nc = T.  No checkpoint ships for this script: seeded
    default init.  Fixtures: decoder outputs (both tensors) for B in {1, 4}, T in {1, 2, 15};
    one training step (reference LossFunc, :293-335) with every parameter gradient; one bare
    propagate() per flow and aggregation."""
    sys.path.insert(0, os.path.join(REF, 'quantum'))
    import error_generate as eg
    L = 5
    Hnp, _ = eg.generate_PCM(2 * L * L - 2, L)
    H = torch.from_numpy(Hnp).t()
    hp = eg.H_Prep(H.t())
    H_prep = torch.from_numpy(hp.get_H_Prep())
    V, C = H.shape
    N = V + C
    names = {'MessagePassing', 'GraphConv', 'GNNI', 'LossFunc'}
    ns = load_ref('quantum/decoder_v3_0.py', names)
    ns['rows'], ns['cols'], ns['BATCH_SIZE'], ns['H'], ns['Nc'] = V, C, 1, H, 15
    set_seed(701)
    sd = {k: v.clone() for k, v in ns['GNNI'](15).state_dict().items()}
    arrays = dict(sd_to_np(sd))
    for B, seed in ((1, 702), (4, 703)):
        x, y = toric_inputs(eg, H, L, [0.05, 0.1], B, seed)
        arrays[f'x_B{B}'], arrays[f'y_B{B}'] = x.numpy(), y.numpy()
        for T in (1, 2, 15):
            ns['Nc'] = T
            out, _ = run_model(ns, H, x, B, T, sd)
            arrays[f'out0_B{B}_T{T}'] = out[0].numpy()
            arrays[f'out1_B{B}_T{T}'] = out[1].numpy()
    save('v30_toric5', **arrays)

    # one training step at B = 4, T = 15 (reference LossFunc on the two outputs)
    B, T = 4, 15
    x, y = toric_inputs(eg, H, L, [0.05, 0.1], B, 704)
    ns['rows'], ns['cols'], ns['BATCH_SIZE'], ns['H'], ns['Nc'] = V, C, B, H, T
    model = ns['GNNI'](T)
    model.load_state_dict(sd)
    data = types.SimpleNamespace(x=x, edge_index=batch_edge_index(single_edge_index(H), B, N), y=y)
    pred = model(data)
    loss = ns['LossFunc'](H, H_prep)(pred, data)
    loss.backward()
    save('train_v30_L5', x=x.numpy(), y=y.numpy(), loss=np.array(loss.item()), T=np.array(T),
         pred0=pred[0].detach().numpy(), pred1=pred[1].detach().numpy(),
         **sd_to_np(sd), **grads_of(model))

    # bare propagate() per flow / aggregation on random edge states
    B = 3
    ei = batch_edge_index(single_edge_index(H), B, N)
    ei = torch.stack([ei[0], ei[1] + V])
    g = torch.Generator().manual_seed(705)
    E = ei.size(1)
    m = (torch.randn(E, 1, generator=g) * 3).double()
    xv = torch.randn(B, V, generator=g) * 2
    xc = torch.where(torch.rand(B, C, generator=g) < 0.3, -1.0, 1.0)
    extra = torch.cat([xv, xc], dim=1).reshape(B * N, 1).double()
    prop = {'v30/edge_index': ei.numpy(), 'v30/msg': m.numpy(), 'v30/extra': extra.numpy()}
    for flow in ('source_to_target', 'target_to_source'):
        for aggr in ('add', 'max'):
            mp = ns['MessagePassing'](aggr, flow)
            with torch.no_grad():
                out = mp.propagate(edge_index=ei, size=(N * B, N * B), x=m, extra=extra)
            prop[f'v30/{flow}/{aggr}'] = out.numpy()
    save('propagate_ops_v30', **prop)


def _ref_edge_types(eg_path, L, H):
    """The 8 edge types of quantum/decoder_v2_2.py:226-250 from the reference itself: the
    shipped generate_PCM builds them as its local `H_prime` (error_generate.py:92-124) but
    returns `H_one` instead, so the function is exec'd with its return changed to
    (H, H_prime).  Types = H_prime.long() at the edges, reference edge order."""
    tree = ast.parse(open(eg_path).read(), eg_path)
    fns = [n for n in tree.body if isinstance(n, ast.FunctionDef)]   # generate_PCM + helpers
    fn = [n for n in fns if n.name == 'generate_PCM'][0]
    ret = [n for n in ast.walk(fn) if isinstance(n, ast.Return)][-1]
    ret.value = ast.Tuple(elts=[ast.Name('H', ast.Load()), ast.Name('H_prime', ast.Load())],
                          ctx=ast.Load())
    ns = {'np': np, 'math': math, 'torch': torch}
    exec(compile(ast.fix_missing_locations(ast.Module(body=fns, type_ignores=[])), eg_path,
                 'exec'), ns)
    Hc, Hp = ns['generate_PCM'](2 * L * L - 2, L)
    assert np.array_equal(np.asarray(Hc).T, H.numpy())
    Hp = torch.from_numpy(np.asarray(Hp)).t()               # [V, C] like H
    idx = single_edge_index(H)
    return Hp[idx[0], idx[1]].to(torch.long)


def gen_v22():
    """quantum/decoder_v2_2.py (neural BP with edge-type-shared weights, per-layer readout
    list) at toric L = 4, Nc = 25.  The script's module top level cannot run against the
    shipped error_generate (its H_prime, the `generate_PCM` second value, now carries labels
    up to 31 and `feat_onehot.scatter_` into 8 columns fails); load_ref keeps the classes
    and the fixtures inject `feat_onehot` built from the reference's own 8-type H_prime
    (_ref_edge_types) with rows/cols/BATCH_SIZE/H/nb_digits/logical.  Weights: the script's
    init (ones, W_pr 0.5, weight -4) perturbed seeded so every path is exercised.
    Fixtures: per-layer readouts for B in {1, 8}, T in {1, 2, 25}; one training step
    (reference LossFunc, train=1: the sum over all layers) with every parameter gradient."""
    sys.path.insert(0, os.path.join(REF, 'quantum'))
    import error_generate as eg
    L, NC = 4, 25
    Hnp, _ = eg.generate_PCM(2 * L * L - 2, L)
    H = torch.from_numpy(Hnp).t()
    hp = eg.H_Prep(H.t())
    H_prep = torch.from_numpy(hp.get_H_Prep())
    logical, _ = hp.get_logical(H_prep)
    V, C = H.shape
    N = V + C
    types_ = _ref_edge_types(os.path.join(REF, 'quantum', 'error_generate.py'), L, H)
    E = types_.numel()
    onehot = torch.zeros(E, 8, dtype=torch.float64)
    onehot.scatter_(1, types_.unsqueeze(1), 1)

    def setup(B):
        ns['rows'], ns['cols'], ns['BATCH_SIZE'], ns['H'] = V, C, B, H
        ns['feat_onehot'] = onehot.repeat(B, 1)

    ns = load_ref('quantum/decoder_v2_2.py', {'MessagePassing', 'GraphConv', 'GNNI', 'LossFunc'},
                  nb_digits=8, logical=logical)
    setup(1)
    set_seed(221)
    model = ns['GNNI'](NC)
    with torch.no_grad():
        for k, p in model.named_parameters():
            if k == 'weight':
                p.fill_(-1.0)
            else:
                p.mul_(1 + 0.25 * torch.randn(p.shape, dtype=p.dtype))
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    arrays = dict(sd_to_np(sd))
    arrays['edge_types'] = types_.numpy()
    for B, xs in ((1, 222), (8, 223)):
        x, y = toric_inputs(eg, H, L, [0.05, 0.1], B, xs)
        arrays[f'x_B{B}'], arrays[f'y_B{B}'] = x.numpy(), y.numpy()
        setup(B)
        for T in (1, 2, NC):
            m = ns['GNNI'](T)
            m.load_state_dict({k: v for k, v in sd.items()
                               if not k.startswith('layers.') or int(k.split('.')[1]) < 2 * T})
            data = types.SimpleNamespace(x=x, edge_index=batch_edge_index(single_edge_index(H), B, N))
            with torch.no_grad():
                out = m(data)
            assert len(out) == T
            arrays[f'out_B{B}_T{T}'] = torch.stack([o.reshape(-1) for o in out]).numpy()
    save('v22_toric4', **arrays)

    # one training step at B = 4, T = NC (reference LossFunc, train=1: every layer's readout)
    B = 4
    x, y = toric_inputs(eg, H, L, [0.05, 0.1], B, 224)
    setup(B)
    model = ns['GNNI'](NC)
    model.load_state_dict(sd)
    data = types.SimpleNamespace(x=x, edge_index=batch_edge_index(single_edge_index(H), B, N), y=y)
    pred = model(data)
    loss = ns['LossFunc'](H, H_prep)(pred, data, 1)
    loss.backward()
    save('train_v22_L4', x=x.numpy(), y=y.numpy(), loss=np.array(loss.item()), T=np.array(NC),
         edge_types=types_.numpy(), pred=torch.stack([p.detach().reshape(-1) for p in pred]).numpy(),
         **sd_to_np(sd), **grads_of(model))


if __name__ == '__main__':
    torch.set_num_threads(1)
    which = sys.argv[1:] or ['classical', 'quantum', 'training', 'neural_bp', 'ldpc', 'fer', 'v30',
                             'v22']
    if 'classical' in which:
        gen_classical()
    if 'quantum' in which:
        gen_quantum()
    if 'training' in which:
        gen_training()
    if 'neural_bp' in which:
        gen_neural_bp()
    if 'ldpc' in which:
        gen_ldpc()
    if 'fer' in which:
        gen_fer()
    if 'v30' in which:
        gen_v30()
    if 'v22' in which:
        gen_v22()
