"""Synthetic decoder inputs in the reference's batch layout (graph-major, N = V + C rows).

* classical (classical/CGNNI.py:125-147 `Gen_Data`, :157-161 `CustomDataset`): BPSK of a
  fixed codeword, AWGN with sigma^2 = 10^(-SNR/10), LLR = 2 y / sigma^2 at the variable rows,
  zeros at the check rows; SNR cycles over a grid per codeword.
* toric (quantum/error_generate.py:252-278 `gen_syn`): per codeword p drawn from a grid,
  independent X/Z flips with probability p, prior log((1-p)/p) at the variable rows and
  syndrome (-1)^(H^T e) at the check rows; labels y = e.

On a GPU both samplers run as HIP kernels (`gnnd_sample_toric` / `gnnd_sample_awgn`,
Philox4x32-10 counter-based streams: codeword b draws from (seed, offset + b) only, so a
data-parallel shard passing offset = its start reproduces its slice of the global batch
exactly).  `engine='torch'` (and CPU tensors) use the torch-generator formulation, kept as
the statistical cross-check.  The distributions match the reference; the random streams do
not (the reference draws with numpy / torch CPU generators).  Generation is outside every
timed region.
"""
import math

import numpy as np
import torch

_GRAPHS = {}


def _resolved(device):
    """torch.device with the index resolved ('cuda' -> the current device), so a cached
    graph never serves another GPU after a set_device."""
    d = torch.device(device)
    if d.type == 'cuda' and d.index is None:
        d = torch.device('cuda', torch.cuda.current_device())
    return d


def _graph_of(H, device):
    """Cached device graph of H (keyed by content and the resolved device).  A TannerGraph
    passed as H is used as is: no host copy or hashing of H inside a caller's timed loop."""
    from .graph import TannerGraph
    dev = _resolved(device)
    if isinstance(H, TannerGraph):
        if _resolved(H.device) != dev:
            raise ValueError(f'the TannerGraph passed as H lives on {H.device}, but the batch is '
                             f'requested on {dev}: pass the graph of that device (or the matrix)')
        return H, None
    Hn = (np.asarray(H.detach().cpu() if isinstance(H, torch.Tensor) else H) != 0).astype(np.uint8)
    key = (Hn.shape, hash(Hn.tobytes()), str(dev))
    g = _GRAPHS.get(key)
    if g is None:
        if len(_GRAPHS) > 32:
            _GRAPHS.clear()
        g = _GRAPHS[key] = TannerGraph(Hn, device=dev)
    return g, key


def _engine(engine, device):
    if engine == 'auto':
        return 'hip' if torch.device(device).type == 'cuda' else 'torch'
    if engine not in ('hip', 'torch'):
        raise ValueError(f'engine must be auto, hip or torch, got {engine!r}')
    return engine


def awgn_batch(H, B, snrs=(1, 2, 3, 4, 5, 6), codeword_bit=1, seed=0, device='cuda',
               dtype=torch.float32, codewords='fixed', offset=0, engine='auto'):
    """codewords='fixed': every codeword is the constant word `codeword_bit` (default 1:
    the reference's Gen_Data input is the all-ones word, classical/CGNNI.py:195, modulated
    to -1; classical/BP.py decodes the all-zeros word, pass 0); 'random': uniform random
    codewords of H (random GF(2) combinations of the generator rows,
    codes.gf2_generator), labels = their bits.  SNR of codeword b = snrs[(offset + b) %
    len(snrs)]."""
    if codewords not in ('fixed', 'random'):
        raise ValueError(f'codewords must be "fixed" or "random", got {codewords!r}')
    if _engine(engine, device) == 'hip':
        from . import ops
        g, _ = _graph_of(H, device)
        cols, k = None, 0
        if codewords == 'random':
            ent = getattr(g, '_gen_cols', None)        # generator columns, cached on the graph
            if ent is None:
                from .codes import gf2_generator
                c, k = ops.pack_generator_columns(gf2_generator(np.asarray(g.H)))
                ent = g._gen_cols = (c.to(g.device), k)
            cols, k = ent
        return ops.sample_awgn(g, B, snrs, cols, k, codeword_bit, seed, offset, dtype, device)
    if offset:
        raise ValueError('offset needs the HIP sampler (engine="hip")')
    V, C = H.shape
    g = torch.Generator(device=device).manual_seed(seed)
    snr = torch.tensor([snrs[b % len(snrs)] for b in range(B)], dtype=torch.float32, device=device)
    sigma = torch.sqrt(1.0 / (10 ** (snr / 10)))
    if codewords == 'random':
        from .codes import gf2_generator
        G = torch.as_tensor(gf2_generator(H), dtype=torch.float32, device=device)
        msg = torch.randint(0, 2, (B, G.shape[0]), generator=g, device=device).float()
        bits = torch.remainder(msg @ G, 2)
    else:
        bits = torch.full((B, V), float(codeword_bit), device=device)
    y = (1 - 2 * bits) + sigma[:, None] * torch.randn(B, V, generator=g, device=device)
    llr = 2 * y / (sigma[:, None] ** 2)
    x = torch.cat([llr, torch.zeros(B, C, device=device)], dim=1)
    return x.reshape(B * (V + C), 1).to(dtype), bits.reshape(B * V, 1).to(dtype)


def toric_batch(H, B, ps=(0.01, 0.02, 0.03, 0.04, 0.05, 0.06, 0.07, 0.08, 0.09, 0.1), seed=0,
                device='cuda', dtype=torch.float64, offset=0, engine='auto'):
    if _engine(engine, device) == 'hip':
        from . import ops
        g, _ = _graph_of(H, device)
        return ops.sample_toric(g, B, ps, seed, offset, dtype, device)
    if offset:
        raise ValueError('offset needs the HIP sampler (engine="hip")')
    Ht = torch.as_tensor(H, dtype=torch.float32, device=device)    # [V, C]
    V, C = Ht.shape
    g = torch.Generator(device=device).manual_seed(seed)
    pgrid = torch.tensor(ps, dtype=torch.float64, device=device)
    p = pgrid[torch.randint(len(ps), (B,), generator=g, device=device)]
    e = (torch.rand(B, V, generator=g, device=device, dtype=torch.float64) < p[:, None]).float()
    syn = torch.remainder(e @ Ht, 2)
    prior = torch.log((1 - p) / p)[:, None].expand(B, V)
    x = torch.cat([prior.to(torch.float64), (1 - 2 * syn).to(torch.float64)], dim=1)
    return x.reshape(B * (V + C), 1).to(dtype), e.reshape(B * V, 1).to(dtype)


def make_batch(x, graph, device=None):
    """A minimal PyG-style batch object: .x, .edge_index (collated, unshifted)."""
    class Batch:
        pass
    b = Batch()
    b.x = x
    b.edge_index = graph.batched_edge_index(x.numel() // graph.N, 0, device or x.device)
    return b
