"""Tensor-level entry points over the C ABI (torch tensors only as device-memory plumbing).

Every function here launches HIP kernels from libgnnd.so on the current HIP stream and
never synchronises the host.  Inputs must already be on the GPU: there is no CPU path.
"""
import ctypes

import torch

from . import _lib
from .graph import TannerGraph, current_stream, dtype_code

MODELS = ('v24', 'qgnni', 'qbp', 'cgnni', 'cbp', 'nbp', 'v10', 'v30', 'v22')
WEIGHTED_BP = ('nbp', 'v10', 'v22')      # per-edge weight tables: count depends on the graph and T


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _require_gpu(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError('gnndecode runs on the GPU only (HIP/gfx950); got a CPU tensor')


def propagate_width(variant, flow):
    return _lib.get().gnnd_propagate_width(_lib.VARIANT[variant], _lib.FLOW[flow])


def _tiled_batch(graph, edge_index, nE, dim_size, extra, aggr, chk_shift):
    """Batch size if edge_index is `graph` tiled over codewords, else None."""
    if graph is None or aggr == 'mean':
        return None
    shift = graph.V if chk_shift is None else chk_shift
    if (dim_size == (nE // graph.E) * graph.N and (extra is None or extra.size(0) == dim_size)
            and graph.is_tiled(edge_index, shift)):
        return nE // graph.E
    return None


def _propagate_fwd(variant, flow, aggr, edge_index, msg, extra, dim_size, B):
    nE = msg.size(0)
    F = propagate_width(variant, flow)
    out = torch.empty(nE, F, dtype=msg.dtype, device=msg.device)
    v, f, a = _lib.VARIANT[variant], _lib.FLOW[flow], _lib.AGGR[aggr]
    dt = dtype_code(msg.dtype)
    stream = current_stream(msg.device)
    if B is not None:
        _lib.call('gnnd_propagate_tiled', B[0].handle, v, f, a, dt, _ptr(msg), _ptr(extra),
                  _ptr(out), B[1], stream)
        return out
    ei = edge_index if edge_index.stride(1) == 1 else edge_index.contiguous()
    ws_bytes = ctypes.c_int64()
    _lib.call('gnnd_propagate_generic_workspace', v, f, a, dt, nE, dim_size, ctypes.byref(ws_bytes))
    ws = torch.empty(max(ws_bytes.value, 1), dtype=torch.uint8, device=msg.device)
    _lib.call('gnnd_propagate_generic', v, f, a, dt, _ptr(ei), ei.stride(0), nE, _ptr(msg),
              _ptr(extra), dim_size, _ptr(out), _ptr(ws), ws_bytes.value, stream)
    return out


def _propagate_bwd(variant, flow, aggr, edge_index, msg, extra, grad_out, dim_size, B):
    grad_out = grad_out.contiguous()
    gmsg = torch.empty_like(msg)
    v, f, a = _lib.VARIANT[variant], _lib.FLOW[flow], _lib.AGGR[aggr]
    dt = dtype_code(msg.dtype)
    stream = current_stream(msg.device)
    if B is not None:
        _lib.call('gnnd_propagate_tiled_bwd', B[0].handle, v, f, a, dt, _ptr(msg), _ptr(extra),
                  _ptr(grad_out), _ptr(gmsg), B[1], stream)
        return gmsg
    ei = edge_index if edge_index.stride(1) == 1 else edge_index.contiguous()
    nb = ctypes.c_int64()
    _lib.call('gnnd_propagate_generic_bwd_workspace', v, f, a, dt, msg.size(0), dim_size,
              ctypes.byref(nb))
    ws = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=msg.device)
    _lib.call('gnnd_propagate_generic_bwd', v, f, a, dt, _ptr(ei), ei.stride(0), msg.size(0),
              _ptr(msg), _ptr(extra), _ptr(grad_out), dim_size, _ptr(gmsg), _ptr(ws),
              nb.value, stream)
    return gmsg


def _propagate_impl(variant, flow, aggr, edge_index, msg, extra, dim_size, graph, chk_shift):
    """gnnd::propagate implementation (gnndecode.library): tiled kernel when `graph` matches
    the batched edge_index, else the generic kernels."""
    b = _tiled_batch(graph, edge_index, msg.size(0), dim_size, extra, aggr, chk_shift)
    return _propagate_fwd(variant, flow, aggr, edge_index, msg, extra, dim_size,
                          (graph, b) if b is not None else None)


def _propagate_bwd_impl(variant, flow, aggr, edge_index, msg, extra, grad_out, dim_size, graph,
                        chk_shift):
    b = _tiled_batch(graph, edge_index, msg.size(0), dim_size, extra, aggr, chk_shift)
    return _propagate_bwd(variant, flow, aggr, edge_index, msg, extra, grad_out, dim_size,
                          (graph, b) if b is not None else None)


def propagate(variant, flow, aggr, edge_index, msg, extra, dim_size, graph=None, chk_shift=None):
    """One reference `propagate` body on the device (torch op gnnd::propagate).

    msg [nE, 1] per-edge message, extra [dim_size, 1] node tensor (or None for CGNNI's
    `post=None`), edge_index int64 [2, nE].  Uses the tiled LDS kernel when `graph` matches
    the batched edge_index, otherwise the generic (atomic) kernels.  Differentiable w.r.t.
    `msg` (aggr 'add') through HIP backward kernels (gnnd::propagate_bwd).
    Returns [nE, F] with F = propagate_width(variant, flow).
    """
    _require_gpu(edge_index, msg, extra)
    if msg.dim() == 1:
        msg = msg.unsqueeze(1)
    if msg.size(-1) != 1:
        raise ValueError('per-edge message must have one feature column (reference models)')
    msg = msg.contiguous()
    dtype_code(msg.dtype)
    if extra is not None:
        if extra.dim() == 1:
            extra = extra.unsqueeze(1)
        extra = extra.detach().to(msg.dtype).contiguous()
    nE = msg.size(0)
    if edge_index.size(1) != nE:
        raise ValueError('edge_index and message disagree on the number of edges')
    if extra is None and variant != 'cgnni':
        raise ValueError(f'{variant}: propagate needs `extra`')
    if msg.requires_grad and torch.is_grad_enabled() and aggr != 'add':
        raise NotImplementedError(f'no backward for aggr={aggr!r}')
    if torch.compiler.is_compiling():
        # traced (torch.compile / FX): the registered op gnnd::propagate (gnndecode.library)
        return torch.ops.gnnd.propagate(variant, flow, aggr, edge_index, msg, extra,
                                        int(dim_size), graph.gid if graph is not None else -1,
                                        -1 if chk_shift is None else int(chk_shift))
    # eager: the same implementation without the dispatcher round trip
    if msg.requires_grad and torch.is_grad_enabled():
        return _PropagateFn.apply(msg, variant, flow, aggr, edge_index, extra, int(dim_size),
                                  graph, chk_shift)
    return _propagate_impl(variant, flow, aggr, edge_index, msg, extra, dim_size, graph, chk_shift)


class _PropagateFn(torch.autograd.Function):
    """Eager autograd of propagate (the traced path uses gnnd::propagate's registered
    autograd): HIP backward w.r.t. the per-edge message, extra is data."""

    @staticmethod
    def forward(ctx, msg, variant, flow, aggr, edge_index, extra, dim_size, graph, chk_shift):
        ctx.save_for_backward(msg, edge_index, extra)
        ctx.args = (variant, flow, aggr, dim_size, graph, chk_shift)
        return _propagate_impl(variant, flow, aggr, edge_index, msg, extra, dim_size, graph,
                               chk_shift)

    @staticmethod
    def backward(ctx, grad_out):
        msg, edge_index, extra = ctx.saved_tensors
        variant, flow, aggr, dim_size, graph, chk_shift = ctx.args
        gmsg = _propagate_bwd_impl(variant, flow, aggr, edge_index, msg, extra,
                                   grad_out.contiguous(), dim_size, graph, chk_shift)
        return gmsg, None, None, None, None, None, None, None, None


def weights_count(model, graph=None, iters=None):
    """Packed weight count of a fused decoder (gnnd.h); the weighted-BP models need the
    graph and the iteration count."""
    n = ctypes.c_int64()
    if model in WEIGHTED_BP:
        if graph is None or iters is None:
            raise ValueError(f'{model}: the weight count depends on the graph and T')
        _lib.call('gnnd_decode_weights_count', graph.handle, _lib.VARIANT[model], int(iters),
                  ctypes.byref(n))
    else:
        _lib.call('gnnd_weights_count', _lib.VARIANT[model], ctypes.byref(n))
    return n.value


def prepared_count(model, dtype, graph=None, iters=None, priors=0):
    """Elements of the kernel-layout weights (gnnd_prepared_weights_count[_priors]): the packed
    count, except decoder_v2_4, whose prepared weights carry the check-MLP table and the
    channel-prior section (fp64: `priors` tables of the variable-side MLP)."""
    if model in WEIGHTED_BP:
        return weights_count(model, graph, iters)
    n = ctypes.c_int64()
    _lib.call('gnnd_prepared_weights_count_priors', _lib.VARIANT[model],
              dtype_code(torch.float32 if dtype == torch.bfloat16 else dtype), int(priors),
              ctypes.byref(n))
    return n.value


def prepare_weights(model, flat, priors=None):
    """Kernel-layout copy of a packed weight vector (gnnd_prepare_weights).  The weighted-BP
    tables are used as packed.  `priors` (fp64 decoder_v2_4): the channel-prior LLRs x_v the
    inputs will carry (e.g. channel_priors(graph, x)); the prepared weights then hold the
    variable-side MLP tabulated per prior (gnnd_prepare_weights_priors)."""
    _require_gpu(flat)
    flat = flat.contiguous()
    if model in WEIGHTED_BP:
        return flat
    n = weights_count(model)
    if n == 0:
        return None
    if flat.numel() != n:
        raise ValueError(f'{model}: expected {n} packed weights, got {flat.numel()}')
    pv = [float(v) for v in (priors if priors is not None else [])]
    out = torch.empty(prepared_count(model, flat.dtype, priors=len(pv)), dtype=flat.dtype,
                      device=flat.device)
    arr = (ctypes.c_double * max(len(pv), 1))(*pv)
    _lib.call('gnnd_prepare_weights_priors', _lib.VARIANT[model], dtype_code(flat.dtype), _ptr(flat),
              _ptr(out), arr, len(pv), current_stream(flat.device))
    return out


def channel_priors(graph, x, limit=64):
    """The distinct variable-node inputs x_v of a batch x [B*N] (the channel-prior LLRs of the
    reference's gen_syn inputs: one per codeword, from a short p list) -- the keys for
    prepare_weights(priors=...).  One device-to-host copy (setup, not the decode path); raises
    ValueError when there are more than `limit` (<= 64) distinct values."""
    xv = x.reshape(-1, graph.N)[:, :graph.V]
    u = torch.unique(xv).cpu().tolist()
    if len(u) > limit:
        raise ValueError(f'{len(u)} distinct priors (at most {limit} tables)')
    return u


def v24_var_mlp_table(prepared_weights, u, xv=None):
    """gnnd_v24_var_mlp_table: decoder_v2_4's variable-side MLP through the channel-prior tables
    at fp64 points (u, x_v) -> (y, hit) with y = tanh(ggc1.mlp(u, x_v) / 2), the check step's
    pre-op of the MLP output that the tables hold; xv None: the readout MLP's table at u,
    y = mlp(u).  y is NaN where hit is False."""
    _require_gpu(prepared_weights, u)
    u = u.to(torch.float64).contiguous()
    if xv is not None:
        xv = xv.to(torch.float64).contiguous()
        if u.shape != xv.shape:
            raise ValueError('u and x need the same shape')
    y = torch.full_like(u, float('nan'))
    hit = torch.zeros(u.shape, dtype=torch.int32, device=u.device)
    _lib.call('gnnd_v24_var_mlp_table', _ptr(prepared_weights), _ptr(u),
              _ptr(xv) if xv is not None else None, _ptr(y), _ptr(hit), u.numel(),
              current_stream(u.device))
    return y, hit.bool()


def decode_out_rows(graph, model, B, iters=1):
    """Rows of gnnd_decode's output: B*V, 2*B*N for decoder_v3_0's two-output readout,
    iters*B*V for decoder_v2_2's per-iteration readout list."""
    if model == 'v30':
        return 2 * B * graph.N
    return iters * B * graph.V if model == 'v22' else B * graph.V


def decode(graph: TannerGraph, model, x, iters, prepared_weights=None, out=None):
    """Fused T-iteration decode: x [B*N(,1)] -> P(bit=1) [B*V, 1] (v30: [2*B*N, 1], the
    two readout tensors of quantum/decoder_v3_0.py:287-288 stacked; v22: [T*B*V, 1], the
    per-iteration readouts of quantum/decoder_v2_2.py:341-347 stacked).  Traced code
    (torch.compile / FX) gets the registered ops gnnd::decode / gnnd::decode_out."""
    if torch.compiler.is_compiling():
        if out is None:
            return torch.ops.gnnd.decode(graph.gid, model, x, int(iters), prepared_weights)
        torch.ops.gnnd.decode_out(graph.gid, model, x, int(iters), prepared_weights, out)
        return out
    _require_gpu(x, prepared_weights)
    x = x.contiguous()
    if x.numel() % graph.N:
        raise ValueError(f'x has {x.numel()} rows, not a multiple of N={graph.N}')
    B = x.numel() // graph.N
    wdt = torch.float32 if x.dtype == torch.bfloat16 else x.dtype   # bf16 storage, fp32 math
    nw = prepared_count(model, wdt, graph, iters)
    # (fp64 decoder_v2_4 prepared with channel-prior tables: more)
    if nw and (prepared_weights is None or prepared_weights.numel() < nw or
               (prepared_weights.numel() != nw and not (model == 'v24' and wdt == torch.float64))):
        raise ValueError(f'{model}: needs {nw} prepared weights (prepare_weights)')
    if prepared_weights is not None and prepared_weights.dtype != wdt:
        raise TypeError(f'{x.dtype} inputs need {wdt} prepared weights')
    rows = decode_out_rows(graph, model, B, int(iters))
    if out is None:
        out = torch.empty(rows, 1, dtype=x.dtype, device=x.device)
    elif out.numel() != rows or not out.is_contiguous() or out.dtype != x.dtype:
        raise ValueError(f'out must be a contiguous {x.dtype} tensor of {rows} values')
    _decode_impl(graph, model, x, iters, prepared_weights, out)
    return out


def _decode_impl(graph, model, x, iters, prepared_weights, out):
    """gnnd::decode / gnnd::decode_out implementation (gnndecode.library)."""
    _lib.call('gnnd_decode', graph.handle, _lib.VARIANT[model], dtype_code(x.dtype),
              _ptr(prepared_weights), _ptr(x), _ptr(out), x.numel() // graph.N, int(iters),
              current_stream(x.device))


def decode_plan(graph, model, dtype):
    """{'cw', 'lds', 'kernel', 'items_per_lane'} of the fused decoder's launch plan."""
    plan = (ctypes.c_int32 * 5)()
    _lib.call('gnnd_decode_plan', graph.handle, _lib.VARIANT[model], dtype_code(dtype), plan)
    return {'cw': plan[0], 'lds': plan[1],
            'kernel': 'decode_resident_kernel' if plan[2] else 'decode_kernel',
            'items_per_lane': plan[3], 'var_group': plan[4]}


def decode_tile(graph, model, dtype):
    cw, lds = ctypes.c_int32(), ctypes.c_int32()
    _lib.call('gnnd_decode_tile', graph.handle, _lib.VARIANT[model], dtype_code(dtype),
              ctypes.byref(cw), ctypes.byref(lds))
    return cw.value, lds.value


# ---------------------------------------------------------------------------------------
# fused training step (decoder_v2_4): forward with tape + one-launch reverse pass
# ---------------------------------------------------------------------------------------
def train_forward(graph, model, x, prepared_weights, iters):
    """gnnd_train_fwd: the fused decode plus the training tape (models v24, v30; nbp, v22 fp64).
    Returns (out, tape)."""
    _require_gpu(x, prepared_weights)
    x = x.contiguous()
    B = x.numel() // graph.N
    dt = dtype_code(x.dtype)
    # (decoder_v2_4 reads its prepared layout -- fp64: with the check-MLP table; the other
    # models' training forwards read the plain weights at its head)
    nw = (prepared_count(model, x.dtype, graph, iters) if model == 'v24'
          else weights_count(model, graph, iters))
    if nw and (prepared_weights is None or prepared_weights.numel() < nw):
        raise ValueError(f'{model}: needs {nw} prepared weights (prepare_weights)')
    nb = ctypes.c_int64()
    _lib.call('gnnd_train_tape_bytes', graph.handle, _lib.VARIANT[model], dt, B, int(iters),
              ctypes.byref(nb))
    tape = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=x.device)
    # v30: the two readout tensors [2][B*N]; v22: every layer's readout [T][B*V] (gnnd_decode's
    # layouts)
    nout = 2 * B * graph.N if model == 'v30' else iters * B * graph.V if model == 'v22' else B * graph.V
    out = torch.empty(nout, 1, dtype=x.dtype, device=x.device)
    _lib.call('gnnd_train_fwd', graph.handle, _lib.VARIANT[model], dt, _ptr(prepared_weights),
              _ptr(x), _ptr(out), _ptr(tape), B, int(iters), current_stream(x.device))
    return out, tape


def train_forward_loss(graph, model, x, prepared_weights, iters, y, logical_mask, n_logical,
                       logical_only):
    """gnnd_train_fwd_loss: train_forward plus decoder_v2_4's syndrome loss in the forward's
    epilogue.  Returns (out, tape, d loss / d out, per-codeword-and-component losses), or None
    when the plan does not take it (fp32 V24 unit-split small batches only): then
    train_backward_loss_partial computes the same loss in the reverse pass."""
    _require_gpu(x, prepared_weights)
    x = x.contiguous()
    B = x.numel() // graph.N
    dt = dtype_code(x.dtype)
    nb = ctypes.c_int64()
    _lib.call('gnnd_train_tape_bytes', graph.handle, _lib.VARIANT[model], dt, B, int(iters),
              ctypes.byref(nb))
    nl = ctypes.c_int64()
    _lib.call('gnnd_train_loss_count', graph.handle, B, ctypes.byref(nl))
    tape = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=x.device)
    out = torch.empty(B * graph.V, 1, dtype=x.dtype, device=x.device)
    gout = torch.empty_like(out)
    loss_b = torch.empty(max(nl.value, 1), dtype=x.dtype, device=x.device)[:nl.value]
    y = y.to(x.dtype).contiguous()
    ok = _lib.call_or_unsupported(
        'gnnd_train_fwd_loss', graph.handle, _lib.VARIANT[model], dt, _ptr(prepared_weights),
        _ptr(x), _ptr(out), _ptr(tape), _ptr(y), _ptr(logical_mask), int(n_logical),
        int(bool(logical_only)), _ptr(gout), _ptr(loss_b), B, int(iters), current_stream(x.device))
    return (out, tape, gout, loss_b) if ok else None


def train_backward(graph, model, plain_weights, x, out, grad_out, tape, iters):
    """gnnd_train_bwd: d loss / d (plain packed weights) from d loss / d out."""
    B = x.numel() // graph.N
    dt = dtype_code(x.dtype)
    nb = ctypes.c_int64()
    _lib.call('gnnd_train_workspace_bytes', graph.handle, _lib.VARIANT[model], dt, B, int(iters),
              ctypes.byref(nb))
    ws = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=x.device)
    gw = torch.empty_like(plain_weights)
    grad_out = grad_out.contiguous()
    _lib.call('gnnd_train_bwd', graph.handle, _lib.VARIANT[model], dt, _ptr(plain_weights), _ptr(x),
              _ptr(out), _ptr(grad_out), _ptr(tape), _ptr(gw), _ptr(ws), nb.value, B, int(iters),
              current_stream(x.device))
    return gw


def train_backward_partial(graph, model, plain_weights, x, out, grad_out, tape, iters, ws=None):
    """gnnd_train_bwd_partial: the reverse pass leaving its per-workgroup gradient rows in a
    workspace.  Returns (workspace, rows); reduce with train_update."""
    B = x.numel() // graph.N
    dt = dtype_code(x.dtype)
    nr = ctypes.c_int64()
    _lib.call('gnnd_train_bwd_rows', graph.handle, _lib.VARIANT[model], dt, B, ctypes.byref(nr))
    nb = ctypes.c_int64()
    _lib.call('gnnd_train_workspace_bytes', graph.handle, _lib.VARIANT[model], dt, B, int(iters),
              ctypes.byref(nb))
    if ws is None or ws.numel() < nb.value:
        ws = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=x.device)
    grad_out = grad_out.contiguous()
    _lib.call('gnnd_train_bwd_partial', graph.handle, _lib.VARIANT[model], dt, _ptr(plain_weights),
              _ptr(x), _ptr(out), _ptr(grad_out), _ptr(tape), _ptr(ws), nb.value, B, int(iters),
              current_stream(x.device))
    return ws, int(nr.value)


def train_backward_loss_partial(graph, model, plain_weights, x, out, y, logical_mask, n_logical,
                                logical_only, tape, iters, ws=None):
    """gnnd_train_bwd_loss_partial: the reverse pass with the syndrome loss fused in (no
    d loss / d out tensor).  Returns (workspace, rows, per-codeword-and-component losses), or
    None when the graph's tables plus the loss arrays exceed the workgroup's LDS (nothing
    launched: use the syndrome-loss kernel and train_backward_partial instead)."""
    B = x.numel() // graph.N
    dt = dtype_code(x.dtype)
    nr = ctypes.c_int64()
    _lib.call('gnnd_train_bwd_rows', graph.handle, _lib.VARIANT[model], dt, B, ctypes.byref(nr))
    nb = ctypes.c_int64()
    _lib.call('gnnd_train_workspace_bytes', graph.handle, _lib.VARIANT[model], dt, B, int(iters),
              ctypes.byref(nb))
    nl = ctypes.c_int64()
    _lib.call('gnnd_train_loss_count', graph.handle, B, ctypes.byref(nl))
    if ws is None or ws.numel() < nb.value:
        ws = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=x.device)
    loss_b = torch.empty(max(nl.value, 1), dtype=x.dtype, device=x.device)[:nl.value]
    y = y.to(x.dtype).contiguous()
    ok = _lib.call_or_unsupported(
        'gnnd_train_bwd_loss_partial', graph.handle, _lib.VARIANT[model], dt,
        _ptr(plain_weights), _ptr(x), _ptr(out), _ptr(y), _ptr(logical_mask), int(n_logical),
        int(bool(logical_only)), _ptr(tape), _ptr(loss_b), _ptr(ws), nb.value, B, int(iters),
        current_stream(x.device))
    return (ws, int(nr.value), loss_b) if ok else None


def train_update(model, dtype, rows=None, n_rows=0, grad=None, loss_b=None, loss=None,
                 param=None, exp_avg=None, exp_avg_sq=None, step=None, sync=None, lr=3e-4,
                 betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, prepared=None, device=None):
    """gnnd_train_update: reduce the reverse pass's rows (and the per-codeword losses) and/or
    apply Adam + the kernel-layout weight copy, in one launch (see include/gnnd.h)."""
    dev = device or (param.device if param is not None else grad.device)
    _lib.call('gnnd_train_update', _lib.VARIANT[model], dtype_code(dtype), _ptr(rows), int(n_rows),
              _ptr(grad), _ptr(loss_b), 0 if loss_b is None else loss_b.numel(), _ptr(loss),
              _ptr(param), _ptr(exp_avg), _ptr(exp_avg_sq), _ptr(step), _ptr(sync), float(lr),
              float(betas[0]), float(betas[1]), float(eps), float(weight_decay), _ptr(prepared),
              current_stream(dev))


class FusedTrainFn(torch.autograd.Function):
    """out = decode(weights, x) with a one-launch HIP backward to the packed weights."""

    @staticmethod
    def forward(ctx, flat_w, x, graph, model, iters):
        w = flat_w.detach().to(x.dtype).contiguous()
        out, tape = train_forward(graph, model, x, prepare_weights(model, w), iters)
        ctx.save_for_backward(w, x, out, tape)
        ctx.args = (graph, model, iters, flat_w.dtype)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        w, x, out, tape = ctx.saved_tensors
        graph, model, iters, wdt = ctx.args
        gw = train_backward(graph, model, w, x, out, grad_out.to(x.dtype), tape, iters)
        return gw.to(wdt), None, None, None, None


# ---------------------------------------------------------------------------------------
# training objective: syndrome loss + gradient in one launch (gnnd_syndrome_loss)
# ---------------------------------------------------------------------------------------
def syndrome_loss(graph, logical_rows, logical_only, pred, y):
    """(per-codeword losses [B], d loss / d pred [B*V, 1]) of quantum/decoder_v2_4.py:297-317
    (logical_only: quantum/QGNNI.py:255-290).  logical_rows: int32 [n_l, V] on the device."""
    _require_gpu(pred, y)
    V = graph.V
    pred = pred.contiguous()
    y = y.to(pred.dtype).contiguous()
    B = pred.numel() // V
    if pred.numel() != B * V or y.numel() != pred.numel():
        raise ValueError(f'pred/y must hold B*V values (V = {V})')
    loss_b = torch.empty(B, dtype=pred.dtype, device=pred.device)
    dpred = torch.empty_like(pred)
    lg = logical_rows.contiguous()
    _lib.call('gnnd_syndrome_loss', graph.handle, _ptr(lg), int(lg.size(0)), int(bool(logical_only)),
              dtype_code(pred.dtype), _ptr(pred), _ptr(y), _ptr(loss_b), _ptr(dpred), B,
              current_stream(pred.device))
    return loss_b, dpred


def v24_check_mlp_table(graph, w, u):
    """decoder_v2_4's check-side MLP evaluated through the fp64 decoder's table
    (gnnd_v24_check_mlp_table): (y [n] fp64, valid) where valid says whether the decoder uses
    the table for these weights (y undefined when not).  w: packed fp64 V24 weights (1283,
    prepared here) or prepared ones; u: fp64 inputs within [-(max_dc - 1), max_dc - 1]."""
    _require_gpu(w, u)
    w = w.to(torch.float64).contiguous()
    if w.numel() == weights_count('v24'):
        w = prepare_weights('v24', w)
    u = u.to(torch.float64).contiguous().reshape(-1)
    y = torch.empty_like(u)
    ok = torch.zeros(1, dtype=torch.int32, device=u.device)
    _lib.call('gnnd_v24_check_mlp_table', graph.handle, _ptr(w), _ptr(u), _ptr(y), u.numel(),
              _ptr(ok), current_stream(u.device))
    return y, bool(ok.item())


def decision_errors(graph, logical_rows, pred, y):
    """(bit errors, frame errors, residual-syndrome failures, logical failures) of hard
    decisions pred > 0.5 against y, one HIP launch (gnnd_decision_errors); int64 tensor [4]
    on the device (no host sync).  logical_rows: int32 [n_l, V] or None (classical)."""
    _require_gpu(pred, y)
    V = graph.V
    pred = pred.contiguous()
    y = y.to(pred.dtype).contiguous()
    B = pred.numel() // V
    if pred.numel() != B * V or y.numel() != pred.numel():
        raise ValueError(f'pred/y must hold B*V values (V = {V})')
    counts = torch.empty(4, dtype=torch.int64, device=pred.device)
    if logical_rows is None:
        lg, nl = None, 0
    else:
        lg = logical_rows.to(device=pred.device, dtype=torch.int32).contiguous()
        nl = int(lg.size(0))
    _lib.call('gnnd_decision_errors', graph.handle, _ptr(lg), nl,
              dtype_code(pred.dtype), _ptr(pred), _ptr(y), _ptr(counts), B,
              current_stream(pred.device))
    return counts


class SyndromeLossFn(torch.autograd.Function):
    """Batch-summed syndrome loss; backward scales the kernel's d loss / d pred."""

    @staticmethod
    def forward(ctx, pred, y, graph, logical_rows, logical_only):
        loss_b, dpred = syndrome_loss(graph, logical_rows, logical_only, pred, y)
        ctx.save_for_backward(dpred)
        return loss_b.sum()

    @staticmethod
    def backward(ctx, g):
        (dpred,) = ctx.saved_tensors
        return dpred * g, None, None, None, None


def adam_step(param, grad, exp_avg, exp_avg_sq, step, lr, betas=(0.9, 0.999), eps=1e-8,
              weight_decay=0.0):
    """In-place torch.optim.Adam update of one flat parameter buffer (gnnd_adam_step);
    `step` is a float64 device scalar tensor incremented by the call."""
    _require_gpu(param, grad, exp_avg, exp_avg_sq, step)
    for t in (grad, exp_avg, exp_avg_sq):
        if t.dtype != param.dtype or t.numel() != param.numel() or not t.is_contiguous():
            raise ValueError('adam_step: buffers must match the parameter (dtype, size, contiguous)')
    if step.dtype != torch.float64 or step.numel() != 1:
        raise ValueError('adam_step: step must be a float64 scalar tensor')
    _lib.call('gnnd_adam_step', dtype_code(param.dtype), _ptr(param), _ptr(grad), _ptr(exp_avg),
              _ptr(exp_avg_sq), _ptr(step), param.numel(), float(lr), float(betas[0]),
              float(betas[1]), float(eps), float(weight_decay), current_stream(param.device))


# ---------------------------------------------------------------------------------------
# input synthesis (gnnd_sample_*)
# ---------------------------------------------------------------------------------------
def _doubles(vals):
    vals = [float(v) for v in vals]
    return (ctypes.c_double * len(vals))(*vals), len(vals)


def sample_toric(graph, B, ps, seed=0, offset=0, dtype=torch.float64, device=None):
    """gen_syn inputs on the device (gnnd_sample_toric): x [B*N, 1], y [B*V, 1]."""
    device = device or graph.device
    x = torch.empty(B * graph.N, 1, dtype=dtype, device=device)
    y = torch.empty(B * graph.V, 1, dtype=dtype, device=device)
    _require_gpu(x)
    arr, n = _doubles(ps)
    _lib.call('gnnd_sample_toric', graph.handle, dtype_code(dtype), arr, n, int(seed) & (2**64 - 1),
              int(offset), _ptr(x), _ptr(y), int(B), current_stream(x.device))
    return x, y


def pack_generator_columns(G):
    """Generator [k, V] (0/1) -> [V, ceil(k/32)] uint32 column bit masks (int32 storage)."""
    import numpy as np
    G = np.asarray(G, dtype=np.uint8)
    k, V = G.shape
    kw = (k + 31) // 32
    cols = np.zeros((V, kw), dtype=np.uint64)
    for i in range(k):
        cols[:, i // 32] |= G[i].astype(np.uint64) << np.uint64(i % 32)
    return torch.from_numpy(cols.astype(np.uint32).view(np.int32)), k


def sample_awgn(graph, B, snrs, gen_cols=None, k=0, codeword_bit=1, seed=0, offset=0,
                dtype=torch.float32, device=None):
    """Gen_Data inputs on the device (gnnd_sample_awgn): x [B*N, 1], labels [B*V, 1].
    gen_cols: device int32 [V, ceil(k/32)] from pack_generator_columns (random codewords),
    or None for the constant word `codeword_bit`."""
    device = device or graph.device
    x = torch.empty(B * graph.N, 1, dtype=dtype, device=device)
    y = torch.empty(B * graph.V, 1, dtype=dtype, device=device)
    _require_gpu(x)
    arr, n = _doubles(snrs)
    if gen_cols is not None:
        if gen_cols.dtype != torch.int32 or not gen_cols.is_cuda or gen_cols.size(0) != graph.V:
            raise ValueError('gen_cols must be a device int32 [V, ceil(k/32)] tensor')
        gen_cols = gen_cols.contiguous()
    _lib.call('gnnd_sample_awgn', graph.handle, dtype_code(dtype), arr, n, _ptr(gen_cols), int(k),
              int(codeword_bit), int(seed) & (2**64 - 1), int(offset), _ptr(x), _ptr(y), int(B),
              current_stream(x.device))
    return x, y


def philox4x32_10(counter, key):
    """Host mirror of the device generator (known-answer tests)."""
    c = (ctypes.c_uint32 * 4)(*[int(v) & 0xffffffff for v in counter])
    kk = (ctypes.c_uint32 * 2)(*[int(v) & 0xffffffff for v in key])
    out = (ctypes.c_uint32 * 4)()
    _lib.get().gnnd_philox4x32_10(c, kk, out)
    return list(out)
