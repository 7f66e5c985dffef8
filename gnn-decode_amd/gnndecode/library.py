"""torch.library registration of the device operators.

The public entries of `gnndecode.ops` dispatch to these custom ops whenever they are traced
(torch.compile / FX: `torch.compiler.is_compiling()`), so the decoder is a set of named
operators with fake kernels for shape propagation instead of opaque ctypes calls; eager
calls run the same implementation functions directly (the Python dispatcher round trip of
a custom op costs more than the 0.47 ms headline kernel, measured r02n):

  gnnd::propagate(variant, flow, aggr, edge_index, msg, extra?, dim_size, graph_id, chk_shift)
      one reference `propagate` body (quantum/decoder_v2_4.py:85-148 and the other scripts'
      copies); autograd through gnnd::propagate_bwd
  gnnd::propagate_bwd(..., grad_out, ...)  d out / d msg (HIP backward kernels)
  gnnd::decode(graph_id, model, x, iters, weights?)          fused T-iteration decoder
  gnnd::decode_out(graph_id, model, x, iters, weights?, out)  the same into `out` (mutates)

The single-codeword Tanner graph is a device object owned by libgnnd, not a tensor: ops
take the integer id that `register_graph` hands out (TannerGraph does this on creation;
-1 = no graph: the generic kernels).  Implementations are the ctypes launches in
`gnndecode.ops` (`_propagate_impl`, `_decode_impl`): no CPU kernel is registered, so a CPU
tensor reaching an op fails in the dispatcher instead of falling back.
"""
import weakref
from typing import Optional

import torch
from torch import Tensor

_GRAPHS = {}          # id -> weakref(TannerGraph)
_DIMS = {}            # id -> (V, C, N, E): shapes for the fake kernels
_NEXT = [0]


def register_graph(graph) -> int:
    gid = _NEXT[0]
    _NEXT[0] += 1
    _GRAPHS[gid] = weakref.ref(graph)
    _DIMS[gid] = (graph.V, graph.C, graph.N, graph.E)
    return gid


def graph_of(gid):
    if gid < 0:
        return None
    ref = _GRAPHS.get(gid)
    g = ref() if ref is not None else None
    if g is None:
        raise RuntimeError(f'gnnd: Tanner graph {gid} no longer exists')
    return g


def _out_rows(gid, model, B, iters=1):
    V, C, N, E = _DIMS[gid]
    if model == 'v30':
        return 2 * B * N
    return iters * B * V if model == 'v22' else B * V


# ---------------------------------------------------------------------------------------
# propagate
# ---------------------------------------------------------------------------------------
@torch.library.custom_op('gnnd::propagate', mutates_args=(), device_types='cuda')
def propagate(variant: str, flow: str, aggr: str, edge_index: Tensor, msg: Tensor,
              extra: Optional[Tensor], dim_size: int, graph_id: int, chk_shift: int) -> Tensor:
    from . import ops
    return ops._propagate_impl(variant, flow, aggr, edge_index, msg, extra, dim_size,
                               graph_of(graph_id), None if chk_shift < 0 else chk_shift)


@propagate.register_fake
def _propagate_fake(variant, flow, aggr, edge_index, msg, extra, dim_size, graph_id, chk_shift):
    from . import ops
    return msg.new_empty(msg.size(0), ops.propagate_width(variant, flow))


@torch.library.custom_op('gnnd::propagate_bwd', mutates_args=(), device_types='cuda')
def propagate_bwd(variant: str, flow: str, aggr: str, edge_index: Tensor, msg: Tensor,
                  extra: Optional[Tensor], grad_out: Tensor, dim_size: int, graph_id: int,
                  chk_shift: int) -> Tensor:
    from . import ops
    return ops._propagate_bwd_impl(variant, flow, aggr, edge_index, msg, extra, grad_out,
                                   dim_size, graph_of(graph_id),
                                   None if chk_shift < 0 else chk_shift)


@propagate_bwd.register_fake
def _propagate_bwd_fake(variant, flow, aggr, edge_index, msg, extra, grad_out, dim_size,
                        graph_id, chk_shift):
    return torch.empty_like(msg)


def _prop_setup(ctx, inputs, output):
    variant, flow, aggr, edge_index, msg, extra, dim_size, graph_id, chk_shift = inputs
    ctx.save_for_backward(edge_index, msg, extra)
    ctx.args = (variant, flow, aggr, dim_size, graph_id, chk_shift)


def _prop_backward(ctx, grad_out):
    edge_index, msg, extra = ctx.saved_tensors
    variant, flow, aggr, dim_size, graph_id, chk_shift = ctx.args
    if aggr != 'add':
        raise NotImplementedError(f'no backward for aggr={aggr!r}')
    gmsg = torch.ops.gnnd.propagate_bwd(variant, flow, aggr, edge_index, msg, extra,
                                        grad_out.contiguous(), dim_size, graph_id, chk_shift)
    return None, None, None, None, gmsg, None, None, None, None


torch.library.register_autograd('gnnd::propagate', _prop_backward, setup_context=_prop_setup)


# ---------------------------------------------------------------------------------------
# fused decoder
# ---------------------------------------------------------------------------------------
@torch.library.custom_op('gnnd::decode', mutates_args=(), device_types='cuda')
def decode(graph_id: int, model: str, x: Tensor, iters: int, weights: Optional[Tensor]) -> Tensor:
    from . import ops
    g = graph_of(graph_id)
    out = torch.empty(ops.decode_out_rows(g, model, x.numel() // g.N, iters), 1, dtype=x.dtype,
                      device=x.device)
    ops._decode_impl(g, model, x, iters, weights, out)
    return out


@decode.register_fake
def _decode_fake(graph_id, model, x, iters, weights):
    N = _DIMS[graph_id][2]
    return x.new_empty(_out_rows(graph_id, model, x.numel() // N, iters), 1)


@torch.library.custom_op('gnnd::decode_out', mutates_args=('out',), device_types='cuda')
def decode_out(graph_id: int, model: str, x: Tensor, iters: int, weights: Optional[Tensor],
               out: Tensor) -> None:
    from . import ops
    ops._decode_impl(graph_of(graph_id), model, x, iters, weights, out)


@decode_out.register_fake
def _decode_out_fake(graph_id, model, x, iters, weights, out):
    return None
