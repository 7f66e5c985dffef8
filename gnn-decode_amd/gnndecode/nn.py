"""Drop-in `MessagePassing` operator (the reference's per-script PyG-1.x-style base class).

Interface kept from the reference (quantum/decoder_v2_4.py:66-158, classical/CGNNI.py:33-122):

* `MessagePassing(aggr='add', flow='source_to_target')` — `aggr` in {add, mean, max},
  `flow` in {source_to_target, target_to_source}; `message`/`update` argument names are
  introspected the same way (`message` args minus self; `update` args minus self, aggr_out).
* `propagate(edge_index, extra=None, size=None, **kwargs)` — kwargs carry `x` (per-edge
  messages: the reference's gather is commented out, classical/CGNNI.py:80) and any names
  `update` asks for.  `size` inference and the `_i`/`_j` suffix rules are the reference's.
  The classical scripts name the 2nd parameter `post` (classical/CGNNI.py:52): use
  `ClassicalMessagePassing` / `variant='cgnni'`.
* The aggregation + pre/post-op body between `message` and `update` runs on the GPU
  (libgnnd: gnnd_propagate_tiled / gnnd_propagate_generic).  Each reference script has its
  own body; pick it with the class attribute `variant`:
      'v24'   quantum/decoder_v2_4.py:132-144     'qgnni' quantum/QGNNI.py:101-112
      'qbp'   quantum/BP.py:101-119               'cgnni' classical/CGNNI.py:99-108
      'cbp'   classical/BP.py:99-119
  Bind a `TannerGraph` (`bind_graph`) to use the tiled LDS kernel; otherwise the generic
  atomic kernel handles any edge_index.
"""
import inspect

import torch

from . import ops

special_args = ['edge_index', 'edge_index_i', 'edge_index_j', 'size', 'size_i', 'size_j']
__size_error_msg__ = ('All tensors which should get mapped to the same source'
                      'or target nodes must be of same size in dimension 0.')

AGGRS = ('add', 'mean', 'max')
FLOWS = ('source_to_target', 'target_to_source')


def _positional_names(fn):
    return inspect.getfullargspec(fn)[0]


class MessagePassing(torch.nn.Module):
    variant = 'v24'

    def __init__(self, aggr='add', flow='source_to_target'):
        super().__init__()
        self.aggr = aggr
        assert self.aggr in AGGRS
        self.flow = flow
        assert self.flow in FLOWS
        margs = _positional_names(self.message)[1:]
        self.__special_args__ = [(k, a) for k, a in enumerate(margs) if a in special_args]
        self.__message_args__ = [a for a in margs if a not in special_args]
        self.__update_args__ = _positional_names(self.update)[2:]
        self.graph = None

    def bind_graph(self, graph):
        """Attach the single-codeword TannerGraph so propagate can use the tiled kernel."""
        self.graph = graph
        return self

    # ---------------------------------------------------------------------------------
    def _collect(self, edge_index, size, kwargs):
        """Reference argument handling (quantum/decoder_v2_4.py:86-130)."""
        size = [None, None] if size is None else list(size)
        assert len(size) == 2
        i, j = (0, 1) if self.flow == 'target_to_source' else (1, 0)
        suffix = {'_i': i, '_j': j}
        margs = []
        for name in self.__message_args__:
            side = suffix.get(name[-2:])
            if side is None:
                margs.append(kwargs[name])
                continue
            val = kwargs[name[:-2]]
            if val is not None:
                if isinstance(val, (tuple, list)):
                    assert len(val) == 2
                    other = 1 - side
                    if size[other] is None:
                        size[other] = val[other].size(0)
                    if size[other] != val[other].size(0):
                        raise ValueError(__size_error_msg__)
                    val = val[side]
                if size[side] is None:
                    size[side] = val.size(0)
            margs.append(val)
        if size[0] is None:
            size[0] = size[1]
        if size[1] is None:
            size[1] = size[0]
        kwargs['edge_index'] = edge_index
        kwargs['size'] = size
        for pos, name in self.__special_args__:
            side = suffix.get(name[-2:])
            margs.insert(pos, kwargs[name[:-2]][side] if side is not None else kwargs[name])
        uargs = [kwargs[name] for name in self.__update_args__]
        return margs, uargs, size, i

    def propagate(self, edge_index, extra=None, size=None, **kwargs):
        margs, uargs, size, i = self._collect(edge_index, size, kwargs)
        out = self.message(*margs)
        dim_size = size[i]
        if dim_size is None:
            dim_size = extra.size(0) if extra is not None else int(edge_index[i].max()) + 1
        out = ops.propagate(self.variant, self.flow, self.aggr, edge_index, out, extra,
                            dim_size, graph=self.graph)
        return self.update(out, *uargs)

    def message(self, x_j):
        return x_j

    def update(self, aggr_out):
        return aggr_out


class ClassicalMessagePassing(MessagePassing):
    """classical/CGNNI.py:33-122 flavour: 2nd parameter is `post`, added when not None."""
    variant = 'cgnni'

    def propagate(self, edge_index, post, size=None, **kwargs):
        return super().propagate(edge_index, post, size, **kwargs)


def message_passing_class(variant):
    """The MessagePassing base class of one reference script."""
    if variant == 'cgnni':
        return ClassicalMessagePassing
    return type(f'MessagePassing_{variant}', (MessagePassing,), {'variant': variant})
