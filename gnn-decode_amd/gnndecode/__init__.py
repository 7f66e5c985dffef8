"""gnndecode — MI355X-native (gfx950) GNN belief-propagation decoder.

Drop-in for the `MessagePassing.propagate()` T-iteration decode loop of
ironmanaudi/GNN-decode.  Compute runs in hand-written HIP kernels (libgnnd.so, C ABI in
include/gnnd.h); PyTorch provides device memory, streams and torch.distributed only.
"""
from . import _lib, checkpoint, codes, data, loss, train
from .graph import TannerGraph
from .nn import MessagePassing, ClassicalMessagePassing, message_passing_class
from .models import (DecoderV24, QGNNI, QuantumBP, CGNNI, ClassicalBP, NeuralBP, DecoderV10,
                     DecoderV30, DecoderV22, MODELS, DEFAULT_ITERS, init_weights)
from . import ops
from . import library   # registers the gnnd:: torch ops

__all__ = ['TannerGraph', 'MessagePassing', 'ClassicalMessagePassing', 'message_passing_class',
           'DecoderV24', 'QGNNI', 'QuantumBP', 'CGNNI', 'ClassicalBP', 'NeuralBP', 'DecoderV10',
           'DecoderV30', 'DecoderV22', 'MODELS', 'DEFAULT_ITERS',
           'init_weights', 'ops', 'checkpoint', 'codes', 'data', 'loss', 'train']
