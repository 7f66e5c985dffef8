"""Worker for tests/test_gpu_debug.py (run as a child process with GNND_LIB pointing at
libgnnd_debug.so or the release library): decodes every model on its configs' codes,
propagates on both kernels, samples inputs and runs one fused training step, then prints
one JSON line with the debug flags and a checksum of every output."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gnn-decode_amd'))
import gnndecode as gd  # noqa: E402
from gnndecode import _lib  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    sums = {}
    cases = [('cgnni', 'bch_63_45', torch.float32), ('cgnni', 'ldpc_648_324', torch.float32),
             ('cbp', 'bch_63_45', torch.float32), ('cbp', 'bch_63_45', torch.bfloat16),
             ('qgnni', 'toric_5', torch.float32), ('qgnni', 'toric_5', torch.float64),
             ('qbp', 'toric_5', torch.float32), ('v24', 'toric_5', torch.float32),
             ('v24', 'toric_5', torch.float64), ('nbp', 'toric_4', torch.float32),
             ('v10', 'toric_4', torch.float64), ('v30', 'toric_5', torch.float64),
             ('v22', 'toric_4', torch.float64), ('v22', 'toric_4', torch.float32)]
    for model, code, dt in cases:
        H = gd.codes.get_code(code)
        torch.manual_seed(1)
        m = gd.MODELS[model](gd.DEFAULT_ITERS[model], H).to(dev).eval()
        if code.startswith('toric'):
            x, _ = gd.data.toric_batch(H, 300, seed=2, device=dev,
                                       dtype=torch.float64 if dt == torch.float64 else torch.float32)
        else:
            x, _ = gd.data.awgn_batch(H, 300, seed=2, device=dev, codewords='random')
        x = x.to(dt)
        with torch.no_grad():
            out = m(gd.data.make_batch(x, m.graph(dev)))
        out = torch.cat([o.reshape(-1) for o in out]) if isinstance(out, list) else out
        sums[f'{model}/{code}/{dt}'] = float(out.double().sum())
    H = gd.codes.toric_code(5)
    g = gd.TannerGraph(H, device=dev)
    ei = g.batched_edge_index(3, chk_shift=g.V)
    msg = torch.randn(ei.size(1), 1, dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(3))
    ex = torch.randn(3 * g.N, 1, dtype=torch.float64, device=dev, generator=torch.Generator(dev).manual_seed(4))
    for gr in (g, None):
        for v, f in (('v24', 'target_to_source'), ('qbp', 'target_to_source'), ('v30', 'source_to_target')):
            o = gd.ops.propagate(v, f, 'add', ei, msg, ex, 3 * g.N, graph=gr)
            sums[f'prop/{v}/{f}/{gr is not None}'] = float(o.sum())
    m = gd.DecoderV24(5, H).to(dev)
    lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H)).to(dev)
    tr = gd.train.FusedV24Trainer(m, lf, graph=False)
    x, y = gd.data.toric_batch(H, 64, seed=5, device=dev, dtype=torch.float32)
    m.float()
    tr2 = gd.train.FusedV24Trainer(m, lf, graph=False)
    sums['train'] = float(tr2.step(gd.data.make_batch(x, m.graph(dev)), y))
    del tr
    flags = ctypes_flags()
    print(json.dumps({'debug': _lib.get().gnnd_debug_enabled(), 'flags': flags, 'sums': sums}))


def ctypes_flags():
    import ctypes
    f = ctypes.c_uint32()
    _lib.call('gnnd_debug_flags', ctypes.byref(f))
    return int(f.value)


if __name__ == '__main__':
    main()
