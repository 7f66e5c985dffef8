"""torch.library registration of the device operators (gnndecode/library.py): the gnnd::
ops exist, carry fake kernels (shape propagation without a GPU launch), trace under FX /
torch.compile (aot_eager: no code generation) and pass torch.library.opcheck on the GPU."""
import numpy as np
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

import gnndecode as gd
from gnndecode import library


def test_ops_registered():
    for name in ('propagate', 'propagate_bwd', 'decode', 'decode_out'):
        assert hasattr(torch.ops.gnnd, name), name


@pytest.mark.parametrize('model,rows', [('cgnni', 10 * 63), ('v30', 2 * 10 * 81), ('v22', 25 * 10 * 63)])
def test_decode_fake_kernel_shapes(model, rows):
    gid = 10_000 + len(library._DIMS)
    library._DIMS[gid] = (63, 18, 81, 432)
    with FakeTensorMode():
        x = torch.empty(10 * 81, 1, device='cuda')
        out = torch.ops.gnnd.decode(gid, model, x, 25, None)
        assert tuple(out.shape) == (rows, 1) and out.dtype == x.dtype


@pytest.mark.parametrize('variant,flow,width', [('v24', 'source_to_target', 2), ('qgnni', 'source_to_target', 1),
                                                ('qgnni', 'target_to_source', 2), ('v30', 'target_to_source', 2)])
def test_propagate_fake_kernel_shapes(variant, flow, width):
    with FakeTensorMode():
        msg = torch.empty(300, 1, device='cuda', dtype=torch.float64)
        ei = torch.empty(2, 300, dtype=torch.int64, device='cuda')
        ex = torch.empty(90, 1, device='cuda', dtype=torch.float64)
        out = torch.ops.gnnd.propagate(variant, flow, 'add', ei, msg, ex, 90, -1, -1)
        assert tuple(out.shape) == (300, width)
        g = torch.ops.gnnd.propagate_bwd(variant, flow, 'add', ei, msg, ex, out, 90, -1, -1)
        assert g.shape == msg.shape


@pytest.mark.gpu
def test_compiled_decode_and_propagate_match_eager(golden):
    z = golden('v24_toric5')
    H = golden('toric_L5_graph')['H']
    m = gd.DecoderV24(15, H)
    m.load_state_dict({k[2:]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith('w/')})
    m = m.cuda().eval()
    x = torch.from_numpy(z['x_B4']).cuda()
    data = gd.data.make_batch(x, m.graph(x.device))
    g = m.graph(x.device)
    w = m.prepared_weights(x.dtype, x.device)

    def f(xx):
        return gd.ops.decode(g, 'v24', xx, 15, w)

    eager = f(x)
    comp = torch.compile(f, backend='aot_eager', fullgraph=True)(x)
    assert torch.equal(eager, comp)
    with torch.no_grad():
        assert torch.equal(m(data), eager)

    ei = g.batched_edge_index(4, chk_shift=g.V)
    msg = torch.randn(ei.size(1), 1, dtype=torch.float64, device='cuda', requires_grad=True)

    def p(mm):
        return gd.ops.propagate('v24', 'target_to_source', 'add', ei, mm, x, x.size(0), graph=g).sum()

    a = torch.autograd.grad(p(msg), msg)[0]
    b = torch.autograd.grad(torch.compile(p, backend='aot_eager', fullgraph=True)(msg), msg)[0]
    assert torch.equal(a, b)


@pytest.mark.gpu
def test_opcheck_propagate():
    H = gd.codes.toric_code(4)
    g = gd.TannerGraph(H, device='cuda')
    ei = g.batched_edge_index(2, chk_shift=g.V)
    msg = torch.randn(ei.size(1), 1, dtype=torch.float64, device='cuda', requires_grad=True)
    ex = torch.randn(2 * g.N, 1, dtype=torch.float64, device='cuda')
    for gid in (g.gid, -1):
        torch.library.opcheck(torch.ops.gnnd.propagate,
                              ('v24', 'target_to_source', 'add', ei, msg, ex, 2 * g.N, gid, -1))
