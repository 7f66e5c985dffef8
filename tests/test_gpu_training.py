"""GPU training parity: one forward + reference loss + backward through the HIP propagate
kernels (forward and backward) vs gradients of the reference's own classes (golden)."""
import numpy as np
import pytest
import torch

from conftest import weights_of

pytestmark = pytest.mark.gpu
DEV = 'cuda'

CASES = [  # fixture, model, code, loss kind, dtype tolerance
    ('train_v24_L5', 'v24', ('toric', 5), 'syndrome'),
    ('train_v24_L7', 'v24', ('toric', 7), 'syndrome'),
    ('train_qgnni_L4', 'qgnni', ('toric', 4), 'logical'),
    ('train_cgnni_bch', 'cgnni', ('bch', None), 'classical'),
    ('train_nbp_L4', 'nbp', ('toric', 4), 'syndrome'),
    ('train_v10_L4', 'v10', ('toric', 4), 'syndrome'),
]


def _setup(golden, fx, model, code, kind):
    import gnndecode as gd
    z = golden(fx)
    H = gd.codes.toric_code(code[1]) if code[0] == 'toric' else gd.codes.bch_63_45()
    m = gd.MODELS[model](int(z['T']), H)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()})
    m = m.to(DEV).train()
    if kind == 'classical':
        lf = gd.loss.ClassicalLoss(H).to(DEV)
        loss_fn = lambda p, y: lf(p, y, train=True)
    else:
        lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H), logical_only=(kind == 'logical')).to(DEV)
        loss_fn = lf
    x = torch.from_numpy(z['x']).to(DEV)
    y = torch.from_numpy(z['y']).to(DEV)
    return z, m, loss_fn, gd.data.make_batch(x, m.graph(x.device)), y


def _cases_with_path():
    for c in CASES:
        yield pytest.param(*c, True, id=c[0])
        if c[1] == 'v24':    # decoder_v2_4 also through the layer-by-layer operator path
            yield pytest.param(*c, False, id=c[0] + '-layerwise')


@pytest.mark.parametrize('fx,model,code,kind,fused', list(_cases_with_path()))
def test_training_step_gradients_match_reference(golden, fx, model, code, kind, fused):
    z, m, loss_fn, data, y = _setup(golden, fx, model, code, kind)
    if model == 'v24':
        m.fused_train = fused
    pred = m(data)
    assert pred.requires_grad, 'training forward must build an autograd graph'
    loss = loss_fn(pred, y)
    loss.backward()
    f64 = pred.dtype == torch.float64
    np.testing.assert_allclose(pred.detach().cpu().numpy(), z['pred'],
                               rtol=1e-10 if f64 else 1e-4, atol=1e-12 if f64 else 2e-5)
    assert abs(loss.item() - float(z['loss'])) <= (1e-9 if f64 else 1e-4) * max(1, abs(float(z['loss'])))
    for name, p in m.named_parameters():
        key = 'g/' + name
        if key not in z.files:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, name
            continue
        ref = z[key]
        got = p.grad.detach().cpu().numpy()
        scale = max(np.abs(ref).max(), 1e-30)
        tol = 1e-8 if f64 else 2e-3
        assert np.abs(got - ref).max() <= tol * scale, (name, np.abs(got - ref).max(), scale)


def test_propagate_backward_generic_and_tiled_match_autograd_restatement(golden):
    """d propagate / d msg on both device paths vs torch autograd of the literal formula."""
    import gnndecode as gd
    H = gd.codes.toric_code(5)
    g = gd.TannerGraph(H, device=DEV)
    B = 3
    ei = g.batched_edge_index(B, chk_shift=g.V)
    gen = torch.Generator(device=DEV).manual_seed(0)
    msg = torch.randn(ei.size(1), 1, generator=gen, device=DEV, dtype=torch.float64)
    extra = torch.randn(B * g.N, 1, generator=gen, device=DEV, dtype=torch.float64)
    for flow in ('source_to_target', 'target_to_source'):
        j = 0 if flow == 'source_to_target' else 1
        w = torch.randn(ei.size(1), 2, generator=gen, device=DEV, dtype=torch.float64)
        # literal restatement (torch autograd)
        m0 = msg.clone().requires_grad_(True)
        t = torch.tanh(m0 / 2) if j == 1 else m0
        agg = torch.zeros(B * g.N, 1, dtype=t.dtype, device=DEV).index_add(0, ei[j], t)
        ref_out = torch.cat([agg[ei[j]] - t, extra[ei[j]]], dim=1)
        (ref_out * w).sum().backward()
        for graph in (g, None):
            m1 = msg.clone().requires_grad_(True)
            out = gd.ops.propagate('v24', flow, 'add', ei, m1, extra, B * g.N, graph=graph)
            (out * w).sum().backward()
            np.testing.assert_allclose(out.detach().cpu().numpy(), ref_out.detach().cpu().numpy(),
                                       rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(m1.grad.cpu().numpy(), m0.grad.cpu().numpy(),
                                       rtol=1e-11, atol=1e-12)


@pytest.mark.parametrize('fx,L', [('train_v24_L5', 5), ('train_v24_L7', 7)])
def test_fused_training_step_matches_layerwise_fp32(golden, fx, L):
    """fp32: the fused HIP training step (gnnd_train_fwd/bwd) and the layer-by-layer
    operator path give the same loss and gradients (different fp32 rounding orders)."""
    grads = []
    for fused in (True, False):
        z, m, loss_fn, data, y = _setup(golden, fx, 'v24', ('toric', L), 'syndrome')
        m = m.float()
        m.fused_train = fused
        data.x = data.x.float()
        pred = m(data)
        loss = loss_fn(pred, y.float())
        loss.backward()
        grads.append((loss.item(), {n: p.grad.detach().double().cpu().numpy()
                                    for n, p in m.named_parameters()}))
    (la, ga), (lb, gb) = grads
    assert abs(la - lb) <= 1e-4 * abs(lb)
    for n in gb:
        scale = max(np.abs(gb[n]).max(), 1e-30)
        assert np.abs(ga[n] - gb[n]).max() <= 2e-3 * scale, n


def test_fused_training_step_is_deterministic(golden):
    z, m, loss_fn, data, y = _setup(golden, 'train_v24_L7', 'v24', ('toric', 7), 'syndrome')
    out = []
    for _ in range(2):
        m.zero_grad()
        loss_fn(m(data), y).backward()
        out.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]).clone())
    assert torch.equal(out[0], out[1])


def test_data_parallel_step_on_one_gpu_matches_plain_step(golden):
    """Trainer (all-reduce is a no-op at world size 1) == manual step."""
    import gnndecode as gd
    z, m, loss_fn, data, y = _setup(golden, 'train_v24_L5', 'v24', ('toric', 5), 'syndrome')
    tr = gd.train.Trainer(m, loss_fn)
    before = [p.detach().clone() for p in m.parameters()]
    loss = tr.step(data, y)
    assert abs(float(loss) - float(z['loss'])) <= 1e-9 * abs(float(z['loss']))
    assert any((a != p.detach()).any() for a, p in zip(before, m.parameters()))


def test_graph_captured_trainer_matches_eager(golden):
    """Trainer(graph=True) replays one captured HIP graph per step: same losses and the
    same parameters as eager steps on the same data (fp64, exact order preserved)."""
    import gnndecode as gd
    z, m, loss_fn, data, y = _setup(golden, 'train_v24_L5', 'v24', ('toric', 5), 'syndrome')
    _, m2, _, _, _ = _setup(golden, 'train_v24_L5', 'v24', ('toric', 5), 'syndrome')
    eager = gd.train.Trainer(m, loss_fn, lr=1e-3, capturable=True)
    graphed = gd.train.Trainer(m2, loss_fn, lr=1e-3, graph=True, warmup=2)
    for it in range(5):          # 2 eager warm-up steps, capture at step 3, replays after
        a = float(eager.step(data, y))
        b = float(graphed.step(data, y))
        assert abs(a - b) <= 1e-10 * max(1.0, abs(a)), (it, a, b)
    for (n, p), q in zip(m.named_parameters(), m2.parameters()):
        np.testing.assert_allclose(q.detach().cpu().numpy(), p.detach().cpu().numpy(),
                                   rtol=1e-10, atol=1e-13, err_msg=n)


@pytest.mark.parametrize('fused', [False, True])
def test_graphed_step_static_inputs_skip_copies(golden, fused):
    """After the capture, static_inputs() exposes the buffers the replay reads: stepping with
    them (no input copies) gives the same losses and parameters as stepping with separate
    tensors holding the same batch; new data written into them is what the next step sees."""
    import gnndecode as gd
    z, m, loss_fn, data, y = _setup(golden, 'train_v24_L5', 'v24', ('toric', 5), 'syndrome')
    _, m2, _, data2, y2 = _setup(golden, 'train_v24_L5', 'v24', ('toric', 5), 'syndrome')
    cls = gd.train.FusedV24Trainer if fused else gd.train.Trainer
    a_tr = cls(m, loss_fn, lr=1e-3, graph=True, warmup=1)
    b_tr = cls(m2, loss_fn, lr=1e-3, graph=True, warmup=1)
    assert b_tr.static_inputs() is None
    for _ in range(2):                       # eager warm-up, then the capture
        a_tr.step(data, y)
        b_tr.step(data2, y2)
    sx, sy = b_tr.static_inputs()
    data2.x = sx
    y2 = sy
    for it in range(3):
        la, lb = float(a_tr.step(data, y)), float(b_tr.step(data2, y2))
        assert la == lb, (it, la, lb)
    for (n, p), q in zip(m.named_parameters(), m2.parameters()):
        assert torch.equal(p, q), n
    sx.mul_(-1.0)                            # a new batch written in place
    lb = float(b_tr.step(data2, y2))
    data.x = data.x * -1.0
    la = float(a_tr.step(data, y))
    assert la == lb


@pytest.mark.parametrize('variant', ['qbp', 'cbp', 'nbp', 'v10'])
def test_bp_check_step_backward_matches_torch_autograd(variant):
    """d propagate / d msg of the c->v BP bodies (tiled and generic kernels) vs torch
    autograd of the literal reference formula (quantum/BP.py:102-117, classical/BP.py:
    100-116, quantum/neural_BP.py:109-122), including saturated and clamped messages."""
    import math
    import gnndecode as gd
    H = gd.codes.toric_code(4) if variant != 'cbp' else gd.codes.bch_63_45()
    g = gd.TannerGraph(H, device=DEV)
    B = 3
    ei = g.batched_edge_index(B, chk_shift=g.V)
    gen = torch.Generator(device=DEV).manual_seed(1)
    dt = torch.float64
    msg = torch.randn(ei.size(1), 1, generator=gen, device=DEV, dtype=dt) * 4
    msg[::9] *= 10                                   # beyond +-10 and into tanh saturation
    xc = torch.where(torch.rand(B, g.C, generator=gen, device=DEV) < 0.3, -1.0, 1.0)
    xv = torch.randn(B, g.V, generator=gen, device=DEV)
    extra = torch.cat([xv, xc], 1).reshape(-1, 1).to(dt)
    w = torch.randn(ei.size(1), 1, generator=gen, device=DEV, dtype=dt)
    quantum = variant != 'cbp'
    lo = 1e-7 if variant == 'cbp' else 1e-20
    hi = {'cbp': 1 - 1e-7, 'qbp': 1 - 1e-12}.get(variant, 1 - 1e-15)
    m0 = msg.clone().requires_grad_(True)
    out = m0 if variant in ('nbp', 'v10') else torch.clamp(m0, -10, 10)
    out = torch.tanh(out / 2)
    coeff = torch.where(out < 0, torch.ones_like(out), torch.zeros_like(out))
    out = torch.log(torch.clamp(abs(out), lo, 1e10))
    j = ei[1]
    n = extra.size(0)
    out = torch.zeros(n, 1, dtype=dt, device=DEV).index_add(0, j, out)[j] - out
    coeff = torch.zeros(n, 1, dtype=dt, device=DEV).index_add(0, j, coeff)[j] - coeff
    if quantum:
        coeff = coeff + (1 - extra[j]) / 2
    out = torch.clamp(torch.exp(out) * torch.cos(math.pi * coeff), -hi, hi)
    out = torch.log(1 + out) - torch.log(1 - out) if quantum else torch.log((1 + out) / (1 - out))
    (out * w).sum().backward()
    for graph in (g, None):
        m1 = msg.clone().requires_grad_(True)
        got = gd.ops.propagate(variant, 'target_to_source', 'add', ei, m1, extra, n, graph=graph)
        np.testing.assert_allclose(got.detach().cpu().numpy(), out.detach().cpu().numpy(),
                                   rtol=1e-12, atol=1e-12)
        (got * w).sum().backward()
        np.testing.assert_allclose(m1.grad.cpu().numpy(), m0.grad.cpu().numpy(),
                                   rtol=1e-9, atol=1e-12 * float(m0.grad.abs().max()))


def _dp_worker(rank, world, port, steps, q, fused_trainer=False, graph=False):
    """One rank of a 2-process data-parallel run on the single GPU (gloo all-reduce of the
    flat gradient; the fused HIP training kernels on cuda:0)."""
    import os
    import torch.distributed as dist
    import gnndecode as gd
    from conftest import GOLDEN
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    z = np.load(os.path.join(GOLDEN, 'train_v24_L5.npz'))
    H = gd.codes.toric_code(5)
    m = gd.DecoderV24(int(z['T']), H)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()})
    m = m.to(DEV).train()
    lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H)).to(DEV)
    x = torch.from_numpy(z['x']).to(DEV).view(-1, H.shape[0] + H.shape[1])
    y = torch.from_numpy(z['y']).to(DEV).view(-1, H.shape[0])
    s, e = gd.train.shard_bounds(x.size(0), rank, world)
    xs, ys = x[s:e].reshape(-1, 1).contiguous(), y[s:e].reshape(-1, 1).contiguous()
    # graph=True: compute and Adam replay as two HIP graphs with the (gloo) all-reduce issued
    # eagerly between them (gnndecode/train.py _GraphedStep)
    if fused_trainer:
        tr = gd.train.FusedV24Trainer(m, lf, lr=1e-3, graph=graph, warmup=1)
    else:
        tr = gd.train.Trainer(m, lf, lr=1e-3, graph=graph, warmup=1, capturable=True)
    data = gd.data.make_batch(xs, m.graph(xs.device))
    losses = [float(tr.step(data, ys)) for _ in range(steps)]
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu()
    q.put((rank, losses, flat.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('fused_trainer,graph', [(False, False), (True, False), (True, True),
                                                  (False, True)],
                         ids=['torch-trainer', 'fused-trainer', 'fused-trainer-graph',
                              'torch-trainer-graph'])
def test_two_rank_fused_training_equals_full_batch(golden, fused_trainer, graph):
    """Config 5's data-parallel step with the fused HIP kernels: 2 ranks (gloo, both on the
    one GPU), each a shard of the batch, SUM all-reduce -> same parameters and losses as a
    single full-batch process (the reference loss is a sum)."""
    import socket
    import torch.multiprocessing as mp
    import gnndecode as gd
    sock = socket.socket()
    sock.bind(('127.0.0.1', 0))
    port = sock.getsockname()[1]
    sock.close()
    steps, world = 2, 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, steps, q, fused_trainer, graph))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    z, m, loss_fn, data, y = _setup(golden, 'train_v24_L5', 'v24', ('toric', 5), 'syndrome')
    # the worker's torch Trainer runs capturable Adam (device step count); the full-batch
    # reference uses the same form (the host-step form rounds differently)
    tr = gd.train.Trainer(m, loss_fn, lr=1e-3, capturable=not fused_trainer)
    ref_losses = [float(tr.step(data, y)) for _ in range(steps)]
    ref = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu()
    for rank, losses, flat in res:
        flat = torch.tensor(flat, dtype=torch.float64)
        assert flat.tolist() == res[0][2]                 # ranks bitwise equal
        assert torch.allclose(flat, ref, rtol=1e-10, atol=1e-12), \
            float((flat - ref).abs().max())
        assert all(abs(a - b) <= 1e-9 * max(1, abs(b)) for a, b in zip(losses, ref_losses))


@pytest.mark.parametrize('dtype', [torch.float64, torch.float32])
@pytest.mark.parametrize('logical_only', [False, True])
@pytest.mark.parametrize('Ld', [5, 7])
def test_fused_syndrome_loss_matches_reference_formula(dtype, logical_only, Ld):
    """gnnd_syndrome_loss (one launch: loss and d loss / d pred) equals the reference's
    LossFunc formula (quantum/decoder_v2_4.py:297-317) under torch autograd."""
    import gnndecode as gd
    H = gd.codes.toric_code(Ld)
    lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H), logical_only=logical_only).to(DEV)
    B, V = 37, H.shape[0]
    g = torch.Generator(device='cpu').manual_seed(Ld)
    pred = torch.rand(B * V, 1, generator=g, dtype=torch.float64).to(dtype).to(DEV)
    y = (torch.rand(B * V, 1, generator=g) < 0.1).to(dtype).to(DEV)
    pred[:V] = 0.0                      # integer-valued rows: sin(k pi / 2) edge cases
    p1 = pred.clone().requires_grad_(True)
    p2 = pred.clone().requires_grad_(True)
    l1 = lf(p1, y)
    l1.backward()
    l2 = lf.reference_forward(p2, y)
    l2.backward()
    tol = 1e-12 if dtype == torch.float64 else 2e-5
    assert abs(l1.item() - l2.item()) <= tol * max(1.0, abs(l2.item()))
    torch.testing.assert_close(p1.grad, p2.grad, rtol=tol, atol=tol)


@pytest.mark.parametrize('dtype', [torch.float64, torch.float32])
def test_fused_adam_matches_torch_adam(dtype):
    import gnndecode as gd
    g = torch.Generator(device='cpu').manual_seed(3)
    p0 = torch.randn(1283, generator=g, dtype=torch.float64).to(dtype)
    ref = torch.nn.Parameter(p0.clone().to(DEV))
    opt = torch.optim.Adam([ref], lr=3e-4, weight_decay=1e-9, foreach=False)
    flat = p0.clone().to(DEV)
    m, v = torch.zeros_like(flat), torch.zeros_like(flat)
    step = torch.zeros(1, dtype=torch.float64, device=DEV)
    tol = 1e-13 if dtype == torch.float64 else 2e-6
    for _ in range(6):
        gr = torch.randn(1283, generator=g, dtype=torch.float64).to(dtype).to(DEV)
        ref.grad = gr.clone()
        opt.step()
        gd.ops.adam_step(flat, gr, m, v, step, 3e-4, (0.9, 0.999), 1e-8, 1e-9)
        torch.testing.assert_close(flat, ref.detach(), rtol=tol, atol=tol * 1e-3)
    assert step.item() == 6.0


def test_fused_v24_trainer_matches_torch_trainer():
    """FusedV24Trainer (flat parameter views, one-launch loss, HIP Adam, HIP-graph step)
    follows the torch-optimizer Trainer on the same seeded data (fp64, toric d=5)."""
    import gnndecode as gd
    H = gd.codes.toric_code(5)
    lg = gd.codes.toric_logicals(H)
    torch.manual_seed(0)
    a = gd.MODELS['v24'](15, H).to(DEV)
    b = gd.MODELS['v24'](15, H).to(DEV)
    b.load_state_dict(a.state_dict())
    ta = gd.train.Trainer(a, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=False)
    tb = gd.train.FusedV24Trainer(b, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=True, warmup=1)
    keys = sorted(a.state_dict())
    assert sorted(b.state_dict()) == keys
    for s in range(4):
        x, y = gd.data.toric_batch(H, 24, seed=100 + s, device=DEV)
        la = ta.step(gd.data.make_batch(x, a.graph(x.device)), y)
        lb = tb.step(gd.data.make_batch(x, b.graph(x.device)), y)
        assert abs(la.item() - lb.item()) <= 1e-9 * max(1.0, abs(la.item()))
    for k in keys:
        torch.testing.assert_close(b.state_dict()[k], a.state_dict()[k], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize('dtype', [torch.float64, torch.float32])
def test_fused_training_large_batch_equals_sum_of_chunks(dtype):
    """B > 1024: the reverse pass loops each workgroup over a strided set of codewords (one
    gradient row per workgroup).  The reference loss is a sum, so the full-batch gradient
    equals the sum of the gradients of chunks that each take the one-codeword-per-workgroup
    path."""
    import gnndecode as gd
    H = gd.codes.toric_code(5)
    torch.manual_seed(3)
    m = gd.MODELS['v24'](4, H).to(DEV).to(dtype).train()
    m.fused_train = True
    lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H)).to(DEV)
    x, y = gd.data.toric_batch(H, 2500, seed=11, device=DEV, dtype=dtype)
    V, N = H.shape[0], H.shape[0] + H.shape[1]

    def grads(xs, ys):
        m.zero_grad()
        loss = lf(m(gd.data.make_batch(xs, m.graph(xs.device))), ys)
        loss.backward()
        return loss.item(), torch.cat([p.grad.reshape(-1) for p in m.parameters()]).double()

    lf_full, g_full = grads(x, y)
    lsum, gsum = 0.0, torch.zeros_like(g_full)
    for b0, b1 in ((0, 1000), (1000, 2000), (2000, 2500)):
        l, gc = grads(x[b0 * N:b1 * N], y[b0 * V:b1 * V])
        lsum += l
        gsum += gc
    tol = 1e-10 if dtype == torch.float64 else 2e-4
    assert abs(lf_full - lsum) <= tol * abs(lsum)
    assert (g_full - gsum).abs().max().item() <= tol * gsum.abs().max().item()


@pytest.mark.parametrize('kind', ['graph-trainer', 'fused-trainer-eager', 'fused-trainer-graph'])
def test_eval_after_device_side_training_uses_current_weights(kind):
    """Optimizer steps that run on the device (HIP-graph replay, gnnd_adam_step) do not bump
    parameter versions; the eval decode must still use the updated weights."""
    import gnndecode as gd
    H = gd.codes.toric_code(4)
    torch.manual_seed(5)
    m = gd.MODELS['v24'](3, H).to(DEV).float()
    lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H)).to(DEV)
    x, y = gd.data.toric_batch(H, 32, seed=2, device=DEV, dtype=torch.float32)
    data = gd.data.make_batch(x, m.graph(x.device))
    m.eval()
    with torch.no_grad():
        m(data)                                   # fill the prepared-weight cache
    if kind == 'graph-trainer':
        tr = gd.train.Trainer(m, lf, lr=1e-2, graph=True, warmup=1)
    else:
        m.fused_train = True
        tr = gd.train.FusedV24Trainer(m, lf, lr=1e-2, graph=(kind == 'fused-trainer-graph'), warmup=1)
    for _ in range(4):
        tr.step(data, y)
    torch.cuda.synchronize()
    m.eval()
    with torch.no_grad():
        got = m(data)
        fresh = gd.MODELS['v24'](3, H).to(DEV).float().eval()
        fresh.load_state_dict({k: v.clone() for k, v in m.state_dict().items()})
        ref = fresh(data)
    assert torch.equal(got, ref)


@pytest.mark.parametrize('fused', [True, False], ids=['fused-trainer', 'torch-trainer'])
def test_graphed_step_with_rccl_collective_one_rank(fused):
    """The multi-GPU step shape on the one-GPU box: a 1-rank RCCL ("nccl") process group with
    force_collective=True runs the split capture (compute graph -> eager RCCL all_reduce ->
    Adam graph).  A 1-rank SUM is the identity, so losses and parameters equal the
    single-graph step bit for bit."""
    import socket
    import torch.distributed as dist
    import gnndecode as gd
    sock = socket.socket()
    sock.bind(('127.0.0.1', 0))
    port = sock.getsockname()[1]
    sock.close()
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1,
                            device_id=torch.device(DEV, torch.cuda.current_device()))
    try:
        H = gd.codes.toric_code(5)
        lg = gd.codes.toric_logicals(H)
        torch.manual_seed(11)
        a = gd.MODELS['v24'](5, H).to(DEV)
        b = gd.MODELS['v24'](5, H).to(DEV)
        b.load_state_dict(a.state_dict())
        if fused:
            ta = gd.train.FusedV24Trainer(a, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=True, warmup=1)
            tb = gd.train.FusedV24Trainer(b, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=True, warmup=1,
                                          force_collective=True)
        else:
            ta = gd.train.Trainer(a, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=True, warmup=1)
            tb = gd.train.Trainer(b, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=True, warmup=1,
                                  force_collective=True)
        x, y = gd.data.toric_batch(H, 48, seed=3, device=DEV)
        for s in range(4):
            la = ta.step(gd.data.make_batch(x, a.graph(x.device)), y)
            lb = tb.step(gd.data.make_batch(x, b.graph(x.device)), y)
            assert la.item() == lb.item()
        assert tb._g_apply is not None and ta._g_apply is None
        for k, v in a.state_dict().items():
            assert torch.equal(b.state_dict()[k], v), k
    finally:
        dist.destroy_process_group()


def _v24_checkpoint_model(H, T, dtype):
    """decoder_v2_4 at the reference's training start: its own checkpoint (the shipped
    epoch-67 weights, L-independent shapes, converted to weights/v24_toric_5.npz), as
    quantum/decoder_v2_4.py:322 loads one before its Adam loop."""
    import os
    import gnndecode as gd
    z = np.load(os.path.join(os.path.dirname(gd.__file__), 'weights', 'v24_toric_5.npz'))
    m = gd.MODELS['v24'](T, H)
    m.load_state_dict({k: torch.from_numpy(z[k]) for k in z.files})
    return m.to(DEV).to(dtype).train(), {k: z[k].astype(np.float64) for k in z.files}


def test_config5_trajectory_matches_oracle_L7_B128_f64():
    """Config 5 at the reference's precision and size: 10 fused training steps (forward + tape,
    reverse pass with the fused syndrome loss, fused Adam epilogue) on toric L=7, B=128, fp64,
    from the reference checkpoint, against the oracle's restatement of the reference training
    step (oracle/torch_train.py V24Step: forward, LossFunc, autograd backward, torch Adam lr
    3e-4 wd 1e-9) on the same codewords.  The loss must move (non-integer, changing) and every
    step's loss must agree to 1e-9 relative, the parameters after 10 steps to 1e-10."""
    import gnndecode as gd
    import torch_train
    H = gd.codes.toric_code(7)
    lg = gd.codes.toric_logicals(H)
    T, B, K = 15, 128, 10
    m, w = _v24_checkpoint_model(H, T, torch.float64)
    x, y = gd.data.toric_batch(H, B, seed=2024, device=DEV, dtype=torch.float64)
    tr = gd.train.FusedV24Trainer(m, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=False)
    data = gd.data.make_batch(x, m.graph(x.device))
    got = [float(tr.step(data, y)) for _ in range(K)]
    st = torch_train.V24Step(H, lg, w, T)
    N, V = H.shape[0] + H.shape[1], H.shape[0]
    xs, ys = x.view(-1, N).cpu().reshape(-1, 1), y.view(-1, V).cpu()
    ref = [st.step(xs, ys) for _ in range(K)]
    assert len(set(ref)) == K and all(r != round(r) for r in ref), ref     # the loss moves
    for s, (a, b) in enumerate(zip(got, ref)):
        assert abs(a - b) <= 1e-9 * abs(b), (s, a, b)
    sd = m.state_dict()
    for k, p in st.p.items():
        d = float((sd[k].detach().cpu() - p.detach()).abs().max())
        assert d <= 1e-10, (k, d)


def test_fused_v24_trainer_sees_weights_loaded_after_construction():
    """load_state_dict (or any in-place parameter edit) after FusedV24Trainer was built: the next
    step must run on the loaded weights.  The parameters are views of the trainer's flat buffer
    that keep their own version counters, so the trainer tracks those."""
    import gnndecode as gd
    H = gd.codes.toric_code(5)
    lg = gd.codes.toric_logicals(H)
    torch.manual_seed(21)
    a = gd.MODELS['v24'](5, H).to(DEV)
    other = gd.MODELS['v24'](5, H).to(DEV)            # different (seeded) weights
    ta = gd.train.FusedV24Trainer(a, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=False)
    a.load_state_dict(other.state_dict())
    b = gd.MODELS['v24'](5, H).to(DEV)
    b.load_state_dict(other.state_dict())
    tb = gd.train.FusedV24Trainer(b, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=False)
    x, y = gd.data.toric_batch(H, 32, seed=9, device=DEV)
    for _ in range(2):
        la = float(ta.step(gd.data.make_batch(x, a.graph(x.device)), y))
        lb = float(tb.step(gd.data.make_batch(x, b.graph(x.device)), y))
        assert la == lb, (la, lb)
    for k, v in b.state_dict().items():
        assert torch.equal(a.state_dict()[k], v), k
