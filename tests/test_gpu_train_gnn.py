"""Fused training of the 10-hidden-unit GNN decoders (gnnd_train_gnn.hip, FusedGnnTrainer):
CGNNI (classical/CGNNI.py:314-338, fp32) and QGNNI (quantum/QGNNI.py:294-320, fp64).  The
forward with tape + reverse pass give the reference's own autograd gradients (goldens generated
by exec'ing the reference classes, tests/golden/make_golden.py), and the trainer follows the
torch-optimizer Trainer on the layer-by-layer operator path."""
import numpy as np
import pytest
import torch

from conftest import weights_of

pytestmark = pytest.mark.gpu
DEV = 'cuda'

CASES = [('train_cgnni_bch', 'cgnni', ('bch', None)), ('train_qgnni_L4', 'qgnni', ('toric', 4))]


def _setup(golden, fx, model, code, f64=False):
    """f64: CGNNI in double as well (its fp32 reference dtype aside), so two implementations'
    trajectories can be compared without fp32 rounding noise in Adam's first steps."""
    import gnndecode as gd
    z = golden(fx)
    H = gd.codes.toric_code(code[1]) if code[0] == 'toric' else gd.codes.bch_63_45()
    m = gd.MODELS[model](int(z['T']), H)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()})
    m = m.to(DEV).train()
    if model == 'cgnni':
        lf = gd.loss.ClassicalLoss(H).to(DEV)
    else:
        lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H), logical_only=True).to(DEV)
    x = torch.from_numpy(z['x']).to(DEV)
    y = torch.from_numpy(z['y']).to(DEV)
    if f64:
        m, x, y = m.double(), x.double(), y.double()
    return z, m, lf, H, x, y


def _golden_flat(z, model):
    msg = 'ggc2.mlp2' if model == 'cgnni' else 'ggc2.mlp'
    parts = []
    for pre in (msg, 'mlp'):
        for k in ('0.weight', '0.bias', '2.weight', '2.bias'):
            parts.append(np.asarray(z[f'g/{pre}.{k}'], np.float64).reshape(-1))
    return np.concatenate(parts)


@pytest.mark.parametrize('fx,model,code', CASES, ids=[c[0] for c in CASES])
def test_fused_gnn_gradients_match_reference(golden, fx, model, code):
    """gnnd_train_fwd + the reference LossFunc + gnnd_train_bwd == the reference autograd
    gradients (fp64 QGNNI to 1e-8 of the largest; fp32 CGNNI to 2e-3, the fp32 tolerance of
    tests/test_gpu_training.py)."""
    import gnndecode as gd
    z, m, lf, H, x, y = _setup(golden, fx, model, code)
    g = m.graph(x.device)
    w = m.packed_weights().detach().to(x.dtype).contiguous()
    out, tape = gd.ops.train_forward(g, model, x, w, m.Nc)
    f64 = x.dtype == torch.float64
    np.testing.assert_allclose(out.cpu().numpy(), z['pred'], rtol=1e-10 if f64 else 1e-4,
                               atol=1e-12 if f64 else 2e-5)
    tr = gd.train.FusedGnnTrainer(m, lf, graph=False)
    loss_b, d = tr._loss_grad(out, y)
    assert abs(float(loss_b.sum()) - float(z['loss'])) <= (1e-9 if f64 else 1e-4) * max(1.0, abs(float(z['loss'])))
    gw = gd.ops.train_backward(g, model, w, x, out, d, tape, m.Nc).double().cpu().numpy()
    ref = _golden_flat(z, model)
    tol = 1e-8 if f64 else 2e-3
    assert np.abs(gw - ref).max() <= tol * np.abs(ref).max(), (np.abs(gw - ref).max(), np.abs(ref).max())


@pytest.mark.parametrize('fx,model,code', CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize('graph', [False, True], ids=['eager', 'graph'])
def test_fused_gnn_trainer_follows_torch_trainer(golden, fx, model, code, graph):
    """FusedGnnTrainer (flat parameter views, HIP forward/reverse pass, fused Adam epilogue)
    follows the torch-optimizer Trainer on the layer-by-layer propagate path over 4 steps
    (fp64 for both models: CGNNI's kernels are dtype templates)."""
    import gnndecode as gd
    z, a, lf, H, x, y = _setup(golden, fx, model, code, f64=True)
    _, b, lf2, _, _, _ = _setup(golden, fx, model, code, f64=True)
    if model == 'cgnni':
        loss_a = lambda p, yy: lf(p, yy, train=True)
    else:
        loss_a = lf
    ta = gd.train.Trainer(a, loss_a, graph=False)
    tb = gd.train.FusedGnnTrainer(b, lf2, graph=graph, warmup=1)
    f64 = x.dtype == torch.float64
    for s in range(4):
        la = float(ta.step(gd.data.make_batch(x, a.graph(x.device)), y))
        lb = float(tb.step(gd.data.make_batch(x, b.graph(x.device)), y))
        assert abs(la - lb) <= (1e-9 if f64 else 1e-4) * max(1.0, abs(la)), (s, la, lb)
    for k, v in a.state_dict().items():
        torch.testing.assert_close(b.state_dict()[k], v, rtol=1e-9 if f64 else 1e-4,
                                   atol=1e-12 if f64 else 1e-6, msg=k)


def test_fused_qgnni_large_batch_equals_sum_of_chunks():
    """B > 1024: the reverse pass loops each workgroup over a strided set of codewords (one
    gradient row per workgroup); the logical |sin| loss is a sum, so the full-batch gradient
    equals the sum of its chunks' (fp64)."""
    import gnndecode as gd
    H = gd.codes.toric_code(4)
    torch.manual_seed(7)
    m = gd.MODELS['qgnni'](6, H).to(DEV).train()
    lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H), logical_only=True).to(DEV)
    x, y = gd.data.toric_batch(H, 2300, seed=4, device=DEV)
    g = m.graph(x.device)
    w = m.packed_weights().detach().contiguous()
    N, V = g.N, g.V

    def grads(xs, ys):
        out, tape = gd.ops.train_forward(g, 'qgnni', xs, w, m.Nc)
        lb, d = lf.per_codeword(out, ys)
        return float(lb.sum()), gd.ops.train_backward(g, 'qgnni', w, xs, out, d, tape, m.Nc)

    lfull, gfull = grads(x, y)
    lsum, gsum = 0.0, torch.zeros_like(gfull)
    for b0, b1 in ((0, 1000), (1000, 2000), (2000, 2300)):
        l, gc = grads(x[b0 * N:b1 * N].contiguous(), y[b0 * V:b1 * V].contiguous())
        lsum += l
        gsum += gc
    assert abs(lfull - lsum) <= 1e-10 * abs(lsum)
    assert (gfull - gsum).abs().max().item() <= 1e-10 * gsum.abs().max().item()


def _dp_worker(rank, world, port, q, model, odd=False):
    import os
    import torch.distributed as dist
    import gnndecode as gd
    from conftest import GOLDEN
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    fx = 'train_cgnni_bch' if model == 'cgnni' else 'train_qgnni_L4'
    z = np.load(os.path.join(GOLDEN, fx + '.npz'))
    H = gd.codes.bch_63_45() if model == 'cgnni' else gd.codes.toric_code(4)
    m = gd.MODELS[model](int(z['T']), H)
    m.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()})
    m = m.to(DEV).double().train()
    lf = (gd.loss.ClassicalLoss(H) if model == 'cgnni' else
          gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H), logical_only=True)).to(DEV)
    N, V = H.shape[0] + H.shape[1], H.shape[0]
    x = torch.from_numpy(z['x']).to(DEV).double().view(-1, N)
    y = torch.from_numpy(z['y']).to(DEV).double().view(-1, V)
    if odd:                                  # an odd global batch: unequal shards
        n = x.size(0) - 1 if x.size(0) % 2 == 0 else x.size(0)
        x, y = x[:n], y[:n]
    s, e = gd.train.shard_bounds(x.size(0), rank, world)
    xs, ys = x[s:e].reshape(-1, 1).contiguous(), y[s:e].reshape(-1, 1).contiguous()
    tr = gd.train.FusedGnnTrainer(m, lf, graph=False)
    losses = [float(tr.step(gd.data.make_batch(xs, m.graph(xs.device)), ys)) for _ in range(2)]
    q.put((rank, losses, tr.flat.double().cpu().tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('model,odd', [('qgnni', False), ('cgnni', False), ('cgnni', True)])
def test_two_rank_fused_gnn_training_equals_full_batch(golden, model, odd):
    """Data-parallel FusedGnnTrainer: 2 gloo ranks on the one GPU, each half of the batch, one
    all_reduce of [gradient | loss] per step (SUM for QGNNI's summed loss; for CGNNI's mean loss
    each rank's mean weighted by its shard size, so an odd global batch -- unequal shards --
    still gives the full-batch mean) -> the single-process full-batch parameters and losses
    (fp64)."""
    import socket
    import torch.multiprocessing as mp
    import gnndecode as gd
    sock = socket.socket()
    sock.bind(('127.0.0.1', 0))
    port = sock.getsockname()[1]
    sock.close()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q, model, odd)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    fx = 'train_cgnni_bch' if model == 'cgnni' else 'train_qgnni_L4'
    z, m, lf, H, x, y = _setup(golden, fx, model, ('bch', None) if model == 'cgnni' else ('toric', 4), f64=True)
    if odd:
        N, V = H.shape[0] + H.shape[1], H.shape[0]
        n = x.numel() // N
        n = n - 1 if n % 2 == 0 else n
        x, y = x[:n * N].contiguous(), y[:n * V].contiguous()
    tr = gd.train.FusedGnnTrainer(m, lf, graph=False)
    ref_losses = [float(tr.step(gd.data.make_batch(x, m.graph(x.device)), y)) for _ in range(2)]
    ref = tr.flat.double().cpu()
    for rank, losses, flat in res:
        flat = torch.tensor(flat, dtype=torch.float64)
        assert flat.tolist() == res[0][2]                 # ranks bitwise equal
        assert torch.allclose(flat, ref, rtol=1e-10, atol=1e-12), float((flat - ref).abs().max())
        assert all(abs(a - b) <= 1e-9 * max(1, abs(b)) for a, b in zip(losses, ref_losses))
