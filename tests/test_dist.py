"""Multi-process data-parallel logic on CPU (gloo, world_size 2): shard bounds, the single
flat SUM all-reduce, and that 2-rank training equals 1-process full-batch training."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gnndecode import train


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_bounds_cover_exactly():
    for B in (0, 1, 7, 64, 65536, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [train.shard_bounds(B, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1


class _Toy(torch.nn.Module):
    """Stand-in decoder with the reference's parameter structure (two MLPs, fp64)."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.mlp = torch.nn.Sequential(torch.nn.Linear(2, 16), torch.nn.Softplus(),
                                       torch.nn.Linear(16, 1)).double()

    def forward(self, x):
        return torch.sigmoid(-self.mlp(x))


def _sum_loss(pred, y):
    return torch.abs(torch.sin((pred + y) * 3.14159 / 2)).sum()


def _data(B, seed=1):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(B, 2, generator=g, dtype=torch.float64), \
        (torch.rand(B, 1, generator=g) < 0.3).double()


def _worker(rank, world, port, B, steps, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    model = _Toy()
    tr = train.Trainer(model, _sum_loss, lr=1e-2)
    x, y = _data(B)
    s, e = train.shard_bounds(B, rank, world)
    losses = [float(tr.step(x[s:e], y[s:e])) for _ in range(steps)]
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    # plain list, not a tensor: a tensor goes through fd sharing, which races the
    # worker's exit
    q.put((rank, losses, flat.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_training_equals_full_batch():
    B, steps, world = 10, 3, 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process, full batch
    model = _Toy()
    tr = train.Trainer(model, _sum_loss, lr=1e-2)
    x, y = _data(B)
    ref_losses = [float(tr.step(x, y)) for _ in range(steps)]
    ref_flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    for rank, losses, flat in res:
        flat = torch.tensor(flat, dtype=torch.float64)
        assert flat.tolist() == res[0][2]     # ranks bitwise equal
        assert torch.allclose(flat, ref_flat, rtol=1e-12, atol=1e-13)
        assert all(abs(a - b) <= 1e-10 * max(1, abs(b)) for a, b in zip(losses, ref_losses))


def _local_worker(rank, world, port, B, steps, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    if rank == 0:
        # a check rank 0 runs on its own inside the 2-rank job (bench.py's trajectory parity):
        # group=LOCAL, so its steps issue no collective (the other rank is not in them)
        model = _Toy()
        tr = train.Trainer(model, _sum_loss, lr=1e-2, group=train.LOCAL)
        x, y = _data(B)
        losses = [float(tr.step(x, y)) for _ in range(steps)]
        q.put((rank, losses))
    dist.barrier()
    dist.destroy_process_group()


def test_local_trainer_in_a_multi_rank_job_issues_no_collective():
    B, steps, world = 10, 3, 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_local_worker, args=(r, world, port, B, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    rank, losses = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    model = _Toy()
    tr = train.Trainer(model, _sum_loss, lr=1e-2)
    x, y = _data(B)
    assert losses == [float(tr.step(x, y)) for _ in range(steps)]
    assert not train._collective(train.LOCAL, True)


def _reduce_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    # FusedGnnTrainer's CGNNI reduce on its own (no device kernels): [gradient | loss | count]
    tr = train.FusedGnnTrainer.__new__(train.FusedGnnTrainer)
    tr.model = type('M', (), {'kind': 'cgnni'})()
    tr.group = None
    n = 4
    tr._gbuf = torch.zeros(n + 2, dtype=torch.float64)
    tr._gl, tr._count = tr._gbuf[:n + 1], tr._gbuf[n + 1]
    sizes = [1, 1, 0]                   # global batch 2 over 3 ranks: rank 2's shard is empty
    assert [e - s for s, e in (train.shard_bounds(2, r, world) for r in range(world))] == sizes
    tr._nb = sizes[rank]
    if tr._nb:
        tr._gl.copy_(torch.arange(n + 1, dtype=torch.float64) * (rank + 1))
    else:
        tr._gl.fill_(float('nan'))      # the mean over zero codewords
    tr._reduce(None, None)
    q.put((rank, tr._gl.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_cgnni_reduce_with_an_empty_shard_gloo3():
    """global batch < world leaves a rank with no codewords; its NaN mean must not
    reach the summed gradient (3 gloo ranks, global batch 2)."""
    world = 3
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reduce_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = [(1.0 * i + 2.0 * i) / 2 for i in range(5)]     # the full-batch mean of ranks 0, 1
    for _, gl in res:
        assert gl == want
