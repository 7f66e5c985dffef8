"""Data-parallel training of the reference decoders.

One process per GPU (`torch.distributed`, backend "nccl" = RCCL on ROCm).  Every rank draws
its own shard of the global batch, runs the layer-by-layer decoder (HIP propagate forward and
backward kernels, torch autograd through the MLPs), and the summed loss's gradients are
all-reduced with SUM in ONE flat bucket (decoder_v2_4 has 1 283 parameters, ~10 KB in
fp64: latency-bound, a single RCCL call per step).  SUM, not mean: the reference loss is a
sum over the batch (quantum/decoder_v2_4.py:314-317), so the all-reduced gradient equals the
single-process full-batch gradient.  Then every rank applies the same Adam step
(quantum/decoder_v2_4.py:323: lr 3e-4, weight_decay 1e-9), so parameters stay bitwise equal.
"""
import torch
import torch.distributed as dist


def shard_bounds(global_batch, rank, world):
    """Contiguous codeword shard [start, end) of rank r (sizes differ by at most one)."""
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def flat_grads(params):
    return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                      for p in params])


def allreduce_grads(params, group=None):
    """all_reduce(SUM) of every parameter gradient as one contiguous bucket."""
    params = [p for p in params if p.requires_grad]
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    flat = flat_grads(params)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    off = 0
    for p in params:
        n = p.numel()
        if p.grad is None:
            p.grad = torch.zeros_like(p)
        p.grad.copy_(flat[off:off + n].view_as(p))
        off += n


class Trainer:
    """zero_grad -> forward -> summed loss -> backward -> all_reduce(SUM) -> Adam."""

    def __init__(self, model, loss_fn, lr=3e-4, weight_decay=1e-9, group=None):
        self.model = model
        self.loss_fn = loss_fn
        self.group = group
        self.opt = torch.optim.Adam(model.parameters(), lr, weight_decay=weight_decay)

    def step(self, data, y):
        self.model.train()
        self.opt.zero_grad(set_to_none=False)
        pred = self.model(data)
        loss = self.loss_fn(pred, y)
        loss.backward()
        allreduce_grads(self.model.parameters(), self.group)
        self.opt.step()
        total = loss.detach().clone()
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1:
            dist.all_reduce(total, op=dist.ReduceOp.SUM, group=self.group)
        return total
