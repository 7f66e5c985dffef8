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

from . import ops


def _invalidate(model):
    """Drop the model's cached prepared weights after an optimizer step that ran on the
    device (graph replay, fused Adam): parameter versions do not see those updates."""
    fn = getattr(model, 'invalidate_weight_cache', None)
    if fn is not None:
        fn()


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
    """zero_grad -> forward -> summed loss -> backward -> all_reduce(SUM) -> Adam.

    `graph=True` captures that whole step (the layer-by-layer decoder launches ~900 small
    kernels per step for T = 15) in one HIP graph after a few eager warm-up steps and
    replays it; inputs are copied into static buffers first.  Same arithmetic, same order.
    Requires a fixed batch shape and edge_index; Adam runs in its capturable form."""

    def __init__(self, model, loss_fn, lr=3e-4, weight_decay=1e-9, group=None, graph=False,
                 warmup=3, capturable=None):
        self.model = model
        self.loss_fn = loss_fn
        self.group = group
        self.use_graph = graph
        self.warmup = warmup
        # capturable Adam (device-side step count) is required under capture; its update
        # rounds differently from the host-step form, so pass capturable=True to compare an
        # eager run against a graphed one bit for bit
        self.opt = torch.optim.Adam(model.parameters(), lr, weight_decay=weight_decay,
                                    capturable=graph if capturable is None else capturable)
        self._graph = None
        self._eager_steps = 0

    def _dist(self):
        return dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1

    def _body(self, data, y):
        self.opt.zero_grad(set_to_none=False)
        pred = self.model(data)
        loss = self.loss_fn(pred, y)
        loss.backward()
        allreduce_grads(self.model.parameters(), self.group)
        self.opt.step()
        total = loss.detach().clone()
        if self._dist():
            dist.all_reduce(total, op=dist.ReduceOp.SUM, group=self.group)
        return total

    def step(self, data, y):
        out = self._step(data, y)
        _invalidate(self.model)
        return out

    def _step(self, data, y):
        self.model.train()
        if not self.use_graph:
            return self._body(data, y)
        if self._graph is None:
            if self._eager_steps < self.warmup:
                # eager warm-up on a side stream (allocator pools, cached graph checks)
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    out = self._body(data, y)
                torch.cuda.current_stream().wait_stream(s)
                self._eager_steps += 1
                return out
            self._sx = data.x.clone()
            self._sy = y.clone()
            self._sdata = _StaticBatch(self._sx, data.edge_index)
            self._graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._graph):
                self._sloss = self._body(self._sdata, self._sy)
        self._sx.copy_(data.x)
        self._sy.copy_(y)
        self._graph.replay()
        return self._sloss


class _StaticBatch:
    def __init__(self, x, edge_index):
        self.x = x
        self.edge_index = edge_index


class FusedV24Trainer:
    """decoder_v2_4 training step (quantum/decoder_v2_4.py:320-348) as a handful of HIP
    launches, the whole step captured in one HIP graph:

        prepare weights -> forward with tape (gnnd_train_fwd) -> syndrome loss and
        d loss / d out (gnnd_syndrome_loss) -> reverse pass to the flat gradient
        (gnnd_train_bwd) -> [one RCCL all_reduce(SUM) of that gradient] -> Adam on the
        flat parameter buffer (gnnd_adam_step)

    The model's parameters are re-bound as VIEWS of one flat buffer in the gnnd.h packed
    layout, so nothing is packed, split, zeroed or accumulated per parameter (the torch
    path, `Trainer`, spends ~80 small kernels per step on that, the loss graph and Adam).
    state_dict / load_state_dict keep working on the views.  Same update as `Trainer`
    (torch.optim.Adam's order; lr 3e-4, weight decay 1e-9 of the reference)."""

    def __init__(self, model, loss_fn, lr=3e-4, weight_decay=1e-9, betas=(0.9, 0.999), eps=1e-8,
                 group=None, graph=True, warmup=2):
        from .models import DecoderV24
        if not isinstance(model, DecoderV24):
            raise TypeError('FusedV24Trainer trains decoder_v2_4 (DecoderV24) models')
        self.model, self.loss_fn, self.group = model, loss_fn, group
        self.lr, self.wd, self.betas, self.eps = lr, weight_decay, betas, eps
        self.use_graph, self.warmup = graph, warmup
        flat = model.packed_weights().detach().clone().contiguous()
        off = 0
        for seq, split in ((model.ggc1.mlp, True), (model.ggc2.mlp, False), (model.mlp, False)):
            W1, b1, W2, b2 = seq[0].weight, seq[0].bias, seq[2].weight, seq[2].bias
            hidden, fan_in = W1.shape
            n = hidden * fan_in
            W1.data = (flat[off:off + n].view(fan_in, hidden).t() if split
                       else flat[off:off + n].view(hidden, fan_in))
            off += n
            b1.data = flat[off:off + hidden]
            off += hidden
            W2.data = flat[off:off + hidden].view(1, hidden)
            off += hidden
            b2.data = flat[off:off + 1]
            off += 1
        assert off == flat.numel()
        self.flat = flat
        self.exp_avg = torch.zeros_like(flat)
        self.exp_avg_sq = torch.zeros_like(flat)
        self.step_count = torch.zeros(1, dtype=torch.float64, device=flat.device)
        self._graph = None
        self._eager_steps = 0

    def _dist(self):
        return dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1

    def _body(self, x, y):
        m = self.model
        g = m.graph(x.device)
        w = self.flat if self.flat.dtype == x.dtype else self.flat.to(x.dtype)
        out, tape = ops.train_forward(g, m.kind, x, ops.prepare_weights(m.kind, w), m.Nc)
        lf = self.loss_fn
        loss_b, dpred = ops.syndrome_loss(lf._graph(x.device), lf.logical_rows, lf.logical_only,
                                          out, y)
        gw = ops.train_backward(g, m.kind, w, x, out, dpred, tape, m.Nc).to(self.flat.dtype)
        total = loss_b.sum()
        if self._dist():
            dist.all_reduce(gw, op=dist.ReduceOp.SUM, group=self.group)
            dist.all_reduce(total, op=dist.ReduceOp.SUM, group=self.group)
        ops.adam_step(self.flat, gw, self.exp_avg, self.exp_avg_sq, self.step_count, self.lr,
                      self.betas, self.eps, self.wd)
        return total

    def step(self, data, y):
        out = self._step(data, y)
        _invalidate(self.model)      # parameters changed on the device (gnnd_adam_step)
        return out

    def _step(self, data, y):
        self.model.train()
        x = data.x if data.x.dim() == 2 else data.x.unsqueeze(1)
        if not self.use_graph:
            return self._body(x, y)
        if self._graph is None:
            if self._eager_steps < self.warmup:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    out = self._body(x, y)
                torch.cuda.current_stream().wait_stream(s)
                self._eager_steps += 1
                return out
            self._sx, self._sy = x.clone(), y.clone()
            self._graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._graph):
                self._sloss = self._body(self._sx, self._sy)
        self._sx.copy_(x)
        self._sy.copy_(y)
        self._graph.replay()
        return self._sloss
