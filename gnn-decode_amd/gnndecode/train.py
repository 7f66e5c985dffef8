"""Data-parallel training of the reference decoders.

One process per GPU (`torch.distributed`, backend "nccl" = RCCL on ROCm).  Every rank draws
its own shard of the global batch, runs the decoder forward and reverse pass on the HIP
kernels, and the summed loss's gradients are all-reduced with SUM in ONE flat bucket
(decoder_v2_4 has 1 283 parameters, ~10 KB in fp64: latency-bound, a single RCCL call per
step).  SUM, not mean: the reference loss is a sum over the batch
(quantum/decoder_v2_4.py:314-317), so the all-reduced gradient equals the single-process
full-batch gradient.  Then every rank applies the same Adam step, so parameters stay
bitwise equal.

HIP graphs and collectives.  A step is captured in HIP graphs for launch-bound batches, but
the RCCL all-reduce is NOT captured: with a collective in play (world size > 1, or
`force_collective`) the step is split into a compute graph (forward, loss, reverse pass ->
flat gradient) and an optimizer graph (Adam), and the all-reduce of the flat gradient runs
eagerly on the same stream between the two replays.  Single-rank runs keep one graph.

Optimizer settings per model follow the reference scripts (`REFERENCE_OPTIM`).
"""
import os

import torch
import torch.distributed as dist

from . import ops

# (lr, weight_decay) of torch.optim.Adam in each reference training script
REFERENCE_OPTIM = {
    'v24': (3e-4, 1e-9),      # quantum/decoder_v2_4.py:193, 323
    'qgnni': (3e-4, 5e-4),    # quantum/QGNNI.py:161, 294
    'nbp': (3e-4, 0.0),       # quantum/neural_BP.py:177, 378
    'v10': (3e-4, 0.0),       # quantum/decoder_v1_0.py:177, 377
    'v30': (3e-4, 5e-4),      # quantum/decoder_v3_0.py:173, 341
    'v22': (2e-4, 0.0),       # quantum/decoder_v2_2.py:207, 408
    'cgnni': (3e-4, 5e-4),    # classical/CGNNI.py:204, 314
}


def reference_optim(model):
    """(lr, weight_decay) of the reference script that trains `model` (a decoder or kind)."""
    kind = model if isinstance(model, str) else getattr(model, 'kind', None)
    if kind not in REFERENCE_OPTIM:
        raise ValueError(f'no reference optimizer settings for model {kind!r}')
    return REFERENCE_OPTIM[kind]


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


# group=LOCAL: a trainer of this process alone, never issuing a collective even inside an
# initialised N-rank job (e.g. a check one rank runs on its own: bench.py's trajectory parity)
LOCAL = 'local'


def _collective(group, force):
    if group is LOCAL or group == LOCAL:
        return False
    if not dist.is_available() or not dist.is_initialized():
        return False
    return force or dist.get_world_size(group) > 1


def allreduce_grads(params, group=None, force=False):
    """all_reduce(SUM) of every parameter gradient as one contiguous bucket."""
    params = [p for p in params if p.requires_grad]
    if not _collective(group, force):
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


class _GraphedStep:
    """Shared capture logic: `warmup` eager steps on a side stream, then HIP graphs.

    Subclasses provide `_compute(x, y) -> (loss_tensor, [grad tensors])` (no collective)
    and `_apply()` (the optimizer update from the gradients).  Without a collective both
    run in ONE captured graph; with one, `_compute` and `_apply` are two graphs and the
    all-reduce of the gradients (and of the loss) is issued eagerly in between."""

    def _init_graph(self, graph, warmup, group, force_collective):
        if graph and warmup < 1:
            raise ValueError('graph=True needs warmup >= 1: the first eager step builds the '
                             'device graph tables and allocator pools that capture reuses')
        self.use_graph, self.warmup, self.group = graph, warmup, group
        self.force_collective = force_collective
        self._g_compute = self._g_apply = None
        self._eager_steps = 0

    def _dist(self):
        return _collective(self.group, self.force_collective)

    def _reduce(self, loss, grads):
        for gr in grads:
            dist.all_reduce(gr, op=dist.ReduceOp.SUM, group=self.group)
        dist.all_reduce(loss, op=dist.ReduceOp.SUM, group=self.group)

    def _eager(self, x, y):
        loss, grads = self._compute(x, y)
        if self._dist():
            self._reduce(loss, grads)
        self._apply()
        return loss

    def static_inputs(self):
        """(x, y) buffers the captured step reads (None before the capture): write the next
        batch into them to skip the per-step input copies."""
        if not self.use_graph or self._g_compute is None:
            return None
        return self._sx, self._sy

    def _run(self, x, y, copy_loss=True):
        if not self.use_graph:
            # (copy_loss=False: the step's loss buffer itself, as for the captured step)
            out = self._eager(x, y).detach()
            return out.clone() if copy_loss else out
        if self._g_compute is None:
            if self._eager_steps < self.warmup:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    out = self._eager(x, y).detach().clone()
                torch.cuda.current_stream().wait_stream(s)
                self._eager_steps += 1
                return out
            self._sx, self._sy = x.clone(), y.clone()
            self._g_compute = torch.cuda.CUDAGraph()
            if self._dist():
                with torch.cuda.graph(self._g_compute):
                    self._sloss, self._sgrads = self._compute(self._sx, self._sy)
                self._g_apply = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self._g_apply):
                    self._apply()
            else:
                with torch.cuda.graph(self._g_compute):
                    self._sloss, self._sgrads = self._compute(self._sx, self._sy)
                    self._apply()
        # inputs already in the graph's static buffers (static_inputs(): a sampler writing
        # there directly) need no copy
        if x.data_ptr() != self._sx.data_ptr():
            self._sx.copy_(x)
        if y.data_ptr() != self._sy.data_ptr():
            self._sy.copy_(y)
        self._g_compute.replay()
        if self._g_apply is not None:
            self._reduce(self._sloss, self._sgrads)      # eager RCCL between the two graphs
            self._g_apply.replay()
        # the static buffer is reused by the next replay: a copy unless the caller reads it
        # before the next step (copy_loss=False skips the one extra copy launch per step)
        return self._sloss.clone() if copy_loss else self._sloss


class Trainer(_GraphedStep):
    """zero_grad -> forward -> summed loss -> backward -> [all_reduce(SUM)] -> Adam, for any
    model (the layer-by-layer decoder on the HIP propagate kernels and their backward
    kernels, torch autograd through the MLPs).

    `graph=True` captures the step (~900 small kernels for T = 15) in HIP graphs after
    `warmup` eager steps (see `_GraphedStep` for where the collective goes).  Requires a
    fixed batch shape and edge_index; Adam runs in its capturable form.  lr and weight decay
    default to the reference script's values for the model (`REFERENCE_OPTIM`)."""

    def __init__(self, model, loss_fn, lr=None, weight_decay=None, group=None, graph=False,
                 warmup=3, capturable=None, force_collective=False):
        self.model = model
        self.loss_fn = loss_fn
        rlr, rwd = reference_optim(model) if getattr(model, 'kind', None) in REFERENCE_OPTIM \
            else (3e-4, 0.0)
        lr = rlr if lr is None else lr
        weight_decay = rwd if weight_decay is None else weight_decay
        self._init_graph(graph, warmup, group, force_collective)
        # capturable Adam (device-side step count) is required under capture; its update
        # rounds differently from the host-step form, so pass capturable=True to compare an
        # eager run against a graphed one bit for bit
        self.opt = torch.optim.Adam(model.parameters(), lr, weight_decay=weight_decay,
                                    capturable=graph if capturable is None else capturable)
        self._edge_index = None

    def _compute(self, x, y):
        self.opt.zero_grad(set_to_none=False)
        # a PyG-style batch (.x, .edge_index) or a plain input tensor
        pred = self.model(x if self._edge_index is None else _StaticBatch(x, self._edge_index))
        # losses that need the decoder input too (V30Loss: the syndrome rows of x)
        loss = (self.loss_fn(pred, y, x) if getattr(self.loss_fn, 'needs_input', False)
                else self.loss_fn(pred, y))
        loss.backward()
        params = [p for p in self.model.parameters() if p.requires_grad]
        grads = []
        if self._dist():
            # one flat bucket; _apply scatters it back into the .grad tensors
            self._flat = flat_grads(params)
            grads = [self._flat]
        return loss.detach().clone(), grads

    def _apply(self):
        if self._dist():
            off = 0
            for p in self.model.parameters():
                if not p.requires_grad:
                    continue
                n = p.numel()
                p.grad.copy_(self._flat[off:off + n].view_as(p))
                off += n
        self.opt.step()

    def step(self, data, y):
        self.model.train()
        ei = getattr(data, 'edge_index', None)
        if not self.use_graph or self._edge_index is None:
            self._edge_index = ei
        elif ei is not None and ei.shape != self._edge_index.shape:
            raise ValueError('graph=True needs a fixed edge_index shape across steps')
        # graph mode keeps the first step's edge_index (checked on the device while eager):
        # a per-batch tensor would need a host-synchronising layout check inside the capture
        x = data.x if hasattr(data, 'x') else data
        out = self._run(x, y)
        _invalidate(self.model)
        return out


class _StaticBatch:
    def __init__(self, x, edge_index):
        self.x = x
        self.edge_index = edge_index


class FusedV24Trainer(_GraphedStep):
    """decoder_v2_4 training step (quantum/decoder_v2_4.py:320-348) as four HIP launches:

        forward with tape (gnnd_train_fwd) -> syndrome loss and d loss / d out
        (gnnd_syndrome_loss) -> reverse pass to per-workgroup gradient rows
        (gnnd_train_bwd_partial; with the syndrome loss of a SyndromeLoss computed inside
        it, gnnd_train_bwd_loss_partial, the loss launch goes too; loss_in_forward=True computes
        it in the unit-split forward's epilogue instead, gnnd_train_fwd_loss, the same bits,
        measured slower) -> fused epilogue
        (gnnd_train_update: fixed-order row
        reduction, the batch loss, Adam, and the kernel-layout weights the next forward reads)

    With a collective in play the epilogue is split around the RCCL all_reduce(SUM) of the
    flat gradient: update(rows -> gradient, loss) -> all_reduce -> update(Adam, weights).
    On a split Tanner graph (the toric code's two disconnected halves, TannerGraph.components)
    the forward and the reverse pass run every component of a codeword in its own workgroup.

    The model's parameters are re-bound as VIEWS of one flat buffer in the gnnd.h packed
    layout, so nothing is packed, split, zeroed or accumulated per parameter (the torch
    path, `Trainer`, spends ~80 small kernels per step on that, the loss graph and Adam).
    state_dict / load_state_dict keep working on the views (an in-place change of a
    parameter re-prepares the kernel-layout weights before the next step).  Same update as
    `Trainer` (torch.optim.Adam's order; lr 3e-4, weight decay 1e-9 of the reference)."""

    def __init__(self, model, loss_fn, lr=None, weight_decay=None, betas=(0.9, 0.999), eps=1e-8,
                 group=None, graph=True, warmup=2, force_collective=False, fuse_loss=True,
                 loss_in_forward=None):
        from .models import DecoderV24
        if not isinstance(model, DecoderV24):
            raise TypeError('FusedV24Trainer trains decoder_v2_4 (DecoderV24) models')
        rlr, rwd = REFERENCE_OPTIM['v24']
        self.model, self.loss_fn = model, loss_fn
        self.lr = rlr if lr is None else lr
        self.wd = rwd if weight_decay is None else weight_decay
        self.betas, self.eps = betas, eps
        self.fuse_loss, self._fuse_ok = fuse_loss, {}
        # default off: measured 2-4 % slower than the reverse pass's own loss at B = 16 / 128
        # (profiles/r03/experiments/train_loss_in_forward_ab_r03ae.txt); GNND_LOSS_IN_FORWARD=1
        # turns it on for A/B runs
        self.loss_in_forward = (os.environ.get('GNND_LOSS_IN_FORWARD', '0') == '1'
                                if loss_in_forward is None else loss_in_forward)
        self._init_graph(graph, warmup, group, force_collective)
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
        self._sync = torch.zeros(1, dtype=torch.int32, device=flat.device)   # gnnd_train_update
        # flat gradient and batch loss side by side: ONE all_reduce(SUM) carries both
        self._gbuf = torch.zeros(flat.numel() + 1, dtype=flat.dtype, device=flat.device)
        self._gw = self._gbuf[:flat.numel()]
        self._loss = self._gbuf[flat.numel()]
        # kernel-layout weights of the current parameters: written by the fused epilogue after
        # every update, re-prepared here when the parameters change outside the trainer
        self.prepared = ops.prepare_weights('v24', flat)
        self._prep_version = self._param_versions()
        # device graph tables now, never inside a capture
        model.graph(flat.device)
        loss_fn._graph(flat.device)

    def _reduce(self, loss, grads):
        # _compute returned views of self._gbuf: one RCCL call for the gradient and the loss
        dist.all_reduce(self._gbuf, op=dist.ReduceOp.SUM, group=self.group)

    def _fused_loss_mask(self, g, device):
        """Logical-row masks for the reverse pass's fused loss, or None (loss kernel path):
        needs a SyndromeLoss with <= 32 logical rows, each inside one graph component."""
        from .loss import SyndromeLoss
        lf = self.loss_fn
        if not self.fuse_loss or not isinstance(lf, SyndromeLoss):
            return None
        key = (g.components, str(device))
        ok = self._fuse_ok.get(key)
        if ok is None:
            ok = self._fuse_ok[key] = (lf.logical_rows.size(0) <= 32 and
                                       lf.rows_within_components(g.components))
        return lf.logical_mask(device) if ok else None

    def _param_versions(self):
        # a parameter re-bound with `p.data = flat[...]` keeps its OWN version counter: an
        # in-place change through it (load_state_dict, p.copy_) bumps that counter, not the
        # flat buffer's, so both are tracked
        return (self.flat._version,) + tuple(p._version for p in self.model.parameters())

    def _refresh_prepared(self):
        v = self._param_versions()
        if v != self._prep_version:
            self.prepared.copy_(ops.prepare_weights('v24', self.flat))
            self._prep_version = v

    def _compute(self, x, y):
        m = self.model
        g = m.graph(x.device)
        lf = self.loss_fn
        if self.flat.dtype != x.dtype:           # mixed precision: the unfused update path
            w = self.flat.to(x.dtype)
            out, tape = ops.train_forward(g, m.kind, x, ops.prepare_weights(m.kind, w), m.Nc)
            loss_b, dpred = lf.per_codeword(out, y)
            self._gw.copy_(ops.train_backward(g, m.kind, w, x, out, dpred, tape, m.Nc))
            self._loss.copy_(loss_b.sum())
            self._pending = None
            return self._loss, [self._gw]
        lmask = self._fused_loss_mask(g, x.device)
        fl = None
        if lmask is not None and self.loss_in_forward:
            # small batches (unit-split forward): the syndrome loss in the forward's epilogue,
            # the reverse pass reads d loss / d out (same bits as the reverse pass's own loss)
            fl = ops.train_forward_loss(g, m.kind, x, self.prepared, m.Nc, y, lmask,
                                        lf.logical_rows.size(0), lf.logical_only)
        if fl is not None:
            out, tape, dpred, loss_b = fl
            ws, nrows = ops.train_backward_partial(g, m.kind, self.flat, x, out, dpred, tape, m.Nc)
        else:
            out, tape = ops.train_forward(g, m.kind, x, self.prepared, m.Nc)
            r = None
            if lmask is not None:
                # the syndrome loss computed inside the reverse pass (no loss launch); None when
                # its tables exceed the workgroup's LDS: remembered, the loss kernel path instead
                r = ops.train_backward_loss_partial(
                    g, m.kind, self.flat, x, out, y, lmask, lf.logical_rows.size(0), lf.logical_only,
                    tape, m.Nc)
                if r is None:
                    self._fuse_ok[(g.components, str(x.device))] = False
            if r is not None:
                ws, nrows, loss_b = r
            else:
                loss_b, dpred = lf.per_codeword(out, y)
                ws, nrows = ops.train_backward_partial(g, m.kind, self.flat, x, out, dpred, tape, m.Nc)
        if self._dist():
            # rows -> flat gradient and batch loss, for the all-reduce
            ops.train_update('v24', x.dtype, rows=ws, n_rows=nrows, grad=self._gw,
                             loss_b=loss_b, loss=self._loss)
            self._pending = None
            return self._loss, [self._gw]
        self._pending = (ws, nrows, loss_b)      # reduced by the fused epilogue in _apply
        return self._loss, []

    def _apply(self):
        kw = dict(param=self.flat, exp_avg=self.exp_avg, exp_avg_sq=self.exp_avg_sq,
                  step=self.step_count, sync=self._sync, lr=self.lr, betas=self.betas,
                  eps=self.eps, weight_decay=self.wd, prepared=self.prepared)
        if self._pending is not None:            # single rank: everything in one launch
            ws, nrows, loss_b = self._pending
            ops.train_update('v24', self.flat.dtype, rows=ws, n_rows=nrows, loss_b=loss_b,
                             loss=self._loss, **kw)
        else:                                    # the (all-reduced) flat gradient
            ops.train_update('v24', self.flat.dtype, grad=self._gw, **kw)

    def step(self, data, y, copy_loss=True):
        """One training step; returns the batch loss (copy_loss=False: the graph's static loss
        buffer itself, valid until the next step)."""
        self.model.train()
        x = data.x if data.x.dim() == 2 else data.x.unsqueeze(1)
        self._refresh_prepared()
        out = self._run(x, y, copy_loss)
        _invalidate(self.model)      # parameters changed on the device (gnnd_train_update)
        return out


class FusedV30Trainer(_GraphedStep):
    """decoder_v3_0 training step (quantum/decoder_v3_0.py:339-356) on the HIP kernels:

        forward with tape (gnnd_train_fwd, model V30: every iteration's edge states before and
        after ggc1) -> the reference LossFunc (loss.V30Loss) and d loss / d [out0, out1] by
        torch autograd on the two readout tensors -> reverse pass to per-workgroup gradient
        rows (gnnd_train_bwd_partial) -> fused epilogue (gnnd_train_update: fixed-order row
        reduction, Adam, the weights the next forward reads)

    all in one HIP graph (with a collective: split around the all_reduce(SUM) of the flat
    gradient, as FusedV24Trainer).  The 137 trained parameters (ggc1.mlp1/rnn1, ggc2.mlp2/
    rnn2, mlp) are re-bound as views of the flat packed buffer; the reference's unused
    ggc1.mlp2/rnn2 and ggc2.mlp1/rnn1 keep their storage and never change (torch's Adam
    skips parameters without a gradient).  Adam as the script: lr 3e-4, weight decay 5e-4."""

    def __init__(self, model, loss_fn, lr=None, weight_decay=None, betas=(0.9, 0.999), eps=1e-8,
                 group=None, graph=True, warmup=2, force_collective=False):
        from .models import DecoderV30
        if not isinstance(model, DecoderV30):
            raise TypeError('FusedV30Trainer trains decoder_v3_0 (DecoderV30) models')
        rlr, rwd = REFERENCE_OPTIM['v30']
        self.model, self.loss_fn = model, loss_fn
        self.lr = rlr if lr is None else lr
        self.wd = rwd if weight_decay is None else weight_decay
        self.betas, self.eps = betas, eps
        self._init_graph(graph, warmup, group, force_collective)
        flat = model.packed_weights().detach().clone().contiguous()
        off = 0

        def bind(p, shape):
            nonlocal off
            n = p.numel()
            p.data = flat[off:off + n].view(shape)
            off += n
        # gnnd.h V30 layout: mlp {W1, b1, W2, b2}, GRU {w_ih, w_hh, b_ih, b_hh}
        mlp = lambda q: (q[0].weight, q[0].bias, q[2].weight, q[2].bias)
        gru = lambda c: (c.weight_ih, c.weight_hh, c.bias_ih, c.bias_hh)
        for group in (mlp(model.ggc1.mlp1), gru(model.ggc1.rnn1), mlp(model.ggc2.mlp2),
                      gru(model.ggc2.rnn2), mlp(model.mlp)):
            for p in group:
                bind(p, p.shape)
        assert off == flat.numel()
        self.flat = flat
        self.exp_avg = torch.zeros_like(flat)
        self.exp_avg_sq = torch.zeros_like(flat)
        self.step_count = torch.zeros(1, dtype=torch.float64, device=flat.device)
        self._sync = torch.zeros(1, dtype=torch.int32, device=flat.device)
        self._loss = torch.zeros((), dtype=flat.dtype, device=flat.device)
        self._gw = torch.zeros_like(flat)
        model.graph(flat.device)                 # device graph tables now, never in a capture

    def _loss_grad(self, out, x, y):
        """The reference LossFunc on [out0, out1] and its gradient w.r.t. both tensors: the
        check term by gnnd_syndrome_loss and the BCE term elementwise (V30Loss.loss_and_grad),
        or torch autograd on the loss where that does not apply."""
        lg = getattr(self.loss_fn, 'loss_and_grad', None)
        res = lg(out, y, x) if lg is not None else None
        if res is not None:
            return res[0].detach(), res[1]
        o = out.detach().requires_grad_(True)
        n = o.size(0) // 2
        with torch.enable_grad():
            loss = self.loss_fn([o[:n], o[n:]], y, x)
            (d,) = torch.autograd.grad(loss, o)
        return loss.detach(), d

    def _compute(self, x, y):
        m = self.model
        g = m.graph(x.device)
        w = self.flat if self.flat.dtype == x.dtype else self.flat.to(x.dtype)
        out, tape = ops.train_forward(g, 'v30', x, w, m.Nc)
        loss, d = self._loss_grad(out, x, y)
        if self.flat.dtype != x.dtype or self._dist():
            gw = ops.train_backward(g, 'v30', w, x, out, d, tape, m.Nc)
            self._gw.copy_(gw.to(self.flat.dtype))
            self._loss.copy_(loss.to(self.flat.dtype))
            self._pending = None
            return self._loss, [self._gw]
        ws, nrows = ops.train_backward_partial(g, 'v30', w, x, out, d, tape, m.Nc)
        self._pending = (ws, nrows, loss.reshape(1))
        return self._loss, []

    def _apply(self):
        kw = dict(param=self.flat, exp_avg=self.exp_avg, exp_avg_sq=self.exp_avg_sq,
                  step=self.step_count, sync=self._sync, lr=self.lr, betas=self.betas,
                  eps=self.eps, weight_decay=self.wd)
        if self._pending is not None:            # single rank: rows -> gradient -> Adam
            ws, nrows, loss1 = self._pending
            ops.train_update('v30', self.flat.dtype, rows=ws, n_rows=nrows, loss_b=loss1,
                             loss=self._loss, **kw)
        else:
            ops.train_update('v30', self.flat.dtype, grad=self._gw, **kw)

    def step(self, data, y, copy_loss=True):
        """One training step; returns the batch loss (copy_loss=False: the graph's static loss
        buffer itself, valid until the next step)."""
        self.model.train()
        x = data.x if data.x.dim() == 2 else data.x.unsqueeze(1)
        out = self._run(x, y, copy_loss)
        _invalidate(self.model)
        return out


class FusedGnnTrainer(_GraphedStep):
    """Training step of the 10-hidden-unit GNN decoders on the HIP kernels:
    CGNNI (classical/CGNNI.py:314-338, fp32) and QGNNI (quantum/QGNNI.py:294-320, fp64):

        forward with tape (gnnd_train_fwd, models CGNNI / QGNNI: every iteration's tanh outputs
        and the readout inputs) -> the reference LossFunc and d loss / d pred (QGNNI: the
        logical |sin| loss on gnnd_syndrome_loss; CGNNI: the script's BCE + syndrome loss by
        torch autograd on the B*V predictions) -> reverse pass to per-workgroup gradient rows
        (gnnd_train_bwd_partial) -> fused epilogue (gnnd_train_update: fixed-order row
        reduction, Adam)

    one HIP graph per step (with a collective: split around the all_reduce(SUM) of the flat
    gradient, as FusedV24Trainer).  The 62 trained parameters (the c->v message MLP: CGNNI
    ggc2.mlp2, QGNNI ggc2.mlp; the readout mlp) are re-bound as views of the flat packed
    buffer (gnnd.h layout); the reference's unused MLPs (ggc1's, CGNNI's ggc2.mlp1 and GRU)
    keep their storage and never change (torch's Adam skips parameters without a gradient).
    Adam as the scripts: lr 3e-4, weight decay 5e-4."""

    def __init__(self, model, loss_fn, lr=None, weight_decay=None, betas=(0.9, 0.999), eps=1e-8,
                 group=None, graph=True, warmup=2, force_collective=False):
        from .models import CGNNI, QGNNI
        if not isinstance(model, (CGNNI, QGNNI)):
            raise TypeError('FusedGnnTrainer trains CGNNI and QGNNI models')
        rlr, rwd = REFERENCE_OPTIM[model.kind]
        self.model, self.loss_fn = model, loss_fn
        self.lr = rlr if lr is None else lr
        self.wd = rwd if weight_decay is None else weight_decay
        self.betas, self.eps = betas, eps
        self._init_graph(graph, warmup, group, force_collective)
        flat = model.packed_weights().detach().clone().contiguous()
        msg = model.ggc2.mlp2 if model.kind == 'cgnni' else model.ggc2.mlp
        off = 0
        for seq in (msg, model.mlp):
            for p in (seq[0].weight, seq[0].bias, seq[2].weight, seq[2].bias):
                n = p.numel()
                p.data = flat[off:off + n].view(p.shape)
                off += n
        assert off == flat.numel() == 62
        self.flat = flat
        self.exp_avg = torch.zeros_like(flat)
        self.exp_avg_sq = torch.zeros_like(flat)
        self.step_count = torch.zeros(1, dtype=torch.float64, device=flat.device)
        self._sync = torch.zeros(1, dtype=torch.int32, device=flat.device)
        # [gradient | loss | codewords of this rank] (the count weights CGNNI's mean, _reduce)
        self._gbuf = torch.zeros(flat.numel() + 2, dtype=flat.dtype, device=flat.device)
        self._gw = self._gbuf[:flat.numel()]
        self._loss = self._gbuf[flat.numel()]
        self._gl = self._gbuf[:flat.numel() + 1]
        self._count = self._gbuf[flat.numel() + 1]
        self._nb = 0
        model.graph(flat.device)                 # device graph tables now, never in a capture
        g = getattr(loss_fn, '_graph', None)
        if g is not None:
            g(flat.device)

    def _reduce(self, loss, grads):
        if self.model.kind == 'cgnni':
            # CGNNI's LossFunc is a MEAN over the batch (classical/CGNNI.py:302-303): each rank's
            # mean gradient and loss weighted by its codeword count, summed, divided by the
            # global count -- the full-batch mean for any shard sizes (shard_bounds of an odd
            # global batch gives unequal shards)
            # (an empty shard -- global batch < world -- has a NaN mean; it contributes nothing,
            # and NaN * 0 would still be NaN: zero it)
            if self._nb == 0:
                self._gl.zero_()
            else:
                self._gl.mul_(float(self._nb))
            self._count.fill_(float(self._nb))
            dist.all_reduce(self._gbuf, op=dist.ReduceOp.SUM, group=self.group)
            self._gl.div_(self._count)
        else:
            dist.all_reduce(self._gbuf, op=dist.ReduceOp.SUM, group=self.group)

    def _loss_grad(self, out, y):
        """(per-codeword (or batch) losses, d loss / d pred)."""
        pc = getattr(self.loss_fn, 'per_codeword', None)
        if pc is not None:                       # SyndromeLoss: one gnnd_syndrome_loss launch
            return pc(out, y)
        o = out.detach().requires_grad_(True)
        with torch.enable_grad():
            loss = self.loss_fn(o, y, train=True) if self.model.kind == 'cgnni' else self.loss_fn(o, y)
            (d,) = torch.autograd.grad(loss, o)
        return loss.detach().reshape(1), d

    def _compute(self, x, y):
        m = self.model
        g = m.graph(x.device)
        w = self.flat if self.flat.dtype == x.dtype else self.flat.to(x.dtype)
        out, tape = ops.train_forward(g, m.kind, x, w, m.Nc)
        self._nb = out.shape[0] // g.V           # codewords of this rank's shard
        loss_b, d = self._loss_grad(out, y)
        if self.flat.dtype != x.dtype or self._dist():
            gw = ops.train_backward(g, m.kind, w, x, out, d, tape, m.Nc)
            self._gw.copy_(gw)
            self._loss.copy_(loss_b.sum())
            self._pending = None
            return self._loss, [self._gw]
        ws, nrows = ops.train_backward_partial(g, m.kind, w, x, out, d, tape, m.Nc)
        self._pending = (ws, nrows, loss_b)
        return self._loss, []

    def _apply(self):
        kw = dict(param=self.flat, exp_avg=self.exp_avg, exp_avg_sq=self.exp_avg_sq,
                  step=self.step_count, sync=self._sync, lr=self.lr, betas=self.betas,
                  eps=self.eps, weight_decay=self.wd)
        if self._pending is not None:            # single rank: rows -> gradient -> Adam
            ws, nrows, loss_b = self._pending
            ops.train_update(self.model.kind, self.flat.dtype, rows=ws, n_rows=nrows, loss_b=loss_b,
                             loss=self._loss, **kw)
        else:
            ops.train_update(self.model.kind, self.flat.dtype, grad=self._gw, **kw)

    def step(self, data, y, copy_loss=True):
        """One training step; returns the batch loss (copy_loss=False: the step's static loss
        buffer itself, valid until the next step)."""
        self.model.train()
        x = data.x if data.x.dim() == 2 else data.x.unsqueeze(1)
        out = self._run(x, y, copy_loss)
        _invalidate(self.model)
        return out


class FusedWbpTrainer(_GraphedStep):
    """Weighted-BP training step on the HIP kernels, fp64 (the scripts' dtype):
    NeuralBP (quantum/neural_BP.py:370-395), decoder_v2_2 (quantum/decoder_v2_2.py:421-443)
    and decoder_v1_0 (quantum/decoder_v1_0.py:377-403: the check-side layers' W and alpha).

        packed per-edge weights (ONE gather from the flat parameter buffer; V22: the 8 edge-type
        weights expanded per edge, sigmoid(weight)) -> forward with tape (gnnd_train_fwd) ->
        syndrome loss and d loss / d out of the readout (gnnd_syndrome_loss; V22: of every
        layer's readout at once, PerLayerLoss) -> reverse pass to the per-edge weight gradient
        (gnnd_train_bwd) -> type sums (V22: one [2T+2, E] x [E, 8] GEMM, deterministic) and
        sigmoid' -> flat gradient -> Adam (gnnd_adam_step)

    ~12 launches in one HIP graph (with a collective: compute and Adam graphs around the
    all_reduce(SUM) of the flat gradient).  The trained parameters (the source_to_target
    layers' W, W_p, the readout W / W_pr, and weight / alpha) are re-bound as views of one
    flat buffer; the target_to_source layers' unused W, W_p keep their storage and never
    change (torch's Adam skips parameters without a gradient).  Adam as the scripts (NBP
    lr 3e-4, V22 lr 2e-4, no decay), torch.optim.Adam's update order."""

    def __init__(self, model, loss_fn, lr=None, weight_decay=None, betas=(0.9, 0.999), eps=1e-8,
                 group=None, graph=True, warmup=2, force_collective=False):
        from .models import DecoderV10, DecoderV22, NeuralBP
        if not isinstance(model, (DecoderV10, DecoderV22, NeuralBP)):
            raise TypeError('FusedWbpTrainer trains NeuralBP, DecoderV22 and DecoderV10 models')
        rlr, rwd = REFERENCE_OPTIM[model.kind]
        self.model, self.loss_fn = model, loss_fn
        self.lr = rlr if lr is None else lr
        self.wd = rwd if weight_decay is None else weight_decay
        self.betas, self.eps = betas, eps
        self._init_graph(graph, warmup, group, force_collective)
        T = model.Nc
        v22 = model.kind == 'v22'
        tail = model.weight if v22 else model.alpha
        if model.kind == 'v10':
            # decoder_v1_0: only the target_to_source layers' W enter the forward
            # (quantum/decoder_v1_0.py:246-247); the source_to_target layers' W never change
            params = [model.layers[2 * t + 1].W for t in range(T)] + [model.alpha]
        else:
            params = ([q for t in range(T) for q in (model.layers[2 * t].W, model.layers[2 * t].W_p)]
                      + [model.W, model.W_pr if v22 else model.W_p, tail])
        dev = tail.device
        flat = torch.cat([q.detach().reshape(-1) for q in params]).contiguous()
        off = 0
        for q in params:
            n = q.numel()
            q.data = flat[off:off + n].view(q.shape)
            off += n
        self.flat, self.params = flat, params
        self.exp_avg = torch.zeros_like(flat)
        self.exp_avg_sq = torch.zeros_like(flat)
        self.step_count = torch.zeros(1, dtype=torch.float64, device=dev)
        self._grad = torch.zeros_like(flat)
        E = model.E
        if v22:
            # packed position (block k of 2T + 2, edge e) reads flat[8 k + type(e)]
            types = model.types.to(dev)
            blocks = torch.arange(2 * T + 2, device=dev).unsqueeze(1)
            self._gather = (8 * blocks + types.unsqueeze(0)).reshape(-1)
            self._onehot = torch.nn.functional.one_hot(types, 8).to(torch.float64)   # [E, 8]
        else:
            self._gather = None                  # identity: the tables ARE the parameters
        self._E = E
        model.graph(dev)                         # device graph tables now, never in a capture
        getattr(loss_fn, 'inner', loss_fn)._graph(dev)

    def _packed(self):
        if self._gather is None:
            return self.flat
        p = torch.empty(self._gather.numel() + 1, dtype=self.flat.dtype, device=self.flat.device)
        torch.index_select(self.flat, 0, self._gather, out=p[:-1])
        torch.sigmoid(self.flat[-1:], out=p[-1:])
        return p

    def _loss_grad(self, out, y):
        """Per-codeword losses and d loss / d out of the readout(s)."""
        m = self.model
        if m.kind == 'v22':                      # PerLayerLoss(train=True): every layer
            yy = y.reshape(1, -1).expand(m.Nc, -1).reshape(-1, 1)
            return self.loss_fn.inner.per_codeword(out, yy)
        return self.loss_fn.per_codeword(out, y)

    def _compute(self, x, y):
        m = self.model
        if x.dtype != torch.float64:
            raise ValueError('FusedWbpTrainer trains in fp64 (the reference scripts\' dtype)')
        g = m.graph(x.device)
        w = self._packed()
        out, tape = ops.train_forward(g, m.kind, x, w, m.Nc)
        loss_b, dpred = self._loss_grad(out, y)
        gw = ops.train_backward(g, m.kind, w, x, out, dpred, tape, m.Nc)
        if self._gather is None:
            self._grad.copy_(gw)
        else:                                    # type sums, then sigmoid'(weight)
            nb = 2 * m.Nc + 2
            torch.mm(gw[:-1].view(nb, self._E), self._onehot, out=self._grad[:-1].view(nb, 8))
            a = w[-1:]
            torch.mul(gw[-1:], a * (1 - a), out=self._grad[-1:])
        loss = loss_b.sum()
        return loss, [self._grad] if self._dist() else []

    def _apply(self):
        ops.adam_step(self.flat, self._grad, self.exp_avg, self.exp_avg_sq, self.step_count,
                      self.lr, self.betas, self.eps, self.wd)

    def step(self, data, y, copy_loss=True):
        self.model.train()
        x = data.x if data.x.dim() == 2 else data.x.unsqueeze(1)
        out = self._run(x, y, copy_loss)
        _invalidate(self.model)
        return out
