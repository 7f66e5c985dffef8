"""Training objectives and decode metrics of the reference (device tensors).

* `SyndromeLoss` — quantum/decoder_v2_4.py:297-317: sum |sin(pi/2 H^T (y + p))| +
  sum |sin(pi/2 Lambda (y + p))| over the batch (a SUM, so data-parallel gradients
  all-reduce with SUM).  `logical_only=True` is quantum/QGNNI.py:255-290 (Lambda term only).
* `ClassicalLoss` — classical/CGNNI.py:287-309: lambda * mean BCE + (1 - lambda) * mean
  |sin(pi/2 H^T p)| (train) or mean BCE (test), lambda = 0.8 (classical/CGNNI.py:206).
* `V30Loss` — quantum/decoder_v3_0.py:293-335 (GRU decoder; the script's batching kept).
* `PerLayerLoss` — quantum/decoder_v2_2.py:350-380: SyndromeLoss summed over the per-layer
  readout list of DecoderV22 (train), or the last layer (test).
* `toric_failures` — hard FER rule of quantum/neural_BP.py:338-348 (non-zero residual
  syndrome, or zero syndrome with a logical flip).

The reference builds [V, B] matrices with an O(B) torch.cat loop; here the same matrices are
views ([B*V,1] -> [B, V] -> transpose), identical values.
"""
import math

import numpy as np

import torch


def _cols(t, V):
    return t.reshape(-1, V).t()          # [V, B], column b = codeword b


class SyndromeLoss(torch.nn.Module):
    """On GPU tensors (fp32/fp64) the loss and its gradient come from ONE HIP launch
    (`gnnd_syndrome_loss`, ops.SyndromeLossFn); `reference_forward` is the reference's
    formula in torch ops (CPU tensors and the tests' cross-check)."""

    def __init__(self, H, logical, logical_only=False, fused=True):
        super().__init__()
        self.H_np = H.detach().cpu().numpy() if isinstance(H, torch.Tensor) else H
        H = torch.as_tensor(H, dtype=torch.float64)
        self.V = H.size(0)
        self.register_buffer('Ht', H.t().contiguous())                      # [C, V]
        self.register_buffer('logical', torch.as_tensor(logical, dtype=torch.float64))
        self.register_buffer('logical_rows', (torch.as_tensor(logical) != 0).to(torch.int32))
        self.logical_only = logical_only
        self.fused = fused
        self._graphs = {}
        self._casts = {}

    def _graph(self, device):
        g = self._graphs.get(device)
        if g is None:
            from .graph import TannerGraph
            g = self._graphs[device] = TannerGraph(self.H_np, device)
        return g

    def _cast(self, t, dtype):      # cached dtype copies of the constant matrices
        key = (id(t), dtype, t.device)
        c = self._casts.get(key)
        if c is None:
            c = self._casts[key] = t.to(dtype)
        return c

    def logical_mask(self, device):
        """int32 [V] bit masks of the logical rows (bit l: variable in row l), for the reverse
        pass's fused loss (gnnd_train_bwd_loss_partial); None if there are more than 32 rows."""
        nl = int(self.logical_rows.size(0))
        if nl > 32:
            return None
        key = ('lmask', torch.device(device))
        m = self._casts.get(key)
        if m is None:
            rows = (self.logical_rows.cpu().numpy() != 0).astype(np.int64)
            bits = (rows << np.arange(nl, dtype=np.int64)[:, None]).sum(0) if nl else np.zeros(self.V, np.int64)
            m = self._casts[key] = torch.as_tensor(bits.astype(np.uint32).view(np.int32), device=device)
        return m

    def rows_within_components(self, ncomp):
        """True iff every logical row's support lies inside one of `ncomp` equal contiguous
        variable blocks (the split Tanner graph's components)."""
        if ncomp <= 1:
            return True
        rows = self.logical_rows.cpu().numpy() != 0
        Vk = self.V // ncomp
        for r in rows:
            blocks = {int(v) // Vk for v in np.nonzero(r)[0]}
            if len(blocks) > 1:
                return False
        return True

    def per_codeword(self, pred, y):
        """(loss per codeword [B], d loss / d pred): the fused kernel, or the reference formula
        under autograd where the kernel does not apply (more than 32 logical rows, or graph
        tables beyond the LDS budget)."""
        from . import _lib, ops
        if pred.is_cuda and pred.dtype in (torch.float32, torch.float64):
            try:
                return ops.syndrome_loss(self._graph(pred.device), self.logical_rows,
                                         self.logical_only, pred, y)
            except _lib.GnndError as e:
                if e.status != _lib.ERR_UNSUPPORTED:
                    raise
        with torch.enable_grad():
            p = pred.detach().clone().requires_grad_(True)
            s = _cols(y, self.V).to(p.dtype) + _cols(p, self.V)              # [V, B]
            t = torch.abs(torch.sin(torch.matmul(self._cast(self.logical, p.dtype), s) * math.pi / 2)).sum(0)
            if not self.logical_only:
                t = torch.abs(torch.sin(torch.matmul(self._cast(self.Ht, p.dtype), s) * math.pi / 2)).sum(0) + t
            t.sum().backward()
        return t.detach(), p.grad

    def reference_forward(self, pred, y):
        s = _cols(y, self.V).to(pred.dtype) + _cols(pred, self.V)
        loss = torch.abs(torch.sin(torch.matmul(self._cast(self.logical, pred.dtype), s) * math.pi / 2)).sum()
        if not self.logical_only:
            loss = torch.abs(torch.sin(torch.matmul(self._cast(self.Ht, pred.dtype), s) * math.pi / 2)).sum() + loss
        return loss

    def forward(self, pred, y):
        if self.fused and pred.is_cuda and pred.dtype in (torch.float32, torch.float64):
            from . import _lib
            from .ops import SyndromeLossFn
            try:
                return SyndromeLossFn.apply(pred, y, self._graph(pred.device), self.logical_rows,
                                            self.logical_only)
            except _lib.GnndError as e:      # > 32 logical rows / tables beyond the LDS budget
                if e.status != _lib.ERR_UNSUPPORTED:
                    raise
        return self.reference_forward(pred, y)


class ClassicalLoss(torch.nn.Module):
    def __init__(self, H, lambda_a=0.8):
        super().__init__()
        H = torch.as_tensor(H, dtype=torch.float32)
        self.V = H.size(0)
        self.register_buffer('Ht', H.t().contiguous())                      # [C, V]
        self.lambda_a = lambda_a

    def forward(self, pred, y, train=True):
        loss_a = (1 - y).mul(torch.log(1 - pred)) + y.mul(torch.log(pred))
        if not train:
            return torch.sum(loss_a) / (-1 * torch.numel(loss_a))
        loss_c = torch.abs(torch.sin(torch.matmul(self.Ht.to(pred.dtype), _cols(pred, self.V)) * math.pi / 2))
        return (torch.sum(self.lambda_a * loss_a) / (-1 * torch.numel(loss_a))
                + torch.sum((1 - self.lambda_a) * loss_c) / torch.numel(loss_c))


class V30Loss(torch.nn.Module):
    """quantum/decoder_v3_0.py:293-335 (LossFunc of the GRU edge-state decoder), restated
    literally on `preds` = DecoderV30's [out0, out1]:

        loss = sum |sin(pi/2 H^T (y_0 + res))| + sum BCE(|sin(pi/2 res_p)|, syn)

    with the script's own batching, kept as is: `tmp` is the FIRST codeword's y for every
    column (the loop extending it is commented out, :308), and the columns of res / res_p
    are sliced from the [B*N] outputs at stride V (= max(H.size())), not N (:307-310); only
    syn steps by N.  Needs the decoder input x for the syndrome (`needs_input`: the
    trainers call loss_fn(pred, y, x))."""
    needs_input = True

    def __init__(self, H):
        super().__init__()
        H = torch.as_tensor(H, dtype=torch.float64)
        self.a, self.b = max(H.shape), min(H.shape)
        self.register_buffer('Ht', H.t().contiguous())                      # [C, V]

    def loss_and_grad(self, out, y, x):
        """(loss, d loss / d out) for the fused trainer, out = [out0; out1] as one [2*B*N]
        tensor.  The check term is gnnd_syndrome_loss on out0's first B*V rows (column k =
        rows kV..kV+V-1, the script's stride-V slicing) with every column's y = the first
        codeword's (`tmp`); the BCE term and its gradient are elementwise on the strided
        [B, C] gathers of out1 and x (torch autograd's formulas: BCE' = (1 - s)/(1 - q) - s/q,
        q = |sin(pi/2 r)|).  None when the BCE rows of neighbouring columns overlap (C > V)."""
        a, b = self.a, self.b
        N = a + b
        B = y.numel() // a
        if b > a or out.dtype not in (torch.float32, torch.float64):
            return None
        syn_loss = getattr(self, '_syn', {}).get(out.device)
        if syn_loss is None:                     # the check term: H^T s rows, no logical rows
            syn_loss = SyndromeLoss(self.Ht.t().cpu(), torch.zeros(0, a)).to(out.device)
            self._syn = {**getattr(self, '_syn', {}), out.device: syn_loss}
        o = out.reshape(-1)
        n = B * N
        ycols = y.reshape(-1)[:a].to(o.dtype).repeat(B)
        loss_a, d_a = syn_loss.per_codeword(o[:B * a], ycols)
        key = (B, out.device)
        cache = getattr(self, '_bce_idx', {})
        if key not in cache:                     # (rows of out1, rows of x) of the BCE term
            k = torch.arange(B, device=out.device).unsqueeze(1)
            j = torch.arange(b, device=out.device)
            cache[key] = (n + k * a + a + j, k * N + a + j)
            self._bce_idx = cache
        ri, xi = cache[key]
        r = o[ri]
        syn = x.reshape(-1)[xi].to(o.dtype)
        h = r * math.pi / 2
        sn = torch.sin(h)
        q = torch.abs(sn)
        bce = -1 * (1 - syn).mul(torch.log(1 - q)) - syn.mul(torch.log(q))
        gq = (1 - syn) / (1 - q) - syn / q
        gr = gq * torch.sgn(sn) * torch.cos(h) * (math.pi / 2)
        d = torch.zeros_like(o)
        d[:B * a] = d_a.reshape(-1)
        d[ri] = gr                               # (distinct rows: b <= a)
        return loss_a.sum() + bce.sum(), d.view_as(out)

    def forward(self, preds, y, x):
        a, b = self.a, self.b
        N = a + b
        B = y.numel() // a
        dev = y.device
        k = torch.arange(B, device=dev).unsqueeze(1)
        p0, p1, xf = preds[0].reshape(-1), preds[1].reshape(-1), x.reshape(-1)
        res = p0[k * a + torch.arange(a, device=dev)].t()                   # [a, B]
        res_p = p1[k * a + a + torch.arange(b, device=dev)].t()             # [b, B]
        syn = xf[k * N + a + torch.arange(b, device=dev)].t().to(res_p.dtype)
        tmp = y.reshape(-1)[:a].unsqueeze(1).to(res.dtype)                  # [a, 1]
        loss_a = torch.matmul(self.Ht.to(res.dtype), tmp + res)
        res_p = torch.abs(torch.sin(res_p * math.pi / 2))
        loss_b = -1 * (1 - syn).mul(torch.log(1 - res_p)) - syn.mul(torch.log(res_p))
        return torch.abs(torch.sin(loss_a * math.pi / 2)).sum() + loss_b.sum()


class PerLayerLoss(torch.nn.Module):
    """quantum/decoder_v2_2.py:350-380 (LossFunc of the edge-type decoder, whose GNNI returns
    one readout per layer): train=True sums the syndrome + logical loss of SyndromeLoss over
    EVERY layer's readout (in layer order), train=False takes the last layer only."""

    def __init__(self, H, logical, fused=True):
        super().__init__()
        self.inner = SyndromeLoss(H, logical, fused=fused)

    def forward(self, preds, y, train=True):
        preds = preds if train else preds[-1:]
        loss = None
        for p in preds:
            term = self.inner(p, y)
            loss = term if loss is None else loss + term
        return loss


def toric_failures(H, logical, y, pred, graph=None):
    """(residual-syndrome failures, logical failures) for hard decisions pred > 0.5
    (quantum/neural_BP.py:333-348).  With a TannerGraph of H and CUDA fp32/fp64 tensors the
    counts come from one HIP launch (ops.decision_errors); otherwise torch ops."""
    if graph is not None and pred.is_cuda and pred.dtype in (torch.float32, torch.float64):
        from .ops import decision_errors
        lg = (torch.as_tensor(logical) != 0).to(torch.int32)
        c = decision_errors(graph, lg, pred, y).tolist()
        return int(c[2]), int(c[3])
    Ht = torch.as_tensor(H, dtype=torch.float32, device=pred.device).t()
    lg = torch.as_tensor(logical, dtype=torch.float32, device=pred.device)
    V = Ht.size(1)
    e = torch.remainder(_cols(y, V).float() + (_cols(pred, V) > 0.5).float(), 2)
    bad_syn = (torch.remainder(Ht @ e, 2) != 0).any(dim=0)
    bad_log = (~bad_syn) & (torch.remainder(lg @ e, 2) != 0).any(dim=0)
    return int(bad_syn.sum()), int(bad_log.sum())
