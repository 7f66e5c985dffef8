"""The reference decoders on the MI355X operator (same layer names and state_dict keys).

Each class mirrors one reference script's `GNNI` (paths relative to
/root/reference/GNN-decode/) so its checkpoints load with `load_state_dict`:

  DecoderV24   quantum/decoder_v2_4.py:230-294   keys ggc1.mlp.{0,2}.*, ggc2.mlp.*, mlp.*
  QGNNI        quantum/QGNNI.py:186-252           keys ggc{1,2}.mlp.*, mlp.*
  QuantumBP    quantum/BP.py:179-219              (no parameters)
  CGNNI        classical/CGNNI.py:212-284         keys ggc{1,2}.mlp{1,2}.*, ggc{1,2}.rnn.*, mlp.*
  ClassicalBP  classical/BP.py:216-259            (no parameters)
  NeuralBP     quantum/neural_BP.py:236-314       keys layers.{i}.W, layers.{i}.W_p, W, W_p, alpha
  DecoderV10   quantum/decoder_v1_0.py:236-313    keys layers.{i}.W, alpha
  DecoderV30   quantum/decoder_v3_0.py:199-290    keys ggc{1,2}.mlp{1,2}.*, ggc{1,2}.rnn{1,2}.*,
                                                  mlp.*  (GRU edge states, two-output readout)
  DecoderV22   quantum/decoder_v2_2.py:272-347    keys layers.{i}.W, layers.{i}.W_p, W, W_pr,
                                                  weight  (edge-type weights, per-layer readout)

Differences from the reference, all at the call boundary: the parity-check matrix is
passed to the constructor (`GNNI(Nc, H)`) instead of being read from module globals
(`rows`, `cols`, `BATCH_SIZE`), and the batch size is derived from `data.x`.

`forward(data)` runs the fused single-launch decoder (libgnnd `gnnd_decode`) whenever the
batch is the tiled Tanner graph and no autograd graph is requested (eval mode or
no_grad); otherwise (training) it runs the reference's layer-by-layer loop on the device
operator (`MessagePassing.propagate` -> gnnd_propagate_*, with HIP backward kernels) and
torch autograd through the MLPs.
"""
import torch

from . import ops
from .graph import TannerGraph
from .nn import MessagePassing, ClassicalMessagePassing, message_passing_class

_MP = {v: message_passing_class(v) for v in ('v24', 'qgnni', 'qbp', 'cbp', 'nbp', 'v10', 'v30')}
_MP['cgnni'] = ClassicalMessagePassing


def _mlp(fan_in, hidden, act, dtype):
    return torch.nn.Sequential(torch.nn.Linear(fan_in, hidden).to(dtype), act,
                               torch.nn.Linear(hidden, 1).to(dtype))


def init_weights(m):
    """quantum/decoder_v2_4.py:211-215: Kaiming-normal weights, zero bias."""
    if type(m) == torch.nn.Linear:
        torch.nn.init.kaiming_normal_(m.weight, a=0, mode='fan_in')
        m.bias.data.fill_(0)


class _SkinnyLinear(torch.autograd.Function):
    """y = x W^T + b for the per-edge MLPs (in or out width <= 2 on one side, rows = edges
    x batch).  Same forward as torch.nn.Linear; the backward forms the weight gradient as a
    fused multiply + column reduction over the rows instead of a K = rows GEMM: hipBLASLt
    runs those tall-skinny GEMMs at ~0.1 TFLOP/s (100-190 us each, 56 % of a decoder_v2_4
    training step, profiles/r01/train_v24_kernel_stats.csv), the reduction streams the
    operands once."""

    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        return torch.addmm(b, x, W.t())

    @staticmethod
    def backward(ctx, gy):
        x, W = ctx.saved_tensors
        gx = gW = gb = None
        if ctx.needs_input_grad[0]:
            gx = gy * W if W.size(0) == 1 else gy @ W          # [n,1]*[1,in] or [n,out]@[out,in]
        if ctx.needs_input_grad[1]:
            if W.size(1) == 1:
                gW = (gy * x).sum(0).unsqueeze(1)                # [out, 1]
            elif W.size(0) == 1:
                gW = (x * gy).sum(0).unsqueeze(0)                # [1, in]
            else:
                gW = torch.stack([(gy * x[:, i:i + 1]).sum(0) for i in range(W.size(1))], 1)
        if ctx.needs_input_grad[2]:
            gb = gy.sum(0)
        return gx, gW, gb


def _apply_mlp(seq, u):
    """seq = Sequential(Linear, activation, Linear) evaluated with _SkinnyLinear (training)."""
    if not torch.is_grad_enabled():
        return seq(u)
    h = _SkinnyLinear.apply(u, seq[0].weight, seq[0].bias)
    return _SkinnyLinear.apply(seq[1](h), seq[2].weight, seq[2].bias)


def _flat_mlp(seq, split_inputs=False):
    W1 = seq[0].weight
    parts = [W1[:, k] for k in range(W1.size(1))] if split_inputs else [W1.reshape(-1)]
    return parts + [seq[0].bias.reshape(-1), seq[2].weight.reshape(-1), seq[2].bias.reshape(-1)]


# ---------------------------------------------------------------------------------------
# layers
# ---------------------------------------------------------------------------------------
class GraphConvV24(_MP['v24']):
    """quantum/decoder_v2_4.py:230-257."""

    def __init__(self, flow, aggr='add', bias=True):
        super().__init__(aggr, flow)
        fan_in = 2 if flow == 'source_to_target' else 1
        self.mlp = _mlp(fan_in, 128, torch.nn.Softplus(), torch.float64)
        self.mlp.apply(init_weights)

    def forward(self, m, edge_index, x, size=None):
        x = x if x.dim() == 2 else x.unsqueeze(-1)
        size = size or (x.size(0), x.size(0))
        return self.propagate(edge_index=edge_index, size=size, x=m, extra=x)

    def update(self, aggr_out):
        if self.flow == 'source_to_target':
            return _apply_mlp(self.mlp, aggr_out.to(self.mlp[0].weight.dtype)).to(aggr_out.dtype)
        u = aggr_out[:, 0:1].to(self.mlp[0].weight.dtype)
        return _apply_mlp(self.mlp, u).to(aggr_out.dtype) * aggr_out[:, 1:2]


class GraphConvQGNNI(_MP['qgnni']):
    """quantum/QGNNI.py:186-214."""

    def __init__(self, flow, aggr='add', bias=True):
        super().__init__(aggr, flow)
        self.mlp = _mlp(1, 10, torch.nn.ReLU(), torch.float64)

    def forward(self, m, edge_index, x, size=None):
        x = x if x.dim() == 2 else x.unsqueeze(-1)
        size = size or (x.size(0), x.size(0))
        return self.propagate(edge_index=edge_index, size=size, x=m, extra=x)

    def update(self, aggr_out):
        if self.flow == 'target_to_source':
            u = aggr_out[:, 0:1].to(self.mlp[0].weight.dtype)
            return _apply_mlp(self.mlp, u).to(aggr_out.dtype) * aggr_out[:, 1:2]
        return aggr_out


class GatedGraphConvBP(MessagePassing):
    """quantum/BP.py:179-188 and classical/BP.py:216-228 (variant set per script)."""

    def __init__(self, flow, variant, aggr='add', bias=True):
        super().__init__(aggr, flow)
        self.variant = variant

    def forward(self, m, edge_index, x=None, size=None):
        if x is not None:
            x = x if x.dim() == 2 else x.unsqueeze(-1)
        n = x.size(0) if x is not None else None
        size = size or (n, n)
        return self.propagate(edge_index=edge_index, size=size, x=m, extra=x)


class GatedGraphConvCGNNI(ClassicalMessagePassing):
    """classical/CGNNI.py:212-242 (mlp1 and rnn exist for state_dict compatibility only)."""

    def __init__(self, flow, aggr='add', bias=True):
        super().__init__(aggr, flow)
        self.mlp1 = _mlp(1, 10, torch.nn.ReLU(), torch.float32)
        self.mlp2 = _mlp(1, 10, torch.nn.ReLU(), torch.float32)
        self.rnn = torch.nn.GRUCell(1, 1, bias=bias)

    def forward(self, m, edge_index, x=None, size=None):
        if x is not None:
            x = x if x.dim() == 2 else x.unsqueeze(-1)
        n = x.size(0) if x is not None else None
        size = size or (n, n)
        return self.propagate(edge_index=edge_index, size=size, x=m, post=x)

    def update(self, aggr_out):
        if self.flow == 'target_to_source':
            return _apply_mlp(self.mlp2, aggr_out.to(self.mlp2[0].weight.dtype)).to(aggr_out.dtype)
        return aggr_out


def _edge_param(E, value):
    return torch.nn.Parameter(torch.full((E, 1), float(value), dtype=torch.float64))


class GraphConvNBP(_MP['nbp']):
    """quantum/neural_BP.py:236-260.  Per-edge W scales the v->c input messages and W_p the
    prior in `update`; both act in the source_to_target layer only (the target_to_source
    layer's pair exists as unused parameters, as in the reference)."""

    def __init__(self, flow, E, aggr='add', bias=True):
        super().__init__(aggr, flow)
        self.W = _edge_param(E, 1.0)
        self.W_p = _edge_param(E, 1.0)

    def forward(self, m, edge_index, x, prev=None, size=None):
        x = x if x.dim() == 2 else x.unsqueeze(-1)
        if self.flow == 'source_to_target':
            m = m.mul(self.W.repeat(m.size(0) // self.W.size(0), 1))
        size = size or (x.size(0), x.size(0))
        return self.propagate(edge_index=edge_index, size=size, x=m, extra=x)

    def update(self, aggr_out):
        if self.flow == 'source_to_target':
            B = aggr_out.size(0) // self.W_p.size(0)
            return aggr_out[:, 0:1] + aggr_out[:, 1:2].mul(self.W_p.repeat(B, 1))
        return aggr_out


class GraphConvV22(_MP['nbp']):
    """quantum/decoder_v2_2.py:272-296: neural_BP's layer (the script's propagate body is
    neural_BP.py's) with W, W_p shared by the 8 edge types: `m.mul(feat_onehot) @ W` is
    m_e W[type(e)] exactly (one non-zero product per row), so the layer gathers W[type]."""

    def __init__(self, flow, types, aggr='add', bias=True):
        super().__init__(aggr, flow)
        self.W = torch.nn.Parameter(torch.ones(8, 1, dtype=torch.float64))
        self.W_p = torch.nn.Parameter(torch.ones(8, 1, dtype=torch.float64))
        self.register_buffer('types', types, persistent=False)

    def forward(self, m, edge_index, x, prev=None, size=None):
        x = x if x.dim() == 2 else x.unsqueeze(-1)
        if self.flow == 'source_to_target':
            w = self.W[self.types.to(m.device)]
            m = m.mul(w.repeat(m.size(0) // w.size(0), 1))
        size = size or (x.size(0), x.size(0))
        return self.propagate(edge_index=edge_index, size=size, x=m, extra=x)

    def update(self, aggr_out):
        if self.flow == 'source_to_target':
            wp = self.W_p[self.types.to(aggr_out.device)]
            return aggr_out[:, 0:1] + aggr_out[:, 1:2].mul(wp.repeat(aggr_out.size(0) // wp.size(0), 1))
        return aggr_out


class GraphConvV10(_MP['v10']):
    """quantum/decoder_v1_0.py:236-252: per-edge W scales the c->v layer's input."""

    def __init__(self, flow, E, aggr='add', bias=True):
        super().__init__(aggr, flow)
        self.W = _edge_param(E, 1.0)

    def forward(self, m, edge_index, x, prev=None, size=None):
        x = x if x.dim() == 2 else x.unsqueeze(-1)
        if self.flow != 'source_to_target':
            m = m.mul(self.W.repeat(m.size(0) // self.W.size(0), 1))
        size = size or (x.size(0), x.size(0))
        return self.propagate(edge_index=edge_index, size=size, x=m, extra=x)


class GraphConvV30(_MP['v30']):
    """quantum/decoder_v3_0.py:199-242: propagate (no pre-op, cat extra[idx_j]) -> mlp1 / mlp2
    (Linear(2,10) ReLU Linear(10,1)) -> GRUCell(input = the edge state, hidden = the MLP
    output).  Both layers own mlp1, mlp2, rnn1 and rnn2 (ggc1 uses mlp1/rnn1, ggc2
    mlp2/rnn2), as in the reference, so state_dicts load unchanged."""

    def __init__(self, flow, aggr='add', bias=True):
        super().__init__(aggr, flow)
        self.mlp1 = _mlp(2, 10, torch.nn.ReLU(), torch.float64)
        self.mlp2 = _mlp(2, 10, torch.nn.ReLU(), torch.float64)
        self.rnn1 = torch.nn.GRUCell(1, 1, bias=bias).double()
        self.rnn2 = torch.nn.GRUCell(1, 1, bias=bias).double()

    def forward(self, m, edge_index, x, size=None):
        x = x if x.dim() == 2 else x.unsqueeze(-1)
        size = size or (x.size(0), x.size(0))
        mes = self.propagate(edge_index=edge_index, size=size, x=m, extra=x)
        rnn = self.rnn2 if self.flow == 'target_to_source' else self.rnn1
        dt = rnn.weight_ih.dtype
        return rnn(m.to(dt), mes.to(dt)).to(m.dtype)

    def update(self, aggr_out):
        seq = self.mlp2 if self.flow == 'target_to_source' else self.mlp1
        return _apply_mlp(seq, aggr_out.to(seq[0].weight.dtype)).to(aggr_out.dtype)


def _flat_gru(cell):
    z = torch.zeros(3, dtype=cell.weight_ih.dtype, device=cell.weight_ih.device)
    return [cell.weight_ih.reshape(-1), cell.weight_hh.reshape(-1),
            cell.bias_ih.reshape(-1) if cell.bias else z, cell.bias_hh.reshape(-1) if cell.bias else z]


# ---------------------------------------------------------------------------------------
# decoders
# ---------------------------------------------------------------------------------------
class _Decoder(torch.nn.Module):
    kind = None            # libgnnd model name
    classical = False

    def __init__(self, Nc, H):
        super().__init__()
        self.Nc = Nc
        self.H = torch.as_tensor(H).detach().cpu()
        self.rows, self.cols = int(self.H.size(0)), int(self.H.size(1))
        self._graphs = {}
        self._wcache = None
        self._priors = ()

    # ---- graph / weights on the device ------------------------------------------------
    def graph(self, device):
        key = str(device)
        g = self._graphs.get(key)
        if g is None:
            g = TannerGraph(self.H, device=device)
            self._graphs[key] = g
            for mod in self.modules():
                if isinstance(mod, MessagePassing):
                    mod.bind_graph(g)
        return g

    def packed_weights(self):
        """Flat weights in the gnnd.h layout (model parameter dtype)."""
        return None

    def invalidate_weight_cache(self):
        """Forget the prepared (packed) weights.  The cache key tracks parameter versions,
        which device-side updates do not bump: a replayed HIP graph's optimizer step and the
        fused trainer's gnnd_adam_step.  The trainers call this after every step."""
        self._wcache = None

    def set_channel_priors(self, priors):
        """decoder_v2_4, fp64: the channel-prior LLRs x_v the inputs carry (one per codeword in
        the reference's gen_syn data; e.g. ops.channel_priors(graph, x)).  The fused decoder then
        reads the variable-side MLP from a table per prior (gnnd_prepare_weights_priors); inputs
        with other priors still decode exactly (the 128 units).  () to clear."""
        if priors and self.kind != 'v24':
            raise ValueError('channel-prior tables: decoder_v2_4 only')
        self._priors = tuple(float(v) for v in priors)
        self._wcache = None

    def prepared_weights(self, dtype, device):
        key = (dtype, str(device), tuple(p._version for p in self.parameters()),
               tuple(p.data_ptr() for p in self.parameters()), self._priors)
        if self._wcache is not None and self._wcache[0] == key:
            return self._wcache[1]
        flat = self.packed_weights()
        if flat is None:
            return None
        pri = self._priors if dtype == torch.float64 else None
        prep = ops.prepare_weights(self.kind, flat.detach().to(device=device, dtype=dtype), priors=pri)
        self._wcache = (key, prep)
        return prep

    def fused_ok(self, x, edge_index):
        dts = (torch.float32, torch.float64, torch.bfloat16) if self.kind in ('cgnni', 'cbp') \
            else (torch.float32, torch.float64)
        if not x.is_cuda or x.dtype not in dts:
            return False
        if torch.is_grad_enabled() and self.training and any(p.requires_grad for p in self.parameters()):
            return False
        g = self.graph(x.device)
        if x.numel() % g.N or edge_index.size(1) != (x.numel() // g.N) * g.E:
            return False
        return g.is_tiled(edge_index, 0)

    def forward(self, data):
        x, edge_index = data.x, data.edge_index
        if x.dim() == 1:
            x = x.unsqueeze(1)
        if self.fused_ok(x, edge_index):
            g = self.graph(x.device)
            # bf16 inputs (classical models): bf16 storage, fp32 weights and arithmetic
            wdt = torch.float32 if x.dtype == torch.bfloat16 else x.dtype
            return ops.decode(g, self.kind, x, self.Nc, self.prepared_weights(wdt, x.device))
        if not x.is_cuda:
            raise RuntimeError('gnndecode runs on the GPU only (HIP/gfx950); move data to cuda')
        self.graph(x.device)      # training: autograd through the HIP propagate kernels
        return self.forward_layers(x, edge_index)

    # ---- reference layer-by-layer loop on the device operator ---------------------------
    def _shifted(self, edge_index):
        # cached per input tensor: the same shifted tensor keeps the propagate ops' tiled-
        # structure check cached (no device round trip per step; required under graph capture)
        c = getattr(self, '_shift_cache', None)
        if c is not None and c[0]() is edge_index and c[1] == edge_index._version:
            return c[2]
        import weakref
        out = torch.stack([edge_index[0], edge_index[1] + self.rows])
        self._shift_cache = (weakref.ref(edge_index), edge_index._version, out)
        return out

    def _var_rows(self, t, B):
        N = self.rows + self.cols
        return t.reshape(B, N, -1)[:, :self.rows].reshape(B * self.rows, -1)

    def _var_sum(self, m, edge_index, nodes):
        out = torch.zeros(nodes, m.size(1), dtype=m.dtype, device=m.device)
        return out.index_add_(0, edge_index[0], m)

    def forward_layers(self, x, edge_index):
        raise NotImplementedError


class DecoderV24(_Decoder):
    """quantum/decoder_v2_4.py:260-294 (T = Nc = 15 in the reference).

    Training (grad enabled, tiled batch) runs the fused HIP step (ops.FusedTrainFn:
    gnnd_train_fwd + gnnd_train_bwd, two launches per step) unless `fused_train` is False,
    which selects the reference's layer-by-layer loop on the propagate kernels."""
    kind = 'v24'
    fused_train = True

    def forward(self, data):
        x, edge_index = data.x, data.edge_index
        if x.dim() == 1:
            x = x.unsqueeze(1)
        if (self.fused_train and x.is_cuda and torch.is_grad_enabled() and self.training
                and any(p.requires_grad for p in self.parameters())
                and x.dtype in (torch.float32, torch.float64)):
            g = self.graph(x.device)
            if (x.numel() % g.N == 0 and edge_index.size(1) == (x.numel() // g.N) * g.E
                    and g.is_tiled(edge_index, 0)):
                return ops.FusedTrainFn.apply(self.packed_weights(), x, g, self.kind, self.Nc)
        return super().forward(data)

    def __init__(self, Nc, H):
        super().__init__(Nc, H)
        self.ggc1 = GraphConvV24('source_to_target')
        self.ggc2 = GraphConvV24('target_to_source')
        self.mlp = _mlp(1, 128, torch.nn.Softplus(), torch.float64)
        self.mlp.apply(init_weights)

    def packed_weights(self):
        return torch.cat(_flat_mlp(self.ggc1.mlp, split_inputs=True) + _flat_mlp(self.ggc2.mlp)
                         + _flat_mlp(self.mlp))

    def forward_layers(self, x, ei):
        B = x.size(0) // (self.rows + self.cols)
        ei = self._shifted(ei)
        m = torch.zeros(ei.size(1), 1, dtype=x.dtype, device=x.device)
        for _ in range(self.Nc):
            m_p = m
            m = self.ggc1(m, ei, x)
            m = self.ggc2(m, ei, x) + m_p
        f = _apply_mlp(self.mlp, m.to(self.mlp[0].weight.dtype)).to(x.dtype)
        res = self._var_rows(self._var_sum(f, ei, x.size(0)), B) + self._var_rows(x, B)
        return torch.sigmoid(-res)


class QGNNI(_Decoder):
    """quantum/QGNNI.py:217-252 (T = 25)."""
    kind = 'qgnni'

    def __init__(self, Nc, H):
        super().__init__(Nc, H)
        self.ggc1 = GraphConvQGNNI('source_to_target')
        self.ggc2 = GraphConvQGNNI('target_to_source')
        self.mlp = _mlp(1, 10, torch.nn.ReLU(), torch.float64)

    def packed_weights(self):
        return torch.cat(_flat_mlp(self.ggc2.mlp) + _flat_mlp(self.mlp))

    def forward_layers(self, x, ei):
        B = x.size(0) // (self.rows + self.cols)
        ei = self._shifted(ei)
        m = torch.zeros(ei.size(1), 1, dtype=x.dtype, device=x.device)
        for _ in range(self.Nc):
            m_p = m
            m = self.ggc1(m, ei, x)
            m = self.ggc2(m, ei, x) + m_p
        r = self._var_rows(self._var_sum(m, ei, x.size(0)) + x, B)
        return torch.sigmoid(-_apply_mlp(self.mlp, r.to(self.mlp[0].weight.dtype)).to(x.dtype))


class QuantumBP(_Decoder):
    """quantum/BP.py:191-219 (T = 10)."""
    kind = 'qbp'

    def __init__(self, Nc, H):
        super().__init__(Nc, H)
        self.ggc1 = GatedGraphConvBP('source_to_target', 'qbp')
        self.ggc2 = GatedGraphConvBP('target_to_source', 'qbp')

    def forward_layers(self, x, ei):
        B = x.size(0) // (self.rows + self.cols)
        ei = self._shifted(ei)
        m = torch.zeros(ei.size(1), 1, dtype=x.dtype, device=x.device)
        for _ in range(self.Nc):
            m = self.ggc1(m, ei, x)
            m = self.ggc2(m, ei, x)
        res = self._var_rows(self._var_sum(m, ei, x.size(0)), B) + self._var_rows(x, B)
        return torch.sigmoid(-res)


class CGNNI(_Decoder):
    """classical/CGNNI.py:248-284 (T = 25)."""
    kind = 'cgnni'
    classical = True

    def __init__(self, Nc, H):
        super().__init__(Nc, H)
        self.ggc1 = GatedGraphConvCGNNI('source_to_target')
        self.ggc2 = GatedGraphConvCGNNI('target_to_source')
        self.mlp = _mlp(1, 10, torch.nn.ReLU(), torch.float32)

    def packed_weights(self):
        return torch.cat(_flat_mlp(self.ggc2.mlp2) + _flat_mlp(self.mlp))

    def forward_layers(self, x, ei):
        B = x.size(0) // (self.rows + self.cols)
        ei = self._shifted(ei)
        m = torch.zeros(ei.size(1), 1, dtype=x.dtype, device=x.device)
        for _ in range(self.Nc):
            m_p = m
            m = self.ggc1(m, ei, x)
            m = self.ggc2(m, ei) + m_p
        r = self._var_rows(self._var_sum(m, ei, x.size(0)) + x, B)
        res = torch.sigmoid(-_apply_mlp(self.mlp, r.to(self.mlp[0].weight.dtype)).to(x.dtype))
        return torch.clamp(res, 1e-7, 1 - 1e-7)


class ClassicalBP(_Decoder):
    """classical/BP.py:231-259 (T = 25)."""
    kind = 'cbp'
    classical = True

    def __init__(self, Nc, H):
        super().__init__(Nc, H)
        self.ggc1 = GatedGraphConvBP('source_to_target', 'cbp')
        self.ggc2 = GatedGraphConvBP('target_to_source', 'cbp')

    def forward_layers(self, x, ei):
        B = x.size(0) // (self.rows + self.cols)
        ei = self._shifted(ei)
        m = torch.zeros(ei.size(1), 1, dtype=x.dtype, device=x.device)
        for _ in range(self.Nc):
            m = self.ggc1(m, ei, x)
            m = self.ggc2(m, ei, x)   # classical/BP.py:246 passes no x; the body ignores it
        res = self._var_rows(self._var_sum(m, ei, x.size(0)) + x, B)
        return torch.clamp(torch.sigmoid(-res), 1e-7, 1 - 1e-7)


class _WeightedBP(_Decoder):
    """Shared plumbing of the weighted ("neural") BP decoders: Nc pairs of layers with
    per-edge weight tables, residual m = c2v + m_prev @ alpha."""
    layer_cls = None

    def __init__(self, Nc, H):
        super().__init__(Nc, H)
        self.E = int(self.H.sum())
        layers = []
        for _ in range(Nc):
            layers.append(self.layer_cls('source_to_target', self.E))
            layers.append(self.layer_cls('target_to_source', self.E))
        self.layers = torch.nn.Sequential(*layers)
        self.alpha = torch.nn.Parameter(torch.zeros(1, 1, dtype=torch.float64))

    def prepared_weights(self, dtype, device):
        flat = self.packed_weights()
        return ops.prepare_weights(self.kind, flat.detach().to(device=device, dtype=dtype))

    def _messages(self, x, ei):
        m = torch.zeros(ei.size(1), 1, dtype=x.dtype, device=x.device)
        alpha = self.alpha.to(x.dtype)
        for i in range(0, len(self.layers), 2):
            m_p = m
            m = self.layers[i](m, ei, x)
            m = self.layers[i + 1](m, ei, x) + torch.matmul(m_p, alpha)
        return m


class NeuralBP(_WeightedBP):
    """quantum/neural_BP.py:263-314 (Nc = 15, toric L = 4 in the reference)."""
    kind = 'nbp'
    layer_cls = GraphConvNBP

    def __init__(self, Nc, H):
        super().__init__(Nc, H)
        self.W = _edge_param(self.E, 1.0)
        self.W_p = _edge_param(self.E, 0.5)

    def packed_weights(self):
        per = [torch.cat([self.layers[2 * t].W.reshape(-1), self.layers[2 * t].W_p.reshape(-1)])
               for t in range(self.Nc)]
        return torch.cat(per + [self.W.reshape(-1), self.W_p.reshape(-1), self.alpha.reshape(-1)])

    def forward_layers(self, x, ei):
        B = x.size(0) // (self.rows + self.cols)
        ei = self._shifted(ei)
        m = self._messages(x, ei)
        m = m.mul(self.W.repeat(B, 1).to(x.dtype))
        prior = x[ei[0]].mul(self.W_p.repeat(B, 1).to(x.dtype))
        res = (self._var_rows(self._var_sum(m, ei, x.size(0)), B)
               + self._var_rows(self._var_sum(prior, ei, x.size(0)), B))
        return torch.sigmoid(-res)


class DecoderV10(_WeightedBP):
    """quantum/decoder_v1_0.py:263-313 (Nc = 15, toric L = 4 in the reference)."""
    kind = 'v10'
    layer_cls = GraphConvV10

    def packed_weights(self):
        return torch.cat([self.layers[2 * t + 1].W.reshape(-1) for t in range(self.Nc)]
                         + [self.alpha.reshape(-1)])

    def forward_layers(self, x, ei):
        B = x.size(0) // (self.rows + self.cols)
        ei = self._shifted(ei)
        m = self._messages(x, ei)
        res = self._var_rows(self._var_sum(m, ei, x.size(0)), B) + self._var_rows(x, B)
        return torch.sigmoid(-res)


class DecoderV30(_Decoder):
    """quantum/decoder_v3_0.py:245-290 (Nc = 15, toric L = 8 in the script): per-edge GRU
    states updated on the variable side (ggc1) then the check side (ggc2) each iteration.
    `forward` returns the reference's two-element list [sigmoid(-res), sigmoid(-res_p)],
    each [B*N, 1]: res = mlp(S_v(m)) + x (check rows: mlp(0) + x_c), res_p = mlp(S_c(m_p))
    (variable rows: mlp(0)), m_p = the edge states after ggc1 of the last iteration (the
    script keys that on its module-global Nc; here on self.Nc, the same when they agree)."""
    kind = 'v30'

    def __init__(self, Nc, H):
        super().__init__(Nc, H)
        self.ggc1 = GraphConvV30('source_to_target')
        self.ggc2 = GraphConvV30('target_to_source')
        self.mlp = _mlp(1, 10, torch.nn.ReLU(), torch.float64)

    def packed_weights(self):
        return torch.cat(_flat_mlp(self.ggc1.mlp1) + _flat_gru(self.ggc1.rnn1)
                         + _flat_mlp(self.ggc2.mlp2) + _flat_gru(self.ggc2.rnn2)
                         + _flat_mlp(self.mlp))

    def forward(self, data):
        x, edge_index = data.x, data.edge_index
        if x.dim() == 1:
            x = x.unsqueeze(1)
        if self.fused_ok(x, edge_index):
            g = self.graph(x.device)
            out = ops.decode(g, self.kind, x, self.Nc, self.prepared_weights(x.dtype, x.device))
            n = out.size(0) // 2
            return [out[:n], out[n:]]
        if not x.is_cuda:
            raise RuntimeError('gnndecode runs on the GPU only (HIP/gfx950); move data to cuda')
        self.graph(x.device)
        return self.forward_layers(x, edge_index)

    def forward_layers(self, x, ei):
        ei = self._shifted(ei)
        m = torch.zeros(ei.size(1), 1, dtype=x.dtype, device=x.device)
        m_p = m
        for i in range(self.Nc):
            m = self.ggc1(m, ei, x)
            if i == self.Nc - 1:
                m_p = m
            m = self.ggc2(m, ei, x)
        n = x.size(0)
        mdt = self.mlp[0].weight.dtype
        s_v = torch.zeros(n, 1, dtype=m.dtype, device=m.device).index_add_(0, ei[0], m)
        s_c = torch.zeros(n, 1, dtype=m.dtype, device=m.device).index_add_(0, ei[1], m_p)
        res = _apply_mlp(self.mlp, s_v.to(mdt)).to(x.dtype) + x
        res_p = _apply_mlp(self.mlp, s_c.to(mdt)).to(x.dtype)
        return [torch.sigmoid(-res), torch.sigmoid(-res_p)]


def _toric_types(H):
    """Edge types of a toric H (codes.toric_edge_types), or None if H is not toric_code(L)."""
    from . import codes
    V, C = H.shape
    L = int(round((V / 4) ** 0.5))
    if L < 2 or 4 * L * L != V or 2 * L * L - 2 != C:
        return None
    if not torch.equal(H.to(torch.uint8), torch.as_tensor(codes.toric_code(L)).to(torch.uint8)):
        return None
    return torch.as_tensor(codes.toric_edge_types(L))


class DecoderV22(_WeightedBP):
    """quantum/decoder_v2_2.py:299-347 (Nc = 25, toric L = 6 in the script): neural BP with
    the per-layer weights W, W_p, the readout W, W_pr shared by the 8 edge types (the script's
    one-hot `feat_onehot` from H_prime; `edge_types` [E] in reference edge order, default
    codes.toric_edge_types for a toric H) and residual m_p @ sigmoid(weight).  `forward`
    returns the script's list of Nc per-layer readouts sigmoid(-(S_v(m_t W) + S_v(x W_pr))),
    each [B*V, 1]; the fused decoder computes all of them in one launch."""
    kind = 'v22'

    def __init__(self, Nc, H, edge_types=None):
        _Decoder.__init__(self, Nc, H)
        self.E = int(self.H.sum())
        types = _toric_types(self.H) if edge_types is None else torch.as_tensor(edge_types)
        if types is None:
            raise ValueError('DecoderV22 needs edge_types [E] for a non-toric H')
        types = types.to(torch.long).reshape(-1)
        if types.numel() != self.E or int(types.min()) < 0 or int(types.max()) > 7:
            raise ValueError('edge_types must hold E values in [0, 8)')
        layers = []
        for _ in range(Nc):
            layers.append(GraphConvV22('source_to_target', types))
            layers.append(GraphConvV22('target_to_source', types))
        self.layers = torch.nn.Sequential(*layers)
        self.register_buffer('types', types, persistent=False)
        self.W = torch.nn.Parameter(torch.ones(8, 1, dtype=torch.float64))
        self.W_pr = torch.nn.Parameter(torch.ones(8, 1, dtype=torch.float64) * 0.5)
        self.weight = torch.nn.Parameter(torch.full((1, 1), -4.0, dtype=torch.float64))

    def packed_weights(self):
        """gnnd.h V22 layout: the NBP per-edge tables with every type weight expanded."""
        t = self.types.to(self.W.device)
        per = [torch.cat([self.layers[2 * i].W[t].reshape(-1), self.layers[2 * i].W_p[t].reshape(-1)])
               for i in range(self.Nc)]
        return torch.cat(per + [self.W[t].reshape(-1), self.W_pr[t].reshape(-1),
                                torch.sigmoid(self.weight).reshape(-1)])

    def fused_ok(self, x, edge_index):
        """The fused decoder_v2_2 kernel runs on register-resident plans only (its per-layer
        readout list); a plan that is not resident (utilisation below 0.5, fp64 items beyond
        the residency budget, GNND_NO_RESIDENT / GNND_NO_F64_RESIDENT) takes the layer path."""
        if not super().fused_ok(x, edge_index):
            return False
        key = ('resident', str(x.device), x.dtype)
        ok = self._plan_ok.get(key) if hasattr(self, '_plan_ok') else None
        if ok is None:
            if not hasattr(self, '_plan_ok'):
                self._plan_ok = {}
            plan = ops.decode_plan(self.graph(x.device), self.kind, x.dtype)
            ok = self._plan_ok[key] = plan['kernel'] == 'decode_resident_kernel'
        return ok

    def forward(self, data):
        from . import _lib
        x, edge_index = data.x, data.edge_index
        if x.dim() == 1:
            x = x.unsqueeze(1)
        if self.fused_ok(x, edge_index):
            g = self.graph(x.device)
            try:
                out = ops.decode(g, self.kind, x, self.Nc, self.prepared_weights(x.dtype, x.device))
                return list(out.chunk(self.Nc, 0)) if self.Nc else []
            except _lib.GnndError as e:          # not register-resident after all: layer path
                if e.status != _lib.ERR_UNSUPPORTED:
                    raise
        if not x.is_cuda:
            raise RuntimeError('gnndecode runs on the GPU only (HIP/gfx950); move data to cuda')
        self.graph(x.device)
        return self.forward_layers(x, edge_index)

    def forward_layers(self, x, ei):
        B = x.size(0) // (self.rows + self.cols)
        ei = self._shifted(ei)
        t = self.types.to(x.device)
        m = torch.zeros(ei.size(1), 1, dtype=x.dtype, device=x.device)
        alpha = torch.sigmoid(self.weight).to(x.dtype)
        results = []
        for i in range(0, len(self.layers), 2):
            m_p = m
            m = self.layers[i](m, ei, x)
            m = self.layers[i + 1](m, ei, x) + torch.matmul(m_p, alpha)
            results.append(m)
        prior = x[ei[0]].mul(self.W_pr[t].repeat(B, 1).to(x.dtype))
        sp = self._var_rows(self._var_sum(prior, ei, x.size(0)), B)
        w = self.W[t].repeat(B, 1).to(x.dtype)
        return [torch.sigmoid(-(self._var_rows(self._var_sum(r.mul(w), ei, x.size(0)), B) + sp))
                for r in results]


MODELS = {'v24': DecoderV24, 'qgnni': QGNNI, 'qbp': QuantumBP, 'cgnni': CGNNI, 'cbp': ClassicalBP,
          'nbp': NeuralBP, 'v10': DecoderV10, 'v30': DecoderV30, 'v22': DecoderV22}
DEFAULT_ITERS = {'v24': 15, 'qgnni': 25, 'qbp': 10, 'cgnni': 25, 'cbp': 25, 'nbp': 15, 'v10': 15,
                 'v30': 15, 'v22': 25}
