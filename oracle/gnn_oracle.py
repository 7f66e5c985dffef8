"""ORACLE — test infrastructure only.  CPU (numpy) restatement of the reference hot path.

This module is the CHECKER for the HIP path.  Only `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg may import it; the product package (`gnn-decode_amd/gnndecode`)
never does, and has no CPU fallback.

It restates, in vectorised numpy, the `MessagePassing.propagate()` T-iteration decode loop of
ironmanaudi/GNN-decode (paths relative to /root/reference/GNN-decode/):

* `propagate()`           quantum/decoder_v2_4.py:85-148, quantum/QGNNI.py:54-116,
                          quantum/BP.py:54-124, classical/CGNNI.py:52-112, classical/BP.py:52-123
* `scatter_`              quantum/decoder_v2_4.py:34-51 (PyG-1.x utils.scatter_ replica),
                          local `scatter_mean` quantum/decoder_v2_4.py:27-31
* `GNNI.forward()`        classical/CGNNI.py:259-284, classical/BP.py:239-259,
                          quantum/BP.py:199-219, quantum/QGNNI.py:228-252,
                          quantum/decoder_v2_4.py:272-294
* `update()` MLPs         classical/CGNNI.py:238-242, quantum/QGNNI.py:207-214,
                          quantum/decoder_v2_4.py:253-257
* weighted ("neural") BP  quantum/neural_BP.py:59-143 (propagate), :236-314 (layers, GNNI);
                          quantum/decoder_v1_0.py:60-133, :236-313
* GRU edge-state GNN      quantum/decoder_v3_0.py:59-122 (propagate), :199-290 (layers, GNNI)

Parity pinning: every function here is checked against golden vectors produced by running the
reference's own class definitions (tests/golden/make_golden.py) in tests/test_oracle_golden.py.
Aggregations use `np.add.at`, which accumulates sequentially in edge order — the order of
CPU torch_scatter / `index_add_` — so leave-one-out sums match the reference bit for bit up
to the BLAS summation order inside the MLPs.

Batch layout (A10): graph-major.  `x` is [B*N, 1] with N = V + C per codeword
(variable rows first, then check rows), output is [B*V, 1].
"""
import numpy as np

SCRIPTS = ('v24', 'qgnni', 'qbp', 'cgnni', 'cbp', 'nbp', 'v10', 'v30', 'v22')


def tanner_edges(H):
    """Single-codeword edge list of H [V, C], sorted by (v, c) like `H.to_sparse()._indices()`
    (quantum/decoder_v2_4.py:164-165, classical/CGNNI.py:153-154)."""
    v, c = np.nonzero(np.asarray(H))
    return v.astype(np.int64), c.astype(np.int64)


def batched_edge_index(H, B):
    """PyG-1.x collation (node offset b*N) followed by GNNI.forward's check shift by V
    (quantum/decoder_v2_4.py:277)."""
    V, C = np.asarray(H).shape
    N = V + C
    v, c = tanner_edges(H)
    off = np.repeat(np.arange(B, dtype=np.int64) * N, v.size)
    return np.stack([np.tile(v, B) + off, np.tile(c, B) + V + off])


# ---------------------------------------------------------------------------------------
# scatter_ / propagate (operator level)
# ---------------------------------------------------------------------------------------
def scatter_(name, src, index, dim_size):
    """PyG-1.x `scatter_` (quantum/decoder_v2_4.py:34-51): add / local leave-one-out mean /
    max with fill -1e9 mapped to 0."""
    src = np.asarray(src)
    out_shape = (dim_size,) + src.shape[1:]
    if name == 'add':
        out = np.zeros(out_shape, src.dtype)
        np.add.at(out, index, src)
        return out
    if name == 'mean':   # the local scatter_mean is already gathered & leave-one-out (:27-31)
        s = np.zeros(out_shape, src.dtype)
        np.add.at(s, index, src)
        cnt = np.zeros(out_shape, src.dtype)
        np.add.at(cnt, index, np.ones_like(src))
        num = s[index] - src
        den = np.maximum(cnt[index] - 1, 1)
        return num / den
    if name == 'max':
        out = np.full(out_shape, -1e9, src.dtype)
        np.maximum.at(out, index, src)
        out[out == src.dtype.type(-1e9)] = 0
        return out
    raise ValueError(name)


def _extrinsic(aggr, src, idx, dim_size):
    """`scatter_(aggr, out, idx, dim_size)[idx] - out` (quantum/decoder_v2_4.py:136,138).
    For 'mean' the reference's scatter_mean already returns the gathered leave-one-out
    mean, which is then indexed again by `[idx]` — restated literally."""
    agg = scatter_(aggr, src, idx, dim_size)
    return agg[idx] - src


def propagate(script, flow, aggr, edge_index, msg, extra, dim_size):
    """Bare `MessagePassing.propagate(edge_index, extra, size=(dim_size,)*2, x=msg)` with the
    base class's identity `message`/`update`, per reference script variant:

    * v24   quantum/decoder_v2_4.py:132-146  (c->v tanh(x/2); both flows cat extra[idx_j])
    * qgnni quantum/QGNNI.py:101-114         (c->v tanh(x/2), cat; v->c + extra)
    * qbp   quantum/BP.py:101-121            (c->v log-domain BP with syndrome; v->c + extra)
    * cgnni classical/CGNNI.py:99-110        (c->v tanh(x/2); `post` added if not None)
    * cbp   classical/BP.py:99-121           (c->v log-domain BP; v->c + extra)
    * nbp   quantum/neural_BP.py:108-131     (c->v BP without the +-10 pre-clamp, p clamp
                                              1 - 1e-15; v->c cat extra[idx_j])
    * v10   quantum/decoder_v1_0.py:109-131  (c->v as nbp; v->c + extra)
    * v30   quantum/decoder_v3_0.py:106-118  (no pre-op on either side; both flows cat)
    """
    ei = np.asarray(edge_index)
    i, j = (0, 1) if flow == 'target_to_source' else (1, 0)
    idx = ei[j]
    out = np.asarray(msg)
    dt = out.dtype.type
    if script in ('nbp', 'v10'):
        if flow == 'target_to_source':
            return _nbp_check_literal(aggr, out, extra[idx], idx, dim_size)
        out = _extrinsic(aggr, out, idx, dim_size)
        if script == 'v10':
            return out + extra[idx]
        return np.concatenate([out, extra[idx]], axis=1)
    if script in ('qbp', 'cbp') and flow == 'target_to_source':
        lo = 1e-20 if script == 'qbp' else 1e-7
        hi = 1 - 1e-12 if script == 'qbp' else 1 - 1e-7
        out = np.clip(out, dt(-10), dt(10))
        out = np.tanh(out / dt(2))
        coeff = np.where(out < 0, dt(1), dt(0))
        out = np.abs(out)
        out = np.clip(out, dt(lo), dt(1e10))
        out = np.log(out)
        out = _extrinsic(aggr, out, idx, dim_size)
        coeff = _extrinsic(aggr, coeff, idx, dim_size)
        if script == 'qbp':
            coeff = np.cos(dt(np.pi) * (coeff + (dt(1) - extra[idx]) / dt(2)))
        else:
            coeff = np.cos(dt(np.pi) * coeff)
        out = np.exp(out) * coeff
        out = np.clip(out, dt(-hi), dt(hi))
        if script == 'qbp':
            out = np.log(dt(1) + out) - np.log(dt(1) - out)
        else:
            out = np.log((dt(1) + out) / (dt(1) - out))
        return out
    if flow == 'target_to_source' and script != 'v30':
        out = np.tanh(out / dt(2))
    out = _extrinsic(aggr, out, idx, dim_size)
    if script in ('qbp', 'cbp'):                       # v->c
        return out + extra[idx]
    if script == 'cgnni':
        return out if extra is None else out + extra[idx]
    if script == 'qgnni' and flow == 'source_to_target':
        return out + extra[idx]
    return np.concatenate([out, extra[idx]], axis=1)  # v24, v30 both flows, qgnni c->v


def _nbp_check_literal(aggr, a, s_e, idx, dim_size):
    """c->v step of quantum/neural_BP.py:109-122 / quantum/decoder_v1_0.py:109-122 (same
    text): tanh(a/2) with NO pre-clamp, sign count, log|t| clamped to [1e-20, 1e10],
    leave-one-out sums at the check, cos(pi (n + (1 - s)/2)), p clamped to +-(1 - 1e-15),
    log(1 + p) - log(1 - p).  s_e = extra[idx_j] (syndrome +-1 at the edge's check)."""
    dt = a.dtype.type
    t = np.tanh(a / dt(2))
    coeff = np.where(t < 0, dt(1), dt(0))
    mag = np.log(np.clip(np.abs(t), dt(1e-20), dt(1e10)))
    lam = _extrinsic(aggr, mag, idx, dim_size)
    n = _extrinsic(aggr, coeff, idx, dim_size)
    p = np.exp(lam) * np.cos(dt(np.pi) * (n + (dt(1) - s_e) / dt(2)))
    p = np.clip(p, dt(-1 + 1e-15), dt(1 - 1e-15))
    return np.log(dt(1) + p) - np.log(dt(1) - p)


# ---------------------------------------------------------------------------------------
# per-edge MLPs (torch.nn.Linear: y = x W^T + b)
# ---------------------------------------------------------------------------------------
def linear(x, W, b):
    return x @ np.asarray(W, x.dtype).T + np.asarray(b, x.dtype)


def softplus(x, threshold=20.0):
    """torch.nn.Softplus(beta=1, threshold=20)."""
    with np.errstate(over='ignore'):
        return np.where(x > threshold, x, np.log1p(np.exp(np.minimum(x, threshold))))


def relu(x):
    return np.maximum(x, 0)


def mlp(w, prefix, x, act):
    h = linear(x, w[prefix + '0.weight'], w[prefix + '0.bias'])
    return linear(act(h), w[prefix + '2.weight'], w[prefix + '2.bias'])


def sigmoid(x):
    with np.errstate(over='ignore'):
        return 1 / (1 + np.exp(-x))


# ---------------------------------------------------------------------------------------
# whole-decoder restatements (single-graph structure, vectorised over the batch)
# ---------------------------------------------------------------------------------------
class _Graph:
    def __init__(self, H):
        H = np.asarray(H)
        self.V, self.C = H.shape
        self.N = self.V + self.C
        self.v, self.c = tanner_edges(H)
        self.E = self.v.size

    def sum_var(self, m):           # m [B, E] -> [B, V]
        out = np.zeros((m.shape[0], self.V), m.dtype)
        np.add.at(out, (slice(None), self.v), m)
        return out

    def sum_chk(self, m):
        out = np.zeros((m.shape[0], self.C), m.dtype)
        np.add.at(out, (slice(None), self.c), m)
        return out


def _split_x(g, x):
    x = np.asarray(x).reshape(-1, g.N)
    return x[:, :g.V], x[:, g.V:]


def _edge_mlp(w, prefix, u, act):
    """Row-wise MLP on a per-edge scalar (or stacked feature) tensor [..., F] -> [...]."""
    return mlp(w, prefix, u, act)[..., 0]


def decode_cgnni(H, w, x, T):
    """classical/CGNNI.py:259-284 (fp32, T=25)."""
    g = _Graph(H)
    xv, _ = _split_x(g, x)
    dt = xv.dtype.type
    m = np.zeros((xv.shape[0], g.E), xv.dtype)
    for _ in range(T):
        m_p = m
        a = g.sum_var(m)[:, g.v] - m + xv[:, g.v]                  # ggc1: v->c, post = x
        t = np.tanh(a / dt(2))                                       # ggc2: c->v
        u = g.sum_chk(t)[:, g.c] - t
        m = _edge_mlp(w, 'ggc2.mlp2.', u[..., None], relu) + m_p
    r = g.sum_var(m) + xv
    r = _edge_mlp(w, 'mlp.', r[..., None], relu)
    out = np.clip(sigmoid(-r), dt(1e-7), dt(1 - 1e-7))
    return out.reshape(-1, 1)


def _bp_check(g, a, s, quantum):
    dt = a.dtype.type
    lo = 1e-20 if quantum else 1e-7
    hi = 1 - 1e-12 if quantum else 1 - 1e-7
    t = np.tanh(np.clip(a, dt(-10), dt(10)) / dt(2))
    coeff = np.where(t < 0, dt(1), dt(0))
    mag = np.log(np.clip(np.abs(t), dt(lo), dt(1e10)))
    lam = g.sum_chk(mag)[:, g.c] - mag
    n = g.sum_chk(coeff)[:, g.c] - coeff
    if quantum:
        n = n + (dt(1) - s[:, g.c]) / dt(2)
    p = np.clip(np.exp(lam) * np.cos(dt(np.pi) * n), dt(-hi), dt(hi))
    if quantum:
        return np.log(dt(1) + p) - np.log(dt(1) - p)
    return np.log((dt(1) + p) / (dt(1) - p))


def decode_bp(H, x, T, quantum):
    """classical/BP.py:239-259 (fp32, clamp output) / quantum/BP.py:199-219 (fp64)."""
    g = _Graph(H)
    xv, xc = _split_x(g, x)
    dt = xv.dtype.type
    m = np.zeros((xv.shape[0], g.E), xv.dtype)
    for _ in range(T):
        a = g.sum_var(m)[:, g.v] - m + xv[:, g.v]
        m = _bp_check(g, a, xc, quantum)
    r = g.sum_var(m) + xv
    out = sigmoid(-r)
    if not quantum:
        out = np.clip(out, dt(1e-7), dt(1 - 1e-7))
    return out.reshape(-1, 1)


def decode_qgnni(H, w, x, T):
    """quantum/QGNNI.py:228-252 (fp64, T=25)."""
    g = _Graph(H)
    xv, xc = _split_x(g, x)
    dt = xv.dtype.type
    m = np.zeros((xv.shape[0], g.E), xv.dtype)
    for _ in range(T):
        m_p = m
        a = g.sum_var(m)[:, g.v] - m + xv[:, g.v]
        t = np.tanh(a / dt(2))
        u = g.sum_chk(t)[:, g.c] - t
        m = _edge_mlp(w, 'ggc2.mlp.', u[..., None], relu) * xc[:, g.c] + m_p
    r = g.sum_var(m) + xv
    return sigmoid(-_edge_mlp(w, 'mlp.', r[..., None], relu)).reshape(-1, 1)


def decode_v24(H, w, x, T):
    """quantum/decoder_v2_4.py:272-294 (fp64, T=15)."""
    g = _Graph(H)
    xv, xc = _split_x(g, x)
    dt = xv.dtype.type
    m = np.zeros((xv.shape[0], g.E), xv.dtype)
    for _ in range(T):
        m_p = m
        ext = g.sum_var(m)[:, g.v] - m
        a = _edge_mlp(w, 'ggc1.mlp.', np.stack([ext, xv[:, g.v]], axis=-1), softplus)
        t = np.tanh(a / dt(2))
        u = g.sum_chk(t)[:, g.c] - t
        m = _edge_mlp(w, 'ggc2.mlp.', u[..., None], softplus) * xc[:, g.c] + m_p
    r = g.sum_var(_edge_mlp(w, 'mlp.', m[..., None], softplus)) + xv
    return sigmoid(-r).reshape(-1, 1)


def _nbp_check(g, a, s):
    """_nbp_check_literal on the single-graph structure: a [B, E], s [B, C]."""
    dt = a.dtype.type
    t = np.tanh(a / dt(2))
    coeff = np.where(t < 0, dt(1), dt(0))
    mag = np.log(np.clip(np.abs(t), dt(1e-20), dt(1e10)))
    lam = g.sum_chk(mag)[:, g.c] - mag
    n = g.sum_chk(coeff)[:, g.c] - coeff
    p = np.exp(lam) * np.cos(dt(np.pi) * (n + (dt(1) - s[:, g.c]) / dt(2)))
    p = np.clip(p, dt(-1 + 1e-15), dt(1 - 1e-15))
    return np.log(dt(1) + p) - np.log(dt(1) - p)


def _edge_w(w, key, dt):
    return np.asarray(w[key], dt).reshape(-1)


def decode_nbp(H, w, x, T):
    """quantum/neural_BP.py:263-314 (fp64, Nc = 15).  Layer 2t (source_to_target,
    :245-260): m <- m * W (per edge), a = LOO_v(m) + x_v * W_p; layer 2t+1 (c->v, its W/W_p
    unused): BP check step; residual m = c2v + m_prev @ alpha.  Readout: sigmoid(-(sum_v
    m * W + sum_v x_v * W_p)) with the GNNI-level W, W_p."""
    g = _Graph(H)
    xv, xc = _split_x(g, x)
    dt = xv.dtype.type
    m = np.zeros((xv.shape[0], g.E), xv.dtype)
    alpha = dt(np.asarray(w['alpha'], dt).reshape(()))
    for t in range(T):
        m_p = m
        mw = m * _edge_w(w, f'layers.{2 * t}.W', dt)
        a = (g.sum_var(mw)[:, g.v] - mw) + xv[:, g.v] * _edge_w(w, f'layers.{2 * t}.W_p', dt)
        m = _nbp_check(g, a, xc) + m_p * alpha
    r = g.sum_var(m * _edge_w(w, 'W', dt)) + g.sum_var(xv[:, g.v] * _edge_w(w, 'W_p', dt))
    return sigmoid(-r).reshape(-1, 1)


def decode_v22(H, w, x, T):
    """quantum/decoder_v2_2.py:318-347 (fp64, Nc = 25): decode_nbp with every weight shared
    by edge type (`m.mul(feat_onehot) @ W` = m_e W[type(e)], :284, :292, :339, :342; types
    w['edge_types'] [E] in reference edge order), residual m_p @ sigmoid(weight) (:336), and
    the readout taken after EVERY layer pair (:337-346): returns the list of T arrays
    sigmoid(-(sum_v m_t W + sum_v x_v W_pr)), each [B*V, 1]."""
    g = _Graph(H)
    xv, xc = _split_x(g, x)
    dt = xv.dtype.type
    ty = np.asarray(w['edge_types']).reshape(-1).astype(np.int64)
    tw = lambda key: np.asarray(w[key], dt).reshape(-1)[ty]
    m = np.zeros((xv.shape[0], g.E), xv.dtype)
    alpha = sigmoid(np.asarray(w['weight'], dt).reshape(()))
    results = []
    for t in range(T):
        m_p = m
        mw = m * tw(f'layers.{2 * t}.W')
        a = (g.sum_var(mw)[:, g.v] - mw) + xv[:, g.v] * tw(f'layers.{2 * t}.W_p')
        m = _nbp_check(g, a, xc) + m_p * alpha
        results.append(m)
    sp = g.sum_var(xv[:, g.v] * tw('W_pr'))
    return [sigmoid(-(g.sum_var(r * tw('W')) + sp)).reshape(-1, 1) for r in results]


def decode_v10(H, w, x, T):
    """quantum/decoder_v1_0.py:282-313 (fp64, Nc = 15).  Layer 2t (source_to_target,
    :245-252): a = LOO_v(m) + x_v; layer 2t+1: a * W (per edge), BP check step; residual
    m = c2v + m_prev @ alpha.  Readout sigmoid(-(sum_v m + x_v))."""
    g = _Graph(H)
    xv, xc = _split_x(g, x)
    dt = xv.dtype.type
    m = np.zeros((xv.shape[0], g.E), xv.dtype)
    alpha = dt(np.asarray(w['alpha'], dt).reshape(()))
    for t in range(T):
        m_p = m
        a = g.sum_var(m)[:, g.v] - m + xv[:, g.v]
        m = _nbp_check(g, a * _edge_w(w, f'layers.{2 * t + 1}.W', dt), xc) + m_p * alpha
    r = g.sum_var(m) + xv
    return sigmoid(-r).reshape(-1, 1)


def gru_cell(w, prefix, inp, h):
    """torch.nn.GRUCell(1, 1)(inp, h) elementwise (ATen gru_cell: r = sig(h_r + i_r),
    z = sig(h_z + i_z), n = tanh(i_n + r h_n), h' = (h - n) z + n)."""
    dt = inp.dtype
    wi = np.asarray(w[prefix + 'weight_ih'], dt).reshape(3)
    wh = np.asarray(w[prefix + 'weight_hh'], dt).reshape(3)
    bi = np.asarray(w.get(prefix + 'bias_ih', np.zeros(3)), dt).reshape(3)
    bh = np.asarray(w.get(prefix + 'bias_hh', np.zeros(3)), dt).reshape(3)
    gi = [inp * wi[k] + bi[k] for k in range(3)]
    gh = [h * wh[k] + bh[k] for k in range(3)]
    r = sigmoid(gh[0] + gi[0])
    z = sigmoid(gh[1] + gi[1])
    n = np.tanh(gi[2] + r * gh[2])
    return (h - n) * z + n


def decode_v30(H, w, x, T):
    """quantum/decoder_v3_0.py:256-290 (fp64, Nc = 15).  Edge states m: ggc1 (:226-229)
    mes = mlp1([LOO_v(m), x_v]), m = rnn1(m, mes); m_p = m at the last iteration; ggc2
    mes = mlp2([LOO_c(m), x_c]), m = rnn2(m, mes).  Returns the two readout tensors
    [B*N, 1]: sigmoid(-(mlp(S_v(m)) + x)) and sigmoid(-mlp(S_c(m_p))) (zero sums on the
    other side's rows)."""
    g = _Graph(H)
    xv, xc = _split_x(g, x)
    B = xv.shape[0]
    m = np.zeros((B, g.E), xv.dtype)
    m_p = m
    for i in range(T):
        u = g.sum_var(m)[:, g.v] - m
        m = gru_cell(w, 'ggc1.rnn1.', m, _edge_mlp(w, 'ggc1.mlp1.', np.stack([u, xv[:, g.v]], -1), relu))
        if i == T - 1:
            m_p = m
        u = g.sum_chk(m)[:, g.c] - m
        m = gru_cell(w, 'ggc2.rnn2.', m, _edge_mlp(w, 'ggc2.mlp2.', np.stack([u, xc[:, g.c]], -1), relu))
    sv = np.concatenate([g.sum_var(m), np.zeros((B, g.C), m.dtype)], 1)
    sc = np.concatenate([np.zeros((B, g.V), m.dtype), g.sum_chk(m_p)], 1)
    xs = np.concatenate([xv, xc], 1)
    res = _edge_mlp(w, 'mlp.', sv[..., None], relu) + xs
    res_p = _edge_mlp(w, 'mlp.', sc[..., None], relu)
    return sigmoid(-res).reshape(-1, 1), sigmoid(-res_p).reshape(-1, 1)


def decode(model, H, x, T, w=None):
    if model == 'cgnni':
        return decode_cgnni(H, w, x, T)
    if model == 'cbp':
        return decode_bp(H, x, T, quantum=False)
    if model == 'qbp':
        return decode_bp(H, x, T, quantum=True)
    if model == 'qgnni':
        return decode_qgnni(H, w, x, T)
    if model == 'v24':
        return decode_v24(H, w, x, T)
    if model == 'nbp':
        return decode_nbp(H, w, x, T)
    if model == 'v10':
        return decode_v10(H, w, x, T)
    if model == 'v30':
        return decode_v30(H, w, x, T)
    if model == 'v22':
        return decode_v22(H, w, x, T)
    raise ValueError(model)


# ---------------------------------------------------------------------------------------
# metrics (quantum/neural_BP.py:338-348 hard FER rule; classical BER)
# ---------------------------------------------------------------------------------------
def hard_decisions(p):
    return (np.asarray(p) > 0.5).astype(np.uint8)


def toric_failures(H, logical, y, p_hat):
    """Residual-syndrome failure + logical failure counts for e + ê
    (quantum/neural_BP.py:338-348 rule).  H [V, C], logical [4, V]."""
    H = np.asarray(H, np.int64)
    V = H.shape[0]
    e = (np.asarray(y).reshape(-1, V).astype(np.int64) + hard_decisions(p_hat).reshape(-1, V)) % 2
    syn = (e @ H) % 2
    bad_syn = syn.any(axis=1)
    lg = (e @ np.asarray(logical, np.int64).T) % 2
    bad_log = (~bad_syn) & lg.any(axis=1)
    return int(bad_syn.sum()), int(bad_log.sum())
