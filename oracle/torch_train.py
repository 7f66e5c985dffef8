"""ORACLE — test/measurement infrastructure only: a CPU torch-autograd restatement of the
reference's decoder_v2_4 training step, the `cpu_baseline` of `bench.py --mode train`.

quantum/decoder_v2_4.py:320-348 trains with torch autograd: GNNI.forward (:272-294, the
T-iteration loop of A2-A7), LossFunc (:297-317, the summed |sin| syndrome + logical loss),
`loss.backward()` and Adam(lr 3e-4, weight_decay 1e-9).  This module restates that step
vectorised over the batch on the single-graph structure (index_add in edge order for the
scatter sums, the same MLP shapes and Softplus), so a CPU core runs the reference's own
arithmetic without its O(B) torch.cat loops.  Checked against the reference-generated
training goldens (tests/test_oracle_golden.py).  Only bench.py's cpu_baseline and tests/
use it; the product package never does.
"""
import numpy as np
import torch
import torch.nn.functional as F

from gnn_oracle import tanner_edges


class V24Step:
    """One decoder_v2_4 training step on CPU: forward, reference loss, backward, Adam."""

    def __init__(self, H, logical, weights, T, dtype=torch.float64, lr=3e-4, weight_decay=1e-9):
        H = np.asarray(H)
        self.V, self.C = H.shape
        v, c = tanner_edges(H)
        self.v, self.c = torch.from_numpy(v), torch.from_numpy(c)
        self.E, self.T, self.dt = v.size, T, dtype
        self.Ht = torch.as_tensor(H.T, dtype=dtype)                   # [C, V]
        self.Lg = torch.as_tensor(np.asarray(logical), dtype=dtype)   # [4, V]
        self.p = {k: torch.as_tensor(np.asarray(a), dtype=dtype).clone().requires_grad_(True)
                  for k, a in weights.items()}
        self.opt = torch.optim.Adam(list(self.p.values()), lr, weight_decay=weight_decay)

    def _mlp(self, pre, u):
        h = F.softplus(F.linear(u, self.p[pre + '0.weight'], self.p[pre + '0.bias']))
        return F.linear(h, self.p[pre + '2.weight'], self.p[pre + '2.bias'])[..., 0]

    def _sum(self, m, idx, n):
        return torch.zeros(m.size(0), n, dtype=m.dtype).index_add_(1, idx, m)

    def forward(self, x):
        """x [B*N, 1] -> P(bit = 1) [B, V] (quantum/decoder_v2_4.py:272-294)."""
        N = self.V + self.C
        x = x.reshape(-1, N)
        xv, xc = x[:, :self.V], x[:, self.V:]
        m = torch.zeros(x.size(0), self.E, dtype=self.dt)
        for _ in range(self.T):
            m_p = m
            ext = self._sum(m, self.v, self.V)[:, self.v] - m
            a = self._mlp('ggc1.mlp.', torch.stack([ext, xv[:, self.v]], -1))
            t = torch.tanh(a / 2)
            u = self._sum(t, self.c, self.C)[:, self.c] - t
            m = self._mlp('ggc2.mlp.', u[..., None]) * xc[:, self.c] + m_p
        r = self._sum(self._mlp('mlp.', m[..., None]), self.v, self.V) + xv
        return torch.sigmoid(-r)

    def loss(self, pred, y):
        """quantum/decoder_v2_4.py:304-317: sum |sin(pi/2 H^T(y+p))| + |sin(pi/2 L(y+p))|."""
        e = (pred + y.reshape(pred.shape)).t()                         # [V, B]
        return torch.abs(torch.sin(self.Ht @ e * (np.pi / 2))).sum() + \
            torch.abs(torch.sin(self.Lg @ e * (np.pi / 2))).sum()

    def step(self, x, y):
        self.opt.zero_grad()
        pred = self.forward(x)
        loss = self.loss(pred, y)
        loss.backward()
        self.opt.step()
        return float(loss.detach())
