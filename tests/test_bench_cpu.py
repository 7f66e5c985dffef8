"""bench.py's CPU-baseline leg on CPU tensors (no GPU): the 1-thread oracle leg, the
all-cores leg (oracle/cpu_pool.py child process) and the reported fields."""
import numpy as np
import torch

import bench
import gnn_oracle as O


def test_cpu_baseline_fields_and_all_cores_leg(golden):
    from conftest import weights_of
    z = golden('cgnni_bch')
    H = golden('bch_63_45_graph')['H']
    w = {k: torch.from_numpy(np.array(v)) for k, v in weights_of(z).items()}
    B, V, C = 2048, 63, 18
    g = torch.Generator().manual_seed(0)
    llr = 4 + 2 * torch.randn(B, V, generator=g)
    x = torch.cat([llr, torch.zeros(B, C)], 1).reshape(-1, 1).float()
    out = torch.from_numpy(O.decode('cgnni', H, x.numpy(), 3, {k: v.numpy() for k, v in w.items()}))
    labels = torch.zeros(B * V, 1)

    import types
    G = types.SimpleNamespace(N=V + C, V=V)
    res = bench.cpu_baseline('cgnni', H, w, x, out, labels, G, 3, 2.0)
    assert res['value_1_thread'] > 0 and res['parity_hard_decision_mismatches'] == 0
    assert res['parity_max_abs_err'] == 0.0
    assert res['cpu_model'] is None or isinstance(res['cpu_model'], str)
    if bench.cpu_workers() > 1:
        assert res['value_all_cores'] and res['cores'] == bench.cpu_workers(), res['sample']
        assert res['value'] == res['value_all_cores']


def test_bench_module_names_resolve():
    """Every global name bench.py reads is bound somewhere in the module (a renamed constant
    used only on the GPU path would otherwise fail first in the driver's round-end run)."""
    import ast
    import builtins
    src = open(bench.__file__).read()
    tree = ast.parse(src)
    bound = {'__file__', '__name__'}
    for n in ast.walk(tree):
        if isinstance(n, (ast.FunctionDef, ast.ClassDef)):
            bound.add(n.name)
        elif isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
            bound.add(n.id)
        elif isinstance(n, ast.arg):
            bound.add(n.arg)
        elif isinstance(n, (ast.Import, ast.ImportFrom)):
            for a in n.names:
                bound.add((a.asname or a.name).split('.')[0])
        elif isinstance(n, ast.ExceptHandler) and n.name:
            bound.add(n.name)
    missing = sorted({n.id for n in ast.walk(tree)
                      if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load)
                      and n.id not in bound and not hasattr(builtins, n.id)})
    assert not missing, missing


def test_issue_model_is_a_lower_bound_on_committed_counts():
    """The cycle-weighted issue model on the committed per-class counts: the headline line's
    issue time stays below its measured kernel time (issue_frac <= 1)."""
    cls = bench.load_pmc_classes('cgnni_bch_63_45_T25_f32')
    assert cls is not None
    m = bench.issue_model(cls, 65536, 0.469e-3)
    assert 0.5 < m['issue_frac'] <= 1.0, m
    assert bench.TRANS_OPS_PER_S > 0


def test_launch_mode_option(monkeypatch):
    """--launch: auto by default (eager stream launches for the fused trainers, a captured graph
    for the torch Trainer); --no-graph still forces eager."""
    import sys
    monkeypatch.setattr(sys, 'argv', ['bench.py'])
    a = bench.parse()
    assert a.launch == 'auto' and not a.no_graph
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--mode', 'train', '--launch', 'graph'])
    assert bench.parse().launch == 'graph'
