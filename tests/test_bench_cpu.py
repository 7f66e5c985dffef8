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


def _full_size_record():
    """The round-4 default run's full record (20 KB, every nested field), widened to the round-5
    config list and an 8-rank job: the largest line the driver can see."""
    import json
    import os
    r = json.load(open(os.path.join(os.path.dirname(bench.__file__), 'profiles', 'r04',
                                    'bench_r04ad.json')))
    c = r['configs']
    c['config5_toric7_v24_train_b16'] = dict(c['config5_toric7_v24_train_global128'])
    c['config5_toric7_v24_train_b16_f64'] = dict(c['config5_toric7_v24_train_global128_f64'])
    # round 6: config 2 in bf16 and the BP decoders (transcendental-bound rooflines)
    c['config2_bch_cgnni_bf16'] = json.loads(json.dumps(r))
    c['config2_bch_cgnni_bf16'].pop('configs')
    for n in ('bp_bch_cbp_f32', 'bp_ldpc648_cbp_f32', 'bp_toric5_qbp_f64'):
        e = json.loads(json.dumps(c['config4_ldpc648_cgnni_shard']))
        e['roofline'].update(bound='transcendental', unit='Tops/s', frac_flop=0.1)
        c[n] = e
    assert set(c) == {n for n, _, _ in bench.SUB_CONFIGS}
    r['scaling_efficiency_global128'] = bench.strong_scaling(c)
    r['dist'] = {'backend': 'nccl', 'world_size': 8,
                 'ranks': [{'rank': i, 'device': i, 'host': 'h' * 24, 'pci_bus': 10 + i}
                           for i in range(8)]}
    return r


def test_driver_line_fits_and_keeps_every_config():
    """the stdout line stays <= 6 KB (the driver keeps the last 8 KB of
    stdout + stderr) and still carries value, roofline, cpu_baseline and parity per config."""
    import json
    r = _full_size_record()
    assert len(json.dumps(r)) > 15000                 # the uncompacted record would not fit
    s = bench.driver_line(r, 'gpurun_out/bench_full.json')
    assert len(s) <= bench.LINE_LIMIT
    line = json.loads(s)
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step',
              'higher_is_better', 'scaling', 'vs_baseline', 'dtype', 'config', 'roofline',
              'cpu_baseline'):
        assert k in line, k
    for k in ('bound', 'achieved', 'peak', 'unit', 'frac', 'traffic'):
        assert k in line['roofline'], k
    for k in ('value', 'unit', 'cores', 'kind'):
        assert k in line['cpu_baseline'], k
    assert set(line['configs']) == set(r['configs'])
    for name, e in line['configs'].items():
        assert e['value'] > 0 and e['ms_per_step'] > 0, name
        assert e['roofline']['frac'] > 0 and 'traffic' in e['roofline'], name
        assert e['roofline']['bound'], name
        if '_b16' not in name:          # (the per-GPU-16 points may shed their CPU legs)
            assert e['cpu_baseline']['value'] > 0, name
        assert e['parity'], name
    for n in ('bp_bch_cbp_f32', 'bp_ldpc648_cbp_f32', 'bp_toric5_qbp_f64'):
        assert line['configs'][n]['roofline']['bound'] == 'transcendental'
        assert line['configs'][n]['roofline']['frac_flop'] > 0
    assert line['dist']['world_size'] == 8 and len(line['dist']['ranks']) == 8
    assert line['scaling_efficiency_global128']['f32']['eff_8gpu'] > 0
    # a line over the limit sheds optional detail, never a contract field, and asserts
    tight = bench.driver_line(r, None, limit=len(s) - 50)
    assert len(tight) <= len(s) - 50 and 'cpu_baseline' in json.loads(tight)
    # far over: the contract fields alone, no exception after the whole run
    tiny = json.loads(bench.driver_line(r, 'f.json', limit=1500))
    assert tiny['value'] == line['value'] and tiny['full_record'] == 'f.json'
    assert 'roofline' in tiny and 'configs' not in tiny


def _rank_map_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    # a CPU stand-in for "this rank's GPU": device index = rank
    m = bench.rank_map(torch.device('cpu'))
    q.put((rank, m))
    dist.barrier()
    dist.destroy_process_group()


def test_rank_map_gathers_every_rank_gloo():
    """every rank's entry reaches every rank (all_gather_object), with the
    backend and world size as the process group reports them."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_map_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    for rank, m in res:
        assert m['backend'] == 'gloo' and m['world_size'] == 2
        assert [q_['rank'] for q_ in m['ranks']] == [0, 1]
    assert res[0][1] == res[1][1]
    single = bench.rank_map(torch.device('cpu'))
    assert single['world_size'] == 1 and single['ranks'][0]['rank'] == 0
