#!/usr/bin/env python3
"""Benchmark: codewords/s of the fused T-iteration GNN decode on MI355X (BASELINE.json metric).

Default workload = BASELINE.json configs[1]: BCH(63,45) Tanner-graph GNN decode
(classical/CGNNI.py architecture, T = 25), batch 65 536 codewords per GPU, synthetic AWGN
(SNR grid 1..6 dB), inputs resident in HBM before the timed region.  One "step" = one
launch of the fused decoder over the whole batch (all T iterations + readout).

Multi-GPU: one process per GPU (torchrun).  Codewords are independent, so every rank
decodes its own batch (weak scaling) with no data-path collective; ranks only barrier
around the timed region and all_reduce(MAX) the elapsed time.

Output: one JSON line on rank 0 (see DESIGN.md §Measurement for every field).
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'gnn-decode_amd'))

import gnndecode as gd  # noqa: E402

# Algorithmic FLOPs per codeword: per edge per iteration the v->c side
# costs 3 (variable sum, leave-one-out, + x) and the c->v side 55 (/2, check sum,
# leave-one-out, MLP 1->10->1 = 51, residual); readout 55 per variable.  Transcendentals
# (tanh, softplus) are counted separately and not included in FLOPs.
# Weighted BP (NBP/V10) adds the per-edge weight products and the residual to BP's 17.
# Second value: transcendental FUNCTIONS per codeword (tanh, softplus, exp, log); each needs
# at least two hardware transcendental ops (exp + log / rcp), which is what the
# transcendental roofline below prices.
def flops_per_codeword(model, g, T):
    E, V = g.E, g.V
    if model in ('cgnni', 'qgnni'):
        return 58 * E * T + 55 * V, E * T
    if model in ('cbp', 'qbp'):
        return 17 * E * T + 4 * V, 6 * E * T
    if model == 'nbp':
        return 22 * E * T + 4 * E + 4 * V, 6 * E * T
    if model == 'v22':           # nbp + a readout (2 E products/sums + sigmoid) every iteration
        return 26 * E * T + 4 * E * T + 4 * V * T, 6 * E * T + V * T
    if model == 'v10':
        return 20 * E * T + 4 * V, 6 * E * T
    if model == 'v24':
        return 1417 * E * T + 514 * E + 2 * V, 256 * E * T + 128 * E
    if model == 'v30':
        # per edge and iteration, both sides: leave-one-out 2, MLP 2->10->1 ReLU 71, GRUCell
        # 19 (+ 2 sigmoid, 1 tanh); readout MLP 1->10->1 (51) for both outputs of every node
        return 184 * E * T + 102 * g.N, 6 * E * T + 2 * g.N
    raise ValueError(model)


# Hardware transcendental ops (v_exp / v_log / v_rcp_f32) the fp32 BP check step issues per edge
# and iteration (decode_resident_kernel, ratio form since r06: E = 2^-|a'| and two v_log_f32 of
# D n_e +- N d_e; bp_ratio_msg).  The product form it replaced issued 5 (tanh = exp + rcp, the
# leave-one-out rcp, atanh = rcp + log) and the reference's formula 6 (tanh, log, exp, log of a
# quotient); the line reports the same throughput priced at those counts beside `frac`.
HW_TRANS_PER_EDGE = {'cbp': 3, 'qbp': 3}
TRANS_PER_EDGE_PRODUCT_FORM = 5
TRANS_PER_EDGE_REFERENCE = 6

PEAK_FP32_TFLOPS = 157.3      # MI355X_MICROARCH.md: FP32 vector = FP32 MFMA dense peak
PEAK_FP64_TFLOPS = 78.6
PEAK_HBM_GBS = 8000.0
PEAK_L2_GBS = 34500.0         # MI355X_MICROARCH.md § L2: ~34.5 TB/s aggregate (8 XCDs)
# fp64 decoder_v2_4 with channel-prior tables (gnnd_prepare_weights_priors): per edge and
# iteration the variable-side MLP is ONE 64-byte table cell (8 fp64 Taylor coefficients) read
# from the L2-resident tables (the check-side MLP one 96-byte LDS entry), per edge one
# readout-MLP cell
V24_TABLE_CELL_BYTES = 64


def parse():
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=1)
    p.add_argument('--steps', type=int, default=200)   # ~0.13 s timed: barrier jitter < 1 %
    p.add_argument('--warmup', type=int, default=10)
    p.add_argument('--prewarm-s', type=float, default=1.0,
                   help='decode mode: untimed seconds of steps before the W warm-up steps '
                        '(GPU clocks ramp over the first tens of ms of load; the K timed '
                        'steps then measure the steady state)')
    p.add_argument('--model', default=None, choices=list(gd.MODELS),
                   help='default: cgnni (decode: the headline), v24 (--mode train: config 5)')
    p.add_argument('--code', default='bch_63_45')
    p.add_argument('--batch', type=int, default=65536, help='codewords per GPU')
    p.add_argument('--iters', type=int, default=None)
    p.add_argument('--dtype', default='f32', choices=['f32', 'f64', 'bf16'],
                   help='bf16 (decode, classical models): bf16 x/out in HBM, fp32 arithmetic')
    p.add_argument('--cpu-seconds', type=float, default=12.0,
                   help='bounded CPU-baseline sample (0 disables)')
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--weights', default='auto', choices=['auto', 'random'],
                   help='auto: the shipped trained weights of this model/code when present '
                        '(gnndecode/weights/<model>_<code>.npz), else random init')
    p.add_argument('--no-graph', action='store_true',
                   help='train mode: eager steps instead of one captured HIP graph per step')
    p.add_argument('--launch', default='auto', choices=['auto', 'graph', 'eager'],
                   help='train mode: auto = eager stream launches for the fused trainers (three '
                        'kernels per step; a HIP graph replay leaves ~9 us idle between steps on '
                        'ROCm 7.2, eager launches none: profiles/r03/experiments/'
                        'train_graph_vs_eager_r03ac.txt), a captured graph for the torch Trainer'),
    p.add_argument('--layerwise', action='store_true',
                   help='train mode: the layer-by-layer operator path instead of the fused '
                        'decoder_v2_4 training kernels')
    p.add_argument('--torch-trainer', action='store_true',
                   help='train mode: torch autograd/optimizer Trainer around the fused kernels '
                        'instead of FusedV24Trainer')
    p.add_argument('--configs', default='auto', choices=['auto', 'on', 'off'],
                   help='decode mode: also time BASELINE configs 3-5 in the same process and nest '
                        'them under "configs" (auto: for the default headline workload)')
    p.add_argument('--priors', default='auto', choices=['auto', 'off'],
                   help='fp64 decoder_v2_4 decodes: tabulate the variable-side MLP per channel '
                        'prior of the batch (gnnd_prepare_weights_priors; auto) or not (off)')
    p.add_argument('--mode', default='decode', choices=['decode', 'train', 'sample'],
                   help='train = config 5: decoder_v2_4 (or --model qgnni/nbp/v10) training '
                        'step (DP, RCCL all-reduce); sample = the on-device input synthesis '
                        'kernel alone (gnnd_sample_*, HBM-write bound)')
    return p.parse_args()


# provenance of the shipped weights (gnn-decode_amd/gnndecode/weights/README.md)
WEIGHT_SOURCES = {
    'cgnni_bch_63_45': 'trained by tools/train_cgnni_bch.py',
    'cgnni_ldpc_648_324': 'trained by tools/train_cgnni_bch.py --code ldpc_648_324',
    'qgnni_toric_5': 'trained by tools/train_qgnni_toric.py',
    'v24_toric_5': 'reference checkpoint quantum/new_model/decoder_parameters_epoch67.pkl, converted',
}


def load_pmc(tag):
    """Committed rocprofv3 --pmc summary of this workload (profiles/pmc_<tag>.json) or {}."""
    path = os.path.join(ROOT, 'profiles', f'pmc_{tag}.json')
    if not os.path.exists(path):
        return {}
    try:
        with open(path) as f:
            return json.load(f)
    except Exception:
        return {}


# Issue model: a kernel's VALU issue time from its per-class instruction
# counts (rocprofv3 SQ_INSTS_VALU_* passes, tools/pmc_classes.sh; committed per codeword as
# profiles/pmc_classes_<tag>.json) times each class's issue cycles per wave64 instruction on one
# SIMD, over the 1 024 SIMDs at the 2.4 GHz peak engine clock; `issue_frac` = that time / the
# measured kernel time.  Cycles (MI355X_MICROARCH.md constants; ratios confirmed by
# tools/micro/issue_cost.hip, profiles/r03/issue_cost_r03f.txt): plain VOP2 fp32 / int / move 2,
# packed fp32 (v_pk_*) 4, fp64 add/mul/fma 4, fp32 transcendental 8, fp64 transcendental 16.
# The micro measured VOP3-encoded forms (v_fma_f32, v_bfe_u32, v_lshl_add_u64, a VOP3
# v_cndmask) at up to 2x their VOP2 cost and everything ~1.2x slower in ns than 2.4 GHz cycles,
# so the model is a LOWER bound on issue time: issue_frac <= 1 for a sound count, and the gap
# to 1 is issue slack plus VOP3 / clock effects.  FP32 FMA/ADD/MUL are split into packed and
# plain forms by SQ_INSTS_VALU_FLOPS_FP32 (a packed op counts twice); unclassified VALU
# (moves, DPP, selects, bit ops) at 2 cycles.
ISSUE_CYCLES = {'pk_f32': 4, 'fma_f32': 2, 'addmul_f32': 2, 'trans_f32': 8, 'f64': 4,
                'trans_f64': 16, 'int32': 2, 'int64': 4, 'cvt': 2, 'other': 2}
N_SIMDS = 256 * 4
CLOCK_HZ = 2.4e9
# Transcendental ops (v_exp/v_log/v_rcp_f32): 8 issue cycles per wave64 op per SIMD
# (MI355X_MICROARCH.md constants; measured 3.5 ns per op per SIMD-wave in
# tools/micro/issue_mix.hip = 18.7 T/s): 1024 SIMDs x 64 lanes / 8 cycles x 2.4 GHz.
TRANS_OPS_PER_S = N_SIMDS * 64 / ISSUE_CYCLES['trans_f32'] * CLOCK_HZ


def load_pmc_classes(tag):
    path = os.path.join(ROOT, 'profiles', f'pmc_classes_{tag}.json')
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def issue_model(cls, codewords, kernel_s):
    """Issue-time model of one launch over `codewords` from per-codeword class counts."""
    c = {k[len('SQ_INSTS_VALU_'):] if k != 'SQ_INSTS_VALU' else 'ALL': v * codewords
         for k, v in cls['per_codeword'].items() if k.startswith('SQ_INSTS_VALU')}
    g = lambda k: c.get(k, 0.0)
    fma, addmul = g('FMA_F32'), g('ADD_F32') + g('MUL_F32')
    scalar_flops = 2 * fma + addmul
    pk = min(1.0, max(0.0, g('FLOPS_FP32') / scalar_flops - 1.0)) if scalar_flops else 0.0
    f64 = g('ADD_F64') + g('MUL_F64') + g('FMA_F64')
    known = fma + addmul + g('TRANS_F32') + f64 + g('TRANS_F64') + g('INT32') + g('INT64') + g('CVT')
    other = max(0.0, g('ALL') - known)
    cy = ISSUE_CYCLES
    cycles = (pk * (fma + addmul) * cy['pk_f32'] +
              (1 - pk) * (fma * cy['fma_f32'] + addmul * cy['addmul_f32']) +
              g('TRANS_F32') * cy['trans_f32'] + f64 * cy['f64'] + g('TRANS_F64') * cy['trans_f64'] +
              g('INT32') * cy['int32'] + g('INT64') * cy['int64'] + g('CVT') * cy['cvt'] +
              other * cy['other'])
    t = cycles / N_SIMDS / CLOCK_HZ
    return {'issue_model_ms': t * 1e3, 'issue_frac': t / kernel_s, 'packed_fp32_frac': pk,
            'valu_insts_per_launch': g('ALL'),
            'unclassified_valu_frac': other / g('ALL') if g('ALL') else None,
            'counts_source': f"profiles/pmc_classes_{cls['tag']}.json ({cls['source']})",
            'cycles_per_wave64_inst': ISSUE_CYCLES,
            'note': 'lower bound on VALU issue time (VOP3 forms and the clock measured up to 2x / '
                    '1.2x slower, profiles/r03/issue_cost_r03f.txt)'}


def cpu_model():
    """`lscpu` "Model name" of this host (read from /proc/cpuinfo, no subprocess)."""
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.lower().startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_workers():
    """Worker processes for the all-cores leg: the cores this process may run on, capped at
    16 (the GPU box's CPU share per GPU; os.cpu_count() there shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(model, H, state, x_dev, out_dev, labels, g, T, seconds, out_bf16=False,
                 all_cores_leg=True, chunk=512):
    """Time the oracle (numpy restatement of the reference path) on a bounded sample of this
    workload: (1) one thread, comparing its outputs with the GPU's on the same codewords
    (parity, matched BER); (2) all cores: one single-threaded worker process per core
    (spawned, never forked from this GPU process) decoding further chunks of the same batch;
    (3) for the fp64 quantum scripts run in fp32 on the GPU, the fp32 oracle beside the fp64
    one.  `value` is the all-cores figure; the 1-thread figure and the CPU model sit beside it."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import numpy as np
    import gnn_oracle
    try:
        from threadpoolctl import threadpool_limits
        limiter = threadpool_limits(limits=1)
    except Exception:
        limiter = None
    w = {k: v.detach().cpu().numpy() for k, v in state.items()}
    x_all = x_dev.view(-1, g.N)
    o_all = out_dev.view(-1, g.V)
    # fp32 classical BP is ill-conditioned near its clamps: also decode the first chunks in
    # fp64 and count how often EACH fp32 implementation (GPU, numpy oracle) disagrees with it
    cond = model == 'cbp' and x_dev.dtype == torch.float32
    # the quantum scripts compute in fp64: their oracle (the reference's arithmetic) runs in
    # fp64 whatever the GPU dtype
    quantum = model in ('qbp', 'qgnni', 'v24', 'nbp', 'v10', 'v30', 'v22')

    def oracle_vars(xs_):
        r = gnn_oracle.decode(model, H, xs_, T, w)
        if model == 'v30':                 # first readout tensor, variable rows
            r = r[0].reshape(-1, g.N)[:, :g.V].reshape(-1, 1)
        if model == 'v22':                 # the last layer's readout
            r = r[-1]
        return r
    ref_dt = np.float64 if quantum else None
    t1 = seconds / 2                      # 1-thread leg, then the all-cores leg
    done, t_total, max_err, mism = 0, 0.0, 0.0, 0
    err_gpu = err_orc = 0
    c_bits = c_gpu = c_orc = 0
    while (t_total < t1 or done == 0) and done + chunk <= x_all.size(0):
        xs = x_all[done:done + chunk].cpu().numpy().reshape(-1, 1)
        if ref_dt is not None:
            xs = xs.astype(ref_dt)
        t0 = time.perf_counter()
        ref = oracle_vars(xs)
        t_total += time.perf_counter() - t0
        got = o_all[done:done + chunk].double().cpu().numpy().reshape(-1, 1)
        if out_bf16:       # the GPU stored its outputs in bf16: round the oracle's the same way
            ref = torch.from_numpy(np.ascontiguousarray(ref, np.float32)).bfloat16().double().numpy()
        ref = ref.astype(np.float64)
        max_err = max(max_err, float(np.abs(got - ref).max()))
        mism += int(((got > 0.5) != (ref > 0.5)).sum())
        lab = labels.view(-1, g.V)[done:done + chunk].double().cpu().numpy().reshape(-1, 1) > 0.5
        err_gpu += int(((got > 0.5) != lab).sum())
        err_orc += int(((ref > 0.5) != lab).sum())
        if cond and c_bits < 8 * chunk * g.V:
            r64 = gnn_oracle.decode(model, H, xs.astype(np.float64), T, w)
            c_bits += r64.size
            c_gpu += int(((got > 0.5) != (r64 > 0.5)).sum())
            c_orc += int(((ref > 0.5) != (r64 > 0.5)).sum())
        done += chunk
    one_thread = done / t_total if t_total > 0 else None
    same_prec = None
    if quantum and x_dev.dtype == torch.float32 and done:
        xs = x_all[:chunk].cpu().numpy().reshape(-1, 1)           # fp32 oracle, same chunk
        t0 = time.perf_counter()
        oracle_vars(xs)
        same_prec = chunk / (time.perf_counter() - t0)
    if limiter is not None and hasattr(limiter, 'unregister'):
        limiter.unregister()

    # all cores: single-threaded worker processes (oracle/cpu_pool.py, a child process that
    # forks its workers; this GPU process is never forked) over chunks of the same batch
    nw = cpu_workers()
    all_cores, sample_all = None, ''
    if nw > 1 and one_thread and all_cores_leg:
        import subprocess
        import tempfile
        per = max(1, int(one_thread * t1 / chunk))                 # ~t1 s of chunks per worker
        n_chunks = min(nw * per, x_all.size(0) // chunk)
        xs = x_all[:n_chunks * chunk].cpu().numpy().reshape(n_chunks, chunk * g.N, 1)
        if ref_dt is not None:
            xs = xs.astype(ref_dt)
        with tempfile.TemporaryDirectory() as td:
            sp = os.path.join(td, 'sample.npz')
            np.savez(sp, model=np.array(model), T=np.array(T), H=np.asarray(H, np.uint8), x=xs,
                     **{'w/' + k: v for k, v in w.items()})
            r = subprocess.run([sys.executable, os.path.join(ROOT, 'oracle', 'cpu_pool.py'), sp,
                                str(nw)], capture_output=True, text=True, timeout=600)
        if r.returncode == 0 and r.stdout.strip():
            pr = json.loads(r.stdout.strip().splitlines()[-1])
            all_cores = pr['codewords'] / pr['seconds']
            sample_all = (f"; all cores: {pr['codewords']} codewords on {nw} single-threaded "
                          f"worker processes in {pr['seconds']:.1f} s")
        else:
            sample_all = f'; all-cores leg failed: {r.stderr.strip()[-300:]}'
    res = {'value': all_cores if all_cores else one_thread, 'unit': 'codewords/s',
           'cores': nw if all_cores else 1, 'kind': 'port',
           'cpu_model': cpu_model(),
           'value_1_thread': one_thread,
           'value_all_cores': all_cores,
           'sample': f'{done} codewords of the same batch (chunks of {chunk}), oracle/gnn_oracle.py '
                     f'numpy restatement ({"fp64" if ref_dt is not None else str(x_dev.dtype)[6:]}), '
                     f'1 thread, {t_total:.1f} s' + sample_all,
           'parity_max_abs_err': max_err, 'parity_hard_decision_mismatches': mism,
           'parity_bits_compared': done * g.V,
           # "matched BER": bit error rate of the GPU and of the oracle on the same sample
           'sample_ber_gpu': err_gpu / max(1, done * g.V),
           'sample_ber_oracle': err_orc / max(1, done * g.V)}
    if same_prec is not None:
        res['value_1_thread_same_precision_f32'] = same_prec
    if cond:
        res['conditioning_vs_f64_oracle'] = {'bits': c_bits, 'gpu_f32_mismatches': c_gpu,
                                             'oracle_f32_mismatches': c_orc}
    return res


def train_cpu_baseline(H, model, T, x, y, batch, seconds):
    """The reference's training step restated in CPU torch autograd (oracle/torch_train.py,
    pinned to the reference-generated gradients) on the same data: 1 thread, then all the
    cores this host gives the process (torch intra-op threads).  Steps of the reference's
    BATCH_SIZE = 128 (quantum/decoder_v2_4.py:192), samples/s."""
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import torch_train
    w = {k: v.detach().cpu().double().numpy() for k, v in model.state_dict().items()}
    lg = gd.codes.toric_logicals(H)
    N, V = H.shape[0] + H.shape[1], H.shape[0]
    bs = min(128, batch)
    xs = x.view(-1, N)[:bs].detach().cpu().double().reshape(-1, 1)
    ys = y.view(-1, V)[:bs].detach().cpu().double()
    prev = torch.get_num_threads()
    res = {'unit': 'samples/s', 'kind': 'port', 'cpu_model': cpu_model()}
    for label, nt in (('1_thread', 1), ('all_cores', cpu_workers())):
        torch.set_num_threads(nt)
        st = torch_train.V24Step(H, lg, w, T)
        st.step(xs, ys)                                    # warm-up (allocator, page-in)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds / 2:
            st.step(xs, ys)
            n += 1
        res['value_' + label] = n * bs / (time.perf_counter() - t0)
        res['threads_' + label] = nt
    torch.set_num_threads(prev)
    res['value'] = res['value_all_cores']
    res['cores'] = res['threads_all_cores']
    res['sample'] = (f'oracle/torch_train.py V24Step (reference forward + LossFunc + backward + Adam, '
                     f'fp64 as the reference), steps of {bs} samples, ~{seconds / 2:.0f} s per leg')
    return res


def sample_main(a, world, rank, dev):
    """§8(f)1: the on-device input synthesis kernel alone (gnnd_sample_awgn with random
    codewords for classical codes, gnnd_sample_toric for toric codes), one launch per step
    over --batch codewords per GPU; each rank draws its slice of the global batch (offset =
    rank * batch).  HBM-write bound: (N + V) values written per codeword."""
    H = gd.codes.get_code(a.code)
    classical = not a.code.startswith('toric')
    dtype = torch.float64 if a.dtype == 'f64' else torch.float32
    if a.dtype == 'bf16':
        raise SystemExit('--mode sample writes f32 or f64')
    off = rank * a.batch

    def step():
        if classical:
            return gd.data.awgn_batch(H, a.batch, codewords='random', seed=a.seed, offset=off,
                                      device=dev, dtype=dtype)
        return gd.data.toric_batch(H, a.batch, seed=a.seed, offset=off, device=dev, dtype=dtype)

    for _ in range(max(a.warmup, 3)):
        step()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(a.steps):
        x, y = step()
    ev1.record()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_s = ev0.elapsed_time(ev1) / 1e3 / a.steps
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    if rank == 0:
        V, C = H.shape
        esz = 8 if dtype == torch.float64 else 4
        bytes_step = (V + C + V) * esz * a.batch
        achieved = bytes_step / kernel_s / 1e9
        print(json.dumps({
            'metric': 'synthesized codewords/sec (whole node), on-device decoder-input sampler',
            'value': world * a.batch * a.steps / elapsed, 'unit': 'codewords/s', 'n_gpus': world,
            'steps': a.steps, 'warmup': a.warmup, 'ms_per_step': elapsed / a.steps * 1e3,
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': a.dtype,
            'data': 'synthetic (Philox4x32-10 on device)',
            'config': {'workload': f'{a.code} {"AWGN random codewords" if classical else "toric gen_syn"} '
                                   f'sampler, batch={a.batch}/GPU',
                       'global_batch': a.batch * world, 'parallelism': f'dp{world} (offset shards)'},
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': PEAK_HBM_GBS, 'unit': 'GB/s',
                         'frac': achieved / PEAK_HBM_GBS, 'traffic': None,
                         'kernel': 'sample_awgn_kernel' if classical else 'sample_toric_kernel',
                         'bytes_written_per_launch': bytes_step, 'kernel_ms': kernel_s * 1e3},
            'cpu_baseline': None}), flush=True)


_ONE_RANK_GROUP = []


def one_rank_group(dev):
    """A 1-rank RCCL process group for the collective-inclusive training timing of a plain
    (non-torchrun) 1-GPU run; created once, destroyed at the end of main()."""
    if dist.is_initialized():
        return True
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1,
                            device_id=dev)
    _ONE_RANK_GROUP.append(True)
    return True


def drop_one_rank_group():
    """Destroy the 1-rank group right after the collective timing, so later configs are timed
    without a barrier / all_reduce inside their timed region."""
    if _ONE_RANK_GROUP and dist.is_initialized():
        dist.destroy_process_group()
        _ONE_RANK_GROUP.clear()


def v24_start_weights(model, code):
    """decoder_v2_4 training starts from the reference's checkpoint, as the script does
    (quantum/decoder_v2_4.py:322 loads decoder_parameters_epoch1.pkl before its Adam loop).
    The shipped epoch-67 checkpoint (quantum/new_model/decoder_parameters_epoch67.pkl, converted
    to weights/v24_toric_5.npz) has L-independent shapes (1 283 parameters), so it loads at any
    L.  Returns the weight source string."""
    wfile = os.path.join(ROOT, 'gnn-decode_amd', 'gnndecode', 'weights', 'v24_toric_5.npz')
    if not os.path.exists(wfile):
        return 'random init (seeded): weights/v24_toric_5.npz missing'
    z = np.load(wfile)                           # plain arrays (allow_pickle off)
    model.load_state_dict({k: torch.from_numpy(z[k]) for k in z.files})
    return (f'{os.path.relpath(wfile, ROOT)} (reference epoch-67 checkpoint, trained at L=5, '
            f'loaded at {code})')


TIMED_NS = [0, 0]       # monotonic-ns window of the last time_train_steps call


def time_train_steps(tr, data, y, steps, fused_tr):
    """K timed steps bracketed by barrier + synchronize; returns (elapsed max over ranks, host
    issue seconds, last loss tensor)."""
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    mono0 = time.monotonic_ns()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(steps):
        # the loss stays in the step's static buffer (read after the timed region), no copy
        loss = tr.step(data, y, copy_loss=False) if fused_tr else tr.step(data, y)
    ev1.record()
    # host time to issue the K steps (before the final synchronize): close to the wall time
    # per step means the step is host-bound (the GPU waits between steps)
    issue_s = time.perf_counter() - t0
    torch.cuda.synchronize()
    TIMED_NS[:] = [mono0, time.monotonic_ns()]
    if dist.is_initialized():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # GPU time of the K steps on the stream the trainers launch on (torch's current stream)
    gpu_s = ev0.elapsed_time(ev1) / 1e3
    t = torch.tensor([elapsed], dtype=torch.float64, device=y.device)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item()), issue_s, loss, gpu_s


def train_run(a, world, rank, dev, cpu='full'):
    """Config 5: decoder_v2_4 training on the toric code (default L=7), each rank a shard of
    size --batch, one flat all_reduce(SUM) of the gradient per step (gnndecode.train).
    decoder_v2_4 starts from the reference checkpoint (v24_start_weights).
    cpu='full' / 'parity': the CPU training baseline (oracle/torch_train.py), and for 'parity'
    also a K=10-step trajectory of the fused GPU trainer against the oracle's training steps
    on the same codewords; 'off'.  Returns the result dict on rank 0."""
    model_name = a.model if a.model in ('v24', 'qgnni', 'nbp', 'v10', 'v22', 'v30', 'cgnni') else 'v24'
    classical = model_name == 'cgnni'       # classical/CGNNI.py trains on a classical code
    code = a.code if (a.code.startswith('toric') or classical) else 'toric_7'
    T = a.iters or gd.DEFAULT_ITERS[model_name]
    dtype = torch.float64 if a.dtype == 'f64' else torch.float32
    H = gd.codes.get_code(code)
    torch.manual_seed(a.seed)
    model = gd.MODELS[model_name](T, H)
    wsrc = 'seeded reference init'
    if model_name == 'v24' and a.weights == 'auto':
        wsrc = v24_start_weights(model, code)
    model = model.to(dev).to(dtype)
    init_state = {k: v.detach().clone() for k, v in model.state_dict().items()}
    fused = (model_name in ('v24', 'v30', 'qgnni', 'cgnni') or
             (model_name in ('nbp', 'v22', 'v10') and dtype == torch.float64)) and not a.layerwise
    if model_name == 'v24':
        model.fused_train = fused
    if model_name == 'v22':          # decoder_v2_2's LossFunc: every layer's readout
        lf = gd.loss.PerLayerLoss(H, gd.codes.toric_logicals(H)).to(dev)
    elif model_name == 'v30':        # decoder_v3_0's LossFunc (two-output readout)
        lf = gd.loss.V30Loss(H).to(dev)
    elif classical:                  # classical/CGNNI.py LossFunc (BCE + syndrome term)
        lf = gd.loss.ClassicalLoss(H).to(dev)
    else:
        lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H),
                                  logical_only=(model_name == 'qgnni')).to(dev)
    parity = None
    if cpu == 'parity' and rank == 0 and model_name == 'v24' and fused and not a.torch_trainer:
        parity = train_trajectory(H, init_state, T, dev, dtype, a.seed)
    launch = getattr(a, 'launch', 'auto')
    if a.no_graph:
        launch = 'eager'
    fused_v24 = fused and model_name == 'v24' and not a.torch_trainer
    if launch == 'auto':
        # the fused V24 step is three kernels: eager stream launches leave no idle time between
        # steps, graph replays ~9 us (r03ac); the torch Trainer (~80 launches) keeps its graph
        launch = 'eager' if fused_v24 else 'graph'
    use_graph = launch == 'graph'
    if fused and model_name in ('nbp', 'v22', 'v10'):
        # packed per-edge weights -> fwd+tape -> syndrome loss -> reverse pass -> Adam (fp64)
        tr = gd.train.FusedWbpTrainer(model, lf, graph=use_graph, warmup=2)
    elif fused and model_name == 'v30':
        # fwd+tape -> reference LossFunc (torch) -> reverse pass -> [all_reduce] -> Adam
        tr = gd.train.FusedV30Trainer(model, lf, graph=use_graph, warmup=2)
    elif fused and model_name in ('qgnni', 'cgnni'):
        # fwd+tape -> reference LossFunc -> reverse pass -> [all_reduce] -> fused epilogue
        tr = gd.train.FusedGnnTrainer(model, lf, graph=use_graph, warmup=2)
    elif fused_v24:
        # fwd+tape (+ fused syndrome loss) -> reverse pass -> [all_reduce] -> fused epilogue
        tr = gd.train.FusedV24Trainer(model, lf, graph=use_graph, warmup=2)
    else:
        loss = (lambda p, yy: lf(p, yy, train=True)) if classical else lf
        tr = gd.train.Trainer(model, loss, graph=use_graph, warmup=2)   # captured after 2 eager steps
    if classical:                    # random codewords under AWGN (Gen_Data.AWGN)
        x, y = gd.data.awgn_batch(H, a.batch, codewords='random', seed=a.seed, offset=rank * a.batch,
                                  device=dev, dtype=dtype)
    else:
        x, y = gd.data.toric_batch(H, a.batch, seed=a.seed, offset=rank * a.batch, device=dev,
                                   dtype=dtype)
    data = gd.data.make_batch(x, model.graph(dev))
    for _ in range(a.warmup):
        tr.step(data, y)
    # the batch lives in the captured step's static input buffers (as an on-device sampler
    # writing there would): no per-step input copies
    st = tr.static_inputs()
    if st is not None:
        data.x, y = st
    fused_tr = isinstance(tr, (gd.train.FusedV24Trainer, gd.train.FusedV30Trainer,
                               gd.train.FusedWbpTrainer, gd.train.FusedGnnTrainer))
    elapsed, issue_s, loss, gpu_s = time_train_steps(tr, data, y, a.steps, fused_tr)
    timed_ns = list(TIMED_NS)
    # the same step with its RCCL all_reduce(SUM) of the flat gradient + loss actually issued:
    # N > 1 runs already contain it; a 1-GPU run times it on a 1-rank RCCL group
    # (force_collective), from the same starting weights on the same batch
    coll = None
    if fused_v24 and model_name == 'v24':
        if world > 1:
            coll = {'ms_per_step': elapsed / a.steps * 1e3, 'note': 'the timed step above (world > 1)'}
        elif getattr(a, 'collective', True):
            one_rank_group(dev)
            m2 = gd.MODELS['v24'](T, H).to(dev).to(dtype)
            m2.load_state_dict(init_state)
            tr2 = gd.train.FusedV24Trainer(m2, lf, graph=use_graph, warmup=2, force_collective=True)
            d2 = gd.data.make_batch(x, m2.graph(dev))
            for _ in range(a.warmup):
                tr2.step(d2, y)
            st2 = tr2.static_inputs()
            if st2 is not None:
                d2.x, y2 = st2
            else:
                y2 = y
            el2, iss2, _, _ = time_train_steps(tr2, d2, y2, a.steps, True)
            coll = {'ms_per_step': el2 / a.steps * 1e3, 'host_issue_ms_per_step': iss2 / a.steps * 1e3,
                    'note': 'FusedV24Trainer(force_collective=True) on a 1-rank RCCL group: '
                            'compute -> gnnd_train_update(rows -> flat gradient, loss) -> ONE '
                            'all_reduce(SUM) of [gradient | loss] -> gnnd_train_update(Adam)'}
            del tr2, m2
            drop_one_rank_group()
    if rank == 0:
        step_s = elapsed / a.steps
        roof = None
        if model_name in ('v24', 'v30', 'nbp', 'v22', 'v10', 'qgnni', 'cgnni') and fused:
            # training ~ 3x the forward's algorithmic FLOPs: forward, the
            # reverse pass through every MLP (2x); transcendentals: forward Softplus + the
            # backward sigmoid of every unit.  Whole step over its wall time per step.
            g = model.graph(dev)
            fl, trans = flops_per_codeword(model_name, g, T)
            peak = PEAK_FP32_TFLOPS if dtype == torch.float32 else PEAK_FP64_TFLOPS
            achieved = 3 * fl * a.batch / step_s / 1e12
            roof = {'bound': 'valu', 'achieved': achieved, 'peak': peak, 'unit': 'TFLOP/s',
                    'frac': achieved / peak, 'traffic': None,
                    'kernel': train_path_string(tr, model_name, use_graph),
                    'flops_per_sample': 3 * fl, 'transcendentals_per_sample': 2 * trans,
                    'step_ms': step_s * 1e3,
                    # event-timed GPU time per step (all the step's kernels, same stream)
                    'kernel_ms': gpu_s / a.steps * 1e3}
        cpu_res = None
        if model_name == 'v24' and a.cpu_seconds > 0 and world == 1 and cpu in ('full', 'parity'):
            cpu_res = train_cpu_baseline(H, model, T, x, y, a.batch, a.cpu_seconds)
        res = {
            'metric': f'training samples/sec (whole node), {model_name} step with RCCL grad all-reduce',
            'value': world * a.batch * a.steps / elapsed, 'unit': 'samples/s', 'n_gpus': world,
            'steps': a.steps, 'warmup': a.warmup, 'ms_per_step': elapsed / a.steps * 1e3,
            'timed_region_ns': timed_ns,
            'host_issue_ms_per_step': issue_s / a.steps * 1e3,
            'ms_per_step_with_collective': coll['ms_per_step'] if coll else None,
            'collective': coll,
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': a.dtype,
            'data': (f'synthetic {"AWGN random codewords" if classical else "toric errors"} '
                     f'(on-device sampler, seeded); start weights: {wsrc}'),
            'config': {'workload': f'{code} {model_name} training step, T={T}, batch={a.batch}/GPU',
                       'global_batch': a.batch * world, 'parallelism': f'dp{world}',
                       'last_loss': float(loss),
                       'params': sum(p.numel() for p in model.parameters()),
                       'hip_graph': use_graph,
                       'path': train_path_string(tr, model_name, use_graph),
                       'graph_components': model.graph(dev).components},
            'roofline': roof, 'cpu_baseline': cpu_res, 'parity': parity}
        return res
    return None


def train_path_string(tr, model_name, use_graph):
    """What one timed training step launches, from the trainer actually used."""
    how = 'one captured HIP graph per step' if use_graph else 'eager stream launches'
    if isinstance(tr, gd.train.FusedV24Trainer):
        fused_loss = any(tr._fuse_ok.values()) if tr._fuse_ok else False
        if fused_loss and tr.loss_in_forward:
            k = 'gnnd_train_fwd_loss (forward + tape + syndrome loss), gnnd_train_bwd_partial'
        elif fused_loss:
            k = 'gnnd_train_fwd (forward + tape), gnnd_train_bwd_loss_partial (reverse pass with the syndrome loss)'
        else:
            k = 'gnnd_train_fwd, gnnd_syndrome_loss, gnnd_train_bwd_partial'
        return f'FusedV24Trainer ({how}): {k}, gnnd_train_update (row reduction + loss + Adam + next weights)'
    if isinstance(tr, gd.train.FusedV30Trainer):
        return (f'FusedV30Trainer ({how}): gnnd_train_fwd (V30), V30Loss.loss_and_grad, '
                f'gnnd_train_bwd_partial, gnnd_train_update')
    if isinstance(tr, gd.train.FusedGnnTrainer):
        return (f'FusedGnnTrainer ({how}): gnnd_train_fwd ({model_name}), the reference LossFunc '
                f'and d loss / d pred, gnnd_train_bwd_partial, gnnd_train_update')
    if isinstance(tr, gd.train.FusedWbpTrainer):
        return (f'FusedWbpTrainer ({how}): packed weights, gnnd_train_fwd, gnnd_syndrome_loss, '
                f'gnnd_train_bwd, gnnd_adam_step')
    return f'Trainer ({how}): layer-by-layer propagate ops / fused forward, torch loss + Adam'


_TRAJ_CACHE = {}


def train_trajectory(H, init_state, T, dev, dtype, seed, n=64, K=10):
    """K training steps of the fused GPU trainer (FusedV24Trainer, eager) against the oracle's
    reference training step (oracle/torch_train.py V24Step, fp64: forward, LossFunc, backward,
    Adam lr 3e-4 wd 1e-9) from the same start weights on the same n seeded codewords; every
    step's two losses and the largest parameter difference after K steps.  Cached per dtype
    (the trajectory does not depend on the timed batch)."""
    key = (str(dtype), T, H.shape)
    if key in _TRAJ_CACHE:
        return dict(_TRAJ_CACHE[key], cached=True)
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import torch_train
    lg = gd.codes.toric_logicals(H)
    N, V = H.shape[0] + H.shape[1], H.shape[0]
    x, y = gd.data.toric_batch(H, n, seed=seed + 7, device=dev, dtype=dtype)
    m = gd.MODELS['v24'](T, H).to(dev).to(dtype)
    m.load_state_dict(init_state)
    lf = gd.loss.SyndromeLoss(H, lg).to(dev)
    # (rank 0 alone runs this check: LOCAL, so an N-rank job's trainer issues no collective)
    tr = gd.train.FusedV24Trainer(m, lf, graph=False, group=gd.train.LOCAL)
    data = gd.data.make_batch(x, m.graph(dev))
    gpu_losses = [float(tr.step(data, y)) for _ in range(K)]
    w = {k: v.detach().cpu().double().numpy() for k, v in init_state.items()}
    st = torch_train.V24Step(H, lg, w, T)
    xs, ys = x.view(-1, N).cpu().double().reshape(-1, 1), y.view(-1, V).cpu().double()
    t0 = time.perf_counter()
    ref_losses = [st.step(xs, ys) for _ in range(K)]
    osec = time.perf_counter() - t0
    sd = m.state_dict()
    pdiff = max(float((sd[k].detach().double().cpu() - st.p[k].detach()).abs().max()) for k in st.p)
    pscale = max(float(st.p[k].detach().abs().max()) for k in st.p)
    moved = max(float((st.p[k].detach() - torch.as_tensor(w[k])).abs().max()) for k in st.p)
    rel = [abs(a_ - b_) / max(1e-30, abs(b_)) for a_, b_ in zip(gpu_losses, ref_losses)]
    res = {'codewords': n, 'steps': K, 'loss_gpu': gpu_losses, 'loss_oracle_f64': ref_losses,
           'loss_max_rel_err': max(rel), 'param_max_abs_diff': pdiff, 'param_max_abs': pscale,
           'param_max_abs_change_oracle': moved,
           'oracle': 'oracle/torch_train.py V24Step (forward + LossFunc + backward + Adam, fp64)',
           'oracle_seconds': osec}
    _TRAJ_CACHE[key] = res
    return res


def decode_run(a, world, rank, dev, cpu='full'):
    """One decode workload (a.model / a.code / a.batch per GPU / a.dtype): K timed launches,
    BER/FER, roofline; cpu='full' times the oracle (1 thread + all cores), 'parity' a bounded
    oracle sample (1 thread, with matched-BER parity, + a short all-cores leg), 'off' none.  Returns the result
    dict on rank 0 (None elsewhere)."""
    T = a.iters or gd.DEFAULT_ITERS[a.model]
    # bf16: storage type of x / out only (classical models); weights and arithmetic fp32
    io_dtype = {'f32': torch.float32, 'f64': torch.float64, 'bf16': torch.bfloat16}[a.dtype]
    dtype = torch.float64 if a.dtype == 'f64' else torch.float32
    if a.dtype == 'bf16' and a.model not in ('cgnni', 'cbp'):
        raise SystemExit('--dtype bf16 is the classical models\' storage mode (cgnni, cbp)')

    H = gd.codes.get_code(a.code)
    torch.manual_seed(a.seed)
    model = gd.MODELS[a.model](T, H).to(dev).eval()
    wfile = os.path.join(ROOT, 'gnn-decode_amd', 'gnndecode', 'weights', f'{a.model}_{a.code}.npz')
    trained = a.weights == 'auto' and os.path.exists(wfile)
    if trained:
        z = np.load(wfile)                       # plain arrays (allow_pickle off)
        model.load_state_dict({k: torch.from_numpy(z[k]) for k in z.files})
    g = model.graph(dev)
    state = dict(model.state_dict())
    if a.model == 'v22':                         # the oracle takes the edge types with the weights
        state['edge_types'] = model.types
    classical = a.model in ('cgnni', 'cbp')
    # each rank draws its slice [rank*batch, (rank+1)*batch) of ONE global batch (Philox keyed
    # by the global codeword index): the all-reduced BER/FER counts of an N-GPU run equal a
    # single-GPU decode of the same N*batch codewords
    off = rank * a.batch
    if classical:
        # uniform random codewords (the CGNNI decoder is not symmetric under codeword
        # translation, so the reference's constant-word input would flatter it)
        x, labels = gd.data.awgn_batch(H, a.batch, codewords='random', seed=a.seed, offset=off,
                                       device=dev, dtype=dtype)
    else:
        x, labels = gd.data.toric_batch(H, a.batch, seed=a.seed, offset=off, device=dev, dtype=dtype)
    if io_dtype != dtype:
        x = x.to(io_dtype)                       # bf16 storage (outside the timed region)
    # fp64 decoder_v2_4: the batch's channel priors (one per codeword, the reference's p list)
    # registered before the timed region, so the prepared weights carry the variable-side MLP
    # per prior (setup work, like the weights themselves)
    n_priors = 0
    if a.model == 'v24' and dtype == torch.float64 and getattr(a, 'priors', 'auto') == 'auto':
        try:
            pri = gd.ops.channel_priors(g, x)
        except ValueError:
            pri = []
        model.set_channel_priors(pri)
        n_priors = len(pri)
    w = model.prepared_weights(dtype, dev)
    out = torch.empty(gd.ops.decode_out_rows(g, a.model, a.batch, T), 1, dtype=io_dtype, device=dev)

    def step():
        gd.ops.decode(g, a.model, x, T, w, out=out)

    t_pre = time.perf_counter()
    while time.perf_counter() - t_pre < a.prewarm_s:
        for _ in range(20):
            step()
        torch.cuda.synchronize()
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    mono0 = time.monotonic_ns()           # the profiler's clock: tools/prof_vs_line.py windows
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(a.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    mono1 = time.monotonic_ns()
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_s = ev0.elapsed_time(ev1) / 1e3 / a.steps        # HIP events, same stream
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    elapsed_decode_only = None
    if n_priors > 0:
        # The channel-prior tables depend on the weights and the channel's prior list only, but
        # the line's value does not take them as given: a second timed region rebuilds the
        # whole prepared layout (check-MLP table, prior tables, readout table:
        # gnnd_prepare_weights_priors) before EVERY decode, and `value` / `ms_per_step` are that
        # region's; the first region (decode launches only) gives the kernel's roofline.
        flat_dev = model.packed_weights().detach().to(device=dev, dtype=dtype).contiguous()
        pri_t = list(model._priors)

        def step_build():
            wt = gd.ops.prepare_weights(a.model, flat_dev, priors=pri_t)
            gd.ops.decode(g, a.model, x, T, wt, out=out)

        for _ in range(max(2, a.warmup)):
            step_build()
        torch.cuda.synchronize()
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize()
        mono0 = time.monotonic_ns()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step_build()
        torch.cuda.synchronize()
        mono1 = time.monotonic_ns()
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        if dist.is_initialized():
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed_decode_only, elapsed = elapsed, float(t.item())

    # hard-decision error rate of this batch (outside the timed region)
    with torch.no_grad():
        # one launch: bit errors, frame errors, residual-syndrome / logical failures (toric)
        lg = None if classical else (torch.as_tensor(gd.codes.toric_logicals(H)) != 0).to(torch.int32)
        pred = out.float() if io_dtype == torch.bfloat16 else out
        if a.model == 'v30':                     # variable rows of the first readout tensor
            pred = out[:a.batch * g.N].view(a.batch, g.N)[:, :g.V].reshape(-1, 1).contiguous()
        if a.model == 'v22':                     # the last layer's readout
            pred = out[-a.batch * g.V:]
        counts = gd.ops.decision_errors(g, lg, pred, labels)
        if dist.is_initialized():
            dist.all_reduce(counts)
        errs = counts[0]
        # uncoded reference point: hard decision on the channel LLR alone (classical codes)
        # (quantum: the error rate of not correcting at all, i.e. the fraction of flipped qubits)
        ch_errs = ((x.view(a.batch, g.N)[:, :g.V] < 0).reshape(-1, 1).to(labels.dtype) != labels).sum() \
            if classical else labels.sum()
        if dist.is_initialized():
            dist.all_reduce(ch_errs)
    ber = float(errs.item()) / (a.batch * g.V * world)
    cl = counts.tolist()
    fer = (cl[1] if classical else cl[2] + cl[3]) / (a.batch * world)
    ch_ber = float(ch_errs.item()) / (a.batch * g.V * world)

    if rank == 0:
        # SURVEY §8(d)'s algorithmic count: `frac` is always this fraction
        fl, trans = flops_per_codeword(a.model, g, T)
        achieved = fl * a.batch / kernel_s / 1e12
        peak = PEAK_FP32_TFLOPS if dtype == torch.float32 else PEAK_FP64_TFLOPS
        frac_alg = achieved / peak
        frac_sp = None
        if a.model == 'v24' and dtype == torch.float64:
            # fp64 has no hardware exp/log: the fraction with each Softplus priced at the fp64
            # FLOPs of a minimal table form (11 FMAs + 6 adds/muls = 28), reported beside it only
            frac_sp = (fl + 28 * trans) * a.batch / kernel_s / 1e12 / peak
        trans_frac = 2 * trans * a.batch / kernel_s / TRANS_OPS_PER_S
        # fp32 BP: the hardware transcendental ops (v_exp/v_log/v_rcp_f32) the kernel issues per
        # edge and iteration, at their 8-cycle issue rate: the binding roofline
        hw_ops = HW_TRANS_PER_EDGE.get(a.model) if dtype == torch.float32 else None
        trans_hw = None
        if hw_ops:
            ops_s = hw_ops * g.E * T * a.batch / kernel_s
            trans_hw = {'achieved': ops_s / 1e12, 'peak': TRANS_OPS_PER_S / 1e12, 'unit': 'Tops/s',
                        'frac': ops_s / TRANS_OPS_PER_S, 'ops_per_edge_iteration': hw_ops}
        esz = {torch.float32: 4, torch.float64: 8, torch.bfloat16: 2}[io_dtype]
        io_bytes = (g.N + gd.ops.decode_out_rows(g, a.model, 1, T)) * esz * a.batch
        plan = gd.ops.decode_plan(g, a.model, dtype)
        # (the prior-table kernel is another kernel: its PMC files carry their own tag)
        ptag = '_ptab' if n_priors > 0 else ''
        tag = f'{a.model}_{a.code}_B{a.batch}_T{T}_{a.dtype}{ptag}'
        pmc = load_pmc(tag)
        traffic = pmc.get('hbm_bytes_per_launch')
        cls = load_pmc_classes(f'{a.model}_{a.code}_T{T}_{a.dtype}{ptag}')
        res = {
            'metric': 'codewords/sec (whole node) at matched BER, T-iter GNN decode',
            'value': world * a.batch * a.steps / elapsed,
            'unit': 'codewords/s',
            'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup, 'prewarm_s': a.prewarm_s,
            'ms_per_step': elapsed / a.steps * 1e3, 'timed_region_ns': [mono0, mono1],
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            'dtype': a.dtype, 'data': 'synthetic (on-device AWGN/toric sampler, seeded); ' +
                                      ('trained weights' if trained else 'random-init weights'),
            'config': {'workload': f'{a.code} {a.model} decode, T={T}, batch={a.batch}/GPU',
                       'code': a.code, 'model': a.model, 'iters': T, 'batch_per_gpu': a.batch,
                       'global_batch': a.batch * world, 'parallelism': f'dp{world} (codeword shards)',
                       'codewords_per_workgroup': plan['cw'], 'lds_bytes_per_workgroup': plan['lds'],
                       'items_per_lane': plan['items_per_lane'],
                       'channel_prior_tables': n_priors,
                       'hard_decision_error_rate': ber,
                       # classical: codewords with a bit error; toric: residual-syndrome or
                       # logical failures (quantum/neural_BP.py:333-348)
                       'frame_error_rate': fer,
                       'channel_hard_decision_error_rate': ch_ber,
                       'weights': (f'{os.path.relpath(wfile, ROOT)} ({WEIGHT_SOURCES.get(a.model + "_" + a.code, "")})'
                                   if trained else 'random init (seeded)') +
                                  ': compute cost is weight-independent; BER parity vs the '
                                  'oracle is in cpu_baseline'},
            'roofline': {'bound': 'valu', 'achieved': achieved, 'peak': peak, 'unit': 'TFLOP/s',
                         'frac': frac_alg, 'traffic': traffic,
                         'kernel': f"{plan['kernel']}<{a.model}, {a.dtype}>",
                         # per-class VALU counts x measured per-class issue costs (ISSUE_NS)
                         'issue_model': issue_model(cls, a.batch, kernel_s) if cls else None,
                         'kernel_ms': kernel_s * 1e3,
                         'flops_per_codeword': fl, 'transcendentals_per_codeword': trans,
                         'frac_algorithmic_count': frac_alg,
                         'frac_softplus_priced_28flop': frac_sp,
                         # >= 2 hardware transcendental ops per function vs the 8-cycle issue
                         # rate (fp32; fp64 has no hardware transcendentals)
                         'transcendental_op_frac': trans_frac if dtype == torch.float32 else None,
                         'hbm_io_bytes_per_launch': io_bytes,
                         'hbm_io_frac': io_bytes / kernel_s / 1e9 / PEAK_HBM_GBS},
        }
        if n_priors > 0:
            # the table form: the kernel reads a table cell where the reference evaluates 128
            # hidden units, so the reference's FLOP count over the kernel time can exceed the
            # FP64 peak (frac_flop); the roofline is the table reads' L2 bandwidth
            tb = V24_TABLE_CELL_BYTES * g.E * (T + 1) * a.batch
            res['roofline'].update(bound='l2', achieved=tb / kernel_s / 1e9, peak=PEAK_L2_GBS,
                                   unit='GB/s', frac=tb / kernel_s / 1e9 / PEAK_L2_GBS,
                                   frac_flop=frac_alg, table_bytes_per_launch=tb,
                                   note='variable-side and readout MLPs from channel-prior tables '
                                        '(one 64-B cell per edge-iteration); frac_flop = the '
                                        "reference's FLOPs per codeword over the FP64 peak")
            res['table_build'] = 'per step (value, ms_per_step: prepare + decode every step)'
            res['ms_per_step_decode_only'] = elapsed_decode_only / a.steps * 1e3
            res['value_decode_only'] = world * a.batch * a.steps / elapsed_decode_only
        if trans_hw is not None:
            # transcendental-bound (fp32 BP): the binding roofline; the FLOP fraction beside it
            rf = res['roofline']
            rf.update(bound='transcendental', achieved=trans_hw['achieved'], peak=trans_hw['peak'],
                      unit=trans_hw['unit'], frac=trans_hw['frac'], frac_flop=frac_alg,
                      trans_ops_per_edge_iteration=hw_ops,
                      frac_at_product_form_ops=trans_hw['frac'] * TRANS_PER_EDGE_PRODUCT_FORM / hw_ops,
                      frac_at_reference_ops=trans_hw['frac'] * TRANS_PER_EDGE_REFERENCE / hw_ops)
        if a.cpu_seconds > 0 and world == 1 and cpu != 'off':
            # the oracle decodes the same (for bf16: widened) inputs in fp32
            res['cpu_baseline'] = cpu_baseline(a.model, H, state, x.to(dtype), pred, labels, g, T,
                                               a.cpu_seconds, out_bf16=io_dtype == torch.bfloat16,
                                               all_cores_leg=cpu in ('full', 'parity'),
                                               chunk=512 if cpu == 'full' else 128)
        else:
            res['cpu_baseline'] = None
        return res
    return None


# BASELINE.json configs[2..4] timed in the same process as the headline (configs[1]) and
# nested under "configs" of its JSON line: (name, mode, overrides).  Config 5's entries fix the
# GLOBAL batch (per-GPU batch = global / world): an N-GPU run of the driver then measures the
# strong scaling of the reference's batch directly (t_N(global) vs the 1-GPU line's t_1).
SUB_CONFIGS = [
    ('config3_toric5_v24_f64', 'decode', dict(model='v24', code='toric_5', batch=65536, dtype='f64',
                                              steps=10, warmup=2, prewarm_s=0.3)),
    # config 2 as BASELINE writes it: bf16 x / out in HBM, fp32 weights and arithmetic
    ('config2_bch_cgnni_bf16', 'decode', dict(model='cgnni', code='bch_63_45', batch=65536,
                                              dtype='bf16', steps=20, warmup=2, prewarm_s=0.3)),
    # the decoders SURVEY §8(d) names as the matched-BER references: classical BP
    # (classical/BP.py:231-259) on configs 1/2's BCH and config 4's LDPC, quantum BP
    # (quantum/BP.py:191-219) on config 3's toric-5 in the reference dtype
    ('bp_bch_cbp_f32', 'decode', dict(model='cbp', code='bch_63_45', batch=65536, dtype='f32',
                                      steps=20, warmup=2, prewarm_s=0.3)),
    ('bp_ldpc648_cbp_f32', 'decode', dict(model='cbp', code='ldpc_648_324', batch=131072, dtype='f32',
                                          steps=10, warmup=2, prewarm_s=0.3)),
    ('bp_toric5_qbp_f64', 'decode', dict(model='qbp', code='toric_5', batch=65536, dtype='f64',
                                         steps=20, warmup=2, prewarm_s=0.3)),
    ('config4_ldpc648_cgnni_shard', 'decode', dict(model='cgnni', code='ldpc_648_324', batch=131072,
                                                   dtype='f32', steps=20, warmup=2, prewarm_s=0.3)),
    # (200 / 100 timed steps: ~40 / ~120 ms, so the synchronize/barrier around the timed region
    # is < 0.2 % of it; 30 steps of a 0.21 ms step left ~1 %)
    ('config5_toric7_v24_train_global128', 'train', dict(model='v24', code='toric_7', gbatch=128,
                                                          dtype='f32', steps=200, warmup=5)),
    ('config5_toric7_v24_train_global1024', 'train', dict(model='v24', code='toric_7', gbatch=1024,
                                                           dtype='f32', steps=100, warmup=5)),
    # the reference's own precision (quantum/decoder_v2_4.py:237-243 .double() MLPs, :278 fp64
    # messages); the f32 entries above are the perf mode
    ('config5_toric7_v24_train_global128_f64', 'train', dict(model='v24', code='toric_7', gbatch=128,
                                                              dtype='f64', steps=200, warmup=5)),
    ('config5_toric7_v24_train_global1024_f64', 'train', dict(model='v24', code='toric_7',
                                                               gbatch=1024, dtype='f64', steps=50,
                                                               warmup=3)),
    # per-GPU batch 16 = the reference's global 128 over 8 GPUs: t1(128) / (8 t1(16)) is the
    # strong-scaling efficiency at the reference's batch (scaling_efficiency_global128)
    ('config5_toric7_v24_train_b16', 'train', dict(model='v24', code='toric_7', batch=16,
                                                   dtype='f32', steps=200, warmup=5)),
    ('config5_toric7_v24_train_b16_f64', 'train', dict(model='v24', code='toric_7', batch=16,
                                                       dtype='f64', steps=200, warmup=5)),
]


def sub_config_results(a, world, rank, dev):
    out = {}
    traj_done = set()
    for name, mode, ov in SUB_CONFIGS:
        sa = argparse.Namespace(**vars(a))
        for k, v in ov.items():
            setattr(sa, k, v)
        sa.iters, sa.weights, sa.seed = None, 'auto', a.seed
        sa.cpu_seconds = min(a.cpu_seconds, 2.0)
        t0 = time.perf_counter()
        if mode == 'train':
            # global-batch entries split the batch over the ranks; per-GPU entries keep it
            sa.batch = max(1, sa.gbatch // world) if 'gbatch' in ov else sa.batch
            sa.no_graph = sa.layerwise = sa.torch_trainer = False
            # the 10-step trajectory against the oracle runs once per dtype (it does not
            # depend on the timed batch); later entries of that dtype time the CPU leg only
            cpu = 'parity' if sa.dtype not in traj_done else 'full'
            traj_done.add(sa.dtype)
            r = train_run(sa, world, rank, dev, cpu=cpu)
        else:
            r = decode_run(sa, world, rank, dev, cpu='parity')
        if rank == 0:
            r['wall_s'] = time.perf_counter() - t0
            out[name] = r
    return out


# ---------------------------------------------------------------------------------------------
# The driver keeps only the last 8 KB of a run's stdout (+ stderr): the JSON line it parses must
# fit with room to spare.  The full record (every field above) goes to a file; stdout carries a
# compact line holding, per config, the value, the roofline, the CPU baseline and a parity
# summary.
LINE_LIMIT = 6144


def _r(v, sig=5):
    """Round a float to `sig` significant digits (ints, None and strings pass through)."""
    if isinstance(v, float) and math.isfinite(v) and v != 0.0:
        return float(f'{v:.{sig}g}')
    return v


def _pick(d, keys, sig=5):
    if not d:
        return None
    return {k: _r(d[k], sig) for k in keys if k in d and d[k] is not None}


def compact_parity(r):
    """Parity summary of one result: decode = oracle sample (bits compared, hard-decision
    mismatches, max abs error); train = the 10-step trajectory vs the fp64 oracle."""
    cb = r.get('cpu_baseline') or {}
    if 'parity_bits_compared' in cb:
        return {'bits': cb['parity_bits_compared'], 'mismatches': cb['parity_hard_decision_mismatches'],
                'max_abs_err': _r(cb['parity_max_abs_err'], 3)}
    p = r.get('parity')
    if p:
        return {'steps': p['steps'], 'codewords': p['codewords'],
                'loss_max_rel_err': _r(p['loss_max_rel_err'], 3),
                'param_max_abs_diff': _r(p['param_max_abs_diff'], 3)}
    return None


def compact_entry(r, top=False):
    """The driver-line form of one result dict (decode or train)."""
    keys = ['value', 'unit', 'ms_per_step', 'steps', 'dtype']
    if top:
        keys = ['metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step',
                'higher_is_better', 'scaling', 'vs_baseline', 'dtype', 'data']
    e = {k: _r(r[k], 7) if k == 'value' else _r(r[k]) for k in keys if k in r}
    c = r.get('config') or {}
    if top:
        e['config'] = _pick(c, ['workload', 'code', 'model', 'iters', 'global_batch', 'parallelism',
                                'hard_decision_error_rate', 'frame_error_rate',
                                'channel_hard_decision_error_rate'], 4)
    else:
        e['workload'] = c.get('workload')
        if 'ms_per_step_with_collective' in r:
            e['ms_per_step_with_collective'] = _r(r['ms_per_step_with_collective'])
        if 'ms_per_step_decode_only' in r:          # prior tables rebuilt in every timed step
            e['ms_per_step_decode_only'] = _r(r['ms_per_step_decode_only'])
        if 'hard_decision_error_rate' in c:
            e['ber'] = _r(c['hard_decision_error_rate'], 4)
    rf = r.get('roofline') or {}
    roof = _pick(rf, (['bound', 'achieved', 'peak', 'unit', 'frac', 'traffic', 'kernel_ms',
                       'frac_algorithmic_count', 'hbm_io_frac', 'kernel'] if top else
                      ['bound', 'frac', 'achieved', 'peak', 'traffic', 'kernel_ms', 'frac_flop']), 4)
    if roof is not None:
        roof.setdefault('traffic', None)
        im = rf.get('issue_model')
        if im:
            roof['issue_frac'] = _r(im['issue_frac'], 3)
    e['roofline'] = roof
    cb = r.get('cpu_baseline')
    e['cpu_baseline'] = _pick(cb, ['value', 'unit', 'cores', 'kind', 'value_1_thread', 'sample',
                                   'cpu_model'] if top else ['value', 'value_1_thread', 'cores'], 4)
    e['parity'] = compact_parity(r)
    return e


def strong_scaling(cfgs):
    """Strong-scaling efficiency of config 5 at the reference's global batch of 128 over 8 GPUs
    from this 1-GPU line: t1(128) / (8 t1(16)) per dtype (collective excluded; with it, the
    collective-inclusive step times).  Only meaningful on a 1-GPU run."""
    out = {}
    for dt in ('', '_f64'):
        a = cfgs.get('config5_toric7_v24_train_global128' + dt)
        b = cfgs.get('config5_toric7_v24_train_b16' + dt)
        if not a or not b or a.get('n_gpus') != 1:
            continue
        e = {'t1_128_ms': _r(a['ms_per_step'], 4), 't1_16_ms': _r(b['ms_per_step'], 4),
             'eff_8gpu': _r(a['ms_per_step'] / (8 * b['ms_per_step']), 3)}
        if a.get('ms_per_step_with_collective') and b.get('ms_per_step_with_collective'):
            e['eff_8gpu_with_collective'] = _r(a['ms_per_step_with_collective'] /
                                               (8 * b['ms_per_step_with_collective']), 3)
        out['f64' if dt else 'f32'] = e
    return out or None


def driver_line(res, full_path=None, limit=LINE_LIMIT):
    """Compact JSON line for stdout; asserts it fits `limit` bytes (optional detail is
    dropped first)."""
    line = compact_entry(res, top=True)
    if res.get('dist') is not None:
        dd = res['dist']
        # [rank, device, PCI bus] per rank, the hosts once
        line['dist'] = {'backend': dd['backend'], 'world_size': dd['world_size'],
                        'ranks': [[q['rank'], q['device'], q.get('pci_bus')] for q in dd['ranks']],
                        'hosts': sorted({q.get('host') for q in dd['ranks']})}
    if res.get('scaling_efficiency_global128') is not None:
        line['scaling_efficiency_global128'] = res['scaling_efficiency_global128']
    if res.get('configs'):
        line['configs'] = {n: compact_entry(r) for n, r in res['configs'].items()}
    if full_path:
        line['full_record'] = full_path
    s = json.dumps(line, separators=(',', ':'))
    # shed optional detail until the line fits (never the contract fields): the headline's
    # free text first, then per-config detail in order of decreasing expendability
    cfg = line.get('configs') or {}
    b16 = [e for n, e in cfg.items() if '_b16' in n]      # the per-GPU-16 strong-scaling points

    def each(fn, es=None):
        return lambda: [fn(e) for e in (cfg.values() if es is None else es)]
    sheds = [lambda: (line.get('cpu_baseline') or {}).pop('sample', None),
             lambda: (line.get('cpu_baseline') or {}).pop('cpu_model', None),
             lambda: (line.get('roofline') or {}).pop('kernel', None),
             lambda: line.pop('data', None),
             each(lambda e: (e.pop('unit', None), e.pop('steps', None))),
             each(lambda e: e.pop('cpu_baseline', None), b16),
             each(lambda e: (e.get('roofline') or {}).pop('peak', None)),
             each(lambda e: (e.get('roofline') or {}).pop('achieved', None)),
             each(lambda e: e.pop('workload', None)),
             each(lambda e: e.pop('cpu_baseline', None)),
             each(lambda e: e.pop('parity', None))]
    s = json.dumps(line, separators=(',', ':'))
    for shed in sheds:
        if len(s) <= limit:
            break
        shed()
        s = json.dumps(line, separators=(',', ':'))
    if len(s) > limit:
        # last resort: the contract fields alone, the full record named; never an
        # exception after the whole run
        keep = ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step',
                'higher_is_better', 'scaling', 'vs_baseline', 'dtype', 'config', 'roofline',
                'cpu_baseline', 'full_record')
        s = json.dumps({k: line[k] for k in keep if k in line}, separators=(',', ':'))
        print(f'bench: driver line over {limit} bytes; configs left to {full_path}', file=sys.stderr)
    return s


def rank_map(dev):
    """Backend, world size and every rank's device, gathered to all ranks:
    an N-GPU line shows that the backend saw N ranks on N distinct GPUs."""
    import socket
    me = {'rank': dist.get_rank() if dist.is_initialized() else 0,
          'device': dev.index if dev.type == 'cuda' else -1,
          'host': socket.gethostname()[:24]}
    if dev.type == 'cuda':
        try:
            me['pci_bus'] = torch.cuda.get_device_properties(dev).pci_bus_id
        except Exception:
            pass
    if not dist.is_initialized():
        return {'backend': None, 'world_size': 1, 'ranks': [me]}
    ranks = [None] * dist.get_world_size()
    dist.all_gather_object(ranks, me)
    return {'backend': str(dist.get_backend()), 'world_size': dist.get_world_size(),
            'ranks': ranks}


def write_full_record(res):
    """The full record (every nested field) under gpurun_out/ (merged back by gpurun; scratch on
    the driver's box) or $GNND_BENCH_FULL."""
    path = os.environ.get('GNND_BENCH_FULL', os.path.join('gpurun_out', 'bench_full.json'))
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, 'w') as f:
            json.dump(res, f, indent=1)
        return path
    except OSError:
        return None


def main():
    a = parse()
    if a.model is None:
        a.model = 'v24' if a.mode == 'train' else 'cgnni'
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # (GNND_BENCH_BACKEND=gloo: a rehearsal of the N-rank flow with several ranks on one GPU,
    # which RCCL refuses; ranks then share the visible GPUs round-robin)
    backend = os.environ.get('GNND_BENCH_BACKEND', 'nccl')
    if backend != 'nccl':
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1 or 'TORCHELASTIC_RUN_ID' in os.environ:
        # any torchrun launch (also --nproc-per-node 1) brings up RCCL, so the N>1 code path is
        # the one a 1-GPU torchrun run exercises; bind the communicator to this rank's GPU
        # (barriers then never touch GPU 0)
        dist.init_process_group(backend, device_id=dev)
    res = None
    ranks = rank_map(dev)
    if a.mode == 'train':
        res = train_run(a, world, rank, dev, cpu='full')
    elif a.mode == 'sample':
        sample_main(a, world, rank, dev)
    else:
        res = decode_run(a, world, rank, dev)
        # the default run (the headline workload) also times every other BASELINE config
        headline = a.model == 'cgnni' and a.code == 'bch_63_45' and a.dtype == 'f32'
        if (a.configs == 'on' or (a.configs == 'auto' and headline)):
            sub = sub_config_results(a, world, rank, dev)
            if rank == 0:
                res['configs'] = sub
                res['scaling_efficiency_global128'] = strong_scaling(sub)
    if rank == 0 and res is not None:
        res['dist'] = ranks
        print(driver_line(res, write_full_record(res)), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
