"""Component split of disconnected Tanner graphs (gnnd_graph::comp, TannerGraph.components).

The toric code's H is block diagonal (quantum/error_generate.py:39-132: X and Z halves, every
logical row inside one half), so decoder_v2_4 decodes and trains each component of a codeword
in its own workgroup — below one codeword per CU (split_pays; larger batches fill the chip whole
and run whole-graph workgroups, so the larger-B cases here check that path's equality too).  The components share no edge and the per-edge arithmetic is the same,
so the split decode must equal the whole-graph decode BIT FOR BIT (forward outputs and the
training tape); the reverse pass sums its per-workgroup gradient rows in a different grouping
(fp rounding only).  Also: the fused optimizer epilogue (gnnd_train_update) against the
separate reduce / Adam / prepare kernels."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _toric(L):
    import gnndecode as gd
    return gd.codes.toric_code(L)


def test_components_detected():
    import gnndecode as gd
    for L in (4, 5, 7):
        assert gd.TannerGraph(_toric(L), device=DEV).components == 2
    assert gd.TannerGraph(gd.codes.bch_63_45(), device=DEV).components == 1
    assert gd.TannerGraph(gd.codes.get_code('ldpc_648_324'), device=DEV).components == 1


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('L,B', [(5, 1), (5, 128), (7, 128), (7, 700), (5, 5000)])
def test_split_decode_is_bit_identical(dtype, L, B):
    import gnndecode as gd
    H = _toric(L)
    torch.manual_seed(L)
    m = gd.MODELS['v24'](15, H).to(DEV).to(dtype).eval()
    g = m.graph(DEV)
    assert g.components == 2
    x, _ = gd.data.toric_batch(H, B, seed=B, device=DEV, dtype=dtype)
    w = m.prepared_weights(dtype, DEV)
    try:
        g.set_split(True)
        a = gd.ops.decode(g, 'v24', x, 15, w)
        g.set_split(False)
        b = gd.ops.decode(g, 'v24', x, 15, w)
    finally:
        g.set_split(True)
    assert torch.equal(a, b)


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('B', [3, 128, 1500])
def test_split_training_tape_and_gradient(dtype, B):
    """Training forward (output + every tape row) bit-identical split vs whole; reverse-pass
    gradient equal up to the grouping of its fixed-order row sums."""
    import gnndecode as gd
    H = _toric(5)
    torch.manual_seed(2)
    T = 6
    m = gd.MODELS['v24'](T, H).to(DEV).to(dtype)
    g = m.graph(DEV)
    lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H)).to(DEV)
    x, y = gd.data.toric_batch(H, B, seed=7, device=DEV, dtype=dtype)
    flat = m.packed_weights().detach().to(dtype).contiguous()
    prep = gd.ops.prepare_weights('v24', flat)
    res = []
    try:
        for split in (True, False):
            g.set_split(split)
            out, tape = gd.ops.train_forward(g, 'v24', x, prep, T)
            _, dpred = gd.ops.syndrome_loss(lf._graph(DEV), lf.logical_rows, False, out, y)
            gw = gd.ops.train_backward(g, 'v24', flat, x, out, dpred, tape, T)
            res.append((out, tape, gw))
    finally:
        g.set_split(True)
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
    tol = 1e-12 if dtype == torch.float64 else 2e-5
    ga, gb = res[0][2].double(), res[1][2].double()
    assert (ga - gb).abs().max().item() <= tol * max(1.0, gb.abs().max().item())


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
def test_fused_update_matches_separate_kernels(dtype):
    """gnnd_train_update (row reduction + loss sum + Adam + kernel-layout weights, one launch)
    vs gnnd_train_bwd's reduction, torch.sum, gnnd_adam_step and gnnd_prepare_weights."""
    import gnndecode as gd
    n = 1283
    gen = torch.Generator(device='cpu').manual_seed(4)
    for rows in (1, 7, 256, 1024):
        R = torch.randn(rows, n, generator=gen, dtype=torch.float64).to(dtype).to(DEV)
        loss_b = torch.rand(333, generator=gen, dtype=torch.float64).to(dtype).to(DEV)
        p0 = torch.randn(n, generator=gen, dtype=torch.float64).to(dtype).to(DEV)
        pa, pb = p0.clone(), p0.clone()
        ma, va, mb, vb = (torch.zeros_like(p0) for _ in range(4))
        sa = torch.zeros(1, dtype=torch.float64, device=DEV)
        sb = torch.zeros(1, dtype=torch.float64, device=DEV)
        sync = torch.zeros(1, dtype=torch.int32, device=DEV)
        loss = torch.zeros((), dtype=dtype, device=DEV)
        grad = torch.zeros_like(p0)
        # (the kernel layout: fp64 carries the check-MLP table after the weights)
        prep = torch.zeros(gd.ops.prepared_count('v24', dtype), dtype=dtype, device=DEV)
        for it in range(3):
            gd.ops.train_update('v24', dtype, rows=R, n_rows=rows, grad=grad, loss_b=loss_b,
                                loss=loss, param=pa, exp_avg=ma, exp_avg_sq=va, step=sa, sync=sync,
                                lr=1e-3, weight_decay=1e-9, prepared=prep)
            ref_g = R.double().sum(0)
            tol = 1e-12 if dtype == torch.float64 else 2e-5
            assert (grad.double() - ref_g).abs().max().item() <= tol * max(1.0, ref_g.abs().max().item())
            assert abs(loss.item() - loss_b.double().sum().item()) <= tol * loss_b.double().sum().item()
            gd.ops.adam_step(pb, grad.clone(), mb, vb, sb, 1e-3, (0.9, 0.999), 1e-8, 1e-9)
            assert torch.equal(pa, pb), (rows, it)
            assert torch.equal(prep, gd.ops.prepare_weights('v24', pa)), (rows, it)
            assert sa.item() == it + 1 and sync.item() == 0


def test_fused_trainer_split_vs_whole_graph():
    """FusedV24Trainer on the split graph follows the whole-graph trainer (fp64, toric d=7,
    one-codeword-per-workgroup and looping batches)."""
    import gnndecode as gd
    H = _toric(7)
    lg = gd.codes.toric_logicals(H)
    for B in (16, 1100):
        torch.manual_seed(0)
        a = gd.MODELS['v24'](5, H).to(DEV)
        b = gd.MODELS['v24'](5, H).to(DEV)
        b.load_state_dict(a.state_dict())
        ta = gd.train.FusedV24Trainer(a, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=True, warmup=1)
        tb = gd.train.FusedV24Trainer(b, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=True, warmup=1)
        gb = b.graph(torch.device(DEV, torch.cuda.current_device()))   # the trainer's graph
        gb.set_split(False)
        try:
            for s in range(3):
                x, y = gd.data.toric_batch(H, B, seed=s, device=DEV)
                la = ta.step(gd.data.make_batch(x, a.graph(DEV)), y)
                lb = tb.step(gd.data.make_batch(x, gb), y)
                assert abs(la.item() - lb.item()) <= 1e-11 * max(1.0, abs(lb.item()))
        finally:
            gb.set_split(True)
        for k, v in a.state_dict().items():
            torch.testing.assert_close(b.state_dict()[k], v, rtol=1e-10, atol=1e-13)
        assert ta.step_count.item() == 3.0


@pytest.mark.parametrize('dtype', [torch.float32, torch.float64])
@pytest.mark.parametrize('logical_only', [False, True])
@pytest.mark.parametrize('split', [True, False])
def test_fused_loss_reverse_pass_matches_loss_kernel(dtype, logical_only, split):
    """gnnd_train_bwd_loss_partial (syndrome loss computed per codeword component inside the
    reverse pass) = gnnd_syndrome_loss + gnnd_train_bwd_partial: per-codeword losses and the
    reduced gradient."""
    import gnndecode as gd
    H = _toric(5)
    torch.manual_seed(4)
    T = 5
    m = gd.MODELS['v24'](T, H).to(DEV).to(dtype)
    g = m.graph(DEV)
    lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H), logical_only=logical_only).to(DEV)
    assert lf.rows_within_components(2)
    B = 100                      # below one codeword per CU: the split applies (split_pays)
    x, y = gd.data.toric_batch(H, B, seed=9, device=DEV, dtype=dtype)
    flat = m.packed_weights().detach().to(dtype).contiguous()
    prep = gd.ops.prepare_weights('v24', flat)
    try:
        g.set_split(split)
        K = g.components if split else 1
        out, tape = gd.ops.train_forward(g, 'v24', x, prep, T)
        loss_b, dpred = gd.ops.syndrome_loss(lf._graph(DEV), lf.logical_rows, logical_only, out, y)
        ws, nrows = gd.ops.train_backward_partial(g, 'v24', flat, x, out, dpred, tape, T)
        ga = torch.zeros_like(flat)
        gd.ops.train_update('v24', dtype, rows=ws, n_rows=nrows, grad=ga, device=x.device)
        ws2, nrows2, lb2 = gd.ops.train_backward_loss_partial(
            g, 'v24', flat, x, out, y, lf.logical_mask(x.device), lf.logical_rows.size(0),
            logical_only, tape, T)
        gb = torch.zeros_like(flat)
        gd.ops.train_update('v24', dtype, rows=ws2, n_rows=nrows2, grad=gb, device=x.device)
    finally:
        g.set_split(True)
    tol = 1e-12 if dtype == torch.float64 else 2e-5
    assert lb2.numel() == B * K
    per_cw = lb2.view(B, K).double().sum(1)
    assert (per_cw - loss_b.double()).abs().max().item() <= tol * max(1.0, loss_b.abs().max().item())
    tolg = 1e-11 if dtype == torch.float64 else 1e-4
    assert (ga.double() - gb.double()).abs().max().item() <= tolg * max(1.0, ga.abs().max().item())


def test_fused_trainer_fused_loss_vs_loss_kernel():
    import gnndecode as gd
    H = _toric(7)
    lg = gd.codes.toric_logicals(H)
    torch.manual_seed(1)
    a = gd.MODELS['v24'](4, H).to(DEV)
    b = gd.MODELS['v24'](4, H).to(DEV)
    b.load_state_dict(a.state_dict())
    ta = gd.train.FusedV24Trainer(a, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=True, warmup=1)
    tb = gd.train.FusedV24Trainer(b, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=True, warmup=1,
                                  fuse_loss=False)
    for s in range(3):
        x, y = gd.data.toric_batch(H, 64, seed=20 + s, device=DEV)
        la = ta.step(gd.data.make_batch(x, a.graph(x.device)), y)
        lb = tb.step(gd.data.make_batch(x, b.graph(x.device)), y)
        assert abs(la.item() - lb.item()) <= 1e-11 * max(1.0, abs(lb.item()))
    for k, v in a.state_dict().items():
        torch.testing.assert_close(b.state_dict()[k], v, rtol=1e-10, atol=1e-13)


def test_syndrome_loss_large_code_uses_big_lds_or_falls_back():
    """toric L = 20 (fp64) exceeded the loss kernel's 64 KB cap and raised; the cap is
    now the device limit (opt-in LDS), and beyond it SyndromeLoss falls back to the reference
    formula (L = 32)."""
    import gnndecode as gd
    for L in (20, 32):
        H = _toric(L)
        lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H)).to(DEV)
        B, V = 6, H.shape[0]
        gen = torch.Generator(device='cpu').manual_seed(L)
        pred = torch.rand(B * V, 1, generator=gen, dtype=torch.float64).to(DEV)
        y = (torch.rand(B * V, 1, generator=gen) < 0.05).double().to(DEV)
        p1 = pred.clone().requires_grad_(True)
        p2 = pred.clone().requires_grad_(True)
        l1 = lf(p1, y)
        l1.backward()
        l2 = lf.reference_forward(p2, y)
        l2.backward()
        assert abs(l1.item() - l2.item()) <= 1e-10 * abs(l2.item())
        torch.testing.assert_close(p1.grad, p2.grad, rtol=1e-10, atol=1e-12)
        lb, dp = lf.per_codeword(pred, y)
        assert abs(lb.sum().item() - l2.item()) <= 1e-10 * abs(l2.item())


@pytest.mark.parametrize('logical_only', [False, True])
@pytest.mark.parametrize('L,B', [(7, 16), (7, 128), (5, 100)])
def test_forward_loss_equals_reverse_pass_loss(logical_only, L, B):
    """gnnd_train_fwd_loss (the syndrome loss in the unit-split forward's epilogue, fp32 small
    batches) gives the SAME BITS as the reverse pass's fused loss: outputs, per-codeword-and-
    component losses and the gradient rows of gnnd_train_bwd_partial on its d loss / d out."""
    import gnndecode as gd
    H = _toric(L)
    torch.manual_seed(L + B)
    T = 6
    m = gd.MODELS['v24'](T, H).to(DEV).float()
    g = m.graph(DEV)
    lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H), logical_only=logical_only).to(DEV)
    x, y = gd.data.toric_batch(H, B, seed=B, device=DEV, dtype=torch.float32)
    flat = m.packed_weights().detach().contiguous()
    prep = gd.ops.prepare_weights('v24', flat)
    lm, nl = lf.logical_mask(x.device), lf.logical_rows.size(0)
    r = gd.ops.train_forward_loss(g, 'v24', x, prep, T, y, lm, nl, logical_only)
    assert r is not None                       # small batch: the unit-split plan takes it
    out1, tape1, dpred, lb1 = r
    ws1, n1 = gd.ops.train_backward_partial(g, 'v24', flat, x, out1, dpred, tape1, T)
    out2, tape2 = gd.ops.train_forward(g, 'v24', x, prep, T)
    ws2, n2, lb2 = gd.ops.train_backward_loss_partial(g, 'v24', flat, x, out2, y, lm, nl,
                                                      logical_only, tape2, T)
    assert torch.equal(out1, out2) and torch.equal(tape1, tape2)
    assert torch.equal(lb1, lb2)
    assert n1 == n2
    nbytes = n1 * flat.numel() * flat.element_size()
    assert torch.equal(ws1[:nbytes], ws2[:nbytes])


def test_forward_loss_declines_large_batches_and_fp64():
    """Outside the unit-split fp32 plans gnnd_train_fwd_loss launches nothing (None), and the
    fused trainer keeps the reverse pass's loss (its steps equal loss_in_forward=False)."""
    import gnndecode as gd
    H = _toric(5)
    m = gd.MODELS['v24'](4, H).to(DEV).float()
    g = m.graph(DEV)
    lf = gd.loss.SyndromeLoss(H, gd.codes.toric_logicals(H)).to(DEV)
    lm, nl = lf.logical_mask(DEV), lf.logical_rows.size(0)
    x, y = gd.data.toric_batch(H, 4096, seed=3, device=DEV, dtype=torch.float32)
    prep = gd.ops.prepare_weights('v24', m.packed_weights().detach().contiguous())
    assert gd.ops.train_forward_loss(g, 'v24', x, prep, 4, y, lm, nl, False) is None
    m64 = gd.MODELS['v24'](4, H).to(DEV).double()
    x64, y64 = gd.data.toric_batch(H, 16, seed=3, device=DEV, dtype=torch.float64)
    p64 = gd.ops.prepare_weights('v24', m64.packed_weights().detach().contiguous())
    assert gd.ops.train_forward_loss(m64.graph(DEV), 'v24', x64, p64, 4, y64, lm, nl, False) is None


def test_fused_trainer_loss_in_forward_steps_equal():
    import gnndecode as gd
    H = _toric(7)
    lg = gd.codes.toric_logicals(H)
    torch.manual_seed(5)
    a = gd.MODELS['v24'](4, H).to(DEV).float()
    b = gd.MODELS['v24'](4, H).to(DEV).float()
    b.load_state_dict(a.state_dict())
    ta = gd.train.FusedV24Trainer(a, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=False,
                                  loss_in_forward=True)
    tb = gd.train.FusedV24Trainer(b, gd.loss.SyndromeLoss(H, lg).to(DEV), graph=False,
                                  loss_in_forward=False)
    for s in range(3):
        x, y = gd.data.toric_batch(H, 128, seed=30 + s, device=DEV, dtype=torch.float32)
        data = gd.data.make_batch(x, a.graph(DEV))
        la, lb = ta.step(data, y), tb.step(data, y)
        assert torch.equal(la, lb), s
    assert torch.equal(ta.flat, tb.flat)
