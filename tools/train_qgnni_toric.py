#!/usr/bin/env python3
"""Train the reference's QGNNI (quantum/QGNNI.py, T = 25) on the toric code with this
framework's training path (HIP propagate forward/backward kernels, captured HIP graph) and
save the weights as .npz (state_dict keys of quantum/QGNNI.py).

The reference ships no QGNNI checkpoint for L = 5.  Errors: the reference generator
(p drawn from {0.01..0.10}, quantum/decoder_v2_4.py:187, error_generate.gen_syn).  Loss:
decoder_v2_4's syndrome + logical loss (quantum/decoder_v2_4.py:297-317; the QGNNI script's
logical-only loss gives no signal for the residual syndrome), fused (gnnd_syndrome_loss).
Init: readout MLP = identity (the prior's decision at step 0), message MLP output 0.
usage: python tools/train_qgnni_toric.py [--L 5] [--steps 3000] [--batch 256] [--lr 1e-3]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gnn-decode_amd'))
import gnndecode as gd  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--L', type=int, default=5)
    p.add_argument('--steps', type=int, default=3000)
    p.add_argument('--batch', type=int, default=256)
    p.add_argument('--lr', type=float, default=1e-3)
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--out', default=None)
    # the shipped qgnni_toric_5.npz was trained with decoder_v2_4's weight decay 1e-9
    # (weights/README.md); quantum/QGNNI.py:294 uses 5e-4 (gnndecode.train.REFERENCE_OPTIM)
    p.add_argument('--weight-decay', type=float, default=1e-9)
    a = p.parse_args()
    code = f'toric_{a.L}'
    out = a.out or os.path.join(ROOT, 'gnn-decode_amd', 'gnndecode', 'weights', f'qgnni_{code}.npz')
    dev = torch.device('cuda')
    H = gd.codes.get_code(code)
    torch.manual_seed(a.seed)
    model = gd.MODELS['qgnni'](25, H).to(dev).train()
    with torch.no_grad():
        ro = model.mlp
        for t in (ro[0].weight, ro[0].bias, ro[2].weight, ro[2].bias):
            t.zero_()
        ro[0].weight[0, 0], ro[0].weight[1, 0] = 1.0, -1.0
        ro[2].weight[0, 0], ro[2].weight[0, 1] = 1.0, -1.0
        mm = model.ggc2.mlp
        mm[2].weight.zero_()
        mm[2].bias.zero_()
    g = model.graph(dev)
    logical = gd.codes.toric_logicals(H)
    lf = gd.loss.SyndromeLoss(H, logical).to(dev)
    lg = (torch.as_tensor(logical) != 0).to(torch.int32).to(dev)
    tr = gd.train.Trainer(model, lf, lr=a.lr, weight_decay=a.weight_decay, graph=True, warmup=2)
    xe, ye = gd.data.toric_batch(H, 8192, seed=10 ** 6, device=dev)
    de = gd.data.make_batch(xe, g)

    def evaluate():
        model.eval()
        with torch.no_grad():
            c = gd.ops.decision_errors(g, lg, model(de), ye).tolist()
        model.train()
        return c[0] / ye.numel(), (c[2] + c[3]) / 8192

    ber0, fer0 = evaluate()
    best, best_state = (fer0, ber0), {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    print(f'step 0: eval BER {ber0:.5f} FER {fer0:.5f} (uncorrected BER {float(ye.mean()):.5f})', flush=True)
    data, t0 = None, time.time()
    for s in range(a.steps):
        x, y = gd.data.toric_batch(H, a.batch, seed=a.seed * 10 ** 7 + s, device=dev)
        if data is None:
            data = gd.data.make_batch(x, g)      # one edge_index for the captured graph
        data.x = x
        loss = tr.step(data, y)
        if s % 100 == 99 or s == a.steps - 1:
            ber, fer = evaluate()
            if (fer, ber) < best:
                best, best_state = (fer, ber), {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
            print(f'step {s + 1}: loss {float(loss):.3f}  eval BER {ber:.5f} FER {fer:.5f} '
                  f'(best FER {best[0]:.5f})  {time.time() - t0:.0f} s', flush=True)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    gd.checkpoint.save_npz(best_state, out)
    print(f'saved {out}: eval FER {best[0]:.5f} BER {best[1]:.5f}', flush=True)


if __name__ == '__main__':
    main()
