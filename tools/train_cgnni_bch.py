#!/usr/bin/env python3
"""Train the reference's classical GNNI (classical/CGNNI.py, T = 25) on BCH(63,45) (or LDPC) with this
framework's training path (HIP propagate forward/backward kernels, captured HIP graph) and
save the weights as .npz (state_dict keys of classical/CGNNI.py).

The reference's own checkpoints were trained on one constant all-ones word
(classical/CGNNI.py:195) and decode nothing (BER 1.0); this trains on uniform random BCH
codewords (codes.gf2_generator) with the reference's loss (classical/CGNNI.py:293-309,
lambda 0.8) and SNR grid {1..6} dB, Adam (weight decay 5e-4 as the reference).  The
weights give bench.py a decoder whose hard decisions beat the channel's.
usage: python tools/train_cgnni_bch.py [--code bch_63_45|ldpc_648_324] [--steps 3000]
       [--batch 256] [--lr 1e-3] [--out gnn-decode_amd/gnndecode/weights/cgnni_<code>.npz]"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'gnn-decode_amd'))
import gnndecode as gd  # noqa: E402


def ber(model, x, y, g):
    model.eval()
    with torch.no_grad():
        pred = model(gd.data.make_batch(x, g))
    model.train()
    return float(((pred > 0.5).float() != y).float().mean())


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--steps', type=int, default=3000)
    p.add_argument('--batch', type=int, default=256)
    p.add_argument('--lr', type=float, default=1e-3)
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--init', default='identity', choices=['identity', 'random'],
                   help='identity: readout MLP = identity, message MLP output 0 (channel '
                        'decisions at step 0); random: the reference init')
    p.add_argument('--code', default='bch_63_45')
    p.add_argument('--out', default=None)
    a = p.parse_args()
    dev = torch.device('cuda')
    if a.out is None:
        a.out = os.path.join(ROOT, 'gnn-decode_amd', 'gnndecode', 'weights', f'cgnni_{a.code}.npz')
    H = gd.codes.get_code(a.code)
    V = H.shape[0]
    torch.manual_seed(a.seed)
    model = gd.MODELS['cgnni'](25, H).to(dev).train()
    if a.init == 'identity':
        # start from the channel decision: readout MLP = identity (relu(s) - relu(-s)),
        # message MLP output 0 (layer-2 zero, layer 1 random so its gradient is not)
        with torch.no_grad():
            ro = model.mlp
            ro[0].weight.zero_(); ro[0].bias.zero_(); ro[2].weight.zero_(); ro[2].bias.zero_()
            ro[0].weight[0, 0], ro[0].weight[1, 0] = 1.0, -1.0
            ro[2].weight[0, 0], ro[2].weight[0, 1] = 1.0, -1.0
            mm = model.ggc2.mlp2
            mm[2].weight.zero_(); mm[2].bias.zero_()
    g = model.graph(dev)
    lf = gd.loss.ClassicalLoss(H).to(dev)
    tr = gd.train.Trainer(model, lambda pr, y: lf(pr, y, train=True), lr=a.lr,
                          weight_decay=5e-4, graph=True, warmup=2)
    xe, ye = gd.data.awgn_batch(H, 4096, seed=10 ** 6, device=dev, codewords='random')
    ch = float(((xe.view(4096, -1)[:, :V] < 0).reshape(-1, 1).float() != ye).float().mean())
    best, best_state = 2.0, None
    t0 = time.time()
    data = None
    for s in range(a.steps):
        x, y = gd.data.awgn_batch(H, a.batch, seed=a.seed * 10 ** 7 + s, device=dev, codewords='random')
        if data is None:
            data = gd.data.make_batch(x, g)      # one edge_index for the captured graph
        data.x = x
        loss = tr.step(data, y)
        if s % 100 == 99 or s == a.steps - 1:
            b = ber(model, xe, ye, g)
            if b < best:
                best, best_state = b, {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
            print(f'step {s + 1}: loss {float(loss):.5f}  eval BER {b:.5f} (channel {ch:.5f}, best {best:.5f})'
                  f'  {time.time() - t0:.0f} s', flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    gd.checkpoint.save_npz(best_state, a.out)
    print(f'saved {a.out}: eval BER {best:.5f} vs channel {ch:.5f}', flush=True)


if __name__ == '__main__':
    main()
