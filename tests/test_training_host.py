"""Training objectives and logical operators vs the reference (CPU, golden fixtures)."""
import numpy as np
import torch

from gnndecode import codes, loss as L


def test_toric_logicals_match_reference(golden):
    for Ld in (4, 5, 7):
        lg = codes.toric_logicals(codes.toric_code(Ld))
        np.testing.assert_array_equal(lg, golden(f'toric_L{Ld}_graph')['logical'])


def test_syndrome_loss_matches_reference_lossfunc(golden):
    for name, Ld, logical_only in (('train_v24_L5', 5, False), ('train_v24_L7', 7, False),
                                   ('train_qgnni_L4', 4, True)):
        z = golden(name)
        H = codes.toric_code(Ld)
        f = L.SyndromeLoss(H, codes.toric_logicals(H), logical_only=logical_only)
        got = f(torch.from_numpy(z['pred']), torch.from_numpy(z['y'])).item()
        assert abs(got - float(z['loss'])) <= 1e-10 * max(1.0, abs(float(z['loss'])))


def test_classical_loss_matches_reference_lossfunc(golden):
    z = golden('train_cgnni_bch')
    f = L.ClassicalLoss(codes.bch_63_45())
    got = f(torch.from_numpy(z['pred']), torch.from_numpy(z['y']), train=True).item()
    assert abs(got - float(z['loss'])) <= 1e-6 * max(1.0, abs(float(z['loss'])))


def test_toric_failures_counts():
    H = codes.toric_code(5)
    lg = codes.toric_logicals(H)
    y = torch.zeros(3 * 100, 1, dtype=torch.float64)
    y[0] = 1                                   # codeword 0: single flip, not corrected
    pred = torch.zeros_like(y)
    assert L.toric_failures(H, lg, y, pred) == (1, 0)
    pred[0] = 0.9                              # corrected
    assert L.toric_failures(H, lg, y, pred) == (0, 0)
