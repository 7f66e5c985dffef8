"""Native code construction vs the reference's matrices (golden fixtures).  CPU only."""
import numpy as np

from gnndecode import codes


def test_bch_63_45_matches_reference_file(golden):
    H = codes.bch_63_45()
    assert H.shape == (63, 18)
    np.testing.assert_array_equal(H, golden('bch_63_45_graph')['H'])
    # all-ones is a codeword (classical/CGNNI.py:195 decodes it)
    assert not ((np.ones(63, np.int64) @ H) % 2).any()


def test_toric_matches_generate_pcm(golden):
    for L in (4, 5, 7):
        H = codes.toric_code(L)
        ref = golden(f'toric_L{L}_graph')
        np.testing.assert_array_equal(H, ref['H'])
        v, c = np.nonzero(H)
        np.testing.assert_array_equal(np.stack([v, c]), ref['edge_index'])
        assert H.sum() == 8 * L * L - 8                 # E = 8L^2 - 8
        assert (H.sum(axis=0) == 4).all()               # check degree 4
        # the reference logical operators commute with every stabiliser (plain GF(2) dot,
        # as LossFunc uses them, quantum/decoder_v2_4.py:314-315) after the X/Z swap
        n = 2 * L * L
        Hs = H.T.astype(np.int64)
        lg = ref['logical'].astype(np.int64)
        sw = np.concatenate([lg[:, n:], lg[:, :n]], axis=1)
        assert not ((sw @ Hs.T) % 2).any()


def test_wifi_ldpc_structure():
    """802.11n LDPC(648,324): not in the reference (unverified base
    matrix).  Structural checks only."""
    H = codes.wifi_ldpc_648()
    assert H.shape == (648, 324)
    assert H.sum() == 2376
    assert codes.gf2_rank(H.T) == 324
    # dual-diagonal parity part: base column 12 has shifts at rows 0, 6, 11
    assert (H.sum(axis=0) >= 7).all() and (H.sum(axis=0) <= 8).all()
    # the all-zero word is a codeword
    assert not ((np.zeros(648, np.int64) @ H) % 2).any()
