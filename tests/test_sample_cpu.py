"""Input-synthesis host pieces (no GPU): the Philox4x32-10 generator behind gnnd_sample_*
against the Random123 known-answer vectors (Salmon et al., SC'11, kat_vectors for
philox4x32_10), and the generator-column packing used for random codewords."""
import numpy as np

from gnndecode import codes, ops


def test_philox4x32_10_known_answers():
    kat = [
        ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
        ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
        ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
         (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
    ]
    for ctr, key, want in kat:
        assert ops.philox4x32_10(ctr, key) == list(want), (ctr, key)


def test_generator_column_packing_reencodes():
    H = codes.bch_63_45()
    G = codes.gf2_generator(H)                     # [k, V]
    cols, k = ops.pack_generator_columns(G)
    assert k == G.shape[0] and tuple(cols.shape) == (H.shape[0], (k + 31) // 32)
    rng = np.random.default_rng(0)
    c32 = cols.numpy().view(np.uint32)
    for _ in range(20):
        m = rng.integers(0, 2, k).astype(np.uint8)
        words = np.zeros(c32.shape[1], np.uint32)
        for i in range(k):
            words[i // 32] |= np.uint32(int(m[i]) << (i % 32))
        # codeword bit v = parity of popcount(message words & column mask v), as the kernel
        bits = np.array([sum(bin(int(a) & int(b)).count('1') for a, b in zip(words, c32[v])) % 2
                         for v in range(H.shape[0])])
        np.testing.assert_array_equal(bits, (m.astype(np.int64) @ G.astype(np.int64)) % 2)
        assert not ((bits @ np.asarray(H, np.int64)) % 2).any()
