"""Philox4x32-10 known-answer vectors (Random123 kat_vectors, Salmon et al. SC'11)."""
import numpy as np

import oracle

KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox_known_answers():
    for ctr, key, want in KAT:
        got = oracle.test_philox(1, *ctr, *key)[0]
        assert tuple(int(v) for v in got) == want


def test_uniform_words_look_uniform():
    w = oracle.test_philox(50000, 0, 1, 2, 3, 42, 0).reshape(-1)
    u = (w >> 8).astype(np.float64) / 2**24
    assert abs(u.mean() - 0.5) < 0.005 and abs(u.var() - 1 / 12) < 0.002


def test_fields6_partition_126_bits():
    """gr_fields6: six 21-bit fields = bits [21j, 21j+21) of the little-endian 128-bit draw."""
    rng = np.random.default_rng(7)
    w = rng.integers(0, 2**32, size=(256, 4), dtype=np.uint64).astype(np.uint32)
    got = oracle.test_fields6(w)
    for r in range(w.shape[0]):
        big = sum(int(w[r, k]) << (32 * k) for k in range(4))
        want = [(big >> (21 * j)) & ((1 << 21) - 1) for j in range(6)]
        assert got[r].tolist() == want
    # single-bit probes: every bit 0..125 lands in exactly one field, 126/127 in none
    for b in range(128):
        big = 1 << b
        ww = np.array([[(big >> (32 * k)) & 0xFFFFFFFF for k in range(4)]], np.uint32)
        f = oracle.test_fields6(ww)[0]
        assert int((f != 0).sum()) == (1 if b < 126 else 0)
